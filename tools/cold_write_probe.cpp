// Where the atomic label-file write's time goes when the cycle starts on
// idle cores (the deployed daemon sleeps 60 s between cycles).  Each sample
// sleeps first, then times every syscall of one write.  Variants:
//   path     : the daemon's write (temp in <dir>/gfd-tmp, rename over <dir>/gfd)
//   spin     : the same after a 300 us busy loop (diagnostic: does a core at
//              full clock make the syscalls cheap again?)
// Run against the output directory under test and against /dev/shm (tmpfs)
// to separate file-system work from CPU wake-up.
//   g++ -O2 -std=c++17 tools/cold_write_probe.cpp -o build/cold_write_probe
// Usage: cold_write_probe <dir> [samples=10] [sleep_ms=1000]
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Acc {
  std::string name;
  std::vector<double> t;
  void print() {
    std::sort(t.begin(), t.end());
    std::printf("  %-8s p50 %7.1f us  max %7.1f us\n", name.c_str(), t[t.size() / 2], t.back());
  }
};

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <dir> [samples] [sleep_ms]\n", argv[0]);
    return 2;
  }
  std::string dir = argv[1];
  int samples = argc > 2 ? std::atoi(argv[2]) : 10;
  int sleep_ms = argc > 3 ? std::atoi(argv[3]) : 1000;
  std::string tmp_dir = dir + "/gfd-tmp";
  mkdir(dir.c_str(), 0755);
  mkdir(tmp_dir.c_str(), 0755);
  std::string contents(900, 'x');
  for (int spin : {0, 1}) {
    Acc op{"open"}, wr{"write"}, cl{"close"}, rn{"rename"}, whole{"whole"};
    for (int i = 0; i < samples; ++i) {
      std::this_thread::sleep_for(std::chrono::milliseconds(sleep_ms));
      if (spin) {
        double until = now_us() + 300;
        while (now_us() < until) {
        }
      }
      std::string tmp = tmp_dir + "/gfd-" + std::to_string(i);
      double t0 = now_us();
      int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_EXCL | O_CLOEXEC, 0644);
      double t1 = now_us();
      if (fd < 0 || ::write(fd, contents.data(), contents.size()) != static_cast<ssize_t>(contents.size())) return 1;
      double t2 = now_us();
      ::close(fd);
      double t3 = now_us();
      if (::rename(tmp.c_str(), (dir + "/gfd").c_str()) != 0) return 1;
      double t4 = now_us();
      op.t.push_back(t1 - t0);
      wr.t.push_back(t2 - t1);
      cl.t.push_back(t3 - t2);
      rn.t.push_back(t4 - t3);
      whole.t.push_back(t4 - t0);
    }
    std::printf("%s, %d samples, %d ms idle before each%s\n", dir.c_str(), samples, sleep_ms,
                spin ? ", 300 us busy loop first" : "");
    for (Acc* a : {&op, &wr, &cl, &rn, &whole}) a->print();
  }
  return 0;
}
