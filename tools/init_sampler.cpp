// Samples what the thread calling amdsmi_init is doing (scheduler state,
// current syscall, kernel wait channel) every ~50 us, to find where its
// ~25 ms go.  No ptrace/strace needed: reads /proc/self/task/<tid>/...
//   g++ -O2 -std=c++17 -I/opt/rocm/include tools/init_sampler.cpp -ldl -lpthread -o build/init_sampler
#include <amd_smi/amdsmi.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <thread>

static std::string slurp(const std::string& p) {
  int fd = open(p.c_str(), O_RDONLY);
  if (fd < 0) return "";
  char buf[512];
  ssize_t n = read(fd, buf, sizeof(buf) - 1);
  close(fd);
  if (n <= 0) return "";
  buf[n] = 0;
  return buf;
}

int main() {
  void* h = dlopen("libamd_smi.so.26", RTLD_NOW);
  if (!h) h = dlopen("/opt/rocm/lib/libamd_smi.so", RTLD_NOW);
  if (!h) return 1;
  auto init = reinterpret_cast<amdsmi_status_t (*)(uint64_t)>(dlsym(h, "amdsmi_init"));
  auto fini = reinterpret_cast<amdsmi_status_t (*)()>(dlsym(h, "amdsmi_shut_down"));
  pid_t tid = static_cast<pid_t>(syscall(SYS_gettid));
  std::string base = "/proc/self/task/" + std::to_string(tid) + "/";
  std::atomic<bool> done{false};
  std::map<std::string, int> hist;
  int samples = 0;
  std::thread sampler([&] {
    while (!done.load()) {
      std::string stat = slurp(base + "stat");
      char state = '?';
      auto rp = stat.rfind(')');
      if (rp != std::string::npos && rp + 2 < stat.size()) state = stat[rp + 2];
      std::string sc = slurp(base + "syscall");
      std::string nr = sc.substr(0, sc.find(' '));
      while (!nr.empty() && (nr.back() == '\n')) nr.pop_back();
      std::string wchan = slurp(base + "wchan");
      hist[std::string(1, state) + " syscall=" + nr + " wchan=" + wchan]++;
      ++samples;
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(5));
  auto t = std::chrono::steady_clock::now();
  amdsmi_status_t st = init(AMDSMI_INIT_AMD_GPUS);
  double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
  done = true;
  sampler.join();
  fini();
  std::printf("amdsmi_init st=%d %.3f ms, %d samples (incl. 5 ms idle lead-in)\n", st, ms, samples);
  for (auto& [k, v] : hist) std::printf("%6d  %s\n", v, k.c_str());
  return 0;
}
