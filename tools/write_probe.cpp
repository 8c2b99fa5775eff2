// Per-syscall cost of the atomic label-file write on a real node.
//   g++ -O2 -std=c++17 -Isrc tools/write_probe.cpp build/libgfdcore.a -o build/write_probe
// Usage: write_probe <output-file>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "lm/labels.h"
#include "util/fs.h"

using namespace gfd;

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Acc {
  const char* name;
  std::vector<double> t;
  void add(double v) { t.push_back(v); }
  void print() {
    std::sort(t.begin(), t.end());
    std::printf("%-14s p50 %.1f us\n", name, t[t.size() / 2]);
  }
};

int main(int argc, char** argv) {
  std::string path = argc > 1 ? argv[1] : "/tmp/gfd-write-probe/gfd";
  std::string dir = fs::dirname(fs::absolute(path));
  fs::mkdir_all(dir);
  std::string tmp_dir = dir + "/gfd-tmp";
  std::string contents(900, 'x');
  Acc mk{"mkdir_all"}, st{"mkstemp"}, wr{"write"}, ch{"fchmod"}, cl{"close"}, rn{"rename"}, whole{"whole"};
  for (int i = 0; i < 300; ++i) {
    double a = now_us();
    fs::mkdir_all(tmp_dir);
    double b = now_us();
    std::string tmpl = tmp_dir + "/gfd-XXXXXX";
    int fd = ::mkstemp(tmpl.data());
    double c = now_us();
    if (::write(fd, contents.data(), contents.size()) < 0) return 1;
    double d = now_us();
    ::fchmod(fd, 0644);
    double e = now_us();
    ::close(fd);
    double f = now_us();
    ::rename(tmpl.c_str(), path.c_str());
    double g = now_us();
    mk.add(b - a), st.add(c - b), wr.add(d - c), ch.add(e - d), cl.add(f - e), rn.add(g - f);
    double h = now_us();
    lm::write_file_atomically(path, contents, 0644);
    whole.add(now_us() - h);
  }
  // Variants: descriptor-relative calls on kept-open directory fds (no path
  // walk), and a temporary in the target directory itself (same-directory
  // rename; NFD would see the temporary, so for comparison only).
  Acc rel{"dirfd-relative"}, same{"same-dir"};
  int tmpfd = ::open(tmp_dir.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
  int outfd = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
  std::string base = fs::basename(path);
  for (int i = 0; i < 300; ++i) {
    double a = now_us();
    std::string name = "gfd-" + std::to_string(i);
    int fd = ::openat(tmpfd, name.c_str(), O_WRONLY | O_CREAT | O_EXCL | O_CLOEXEC, 0644);
    if (fd < 0 || ::write(fd, contents.data(), contents.size()) < 0) return 1;
    ::close(fd);
    ::renameat(tmpfd, name.c_str(), outfd, base.c_str());
    rel.add(now_us() - a);
    double b = now_us();
    std::string dot = dir + "/.gfd-" + std::to_string(i);
    fd = ::open(dot.c_str(), O_WRONLY | O_CREAT | O_EXCL | O_CLOEXEC, 0644);
    if (fd < 0 || ::write(fd, contents.data(), contents.size()) < 0) return 1;
    ::close(fd);
    ::rename(dot.c_str(), path.c_str());
    same.add(now_us() - b);
  }
  for (Acc* x : {&mk, &st, &wr, &ch, &cl, &rn, &whole, &rel, &same}) x->print();
  return 0;
}
