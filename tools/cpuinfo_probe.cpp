// Cost of detecting "running in a VM" (the CPU hypervisor flag) per source:
// reading the start of /proc/cpuinfo (16 KB, 4 KB) vs the CPUID bit the
// kernel's flag is set from (leaf 1, ECX bit 31).  Cold (first) and warm.
//   g++ -O2 -std=c++17 tools/cpuinfo_probe.cpp -o build/cpuinfo_probe
#include <cpuid.h>
#include <fcntl.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <string>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static bool from_file(size_t max) {
  std::string buf(max, '\0');
  int fd = open("/proc/cpuinfo", O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  size_t off = 0;
  while (off < max) {
    ssize_t n = read(fd, &buf[off], max - off);
    if (n <= 0) break;
    off += static_cast<size_t>(n);
  }
  close(fd);
  buf.resize(off);
  auto f = buf.find("\nflags");
  if (f == std::string::npos) return false;
  auto e = buf.find('\n', f + 1);
  return (buf.substr(f, e - f) + " ").find(" hypervisor ") != std::string::npos;
}

static bool from_cpuid() {
  unsigned a, b, c, d;
  if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
  return (c >> 31) & 1;
}

int main() {
  for (int rep = 0; rep < 3; ++rep) {
    double t0 = now_us();
    bool f16 = from_file(16384);
    double t1 = now_us();
    bool f4 = from_file(4096);
    double t2 = now_us();
    bool c = from_cpuid();
    double t3 = now_us();
    std::printf("rep %d: cpuinfo 16KB %.1f us (%d)  cpuinfo 4KB %.1f us (%d)  cpuid %.2f us (%d)\n", rep, t1 - t0, f16,
                t2 - t1, f4, t3 - t2, c);
  }
  return 0;
}
