// Cost of finding the AMD GPU functions of the PCI bus that no listed driver
// binds (sriov/bound.h), by method, on the machine it runs on.
//
//   g++ -O2 -std=c++17 -o build/bus_pass_probe tools/bus_pass_probe.cpp
//   build/bus_pass_probe [rounds]
//
// (a) vendor:   open/read/close <fn>/vendor of every function (the
//               reference's pass, SysfsAmdPCI's first scan);
// (b) driver:   fstatat(<fn>/driver, AT_SYMLINK_NOFOLLOW) of every function
//               relative to one /sys/bus/pci/devices descriptor, then the
//               vendor of the unbound ones only;
// (c) readlink: readlinkat(<fn>/driver) of every function (the driver's
//               name), vendor of the unbound ones;
// (d) procfs:   one read of /proc/bus/pci/devices (vendor and driver of
//               every function, without the PCI domain).
#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static std::vector<std::string> list_functions(const char* dir) {
  std::vector<std::string> out;
  DIR* d = opendir(dir);
  if (!d) return out;
  while (dirent* e = readdir(d))
    if (e->d_name[0] != '.') out.push_back(e->d_name);
  closedir(d);
  std::sort(out.begin(), out.end());
  return out;
}

static bool read_small(int dirfd, const std::string& rel, char* buf, size_t n) {
  int fd = openat(dirfd, rel.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  ssize_t r = read(fd, buf, n - 1);
  close(fd);
  if (r < 0) return false;
  buf[r] = 0;
  return true;
}

int main(int argc, char** argv) {
  int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  const char* dir = "/sys/bus/pci/devices";
  auto fns = list_functions(dir);
  int devfd = open(dir, O_RDONLY | O_DIRECTORY | O_CLOEXEC);
  std::printf("pci functions: %zu\n", fns.size());
  for (int round = 0; round < rounds; ++round) {
    char buf[256];
    // (a)
    double t0 = now_us();
    int amd_a = 0;
    for (const auto& f : fns) {
      std::string p = std::string(dir) + "/" + f + "/vendor";
      int fd = open(p.c_str(), O_RDONLY | O_CLOEXEC);
      if (fd < 0) continue;
      ssize_t r = read(fd, buf, sizeof(buf) - 1);
      close(fd);
      if (r > 0 && std::strncmp(buf, "0x1002", 6) == 0) ++amd_a;
    }
    double ta = now_us() - t0;
    // (b)
    t0 = now_us();
    int unbound = 0, amd_unbound = 0;
    for (const auto& f : fns) {
      struct stat st;
      if (fstatat(devfd, (f + "/driver").c_str(), &st, AT_SYMLINK_NOFOLLOW) == 0) continue;
      ++unbound;
      if (read_small(devfd, f + "/vendor", buf, sizeof(buf)) && std::strncmp(buf, "0x1002", 6) == 0) ++amd_unbound;
    }
    double tb = now_us() - t0;
    // (c)
    t0 = now_us();
    int bound_c = 0;
    for (const auto& f : fns) {
      ssize_t r = readlinkat(devfd, (f + "/driver").c_str(), buf, sizeof(buf) - 1);
      if (r > 0) {
        ++bound_c;
        continue;
      }
      read_small(devfd, f + "/vendor", buf, sizeof(buf));
    }
    double tc = now_us() - t0;
    // (d)
    t0 = now_us();
    size_t bytes = 0;
    int pfd = open("/proc/bus/pci/devices", O_RDONLY | O_CLOEXEC);
    if (pfd >= 0) {
      static char big[1 << 20];
      ssize_t r;
      while ((r = read(pfd, big, sizeof(big))) > 0) bytes += static_cast<size_t>(r);
      close(pfd);
    }
    double td = now_us() - t0;
    std::printf("round %d: (a) vendor %.1f us (%d AMD)  (b) driver-stat %.1f us (%d unbound, %d AMD)  "
                "(c) readlink %.1f us (%d bound)  (d) procfs %.1f us (%zu bytes)\n",
                round, ta, amd_a, tb, unbound, amd_unbound, tc, bound_c, td, bytes);
  }
  return 0;
}
