// Where does amdsmi_init's ~25 ms go?  Times open("/dev/kfd") (KFD process
// creation) on its own, then amdsmi_init in the same process.
//   g++ -O2 -std=c++17 -I/opt/rocm/include tools/kfd_open_probe.cpp -ldl -o build/kfd_open_probe
#include <amd_smi/amdsmi.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main(int argc, char** argv) {
  bool open_kfd_first = argc > 1 && std::strcmp(argv[1], "kfd-first") == 0;
  void* h = dlopen("libamd_smi.so.26", RTLD_NOW);
  if (!h) h = dlopen("/opt/rocm/lib/libamd_smi.so", RTLD_NOW);
  if (!h) {
    std::printf("dlopen failed: %s\n", dlerror());
    return 1;
  }
  auto init = reinterpret_cast<amdsmi_status_t (*)(uint64_t)>(dlsym(h, "amdsmi_init"));
  auto fini = reinterpret_cast<amdsmi_status_t (*)()>(dlsym(h, "amdsmi_shut_down"));
  int fd = -1;
  if (open_kfd_first) {
    auto t = std::chrono::steady_clock::now();
    fd = open("/dev/kfd", O_RDWR | O_CLOEXEC);
    std::printf("open(/dev/kfd) = %d: %.3f ms\n", fd, ms_since(t));
  }
  for (int i = 0; i < 3; ++i) {
    auto t = std::chrono::steady_clock::now();
    amdsmi_status_t st = init(AMDSMI_INIT_AMD_GPUS);
    double a = ms_since(t);
    t = std::chrono::steady_clock::now();
    fini();
    std::printf("amdsmi_init #%d st=%d: %.3f ms, shut_down %.3f ms\n", i, st, a, ms_since(t));
  }
  if (fd >= 0) close(fd);
  return 0;
}
