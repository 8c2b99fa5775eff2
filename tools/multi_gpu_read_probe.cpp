// How the per-GPU attribute reads of one labeling cycle scale with the number
// of GPUs on a real 8-GPU host, using the pool exactly like a cycle does (one
// work item per GPU, one GPU's reads on one thread).  The amdgpu PCI
// attributes of GPUs not allocated to the container are still readable, so a
// 1-GPU box can measure the 2/4/8-GPU fan-out.
//   g++ -O2 -std=c++17 -Isrc tools/multi_gpu_read_probe.cpp build/libgfdcore.a -lpthread -o build/multi_gpu_read_probe
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <ctime>
#include <type_traits>
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>

#include "util/fs.h"
#include "util/pool.h"
#include "util/strings.h"

using namespace gfd;

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const std::string dir = "/sys/bus/pci/devices/";
  std::vector<std::string> gpus;
  for (const auto& name : fs::list_dir(dir)) {
    auto v = fs::read_trimmed(dir + name + "/vendor");
    auto c = fs::read_trimmed(dir + name + "/class");
    if (v && *v == "0x1002" && c && str::starts_with(*c, "0x12") && fs::exists(dir + name + "/mem_info_vram_total"))
      gpus.push_back(name);
  }
  std::printf("GPUs with readable amdgpu attributes: %zu\n", gpus.size());
  static const char* kAttrs[] = {"current_compute_partition", "current_memory_partition", "mem_info_vram_total",
                                 "xgmi_num_links", "available_memory_partition", "available_compute_partition"};
  auto read_gpu = [&](size_t i) {
    for (const char* a : kAttrs) fs::read_trimmed(dir + gpus[i] + "/" + a);
  };
  for (size_t n : {1, 2, 4, 8}) {
    if (n > gpus.size()) break;
    std::vector<double> t;
    for (int it = 0; it < 600; ++it) {
      double a = now_us();
      WorkerPool::instance().parallel_for(n, read_gpu, 8);
      t.push_back(now_us() - a);
    }
    t.erase(t.begin(), t.begin() + 100);
    std::sort(t.begin(), t.end());
    std::printf("%zu GPU(s): %zu attribute reads, p50 %.1f us, p90 %.1f us\n", n, n * 6, t[t.size() / 2],
                t[t.size() * 9 / 10]);
  }
  // Per attribute: 8 GPUs on 8 lanes vs on one thread, and the pool's own
  // fan-out cost (empty items).
  // Median of f's duration, or of f's return value if it measures itself.
  auto p50 = [](auto&& f, int iters) {
    std::vector<double> t;
    for (int it = 0; it < iters; ++it) {
      double a = now_us();
      if constexpr (std::is_same_v<decltype(f()), double>) {
        t.push_back(f());
      } else {
        f();
        t.push_back(now_us() - a);
      }
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
  };
  if (gpus.size() >= 8) {
    std::printf("pool fan-out, 8 empty items: p50 %.1f us\n",
                p50([&] { WorkerPool::instance().parallel_for(8, [](size_t) {}, 8); }, 500));
    for (const char* a : kAttrs) {
      double par = p50([&] { WorkerPool::instance().parallel_for(8, [&](size_t i) { fs::read_trimmed(dir + gpus[i] + "/" + a); }, 8); }, 400);
      double ser = p50([&] { for (size_t i = 0; i < 8; ++i) fs::read_trimmed(dir + gpus[i] + "/" + a); }, 400);
      double one = p50([&] { fs::read_trimmed(dir + gpus[0] + "/" + a); }, 400);
      std::printf("%-28s 1 read %.1f us | 8 GPUs: 8 lanes %.1f us, serial %.1f us\n", a, one, par, ser);
    }
    // Non-amdgpu sysfs attribute of the same devices (PCI core handler).
    double par = p50([&] { WorkerPool::instance().parallel_for(8, [&](size_t i) { fs::read_trimmed(dir + gpus[i] + "/vendor"); }, 8); }, 400);
    double ser = p50([&] { for (size_t i = 0; i < 8; ++i) fs::read_trimmed(dir + gpus[i] + "/vendor"); }, 400);
    std::printf("%-28s 8 GPUs: 8 lanes %.1f us, serial %.1f us\n", "vendor (PCI core)", par, ser);
  }
  // The same reads through descriptors kept open across cycles: pread at
  // offset 0 makes kernfs call the attribute's show() again (a fresh value),
  // without the path walk, open and close.
  {
    std::vector<std::vector<int>> fds(gpus.size());
    for (size_t i = 0; i < gpus.size(); ++i)
      for (const char* a : kAttrs) fds[i].push_back(::open((dir + gpus[i] + "/" + a).c_str(), O_RDONLY | O_CLOEXEC));
    auto pread_gpu = [&](size_t i) {
      char buf[4096];
      for (int fd : fds[i]) (void)!::pread(fd, buf, sizeof(buf), 0);
    };
    std::printf("kept-open fds + pread: 1 GPU %.1f us\n", p50([&] { pread_gpu(0); }, 500));
    if (gpus.size() >= 8) {
      // Lanes sweep for 8 GPUs, back to back and with a 2 ms idle gap before
      // each sample (the daemon sleeps between cycles: workers park, cores idle).
      for (bool gap : {false, true}) {
        std::printf("8 GPUs, kept-open fds + pread, %s:", gap ? "2 ms idle before each" : "back to back");
        for (size_t lanes : {1, 2, 4, 8}) {
          double v = p50([&] {
            if (gap) {
              struct timespec ts{0, 2000000};
              nanosleep(&ts, nullptr);
            }
            double a = now_us();
            if (lanes == 1)
              for (size_t i = 0; i < 8; ++i) pread_gpu(i);
            else
              WorkerPool::instance().parallel_for(8, pread_gpu, lanes);
            return now_us() - a;
          }, 400);
          std::printf("  %zu lane(s) %.1f us", lanes, v);
        }
        std::printf("\n");
      }
    }
    for (auto& v : fds)
      for (int fd : v) ::close(fd);
  }
  // Serial reference: all GPUs on one thread.
  if (gpus.size() >= 8) {
    std::vector<double> t;
    for (int it = 0; it < 300; ++it) {
      double a = now_us();
      for (size_t i = 0; i < 8; ++i) read_gpu(i);
      t.push_back(now_us() - a);
    }
    std::sort(t.begin(), t.end());
    std::printf("8 GPUs serial on one thread: p50 %.1f us\n", t[t.size() / 2]);
  }
  return 0;
}
