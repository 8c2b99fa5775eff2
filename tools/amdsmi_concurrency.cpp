// Probe: does amd-smi serialise concurrent queries?  Times the per-GPU query
// set the backend issues (a) sequentially, (b) split over 3 threads on the
// same GPU, (c) the same set issued from 8 threads at once (stress; checks
// for deadlocks / errors).  Build:
//   g++ -O2 -std=c++17 -I/opt/rocm/include tools/amdsmi_concurrency.cpp \
//       -o build/amdsmi_concurrency -L/opt/rocm/lib -lamd_smi -lpthread -Wl,-rpath,/opt/rocm/lib
#include <amd_smi/amdsmi.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static std::atomic<int> g_errors{0};

static void part_a(amdsmi_processor_handle p) {  // identity / memory / partitions
  amdsmi_asic_info_t asic;
  if (amdsmi_get_gpu_asic_info(p, &asic) != AMDSMI_STATUS_SUCCESS) g_errors++;
  uint64_t total;
  if (amdsmi_get_gpu_memory_total(p, AMDSMI_MEM_TYPE_VRAM, &total) != AMDSMI_STATUS_SUCCESS) g_errors++;
  amdsmi_kfd_info_t kfd;
  if (amdsmi_get_gpu_kfd_info(p, &kfd) != AMDSMI_STATUS_SUCCESS) g_errors++;
  char buf[64];
  if (amdsmi_get_gpu_compute_partition(p, buf, sizeof(buf)) != AMDSMI_STATUS_SUCCESS) g_errors++;
  if (amdsmi_get_gpu_memory_partition(p, buf, sizeof(buf)) != AMDSMI_STATUS_SUCCESS) g_errors++;
  amdsmi_memory_partition_config_t cfg;
  if (amdsmi_get_gpu_memory_partition_config(p, &cfg) != AMDSMI_STATUS_SUCCESS) g_errors++;
}
static void part_b(amdsmi_processor_handle p) {  // xgmi
  amdsmi_xgmi_link_status_t ls;
  if (amdsmi_get_gpu_xgmi_link_status(p, &ls) != AMDSMI_STATUS_SUCCESS) g_errors++;
}
static void part_c(amdsmi_processor_handle p) {  // virtualization
  amdsmi_virtualization_mode_t vm;
  if (amdsmi_get_gpu_virtualization_mode(p, &vm) != AMDSMI_STATUS_SUCCESS) g_errors++;
}

int main() {
  if (amdsmi_init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) return 1;
  uint32_t ns = 0;
  amdsmi_get_socket_handles(&ns, nullptr);
  std::vector<amdsmi_socket_handle> socks(ns);
  amdsmi_get_socket_handles(&ns, socks.data());
  uint32_t np = 0;
  amdsmi_get_processor_handles(socks[0], &np, nullptr);
  std::vector<amdsmi_processor_handle> procs(np);
  amdsmi_get_processor_handles(socks[0], &np, procs.data());
  amdsmi_processor_handle p = procs[0];
  for (int i = 0; i < 20; ++i) part_a(p), part_b(p), part_c(p);  // warm

  const int R = 200;
  std::vector<double> seq, split;
  for (int r = 0; r < R; ++r) {
    double t0 = now_us();
    part_a(p);
    part_b(p);
    part_c(p);
    seq.push_back(now_us() - t0);
  }
  for (int r = 0; r < R; ++r) {
    double t0 = now_us();
    std::thread tb([&] { part_b(p); });
    std::thread tc([&] { part_c(p); });
    part_a(p);
    tb.join();
    tc.join();
    split.push_back(now_us() - t0);
  }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  double t0 = now_us();
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t)
    th.emplace_back([&] {
      for (int r = 0; r < 50; ++r) part_a(p), part_b(p), part_c(p);
    });
  for (auto& t : th) t.join();
  double stress = now_us() - t0;
  printf("sequential median %.1f us; split-3-threads median %.1f us; 8 threads x 50 full sets %.1f ms (%.1f us/set); errors %d\n",
         med(seq), med(split), stress / 1000, stress / 400, g_errors.load());
  amdsmi_shut_down();
  return 0;
}
