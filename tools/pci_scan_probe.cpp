// Cost breakdown of the SR-IOV PCI scan on a real node.
//   g++ -O2 -std=c++17 -Isrc tools/pci_scan_probe.cpp build/libgfdcore.a -o build/pci_scan_probe
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>

#include "sriov/pci.h"
#include "sriov/sriov.h"
#include "util/fs.h"
#include "util/trace.h"

using namespace gfd;

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class F>
static double p50(int n, F f) {
  std::vector<double> t;
  for (int i = 0; i < n; ++i) {
    double a = now_us();
    f();
    t.push_back(now_us() - a);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main() {
  const std::string dir = "/sys/bus/pci/devices";
  int err = 0;
  auto entries = fs::list_dir_ino(dir, &err);
  std::printf("pci functions: %zu\n", entries.size());
  std::printf("list_dir_ino p50: %.1f us\n", p50(200, [&] { fs::list_dir_ino(dir, &err); }));
  fs::DirListing listing;
  bool changed = false;
  std::printf("DirListing read (open fd, getdents64 + compare) p50: %.1f us\n",
              p50(200, [&] { listing.read(dir, &changed); }));
  std::printf("read /proc/bus/pci/devices p50: %.1f us\n",
              p50(50, [&] { fs::read_file("/proc/bus/pci/devices", 4u << 20); }));
  sriov::SysfsAmdPCI pci("/");
  trace::begin_cycle();
  std::printf("Devices() first: %.1f us\n", p50(1, [&] { pci.Devices(); }));
  std::printf("first-scan phases: %s\n", trace::summary(0).c_str());
  auto devs = pci.Devices();
  std::printf("amd gpu functions: %zu\n", devs.size());
  std::printf("Devices() steady p50: %.1f us\n", p50(200, [&] { pci.Devices(); }));
  if (!devs.empty()) {
    std::string f = devs[0].path + "/sriov_numvfs";
    std::printf("read sriov_numvfs p50: %.1f us\n", p50(200, [&] { fs::read_trimmed(f); }));
  }
  for (int i = 0; i < 3; ++i) {
    trace::begin_cycle();
    pci.Devices();
    std::printf("phases: %s\n", trace::summary(0).c_str());
  }
  // Serial NumVFs refresh for comparison.
  std::printf("serial 8x numvfs p50: %.1f us\n", p50(200, [&] {
    for (auto& d : devs) fs::read_trimmed(d.path + "/sriov_numvfs");
  }));
  auto lib = sriov::new_sriov_lib("/");
  std::printf("sriov lib Devices() p50: %.1f us\n", p50(200, [&] { lib->Devices(); }));
  return 0;
}
