// libFuzzer target: a labeling cycle of the amd-smi backend (over the
// scriptable fake libamd_smi) on a node whose sysfs files hold arbitrary
// bytes - the attributes that backend reads directly (partition modes, VRAM,
// xGMI table, product name, KFD node properties, memory banks).  As for
// fuzz_sysfs.cpp: labels or gfd::Error, no crash, only valid label values.
//
// The first three NUL-separated fields script what the fake library itself
// answers - the market name, the compute-partition string, and
// "cus,xcds,vram_mib,links,virt,parts" - so amd-smi's own values are
// arbitrary too; the fake reports that GPU at 0000:75:00.0 with KFD nodes
// from 1.  The remaining fields are the sysfs files.
#include <dlfcn.h>
#include <sys/stat.h>
#include <unistd.h>

#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <optional>
#include <string>

#include "cli/daemon.h"
#include "config/config.h"
#include "lm/labels.h"
#include "resource/amdsmi.h"
#include "sriov/sriov.h"
#include "util/error.h"
#include "util/fs.h"

namespace {

const char* const kFiles[] = {
    "sys/class/kfd/kfd/topology/nodes/1/properties",
    "sys/class/kfd/kfd/topology/nodes/2/properties",
    "sys/class/kfd/kfd/topology/nodes/1/mem_banks/0/properties",
    "sys/class/kfd/kfd/topology/generation_id",
    "sys/bus/pci/devices/0000:75:00.0/current_compute_partition",
    "sys/bus/pci/devices/0000:75:00.0/current_memory_partition",
    "sys/bus/pci/devices/0000:75:00.0/available_compute_partition",
    "sys/bus/pci/devices/0000:75:00.0/available_memory_partition",
    "sys/bus/pci/devices/0000:75:00.0/xgmi_num_links",
    "sys/bus/pci/devices/0000:75:00.0/mem_info_vram_total",
    "sys/bus/pci/devices/0000:75:00.0/product_name",
    "sys/bus/pci/devices/0000:75:00.0/device",
    "sys/bus/pci/devices/0000:75:00.0/compute_partition_config/dec/num_inst",
    "sys/module/amdgpu/version",
};

std::string g_root;
int (*g_configure)(const char*) = nullptr;

}  // namespace

extern "C" int LLVMFuzzerInitialize(int*, char***) {
  // The fake library next to this executable (built by the same CMake tree).
  char exe[PATH_MAX] = {0};
  if (readlink("/proc/self/exe", exe, sizeof(exe) - 1) <= 0) std::abort();
  std::string dir = gfd::fs::dirname(exe);
  std::string lib = dir + "/libfake_amdsmi.so";
  if (!gfd::fs::exists(lib)) lib = dir + "/libfuzz_fake_amdsmi.so";
  setenv("GFD_AMDSMI_LIBRARY", lib.c_str(), 1);
  char d[] = "/tmp/gfd-fuzz-amdsmi-XXXXXX";
  if (!mkdtemp(d)) std::abort();
  g_root = d;
  for (int n = 1; n <= 8; ++n) gfd::fs::mkdir_all(g_root + "/sys/class/kfd/kfd/topology/nodes/" + std::to_string(n) + "/mem_banks/0");
  gfd::fs::mkdir_all(g_root + "/sys/bus/pci/devices/0000:75:00.0/compute_partition_config/dec");
  gfd::fs::mkdir_all(g_root + "/sys/module/amdgpu");
  std::atexit([] { gfd::fs::remove_all(g_root); });
  return 0;
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (!g_configure) {
    std::string lib = std::getenv("GFD_AMDSMI_LIBRARY");
    void* h = dlopen(lib.c_str(), RTLD_NOW);  // the same handle the backend gets
    if (!h) std::abort();
    g_configure = reinterpret_cast<int (*)(const char*)>(dlsym(h, "fake_amdsmi_configure"));
    if (!g_configure) std::abort();
  }
  std::string in(reinterpret_cast<const char*>(data), size);
  auto next_field = [&](size_t& pos) -> std::optional<std::string> {
    if (pos > in.size()) return std::nullopt;
    size_t end = in.find('\0', pos);
    if (end == std::string::npos) end = in.size();
    std::string f = in.substr(pos, end - pos);
    pos = end + 1;
    return f;
  };
  auto clean = [](std::string v) {  // the fake's spec separators
    for (char& c : v)
      if (c == ';' || c == '|' || c == '\n' || c == '=') c = '_';
    return v.substr(0, 64);
  };
  size_t pos = 0;
  std::string name = clean(next_field(pos).value_or("AMD Instinct MI355 OAM"));
  std::string mode = clean(next_field(pos).value_or("SPX"));
  unsigned long nums[6] = {256, 8, 294896, 7, 1, 1};  // cus, xcds, vram_mib, links, virt, parts
  {
    std::string f = next_field(pos).value_or("");
    size_t i = 0;
    for (const char* p = f.c_str(); *p && i < 6; ++i) {
      char* end = nullptr;
      nums[i] = std::strtoul(p, &end, 10);
      if (end == p) break;
      p = *end == ',' ? end + 1 : end;
    }
  }
  unsigned long parts = nums[5] % 9;  // 0..8 partitions
  char spec[512];
  std::snprintf(spec, sizeof(spec),
                "bdf=0000:75:00.0;mode=%s;parts=%lu;name=%s;cus=%lu;xcds=%lu;vram_mib=%lu;links=%lu;virt=%lu;kfd_base=1\n",
                mode.c_str(), parts, name.c_str(), nums[0] % 100000, nums[1] % 1000, nums[2] % (1ul << 40),
                nums[3] % 64, nums[4] % 8);
  g_configure(spec);
  for (const char* f : kFiles) {
    std::string path = g_root + "/" + f;
    auto v = next_field(pos);
    if (!v) {
      ::unlink(path.c_str());
      continue;
    }
    gfd::lm::write_file_atomically(path, *v, 0644);
  }
  static const char* const kStrategies[] = {"none", "single", "mixed"};
  gfd::config::Config c;
  c.flags.mig_strategy = kStrategies[(size / 2) % 3];
  c.flags.gfd.machine_type_file = "";
  c.flags.gfd.sysfs_root = g_root;
  gfd::resource::AmdSmiOptions o;
  o.root = g_root;
  o.persistent = false;
  gfd::resource::AmdSmiManager m(o);
  try {
    auto result = gfd::cli::label_cycle(m, gfd::sriov::new_sriov_lib(g_root), c, gfd::lm::empty(), false);
    for (const auto& [k, v] : result.labels)
      if (gfd::lm::sanitize_label_value(v) != v) {
        std::fprintf(stderr, "invalid label value %s=%s\n", k.c_str(), v.c_str());
        std::abort();
      }
  } catch (const gfd::Error&) {
  }
  return 0;
}
