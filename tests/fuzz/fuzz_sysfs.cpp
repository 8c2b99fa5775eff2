// libFuzzer target: a whole labeling cycle of the KFD-sysfs backend over a
// node whose driver-published files hold arbitrary bytes.
//
// The daemon trusts no sysfs text: KFD node properties, amdgpu attributes
// (partition modes, VRAM, xGMI table, product name), SR-IOV counts, the PCI
// device table, DMI and version files may be empty, truncated, huge or
// nonsense on a broken or future driver.  A cycle must then produce labels
// or fail with gfd::Error - never crash or trip a sanitizer - and every
// label it writes must be a valid Kubernetes label value.
//
// The input is split on NUL bytes; field i replaces file kFiles[i] (a
// missing field removes the file).  One fixed tree under /tmp is rewritten
// for every input and a fresh manager reads it (nothing cached between runs).
#include <sys/stat.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "cli/daemon.h"
#include "config/config.h"
#include "lm/labels.h"
#include "resource/sysfs.h"
#include "sriov/sriov.h"
#include "util/error.h"
#include "util/fs.h"

namespace {

const char* const kFiles[] = {
    "sys/class/kfd/kfd/topology/nodes/1/properties",
    "sys/class/kfd/kfd/topology/nodes/2/properties",
    "sys/class/kfd/kfd/topology/nodes/1/mem_banks/0/properties",
    "sys/bus/pci/devices/0000:75:00.0/current_compute_partition",
    "sys/bus/pci/devices/0000:75:00.0/current_memory_partition",
    "sys/bus/pci/devices/0000:75:00.0/available_compute_partition",
    "sys/bus/pci/devices/0000:75:00.0/available_memory_partition",
    "sys/bus/pci/devices/0000:75:00.0/xgmi_num_links",
    "sys/bus/pci/devices/0000:75:00.0/mem_info_vram_total",
    "sys/bus/pci/devices/0000:75:00.0/product_name",
    "sys/bus/pci/devices/0000:75:00.0/device",
    "sys/bus/pci/devices/0000:75:00.0/sriov_numvfs",
    "sys/bus/pci/devices/0000:75:00.0/sriov_totalvfs",
    "sys/bus/pci/devices/0000:75:00.0/class",
    "sys/bus/pci/devices/0000:75:00.0/config",
    "proc/bus/pci/devices",
    "sys/class/dmi/id/product_name",
    "sys/module/amdgpu/version",
    "opt/rocm/.info/version",
};

const std::string& root() {
  static const std::string r = [] {
    char d[] = "/tmp/gfd-fuzz-sysfs-XXXXXX";
    if (!mkdtemp(d)) std::abort();
    std::string s = d;
    gfd::fs::mkdir_all(s + "/sys/class/kfd/kfd/topology/nodes/0");
    gfd::fs::mkdir_all(s + "/sys/class/kfd/kfd/topology/nodes/1/mem_banks/0");
    gfd::fs::mkdir_all(s + "/sys/class/kfd/kfd/topology/nodes/2");
    gfd::fs::mkdir_all(s + "/sys/bus/pci/devices/0000:75:00.0");
    gfd::fs::mkdir_all(s + "/sys/class/dmi/id");
    gfd::fs::mkdir_all(s + "/sys/module/amdgpu");
    gfd::fs::mkdir_all(s + "/opt/rocm/.info");
    gfd::fs::mkdir_all(s + "/proc/bus/pci");
    gfd::lm::write_file_atomically(s + "/sys/class/kfd/kfd/topology/nodes/0/properties", "cpu_cores_count 64\n", 0644);
    gfd::lm::write_file_atomically(s + "/sys/bus/pci/devices/0000:75:00.0/vendor", "0x1002\n", 0644);
    // Enough other functions for the whole-bus scan's parallel path (more
    // than 16 unread functions), and amdgpu's driver directory naming the
    // GPU (the driver-directed scan).  proc/bus/pci/devices stays in the
    // file list (no reader since round 5) so the corpus keeps its meaning.
    for (int i = 0; i < 24; ++i) {
      char name[32];
      std::snprintf(name, sizeof(name), "0000:%02x:%02x.0", i / 8, i % 8);
      std::string dev = s + "/sys/bus/pci/devices/" + name;
      gfd::fs::mkdir_all(dev);
      gfd::lm::write_file_atomically(dev + "/vendor", i % 5 ? "0x1022\n" : "0x1002\n", 0644);
      gfd::lm::write_file_atomically(dev + "/class", i % 3 ? "0x060400\n" : "0x120000\n", 0644);
    }
    gfd::fs::mkdir_all(s + "/sys/bus/pci/drivers/amdgpu/0000:75:00.0");
    gfd::lm::write_file_atomically(s + "/sys/bus/pci/drivers/amdgpu/bind", "", 0644);
    // Not root(): by exit time the static it returns may already be
    // destroyed (its destructor was registered after this handler).
    static const std::string* const tree = new std::string(s);
    std::atexit([] { gfd::fs::remove_all(*tree); });
    return s;
  }();
  return r;
}

}  // namespace

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  const std::string& r = root();
  std::string in(reinterpret_cast<const char*>(data), size);
  size_t pos = 0;
  for (const char* f : kFiles) {
    std::string path = r + "/" + f;
    if (pos > in.size()) {
      ::unlink(path.c_str());
      continue;
    }
    size_t end = in.find('\0', pos);
    if (end == std::string::npos) end = in.size();
    gfd::lm::write_file_atomically(path, in.substr(pos, end - pos), 0644);
    pos = end + 1;
  }
  static const char* const kStrategies[] = {"none", "single", "mixed"};
  gfd::config::Config c;
  c.flags.mig_strategy = kStrategies[size % 3];
  c.flags.gfd.machine_type_file = r + "/sys/class/dmi/id/product_name";
  c.flags.gfd.sysfs_root = r;
  gfd::resource::SysfsOptions o;
  o.root = r;
  o.versions.root = r;
  gfd::resource::SysfsManager m(o);
  try {
    auto result = gfd::cli::label_cycle(m, gfd::sriov::new_sriov_lib(r), c, gfd::lm::empty(), false);
    for (const auto& [k, v] : result.labels)
      if (gfd::lm::sanitize_label_value(v) != v) {  // a value NFD would reject
        std::fprintf(stderr, "invalid label value %s=%s\n", k.c_str(), v.c_str());
        std::abort();
      }
  } catch (const gfd::Error&) {
  }
  return 0;
}
