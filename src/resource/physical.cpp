#include "resource/physical.h"

#include <algorithm>
#include <mutex>
#include <set>

#include "resource/pci_ids.h"
#include "util/fs.h"
#include "util/log.h"
#include "util/strings.h"

namespace gfd::resource {

bool all_pci_functions(const std::string& root, const std::vector<std::string>& bdfs) {
  for (const auto& b : bdfs)
    if (!fs::exists(fs::join(root, "sys/bus/pci/devices/" + b + "/device"))) return false;
  return true;
}

void log_identity_mismatch(const std::string& slot, size_t members) {
  static std::mutex mu;
  static std::set<std::string> logged;
  std::lock_guard<std::mutex> lk(mu);
  if (!logged.insert(slot).second) return;
  log::printf("Warning: the %zu partitions of the GPU at %s report different serial numbers; counted as one GPU "
              "(grouped by PCI slot and device ID)", members, slot.c_str());
}

bool partition_index_in_function_bits(const GfxTarget& t) { return t.major == 9 && t.minor >= 4; }

std::string bdf_slot(const std::string& bdf) {
  auto dot = bdf.rfind('.');
  return dot == std::string::npos ? bdf : bdf.substr(0, dot);
}

std::string classify_virtualization(const std::string& pci_dir, uint32_t device_id, bool in_vm, bool has_physfn) {
  if (is_mxgpu_vf(device_id) || has_physfn) return "guest";
  if (auto nv = fs::attrs().read_trimmed(fs::join(pci_dir, "sriov_numvfs")); nv && str::parse_uint(*nv).value_or(0) > 0)
    return "host";
  return in_vm ? "passthrough" : "baremetal";
}

// AMD's CLI names a partition's primary at bdf[:10] + ".0"
// (/opt/rocm/libexec/amdsmi_cli/amdsmi_helpers.py:1700-1718): for every
// layout the tests cover, the function found here is that address
// (tests/test_amd_partition_rules.py).
std::string resolve_parent_bdf(const std::string& root, std::vector<std::string> member_bdfs, uint32_t device_id) {
  if (member_bdfs.empty()) return "";
  std::sort(member_bdfs.begin(), member_bdfs.end());
  member_bdfs.erase(std::unique(member_bdfs.begin(), member_bdfs.end()), member_bdfs.end());
  std::vector<std::string> candidates = member_bdfs;
  std::string fn0 = bdf_slot(member_bdfs.front()) + ".0";
  if (std::find(candidates.begin(), candidates.end(), fn0) == candidates.end()) candidates.push_back(fn0);
  for (const auto& c : candidates) {
    // Read once per topology (callers cache the result), so a plain read.
    auto dev = fs::read_trimmed(fs::join(root, "sys/bus/pci/devices/" + c + "/device"));
    if (!dev) continue;
    std::string hex = *dev;
    if (hex.size() > 2 && hex[0] == '0' && (hex[1] == 'x' || hex[1] == 'X')) hex.erase(0, 2);
    auto id = str::parse_uint(hex, 16);
    if (!id) continue;
    if (device_id == 0 || *id == device_id) return c;
  }
  return member_bdfs.front();
}

uint64_t kfd_node_memory_bytes(const std::string& node_dir) {
  uint64_t total = 0;
  std::string banks = fs::join(node_dir, "mem_banks");
  for (const auto& b : fs::list_dir(banks)) {
    auto r = fs::read_file(fs::join(banks, b + "/properties"));
    if (!r.ok()) continue;
    uint64_t heap = 0, size = 0;
    for (const auto& line : str::split(r.data, '\n')) {
      auto kv = str::split_n(line, ' ', 2);
      if (kv.size() != 2) continue;
      if (kv[0] == "heap_type") heap = str::parse_uint(kv[1]).value_or(0);
      if (kv[0] == "size_in_bytes") size = str::parse_uint(kv[1]).value_or(0);
    }
    // HSA_HEAPTYPE_FRAME_BUFFER_PUBLIC (1) / _PRIVATE (2): device-local HBM.
    if (heap == 1 || heap == 2) total += size;
  }
  return total;
}

Attributes partition_engine_counts(const std::string& root, const std::string& parent_bdf) {
  static const std::pair<const char*, const char*> kEngines[] = {{"dec", "engines.decoder"}, {"jpeg", "engines.jpeg"}};
  Attributes out;
  std::string cfg = fs::join(root, "sys/bus/pci/devices/" + parent_bdf + "/compute_partition_config");
  for (const auto& [res, label] : kEngines) {
    auto v = fs::attrs().read_trimmed(cfg + "/" + res + "/num_inst");
    if (!v) continue;
    if (auto n = str::parse_uint(*v)) out[label] = std::to_string(*n);
  }
  return out;
}

Attributes partition_attributes(uint64_t memory_mib, uint32_t compute_units, uint32_t xcds, int sdma,
                                const Attributes& engines, const std::string& compute_partition,
                                const std::string& memory_partition) {
  Attributes a = engines;
  a["memory"] = std::to_string(memory_mib);
  a["compute-units"] = std::to_string(compute_units);
  a["xcds"] = std::to_string(xcds);
  if (sdma >= 0) a["engines.dma"] = std::to_string(sdma);
  if (!compute_partition.empty()) a["compute-partition"] = compute_partition;
  if (!memory_partition.empty()) a["memory-partition"] = memory_partition;
  return a;
}

}  // namespace gfd::resource
