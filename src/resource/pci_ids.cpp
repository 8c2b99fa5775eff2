#include "resource/pci_ids.h"

#include "util/strings.h"

namespace gfd::resource {

namespace {

struct Id {
  uint32_t id;
  const char* name;
  bool vf;
};

constexpr Id kIds[] = {
    {0x75a3, "AMD Instinct MI355X", false}, {0x75a0, "AMD Instinct MI350X", false},
    {0x75b3, "AMD Instinct MI355X VF", true}, {0x74a5, "AMD Instinct MI325X", false},
    {0x74b9, "AMD Instinct MI325X VF", true}, {0x74a1, "AMD Instinct MI300X", false},
    {0x74a9, "AMD Instinct MI300X HF", false}, {0x74b5, "AMD Instinct MI300X VF", true},
    {0x74a0, "AMD Instinct MI300A", false}, {0x740c, "AMD Instinct MI250X/MI250", false},
    {0x740f, "AMD Instinct MI210", false}, {0x738c, "AMD Instinct MI100", false},
};

}  // namespace

std::string device_name(uint32_t device_id) {
  for (const auto& e : kIds)
    if (e.id == device_id) return e.name;
  return str::format("AMD-GPU-0x%04x", static_cast<unsigned>(device_id));
}

bool is_mxgpu_vf(uint32_t device_id) {
  for (const auto& e : kIds)
    if (e.id == device_id) return e.vf;
  return false;
}

bool is_mxgpu_vf(const std::string& device_id) {
  auto v = str::parse_uint_auto(str::trim(device_id));
  return v && is_mxgpu_vf(static_cast<uint32_t>(*v));
}

std::string amd_uuid(uint64_t unique_id, uint32_t device_id) {
  if (unique_id == 0) return "";
  return str::format("%02xff%04x-0000-1000-80%02x-%012llx", static_cast<unsigned>(unique_id >> 56),
                     static_cast<unsigned>(device_id & 0xffff), static_cast<unsigned>((unique_id >> 48) & 0xff),
                     static_cast<unsigned long long>(unique_id & 0xffffffffffffULL));
}

}  // namespace gfd::resource
