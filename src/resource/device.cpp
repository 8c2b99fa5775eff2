#include "resource/types.h"

#include "util/error.h"
#include "util/strings.h"

namespace gfd::resource {

// ---------------------------------------------------------------------------
// GfxTarget

namespace {
char hex_digit(int v) { return static_cast<char>(v < 10 ? '0' + v : 'a' + (v - 10)); }
}  // namespace

std::string GfxTarget::name() const {
  if (!valid()) return "";
  std::string s = "gfx" + std::to_string(major);
  s.push_back(hex_digit(minor % 16));
  s.push_back(hex_digit(stepping % 16));
  return s;
}

std::optional<GfxTarget> parse_gfx_target(const std::string& in) {
  std::string s = str::to_lower(str::trim(in));
  auto colon = s.find(':');
  if (colon != std::string::npos) s = s.substr(0, colon);
  if (!str::starts_with(s, "gfx") || s.size() < 6) return std::nullopt;
  std::string digits = s.substr(3);
  // The last two characters are minor and stepping (hex); the rest is major.
  std::string maj = digits.substr(0, digits.size() - 2);
  auto major = str::parse_uint(maj, 10);
  auto minor = str::parse_uint(digits.substr(digits.size() - 2, 1), 16);
  auto step = str::parse_uint(digits.substr(digits.size() - 1, 1), 16);
  if (!major || !minor || !step || *major == 0) return std::nullopt;
  GfxTarget t;
  t.major = static_cast<int>(*major);
  t.minor = static_cast<int>(*minor);
  t.stepping = static_cast<int>(*step);
  return t;
}

GfxTarget gfx_target_from_kfd(uint64_t v) {
  GfxTarget t;
  if (v >= 1000000) return t;  // major > 99: not a target KFD reports (unknown)
  t.major = static_cast<int>(v / 10000);
  t.minor = static_cast<int>((v / 100) % 100);
  t.stepping = static_cast<int>(v % 100);
  return t;
}

GfxTarget gfx_target_from_amdsmi(uint64_t v) {
  // amd-smi reports the target as an integer whose hex digits spell the
  // name, e.g. 0x950 for gfx950, 0x90a for gfx90a, 0x1100 for gfx1100.
  GfxTarget t;
  if (v == 0 || v > 0xFFFF) return t;  // at most two major digits (gfx12xx); else unknown
  t.stepping = static_cast<int>(v & 0xF);
  t.minor = static_cast<int>((v >> 4) & 0xF);
  uint64_t maj_hex = v >> 8;
  // Major is printed in decimal inside the hex spelling (0x11 -> 11).
  int maj = 0, mul = 1;
  while (maj_hex) {
    maj += static_cast<int>(maj_hex & 0xF) * mul;
    mul *= 10;
    maj_hex >>= 4;
  }
  t.major = maj;
  return t;
}

std::string arch_family(const GfxTarget& t) {
  switch (t.major) {
    case 9:
      if (t.minor == 5) return "cdna4";
      if (t.minor == 4) return "cdna3";
      if (t.minor == 0 && t.stepping == 10) return "cdna2";  // gfx90a
      if (t.minor == 0 && t.stepping == 8) return "cdna1";   // gfx908
      if (t.minor == 0) return "gcn5";                        // gfx900/906
      return "undefined";
    case 10:
      if (t.minor == 1) return "rdna1";
      if (t.minor == 3) return "rdna2";
      return "undefined";
    case 11:
      return "rdna3";
    case 12:
      return "rdna4";
    default:
      return "undefined";
  }
}

std::string partition_mode(const std::string& raw) {
  std::string t = str::trim(raw);
  if (t.empty() || t.size() > 16) return "";
  for (char c : t)
    if (!((c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'))) return "";
  return str::to_upper(t);
}

std::vector<std::string> partition_mode_list(const std::string& raw) {
  std::vector<std::string> out;
  for (const auto& p : str::split(raw, ','))
    if (auto m = partition_mode(p); !m.empty()) out.push_back(m);
  return out;
}

std::string partition_profile_name(const std::string& compute_partition, uint32_t xcds, uint64_t memory_mib) {
  uint64_t gb = (memory_mib + 512) / 1024;
  std::string mode = str::to_lower(compute_partition.empty() ? std::string("xcp") : compute_partition);
  return mode + "." + std::to_string(xcds) + "xcd." + std::to_string(gb) + "gb";
}

// ---------------------------------------------------------------------------
// SnapshotDevice

std::shared_ptr<SnapshotDevice> SnapshotDevice::gpu(DeviceInfo info, bool partitioned, bool partition_capable) {
  auto d = std::make_shared<SnapshotDevice>();
  d->info_ = std::move(info);
  d->partitioned_ = partitioned;
  d->partition_capable_ = partition_capable;
  return d;
}

std::shared_ptr<SnapshotDevice> SnapshotDevice::partition(DeviceInfo info) {
  auto d = std::make_shared<SnapshotDevice>();
  d->info_ = std::move(info);
  d->is_partition_ = true;
  return d;
}

void SnapshotDevice::set_partitions(std::vector<std::shared_ptr<SnapshotDevice>> parts) {
  partitions_ = std::move(parts);
  for (auto& p : partitions_) p->parent_ = shared_from_this();
}

void SnapshotDevice::check(const char* method) const {
  auto it = info_.errors.find(method);
  if (it != info_.errors.end()) throw Error(it->second);
}

bool SnapshotDevice::IsPartitioned() const {
  check("IsPartitioned");
  if (is_partition_) throw Error("IsPartitioned is not supported for compute partitions");
  return partitioned_;
}

bool SnapshotDevice::IsPartitionCapable() const {
  check("IsPartitionCapable");
  if (is_partition_) throw Error("IsPartitionCapable is not supported for compute partitions");
  return partition_capable_;
}

std::vector<DevicePtr> SnapshotDevice::GetPartitions() const {
  check("GetPartitions");
  if (is_partition_) throw Error("GetPartitions is not supported for compute partitions");
  return std::vector<DevicePtr>(partitions_.begin(), partitions_.end());
}

Attributes SnapshotDevice::GetAttributes() const {
  check("GetAttributes");
  if (!is_partition_) throw Error("GetAttributes is not supported for full GPUs");
  return info_.attributes;
}

std::string SnapshotDevice::GetName() const {
  check("GetName");
  return info_.name;
}

uint64_t SnapshotDevice::GetTotalMemoryMiB() const {
  check("GetTotalMemoryMiB");
  return info_.memory_mib;
}

DevicePtr SnapshotDevice::GetParent() const {
  check("GetParent");
  if (!is_partition_) throw Error("GetParent is not supported for full GPUs");
  auto p = parent_.lock();
  if (!p) throw Error("compute partition has no parent GPU");
  return p;
}

GfxTarget SnapshotDevice::GetGfxTarget() const {
  check("GetGfxTarget");
  if (is_partition_) throw Error("GetGfxTarget is not supported for compute partitions");
  return info_.gfx;
}

}  // namespace gfd::resource
