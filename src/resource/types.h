// Resource abstraction: the seam between labelers and device backends.
//
// Reference: internal/resource/types.go:22-42 (Manager / Device interfaces).
// MI355X mapping of the Device methods:
//   IsMigEnabled                       -> IsPartitioned: the GPU runs in a
//                                         multi-partition compute mode
//                                         (DPX/QPX/CPX; SPX is "not enabled")
//   IsMigCapable                       -> IsPartitionCapable: the GPU supports
//                                         more than one compute partition mode
//   GetMigDevices                      -> GetPartitions: one device per compute
//                                         partition (XCP) of a partitioned GPU
//   GetAttributes                      -> partition attributes (memory, CUs,
//                                         XCDs, engines, partition modes)
//   GetDeviceHandleFromMigDeviceHandle -> GetParent
//   GetCudaComputeCapability           -> GetGfxTarget (gfx950 -> 9.5.0)
//
// Design difference (MI355X-first): a backend enumerates the node ONCE per
// Init/Shutdown window and every Device is a value snapshot of what the
// driver reported.  The reference re-enumerates through NVML four times per
// cycle and re-dlopens libnvidia-ml per device; here every
// accessor is a memory read.  Per-method error injection keeps the
// reference's fault-injection tests expressible (resource/testing/).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <optional>
#include <string>
#include <vector>

namespace gfd::resource {

// AMDGPU ISA target, the analogue of a CUDA compute capability.
// gfx950 -> {9,5,0}; gfx90a -> {9,0,10}; gfx1100 -> {11,0,0}.
struct GfxTarget {
  int major = 0;
  int minor = 0;
  int stepping = 0;

  bool valid() const { return major != 0; }
  // "gfx950", "gfx90a", "gfx1100".
  std::string name() const;
  bool operator==(const GfxTarget& o) const { return major == o.major && minor == o.minor && stepping == o.stepping; }
};

// Parse "gfx950", "gfx90a", "gfx942:sramecc+:xnack-".  nullopt if malformed.
std::optional<GfxTarget> parse_gfx_target(const std::string& s);
// KFD topology `gfx_target_version` (e.g. 90500, 90010) -> GfxTarget.
GfxTarget gfx_target_from_kfd(uint64_t v);
// amd-smi asic_info.target_graphics_version (e.g. 0x950 / 950 / 0x90a).
GfxTarget gfx_target_from_amdsmi(uint64_t v);
// Architecture family label (internal/lm/resource.go:261-284 analogue):
// gfx908 cdna1, gfx90a cdna2, gfx94x cdna3, gfx95x cdna4, gfx10.1 rdna1,
// gfx10.3 rdna2, gfx11 rdna3, gfx12 rdna4, gfx9.0.x gcn5; else "undefined".
std::string arch_family(const GfxTarget& t);

// Partition profile name, the analogue of a MIG profile ("3g.20gb"):
// "<mode>.<xcds>xcd.<gb>gb", e.g. "cpx.1xcd.36gb" for one XCD of an MI355X in
// CPX/NPS1 (288 GB / 8).  GB is memory rounded to the nearest GiB.  The name
// is a valid DNS-1123 label sequence so it can be embedded in resource names.
std::string partition_profile_name(const std::string& compute_partition, uint32_t xcds, uint64_t memory_mib);
// A compute / memory partition mode as the driver spells it (SPX, CPX,
// NPS1, ...): trimmed and upper-cased, or "" when the text is not a short
// alphanumeric token (an unreadable or malformed attribute must not end up
// in a label name or value - found by tests/fuzz/fuzz_sysfs.cpp).
std::string partition_mode(const std::string& raw);
// "SPX, DPX, QPX, CPX" -> {"SPX", "DPX", "QPX", "CPX"}; malformed entries dropped.
std::vector<std::string> partition_mode_list(const std::string& raw);

// Ordered so label generation is deterministic.
using Attributes = std::map<std::string, std::string>;

class Device;
using DevicePtr = std::shared_ptr<Device>;

// Everything a backend learns about one GPU or one partition.
struct DeviceInfo {
  std::string name;             // product / market name, or partition profile
  std::string bdf;              // 0000:d9:00.0
  std::string uuid;
  int index = -1;               // enumeration index among physical GPUs
  uint32_t vendor_id = 0;
  uint32_t device_id = 0;
  GfxTarget gfx;
  uint32_t compute_units = 0;
  uint32_t xcds = 0;            // XCCs visible to this device / partition
  uint64_t memory_mib = 0;
  std::string compute_partition;  // SPX, DPX, TPX, QPX, CPX ("" unknown)
  std::string memory_partition;   // NPS1, NPS2, NPS4, NPS8 ("" unknown)
  std::vector<std::string> available_compute_partitions;
  std::vector<std::string> available_memory_partitions;
  int xgmi_links = -1;            // active xGMI links, -1 unknown
  std::string virtualization;     // baremetal | host | guest | passthrough | ""
  int partition_id = -1;          // partitions only
  Attributes attributes;          // partitions only
  // Fault injection: method name -> error message (tests / mock fixtures).
  std::map<std::string, std::string> errors;
};

class Device {
 public:
  virtual ~Device() = default;

  virtual bool IsPartitioned() const = 0;
  virtual bool IsPartitionCapable() const = 0;
  virtual std::vector<DevicePtr> GetPartitions() const = 0;
  virtual Attributes GetAttributes() const = 0;
  virtual std::string GetName() const = 0;
  virtual uint64_t GetTotalMemoryMiB() const = 0;
  virtual DevicePtr GetParent() const = 0;
  virtual GfxTarget GetGfxTarget() const = 0;

  // Raw snapshot (node-level labelers read xGMI/partition/virtualization).
  virtual const DeviceInfo& Info() const = 0;
  virtual bool IsPartition() const = 0;
};

// Snapshot-backed device used by every backend.
class SnapshotDevice : public Device, public std::enable_shared_from_this<SnapshotDevice> {
 public:
  // A physical GPU.  `partitioned` selects the IsMigEnabled analogue.
  static std::shared_ptr<SnapshotDevice> gpu(DeviceInfo info, bool partitioned, bool partition_capable);
  // A compute partition of `parent`.
  static std::shared_ptr<SnapshotDevice> partition(DeviceInfo info);

  // Attach partitions to a GPU (sets their parent pointer).
  void set_partitions(std::vector<std::shared_ptr<SnapshotDevice>> parts);

  bool IsPartitioned() const override;
  bool IsPartitionCapable() const override;
  std::vector<DevicePtr> GetPartitions() const override;
  Attributes GetAttributes() const override;
  std::string GetName() const override;
  uint64_t GetTotalMemoryMiB() const override;
  DevicePtr GetParent() const override;
  GfxTarget GetGfxTarget() const override;
  const DeviceInfo& Info() const override { return info_; }
  bool IsPartition() const override { return is_partition_; }

  DeviceInfo& mutable_info() { return info_; }

 private:
  void check(const char* method) const;

  DeviceInfo info_;
  bool is_partition_ = false;
  bool partitioned_ = false;
  bool partition_capable_ = false;
  std::vector<std::shared_ptr<SnapshotDevice>> partitions_;
  std::weak_ptr<SnapshotDevice> parent_;
};

struct RuntimeVersion {
  unsigned major = 0;
  unsigned minor = 0;
};

// Where the node's driver and ROCm versions are read from (resource/versions.h).
struct VersionSources {
  std::string root = "/";         // sysfs root (synthetic trees in tests)
  std::string host_root;          // host filesystem mount point ("" = none)
  std::string rocm_version_file;  // explicit ROCm version file ("" = discover)
  // Whether the answer may be kept across calls (a loop daemon's; a oneshot
  // Job asks once and keeps nothing: rocm_version).
  bool keep = false;
};

// Reference: resource.Manager (types.go:22-28).  GetCudaDriverVersion maps
// to GetRuntimeVersion (the node's ROCm major/minor; nullopt when the node
// has no ROCm release installed).
class Manager {
 public:
  virtual ~Manager() = default;
  virtual void Init() = 0;
  virtual void Shutdown() = 0;
  virtual std::vector<DevicePtr> GetDevices() = 0;
  virtual std::string GetDriverVersion() = 0;
  virtual std::optional<RuntimeVersion> GetRuntimeVersion() = 0;
  virtual std::string Name() const = 0;
  // For managers whose version queries are plain reads of node files
  // (resource::driver_version / rocm_version from these sources) and touch
  // no manager state: the daemon then reads them on a worker, overlapped
  // with enumeration.  nullopt: ask the manager, inside the Init window.
  virtual std::optional<VersionSources> VersionFiles() const { return std::nullopt; }
  // Work a manager may start in the background before its first Init (the
  // warm-start manager's library initialisation).  The daemon calls it once,
  // in loop mode, when the manager is built.
  virtual void Prepare() {}
};

using ManagerPtr = std::shared_ptr<Manager>;

}  // namespace gfd::resource
