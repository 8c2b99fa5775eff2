// KFD-topology / DRM sysfs backend.
//
// Reference analogue: the CUDA-driver (Tegra) fallback manager,
// internal/resource/cuda-lib.go:25-88 + cuda-device.go:25-98, which is used
// when NVML is absent.  On MI355X the fallback needs no device context at
// all: everything the labels need is published by amdgpu/KFD in sysfs:
//   /sys/class/kfd/kfd/topology/nodes/N/properties   gfx_target_version,
//       simd_count, simd_per_cu, num_xcc, location_id, domain, device_id,
//       unique_id, drm_render_minor, num_sdma_engines
//   /sys/class/kfd/kfd/topology/nodes/N/mem_banks/M/properties  size_in_bytes
//   /sys/bus/pci/devices/<bdf>/{product_name, current_compute_partition,
//       available_compute_partition, current_memory_partition,
//       available_memory_partition, mem_info_vram_total, xgmi_num_links}
// (layout verified on the MI355X pool, see profiles/hw_probe.md).
// A compute-partitioned GPU (DPX/QPX/CPX) appears as several KFD nodes that
// share one PCI location; they are regrouped into one parent with partitions.
//
// KFD nodes the container may not open (EPERM — GPUs not allocated to this
// pod) are skipped, exactly like amd-smi only reports accessible GPUs.
// `root` prefixes every path so synthetic trees (tests, benchmarks) work.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "resource/filter.h"
#include "resource/types.h"
#include "util/fs.h"

namespace gfd::resource {

struct SysfsOptions {
  std::string root = "/";
  DeviceFilter filter;
  VersionSources versions;  // its root is `root`
};

class SysfsManager : public Manager {
 public:
  explicit SysfsManager(SysfsOptions opts);
  void Init() override;
  void Shutdown() override;
  std::vector<DevicePtr> GetDevices() override;
  std::string GetDriverVersion() override;
  std::optional<RuntimeVersion> GetRuntimeVersion() override;
  std::string Name() const override { return "sysfs"; }
  std::optional<VersionSources> VersionFiles() const override { return opts_.versions; }

  // Enumerate without the Init/Shutdown protocol (used by GetDevices).
  std::vector<DevicePtr> enumerate();

  // GPU nodes of one KFD topology generation, grouped by physical GPU.
  struct Topology;

 private:
  std::shared_ptr<const Topology> read_topology() const;

  SysfsOptions opts_;
  fs::KeptAttr generation_attr_{""};  // topology/generation_id (set in the constructor)
  std::string topology_;
  // The parsed GPU nodes are kept while KFD's topology generation_id (read
  // in Init) is unchanged: KFD rebuilds the topology and bumps the generation
  // whenever a node appears, disappears or changes (partition switch, driver
  // reload, hot-plug), so an unchanged generation means unchanged node
  // properties.  The per-GPU attributes (memory, partition modes, links,
  // SR-IOV state) are still read every cycle.
  std::string generation_;
  std::string cached_generation_;
  std::shared_ptr<const Topology> cached_;
  bool in_vm_ = false;  // CPU reports a hypervisor (fixed for the process)
  bool initialized_ = false;
  bool have_snapshot_ = false;
  std::vector<DevicePtr> snapshot_;
};

// True if <root>/proc/cpuinfo reports the "hypervisor" CPU flag.
bool running_in_vm(const std::string& root);

// True if a KFD topology is present under `root`.
bool has_kfd_topology(const std::string& root, std::string* reason);

}  // namespace gfd::resource
