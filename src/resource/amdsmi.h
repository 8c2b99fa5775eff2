// amd-smi backend: the primary MI355X device enumerator.
//
// Reference analogue: the NVML manager (internal/resource/nvml-lib.go:24-97,
// nvml-device.go, nvml-mig-device.go) on top of the vendored cgo binding
// go-nvml (pkg/nvml/init.go:25-218) and its dlopen wrapper (pkg/dl).
//
// MI355X-first differences, all measured on the pool (profiles/hw_probe.md):
//   * libamd_smi is dlopen'ed ONCE per process and its ~20 entry points bound
//     once (the reference dlopens libnvidia-ml 2N+1 times per cycle).
//   * amdsmi_init costs ~25 ms while all per-GPU queries together cost
//     ~0.5 ms, so the default session mode keeps the library initialised
//     across cycles ("persistent") and re-initialises only when the KFD
//     topology generation changes (a partition-mode switch or driver reload)
//     or a query reports a stale handle.  "per-cycle" reproduces the
//     reference's Init/Shutdown-every-cycle behaviour.
//   * the node is enumerated once per cycle into value snapshots; per-GPU
//     queries run in parallel across physical GPUs on multi-GPU nodes.
//   * the virtualization mode, fixed at driver probe, is queried once per
//     session instead of every cycle.
//   * an unpartitioned GPU's values are read once per session: the compute
//     partition mode (amdgpu reads an XCP register for it, which can wake
//     the GPU), memory partition mode, VRAM and xGMI links change only with
//     a partition / NPS switch or driver reload, which re-initialise the
//     session.  They come straight from the amdgpu sysfs attributes the library
//     itself reads for them - for an unpartitioned GPU and for the parent
//     function of a partitioned one, whose partitions' KFD nodes and counts
//     are kept per session; everything else goes through amd-smi.  The
//     test-only Config::amdsmi_library_only (AmdSmiOptions::sysfs_values =
//     false) sends every query through the library instead.
//   * compute partitions (DPX/QPX/CPX) are separate amd-smi processors on
//     one PCI slot (their function bits may carry the partition index); they
//     are regrouped into parent GPUs by PCI slot and device ID, and split
//     by ASIC serial only for SR-IOV functions (resource/physical.h,
//     split_by_identity).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "resource/filter.h"
#include "resource/types.h"
#include "util/fs.h"

namespace gfd::resource {

struct AmdSmiOptions {
  bool persistent = true;       // keep amdsmi initialised across cycles
  std::string root = "/";       // for the KFD generation check / sysfs hints
  DeviceFilter filter;
  int threads = 0;              // 0 = auto (one per physical GPU, max 8)
  bool sysfs_values = true;     // false: every value through the library (test hook)
  VersionSources versions;  // its root is `root`
};

// Process-wide handle to libamd_smi (opened on first use).
class AmdSmiLib;
// True if libamd_smi can be loaded; `reason` explains either way.
bool has_amdsmi(std::string* reason);

class AmdSmiManager : public Manager {
 public:
  explicit AmdSmiManager(AmdSmiOptions opts);
  ~AmdSmiManager() override;
  void Init() override;
  void Shutdown() override;
  std::vector<DevicePtr> GetDevices() override;
  std::string GetDriverVersion() override;
  std::optional<RuntimeVersion> GetRuntimeVersion() override;
  std::string Name() const override { return opts_.persistent ? "amdsmi(persistent)" : "amdsmi"; }
  std::optional<VersionSources> VersionFiles() const override { return opts_.versions; }

  // Number of amdsmi_init calls made by this manager (tests / benchmarks).
  int init_count() const { return init_count_; }

  // Per-session facts of an unpartitioned GPU's KFD node (see kfd_node_).
  struct KfdNodeFacts {
    uint32_t node_id = 0xFFFFFFFFu;  // 0xFFFFFFFF: none (amd-smi reported none, or not asked yet)
    uint32_t num_xcc = 0;
    bool known = false;  // node and XCD count found for this session
  };
  // Per-session values of an unpartitioned GPU (see session_values_).
  struct SessionValues {
    std::string memory_partition;
    uint64_t vram = 0;
    int xgmi_links = -1;
  };
  // Per-session facts of one compute partition (see partition_facts_).
  struct PartitionFacts {
    void* handle = nullptr;        // amd-smi processor handle
    uint32_t node_id = 0xFFFFFFFFu;  // KFD node (0xFFFFFFFF: not known yet)
    uint32_t partition_id = 0;
    uint32_t num_xcc = 0;
    int sdma = -1;
    uint64_t mem_bytes = 0;
  };
  // The partition modes a GPU supports (see available_).
  struct AvailableModes {
    bool known = false;
    std::vector<std::string> memory, compute;
  };
  // Per-session ASIC identity of one processor (see identity_).
  struct Identity {
    std::string market_name;
    uint32_t vendor_id = 0, device_id = 0, cus = 0;
    uint64_t gfx = 0;
    std::string uuid;
  };

 private:
  std::vector<DevicePtr> snapshot();
  void library_init();
  void library_shutdown();
  std::string read_generation() const;

  AmdSmiOptions opts_;
  mutable fs::KeptAttr generation_attr_{""};  // topology/generation_id (set in the constructor)
  AmdSmiLib* lib_ = nullptr;
  bool lib_initialized_ = false;
  bool in_window_ = false;
  bool have_snapshot_ = false;
  std::vector<DevicePtr> snapshot_;
  std::string generation_;
  int init_count_ = 0;
  // Virtualization mode per BDF for the lifetime of one amd-smi session.
  // amdgpu decides baremetal/host/guest/passthrough once, when it probes the
  // device; a driver reload invalidates the handles and re-initialises the
  // session, which clears this.  Saves ~100 us per GPU per cycle (the most
  // expensive amd-smi call left on the hot path, profiles/).
  std::map<std::string, std::string> virt_mode_;
  // KFD topology node of each unpartitioned GPU (by BDF) and its XCD count
  // (num_xcc) for the lifetime of one session: KFD rebuilds its topology and
  // bumps the generation whenever a node changes (a partition switch changes
  // num_xcc), and a new generation re-initialises the session, which clears
  // this - the same rule the sysfs backend applies to node properties.  The
  // per-cycle values of an unpartitioned GPU (VRAM, compute/memory
  // partition) are read from the amdgpu attributes amd-smi itself reads,
  // ~1 us each through kept-open descriptors instead of 11-18 us per
  // library call.
  std::map<std::string, KfdNodeFacts> kfd_node_;
  // The same for each compute partition of a partitioned GPU (by processor
  // handle): its KFD node, partition id, XCD and SDMA counts and its share
  // of HBM, all fixed until a partition/NPS switch - which rebuilds the KFD
  // topology, bumps its generation and re-initialises the session.  The
  // partition modes themselves are the parent's amdgpu attributes (the
  // compute mode once per session, compute_mode_; the memory mode every
  // cycle) - not two library calls per partition.
  std::map<void*, PartitionFacts> partition_facts_;
  // Parent PCI function of each physical GPU (key: its processors' BDFs),
  // for the lifetime of one session: processor addresses and PCI functions
  // only change with a driver reload or partition switch, which re-initialise.
  std::map<std::string, std::string> parent_bdf_;
  // Supported compute and memory partition modes of each physical GPU (by
  // BDF) for the lifetime of one session: what amdgpu offers follows from
  // the ASIC and, for compute modes, the current memory partition.  A memory
  // partition switch resets the GPU and a compute partition switch rebuilds
  // its KFD nodes; either bumps the topology generation, and so does a
  // driver reload, and a new generation re-initialises the session, which
  // clears this.  (Until round 5 the entry was also keyed by the current
  // modes; since every mode change re-initialises the session, that key
  // could never reject an entry - the mutation check showed it unobservable,
  // profiles/differential_mutations_r5.txt - and it is gone.)  Saves two
  // attribute reads per GPU per cycle.
  std::map<std::string, AvailableModes> available_;
  // Compute partition mode of each physical GPU (by BDF) for the lifetime of
  // one session, read once from current_compute_partition (see
  // session_compute_mode in amdsmi.cpp: that read can wake the GPU).  The
  // memory partition mode is read every cycle (an NBIO register, no wake).
  std::map<std::string, std::string> compute_mode_;
  // Memory partition mode, VRAM and xGMI link count of each unpartitioned
  // GPU (by BDF) for the lifetime of one session: fixed for a driver
  // instance but for a partition / NPS switch, which rebuilds the KFD
  // topology (a new generation re-initialises the session, which clears
  // this) - the same rule the KFD backend applies to its node properties.
  std::map<std::string, SessionValues> session_values_;
  // PCI address of each processor (by handle) for the lifetime of one
  // session, checked once against sysfs and the processor's KFD node
  // (checked_bdf in amdsmi.cpp): amd-smi reads it through libdrm and, when
  // it could not load libdrm_amdgpu, returns uninitialised bytes with
  // success (measured on the pool).  Also saves the call on every cycle.
  std::map<void*, std::string> proc_bdf_;
  // ASIC identity of each processor (by handle) for the lifetime of one
  // session: market name (after the FRU fallback), vendor / device ID, CU
  // count, gfx target and the UUID derived from the ASIC serial - read-only
  // properties of the ASIC, and a partition's CU count changes only with a
  // partition switch, which re-initialises the session.  amdsmi_get_gpu_asic_info
  // was the costliest call left in a cycle (17-28 us after an idle second,
  // profiles/amdsmi_calls_cold_r4.txt).
  std::map<void*, Identity> identity_;
  // The physical GPUs (BDFs, index order) the device filter was last checked against.
  std::vector<std::string> selected_from_;
};

}  // namespace gfd::resource
