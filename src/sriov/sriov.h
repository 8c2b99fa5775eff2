// SR-IOV function discovery: the MI355X replacement for vGPU detection.
//
// Reference: internal/vgpu/vgpu.go:25-153 (Interface, Lib.Devices,
// IsVGPUDevice, Device.GetInfo) which finds NVIDIA vGPU guests through the
// "VF" signature of a vendor-specific PCI capability and reads the host
// driver version/branch from its records.
//
// AMD MxGPU partitions a GPU with standard PCIe SR-IOV, so a function is
// SR-IOV relevant when it is
//   * a virtual function seen from the host (sysfs `physfn` link),
//   * a virtual function seen from a guest (a VF device ID; amd-smi's
//     virtualization mode "guest" is folded in by the labeler), or
//   * a physical function with VFs enabled (SR-IOV extended capability
//     NumVFs > 0, or sysfs sriov_numvfs > 0 when the extended config space is
//     not readable by an unprivileged pod).
// The host driver of an MxGPU host is GIM (the SR-IOV "GPU-IOV module"); its
// version is the analogue of the reference's vgpu.host-driver-version and is
// read from the module's sysfs entry on the host.  A guest has no view of it:
// AMD puts no host-driver record in the VF's config space (NVIDIA's vGPU
// vendor capability has one), the PF2VF message amdgpu receives carries no
// host driver version, and amd-smi reports only the guest's own driver - so
// on guests that label is absent (docs/PARITY.md, "parity unpinned").
#pragma once

#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "sriov/pci.h"

namespace gfd::sriov {

struct Info {
  std::string role;        // "pf" or "vf"
  int total_vfs = -1;      // PF only
  int num_vfs = -1;        // PF only
  std::string vf_device;   // PF only: VF device ID from the SR-IOV capability
  std::string physfn;      // VF only (host view): PF address
};

class Function {
 public:
  Function(PCIDevice pci, Info info) : pci_(std::move(pci)), info_(std::move(info)) {}
  const PCIDevice& pci() const { return pci_; }
  // vgpu Device.GetInfo analogue.
  const Info& GetInfo() const { return info_; }

 private:
  PCIDevice pci_;
  Info info_;
};

// SR-IOV capability fields (PCIe Base 5.0 §9.3.3).
struct SriovCapability {
  uint16_t initial_vfs = 0;
  uint16_t total_vfs = 0;
  uint16_t num_vfs = 0;
  uint16_t vf_offset = 0;
  uint16_t vf_stride = 0;
  uint16_t vf_device_id = 0;
  bool vf_enable = false;
};
std::optional<SriovCapability> parse_sriov_capability(const std::string& cap);

// True for known AMD Instinct virtual-function device IDs (guest view).
bool is_vf_device_id(const std::string& device_id);

class Interface {
 public:
  virtual ~Interface() = default;
  virtual std::vector<Function> Devices() = 0;
  // Version of the SR-IOV host driver (GIM) loaded on this node; nullopt
  // when it is not (bare metal, amdgpu-only hosts, guests).
  virtual std::optional<std::string> HostDriverVersion() { return std::nullopt; }
};

class Lib : public Interface {
 public:
  explicit Lib(std::shared_ptr<AmdPCI> pci, std::string root = "") : pci_(std::move(pci)), root_(std::move(root)) {}
  // Thread-safe (one scan at a time): the daemon may start the first scan on
  // a worker while it selects the backend (cli::start).
  std::vector<Function> Devices() override;
  // <root>/sys/module/gim/version (no root: not looked up).
  std::optional<std::string> HostDriverVersion() override;
  // Classifies one PCI function; nullopt if it is not SR-IOV relevant.
  static std::optional<Info> Classify(const PCIDevice& d);

 private:
  std::shared_ptr<AmdPCI> pci_;
  std::string root_;
  std::mutex mu_;
  bool have_ = false;                // functions_ classifies the source's last result
  std::vector<Function> functions_;  // (kept while the source reports no change)
};

// The node's SR-IOV functions (sriov/bound.h): the functions the listed
// drivers bind and their VFs, and inside a VM also the bus's AMD functions
// no listed driver binds.  A Job and the daemon read the same sources.
std::shared_ptr<Interface> new_sriov_lib(const std::string& root);
std::shared_ptr<Interface> new_mock_sriov();
// A library that reports no functions (e.g. when PCI scanning is disabled).
std::shared_ptr<Interface> new_empty_sriov();

}  // namespace gfd::sriov
