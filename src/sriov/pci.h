// PCI function discovery and configuration-space parsing for AMD GPUs.
//
// Reference: internal/vgpu/pciutil.go:27-204 (NvidiaPCI, PCIDevice,
// GetVendorSpecificCapability, GetByte/GetWord/GetLong, MockNvidiaPCI).
// NVIDIA's vGPU guests are identified by a vendor-specific capability
// (ID 0x09, signature "VF") that the host driver writes into the virtual
// config space.  AMD MxGPU uses standard PCIe SR-IOV instead, so besides the
// classic capability-list walk this module walks the PCIe *extended*
// capability list (offset 0x100+) to find the SR-IOV capability (ID 0x0010)
// of physical functions, and reads the world-readable sysfs attributes
// (sriov_totalvfs, sriov_numvfs, physfn) that the kernel derives from it.
//
// Unprivileged readers only see the first 64 bytes of config space (measured
// on the MI355X pool), so the walkers report that case as an error exactly
// like the reference, and the SR-IOV library falls back to sysfs.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <optional>
#include <string>
#include <vector>

#include "util/fs.h"

namespace gfd::sriov {

inline constexpr const char* kPciDevicesRoot = "sys/bus/pci/devices";
inline constexpr const char* kAmdVendorId = "0x1002";

// Standard configuration header / capability list (PCI Local Bus 3.0 §6.7).
inline constexpr int kPciStatusByte = 0x06;
inline constexpr int kPciStatusCapabilityList = 0x10;
inline constexpr int kPciCapabilityList = 0x34;
inline constexpr int kPciCapabilityListId = 0;
inline constexpr int kPciCapabilityListNext = 1;
inline constexpr int kPciCapabilityLength = 2;
inline constexpr int kPciCapabilityVendorSpecificId = 0x09;
inline constexpr int kPciCapabilityExpressId = 0x10;
// PCIe extended capabilities (PCIe Base 5.0 §7.6).
inline constexpr int kPciExtendedCapabilityStart = 0x100;
inline constexpr int kPciExtCapSriovId = 0x0010;
inline constexpr int kPciExtCapVendorSpecificId = 0x000B;
inline constexpr size_t kPciConfigSpaceSize = 256;
inline constexpr size_t kPciExpressConfigSpaceSize = 4096;

struct PCIDevice {
  std::string path;
  std::string address;   // 0000:d9:00.0
  std::string vendor;    // 0x1002
  std::string device;    // 0x75a3
  std::string class_code;  // first 4 hex digits of class, e.g. "0x12"
  std::string config;    // raw configuration space bytes (may be truncated)
  // sysfs-derived SR-IOV facts (-1 / "" = attribute absent).
  int sriov_totalvfs = -1;
  int sriov_numvfs = -1;
  std::string sriov_vf_device;  // e.g. 0x75b3
  std::string physfn;    // PF address if this function is a VF on the host

  // Classic capability-list walk for `cap_id` (pciutil.go:115-149: loop and
  // broken-chain detection).  Returns the capability bytes (length taken from
  // the capability's length byte, or 2 if it has none), nullopt if absent.
  // Throws gfd::Error if fewer than 256 bytes of config space are available.
  std::optional<std::string> GetCapability(int cap_id) const;
  // pciutil.go GetVendorSpecificCapability (ID 0x09).
  std::optional<std::string> GetVendorSpecificCapability() const { return GetCapability(kPciCapabilityVendorSpecificId); }
  // PCIe extended capability walk.  Returns the capability body starting at
  // its header; nullopt if absent.  Throws if config space is < 4096 bytes.
  std::optional<std::string> GetExtendedCapability(int ext_id, size_t length) const;
};

uint8_t GetByte(const std::string& buf, size_t pos);
uint16_t GetWord(const std::string& buf, size_t pos);
uint32_t GetLong(const std::string& buf, size_t pos);

// Source of AMD PCI functions (NvidiaPCI analogue).
class AmdPCI {
 public:
  virtual ~AmdPCI() = default;
  virtual std::vector<PCIDevice> Devices() = 0;
  // Like Devices(), but false - and *out untouched - when the functions are
  // the ones this source's previous call returned (a kept result: nothing
  // to copy or classify again).
  virtual bool DevicesIfChanged(std::vector<PCIDevice>* out) {
    *out = Devices();
    return true;
  }
};

// Walks <root>/sys/bus/pci/devices and keeps vendor 0x1002 display (0x03)
// and processing-accelerator (0x12) functions: the reference's approach
// (pciutil.go:70-112), and since round 4 only the fallback of the
// driver-directed source (sriov/bound.h) for nodes where neither amdgpu nor
// gim binds anything.
//
// Cost model (measured on the MI355X pool, ~1.3 ms per scan before this):
// a large server has hundreds of PCI functions and the reference reads
// `vendor` (and, for its vendor, the whole config space) of every one of them
// every cycle.  Here:
//   * the bus is re-listed every call (hot-plug is seen immediately) through
//     a directory descriptor kept open (fs::DirListing), but the immutable
//     identity of a function (vendor, class, device ID) is kept per (address,
//     sysfs inode) - a removed and re-added device gets a new inode and is
//     re-read;
//   * the listing itself is skipped while /sys/kernel/uevent_seqnum, which
//     every device addition or removal increments, is unchanged;
//   * the mutable SR-IOV state comes from the kernel's sysfs attributes
//     (sriov_numvfs), which cost no PCI config cycles, and is re-read whenever
//     the listing changed - enabling or disabling VFs adds or removes their
//     PCI functions, so an unchanged listing means unchanged NumVFs;
//   * configuration space (a 4 KiB read = ~1000 config cycles when
//     privileged) is read only for functions whose SR-IOV state sysfs does not
//     publish.
// Measured on an 8-GPU MI355X host with 367 PCI functions: ~1.5 ms first
// scan; then 15 us when the listing is read (one getdents64 pass) and ~1 us
// when uevent_seqnum shows nothing was added or removed
// (profiles/pci_scan_probe.txt).
class SysfsAmdPCI : public AmdPCI {
 public:
  explicit SysfsAmdPCI(std::string root = "/")
      : root_(std::move(root)), seqnum_attr_(fs::join(root_, "sys/kernel/uevent_seqnum")) {}
  std::vector<PCIDevice> Devices() override;
  // The addresses of the AMD display / accelerator functions on the bus,
  // sorted: Devices() without the per-function SR-IOV state (the
  // driver-directed source, sriov/bound.h, reads that itself for the
  // functions no driver it lists binds).  Same cost model: nothing read
  // while uevent_seqnum is unchanged, one listing when it moved, identities
  // only of functions not seen before.
  std::vector<std::string> amd_functions();

 private:
  // Brings the listing and the identity cache up to date with the bus.
  void update();
  // Immutable for the lifetime of a sysfs object: vendor/class/device,
  // TotalVFs and the VF device ID (read-only SR-IOV capability fields), and
  // a VF's physfn link.  Only NumVFs is re-read every call.
  struct Identity {
    uint64_t ino = 0;
    bool relevant = false;  // AMD display / accelerator function
    std::string class_code;
    std::string device;
    int sriov_totalvfs = -1;
    std::string sriov_vf_device;
    std::string physfn;
    int sriov_numvfs = -1;  // last NumVFs read; -1 = re-read (listing changed)
  };
  static Identity read_identity(const std::string& addr, const std::string& path, uint64_t ino);
  std::string root_;
  fs::KeptAttr seqnum_attr_;  // /sys/kernel/uevent_seqnum
  fs::DirListing listing_;
  bool scanned_ = false;
  std::string seqnum_;  // /sys/kernel/uevent_seqnum at the last scan
  std::vector<std::pair<std::string, Identity>> cache_;  // sorted by address
};

// Built-in mock with synthetic MI300X/MI355X configuration spaces:
//   "passthrough": a PF without SR-IOV capability,
//   "pf":          a PF with an SR-IOV capability (TotalVFs 8, NumVFs 4),
//   "vf":          a VF (device 0x74b5) whose physfn is the "pf" device.
class MockAmdPCI : public AmdPCI {
 public:
  MockAmdPCI();
  explicit MockAmdPCI(std::vector<PCIDevice> devices) : devices_(std::move(devices)) {}
  std::vector<PCIDevice> Devices() override { return devices_; }
  static std::string passthrough_config();
  static std::string pf_config(uint16_t total_vfs, uint16_t num_vfs, uint16_t vf_device);
  static std::string vf_config(uint16_t device);

 private:
  std::vector<PCIDevice> devices_;
};

}  // namespace gfd::sriov
