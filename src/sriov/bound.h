// SR-IOV discovery through the drivers that bind AMD GPU functions.
//
// Reference: internal/vgpu/pciutil.go:70-112 lists every function on the PCI
// bus and reads the vendor of each - 367 functions on an 8xMI355X host, most
// of a oneshot Job's cycle (~1 ms cold, profiles/oneshot_breakdown_r3.txt).
// The functions that matter are far fewer and the kernel already knows
// them: every AMD GPU function a node uses is bound to amdgpu (bare metal, a
// passthrough guest, an SR-IOV guest's VF), on an MxGPU host its physical
// functions to the GIM host driver, and a function handed to a VM to
// vfio-pci, pci-pf-stub or pci-stub; a PF's enabled VFs are its
// `virtfn<N>` links.  So this source lists, for the loaded ones of those
// drivers (drivers()),
//   <root>/sys/bus/pci/drivers/<driver>/<address>
// reads the identity and SR-IOV attributes of the AMD functions among them
// (about six small sysfs reads per GPU), adds the VFs their `virtfn*` links
// name, and returns them in the same form as the full-bus scan
// (SysfsAmdPCI), so sriov::Lib classifies them identically.
//
// When none of the drivers binds anything - an SR-IOV guest whose amdgpu is
// not loaded, or a node without AMD GPUs - the whole-bus scan (SysfsAmdPCI)
// is the answer.  Inside a VM (`merge_unbound`, the CPU's hypervisor flag) the
// bus also decides which AMD functions exist: whenever uevent_seqnum moved,
// the AMD display / accelerator functions of the bus that no listed driver
// binds - a guest VF amdgpu failed to probe - are read too
// (SysfsAmdPCI::amd_functions: one listing through a kept descriptor,
// identities only of functions not seen before), so the result is the
// reference's whole-bus result (pciutil.go:70-112) function for function.
// A VM's bus is small.  On a host, listing the bus costs 0.1-0.2 ms after an
// idle second (367 functions, profiles/cadence_r6.txt) on every cycle whose
// counter moved - most cycles of a busy node at the deployed cadence - and
// finds nothing the labels use: every function with SR-IOV state is a PF
// whose driver enabled its VFs (gim, vfio-pci, pci-pf-stub: listed) or a VF
// that PF's `virtfn*` links name.  So a host is read through the drivers;
// an unbound AMD function without VFs (a GPU amdgpu failed to probe) is the
// one thing it does not list, and the SR-IOV labeler classifies such a
// function as nothing.
//
// Like the full scan, the result is kept while /sys/kernel/uevent_seqnum is
// unchanged: binding, unbinding, adding or removing a function (VFs
// included, so any NumVFs change) sends a uevent.  A moved counter is not
// enough to re-read everything - every container start on a node (veth,
// loop and cgroup devices) sends uevents too: measured on the pool, 4 of 11
// cycles 1 s apart found it moved and paid a 0.25 ms re-read.  So the
// driver directories (and in a VM the bus) are re-listed (names and inode
// numbers: a function removed and re-added under the same address gets a
// new entry), and on a host the PFs' VF links looked at; only a difference
// re-reads the functions.  Directories are read through descriptors kept
// open (fs::DirListing): no path walk, open or close per check.
#pragma once

#include <array>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "sriov/pci.h"
#include "util/fs.h"

namespace gfd::sriov {

class BoundAmdPCI : public AmdPCI {
 public:
  // `bus`: the whole-bus scan - the answer when no function is bound, and
  // the source of the AMD functions no listed driver binds.  May be null:
  // then only bound functions and their VFs are reported (tests).
  // `merge_unbound`: whether the AMD functions no listed driver binds are
  // looked for on the bus (else the bus is read only when nothing is bound).
  explicit BoundAmdPCI(std::string root = "/", std::shared_ptr<SysfsAmdPCI> bus = nullptr, bool merge_unbound = true)
      : root_(std::move(root)),
        fallback_(std::move(bus)),
        merge_unbound_(merge_unbound),
        seqnum_attr_(fs::join(root_, "sys/kernel/uevent_seqnum")) {}
  std::vector<PCIDevice> Devices() override;
  bool DevicesIfChanged(std::vector<PCIDevice>* out) override;
  // Whether the last Devices() came from the fallback scan.
  bool used_fallback() const { return fell_back_; }

  // The drivers whose bound functions are the node's AMD GPU functions.
  static const std::vector<std::string>& drivers();

 private:
  // Reads `bound`, the `unbound` AMD functions and the VFs of every PF
  // among them; the directories of SR-IOV PFs go to *pf_dirs.
  std::vector<PCIDevice> scan_bound(const std::vector<std::string>& bound, const std::vector<std::string>& unbound,
                                    std::map<std::string, std::unique_ptr<fs::Dir>>* pf_dirs);
  // (address, inode) of every function in the driver directories, sorted.
  std::vector<std::pair<std::string, uint64_t>> list_bound();
  // The bus's AMD functions that are not in `bound` (none without a bus source).
  std::vector<std::string> list_unbound(const std::vector<std::pair<std::string, uint64_t>>& bound);
  // Whether last_ still describes the node: same bound and unbound
  // functions, same VFs.
  bool still_valid(const std::vector<std::pair<std::string, uint64_t>>& bound, const std::vector<std::string>& unbound);
  // Brings last_ up to date; true if it was re-read (or the fallback used).
  bool refresh();
  std::string root_;
  std::shared_ptr<SysfsAmdPCI> fallback_;
  bool merge_unbound_ = true;
  fs::KeptAttr seqnum_attr_;  // /sys/kernel/uevent_seqnum
  bool have_ = false;
  bool fell_back_ = false;
  std::string seqnum_;  // /sys/kernel/uevent_seqnum of the kept result
  std::vector<std::pair<std::string, uint64_t>> bound_;  // list_bound() of the kept result
  std::vector<std::string> unbound_;                      // list_unbound() of the kept result
  std::vector<PCIDevice> last_;
  std::array<fs::DirListing, 5> listings_;  // one per drivers() entry
  fs::DirListing drivers_;                   // sys/bus/pci/drivers
  std::array<bool, 5> loaded_{};             // drivers() entries with a directory there
  std::map<std::string, std::unique_ptr<fs::Dir>> pf_dirs_;  // of last_'s SR-IOV PFs, opened by the scan
};

}  // namespace gfd::sriov
