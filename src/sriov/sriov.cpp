#include "sriov/sriov.h"

#include "sriov/bound.h"

#include "resource/pci_ids.h"
#include "resource/sysfs.h"
#include "util/error.h"
#include "util/strings.h"

namespace gfd::sriov {

std::optional<SriovCapability> parse_sriov_capability(const std::string& cap) {
  if (cap.size() < 0x1c) return std::nullopt;
  if ((GetLong(cap, 0) & 0xFFFF) != kPciExtCapSriovId) return std::nullopt;
  SriovCapability c;
  c.vf_enable = (GetWord(cap, 0x08) & 0x1) != 0;
  c.initial_vfs = GetWord(cap, 0x0c);
  c.total_vfs = GetWord(cap, 0x0e);
  c.num_vfs = GetWord(cap, 0x10);
  c.vf_offset = GetWord(cap, 0x14);
  c.vf_stride = GetWord(cap, 0x16);
  c.vf_device_id = GetWord(cap, 0x1a);
  return c;
}

bool is_vf_device_id(const std::string& device_id) { return resource::is_mxgpu_vf(device_id); }

std::optional<Info> Lib::Classify(const PCIDevice& d) {
  if (!d.physfn.empty()) {
    Info i;
    i.role = "vf";
    i.physfn = d.physfn;
    return i;
  }
  if (is_vf_device_id(d.device)) {
    Info i;
    i.role = "vf";
    return i;
  }
  // Physical function: the kernel's sysfs view of the SR-IOV capability is
  // authoritative and free; walk the configuration space only when the
  // kernel does not publish it.
  if (d.sriov_totalvfs >= 0) {
    if (d.sriov_numvfs <= 0) return std::nullopt;
    Info i;
    i.role = "pf";
    i.total_vfs = d.sriov_totalvfs;
    i.num_vfs = d.sriov_numvfs;
    i.vf_device = d.sriov_vf_device;
    return i;
  }
  if (d.config.size() >= kPciExpressConfigSpaceSize) {
    auto cap = d.GetExtendedCapability(kPciExtCapSriovId, 0x40);
    if (!cap) return std::nullopt;
    auto c = parse_sriov_capability(*cap);
    if (!c || c->num_vfs == 0 || !c->vf_enable) return std::nullopt;
    Info i;
    i.role = "pf";
    i.total_vfs = c->total_vfs;
    i.num_vfs = c->num_vfs;
    i.vf_device = str::format("0x%04x", c->vf_device_id);
    return i;
  }
  return std::nullopt;
}

std::vector<Function> Lib::Devices() {
  std::vector<PCIDevice> devices;
  std::lock_guard<std::mutex> lk(mu_);
  try {
    // A kept result (the source's own change detection, sriov/bound.h) was
    // classified already: no copy of the functions, no classification.
    if (!pci_->DevicesIfChanged(&devices)) {
      if (have_) return functions_;
      devices = pci_->Devices();
    }
  } catch (const std::exception& e) {
    have_ = false;
    throw Error(std::string("error getting AMD specific PCI devices: ") + e.what());
  }
  have_ = false;  // until classified
  std::vector<Function> out;
  for (auto& d : devices) {
    std::optional<Info> info;
    try {
      info = Classify(d);
    } catch (const std::exception& e) {
      throw Error("unable to read SR-IOV capability for " + d.address + ": " + e.what());
    }
    if (info) out.emplace_back(std::move(d), std::move(*info));
  }
  functions_ = out;
  have_ = true;
  return out;
}

std::optional<std::string> Lib::HostDriverVersion() {
  if (root_.empty()) return std::nullopt;
  auto v = fs::attrs().read_trimmed(fs::join(root_, "sys/module/gim/version"));
  if (!v || v->empty()) return std::nullopt;
  return v;
}

namespace {
class EmptyLib : public Interface {
 public:
  std::vector<Function> Devices() override { return {}; }
};
}  // namespace

std::shared_ptr<Interface> new_sriov_lib(const std::string& root) {
  // The functions the listed drivers bind and the VFs of those PFs, plus the
  // bus's AMD functions no listed driver binds (sriov/bound.h).
  bool merge_unbound = resource::running_in_vm(root);
  return std::make_shared<Lib>(std::make_shared<BoundAmdPCI>(root, std::make_shared<SysfsAmdPCI>(root), merge_unbound),
                               root);
}

std::shared_ptr<Interface> new_mock_sriov() { return std::make_shared<Lib>(std::make_shared<MockAmdPCI>()); }

std::shared_ptr<Interface> new_empty_sriov() { return std::make_shared<EmptyLib>(); }

}  // namespace gfd::sriov
