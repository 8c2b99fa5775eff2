#include "sriov/bound.h"

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <optional>
#include <set>

#include "util/error.h"
#include "util/fs.h"
#include "util/pool.h"
#include "util/strings.h"
#include "util/trace.h"

namespace gfd::sriov {

namespace {

// "DDDD:BB:DD.F" (a driver directory also holds bind, unbind, new_id,
// module, uevent...).
bool is_pci_address(const std::string& name) {
  size_t n = name.size();
  if (n < 12 || name[n - 2] != '.' || name[n - 5] != ':' || name[n - 8] != ':') return false;
  for (size_t i = 0; i < n; ++i) {
    if (i == n - 2 || i == n - 5 || i == n - 8) continue;
    char c = name[i];
    if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'))) return false;
  }
  return true;
}

// The function at `dir` as SysfsAmdPCI reports it, or nullopt when it is not
// an AMD (0x1002) display (0x03) or processing-accelerator (0x12) function:
// amdgpu's and gim's ID tables name vendor 0x1002 only, but vfio-pci and the
// stub drivers bind anything.
// Class and device ID from the function's `uevent` (PCI_CLASS=120000,
// PCI_ID=1002:75A3): one read instead of `class` and `device`.  The kernel
// prints PCI_CLASS with %04X, so a display function's leading zero is gone
// (0x038000 is "38000"): the value is parsed and re-padded to the six digits
// of the `class` attribute.
bool from_uevent(const fs::Dir& dir, std::string* cls, std::string* vendor, std::string* device) {
  auto r = dir.read_attr("uevent");
  if (!r.ok()) return false;
  std::string c, id;
  for (const auto& line : str::split(r.data, '\n')) {
    if (str::starts_with(line, "PCI_CLASS=")) c = line.substr(10);
    if (str::starts_with(line, "PCI_ID=")) id = line.substr(7);
  }
  auto colon = id.find(':');
  if (c.empty() || c.size() > 6 || colon == std::string::npos) return false;
  *vendor = "0x" + str::to_lower(id.substr(0, colon));
  char* end = nullptr;
  unsigned long v = std::strtoul(c.c_str(), &end, 16);
  if (end == c.c_str() || *end != 0) return false;
  char buf[16];
  std::snprintf(buf, sizeof(buf), "0x%06lx", v);
  *cls = buf;
  *device = "0x" + str::to_lower(id.substr(colon + 1));
  return true;
}

// `keep`: the function's directory, handed over when it is an SR-IOV PF (the
// later checks look its VF links up through it).
std::optional<PCIDevice> read_function(const std::string& path, const std::string& addr, const std::string& physfn,
                                       std::unique_ptr<fs::Dir>* keep) {
  auto owned = std::make_unique<fs::Dir>(path);
  const fs::Dir& dir = *owned;
  std::string c, vendor, device;
  bool have_device = from_uevent(dir, &c, &vendor, &device);
  if (!have_device) {
    auto v = dir.read_attr("vendor", 64);
    if (!v.ok()) throw Error("unable to read PCI device vendor id for " + addr + ": " + fs::errno_str(v.err));
    vendor = str::trim(v.data);
  }
  // vfio-pci and the stub drivers bind any vendor's functions.
  if (vendor != kAmdVendorId) return std::nullopt;
  if (!have_device) {
    auto cls = dir.read_attr("class", 64);
    if (!cls.ok()) throw Error("unable to read PCI device class for " + addr + ": " + fs::errno_str(cls.err));
    c = str::trim(cls.data);
  }
  if (!str::starts_with(c, "0x03") && !str::starts_with(c, "0x12")) return std::nullopt;
  PCIDevice d;
  d.path = path;
  d.address = addr;
  d.vendor = kAmdVendorId;
  d.class_code = c.substr(0, 4);
  d.device = have_device ? device : dir.read_trimmed("device").value_or("");
  if (auto t = dir.read_trimmed("sriov_totalvfs")) d.sriov_totalvfs = static_cast<int>(str::parse_uint(*t).value_or(0));
  if (d.sriov_totalvfs == 0) {
    d.sriov_numvfs = 0;  // SR-IOV capable in name only
  } else if (d.sriov_totalvfs > 0 && dir.lookup("virtfn0") == ENOENT) {
    // The kernel links every VF it enables as virtfn<N> (the check below
    // relies on it too): no link, no VFs - a lookup instead of a
    // sriov_numvfs read, whose show() waits for the device lock.
    d.sriov_numvfs = 0;
  } else if (d.sriov_totalvfs > 0) {
    if (auto n = dir.read_trimmed("sriov_numvfs")) d.sriov_numvfs = static_cast<int>(str::parse_uint(*n).value_or(0));
    if (d.sriov_numvfs > 0) d.sriov_vf_device = dir.read_trimmed("sriov_vf_device").value_or("");
  }
  if (!physfn.empty()) {
    d.physfn = physfn;
  } else if (d.sriov_totalvfs < 0) {
    // Only a function without an SR-IOV capability of its own can be a VF
    // (a PF's VFs have none; every PF that has one publishes sriov_totalvfs).
    std::string link = dir.read_link("physfn");
    if (!link.empty()) d.physfn = fs::basename(link);
  }
  // Configuration space only where sysfs publishes no SR-IOV state.
  if (d.sriov_totalvfs < 0 && d.physfn.empty()) {
    auto cfg = dir.read_attr("config", kPciExpressConfigSpaceSize);
    if (!cfg.ok()) throw Error("unable to read PCI configuration space for " + addr + ": " + fs::errno_str(cfg.err));
    d.config = std::move(cfg.data);
  }
  if (d.sriov_totalvfs > 0) *keep = std::move(owned);
  return d;
}

}  // namespace

const std::vector<std::string>& BoundAmdPCI::drivers() {
  // amdgpu (bare metal, a passthrough or SR-IOV guest), gim (an MxGPU
  // host's PFs), and what hands a GPU to a VM or enables VFs without a GPU
  // driver: vfio-pci, pci-pf-stub, pci-stub.  No other in-tree driver's ID
  // table names an AMD GPU function.
  static const std::vector<std::string> names{"amdgpu", "gim", "vfio-pci", "pci-pf-stub", "pci-stub"};
  return names;
}

std::vector<PCIDevice> BoundAmdPCI::scan_bound(const std::vector<std::string>& bound_only,
                                               const std::vector<std::string>& unbound,
                                               std::map<std::string, std::unique_ptr<fs::Dir>>* pf_dirs) {
  // The unbound functions are read like the bound ones: a VF among them
  // finds its PF through its physfn link, as the whole-bus scan does.
  std::vector<std::string> bound = bound_only;
  bound.insert(bound.end(), unbound.begin(), unbound.end());
  std::string devices = fs::join(root_, kPciDevicesRoot);
  // Two functions per lane - the 8 GPUs of an MI355X host are ~40 small
  // reads, 0.23 ms on one cold thread - but only on workers already parked:
  // in a oneshot Job, creating threads for them made the scan slower (0.39
  // ms), and it is overlapped with enumeration anyway.
  constexpr size_t kChunk = 2;
  std::vector<std::optional<PCIDevice>> found(bound.size());
  std::vector<std::unique_ptr<fs::Dir>> dirs;
  // The old directories stay open until the new ones are: a re-read never
  // dips below the descriptors a steady daemon holds.
  std::map<std::string, std::unique_ptr<fs::Dir>> fresh;
  auto read_all = [&](const std::vector<std::string>& addrs, const std::vector<std::string>& pfs) {
    size_t chunks = (addrs.size() + kChunk - 1) / kChunk;
    found.assign(addrs.size(), std::nullopt);
    dirs.clear();
    dirs.resize(addrs.size());
    WorkerPool::instance().parallel_for(
        chunks,
        [&](size_t c) {
          for (size_t i = c * kChunk; i < std::min(addrs.size(), (c + 1) * kChunk); ++i)
            found[i] = read_function(fs::join(devices, addrs[i]), addrs[i], pfs.empty() ? "" : pfs[i], &dirs[i]);
        },
        1 + WorkerPool::instance().idle_workers());
    for (size_t i = 0; i < addrs.size(); ++i)
      if (dirs[i]) fresh[addrs[i]] = std::move(dirs[i]);
  };
  read_all(bound, {});
  std::vector<PCIDevice> out;
  std::set<std::string> seen(bound.begin(), bound.end());
  std::vector<std::string> vfs, vf_pfs;  // VF addresses and their PFs
  for (size_t i = 0; i < bound.size(); ++i) {
    if (!found[i]) continue;
    if (found[i]->sriov_numvfs > 0) {
      // The PF's enabled VFs, bound to whatever hands them to VMs (or
      // nothing): "virtfn0" -> "../0000:d9:00.1".
      for (const auto& e : fs::list_dir(found[i]->path)) {
        if (e.rfind("virtfn", 0) != 0) continue;
        std::string vf = fs::basename(fs::read_link(fs::join(found[i]->path, e)));
        if (is_pci_address(vf) && seen.insert(vf).second) {
          vfs.push_back(vf);
          vf_pfs.push_back(bound[i]);
        }
      }
    }
    out.push_back(std::move(*found[i]));
  }
  if (!vfs.empty()) {
    read_all(vfs, vf_pfs);
    for (auto& d : found)
      if (d) out.push_back(std::move(*d));
  }
  std::sort(out.begin(), out.end(), [](const PCIDevice& a, const PCIDevice& b) { return a.address < b.address; });
  pf_dirs->swap(fresh);
  return out;
}

std::vector<std::pair<std::string, uint64_t>> BoundAmdPCI::list_bound() {
  std::vector<std::pair<std::string, uint64_t>> bound;
  // Which of the listed drivers are loaded (a driver that is not has no
  // directory, and nothing is bound to it): one listing of the PCI drivers
  // through a kept descriptor, instead of a failing open - a whole path walk,
  // ~10-15 us after an idle second - per absent driver.
  bool loaded_changed = true;
  if (drivers_.read(fs::join(root_, "sys/bus/pci/drivers"), &loaded_changed) != 0) {
    loaded_.fill(true);  // unreadable: try every driver directory
  } else if (loaded_changed) {
    auto names = drivers_.entries();
    for (size_t i = 0; i < loaded_.size(); ++i)
      loaded_[i] = std::any_of(names.begin(), names.end(), [&](const auto& e) { return e.first == drivers()[i]; });
  }
  for (size_t i = 0; i < listings_.size(); ++i) {
    bool changed = false;
    if (!loaded_[i]) continue;
    if (listings_[i].read(fs::join(root_, "sys/bus/pci/drivers/" + drivers()[i]), &changed) != 0) continue;
    for (auto& e : listings_[i].entries())
      if (is_pci_address(e.first)) bound.push_back(std::move(e));
  }
  std::sort(bound.begin(), bound.end());
  bound.erase(std::unique(bound.begin(), bound.end(),
                          [](const auto& a, const auto& b) { return a.first == b.first; }),
              bound.end());
  return bound;
}

std::vector<std::string> BoundAmdPCI::list_unbound(const std::vector<std::pair<std::string, uint64_t>>& bound) {
  std::vector<std::string> out;
  if (!fallback_ || !merge_unbound_) return out;
  int64_t t0 = trace::stamp();
  auto amd = fallback_->amd_functions();  // sorted, like `bound`
  auto b = bound.begin();
  for (auto& addr : amd) {
    while (b != bound.end() && b->first < addr) ++b;
    if (b == bound.end() || b->first != addr) out.push_back(std::move(addr));
  }
  trace::record_since("pci.bus", t0);
  return out;
}

bool BoundAmdPCI::still_valid(const std::vector<std::pair<std::string, uint64_t>>& bound,
                              const std::vector<std::string>& unbound) {
  if (!have_ || fell_back_ || bound != bound_ || unbound != unbound_) return false;
  // With the bus merged in (a VM), every AMD function - a VF included,
  // bound or not - is in `bound` or `unbound`: a VF enabled or removed
  // changed one of the two listings.  Without it (a host), the PFs' VF
  // links are the check.
  if (fallback_ && merge_unbound_) return true;
  for (const auto& d : last_) {
    if (d.sriov_totalvfs <= 0) continue;
    // The kernel links every VF it creates as <pf>/virtfn<N> and removes the
    // links with the VFs, so the links are the PF's NumVFs: a lookup in the
    // directory the scan opened instead of a sriov_numvfs read (whose show()
    // also takes the device lock).  8 PFs: 0.019 ms vs 0.028-0.030 ms, and
    // no first check that opens 8 attribute files, 0.14-0.17 ms
    // (profiles/sriov_check_r4.txt).
    if (d.sriov_numvfs <= 0) {
      // No VFs: one lookup, through the PF's directory the scan opened.
      auto& dir = pf_dirs_[d.address];
      if (!dir) dir = std::make_unique<fs::Dir>(d.path);
      if (dir->err() != 0 || dir->lookup("virtfn0") != ENOENT) return false;  // (a PF gone: re-read)
      continue;
    }
    // VFs: the same links to the same functions (a VF removed on its own
    // with `remove` leaves NumVFs as it was).
    std::vector<std::string> now, kept;
    for (const auto& e : fs::list_dir(d.path))
      if (e.rfind("virtfn", 0) == 0) now.push_back(fs::basename(fs::read_link(fs::join(d.path, e))));
    for (const auto& v : last_)
      if (v.physfn == d.address) kept.push_back(v.address);
    std::sort(now.begin(), now.end());
    std::sort(kept.begin(), kept.end());
    if (now != kept) return false;
  }
  return true;
}

std::vector<PCIDevice> BoundAmdPCI::Devices() {
  refresh();
  return fell_back_ && fallback_ ? fallback_->Devices() : last_;
}

bool BoundAmdPCI::DevicesIfChanged(std::vector<PCIDevice>* out) {
  bool changed = refresh();
  if (fell_back_ && fallback_) {
    *out = fallback_->Devices();
    return true;
  }
  if (changed) *out = last_;
  return changed;
}

bool BoundAmdPCI::refresh() {
  int64_t t0 = trace::stamp();
  // A booted kernel has sent thousands of uevents; "" or "0" is an emulated
  // sysfs that never counts, and is not trusted.
  std::optional<std::string> seqnum;
  if (std::string s; seqnum_attr_.read(&s) && !s.empty() && s != "0") seqnum = std::move(s);
  if (have_ && seqnum && *seqnum == seqnum_) {
    trace::record_since("pci.bound(kept)", t0);
    return fell_back_;
  }
  auto bound = list_bound();
  // Whatever the bus holds that the listed drivers do not bind (empty when
  // nothing is bound: the bus scan below is the whole answer then).
  std::vector<std::string> unbound = bound.empty() ? std::vector<std::string>{} : list_unbound(bound);
  int64_t t_list = trace::stamp();
  if (seqnum && still_valid(bound, unbound)) {
    // The counter moved for some other device (a container's veth...).
    seqnum_ = *seqnum;
    int64_t t_end = trace::stamp();
    trace::record("pci.list", t_list - t0);
    trace::record("pci.vfs", t_end - t_list);
    trace::record("pci.bound(checked)", t_end - t0);
    return false;
  }
  trace::record_since("pci.drivers", t0);
  if (bound.empty()) {
    // Nothing bound: a guest whose amdgpu is not loaded still shows its VF
    // on the bus (the caller asks the fallback scan).
    fell_back_ = true;
    last_.clear();
    pf_dirs_.clear();
  } else {
    int64_t t1 = trace::stamp();
    std::vector<std::string> names;
    for (const auto& e : bound) names.push_back(e.first);
    last_ = scan_bound(names, unbound, &pf_dirs_);
    trace::record_since("pci.bound", t1);
    fell_back_ = false;
  }
  have_ = true;
  bound_ = std::move(bound);
  unbound_ = std::move(unbound);
  seqnum_ = seqnum.value_or("");
  return true;
}

}  // namespace gfd::sriov
