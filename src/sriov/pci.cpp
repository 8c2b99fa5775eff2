#include "sriov/pci.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string_view>
#include <unordered_map>
#include <unordered_set>

#include "util/error.h"
#include "util/fs.h"
#include "util/pool.h"
#include "util/trace.h"
#include "util/strings.h"

namespace gfd::sriov {

uint8_t GetByte(const std::string& buf, size_t pos) { return static_cast<uint8_t>(buf.at(pos)); }

uint16_t GetWord(const std::string& buf, size_t pos) {
  return static_cast<uint16_t>(GetByte(buf, pos) | (GetByte(buf, pos + 1) << 8));
}

uint32_t GetLong(const std::string& buf, size_t pos) {
  return static_cast<uint32_t>(GetByte(buf, pos)) | (static_cast<uint32_t>(GetByte(buf, pos + 1)) << 8) |
         (static_cast<uint32_t>(GetByte(buf, pos + 2)) << 16) | (static_cast<uint32_t>(GetByte(buf, pos + 3)) << 24);
}

std::optional<std::string> PCIDevice::GetCapability(int cap_id) const {
  if (config.size() < kPciConfigSpaceSize)
    throw Error("entire PCI configuration is not read for device " + address +
                ". Please run GFD with privileged mode to read complete PCI configuration data");
  if ((GetByte(config, kPciStatusByte) & kPciStatusCapabilityList) == 0) return std::nullopt;
  bool visited[256] = {false};
  int pos = GetByte(config, kPciCapabilityList) & 0xFC;
  while (pos != 0) {
    if (pos + kPciCapabilityLength >= static_cast<int>(kPciConfigSpaceSize)) break;  // malformed pointer
    int id = GetByte(config, static_cast<size_t>(pos + kPciCapabilityListId));
    int next = GetByte(config, static_cast<size_t>(pos + kPciCapabilityListNext)) & 0xFC;
    if (visited[pos]) break;  // chain looped
    if (id == 0xff) break;    // chain broken
    if (id == cap_id) {
      // Vendor-specific capabilities carry their length in byte 2; others
      // are returned as header + following bytes up to the next capability.
      size_t len = id == kPciCapabilityVendorSpecificId ? GetByte(config, static_cast<size_t>(pos + kPciCapabilityLength))
                                                        : 2;
      if (len < 2) len = 2;
      if (static_cast<size_t>(pos) + len > config.size()) len = config.size() - static_cast<size_t>(pos);
      return config.substr(static_cast<size_t>(pos), len);
    }
    visited[pos] = true;
    pos = next;
  }
  return std::nullopt;
}

std::optional<std::string> PCIDevice::GetExtendedCapability(int ext_id, size_t length) const {
  if (config.size() < kPciExpressConfigSpaceSize)
    throw Error("PCIe extended configuration space is not readable for device " + address +
                " (" + std::to_string(config.size()) + " bytes); run privileged to read it");
  bool visited[kPciExpressConfigSpaceSize / 4] = {false};
  size_t pos = kPciExtendedCapabilityStart;
  while (pos != 0 && pos + 4 <= config.size()) {
    uint32_t header = GetLong(config, pos);
    if (header == 0 || header == 0xFFFFFFFFu) break;
    if (visited[pos / 4]) break;
    visited[pos / 4] = true;
    int id = static_cast<int>(header & 0xFFFF);
    size_t next = (header >> 20) & 0xFFC;
    if (id == ext_id) {
      size_t len = std::min(length, config.size() - pos);
      return config.substr(pos, len);
    }
    if (next != 0 && next < kPciExtendedCapabilityStart) break;  // malformed
    pos = next;
  }
  return std::nullopt;
}

namespace {

// Vendor and device ID (vendor << 16 | device) of every PCI function from
// procfs' one-file device table
// (/proc/bus/pci/devices: one "BBDF\tVVVVDDDD\t..." line per function, BBDF =
// bus << 8 | devfn, all hex).  One read instead of one `vendor` file per
// function - 367 files on an 8-GPU MI355X host.  The table has no PCI
// domain, so a bus/devfn listed twice is dropped (those functions are read
// from sysfs).  Empty when the table cannot be read.
struct ProcFunction {
  uint32_t id = 0;    // vendor << 16 | device
  bool port = false;  // bound to pcieport: a PCIe port (bridge), never a GPU
};

std::unordered_map<uint32_t, ProcFunction> proc_pci_functions(const std::string& root) {
  std::unordered_map<uint32_t, ProcFunction> out;
  auto r = fs::read_file(fs::join(root, "proc/bus/pci/devices"), 4u << 20);
  if (!r.ok()) return out;
  std::unordered_set<uint32_t> dup;
  const char* p = r.data.c_str();
  const char* end = p + r.data.size();
  // The kernel's line (drivers/pci/proc.c, show_device): bus/devfn,
  // vendor/device, irq, 7 resource starts, 7 sizes, then the bound driver's
  // name (empty if none) - 18 tab-separated fields.
  constexpr int kDriverField = 17;
  while (p < end) {
    const char* eol = static_cast<const char*>(std::memchr(p, '\n', static_cast<size_t>(end - p)));
    if (!eol) eol = end;
    char* q = nullptr;
    unsigned long bbdf = std::strtoul(p, &q, 16);
    if (q && q < eol && *q == '\t') {
      char* q2 = nullptr;
      unsigned long id = std::strtoul(q + 1, &q2, 16);
      if (q2 && q2 > q + 1 && q2 <= eol) {
        ProcFunction f;
        f.id = static_cast<uint32_t>(id);
        int tabs = 0;
        const char* last = p;
        for (const char* c = p; c < eol; ++c)
          if (*c == '\t') {
            ++tabs;
            last = c + 1;
          }
        f.port = tabs == kDriverField && std::string_view(last, static_cast<size_t>(eol - last)) == "pcieport";
        auto key = static_cast<uint32_t>(bbdf & 0xffff);
        if (!out.emplace(key, f).second) dup.insert(key);
      }
    }
    p = eol + 1;
  }
  for (auto k : dup) out.erase(k);
  return out;
}

// "DDDD:BB:DD.F" (sysfs' PCI device names; the domain may be longer) ->
// bus << 8 | dev << 3 | fn.  Hand-parsed: sscanf cost ~0.2 us per name,
// 70 us for the ~350 names a cold scan looks up.
std::optional<uint32_t> bus_devfn(const std::string& addr) {
  auto hex = [](char c) -> int {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  };
  // The fixed-width tail ":BB:DD.F" after a domain of 4+ hex digits.
  size_t n = addr.size();
  if (n < 12) return std::nullopt;
  const char* t = addr.c_str() + n - 8;
  for (size_t i = 0; i + 8 < n; ++i)
    if (hex(addr[i]) < 0) return std::nullopt;
  int b1 = hex(t[1]), b0 = hex(t[2]), d1 = hex(t[4]), d0 = hex(t[5]), f = hex(t[7]);
  if (t[0] != ':' || t[3] != ':' || t[6] != '.' || b1 < 0 || b0 < 0 || d1 < 0 || d0 < 0 || f < 0) return std::nullopt;
  unsigned bus = static_cast<unsigned>(b1 << 4 | b0), dev = static_cast<unsigned>(d1 << 4 | d0);
  if (dev > 0x1f || f > 7) return std::nullopt;
  return static_cast<uint32_t>((bus << 8) | (dev << 3) | static_cast<unsigned>(f));
}

}  // namespace

SysfsAmdPCI::Identity SysfsAmdPCI::read_identity(const std::string& addr, const std::string& p, uint64_t ino,
                                                 uint32_t device_id, bool amd) {
  Identity id;
  id.ino = ino;
  if (device_id == 0 && !amd) {
    auto vendor = fs::read_file(fs::join(p, "vendor"), 64);
    if (!vendor.ok()) throw Error("unable to read PCI device vendor id for " + addr + ": " + fs::errno_str(vendor.err));
    if (str::trim(vendor.data) != kAmdVendorId) return id;
  }
  auto cls = fs::read_file(fs::join(p, "class"), 64);
  if (!cls.ok()) throw Error("unable to read PCI device class for " + addr + ": " + fs::errno_str(cls.err));
  std::string c = str::trim(cls.data);
  // Display controllers (0x03xxxx) and processing accelerators (0x12xxxx).
  if (!str::starts_with(c, "0x03") && !str::starts_with(c, "0x12")) return id;
  id.relevant = true;
  id.class_code = c.substr(0, 4);
  id.device = device_id ? str::format("0x%04x", device_id) : fs::read_trimmed(fs::join(p, "device")).value_or("");
  if (auto t = fs::read_trimmed(fs::join(p, "sriov_totalvfs")))
    id.sriov_totalvfs = static_cast<int>(str::parse_uint(*t).value_or(0));
  if (id.sriov_totalvfs > 0) id.sriov_vf_device = fs::read_trimmed(fs::join(p, "sriov_vf_device")).value_or("");
  std::string link = fs::read_link(fs::join(p, "physfn"));
  if (!link.empty()) id.physfn = fs::basename(link);
  return id;
}

std::vector<PCIDevice> SysfsAmdPCI::Devices() {
  std::string dir = fs::join(root_, kPciDevicesRoot);
  int64_t t0 = trace::now_ns();
  // The kernel's uevent sequence number goes up with every device added to
  // or removed from the system - a PCI function, an SR-IOV VF included
  // (device_add / device_del -> kobject_uevent; PCI devices pass the devices
  // kset's uevent filter).  Read before the listing, so an event racing with
  // this scan shows up as a new number next time.  Unchanged since the last
  // scan: the bus listing is unchanged too, and is not read.
  // A booted kernel has sent thousands of uevents; "0" would be an emulated
  // sysfs that never counts, and is not trusted.
  auto seqnum = fs::attrs().read_trimmed(fs::join(root_, "sys/kernel/uevent_seqnum"));
  if (seqnum && (seqnum->empty() || *seqnum == "0")) seqnum.reset();
  bool changed = true;
  if (seqnum && *seqnum == seqnum_ && scanned_) {
    changed = false;
  } else {
    int err = listing_.read(dir, &changed);
    if (err != 0) throw Error("unable to read PCI bus devices: open " + dir + ": " + fs::errno_str(err));
  }
  trace::record("pci.list", trace::now_ns() - t0);

  // Merge the (sorted) listing with the (sorted) identity cache: entries
  // whose sysfs inode is unchanged reuse their identity, new or re-created
  // ones are read.  Skipped entirely when the bus listing is unchanged.
  std::vector<std::pair<std::string, Identity>> next;
  std::vector<size_t> misses;
  if (changed) {
    auto entries = listing_.entries();
    next.reserve(entries.size());
    auto hit = cache_.begin();
    for (auto& [addr, ino] : entries) {
      while (hit != cache_.end() && hit->first < addr) ++hit;
      if (hit != cache_.end() && hit->first == addr && hit->second.ino == ino && ino != 0) {
        // Copied, not moved: if an identity read below fails, cache_ must
        // still be intact for the next scan.
        next.emplace_back(std::move(addr), hit->second);
        next.back().second.sriov_numvfs = -1;  // re-read below
      } else {
        misses.push_back(next.size());
        Identity fresh;
        fresh.ino = ino;
        next.emplace_back(std::move(addr), std::move(fresh));
      }
    }
  }
  // Identity reads (vendor, class, ...) of functions not seen before: every
  // function on the first scan (~5 us each, 2 ms for 367 functions on an
  // 8-GPU host) - the whole cost of a oneshot Job's scan.  A cold scan first
  // takes the vendor IDs of all functions from procfs' device table and
  // reads sysfs only for AMD functions (and any the table cannot place); the
  // remaining reads are spread over the worker pool in chunks.  A hot-plugged
  // function or two is read inline.
  constexpr size_t kChunk = 16;
  size_t chunk = kChunk;
  std::vector<uint32_t> known_device;  // aligned with misses: device ID from procfs, 0 = unknown
  // Functions bound to amdgpu (AMD's: its ID table names vendor 0x1002 only)
  // in a cold scan: their identity reads start on the pool at once and run
  // while this thread reads the procfs table (0.5-0.65 ms on a 367-function
  // host: the kernel restarts its device walk for every page it hands out),
  // which then only has to name the other AMD functions (none on the pool's
  // hosts once the PCIe ports are skipped).
  std::vector<size_t> early;
  WorkerPool::Task early_task;
  struct EarlyGuard {  // the task reads `next`: it must be done before it goes
    WorkerPool::Task* t;
    bool armed = false;
    ~EarlyGuard() {
      if (armed) t->cancel_or_wait();
    }
  } early_guard{&early_task};
  if (misses.size() > kChunk) {
    int64_t tp = trace::now_ns();
    std::vector<char> miss(next.size(), 0);
    for (size_t m : misses) miss[m] = 1;
    for (const auto& name : fs::list_dir(fs::join(root_, "sys/bus/pci/drivers/amdgpu"))) {
      if (!bus_devfn(name)) continue;  // bind, unbind, module, ...
      auto it = std::lower_bound(next.begin(), next.end(), name,
                                 [](const std::pair<std::string, Identity>& e, const std::string& n) { return e.first < n; });
      size_t i = static_cast<size_t>(it - next.begin());
      if (it != next.end() && it->first == name && miss[i]) {
        early.push_back(i);
        miss[i] = 0;
      }
    }
    if (!early.empty()) {
      misses.erase(std::remove_if(misses.begin(), misses.end(), [&](size_t m) { return !miss[m]; }), misses.end());
      early_task = WorkerPool::instance().submit([&] {
        constexpr size_t kEarlyChunk = 2;
        WorkerPool::instance().parallel_for((early.size() + kEarlyChunk - 1) / kEarlyChunk, [&](size_t c) {
          for (size_t k = c * kEarlyChunk; k < std::min(early.size(), (c + 1) * kEarlyChunk); ++k) {
            auto& [addr, id] = next[early[k]];
            id = read_identity(addr, fs::join(dir, addr), id.ino, 0, true);
          }
        });
      });
      early_guard.armed = true;
    }
    trace::record("pci.amdgpu", trace::now_ns() - tp);
    tp = trace::now_ns();
    auto table = proc_pci_functions(root_);
    trace::record("pci.proc_table", trace::now_ns() - tp);
    if (!table.empty()) {
      uint32_t amd = static_cast<uint32_t>(std::strtoul(kAmdVendorId, nullptr, 16));
      std::vector<size_t> amd_or_unknown;
      for (size_t m : misses) {
        auto key = bus_devfn(next[m].first);
        auto v = key ? table.find(*key) : table.end();
        if (v == table.end()) {
          amd_or_unknown.push_back(m);
          known_device.push_back(0);
        } else if ((v->second.id >> 16) == amd && (v->second.id & 0xffff) != 0 && !v->second.port) {
          amd_or_unknown.push_back(m);
          known_device.push_back(v->second.id & 0xffff);
        }
        // else: another vendor's function, or an AMD PCIe port (the switch
        // ports next to every MI355X: half the host's AMD functions) -
        // identity stays "not relevant"
      }
      misses.swap(amd_or_unknown);
      // A few functions per lane (~2-4 reads each now that vendor and device
      // come from the table).  Lane count does not matter on the pool's
      // 16-AMD-function hosts: 1, 2, 4, 8 or all 16 per lane gave the same
      // Job process within 0.04 ms (profiles/pci_cold_ab.txt).
      chunk = 2;
    }
  }
  auto read_chunk = [&](size_t c) {
    for (size_t k = c * chunk; k < std::min(misses.size(), (c + 1) * chunk); ++k) {
      auto& [addr, id] = next[misses[k]];
      id = read_identity(addr, fs::join(dir, addr), id.ino, k < known_device.size() ? known_device[k] : 0);
    }
  };
  size_t chunks = (misses.size() + chunk - 1) / chunk;
  try {
    if (chunks > 1)
      WorkerPool::instance().parallel_for(chunks, read_chunk);
    else if (chunks == 1)
      read_chunk(0);
    if (early_guard.armed) {
      early_guard.armed = false;
      early_task.run_or_wait();
    }
  } catch (...) {
    listing_.reset();  // the next scan must see this listing as changed again
    throw;
  }
  if (changed) cache_.swap(next);
  scanned_ = true;
  seqnum_ = seqnum.value_or("");
  int64_t t1 = trace::now_ns();
  trace::record("pci.identity", t1 - t0);

  std::vector<PCIDevice> out;
  std::vector<Identity*> ids;
  for (auto& [addr, id] : cache_) {
    if (!id.relevant) continue;
    PCIDevice d;
    d.path = fs::join(dir, addr);
    d.address = addr;
    d.vendor = kAmdVendorId;
    d.class_code = id.class_code;
    d.device = id.device;
    d.sriov_totalvfs = id.sriov_totalvfs;
    d.sriov_vf_device = id.sriov_vf_device;  // cleared below unless VFs are enabled
    d.physfn = id.physfn;
    out.push_back(std::move(d));
    ids.push_back(&id);
  }

  // Mutable state: NumVFs of SR-IOV capable functions (one ~3 us sysfs read
  // each), and the raw configuration space of functions whose SR-IOV state
  // sysfs does not publish.  Serial on purpose: spreading the 8 reads of an
  // 8-GPU host over the pool measured 40-56 us vs 26 us serial (worker
  // wake-up costs more than the reads).
  //
  // NumVFs is re-read only when the bus listing changed: the kernel creates
  // (and removes) one PCI function per VF when NumVFs is written, and refuses
  // to change a non-zero NumVFs to another non-zero value without going
  // through 0 (drivers/pci/iov.c, sriov_numvfs_store: -EBUSY), so NumVFs
  // cannot change while the listing - names and inode numbers - stays the same.
  auto refresh = [&](size_t i) {
    PCIDevice& d = out[i];
    Identity& id = *ids[i];
    if (d.sriov_totalvfs == 0) {
      d.sriov_numvfs = 0;  // SR-IOV capable in name only: no VFs possible
    } else if (d.sriov_totalvfs > 0) {
      if (id.sriov_numvfs < 0)
        if (auto n = fs::read_trimmed(fs::join(d.path, "sriov_numvfs")))
          id.sriov_numvfs = static_cast<int>(str::parse_uint(*n).value_or(0));
      d.sriov_numvfs = id.sriov_numvfs;
    }
    if (d.sriov_numvfs <= 0) d.sriov_vf_device.clear();
    if (d.sriov_totalvfs < 0 && d.physfn.empty()) {
      auto cfg = fs::read_file(fs::join(d.path, "config"), kPciExpressConfigSpaceSize);
      if (!cfg.ok()) throw Error("unable to read PCI configuration space for " + d.address + ": " + fs::errno_str(cfg.err));
      d.config = std::move(cfg.data);
    }
  };
  int64_t t2 = trace::now_ns();
  trace::record("pci.build", t2 - t1);
  for (size_t i = 0; i < out.size(); ++i) refresh(i);
  trace::record("pci.refresh", trace::now_ns() - t2);
  return out;
}

// ---------------------------------------------------------------------------
// Mock configuration spaces

namespace {

void put16(std::string& b, size_t pos, uint16_t v) {
  b[pos] = static_cast<char>(v & 0xff);
  b[pos + 1] = static_cast<char>(v >> 8);
}
void put32(std::string& b, size_t pos, uint32_t v) {
  for (int i = 0; i < 4; ++i) b[pos + static_cast<size_t>(i)] = static_cast<char>((v >> (8 * i)) & 0xff);
}

// Type-0 header of an AMD processing accelerator with the capability chain
// PM(0x48) -> PCIe(0x64) -> MSI(0xa0) -> MSI-X(0xc0) and the extended chain
// AER(0x100) -> ARI(0x150) -> [SR-IOV(0x200)] -> VSEC(0x300).
std::string base_config(uint16_t device, bool with_sriov, uint16_t total_vfs, uint16_t num_vfs, uint16_t vf_device) {
  std::string b(kPciExpressConfigSpaceSize, '\0');
  put16(b, 0x00, 0x1002);
  put16(b, 0x02, device);
  put16(b, 0x04, 0x0407);
  put16(b, 0x06, 0x0010);  // capability list present
  b[0x0b] = 0x12;          // class: processing accelerator
  put16(b, 0x2c, 0x1002);
  put16(b, 0x2e, device);
  b[0x34] = 0x48;
  // PM
  b[0x48] = 0x01;
  b[0x49] = 0x64;
  put16(b, 0x4a, 0x0003);
  // PCI Express
  b[0x64] = 0x10;
  b[0x65] = static_cast<char>(0xa0);
  put16(b, 0x66, 0x0002);
  // MSI
  b[0xa0] = 0x05;
  b[0xa1] = static_cast<char>(0xc0);
  // MSI-X
  b[0xc0] = 0x11;
  b[0xc1] = 0x00;
  // Extended: AER @0x100 -> ARI @0x150 -> SR-IOV @0x200 -> VSEC @0x300
  uint16_t after_ari = with_sriov ? 0x200 : 0x300;
  put32(b, 0x100, 0x0001u | (1u << 16) | (0x150u << 20));
  put32(b, 0x150, 0x000Eu | (1u << 16) | (static_cast<uint32_t>(after_ari) << 20));
  if (with_sriov) {
    put32(b, 0x200, 0x0010u | (1u << 16) | (0x300u << 20));
    put16(b, 0x208, num_vfs ? 0x0001 : 0x0000);  // SR-IOV control: VF enable
    put16(b, 0x20c, total_vfs);                  // InitialVFs
    put16(b, 0x20e, total_vfs);                  // TotalVFs
    put16(b, 0x210, num_vfs);                    // NumVFs
    put16(b, 0x214, 1);                          // First VF offset
    put16(b, 0x216, 1);                          // VF stride
    put16(b, 0x21a, vf_device);                  // VF device ID
  }
  // AMD vendor-specific extended capability (VSEC) terminates the chain.
  put32(b, 0x300, 0x000Bu | (1u << 16) | (0u << 20));
  put32(b, 0x304, 0x1002u | (1u << 16) | (0x10u << 20));
  return b;
}

}  // namespace

std::string MockAmdPCI::passthrough_config() { return base_config(0x75a3, false, 0, 0, 0); }

std::string MockAmdPCI::pf_config(uint16_t total_vfs, uint16_t num_vfs, uint16_t vf_device) {
  return base_config(0x74a1, true, total_vfs, num_vfs, vf_device);
}

std::string MockAmdPCI::vf_config(uint16_t device) { return base_config(device, false, 0, 0, 0); }

MockAmdPCI::MockAmdPCI() {
  PCIDevice passthrough;
  passthrough.address = "passthrough";
  passthrough.vendor = kAmdVendorId;
  passthrough.device = "0x75a3";
  passthrough.class_code = "0x12";
  passthrough.config = passthrough_config();
  passthrough.sriov_totalvfs = 1;
  passthrough.sriov_numvfs = 0;

  PCIDevice pf;
  pf.address = "pf";
  pf.vendor = kAmdVendorId;
  pf.device = "0x74a1";
  pf.class_code = "0x12";
  pf.config = pf_config(8, 4, 0x74b5);
  pf.sriov_totalvfs = 8;
  pf.sriov_numvfs = 4;
  pf.sriov_vf_device = "0x74b5";

  PCIDevice vf;
  vf.address = "vf";
  vf.vendor = kAmdVendorId;
  vf.device = "0x74b5";
  vf.class_code = "0x12";
  vf.config = vf_config(0x74b5);
  vf.physfn = "pf";

  devices_ = {passthrough, pf, vf};
}

}  // namespace gfd::sriov
