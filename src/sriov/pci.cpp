#include "sriov/pci.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

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

SysfsAmdPCI::Identity SysfsAmdPCI::read_identity(const std::string& addr, const std::string& p, uint64_t ino) {
  Identity id;
  id.ino = ino;
  auto vendor = fs::read_file(fs::join(p, "vendor"), 64);
  if (!vendor.ok()) throw Error("unable to read PCI device vendor id for " + addr + ": " + fs::errno_str(vendor.err));
  if (str::trim(vendor.data) != kAmdVendorId) return id;
  auto cls = fs::read_file(fs::join(p, "class"), 64);
  if (!cls.ok()) throw Error("unable to read PCI device class for " + addr + ": " + fs::errno_str(cls.err));
  std::string c = str::trim(cls.data);
  // Display controllers (0x03xxxx) and processing accelerators (0x12xxxx).
  if (!str::starts_with(c, "0x03") && !str::starts_with(c, "0x12")) return id;
  id.relevant = true;
  id.class_code = c.substr(0, 4);
  id.device = fs::read_trimmed(fs::join(p, "device")).value_or("");
  if (auto t = fs::read_trimmed(fs::join(p, "sriov_totalvfs")))
    id.sriov_totalvfs = static_cast<int>(str::parse_uint(*t).value_or(0));
  if (id.sriov_totalvfs > 0) id.sriov_vf_device = fs::read_trimmed(fs::join(p, "sriov_vf_device")).value_or("");
  std::string link = fs::read_link(fs::join(p, "physfn"));
  if (!link.empty()) id.physfn = fs::basename(link);
  return id;
}

void SysfsAmdPCI::update() {
  std::string dir = fs::join(root_, kPciDevicesRoot);
  int64_t t0 = trace::stamp();
  // The kernel's uevent sequence number goes up with every device added to
  // or removed from the system - a PCI function, an SR-IOV VF included
  // (device_add / device_del -> kobject_uevent; PCI devices pass the devices
  // kset's uevent filter).  Read before the listing, so an event racing with
  // this scan shows up as a new number next time.  Unchanged since the last
  // scan: the bus listing is unchanged too, and is not read.
  // A booted kernel has sent thousands of uevents; "0" would be an emulated
  // sysfs that never counts, and is not trusted.
  std::optional<std::string> seqnum;
  if (std::string s; seqnum_attr_.read(&s) && !s.empty() && s != "0") seqnum = std::move(s);
  bool changed = true;
  if (seqnum && *seqnum == seqnum_ && scanned_) {
    changed = false;
  } else {
    int err = listing_.read(dir, &changed);
    if (err != 0) throw Error("unable to read PCI bus devices: open " + dir + ": " + fs::errno_str(err));
  }
  trace::record_since("pci.list", t0);

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
  // function on the first scan (~5 us each: 2 ms for the 367 functions of an
  // 8-GPU host), spread over the worker pool in chunks; a hot-plugged
  // function or two is read inline.  The driver-directed source
  // (sriov/bound.h) runs this whenever uevent_seqnum moved, for the AMD
  // functions no driver it lists binds; a daemon pays the first, full pass in
  // its start-up prefetch, and later passes read only the listing.
  constexpr size_t kChunk = 16;
  auto read_chunk = [&](size_t c) {
    for (size_t k = c * kChunk; k < std::min(misses.size(), (c + 1) * kChunk); ++k) {
      auto& [addr, id] = next[misses[k]];
      id = read_identity(addr, fs::join(dir, addr), id.ino);
    }
  };
  size_t chunks = (misses.size() + kChunk - 1) / kChunk;
  try {
    if (chunks > 1)
      WorkerPool::instance().parallel_for(chunks, read_chunk);
    else if (chunks == 1)
      read_chunk(0);
  } catch (...) {
    listing_.reset();  // the next scan must see this listing as changed again
    throw;
  }
  if (changed) cache_.swap(next);
  scanned_ = true;
  seqnum_ = seqnum.value_or("");
  trace::record_since("pci.identity", t0);
}

std::vector<std::string> SysfsAmdPCI::amd_functions() {
  update();
  std::vector<std::string> out;
  for (const auto& [addr, id] : cache_)
    if (id.relevant) out.push_back(addr);
  return out;
}

std::vector<PCIDevice> SysfsAmdPCI::Devices() {
  update();
  std::string dir = fs::join(root_, kPciDevicesRoot);
  int64_t t1 = trace::stamp();
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
  int64_t t2 = trace::stamp();
  trace::record("pci.build", t2 - t1);
  for (size_t i = 0; i < out.size(); ++i) refresh(i);
  trace::record_since("pci.refresh", t2);
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
