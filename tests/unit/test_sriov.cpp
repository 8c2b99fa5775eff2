// SR-IOV / PCI tests.  Ports of internal/vgpu/pciutil_test.go and
// vgpu_test.go (capability walk, device classification, info), adapted to
// PCIe SR-IOV.
#include "lm/labels.h"
#include "lm/node.h"
#include "sriov/bound.h"
#include "sriov/pci.h"
#include "sriov/sriov.h"
#include "test.h"
#include "util/fs.h"
#include "util/strings.h"

#include <algorithm>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>

using namespace gfd;
using namespace gfd::sriov;

namespace {
PCIDevice find(const std::string& addr) {
  for (auto& d : MockAmdPCI().Devices())
    if (d.address == addr) return d;
  throw std::runtime_error("no mock device " + addr);
}
}  // namespace

TEST(Pci_MockDevicesAreAmd) {
  for (const auto& d : MockAmdPCI().Devices()) {
    EXPECT_EQ(GetWord(d.config, 0), static_cast<uint16_t>(0x1002));
    EXPECT_EQ(d.config.size(), kPciExpressConfigSpaceSize);
  }
}

TEST(Pci_CapabilityWalkFindsExpressCapability) {
  for (const auto& d : MockAmdPCI().Devices()) {
    auto cap = d.GetCapability(kPciCapabilityExpressId);
    EXPECT_TRUE(cap.has_value());
    EXPECT_EQ(GetByte(*cap, 0), static_cast<uint8_t>(0x10));
    // No vendor-specific (0x09) capability on AMD functions.
    EXPECT_FALSE(d.GetVendorSpecificCapability().has_value());
  }
}

TEST(Pci_ReferenceConfigDumpsVendorCapability) {
  // internal/vgpu/pciutil_test.go:26-42 on the reference's own two
  // configuration-space dumps (tests/fixtures/pci/README.md): the generic
  // capability walk finds the vendor-specific capability with the lengths
  // the reference expects, and the vGPU one carries the 'VF' signature.
  struct Case {
    const char* file;
    size_t length;
  };
  for (const Case& c : {Case{"nvidia-passthrough.cfg", 20}, Case{"nvidia-vgpu.cfg", 27}}) {
    PCIDevice d;
    d.config = fs::read_file(std::string(GFD_SOURCE_DIR) + "/tests/fixtures/pci/" + c.file).data;
    EXPECT_EQ(d.config.size(), static_cast<size_t>(256));
    EXPECT_EQ(GetWord(d.config, 0), static_cast<uint16_t>(0x10de));
    auto cap = d.GetVendorSpecificCapability();
    EXPECT_TRUE(cap.has_value());
    EXPECT_EQ(cap->size(), c.length);
    EXPECT_EQ(cap->substr(3, 2) == "VF", std::string(c.file) == "nvidia-vgpu.cfg");
  }
}

TEST(Pci_CapabilityWalkRequiresFullConfig) {
  PCIDevice d = find("passthrough");
  d.config.resize(64);  // what an unprivileged reader sees
  EXPECT_THROW_MSG(d.GetCapability(kPciCapabilityExpressId), "Please run GFD with privileged mode");
  EXPECT_THROW_MSG(d.GetExtendedCapability(kPciExtCapSriovId, 0x40), "extended configuration space is not readable");
}

TEST(Pci_CapabilityWalkNoCapList) {
  PCIDevice d = find("passthrough");
  d.config[kPciStatusByte] = 0;
  EXPECT_FALSE(d.GetCapability(kPciCapabilityExpressId).has_value());
}

TEST(Pci_CapabilityWalkDetectsLoop) {
  PCIDevice d = find("passthrough");
  d.config[0xc1] = 0x48;  // MSI-X -> PM: loop; PCIe cap is still found first
  EXPECT_TRUE(d.GetCapability(kPciCapabilityExpressId).has_value());
  EXPECT_FALSE(d.GetCapability(0x42).has_value());  // terminates despite the loop
}

TEST(Pci_CapabilityWalkBrokenChain) {
  PCIDevice d = find("passthrough");
  d.config[0x64] = static_cast<char>(0xff);  // PCIe cap id 0xff: chain broken
  EXPECT_FALSE(d.GetCapability(kPciCapabilityExpressId).has_value());
}

TEST(Pci_ExtendedWalkFindsSriovOnPF) {
  PCIDevice pf = find("pf");
  auto cap = pf.GetExtendedCapability(kPciExtCapSriovId, 0x40);
  EXPECT_TRUE(cap.has_value());
  auto c = parse_sriov_capability(*cap);
  EXPECT_TRUE(c.has_value());
  EXPECT_EQ(c->total_vfs, static_cast<uint16_t>(8));
  EXPECT_EQ(c->num_vfs, static_cast<uint16_t>(4));
  EXPECT_EQ(c->vf_device_id, static_cast<uint16_t>(0x74b5));
  EXPECT_TRUE(c->vf_enable);
  EXPECT_FALSE(find("passthrough").GetExtendedCapability(kPciExtCapSriovId, 0x40).has_value());
  EXPECT_TRUE(find("passthrough").GetExtendedCapability(kPciExtCapVendorSpecificId, 0x10).has_value());
}

TEST(Pci_ExtendedWalkDetectsLoop) {
  PCIDevice d = find("passthrough");
  // AER next -> 0x100 (itself).
  uint32_t hdr = 0x0001u | (1u << 16) | (0x100u << 20);
  for (int i = 0; i < 4; ++i) d.config[0x100 + i] = static_cast<char>((hdr >> (8 * i)) & 0xff);
  EXPECT_FALSE(d.GetExtendedCapability(kPciExtCapSriovId, 0x40).has_value());
}

TEST(Sriov_Classify) {
  EXPECT_FALSE(Lib::Classify(find("passthrough")).has_value());
  auto pf = Lib::Classify(find("pf"));
  EXPECT_TRUE(pf.has_value());
  EXPECT_EQ(pf->role, std::string("pf"));
  EXPECT_EQ(pf->num_vfs, 4);
  EXPECT_EQ(pf->total_vfs, 8);
  EXPECT_EQ(pf->vf_device, std::string("0x74b5"));
  auto vf = Lib::Classify(find("vf"));
  EXPECT_TRUE(vf.has_value());
  EXPECT_EQ(vf->role, std::string("vf"));
  EXPECT_EQ(vf->physfn, std::string("pf"));
}

TEST(Sriov_ClassifyGuestVFByDeviceId) {
  PCIDevice d = find("passthrough");
  d.device = "0x74b5";
  auto i = Lib::Classify(d);
  EXPECT_TRUE(i.has_value());
  EXPECT_EQ(i->role, std::string("vf"));
}

TEST(Sriov_TruncatedConfigFallsBackToSysfs) {
  PCIDevice d = find("pf");
  d.config.resize(64);
  auto i = Lib::Classify(d);
  EXPECT_TRUE(i.has_value());
  EXPECT_EQ(i->role, std::string("pf"));
  EXPECT_EQ(i->num_vfs, 4);
  d.sriov_numvfs = 0;
  EXPECT_FALSE(Lib::Classify(d).has_value());
}

TEST(Sriov_PFWithVFsDisabledIsNotReported) {
  PCIDevice d = find("pf");
  d.sriov_numvfs = 0;
  EXPECT_FALSE(Lib::Classify(d).has_value());
  // Same through the configuration space when sysfs publishes nothing.
  d.sriov_totalvfs = d.sriov_numvfs = -1;
  d.config = MockAmdPCI::pf_config(8, 0, 0x74b5);
  EXPECT_FALSE(Lib::Classify(d).has_value());
}

TEST(Sriov_ConfigSpaceOnlyClassification) {
  PCIDevice d = find("pf");
  d.sriov_totalvfs = d.sriov_numvfs = -1;
  d.sriov_vf_device.clear();
  auto i = Lib::Classify(d);
  EXPECT_TRUE(i.has_value());
  EXPECT_EQ(i->role, std::string("pf"));
  EXPECT_EQ(i->total_vfs, 8);
  EXPECT_EQ(i->num_vfs, 4);
  EXPECT_EQ(i->vf_device, std::string("0x74b5"));
  // Truncated config and no sysfs attributes: nothing can be said.
  d.config.resize(64);
  EXPECT_FALSE(Lib::Classify(d).has_value());
}

TEST(Sriov_LabelerReportsPresenceAndRole) {
  auto labels = lm::NewSriovLabeler(new_mock_sriov())->GetLabels();
  EXPECT_EQ(labels["amd.com/sriov.present"], std::string("true"));
  // A PF with VFs enabled makes this an SR-IOV host.
  EXPECT_EQ(labels["amd.com/sriov.role"], std::string("pf"));
  EXPECT_EQ(labels["amd.com/sriov.num-vfs"], std::string("4"));
  EXPECT_EQ(labels["amd.com/sriov.total-vfs"], std::string("8"));
}

TEST(Sriov_LabelerGuestRole) {
  PCIDevice vf = find("passthrough");
  vf.device = "0x74b5";  // a VF as seen inside a guest (no physfn link)
  auto lib = std::make_shared<Lib>(std::make_shared<MockAmdPCI>(std::vector<PCIDevice>{vf}));
  auto labels = lm::NewSriovLabeler(lib)->GetLabels();
  EXPECT_EQ(labels, (lm::Labels{{"amd.com/sriov.present", "true"}, {"amd.com/sriov.role", "vf"}}));
}

TEST(Sriov_LabelerSumsVfsOverPFs) {
  PCIDevice a = find("pf"), b = find("pf");
  b.address = "pf2";
  b.sriov_numvfs = 2;
  auto lib = std::make_shared<Lib>(std::make_shared<MockAmdPCI>(std::vector<PCIDevice>{a, b}));
  auto labels = lm::NewSriovLabeler(lib)->GetLabels();
  EXPECT_EQ(labels["amd.com/sriov.num-vfs"], std::string("6"));
  EXPECT_EQ(labels["amd.com/sriov.total-vfs"], std::string("16"));
}

TEST(Sriov_LabelerEmptyWhenNoFunctions) {
  auto lib = std::make_shared<Lib>(std::make_shared<MockAmdPCI>(std::vector<PCIDevice>{find("passthrough")}));
  EXPECT_EQ(lm::NewSriovLabeler(lib)->GetLabels(), lm::Labels{});
}

namespace {
// A source that reports "unchanged" on demand, and counts full reads.
struct ScriptedPCI : AmdPCI {
  std::vector<PCIDevice> devices;
  bool changed = true;
  int full_reads = 0;
  std::vector<PCIDevice> Devices() override {
    ++full_reads;
    return devices;
  }
  bool DevicesIfChanged(std::vector<PCIDevice>* out) override {
    if (!changed) return false;
    *out = Devices();
    return true;
  }
};
}  // namespace

TEST(Sriov_LibClassifiesOnlyWhatTheSourceReadAgain) {
  auto src = std::make_shared<ScriptedPCI>();
  PCIDevice pf = find("pf");
  src->devices = {pf};
  Lib lib(src);
  EXPECT_EQ(lib.Devices().size(), static_cast<size_t>(1));
  EXPECT_EQ(src->full_reads, 1);
  // Kept by the source: the classified functions again, nothing copied.
  src->changed = false;
  src->devices.clear();  // (not looked at)
  for (int i = 0; i < 3; ++i) EXPECT_EQ(lib.Devices().size(), static_cast<size_t>(1));
  EXPECT_EQ(src->full_reads, 1);
  // Re-read by the source: classified anew.
  src->changed = true;
  EXPECT_EQ(lib.Devices().size(), static_cast<size_t>(0));
  EXPECT_EQ(src->full_reads, 2);
  // A Lib that never classified asks for the whole list even when the
  // source reports no change.
  src->changed = false;
  src->devices = {pf, pf};
  Lib fresh(src);
  EXPECT_EQ(fresh.Devices().size(), static_cast<size_t>(2));
  EXPECT_EQ(src->full_reads, 3);
}

TEST(Sriov_SysfsScanMissingRootErrors) {
  auto lib = new_sriov_lib("/nonexistent-gfd-root");
  EXPECT_THROW_MSG(lib->Devices(), "unable to read PCI bus devices");
}

namespace {
void put_file(const std::string& path, const std::string& content) {
  fs::mkdir_all(fs::dirname(path));
  FILE* f = std::fopen(path.c_str(), "w");
  if (!f) throw std::runtime_error("cannot write " + path);
  std::fputs(content.c_str(), f);
  std::fclose(f);
}

// A host with `filler` non-AMD functions, 4 MI355X PFs without VFs and one
// PF (0000:c1:00.0) with `vfs` VFs enabled.
std::string pci_host(int filler, int vfs) {
  char d[] = "/tmp/gfd-pci-XXXXXX";
  if (!mkdtemp(d)) throw std::runtime_error("mkdtemp");
  std::string dev = std::string(d) + "/sys/bus/pci/devices/";
  for (int i = 0; i < filler; ++i) {
    std::string p = dev + str::format("0000:%02x:%02x.%d", i / 32, i % 32, 0);
    put_file(p + "/vendor", "0x1022\n");
    put_file(p + "/class", "0x060000\n");
  }
  auto gpu = [&](const std::string& bdf, int total, int num) {
    put_file(dev + bdf + "/vendor", "0x1002\n");
    put_file(dev + bdf + "/class", "0x120000\n");
    put_file(dev + bdf + "/device", "0x75a3\n");
    put_file(dev + bdf + "/sriov_totalvfs", std::to_string(total) + "\n");
    put_file(dev + bdf + "/sriov_numvfs", std::to_string(num) + "\n");
    put_file(dev + bdf + "/sriov_vf_device", "0x75b3\n");
  };
  for (int g = 0; g < 4; ++g) gpu(str::format("0000:%02x:00.0", 0x11 + 0x10 * g), 1, 0);
  gpu("0000:c1:00.0", 8, vfs);
  for (int v = 0; v < vfs; ++v) {
    std::string p = dev + str::format("0000:c1:00.%d", v + 1);
    put_file(p + "/vendor", "0x1002\n");
    put_file(p + "/class", "0x120000\n");
    put_file(p + "/device", "0x75b3\n");
    if (symlink("../0000:c1:00.0", (p + "/physfn").c_str()) != 0) throw std::runtime_error("symlink");
  }
  return d;
}
}  // namespace

TEST(Sriov_SysfsScanColdParallelThenIncremental) {
  // 200 filler functions force the parallel cold-scan path (>16 misses).
  std::string root = pci_host(200, 2);
  SysfsAmdPCI pci(root);
  auto devs = pci.Devices();
  EXPECT_EQ(devs.size(), static_cast<size_t>(7));  // 4 PFs + 1 PF with 2 VFs
  int pfs_with_vfs = 0, vfs = 0;
  for (const auto& d : devs) {
    if (d.sriov_numvfs > 0) {
      ++pfs_with_vfs;
      EXPECT_EQ(d.address, std::string("0000:c1:00.0"));
      EXPECT_EQ(d.sriov_totalvfs, 8);
      EXPECT_EQ(d.sriov_vf_device, std::string("0x75b3"));
    }
    if (!d.physfn.empty()) {
      ++vfs;
      EXPECT_EQ(d.physfn, std::string("0000:c1:00.0"));
    }
    if (d.sriov_numvfs == 0) EXPECT_EQ(d.sriov_vf_device, std::string(""));
  }
  EXPECT_EQ(pfs_with_vfs, 1);
  EXPECT_EQ(vfs, 2);
  // NumVFs is re-read when the listing changes.  Enabling VFs is what changes
  // it: the kernel adds one PCI function per VF (and refuses N -> M without
  // going through 0), so a NumVFs write never leaves the listing unchanged.
  std::string dev = root + "/sys/bus/pci/devices/";
  put_file(dev + "0000:11:00.0/sriov_numvfs", "1\n");
  int on = 0;
  for (const auto& d : pci.Devices())
    if (d.address == "0000:11:00.0") on = d.sriov_numvfs;
  EXPECT_EQ(on, 0);  // same listing: the value of the previous scan stands
  put_file(dev + "0000:11:00.1/vendor", "0x1002\n");
  put_file(dev + "0000:11:00.1/class", "0x120000\n");
  put_file(dev + "0000:11:00.1/device", "0x75b3\n");
  if (symlink("../0000:11:00.0", (dev + "0000:11:00.1/physfn").c_str()) != 0) throw std::runtime_error("symlink");
  int vfs_of_11 = 0;
  for (const auto& d : pci.Devices()) {
    if (d.address == "0000:11:00.0") on = d.sriov_numvfs;
    if (d.physfn == "0000:11:00.0") ++vfs_of_11;
  }
  EXPECT_EQ(on, 1);
  EXPECT_EQ(vfs_of_11, 1);
  // A function removed and re-created (new sysfs inode) is re-identified.
  // (Parked elsewhere, not deleted, so this filesystem cannot hand the new
  // directory the old inode number - kernfs allocates them cyclically.)
  if (rename((root + "/sys/bus/pci/devices/0000:21:00.0").c_str(), (root + "/parked").c_str()) != 0)
    throw std::runtime_error("rename");
  put_file(root + "/sys/bus/pci/devices/0000:21:00.0/vendor", "0x8086\n");
  put_file(root + "/sys/bus/pci/devices/0000:21:00.0/class", "0x020000\n");
  bool still_there = false;
  for (const auto& d : pci.Devices()) still_there |= d.address == "0000:21:00.0";
  EXPECT_FALSE(still_there);
  // Errors from the parallel cold scan surface like serial ones.
  SysfsAmdPCI cold(root);
  fs::remove_all(root + "/sys/bus/pci/devices/0000:00:05.0/vendor");
  fs::mkdir_all(root + "/sys/bus/pci/devices/0000:00:05.0/vendor");  // unreadable attribute
  EXPECT_THROW_MSG(cold.Devices(), "unable to read PCI device vendor id for 0000:00:05.0");
  fs::remove_all(root);
}

TEST(Fs_DirListingReportsChangesAndSurvivesRecreation) {
  char d[] = "/tmp/gfd-dirlist-XXXXXX";
  if (!mkdtemp(d)) throw std::runtime_error("mkdtemp");
  std::string dir = std::string(d) + "/devices";
  put_file(dir + "/0000:01:00.0/vendor", "0x1002\n");
  put_file(dir + "/0000:02:00.0/vendor", "0x1002\n");
  fs::DirListing l;
  bool changed = false;
  EXPECT_EQ(l.read(dir, &changed), 0);
  EXPECT_TRUE(changed);  // first read
  auto e = l.entries();
  EXPECT_EQ(e.size(), static_cast<size_t>(2));
  EXPECT_EQ(e[0].first, std::string("0000:01:00.0"));
  EXPECT_EQ(e[1].first, std::string("0000:02:00.0"));
  EXPECT_TRUE(e[0].second != 0 && e[0].second != e[1].second);
  EXPECT_EQ(l.read(dir, &changed), 0);
  EXPECT_FALSE(changed);
  put_file(dir + "/0000:00:01.0/vendor", "0x1022\n");
  EXPECT_EQ(l.read(dir, &changed), 0);
  EXPECT_TRUE(changed);
  EXPECT_EQ(l.entries().front().first, std::string("0000:00:01.0"));
  // The directory removed and created again: the open descriptor is stale
  // and the listing looks the path up again.
  fs::remove_all(dir);
  put_file(dir + "/0000:03:00.0/vendor", "0x1002\n");
  EXPECT_EQ(l.read(dir, &changed), 0);
  EXPECT_TRUE(changed);
  EXPECT_EQ(l.entries().size(), static_cast<size_t>(1));
  fs::remove_all(dir);
  EXPECT_TRUE(l.read(dir, &changed) != 0);
  fs::remove_all(d);
}

TEST(Fs_AttrReaderKeepsOnlySysfsDescriptors) {
  char d[] = "/tmp/gfd-attr-XXXXXX";
  if (!mkdtemp(d)) throw std::runtime_error("mkdtemp");
  std::string f = std::string(d) + "/attr";
  put_file(f, "SPX\n");
  // A regular file may be replaced under an open descriptor: never kept, and
  // a replacement is seen.
  fs::AttrReader plain;
  EXPECT_EQ(plain.read_trimmed(f).value_or(""), std::string("SPX"));
  EXPECT_EQ(plain.open_count(), static_cast<size_t>(0));
  put_file(f, "CPX\n");
  EXPECT_EQ(plain.read_trimmed(f).value_or(""), std::string("CPX"));
  EXPECT_FALSE(plain.read_trimmed(std::string(d) + "/missing").has_value());
  // Kept descriptors re-read from offset 0 every time (what kernfs turns
  // into a fresh show() call): an in-place rewrite is seen.
  fs::AttrReader kept;
  kept.keep_all_for_testing(true);
  EXPECT_EQ(kept.read_trimmed(f).value_or(""), std::string("CPX"));
  EXPECT_EQ(kept.open_count(), static_cast<size_t>(1));
  {
    FILE* fp = std::fopen(f.c_str(), "r+");
    std::fputs("DPX\n", fp);
    std::fclose(fp);
  }
  EXPECT_EQ(kept.read_trimmed(f).value_or(""), std::string("DPX"));
  EXPECT_EQ(kept.open_count(), static_cast<size_t>(1));
  kept.clear();
  EXPECT_EQ(kept.open_count(), static_cast<size_t>(0));
  // Real sysfs (when present) is kept open.
  fs::AttrReader sys;
  if (sys.read_trimmed("/sys/kernel/mm/transparent_hugepage/enabled") || sys.read_trimmed("/sys/kernel/uevent_seqnum"))
    EXPECT_EQ(sys.open_count(), static_cast<size_t>(1));
  fs::remove_all(d);
}

TEST(Fs_KeptReadsAreWholeAtAnySize) {
  // A first read shorter than a page is the whole attribute (one pread); a
  // longer one keeps reading to the end.
  char d[] = "/tmp/gfd-attr-size-XXXXXX";
  EXPECT_TRUE(mkdtemp(d) != nullptr);
  std::string f = std::string(d) + "/attr";
  fs::AttrReader kept;
  kept.keep_all_for_testing(true);
  for (size_t n : {size_t{5}, size_t{4095}, size_t{4096}, size_t{6000}, size_t{20000}, size_t{7}}) {
    std::string body(n, 'x');
    for (size_t i = 0; i < n; i += 97) body[i] = static_cast<char>('a' + i % 26);
    FILE* fp = std::fopen(f.c_str(), "w");  // same inode: the kept descriptor reads it
    std::fwrite(body.data(), 1, body.size(), fp);
    std::fclose(fp);
    auto r = kept.read(f);
    EXPECT_TRUE(r.ok());
    EXPECT_EQ(r.data.size(), n);
    EXPECT_TRUE(r.data == body);
  }
  EXPECT_EQ(kept.open_count(), static_cast<size_t>(1));
  EXPECT_EQ(kept.read(f, 3).data, std::string("axx"));
  fs::remove_all(d);
}

TEST(Fs_KeptAttrReadsFreshOffSysfsAndKeepsOnSysfs) {
  char d[] = "/tmp/gfd-kept-attr-XXXXXX";
  EXPECT_TRUE(mkdtemp(d) != nullptr);
  std::string f = std::string(d) + "/generation_id";
  fs::KeptAttr a(f);
  std::string v;
  EXPECT_FALSE(a.read(&v));  // missing
  put_file(f, " 7\n");
  EXPECT_TRUE(a.read(&v));
  EXPECT_EQ(v, std::string("7"));
  put_file(f, "8\n");  // replaced (a new inode): off sysfs nothing is kept
  EXPECT_TRUE(a.read(&v));
  EXPECT_EQ(v, std::string("8"));
  fs::remove_all(d);
  EXPECT_FALSE(a.read(&v));
  // Real sysfs (when present): read through the kept descriptor, fresh each time.
  fs::KeptAttr seq("/sys/kernel/uevent_seqnum");
  std::string s1, s2;
  if (seq.read(&s1)) {
    EXPECT_TRUE(seq.read(&s2));
    EXPECT_TRUE(str::parse_uint(s2).value_or(0) >= str::parse_uint(s1).value_or(0));
  }
}

TEST(Fs_AttrReaderDropsADescriptorThatStopsReading) {
  // The CPU-side analogue of a sysfs attribute whose device went away (reads
  // on the kept descriptor fail with ENODEV): a /proc file of a process that
  // has been reaped fails with ESRCH.  The descriptor is dropped and the path
  // looked up again, which then fails too.
  int pipefd[2];
  EXPECT_TRUE(::pipe(pipefd) == 0);
  pid_t pid = ::fork();
  if (pid == 0) {
    char c;
    ::close(pipefd[1]);
    while (::read(pipefd[0], &c, 1) > 0) {
    }
    ::_exit(0);
  }
  ::close(pipefd[0]);
  std::string path = "/proc/" + std::to_string(pid) + "/stat";
  fs::AttrReader r;
  r.keep_all_for_testing(true);
  EXPECT_TRUE(r.read_trimmed(path).has_value());
  EXPECT_EQ(r.open_count(), static_cast<size_t>(1));
  ::close(pipefd[1]);  // the child sees EOF and exits
  int status = 0;
  EXPECT_EQ(::waitpid(pid, &status, 0), pid);
  auto gone = r.read(path);
  EXPECT_FALSE(gone.ok());
  EXPECT_EQ(r.open_count(), static_cast<size_t>(0));
}

TEST(Sriov_ListingSkippedWhileUeventSeqnumUnchanged) {
  std::string root = pci_host(20, 0);
  std::string dev = root + "/sys/bus/pci/devices/";
  put_file(root + "/sys/kernel/uevent_seqnum", "1000\n");
  SysfsAmdPCI pci(root);
  EXPECT_EQ(pci.Devices().size(), static_cast<size_t>(5));
  // A function appears without a uevent (impossible on a real kernel): the
  // listing is not read again...
  put_file(dev + "0000:e1:00.0/vendor", "0x1002\n");
  put_file(dev + "0000:e1:00.0/class", "0x120000\n");
  put_file(dev + "0000:e1:00.0/device", "0x75a3\n");
  put_file(dev + "0000:e1:00.0/sriov_totalvfs", "0\n");
  EXPECT_EQ(pci.Devices().size(), static_cast<size_t>(5));
  // ... the uevent that device_add() sends makes the next scan see it.
  put_file(root + "/sys/kernel/uevent_seqnum", "1001\n");
  EXPECT_EQ(pci.Devices().size(), static_cast<size_t>(6));
  // Without the counter every scan reads the listing.
  fs::remove_all(root + "/sys/kernel/uevent_seqnum");
  fs::remove_all(dev + "0000:e1:00.0");
  EXPECT_EQ(pci.Devices().size(), static_cast<size_t>(5));
  fs::remove_all(root);
}

TEST(Fs_AttrReaderCheckedFollowsReplacedFiles) {
  char d[] = "/tmp/gfd-checked-XXXXXX";
  if (!mkdtemp(d)) throw std::runtime_error("mkdtemp");
  std::string f = std::string(d) + "/version";
  put_file(f, "7.2.0\n");
  fs::AttrReader r;
  EXPECT_EQ(r.read_checked_trimmed(f).value_or(""), std::string("7.2.0"));
  EXPECT_EQ(r.open_count(), static_cast<size_t>(1));
  EXPECT_EQ(r.read_checked_trimmed(f).value_or(""), std::string("7.2.0"));
  put_file(f, "7.3.1\n");  // replaced (rename over it): a new inode
  EXPECT_EQ(r.read_checked_trimmed(f).value_or(""), std::string("7.3.1"));
  {
    FILE* fp = std::fopen(f.c_str(), "r+");  // rewritten in place
    std::fputs("7.4.0\n", fp);
    std::fclose(fp);
  }
  EXPECT_EQ(r.read_checked_trimmed(f).value_or(""), std::string("7.4.0"));
  fs::remove_all(f);
  EXPECT_FALSE(r.read_checked_trimmed(f).has_value());
  EXPECT_EQ(r.open_count(), static_cast<size_t>(0));
  fs::remove_all(d);
}

TEST(Sriov_FailedScanLeavesStateForTheNextOne) {
  std::string root = pci_host(20, 0);
  std::string dev = root + "/sys/bus/pci/devices/";
  SysfsAmdPCI pci(root);
  EXPECT_EQ(pci.Devices().size(), static_cast<size_t>(5));
  // A new function whose vendor cannot be read yet: the scan fails ...
  fs::mkdir_all(dev + "0000:e1:00.0/vendor");
  put_file(dev + "0000:e1:00.0/class", "0x120000\n");
  put_file(dev + "0000:e1:00.0/device", "0x75a3\n");
  put_file(dev + "0000:e1:00.0/sriov_totalvfs", "0\n");
  EXPECT_THROW_MSG(pci.Devices(), "unable to read PCI device vendor id for 0000:e1:00.0");
  // ... and the next one, over the same listing, reads it again and keeps
  // the identities it already had.
  fs::remove_all(dev + "0000:e1:00.0/vendor");
  put_file(dev + "0000:e1:00.0/vendor", "0x1002\n");
  auto devs = pci.Devices();
  EXPECT_EQ(devs.size(), static_cast<size_t>(6));
  for (const auto& d : devs) EXPECT_EQ(d.device, std::string("0x75a3"));
  fs::remove_all(root);
}

// ---------------------------------------------------------------------------
// Driver-directed discovery (sriov/bound.h)

namespace {
void bind_driver(const std::string& root, const std::string& driver, const std::string& bdf) {
  std::string dir = root + "/sys/bus/pci/drivers/" + driver;
  fs::mkdir_all(dir);
  put_file(dir + "/bind", "");
  put_file(dir + "/unbind", "");
  if (symlink(("../../devices/" + bdf).c_str(), (dir + "/" + bdf).c_str()) != 0) throw std::runtime_error("symlink");
}

// pci_host() as a GIM host binds it: the 4 plain PFs to amdgpu, the PF with
// VFs to gim, its VFs named by virtfn links (and bound to nothing).
std::string bound_host(int filler, int vfs) {
  std::string root = pci_host(filler, vfs);
  for (int g = 0; g < 4; ++g) {
    std::string bdf = str::format("0000:%02x:00.0", 0x11 + 0x10 * g);
    bind_driver(root, "amdgpu", bdf);
    // The 4 plain PFs carry a uevent (class and ID in one read); the PF with
    // VFs does not, so both ways of reading them are compared below.
    put_file(root + "/sys/bus/pci/devices/" + bdf + "/uevent",
             "DRIVER=amdgpu\nPCI_CLASS=120000\nPCI_ID=1002:75A3\nPCI_SLOT_NAME=" + bdf + "\n");
  }
  bind_driver(root, "gim", "0000:c1:00.0");
  std::string pf = root + "/sys/bus/pci/devices/0000:c1:00.0/";
  for (int v = 0; v < vfs; ++v)
    if (symlink(str::format("../0000:c1:00.%d", v + 1).c_str(), (pf + "virtfn" + std::to_string(v)).c_str()) != 0)
      throw std::runtime_error("symlink");
  return root;
}

std::string describe(const std::vector<PCIDevice>& devs) {
  std::string out;
  for (const auto& d : devs)
    out += d.address + " " + d.vendor + " " + d.device + " " + d.class_code + " " + std::to_string(d.sriov_totalvfs) +
           " " + std::to_string(d.sriov_numvfs) + " " + d.sriov_vf_device + " " + d.physfn + " cfg" +
           std::to_string(d.config.size()) + "\n";
  return out;
}
}  // namespace

TEST(Bound_SameFunctionsAsTheFullBusScan) {
  // The full scan reads 300 + 9 functions; the bound scan 5 + 3 VFs - and
  // both hand sriov::Lib the same functions, field for field.
  std::string root = bound_host(300, 3);
  BoundAmdPCI bound(root);
  SysfsAmdPCI full(root);
  auto b = bound.Devices();
  EXPECT_FALSE(bound.used_fallback());
  EXPECT_EQ(b.size(), static_cast<size_t>(8));
  EXPECT_EQ(describe(b), describe(full.Devices()));
  auto labels = lm::NewSriovLabeler(std::make_shared<Lib>(std::make_shared<BoundAmdPCI>(root)))->GetLabels();
  auto want = lm::NewSriovLabeler(std::make_shared<Lib>(std::make_shared<SysfsAmdPCI>(root)))->GetLabels();
  EXPECT_EQ(labels, want);
  EXPECT_EQ(labels["amd.com/sriov.num-vfs"], std::string("3"));
  fs::remove_all(root);
}

TEST(Bound_DisplayClassFromUeventKeepsItsLeadingZero) {
  // The kernel prints PCI_CLASS with %04X: a display-class MxGPU PF (0x038000,
  // V620/V710 hosts, MI2xx) appears as "38000".  Read as "0x38000" it failed
  // the 0x03 check and every such PF and VF vanished.
  std::string root = bound_host(4, 2);
  std::string dev = root + "/sys/bus/pci/devices/";
  for (const char* bdf : {"0000:11:00.0", "0000:c1:00.0", "0000:c1:00.1", "0000:c1:00.2"}) {
    put_file(dev + bdf + "/class", "0x038000\n");
    put_file(dev + bdf + "/uevent", std::string("DRIVER=amdgpu\nPCI_CLASS=38000\nPCI_ID=1002:73A1\nPCI_SLOT_NAME=") +
                                        bdf + "\n");
    put_file(dev + bdf + "/device", "0x73a1\n");
  }
  auto b = BoundAmdPCI(root).Devices();
  EXPECT_EQ(b.size(), static_cast<size_t>(7));
  EXPECT_EQ(describe(b), describe(SysfsAmdPCI(root).Devices()));
  for (const auto& d : b)
    if (d.address == "0000:c1:00.0") EXPECT_EQ(d.class_code, std::string("0x03"));
  // Garbage in PCI_CLASS falls back to the `class` attribute.
  put_file(dev + std::string("0000:11:00.0/uevent"), "PCI_CLASS=zz\nPCI_ID=1002:73A1\n");
  EXPECT_EQ(describe(BoundAmdPCI(root).Devices()), describe(SysfsAmdPCI(root).Devices()));
  fs::remove_all(root);
}

TEST(Bound_NeverReadsFunctionsNoDriverBinds) {
  // An unbound AMD function whose class cannot be read: the full scan fails
  // on it, the bound scan never looks.
  std::string root = bound_host(10, 0);
  std::string odd = root + "/sys/bus/pci/devices/0000:e1:00.0";
  put_file(odd + "/vendor", "0x1002\n");
  fs::mkdir_all(odd + "/class");  // reads fail (EISDIR)
  BoundAmdPCI bound(root);
  EXPECT_EQ(bound.Devices().size(), static_cast<size_t>(5));
  EXPECT_THROW_MSG(SysfsAmdPCI(root).Devices(), "unable to read PCI device class for 0000:e1:00.0");
  fs::remove_all(root);
}

TEST(Bound_WithTheBusSeesAVfioPfAndItsVfs) {
  // A host whose GPUs are bound to amdgpu, except the SR-IOV PF handed to
  // vfio-pci (its VFs enabled by vfio-pci and bound to nothing): the
  // functions are the whole-bus scan's, field for field, and so are the
  // labels - vfio-pci is one of the listed drivers; a function no driver
  // binds needs the bus (below).
  std::string root = pci_host(40, 2);
  std::string dev = root + "/sys/bus/pci/devices/";
  for (int g = 0; g < 4; ++g) bind_driver(root, "amdgpu", str::format("0000:%02x:00.0", 0x11 + 0x10 * g));
  bind_driver(root, "vfio-pci", "0000:c1:00.0");
  for (int v = 0; v < 2; ++v)
    EXPECT_EQ(symlink(str::format("../0000:c1:00.%d", v + 1).c_str(), (dev + "0000:c1:00.0/virtfn" + std::to_string(v)).c_str()), 0);
  put_file(root + "/sys/kernel/uevent_seqnum", "100\n");
  // vfio-pci also binds other vendors' functions: not reported.
  std::string nic = dev + "0000:e9:00.0";
  put_file(nic + "/vendor", "0x15b3\n");
  put_file(nic + "/class", "0x020000\n");
  bind_driver(root, "vfio-pci", "0000:e9:00.0");
  EXPECT_EQ(describe(BoundAmdPCI(root).Devices()), describe(SysfsAmdPCI(root).Devices()));
  auto bus = std::make_shared<SysfsAmdPCI>(root);
  BoundAmdPCI bound(root, bus);
  auto b = bound.Devices();
  EXPECT_FALSE(bound.used_fallback());
  EXPECT_EQ(b.size(), static_cast<size_t>(7));
  EXPECT_EQ(describe(b), describe(SysfsAmdPCI(root).Devices()));
  auto labels = lm::NewSriovLabeler(std::make_shared<Lib>(std::make_shared<BoundAmdPCI>(root, std::make_shared<SysfsAmdPCI>(root))))->GetLabels();
  auto want = lm::NewSriovLabeler(std::make_shared<Lib>(std::make_shared<SysfsAmdPCI>(root)))->GetLabels();
  EXPECT_EQ(labels, want);
  EXPECT_EQ(labels["amd.com/sriov.num-vfs"], std::string("2"));
  // Rebinding the PF from vfio-pci to gim (a uevent) changes no function.
  fs::remove_all(root + "/sys/bus/pci/drivers/vfio-pci/0000:c1:00.0");
  bind_driver(root, "gim", "0000:c1:00.0");
  put_file(root + "/sys/kernel/uevent_seqnum", "101\n");
  EXPECT_EQ(describe(bound.Devices()), describe(SysfsAmdPCI(root).Devices()));
  // An AMD function hot-added and bound to nothing is seen once the counter
  // moves; one removed is gone.
  std::string extra = dev + "0000:e1:00.0";
  put_file(extra + "/vendor", "0x1002\n");
  put_file(extra + "/class", "0x030000\n");
  put_file(extra + "/device", "0x75a3\n");
  put_file(extra + "/sriov_totalvfs", "0\n");
  put_file(root + "/sys/kernel/uevent_seqnum", "102\n");
  auto after = bound.Devices();
  EXPECT_EQ(after.size(), static_cast<size_t>(8));
  EXPECT_EQ(describe(after), describe(SysfsAmdPCI(root).Devices()));
  EXPECT_EQ(BoundAmdPCI(root).Devices().size(), static_cast<size_t>(7));  // without the bus: not seen
  EXPECT_EQ(BoundAmdPCI(root, std::make_shared<SysfsAmdPCI>(root), false).Devices().size(), static_cast<size_t>(7));
  fs::remove_all(extra);
  put_file(root + "/sys/kernel/uevent_seqnum", "103\n");
  EXPECT_EQ(describe(bound.Devices()), describe(SysfsAmdPCI(root).Devices()));
  // A counter moved for some other device: nothing is read again (a function
  // whose class became unreadable would fail a re-read).
  fs::remove_all(dev + "0000:11:00.0/class");
  fs::mkdir_all(dev + "0000:11:00.0/class");
  put_file(root + "/sys/kernel/uevent_seqnum", "150\n");
  EXPECT_EQ(bound.Devices().size(), static_cast<size_t>(7));
  fs::remove_all(root);
}

TEST(Bound_WithTheBusSeesAGuestVfAmdgpuDidNotProbe) {
  // A guest with two VFs: amdgpu bound one and failed to probe the other.
  // Both are the guest's AMD functions, as the whole-bus scan reports them.
  char d[] = "/tmp/gfd-pci-XXXXXX";
  EXPECT_TRUE(mkdtemp(d) != nullptr);
  std::string root = d;
  for (const char* bdf : {"0000:00:05.0", "0000:00:06.0"}) {
    std::string p = root + "/sys/bus/pci/devices/" + bdf;
    put_file(p + "/vendor", "0x1002\n");
    put_file(p + "/class", "0x120000\n");
    put_file(p + "/device", "0x75b3\n");
    put_file(p + "/config", std::string(64, '\x02'));
  }
  for (int i = 0; i < 12; ++i) {  // the VM's chipset and virtio functions
    std::string p = root + "/sys/bus/pci/devices/" + str::format("0000:00:%02x.0", 0x10 + i);
    put_file(p + "/vendor", "0x1af4\n");
    put_file(p + "/class", "0x010000\n");
  }
  bind_driver(root, "amdgpu", "0000:00:05.0");
  put_file(root + "/sys/kernel/uevent_seqnum", "7\n");
  EXPECT_EQ(BoundAmdPCI(root).Devices().size(), static_cast<size_t>(1));  // the gap without the bus
  BoundAmdPCI bound(root, std::make_shared<SysfsAmdPCI>(root));
  auto b = bound.Devices();
  EXPECT_EQ(b.size(), static_cast<size_t>(2));
  EXPECT_EQ(describe(b), describe(SysfsAmdPCI(root).Devices()));
  auto fns = Lib(std::make_shared<BoundAmdPCI>(root, std::make_shared<SysfsAmdPCI>(root))).Devices();
  EXPECT_EQ(fns.size(), static_cast<size_t>(2));
  for (const auto& f : fns) EXPECT_EQ(f.GetInfo().role, std::string("vf"));
  fs::remove_all(root);
}

TEST(Bound_ADriverLoadedLaterIsListed) {
  // Only the listed drivers that are loaded are read (one listing of
  // sys/bus/pci/drivers says which); one that loads later - vfio-pci taking
  // a GPU for a VM - is read from then on.
  std::string root = bound_host(3, 0);
  put_file(root + "/sys/kernel/uevent_seqnum", "10\n");
  BoundAmdPCI bound(root);
  EXPECT_EQ(bound.Devices().size(), static_cast<size_t>(5));
  fs::remove_all(root + "/sys/bus/pci/drivers/amdgpu/0000:41:00.0");
  bind_driver(root, "vfio-pci", "0000:41:00.0");
  put_file(root + "/sys/kernel/uevent_seqnum", "11\n");
  auto devs = bound.Devices();
  EXPECT_EQ(devs.size(), static_cast<size_t>(5));
  bool seen = false;
  for (const auto& d : devs) seen |= d.address == "0000:41:00.0";
  EXPECT_TRUE(seen);
  // Unloaded again: its directory is gone, nothing is read from it.
  fs::remove_all(root + "/sys/bus/pci/drivers/vfio-pci");
  put_file(root + "/sys/kernel/uevent_seqnum", "12\n");
  EXPECT_EQ(bound.Devices().size(), static_cast<size_t>(4));
  fs::remove_all(root);
}

TEST(Bound_FallsBackToTheBusWhenNothingIsBound) {
  // A guest whose amdgpu is not loaded: its VF is on the bus, bound to nothing.
  std::string root = pci_host(5, 0);
  fs::mkdir_all(root + "/sys/bus/pci/drivers/amdgpu");  // module loaded, nothing bound
  BoundAmdPCI bound(root, std::make_shared<SysfsAmdPCI>(root));
  auto devs = bound.Devices();
  EXPECT_TRUE(bound.used_fallback());
  EXPECT_EQ(devs.size(), static_cast<size_t>(5));
  EXPECT_EQ(BoundAmdPCI(root).Devices().size(), static_cast<size_t>(0));  // no fallback given
  fs::remove_all(root);
}

TEST(Bound_GuestVFOnAmdgpu) {
  // Inside a VM: the VF is an ordinary function to the guest kernel - no
  // physfn link, no SR-IOV attributes - bound to amdgpu; its VF device ID
  // makes it a VF, and its (unprivileged, 64-byte) config space is read
  // because sysfs publishes no SR-IOV state for it.
  char d[] = "/tmp/gfd-pci-XXXXXX";
  EXPECT_TRUE(mkdtemp(d) != nullptr);
  std::string root = d;
  std::string p = root + "/sys/bus/pci/devices/0000:00:05.0";
  put_file(p + "/vendor", "0x1002\n");
  put_file(p + "/class", "0x120000\n");
  put_file(p + "/device", "0x75b3\n");
  put_file(p + "/config", std::string(64, '\x02'));
  bind_driver(root, "amdgpu", "0000:00:05.0");
  auto fns = Lib(std::make_shared<BoundAmdPCI>(root)).Devices();
  EXPECT_EQ(fns.size(), static_cast<size_t>(1));
  EXPECT_EQ(fns[0].GetInfo().role, std::string("vf"));
  EXPECT_EQ(fns[0].pci().config.size(), static_cast<size_t>(64));
  fs::remove_all(root);
}

TEST(Bound_KeptWhileUeventSeqnumUnchanged) {
  std::string root = bound_host(3, 2);
  std::string dev = root + "/sys/bus/pci/devices/";
  put_file(root + "/sys/kernel/uevent_seqnum", "4242\n");
  BoundAmdPCI bound(root, std::make_shared<SysfsAmdPCI>(root));
  EXPECT_EQ(bound.Devices().size(), static_cast<size_t>(7));
  // A VF removed behind a constant seqnum (impossible on a real kernel: the
  // removal sends a uevent) is not noticed...
  fs::remove_all(dev + "0000:c1:00.0/virtfn1");
  fs::remove_all(dev + "0000:c1:00.2");
  EXPECT_EQ(bound.Devices().size(), static_cast<size_t>(7));
  // ...until the seqnum moves.
  put_file(root + "/sys/kernel/uevent_seqnum", "4243\n");
  EXPECT_EQ(bound.Devices().size(), static_cast<size_t>(6));
  // A counter that moved for another device (a container's veth, say):
  // the functions are not read again - here one whose class has become
  // unreadable would make a re-read fail.
  fs::remove_all(dev + "0000:11:00.0/class");
  fs::mkdir_all(dev + "0000:11:00.0/class");
  put_file(root + "/sys/kernel/uevent_seqnum", "4300\n");
  EXPECT_EQ(bound.Devices().size(), static_cast<size_t>(6));
  fs::remove_all(dev + "0000:11:00.0/class");
  put_file(dev + "0000:11:00.0/class", "0x120000\n");
  // A function removed and re-added under the same address (a new entry in
  // the driver directory) is read again.
  fs::remove_all(root + "/sys/bus/pci/drivers/amdgpu/0000:21:00.0");
  put_file(root + "/sys/bus/pci/drivers/amdgpu/placeholder", "");  // takes the freed inode number (kernfs never reuses one)
  bind_driver(root, "amdgpu", "0000:21:00.0");
  put_file(dev + "0000:21:00.0/device", "0x75a0\n");
  fs::remove_all(dev + "0000:21:00.0/uevent");
  put_file(root + "/sys/kernel/uevent_seqnum", "4301\n");
  auto devs = bound.Devices();
  EXPECT_EQ(devs.size(), static_cast<size_t>(6));
  bool seen = false;
  for (const auto& d : devs) seen |= d.address == "0000:21:00.0" && d.device == "0x75a0";
  EXPECT_TRUE(seen);
  // VFs enabled on a PF that had none (the kernel adds the VF functions and
  // the PF's virtfn links) are seen once the seqnum moves...
  std::string vf = dev + "0000:11:00.1";
  put_file(vf + "/vendor", "0x1002\n");
  put_file(vf + "/class", "0x120000\n");
  put_file(vf + "/device", "0x75b3\n");
  EXPECT_EQ(symlink("../0000:11:00.0", (vf + "/physfn").c_str()), 0);
  EXPECT_EQ(symlink("../0000:11:00.1", (dev + "0000:11:00.0/virtfn0").c_str()), 0);
  put_file(dev + "0000:11:00.0/sriov_numvfs", "1\n");
  EXPECT_EQ(bound.Devices().size(), static_cast<size_t>(6));  // same seqnum: kept
  put_file(root + "/sys/kernel/uevent_seqnum", "4302\n");
  EXPECT_EQ(bound.Devices().size(), static_cast<size_t>(7));
  // ...and disabled again.
  fs::remove_all(dev + "0000:11:00.0/virtfn0");
  fs::remove_all(vf);
  put_file(dev + "0000:11:00.0/sriov_numvfs", "0\n");
  put_file(root + "/sys/kernel/uevent_seqnum", "4303\n");
  EXPECT_EQ(bound.Devices().size(), static_cast<size_t>(6));
  // Nothing reads sriov_numvfs while the listings stand (its show() waits
  // for the device lock): a value no change of the bus backs is not read.
  std::string numvfs = dev + "0000:31:00.0/sriov_numvfs";
  put_file(numvfs, "3\n");
  put_file(root + "/sys/kernel/uevent_seqnum", "4304\n");
  for (const auto& d : bound.Devices())
    if (d.address == "0000:31:00.0") EXPECT_EQ(d.sriov_numvfs, 0);
  put_file(numvfs, "0\n");
  // An emulated sysfs that never counts ("0") is re-read every time.
  put_file(root + "/sys/kernel/uevent_seqnum", "0\n");
  fs::remove_all(dev + "0000:c1:00.0/virtfn0");
  fs::remove_all(dev + "0000:c1:00.1");
  EXPECT_EQ(bound.Devices().size(), static_cast<size_t>(5));
  // Without the bus (a host): the driver listings and the PFs' VF links are
  // the check.  Nothing is re-read while they stand...
  BoundAmdPCI host(root);
  put_file(root + "/sys/kernel/uevent_seqnum", "5000\n");
  EXPECT_EQ(host.Devices().size(), static_cast<size_t>(5));
  fs::remove_all(dev + "0000:11:00.0/class");
  fs::mkdir_all(dev + "0000:11:00.0/class");
  fs::remove_all(dev + "0000:11:00.0/uevent");
  put_file(root + "/sys/kernel/uevent_seqnum", "5001\n");
  EXPECT_EQ(host.Devices().size(), static_cast<size_t>(5));
  fs::remove_all(dev + "0000:11:00.0/class");
  put_file(dev + "0000:11:00.0/class", "0x120000\n");
  // ...and VFs enabled behind unchanged driver listings are seen through
  // their PF's links.
  std::string vf31 = dev + "0000:31:00.1";
  put_file(vf31 + "/vendor", "0x1002\n");
  put_file(vf31 + "/class", "0x120000\n");
  put_file(vf31 + "/device", "0x75b3\n");
  EXPECT_EQ(symlink("../0000:31:00.0", (vf31 + "/physfn").c_str()), 0);
  EXPECT_EQ(symlink("../0000:31:00.1", (dev + "0000:31:00.0/virtfn0").c_str()), 0);
  put_file(dev + "0000:31:00.0/sriov_numvfs", "1\n");
  put_file(root + "/sys/kernel/uevent_seqnum", "5002\n");
  EXPECT_EQ(host.Devices().size(), static_cast<size_t>(6));
  fs::remove_all(root);
}
