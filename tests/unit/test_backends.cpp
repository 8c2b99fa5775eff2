// Backend tests: KFD-sysfs enumeration over synthetic trees, the device
// filter, ISA/version parsing, fallback, mock fixtures and backend selection.
// (The reference tests its NVML adapter only through mocks; the sysfs
// backend here is fully testable on CPU because it only reads files.)
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <condition_variable>
#include <fstream>
#include <mutex>

#include "config/config.h"
#include "lm/labels.h"
#include "resource/amdsmi.h"
#include "resource/factory.h"
#include "resource/filter.h"
#include "resource/managers.h"
#include "resource/pci_ids.h"
#include "resource/sysfs.h"
#include "resource/versions.h"
#include "test.h"
#include "util/fs.h"
#include "util/log.h"
#include "util/strings.h"
#include "util/trace.h"

using namespace gfd;
using namespace gfd::resource;

namespace {

void put(const std::string& path, const std::string& content) {
  fs::mkdir_all(fs::dirname(path));
  lm::write_file_atomically(path, content, 0644);
  fs::remove_all(fs::join(fs::dirname(path), "gfd-tmp"));
}

std::string kfd_props(uint64_t gfx, uint64_t simd, uint64_t xcc, uint64_t location, uint64_t render, uint64_t unique) {
  return str::format(
      "cpu_cores_count 0\nsimd_count %llu\nmem_banks_count 1\nsimd_per_cu 4\ngfx_target_version %llu\n"
      "vendor_id 4098\ndevice_id 30115\nlocation_id %llu\ndomain 0\ndrm_render_minor %llu\nunique_id %llu\n"
      "num_sdma_engines 2\nnum_xcc %llu\nlocal_mem_size 0\n",
      (unsigned long long)simd, (unsigned long long)gfx, (unsigned long long)location, (unsigned long long)render,
      (unsigned long long)unique, (unsigned long long)xcc);
}

struct Tree {
  std::string root;
  Tree() {
    char d[] = "/tmp/gfd-sysfs-XXXXXX";
    if (!mkdtemp(d)) throw std::runtime_error("mkdtemp");
    root = d;
    std::string nodes = root + "/sys/class/kfd/kfd/topology/nodes";
    put(nodes + "/0/properties", "cpu_cores_count 128\nsimd_count 0\ngfx_target_version 0\n");
    put(root + "/sys/class/kfd/kfd/topology/generation_id", "1\n");
    put(root + "/sys/module/amdgpu/version", "6.12.12\n");
    put(root + "/opt/rocm/.info/version", "7.2.0-43\n");
    // GPU A: SPX at d9:00.0 (node 1).
    put(nodes + "/1/properties", kfd_props(90500, 1024, 8, 0xd900, 128, 0x3a7c178b7c5e4d5cULL));
    put(nodes + "/1/mem_banks/0/properties", "heap_type 1\nsize_in_bytes 309220868096\n");
    pci("0000:d9:00.0", "SPX", "NPS1", 309220868096ULL);
    // GPU B: CPX at 23:00.0 (nodes 2..9, one XCD each, 36 GiB each).
    for (int p = 0; p < 8; ++p) {
      std::string n = nodes + "/" + std::to_string(2 + p);
      put(n + "/properties", kfd_props(90500, 128, 1, 0x2300, 136 + p, 0x75c7dc68fc70d513ULL));
      put(n + "/mem_banks/0/properties", "heap_type 1\nsize_in_bytes 38652608512\n");
    }
    pci("0000:23:00.0", "CPX", "NPS1", 309220868096ULL);
  }
  void pci(const std::string& bdf, const std::string& cp, const std::string& mp, uint64_t vram) {
    std::string d = root + "/sys/bus/pci/devices/" + bdf;
    put(d + "/vendor", "0x1002\n");
    put(d + "/device", "0x75a3\n");
    put(d + "/class", "0x120000\n");
    put(d + "/product_name", "AMD Instinct MI355 OAM\n");
    put(d + "/current_compute_partition", cp + "\n");
    put(d + "/available_compute_partition", "SPX, DPX, QPX, CPX\n");
    put(d + "/current_memory_partition", mp + "\n");
    put(d + "/available_memory_partition", "NPS1, NPS2\n");
    put(d + "/mem_info_vram_total", std::to_string(vram) + "\n");
    put(d + "/xgmi_num_links", "01 01 01 01 01 01 00 01\n");
    put(d + "/sriov_totalvfs", "1\n");
    put(d + "/sriov_numvfs", "0\n");
    put(d + "/config", std::string(64, '\0'));
  }
  ~Tree() { fs::remove_all(root); }
};

}  // namespace

TEST(Sysfs_TopologyKeptPerKfdGeneration) {
  Tree t;
  std::string nodes = t.root + "/sys/class/kfd/kfd/topology/nodes";
  SysfsManager m(SysfsOptions{t.root, DeviceFilter(), {}});
  auto cycle = [&] {
    m.Init();
    auto d = m.GetDevices();
    m.Shutdown();
    return d;
  };
  EXPECT_EQ(cycle()[1]->Info().xcds, static_cast<uint32_t>(8));
  // A node property rewritten without a new generation (KFD never does that)
  // is not re-read; per-GPU attributes still are.
  put(nodes + "/1/properties", kfd_props(90500, 1024, 4, 0xd900, 128, 0x3a7c178b7c5e4d5cULL));
  put(t.root + "/sys/bus/pci/devices/0000:d9:00.0/current_memory_partition", "NPS2\n");
  auto d = cycle();
  EXPECT_EQ(d[1]->Info().xcds, static_cast<uint32_t>(8));
  EXPECT_EQ(d[1]->Info().memory_partition, std::string("NPS2"));
  // KFD re-enumerates (partition switch, driver reload): new generation.
  put(t.root + "/sys/class/kfd/kfd/topology/generation_id", "2\n");
  EXPECT_EQ(cycle()[1]->Info().xcds, static_cast<uint32_t>(4));
  // A GPU removed together with a generation bump disappears.
  fs::remove_all(nodes + "/1");
  put(t.root + "/sys/class/kfd/kfd/topology/generation_id", "3\n");
  EXPECT_EQ(cycle().size(), static_cast<size_t>(1));
  // Without generation_id nothing is kept.
  fs::remove_all(t.root + "/sys/class/kfd/kfd/topology/generation_id");
  put(nodes + "/1/properties", kfd_props(90500, 1024, 8, 0xd900, 128, 0x3a7c178b7c5e4d5cULL));
  EXPECT_EQ(cycle().size(), static_cast<size_t>(2));
}

TEST(Sysfs_ComputeModeReadOncePerKfdGeneration) {
  // current_compute_partition makes amdgpu read an XCP register, which can
  // wake the GPU: it is read when the topology is, not every cycle.
  Tree t;
  SysfsManager m(SysfsOptions{t.root, DeviceFilter(), {}});
  std::string attr = t.root + "/sys/bus/pci/devices/0000:d9:00.0/current_compute_partition";
  auto cycle = [&](int* reads) {
    m.Init();
    trace::begin_cycle();
    auto d = m.GetDevices();
    *reads = 0;
    for (const auto& p : trace::phases()) *reads += p.first == "compute_partition(read)";
    m.Shutdown();
    return d;
  };
  int reads = 0;
  EXPECT_EQ(cycle(&reads)[1]->Info().compute_partition, std::string("SPX"));
  EXPECT_EQ(reads, 2);  // both GPUs
  put(attr, "DPX\n");  // no real switch leaves the generation as it was
  EXPECT_EQ(cycle(&reads)[1]->Info().compute_partition, std::string("SPX"));
  EXPECT_EQ(reads, 0);
  put(t.root + "/sys/class/kfd/kfd/topology/generation_id", "2\n");
  EXPECT_EQ(cycle(&reads)[1]->Info().compute_partition, std::string("DPX"));
  EXPECT_EQ(reads, 2);
  EXPECT_EQ(cycle(&reads)[1]->Info().compute_partition, std::string("DPX"));
  EXPECT_EQ(reads, 0);
}

TEST(Sysfs_EnumeratesSpxAndCpxGpus) {
  Tree t;
  SysfsManager m(SysfsOptions{t.root, DeviceFilter(), {}});
  m.Init();
  auto devs = m.GetDevices();
  EXPECT_EQ(devs.size(), static_cast<size_t>(2));
  // Sorted by BDF: 23:00.0 (CPX) first, d9:00.0 (SPX) second.
  const auto& cpx = *devs[0];
  EXPECT_EQ(cpx.Info().bdf, std::string("0000:23:00.0"));
  EXPECT_TRUE(cpx.IsPartitioned());
  EXPECT_TRUE(cpx.IsPartitionCapable());
  EXPECT_EQ(cpx.GetPartitions().size(), static_cast<size_t>(8));
  EXPECT_EQ(cpx.GetTotalMemoryMiB(), static_cast<uint64_t>(294896));
  EXPECT_EQ(cpx.Info().compute_units, static_cast<uint32_t>(256));
  EXPECT_EQ(cpx.Info().xcds, static_cast<uint32_t>(8));
  auto p0 = cpx.GetPartitions()[0];
  EXPECT_EQ(p0->GetName(), std::string("cpx.1xcd.36gb"));
  EXPECT_EQ(p0->GetAttributes().at("compute-units"), std::string("32"));
  EXPECT_EQ(p0->GetAttributes().at("memory"), std::string("36862"));
  EXPECT_EQ(p0->GetParent().get(), devs[0].get());

  const auto& spx = *devs[1];
  EXPECT_EQ(spx.GetName(), std::string("AMD Instinct MI355 OAM"));
  EXPECT_FALSE(spx.IsPartitioned());
  EXPECT_EQ(spx.GetGfxTarget().name(), std::string("gfx950"));
  EXPECT_EQ(spx.GetTotalMemoryMiB(), static_cast<uint64_t>(294896));
  EXPECT_EQ(spx.Info().compute_units, static_cast<uint32_t>(256));
  EXPECT_EQ(spx.Info().xgmi_links, 7);
  EXPECT_EQ(spx.Info().uuid, std::string("3aff75a3-0000-1000-807c-178b7c5e4d5c"));
  EXPECT_EQ(spx.Info().compute_partition, std::string("SPX"));
  EXPECT_EQ(spx.Info().available_memory_partitions, (std::vector<std::string>{"NPS1", "NPS2"}));
  EXPECT_EQ(m.GetDriverVersion(), std::string("6.12.12"));
  EXPECT_EQ(m.GetRuntimeVersion()->major, 7u);
  EXPECT_EQ(m.GetRuntimeVersion()->minor, 2u);
  m.Shutdown();
}

TEST(Sysfs_VisibleDeviceFilter) {
  Tree t;
  SysfsManager m(SysfsOptions{t.root, DeviceFilter::parse("1"), {}});
  m.Init();
  auto devs = m.GetDevices();
  EXPECT_EQ(devs.size(), static_cast<size_t>(1));
  EXPECT_EQ(devs[0]->Info().bdf, std::string("0000:d9:00.0"));
  SysfsManager m2(SysfsOptions{t.root, DeviceFilter::parse("0000:23:00.0"), {}});
  m2.Init();
  EXPECT_EQ(m2.GetDevices()[0]->Info().bdf, std::string("0000:23:00.0"));
}

TEST(Sysfs_UnreadableNodesAreSkipped) {
  Tree t;
  // Node 1 becomes unreadable like GPUs not allocated to the container.
  ::unlink((t.root + "/sys/class/kfd/kfd/topology/nodes/1/properties").c_str());
  fs::mkdir_all(t.root + "/sys/class/kfd/kfd/topology/nodes/1/properties");  // read fails (EISDIR)
  SysfsManager m(SysfsOptions{t.root, DeviceFilter(), {}});
  m.Init();
  EXPECT_EQ(m.GetDevices().size(), static_cast<size_t>(1));
}

TEST(Sysfs_SnapshotOncePerWindow) {
  Tree t;
  SysfsManager m(SysfsOptions{t.root, DeviceFilter(), {}});
  m.Init();
  auto a = m.GetDevices();
  auto b = m.GetDevices();
  EXPECT_EQ(a[0].get(), b[0].get());
  m.Shutdown();
  m.Init();
  EXPECT_FALSE(m.GetDevices()[0].get() == a[0].get());
}

TEST(Sysfs_MissingTopologyIsInitError) {
  SysfsManager m(SysfsOptions{"/nonexistent-gfd", DeviceFilter(), {}});
  EXPECT_THROW_MSG(m.Init(), "KFD topology not available");
  std::string reason;
  EXPECT_FALSE(has_kfd_topology("/nonexistent-gfd", &reason));
}

TEST(Filter_Parse) {
  auto f = DeviceFilter::parse("0, 2-3,d9:00.0");
  EXPECT_TRUE(f.matches(0, ""));
  EXPECT_FALSE(f.matches(1, ""));
  EXPECT_TRUE(f.matches(3, ""));
  EXPECT_TRUE(f.matches(7, "0000:D9:00.0"));
  EXPECT_TRUE(DeviceFilter::parse("").all());
  EXPECT_TRUE(DeviceFilter::parse("all").all());
  EXPECT_THROW_MSG(DeviceFilter::parse("3-1"), "invalid device range");
  EXPECT_THROW_MSG(DeviceFilter::parse("x"), "invalid device");
  EXPECT_THROW_MSG(DeviceFilter::parse("0000:zz"), "invalid PCI address '0000:zz'");
  EXPECT_THROW_MSG(DeviceFilter::parse("d9:20.0"), "invalid PCI address");  // device > 0x1f
  EXPECT_THROW_MSG(DeviceFilter::parse("d9:00.8"), "invalid PCI address");  // function > 7
  EXPECT_TRUE(DeviceFilter::parse("10000:d9:00.0").matches(0, "10000:d9:00.0"));  // 5-digit domain
}

namespace {
// stderr of `f` (the logger writes there; the test binary silences it).
template <typename F>
std::string stderr_of(F&& f) {
  bool was_quiet = gfd::log::set_quiet(false);
  std::fflush(stderr);
  FILE* tmp = std::tmpfile();
  int saved = ::dup(2);
  ::dup2(::fileno(tmp), 2);
  f();
  std::fflush(stderr);
  ::dup2(saved, 2);
  ::close(saved);
  gfd::log::set_quiet(was_quiet);
  std::string out;
  std::rewind(tmp);
  for (int c; (c = std::fgetc(tmp)) != EOF;) out.push_back(static_cast<char>(c));
  std::fclose(tmp);
  return out;
}
}  // namespace

TEST(Filter_ItemsSelectingNoGpuAreLoggedOnce) {
  auto f = DeviceFilter::parse("1,5,0000:aa:00.0");
  std::vector<std::string> node{"0000:23:00.0", "0000:d9:00.0"};
  std::string first = stderr_of([&] { f.check_selection(node); });
  EXPECT_TRUE(first.find("--visible-devices '1,5,0000:aa:00.0': 5, 0000:aa:00.0 select none of the node's 2 GPU(s)") !=
              std::string::npos);
  // Every cycle checks; the same outcome is not logged again, a new one is.
  EXPECT_EQ(stderr_of([&] { f.check_selection(node); }), std::string());
  node.push_back("0000:aa:00.0");
  EXPECT_TRUE(stderr_of([&] { f.check_selection(node); }).find("5 selects none of the node's 3 GPU(s)") !=
              std::string::npos);
  // Everything selected something: nothing to say.
  EXPECT_EQ(stderr_of([&] { DeviceFilter::parse("0-1").check_selection(node); }), std::string());
}

TEST(GfxTarget_Parsing) {
  EXPECT_EQ(parse_gfx_target("gfx950")->name(), std::string("gfx950"));
  EXPECT_EQ(parse_gfx_target("gfx90a:sramecc+:xnack-")->stepping, 10);
  EXPECT_EQ(parse_gfx_target("gfx1100")->major, 11);
  EXPECT_FALSE(parse_gfx_target("sm_90").has_value());
  EXPECT_EQ(gfx_target_from_kfd(90500).name(), std::string("gfx950"));
  EXPECT_EQ(gfx_target_from_kfd(90010).name(), std::string("gfx90a"));
  // amd-smi spells the target in hex digits (measured: 0x950 on MI355X).
  EXPECT_EQ(gfx_target_from_amdsmi(0x950).name(), std::string("gfx950"));
  EXPECT_EQ(gfx_target_from_amdsmi(0x942).name(), std::string("gfx942"));
  EXPECT_EQ(gfx_target_from_amdsmi(0x1100).name(), std::string("gfx1100"));
  EXPECT_FALSE(gfx_target_from_amdsmi(0).valid());
  // Out-of-range values are unknown targets, not overflowed majors
  // (tests/fuzz/corpus/sysfs/regress-huge-gfx-target).
  EXPECT_FALSE(gfx_target_from_kfd(18446744073709551615ULL).valid());
  EXPECT_FALSE(gfx_target_from_amdsmi(0xFFFFFFFFFFFFFFFFULL).valid());
}

TEST(PartitionMode_OnlyShortAlphanumericTokens) {
  EXPECT_EQ(partition_mode(" cpx\n"), std::string("CPX"));
  EXPECT_EQ(partition_mode("NPS4"), std::string("NPS4"));
  EXPECT_EQ(partition_mode("SPX, DPX"), std::string(""));  // a list where one mode belongs
  EXPECT_EQ(partition_mode(""), std::string(""));
  EXPECT_EQ(partition_mode(std::string(17, 'A')), std::string(""));
  EXPECT_EQ(partition_mode_list("SPX, DPX, QPX, CPX\n"), (std::vector<std::string>{"SPX", "DPX", "QPX", "CPX"}));
  EXPECT_EQ(partition_mode_list("NPS1, N/A, , NPS2"), (std::vector<std::string>{"NPS1", "NPS2"}));
}

TEST(PartitionProfileName) {
  EXPECT_EQ(partition_profile_name("CPX", 1, 36862), std::string("cpx.1xcd.36gb"));
  EXPECT_EQ(partition_profile_name("DPX", 4, 147448), std::string("dpx.4xcd.144gb"));
  EXPECT_EQ(partition_profile_name("", 2, 1024), std::string("xcp.2xcd.1gb"));
}

TEST(Versions_Extract) {
  EXPECT_EQ(*extract_version("6.18.54-ant.1"), std::string("6.18.54"));
  EXPECT_EQ(*extract_version("Linuxversion6.18.54-ant.1(nixbld@localhost)(gcc(GCC)15.3.0"), std::string("6.18.54"));
  EXPECT_EQ(*extract_version("6.12.12.60200"), std::string("6.12.12"));
  EXPECT_EQ(*extract_version("amdgpu 400.300"), std::string("400.300"));
  EXPECT_FALSE(extract_version("no version here 7").has_value());
}

// ---- Node-true ROCm version (resource/versions.h) ----

namespace {
std::string mktemp_dir() {
  char d[] = "/tmp/gfd-rocm-XXXXXX";
  if (!mkdtemp(d)) throw std::runtime_error("mkdtemp");
  return d;
}
void link(const std::string& target, const std::string& path) {
  fs::mkdir_all(fs::dirname(path));
  EXPECT_EQ(symlink(target.c_str(), path.c_str()), 0);
}
}  // namespace

TEST(ResolveInRoot_FollowsHostSymlinksUnderTheMount) {
  std::string host = mktemp_dir();
  put(host + "/opt/rocm-6.4.1/.info/version", "6.4.1-120\n");
  link("/opt/rocm-6.4.1", host + "/opt/rocm");         // absolute: re-rooted
  link("rocm-6.4.1", host + "/opt/rocm-rel");          // relative
  link("../opt/./rocm", host + "/usr/rocm-up");        // .. and . through another link
  EXPECT_EQ(fs::resolve_in_root(host, "opt/rocm/.info/version"), host + "/opt/rocm-6.4.1/.info/version");
  EXPECT_EQ(fs::resolve_in_root(host, "/opt/rocm-rel/.info/version"), host + "/opt/rocm-6.4.1/.info/version");
  EXPECT_EQ(fs::resolve_in_root(host, "usr/rocm-up/.info/version"), host + "/opt/rocm-6.4.1/.info/version");
  EXPECT_EQ(fs::resolve_in_root(host, "../../../opt/rocm/.info/version"), host + "/opt/rocm-6.4.1/.info/version");
  EXPECT_EQ(fs::resolve_in_root(host, "opt/missing/.info/version"), std::string());
  link("/loop-b", host + "/loop-a");
  link("/loop-a", host + "/loop-b");
  EXPECT_EQ(fs::resolve_in_root(host, "loop-a/x"), std::string());
  fs::remove_all(host);
}

TEST(RocmVersion_HostRootWinsOverTheImage) {
  std::string image = mktemp_dir(), host = mktemp_dir();
  put(image + "/opt/rocm/.info/version", "7.2.0\n");  // the container image's own
  put(host + "/opt/rocm-6.4.1/.info/version", "6.4.1-120\n");
  link("/opt/rocm-6.4.1", host + "/opt/rocm");
  VersionSources s;
  s.root = image;
  std::string source;
  EXPECT_EQ(rocm_version(s)->major, 7u);  // without a host root: this root
  s.host_root = host;
  auto v = rocm_version(s, &source);
  EXPECT_TRUE(v.has_value());
  EXPECT_EQ(v->major, 6u);
  EXPECT_EQ(v->minor, 4u);
  EXPECT_EQ(source, host + "/opt/rocm-6.4.1/.info/version");
  fs::remove_all(image);
  fs::remove_all(host);
}

TEST(RocmVersion_AlternativesLinkOutsideTheMountUsesNewestInstall) {
  std::string host = mktemp_dir();
  put(host + "/opt/rocm-6.4.1/.info/version", "6.4.1\n");
  put(host + "/opt/rocm-7.0.2/.info/version", "7.0.2\n");
  put(host + "/opt/rocm-7.10.0/.info/version", "7.10.0\n");  // numeric, not lexical, order
  link("/etc/alternatives/rocm", host + "/opt/rocm");  // /etc is not mounted
  VersionSources s;
  s.host_root = host;
  auto v = rocm_version(s);
  EXPECT_TRUE(v.has_value());
  EXPECT_EQ(v->major, 7u);
  EXPECT_EQ(v->minor, 10u);
  fs::remove_all(host);
}

TEST(RocmVersion_DriverOnlyHostHasNone) {
  std::string image = mktemp_dir(), host = mktemp_dir();
  put(image + "/opt/rocm/.info/version", "7.2.0\n");
  fs::mkdir_all(host + "/opt/containerd");
  VersionSources s;
  s.root = image;
  s.host_root = host;
  EXPECT_FALSE(rocm_version(s).has_value());  // never the image's version
  fs::remove_all(image);
  fs::remove_all(host);
}

TEST(RocmVersion_HostRootWithoutOptIsAMissingMount) {
  // --host-root set but the host's /opt not mounted there: an error (the
  // cycle fails), not a silent drop of amd.com/rocm.runtime.*.
  std::string image = mktemp_dir(), host = mktemp_dir();
  put(image + "/opt/rocm/.info/version", "7.2.0\n");
  VersionSources s;
  s.root = image;
  s.host_root = host;
  EXPECT_THROW_MSG(rocm_version(s), "has no opt/ directory");
  fs::remove_all(image);
  fs::remove_all(host);
}

TEST(RocmVersion_KeptOnlyWhileThePathToItIsUnchanged) {
  // The answer is kept across calls (fs::DirWatch on the directories the
  // lookup walked); every way a node's ROCm version changes is seen at the
  // next call: the file rewritten in place, replaced by a rename, the
  // symlink repointed, the target directory renamed away, the file removed
  // and created again.  Both lookups: a synthetic root and a host root.
  for (bool host_mode : {false, true}) {
    std::string d = mktemp_dir();
    put(d + "/opt/rocm-7.1.0/.info/version", "7.1.0\n");
    put(d + "/opt/rocm-7.2.0/.info/version", "7.2.0\n");
    link(host_mode ? "/opt/rocm-7.1.0" : "rocm-7.1.0", d + "/opt/rocm");
    VersionSources s;
    s.keep = true;  // a loop daemon's
    (host_mode ? s.host_root : s.root) = d;
    auto minor = [&] {
      auto v = rocm_version(s);
      return v ? static_cast<int>(v->minor) : -1;
    };
    for (int i = 0; i < 4; ++i) EXPECT_EQ(minor(), 1);  // kept from the third call on
    {
      std::ofstream f(d + "/opt/rocm-7.1.0/.info/version", std::ios::trunc);  // same inode
      f << "7.3.0\n";
    }
    EXPECT_EQ(minor(), 3);
    EXPECT_EQ(minor(), 3);
    put(d + "/opt/rocm-7.1.0/.info/version.new", "7.4.0\n");
    EXPECT_EQ(std::rename((d + "/opt/rocm-7.1.0/.info/version.new").c_str(),
                          (d + "/opt/rocm-7.1.0/.info/version").c_str()), 0);
    EXPECT_EQ(minor(), 4);
    EXPECT_EQ(minor(), 4);
    EXPECT_EQ(std::remove((d + "/opt/rocm").c_str()), 0);
    link(host_mode ? "/opt/rocm-7.2.0" : "rocm-7.2.0", d + "/opt/rocm");
    EXPECT_EQ(minor(), 2);
    EXPECT_EQ(minor(), 2);
    EXPECT_EQ(std::rename((d + "/opt/rocm-7.2.0").c_str(), (d + "/opt/old-7.2.0").c_str()), 0);
    EXPECT_EQ(minor(), host_mode ? 4 : -1);  // a host root falls back to the newest install left
    EXPECT_EQ(std::rename((d + "/opt/old-7.2.0").c_str(), (d + "/opt/rocm-7.2.0").c_str()), 0);
    EXPECT_EQ(minor(), 2);
    EXPECT_EQ(minor(), 2);
    EXPECT_EQ(std::remove((d + "/opt/rocm-7.2.0/.info/version").c_str()), 0);
    EXPECT_EQ(minor(), host_mode ? 4 : -1);
    EXPECT_EQ(minor(), host_mode ? 4 : -1);
    put(d + "/opt/rocm-7.2.0/.info/version", "7.5.0\n");
    EXPECT_EQ(minor(), 5);
    EXPECT_EQ(minor(), 5);
    fs::remove_all(d);
  }
}

TEST(DirWatch_SeesEntryChangesOnly) {
  std::string d = mktemp_dir();
  fs::mkdir_all(d + "/a");
  put(d + "/a/f", "1");
  fs::DirWatch w;
  EXPECT_FALSE(w.unchanged());  // nothing armed
  EXPECT_TRUE(w.arm({d, d + "/a"}));
  EXPECT_TRUE(w.unchanged());
  {
    std::ofstream f(d + "/a/f", std::ios::app);  // contents: not an entry change
    f << "2";
  }
  EXPECT_TRUE(w.unchanged());
  put(d + "/a/g", "x");  // an entry created
  EXPECT_FALSE(w.unchanged());
  EXPECT_FALSE(w.unchanged());  // disarmed until armed again
  EXPECT_TRUE(w.arm({d, d + "/a"}));
  EXPECT_TRUE(w.unchanged());
  EXPECT_EQ(std::rename((d + "/a").c_str(), (d + "/b").c_str()), 0);
  EXPECT_FALSE(w.unchanged());
  EXPECT_FALSE(w.arm({d + "/missing"}));
  EXPECT_FALSE(w.unchanged());
  // Two sets sharing a directory (one inotify watch): dropping one leaves
  // the other's watch in place.
  fs::mkdir_all(d + "/c");
  {
    fs::DirWatch x, y;
    EXPECT_TRUE(x.arm({d + "/c"}));
    EXPECT_TRUE(y.arm({d, d + "/c"}));
    EXPECT_TRUE(x.arm({d}));  // x leaves c
    EXPECT_TRUE(x.unchanged() && y.unchanged());
    put(d + "/c/h", "x");
    EXPECT_FALSE(y.unchanged());
    EXPECT_TRUE(x.unchanged());
  }
  fs::remove_all(d);
}

TEST(RocmVersion_ExplicitFileMustBeReadable) {
  std::string d = mktemp_dir();
  VersionSources s;
  s.rocm_version_file = d + "/version";
  EXPECT_THROW_MSG(rocm_version(s), "unable to read the ROCm version file");
  put(d + "/version", "not a version\n");
  EXPECT_THROW_MSG(rocm_version(s), "not X.Y[.Z]");
  put(d + "/version", "6.3.3\n");
  s.host_root = "/nonexistent";  // the explicit file wins
  EXPECT_EQ(rocm_version(s)->minor, 3u);
  fs::remove_all(d);
}

TEST(MockFixture_Loads) {
  auto m = mock_manager_from_node(yaml::parse(R"(
driverVersion: 6.8.5
runtimeVersion: "6.4"
devices:
- name: MOCKMODEL
  gfx: gfx942
  memoryMiB: 196592
  xgmiLinks: 7
  availableComputePartitions: [SPX, CPX]
- name: MOCKMODEL
  partitioned: true
  computePartition: CPX
  partitions:
  - name: cpx.1xcd.24gb
    attributes: {memory: 24576, xcds: 1}
  errors: {GetName: "injected"}
)"));
  EXPECT_EQ(m->devices.size(), static_cast<size_t>(2));
  EXPECT_EQ(m->driver_version, std::string("6.8.5"));
  EXPECT_EQ(m->runtime_version->minor, 4u);
  EXPECT_TRUE(m->devices[0]->IsPartitionCapable());
  EXPECT_EQ(m->devices[0]->GetGfxTarget().name(), std::string("gfx942"));
  EXPECT_EQ(m->devices[1]->GetPartitions()[0]->GetAttributes().at("memory"), std::string("24576"));
  EXPECT_THROW_MSG(m->devices[1]->GetName(), "injected");
}

TEST(Factory_ExplicitBackends) {
  config::Config c;
  c.flags.gfd.backend = "null";
  EXPECT_EQ(get_manager(c)->Name(), std::string("null"));
  c.flags.gfd.backend = "sysfs";
  EXPECT_EQ(get_manager(c)->Name(), std::string("sysfs"));
  c.flags.gfd.backend = "bogus";
  EXPECT_THROW_MSG(get_manager(c), "unknown backend 'bogus'");
  c.flags.gfd.backend = "mock";
  EXPECT_THROW_MSG(get_manager(c), "requires --mock-file");
  c.flags.gfd.backend = "amdsmi";
  c.flags.gfd.amdsmi_session = "sometimes";
  EXPECT_THROW_MSG(get_manager(c), "unknown amd-smi session mode");
}

TEST(Factory_FailOnInitErrorWrapsInFallback) {
  config::Config c;
  c.flags.gfd.backend = "null";
  c.flags.fail_on_init_error = false;
  EXPECT_TRUE(new_manager(c)->Name().rfind("fallback(", 0) == 0);
  c.flags.fail_on_init_error = true;
  EXPECT_EQ(new_manager(c)->Name(), std::string("null"));
}

TEST(Preference_FirstManagerThatInitialisesIsKeptUntilRebuilt) {
  auto a = std::make_shared<MockManager>();
  a->with_error_on_init("no driver");
  auto b = std::make_shared<MockManager>(std::vector<DevicePtr>{new_full_gpu()});
  PreferenceManager p({a, b});
  p.Init();
  EXPECT_EQ(p.chosen(), static_cast<size_t>(1));
  EXPECT_EQ(p.GetDevices().size(), static_cast<size_t>(1));
  p.Shutdown();
  // Init runs every cycle; the failed candidate is not retried.
  p.Init();
  EXPECT_EQ(a->init_calls, 1);
  EXPECT_EQ(b->init_calls, 2);
  EXPECT_EQ(b->shutdown_calls, 1);
}

TEST(Preference_PreferredManagerUsedWhenItInitialises) {
  auto a = std::make_shared<MockManager>(std::vector<DevicePtr>{new_full_gpu(), new_full_gpu()});
  auto b = std::make_shared<MockManager>();
  PreferenceManager p({a, b});
  p.Init();
  EXPECT_EQ(p.chosen(), static_cast<size_t>(0));
  EXPECT_EQ(p.GetDevices().size(), static_cast<size_t>(2));
  EXPECT_EQ(b->init_calls, 0);
}

TEST(Preference_EveryCandidateFailingIsAnInitError) {
  auto a = std::make_shared<MockManager>();
  a->with_error_on_init("no driver");
  auto b = std::make_shared<MockManager>();
  b->with_error_on_init("no topology");
  auto p = std::make_shared<PreferenceManager>(std::vector<ManagerPtr>{a, b});
  EXPECT_THROW_MSG(p->Init(), "mock: no driver; mock: no topology");
  // Without failOnInitError the daemon then labels with the Null manager.
  FallbackManager f(p);
  f.Init();
  EXPECT_TRUE(f.fell_back());
  EXPECT_EQ(f.Name(), std::string("fallback(null)"));
}

namespace {
// Cycles (Init, GetDevices, Shutdown) until the preferred manager is in use
// or 2 s passed; returns the device counts seen.
std::vector<size_t> cycle_until_warm(WarmStartManager& w) {
  std::vector<size_t> seen;
  for (int i = 0; i < 2000 && !w.warmed(); ++i) {
    w.Init();
    seen.push_back(w.GetDevices().size());
    w.Shutdown();
    usleep(1000);
  }
  return seen;
}
}  // namespace

TEST(WarmStart_FirstCycleFromQuickThenPreferred) {
  // Both describe the node alike: the preferred manager takes over.
  auto smi = std::make_shared<MockManager>(std::vector<DevicePtr>{new_full_gpu(), new_full_gpu()});
  auto kfd = std::make_shared<MockManager>(std::vector<DevicePtr>{new_full_gpu(), new_full_gpu()});
  WarmStartManager w(smi, kfd);
  cycle_until_warm(w);
  EXPECT_TRUE(w.warmed());
  EXPECT_TRUE(kfd->init_calls >= 1);  // the first cycle: the quick manager
  int kfd_inits = kfd->init_calls, smi_inits = smi->init_calls;
  w.Init();
  EXPECT_EQ(w.GetDevices().size(), static_cast<size_t>(2));
  w.Shutdown();
  w.Init();  // switched for good
  w.Shutdown();
  EXPECT_EQ(kfd->init_calls, kfd_inits);
  EXPECT_EQ(smi->init_calls, smi_inits + 2);
}

TEST(WarmStart_APreferredManagerThatDisagreesIsNotSwitchedTo) {
  // The quick manager's labels are published; the preferred one, ready,
  // describes the GPUs differently: the daemon keeps the quick one (its
  // labels do not change) until the next restart, and releases the other.
  auto smi = std::make_shared<MockManager>(std::vector<DevicePtr>{new_full_gpu(), new_full_gpu()});
  auto kfd = std::make_shared<MockManager>(std::vector<DevicePtr>{new_full_gpu()});
  {
    WarmStartManager w(smi, kfd);
    for (int i = 0; i < 300; ++i) {
      w.Init();
      EXPECT_EQ(w.GetDevices().size(), static_cast<size_t>(1));
      w.Shutdown();
      usleep(1000);
    }
    EXPECT_FALSE(w.warmed());
    EXPECT_EQ(smi->init_calls, 2);  // the warmer, and the second look before deciding
  }
  EXPECT_EQ(smi.use_count(), 1L);  // released at the decision, not kept warm
}

TEST(WarmStart_ADifferenceThatGoesAwayDoesNotDecide) {
  // The node changed between the warmer's snapshot and the published one (a
  // partition switch during start-up): the published labels said one GPU,
  // the warmer saw two, and now both managers see two.  The second look
  // finds them agreeing, and the preferred manager takes over.
  auto smi = std::make_shared<MockManager>(std::vector<DevicePtr>{new_full_gpu(), new_full_gpu()});
  auto kfd = std::make_shared<MockManager>(std::vector<DevicePtr>{new_full_gpu()});
  WarmStartManager w(smi, kfd);
  w.Init();  // starts the warmer; labels from kfd
  EXPECT_EQ(w.GetDevices().size(), static_cast<size_t>(1));
  w.Shutdown();
  usleep(300 * 1000);  // the warmer (the mock initialises at once) is done
  kfd->devices.push_back(new_full_gpu());  // the change reaches the quick manager too
  w.Init();  // decides: published 1 vs warmer 2, then 2 and 2 on the second look
  EXPECT_TRUE(w.warmed());
  EXPECT_EQ(smi->init_calls, 3);  // the warmer, the second look, then this cycle (read after Init joined the warmer)
  EXPECT_EQ(w.GetDevices().size(), static_cast<size_t>(2));
  w.Shutdown();
}

TEST(WarmStart_PrepareStartsThePreferredManagerBeforeTheFirstCycle) {
  // The daemon calls Prepare() when it builds the manager: the library's
  // initialisation runs during start-up, so the first cycle can already
  // use it; a second Prepare (or the first Init) starts no second warmer.
  auto smi = std::make_shared<MockManager>(std::vector<DevicePtr>{new_full_gpu(), new_full_gpu()});
  auto kfd = std::make_shared<MockManager>(std::vector<DevicePtr>{new_full_gpu()});
  WarmStartManager w(smi, kfd);
  w.Prepare();
  w.Prepare();
  usleep(300 * 1000);  // the mock initialises at once
  w.Init();
  EXPECT_TRUE(w.warmed());
  EXPECT_EQ(w.GetDevices().size(), static_cast<size_t>(2));
  w.Shutdown();
  EXPECT_EQ(smi->init_calls, 2);  // the warmer, then the first cycle
  EXPECT_EQ(kfd->init_calls, 0);
}

TEST(WarmStart_PreferredFailingInTheBackgroundKeepsQuick) {
  auto smi = std::make_shared<MockManager>();
  smi->with_error_on_init("no driver");
  auto kfd = std::make_shared<MockManager>(std::vector<DevicePtr>{new_full_gpu()});
  WarmStartManager w(smi, kfd);
  for (int i = 0; i < 50; ++i) {
    w.Init();
    EXPECT_EQ(w.GetDevices().size(), static_cast<size_t>(1));
    w.Shutdown();
    usleep(1000);
  }
  EXPECT_FALSE(w.warmed());
  EXPECT_EQ(smi->init_calls, 1);  // tried once, in the background; never retried
}

TEST(WarmStart_PreferredFailingLaterFallsBackForGood) {
  auto smi = std::make_shared<MockManager>(std::vector<DevicePtr>{new_full_gpu()});
  auto kfd = std::make_shared<MockManager>(std::vector<DevicePtr>{new_full_gpu()});
  WarmStartManager w(smi, kfd);
  cycle_until_warm(w);
  EXPECT_TRUE(w.warmed());
  smi->with_error_on_init("driver reloaded");
  int kfd_inits = kfd->init_calls;
  w.Init();
  EXPECT_EQ(w.GetDevices().size(), static_cast<size_t>(1));
  w.Shutdown();
  EXPECT_FALSE(w.warmed());
  EXPECT_EQ(kfd->init_calls, kfd_inits + 1);
  int smi_inits = smi->init_calls;
  w.Init();
  w.Shutdown();
  EXPECT_EQ(smi->init_calls, smi_inits);
}

TEST(WarmStart_DestructorWaitsForTheWarmer) {
  auto smi = std::make_shared<MockManager>();
  auto kfd = std::make_shared<MockManager>();
  {
    WarmStartManager w(smi, kfd);
    w.Init();
    w.Shutdown();
  }  // must not leave a running thread behind (TSan / std::terminate)
  EXPECT_EQ(smi->init_calls, 1);
}

namespace {
// A preferred manager whose Init blocks until released: a library wedged in
// its initialisation.
struct BlockingManager : MockManager {
  std::mutex mu;
  std::condition_variable cv;
  bool released = false, finished = false;
  void Init() override {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return released; });
  }
  void release() {
    std::lock_guard<std::mutex> lk(mu);
    released = true;
    cv.notify_all();
  }
};
}  // namespace

TEST(WarmStart_DestructorDoesNotWaitForeverForAWedgedInit) {
  auto smi = std::make_shared<BlockingManager>();
  auto kfd = std::make_shared<MockManager>(std::vector<DevicePtr>{new_full_gpu()});
  auto t0 = std::chrono::steady_clock::now();
  {
    WarmStartManager w(smi, kfd);
    w.teardown_wait_ms = 50;
    w.Init();
    EXPECT_EQ(w.GetDevices().size(), static_cast<size_t>(1));
    w.Shutdown();
  }  // SIGTERM / SIGHUP: the manager goes while the warmer is stuck
  auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
  EXPECT_TRUE(ms < 2000);
  smi->release();  // the detached warmer finishes on its own (it owns smi)
  for (int i = 0; i < 2000 && smi.use_count() > 1; ++i) usleep(1000);
  EXPECT_EQ(smi.use_count(), 1L);
}

TEST(WarmStart_ReloadWaitsForTheWedgedWarmerInsteadOfStartingAnother) {
  // a library init wedged while holding amd-smi's process-wide
  // lock; every SIGHUP used to start (and then abandon) one more warmer
  // blocked behind it.  Now a reloaded manager labels from the quick one
  // until the old warmer finishes, and only then starts its own.
  auto wedged = std::make_shared<BlockingManager>();
  auto kfd = std::make_shared<MockManager>(std::vector<DevicePtr>{new_full_gpu()});
  {
    WarmStartManager w(wedged, kfd);
    w.teardown_wait_ms = 20;
    w.Init();
    w.Shutdown();
  }  // SIGHUP: torn down with its warmer stuck
  EXPECT_TRUE(warmer_left_running());
  auto smi = std::make_shared<MockManager>(std::vector<DevicePtr>{new_full_gpu()});
  {
    WarmStartManager w2(smi, kfd);
    int kfd_inits = kfd->init_calls;
    for (int i = 0; i < 5; ++i) {  // reloads' cycles: no second warmer
      w2.Init();
      EXPECT_EQ(w2.GetDevices().size(), static_cast<size_t>(1));
      w2.Shutdown();
    }
    EXPECT_EQ(smi->init_calls, 0);
    EXPECT_EQ(kfd->init_calls, kfd_inits + 5);
    wedged->release();
    for (int i = 0; i < 2000 && warmer_left_running(); ++i) usleep(1000);
    EXPECT_FALSE(warmer_left_running());
    cycle_until_warm(w2);
    EXPECT_TRUE(w2.warmed());
    EXPECT_TRUE(smi->init_calls >= 2);  // its own warmer, then the cycle that switched
  }
  for (int i = 0; i < 2000 && wedged.use_count() > 1; ++i) usleep(1000);
  EXPECT_EQ(wedged.use_count(), 1L);
}

TEST(DeviceSummary_ShowsWhatTheLabelsDependOn) {
  auto a = device_summary({new_full_gpu()});
  EXPECT_EQ(a, device_summary({new_full_gpu()}));
  EXPECT_TRUE(a != device_summary({new_full_gpu(), new_full_gpu()}));
  EXPECT_TRUE(a.find("MOCKMODEL") != std::string::npos);
  EXPECT_TRUE(a.find("mem=300MiB") != std::string::npos);
}

TEST(AmdSmi_InitFailsCleanlyWithoutDriver) {
  // In the CPU container libamd_smi loads but there is no amdgpu driver:
  // amdsmi_init returns DRIVER_NOT_LOADED, which must surface as an Init error.
  std::string reason;
  if (std::getenv("GFD_AMDSMI_LIBRARY")) return;  // a substituted library (fake tests)
  if (!has_amdsmi(&reason)) return;  // library not installed: nothing to check
  if (fs::exists("/dev/kfd")) return;  // a real GPU node: covered by GPU tests
  AmdSmiManager m(AmdSmiOptions{});
  EXPECT_THROW_MSG(m.Init(), "amdsmi_init failed");
  EXPECT_EQ(m.init_count(), 0);
}

TEST(PciIds_NamesAndVirtualFunctions) {
  EXPECT_EQ(device_name(0x75a3), std::string("AMD Instinct MI355X"));
  EXPECT_EQ(device_name(0x1234), std::string("AMD-GPU-0x1234"));
  EXPECT_TRUE(is_mxgpu_vf(0x75b3));
  EXPECT_TRUE(is_mxgpu_vf(std::string("0x74B5\n")));
  EXPECT_FALSE(is_mxgpu_vf(0x75a3));
  EXPECT_FALSE(is_mxgpu_vf(std::string("garbage")));
}

TEST(Sysfs_HypervisorFlagFromFirstCpu) {
  Tree t;
  EXPECT_FALSE(running_in_vm(t.root));  // no /proc/cpuinfo under the root
  put(t.root + "/proc/cpuinfo", "processor\t: 0\nflags\t\t: fpu vme hypervisor lahf_lm\n\nprocessor\t: 1\n");
  EXPECT_TRUE(running_in_vm(t.root));
  put(t.root + "/proc/cpuinfo", "processor\t: 0\nflags\t\t: fpu vme hypervisorx\n");
  EXPECT_FALSE(running_in_vm(t.root));
  put(t.root + "/proc/cpuinfo", "processor\t: 0\nflags\t\t: fpu hypervisor\n");
  EXPECT_TRUE(running_in_vm(t.root));  // flag at the end of the line
}
