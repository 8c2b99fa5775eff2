// Labeler unit tests.  Ports of internal/lm/resource_test.go:27-304 and
// internal/lm/nvml_test.go:11-77, re-expressed for the amd.com schema.
#include <fcntl.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <thread>

#include "lm/keys.h"
#include "lm/labels.h"
#include "lm/node.h"
#include "lm/resource.h"
#include "resource/managers.h"
#include "resource/versions.h"
#include "test.h"
#include "util/fs.h"
#include "util/trace.h"

using namespace gfd;
using lm::Labels;

namespace {

config::ReplicatedResource replicated(const std::string& name, int replicas, const std::string& rename = "") {
  config::ReplicatedResource r;
  r.name = name;
  r.rename = rename;
  r.replicas = replicas;
  r.devices.all = true;
  return r;
}

config::Config sharing_config(std::vector<config::ReplicatedResource> rs) {
  config::Config c;
  c.sharing.time_slicing.resources = std::move(rs);
  return c;
}

Labels full_gpu(const std::string& count, const std::string& replicas, const std::string& product) {
  return Labels{
      {"amd.com/gpu.count", count},          {"amd.com/gpu.replicas", replicas},
      {"amd.com/gpu.memory", "300"},         {"amd.com/gpu.product", product},
      {"amd.com/gpu.family", "cdna4"},       {"amd.com/gpu.arch", "gfx950"},
      {"amd.com/gpu.compute.major", "9"},    {"amd.com/gpu.compute.minor", "5"},
      {"amd.com/gpu.compute-units", "256"},  {"amd.com/gpu.xcds", "8"},
  };
}

Labels partition_labels(const std::string& res, const std::string& replicas, const std::string& product) {
  return Labels{
      {res + ".count", "1"},
      {res + ".replicas", replicas},
      {res + ".memory", "300"},
      {res + ".product", product},
      {res + ".compute-units", "0"},
      {res + ".xcds", "1"},
      {res + ".engines.dma", "0"},
      {res + ".engines.decoder", "0"},
      {res + ".engines.encoder", "0"},
      {res + ".engines.jpeg", "0"},
      {res + ".compute-partition", "CPX"},
      {res + ".memory-partition", "NPS1"},
  };
}

}  // namespace

TEST(GPUResourceLabeler_ZeroCountReturnsEmpty) {
  config::Config c;
  EXPECT_EQ(lm::NewGPUResourceLabels(&c, *resource::new_full_gpu(), 0), Labels{});
}

TEST(GPUResourceLabeler_NoSharing) {
  config::Config c;
  EXPECT_EQ(lm::NewGPUResourceLabels(&c, *resource::new_full_gpu(), 1), full_gpu("1", "1", "MOCKMODEL"));
}

TEST(GPUResourceLabeler_SharingIgnoresNonMatchingResource) {
  auto c = sharing_config({replicated("amd.com/not-gpu", 2)});
  EXPECT_EQ(lm::NewGPUResourceLabels(&c, *resource::new_full_gpu(), 1), full_gpu("1", "1", "MOCKMODEL"));
}

TEST(GPUResourceLabeler_SharedAppendsSuffix) {
  auto c = sharing_config({replicated("amd.com/gpu", 2)});
  EXPECT_EQ(lm::NewGPUResourceLabels(&c, *resource::new_full_gpu(), 1), full_gpu("1", "2", "MOCKMODEL-SHARED"));
}

TEST(GPUResourceLabeler_RenamedDoesNotAppendSuffix) {
  auto c = sharing_config({replicated("amd.com/gpu", 2, "amd.com/gpu.shared")});
  EXPECT_EQ(lm::NewGPUResourceLabels(&c, *resource::new_full_gpu(), 1), full_gpu("1", "2", "MOCKMODEL"));
}

TEST(GPUResourceLabeler_WithoutSharingHasZeroReplicas) {
  EXPECT_EQ(lm::NewGPUResourceLabelsWithoutSharing(*resource::new_full_gpu(), 2), full_gpu("2", "0", "MOCKMODEL"));
}

TEST(GPUResourceLabeler_ZeroMemoryOmitsMemoryLabel) {
  auto d = resource::new_full_gpu();
  d->mutable_info().memory_mib = 0;
  config::Config c;
  auto l = lm::NewGPUResourceLabels(&c, *d, 1);
  EXPECT_TRUE(l.find("amd.com/gpu.memory") == l.end());
}

TEST(GPUResourceLabeler_ProductNameIsSanitized) {
  auto d = resource::new_full_gpu();
  d->mutable_info().name = "AMD Instinct MI250X/MI250 (OAM)";
  config::Config c;
  auto l = lm::NewGPUResourceLabels(&c, *d, 1);
  EXPECT_EQ(l["amd.com/gpu.product"], std::string("AMD-Instinct-MI250X-MI250--OAM"));
}

TEST(GPUResourceLabeler_NameErrorIsWrapped) {
  auto d = resource::new_full_gpu();
  d->mutable_info().errors["GetName"] = "boom";
  config::Config c;
  EXPECT_THROW_MSG(lm::NewGPUResourceLabels(&c, *d, 1), "failed to get device model: boom");
}

TEST(GPUResourceLabeler_UnknownIsaOmitsArchLabels) {
  auto d = resource::new_full_gpu();
  d->mutable_info().gfx = {};
  config::Config c;
  auto l = lm::NewGPUResourceLabels(&c, *d, 1);
  EXPECT_TRUE(l.find("amd.com/gpu.family") == l.end());
  EXPECT_TRUE(l.find("amd.com/gpu.arch") == l.end());
  EXPECT_TRUE(l.find("amd.com/gpu.compute.major") == l.end());
}

TEST(ArchFamilyMapping) {
  using resource::arch_family;
  using resource::GfxTarget;
  EXPECT_EQ(arch_family(GfxTarget{9, 5, 0}), std::string("cdna4"));
  EXPECT_EQ(arch_family(GfxTarget{9, 4, 2}), std::string("cdna3"));
  EXPECT_EQ(arch_family(GfxTarget{9, 0, 10}), std::string("cdna2"));
  EXPECT_EQ(arch_family(GfxTarget{9, 0, 8}), std::string("cdna1"));
  EXPECT_EQ(arch_family(GfxTarget{9, 0, 6}), std::string("gcn5"));
  EXPECT_EQ(arch_family(GfxTarget{10, 3, 0}), std::string("rdna2"));
  EXPECT_EQ(arch_family(GfxTarget{11, 0, 0}), std::string("rdna3"));
  EXPECT_EQ(arch_family(GfxTarget{12, 0, 1}), std::string("rdna4"));
  EXPECT_EQ(arch_family(GfxTarget{8, 0, 3}), std::string("undefined"));
}

// ---- Partition resource labeler (resource_test.go TestMigResourceLabeler) ----

namespace {
resource::DevicePtr partition_under_parent() {
  auto p = resource::new_partition("cpx", 1, 300);
  static std::vector<std::shared_ptr<resource::SnapshotDevice>> keep;  // parents must outlive partitions
  keep.push_back(resource::new_partitioned_gpu({p}));
  return p;
}
}  // namespace

TEST(PartitionResourceLabeler_ZeroCountReturnsEmpty) {
  config::Config c;
  EXPECT_EQ(lm::NewPartitionResourceLabels("", &c, *partition_under_parent(), 0), Labels{});
}

TEST(PartitionResourceLabeler_NoSharing) {
  config::Config c;
  EXPECT_EQ(lm::NewPartitionResourceLabels("amd.com/gpu", &c, *partition_under_parent(), 1),
            partition_labels("amd.com/gpu", "1", "MOCKMODEL-PARTITION-cpx.1xcd.300gb"));
}

TEST(PartitionResourceLabeler_SharedAppendsSuffix) {
  auto c = sharing_config({replicated("amd.com/gpu", 2)});
  EXPECT_EQ(lm::NewPartitionResourceLabels("amd.com/gpu", &c, *partition_under_parent(), 1),
            partition_labels("amd.com/gpu", "2", "MOCKMODEL-PARTITION-cpx.1xcd.300gb-SHARED"));
}

TEST(PartitionResourceLabeler_RenamedDoesNotAppendSuffix) {
  auto c = sharing_config({replicated("amd.com/gpu", 2, "amd.com/gpu.shared")});
  EXPECT_EQ(lm::NewPartitionResourceLabels("amd.com/gpu", &c, *partition_under_parent(), 1),
            partition_labels("amd.com/gpu", "2", "MOCKMODEL-PARTITION-cpx.1xcd.300gb"));
}

TEST(PartitionResourceLabeler_MixedAppendsShared) {
  auto c = sharing_config({replicated("amd.com/gpu", 2, "amd.com/gpu.shared"),
                           replicated("amd.com/partition-cpx.1xcd.1gb", 2)});
  EXPECT_EQ(lm::NewPartitionResourceLabels("amd.com/partition-cpx.1xcd.1gb", &c, *partition_under_parent(), 1),
            partition_labels("amd.com/partition-cpx.1xcd.1gb", "2", "MOCKMODEL-PARTITION-cpx.1xcd.300gb-SHARED"));
}

TEST(PartitionResourceLabeler_MixedRenameDoesNotAppend) {
  auto c = sharing_config({replicated("amd.com/partition-cpx.1xcd.1gb", 2, "amd.com/partition-cpx.1xcd.1gb.shared")});
  EXPECT_EQ(lm::NewPartitionResourceLabels("amd.com/partition-cpx.1xcd.1gb", &c, *partition_under_parent(), 1),
            partition_labels("amd.com/partition-cpx.1xcd.1gb", "2", "MOCKMODEL-PARTITION-cpx.1xcd.300gb"));
}

TEST(PartitionResourceLabeler_OrphanPartitionErrors) {
  auto p = resource::new_partition("cpx", 1, 300);
  config::Config c;
  EXPECT_THROW_MSG(lm::NewPartitionResourceLabels("amd.com/gpu", &c, *p, 1), "failed to get parent of compute partition");
}

// ---- Capability labeler (nvml_test.go TestMigCapabilityLabeler) ----

namespace {
Labels capability(std::vector<resource::DevicePtr> devs) {
  resource::MockManager m(std::move(devs));
  return lm::NewPartitionCapabilityLabeler(m)->GetLabels();
}
}  // namespace

TEST(CapabilityLabeler_NoDevicesReturnsEmpty) { EXPECT_EQ(capability({}), Labels{}); }

TEST(CapabilityLabeler_SingleNonCapable) {
  EXPECT_EQ(capability({resource::new_full_gpu()}), (Labels{{"amd.com/gpu.partition.capable", "false"}}));
}

TEST(CapabilityLabeler_MultipleNonCapable) {
  EXPECT_EQ(capability({resource::new_full_gpu(), resource::new_full_gpu()}),
            (Labels{{"amd.com/gpu.partition.capable", "false"}}));
}

TEST(CapabilityLabeler_SingleCapable) {
  EXPECT_EQ(capability({resource::new_partitioned_gpu()}), (Labels{{"amd.com/gpu.partition.capable", "true"}}));
}

TEST(CapabilityLabeler_OneCapableAmongMany) {
  EXPECT_EQ(capability({resource::new_full_gpu(), resource::new_partitioned_gpu()}),
            (Labels{{"amd.com/gpu.partition.capable", "true"}}));
}

// ---- Version labeler (nvml.go:75-106) ----

TEST(VersionLabeler_ParsesDriverAndRuntime) {
  resource::MockManager m({resource::new_full_gpu()});
  m.driver_version = "6.18.54";
  m.runtime_version = {7, 2};
  EXPECT_EQ(lm::NewVersionLabeler(m)->GetLabels(), (Labels{{"amd.com/driver.major", "6"},
                                                            {"amd.com/driver.minor", "18"},
                                                            {"amd.com/driver.rev", "54"},
                                                            {"amd.com/rocm.runtime.major", "7"},
                                                            {"amd.com/rocm.runtime.minor", "2"}}));
}

TEST(VersionLabeler_TwoPartVersionHasEmptyRev) {
  resource::MockManager m({resource::new_full_gpu()});
  m.driver_version = "400.300";
  auto l = lm::NewVersionLabeler(m)->GetLabels();
  EXPECT_EQ(l["amd.com/driver.major"], std::string("400"));
  EXPECT_EQ(l["amd.com/driver.rev"], std::string(""));
}

TEST(VersionLabeler_RejectsBadFormat) {
  resource::MockManager m({resource::new_full_gpu()});
  m.driver_version = "1.2.3.4";
  EXPECT_THROW_MSG(lm::NewVersionLabeler(m), "does not match format \"X.Y[.Z]\"");
  m.driver_version = "garbage";
  EXPECT_THROW_MSG(lm::NewVersionLabeler(m), "does not match format");
}

TEST(VersionLabeler_RuntimeErrorPropagates) {
  resource::MockManager m({resource::new_full_gpu()});
  m.runtime_error = "no rocm";
  EXPECT_THROW_MSG(lm::NewVersionLabeler(m), "error getting ROCm runtime version: no rocm");
}

TEST(DriverVersion_BuiltinAndLoadableAmdgpu) {
  char d[] = "/tmp/gfd-drv-XXXXXX";
  if (!mkdtemp(d)) throw std::runtime_error("mkdtemp");
  std::string root = d;
  fs::mkdir_all(root + "/proc/sys/kernel");
  lm::write_file_atomically(root + "/proc/sys/kernel/osrelease", "6.18.54-ant.1\n", 0644);
  // Not loaded: the kernel release; asked again every time.
  EXPECT_EQ(resource::driver_version(root), std::string("6.18.54"));
  // Built in (parameters only): the kernel release, decided for good.
  fs::mkdir_all(root + "/sys/module/amdgpu/parameters");
  EXPECT_EQ(resource::driver_version(root), std::string("6.18.54"));
  lm::write_file_atomically(root + "/sys/module/amdgpu/version", "6.12.12\n", 0644);  // cannot happen without a reboot
  EXPECT_EQ(resource::driver_version(root), std::string("6.18.54"));
  // A loadable (DKMS) module: its version, re-read every time.
  std::string dkms = root + "/dkms";
  fs::mkdir_all(dkms + "/sys/module/amdgpu");
  lm::write_file_atomically(dkms + "/sys/module/amdgpu/initstate", "live\n", 0644);
  lm::write_file_atomically(dkms + "/sys/module/amdgpu/version", "6.12.12\n", 0644);
  EXPECT_EQ(resource::driver_version(dkms), std::string("6.12.12"));
  lm::write_file_atomically(dkms + "/sys/module/amdgpu/version", "6.14.3\n", 0644);
  EXPECT_EQ(resource::driver_version(dkms), std::string("6.14.3"));
  // An in-tree loadable module (no `version`): the kernel release; then the
  // module reloaded as a DKMS build (a new module directory): its version.
  std::string intree = root + "/intree";
  fs::mkdir_all(intree + "/proc/sys/kernel");
  lm::write_file_atomically(intree + "/proc/sys/kernel/osrelease", "6.18.54-ant.1\n", 0644);
  fs::mkdir_all(intree + "/sys/module/amdgpu");
  lm::write_file_atomically(intree + "/sys/module/amdgpu/initstate", "live\n", 0644);
  EXPECT_EQ(resource::driver_version(intree), std::string("6.18.54"));
  EXPECT_EQ(resource::driver_version(intree), std::string("6.18.54"));
  fs::remove_all(intree + "/sys/module/amdgpu");
  fs::mkdir_all(intree + "/sys/module/amdgpu");
  lm::write_file_atomically(intree + "/sys/module/amdgpu/initstate", "live\n", 0644);
  lm::write_file_atomically(intree + "/sys/module/amdgpu/version", "6.16.1\n", 0644);
  EXPECT_EQ(resource::driver_version(intree), std::string("6.16.1"));
  fs::remove_all(root);
}

// Facts read on the daemon's worker (file-backed managers) give the same
// labels and errors as asking the manager.
TEST(NodeFacts_PrefetchedVersionsMatchManager) {
  char d[] = "/tmp/gfd-facts-XXXXXX";
  if (!mkdtemp(d)) throw std::runtime_error("mkdtemp");
  std::string root = d;
  fs::mkdir_all(root + "/sys/module/amdgpu");
  lm::write_file_atomically(root + "/sys/module/amdgpu/version", "6.12.12\n", 0644);
  config::Config c;
  c.flags.gfd.machine_type_file = root + "/missing-dmi";
  resource::VersionSources src;
  src.root = root;
  lm::NodeFacts f = lm::ReadNodeFacts(c, src);
  EXPECT_TRUE(f.have_versions);
  EXPECT_EQ(f.driver_version, std::string("6.12.12"));
  EXPECT_FALSE(f.runtime_version.has_value());  // no opt/rocm/.info/version in this root
  EXPECT_TRUE(f.runtime_error.empty());         // ... which is not an error: no ROCm on the node
  EXPECT_EQ(f.machine, (Labels{{"amd.com/gpu.machine", "unknown"}}));
  EXPECT_TRUE(f.machine_warning.find("error getting machine type") != std::string::npos);
  resource::MockManager m({resource::new_full_gpu()});
  auto no_rocm = lm::NewDeviceLabeler(m, c, [&]() -> const lm::NodeFacts& { return f; })->GetLabels();
  EXPECT_EQ(no_rocm["amd.com/driver.major"], std::string("6"));
  EXPECT_EQ(no_rocm.count("amd.com/rocm.runtime.major"), static_cast<size_t>(0));
  // An explicitly configured version file that cannot be read is an error.
  resource::VersionSources bad = src;
  bad.rocm_version_file = root + "/nope";
  f = lm::ReadNodeFacts(c, bad);
  EXPECT_THROW_MSG(lm::NewDeviceLabeler(m, c, [&]() -> const lm::NodeFacts& { return f; }),
                   "error getting ROCm runtime version: unable to read the ROCm version file");
  fs::mkdir_all(root + "/opt/rocm/.info");
  lm::write_file_atomically(root + "/opt/rocm/.info/version", "7.2.0-43\n", 0644);
  f = lm::ReadNodeFacts(c, src);
  auto l = lm::NewDeviceLabeler(m, c, [&]() -> const lm::NodeFacts& { return f; })->GetLabels();
  EXPECT_EQ(l["amd.com/driver.minor"], std::string("12"));
  EXPECT_EQ(l["amd.com/rocm.runtime.major"], std::string("7"));
  EXPECT_EQ(l["amd.com/gpu.machine"], std::string("unknown"));
  // Without a version root the manager is asked (mock: 6.12.12 / 7.2).
  EXPECT_FALSE(lm::ReadNodeFacts(c, std::nullopt).have_versions);
  // Several labelers failing: the error reported is the first in the
  // reference's construction order (version before resources), although
  // the resource labeler is built first here.
  config::Config bogus = c;
  bogus.flags.mig_strategy = "bogus";
  EXPECT_THROW_MSG(lm::NewDeviceLabeler(m, bogus, [&]() -> const lm::NodeFacts& { return f; }),
                   "unknown strategy: bogus");
  f = lm::ReadNodeFacts(c, bad);
  EXPECT_THROW_MSG(lm::NewDeviceLabeler(m, bogus, [&]() -> const lm::NodeFacts& { return f; }),
                   "error getting ROCm runtime version: unable to read the ROCm version file");
  fs::remove_all(root);
}

// ---- Machine type / timestamp ----

TEST(MachineTypeLabeler_ReadsAndReplacesSpaces) {
  char tmpl[] = "/tmp/gfd-machine-XXXXXX";
  int fd = mkstemp(tmpl);
  const char content[] = "  WB SERVER E6-IS\n";
  EXPECT_TRUE(write(fd, content, sizeof(content) - 1) > 0);
  close(fd);
  auto l = lm::NewMachineTypeLabeler(tmpl)->GetLabels();
  unlink(tmpl);
  EXPECT_EQ(l["amd.com/gpu.machine"], std::string("WB-SERVER-E6-IS"));
}

TEST(MachineTypeLabeler_MissingFileIsUnknown) {
  EXPECT_EQ(lm::NewMachineTypeLabeler("/nonexistent/gfd/machine")->GetLabels(),
            (Labels{{"amd.com/gpu.machine", "unknown"}}));
  EXPECT_EQ(lm::NewMachineTypeLabeler("")->GetLabels(), (Labels{{"amd.com/gpu.machine", "unknown"}}));
}

TEST(TimestampLabeler_RespectsNoTimestamp) {
  config::Config c;
  EXPECT_EQ(lm::NewTimestampLabeler(c, 1234567890)->GetLabels(), (Labels{{"amd.com/gfd.timestamp", "1234567890"}}));
  c.flags.gfd.no_timestamp = true;
  EXPECT_EQ(lm::NewTimestampLabeler(c, 1234567890)->GetLabels(), Labels{});
}

// ---- Composition and writer (labels.go / list.go) ----

TEST(Merge_LaterLabelersOverride) {
  auto l = lm::merge({lm::from_labels({{"a", "1"}, {"b", "1"}}), lm::empty(), lm::from_labels({{"b", "2"}})})->GetLabels();
  EXPECT_EQ(l, (Labels{{"a", "1"}, {"b", "2"}}));
}

TEST(Render_IsSortedKeyValueLines) {
  EXPECT_EQ(lm::render({{"b", "2"}, {"a", "1"}}), std::string("a=1\nb=2\n"));
}

TEST(WriteToFile_ReusesFilesOnlyOnLocalFileSystems) {
  // A lease sees only this kernel's openers: reuse is allowed where every
  // reader is local (tmpfs here), not on other file systems (procfs stands
  // in for a network one: no lease there could see a remote reader).
  int shm = ::open("/dev/shm", O_RDONLY | O_DIRECTORY);
  EXPECT_TRUE(shm >= 0);
  EXPECT_TRUE(lm::reuse_is_safe(shm));
  ::close(shm);
  int proc = ::open("/proc/self/stat", O_RDONLY);
  EXPECT_TRUE(proc >= 0);
  EXPECT_FALSE(lm::reuse_is_safe(proc));
  ::close(proc);
  EXPECT_FALSE(lm::reuse_is_safe(-1));
}

TEST(WriteToFile_AtomicWithMode0644) {
  char dir[] = "/tmp/gfd-write-XXXXXX";
  EXPECT_TRUE(mkdtemp(dir) != nullptr);
  std::string path = std::string(dir) + "/gfd";
  lm::write_to_file({{"k", "v"}}, path);
  EXPECT_EQ(fs::read_file(path).data, std::string("k=v\n"));
  struct stat st;
  EXPECT_TRUE(stat(path.c_str(), &st) == 0);
  EXPECT_EQ(static_cast<int>(st.st_mode & 0777), 0644);
  EXPECT_TRUE(fs::is_dir(std::string(dir) + "/gfd-tmp"));
  EXPECT_EQ(fs::list_dir(std::string(dir) + "/gfd-tmp").size(), static_cast<size_t>(0));
  lm::remove_output_file(path);
  EXPECT_FALSE(fs::exists(path));
  EXPECT_FALSE(fs::exists(std::string(dir) + "/gfd-tmp"));
  fs::remove_all(dir);
}

TEST(WriteToFile_ReplaceKeepsExactContentsAndStaysFast) {
  // Every cycle after the first replaces the file (rename over it).  On ext4
  // that used to flush the new file inside rename(2) (~55 ms, auto_da_alloc);
  // the writer preallocates there.  Contents and size must stay exact when
  // the label set shrinks, and the median replace must stay far below that.
  char dir[] = "/tmp/gfd-write-XXXXXX";
  EXPECT_TRUE(mkdtemp(dir) != nullptr);
  std::string path = std::string(dir) + "/gfd";
  lm::write_to_file({{"k", std::string(5000, 'v')}}, path);
  std::vector<double> us;
  for (int i = 0; i < 9; ++i) {
    auto t0 = std::chrono::steady_clock::now();
    lm::write_to_file({{"k", std::to_string(i)}}, path);
    us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    EXPECT_EQ(fs::read_file(path).data, "k=" + std::to_string(i) + "\n");
  }
  struct stat st;
  EXPECT_TRUE(stat(path.c_str(), &st) == 0);
  EXPECT_EQ(static_cast<long>(st.st_size), 4L);
  std::sort(us.begin(), us.end());
  EXPECT_TRUE(us[us.size() / 2] < 5000.0);
  fs::remove_all(dir);
}

TEST(WriteToFile_UnwritableDirectoryErrors) {
  EXPECT_THROW_MSG(lm::write_to_file({{"k", "v"}}, "/proc/gfd-cannot-write/here/gfd"), "error atomically writing file");
}

TEST(WriteToFile_FailedWriteLeavesNoTemporaries) {
  // A write that fails part-way (here: the file size limit, EFBIG - as a
  // full disk gives ENOSPC) throws and removes gfd-tmp/, like the
  // reference's deferred cleanup (labels.go:81-96); the old file stays.
  char dir[] = "/tmp/gfd-write-XXXXXX";
  EXPECT_TRUE(mkdtemp(dir) != nullptr);
  std::string path = std::string(dir) + "/gfd";
  lm::write_to_file({{"k", "old"}}, path);
  struct rlimit old_limit;
  ::getrlimit(RLIMIT_FSIZE, &old_limit);
  struct rlimit small = old_limit;
  small.rlim_cur = 64;
  auto old_handler = ::signal(SIGXFSZ, SIG_IGN);
  ::setrlimit(RLIMIT_FSIZE, &small);
  std::string err;
  try {
    lm::write_to_file({{"k", std::string(4096, 'v')}}, path);
  } catch (const std::exception& e) {
    err = e.what();
  }
  ::setrlimit(RLIMIT_FSIZE, &old_limit);
  ::signal(SIGXFSZ, old_handler);
  EXPECT_TRUE(err.find("error writing temporary file") != std::string::npos);
  EXPECT_FALSE(fs::exists(std::string(dir) + "/gfd-tmp"));
  EXPECT_EQ(fs::read_file(path, 64).data, std::string("k=old\n"));
  fs::remove_all(dir);
}

TEST(WriteToFile_LoopWriteThatFailsKeepsTheOldFile) {
  // The rewrite of the kept file fails part-way (EFBIG): it is dropped, the
  // new file the write then tries fails the same way, the error is thrown
  // and the feature file keeps its old contents; the next write works.
  char dir[] = "/tmp/gfd-write-XXXXXX";
  EXPECT_TRUE(mkdtemp(dir) != nullptr);
  std::string path = std::string(dir) + "/gfd";
  lm::write_to_file({{"k", "a"}}, path, true);
  lm::write_to_file({{"k", "old"}}, path, true);
  struct rlimit old_limit;
  ::getrlimit(RLIMIT_FSIZE, &old_limit);
  struct rlimit small = old_limit;
  small.rlim_cur = 64;
  auto old_handler = ::signal(SIGXFSZ, SIG_IGN);
  ::setrlimit(RLIMIT_FSIZE, &small);
  std::string err;
  try {
    lm::write_to_file({{"k", std::string(4096, 'v')}}, path, true);
  } catch (const std::exception& e) {
    err = e.what();
  }
  ::setrlimit(RLIMIT_FSIZE, &old_limit);
  ::signal(SIGXFSZ, old_handler);
  EXPECT_TRUE(err.find("error writing temporary file") != std::string::npos);
  EXPECT_EQ(fs::read_file(path, 64).data, std::string("k=old\n"));
  lm::write_to_file({{"k", "new"}}, path, true);
  EXPECT_EQ(fs::read_file(path).data, std::string("k=new\n"));
  lm::remove_output_file(path);
  fs::remove_all(dir);
}

TEST(WriteToFile_RenameFailureLeavesNoTemporaries) {
  char dir[] = "/tmp/gfd-write-XXXXXX";
  EXPECT_TRUE(mkdtemp(dir) != nullptr);
  // The output path is a non-empty directory: rename(2) refuses it.
  std::string path = std::string(dir) + "/gfd";
  fs::mkdir_all(path + "/keep");
  EXPECT_THROW_MSG(lm::write_to_file({{"k", "v"}}, path), "error moving temporary file to");
  EXPECT_FALSE(fs::exists(std::string(dir) + "/gfd-tmp"));
  EXPECT_TRUE(fs::is_dir(path + "/keep"));
  fs::remove_all(dir);
}

TEST(WriteToFile_RecoversFromABlockedTemporaryDirectory) {
  char dir[] = "/tmp/gfd-write-XXXXXX";
  EXPECT_TRUE(mkdtemp(dir) != nullptr);
  std::string path = std::string(dir) + "/gfd";
  // A regular file where gfd-tmp/ belongs: that cycle fails and clears it,
  // the next one writes.
  EXPECT_TRUE(::close(::open((std::string(dir) + "/gfd-tmp").c_str(), O_CREAT | O_WRONLY, 0644)) == 0);
  EXPECT_THROW_MSG(lm::write_to_file({{"k", "v"}}, path), "fail to create temporary output file");
  EXPECT_FALSE(fs::exists(std::string(dir) + "/gfd-tmp"));
  lm::write_to_file({{"k", "v"}}, path);
  EXPECT_EQ(fs::read_file(path).data, std::string("k=v\n"));
  fs::remove_all(dir);
}

namespace {
// The daemon's loop-mode write.
void loop_write(const Labels& l, const std::string& path) { lm::write_to_file(l, path, true); }
// Files in gfd-tmp/: the kept (swapped-out) feature file.
std::vector<std::string> temp_files(const std::string& dir) {
  std::vector<std::string> out;
  for (const auto& n : fs::list_dir(dir + "/gfd-tmp")) out.push_back(dir + "/gfd-tmp/" + n);
  std::sort(out.begin(), out.end());
  return out;
}
ino_t inode(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0 ? st.st_ino : 0;
}
}  // namespace

TEST(WriteToFile_LoopWritesAlternateTwoFilesAndCreateNone) {
  // The first two loop writes create their files (the second swaps the
  // first out with RENAME_EXCHANGE); from then on each write rewrites the
  // file the previous one swapped out, so the feature file alternates
  // between two inodes and gfd-tmp/ holds exactly the other one.
  char dir[] = "/tmp/gfd-write-XXXXXX";
  EXPECT_TRUE(mkdtemp(dir) != nullptr);
  std::string path = std::string(dir) + "/gfd";
  loop_write({{"k", "0"}}, path);
  ino_t first = inode(path);
  EXPECT_EQ(temp_files(dir).size(), static_cast<size_t>(0));
  loop_write({{"k", "1"}}, path);
  ino_t second = inode(path);
  EXPECT_TRUE(second != first);
  EXPECT_EQ(temp_files(dir).size(), static_cast<size_t>(1));
  EXPECT_EQ(fs::read_file(temp_files(dir)[0]).data, std::string("k=0\n"));
  // Longer, shorter and equal contents: always exact.
  std::vector<std::string> vals{"2", std::string(3000, 'v'), "4", "5", "six", "7"};
  for (size_t i = 0; i < vals.size(); ++i) {
    trace::begin_cycle();
    loop_write({{"k", vals[i]}}, path);
    bool created = false;
    for (const auto& ph : trace::phases()) created |= ph.first == "write.create";
    EXPECT_FALSE(created);
    EXPECT_EQ(fs::read_file(path).data, "k=" + vals[i] + "\n");
    EXPECT_EQ(inode(path), i % 2 == 0 ? first : second);
    EXPECT_EQ(temp_files(dir).size(), static_cast<size_t>(1));
    struct stat st;
    EXPECT_TRUE(stat(path.c_str(), &st) == 0);
    EXPECT_EQ(static_cast<int>(st.st_mode & 0777), 0644);
    EXPECT_EQ(static_cast<size_t>(st.st_size), vals[i].size() + 3);
  }
  // Exit: nothing left behind.
  lm::remove_output_file(path);
  EXPECT_FALSE(fs::exists(std::string(dir) + "/gfd-tmp"));
  EXPECT_FALSE(fs::exists(path));
  fs::remove_all(dir);
}

TEST(WriteToFile_KeptFilesSignalALeaseBreakWithSIGURG) {
  // A reader whose open raced with an exchange can reach the kept file while
  // a write holds its lease; the kernel then signals the holder - SIGIO by
  // default, which terminates a process.  The kept files' descriptors signal
  // SIGURG, ignored by default.
  char dir[] = "/tmp/gfd-write-XXXXXX";
  EXPECT_TRUE(mkdtemp(dir) != nullptr);
  std::string path = std::string(dir) + "/gfd";
  loop_write({{"k", "1"}}, path);
  loop_write({{"k", "2"}}, path);
  int seen = 0, kept_fd = -1;
  std::string kept;
  for (const auto& n : fs::list_dir("/proc/self/fd")) {
    std::string target = fs::read_link("/proc/self/fd/" + n);
    if (target.rfind(std::string(dir) + "/", 0) != 0) continue;
    ++seen;
    EXPECT_EQ(::fcntl(std::atoi(n.c_str()), F_GETSIG), SIGURG);
    if (target.find("/gfd-tmp/") != std::string::npos) {
      kept_fd = std::atoi(n.c_str());
      kept = target;
    }
  }
  EXPECT_EQ(seen, 2);  // the feature file and the kept one
  // A lease break is survived: a write lease on the kept file's descriptor,
  // broken by another process opening the file (`cat`, which waits for the
  // release), signals this process with SIGURG - ignored.
  EXPECT_TRUE(kept_fd >= 0);
  EXPECT_EQ(::fcntl(kept_fd, F_SETLEASE, F_WRLCK), 0);
  pid_t pid = ::fork();
  if (pid == 0) {
    int null = ::open("/dev/null", O_WRONLY);
    ::dup2(null, 1);
    ::execlp("cat", "cat", kept.c_str(), static_cast<char*>(nullptr));
    ::_exit(127);
  }
  ::usleep(100 * 1000);  // the child's open is blocked on the lease meanwhile
  EXPECT_EQ(::fcntl(kept_fd, F_SETLEASE, F_UNLCK), 0);
  int status = 0;
  EXPECT_EQ(::waitpid(pid, &status, 0), pid);
  EXPECT_TRUE(WIFEXITED(status) && WEXITSTATUS(status) == 0);
  lm::remove_output_file(path);
  fs::remove_all(dir);
}

TEST(WriteToFile_AReaderOfTheOldFileKeepsItWhole) {
  // A reader that opened the feature file before a write still has it open
  // when the next write would rewrite it: the write lease is refused, so
  // that write leaves the file to the reader (unlinked) and creates a new
  // one.  The reader reads the old contents, whole.
  char dir[] = "/tmp/gfd-write-XXXXXX";
  EXPECT_TRUE(mkdtemp(dir) != nullptr);
  std::string path = std::string(dir) + "/gfd";
  loop_write({{"k", "a"}}, path);
  loop_write({{"k", "old"}}, path);
  int rfd = ::open(path.c_str(), O_RDONLY);
  EXPECT_TRUE(rfd >= 0);
  ino_t held = inode(path);
  loop_write({{"k", "new"}}, path);  // swaps the held file out
  trace::begin_cycle();
  loop_write({{"k", "newer"}}, path);  // would rewrite it: the reader still has it
  bool created = false;
  for (const auto& ph : trace::phases()) created |= ph.first == "write.create";
  EXPECT_TRUE(created);
  char buf[16] = {};
  EXPECT_EQ(::pread(rfd, buf, sizeof(buf) - 1, 0), static_cast<ssize_t>(6));
  EXPECT_EQ(std::string(buf), std::string("k=old\n"));
  struct stat st;
  EXPECT_TRUE(::fstat(rfd, &st) == 0);
  EXPECT_EQ(st.st_ino, held);
  EXPECT_EQ(static_cast<long>(st.st_nlink), 0L);  // unlinked, the reader's alone
  ::close(rfd);
  EXPECT_EQ(fs::read_file(path).data, std::string("k=newer\n"));
  EXPECT_EQ(temp_files(dir).size(), static_cast<size_t>(1));
  // With the reader gone, writes reuse again.
  trace::begin_cycle();
  loop_write({{"k", "last"}}, path);
  created = false;
  for (const auto& ph : trace::phases()) created |= ph.first == "write.create";
  EXPECT_FALSE(created);
  EXPECT_EQ(fs::read_file(path).data, std::string("k=last\n"));
  lm::remove_output_file(path);
  fs::remove_all(dir);
}

TEST(SweepTempDir_RemovesWhatACrashLeft) {
  char dir[] = "/tmp/gfd-write-XXXXXX";
  EXPECT_TRUE(mkdtemp(dir) != nullptr);
  std::string path = std::string(dir) + "/gfd", tmp = std::string(dir) + "/gfd-tmp";
  fs::mkdir_all(tmp + "/a");  // round-2 layout: subdirectories
  for (const char* n : {"/gfd-amd-abc123", "/a/gfd-def456"})
    EXPECT_TRUE(::close(::open((tmp + n).c_str(), O_CREAT | O_WRONLY, 0644)) == 0);
  lm::sweep_temp_dir(path);
  EXPECT_FALSE(fs::exists(tmp));
  // NVIDIA's GFD on the same node keeps its in-flight file there as
  // gfd-XXXXXX: a sweep leaves it (and so the directory) alone.
  fs::mkdir_all(tmp);
  for (const char* n : {"/gfd-amd-abc123", "/gfd-xyz789"})
    EXPECT_TRUE(::close(::open((tmp + n).c_str(), O_CREAT | O_WRONLY, 0644)) == 0);
  lm::sweep_temp_dir(path);
  EXPECT_FALSE(fs::exists(tmp + "/gfd-amd-abc123"));
  EXPECT_TRUE(fs::exists(tmp + "/gfd-xyz789"));
  fs::remove_all(tmp);
  lm::sweep_temp_dir(path);  // nothing there: fine
  lm::sweep_temp_dir("");    // stdout mode: nothing to do
  fs::remove_all(dir);
}

TEST(WriteToFile_ExchangeNeverSwapsADirectoryIntoTheTemporaryDirectory) {
  // Loop mode replaces the feature file with RENAME_EXCHANGE; a directory
  // where the feature file belongs must fail the write as rename(2) does
  // (EISDIR), stay where it is, and not be removed with gfd-tmp/ at exit.
  char dir[] = "/tmp/gfd-write-XXXXXX";
  EXPECT_TRUE(mkdtemp(dir) != nullptr);
  std::string path = std::string(dir) + "/gfd";
  loop_write({{"k", "1"}}, path);
  loop_write({{"k", "2"}}, path);
  EXPECT_TRUE(::unlink(path.c_str()) == 0);
  EXPECT_TRUE(::mkdir(path.c_str(), 0755) == 0);
  EXPECT_TRUE(::close(::open((path + "/keep").c_str(), O_CREAT | O_WRONLY, 0644)) == 0);
  EXPECT_THROW_MSG(loop_write({{"k", "3"}}, path), "error moving temporary file");
  EXPECT_TRUE(fs::exists(path + "/keep"));
  lm::release_kept_files();
  fs::remove_all(std::string(dir) + "/gfd-tmp");
  EXPECT_TRUE(fs::exists(path + "/keep"));
  fs::remove_all(dir);
}

TEST(WriteToFile_FeatureFileRemovedOrReplacedBetweenCycles) {
  char dir[] = "/tmp/gfd-write-XXXXXX";
  EXPECT_TRUE(mkdtemp(dir) != nullptr);
  std::string path = std::string(dir) + "/gfd";
  loop_write({{"k", "1"}}, path);
  loop_write({{"k", "2"}}, path);
  // Deleted since the last cycle: nothing to swap with, a plain rename.
  EXPECT_TRUE(::unlink(path.c_str()) == 0);
  loop_write({{"k", "3"}}, path);
  EXPECT_EQ(fs::read_file(path).data, std::string("k=3\n"));
  loop_write({{"k", "4"}}, path);
  EXPECT_EQ(fs::read_file(path).data, std::string("k=4\n"));
  // Replaced by someone else's file: it is swapped out and removed, as a
  // rename over it would; it is never rewritten.
  std::string other = std::string(dir) + "/other";
  {
    FILE* f = std::fopen(other.c_str(), "w");
    std::fputs("theirs\n", f);
    std::fclose(f);
  }
  ino_t theirs = inode(other);
  EXPECT_TRUE(::rename(other.c_str(), path.c_str()) == 0);
  loop_write({{"k", "5"}}, path);
  EXPECT_EQ(fs::read_file(path).data, std::string("k=5\n"));
  for (const auto& f : temp_files(dir)) EXPECT_TRUE(inode(f) != theirs);
  loop_write({{"k", "6"}}, path);
  loop_write({{"k", "7"}}, path);
  EXPECT_EQ(fs::read_file(path).data, std::string("k=7\n"));
  EXPECT_TRUE(temp_files(dir).size() <= static_cast<size_t>(1));
  lm::remove_output_file(path);
  EXPECT_FALSE(fs::exists(std::string(dir) + "/gfd-tmp"));
  EXPECT_FALSE(fs::exists(path));
  fs::remove_all(dir);
}

TEST(WriteToFile_KeptFileRemovedBetweenCycles) {
  // gfd-tmp/ emptied by someone else between two cycles: the write finds
  // its kept file gone (or, re-created, a different file under the name)
  // and writes through a new one.
  char dir[] = "/tmp/gfd-write-XXXXXX";
  EXPECT_TRUE(mkdtemp(dir) != nullptr);
  std::string path = std::string(dir) + "/gfd";
  loop_write({{"k", "1"}}, path);
  loop_write({{"k", "2"}}, path);
  EXPECT_EQ(temp_files(dir).size(), static_cast<size_t>(1));
  std::string kept = temp_files(dir)[0];
  fs::remove_all(std::string(dir) + "/gfd-tmp");
  loop_write({{"k", "3"}}, path);
  EXPECT_EQ(fs::read_file(path).data, std::string("k=3\n"));
  // Same name, different file.
  loop_write({{"k", "4"}}, path);
  kept = temp_files(dir)[0];
  EXPECT_TRUE(::unlink(kept.c_str()) == 0);
  {
    FILE* f = std::fopen(kept.c_str(), "w");
    std::fputs("stranger\n", f);
    std::fclose(f);
  }
  loop_write({{"k", "5"}}, path);
  EXPECT_EQ(fs::read_file(path).data, std::string("k=5\n"));
  EXPECT_EQ(fs::read_file(kept).data, std::string("stranger\n"));  // not ours: left alone
  ::unlink(kept.c_str());
  lm::remove_output_file(path);
  fs::remove_all(dir);
}

TEST(WriteToFile_KeptFilesOfEveryPathAreReleased) {
  char a[] = "/tmp/gfd-write-XXXXXX", b[] = "/tmp/gfd-write-XXXXXX";
  EXPECT_TRUE(mkdtemp(a) != nullptr && mkdtemp(b) != nullptr);
  std::string pa = std::string(a) + "/gfd", pb = std::string(b) + "/gfd";
  for (int i = 0; i < 3; ++i) {
    loop_write({{"k", "a" + std::to_string(i)}}, pa);
    loop_write({{"k", "b" + std::to_string(i)}}, pb);
  }
  EXPECT_EQ(temp_files(a).size(), static_cast<size_t>(1));
  EXPECT_EQ(temp_files(b).size(), static_cast<size_t>(1));
  EXPECT_EQ(fs::read_file(pa).data, std::string("k=a2\n"));
  EXPECT_EQ(fs::read_file(pb).data, std::string("k=b2\n"));
  // A session that ends: its kept files go, the feature files stay.
  lm::release_kept_files();
  EXPECT_EQ(temp_files(a).size(), static_cast<size_t>(0));
  EXPECT_EQ(temp_files(b).size(), static_cast<size_t>(0));
  EXPECT_EQ(fs::read_file(pa).data, std::string("k=a2\n"));
  fs::remove_all(a);
  fs::remove_all(b);
}

TEST(ReadFile_LongFileInFullOrCut) {
  // Files longer than a page (the procfs PCI table): contents and the
  // max_bytes cut must be exact.
  char dir[] = "/tmp/gfd-read-XXXXXX";
  EXPECT_TRUE(mkdtemp(dir) != nullptr);
  std::string p = std::string(dir) + "/big";
  std::string data;
  for (int i = 0; i < 20000; ++i) data += std::to_string(i) + "\n";
  {
    int fd = ::open(p.c_str(), O_CREAT | O_WRONLY, 0644);
    EXPECT_TRUE(fd >= 0 && ::write(fd, data.data(), data.size()) == static_cast<ssize_t>(data.size()));
    ::close(fd);
  }
  EXPECT_TRUE(fs::read_file(p, 4u << 20).data == data);
  EXPECT_TRUE(fs::read_file(p, 100000).data == data.substr(0, 100000));
  EXPECT_TRUE(fs::read_file(p, 4096).data == data.substr(0, 4096));
  EXPECT_TRUE(fs::read_file(p, 5000).data == data.substr(0, 5000));
  fs::remove_all(dir);
}

TEST(SanitizeLabelValue) {
  EXPECT_EQ(lm::sanitize_label_value("AMD Instinct MI355 OAM"), std::string("AMD-Instinct-MI355-OAM"));
  EXPECT_EQ(lm::sanitize_label_value("-x-"), std::string("x"));
  EXPECT_EQ(lm::sanitize_label_value(std::string(80, 'a')).size(), static_cast<size_t>(63));
  EXPECT_EQ(lm::sanitize_label_value(""), std::string(""));
}
