// amd-smi backend logic against a scriptable fake libamd_smi
// (tests/fake_amdsmi/fake_amdsmi.cpp).  These tests only run when
// GFD_AMDSMI_LIBRARY points at libfake_amdsmi.so (tests/test_unit_cpp.py
// runs them in a separate process); otherwise they return immediately.
//
// They cover what the pool cannot exercise on real hardware: compute-
// partitioned GPUs (CPX regrouping into physical GPUs under both partition
// address layouts, partition ordering),
// the persistent session's re-initialisation rules, stale handles and the
// market-name fallback.
#include <dlfcn.h>
#include <unistd.h>

#include <cstdlib>

#include "config/config.h"
#include "lm/resource.h"
#include "resource/amdsmi.h"
#include "resource/managers.h"
#include "resource/factory.h"
#include "test.h"
#include "util/fs.h"
#include "util/strings.h"
#include "util/trace.h"

using namespace gfd;
using namespace gfd::resource;

namespace {

struct Fake {
  int (*configure)(const char*) = nullptr;
  int (*init_calls)() = nullptr;
  int (*shutdown_calls)() = nullptr;
  int (*virt_calls)() = nullptr;
  long (*calls)(const char*) = nullptr;
  bool ok = false;

  Fake() {
    const char* lib = std::getenv("GFD_AMDSMI_LIBRARY");
    if (!lib || std::string(lib).find("fake") == std::string::npos) return;
    void* h = dlopen(lib, RTLD_NOW);
    // Asked for the fake but cannot load it: fail loudly rather than let
    // every fake-backed test pass vacuously.
    if (!h) throw std::runtime_error(std::string("cannot load fake amd-smi: ") + dlerror());
    configure = reinterpret_cast<int (*)(const char*)>(dlsym(h, "fake_amdsmi_configure"));
    init_calls = reinterpret_cast<int (*)()>(dlsym(h, "fake_amdsmi_init_calls"));
    shutdown_calls = reinterpret_cast<int (*)()>(dlsym(h, "fake_amdsmi_shutdown_calls"));
    virt_calls = reinterpret_cast<int (*)()>(dlsym(h, "fake_amdsmi_virt_calls"));
    calls = reinterpret_cast<long (*)(const char*)>(dlsym(h, "fake_amdsmi_calls"));
    ok = configure && init_calls && shutdown_calls && virt_calls && calls;
  }
};

Fake& fake() {
  static Fake f;
  return f;
}

const char* kTwoGpus =
    "bdf=0000:d9:00.0;mode=SPX;parts=1;cus=256;xcds=8;vram_mib=294896;links=7;virt=1\n"
    "bdf=0000:23:00.0;mode=CPX;parts=8;cus=32;xcds=1;vram_mib=36862;links=6;virt=1\n";

std::string temp_root() {
  char d[] = "/tmp/gfd-fake-XXXXXX";
  if (!mkdtemp(d)) throw std::runtime_error("mkdtemp");
  return d;
}

void set_generation(const std::string& root, const std::string& gen) {
  fs::mkdir_all(root + "/sys/class/kfd/kfd/topology");
  lm::write_file_atomically(root + "/sys/class/kfd/kfd/topology/generation_id", gen + "\n", 0644);
}

AmdSmiOptions opts(const std::string& root, bool persistent, const std::string& filter = "") {
  AmdSmiOptions o;
  o.root = root;
  o.persistent = persistent;
  o.filter = DeviceFilter::parse(filter);
  return o;
}

#define REQUIRE_FAKE() \
  if (!fake().ok) return

}  // namespace

TEST(AmdSmiFake_RegroupsCpxPartitionsByBdf) {
  REQUIRE_FAKE();
  fake().configure(kTwoGpus);
  std::string root = temp_root();
  AmdSmiManager m(opts(root, false));
  m.Init();
  auto devs = m.GetDevices();
  EXPECT_EQ(devs.size(), static_cast<size_t>(2));
  const auto& cpx = *devs[0];
  EXPECT_EQ(cpx.Info().bdf, std::string("0000:23:00.0"));
  EXPECT_TRUE(cpx.IsPartitioned());
  EXPECT_TRUE(cpx.IsPartitionCapable());  // from the accelerator profile table
  auto parts = cpx.GetPartitions();
  EXPECT_EQ(parts.size(), static_cast<size_t>(8));
  for (size_t i = 0; i < parts.size(); ++i) EXPECT_EQ(parts[i]->Info().partition_id, static_cast<int>(i));
  EXPECT_EQ(parts[0]->GetName(), std::string("cpx.1xcd.36gb"));
  auto attrs = parts[0]->GetAttributes();
  EXPECT_EQ(attrs.at("compute-units"), std::string("32"));
  // No KFD node (engines.dma) and no readable compute_partition_config
  // (decoder / jpeg) in this root: those attributes are unknown, not zero.
  EXPECT_EQ(attrs.count("engines.dma"), static_cast<size_t>(0));
  EXPECT_EQ(attrs.count("engines.decoder"), static_cast<size_t>(0));
  EXPECT_EQ(attrs.at("compute-partition"), std::string("CPX"));
  EXPECT_EQ(cpx.Info().compute_units, static_cast<uint32_t>(256));
  EXPECT_EQ(cpx.Info().xcds, static_cast<uint32_t>(8));
  EXPECT_EQ(cpx.GetTotalMemoryMiB(), static_cast<uint64_t>(8 * 36862));
  EXPECT_EQ(cpx.Info().xgmi_links, 6);

  const auto& spx = *devs[1];
  EXPECT_FALSE(spx.IsPartitioned());
  EXPECT_EQ(spx.GetName(), std::string("AMD Instinct MI355 OAM"));
  EXPECT_EQ(spx.GetGfxTarget().name(), std::string("gfx950"));
  EXPECT_EQ(spx.Info().xgmi_links, 7);
  EXPECT_EQ(spx.Info().virtualization, std::string("baremetal"));
  EXPECT_EQ(spx.Info().available_memory_partitions, (std::vector<std::string>{"NPS1", "NPS2"}));
  m.Shutdown();
  fs::remove_all(root);
}

TEST(AmdSmiFake_GenericMarketNameFallsBackToBoard) {
  REQUIRE_FAKE();
  fake().configure("bdf=0000:d9:00.0;name=AMD Radeon Graphics;board=AMD Instinct MI355X OAM\n");
  std::string root = temp_root();
  AmdSmiManager m(opts(root, false));
  m.Init();
  EXPECT_EQ(m.GetDevices()[0]->GetName(), std::string("AMD Instinct MI355X OAM"));
  m.Shutdown();
  fs::remove_all(root);
}

TEST(AmdSmiFake_UnpartitionedGpuValuesFromSysfs) {
  REQUIRE_FAKE();
  // The library's per-cycle value getters fail; an SPX GPU whose amdgpu
  // attributes are readable never needs them.
  const char* spec =
      "bdf=0000:d9:00.0;mode=SPX;parts=1;cus=256;xcds=8;vram_mib=294896;links=7;virt=1\n"
      "fail=amdsmi_get_gpu_memory_total:2\n"
      "fail=amdsmi_get_gpu_compute_partition:2\n"
      "fail=amdsmi_get_gpu_memory_partition:2\n";
  fake().configure(spec);
  std::string root = temp_root();
  std::string pci = root + "/sys/bus/pci/devices/0000:d9:00.0";
  fs::mkdir_all(pci);
  lm::write_file_atomically(pci + "/current_compute_partition", "SPX\n", 0644);
  lm::write_file_atomically(pci + "/current_memory_partition", "NPS1\n", 0644);
  lm::write_file_atomically(pci + "/mem_info_vram_total", "309220868096\n", 0644);
  std::string gen = root + "/sys/class/kfd/kfd/topology/generation_id";
  fs::mkdir_all(root + "/sys/class/kfd/kfd/topology");
  lm::write_file_atomically(gen, "1\n", 0644);
  AmdSmiManager m(opts(root, true));
  auto mode_read = [] {
    for (const auto& p : trace::phases())
      if (p.first == "compute_partition(read)") return true;
    return false;
  };
  for (int c = 0; c < 2; ++c) {
    m.Init();
    trace::begin_cycle();
    auto devs = m.GetDevices();
    // current_compute_partition (a register read that can wake the GPU) is
    // read by the session's first cycle only.
    EXPECT_EQ(mode_read(), c == 0);
    EXPECT_EQ(devs.size(), static_cast<size_t>(1));
    EXPECT_FALSE(devs[0]->IsPartitioned());
    EXPECT_EQ(devs[0]->GetTotalMemoryMiB(), static_cast<uint64_t>(294896));
    EXPECT_EQ(devs[0]->Info().compute_partition, std::string("SPX"));
    EXPECT_EQ(devs[0]->Info().memory_partition, std::string("NPS1"));
    EXPECT_EQ(devs[0]->Info().xcds, static_cast<uint32_t>(8));  // no KFD node: xcd counter
    EXPECT_EQ(devs[0]->GetName(), std::string("AMD Instinct MI355 OAM"));
    m.Shutdown();
  }
  // The values are the session's: a changed attribute without a new
  // topology generation (no real NPS switch leaves one) is not read again;
  // with one, the session re-initialises and reads it.
  lm::write_file_atomically(pci + "/current_memory_partition", "NPS2\n", 0644);
  m.Init();
  EXPECT_EQ(m.GetDevices()[0]->Info().memory_partition, std::string("NPS1"));
  m.Shutdown();
  lm::write_file_atomically(gen, "2\n", 0644);
  m.Init();
  EXPECT_EQ(m.GetDevices()[0]->Info().memory_partition, std::string("NPS2"));
  m.Shutdown();
  // The compute mode is read once per session: a changed attribute without
  // a new topology generation (which no real partition switch leaves) is
  // not read again.
  lm::write_file_atomically(pci + "/current_compute_partition", "CPX\n", 0644);
  m.Init();
  EXPECT_EQ(m.GetDevices()[0]->Info().compute_partition, std::string("SPX"));
  m.Shutdown();
  // With the generation a switch bumps: the session re-initialises and reads
  // the mode again.  Not SPX per sysfs: every value goes through the library
  // (whose injected failures then leave them unset).
  lm::write_file_atomically(gen, "3\n", 0644);
  m.Init();
  EXPECT_EQ(m.GetDevices()[0]->GetTotalMemoryMiB(), static_cast<uint64_t>(0));
  EXPECT_EQ(m.GetDevices()[0]->Info().compute_partition, std::string(""));
  m.Shutdown();
  fs::remove_all(root);
}

TEST(AmdSmiFake_PerCycleSessionInitsEveryWindow) {
  REQUIRE_FAKE();
  fake().configure(kTwoGpus);
  std::string root = temp_root();
  int i0 = fake().init_calls(), s0 = fake().shutdown_calls();
  {
    AmdSmiManager m(opts(root, false));
    for (int c = 0; c < 3; ++c) {
      m.Init();
      EXPECT_EQ(m.GetDevices().size(), static_cast<size_t>(2));
      m.Shutdown();
    }
    EXPECT_EQ(m.init_count(), 3);
  }
  EXPECT_EQ(fake().init_calls() - i0, 3);
  EXPECT_EQ(fake().shutdown_calls() - s0, 3);
  fs::remove_all(root);
}

TEST(AmdSmiFake_PersistentSessionInitsOnceAndReinitsOnTopologyChange) {
  REQUIRE_FAKE();
  fake().configure(kTwoGpus);
  std::string root = temp_root();
  set_generation(root, "7");
  int i0 = fake().init_calls(), s0 = fake().shutdown_calls();
  {
    AmdSmiManager m(opts(root, true));
    for (int c = 0; c < 3; ++c) {
      m.Init();
      m.GetDevices();
      m.Shutdown();
    }
    EXPECT_EQ(fake().init_calls() - i0, 1);
    EXPECT_EQ(fake().shutdown_calls() - s0, 0);
    // A partition-mode switch bumps the KFD generation: re-initialise.
    fake().configure("bdf=0000:d9:00.0;mode=DPX;parts=2;cus=128;xcds=4;vram_mib=147448\n");
    set_generation(root, "8");
    m.Init();
    auto devs = m.GetDevices();
    m.Shutdown();
    EXPECT_EQ(fake().init_calls() - i0, 2);
    EXPECT_EQ(devs.size(), static_cast<size_t>(1));
    EXPECT_EQ(devs[0]->GetPartitions().size(), static_cast<size_t>(2));
    EXPECT_EQ(devs[0]->GetPartitions()[0]->GetName(), std::string("dpx.4xcd.144gb"));
  }
  // Destroying the manager releases the library.
  EXPECT_EQ(fake().shutdown_calls() - s0, 2);
  fs::remove_all(root);
}

TEST(AmdSmiFake_UuidFromAsicSerial) {
  REQUIRE_FAKE();
  fake().configure(kTwoGpus);
  std::string root = temp_root();
  AmdSmiManager m(opts(root, true));
  m.Init();
  auto devs = m.GetDevices();
  m.Shutdown();
  // amd-smi's spelling (verified against `amd-smi list` on the pool).
  EXPECT_EQ(devs[1]->Info().bdf, std::string("0000:d9:00.0"));
  EXPECT_EQ(devs[1]->Info().uuid, std::string("3aff75a3-0000-1000-807c-178b7c5ed95c"));  // "0x..." serial
  EXPECT_EQ(devs[0]->Info().uuid, std::string("3aff75a3-0000-1000-807c-178b7c5e235c"));  // bare hex serial
  fs::remove_all(root);
}

TEST(AmdSmiFake_VirtualizationModeQueriedOncePerSession) {
  REQUIRE_FAKE();
  fake().configure(kTwoGpus);
  std::string root = temp_root();
  set_generation(root, "1");
  int v0 = fake().virt_calls();
  AmdSmiManager m(opts(root, true));
  for (int c = 0; c < 4; ++c) {
    m.Init();
    auto devs = m.GetDevices();
    m.Shutdown();
    EXPECT_EQ(devs[0]->Info().virtualization, std::string("baremetal"));
  }
  EXPECT_EQ(fake().virt_calls() - v0, 2);  // once per physical GPU
  // A driver reload (new KFD generation) starts a new session: query again.
  fake().configure("bdf=0000:d9:00.0;mode=SPX;parts=1;cus=256;xcds=8;vram_mib=294896;virt=3\n");
  set_generation(root, "2");
  m.Init();
  auto devs = m.GetDevices();
  m.Shutdown();
  EXPECT_EQ(fake().virt_calls() - v0, 3);
  EXPECT_EQ(devs[0]->Info().virtualization, std::string("guest"));
  // Per-cycle sessions query every cycle.
  AmdSmiManager pc(opts(root, false));
  for (int c = 0; c < 2; ++c) {
    pc.Init();
    pc.GetDevices();
    pc.Shutdown();
  }
  EXPECT_EQ(fake().virt_calls() - v0, 5);
  fs::remove_all(root);
}

TEST(AmdSmiFake_AsicIdentityQueriedOncePerSession) {
  // amdsmi_get_gpu_asic_info (market name, IDs, CUs, gfx target, serial):
  // once per processor per session - 1 + 8 processors here - not per cycle,
  // and again after a re-initialisation.
  REQUIRE_FAKE();
  fake().configure(kTwoGpus);
  std::string root = temp_root();
  set_generation(root, "1");
  long a0 = fake().calls("amdsmi_get_gpu_asic_info");
  AmdSmiManager m(opts(root, true));
  std::string first;
  for (int c = 0; c < 4; ++c) {
    m.Init();
    auto devs = m.GetDevices();
    m.Shutdown();
    std::string d = device_summary(devs);
    if (c == 0) first = d;
    EXPECT_EQ(d, first);  // the cached identity describes the GPUs the same way
    EXPECT_EQ(devs[1]->GetName(), devs[1]->Info().name);
  }
  EXPECT_EQ(fake().calls("amdsmi_get_gpu_asic_info") - a0, 9L);
  set_generation(root, "2");  // partition switch / driver reload: new session
  m.Init();
  m.GetDevices();
  m.Shutdown();
  EXPECT_EQ(fake().calls("amdsmi_get_gpu_asic_info") - a0, 18L);
  fs::remove_all(root);
}

TEST(AmdSmiFake_SupportedPartitionModesKeptWhileTheModesStay) {
  // Which partition modes a GPU supports is read once per session while its
  // current modes stay - not per cycle - and again after a re-initialisation.
  REQUIRE_FAKE();
  fake().configure(kTwoGpus);
  std::string root = temp_root();
  set_generation(root, "1");
  long m0 = fake().calls("amdsmi_get_gpu_memory_partition_config");
  long p0 = fake().calls("amdsmi_get_gpu_accelerator_partition_profile_config");
  AmdSmiManager m(opts(root, true));
  std::string first;
  for (int c = 0; c < 4; ++c) {
    m.Init();
    auto devs = m.GetDevices();
    m.Shutdown();
    std::string d;
    for (const auto& g : devs)
      d += str::join(g->Info().available_compute_partitions, ",") + "/" +
           str::join(g->Info().available_memory_partitions, ",") + ";";
    if (c == 0) first = d;
    EXPECT_EQ(d, first);
  }
  EXPECT_EQ(first, std::string("SPX,DPX,QPX,CPX/NPS1,NPS2;SPX,DPX,QPX,CPX/NPS1,NPS2;"));
  EXPECT_EQ(fake().calls("amdsmi_get_gpu_memory_partition_config") - m0, 2L);
  EXPECT_EQ(fake().calls("amdsmi_get_gpu_accelerator_partition_profile_config") - p0, 2L);
  set_generation(root, "2");  // partition switch / driver reload: new session
  m.Init();
  m.GetDevices();
  m.Shutdown();
  EXPECT_EQ(fake().calls("amdsmi_get_gpu_memory_partition_config") - m0, 4L);
  fs::remove_all(root);
}

TEST(AmdSmiFake_StaleHandlesTriggerOneReinit) {
  REQUIRE_FAKE();
  fake().configure((std::string(kTwoGpus) + "stale_after=5\n").c_str());
  std::string root = temp_root();
  int i0 = fake().init_calls();
  AmdSmiManager m(opts(root, true));
  m.Init();
  auto devs = m.GetDevices();  // first snapshot hits NOT_INIT midway -> re-init + retry
  EXPECT_EQ(devs.size(), static_cast<size_t>(2));
  EXPECT_EQ(fake().init_calls() - i0, 2);
  m.Shutdown();
  fs::remove_all(root);
}

TEST(AmdSmiFake_StaleHandlesAreFatalPerCycle) {
  REQUIRE_FAKE();
  fake().configure((std::string(kTwoGpus) + "stale_after=5\n").c_str());
  std::string root = temp_root();
  AmdSmiManager m(opts(root, false));
  m.Init();
  EXPECT_THROW_MSG(m.GetDevices(), "NOT_INIT");
  m.Shutdown();
  fs::remove_all(root);
}

TEST(AmdSmiFake_InitFailureSurfaces) {
  REQUIRE_FAKE();
  fake().configure("init_status=34\n");
  std::string root = temp_root();
  AmdSmiManager m(opts(root, true));
  EXPECT_THROW_MSG(m.Init(), "amdsmi_init failed: AMDSMI_STATUS_DRIVER_NOT_LOADED");
  fs::remove_all(root);
}

TEST(AmdSmiFake_AutoBackendFallsBackToSysfsWhenInitFails) {
  REQUIRE_FAKE();
  fake().configure("init_status=34\n");
  std::string root = temp_root();
  fs::mkdir_all(root + "/sys/class/kfd/kfd/topology/nodes");
  set_generation(root, "1");
  config::Config c;
  c.flags.gfd.backend = "auto";
  c.flags.gfd.sysfs_root = root;
  int i0 = fake().init_calls();
  auto m = get_manager(c);  // daemon mode: amd-smi initialises in the background
  for (int i = 0; i < 200; ++i) {
    m->Init();
    EXPECT_EQ(m->Name(), std::string("sysfs"));
    EXPECT_EQ(m->GetDevices().size(), static_cast<size_t>(0));
    m->Shutdown();
    usleep(1000);
  }
  EXPECT_EQ(fake().init_calls() - i0, 1);  // amd-smi is not retried every cycle
  fs::remove_all(root);
}

TEST(AmdSmiFake_AutoBackendSwitchesToAmdsmiOnceInitialised) {
  REQUIRE_FAKE();
  fake().configure(kTwoGpus);
  std::string root = temp_root();
  fs::mkdir_all(root + "/sys/class/kfd/kfd/topology/nodes");  // a KFD topology without GPUs
  set_generation(root, "1");
  config::Config c;
  c.flags.gfd.backend = "auto";
  c.flags.gfd.sysfs_root = root;
  auto m = get_manager(c);
  m->Init();
  EXPECT_EQ(m->Name(), std::string("sysfs"));  // the first cycle does not wait for amdsmi_init
  m->Shutdown();
  size_t n = 0;
  for (int i = 0; i < 2000 && n == 0; ++i) {
    usleep(1000);
    m->Init();
    n = m->GetDevices().size();
    m->Shutdown();
  }
  EXPECT_EQ(n, static_cast<size_t>(2));  // the fake's GPUs: amd-smi took over
  EXPECT_EQ(m->Name(), std::string("amdsmi(persistent)"));
  fs::remove_all(root);
}

TEST(AmdSmiFake_VisibleDevicesFilter) {
  REQUIRE_FAKE();
  fake().configure(kTwoGpus);
  std::string root = temp_root();
  AmdSmiManager m(opts(root, false, "1"));
  m.Init();
  auto devs = m.GetDevices();
  EXPECT_EQ(devs.size(), static_cast<size_t>(1));
  EXPECT_EQ(devs[0]->Info().bdf, std::string("0000:d9:00.0"));
  m.Shutdown();
  fs::remove_all(root);
}

TEST(AmdSmiFake_EightGpuNodeInParallel) {
  REQUIRE_FAKE();
  std::string spec;
  for (int i = 0; i < 8; ++i) spec += "bdf=0000:" + std::to_string(10 + i) + ":00.0;links=7\n";
  fake().configure(spec.c_str());
  std::string root = temp_root();
  AmdSmiManager m(opts(root, true));
  for (int c = 0; c < 20; ++c) {
    m.Init();
    EXPECT_EQ(m.GetDevices().size(), static_cast<size_t>(8));
    m.Shutdown();
  }
  fs::remove_all(root);
}

TEST(AmdSmiFake_SingleStrategyOverCpxNode) {
  REQUIRE_FAKE();
  fake().configure("bdf=0000:23:00.0;mode=CPX;parts=8;cus=32;xcds=1;vram_mib=36862\n"
                   "bdf=0000:24:00.0;mode=CPX;parts=8;cus=32;xcds=1;vram_mib=36862\n");
  std::string root = temp_root();
  AmdSmiManager m(opts(root, false));
  config::Config c;
  c.flags.mig_strategy = "single";
  m.Init();
  auto l = lm::NewResourceLabeler(m, c)->GetLabels();
  m.Shutdown();
  EXPECT_EQ(l["amd.com/gpu.count"], std::string("16"));
  EXPECT_EQ(l["amd.com/gpu.product"], std::string("AMD-Instinct-MI355-OAM-PARTITION-cpx.1xcd.36gb"));
  EXPECT_EQ(l["amd.com/gpu.memory"], std::string("36862"));
  EXPECT_EQ(l["amd.com/gpu.compute-units"], std::string("32"));
  EXPECT_EQ(l["amd.com/partition.strategy"], std::string("single"));
  fs::remove_all(root);
}

// ---- Partition layouts (resource/physical.h) --------------------------------
// Current kernels put the partition index in the PCI function bits of each
// partition's address (kfd_topology.c ORs the XCP node id into location_id);
// older ones give every partition the parent's address.  amd-smi groups
// processors into one socket per domain:bus:device; `sockets=one` checks the
// backend does not depend on that.  Every combination must label the same.

namespace {
const char* kLayouts[][2] = {{"partition_bdf=function", "sockets=slot"},
                             {"partition_bdf=function", "sockets=one"},
                             {"partition_bdf=shared", "sockets=slot"},
                             {"partition_bdf=shared", "sockets=one"}};

std::string with_layout(const char* const layout[2], const std::string& gpus) {
  return std::string(layout[0]) + "\n" + layout[1] + "\n" + gpus;
}

lm::Labels strategy_labels(const std::string& spec, const std::string& strategy, const std::string& root) {
  fake().configure(spec.c_str());
  AmdSmiManager m(opts(root, false));
  config::Config c;
  c.flags.mig_strategy = strategy;
  m.Init();
  auto l = lm::NewResourceLabeler(m, c)->GetLabels();
  m.Shutdown();
  return l;
}

const std::string kTwoCpx =
    "bdf=0000:23:00.0;mode=CPX;parts=8;cus=32;xcds=1;vram_mib=36862\n"
    "bdf=0000:24:00.0;mode=CPX;parts=8;cus=32;xcds=1;vram_mib=36862\n";
}  // namespace

TEST(AmdSmiFake_CpxSingleAndMixedUnderEveryLayout) {
  REQUIRE_FAKE();
  std::string root = temp_root();
  for (const auto& layout : kLayouts) {
    auto single = strategy_labels(with_layout(layout, kTwoCpx), "single", root);
    EXPECT_EQ(single["amd.com/gpu.count"], std::string("16"));
    EXPECT_EQ(single["amd.com/gpu.product"], std::string("AMD-Instinct-MI355-OAM-PARTITION-cpx.1xcd.36gb"));
    EXPECT_EQ(single["amd.com/gpu.memory"], std::string("36862"));
    auto mixed = strategy_labels(with_layout(layout, kTwoCpx), "mixed", root);
    EXPECT_EQ(mixed["amd.com/partition-cpx.1xcd.36gb.count"], std::string("16"));
    EXPECT_EQ(mixed["amd.com/gpu.count"], std::string("2"));
    EXPECT_EQ(mixed["amd.com/gpu.replicas"], std::string("0"));
  }
  fs::remove_all(root);
}

TEST(AmdSmiFake_PartitionAddressesAndParent) {
  REQUIRE_FAKE();
  fake().configure(("partition_bdf=function\n" + kTwoCpx).c_str());
  std::string root = temp_root();
  AmdSmiManager m(opts(root, false));
  m.Init();
  auto devs = m.GetDevices();
  EXPECT_EQ(devs.size(), static_cast<size_t>(2));
  EXPECT_EQ(devs[0]->Info().bdf, std::string("0000:23:00.0"));
  EXPECT_EQ(devs[1]->Info().bdf, std::string("0000:24:00.0"));
  auto parts = devs[1]->GetPartitions();
  EXPECT_EQ(parts.size(), static_cast<size_t>(8));
  for (size_t i = 0; i < parts.size(); ++i) {
    EXPECT_EQ(parts[i]->Info().partition_id, static_cast<int>(i));
    EXPECT_EQ(parts[i]->Info().bdf, "0000:24:00." + std::to_string(i));
    EXPECT_EQ(parts[i]->GetParent().get(), devs[1].get());
  }
  m.Shutdown();
  fs::remove_all(root);
}

TEST(AmdSmiFake_OnePartitionVisibleReadsParentAttributes) {
  REQUIRE_FAKE();
  // A pod allocated partition 3 of a CPX GPU: the one processor reports
  // 0000:23:00.3, which is not a PCI function; the GPU-wide attributes live
  // on 0000:23:00.0.
  std::string root = temp_root();
  std::string pci = root + "/sys/bus/pci/devices/0000:23:00.0";
  fs::mkdir_all(pci);
  lm::write_file_atomically(pci + "/device", "0x75a3\n", 0644);
  lm::write_file_atomically(pci + "/xgmi_num_links", "01 01 01 00 01 01 01 01\n", 0644);
  lm::write_file_atomically(pci + "/available_memory_partition", "NPS1, NPS2, NPS4\n", 0644);
  fake().configure("partition_bdf=function\nbdf=0000:23:00.0;mode=CPX;parts=8;cus=32;xcds=1;vram_mib=36862;visible=3\n");
  AmdSmiManager m(opts(root, false));
  m.Init();
  auto devs = m.GetDevices();
  EXPECT_EQ(devs.size(), static_cast<size_t>(1));
  EXPECT_EQ(devs[0]->Info().bdf, std::string("0000:23:00.0"));
  EXPECT_TRUE(devs[0]->IsPartitioned());
  EXPECT_EQ(devs[0]->Info().xgmi_links, 7);
  EXPECT_EQ(devs[0]->Info().available_memory_partitions, (std::vector<std::string>{"NPS1", "NPS2", "NPS4"}));
  auto parts = devs[0]->GetPartitions();
  EXPECT_EQ(parts.size(), static_cast<size_t>(1));
  EXPECT_EQ(parts[0]->Info().partition_id, 3);
  EXPECT_EQ(parts[0]->Info().bdf, std::string("0000:23:00.3"));
  m.Shutdown();
  config::Config c;
  c.flags.mig_strategy = "single";
  m.Init();
  auto l = lm::NewResourceLabeler(m, c)->GetLabels();
  m.Shutdown();
  EXPECT_EQ(l["amd.com/gpu.count"], std::string("1"));
  EXPECT_EQ(l["amd.com/gpu.product"], std::string("AMD-Instinct-MI355-OAM-PARTITION-cpx.1xcd.36gb"));
  fs::remove_all(root);
}

TEST(AmdSmiFake_PartitionedGpuValuesFromAttributesAndSessionCache) {
  REQUIRE_FAKE();
  // A CPX GPU whose parent function publishes its modes and whose 8 KFD
  // partition nodes (2..9) publish XCD/SDMA counts and memory: after the
  // first cycle no partition is queried through amd-smi any more (the
  // partition modes come from two parent attribute reads per cycle).
  std::string root = temp_root();
  set_generation(root, "1");
  std::string pci = root + "/sys/bus/pci/devices/0000:23:00.0";
  fs::mkdir_all(pci);
  lm::write_file_atomically(pci + "/device", "0x75a3\n", 0644);
  lm::write_file_atomically(pci + "/current_compute_partition", "CPX\n", 0644);
  lm::write_file_atomically(pci + "/current_memory_partition", "NPS1\n", 0644);
  for (int n = 2; n < 10; ++n) {
    std::string node = root + "/sys/class/kfd/kfd/topology/nodes/" + std::to_string(n);
    fs::mkdir_all(node + "/mem_banks/0");
    lm::write_file_atomically(node + "/properties", "simd_count 128\nnum_sdma_engines 1\nnum_xcc 1\n", 0644);
    lm::write_file_atomically(node + "/mem_banks/0/properties", "heap_type 1\nsize_in_bytes 38652608512\n", 0644);
  }
  fake().configure("bdf=0000:23:00.0;mode=CPX;parts=8;cus=32;xcds=1;vram_mib=36000;kfd_base=2\n");
  AmdSmiManager m(opts(root, true));
  for (int c = 0; c < 3; ++c) {
    m.Init();
    auto devs = m.GetDevices();
    EXPECT_EQ(devs.size(), static_cast<size_t>(1));
    auto parts = devs[0]->GetPartitions();
    EXPECT_EQ(parts.size(), static_cast<size_t>(8));
    EXPECT_EQ(parts[7]->Info().partition_id, 7);
    EXPECT_EQ(parts[0]->GetTotalMemoryMiB(), static_cast<uint64_t>(36862));  // the KFD node's share, not the library's
    EXPECT_EQ(parts[0]->GetAttributes().at("engines.dma"), std::string("1"));
    EXPECT_EQ(devs[0]->Info().compute_partition, std::string("CPX"));
    m.Shutdown();
  }
  // First cycle only: 8 for the partition facts, and 7 checking the addresses
  // of partitions 1-7, which are no PCI functions of this root (00.1-00.7).
  EXPECT_EQ(fake().calls("amdsmi_get_gpu_kfd_info"), 15L);
  EXPECT_EQ(fake().calls("amdsmi_get_gpu_memory_total"), 0L);
  EXPECT_EQ(fake().calls("amdsmi_get_gpu_compute_partition"), 0L);
  EXPECT_EQ(fake().calls("amdsmi_get_gpu_memory_partition"), 0L);
  fs::remove_all(root);
}

TEST(AmdSmiFake_DistinctGpusOnOneSlotStaySeparate) {
  REQUIRE_FAKE();
  // Two SR-IOV virtual functions a guest sees on one slot (ARI): different
  // ASIC serials and each a PCI function of its own, so two GPUs, not one
  // GPU with two partitions.
  fake().configure(
      "bdf=0000:05:00.0;mode=SPX;parts=1;serial=0x1111222233334444\n"
      "bdf=0000:05:00.1;mode=SPX;parts=1;serial=0x5555666677778888\n");
  std::string root = temp_root();
  for (const char* fn : {"0000:05:00.0", "0000:05:00.1"}) {
    fs::mkdir_all(root + "/sys/bus/pci/devices/" + fn);
    lm::write_file_atomically(root + "/sys/bus/pci/devices/" + fn + "/device", "0x75a3\n", 0644);
  }
  AmdSmiManager m(opts(root, false));
  m.Init();
  auto devs = m.GetDevices();
  EXPECT_EQ(devs.size(), static_cast<size_t>(2));
  EXPECT_FALSE(devs[0]->IsPartitioned());
  EXPECT_FALSE(devs[1]->IsPartitioned());
  EXPECT_EQ(devs[0]->Info().bdf, std::string("0000:05:00.0"));
  EXPECT_EQ(devs[1]->Info().bdf, std::string("0000:05:00.1"));
  m.Shutdown();
  fs::remove_all(root);
}

TEST(AmdSmiFake_PartitionsWithTheirOwnSerialsStayOneGpu) {
  REQUIRE_FAKE();
  // A kernel that gives every CPX partition its own ASIC serial: the
  // partitions (0000:05:00.1-7 are not PCI functions) are still one GPU.
  fake().configure("partition_serials=distinct\nbdf=0000:05:00.0;mode=CPX;parts=8;cus=32;xcds=1;vram_mib=36862\n");
  std::string root = temp_root();
  fs::mkdir_all(root + "/sys/bus/pci/devices/0000:05:00.0");
  lm::write_file_atomically(root + "/sys/bus/pci/devices/0000:05:00.0/device", "0x75a3\n", 0644);
  AmdSmiManager m(opts(root, false));
  m.Init();
  auto devs = m.GetDevices();
  EXPECT_EQ(devs.size(), static_cast<size_t>(1));
  EXPECT_TRUE(devs[0]->IsPartitioned());
  EXPECT_EQ(devs[0]->GetPartitions().size(), static_cast<size_t>(8));
  EXPECT_EQ(devs[0]->Info().bdf, std::string("0000:05:00.0"));
  m.Shutdown();
  fs::remove_all(root);
}

// ---- Fault injection: one amd-smi call failing with a chosen status ----

namespace {
std::vector<DevicePtr> devices_with(const std::string& spec, bool persistent = true) {
  fake().configure(spec.c_str());
  std::string root = temp_root();
  AmdSmiManager m(opts(root, persistent));
  m.Init();
  std::vector<DevicePtr> devs;
  try {
    devs = m.GetDevices();
  } catch (...) {
    m.Shutdown();
    fs::remove_all(root);
    throw;
  }
  m.Shutdown();
  fs::remove_all(root);
  return devs;
}
const std::string kOneGpu = "bdf=0000:d9:00.0;mode=SPX;parts=1;cus=256;xcds=8;vram_mib=294896;links=7;virt=1\n";
}  // namespace

TEST(AmdSmiFault_AsicInfoFailureIsAnError) {
  REQUIRE_FAKE();
  EXPECT_THROW_MSG(devices_with("fail=amdsmi_get_gpu_asic_info:7\n" + kOneGpu), "amdsmi_get_gpu_asic_info");
  // NOT_SUPPORTED (no libdrm_amdgpu) falls back to the KFD node; without a
  // readable node there is no identity either, and the call's error stands.
  EXPECT_THROW_MSG(devices_with("fail=amdsmi_get_gpu_asic_info:2\n" + kOneGpu), "AMDSMI_STATUS_NOT_SUPPORTED");
}

TEST(AmdSmiFault_ProcessorHandlesFailureIsAnError) {
  REQUIRE_FAKE();
  // Handle-table calls are checked too (processor type / BDF).
  EXPECT_THROW_MSG(devices_with("fail=amdsmi_get_gpu_device_bdf:10\n" + kOneGpu), "amdsmi_get_gpu_device_bdf");
}

TEST(AmdSmiFault_PersistentStaleStatusRetriesOnceThenFails) {
  REQUIRE_FAKE();
  int i0 = fake().init_calls();
  // NOT_INIT on every ASIC query: one re-initialisation, then the error.
  EXPECT_THROW_MSG(devices_with("fail=amdsmi_get_gpu_asic_info:32\n" + kOneGpu), "amdsmi_get_gpu_asic_info");
  EXPECT_EQ(fake().init_calls() - i0, 2);
}

TEST(AmdSmiFault_OptionalQueriesDegradeToUnknown) {
  REQUIRE_FAKE();
  // Facts the labels can do without: the device is still reported, the
  // affected labels are omitted (memory 0 -> no gpu.memory label, as in
  // the reference's resource.go:63).
  auto devs = devices_with("fail=amdsmi_get_gpu_memory_total:2\nfail=amdsmi_get_gpu_virtualization_mode:2\n"
                           "fail=amdsmi_get_gpu_compute_partition:2\n" + kOneGpu);
  EXPECT_EQ(devs.size(), static_cast<size_t>(1));
  const auto& i = devs[0]->Info();
  EXPECT_EQ(i.memory_mib, static_cast<uint64_t>(0));
  EXPECT_EQ(i.virtualization, std::string(""));
  EXPECT_EQ(i.compute_partition, std::string(""));
  EXPECT_FALSE(devs[0]->IsPartitioned());
  EXPECT_EQ(i.compute_units, static_cast<uint32_t>(256));
}

TEST(AmdSmiFault_KfdInfoFailureFallsBackToXcdCounter) {
  REQUIRE_FAKE();
  auto devs = devices_with("fail=amdsmi_get_gpu_kfd_info:2\n" + kOneGpu);
  EXPECT_EQ(devs[0]->Info().xcds, static_cast<uint32_t>(8));
}

TEST(AmdSmiFault_XgmiFallbackFailureLeavesLinksUnknown) {
  REQUIRE_FAKE();
  // No amdgpu xgmi table under the test root and the link-status query
  // fails: the link count is unknown (-1), not 0.
  auto devs = devices_with("fail=amdsmi_get_gpu_xgmi_link_status:2\n" + kOneGpu);
  EXPECT_EQ(devs[0]->Info().xgmi_links, -1);
}
