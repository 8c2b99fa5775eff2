// Partition-strategy tests.  Ports of internal/lm/mig-strategy_test.go
// (TestMigStrategyNoneLabels, TestMigStrategySingleLabels) plus mixed and
// error cases from cmd/gpu-feature-discovery/mig_test.go.
#include "lm/resource.h"
#include "partition/device_info.h"
#include "resource/managers.h"
#include "test.h"

using namespace gfd;
using lm::Labels;
using resource::new_full_gpu;
using resource::new_partition;
using resource::new_partitioned_gpu;

namespace {

config::Config strategy_config(const std::string& s, int replicas = 0) {
  config::Config c;
  c.flags.mig_strategy = s;
  if (replicas) {
    config::ReplicatedResource r;
    r.name = "amd.com/gpu";
    r.replicas = replicas;
    r.devices.all = true;
    c.sharing.time_slicing.resources.push_back(r);
  }
  return c;
}

Labels resource_labels(std::vector<resource::DevicePtr> devs, const config::Config& c) {
  resource::MockManager m(std::move(devs));
  return lm::NewResourceLabeler(m, c)->GetLabels();
}

Labels with(Labels base, const Labels& extra) {
  for (const auto& kv : extra) base[kv.first] = kv.second;
  return base;
}

const Labels kArch = {{"amd.com/gpu.family", "cdna4"},     {"amd.com/gpu.arch", "gfx950"},
                      {"amd.com/gpu.compute.major", "9"},  {"amd.com/gpu.compute.minor", "5"},
                      {"amd.com/gpu.compute-units", "256"}, {"amd.com/gpu.xcds", "8"}};

Labels gpu(const std::string& count, const std::string& replicas, const std::string& memory,
           const std::string& product) {
  return {{"amd.com/gpu.count", count},
          {"amd.com/gpu.replicas", replicas},
          {"amd.com/gpu.memory", memory},
          {"amd.com/gpu.product", product}};
}

Labels part_attrs(const std::string& mode, const std::string& xcds, const Labels& overrides = {}) {
  Labels l = {{"amd.com/gpu.compute-units", "0"},  {"amd.com/gpu.xcds", xcds},
              {"amd.com/gpu.engines.dma", "0"},    {"amd.com/gpu.engines.decoder", "0"},
              {"amd.com/gpu.engines.encoder", "0"}, {"amd.com/gpu.engines.jpeg", "0"},
              {"amd.com/gpu.compute-partition", mode}, {"amd.com/gpu.memory-partition", "NPS1"}};
  return with(l, overrides);
}

const Labels kSingle = {{"amd.com/partition.strategy", "single"}};
const Labels kInvalid = {{"amd.com/gpu.count", "0"},
                         {"amd.com/gpu.replicas", "0"},
                         {"amd.com/gpu.memory", "0"},
                         {"amd.com/gpu.product", "MOCKMODEL-PARTITION-INVALID"}};

}  // namespace

// ---- strategy none ----

TEST(StrategyNone_NoDevicesReturnsEmpty) { EXPECT_EQ(resource_labels({}, strategy_config("none")), Labels{}); }

TEST(StrategyNone_SingleFullGPU) {
  EXPECT_EQ(resource_labels({new_full_gpu()}, strategy_config("none")), with(gpu("1", "1", "300", "MOCKMODEL"), kArch));
}

TEST(StrategyNone_SharingAppliedToSingleDevice) {
  EXPECT_EQ(resource_labels({new_full_gpu()}, strategy_config("none", 2)),
            with(gpu("1", "2", "300", "MOCKMODEL-SHARED"), kArch));
}

TEST(StrategyNone_SharingAppliedToMultipleDevices) {
  EXPECT_EQ(resource_labels({new_full_gpu(), new_full_gpu()}, strategy_config("none", 2)),
            with(gpu("2", "2", "300", "MOCKMODEL-SHARED"), kArch));
}

TEST(StrategyNone_SharingNotAppliedToPartitionedDevice) {
  EXPECT_EQ(resource_labels({new_partitioned_gpu()}, strategy_config("none", 2)), gpu("1", "0", "300", "MOCKMODEL"));
}

TEST(StrategyNone_SharingNotAppliedToMultiplePartitionedDevices) {
  EXPECT_EQ(resource_labels({new_partitioned_gpu(), new_partitioned_gpu()}, strategy_config("none", 2)),
            gpu("2", "0", "300", "MOCKMODEL"));
}

TEST(StrategyNone_SharingAppliedToPartitionedAndFull) {
  EXPECT_EQ(resource_labels({new_partitioned_gpu(), new_full_gpu()}, strategy_config("none", 2)),
            with(gpu("2", "2", "300", "MOCKMODEL-SHARED"), kArch));
}

// ---- strategy single ----

TEST(StrategySingle_NoDevicesReturnsEmpty) { EXPECT_EQ(resource_labels({}, strategy_config("single")), Labels{}); }

TEST(StrategySingle_SingleFullGPUIsLikeNone) {
  EXPECT_EQ(resource_labels({new_full_gpu()}, strategy_config("single")),
            with(with(gpu("1", "1", "300", "MOCKMODEL"), kArch), kSingle));
}

TEST(StrategySingle_MultipleFullGPUsIsLikeNone) {
  EXPECT_EQ(resource_labels({new_full_gpu(), new_full_gpu()}, strategy_config("single")),
            with(with(gpu("2", "1", "300", "MOCKMODEL"), kArch), kSingle));
}

TEST(StrategySingle_SinglePartitionedGPU) {
  auto l = resource_labels({new_partitioned_gpu({new_partition("cpx", 1, 100)})}, strategy_config("single"));
  EXPECT_EQ(l, with(with(gpu("1", "1", "100", "MOCKMODEL-PARTITION-cpx.1xcd.100gb"), part_attrs("CPX", "1")), kSingle));
}

TEST(StrategySingle_MultiplePartitionedGPUs) {
  resource::Attributes over = {{"compute-units", "12"},   {"engines.dma", "13"}, {"engines.decoder", "14"},
                               {"engines.encoder", "15"}, {"engines.jpeg", "16"}};
  auto l = resource_labels({new_partitioned_gpu({new_partition("cpx", 1, 100, over)}),
                            new_partitioned_gpu({new_partition("cpx", 1, 100, over)})},
                           strategy_config("single"));
  Labels attrs = part_attrs("CPX", "1",
                            {{"amd.com/gpu.compute-units", "12"},
                             {"amd.com/gpu.engines.dma", "13"},
                             {"amd.com/gpu.engines.decoder", "14"},
                             {"amd.com/gpu.engines.encoder", "15"},
                             {"amd.com/gpu.engines.jpeg", "16"}});
  EXPECT_EQ(l, with(with(gpu("2", "1", "100", "MOCKMODEL-PARTITION-cpx.1xcd.100gb"), attrs), kSingle));
}

TEST(StrategySingle_EmptyPartitionedGPUIsInvalid) {
  EXPECT_EQ(resource_labels({new_partitioned_gpu()}, strategy_config("single")), with(kInvalid, kSingle));
}

TEST(StrategySingle_MixedProfilesIsInvalid) {
  auto l = resource_labels({new_partitioned_gpu({new_partition("cpx", 1, 100), new_partition("dpx", 4, 100)})},
                           strategy_config("single"));
  EXPECT_EQ(l, with(kInvalid, kSingle));
}

TEST(StrategySingle_PartitionedAndFullIsInvalid) {
  auto l = resource_labels({new_partitioned_gpu({new_partition("cpx", 1, 100)}), new_full_gpu()},
                           strategy_config("single"));
  EXPECT_EQ(l, with(with(kArch, kInvalid), kSingle));
}

TEST(StrategySingle_EnabledDisabledAndEmptyIsInvalid) {
  auto l = resource_labels(
      {new_partitioned_gpu({new_partition("cpx", 1, 100)}), new_full_gpu(), new_partitioned_gpu()},
      strategy_config("single"));
  EXPECT_EQ(l, with(with(kArch, kInvalid), kSingle));
}

// ---- strategy mixed ----

TEST(StrategyMixed_OneResourcePerProfile) {
  auto l = resource_labels({new_partitioned_gpu({new_partition("cpx", 1, 20), new_partition("qpx", 2, 5)})},
                           strategy_config("mixed"));
  EXPECT_EQ(l["amd.com/partition.strategy"], std::string("mixed"));
  EXPECT_EQ(l["amd.com/gpu.count"], std::string("1"));
  EXPECT_EQ(l["amd.com/gpu.replicas"], std::string("0"));
  EXPECT_EQ(l["amd.com/gpu.product"], std::string("MOCKMODEL"));
  EXPECT_EQ(l["amd.com/partition-cpx.1xcd.20gb.count"], std::string("1"));
  EXPECT_EQ(l["amd.com/partition-cpx.1xcd.20gb.product"], std::string("MOCKMODEL-PARTITION-cpx.1xcd.20gb"));
  EXPECT_EQ(l["amd.com/partition-cpx.1xcd.20gb.memory"], std::string("20"));
  EXPECT_EQ(l["amd.com/partition-qpx.2xcd.5gb.count"], std::string("1"));
  EXPECT_EQ(l["amd.com/partition-qpx.2xcd.5gb.xcds"], std::string("2"));
  EXPECT_EQ(l["amd.com/partition-qpx.2xcd.5gb.replicas"], std::string("1"));
}

TEST(StrategyMixed_CountsAcrossGPUs) {
  auto l = resource_labels({new_partitioned_gpu({new_partition("cpx", 1, 36), new_partition("cpx", 1, 36)}),
                            new_partitioned_gpu({new_partition("cpx", 1, 36), new_partition("cpx", 1, 36)})},
                           strategy_config("mixed"));
  EXPECT_EQ(l["amd.com/partition-cpx.1xcd.36gb.count"], std::string("4"));
  EXPECT_EQ(l["amd.com/gpu.count"], std::string("2"));
}

TEST(StrategyMixed_EmptyPartitionedDevicesIgnored) {
  auto l = resource_labels({new_partitioned_gpu()}, strategy_config("mixed"));
  EXPECT_EQ(l, with(gpu("1", "0", "300", "MOCKMODEL"), {{"amd.com/partition.strategy", "mixed"}}));
}

TEST(Strategy_UnknownErrorsOnlyWithDevices) {
  EXPECT_EQ(resource_labels({}, strategy_config("bogus")), Labels{});
  EXPECT_THROW_MSG(resource_labels({new_full_gpu()}, strategy_config("bogus")), "unknown strategy: bogus");
}

// ---- DeviceInfo (internal/mig/mig.go) ----

TEST(DeviceInfo_SplitsAndCaches) {
  resource::MockManager m({new_full_gpu(), new_partitioned_gpu({new_partition("cpx", 1, 36)}), new_partitioned_gpu()});
  partition::DeviceInfo di(m);
  EXPECT_EQ(di.GetDevicesWithPartitioningEnabled().size(), static_cast<size_t>(2));
  EXPECT_EQ(di.GetDevicesWithPartitioningDisabled().size(), static_cast<size_t>(1));
  EXPECT_TRUE(di.AnyPartitionedDeviceIsEmpty());
  EXPECT_EQ(di.GetAllPartitions().size(), static_cast<size_t>(1));
  EXPECT_EQ(m.get_devices_calls, 1);  // map built once
}

TEST(DeviceInfo_EmptySetIsEmptyByDefinition) {
  resource::MockManager m({new_full_gpu()});
  partition::DeviceInfo di(m);
  EXPECT_TRUE(di.AnyPartitionedDeviceIsEmpty());
}

TEST(DeviceInfo_IsPartitionedErrorPropagates) {
  auto d = new_full_gpu();
  d->mutable_info().errors["IsPartitioned"] = "driver gone";
  resource::MockManager m({d});
  partition::DeviceInfo di(m);
  EXPECT_THROW_MSG(di.GetDevicesMap(), "driver gone");
}

// Several GPUs of one model: the reference keeps the LAST device of each
// name in a map (mig-strategy.go:129-142), so its memory is what the labels
// report when same-named GPUs differ (e.g. after a RAS page retirement).
TEST(StrategyNone_LastDeviceOfAModelRepresentsIt) {
  auto a = new_full_gpu();
  auto b = new_full_gpu();
  a->mutable_info().memory_mib = 294896;
  b->mutable_info().memory_mib = 294880;  // 16 MiB retired
  Labels l = resource_labels({a, b}, strategy_config("none"));
  EXPECT_EQ(l["amd.com/gpu.count"], std::string("2"));
  EXPECT_EQ(l["amd.com/gpu.memory"], std::string("294880"));
  l = resource_labels({b, a}, strategy_config("none"));
  EXPECT_EQ(l["amd.com/gpu.memory"], std::string("294896"));
}
