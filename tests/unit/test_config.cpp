// Config schema tests (vendored config/v1: config.go, replicas.go,
// resources.go, duration.go).
#include "config/config.h"
#include "test.h"
#include "util/duration.h"

using namespace gfd;
using namespace gfd::config;

TEST(Config_EmptyDocumentDefaultsToV1) {
  Config c = parse_config_text("");
  EXPECT_EQ(c.version, std::string("v1"));
  EXPECT_FALSE(c.flags.mig_strategy.has_value());
}

TEST(Config_KeysMatchIgnoringCaseLikeEncodingJson) {
  // The reference decodes through encoding/json, which takes a key that
  // equals a field's name ignoring case; the last such key wins.
  Config c = parse_config_text(
      "Version: v1\nFLAGS:\n  MigStrategy: single\n  migstrategy: mixed\n  Gfd:\n    SleepInterval: 5s\n"
      "Sharing:\n  timeslicing:\n    resources:\n    - name: amd.com/gpu\n      replicas: 4\n");
  EXPECT_EQ(c.mig_strategy(), std::string("mixed"));
  EXPECT_EQ(*c.flags.gfd.sleep_interval, parse_duration("5s"));
  EXPECT_EQ(c.sharing.time_slicing.resources.size(), static_cast<size_t>(1));
  EXPECT_EQ(c.sharing.time_slicing.resources[0].replicas, 4);
  EXPECT_EQ(parse_config_text("flags:\n  migStrategy: single\n  MIGSTRATEGY: mixed\n").mig_strategy(),
            std::string("mixed"));
  EXPECT_EQ(parse_config_text("flags:\n  MIGSTRATEGY: mixed\n  migStrategy: single\n").mig_strategy(),
            std::string("single"));
  // Not inside the bodies the reference decodes itself (TimeSlicing,
  // ReplicatedResource, Resource: exact map lookups).
  EXPECT_THROW_MSG(parse_config_text("sharing:\n  timeSlicing:\n    Resources:\n    - name: amd.com/gpu\n"
                                     "      replicas: 2\n"),
                   "no resources specified");
}

TEST(Config_UnknownVersionRejected) {
  EXPECT_THROW_MSG(parse_config_text("version: v2\n"), "unknown version: v2");
}

TEST(Config_FullFile) {
  Config c = parse_config_text(R"(
version: v1
flags:
  migStrategy: mixed
  failOnInitError: false
  gfd:
    oneshot: true
    noTimestamp: true
    sleepInterval: 1m30s
    outputFile: /tmp/out
    machineTypeFile: /tmp/mt
    backend: sysfs
    visibleDevices: "0-3"
sharing:
  timeSlicing:
    renameByDefault: true
    resources:
    - name: gpu
      replicas: 4
    - name: amd.com/partition-cpx.1xcd.36gb
      devices: [0, "1", "0:3"]
      replicas: 2
      rename: cpx-shared
)");
  EXPECT_EQ(*c.flags.mig_strategy, std::string("mixed"));
  EXPECT_EQ(*c.flags.fail_on_init_error, false);
  EXPECT_EQ(*c.flags.gfd.oneshot, true);
  EXPECT_EQ(*c.flags.gfd.sleep_interval, 90 * kSecond);
  EXPECT_EQ(*c.flags.gfd.output_file, std::string("/tmp/out"));
  EXPECT_EQ(c.backend(), std::string("sysfs"));
  EXPECT_EQ(c.visible_devices(), std::string("0-3"));
  const auto& rs = c.sharing.time_slicing.resources;
  EXPECT_EQ(rs.size(), static_cast<size_t>(2));
  EXPECT_EQ(rs[0].name, std::string("amd.com/gpu"));
  EXPECT_EQ(rs[0].rename, std::string("amd.com/gpu.shared"));  // renameByDefault
  EXPECT_TRUE(rs[0].devices.all);
  EXPECT_EQ(rs[1].rename, std::string("amd.com/cpx-shared"));
  EXPECT_EQ(rs[1].devices.list, (std::vector<std::string>{"0", "1", "0:3"}));
}

TEST(Config_FileSharedWithTheDevicePlugin) {
  // The reference README's config shared with the device plugin: the
  // plugin's keys are accepted (and dropped) ...
  Config c = parse_config_text(R"(
version: v1
flags:
  migStrategy: "none"
  failOnInitError: true
  nvidiaDriverRoot: "/"
  gdsEnabled: false
  plugin:
    passDeviceSpecs: false
    deviceListStrategy: "envvar"
    deviceIDStrategy: "uuid"
  gfd:
    oneshot: false
    noTimestamp: false
    outputFile: /etc/kubernetes/node-feature-discovery/features.d/gfd
    sleepInterval: 60s
)");
  EXPECT_TRUE(c.flags.plugin_present);
  EXPECT_EQ(*c.flags.gfd.sleep_interval, 60 * kSecond);
  EXPECT_EQ(c.mig_strategy(), std::string("none"));
  // ... and type-checked as the reference decodes them.
  EXPECT_THROW_MSG(parse_config_text("flags:\n  plugin:\n    passDeviceSpecs: sometimes\n"),
                   "Go struct field Config.flags.plugin.passDeviceSpecs of type bool");
  EXPECT_THROW_MSG(parse_config_text("flags:\n  plugin: [envvar]\n"),
                   "Go struct field Config.flags.plugin of type PluginCommandLineFlags");
  EXPECT_THROW_MSG(parse_config_text("flags:\n  mofedEnabled: 1\n"), "Config.flags.mofedEnabled of type bool");
  EXPECT_THROW_MSG(parse_config_text("flags:\n  nvidiaDriverRoot: {a: b}\n"),
                   "Config.flags.nvidiaDriverRoot of type string");
}

TEST(Config_JsonFile) {
  Config c = parse_config_text(R"({"version":"v1","flags":{"migStrategy":"single","gfd":{"sleepInterval":5000000000}}})");
  EXPECT_EQ(*c.flags.mig_strategy, std::string("single"));
  EXPECT_EQ(*c.flags.gfd.sleep_interval, 5 * kSecond);
}

TEST(Config_TypeErrors) {
  EXPECT_THROW_MSG(parse_config_text("flags:\n  failOnInitError: maybe\n"), "cannot unmarshal string into Go struct field");
  EXPECT_THROW_MSG(parse_config_text("flags:\n  gfd:\n    sleepInterval: forever\n"), "invalid duration");
  EXPECT_THROW_MSG(parse_config_text("flags: [1]\n"), "cannot unmarshal array");
}

TEST(Config_PlainScalarsAcceptedForStrings) {
  Config c = parse_config_text("flags:\n  migStrategy: 1\n");
  EXPECT_EQ(*c.flags.mig_strategy, std::string("1"));
}

TEST(Config_TimeSlicingValidation) {
  EXPECT_THROW_MSG(parse_config_text("sharing:\n  timeSlicing: {}\n"), "no resources specified");
  EXPECT_THROW_MSG(parse_config_text("sharing:\n  timeSlicing:\n    resources: []\n"), "no resources specified");
  EXPECT_THROW_MSG(parse_config_text("sharing:\n  timeSlicing:\n    resources:\n    - replicas: 2\n"),
                   "no resource name specified");
  EXPECT_THROW_MSG(parse_config_text("sharing:\n  timeSlicing:\n    resources:\n    - name: gpu\n"),
                   "no replicas specified");
  EXPECT_THROW_MSG(parse_config_text("sharing:\n  timeSlicing:\n    resources:\n    - name: gpu\n      replicas: 1\n"),
                   "number of replicas must be >= 2");
  EXPECT_THROW_MSG(
      parse_config_text("sharing:\n  timeSlicing:\n    resources:\n    - name: gpu\n      replicas: 2\n      devices: some\n"),
      "the only valid string input is 'all'");
  EXPECT_THROW_MSG(
      parse_config_text("sharing:\n  timeSlicing:\n    resources:\n    - name: gpu\n      replicas: 2\n      devices: 0\n"),
      "a count of devices must be > 0");
  EXPECT_THROW_MSG(parse_config_text(
                       "sharing:\n  timeSlicing:\n    resources:\n    - name: gpu\n      replicas: 2\n      devices: [x]\n"),
                   "unsupported type for device");
}

TEST(Config_IntegralFloatsAreIntegersLikeTheReferencesJson) {
  // sigs.k8s.io/yaml hands the reference's decoder JSON in which 2.0 is 2.
  auto devices = [](const std::string& v) {
    return parse_config_text("sharing:\n  timeSlicing:\n    resources:\n    - name: gpu\n      replicas: 2.0\n"
                             "      devices: " + v + "\n")
        .sharing.time_slicing.resources[0];
  };
  EXPECT_EQ(devices("2.0").devices.count, 2);
  EXPECT_EQ(devices("2.0").replicas, 2);
  EXPECT_EQ(devices("[1.0, 0]").devices.list, (std::vector<std::string>{"1", "0"}));
  EXPECT_THROW_MSG(devices("2.5"), "unrecognized type for devices spec");
  EXPECT_THROW_MSG(devices("[-1]"), "unsupported type for device");
}

TEST(Config_OutOfRangeNumbersAreTypeErrors) {
  // Found by tests/fuzz/fuzz_config.cpp: a float beyond the integer range
  // was converted with undefined behaviour, a large int silently truncated.
  auto replicas = [](const std::string& v) {
    return parse_config_text("sharing:\n  timeSlicing:\n    resources:\n    - name: gpu\n      replicas: " + v + "\n");
  };
  EXPECT_THROW_MSG(replicas("1e93"), "of type int");
  EXPECT_THROW_MSG(replicas("4294967298"), "of type int");
  EXPECT_THROW_MSG(replicas("2.5"), "of type int");
  EXPECT_EQ(replicas("4.0").sharing.time_slicing.resources[0].replicas, 4);
  EXPECT_THROW_MSG(parse_config_text("flags:\n  gfd:\n    sleepInterval: 1e300\n"), "invalid duration");
  EXPECT_EQ(*parse_config_text("flags:\n  gfd:\n    sleepInterval: 1.5e9\n").flags.gfd.sleep_interval, 1500000000LL);
}

TEST(Config_PartitionDeviceRefs) {
  auto devices = [](const std::string& items) {
    return parse_config_text("sharing:\n  timeSlicing:\n    resources:\n    - name: gpu\n      replicas: 2\n"
                             "      devices:\n" + items)
        .sharing.time_slicing.resources[0]
        .devices.list;
  };
  EXPECT_EQ(devices("      - PARTITION-GPU-3aff75a3-0000-1000-807c-178b7c5e4d5c/3\n"
                    "      - PARTITION-3aff75a3-0000-1000-807c-178b7c5e4d5c/0\n      - \"1:7\"\n")
                .size(),
            static_cast<size_t>(3));
  EXPECT_THROW_MSG(devices("      - PARTITION-nope/1\n"), "unsupported type for device");
  EXPECT_THROW_MSG(devices("      - PARTITION-GPU-3aff75a3-0000-1000-807c-178b7c5e4d5c/x\n"), "unsupported type for device");
  EXPECT_THROW_MSG(devices("      - \"1:x\"\n"), "unsupported type for device");
  EXPECT_THROW_MSG(devices("      - GPU-3aff75a3\n"), "unsupported type for device");
  EXPECT_THROW_MSG(devices("      - -1\n"), "unsupported type for device");
}

TEST(Config_DeviceRefsAcceptUuids) {
  Config c = parse_config_text(
      "sharing:\n  timeSlicing:\n    resources:\n    - name: gpu\n      replicas: 2\n      devices:\n"
      "      - GPU-3aff75a3-0000-1000-807c-178b7c5e4d5c\n      - 3aff75a3-0000-1000-807c-178b7c5e4d5c\n      - 3\n");
  EXPECT_EQ(c.sharing.time_slicing.resources[0].devices.list.size(), static_cast<size_t>(3));
  Config c2 = parse_config_text("sharing:\n  timeSlicing:\n    resources:\n    - name: gpu\n      replicas: 2\n      devices: 2\n");
  EXPECT_EQ(c2.sharing.time_slicing.resources[0].devices.count, 2);
}

TEST(Config_ResourcesSection) {
  Config c = parse_config_text("resources:\n  gpus:\n  - pattern: '*MI355*'\n    name: mi355\n");
  EXPECT_EQ(c.resources.gpus.size(), static_cast<size_t>(1));
  EXPECT_EQ(c.resources.gpus[0].name, std::string("amd.com/mi355"));
  EXPECT_THROW_MSG(parse_config_text("resources:\n  gpus:\n  - name: x\n"), "must have a 'pattern' field set");
}

TEST(ResourceName_PrefixAndValidation) {
  EXPECT_EQ(new_resource_name("gpu"), std::string("amd.com/gpu"));
  EXPECT_EQ(new_resource_name("amd.com/gpu.shared"), std::string("amd.com/gpu.shared"));
  EXPECT_THROW_MSG(new_resource_name("Bad_Name"), "incorrect format for resource name");
  EXPECT_THROW_MSG(new_resource_name(std::string(60, 'a')), "must be 63 characters or less");
  EXPECT_EQ(default_shared_rename("amd.com/gpu"), std::string("amd.com/gpu.shared"));
}

TEST(DisableResourceRenaming) {
  Config c = parse_config_text(
      "resources:\n  gpus:\n  - pattern: x\n    name: y\nsharing:\n  timeSlicing:\n    resources:\n    - name: gpu\n"
      "      replicas: 2\n      rename: foo\n      devices: [0]\n");
  disable_resource_renaming(c);
  EXPECT_TRUE(c.resources.gpus.empty());
  EXPECT_EQ(c.sharing.time_slicing.resources[0].rename, std::string(""));
  EXPECT_TRUE(c.sharing.time_slicing.resources[0].devices.all);
  EXPECT_TRUE(c.sharing.time_slicing.resources[0].devices.list.empty());
}

TEST(DisableResourceRenaming_RenameByDefaultForcesDefault) {
  Config c = parse_config_text(
      "sharing:\n  timeSlicing:\n    renameByDefault: true\n    resources:\n    - name: gpu\n      replicas: 2\n"
      "      rename: custom\n");
  disable_resource_renaming(c);
  EXPECT_EQ(c.sharing.time_slicing.resources[0].rename, std::string("amd.com/gpu.shared"));
}

TEST(Config_JsonDumpRoundTrips) {
  Config c = parse_config_text("flags:\n  migStrategy: single\n  gfd:\n    sleepInterval: 90s\n");
  std::string js = to_json(c);
  EXPECT_TRUE(js.find("\"migStrategy\": \"single\"") != std::string::npos);
  EXPECT_TRUE(js.find("\"sleepInterval\": \"1m30s\"") != std::string::npos);
  Config back = parse_config_text(js);
  EXPECT_EQ(*back.flags.gfd.sleep_interval, 90 * kSecond);
}

TEST(Config_JsonDumpOfResourcesAndSharingRoundTrips) {
  // The start-up "Running with config" dump (the reference marshals its
  // whole Config) must load back as the same resources and sharing.
  Config c = parse_config_text(R"(
resources:
  gpus:
  - pattern: '*MI355*'
    name: mi355
  mig:
  - pattern: 'cpx.*'
    name: cpx
sharing:
  timeSlicing:
    failRequestsGreaterThanOne: true
    resources:
    - name: gpu
      replicas: 4
    - name: amd.com/partition-cpx.1xcd.36gb
      devices: 3
      replicas: 2
      rename: cpx-shared
    - name: mi355
      devices: [0, "1:3"]
      replicas: 8
)");
  Config back = parse_config_text(to_json(c));
  EXPECT_EQ(back.resources.gpus.size(), static_cast<size_t>(1));
  EXPECT_EQ(back.resources.gpus[0].pattern, std::string("*MI355*"));
  EXPECT_EQ(back.resources.gpus[0].name, std::string("amd.com/mi355"));
  EXPECT_EQ(back.resources.partitions.size(), static_cast<size_t>(1));
  EXPECT_EQ(back.resources.partitions[0].name, std::string("amd.com/cpx"));
  const auto& t = back.sharing.time_slicing;
  EXPECT_TRUE(t.fail_requests_greater_than_one);
  EXPECT_FALSE(t.rename_by_default);
  EXPECT_EQ(t.resources.size(), static_cast<size_t>(3));
  EXPECT_TRUE(t.resources[0].devices.all);
  EXPECT_EQ(t.resources[0].replicas, 4);
  EXPECT_EQ(t.resources[1].devices.count, 3);
  EXPECT_EQ(t.resources[1].rename, std::string("amd.com/cpx-shared"));
  EXPECT_EQ(t.resources[2].devices.list, (std::vector<std::string>{"0", "1:3"}));
  EXPECT_EQ(t.resources[2].replicas, 8);
  // renameByDefault survives too.
  Config d = parse_config_text("sharing:\n  timeSlicing:\n    renameByDefault: true\n    resources:\n"
                               "    - name: gpu\n      replicas: 2\n");
  EXPECT_TRUE(parse_config_text(to_json(d)).sharing.time_slicing.rename_by_default);
}

TEST(Duration_ParseGoGrammar) {
  EXPECT_EQ(parse_duration("60s"), 60 * kSecond);
  EXPECT_EQ(parse_duration("1m30s"), 90 * kSecond);
  EXPECT_EQ(parse_duration("1.5h"), static_cast<Nanos>(5400) * kSecond);
  EXPECT_EQ(parse_duration("500ms"), 500 * kMillisecond);
  EXPECT_EQ(parse_duration("2us"), static_cast<Nanos>(2000));
  EXPECT_EQ(parse_duration("2\xC2\xB5s"), static_cast<Nanos>(2000));
  EXPECT_EQ(parse_duration("-1s"), -kSecond);
  EXPECT_EQ(parse_duration("0"), static_cast<Nanos>(0));
  EXPECT_EQ(parse_duration(".5s"), kSecond / 2);
  EXPECT_THROW_MSG(parse_duration(""), "invalid duration");
  EXPECT_THROW_MSG(parse_duration("10"), "missing unit");
  EXPECT_THROW_MSG(parse_duration("10d"), "unknown unit");
  EXPECT_THROW_MSG(parse_duration("s"), "invalid duration");
}

TEST(Duration_FormatGoStyle) {
  EXPECT_EQ(format_duration(60 * kSecond), std::string("1m0s"));
  EXPECT_EQ(format_duration(90 * kSecond), std::string("1m30s"));
  EXPECT_EQ(format_duration(3600 * kSecond), std::string("1h0m0s"));
  EXPECT_EQ(format_duration(1500 * kMillisecond), std::string("1.5s"));
  EXPECT_EQ(format_duration(500 * kMillisecond), std::string("500ms"));
  EXPECT_EQ(format_duration(1500), std::string("1.5\xC2\xB5s"));
  EXPECT_EQ(format_duration(7), std::string("7ns"));
  EXPECT_EQ(format_duration(0), std::string("0s"));
  EXPECT_EQ(format_duration(-kSecond), std::string("-1s"));
}
