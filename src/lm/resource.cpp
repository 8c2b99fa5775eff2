#include "lm/resource.h"

#include <map>

#include "lm/keys.h"
#include "partition/device_info.h"
#include "util/error.h"
#include "util/log.h"
#include "util/strings.h"

namespace gfd::lm {

using resource::Device;
using resource::DevicePtr;

// ---------------------------------------------------------------------------
// ResourceLabeler

Labels ResourceLabeler::product_label(const std::vector<std::string>& parts) const {
  std::vector<std::string> stripped;
  for (const auto& p : parts)
    if (!p.empty()) stripped.push_back(str::replace_all(p, " ", "-"));
  if (stripped.empty()) return {};
  if (is_shared() && !is_renamed()) stripped.push_back("SHARED");
  return single("product", sanitize_label_value(str::join(stripped, "-")));
}

Labels ResourceLabeler::replicas_label() const {
  int replicas = 1;
  if (sharing_disabled()) {
    replicas = 0;
  } else if (const auto* r = replication_info(); r && r->replicas > 1) {
    replicas = r->replicas;
  }
  return single("replicas", std::to_string(replicas));
}

Labels ResourceLabeler::base_labels(int count, const std::vector<std::string>& parts) const {
  Labels l = product_label(parts);
  update(l, "count", std::to_string(count));
  l.merge(replicas_label());  // disjoint keys
  return l;
}

bool ResourceLabeler::is_shared() const {
  const auto* r = replication_info();
  return r && r->replicas > 1;
}

bool ResourceLabeler::is_renamed() const {
  const auto* r = replication_info();
  return r && !r->rename.empty();
}

const config::ReplicatedResource* ResourceLabeler::replication_info() const {
  if (!config_) return nullptr;
  for (const auto& r : config_->sharing.time_slicing.resources)
    if (r.name == resource_name_) return &r;
  return nullptr;
}

// ---------------------------------------------------------------------------
// Resource labels

Labels NewArchitectureLabels(const ResourceLabeler& rl, const Device& device) {
  resource::GfxTarget t = device.GetGfxTarget();
  if (!t.valid()) return {};
  return Labels{
      {rl.key("family"), resource::arch_family(t)},
      {rl.key("arch"), t.name()},
      {rl.key("compute.major"), std::to_string(t.major)},
      {rl.key("compute.minor"), std::to_string(t.minor)},
  };
}

Labels NewGPUResourceLabels(const config::Config* config, const Device& device, int count) {
  if (count == 0) return {};
  std::string model = GFD_WRAP("failed to get device model", device.GetName());
  uint64_t memory = GFD_WRAP("failed to get memory info for device", device.GetTotalMemoryMiB());
  ResourceLabeler rl(keys::kFullGpuResource, config);
  Labels arch = GFD_WRAP("failed to create architecture labels", NewArchitectureLabels(rl, device));

  Labels l = rl.base_labels(count, {model});
  if (memory != 0) rl.update(l, "memory", std::to_string(memory));
  l.merge(arch);  // disjoint keys
  const auto& info = device.Info();
  if (info.compute_units) rl.update(l, "compute-units", std::to_string(info.compute_units));
  if (info.xcds) rl.update(l, "xcds", std::to_string(info.xcds));
  return l;
}

Labels NewPartitionResourceLabels(const std::string& resource_name, const config::Config* config,
                                  const Device& partition, int count) {
  if (count == 0) return {};
  DevicePtr parent = GFD_WRAP("failed to get parent of compute partition", partition.GetParent());
  std::string model = GFD_WRAP("failed to get device model", parent->GetName());
  std::string profile = GFD_WRAP("failed to get compute partition profile name", partition.GetName());
  ResourceLabeler rl(resource_name, config);
  resource::Attributes attrs =
      GFD_WRAP("failed to get compute partition attribute labels", partition.GetAttributes());
  Labels l = rl.base_labels(count, {model, "PARTITION", profile});
  for (const auto& kv : attrs) rl.update(l, kv.first, kv.second);
  return l;
}

// ---------------------------------------------------------------------------
// Strategies

namespace {

struct PartitionResource {
  std::string name;
  DevicePtr device;
  int count = 0;
};

Labels strategy_labels(const std::string& strategy) {
  if (strategy == kStrategyNone) return {};
  return Labels{{keys::kPartitionStrategy, strategy}};
}

// mig-strategy.go:113-179.  Evaluated eagerly.
Labels new_gpu_labels(resource::Manager& manager, const config::Config& config) {
  partition::DeviceInfo di(manager);
  const auto& by_partitioned = GFD_WRAP("error getting map of devices", di.GetDevicesMap());
  if (by_partitioned.empty()) throw Error("no GPU devices detected");

  std::map<std::string, int> counts;
  std::map<std::string, DevicePtr> partitioned;
  std::map<std::string, DevicePtr> full;
  if (auto it = by_partitioned.find(true); it != by_partitioned.end()) {
    for (const auto& d : it->second) {
      std::string name = GFD_WRAP("error getting device name", d->GetName());
      partitioned[name] = d;  // the last device of a model represents it (map assignment, mig-strategy.go:132)
      counts[name]++;
    }
  }
  if (auto it = by_partitioned.find(false); it != by_partitioned.end()) {
    for (const auto& d : it->second) {
      std::string name = GFD_WRAP("error getting device name", d->GetName());
      full[name] = d;  // mig-strategy.go:142
      counts[name]++;
    }
  }
  if (counts.size() > 1) {
    std::vector<std::string> names;
    for (const auto& kv : counts) names.push_back(kv.first);
    log::printf("WARNING: Multiple device types detected: [%s]", str::join(names, " ").c_str());
  }

  Labels out;
  // Partitioned GPUs first, without sharing; full GPUs override them.
  // (Plain pair iteration: GFD_WRAP's lambda cannot capture structured
  // bindings before C++20.)
  for (const auto& entry : partitioned) {
    const Device& d = *entry.second;
    int count = counts[entry.first];
    Labels l = GFD_WRAP("failed to construct labeler", NewGPUResourceLabelsWithoutSharing(d, count));
    move_labels(out, std::move(l));
  }
  for (const auto& entry : full) {
    const Device& d = *entry.second;
    int count = counts[entry.first];
    Labels l = GFD_WRAP("failed to construct labeler", NewGPUResourceLabels(&config, d, count));
    move_labels(out, std::move(l));
  }
  return out;
}

Labels new_partition_device_labels(const std::map<std::string, PartitionResource>& resources,
                                   const config::Config& config) {
  Labels out;
  for (const auto& entry : resources) {
    const PartitionResource& r = entry.second;
    Labels l = GFD_WRAP("failed to construct labeler", NewPartitionResourceLabels(r.name, &config, *r.device, r.count));
    move_labels(out, std::move(l));
  }
  return out;
}

Labels invalid_single_labels(const Device& device, const std::string& reason) {
  log::printf("WARNING: Invalid configuration detected for mig-strategy=single: %s", reason.c_str());
  std::string model = GFD_WRAP("failed to get device model", device.GetName());
  ResourceLabeler rl(keys::kFullGpuResource, nullptr);
  Labels l = rl.product_label({model, "PARTITION", "INVALID"});
  rl.update(l, "count", "0");
  rl.update(l, "replicas", "0");
  rl.update(l, "memory", "0");
  return l;
}

std::map<std::string, PartitionResource> group_partitions(const std::vector<DevicePtr>& parts,
                                                          const std::string& resource_prefix, bool per_profile) {
  std::map<std::string, PartitionResource> resources;
  for (const auto& p : parts) {
    std::string name = GFD_WRAP("unable to get compute partition name", p->GetName());
    auto& r = resources[name];
    if (!r.device) {
      r.device = p;
      r.name = per_profile ? resource_prefix + name : resource_prefix;
    }
    r.count++;
  }
  return resources;
}

// mig-strategy.go:181-241.
Labels single_strategy_labels(resource::Manager& manager, const config::Config& config) {
  partition::DeviceInfo di(manager);
  auto enabled = GFD_WRAP("unable to retrieve list of partitioned devices", di.GetDevicesWithPartitioningEnabled());
  if (enabled.empty()) return {};  // equivalent to strategy none
  bool has_empty = GFD_WRAP("failed to check for empty partitioned devices", di.AnyPartitionedDeviceIsEmpty());
  if (has_empty) return invalid_single_labels(*enabled[0], "at least one partitioned GPU exposes no compute partitions");
  auto disabled = GFD_WRAP("unable to retrieve list of unpartitioned devices", di.GetDevicesWithPartitioningDisabled());
  if (!disabled.empty())
    return invalid_single_labels(*enabled[0], "GPUs with and without compute partitioning detected");
  auto parts = GFD_WRAP("unable to retrieve list of compute partitions", di.GetAllPartitions());
  auto resources = group_partitions(parts, keys::kFullGpuResource, false);
  if (resources.size() != 1)
    return invalid_single_labels(*enabled[0], "more than one compute partition profile present on node");
  return new_partition_device_labels(resources, config);
}

// mig-strategy.go:264-295.  Partitioned GPUs exposing nothing are ignored.
Labels mixed_strategy_labels(resource::Manager& manager, const config::Config& config) {
  partition::DeviceInfo di(manager);
  auto parts = GFD_WRAP("unable to retrieve list of compute partitions", di.GetAllPartitions());
  auto resources = group_partitions(parts, keys::kPartitionResourcePrefix, true);
  return new_partition_device_labels(resources, config);
}

// mig-strategy.go:84-110.
Labels new_partition_labels(resource::Manager& manager, const config::Config& config) {
  std::string strategy = config.mig_strategy();
  Labels l;
  if (strategy == kStrategyNone) {
    // nothing
  } else if (strategy == kStrategySingle) {
    l = GFD_WRAP("failed to create labeler for mig-strategy=single", single_strategy_labels(manager, config));
  } else if (strategy == kStrategyMixed) {
    l = GFD_WRAP("failed to create labeler for mig-strategy=mixed", mixed_strategy_labels(manager, config));
  } else {
    throw Error("unknown strategy: " + strategy);
  }
  Labels out = strategy_labels(strategy);
  move_labels(out, std::move(l));
  return out;
}

}  // namespace

LabelerPtr NewResourceLabeler(resource::Manager& manager, const config::Config& config) {
  auto devices = GFD_WRAP("error getting devices", manager.GetDevices());
  if (devices.empty()) return empty();
  Labels full = GFD_WRAP("failed to construct GPU labeler", new_gpu_labels(manager, config));
  if (config.mig_strategy() == kStrategyNone) return from_labels(std::move(full));
  Labels parts = GFD_WRAP("failed to construct compute partition resource labeler", new_partition_labels(manager, config));
  return merge({from_labels(std::move(full)), from_labels(std::move(parts))});
}

}  // namespace gfd::lm
