// Resource labelers (full GPUs and compute partitions) and the partition
// strategies.
//
// Reference: internal/lm/resource.go:27-284 (resource labelers, product /
// count / replicas / memory / architecture labels, sharing rules) and
// internal/lm/mig-strategy.go:29-309 (none / single / mixed), strategy.go.
#pragma once

#include <string>

#include "config/config.h"
#include "lm/labels.h"
#include "resource/types.h"

namespace gfd::lm {

inline constexpr const char* kStrategyNone = "none";
inline constexpr const char* kStrategySingle = "single";
inline constexpr const char* kStrategyMixed = "mixed";

// Builds labels for one resource name ("amd.com/gpu",
// "amd.com/partition-cpx.1xcd.36gb").  A null config means sharing is
// disabled (replicas=0), as in resource.go:30-33.
class ResourceLabeler {
 public:
  ResourceLabeler(std::string resource_name, const config::Config* config)
      : resource_name_(std::move(resource_name)), config_(config) {}

  std::string key(const std::string& suffix) const { return resource_name_ + "." + suffix; }
  // Values are passed through sanitize_label_value: whatever a driver
  // reports, the file never holds a value NFD would reject.
  Labels single(const std::string& suffix, const std::string& value) const {
    return Labels{{key(suffix), sanitize_label_value(value)}};
  }
  void update(Labels& l, const std::string& suffix, const std::string& value) const {
    l[key(suffix)] = sanitize_label_value(value);
  }

  // product: non-empty parts joined by '-', spaces replaced, "-SHARED" if
  // replicated (>1) and not renamed (resource.go:159-176).
  Labels product_label(const std::vector<std::string>& parts) const;
  Labels replicas_label() const;
  Labels base_labels(int count, const std::vector<std::string>& parts) const;

  bool sharing_disabled() const { return config_ == nullptr; }
  bool is_shared() const;
  bool is_renamed() const;
  const config::ReplicatedResource* replication_info() const;

 private:
  std::string resource_name_;
  const config::Config* config_;
};

// resource.go:36-73.  count==0 -> empty.
Labels NewGPUResourceLabels(const config::Config* config, const resource::Device& device, int count);
inline Labels NewGPUResourceLabelsWithoutSharing(const resource::Device& device, int count) {
  return NewGPUResourceLabels(nullptr, device, count);
}
// resource.go:76-111 (MIG -> partition).  Product is
// <parent model>-PARTITION-<profile>; attributes map 1:1 to labels.
Labels NewPartitionResourceLabels(const std::string& resource_name, const config::Config* config,
                                  const resource::Device& partition, int count);
// family / arch / compute.{major,minor}; empty when the ISA target is unknown
// (the reference omits arch labels when CC major == 0).
Labels NewArchitectureLabels(const ResourceLabeler& rl, const resource::Device& device);

// mig-strategy.go:45-77: full-GPU labels, plus strategy-specific partition
// labels unless the strategy is "none".  Throws on an unknown strategy when
// devices exist.
LabelerPtr NewResourceLabeler(resource::Manager& manager, const config::Config& config);

}  // namespace gfd::lm
