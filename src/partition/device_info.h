// Per-cycle view of the node's GPUs split by partitioning state.
//
// Reference: internal/mig/mig.go:24-124 (DeviceInfo).  "MIG enabled" maps to
// "runs in a multi-partition compute mode (DPX/QPX/CPX)"; the MIG devices of
// a GPU are its compute partitions.  As in the reference the split is
// computed lazily on first use and cached for the lifetime of the object.
#pragma once

#include <map>
#include <vector>

#include "resource/types.h"

namespace gfd::partition {

class DeviceInfo {
 public:
  explicit DeviceInfo(resource::Manager& manager) : manager_(manager) {}

  // {true: partitioned GPUs, false: unpartitioned GPUs}
  const std::map<bool, std::vector<resource::DevicePtr>>& GetDevicesMap();
  std::vector<resource::DevicePtr> GetDevicesWithPartitioningEnabled();
  std::vector<resource::DevicePtr> GetDevicesWithPartitioningDisabled();
  // True if any partitioned GPU exposes no partitions (true for the empty set,
  // by definition, mig.go:85-106).
  bool AnyPartitionedDeviceIsEmpty();
  // All partitions of all partitioned GPUs.
  std::vector<resource::DevicePtr> GetAllPartitions();

 private:
  resource::Manager& manager_;
  bool built_ = false;
  std::map<bool, std::vector<resource::DevicePtr>> map_;
};

}  // namespace gfd::partition
