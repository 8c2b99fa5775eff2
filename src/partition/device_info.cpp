#include "partition/device_info.h"

namespace gfd::partition {

using resource::DevicePtr;

const std::map<bool, std::vector<DevicePtr>>& DeviceInfo::GetDevicesMap() {
  if (built_) return map_;
  std::map<bool, std::vector<DevicePtr>> m;
  for (const auto& d : manager_.GetDevices()) m[d->IsPartitioned()].push_back(d);
  map_ = std::move(m);
  built_ = true;
  return map_;
}

std::vector<DevicePtr> DeviceInfo::GetDevicesWithPartitioningEnabled() {
  const auto& m = GetDevicesMap();
  auto it = m.find(true);
  return it == m.end() ? std::vector<DevicePtr>{} : it->second;
}

std::vector<DevicePtr> DeviceInfo::GetDevicesWithPartitioningDisabled() {
  const auto& m = GetDevicesMap();
  auto it = m.find(false);
  return it == m.end() ? std::vector<DevicePtr>{} : it->second;
}

bool DeviceInfo::AnyPartitionedDeviceIsEmpty() {
  auto enabled = GetDevicesWithPartitioningEnabled();
  if (enabled.empty()) return true;
  for (const auto& d : enabled)
    if (d->GetPartitions().empty()) return true;
  return false;
}

std::vector<DevicePtr> DeviceInfo::GetAllPartitions() {
  std::vector<DevicePtr> out;
  for (const auto& d : GetDevicesWithPartitioningEnabled()) {
    auto parts = d->GetPartitions();
    out.insert(out.end(), parts.begin(), parts.end());
  }
  return out;
}

}  // namespace gfd::partition
