// `--visible-devices` selector: which physical GPUs a backend reports.
//
// The benchmark contract measures label generation "with 1, 2, 4 and 8 GPUs
// visible" (BASELINE.json); amd-smi and the KFD topology always enumerate
// every GPU the container can open, so the restriction is applied inside the
// backend at enumeration time.  Syntax: "" or "all" = every GPU; otherwise a
// comma list of indices ("0,3"), ranges ("0-3") and PCI addresses
// ("0000:d9:00.0").  Indices refer to physical GPUs sorted by PCI address.
// A malformed spec is an error at start-up; a well-formed item that names no
// GPU of the node (an index past the last GPU, an absent address) is logged
// once, since it silently removes that GPU's labels.
#pragma once

#include <mutex>
#include <string>
#include <vector>

namespace gfd::resource {

class DeviceFilter {
 public:
  DeviceFilter() = default;
  // Throws gfd::Error on a malformed spec.
  static DeviceFilter parse(const std::string& spec);

  DeviceFilter(const DeviceFilter& o) : all_(o.all_), spec_(o.spec_), ranges_(o.ranges_), bdfs_(o.bdfs_) {}
  DeviceFilter& operator=(const DeviceFilter& o);

  bool all() const { return all_; }
  bool matches(int index, const std::string& bdf) const;
  // After a selection over the node's physical GPUs (`bdfs`, in index order):
  // logs the items that selected none of them, once per distinct outcome.
  void check_selection(const std::vector<std::string>& bdfs) const;

 private:
  bool all_ = true;
  std::string spec_;
  std::vector<std::pair<int, int>> ranges_;
  std::vector<std::string> bdfs_;
  mutable std::mutex mu_;
  mutable std::string last_report_;  // what check_selection last logged ("" = nothing)
};

}  // namespace gfd::resource
