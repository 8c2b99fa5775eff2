// `--visible-devices` selector: which physical GPUs a backend reports.
//
// The benchmark contract measures label generation "with 1, 2, 4 and 8 GPUs
// visible" (BASELINE.json); amd-smi and the KFD topology always enumerate
// every GPU the container can open, so the restriction is applied inside the
// backend at enumeration time.  Syntax: "" or "all" = every GPU; otherwise a
// comma list of indices ("0,3"), ranges ("0-3") and PCI addresses
// ("0000:d9:00.0").  Indices refer to physical GPUs sorted by PCI address.
#pragma once

#include <string>
#include <vector>

namespace gfd::resource {

class DeviceFilter {
 public:
  DeviceFilter() = default;
  // Throws gfd::Error on a malformed spec.
  static DeviceFilter parse(const std::string& spec);

  bool all() const { return all_; }
  bool matches(int index, const std::string& bdf) const;

 private:
  bool all_ = true;
  std::vector<std::pair<int, int>> ranges_;
  std::vector<std::string> bdfs_;
};

}  // namespace gfd::resource
