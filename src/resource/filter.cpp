#include "resource/filter.h"

#include <algorithm>

#include "util/error.h"
#include "util/strings.h"

namespace gfd::resource {

namespace {
// Normalise "d9:00.0" -> "0000:d9:00.0", lowercase.
std::string normalize_bdf(const std::string& s) {
  std::string b = str::to_lower(s);
  if (std::count(b.begin(), b.end(), ':') == 1) b = "0000:" + b;
  return b;
}
}  // namespace

DeviceFilter DeviceFilter::parse(const std::string& spec) {
  DeviceFilter f;
  std::string s = str::trim(spec);
  if (s.empty() || s == "all") return f;
  f.all_ = false;
  for (const auto& raw : str::split(s, ',')) {
    std::string item = str::trim(raw);
    if (item.empty()) continue;
    if (item.find(':') != std::string::npos) {
      f.bdfs_.push_back(normalize_bdf(item));
      continue;
    }
    auto dash = item.find('-');
    if (dash != std::string::npos) {
      auto lo = str::parse_uint(item.substr(0, dash));
      auto hi = str::parse_uint(item.substr(dash + 1));
      if (!lo || !hi || *hi < *lo) throw Error("invalid device range '" + item + "' in visible devices '" + spec + "'");
      f.ranges_.emplace_back(static_cast<int>(*lo), static_cast<int>(*hi));
      continue;
    }
    auto v = str::parse_uint(item);
    if (!v) throw Error("invalid device '" + item + "' in visible devices '" + spec + "'");
    f.ranges_.emplace_back(static_cast<int>(*v), static_cast<int>(*v));
  }
  return f;
}

bool DeviceFilter::matches(int index, const std::string& bdf) const {
  if (all_) return true;
  for (const auto& r : ranges_)
    if (index >= r.first && index <= r.second) return true;
  if (!bdf.empty()) {
    std::string b = normalize_bdf(bdf);
    for (const auto& x : bdfs_)
      if (x == b) return true;
  }
  return false;
}

}  // namespace gfd::resource
