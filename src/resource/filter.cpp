#include "resource/filter.h"

#include <algorithm>

#include "util/error.h"
#include "util/log.h"
#include "util/strings.h"

namespace gfd::resource {

namespace {
// Normalise "d9:00.0" -> "0000:d9:00.0", lowercase.
std::string normalize_bdf(const std::string& s) {
  std::string b = str::to_lower(s);
  if (std::count(b.begin(), b.end(), ':') == 1) b = "0000:" + b;
  return b;
}

// "dddd:bb:dd.f" with a domain of 4+ hex digits, device < 0x20 (normalised form).
bool valid_bdf(const std::string& b) {
  auto hex = [](char c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f'); };
  size_t n = b.size();
  if (n < 12 || b[n - 8] != ':' || b[n - 5] != ':' || b[n - 2] != '.') return false;
  for (size_t i = 0; i < n; ++i)
    if (i != n - 8 && i != n - 5 && i != n - 2 && !hex(b[i])) return false;
  return b[n - 4] <= '1' && b[n - 1] <= '7';
}
}  // namespace

DeviceFilter& DeviceFilter::operator=(const DeviceFilter& o) {
  if (this != &o) {
    all_ = o.all_;
    spec_ = o.spec_;
    ranges_ = o.ranges_;
    bdfs_ = o.bdfs_;
    std::lock_guard<std::mutex> lk(mu_);
    last_report_.clear();
  }
  return *this;
}

DeviceFilter DeviceFilter::parse(const std::string& spec) {
  DeviceFilter f;
  std::string s = str::trim(spec);
  if (s.empty() || s == "all") return f;
  f.all_ = false;
  f.spec_ = s;
  for (const auto& raw : str::split(s, ',')) {
    std::string item = str::trim(raw);
    if (item.empty()) continue;
    if (item.find(':') != std::string::npos) {
      std::string b = normalize_bdf(item);
      if (!valid_bdf(b)) throw Error("invalid PCI address '" + item + "' in visible devices '" + spec + "'");
      f.bdfs_.push_back(std::move(b));
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

void DeviceFilter::check_selection(const std::vector<std::string>& bdfs) const {
  if (all_) return;
  std::vector<std::string> unmatched;
  for (const auto& r : ranges_)
    if (static_cast<size_t>(r.first) >= bdfs.size())
      unmatched.push_back(r.first == r.second ? std::to_string(r.first)
                                              : std::to_string(r.first) + "-" + std::to_string(r.second));
  for (const auto& b : bdfs_) {
    bool found = false;
    for (const auto& x : bdfs) found |= normalize_bdf(x) == b;
    if (!found) unmatched.push_back(b);
  }
  std::string report;
  if (!unmatched.empty()) {
    report = "Warning: --visible-devices '" + spec_ + "': " + str::join(unmatched, ", ") +
             (unmatched.size() == 1 ? " selects" : " select") + " none of the node's " + std::to_string(bdfs.size()) +
             " GPU(s)";
  }
  std::lock_guard<std::mutex> lk(mu_);
  if (report == last_report_) return;
  last_report_ = report;
  if (!report.empty()) log::printf("%s", report.c_str());
}

}  // namespace gfd::resource
