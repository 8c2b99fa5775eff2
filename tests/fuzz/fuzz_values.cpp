// libFuzzer target: the small value parsers fed from flags, env vars and
// sysfs text - Go durations (--sleep-interval), the --visible-devices
// filter, integer parsing, and label-value sanitising.  Each must accept or
// reject (gfd::Error / nullopt) without crashing; accepted durations must
// round-trip through format_duration, and a sanitised label value must be a
// valid Kubernetes label value.
#include <cstdint>
#include <cstdlib>
#include <string>

#include "lm/labels.h"
#include "resource/filter.h"
#include "util/duration.h"
#include "util/error.h"
#include "util/strings.h"

namespace {
bool valid_label_value(const std::string& v) {
  if (v.size() > 63) return false;
  auto alnum = [](char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); };
  for (char c : v)
    if (!alnum(c) && c != '-' && c != '_' && c != '.') return false;
  return v.empty() || (alnum(v.front()) && alnum(v.back()));
}
}  // namespace

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  std::string s(reinterpret_cast<const char*>(data), size);
  try {
    gfd::Nanos d = gfd::parse_duration(s);
    if (gfd::parse_duration(gfd::format_duration(d)) != d) std::abort();
  } catch (const gfd::Error&) {
  }
  try {
    auto f = gfd::resource::DeviceFilter::parse(s);
    (void)f.matches(0, "0000:75:00.0");
  } catch (const gfd::Error&) {
  }
  (void)gfd::str::parse_uint(s, 16);
  (void)gfd::str::parse_int(s);
  (void)gfd::str::parse_uint_auto(s);
  (void)gfd::str::parse_float(s);
  if (!valid_label_value(gfd::lm::sanitize_label_value(s))) std::abort();
  return 0;
}
