#include "util/trace.h"

#include <cstdio>

namespace gfd::trace {

namespace {
thread_local std::vector<Phase> t_phases;
thread_local int64_t t_top_ns = 0;
thread_local int t_depth = 0;
// Only threads that run (traced) labeling cycles record (detail::t_active);
// spans executed on pool workers would otherwise accumulate forever.
using detail::t_active;
}  // namespace

int& detail::depth() { return t_depth; }

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void begin_cycle(bool on) {
  t_phases.clear();
  t_top_ns = 0;
  t_active = on;
}
const std::vector<Phase>& phases() { return t_phases; }
void record(const std::string& name, int64_t ns) {
  if (t_active) t_phases.emplace_back(name, ns);
}
void record_top(const std::string& name, int64_t ns) {
  if (!t_active) return;
  t_phases.emplace_back(name, ns);
  t_top_ns += ns;
}
int64_t top_level_ns() { return t_top_ns; }

Capture::Capture(bool on) : own_(on && !t_active) {
  if (!own_) return;
  t_phases.clear();
  top_ns_ = t_top_ns;
  t_active = true;
}

std::vector<Phase> Capture::take() {
  std::vector<Phase> out;
  if (own_) out.swap(t_phases);
  return out;
}

Capture::~Capture() {
  if (!own_) return;
  t_phases.clear();
  t_top_ns = top_ns_;
  t_active = false;
}

std::string summary(int64_t total_ns) {
  std::string out;
  char buf[96];
  for (const auto& p : t_phases) {
    snprintf(buf, sizeof(buf), "%s=%.3fms ", p.first.c_str(), static_cast<double>(p.second) / 1e6);
    out += buf;
  }
  int64_t other = total_ns - t_top_ns;
  snprintf(buf, sizeof(buf), "other=%.3fms total=%.3fms", static_cast<double>(other) / 1e6,
           static_cast<double>(total_ns) / 1e6);
  out += buf;
  return out;
}

}  // namespace gfd::trace
