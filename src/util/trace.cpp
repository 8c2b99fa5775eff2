#include "util/trace.h"

#include <cstdio>

namespace gfd::trace {

namespace {
thread_local std::vector<Phase> t_phases;
// Only threads that run labeling cycles record; spans executed on pool
// workers would otherwise accumulate forever.
thread_local bool t_active = false;
}

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void begin_cycle() {
  t_phases.clear();
  t_active = true;
}
const std::vector<Phase>& phases() { return t_phases; }
void record(const std::string& name, int64_t ns) {
  if (t_active) t_phases.emplace_back(name, ns);
}

std::string summary(int64_t total_ns) {
  std::string out;
  char buf[96];
  for (const auto& p : t_phases) {
    snprintf(buf, sizeof(buf), "%s=%.3fms ", p.first.c_str(), static_cast<double>(p.second) / 1e6);
    out += buf;
  }
  snprintf(buf, sizeof(buf), "total=%.3fms", static_cast<double>(total_ns) / 1e6);
  out += buf;
  return out;
}

}  // namespace gfd::trace
