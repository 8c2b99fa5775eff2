// Per-cycle phase timing ("--trace-timing").
//
// The reference has no tracing at all; the headline metric of
// this port is label-generation latency, so every cycle records how long
// each phase took (init, enumerate, label, sriov, write).  Recording is two
// steady_clock reads per phase and is always on; printing is opt-in.
#pragma once

#include <chrono>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace gfd::trace {

using Phase = std::pair<std::string, int64_t>;  // name, nanoseconds

// Start a new cycle (clears the recorded phases of this thread).
void begin_cycle();
// Phases recorded on this thread since begin_cycle(), in completion order.
const std::vector<Phase>& phases();
void record(const std::string& name, int64_t ns);
// "init=25.1ms enumerate=0.4ms ... total=26.0ms"
std::string summary(int64_t total_ns);

int64_t now_ns();

class Span {
 public:
  explicit Span(const char* name) : name_(name), start_(now_ns()) {}
  ~Span() { record(name_, now_ns() - start_); }
  Span(const Span&) = delete;
  Span& operator=(const Span&) = delete;

 private:
  const char* name_;
  int64_t start_;
};

}  // namespace gfd::trace
