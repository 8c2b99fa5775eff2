// Per-cycle phase timing ("--trace-timing").
//
// The reference has no tracing at all; the headline metric of
// this port is label-generation latency, so every cycle records how long
// each phase took (init, enumerate, label, sriov, write).  Recording is two
// steady_clock reads per phase and is always on; printing is opt-in.
//
// Attribution: a Span opened while no other Span is open on the thread is a
// top-level phase; the top-level phases of a cycle are disjoint stretches of
// the cycle thread's time, so total - sum(top-level) is the time no phase
// names ("other" in the summary).  Nested spans and record() calls are
// details (a phase's parts, or work overlapped on a worker) and do not count
// towards the sum.
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
// A detail (not part of the top-level sum).
void record(const std::string& name, int64_t ns);
// A top-level phase measured by hand (time the cycle thread spent in it).
void record_top(const std::string& name, int64_t ns);
// Sum of the top-level phases of this thread's cycle.
int64_t top_level_ns();
// "init=25.1ms enumerate=0.4ms ... other=0.010ms total=26.0ms"
std::string summary(int64_t total_ns);

int64_t now_ns();

namespace detail {
int& depth();
}

// The records a task makes on a pool worker (a thread that runs no cycle and
// so records nothing), to be re-recorded by the cycle thread as details once
// it has joined the task.  On the cycle thread itself (a task it took over)
// the records already are the cycle's, and take() returns none.
class Capture {
 public:
  Capture();
  ~Capture();
  std::vector<Phase> take();
  Capture(const Capture&) = delete;
  Capture& operator=(const Capture&) = delete;

 private:
  bool own_;  // this thread was not recording: the records are ours to hand over
  int64_t top_ns_ = 0;
};

class Span {
 public:
  explicit Span(const char* name) : name_(name), start_(now_ns()) { ++detail::depth(); }
  ~Span() {
    int64_t ns = now_ns() - start_;
    if (--detail::depth() == 0) {
      record_top(name_, ns);
    } else {
      record(name_, ns);
    }
  }
  Span(const Span&) = delete;
  Span& operator=(const Span&) = delete;

 private:
  const char* name_;
  int64_t start_;
};

}  // namespace gfd::trace
