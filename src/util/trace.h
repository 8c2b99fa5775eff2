// Per-cycle phase timing ("--trace-timing").
//
// The reference has no tracing at all; the headline metric of
// this port is label-generation latency, so every cycle records how long
// each phase took (init, enumerate, label, sriov, write).  Recording is two
// steady_clock reads per phase (19 ns each on the MI355X pool's EPYC 9575F,
// build/clock_probe): ~1.5 us of a 15 us back-to-back cycle, so a cycle is
// traced only when asked - the daemon's under --trace-timing, the bindings'
// by default (tests read the phases); an untraced cycle reads no clock for
// its phases and records nothing.
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

// Start a new cycle (clears the recorded phases of this thread); `on`:
// whether it is traced.
void begin_cycle(bool on = true);
// Whether this thread records (a traced cycle, or a Capture on a worker).
inline bool active();
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
inline thread_local bool t_active = false;
}  // namespace detail

inline bool active() { return detail::t_active; }
// A phase boundary: the clock when `on` (by default: when this thread
// records), else 0 - no clock read in an untraced cycle.  Work handed to
// another thread passes the cycle thread's active() as `on`.
inline int64_t stamp(bool on) { return on ? now_ns() : 0; }
inline int64_t stamp() { return stamp(detail::t_active); }
// record(name, now - t0), reading the clock only when this thread records.
inline void record_since(const char* name, int64_t t0) {
  if (detail::t_active) record(name, now_ns() - t0);
}

// The records a task makes on a pool worker (a thread that runs no cycle and
// so records nothing), to be re-recorded by the cycle thread as details once
// it has joined the task.  On the cycle thread itself (a task it took over)
// the records already are the cycle's, and take() returns none.  `on`: the
// cycle's active() (an untraced cycle's task records nothing).
class Capture {
 public:
  explicit Capture(bool on = true);
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
  explicit Span(const char* name) : name_(name), start_(stamp()) { ++detail::depth(); }
  ~Span() {
    if (!detail::t_active) {
      --detail::depth();
      return;
    }
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
