// Cost of the clocks a labeling cycle's phase tracing reads (trace::now_ns:
// steady_clock / CLOCK_MONOTONIC through the vDSO) against the CPU's time
// stamp counter, and of one trace record (two clock reads + the record).
// Usage: build/clock_probe   (prints one JSON line)
#include <x86intrin.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <ctime>

#include "util/trace.h"

int main() {
  using namespace gfd;
  constexpr int N = 2000000;
  volatile int64_t sink = 0;
  auto t0 = trace::now_ns();
  for (int i = 0; i < N; ++i) sink = sink + trace::now_ns();
  auto t1 = trace::now_ns();
  for (int i = 0; i < N; ++i) sink = sink + static_cast<int64_t>(__rdtsc());
  auto t2 = trace::now_ns();
  struct timespec ts;
  for (int i = 0; i < N; ++i) {
    clock_gettime(CLOCK_MONOTONIC_COARSE, &ts);
    sink = sink + ts.tv_nsec;
  }
  auto t3 = trace::now_ns();
  trace::begin_cycle();
  for (int i = 0; i < N / 40; ++i) {
    if (i % 40 == 0) trace::begin_cycle();
    int64_t s = trace::now_ns();
    trace::record("write.unlease", trace::now_ns() - s);
  }
  auto t4 = trace::now_ns();
  std::printf("{\"now_ns\": %.1f, \"rdtsc_ns\": %.1f, \"monotonic_coarse_ns\": %.1f, \"record_ns\": %.1f}\n",
              double(t1 - t0) / N, double(t2 - t1) / N, double(t3 - t2) / N, double(t4 - t3) / (N / 40));
  return static_cast<int>(sink & 0) ;
}
