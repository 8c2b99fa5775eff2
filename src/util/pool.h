// Small persistent worker pool.
//
// A labeling cycle on an 8-GPU node issues a few hundred microseconds of
// driver queries per GPU plus an independent PCI-bus scan.  Spawning threads
// per cycle would cost as much as the work, so a process-wide pool of
// long-lived workers runs (a) the SR-IOV scan concurrently with device
// enumeration and (b) per-GPU amd-smi queries in parallel.
//
// Workers are created lazily on first use and inherit the creating thread's
// signal mask; the daemon blocks its watched signals before the first cycle,
// so workers never steal SIGHUP/SIGTERM from the run loop's sigtimedwait.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "util/affinity.h"

namespace gfd {

class WorkerPool {
 public:
  // Process-wide pool.
  static WorkerPool& instance();

  explicit WorkerPool(size_t max_workers);
  ~WorkerPool();
  WorkerPool(const WorkerPool&) = delete;
  WorkerPool& operator=(const WorkerPool&) = delete;

  class Task {
   public:
    // Blocks until the task ran; rethrows its exception.
    void wait();
    // Runs the task on the calling thread if no worker has started it yet,
    // else waits for it; rethrows its exception.  A late worker wake-up
    // (a core coming out of a deep idle state after the daemon's sleep)
    // then costs the work itself, not the wake-up latency on top of it.
    void run_or_wait();
    // Runs the task on the calling thread if no thread has started it yet
    // (true), else returns false at once: a thread about to wait for another
    // task of the same sequence takes this one over instead of idling.
    bool try_run();
    // Drops the task if no thread has started it, else waits for it (its
    // exception is discarded).  Afterwards fn is not running and never will.
    void cancel_or_wait();

   private:
    friend class WorkerPool;
    struct State {
      std::mutex mu;
      std::condition_variable cv;
      std::atomic<bool> claimed{false};  // a thread has started fn
      std::atomic<bool> finished{false};  // done, readable without the lock (a waiter's spin)
      bool done = false;
      std::exception_ptr error;
      std::function<void()> fn;
      void run();  // claimed by the caller: run fn, publish the result
      // A waiter spins this long (~10 us) before it sleeps on cv: a task
      // another thread is finishing costs its remaining run, not a futex
      // wake-up of the waiter on top (1-2 us back to back).
      void spin() const;
    };
    std::shared_ptr<State> state_;
  };

  // Run fn on a worker (or on the thread that calls run_or_wait first).
  Task submit(std::function<void()> fn);
  // Run fns in order on ONE worker (same core, warm cache); each is still a
  // Task of its own that the caller may run itself (run_or_wait) or drop
  // (cancel_or_wait) if the worker has not reached it yet.
  std::vector<Task> submit_sequence(std::vector<std::function<void()>> fns);
  // Run fn(i) for i in [0, n): the calling thread takes part, at most
  // `max_parallel` (0 = unlimited) run concurrently.  Rethrows the first error.
  // Safe to call from a pool task (nested): completes even if no worker is
  // free, because the caller runs every item nobody else has claimed.
  //
  // `stats` (optional): where the time went - the caller's hand-off (enqueue
  // and wake the helper lanes), the latest start of any item and the longest
  // item, all from the call's start, and how many items the caller ran.
  struct ParallelStats {
    int64_t handoff_ns = 0;     // the caller, before it starts on items itself
    int64_t last_start_ns = 0;  // the last item to start
    int64_t max_item_ns = 0;    // the longest item
    size_t caller_items = 0;
  };
  void parallel_for(size_t n, const std::function<void(size_t)>& fn, size_t max_parallel = 0,
                    ParallelStats* stats = nullptr);

  size_t workers() const;
  // Workers parked right now (a lane given to one of them needs no thread
  // to be created: in a fresh process that costs more than short work).
  size_t idle_workers() const;

  // Workers follow the caller: follow_caller() (called by the thread about
  // to hand out work) keeps every worker on the CPUs that share the L3 cache
  // of the CPU the caller runs on, re-pinning them only when that domain
  // changed.  The caller is left where the scheduler put it.  Off until
  // enabled.  load_topology() reads the host's L3 map (once per process;
  // the daemon calls it at start-up in loop mode, so a cycle only looks its
  // CPU up; a oneshot Job never follows and never reads it).  A domain of
  // which fewer than two CPUs are allowed is not pinned to (every lane on
  // one core).  set_follow(false) returns pinned workers to the caller's
  // allowed set.
  void set_follow(bool on);
  void load_topology();
  void follow_caller();
  // Re-pins done by follow_caller (tests / benchmarks).
  size_t repins() const { return repins_.load(std::memory_order_relaxed); }

 private:
  struct Worker {
    std::condition_variable cv;
    bool woken = false;  // set by wake_one (guarded by mu_)
  };
  void ensure_workers(size_t n);
  void unpin_locked();  // caller holds mu_
  void wake_one();
  void loop(Worker* w);

  size_t max_workers_;
  mutable std::mutex mu_;
  std::deque<std::function<void()>> queue_;
  std::vector<std::unique_ptr<Worker>> workers_;
  std::vector<std::thread> threads_;
  std::vector<Worker*> idle_;  // parked workers, most recently parked last
  size_t waking_ = 0;          // woken, not yet running
  size_t spawning_ = 0;        // threads created but not yet parked
  bool stop_ = false;
  std::atomic<bool> follow_{false};
  const affinity::L3Map* l3_ = nullptr;  // set with follow_
  std::atomic<int> domain_id_{-1};        // L3 domain the workers follow (-1: none yet)
  std::vector<int> domain_;  // CPUs the workers are kept on (follow mode; empty: anywhere)
  std::atomic<size_t> repins_{0};
};

// Lanes for per-GPU work in one cycle: one GPU per lane, at most 8 (the
// pool's size).  Spreading even the light SPX path (a few attribute preads
// per GPU) over one lane per GPU measured fastest at 2, 4 and 8 GPUs, back
// to back and after a 1 s sleep (profiles/hybrid_8gpu_scaling.txt); again in
// round 6 for 8 GPUs, with no per-cycle reads left: 8 lanes 0.0328 ms, 4
// lanes 0.0335, 2 lanes 0.0379 (profiles/hybrid_amdsmi_scaling_r6.txt).
size_t gpu_lanes(size_t n_gpus);

}  // namespace gfd
