#include "util/pool.h"

#include "util/trace.h"

#include <pthread.h>
#include <x86intrin.h>
#include <sched.h>

#include <algorithm>
#include <cstdlib>
#include <atomic>

#include "util/affinity.h"

namespace gfd {

namespace {
void pin(std::thread& t, const std::vector<int>& cpus) {
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus) CPU_SET(c, &set);
  pthread_setaffinity_np(t.native_handle(), sizeof(set), &set);
}
}  // namespace

WorkerPool& WorkerPool::instance() {
  // Leaked on purpose: workers may still be parked at exit.
  static WorkerPool* pool = new WorkerPool(8);
  return *pool;
}

WorkerPool::WorkerPool(size_t max_workers) : max_workers_(max_workers ? max_workers : 1) {}

WorkerPool::~WorkerPool() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
    for (auto& w : workers_) w->cv.notify_one();
  }
  for (auto& t : threads_) t.join();
}

size_t WorkerPool::workers() const {
  std::lock_guard<std::mutex> g(mu_);
  return threads_.size();
}

size_t WorkerPool::idle_workers() const {
  std::lock_guard<std::mutex> g(mu_);
  return idle_.size();
}

void WorkerPool::ensure_workers(size_t n) {
  // Caller holds mu_.  `n` tasks are queued: make sure that many workers are
  // parked, being woken or starting (busy workers may be blocked in a nested
  // parallel_for).
  while (idle_.size() + waking_ + spawning_ < n && threads_.size() < max_workers_) {
    ++spawning_;
    workers_.push_back(std::make_unique<Worker>());
    Worker* w = workers_.back().get();
    threads_.emplace_back([this, w] { loop(w); });
    if (!domain_.empty()) pin(threads_.back(), domain_);
  }
}

void WorkerPool::set_follow(bool on) {
  std::lock_guard<std::mutex> g(mu_);
  follow_.store(on);
  domain_id_.store(-1);
  if (!on && !domain_.empty()) unpin_locked();
}

void WorkerPool::load_topology() {
  if (!follow_.load()) return;
  const affinity::L3Map* map = &affinity::L3Map::host();  // sysfs reads: outside the lock
  std::lock_guard<std::mutex> g(mu_);
  l3_ = map;
}

void WorkerPool::unpin_locked() {
  // Back to wherever the caller may run (the process's placement).
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  if (sched_getaffinity(0, sizeof(allowed), &allowed) == 0)
    for (auto& t : threads_) pthread_setaffinity_np(t.native_handle(), sizeof(allowed), &allowed);
  domain_.clear();
}

void WorkerPool::follow_caller() {
  if (!follow_.load(std::memory_order_relaxed)) return;
  // The common case - the cycle woke on the L3 domain it last ran on - is a
  // vDSO getcpu and a table lookup.
  int cpu = sched_getcpu();
  std::lock_guard<std::mutex> g(mu_);
  if (!l3_) l3_ = &affinity::L3Map::host();  // load_topology() was not called
  int id = l3_->id(cpu);
  if (id < 0 || id == domain_id_.load(std::memory_order_relaxed)) return;
  domain_id_.store(id, std::memory_order_relaxed);
  std::vector<int> domain = affinity::allowed_subset(l3_->cpus(id));
  if (domain.size() < 2) {
    // A pod whose cpuset holds one CPU of this L3: pinning would put every
    // lane on that core.  Leave the workers to the scheduler.
    if (domain_.empty()) return;
    unpin_locked();
    ++repins_;
    return;
  }
  if (domain == domain_) return;
  domain_ = std::move(domain);
  for (auto& t : threads_) pin(t, domain_);
  ++repins_;
}

void WorkerPool::wake_one() {
  // Caller holds mu_.  LIFO: the most recently parked worker is the one
  // whose core still has its stack and the task's data in cache; a FIFO
  // condition variable would rotate every task over all workers (measured:
  // the per-cycle PCI scan took 180 us instead of 86 us once 8 workers
  // existed and took turns).
  if (idle_.empty()) return;
  Worker* w = idle_.back();
  idle_.pop_back();
  w->woken = true;
  ++waking_;
  w->cv.notify_one();
}

void WorkerPool::loop(Worker* w) {
  std::unique_lock<std::mutex> lk(mu_);
  --spawning_;
  for (;;) {
    while (queue_.empty() && !stop_) {
      // Idle workers block at once: the daemon sleeps a minute between
      // cycles, and a spinning worker would only burn a tenant's core.
      w->woken = false;
      idle_.push_back(w);
      w->cv.wait(lk, [&] { return w->woken || stop_; });
      if (w->woken) {
        --waking_;
      } else {
        idle_.erase(std::find(idle_.begin(), idle_.end(), w));  // stopping
      }
    }
    if (queue_.empty()) return;  // stop_ and nothing left to run
    std::function<void()> fn = std::move(queue_.front());
    queue_.pop_front();
    lk.unlock();
    fn();
    fn = nullptr;  // release captures outside the lock
    lk.lock();
  }
}

void WorkerPool::Task::State::run() {
  std::exception_ptr err;
  try {
    fn();
  } catch (...) {
    err = std::current_exception();
  }
  fn = nullptr;  // release captures before publishing
  std::lock_guard<std::mutex> g(mu);
  error = err;
  done = true;
  finished.store(true, std::memory_order_release);
  cv.notify_all();
}

void WorkerPool::Task::State::spin() const {
  for (int i = 0; i < 1000 && !finished.load(std::memory_order_acquire); ++i) _mm_pause();
}

WorkerPool::Task WorkerPool::submit(std::function<void()> fn) {
  Task t;
  t.state_ = std::make_shared<Task::State>();
  t.state_->fn = std::move(fn);
  auto st = t.state_;
  {
    std::lock_guard<std::mutex> g(mu_);
    queue_.emplace_back([st] {
      if (!st->claimed.exchange(true)) st->run();  // else the submitter ran it
    });
    ensure_workers(queue_.size());
    wake_one();
  }
  return t;
}

std::vector<WorkerPool::Task> WorkerPool::submit_sequence(std::vector<std::function<void()>> fns) {
  std::vector<Task> tasks(fns.size());
  std::vector<std::shared_ptr<Task::State>> states;
  for (size_t i = 0; i < fns.size(); ++i) {
    tasks[i].state_ = std::make_shared<Task::State>();
    tasks[i].state_->fn = std::move(fns[i]);
    states.push_back(tasks[i].state_);
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    queue_.emplace_back([states = std::move(states)] {
      for (const auto& st : states)
        if (!st->claimed.exchange(true)) st->run();
    });
    ensure_workers(queue_.size());
    wake_one();
  }
  return tasks;
}

void WorkerPool::Task::wait() {
  if (!state_) return;
  state_->spin();
  std::unique_lock<std::mutex> lk(state_->mu);
  state_->cv.wait(lk, [this] { return state_->done; });
  if (state_->error) std::rethrow_exception(state_->error);
}

void WorkerPool::Task::cancel_or_wait() {
  if (!state_) return;
  if (!state_->claimed.exchange(true)) {
    std::lock_guard<std::mutex> g(state_->mu);
    state_->fn = nullptr;
    state_->done = true;
    state_->finished.store(true, std::memory_order_release);
    state_->cv.notify_all();
    return;
  }
  state_->spin();
  std::unique_lock<std::mutex> lk(state_->mu);
  state_->cv.wait(lk, [this] { return state_->done; });
}

bool WorkerPool::Task::try_run() {
  if (!state_ || state_->claimed.exchange(true)) return false;
  state_->run();
  return true;
}

void WorkerPool::Task::run_or_wait() {
  if (!state_) return;
  if (!state_->claimed.exchange(true)) state_->run();
  wait();
}

void WorkerPool::parallel_for(size_t n, const std::function<void(size_t)>& fn, size_t max_parallel,
                              ParallelStats* stats) {
  if (n == 0) return;
  size_t lanes = max_parallel ? std::min(n, max_parallel) : n;
  const int64_t t0 = stats ? trace::now_ns() : 0;
  if (lanes <= 1) {
    for (size_t i = 0; i < n; ++i) {
      int64_t s0 = stats ? trace::now_ns() : 0;
      fn(i);
      if (stats) {
        stats->last_start_ns = s0 - t0;
        stats->max_item_ns = std::max(stats->max_item_ns, trace::now_ns() - s0);
      }
    }
    if (stats) stats->caller_items = n;
    return;
  }
  // Items are claimed from a shared counter; the caller waits for every
  // *claimed* item to finish, not for the helper lanes to start.  A lane
  // still queued when the caller has drained the range finds nothing left
  // and exits, so nested parallel_for calls (e.g. the PCI scan, itself a
  // pool task, spreading its reads) cannot deadlock on a saturated pool.
  struct Shared {
    std::atomic<size_t> next{0};
    std::mutex mu;
    std::condition_variable cv;
    size_t done = 0;
    std::exception_ptr error;
    const std::function<void(size_t)>* fn;
    size_t n;
  };
  auto sh = std::make_shared<Shared>();
  sh->fn = &fn;
  sh->n = n;
  // Per-item (start, duration) when `stats` is asked for; written by the
  // item's own thread, read after every item is done.
  struct ItemTime {
    int64_t start = 0, ns = 0;
    bool caller = false;
  };
  std::vector<ItemTime> times(stats ? n : 0);
  ItemTime* times_p = stats ? times.data() : nullptr;
  const std::thread::id caller = std::this_thread::get_id();
  auto body = [sh, times_p, caller] {
    for (size_t i = sh->next++; i < sh->n; i = sh->next++) {
      std::exception_ptr err;
      int64_t s0 = times_p ? trace::now_ns() : 0;
      try {
        (*sh->fn)(i);
      } catch (...) {
        err = std::current_exception();
      }
      if (times_p) times_p[i] = {s0, trace::now_ns() - s0, std::this_thread::get_id() == caller};
      std::lock_guard<std::mutex> g(sh->mu);
      if (err && !sh->error) sh->error = err;
      if (++sh->done == sh->n) sh->cv.notify_all();
    }
  };
  // Enqueue every helper lane and wake its worker under one acquisition of
  // the pool lock: per-lane submit (lock, enqueue, notify, unlock) staggers
  // the 8th lane's start by several wake-up latencies on an 8-GPU cycle.
  {
    std::lock_guard<std::mutex> g(mu_);
    for (size_t l = 1; l < lanes; ++l) queue_.emplace_back(body);
    ensure_workers(queue_.size());
    for (size_t l = 1; l < lanes; ++l) wake_one();
  }
  if (stats) stats->handoff_ns = trace::now_ns() - t0;
  body();
  std::exception_ptr error;
  {
    std::unique_lock<std::mutex> lk(sh->mu);
    sh->cv.wait(lk, [&] { return sh->done == sh->n; });
    // Taken out, so that a helper lane dropping the last reference to `sh`
    // later never destroys the exception this thread is handling.
    error = std::move(sh->error);
  }
  if (stats) {
    for (const auto& t : times) {
      stats->last_start_ns = std::max(stats->last_start_ns, t.start - t0);
      stats->max_item_ns = std::max(stats->max_item_ns, t.ns);
      stats->caller_items += t.caller;
    }
  }
  if (error) std::rethrow_exception(error);
}

size_t gpu_lanes(size_t n_gpus) { return std::max<size_t>(1, std::min<size_t>(8, n_gpus)); }

}  // namespace gfd
