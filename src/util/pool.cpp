#include "util/pool.h"

#include <atomic>

namespace gfd {

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
  }
  cv_.notify_all();
  for (auto& t : threads_) t.join();
}

size_t WorkerPool::workers() const {
  std::lock_guard<std::mutex> g(mu_);
  return threads_.size();
}

void WorkerPool::ensure_workers(size_t n) {
  // Caller holds mu_.
  while (threads_.size() < n && threads_.size() < max_workers_) threads_.emplace_back([this] { loop(); });
}

void WorkerPool::loop() {
  for (;;) {
    std::function<void()> fn;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this] { return stop_ || !queue_.empty(); });
      if (stop_ && queue_.empty()) return;
      fn = std::move(queue_.front());
      queue_.pop_front();
    }
    fn();
  }
}

WorkerPool::Task WorkerPool::submit(std::function<void()> fn) {
  Task t;
  t.state_ = std::make_shared<Task::State>();
  auto st = t.state_;
  {
    std::lock_guard<std::mutex> g(mu_);
    ensure_workers(queue_.size() + 1);
    queue_.emplace_back([st, fn = std::move(fn)] {
      std::exception_ptr err;
      try {
        fn();
      } catch (...) {
        err = std::current_exception();
      }
      std::lock_guard<std::mutex> g2(st->mu);
      st->error = err;
      st->done = true;
      st->cv.notify_all();
    });
  }
  cv_.notify_one();
  return t;
}

void WorkerPool::Task::wait() {
  if (!state_) return;
  std::unique_lock<std::mutex> lk(state_->mu);
  state_->cv.wait(lk, [this] { return state_->done; });
  if (state_->error) std::rethrow_exception(state_->error);
}

void WorkerPool::parallel_for(size_t n, const std::function<void(size_t)>& fn, size_t max_parallel) {
  if (n == 0) return;
  size_t lanes = max_parallel ? std::min(n, max_parallel) : n;
  if (lanes <= 1) {
    for (size_t i = 0; i < n; ++i) fn(i);
    return;
  }
  auto next = std::make_shared<std::atomic<size_t>>(0);
  auto body = [next, n, &fn] {
    for (size_t i = (*next)++; i < n; i = (*next)++) fn(i);
  };
  std::vector<Task> tasks;
  tasks.reserve(lanes - 1);
  for (size_t l = 1; l < lanes; ++l) tasks.push_back(submit(body));
  std::exception_ptr first;
  try {
    body();
  } catch (...) {
    first = std::current_exception();
  }
  for (auto& t : tasks) {
    try {
      t.wait();
    } catch (...) {
      if (!first) first = std::current_exception();
    }
  }
  if (first) std::rethrow_exception(first);
}

}  // namespace gfd
