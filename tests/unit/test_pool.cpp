// WorkerPool tests (run under TSan by `make tsan`).
#include <atomic>
#include <chrono>
#include <stdexcept>

#include <sched.h>

#include <string>
#include <vector>

#include "lm/labels.h"
#include "test.h"
#include "util/affinity.h"
#include "util/fs.h"
#include "util/pool.h"
#include "util/strings.h"

using gfd::WorkerPool;
namespace affinity = gfd::affinity;
namespace fs = gfd::fs;
namespace lm = gfd::lm;
namespace str = gfd::str;

TEST(Pool_ParallelForVisitsEveryIndexOnce) {
  WorkerPool pool(4);
  std::vector<std::atomic<int>> hits(1000);
  pool.parallel_for(hits.size(), [&](size_t i) { hits[i]++; });
  for (auto& h : hits) EXPECT_EQ(h.load(), 1);
  EXPECT_TRUE(pool.workers() <= 4);
}

TEST(Pool_ParallelForStatsSayWhereTheTimeWent) {
  WorkerPool pool(4);
  WorkerPool::ParallelStats st;
  std::atomic<int> ran{0};
  pool.parallel_for(
      8,
      [&](size_t) {
        auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(200);
        while (std::chrono::steady_clock::now() < until) {
        }
        ++ran;
      },
      4, &st);
  EXPECT_EQ(ran.load(), 8);
  EXPECT_TRUE(st.max_item_ns >= 200000);
  EXPECT_TRUE(st.handoff_ns >= 0 && st.last_start_ns >= 0);
  // (0 is possible: creating the workers can outlast the helpers' claims.)
  EXPECT_TRUE(st.caller_items <= 8);
  // One lane: everything on the caller.
  WorkerPool::ParallelStats one;
  pool.parallel_for(3, [&](size_t) { ++ran; }, 1, &one);
  EXPECT_EQ(one.caller_items, static_cast<size_t>(3));
  EXPECT_EQ(one.handoff_ns, static_cast<int64_t>(0));
}

TEST(Pool_ParallelForPropagatesFirstError) {
  WorkerPool pool(3);
  std::atomic<int> ran{0};
  EXPECT_THROW_MSG(pool.parallel_for(50,
                                     [&](size_t i) {
                                       ran++;
                                       if (i == 7) throw std::runtime_error("boom at 7");
                                     }),
                   "boom at 7");
  EXPECT_TRUE(ran.load() >= 1);
}

TEST(Pool_SubmitAndWait) {
  WorkerPool pool(2);
  int value = 0;
  auto t = pool.submit([&] { value = 42; });
  t.wait();
  EXPECT_EQ(value, 42);
  auto bad = pool.submit([] { throw std::runtime_error("task failed"); });
  EXPECT_THROW_MSG(bad.wait(), "task failed");
}

TEST(Pool_SerialWhenLimited) {
  WorkerPool pool(8);
  std::atomic<int> concurrent{0}, peak{0};
  pool.parallel_for(
      20,
      [&](size_t) {
        int c = ++concurrent;
        int p = peak.load();
        while (c > p && !peak.compare_exchange_weak(p, c)) {
        }
        --concurrent;
      },
      1);
  EXPECT_EQ(peak.load(), 1);
}

TEST(Pool_ManyRoundsReuseWorkers) {
  WorkerPool pool(4);
  for (int r = 0; r < 200; ++r) {
    std::atomic<int> sum{0};
    pool.parallel_for(8, [&](size_t i) { sum += static_cast<int>(i); });
    EXPECT_EQ(sum.load(), 28);
  }
  EXPECT_TRUE(pool.workers() <= 4);
}

TEST(Pool_NestedParallelForOnSaturatedPoolCompletes) {
  // The PCI scan is a pool task that itself calls parallel_for; with every
  // worker busy the nested call must still finish (caller drains the range).
  WorkerPool pool(1);
  std::atomic<int> inner{0};
  auto t = pool.submit([&] { pool.parallel_for(16, [&](size_t) { inner++; }, 8); });
  t.wait();
  EXPECT_EQ(inner.load(), 16);
  // Two levels deep on a wider pool.
  WorkerPool pool4(4);
  std::atomic<int> leaves{0};
  pool4.parallel_for(8, [&](size_t) { pool4.parallel_for(8, [&](size_t) { leaves++; }, 4); }, 8);
  EXPECT_EQ(leaves.load(), 64);
}

TEST(Pool_RunOrWaitRunsUnstartedTaskInline) {
  // One worker, kept busy: a task queued behind it is run by the caller.
  WorkerPool pool(1);
  std::atomic<bool> release{false};
  auto busy = pool.submit([&] {
    while (!release.load()) std::this_thread::yield();
  });
  std::thread::id ran_on;
  auto t = pool.submit([&] { ran_on = std::this_thread::get_id(); });
  t.run_or_wait();
  EXPECT_TRUE(ran_on == std::this_thread::get_id());
  release = true;
  busy.wait();
  // Its exception reaches the caller either way.
  auto bad = pool.submit([] { throw std::runtime_error("task failed"); });
  EXPECT_THROW_MSG(bad.run_or_wait(), "task failed");
}

TEST(Pool_CancelOrWaitDropsUnstartedTask) {
  WorkerPool pool(1);
  std::atomic<bool> release{false};
  auto busy = pool.submit([&] {
    while (!release.load()) std::this_thread::yield();
  });
  std::atomic<int> ran{0};
  auto t = pool.submit([&] { ran++; });
  t.cancel_or_wait();
  release = true;
  busy.wait();
  auto after = pool.submit([] {});
  after.wait();  // the worker has drained the cancelled task by now
  EXPECT_EQ(ran.load(), 0);
  // A task already finished by a worker: cancel_or_wait returns at once.
  auto done = pool.submit([&] { ran++; });
  done.wait();
  done.cancel_or_wait();
  EXPECT_EQ(ran.load(), 1);
}

TEST(Pool_GpuLanesPolicy) {
  // One GPU per lane, at most the pool's width.
  EXPECT_EQ(gfd::gpu_lanes(0), static_cast<size_t>(1));
  EXPECT_EQ(gfd::gpu_lanes(1), static_cast<size_t>(1));
  EXPECT_EQ(gfd::gpu_lanes(2), static_cast<size_t>(2));
  EXPECT_EQ(gfd::gpu_lanes(8), static_cast<size_t>(8));
  EXPECT_EQ(gfd::gpu_lanes(16), static_cast<size_t>(8));
}

// ---- L3-domain pinning (util/affinity.h) ----

TEST(Affinity_ParseCpuList) {
  EXPECT_TRUE(affinity::parse_cpu_list("0-3,128-129\n") == (std::vector<int>{0, 1, 2, 3, 128, 129}));
  EXPECT_TRUE(affinity::parse_cpu_list("5") == (std::vector<int>{5}));
  EXPECT_TRUE(affinity::parse_cpu_list("3-1").empty());
  EXPECT_TRUE(affinity::parse_cpu_list("x").empty());
}

TEST(Affinity_PinsToTheCurrentL3DomainWithinTheAllowedSet) {
  cpu_set_t before;
  CPU_ZERO(&before);
  EXPECT_TRUE(sched_getaffinity(0, sizeof(before), &before) == 0);
  if (CPU_COUNT(&before) < 2) return;  // nothing to narrow
  // A synthetic topology in which every CPU has an L3 of its own.
  char d[] = "/tmp/gfd-aff-XXXXXX";
  EXPECT_TRUE(mkdtemp(d) != nullptr);
  std::string root = d;
  for (int c = 0; c < CPU_SETSIZE; ++c) {
    if (!CPU_ISSET(c, &before)) continue;
    std::string idx = root + "/sys/devices/system/cpu/cpu" + std::to_string(c) + "/cache/index3";
    fs::mkdir_all(idx);
    lm::write_file_atomically(idx + "/level", "3\n", 0644);
    lm::write_file_atomically(idx + "/shared_cpu_list", std::to_string(c) + "\n", 0644);
  }
  std::string what = affinity::pin_to_current_l3(root);
  cpu_set_t after;
  CPU_ZERO(&after);
  EXPECT_TRUE(sched_getaffinity(0, sizeof(after), &after) == 0);
  EXPECT_EQ(CPU_COUNT(&after), 1);
  EXPECT_TRUE(what.find("threads kept on the 1 CPUs") != std::string::npos);
  // Already within one domain: nothing changes.
  EXPECT_EQ(affinity::pin_to_current_l3(root), std::string(""));
  EXPECT_TRUE(sched_setaffinity(0, sizeof(before), &before) == 0);
  fs::remove_all(root);
}

TEST(Affinity_L3DomainFollowsTheAllowedSetAsItChanges) {
  // A cpuset changed under a running pod (CPU manager): the domain is the
  // cached cache topology intersected with what the thread may use now.
  cpu_set_t before;
  CPU_ZERO(&before);
  EXPECT_TRUE(sched_getaffinity(0, sizeof(before), &before) == 0);
  if (CPU_COUNT(&before) < 2) return;
  std::vector<int> allowed;
  for (int c = 0; c < CPU_SETSIZE; ++c)
    if (CPU_ISSET(c, &before)) allowed.push_back(c);
  // One L3 shared by every allowed CPU.
  char d[] = "/tmp/gfd-aff-XXXXXX";
  EXPECT_TRUE(mkdtemp(d) != nullptr);
  std::string root = d;
  std::vector<std::string> names;
  for (int c : allowed) names.push_back(std::to_string(c));
  for (int c : allowed) {
    std::string idx = root + "/sys/devices/system/cpu/cpu" + std::to_string(c) + "/cache/index3";
    fs::mkdir_all(idx);
    lm::write_file_atomically(idx + "/level", "3\n", 0644);
    lm::write_file_atomically(idx + "/shared_cpu_list", str::join(names, ",") + "\n", 0644);
  }
  int cpu = allowed.front();
  EXPECT_TRUE(affinity::l3_domain(cpu, root) == allowed);
  cpu_set_t one;
  CPU_ZERO(&one);
  CPU_SET(allowed.back(), &one);
  EXPECT_TRUE(sched_setaffinity(0, sizeof(one), &one) == 0);
  EXPECT_TRUE(affinity::l3_domain(cpu, root) == std::vector<int>{allowed.back()});
  EXPECT_TRUE(sched_setaffinity(0, sizeof(before), &before) == 0);
  EXPECT_TRUE(affinity::l3_domain(cpu, root) == allowed);
  fs::remove_all(root);
}

TEST(Pool_WorkersFollowTheCallersL3Domain) {
  // --cpu-affinity=follow: every worker is kept on the CPUs sharing the L3
  // of the CPU the calling thread runs on; the caller itself is untouched.
  int cpu = sched_getcpu();
  std::vector<int> domain = affinity::l3_domain(cpu);
  if (domain.empty()) return;  // no cache topology in sysfs here
  cpu_set_t before;
  EXPECT_TRUE(sched_getaffinity(0, sizeof(before), &before) == 0);
  gfd::WorkerPool pool(2);
  pool.set_follow(true);
  pool.follow_caller();
  std::vector<int> seen;
  pool.submit([&] {
        cpu_set_t s;
        CPU_ZERO(&s);
        sched_getaffinity(0, sizeof(s), &s);
        for (int c = 0; c < CPU_SETSIZE; ++c)
          if (CPU_ISSET(c, &s)) seen.push_back(c);
      })
      .wait();
  EXPECT_TRUE(seen == affinity::l3_domain(sched_getcpu()) || seen == domain);
  cpu_set_t after;
  EXPECT_TRUE(sched_getaffinity(0, sizeof(after), &after) == 0);
  EXPECT_TRUE(CPU_EQUAL(&before, &after));
}
