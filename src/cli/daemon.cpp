#include "cli/daemon.h"

#include <sched.h>
#include <signal.h>
#include <time.h>

#include <cerrno>
#include <cstdlib>
#include <functional>
#include <cstdio>

#include "info/version.h"
#include "lm/node.h"
#include "resource/factory.h"
#include "util/affinity.h"
#include "util/error.h"
#include "util/log.h"
#include "util/pool.h"

namespace gfd::cli {

// ---------------------------------------------------------------------------
// Configuration

void update_from_cli_flags(config::Flags& f, const Context& ctx) {
  auto str_field = [&](std::optional<std::string>& field, const char* name) {
    if (ctx.IsSet(name) || !field) field = ctx.String(name);
  };
  auto bool_field = [&](std::optional<bool>& field, const char* name) {
    if (ctx.IsSet(name) || !field) field = ctx.Bool(name);
  };
  auto dur_field = [&](std::optional<Nanos>& field, const char* name) {
    if (ctx.IsSet(name) || !field) field = ctx.Duration(name);
  };
  // Common flags.
  str_field(f.mig_strategy, "mig-strategy");
  bool_field(f.fail_on_init_error, "fail-on-init-error");
  // GFD flags.
  auto& g = f.gfd;
  bool_field(g.oneshot, "oneshot");
  str_field(g.output_file, "output-file");
  dur_field(g.sleep_interval, "sleep-interval");
  bool_field(g.no_timestamp, "no-timestamp");
  str_field(g.machine_type_file, "machine-type-file");
  str_field(g.backend, "backend");
  str_field(g.sysfs_root, "sysfs-root");
  str_field(g.host_root, "host-root");
  str_field(g.rocm_version_file, "rocm-version-file");
  str_field(g.visible_devices, "visible-devices");
  str_field(g.amdsmi_session, "amdsmi-session");
  str_field(g.mock_file, "mock-file");
  bool_field(g.trace_timing, "trace-timing");
}

config::Config load_config(const Context& ctx) {
  config::Config c;
  try {
    std::string file = ctx.String("config-file");
    if (!file.empty()) {
      try {
        c = config::parse_config_file(file);
      } catch (const std::exception& e) {
        throw Error(std::string("unable to parse config file: ") + e.what());
      }
    }
    update_from_cli_flags(c.flags, ctx);
  } catch (const std::exception& e) {
    throw Error(std::string("unable to finalize config: ") + e.what());
  }
  c.flags.plugin_present = false;  // config.Flags.Plugin = nil (main.go:105)
  return c;
}

// ---------------------------------------------------------------------------
// Signals

namespace {
sigset_t watched_set() {
  sigset_t s;
  sigemptyset(&s);
  sigaddset(&s, SIGHUP);
  sigaddset(&s, SIGINT);
  sigaddset(&s, SIGTERM);
  sigaddset(&s, SIGQUIT);
  return s;
}
}  // namespace

SignalWatcher::SignalWatcher() {
  sigset_t s = watched_set();
  pthread_sigmask(SIG_BLOCK, &s, nullptr);
}

std::optional<int> SignalWatcher::wait(int64_t timeout_ns) {
  sigset_t s = watched_set();
  int64_t deadline = trace::now_ns() + (timeout_ns < 0 ? 0 : timeout_ns);
  for (;;) {
    int64_t left = deadline - trace::now_ns();
    if (left < 0) left = 0;
    struct timespec ts;
    ts.tv_sec = static_cast<time_t>(left / 1000000000LL);
    ts.tv_nsec = static_cast<long>(left % 1000000000LL);
    siginfo_t info;
    int sig = sigtimedwait(&s, &info, &ts);
    if (sig > 0) return sig;
    if (errno == EINTR) continue;
    return std::nullopt;  // EAGAIN: timeout
  }
}

std::string SignalWatcher::name(int sig) {
  switch (sig) {
    case SIGHUP: return "hangup";
    case SIGINT: return "interrupt";
    case SIGTERM: return "terminated";
    case SIGQUIT: return "quit";
    default: return "signal " + std::to_string(sig);
  }
}

// ---------------------------------------------------------------------------
// Labeling

CycleResult label_cycle(resource::Manager& manager, const std::shared_ptr<sriov::Interface>& sriov,
                        const config::Config& config, const lm::LabelerPtr& timestamp, bool write, bool traced) {
  trace::begin_cycle(traced);
  int64_t t0 = trace::now_ns();
  CycleResult r;
  r.cpu_start = sched_getcpu();
  {
    // --cpu-affinity=follow, loop mode only: a oneshot Job has one cycle.
    trace::Span span("placement");
    if (!config.oneshot()) WorkerPool::instance().follow_caller();
  }
  // Work that does not depend on the device backend runs on workers while
  // the backend enumerates: the node facts the device labeler needs after
  // enumeration (machine type, file-backed versions) and the SR-IOV bus scan
  // (the reference evaluates the vGPU labeler after the NVML labeler; only
  // the merge order is observable).  Whichever a worker has not started by
  // the time it is needed runs on this thread instead (run_or_wait).  The
  // tasks never throw; an SR-IOV error is handed back and raised after the
  // device labeler.
  std::optional<resource::VersionSources> version_files;
  {
    trace::Span span("versions");
    version_files = manager.VersionFiles();
  }
  lm::NodeFacts facts;
  lm::Labels sriov_labels;
  std::exception_ptr sriov_error;
  int64_t facts_ns = 0, sriov_ns = 0, facts_start = 0, submitted = 0;

  std::vector<trace::Phase> facts_detail;  // the facts' own records, made on a worker
  auto read_facts = [&] {
    int64_t s0 = trace::stamp(traced);
    facts_start = s0;
    r.cpu_facts = sched_getcpu();
    trace::Capture capture(traced);
    try {
      facts = lm::ReadNodeFacts(config, version_files);
    } catch (...) {
      facts = lm::NodeFacts{};  // fall back to the manager inside the labeler
    }
    facts_detail = capture.take();
    if (traced) facts_ns = trace::now_ns() - s0;
  };
  std::vector<trace::Phase> sriov_detail;  // the lookup's own records, made on a worker
  auto scan_sriov = [&] {
    int64_t s0 = trace::stamp(traced);
    trace::Capture capture(traced);
    try {
      sriov_labels = lm::NewSriovLabeler(sriov)->GetLabels();
    } catch (...) {
      sriov_error = std::current_exception();
    }
    sriov_detail = capture.take();
    if (traced) sriov_ns = trace::now_ns() - s0;
  };
  // Loop mode: both on one worker, in that order (two workers measured
  // slower: each task 1.5-4x longer on the second, colder core,
  // profiles/ab_cycle_tasks.txt).  Whichever of the two the worker has not
  // started when this thread needs it, this thread runs: the SR-IOV lookup
  // before it waits for the node facts, the facts themselves if the worker
  // has not reached them.  Against both on this thread, alternated on one
  // box: back to back 0.0208 vs 0.0241 ms, cycles 1 s apart 0.194-0.228 vs
  // 0.257-0.313 ms (profiles/cycle_tasks_ab_r5.txt).
  //
  // A oneshot Job runs both here, after enumeration: its one cycle would pay
  // a worker thread's creation, which costs more than the work (Job process
  // p50 1.05 vs 1.27 ms with the hand-off and the start-up SR-IOV prefetch,
  // same file).
  const bool overlap = !config.oneshot();
  WorkerPool::Task facts_task, sriov_task;
  if (overlap) {
    trace::Span span("submit");
    submitted = trace::stamp();
    auto seq = WorkerPool::instance().submit_sequence({read_facts, scan_sriov});
    facts_task = seq[0];
    sriov_task = seq[1];
  }
  auto join_facts = [&]() -> const lm::NodeFacts& {
    if (!overlap) {
      read_facts();
      return facts;
    }
    int64_t s0 = trace::stamp();
    if (sriov_task.try_run()) trace::record_since("sriov.self", s0);
    int64_t w0 = trace::stamp();
    facts_task.run_or_wait();
    trace::record_since("facts.wait", w0);  // inside "label"
    return facts;
  };
  lm::LabelerPtr device;
  try {
    device = GFD_WRAP("error creating device labeler", lm::NewDeviceLabeler(manager, config, join_facts));
  } catch (...) {
    // Neither task may outlive this frame (they write its locals).
    facts_task.cancel_or_wait();
    sriov_task.cancel_or_wait();
    throw;
  }
  if (overlap) {
    int64_t j0 = trace::stamp();
    facts_task.cancel_or_wait();  // no devices: the labeler never needed them
    sriov_task.run_or_wait();
    // Where an overlapped cycle waits: how long after the hand-off the node
    // facts started (a worker's wake-up, or this thread taking them over),
    // and how long this thread then waited for the SR-IOV lookup.
    if (traced) trace::record_top("sriov.join", trace::now_ns() - j0);
    trace::record("facts.start", facts_start ? facts_start - submitted : 0);
    trace::record("facts(overlapped)", facts_ns);
    trace::record("sriov(overlapped)", sriov_ns);
  } else {
    {
      trace::Span span("sriov");
      scan_sriov();
    }
    trace::record("facts", facts_ns);
  }
  // Which way the lookup went (kept / checked / re-read) and the node facts'
  // parts, wherever they ran.
  for (const auto& p : facts_detail) trace::record(p.first, p.second);
  for (const auto& p : sriov_detail) trace::record(p.first, p.second);
  if (sriov_error) {
    try {
      std::rethrow_exception(sriov_error);
    } catch (const std::exception& e) {
      throw Error(std::string("error generating labels: ") + e.what());
    }
  }
  {
    trace::Span span("merge");
    // The timestamp labeler lives across cycles (appended); the device
    // labeler and the SR-IOV labels are this cycle's own (moved in).
    // Errors read as the merge of the three would wrap them (lm::merge).
    try {
      try {
        if (timestamp) timestamp->AppendTo(r.labels);
        if (device) device->MoveTo(r.labels);
        lm::from_labels(std::move(sriov_labels))->MoveTo(r.labels);
      } catch (const std::exception& e) {
        throw Error(std::string("error generating labels: ") + e.what());
      }
    } catch (const std::exception& e) {
      throw Error(std::string("error generating labels: ") + e.what());
    }
    device.reset();
  }
  if (r.labels.size() <= 1) log::printf("Warning: no labels generated from any source");
  if (write) {
    {
      trace::Span span("log");
      log::printf("Writing labels to output file");
    }
    trace::Span span("write");
    try {
      lm::write_to_file(r.labels, config.output_file(), !config.oneshot());
    } catch (const std::exception& e) {
      throw Error("error writing file '" + config.output_file() + "': " + e.what());
    }
  }
  r.total_ns = trace::now_ns() - t0;
  r.other_ns = r.total_ns - trace::top_level_ns();
  r.phases = trace::phases();
  r.cpu_end = sched_getcpu();
  return r;
}

bool run(resource::Manager& manager, const std::shared_ptr<sriov::Interface>& sriov, const config::Config& config,
         SignalWatcher* sigs) {
  struct Cleanup {
    const config::Config& c;
    ~Cleanup() {
      if (!c.oneshot() && !c.output_file().empty()) {
        try {
          lm::remove_output_file(c.output_file());
        } catch (const std::exception& e) {
          log::printf("Warning: Error removing output file: %s", e.what());
        }
      }
    }
  } cleanup{config};

  lm::LabelerPtr timestamp = lm::NewTimestampLabeler(config);
  for (;;) {
    // The cycle's log lines ("Writing labels to output file", ...) go out
    // together once the feature file is in place (and on any error).
    log::Hold hold;
    CycleResult r = label_cycle(manager, sriov, config, timestamp, true, config.trace_timing());
    if (config.trace_timing())
      log::printf("Timing: %s cpu=%d,%d,%d", trace::summary(r.total_ns).c_str(), r.cpu_start, r.cpu_end, r.cpu_facts);
    if (config.oneshot()) return false;

    log::printf("Sleeping for %s", format_duration(config.sleep_interval()).c_str());
    hold.flush();
    std::optional<int> sig;
    if (sigs) {
      sig = sigs->wait(config.sleep_interval());
    } else {
      struct timespec ts;
      ts.tv_sec = static_cast<time_t>(config.sleep_interval() / 1000000000LL);
      ts.tv_nsec = static_cast<long>(config.sleep_interval() % 1000000000LL);
      nanosleep(&ts, nullptr);
    }
    if (!sig) continue;  // rerun
    if (*sig == SIGHUP) {
      log::printf("Received SIGHUP, restarting.");
      return true;
    }
    log::printf("Received signal \"%s\", shutting down.", SignalWatcher::name(*sig).c_str());
    return false;
  }
}

namespace {
// Process-level timeline for --trace-timing (a oneshot Job's latency is
// mostly outside the labeling cycle: process start, backend selection and
// library loading, teardown).  Absolute CLOCK_MONOTONIC milliseconds, so a
// parent that timed the spawn can attribute the rest.
struct ProcessTimeline {
  bool enabled = false;
  int64_t main_ns = 0, configured_ns = 0, manager_ns = 0, run_done_ns = 0;
} g_timeline;
}  // namespace

void start(const Context& ctx, SignalWatcher& sigs) {
  for (;;) {
    log::printf("Loading configuration.");
    config::Config c;
    try {
      c = load_config(ctx);
    } catch (const std::exception& e) {
      throw Error(std::string("unable to load config: ") + e.what());
    }
    config::disable_resource_renaming(c);
    // The first SR-IOV scan (every amdgpu/gim-bound function, ~0.3 ms in a
    // fresh process) starts now, on a worker, while this thread logs the
    // configuration and selects the backend; the first cycle then finds its
    // result kept (unchanged uevent counter) or waits for it to finish.
    auto sriov = sriov::new_sriov_lib(c.sysfs_root());
    struct Prefetch {  // never outlives this iteration (an error exits the process)
      WorkerPool::Task task;
      ~Prefetch() { task.cancel_or_wait(); }
    } prefetch;
    // Loop mode only: a Job's worker thread would cost more than it hides
    // (see label_cycle).
    if (!c.oneshot())
      prefetch.task = WorkerPool::instance().submit([sriov] {
        try {
          sriov->Devices();
        } catch (...) {  // the cycle's own scan reports it
        }
      });
    log::printf("\nRunning with config:\n%s", config::to_json(c).c_str());
    // A process killed without its exit cleanup (OOM, SIGKILL, node crash)
    // left its temporary files in <dir>/gfd-tmp: remove them before the
    // first write.  Loop mode only - a oneshot Job leaves the directory to
    // the DaemonSet that may share it.  Every (re)start: a SIGHUP may have
    // moved the output file to a directory a crashed daemon wrote to (the
    // previous run's own gfd-tmp/ is already gone with its exit cleanup).
    if (!c.oneshot() && !c.output_file().empty()) {
      try {
        lm::sweep_temp_dir(c.output_file());
      } catch (const std::exception& e) {
        log::printf("Warning: %s", e.what());
      }
    }
    if (!c.oneshot()) WorkerPool::instance().load_topology();  // before the first cycle
    g_timeline.enabled = c.trace_timing();
    if (!g_timeline.configured_ns) g_timeline.configured_ns = trace::now_ns();

    bool restart;
    {
      resource::ManagerPtr manager = resource::new_manager(c);
      // The warm-start manager's amd-smi initialisation starts here, not in
      // the first cycle's Init.
      if (!c.oneshot()) manager->Prepare();
      if (!g_timeline.manager_ns) g_timeline.manager_ns = trace::now_ns();

      log::printf("Start running");
      restart = run(*manager, sriov, c, &sigs);
      g_timeline.run_done_ns = trace::now_ns();
    }  // the manager (and a persistent amd-smi session) is released here
    if (!restart) return;
  }
}

int gfd_main(int argc, char** argv) {
  const std::string app = "GPU Feature Discovery";
  const std::string usage = "generate labels for AMD devices";
  std::vector<std::string> args(argv + 1, argv + argc);
  auto defs = gfd_flags();
  Context ctx;
  try {
    ctx = Context::parse(defs, args);
  } catch (const UsageError& e) {
    fprintf(stderr, "Incorrect Usage: %s\n\n%s", e.what(), help_text(defs, app, usage, info::version_string()).c_str());
    log::printf("Error: %s", e.what());
    return 1;
  }
  if (ctx.help_requested()) {
    fputs(help_text(defs, app, usage, info::version_string()).c_str(), stdout);
    return 0;
  }
  if (ctx.version_requested()) {
    printf("%s version %s\n", app.c_str(), info::version_string().c_str());
    return 0;
  }
  g_timeline.main_ns = trace::now_ns();
  // CPU placement (util/affinity.h, util/pool.h).  The default, follow,
  // leaves the cycle thread to the scheduler and keeps only the pool's
  // workers on the L3 cache domain it runs on, so a hand-off never crosses
  // the fabric: back to back 0.027-0.050 -> 0.025-0.027 ms, after an idle
  // second 0.24-0.32 -> 0.25-0.28 ms (profiles/affinity_r3.txt).  l3 pins
  // the whole process to the domain it starts on (before any thread exists:
  // workers inherit the mask); none changes nothing.
  std::string placement = ctx.String("cpu-affinity");
  if (placement == "l3") {
    if (std::string pinned = affinity::pin_to_current_l3(); !pinned.empty()) log::printf("CPU affinity: %s", pinned.c_str());
  } else if (placement == "follow") {
    WorkerPool::instance().set_follow(true);
    log::printf("CPU affinity: workers follow the labeling thread's L3 cache domain");
  } else if (placement != "none") {
    log::printf("Error: unknown --cpu-affinity '%s' (expected none, follow or l3)", placement.c_str());
    return 1;
  }
  int rc = 0;
  {
    log::printf("Starting OS watcher.");
    SignalWatcher sigs;
    try {
      start(ctx, sigs);
    } catch (const std::exception& e) {
      log::printf("Exiting");
      log::printf("Error: %s", e.what());
      return 1;
    }
    log::printf("Exiting");
  }
  if (g_timeline.enabled) {
    int64_t end = trace::now_ns();
    auto ms = [](int64_t ns) { return static_cast<double>(ns) / 1e6; };
    log::printf("Process timing: main_at=%.3fms config=%.3fms backend_select=%.3fms run=%.3fms teardown=%.3fms",
                ms(g_timeline.main_ns), ms(g_timeline.configured_ns - g_timeline.main_ns),
                ms(g_timeline.manager_ns - g_timeline.configured_ns), ms(g_timeline.run_done_ns - g_timeline.manager_ns),
                ms(end - g_timeline.run_done_ns));
  }
  return rc;
}

}  // namespace gfd::cli
