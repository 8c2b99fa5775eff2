// Daemon lifecycle: configuration loading, the labeling loop, signals.
//
// Reference: cmd/gpu-feature-discovery/main.go:22-270 (main, loadConfig,
// start, run, removeOutputFile, disableResourceRenamingInConfig) and
// watchers.go:26-31 (newOSWatcher).
#pragma once

#include <memory>
#include <optional>
#include <string>
#include <vector>

#include "cli/flags.h"
#include "config/config.h"
#include "lm/labels.h"
#include "resource/types.h"
#include "sriov/sriov.h"
#include "util/trace.h"

namespace gfd::cli {

// flags.go:75-121: a field is taken from the CLI/env when IsSet, or from the
// flag default when the config file left it unset.
void update_from_cli_flags(config::Flags& f, const Context& ctx);
// main.go:96-107 + config.go:43-57: file (if --config-file) then flags.
config::Config load_config(const Context& ctx);

// Blocks SIGHUP/SIGINT/SIGTERM/SIGQUIT for the process and lets the run loop
// wait for them synchronously (sigtimedwait), which doubles as the sleep
// between labeling cycles.  Must be constructed before any thread starts.
class SignalWatcher {
 public:
  SignalWatcher();
  // Wait up to `timeout_ns`; returns the signal number or nullopt on timeout.
  std::optional<int> wait(int64_t timeout_ns);
  static std::string name(int sig);
};

struct CycleResult {
  lm::Labels labels;
  int64_t total_ns = 0;
  int64_t other_ns = 0;  // total minus the top-level phases (unattributed)
  std::vector<trace::Phase> phases;
  // CPU the cycle thread started / ended on, and the one the node facts ran
  // on (a worker's, or the cycle thread's if it took them over).
  int cpu_start = -1, cpu_end = -1, cpu_facts = -1;
};

// One labeling cycle: build labelers (device + SR-IOV), merge with the
// timestamp labeler, evaluate, and write the feature file if `write`.
// `traced`: record the phases (util/trace.h; the daemon's under
// --trace-timing); untraced, `phases` is empty and other_ns the total.
CycleResult label_cycle(resource::Manager& manager, const std::shared_ptr<sriov::Interface>& sriov,
                        const config::Config& config, const lm::LabelerPtr& timestamp, bool write,
                        bool traced = true);

// main.go:148-210.  Returns true if the caller should reload (SIGHUP).
// `sigs` may be null (oneshot tests).
bool run(resource::Manager& manager, const std::shared_ptr<sriov::Interface>& sriov, const config::Config& config,
         SignalWatcher* sigs);

// main.go:109-146.  Throws gfd::Error on failure.
void start(const Context& ctx, SignalWatcher& sigs);

// Process entry point; returns the exit code.
int gfd_main(int argc, char** argv);

}  // namespace gfd::cli
