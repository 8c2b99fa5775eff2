// Resource managers that do not talk to hardware: Null, the sticky
// fallback-to-Null decorator, and the scripted Mock used by tests and by
// `--backend=mock`.
//
// Reference: internal/resource/null.go:23-57, fallback.go:23-64,
// factory.go:33-39 (WithConfig), testing/resource-testing.go:26-134.
#pragma once

#include <functional>
#include <optional>
#include <string>
#include <vector>

#include "config/config.h"
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>

#include "config/yaml.h"
#include "resource/types.h"

namespace gfd::resource {

// No devices; Init/Shutdown are no-ops; version queries are unsupported.
class NullManager : public Manager {
 public:
  void Init() override {}
  void Shutdown() override {}
  std::vector<DevicePtr> GetDevices() override { return {}; }
  std::string GetDriverVersion() override;
  std::optional<RuntimeVersion> GetRuntimeVersion() override;
  std::string Name() const override { return "null"; }
};

// Becomes a Null manager on the first Init error and stays that way until the
// manager is rebuilt (SIGHUP reload) — the reference's sticky semantics.
class FallbackManager : public Manager {
 public:
  explicit FallbackManager(ManagerPtr wraps);
  void Init() override;
  void Shutdown() override { current_->Shutdown(); }
  std::vector<DevicePtr> GetDevices() override { return current_->GetDevices(); }
  std::string GetDriverVersion() override { return current_->GetDriverVersion(); }
  std::optional<RuntimeVersion> GetRuntimeVersion() override { return current_->GetRuntimeVersion(); }
  std::string Name() const override { return "fallback(" + current_->Name() + ")"; }
  std::optional<VersionSources> VersionFiles() const override { return current_->VersionFiles(); }
  void Prepare() override { current_->Prepare(); }
  bool fell_back() const { return fell_back_; }

 private:
  ManagerPtr current_;
  bool fell_back_ = false;
};

// `--backend=auto` on a node with both amd-smi and a KFD topology: the
// candidates in order of preference (amd-smi, then KFD sysfs).  Init keeps
// the first one whose Init succeeds - an amd-smi library that cannot talk to
// the driver (version skew, no /dev/kfd in the container) still leaves the
// node labelled from sysfs - and the choice sticks until the manager is
// rebuilt (SIGHUP reload).  Init fails only when every candidate failed.
// (The reference simply disables its second backend on such nodes,
// internal/resource/factory.go:55-59.)
class PreferenceManager : public Manager {
 public:
  explicit PreferenceManager(std::vector<ManagerPtr> candidates);
  void Init() override;
  void Shutdown() override { current_->Shutdown(); }
  std::vector<DevicePtr> GetDevices() override { return current_->GetDevices(); }
  std::string GetDriverVersion() override { return current_->GetDriverVersion(); }
  std::optional<RuntimeVersion> GetRuntimeVersion() override { return current_->GetRuntimeVersion(); }
  std::string Name() const override { return current_->Name(); }
  std::optional<VersionSources> VersionFiles() const override { return current_->VersionFiles(); }
  // Index of the candidate in use (0 until an Init fell through).
  size_t chosen() const { return chosen_; }

 private:
  std::vector<ManagerPtr> candidates_;
  ManagerPtr current_;
  size_t chosen_ = 0;
};

// `--backend=auto` in daemon mode on a node with both amd-smi and a KFD
// topology, amd-smi session persistent.  amd-smi's first amdsmi_init costs
// ~25 ms (it parses all of /proc/cpuinfo, profiles/amdsmi_init_profile.txt)
// while the KFD topology answers the same questions with byte-identical
// labels (tests/test_gpu.py).  So the first cycle is labelled from KFD while
// the preferred manager initialises - and takes one snapshot, paying its
// first-query costs - on a background thread; the first cycle
// that finds it ready switches to it for good.  If its initialisation
// failed - or it fails later - the quick manager keeps serving until the
// manager is rebuilt (SIGHUP), as with PreferenceManager.  Switching happens
// only in Init, between cycles.
class WarmStartManager : public Manager {
 public:
  WarmStartManager(ManagerPtr preferred, ManagerPtr quick);
  // Waits for a background initialisation, at most teardown_wait_ms: a
  // library wedged in its init must not keep the daemon from exiting on
  // SIGTERM or reloading on SIGHUP (the warmer is then left to finish alone).
  ~WarmStartManager() override;
  void Init() override;
  void Shutdown() override { current_->Shutdown(); }
  std::vector<DevicePtr> GetDevices() override;
  std::string GetDriverVersion() override { return current_->GetDriverVersion(); }
  std::optional<RuntimeVersion> GetRuntimeVersion() override { return current_->GetRuntimeVersion(); }
  std::string Name() const override { return current_->Name(); }
  std::optional<VersionSources> VersionFiles() const override { return current_->VersionFiles(); }
  // Starts the preferred manager's initialisation now rather than in the
  // first Init (the thread start is then not part of the first cycle).
  void Prepare() override;
  // The preferred manager is the one in use.
  bool warmed() const { return state_ == State::preferred; }
  int64_t teardown_wait_ms = 5000;
  struct Warmer;

 private:
  enum class State { cold, warming, preferred, quick_only };
  void fall_back(const std::string& why);
  // cold -> warming, unless an earlier manager's warmer still runs.
  void start_warmer();
  // Both managers describe the node again, now (device_summary each); true
  // if they agree.
  bool second_look(std::string* quick_now, std::string* preferred_now);
  bool waited_logged_ = false;

  ManagerPtr preferred_, quick_, current_;
  State state_ = State::cold;
  std::thread thread_;
  std::shared_ptr<Warmer> warmer_;
  std::string quick_devices_;  // the quick manager's last devices (device_summary), while warming
};

// Whether a WarmStartManager was torn down while its warmer was still
// initialising the preferred manager and that warmer has not finished: the
// process must then not run static destructors (the warmer may be inside
// the library), so main() leaves with _exit.
bool warmer_left_running();

// What the labels of `devices` depend on, one line per device (and
// partition): compared when the daemon switches backends, so a difference
// between them - and the label change it causes - is logged.
std::string device_summary(const std::vector<DevicePtr>& devices);

// Wrap `m` in a FallbackManager unless failOnInitError is set.
ManagerPtr with_config(ManagerPtr m, const config::Config& c);

// Scripted manager.  Every method can be overridden or made to fail; calls
// are counted so tests can assert on them (moq's call recording).
class MockManager : public Manager {
 public:
  MockManager() = default;
  explicit MockManager(std::vector<DevicePtr> devices);

  void Init() override;
  void Shutdown() override;
  std::vector<DevicePtr> GetDevices() override;
  std::string GetDriverVersion() override;
  std::optional<RuntimeVersion> GetRuntimeVersion() override;
  std::string Name() const override { return "mock"; }

  MockManager& with_error_on_init(std::string msg);

  std::vector<DevicePtr> devices;
  std::optional<std::string> init_error;
  std::optional<std::string> devices_error;
  std::optional<std::string> driver_error;
  std::optional<std::string> runtime_error;
  std::string driver_version = "6.12.12";
  std::optional<RuntimeVersion> runtime_version = RuntimeVersion{7, 2};  // nullopt: no ROCm on the node

  int init_calls = 0;
  int shutdown_calls = 0;
  int get_devices_calls = 0;
};

// ---- Builders mirroring internal/resource/testing/resource-testing.go ----

// A full (unpartitioned) GPU: name MOCKMODEL, gfx950, 300 MiB, 256 CUs, 8 XCDs.
std::shared_ptr<SnapshotDevice> new_full_gpu();
// A GPU in a partitioned compute mode exposing `partitions`.  Like the
// reference's MIG-enabled mock it reports no ISA target (arch labels are
// omitted) and is partition capable.
std::shared_ptr<SnapshotDevice> new_partitioned_gpu(std::vector<std::shared_ptr<SnapshotDevice>> partitions = {});
// Generic mock GPU; `partitioned` selects the IsPartitioned answer.
std::shared_ptr<SnapshotDevice> new_mock_gpu(bool partitioned);
// A compute partition named "<mode>.<xcds>xcd.<gb>gb" whose default
// attributes are memory=<gb>, compute-units=0, xcds=<xcds>, engines.*=0,
// compute-partition=<MODE>, memory-partition=NPS1.  `overrides` replace
// attributes by key.
std::shared_ptr<SnapshotDevice> new_partition(const std::string& mode, int xcds, uint64_t gb,
                                              const Attributes& overrides = {});

// Load a mock manager from a YAML/JSON fixture (format in docs/BACKENDS.md).
std::shared_ptr<MockManager> load_mock_manager(const std::string& path);
std::shared_ptr<MockManager> mock_manager_from_node(const yaml::Node& root);

}  // namespace gfd::resource
