#include "resource/managers.h"

#include "util/error.h"
#include "util/fs.h"
#include "util/log.h"
#include "util/strings.h"
#include "util/trace.h"

namespace gfd::resource {

// ---------------------------------------------------------------------------
// Null / Fallback

std::string NullManager::GetDriverVersion() { throw Error("GetDriverVersion is unsupported"); }
std::optional<RuntimeVersion> NullManager::GetRuntimeVersion() { throw Error("GetRuntimeVersion is unsupported"); }

FallbackManager::FallbackManager(ManagerPtr wraps) : current_(std::move(wraps)) {}

void FallbackManager::Init() {
  try {
    current_->Init();
  } catch (const std::exception& e) {
    log::printf("Warning: failed to initialize resource manager: %s", e.what());
    current_ = std::make_shared<NullManager>();
    fell_back_ = true;
  }
}

PreferenceManager::PreferenceManager(std::vector<ManagerPtr> candidates) : candidates_(std::move(candidates)) {
  if (candidates_.empty()) throw Error("PreferenceManager needs at least one manager");
  current_ = candidates_.front();
}

void PreferenceManager::Init() {
  // Init runs once per labeling cycle: start from the manager in use, so a
  // candidate that failed is not retried before the next reload.
  std::string errors;
  for (size_t i = chosen_; i < candidates_.size(); ++i) {
    try {
      candidates_[i]->Init();
      bool switched = i != chosen_;
      current_ = candidates_[i];
      chosen_ = i;
      if (switched) log::printf("Using the %s manager", current_->Name().c_str());
      return;
    } catch (const std::exception& e) {
      log::printf("Warning: %s manager failed to initialize: %s", candidates_[i]->Name().c_str(), e.what());
      errors += (errors.empty() ? "" : "; ") + candidates_[i]->Name() + ": " + e.what();
    }
  }
  throw Error("no resource manager could be initialized (" + errors + ")");
}

struct WarmStartManager::Warmer {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  std::string error;    // empty: the preferred manager is ready
  std::string devices;  // its first snapshot (device_summary)
  int64_t ns = 0;
};

namespace {
// The warmer a torn-down manager left running (its library init wedged), if
// any.  A wedged amdsmi_init holds the library's process-wide lock, so a new
// warmer would only block behind it: a reloaded daemon waits for this one to
// finish before starting its own, and at most one warmer is ever left
// behind, however many SIGHUPs come.
std::mutex g_orphan_mu;
std::shared_ptr<WarmStartManager::Warmer> g_orphan;

bool orphan_running() {
  std::shared_ptr<WarmStartManager::Warmer> w;
  {
    std::lock_guard<std::mutex> g(g_orphan_mu);
    w = g_orphan;
  }
  if (!w) return false;
  std::lock_guard<std::mutex> lk(w->mu);
  if (!w->done) return true;
  std::lock_guard<std::mutex> g(g_orphan_mu);
  if (g_orphan == w) g_orphan.reset();
  return false;
}
}  // namespace

bool warmer_left_running() { return orphan_running(); }

WarmStartManager::WarmStartManager(ManagerPtr preferred, ManagerPtr quick)
    : preferred_(std::move(preferred)), quick_(std::move(quick)), current_(quick_) {}

WarmStartManager::~WarmStartManager() {
  if (!thread_.joinable()) return;
  std::unique_lock<std::mutex> lk(warmer_->mu);
  // system_clock: a steady_clock wait is pthread_cond_clockwait, which GCC
  // 11's ThreadSanitizer does not intercept (it then reports the waker's lock
  // of `mu` as a double lock); a clock step only moves this bound.
  if (warmer_->cv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(teardown_wait_ms),
                             [&] { return warmer_->done; })) {
    lk.unlock();
    thread_.join();
    return;
  }
  lk.unlock();
  log::printf("Warning: the %s manager is still initializing after %lld ms; not waiting for it",
              preferred_->Name().c_str(), static_cast<long long>(teardown_wait_ms));
  {
    std::lock_guard<std::mutex> g(g_orphan_mu);
    g_orphan = warmer_;
  }
  thread_.detach();  // it owns what it uses (the manager and its state)
}

void WarmStartManager::fall_back(const std::string& why) {
  log::printf("Warning: %s manager failed to initialize: %s", preferred_->Name().c_str(), why.c_str());
  log::printf("Using the %s manager", quick_->Name().c_str());
  state_ = State::quick_only;
  current_ = quick_;
}

std::vector<DevicePtr> WarmStartManager::GetDevices() {
  auto devs = current_->GetDevices();
  if (state_ == State::warming) quick_devices_ = device_summary(devs);
  return devs;
}

void WarmStartManager::Prepare() {
  if (state_ == State::cold) start_warmer();
}

void WarmStartManager::start_warmer() {
  if (orphan_running()) {
    // An earlier manager's warmer is still stuck in the library's init:
    // label from the quick manager and look again next cycle.
    if (!waited_logged_) {
      log::printf("The %s manager of the previous configuration is still initializing; labeling from the %s "
                  "manager until it finishes", preferred_->Name().c_str(), quick_->Name().c_str());
      waited_logged_ = true;
    }
    return;
  }
  // A persistent session stays initialised after Shutdown: the warmer
  // opens it and takes one snapshot - the library's first queries of a
  // device (~1.2 ms on MI355X: ASIC info, KFD node, virtualization mode)
  // and the session caches are paid here too - so the cycle that switches
  // over finds everything ready.
  warmer_ = std::make_shared<Warmer>();
  thread_ = std::thread([w = warmer_, m = preferred_] {
    int64_t t0 = trace::now_ns();
    std::string error, devices;
    try {
      m->Init();
      try {
        devices = device_summary(m->GetDevices());
      } catch (...) {
        m->Shutdown();
        throw;
      }
      m->Shutdown();
    } catch (const std::exception& e) {
      error = e.what();
    }
    std::lock_guard<std::mutex> lk(w->mu);
    w->error = std::move(error);
    w->devices = std::move(devices);
    w->ns = trace::now_ns() - t0;
    w->done = true;
    w->cv.notify_all();
  });
  state_ = State::warming;
  log::printf("Initializing the %s manager in the background; labeling from the %s manager meanwhile",
              preferred_->Name().c_str(), quick_->Name().c_str());
}

// The first comparison used the warmer's snapshot and the quick manager's
// last published one, taken at different times: a node that changed in
// between (a partition switch during start-up) must not keep the daemon off
// the preferred manager for its whole life.  So before deciding, both
// describe the node again, back to back (once per start iteration).
bool WarmStartManager::second_look(std::string* quick_now, std::string* preferred_now) {
  auto describe = [](Manager& m, std::string* out) {
    try {
      m.Init();
      try {
        *out = device_summary(m.GetDevices());
      } catch (...) {
        m.Shutdown();
        throw;
      }
      m.Shutdown();
      return true;
    } catch (const std::exception& e) {
      *out = std::string("(error: ") + e.what() + ")\n";
      return false;
    }
  };
  bool ok = describe(*quick_, quick_now);
  ok = describe(*preferred_, preferred_now) && ok;
  return ok && *quick_now == *preferred_now;
}

void WarmStartManager::Init() {
  if (state_ == State::cold) {
    start_warmer();
  } else if (state_ == State::warming) {
    std::unique_lock<std::mutex> lk(warmer_->mu);
    if (warmer_->done) {
      std::string error = warmer_->error, devices = warmer_->devices;
      int64_t ns = warmer_->ns;
      lk.unlock();
      thread_.join();
      if (!error.empty()) {
        fall_back(error);
      } else if (std::string quick_now, preferred_now;
                 !quick_devices_.empty() && devices != quick_devices_ && !second_look(&quick_now, &preferred_now)) {
        // Labels from the quick manager are published and the preferred
        // one would change them - also when both describe the node again:
        // keep the published source until the next (re)start, like the
        // reference's fallback, which keeps one backend per start iteration
        // (internal/resource/fallback.go:37-44) - the node's labels never
        // flip because a backend finished starting.
        log::printf("Warning: the %s manager (initialized in the background in %.1f ms) describes the GPUs "
                    "differently from the %s manager, whose labels are published; labeling from the %s manager "
                    "until the next restart (SIGHUP):\n%s:\n%s%s:\n%s",
                    preferred_->Name().c_str(), static_cast<double>(ns) / 1e6, quick_->Name().c_str(),
                    quick_->Name().c_str(), quick_->Name().c_str(), quick_now.c_str(), preferred_->Name().c_str(),
                    preferred_now.c_str());
        state_ = State::quick_only;
        current_ = quick_;
        preferred_.reset();  // its session is not used again
      } else {
        log::printf("Using the %s manager (initialized in the background in %.1f ms%s)", preferred_->Name().c_str(),
                    static_cast<double>(ns) / 1e6,
                    devices != quick_devices_ && !quick_devices_.empty()
                        ? "; the node changed while it started, both describe it the same way now"
                        : "");
        state_ = State::preferred;
        current_ = preferred_;
      }
      quick_devices_.clear();
    }
  }
  if (state_ == State::preferred) {
    try {
      preferred_->Init();
      return;
    } catch (const std::exception& e) {
      fall_back(e.what());
    }
  }
  quick_->Init();
}

std::string device_summary(const std::vector<DevicePtr>& devices) {
  std::string out;
  auto line = [&](const Device& d, const std::string& indent) {
    const auto& i = d.Info();
    out += indent + i.bdf + " " + d.GetName() + " " + i.gfx.name() + " cu=" + std::to_string(i.compute_units) +
           " xcd=" + std::to_string(i.xcds) + " mem=" + std::to_string(i.memory_mib) + "MiB " + i.compute_partition + "/" +
           i.memory_partition + " xgmi=" + std::to_string(i.xgmi_links) + " " + i.virtualization + "\n";
  };
  for (const auto& d : devices) {
    line(*d, "");
    if (!d->IsPartition())
      for (const auto& p : d->GetPartitions()) line(*p, "  ");
  }
  return out;
}

ManagerPtr with_config(ManagerPtr m, const config::Config& c) {
  if (c.fail_on_init_error()) return m;
  return std::make_shared<FallbackManager>(std::move(m));
}

// ---------------------------------------------------------------------------
// Mock

MockManager::MockManager(std::vector<DevicePtr> devs) : devices(std::move(devs)) {}

void MockManager::Init() {
  ++init_calls;
  if (init_error) throw Error(*init_error);
}

void MockManager::Shutdown() { ++shutdown_calls; }

std::vector<DevicePtr> MockManager::GetDevices() {
  ++get_devices_calls;
  if (devices_error) throw Error(*devices_error);
  return devices;
}

std::string MockManager::GetDriverVersion() {
  if (driver_error) throw Error(*driver_error);
  return driver_version;
}

std::optional<RuntimeVersion> MockManager::GetRuntimeVersion() {
  if (runtime_error) throw Error(*runtime_error);
  return runtime_version;
}

MockManager& MockManager::with_error_on_init(std::string msg) {
  init_error = std::move(msg);
  return *this;
}

// ---------------------------------------------------------------------------
// Builders

std::shared_ptr<SnapshotDevice> new_mock_gpu(bool partitioned) {
  DeviceInfo info;
  info.name = "MOCKMODEL";
  info.memory_mib = 300;
  if (!partitioned) {
    info.gfx = GfxTarget{9, 5, 0};
    info.compute_units = 256;
    info.xcds = 8;
    info.compute_partition = "SPX";
  } else {
    info.compute_partition = "CPX";
  }
  info.memory_partition = "NPS1";
  return SnapshotDevice::gpu(std::move(info), partitioned, /*partition_capable=*/partitioned);
}

std::shared_ptr<SnapshotDevice> new_full_gpu() { return new_mock_gpu(false); }

std::shared_ptr<SnapshotDevice> new_partitioned_gpu(std::vector<std::shared_ptr<SnapshotDevice>> partitions) {
  auto d = new_mock_gpu(true);
  d->set_partitions(std::move(partitions));
  return d;
}

std::shared_ptr<SnapshotDevice> new_partition(const std::string& mode, int xcds, uint64_t gb,
                                              const Attributes& overrides) {
  DeviceInfo info;
  info.name = str::to_lower(mode) + "." + std::to_string(xcds) + "xcd." + std::to_string(gb) + "gb";
  info.memory_mib = gb;
  info.xcds = static_cast<uint32_t>(xcds);
  info.compute_partition = str::to_upper(mode);
  info.memory_partition = "NPS1";
  info.attributes = {
      {"memory", std::to_string(gb)},
      {"compute-units", "0"},
      {"xcds", std::to_string(xcds)},
      {"engines.dma", "0"},
      {"engines.decoder", "0"},
      {"engines.encoder", "0"},
      {"engines.jpeg", "0"},
      {"compute-partition", str::to_upper(mode)},
      {"memory-partition", "NPS1"},
  };
  for (const auto& kv : overrides) info.attributes[kv.first] = kv.second;
  return SnapshotDevice::partition(std::move(info));
}

// ---------------------------------------------------------------------------
// Fixture loading

namespace {

using yaml::Node;

std::string scalar_or(const Node* n, const std::string& def) { return n && n->is_scalar() && !n->is_null() ? n->text() : def; }

uint64_t uint_or(const Node* n, uint64_t def) {
  if (!n || n->is_null()) return def;
  if (n->kind() == Node::Kind::Int && n->as_int() >= 0) return static_cast<uint64_t>(n->as_int());
  auto v = str::parse_uint_auto(n->text());
  if (!v) throw Error("mock fixture: expected unsigned integer, got '" + n->text() + "'");
  return *v;
}

bool bool_or(const Node* n, bool def) {
  if (!n || n->is_null()) return def;
  if (n->kind() != Node::Kind::Bool) throw Error("mock fixture: expected bool, got '" + n->text() + "'");
  return n->as_bool();
}

std::vector<std::string> string_list(const Node* n) {
  std::vector<std::string> out;
  if (!n || n->is_null()) return out;
  if (n->is_seq()) {
    for (const auto& i : n->items()) out.push_back(i.text());
  } else {
    for (auto& p : str::split(n->text(), ',')) out.push_back(str::trim(p));
  }
  return out;
}

void load_errors(const Node* n, DeviceInfo& info) {
  if (!n || !n->is_map()) return;
  for (const auto& kv : n->entries()) info.errors[kv.first] = kv.second.text();
}

void load_common(const Node& d, DeviceInfo& info) {
  info.name = scalar_or(d.get("name"), info.name);
  info.bdf = scalar_or(d.get("bdf"), info.bdf);
  info.uuid = scalar_or(d.get("uuid"), info.uuid);
  info.memory_mib = uint_or(d.get("memoryMiB"), info.memory_mib);
  info.compute_units = static_cast<uint32_t>(uint_or(d.get("computeUnits"), info.compute_units));
  info.xcds = static_cast<uint32_t>(uint_or(d.get("xcds"), info.xcds));
  info.compute_partition = scalar_or(d.get("computePartition"), info.compute_partition);
  info.memory_partition = scalar_or(d.get("memoryPartition"), info.memory_partition);
  load_errors(d.get("errors"), info);
}

std::shared_ptr<SnapshotDevice> load_partition(const Node& p, int idx) {
  DeviceInfo info;
  info.partition_id = static_cast<int>(uint_or(p.get("partitionId"), static_cast<uint64_t>(idx)));
  load_common(p, info);
  if (const Node* attrs = p.get("attributes"); attrs && attrs->is_map())
    for (const auto& kv : attrs->entries()) info.attributes[kv.first] = kv.second.text();
  return SnapshotDevice::partition(std::move(info));
}

std::shared_ptr<SnapshotDevice> load_device(const Node& d, int idx) {
  DeviceInfo info;
  info.index = idx;
  info.name = "MOCKMODEL";
  load_common(d, info);
  info.vendor_id = static_cast<uint32_t>(uint_or(d.get("vendorId"), 0x1002));
  info.device_id = static_cast<uint32_t>(uint_or(d.get("deviceId"), 0));
  if (const Node* g = d.get("gfx"); g && !g->is_null()) {
    auto t = parse_gfx_target(g->text());
    if (!t) throw Error("mock fixture: invalid gfx target '" + g->text() + "'");
    info.gfx = *t;
  }
  info.available_compute_partitions = string_list(d.get("availableComputePartitions"));
  info.available_memory_partitions = string_list(d.get("availableMemoryPartitions"));
  if (const Node* x = d.get("xgmiLinks"); x && !x->is_null()) info.xgmi_links = static_cast<int>(uint_or(x, 0));
  info.virtualization = scalar_or(d.get("virtualization"), "");
  bool partitioned = bool_or(d.get("partitioned"), false);
  bool capable = bool_or(d.get("partitionCapable"), info.available_compute_partitions.size() > 1 || partitioned);
  auto dev = SnapshotDevice::gpu(std::move(info), partitioned, capable);
  std::vector<std::shared_ptr<SnapshotDevice>> parts;
  if (const Node* ps = d.get("partitions"); ps && ps->is_seq()) {
    int i = 0;
    for (const auto& p : ps->items()) parts.push_back(load_partition(p, i++));
  }
  dev->set_partitions(std::move(parts));
  return dev;
}

}  // namespace

std::shared_ptr<MockManager> mock_manager_from_node(const yaml::Node& root) {
  auto m = std::make_shared<MockManager>();
  if (root.is_null()) return m;
  if (!root.is_map()) throw Error("mock fixture: top level must be a mapping");
  if (const Node* e = root.get("initError"); e && !e->is_null()) m->init_error = e->text();
  if (const Node* e = root.get("devicesError"); e && !e->is_null()) m->devices_error = e->text();
  if (const Node* e = root.get("driverVersionError"); e && !e->is_null()) m->driver_error = e->text();
  if (const Node* e = root.get("runtimeVersionError"); e && !e->is_null()) m->runtime_error = e->text();
  m->driver_version = scalar_or(root.get("driverVersion"), m->driver_version);
  if (const Node* rv = root.get("runtimeVersion"); rv && !rv->is_null() && rv->text().empty()) {
    m->runtime_version = std::nullopt;  // runtimeVersion: "" - a node without ROCm
  } else if (rv && !rv->is_null()) {
    auto parts = str::split(rv->text(), '.');
    auto maj = parts.size() > 0 ? str::parse_uint(parts[0]) : std::nullopt;
    auto min = parts.size() > 1 ? str::parse_uint(parts[1]) : std::optional<uint64_t>(0);
    if (!maj || !min) throw Error("mock fixture: runtimeVersion must be 'MAJOR.MINOR'");
    m->runtime_version = RuntimeVersion{static_cast<unsigned>(*maj), static_cast<unsigned>(*min)};
  }
  if (const Node* ds = root.get("devices"); ds && ds->is_seq()) {
    int i = 0;
    for (const auto& d : ds->items()) m->devices.push_back(load_device(d, i++));
  }
  return m;
}

std::shared_ptr<MockManager> load_mock_manager(const std::string& path) {
  auto r = fs::read_file(path);
  if (!r.ok()) throw Error("unable to read mock device file '" + path + "': " + fs::errno_str(r.err));
  return mock_manager_from_node(yaml::parse(r.data));
}

}  // namespace gfd::resource
