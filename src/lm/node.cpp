#include "lm/node.h"

#include <atomic>
#include <ctime>
#include <exception>
#include <map>

#include "lm/keys.h"
#include "lm/resource.h"
#include "resource/versions.h"
#include "util/error.h"
#include "util/fs.h"
#include "util/log.h"
#include "util/strings.h"
#include "util/trace.h"

namespace gfd::lm {

LabelerPtr NewTimestampLabeler(const config::Config& config, int64_t unix_seconds) {
  if (config.no_timestamp()) return empty();
  return from_labels(Labels{{keys::kTimestamp, std::to_string(unix_seconds)}});
}

LabelerPtr NewTimestampLabeler(const config::Config& config) {
  return NewTimestampLabeler(config, static_cast<int64_t>(time(nullptr)));
}

namespace {

Labels machine_type_labels(const std::string& path, std::string* warning) {
  std::string machine = "unknown";
  if (!path.empty()) {
    auto r = fs::read_dmi(path);  // kept when it is the kernel's DMI (fixed until reboot)
    if (r.ok()) {
      machine = str::trim(r.data);
    } else {
      *warning = "WARNING: error getting machine type from " + path + ": could not open machine type file: open " +
                 path + ": " + fs::errno_str(r.err);
    }
  }
  return Labels{{keys::kMachine, sanitize_label_value(str::replace_all(machine, " ", "-"))}};
}

// nvml.go:75-106: the driver version is fetched and checked before the
// runtime version is asked for.  A node without a ROCm release (nullopt:
// driver-only hosts whose workloads bring ROCm in their images) gets the
// driver labels only; failing to read a source that should be there (an
// explicitly configured version file) is an error, as in the reference.
template <typename DriverFn, typename RuntimeFn>
LabelerPtr version_labeler(DriverFn&& get_driver, RuntimeFn&& get_runtime) {
  std::string driver = GFD_WRAP("error getting driver version", get_driver());
  auto parts = str::split(driver, '.');
  if (parts.size() > 3 || parts.size() < 2)
    throw Error("error getting driver version: Version \"" + driver + "\" does not match format \"X.Y[.Z]\"");
  std::optional<resource::RuntimeVersion> rt = GFD_WRAP("error getting ROCm runtime version", get_runtime());
  Labels l{
      {keys::kDriverMajor, sanitize_label_value(parts[0])},
      {keys::kDriverMinor, sanitize_label_value(parts[1])},
      {keys::kDriverRev, parts.size() > 2 ? sanitize_label_value(parts[2]) : ""},
  };
  if (rt) {
    l[keys::kRuntimeMajor] = std::to_string(rt->major);
    l[keys::kRuntimeMinor] = std::to_string(rt->minor);
  } else {
    static std::atomic<bool> warned{false};
    if (!warned.exchange(true))
      log::printf("WARNING: no ROCm release found on the node; omitting the rocm.runtime labels "
                  "(in a pod, mount the host's /opt and set --host-root)");
  }
  return from_labels(std::move(l));
}

}  // namespace

LabelerPtr NewMachineTypeLabeler(const std::string& path) {
  std::string warning;
  Labels l = machine_type_labels(path, &warning);
  if (!warning.empty()) log::printf("%s", warning.c_str());
  return from_labels(std::move(l));
}

LabelerPtr NewVersionLabeler(resource::Manager& manager) {
  return version_labeler([&] { return manager.GetDriverVersion(); }, [&] { return manager.GetRuntimeVersion(); });
}

NodeFacts ReadNodeFacts(const config::Config& config, const std::optional<resource::VersionSources>& version_files) {
  NodeFacts f;
  {
    trace::Span span("facts.machine");
    f.machine = machine_type_labels(config.machine_type_file(), &f.machine_warning);
  }
  if (version_files) {
    f.have_versions = true;
    {
      trace::Span span("facts.driver");
      f.driver_version = resource::driver_version(version_files->root);
    }
    trace::Span span("facts.runtime");
    try {
      f.runtime_version = resource::rocm_version(*version_files);
    } catch (const std::exception& e) {
      f.runtime_error = e.what();
    }
  }
  return f;
}

LabelerPtr NewPartitionCapabilityLabeler(resource::Manager& manager) {
  auto devices = manager.GetDevices();
  if (devices.empty()) return empty();
  bool capable = false;
  for (const auto& d : devices) {
    capable = GFD_WRAP("error getting partition capability", d->IsPartitionCapable());
    if (capable) break;
  }
  return from_labels(Labels{{keys::kPartitionCapable, str::bool_str(capable)}});
}

LabelerPtr NewTopologyLabeler(resource::Manager& manager) {
  auto devices = manager.GetDevices();
  if (devices.empty()) return empty();
  auto agree = [&](auto get) -> std::string {
    std::string v;
    bool first = true;
    for (const auto& d : devices) {
      std::string x = get(d->Info());
      if (first) {
        v = x;
        first = false;
      } else if (x != v) {
        return "mixed";
      }
    }
    return v;
  };
  Labels l;
  std::string cp = agree([](const resource::DeviceInfo& i) { return i.compute_partition; });
  std::string mp = agree([](const resource::DeviceInfo& i) { return i.memory_partition; });
  std::string vm = agree([](const resource::DeviceInfo& i) { return i.virtualization; });
  if (!cp.empty()) l[keys::kComputePartition] = sanitize_label_value(cp);
  if (!mp.empty()) l[keys::kMemoryPartition] = sanitize_label_value(mp);
  if (!vm.empty()) l[keys::kVirtualization] = sanitize_label_value(vm);
  int links = -1;
  for (const auto& d : devices) {
    int x = d->Info().xgmi_links;
    if (x < 0) continue;
    links = links < 0 ? x : std::min(links, x);
  }
  if (links >= 0) l[keys::kXgmiLinks] = std::to_string(links);
  return from_labels(std::move(l));
}

namespace {

class SriovLabeler : public Labeler {
 public:
  explicit SriovLabeler(std::shared_ptr<sriov::Interface> lib) : lib_(std::move(lib)) {}
  Labels GetLabels() override {
    std::vector<sriov::Function> fns;
    try {
      fns = lib_->Devices();
    } catch (const std::exception& e) {
      throw Error(std::string("unable to get SR-IOV devices: ") + e.what());
    }
    // Node-level summary.  A host with VFs enabled is role "pf" (its own GPUs
    // are physical functions; host-side VFs are handed to VMs), a guest that
    // sees VFs is role "vf".  VF counts are summed over all PFs.
    Labels l;
    if (fns.empty()) return l;
    l[keys::kSriovPresent] = "true";
    bool any_pf = false;
    int total = 0, num = 0;
    for (const auto& f : fns) {
      const auto& info = f.GetInfo();
      if (info.role != "pf") continue;
      any_pf = true;
      total += info.total_vfs > 0 ? info.total_vfs : 0;
      num += info.num_vfs > 0 ? info.num_vfs : 0;
    }
    l[keys::kSriovRole] = any_pf ? "pf" : "vf";
    if (any_pf) {
      l[keys::kSriovTotalVfs] = std::to_string(total);
      l[keys::kSriovNumVfs] = std::to_string(num);
      // vgpu.go:44-52 labels the host driver; an MxGPU host's is GIM.
      if (auto v = lib_->HostDriverVersion()) l[keys::kSriovHostDriverVersion] = sanitize_label_value(*v);
    }
    return l;
  }

 private:
  std::shared_ptr<sriov::Interface> lib_;
};

// Calls Shutdown when leaving scope (the reference's `defer manager.Shutdown()`).
class ShutdownGuard {
 public:
  explicit ShutdownGuard(resource::Manager& m) : m_(m) {}
  ~ShutdownGuard() {
    trace::Span span("shutdown");
    try {
      m_.Shutdown();
    } catch (const std::exception& e) {
      log::printf("Warning: resource manager shutdown failed: %s", e.what());
    }
  }

 private:
  resource::Manager& m_;
};

}  // namespace

LabelerPtr NewSriovLabeler(std::shared_ptr<sriov::Interface> lib) { return std::make_shared<SriovLabeler>(std::move(lib)); }

LabelerPtr NewDeviceLabeler(resource::Manager& manager, const config::Config& config,
                            const std::function<const NodeFacts&()>& facts) {
  {
    trace::Span span("init");
    try {
      manager.Init();
    } catch (const std::exception& e) {
      throw Error(std::string("failed to initialize resource manager: ") + e.what());
    }
  }
  ShutdownGuard guard(manager);

  std::vector<resource::DevicePtr> devices;
  {
    trace::Span span("enumerate");
    devices = GFD_WRAP("error getting devices", manager.GetDevices());
  }
  if (devices.empty()) return empty();

  trace::Span span("label");
  // The device-derived labelers first: the node facts are read on a worker
  // meanwhile (daemon.cpp label_cycle), and are joined only when this
  // thread has nothing else to do.  Their errors wait until the machine and
  // version labelers are built, so that the error reported is the first in
  // the reference's order (nvml.go:44-67: machine type, version, MIG
  // capability, resources).
  std::exception_ptr device_error;
  auto deferred = [&](auto make) -> LabelerPtr {
    if (device_error) return nullptr;
    try {
      return make();
    } catch (...) {
      device_error = std::current_exception();
      return nullptr;
    }
  };
  auto capability = deferred([&] {
    return GFD_WRAP("error creating partition capability labeler", NewPartitionCapabilityLabeler(manager));
  });
  auto topology = deferred([&] { return GFD_WRAP("error creating topology labeler", NewTopologyLabeler(manager)); });
  auto resources =
      deferred([&] { return GFD_WRAP("error creating resource labeler", NewResourceLabeler(manager, config)); });
  const NodeFacts* pre = facts ? &facts() : nullptr;
  LabelerPtr machine, version;
  if (pre) {
    if (!pre->machine_warning.empty()) log::printf("%s", pre->machine_warning.c_str());
    machine = from_labels(pre->machine);
  } else {
    machine = GFD_WRAP("failed to construct machine type labeler", NewMachineTypeLabeler(config.machine_type_file()));
  }
  if (pre && pre->have_versions) {
    version = GFD_WRAP("failed to construct version labeler",
                       version_labeler([&] { return pre->driver_version; },
                                       [&] {
                                         if (!pre->runtime_error.empty()) throw Error(pre->runtime_error);
                                         return pre->runtime_version;
                                       }));
  } else {
    version = GFD_WRAP("failed to construct version labeler", NewVersionLabeler(manager));
  }
  if (device_error) std::rethrow_exception(device_error);
  return merge({machine, version, capability, topology, resources});
}

LabelerPtr NewLabelers(resource::Manager& manager, std::shared_ptr<sriov::Interface> sriov,
                       const config::Config& config) {
  auto device = GFD_WRAP("error creating device labeler", NewDeviceLabeler(manager, config));
  return merge({device, NewSriovLabeler(std::move(sriov))});
}

}  // namespace gfd::lm
