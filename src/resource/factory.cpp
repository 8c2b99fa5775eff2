#include "resource/factory.h"

#include <cstdlib>

#include "resource/amdsmi.h"
#include "resource/managers.h"
#include "resource/sysfs.h"
#include "resource/versions.h"
#include "util/error.h"
#include "util/log.h"
#include "util/strings.h"

namespace gfd::resource {

namespace {

AmdSmiOptions amdsmi_options(const config::Config& c) {
  AmdSmiOptions o;
  std::string mode = c.amdsmi_session();
  if (mode == "persistent") {
    o.persistent = true;
  } else if (mode == "per-cycle") {
    o.persistent = false;
  } else {
    throw Error("unknown amd-smi session mode '" + mode + "' (expected persistent or per-cycle)");
  }
  o.root = c.sysfs_root();
  o.filter = DeviceFilter::parse(c.visible_devices());
  if (const char* t = std::getenv("GFD_AMDSMI_THREADS"); t && *t) o.threads = static_cast<int>(str::parse_uint(t).value_or(0));
  return o;
}

SysfsOptions sysfs_options(const config::Config& c) {
  SysfsOptions o;
  o.root = c.sysfs_root();
  o.filter = DeviceFilter::parse(c.visible_devices());
  return o;
}

bool log_with_reason(bool is, const std::string& reason, std::string tag) {
  if (!is) tag = "non-" + tag;
  log::printf("Detected %s platform: %s", tag.c_str(), reason.c_str());
  return is;
}

// Startup observability: the runtime and driver versions the
// hardware backends will label with.
void log_versions(const std::string& root) {
  auto rv = rocm_version(root);
  std::string drv = host_driver_version(root);
  log::printf("ROCm runtime %s, amdgpu driver %s",
              rv ? (std::to_string(rv->major) + "." + std::to_string(rv->minor)).c_str() : "not found",
              extract_version(drv).value_or(drv).c_str());
}

}  // namespace

ManagerPtr get_manager(const config::Config& c) {
  std::string backend = c.backend();
  if (backend == "mock") {
    if (c.mock_file().empty()) throw Error("--backend=mock requires --mock-file");
    log::printf("Using mock manager (%s)", c.mock_file().c_str());
    return load_mock_manager(c.mock_file());
  }
  if (backend == "null") {
    log::printf("Using empty manager");
    return std::make_shared<NullManager>();
  }
  if (backend == "sysfs") {
    log::printf("Using sysfs (KFD topology) manager");
    log_versions(c.sysfs_root());
    return std::make_shared<SysfsManager>(sysfs_options(c));
  }
  if (backend == "amdsmi") {
    log::printf("Using amd-smi manager");
    log_versions(c.sysfs_root());
    return std::make_shared<AmdSmiManager>(amdsmi_options(c));
  }
  if (backend != "auto") throw Error("unknown backend '" + backend + "' (expected auto, amdsmi, sysfs, null or mock)");

  std::string why;
  bool has_smi = log_with_reason(has_amdsmi(&why), why, "amd-smi");
  bool has_kfd = log_with_reason(has_kfd_topology(c.sysfs_root(), &why), why, "KFD");
  if (has_smi || has_kfd) log_versions(c.sysfs_root());
  if (has_smi && has_kfd) {
    log::printf("Using amd-smi manager, KFD sysfs manager if amd-smi fails to initialize");
    return std::make_shared<PreferenceManager>(std::vector<ManagerPtr>{
        std::make_shared<AmdSmiManager>(amdsmi_options(c)), std::make_shared<SysfsManager>(sysfs_options(c))});
  }
  if (has_smi) {
    log::printf("Using amd-smi manager");
    return std::make_shared<AmdSmiManager>(amdsmi_options(c));
  }
  if (has_kfd) {
    log::printf("Using sysfs (KFD topology) manager");
    return std::make_shared<SysfsManager>(sysfs_options(c));
  }
  log::printf("WARNING: No valid resources detected; using empty manager.");
  return std::make_shared<NullManager>();
}

ManagerPtr new_manager(const config::Config& c) { return with_config(get_manager(c), c); }

}  // namespace gfd::resource
