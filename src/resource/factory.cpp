#include "resource/factory.h"

#include "resource/amdsmi.h"
#include "resource/managers.h"
#include "resource/sysfs.h"
#include "resource/versions.h"
#include "util/error.h"
#include "util/log.h"

namespace gfd::resource {

namespace {

VersionSources version_sources(const config::Config& c) {
  VersionSources v;
  v.root = c.sysfs_root();
  v.host_root = c.host_root();
  v.rocm_version_file = c.rocm_version_file();
  v.keep = !c.oneshot();
  return v;
}

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
  o.versions = version_sources(c);
  o.sysfs_values = !c.amdsmi_library_only;
  return o;
}

SysfsOptions sysfs_options(const config::Config& c) {
  SysfsOptions o;
  o.root = c.sysfs_root();
  o.filter = DeviceFilter::parse(c.visible_devices());
  o.versions = version_sources(c);
  return o;
}

bool log_with_reason(bool is, const std::string& reason, std::string tag) {
  if (!is) tag = "non-" + tag;
  log::printf("Detected %s platform: %s", tag.c_str(), reason.c_str());
  return is;
}

// Startup observability: the runtime and driver versions the
// hardware backends will label with.
void log_versions(const config::Config& c) {
  std::string source, rocm = "not found";
  try {
    if (auto rv = rocm_version(version_sources(c), &source))
      rocm = std::to_string(rv->major) + "." + std::to_string(rv->minor) + " (" + source + ")";
  } catch (const std::exception& e) {
    rocm = e.what();
  }
  std::string drv = host_driver_version(c.sysfs_root());
  log::printf("ROCm runtime %s, amdgpu driver %s", rocm.c_str(), extract_version(drv).value_or(drv).c_str());
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
    log_versions(c);
    return std::make_shared<SysfsManager>(sysfs_options(c));
  }
  if (backend == "amdsmi") {
    log::printf("Using amd-smi manager");
    log_versions(c);
    return std::make_shared<AmdSmiManager>(amdsmi_options(c));
  }
  if (backend != "auto") throw Error("unknown backend '" + backend + "' (expected auto, amdsmi, sysfs, null or mock)");

  std::string why;
  if (c.oneshot()) {
    // Job mode labels once and exits, so amd-smi's ~25 ms amdsmi_init (it
    // parses all of /proc/cpuinfo, profiles/amdsmi_init_profile.txt) would be
    // most of the process's life.  The KFD topology answers the same
    // questions with the same values (tests/test_gpu.py checks the two label
    // files are byte-identical), so a Job reads it and never loads amd-smi.
    if (log_with_reason(has_kfd_topology(c.sysfs_root(), &why), why, "KFD")) {
      log_versions(c);
      log::printf("Using sysfs (KFD topology) manager (oneshot: amd-smi not loaded)");
      return std::make_shared<SysfsManager>(sysfs_options(c));
    }
  }
  bool has_smi = log_with_reason(has_amdsmi(&why), why, "amd-smi");
  bool has_kfd = log_with_reason(has_kfd_topology(c.sysfs_root(), &why), why, "KFD");
  if (has_smi || has_kfd) log_versions(c);
  if (has_smi && has_kfd && c.amdsmi_session() == "persistent") {
    log::printf("Using amd-smi manager (initialized in the background), KFD sysfs manager until then "
                "or if amd-smi fails to initialize");
    return std::make_shared<WarmStartManager>(std::make_shared<AmdSmiManager>(amdsmi_options(c)),
                                              std::make_shared<SysfsManager>(sysfs_options(c)));
  }
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
