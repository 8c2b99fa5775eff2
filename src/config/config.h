// Versioned (v1) daemon configuration.
//
// Same external schema as the config package the reference vendors from the
// device plugin (vendor/github.com/NVIDIA/k8s-device-plugin/api/config/v1):
//   version                                          config.go:33-38
//   flags.{migStrategy,failOnInitError,gfd.{...}}    flags.go:48-72
//   resources.{gpus,mig}[{pattern,name}]             resources.go:36-46
//   sharing.timeSlicing.{renameByDefault,
//       failRequestsGreaterThanOne,
//       resources[{name,rename,devices,replicas}]}   replicas.go:29-41
// with the resource-name prefix switched to `amd.com`.  The file may be YAML
// or JSON.  The `mig*` names are kept so existing manifests keep working;
// on MI355X the "MIG strategy" selects how compute partitions (SPX/DPX/QPX/
// CPX) are exposed.
//
// AMD-specific additions live under flags.gfd (backend selection, sysfs root,
// device filter, timing trace, amd-smi session mode).
#pragma once

#include <optional>
#include <string>
#include <vector>

#include "config/yaml.h"
#include "util/duration.h"

namespace gfd::config {

inline constexpr const char* kVersion = "v1";
inline constexpr const char* kResourceNamePrefix = "amd.com";
inline constexpr const char* kDefaultSharedResourceNameSuffix = ".shared";
inline constexpr size_t kMaxResourceNameLength = 63;

inline constexpr const char* kMigStrategyNone = "none";
inline constexpr const char* kMigStrategySingle = "single";
inline constexpr const char* kMigStrategyMixed = "mixed";

// Defaults of the CLI flags (cmd/gpu-feature-discovery/main.go:33-82).
inline constexpr const char* kDefaultOutputFile = "/etc/kubernetes/node-feature-discovery/features.d/gfd";
inline constexpr const char* kDefaultMachineTypeFile = "/sys/class/dmi/id/product_name";
inline constexpr Nanos kDefaultSleepInterval = 60 * kSecond;

// A fully-qualified Kubernetes extended resource name ("amd.com/gpu").
// Construction validates it (resources.go:48-64): the prefix is added if
// missing, the total length is limited to 63, and the name part must be a
// DNS-1123 subdomain.  Throws gfd::Error on invalid input.
std::string new_resource_name(const std::string& n);
// "amd.com/gpu" -> ("amd.com", "gpu"); names without '/' -> ("", name).
std::pair<std::string, std::string> split_resource_name(const std::string& n);
// name + ".shared" (resources.go:89-91).
std::string default_shared_rename(const std::string& resource_name);
// Kubernetes IsDNS1123Subdomain.
bool is_dns1123_subdomain(const std::string& s);

struct Resource {
  std::string pattern;
  std::string name;
};

struct Resources {
  std::vector<Resource> gpus;
  std::vector<Resource> partitions;  // "mig" key in the file
};

// Union: exactly one of all / count / list is meaningful (replicas.go:45-49).
struct ReplicatedDevices {
  bool all = false;
  int count = 0;
  std::vector<std::string> list;
};

struct ReplicatedResource {
  std::string name;
  std::string rename;
  ReplicatedDevices devices;
  int replicas = 0;
};

struct TimeSlicing {
  bool rename_by_default = false;
  bool fail_requests_greater_than_one = false;
  std::vector<ReplicatedResource> resources;
};

struct Sharing {
  TimeSlicing time_slicing;
};

struct GFDFlags {
  std::optional<bool> oneshot;
  std::optional<bool> no_timestamp;
  std::optional<Nanos> sleep_interval;
  std::optional<std::string> output_file;
  std::optional<std::string> machine_type_file;
  // AMD extensions.
  std::optional<std::string> backend;          // auto | amdsmi | sysfs | null | mock
  std::optional<std::string> sysfs_root;       // root prefix for /sys reads
  std::optional<std::string> host_root;        // host filesystem mount (node-true ROCm version)
  std::optional<std::string> rocm_version_file;  // explicit ROCm .info/version file
  std::optional<std::string> visible_devices;  // "" = all; "0,2-3" or BDFs
  std::optional<std::string> mock_file;        // device fixture for backend=mock
  std::optional<std::string> amdsmi_session;   // per-cycle | persistent
  std::optional<bool> trace_timing;
};

struct Flags {
  std::optional<std::string> mig_strategy;
  std::optional<bool> fail_on_init_error;
  std::optional<std::string> driver_root;
  bool plugin_present = false;  // dropped by loadConfig (main.go:105)
  GFDFlags gfd;
};

struct Config {
  std::string version = kVersion;
  Flags flags;
  Resources resources;
  Sharing sharing;
  // Test hook, not a flag or config key (the Python bindings set it): the
  // amd-smi backend answers every query through the library instead of the
  // amdgpu attributes it reads directly for unpartitioned GPUs.
  bool amdsmi_library_only = false;

  // Convenience accessors; defaults apply if a field was never populated.
  std::string mig_strategy() const { return flags.mig_strategy.value_or(kMigStrategyNone); }
  bool fail_on_init_error() const { return flags.fail_on_init_error.value_or(true); }
  bool oneshot() const { return flags.gfd.oneshot.value_or(false); }
  bool no_timestamp() const { return flags.gfd.no_timestamp.value_or(false); }
  Nanos sleep_interval() const { return flags.gfd.sleep_interval.value_or(kDefaultSleepInterval); }
  std::string output_file() const { return flags.gfd.output_file.value_or(kDefaultOutputFile); }
  std::string machine_type_file() const { return flags.gfd.machine_type_file.value_or(kDefaultMachineTypeFile); }
  std::string backend() const { return flags.gfd.backend.value_or("auto"); }
  std::string sysfs_root() const { return flags.gfd.sysfs_root.value_or("/"); }
  std::string host_root() const { return flags.gfd.host_root.value_or(""); }
  std::string rocm_version_file() const { return flags.gfd.rocm_version_file.value_or(""); }
  std::string visible_devices() const { return flags.gfd.visible_devices.value_or(""); }
  std::string mock_file() const { return flags.gfd.mock_file.value_or(""); }
  std::string amdsmi_session() const { return flags.gfd.amdsmi_session.value_or("persistent"); }
  bool trace_timing() const { return flags.gfd.trace_timing.value_or(false); }
};

// Parse a YAML/JSON config document (config.go:75-99).  Throws gfd::Error
// ("unmarshal error: ..." / "unknown version: ...").
Config parse_config_text(const std::string& text);
// Read + parse; errors are wrapped as "error opening config file: ..." /
// "error parsing config file: ..." (config.go:60-72).
Config parse_config_file(const std::string& path);

// Equivalent of main.go:236-270 disableResourceRenamingInConfig: drops
// `resources`, forces default renames and devices=all in time-slicing, and
// logs what was ignored.
void disable_resource_renaming(Config& c);

// JSON rendering used for the "Running with config" startup log
// (main.go:127-131).
yaml::Node to_node(const Config& c);
std::string to_json(const Config& c);

}  // namespace gfd::config
