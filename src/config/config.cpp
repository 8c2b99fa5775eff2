#include "config/config.h"

#include <cctype>
#include <cmath>
#include <cstring>
#include <limits>

#include "util/error.h"
#include "util/fs.h"
#include "util/log.h"
#include "util/strings.h"

namespace gfd::config {

using yaml::Node;

// ---------------------------------------------------------------------------
// Resource names (resources.go:48-91)

bool is_dns1123_subdomain(const std::string& s) {
  if (s.empty() || s.size() > 253) return false;
  for (const auto& label : str::split(s, '.')) {
    if (label.empty() || label.size() > 63) return false;
    auto alnum = [](char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
    if (!alnum(label.front()) || !alnum(label.back())) return false;
    for (char c : label)
      if (!alnum(c) && c != '-') return false;
  }
  return true;
}

std::pair<std::string, std::string> split_resource_name(const std::string& n) {
  auto parts = str::split_n(n, '/', 2);
  if (parts.size() != 2) return {"", n};
  return {parts[0], parts[1]};
}

std::string new_resource_name(const std::string& in) {
  std::string n = in;
  if (!str::starts_with(n, std::string(kResourceNamePrefix) + "/")) n = std::string(kResourceNamePrefix) + "/" + n;
  if (n.size() > kMaxResourceNameLength)
    throw Error(str::format("fully-qualified resource name must be %zu characters or less: %s", kMaxResourceNameLength,
                            n.c_str()));
  if (!is_dns1123_subdomain(split_resource_name(n).second))
    throw Error("incorrect format for resource name '" + n +
                "': [a lowercase RFC 1123 subdomain must consist of lower case alphanumeric characters, '-' or '.', "
                "and must start and end with an alphanumeric character]");
  return n;
}

std::string default_shared_rename(const std::string& resource_name) {
  return resource_name + kDefaultSharedResourceNameSuffix;
}

// ---------------------------------------------------------------------------
// Typed decoding with json-like error messages.

namespace {

// A struct field's key, matched the way the reference's decoder matches it
// (sigs.k8s.io/yaml -> encoding/json): any key equal to the field's name
// ignoring ASCII case ("MigStrategy", "MIGSTRATEGY"), the last one in the
// document winning.  (A key repeated verbatim keeps its first position here,
// so "a, A, a" picks A where Go picks the second a.)  Not for the bodies the
// reference decodes with its own UnmarshalJSON - TimeSlicing,
// ReplicatedResource, Resource (replicas.go:121-200, resources.go:94-122) -
// which look their keys up exactly in a map.
const Node* field(const Node& n, const char* name) {
  const Node* found = nullptr;
  for (const auto& [k, v] : n.entries()) {
    if (k.size() != std::strlen(name)) continue;
    bool eq = true;
    for (size_t i = 0; i < k.size() && eq; ++i)
      eq = std::tolower(static_cast<unsigned char>(k[i])) == std::tolower(static_cast<unsigned char>(name[i]));
    if (eq) found = &v;
  }
  return found;
}

[[noreturn]] void type_error(const Node& n, const std::string& path, const std::string& want) {
  throw Error("json: cannot unmarshal " + n.kind_name() + " into Go struct field " + path + " of type " + want);
}

// String fields accept any scalar: sigs.k8s.io/yaml converts plain YAML
// ints/floats/bools to strings when the JSON target is a string.
std::optional<std::string> opt_string(const Node* n, const std::string& path) {
  if (!n || n->is_null()) return std::nullopt;
  if (!n->is_scalar()) type_error(*n, path, "string");
  return n->text();
}

std::optional<bool> opt_bool(const Node* n, const std::string& path) {
  if (!n || n->is_null()) return std::nullopt;
  if (n->kind() != Node::Kind::Bool) type_error(*n, path, "bool");
  return n->as_bool();
}

// An integral number inside [lo, hi] (checked before any conversion: a
// float outside the target range has no defined conversion).
std::optional<int64_t> integral_in(const Node& n, double lo, double hi) {
  if (n.kind() == Node::Kind::Int) {
    if (static_cast<double>(n.as_int()) < lo || static_cast<double>(n.as_int()) > hi) return std::nullopt;
    return n.as_int();
  }
  if (n.kind() == Node::Kind::Float) {
    double f = n.as_float();
    if (!(f >= lo && f <= hi) || f != std::trunc(f)) return std::nullopt;
    return static_cast<int64_t>(f);
  }
  return std::nullopt;
}

// Go's int is 64 bits; the fields read as int here (replicas) are counts,
// so a value beyond 32 bits is rejected with Go's type error rather than
// truncated.
int to_int(const Node& n, const std::string& path) {
  if (auto v = integral_in(n, std::numeric_limits<int>::min(), std::numeric_limits<int>::max()))
    return static_cast<int>(*v);
  type_error(n, path, "int");
}

// Duration: a Go duration string or a number of nanoseconds (duration.go:36-53).
// The reference's error names no field (vendored api/config/v1/duration.go:51).
std::optional<Nanos> opt_duration(const Node* n, const std::string& /*path*/) {
  if (!n || n->is_null()) return std::nullopt;
  if (n->kind() == Node::Kind::Int) return static_cast<Nanos>(n->as_int());
  if (n->kind() == Node::Kind::Float) {
    // time.Duration(float64) truncates; outside int64 there is no duration.
    double f = n->as_float();
    if (!(f > -9.2233720368547758e18 && f < 9.2233720368547758e18)) throw Error("invalid duration");
    return static_cast<Nanos>(f);
  }
  if (n->kind() == Node::Kind::String) return parse_duration(n->text());
  throw Error("invalid duration");
}

void require_map(const Node& n, const std::string& path, const std::string& type) {
  if (!n.is_map()) type_error(n, path, type);
}

// ReplicatedDeviceRef (replicas.go:52-120): GPU index, partition index
// "<gpu>:<partition>", or a device UUID ("GPU-<uuid>" or a bare RFC 4122 UUID
// as reported by amd-smi).
bool is_uuid(const std::string& s) {
  if (s.size() != 36) return false;
  for (size_t i = 0; i < s.size(); ++i) {
    bool dash = i == 8 || i == 13 || i == 18 || i == 23;
    if (dash) {
      if (s[i] != '-') return false;
    } else if (!isxdigit(static_cast<unsigned char>(s[i]))) {
      return false;
    }
  }
  return true;
}

bool is_gpu_index(const std::string& s) { return str::parse_uint(s).has_value() && s == str::trim(s); }

bool is_partition_index(const std::string& s) {
  auto parts = str::split_n(s, ':', 2);
  return parts.size() == 2 && is_gpu_index(parts[0]) && is_gpu_index(parts[1]);
}

bool is_device_uuid(const std::string& s) {
  if (is_uuid(s)) return true;
  if (str::starts_with(s, "GPU-")) return is_uuid(s.substr(4));
  if (str::starts_with(s, "PARTITION-")) {
    // PARTITION-<gpu uuid>/<partition>
    auto parts = str::split_n(s.substr(10), '/', 2);
    return parts.size() == 2 && (is_uuid(parts[0]) || (str::starts_with(parts[0], "GPU-") && is_uuid(parts[0].substr(4)))) &&
           is_gpu_index(parts[1]);
  }
  return false;
}

ReplicatedDevices decode_devices(const Node& n) {
  ReplicatedDevices d;
  if (n.kind() == Node::Kind::String) {
    if (n.text() != "all")
      throw Error("devices set as '" + n.text() + "' but the only valid string input is 'all'");
    d.all = true;
    return d;
  }
  // Numbers reach the reference's decoder as JSON written by sigs.k8s.io/yaml,
  // where an integral float is an integer (2.0 -> 2): counts and indices
  // take either.
  if (auto count = integral_in(n, std::numeric_limits<int>::min(), std::numeric_limits<int>::max())) {
    if (*count <= 0) throw Error("devices set as '" + std::to_string(*count) + "' but a count of devices must be > 0");
    d.count = static_cast<int>(*count);
    return d;
  }
  if (n.is_seq()) {
    for (const auto& item : n.items()) {
      if (auto index = integral_in(item, 0, std::numeric_limits<int>::max())) {
        d.list.push_back(std::to_string(*index));
        continue;
      }
      if (item.kind() == Node::Kind::String) {
        const std::string& s = item.text();
        if (is_gpu_index(s) || is_partition_index(s) || is_device_uuid(s)) {
          d.list.push_back(s);
          continue;
        }
      }
      throw Error("unsupported type for device in devices list: " + item.text() + ", " + item.kind_name());
    }
    return d;
  }
  throw Error("unrecognized type for devices spec: " + yaml::to_json(n));
}

ReplicatedResource decode_replicated_resource(const Node& n, const std::string& path) {
  require_map(n, path, "ReplicatedResource");
  ReplicatedResource r;
  const Node* name = n.get("name");
  if (!name) throw Error("no resource name specified");
  auto name_s = opt_string(name, path + ".name");
  r.name = new_resource_name(name_s.value_or(""));
  const Node* devices = n.get("devices");
  if (devices && !devices->is_null())
    r.devices = decode_devices(*devices);
  else
    r.devices.all = true;
  const Node* replicas = n.get("replicas");
  if (!replicas) throw Error("no replicas specified");
  r.replicas = to_int(*replicas, path + ".replicas");
  if (r.replicas < 2) throw Error("number of replicas must be >= 2");
  if (const Node* rename = n.get("rename")) {
    auto rs = opt_string(rename, path + ".rename");
    if (rs) r.rename = new_resource_name(*rs);
  }
  return r;
}

TimeSlicing decode_time_slicing(const Node& n, const std::string& path) {
  require_map(n, path, "TimeSlicing");
  TimeSlicing ts;
  ts.rename_by_default = opt_bool(n.get("renameByDefault"), path + ".renameByDefault").value_or(false);
  ts.fail_requests_greater_than_one =
      opt_bool(n.get("failRequestsGreaterThanOne"), path + ".failRequestsGreaterThanOne").value_or(false);
  const Node* res = n.get("resources");
  if (!res || res->is_null()) throw Error("no resources specified");
  if (!res->is_seq()) type_error(*res, path + ".resources", "[]ReplicatedResource");
  for (const auto& item : res->items()) ts.resources.push_back(decode_replicated_resource(item, path + ".resources"));
  if (ts.resources.empty()) throw Error("no resources specified");
  for (auto& r : ts.resources)
    if (ts.rename_by_default && r.rename.empty()) r.rename = default_shared_rename(r.name);
  return ts;
}

std::vector<Resource> decode_resource_list(const Node* n, const std::string& path) {
  std::vector<Resource> out;
  if (!n || n->is_null()) return out;
  if (!n->is_seq()) type_error(*n, path, "[]Resource");
  for (const auto& item : n->items()) {
    require_map(item, path, "Resource");
    const Node* pattern = item.get("pattern");
    const Node* name = item.get("name");
    if (!pattern) throw Error("resources must have a 'pattern' field set");
    if (!name) throw Error("resources must have a 'name' field set");
    Resource r;
    r.pattern = opt_string(pattern, path + ".pattern").value_or("");
    r.name = new_resource_name(opt_string(name, path + ".name").value_or(""));
    out.push_back(r);
  }
  return out;
}

GFDFlags decode_gfd_flags(const Node& n) {
  GFDFlags g;
  require_map(n, "Config.flags.gfd", "GFDCommandLineFlags");
  g.oneshot = opt_bool(field(n, "oneshot"), "Config.flags.gfd.oneshot");
  g.no_timestamp = opt_bool(field(n, "noTimestamp"), "Config.flags.gfd.noTimestamp");
  g.sleep_interval = opt_duration(field(n, "sleepInterval"), "Config.flags.gfd.sleepInterval");
  g.output_file = opt_string(field(n, "outputFile"), "Config.flags.gfd.outputFile");
  g.machine_type_file = opt_string(field(n, "machineTypeFile"), "Config.flags.gfd.machineTypeFile");
  g.backend = opt_string(field(n, "backend"), "Config.flags.gfd.backend");
  g.sysfs_root = opt_string(field(n, "sysfsRoot"), "Config.flags.gfd.sysfsRoot");
  g.host_root = opt_string(field(n, "hostRoot"), "Config.flags.gfd.hostRoot");
  g.rocm_version_file = opt_string(field(n, "rocmVersionFile"), "Config.flags.gfd.rocmVersionFile");
  g.visible_devices = opt_string(field(n, "visibleDevices"), "Config.flags.gfd.visibleDevices");
  g.mock_file = opt_string(field(n, "mockFile"), "Config.flags.gfd.mockFile");
  g.amdsmi_session = opt_string(field(n, "amdsmiSession"), "Config.flags.gfd.amdsmiSession");
  g.trace_timing = opt_bool(field(n, "traceTiming"), "Config.flags.gfd.traceTiming");
  return g;
}

Node opt_node(const std::optional<std::string>& v) { return v ? Node::string(*v) : Node::null(); }
Node opt_node(const std::optional<bool>& v) { return v ? Node::boolean(*v) : Node::null(); }

}  // namespace

Config parse_config_text(const std::string& text) {
  Config c;
  Node root;
  try {
    root = yaml::parse(text);
    if (!root.is_null()) {
      require_map(root, "Config", "Config");
      if (auto v = opt_string(field(root, "version"), "Config.version")) c.version = *v;
      if (const Node* flags = field(root, "flags"); flags && !flags->is_null()) {
        require_map(*flags, "Config.flags", "Flags");
        c.flags.mig_strategy = opt_string(field(*flags, "migStrategy"), "Config.flags.migStrategy");
        c.flags.fail_on_init_error = opt_bool(field(*flags, "failOnInitError"), "Config.flags.failOnInitError");
        c.flags.driver_root = opt_string(field(*flags, "driverRoot"), "Config.flags.driverRoot");
        // A config file shared with the device plugin carries the plugin's
        // keys too (vendored api/config/v1/flags.go:48-63).  They do not
        // configure this daemon, but they are decoded and type-checked as the
        // reference decodes them, so a file it rejects is rejected here.
        (void)opt_string(field(*flags, "nvidiaDriverRoot"), "Config.flags.nvidiaDriverRoot");
        (void)opt_bool(field(*flags, "gdsEnabled"), "Config.flags.gdsEnabled");
        (void)opt_bool(field(*flags, "mofedEnabled"), "Config.flags.mofedEnabled");
        if (const Node* p = field(*flags, "plugin"); p && !p->is_null()) {
          require_map(*p, "Config.flags.plugin", "PluginCommandLineFlags");
          (void)opt_bool(field(*p, "passDeviceSpecs"), "Config.flags.plugin.passDeviceSpecs");
          (void)opt_string(field(*p, "deviceListStrategy"), "Config.flags.plugin.deviceListStrategy");
          (void)opt_string(field(*p, "deviceIDStrategy"), "Config.flags.plugin.deviceIDStrategy");
          c.flags.plugin_present = true;
        }
        if (const Node* g = field(*flags, "gfd"); g && !g->is_null()) c.flags.gfd = decode_gfd_flags(*g);
      }
      if (const Node* res = field(root, "resources"); res && !res->is_null()) {
        require_map(*res, "Config.resources", "Resources");
        c.resources.gpus = decode_resource_list(field(*res, "gpus"), "Config.resources.gpus");
        c.resources.partitions = decode_resource_list(field(*res, "mig"), "Config.resources.mig");
        if (c.resources.partitions.empty())
          c.resources.partitions = decode_resource_list(field(*res, "partitions"), "Config.resources.partitions");
      }
      if (const Node* sh = field(root, "sharing"); sh && !sh->is_null()) {
        require_map(*sh, "Config.sharing", "Sharing");
        if (const Node* ts = field(*sh, "timeSlicing"); ts && !ts->is_null())
          c.sharing.time_slicing = decode_time_slicing(*ts, "Config.sharing.timeSlicing");
      }
    }
  } catch (const Error& e) {
    throw Error(std::string("unmarshal error: ") + e.what());
  }
  if (c.version.empty()) c.version = kVersion;
  if (c.version != kVersion) throw Error("unknown version: " + c.version);
  return c;
}

Config parse_config_file(const std::string& path) {
  auto r = fs::read_file(path);
  if (!r.ok()) throw Error("error opening config file: open " + path + ": " + fs::errno_str(r.err));
  try {
    return parse_config_text(r.data);
  } catch (const std::exception& e) {
    throw Error(std::string("error parsing config file: ") + e.what());
  }
}

void disable_resource_renaming(Config& c) {
  if (!c.resources.gpus.empty() || !c.resources.partitions.empty())
    log::printf("Customizing the 'resources' field is not yet supported in the config. Ignoring...");
  c.resources.gpus.clear();
  c.resources.partitions.clear();

  auto& ts = c.sharing.time_slicing;
  bool sets_non_default_rename = false;
  bool sets_devices = false;
  for (auto& r : ts.resources) {
    if (!ts.rename_by_default && !r.rename.empty()) {
      sets_non_default_rename = true;
      r.rename.clear();
    }
    if (ts.rename_by_default && r.rename != default_shared_rename(r.name)) {
      sets_non_default_rename = true;
      r.rename = default_shared_rename(r.name);
    }
    if (!r.devices.all) {
      sets_devices = true;
      r.devices.all = true;
      r.devices.count = 0;
      r.devices.list.clear();
    }
  }
  if (sets_non_default_rename)
    log::printf("Setting the 'rename' field in sharing.timeSlicing.resources is not yet supported in the config. Ignoring...");
  if (sets_devices)
    log::printf(
        "Customizing the 'devices' field in sharing.timeSlicing.resources is not yet supported in the config. "
        "Ignoring...");
}

Node to_node(const Config& c) {
  Node root = Node::map();
  root.set("version", Node::string(c.version));

  Node flags = Node::map();
  flags.set("migStrategy", opt_node(c.flags.mig_strategy));
  flags.set("failOnInitError", opt_node(c.flags.fail_on_init_error));
  if (c.flags.driver_root) flags.set("driverRoot", Node::string(*c.flags.driver_root));
  Node gfd = Node::map();
  const auto& g = c.flags.gfd;
  gfd.set("oneshot", opt_node(g.oneshot));
  gfd.set("noTimestamp", opt_node(g.no_timestamp));
  gfd.set("sleepInterval", g.sleep_interval ? Node::string(format_duration(*g.sleep_interval)) : Node::null());
  gfd.set("outputFile", opt_node(g.output_file));
  gfd.set("machineTypeFile", opt_node(g.machine_type_file));
  gfd.set("backend", opt_node(g.backend));
  gfd.set("sysfsRoot", opt_node(g.sysfs_root));
  gfd.set("hostRoot", opt_node(g.host_root));
  gfd.set("rocmVersionFile", opt_node(g.rocm_version_file));
  gfd.set("visibleDevices", opt_node(g.visible_devices));
  if (g.mock_file && !g.mock_file->empty()) gfd.set("mockFile", Node::string(*g.mock_file));
  gfd.set("amdsmiSession", opt_node(g.amdsmi_session));
  gfd.set("traceTiming", opt_node(g.trace_timing));
  flags.set("gfd", gfd);
  root.set("flags", flags);

  auto res_list = [](const std::vector<Resource>& v) {
    if (v.empty()) return Node::null();
    Node s = Node::seq();
    for (const auto& r : v) {
      Node m = Node::map();
      m.set("pattern", Node::string(r.pattern));
      m.set("name", Node::string(r.name));
      s.push(m);
    }
    return s;
  };
  Node resources = Node::map();
  resources.set("gpus", res_list(c.resources.gpus));
  if (!c.resources.partitions.empty()) resources.set("mig", res_list(c.resources.partitions));
  root.set("resources", resources);

  Node ts = Node::map();
  const auto& t = c.sharing.time_slicing;
  if (t.rename_by_default) ts.set("renameByDefault", Node::boolean(true));
  if (t.fail_requests_greater_than_one) ts.set("failRequestsGreaterThanOne", Node::boolean(true));
  if (!t.resources.empty()) {
    Node rs = Node::seq();
    for (const auto& r : t.resources) {
      Node m = Node::map();
      m.set("name", Node::string(r.name));
      if (!r.rename.empty()) m.set("rename", Node::string(r.rename));
      if (r.devices.all) {
        m.set("devices", Node::string("all"));
      } else if (r.devices.count > 0) {
        m.set("devices", Node::integer(r.devices.count));
      } else {
        Node l = Node::seq();
        for (const auto& d : r.devices.list) l.push(Node::string(d));
        m.set("devices", l);
      }
      m.set("replicas", Node::integer(r.replicas));
      rs.push(m);
    }
    ts.set("resources", rs);
  }
  Node sharing = Node::map();
  // An empty timeSlicing would not parse back ("no resources specified").
  if (!t.resources.empty()) sharing.set("timeSlicing", ts);
  root.set("sharing", sharing);
  return root;
}

std::string to_json(const Config& c) { return yaml::to_json(to_node(c), 2); }

}  // namespace gfd::config
