#include "cli/flags.h"

#include <cstdlib>

#include "config/config.h"
#include "util/strings.h"

namespace gfd::cli {

namespace {

std::optional<std::string> lookup_env(const std::string& name, const std::map<std::string, std::string>* env) {
  if (env) {
    auto it = env->find(name);
    if (it == env->end()) return std::nullopt;
    return it->second;
  }
  const char* v = std::getenv(name.c_str());
  if (!v) return std::nullopt;
  return std::string(v);
}

void validate(const FlagDef& d, const std::string& v, const std::string& source) {
  if (d.type == FlagType::Bool && !str::parse_bool(v))
    throw UsageError("could not parse \"" + v + "\" as bool value from " + source + " for flag " + d.name +
                     ": strconv.ParseBool: parsing \"" + v + "\": invalid syntax");
  if (d.type == FlagType::Duration) {
    try {
      parse_duration(v);
    } catch (const std::exception& e) {
      throw UsageError("could not parse \"" + v + "\" as duration value from " + source + " for flag " + d.name + ": " +
                       e.what());
    }
  }
}

}  // namespace

const FlagDef* Context::find(const std::string& name) const {
  for (const auto& d : defs_) {
    if (d.name == name) return &d;
    for (const auto& a : d.aliases)
      if (a == name) return &d;
  }
  return nullptr;
}

Context Context::parse(const std::vector<FlagDef>& defs, const std::vector<std::string>& args,
                       const std::map<std::string, std::string>* env) {
  Context c;
  c.defs_ = defs;
  // Defaults, then environment (flag Apply order in urfave).
  for (const auto& d : defs) {
    Value v;
    v.text = d.default_value;
    for (const auto& e : d.env_vars) {
      auto ev = lookup_env(e, env);
      if (!ev) continue;
      if (d.type == FlagType::String) {
        v.text = *ev;
        v.from_env = true;
      } else if (!ev->empty()) {
        validate(d, *ev, "environment variable \"" + e + "\"");
        v.text = *ev;
        v.from_env = true;
      }
      break;  // first env var present wins
    }
    c.values_[d.name] = v;
  }

  for (size_t i = 0; i < args.size(); ++i) {
    const std::string& a = args[i];
    if (a.size() < 2 || a[0] != '-') {
      c.positional_.assign(args.begin() + static_cast<long>(i), args.end());
      break;
    }
    if (a == "--") {
      c.positional_.assign(args.begin() + static_cast<long>(i) + 1, args.end());
      break;
    }
    std::string body = a.substr(a[1] == '-' ? 2 : 1);
    if (body.empty() || body[0] == '-' || body[0] == '=') throw UsageError("bad flag syntax: " + a);
    std::string name = body, value;
    bool has_value = false;
    auto eq = body.find('=');
    if (eq != std::string::npos) {
      name = body.substr(0, eq);
      value = body.substr(eq + 1);
      has_value = true;
    }
    if (name == "help" || name == "h") {
      c.help_ = true;
      continue;
    }
    if (name == "version" || name == "v") {
      c.version_ = true;
      continue;
    }
    const FlagDef* d = c.find(name);
    if (!d) throw UsageError("flag provided but not defined: -" + name);
    if (d->type == FlagType::Bool) {
      if (!has_value) value = "true";
      if (!str::parse_bool(value)) throw UsageError("invalid boolean value \"" + value + "\" for -" + name + ": parse error");
    } else {
      if (!has_value) {
        if (i + 1 >= args.size()) throw UsageError("flag needs an argument: -" + name);
        value = args[++i];
      }
      if (d->type == FlagType::Duration) {
        try {
          parse_duration(value);
        } catch (const std::exception&) {
          throw UsageError("invalid value \"" + value + "\" for flag -" + name + ": parse error");
        }
      }
    }
    auto& v = c.values_[d->name];
    v.text = value;
    v.from_cli = true;
  }
  return c;
}

bool Context::IsSet(const std::string& name) const {
  const FlagDef* d = find(name);
  if (!d) return false;
  const auto& v = values_.at(d->name);
  return v.from_cli || v.from_env;
}

std::string Context::String(const std::string& name) const {
  const FlagDef* d = find(name);
  return d ? values_.at(d->name).text : std::string();
}

bool Context::Bool(const std::string& name) const {
  const FlagDef* d = find(name);
  if (!d) return false;
  return str::parse_bool(values_.at(d->name).text).value_or(false);
}

Nanos Context::Duration(const std::string& name) const {
  const FlagDef* d = find(name);
  if (!d) return 0;
  try {
    return parse_duration(values_.at(d->name).text);
  } catch (const std::exception&) {
    return 0;
  }
}

std::vector<FlagDef> gfd_flags() {
  using T = FlagType;
  return {
      {"mig-strategy", {}, T::String, config::kMigStrategyNone, {"GFD_MIG_STRATEGY", "MIG_STRATEGY"},
       "the desired strategy for exposing compute partitions (SPX/DPX/QPX/CPX) on GPUs that support it:\n\t\t[none | single | mixed]"},
      {"fail-on-init-error", {}, T::Bool, "true", {"GFD_FAIL_ON_INIT_ERROR", "FAIL_ON_INIT_ERROR"},
       "fail the plugin if an error is encountered during initialization, otherwise block indefinitely"},
      {"oneshot", {}, T::Bool, "false", {"GFD_ONESHOT"}, "Label once and exit"},
      {"no-timestamp", {}, T::Bool, "false", {"GFD_NO_TIMESTAMP"}, "Do not add the timestamp to the labels"},
      {"sleep-interval", {}, T::Duration, "1m0s", {"GFD_SLEEP_INTERVAL"}, "Time to sleep between labeling"},
      {"output-file", {"output", "o"}, T::String, config::kDefaultOutputFile, {"GFD_OUTPUT_FILE"},
       "the path to the NFD feature file (empty: write to stdout)"},
      {"machine-type-file", {}, T::String, config::kDefaultMachineTypeFile, {"GFD_MACHINE_TYPE_FILE"},
       "a path to a file that contains the DMI (SMBIOS) information for the node"},
      {"config-file", {}, T::String, "", {"GFD_CONFIG_FILE", "CONFIG_FILE"},
       "the path to a config file as an alternative to command line options or environment variables"},
      // AMD extensions.
      {"backend", {}, T::String, "auto", {"GFD_BACKEND"},
       "device backend: auto (amd-smi once initialised - in the background, KFD sysfs until then; --oneshot: KFD\n\t\t"
       "sysfs; without amd-smi: KFD sysfs, else none) | amdsmi | sysfs | null | mock"},
      {"sysfs-root", {}, T::String, "/", {"GFD_SYSFS_ROOT"},
       "root prefix for sysfs/procfs reads (synthetic trees for testing)"},
      {"host-root", {}, T::String, "", {"GFD_HOST_ROOT"},
       "where the host's filesystem (at least /opt) is mounted in the container: the ROCm runtime version is\n\t\t"
       "read from <host-root>/opt/rocm/.info/version, following the host's absolute symlinks (empty: this root)"},
      {"rocm-version-file", {}, T::String, "", {"GFD_ROCM_VERSION_FILE"},
       "read the ROCm runtime version from this file (e.g. a mounted /opt/rocm/.info/version); an error if unreadable"},
      {"visible-devices", {}, T::String, "", {"GFD_VISIBLE_DEVICES"},
       "restrict labeling to these physical GPUs: indices, ranges or PCI addresses (\"0,2-3\"); empty = all"},
      {"amdsmi-session", {}, T::String, "persistent", {"GFD_AMDSMI_SESSION"},
       "amd-smi session lifetime: persistent (initialise once, re-init on topology change) | per-cycle"},
      {"mock-file", {}, T::String, "", {"GFD_MOCK_FILE"}, "device fixture (YAML/JSON) for --backend=mock"},
      {"trace-timing", {}, T::Bool, "false", {"GFD_TRACE_TIMING"}, "log per-phase timing of every labeling cycle"},
      {"cpu-affinity", {}, T::String, "follow", {"GFD_CPU_AFFINITY"},
       "CPU placement of the daemon's threads: none (the scheduler decides) | follow (worker threads kept on the\n\t\t"
       "CPUs sharing the L3 cache of the CPU each cycle starts on) | l3 (every thread on the L3 domain of the CPU\n\t\t"
       "the daemon starts on)"},
  };
}

std::string help_text(const std::vector<FlagDef>& defs, const std::string& app_name, const std::string& usage,
                      const std::string& version) {
  std::string out;
  out += "NAME:\n   " + app_name + " - " + usage + "\n\n";
  out += "USAGE:\n   gpu-feature-discovery [global options] [arguments...]\n\n";
  out += "VERSION:\n   " + str::replace_all(version, "\n", "\n   ") + "\n\n";
  out += "GLOBAL OPTIONS:\n";
  for (const auto& d : defs) {
    if (d.hidden) continue;
    std::string suffix = d.type != FlagType::Bool ? " value" : "";
    std::string names = "--" + d.name + suffix;
    for (const auto& a : d.aliases) names += (a.size() == 1 ? ", -" : ", --") + a + suffix;
    std::string line = "   " + names + "\t" + d.usage;
    if (d.type == FlagType::String && !d.default_value.empty())
      line += " (default: \"" + d.default_value + "\")";
    else if (d.type != FlagType::String)
      line += " (default: " + d.default_value + ")";
    std::vector<std::string> envs;
    for (const auto& e : d.env_vars) envs.push_back("$" + e);
    if (!envs.empty()) line += " [" + str::join(envs, ", ") + "]";
    out += line + "\n";
  }
  out += "   --help, -h\tshow help\n";
  out += "   --version, -v\tprint the version\n";
  return out;
}

}  // namespace gfd::cli
