#include "resource/versions.h"

#include <sys/utsname.h>

#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>

#include "util/error.h"
#include "util/fs.h"
#include "util/strings.h"

namespace gfd::resource {

std::optional<std::string> extract_version(const std::string& s) {
  auto digit = [](char c) { return c >= '0' && c <= '9'; };
  for (size_t i = 0; i < s.size(); ++i) {
    if (!digit(s[i]) || (i > 0 && (digit(s[i - 1]) || s[i - 1] == '.'))) continue;
    std::vector<std::string> parts;
    size_t j = i;
    for (;;) {
      size_t st = j;
      while (j < s.size() && digit(s[j])) ++j;
      if (j == st) break;
      parts.push_back(s.substr(st, j - st));
      if (parts.size() == 3 || j + 1 >= s.size() || s[j] != '.' || !digit(s[j + 1])) break;
      ++j;  // skip '.'
    }
    if (parts.size() >= 2) return str::join(parts, ".");
  }
  return std::nullopt;
}

namespace {
// amdgpu built into the kernel: /sys/module/amdgpu exists but has no
// `initstate` (only loadable modules have one) and no `version`.  (The
// MI355X pool's amdgpu is loadable, without a `version`:
// profiles/amdgpu_module_layout.txt.)
// Whether the kernel's amdgpu is built in or loadable is fixed until the
// next boot (a DKMS module cannot replace a built-in driver, and a kernel
// with a loadable amdgpu never grows a built-in one), so it is decided once
// the module directory exists; a built-in driver then skips the failing
// `version` lookup - a path walk every cycle.
bool builtin_amdgpu(const std::string& root) {
  static std::mutex mu;
  static std::map<std::string, bool> known;
  std::lock_guard<std::mutex> g(mu);
  auto it = known.find(root);
  if (it != known.end()) return it->second;
  std::string dir = fs::join(root, "sys/module/amdgpu");
  if (!fs::is_dir(dir)) return false;  // not loaded (yet): ask again next time
  bool builtin = !fs::exists(dir + "/initstate") && !fs::exists(dir + "/version");
  known.emplace(root, builtin);
  return builtin;
}
// Whether the loaded amdgpu module publishes a `version` (a DKMS build does;
// an in-tree module, the MI355X pool's, does not).  Looked up relative to
// the module directory kept open: the failing lookup by path walked
// /sys/module/amdgpu every cycle (facts.driver 0.035 ms after an idle
// second, profiles/bench_fresh_r4.txt r4fin3a).  A reloaded module is a new
// directory: the old one has lost its `initstate` (every loadable module
// has one; this is only asked when the module is not built in) and the path
// is opened again.
bool module_has_version(const std::string& root) {
  static std::mutex mu;
  static std::map<std::string, std::unique_ptr<fs::Dir>> dirs;
  std::lock_guard<std::mutex> g(mu);
  auto& d = dirs[root];
  if (!d || d->lookup("initstate") != 0) d = std::make_unique<fs::Dir>(fs::join(root, "sys/module/amdgpu"));
  return d->err() == 0 && d->lookup("version") == 0;
}
}  // namespace

std::string host_driver_version(const std::string& root) {
  if (!builtin_amdgpu(root) && module_has_version(root))
    if (auto v = fs::attrs().read_trimmed(fs::join(root, "sys/module/amdgpu/version")); v && !v->empty()) return *v;
  if (root != "/" && !root.empty()) {
    // Synthetic trees carry the kernel banner under proc/.
    if (auto v = fs::read_trimmed(fs::join(root, "proc/sys/kernel/osrelease")); v && !v->empty()) return *v;
  }
  struct utsname u;
  if (uname(&u) == 0) return u.release;
  return "";
}

std::optional<RuntimeVersion> parse_runtime_version(const std::string& text) {
  auto ver = extract_version(text);
  if (!ver) return std::nullopt;
  auto parts = str::split(*ver, '.');
  auto maj = str::parse_uint(parts[0]);
  auto min = str::parse_uint(parts[1]);
  if (!maj || !min) return std::nullopt;
  return RuntimeVersion{static_cast<unsigned>(*maj), static_cast<unsigned>(*min)};
}

namespace {

std::optional<RuntimeVersion> read_version_file(const std::string& path) {
  auto v = fs::attrs().read_checked_trimmed(path);
  if (!v) return std::nullopt;
  return parse_runtime_version(*v);
}

// Highest <host_root>/opt/rocm-X.Y.Z/.info/version (versioned installs).
std::optional<RuntimeVersion> newest_versioned_install(const std::string& host_root, std::string* source) {
  std::optional<RuntimeVersion> best;
  for (const auto& name : fs::list_dir(fs::join(host_root, "opt"))) {
    if (name.rfind("rocm-", 0) != 0) continue;
    std::string path = fs::resolve_in_root(host_root, "opt/" + name + "/.info/version");
    if (path.empty()) continue;
    auto v = read_version_file(path);
    if (v && (!best || std::tie(v->major, v->minor) > std::tie(best->major, best->minor))) {
      best = v;
      if (source) *source = path;
    }
  }
  return best;
}

}  // namespace

std::optional<RuntimeVersion> rocm_version(const VersionSources& s, std::string* source) {
  auto from = [&](const std::string& path) -> std::optional<RuntimeVersion> {
    auto v = read_version_file(path);
    if (v && source) *source = path;
    return v;
  };
  if (!s.rocm_version_file.empty()) {
    auto text = fs::attrs().read_checked_trimmed(s.rocm_version_file);
    if (!text) throw Error("unable to read the ROCm version file " + s.rocm_version_file);
    auto v = parse_runtime_version(*text);
    if (!v) throw Error("ROCm version file " + s.rocm_version_file + " holds \"" + *text + "\", not X.Y[.Z]");
    if (source) *source = s.rocm_version_file;
    return v;
  }
  if (!s.host_root.empty()) {
    // A host root without opt/ is a missing mount (the manifests mount the
    // host's /opt at <host-root>/opt), not a node without ROCm: labeling on
    // would silently drop amd.com/rocm.runtime.*, which the reference always
    // emits.  A mounted /opt that holds no ROCm is a node without it.
    if (!fs::is_dir(fs::join(s.host_root, "opt")))
      throw Error("--host-root " + s.host_root + " has no opt/ directory: mount the host's /opt there to read the ROCm "
                  "runtime version");
    std::string path = fs::resolve_in_root(s.host_root, "opt/rocm/.info/version");
    if (!path.empty())
      if (auto v = from(path)) return v;
    return newest_versioned_install(s.host_root, source);
  }
  if (!s.root.empty() && s.root != "/") return from(fs::join(s.root, "opt/rocm/.info/version"));
  if (const char* rp = std::getenv("ROCM_PATH"); rp && *rp)
    if (auto v = from(fs::join(rp, ".info/version"))) return v;
  return from("/opt/rocm/.info/version");
}

std::string driver_version(const std::string& root) {
  std::string raw = host_driver_version(root);
  auto v = extract_version(raw);
  return v ? *v : raw;
}

}  // namespace gfd::resource
