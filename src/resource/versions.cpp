#include "resource/versions.h"

#include <fcntl.h>
#include <sys/utsname.h>
#include <unistd.h>

#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <vector>

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

// One evaluation of the lookup below.  With `walk` set, every path is
// resolved by hand (fs::resolve_in_root) to learn the directories whose
// entries decide the answer, and the file that gave it is kept open.
struct Walk {
  std::vector<std::string> dirs;
  std::string file;      // the file whose contents gave the answer ("": none)
  int fd = -1;           // that file, open
  bool single = true;    // false: the answer compared several files (newest install)
  ~Walk() {
    if (fd >= 0) ::close(fd);
  }
};

std::optional<std::string> read_text(const std::string& path, Walk* walk) {
  if (!walk) {
    auto v = fs::attrs().read_checked_trimmed(path);
    return v;
  }
  std::string real = fs::resolve_in_root("/", fs::absolute(path), &walk->dirs);
  if (real.empty()) return std::nullopt;
  int fd = ::open(real.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return std::nullopt;
  std::string data;
  if (fs::pread_all(fd, 4096, &data) != 0) {
    ::close(fd);
    return std::nullopt;
  }
  if (walk->fd >= 0) ::close(walk->fd);
  walk->fd = fd;
  walk->file = real;
  return str::trim(data);
}

std::optional<RuntimeVersion> read_version_file(const std::string& path, Walk* walk) {
  auto v = read_text(path, walk);
  if (!v) return std::nullopt;
  return parse_runtime_version(*v);
}

// Highest <host_root>/opt/rocm-X.Y.Z/.info/version (versioned installs).
std::optional<RuntimeVersion> newest_versioned_install(const std::string& host_root, std::string* source, Walk* walk) {
  if (walk) walk->single = false;
  std::optional<RuntimeVersion> best;
  for (const auto& name : fs::list_dir(fs::join(host_root, "opt"))) {
    if (name.rfind("rocm-", 0) != 0) continue;
    std::string path = fs::resolve_in_root(host_root, "opt/" + name + "/.info/version");
    if (path.empty()) continue;
    auto v = read_version_file(path, nullptr);
    if (v && (!best || std::tie(v->major, v->minor) > std::tie(best->major, best->minor))) {
      best = v;
      if (source) *source = path;
    }
  }
  return best;
}

std::optional<RuntimeVersion> lookup(const VersionSources& s, std::string* source, Walk* walk) {
  auto from = [&](const std::string& path) -> std::optional<RuntimeVersion> {
    auto v = read_version_file(path, walk);
    if (v && source) *source = path;
    return v;
  };
  if (!s.rocm_version_file.empty()) {
    auto text = read_text(s.rocm_version_file, walk);
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
    std::string path = fs::resolve_in_root(s.host_root, "opt/rocm/.info/version", walk ? &walk->dirs : nullptr);
    if (!path.empty())
      if (auto v = from(path)) return v;
    return newest_versioned_install(s.host_root, source, walk);
  }
  if (!s.root.empty() && s.root != "/") return from(fs::join(s.root, "opt/rocm/.info/version"));
  if (const char* rp = std::getenv("ROCM_PATH"); rp && *rp)
    if (auto v = from(fs::join(rp, ".info/version"))) return v;
  return from("/opt/rocm/.info/version");
}

// The lookup's answer for one set of sources, kept while the directories it
// walked are unchanged (fs::DirWatch): a path walk per cycle - with
// --host-root one lstat per component - becomes one non-blocking read of an
// inotify queue and a pread of the kept file (a version file rewritten in
// place is read fresh; one replaced, a symlink repointed, a directory on
// the way renamed or removed is an entry change in a watched directory).
// Only for sources that may be kept (a loop daemon's; a oneshot Job looks
// up once, and an inotify watch would cost it more than the lookup).  The
// first call looks up plainly; later misses walk by hand, arm the watch,
// and walk again - the answer is kept only if both walks agree, so a change
// racing the first walk is not missed.  Answers from several files (the
// newest-install scan) and errors are not kept.
struct Kept {
  std::string key;
  bool seen = false;
  int plain = 0;  // calls left to look up plainly: nothing to watch (see below)
  fs::DirWatch watch;
  int fd = -1;  // the file the answer came from (-1: no file, no ROCm)
  std::string source;
  bool valid = false;
  ~Kept() {
    if (fd >= 0) ::close(fd);
  }
};

}  // namespace

std::optional<RuntimeVersion> rocm_version(const VersionSources& s, std::string* source) {
  if (!s.keep) return lookup(s, source, nullptr);
  static std::mutex mu;
  static auto* kept = new std::vector<std::unique_ptr<Kept>>();  // leaked: workers may read at exit
  std::string rocm_path;
  if (s.host_root.empty() && s.rocm_version_file.empty() && (s.root.empty() || s.root == "/"))
    if (const char* rp = std::getenv("ROCM_PATH")) rocm_path = rp;
  std::string key = s.rocm_version_file + '\0' + s.host_root + '\0' + s.root + '\0' + rocm_path;
  std::lock_guard<std::mutex> g(mu);
  Kept* k = nullptr;
  for (auto& e : *kept)
    if (e->key == key) k = e.get();
  if (!k) {
    // A few sets of sources at most (one per daemon; tests build many).
    if (kept->size() >= 8) kept->erase(kept->begin());
    kept->push_back(std::make_unique<Kept>());
    k = kept->back().get();
    k->key = key;
  }
  if (k->valid && k->watch.unchanged()) {
    if (k->fd < 0) return std::nullopt;
    std::string data;
    if (fs::pread_all(k->fd, 4096, &data, true) == 0)  // a regular file
      if (auto v = parse_runtime_version(str::trim(data))) {
        if (source) *source = k->source;
        return v;
      }
    // No longer a version: the lookup decides (an error, or the next source).
  }
  k->valid = false;
  if (k->fd >= 0) ::close(k->fd);
  k->fd = -1;
  if (!k->seen || k->plain > 0) {
    k->seen = true;
    if (k->plain > 0) --k->plain;
    return lookup(s, source, nullptr);
  }
  Walk first;
  std::string src;
  auto first_v = lookup(s, &src, &first);
  if (!first.single || !k->watch.arm(first.dirs)) {
    // An answer from several files, a directory on a network file system,
    // no inotify instance left: nothing to keep.  Plain lookups for the
    // next 64 calls (a walk by hand costs more), then another try.
    k->plain = 64;
    if (source && first_v) *source = src;
    return first_v;
  }
  Walk second;
  src.clear();
  auto v = lookup(s, &src, &second);
  if (second.single && second.dirs == first.dirs && second.file == first.file) {
    k->valid = true;
    k->fd = second.fd;
    second.fd = -1;
    k->source = src;
  }
  if (source && v) *source = src;
  return v;
}

std::string driver_version(const std::string& root) {
  std::string raw = host_driver_version(root);
  auto v = extract_version(raw);
  return v ? *v : raw;
}

}  // namespace gfd::resource
