#include "resource/versions.h"

#include <sys/utsname.h>

#include <cstdlib>

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

std::string host_driver_version(const std::string& root) {
  if (auto v = fs::attrs().read_trimmed(fs::join(root, "sys/module/amdgpu/version")); v && !v->empty()) return *v;
  if (root != "/" && !root.empty()) {
    // Synthetic trees carry the kernel banner under proc/.
    if (auto v = fs::read_trimmed(fs::join(root, "proc/sys/kernel/osrelease")); v && !v->empty()) return *v;
  }
  struct utsname u;
  if (uname(&u) == 0) return u.release;
  return "";
}

std::optional<RuntimeVersion> rocm_version(const std::string& root) {
  std::vector<std::string> candidates;
  // A synthetic root is authoritative (deterministic test trees).
  bool synthetic = !root.empty() && root != "/";
  if (synthetic) candidates.push_back(fs::join(root, "opt/rocm/.info/version"));
  if (const char* rp = std::getenv("ROCM_PATH"); rp && *rp && !synthetic)
    candidates.push_back(fs::join(rp, ".info/version"));
  if (!synthetic) candidates.push_back("/opt/rocm/.info/version");
  for (const auto& c : candidates) {
    auto v = fs::attrs().read_checked_trimmed(c);
    if (!v) continue;
    auto ver = extract_version(*v);
    if (!ver) continue;
    auto parts = str::split(*ver, '.');
    auto maj = str::parse_uint(parts[0]);
    auto min = str::parse_uint(parts[1]);
    if (maj && min) return RuntimeVersion{static_cast<unsigned>(*maj), static_cast<unsigned>(*min)};
  }
  return std::nullopt;
}

std::string driver_version(const std::string& root) {
  std::string raw = host_driver_version(root);
  auto v = extract_version(raw);
  return v ? *v : raw;
}

RuntimeVersion runtime_version(const std::string& root) {
  auto v = rocm_version(root);
  if (!v) throw Error("unable to determine the ROCm version (no .info/version under $ROCM_PATH or /opt/rocm)");
  return *v;
}

}  // namespace gfd::resource
