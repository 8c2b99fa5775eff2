#include "info/version.h"

#ifndef GFD_VERSION
#define GFD_VERSION "unknown"
#endif
#ifndef GFD_GIT_COMMIT
#define GFD_GIT_COMMIT ""
#endif

namespace gfd::info {

std::vector<std::string> version_parts() {
  std::vector<std::string> v{GFD_VERSION};
  std::string commit = GFD_GIT_COMMIT;
  if (!commit.empty()) v.push_back("commit: " + commit);
  return v;
}

std::string version_string(const std::vector<std::string>& more) {
  auto v = version_parts();
  v.insert(v.end(), more.begin(), more.end());
  std::string out;
  for (size_t i = 0; i < v.size(); ++i) {
    if (i) out.push_back('\n');
    out += v[i];
  }
  return out;
}

}  // namespace gfd::info
