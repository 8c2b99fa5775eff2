// Build version information (internal/info/version.go:22-43 analogue).
// GFD_VERSION and GFD_GIT_COMMIT are injected by CMake (the reference uses
// `go build -ldflags -X`, Makefile:57-59).
#pragma once

#include <string>
#include <vector>

namespace gfd::info {

// {version, "commit: <sha>"} (commit omitted when unknown).
std::vector<std::string> version_parts();
// version_parts() + extra, joined by newlines.
std::string version_string(const std::vector<std::string>& more = {});

}  // namespace gfd::info
