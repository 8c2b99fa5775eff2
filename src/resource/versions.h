// Driver / ROCm version discovery shared by the hardware backends.
//
// Reference analogue: NVML SystemGetDriverVersion / SystemGetCudaDriverVersion
// (vendored go-nvml system.go:18-36) consumed by internal/lm/nvml.go:75-106.
// On MI355X:
//   * amdgpu built as DKMS exposes /sys/module/amdgpu/version ("6.12.12");
//     an in-tree amdgpu has no module version and amd-smi reports the kernel
//     banner instead ("Linuxversion6.18.54-ant.1(...)", measured on the
//     MI355X pool), so the driver version is the first X.Y[.Z] in that text.
//     Both are node-true from inside a pod: /sys and the kernel are the host's.
//   * the "runtime" version is the ROCm release installed on the node
//     (<prefix>/opt/rocm/.info/version, e.g. "7.2.0").  From a pod that is
//     the host's file, not the image's: the manifests mount the host's /opt
//     and pass --host-root; a node without ROCm userspace (driver-only hosts
//     whose workloads bring ROCm in their images) gets no rocm.runtime labels.
//     The reference's cuda.runtime comes from the driver (nvml.go:75-106);
//     amdgpu publishes no runtime release, so the installed one is reported.
#pragma once

#include <optional>
#include <string>

#include "resource/types.h"

namespace gfd::resource {

// First "X.Y" or "X.Y.Z" numeric run in `s` (digits may not be preceded by a
// digit or '.').  "6.18.54-ant.1" -> "6.18.54"; "Linuxversion6.18.54" ->
// "6.18.54"; nullopt if none.
std::optional<std::string> extract_version(const std::string& s);

// amdgpu driver version as seen from `root` ("/" on a real node): the DKMS
// module version if present, else the running kernel release.  Returns the
// raw string (callers normalise with extract_version).
std::string host_driver_version(const std::string& root);

// Installed ROCm release, from the first source that applies:
//   1. `rocm_version_file`: must be readable and hold X.Y[.Z], else Error;
//   2. `host_root` set: <host_root>/opt/rocm/.info/version resolved with the
//      host's symlinks (fs::resolve_in_root); if that link leads outside the
//      mount (e.g. through /etc/alternatives), the highest
//      <host_root>/opt/rocm-X.Y.Z/.info/version;
//   3. a synthetic `root`: <root>/opt/rocm/.info/version;
//   4. otherwise $ROCM_PATH/.info/version, then /opt/rocm/.info/version.
// nullopt: no ROCm release on the node.  `source`, if given, receives the
// file the version came from.
std::optional<RuntimeVersion> rocm_version(const VersionSources& s, std::string* source = nullptr);

// What the file-backed managers (amd-smi, KFD sysfs) answer for
// GetDriverVersion: the X.Y[.Z] part of host_driver_version, else the raw text.
std::string driver_version(const std::string& root);
// Parse "7.2.0" / "7.2.0-123" -> {7, 2}; nullopt if there is no X.Y.
std::optional<RuntimeVersion> parse_runtime_version(const std::string& text);

}  // namespace gfd::resource
