// Driver / ROCm version discovery shared by the hardware backends.
//
// Reference analogue: NVML SystemGetDriverVersion / SystemGetCudaDriverVersion
// (vendored go-nvml system.go:18-36) consumed by internal/lm/nvml.go:75-106.
// On MI355X:
//   * amdgpu built as DKMS exposes /sys/module/amdgpu/version ("6.12.12");
//     an in-tree amdgpu has no module version and amd-smi reports the kernel
//     banner instead ("Linuxversion6.18.54-ant.1(...)", measured on the
//     MI355X pool), so the driver version is the first X.Y[.Z] in that text.
//   * the "runtime" version is the installed ROCm release
//     ($ROCM_PATH/.info/version, e.g. "7.2.0").
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

// Installed ROCm release.  Looks at $ROCM_PATH/.info/version, then
// <root>/opt/rocm/.info/version.  nullopt if not installed.
std::optional<RuntimeVersion> rocm_version(const std::string& root);

// What the file-backed managers (amd-smi, KFD sysfs) answer for
// GetDriverVersion: the X.Y[.Z] part of host_driver_version, else the raw text.
std::string driver_version(const std::string& root);
// Their GetRuntimeVersion: rocm_version or an error naming where it looked.
RuntimeVersion runtime_version(const std::string& root);

}  // namespace gfd::resource
