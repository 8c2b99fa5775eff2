// Backend selection (internal/resource/factory.go:27-74 analogue).
//
// `--backend=auto` (default) detects the platform and logs why, like the
// reference's "Detected NVML platform: ..." lines:
//   amd-smi loadable            -> AmdSmiManager   (NVML analogue)
//   else KFD topology present   -> SysfsManager    (Tegra/CUDA analogue)
//   else                        -> NullManager
// When both are present amd-smi is preferred and the KFD path takes over if
// amd-smi fails to initialise (PreferenceManager); the reference instead
// disables the second backend ("NVML + Tegra -> Tegra disabled",
// factory.go:53-62).
// Explicit values: amdsmi | sysfs | null | mock (with --mock-file).
#pragma once

#include "config/config.h"
#include "resource/types.h"

namespace gfd::resource {

// Raw backend (no fallback decoration).  Throws on an unknown backend name or
// an unreadable mock fixture.
ManagerPtr get_manager(const config::Config& c);
// get_manager + with_config (fallback to Null on init error unless
// failOnInitError).
ManagerPtr new_manager(const config::Config& c);

}  // namespace gfd::resource
