// Node-level labelers and the top-level labeler assembly.
//
// Reference: internal/lm/labeler.go:33-45 (NewLabelers), nvml.go:29-137
// (NVML labeler, version labeler, MIG-capability labeler), timestamp.go,
// machine-type.go, vgpu.go.
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <optional>
#include <string>

#include "config/config.h"
#include "lm/labels.h"
#include "resource/types.h"
#include "sriov/sriov.h"

namespace gfd::lm {

// amd.com/gfd.timestamp=<unix seconds> unless --no-timestamp.  The value is
// captured when the labeler is built (once per run, main.go:158).
LabelerPtr NewTimestampLabeler(const config::Config& config);
LabelerPtr NewTimestampLabeler(const config::Config& config, int64_t unix_seconds);

// amd.com/gpu.machine from the DMI product name (machine-type.go:30-51).
LabelerPtr NewMachineTypeLabeler(const std::string& machine_type_path);

// amd.com/driver.{major,minor,rev} + amd.com/rocm.runtime.{major,minor}
// (nvml.go:75-106).  The driver version must match X.Y[.Z].
LabelerPtr NewVersionLabeler(resource::Manager& manager);

// amd.com/gpu.partition.capable (nvml.go:110-137).
LabelerPtr NewPartitionCapabilityLabeler(resource::Manager& manager);

// amd.com/gpu.{compute-partition,memory-partition,xgmi.links,
// virtualization-mode}: node-wide facts that have no NVIDIA counterpart.
// A value that differs between GPUs is reported as "mixed" (links: minimum).
LabelerPtr NewTopologyLabeler(resource::Manager& manager);

// SR-IOV labels, evaluated lazily at GetLabels() time like the reference's
// vGPU labeler (lm/vgpu.go:37-55).
LabelerPtr NewSriovLabeler(std::shared_ptr<sriov::Interface> lib);

// Node facts that need no device context: the DMI machine type and, for
// managers whose version queries are plain file reads
// (Manager::VersionFiles), the driver and ROCm versions.  The daemon
// reads them on a worker while the backend enumerates the GPUs.
struct NodeFacts {
  Labels machine;               // amd.com/gpu.machine
  std::string machine_warning;  // logged when the labels are used
  bool have_versions = false;
  std::string driver_version;
  std::optional<resource::RuntimeVersion> runtime_version;  // nullopt: no ROCm on the node
  std::string runtime_error;  // a configured version source failed
};
NodeFacts ReadNodeFacts(const config::Config& config, const std::optional<resource::VersionSources>& version_files);

// The device labeler (NewNVMLLabeler analogue, nvml.go:29-72): Init, defer
// Shutdown, enumerate, and build every device-derived labeler eagerly inside
// that window.  Zero devices -> empty.  `facts`, if given, is called (once,
// after enumeration) for facts read concurrently; it may block until they
// are ready.
LabelerPtr NewDeviceLabeler(resource::Manager& manager, const config::Config& config,
                            const std::function<const NodeFacts&()>& facts = nullptr);

// NewLabelers (labeler.go:33-45): Merge(device labeler, SR-IOV labeler).
LabelerPtr NewLabelers(resource::Manager& manager, std::shared_ptr<sriov::Interface> sriov,
                       const config::Config& config);

}  // namespace gfd::lm
