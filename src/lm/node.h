// Node-level labelers and the top-level labeler assembly.
//
// Reference: internal/lm/labeler.go:33-45 (NewLabelers), nvml.go:29-137
// (NVML labeler, version labeler, MIG-capability labeler), timestamp.go,
// machine-type.go, vgpu.go.
#pragma once

#include <cstdint>
#include <memory>
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

// The device labeler (NewNVMLLabeler analogue, nvml.go:29-72): Init, defer
// Shutdown, enumerate, and build every device-derived labeler eagerly inside
// that window.  Zero devices -> empty.
LabelerPtr NewDeviceLabeler(resource::Manager& manager, const config::Config& config);

// NewLabelers (labeler.go:33-45): Merge(device labeler, SR-IOV labeler).
LabelerPtr NewLabelers(resource::Manager& manager, std::shared_ptr<sriov::Interface> sriov,
                       const config::Config& config);

}  // namespace gfd::lm
