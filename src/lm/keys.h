// Label keys emitted by the daemon (the amd.com/* schema).
//
// Reference schema (README.md:195-263, nvidia.com/*) -> MI355X schema:
//   gfd.timestamp                         -> amd.com/gfd.timestamp
//   cuda.driver.{major,minor,rev}         -> amd.com/driver.{major,minor,rev}
//   cuda.runtime.{major,minor}            -> amd.com/rocm.runtime.{major,minor}
//   gpu.machine                           -> amd.com/gpu.machine
//   gpu.{product,count,replicas,memory}   -> amd.com/gpu.{...} (memory in MiB)
//   gpu.family, gpu.compute.{major,minor} -> amd.com/gpu.{family,arch},
//                                            amd.com/gpu.compute.{major,minor}
//   mig.capable                           -> amd.com/gpu.partition.capable
//   mig.strategy                          -> amd.com/partition.strategy
//   mig-<profile>.*                       -> amd.com/partition-<profile>.*
//   vgpu.present                          -> amd.com/sriov.present (+ role,
//                                            num-vfs, total-vfs)
//   (new) amd.com/gpu.{compute-units,xcds,compute-partition,memory-partition,
//         xgmi.links,virtualization-mode}
#pragma once

namespace gfd::lm::keys {

inline constexpr const char* kPrefix = "amd.com";
inline constexpr const char* kTimestamp = "amd.com/gfd.timestamp";
inline constexpr const char* kDriverMajor = "amd.com/driver.major";
inline constexpr const char* kDriverMinor = "amd.com/driver.minor";
inline constexpr const char* kDriverRev = "amd.com/driver.rev";
inline constexpr const char* kRuntimeMajor = "amd.com/rocm.runtime.major";
inline constexpr const char* kRuntimeMinor = "amd.com/rocm.runtime.minor";
inline constexpr const char* kMachine = "amd.com/gpu.machine";
inline constexpr const char* kPartitionCapable = "amd.com/gpu.partition.capable";
inline constexpr const char* kPartitionStrategy = "amd.com/partition.strategy";
inline constexpr const char* kComputePartition = "amd.com/gpu.compute-partition";
inline constexpr const char* kMemoryPartition = "amd.com/gpu.memory-partition";
inline constexpr const char* kXgmiLinks = "amd.com/gpu.xgmi.links";
inline constexpr const char* kVirtualization = "amd.com/gpu.virtualization-mode";
inline constexpr const char* kSriovPresent = "amd.com/sriov.present";
inline constexpr const char* kSriovRole = "amd.com/sriov.role";
inline constexpr const char* kSriovNumVfs = "amd.com/sriov.num-vfs";
inline constexpr const char* kSriovTotalVfs = "amd.com/sriov.total-vfs";
inline constexpr const char* kSriovHostDriverVersion = "amd.com/sriov.host-driver-version";

// Full-GPU resource and the prefix of per-profile partition resources.
inline constexpr const char* kFullGpuResource = "amd.com/gpu";
inline constexpr const char* kPartitionResourcePrefix = "amd.com/partition-";

}  // namespace gfd::lm::keys
