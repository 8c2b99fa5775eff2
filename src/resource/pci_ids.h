// AMD Instinct PCI device IDs the daemon needs to recognise without a
// management library: marketing names for the KFD-sysfs backend and the
// MxGPU (SR-IOV) virtual-function IDs for both the backends and the SR-IOV
// scanner.  Reference analogue: none (NVML names devices itself; vGPU guests
// are recognised by a vendor capability, internal/vgpu/vgpu.go:93-105).
#pragma once

#include <cstdint>
#include <string>

namespace gfd::resource {

// "AMD Instinct MI355X" for 0x75a3; "AMD-GPU-0x<id>" if unknown.
std::string device_name(uint32_t device_id);

// True for the device ID of an Instinct SR-IOV virtual function (what a
// guest VM sees instead of the physical function's ID).
bool is_mxgpu_vf(uint32_t device_id);

// Same, for the sysfs spelling "0x75b3".
bool is_mxgpu_vf(const std::string& device_id);

// The UUID spelling amd-smi reports, derived from the ASIC serial
// (KFD `unique_id`, amd-smi `asic_serial`) and device ID - measured on the
// pool: serial 0x3a7c178b7c5e4d5c, device 0x75a3 ->
// "3aff75a3-0000-1000-807c-178b7c5e4d5c".  "" for serial 0.
std::string amd_uuid(uint64_t unique_id, uint32_t device_id);

}  // namespace gfd::resource
