// Physical-GPU identity of KFD nodes and amd-smi processors.
//
// Reference analogue: the MIG parent/child walk (internal/mig/mig.go:41-124,
// internal/resource/nvml-mig-device.go:27-134, go-nvlib
// nvlib/device/device.go:91-118), where NVML hands out MIG devices as
// children of their parent's handle.  Neither amd-smi nor KFD has such a
// parent link for compute partitions (XCPs): each partition is a KFD node /
// amd-smi processor of its own, so the backends regroup them.
//
// What identifies the physical GPU of a partition (upstream amdgpu,
// kfd_topology.c): on GC 9.4.3-class parts (gfx94x, gfx950) KFD sets
//     location_id = pci_dev_id(parent) | xcp node_id
// i.e. partition k of a GPU at dddd:bb:00.0 reports dddd:bb:00.k, and
// amd-smi (which takes its BDF from the KFD node) reports the same.  Older
// kernels report the parent's location for every partition.  Domain, bus
// and device number (amd-smi's own "socket id") and the ASIC serial
// (KFD unique_id, amd-smi asic_serial) are the same for every partition
// under both layouts, so they are the grouping key; the function bits are
// ignored for partition-capable families only.  The parent PCI function -
// where amdgpu publishes the GPU-wide attributes (current_compute_partition,
// mem_info_vram_total, xgmi_num_links, ...) - is then the lowest member
// address that is a PCI function of the same device ID (partition 0 reports
// it exactly), else the address with the function bits cleared.
//
// AMD's own CLI (in the ROCm image: /opt/rocm/libexec/amdsmi_cli) follows
// the same model, and tests/test_amd_partition_rules.py runs its code
// against both backends:
//   * a partition's id is amdsmi_get_gpu_kfd_info's current_partition_id
//     (amdsmi_helpers.py:1691-1698) - the amd-smi backend's partition id;
//     the KFD backend reads it from the function bits of the node's
//     location (sysfs.cpp, describe_gpu);
//   * the primary partition of the processor at `bdf` is the one at
//     bdf[:10] + ".0", if its id is 0 (amdsmi_helpers.py:1700-1718) - the
//     parent function resolve_parent_bdf returns;
//   * a processor is primary iff its partition id is 0
//     (amdsmi_helpers.py:1720-1725).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "resource/types.h"

namespace gfd::resource {

// True for ASIC families whose partitions carry their index in the PCI
// function bits (gfx 9.4.x, 9.5.x: MI300, MI325, MI350/MI355).
bool partition_index_in_function_bits(const GfxTarget& t);

// "dddd:bb:dd.f" -> "dddd:bb:dd" (amd-smi's socket id of the function).
std::string bdf_slot(const std::string& bdf);

// The members (KFD nodes or amd-smi processors) that one PCI slot and
// device ID group as one physical GPU, checked against their identities
// (`id_of`: KFD unique_id / amd-smi ASIC serial; `bdf_of`: the member's
// address).  Current kernels give every partition the GPU's serial, so a
// group that agrees is one GPU.  One that disagrees is either a GPU whose
// kernel reports a serial per partition - kept whole, with a warning (once
// per slot), rather than counted as 8 GPUs - or distinct GPUs that share a
// slot (SR-IOV virtual functions behind ARI), told apart by every member
// being a PCI function of its own under <root>/sys/bus/pci/devices
// (partition addresses other than the GPU's own are not): split by serial.
bool all_pci_functions(const std::string& root, const std::vector<std::string>& bdfs);
void log_identity_mismatch(const std::string& slot, size_t members);
template <typename T, typename IdOf, typename BdfOf>
std::vector<std::vector<T>> split_by_identity(const std::string& root, std::vector<T> members, IdOf id_of,
                                              BdfOf bdf_of) {
  bool agree = true;
  for (const auto& m : members) agree = agree && id_of(m) == id_of(members.front());
  if (agree) return {std::move(members)};
  std::vector<std::string> bdfs;
  for (const auto& m : members) bdfs.push_back(bdf_of(m));
  if (!all_pci_functions(root, bdfs)) {
    log_identity_mismatch(bdf_slot(bdfs.front()), members.size());
    return {std::move(members)};
  }
  std::vector<std::vector<T>> out;
  std::vector<decltype(id_of(members.front()))> ids;
  for (auto& m : members) {
    auto id = id_of(m);
    size_t i = 0;
    while (i < ids.size() && !(ids[i] == id)) ++i;
    if (i == ids.size()) {
      ids.push_back(id);
      out.emplace_back();
    }
    out[i].push_back(std::move(m));
  }
  return out;
}

// Parent PCI function of a physical GPU whose members (partitions, or the
// GPU itself) report `member_bdfs`.  `device_id` 0 accepts any device.
// Candidates: the member addresses in ascending order, then the slot's
// function 0; the first with <root>/sys/bus/pci/devices/<bdf>/device equal
// to `device_id` wins.  Without a readable PCI tree (or no match) the lowest
// member address is returned.
std::string resolve_parent_bdf(const std::string& root, std::vector<std::string> member_bdfs, uint32_t device_id);

// amdgpu's own virtualization classification (amdgpu_detect_virtualization)
// from what a container can see, for the PCI function at `pci_dir`: an
// SR-IOV virtual function (MxGPU VF device ID, or a `physfn` link) runs as a
// guest; a physical function with VFs enabled is the host; a whole GPU in a
// VM (`in_vm`: running_in_vm) is passthrough; otherwise bare metal.
std::string classify_virtualization(const std::string& pci_dir, uint32_t device_id, bool in_vm, bool has_physfn);

// Device-local memory (bytes) of a KFD topology node: the sum of its
// frame-buffer memory banks (mem_banks/N/properties, heap types 1 and 2).
// For a partition node that is the partition's share of HBM
// (KFD_XCP_MEMORY_SIZE); 0 if unreadable.
uint64_t kfd_node_memory_bytes(const std::string& node_dir);

// Engine counts per partition that amdgpu publishes for the current compute
// partition mode under the parent function
// (compute_partition_config/{dec,jpeg}/num_inst -> engines.decoder,
// engines.jpeg; mode 0400 on current kernels, so a non-root pod sees none).
// amd-smi's accelerator-partition profile reports the same files and is
// refused to non-root callers the same way (profiles/hw_probe.md).
Attributes partition_engine_counts(const std::string& root, const std::string& parent_bdf);

// The attribute set of one compute partition - built here so that both
// backends label a partition identically.  `sdma` is the partition's KFD
// node num_sdma_engines (-1: unknown, omitted).
Attributes partition_attributes(uint64_t memory_mib, uint32_t compute_units, uint32_t xcds, int sdma,
                                const Attributes& engines, const std::string& compute_partition,
                                const std::string& memory_partition);

}  // namespace gfd::resource
