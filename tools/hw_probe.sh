#!/bin/bash
# Hardware facts the daemon relies on, as a real MI355X node exposes them to an
# unprivileged container: KFD topology, amdgpu PCI attributes, DRM nodes,
# partition configuration, SR-IOV / virtualization traces, amd-smi's own view.
# Source of profiles/hw_probe.md.  Every command is read-only and time-limited.
# Usage (GPU box): tools/hw_probe.sh [outdir-name]
out=gpurun_out/${1:-hw_probe}
mkdir -p "$out"
gpu=$(for c in /sys/class/drm/renderD*; do [ -e "$c/device/vendor" ] && readlink -f "$c/device" && break; done)
{
  echo "== uname"; uname -a
  echo "== rocm version"; cat /opt/rocm/.info/version; readlink -f /opt/rocm
  echo "== dmi"; cat /sys/class/dmi/id/product_name 2>&1
  echo "== id"; id
  echo "== /dev"; ls -la /dev/kfd /dev/dri 2>&1
  echo "== kfd generation"; cat /sys/class/kfd/kfd/topology/generation_id 2>&1
  echo "== kfd nodes"
  for n in /sys/class/kfd/kfd/topology/nodes/*; do
    echo "--- $n"; cat "$n/gpu_id" 2>&1; cat "$n/properties" 2>&1
    for m in "$n"/mem_banks/*; do cat "$m/properties" 2>&1; done
  done
  echo "== drm cards"
  for c in /sys/class/drm/card*; do
    [ -e "$c/device" ] || continue
    echo "--- $c -> $(readlink -f "$c/device")"
    for f in vendor device class current_compute_partition available_compute_partition current_memory_partition \
             available_memory_partition sriov_totalvfs sriov_numvfs product_name serial_number unique_id \
             mem_info_vram_total xgmi_num_links xgmi_physical_id numa_node; do
      printf "%s=" "$f"; head -3 "$c/device/$f" 2>&1
    done
  done
  if [ -n "$gpu" ]; then
    echo "== $gpu: attributes"; ls "$gpu"
    echo "== compute_partition_config"
    for f in $(find "$gpu/compute_partition_config" -type f 2>/dev/null); do echo "$f: $(head -3 "$f" 2>&1)"; done
    echo "== config space as this user"; stat -c '%s bytes, mode %a' "$gpu/config"; od -A x -t x1 -N 64 "$gpu/config"
  fi
  echo "== platform xcp devices (partition render nodes)"; ls /sys/devices/platform/ | grep -i xcp | head -20
  echo "== AMD PCI functions"
  for d in /sys/bus/pci/devices/*; do
    [ "$(cat "$d/vendor")" = "0x1002" ] || continue
    echo "$d class=$(cat "$d/class") device=$(cat "$d/device") driver=$(basename "$(readlink "$d/driver" 2>/dev/null)")"
  done
  echo "== driver modules (amdgpu; gim = the MxGPU SR-IOV host driver)"
  for m in amdgpu gim; do printf "%s: " "$m"; cat "/sys/module/$m/version" 2>&1; done
  echo "== hypervisor flag"; grep -m1 -o -w hypervisor /proc/cpuinfo || echo none
  echo "== amd-smi"; timeout 60 amd-smi version 2>&1; timeout 60 amd-smi list 2>&1
} > "$out/probe.txt" 2>&1
for v in static partition topology xgmi; do timeout 120 amd-smi "$v" --json > "$out/amdsmi_$v.json" 2>&1; done
echo "wrote $out"
