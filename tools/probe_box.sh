#!/bin/bash
# Hardware probe: dumps the driver-visible facts the daemon reads (sysfs, amd-smi).
out=gpurun_out/probe
mkdir -p $out
{
echo "== uname"; uname -a
echo "== nproc"; nproc
echo "== which go"; which go || true
echo "== rocm version"; cat /opt/rocm/.info/version
echo "== dmi"; cat /sys/class/dmi/id/product_name 2>&1
echo "== /dev"; ls -la /dev/kfd /dev/dri 2>&1
echo "== kfd nodes"; ls /sys/class/kfd/kfd/topology/nodes 2>&1
for n in /sys/class/kfd/kfd/topology/nodes/*; do echo "--- $n"; cat $n/name 2>&1; cat $n/gpu_id 2>&1; cat $n/properties 2>&1; ls $n/io_links 2>&1; for l in $n/io_links/*; do echo "link $l"; cat $l/properties 2>&1; done; ls $n/mem_banks 2>&1; for m in $n/mem_banks/*; do cat $m/properties 2>&1; done; done
echo "== kfd generation"; cat /sys/class/kfd/kfd/topology/generation_id 2>&1
echo "== drm"; ls -la /sys/class/drm 2>&1
for c in /sys/class/drm/card*; do [ -e $c/device ] || continue; echo "--- $c"; d=$(readlink -f $c/device); echo $d; for f in vendor device subsystem_vendor subsystem_device revision class current_compute_partition available_compute_partition current_memory_partition available_memory_partition sriov_totalvfs sriov_numvfs product_name product_number serial_number unique_id mem_info_vram_total vbios_version numa_node; do printf "%s=" $f; cat $c/device/$f 2>&1 | head -3; done; ls $c/device 2>&1 | tr '\n' ' '; echo; done
echo "== pci amd devices"; for d in /sys/bus/pci/devices/*; do v=$(cat $d/vendor); if [ "$v" = "0x1002" ]; then echo "$d $(cat $d/class) $(cat $d/device)"; ls -la $d/physfn 2>&1; stat -c %s $d/config; fi; done
echo "== module"; cat /sys/module/amdgpu/version 2>&1; ls /sys/module/amdgpu 2>&1 | head; cat /proc/driver/amdgpu 2>&1 | head
echo "== amd-smi version"; timeout 60 amd-smi version 2>&1
echo "== amd-smi list"; timeout 60 amd-smi list 2>&1
} > $out/probe.txt 2>&1
timeout 120 amd-smi static --json > $out/amdsmi_static.json 2>&1
timeout 120 amd-smi partition --json > $out/amdsmi_partition.json 2>&1
timeout 120 amd-smi topology --json > $out/amdsmi_topology.json 2>&1
timeout 120 amd-smi xgmi --json > $out/amdsmi_xgmi.json 2>&1
echo done
