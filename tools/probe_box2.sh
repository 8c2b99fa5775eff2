#!/bin/bash
# Second hardware probe: amd-smi API values + latency, extra sysfs attributes.
out=gpurun_out/probe2
mkdir -p $out
timeout -k 10 120 ./build/amdsmi_probe 5 > $out/amdsmi_probe.txt 2>&1
echo "rc=$?" >> $out/amdsmi_probe.txt
{
d=$(readlink -f /sys/class/drm/renderD176/device)
echo "dev=$d"
for f in xgmi_num_links xgmi_physical_id xgmi_hive_info xgmi_num_hops xgmi_port_num xgmi_device_id board_info mem_info_vram_vendor compute_partition_config/* uevent; do echo "--- $f"; cat $d/$f 2>&1 | head -20; done
echo "--- xcp"; ls -la $d/xcp 2>&1; ls $d/xcp/* 2>&1 | head -40
echo "--- compute_partition_config"; ls -R $d/compute_partition_config 2>&1 | head -40
for f in $(find $d/compute_partition_config -type f 2>/dev/null); do echo "$f: $(cat $f 2>&1 | head -3)"; done
echo "--- kfd node 8 files"; ls /sys/class/kfd/kfd/topology/nodes/8
echo "--- kfd caches count"; ls /sys/class/kfd/kfd/topology/nodes/8/caches | wc -l
echo "--- proc version"; cat /proc/version; uname -r
echo "--- platform xcp"; ls /sys/devices/platform/ | head -80
echo "--- amdgpu_xcp_42"; ls -la /sys/devices/platform/amdgpu_xcp_42/ 2>&1; cat /sys/devices/platform/amdgpu_xcp_42/uevent 2>&1
echo "--- config size/perm"; ls -la $d/config; od -A x -t x1z -v $d/config | head -20
echo "--- id"; id
} > $out/sysfs2.txt 2>&1
echo done
