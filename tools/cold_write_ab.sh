set -o pipefail
mkdir -p gpurun_out/coldw
{ stat -f -c '%n %T' /tmp /dev/shm "$PWD"; df -h /tmp /dev/shm | head -5; } > gpurun_out/coldw/fs.txt 2>&1
timeout -k 5 120 ./build/cold_write_probe /tmp/gfd-cwp 10 1000 > gpurun_out/coldw/tmp.txt 2>&1 &&
timeout -k 5 120 ./build/cold_write_probe /dev/shm/gfd-cwp 10 1000 > gpurun_out/coldw/shm.txt 2>&1 &&
timeout -k 5 120 env TMPDIR=/dev/shm python3 tools/cold_cycle.py --interval 1s --cycles 10 --backend auto > gpurun_out/coldw/cycle_shm.json 2> gpurun_out/coldw/cycle_shm.err &&
timeout -k 5 120 python3 tools/cold_cycle.py --interval 1s --cycles 10 --backend auto > gpurun_out/coldw/cycle_tmp.json 2> gpurun_out/coldw/cycle_tmp.err
rc=$?
cat gpurun_out/coldw/*.txt gpurun_out/coldw/*.json
exit $rc
