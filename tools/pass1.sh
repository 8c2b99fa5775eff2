set -o pipefail
out=gpurun_out/r3p1
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.txt 2>&1 || { tail -30 $out/pytest_gpu.txt; exit 1; }
tail -3 $out/pytest_gpu.txt
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
timeout -k 10 200 python tools/writer_ab.py /tmp --cycles 10 --reps 2 --interval 1s > $out/writer.txt 2>&1
