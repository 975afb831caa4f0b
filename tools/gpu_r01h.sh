set -o pipefail
OUT=gpurun_out/r01h; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log &&
timeout -k 10 300 python bench.py --sharded --no-cpu > $OUT/bench_sharded.log 2>&1 && tail -1 $OUT/bench_sharded.log | cut -c1-300 &&
timeout -k 10 300 python bench.py --algo scan --no-cpu --steps 5 > $OUT/bench_scan.log 2>&1 && tail -1 $OUT/bench_scan.log | cut -c1-300
