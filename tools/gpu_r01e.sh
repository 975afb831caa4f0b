set -o pipefail
OUT=gpurun_out/r01e; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | cut -c1-300 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --sharded > $OUT/bench_sharded.log 2>&1 && tail -1 $OUT/bench_sharded.log
