set -o pipefail
OUT=gpurun_out/r01g; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --algo index > $OUT/bench_index.log 2>&1 && tail -1 $OUT/bench_index.log | cut -c1-300 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu --algo index > $OUT/kt.log 2>&1 && echo kt-ok
