set -o pipefail
OUT=gpurun_out/r01m; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --no-cpu --steps 10 --warmup 2 > $OUT/kt.log 2>&1 && echo kt-ok
