set -o pipefail
OUT=gpurun_out/r01s; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python tools/batch_probe.py > $OUT/probe.log 2>&1 && cat $OUT/probe.log | tail -2 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | cut -c1-900
