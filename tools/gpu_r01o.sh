set -o pipefail
OUT=gpurun_out/r01o; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "batch or topk_sizes or clustered or adversarial or duplicates or empty or 2p24 or full_batch or prefix_shard" > $OUT/gpu_tests.log 2>&1; rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log
