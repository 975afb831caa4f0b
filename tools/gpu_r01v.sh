set -o pipefail
OUT=gpurun_out/r01v; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "buffer_nodes or deserialize" > $OUT/tests.log 2>&1; tail -15 $OUT/tests.log
