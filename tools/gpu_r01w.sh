set -o pipefail
OUT=gpurun_out/r01w; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "search_batch or crawl" > $OUT/tests.log 2>&1; tail -25 $OUT/tests.log
