set -o pipefail
OUT=gpurun_out/r01x; mkdir -p $OUT
timeout -k 10 400 python -u tools/crawl_bench.py > $OUT/crawl.log 2>&1; rc=$?; tail -3 $OUT/crawl.log; exit $rc
