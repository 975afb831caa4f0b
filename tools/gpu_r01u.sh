set -o pipefail
OUT=gpurun_out/r01u; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "batch or topk_sizes or clustered or adversarial or 2p24 or duplicates or prefix" > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 > $OUT/pmc_fetch.log 2>&1 && echo fetch-ok &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 > $OUT/pmc_write.log 2>&1 && echo write-ok &&
python3 tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_traffic.json > /dev/null && mkdir -p profiles/r01_batch && cp $OUT/pmc_traffic.json profiles/r01_batch/ &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --no-cpu --no-scan --steps 20 --warmup 2 > $OUT/kt.log 2>&1 && echo kt-ok &&
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | cut -c1-300
