# Round evidence on the GPU box: GPU parity suite, PMC HBM traffic (separate FETCH_SIZE /
# WRITE_SIZE passes on the K6 probe), the default bench line (which reads that traffic file),
# and a rocprofv3 kernel trace + stats of the bench.  usage: bash tools/gpu_round.sh <out-tag>
set -o pipefail
TAG=${1:-round}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 > $OUT/fetch.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 > $OUT/write.log 2>&1 &&
python3 tools/pmc_traffic.py $OUT/fetch $OUT/write $OUT/pmc_traffic.json && cp $OUT/pmc_traffic.json profiles/r01_batch/pmc_traffic.json &&
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu > $OUT/kt.log 2>&1 && python3 tools/kt_gaps.py $OUT/kt | grep -E "k_f|gap"
