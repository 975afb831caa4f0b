set -o pipefail
OUT=gpurun_out/r01i; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | cut -c1-250 &&
for r in 0 7; do timeout -k 10 300 python bench.py --simulate-world 8 --simulate-rank $r --no-scan > $OUT/sim8_r$r.log 2>&1 && tail -1 $OUT/sim8_r$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('sim8 rank', d['config']['ids_per_gpu'], d['config']['targets_per_gpu'], d['ms_per_step'], d['value'], d.get('verified_exact'), d['roofline']['kernels_ms'])" || exit 1; done &&
for r in 0 1; do timeout -k 10 300 python bench.py --simulate-world 2 --simulate-rank $r --no-scan > $OUT/sim2_r$r.log 2>&1 && tail -1 $OUT/sim2_r$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('sim2 rank', d['ms_per_step'], d['value'], d.get('verified_exact'))" || exit 1; done &&
timeout -k 10 300 python bench.py --sharded --route broadcast --no-cpu > $OUT/bench_bcast.log 2>&1 && tail -1 $OUT/bench_bcast.log | cut -c1-250
