set -o pipefail
OUT=gpurun_out/r01y2; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] &&
for g in 2 8; do timeout -k 10 300 python bench.py --simulate-world $g --simulate-rank 1 --no-scan > $OUT/sim${g}.log 2>&1 && tail -1 $OUT/sim${g}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('sim$g', d['ms_per_step'], d['value'], d.get('verified_exact'), d['roofline']['kernels_ms'])" || exit 1; done &&
timeout -k 10 300 python bench.py --sharded --route broadcast --no-scan > $OUT/bcast.log 2>&1 && tail -1 $OUT/bcast.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bcast', d['ms_per_step'], d['value'], d.get('verified_exact'))"
