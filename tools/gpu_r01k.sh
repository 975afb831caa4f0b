set -o pipefail
OUT=gpurun_out/r01k; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench.py --no-scan > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N1', d['ms_per_step'], d['value'], d.get('verified_exact'), d['roofline']['kernels_ms'])" &&
for g in 2 8; do timeout -k 10 300 python bench.py --simulate-world $g --simulate-rank 0 --no-scan > $OUT/sim${g}.log 2>&1 && tail -1 $OUT/sim${g}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('sim$g', d['ms_per_step'], d['value'], d.get('verified_exact'), d['roofline']['kernels_ms'])" || exit 1; done
