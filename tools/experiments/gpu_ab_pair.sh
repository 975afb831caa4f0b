# A/B of the in-tree build against one variant library on the cfg-2 headline: alternating 1,000-
# and 20-step benches (ms/step, latency, per-kernel event times), twice.
# usage: bash tools/experiments/gpu_ab_pair.sh <out-tag> <variant.so> [pytest -k selection run first]
set -o pipefail
TAG=$1; V=$2; SEL=$3
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$SEL" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests -k "$SEL" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
b() { timeout -k 10 200 env "$@" python bench.py --no-cpu --no-extra --no-scan --steps $S --warmup $W 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 S=$S', round(d['ms_per_step']*1e3,2), 'us/step lat', round(d.get('latency_ms_per_batch',0)*1e3,1), 'F', [round(x*1e3,1) for x in d['roofline']['kernels_ms'].values()])"; }
for i in 1 2; do
  S=1000 W=100 b X=1 && S=1000 W=100 b DHTGPU_LIB=$V && S=20 W=5 b X=1 && S=20 W=5 b DHTGPU_LIB=$V || exit 1
done | tee $OUT/ab.txt
echo all-ok
