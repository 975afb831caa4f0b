# A/B of two builds of libdhtgpu on the cfg-2 headline: A = opendht_amd/ab/prev.so (an earlier
# commit, built by hand), B = the in-tree build.  GPU tests of B first (default: the K6 parity +
# fuzz suites), then alternating 1,000- and 20-step benches, then the per-kernel event probes.
# usage: bash tools/experiments/gpu_ab_lib.sh <out-tag> [test-selection | none]
set -o pipefail
TAG=$1; SEL=${2:-"tests/test_gpu_parity.py tests/test_gpu_fuzz.py"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
A=opendht_amd/ab/prev.so
if [ "$SEL" != none ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $SEL > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
b() { timeout -k 10 200 env "$@" python bench.py --no-cpu --no-extra --no-scan --steps $S --warmup $W 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 S=$S', round(d['ms_per_step']*1e3,2), 'us/step lat', round(d.get('latency_ms_per_batch',0)*1e3,1), 'F', [round(x*1e3,1) for x in d['roofline']['kernels_ms'].values()])"; }
for i in 1 2; do
  S=1000 W=100 b DHTGPU_LIB=$A && S=1000 W=100 b B=1 && S=20 W=5 b DHTGPU_LIB=$A && S=20 W=5 b B=1 || exit 1
done | tee $OUT/ab.txt
timeout -k 10 120 env DHTGPU_LIB=$A python tools/batch_probe.py --reps 10 > $OUT/probe_A.log 2>&1 && timeout -k 10 120 python tools/batch_probe.py --reps 10 > $OUT/probe_B.log 2>&1 || exit 1
timeout -k 10 200 env DHTGPU_LIB=$A python tools/batch_probe.py --reps 10 --n 134217728 --q 131072 > $OUT/cfg3_A.log 2>&1 && timeout -k 10 200 python tools/batch_probe.py --reps 10 --n 134217728 --q 131072 > $OUT/cfg3_B.log 2>&1 || exit 1
grep -H "phases\|ms/call" $OUT/probe_*.log $OUT/cfg3_*.log
echo done
