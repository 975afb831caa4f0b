# A/B of one library knob (an environment variable) on the cfg-2 headline and the probes.
# usage: bash tools/experiments/gpu_ab_env.sh <out-tag> <VAR=value for B> [test-selection]
# Runs the named GPU tests first (default: the K6 parity + fuzz suites), then alternates
# A (knob unset) and B over 1,000-step and 20-step benches, then the per-kernel event probe.
set -o pipefail
TAG=$1; KNOB=$2; SEL=${3:-"tests/test_gpu_parity.py tests/test_gpu_fuzz.py"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $SEL > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
b() { timeout -k 10 200 env "$@" python bench.py --no-cpu --no-extra --no-scan --steps $S --warmup $W 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$* S=$S', round(d['ms_per_step']*1e3,2), 'us/step lat', round(d.get('latency_ms_per_batch',0)*1e3,1), 'F', [round(x*1e3,1) for x in d['roofline']['kernels_ms'].values()], 'exact', d.get('verified_exact'))"; }
for i in 1 2; do
  S=1000 W=100 b A=1 && S=1000 W=100 b $KNOB && S=20 W=5 b A=1 && S=20 W=5 b $KNOB || exit 1
done | tee $OUT/ab.txt
timeout -k 10 120 python tools/batch_probe.py --reps 10 > $OUT/probe_A.log 2>&1 && timeout -k 10 120 env $KNOB python tools/batch_probe.py --reps 10 > $OUT/probe_B.log 2>&1 || exit 1
grep -H "phases" $OUT/probe_*.log
echo done
