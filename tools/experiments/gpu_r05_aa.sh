# Round 5, pass aa: batches in flight (2 / 3 / 4) with the lighter F4, 1,000 and 20 steps, twice.
set -o pipefail
OUT=gpurun_out/r05aa; mkdir -p $OUT
b() { timeout -k 10 200 python bench.py --no-cpu --no-extra --no-scan --steps $S --warmup $W --inflight $I 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('inflight $I S=$S', round(d['ms_per_step']*1e3,2), 'us/step lat', round(d.get('latency_ms_per_batch',0)*1e3,1))"; }
for i in 1 2; do
  for I in 3 2 4; do
    S=1000 W=100 b && S=20 W=5 b || exit 1
  done
done | tee $OUT/inflight.txt
echo all-ok
