# cfg-2 headline at 2 / 3 / 4 batches in flight (HEAD), 1,000 and 20 steps, rotated twice
set -o pipefail
OUT=gpurun_out/r04infl; mkdir -p $OUT
for i in 1 2; do for inf in 3 2 4; do for st in "1000 100" "20 5"; do
  set -- $st
  echo -n "inflight $inf S=$1: "
  timeout -k 10 200 python bench.py --no-cpu --no-extra --no-scan --steps $1 --warmup $2 --verify 0 --inflight $inf 2>/dev/null |
    python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1e3,2), 'us/step lat', round(d.get('latency_ms_per_batch',0)*1e3,1))" || exit 1
done; done; done | tee $OUT/inflight.txt
