# F2 ring depth (DHT_F2_RING = 2 in-tree, 3 / 4 in opendht_amd/ab/ring{3,4}.so): cfg-3 shard at one
# and two calls in flight, cfg 2 per-kernel probe, cfg-2 bench at 1,000 and 20 steps
set -o pipefail
OUT=gpurun_out/r04ring; mkdir -p $OUT
run() { # $1 label, rest env
  L=$1; shift
  for inf in 1 2; do
    echo "$L cfg3 inflight $inf: $(timeout -k 10 120 env "$@" python tools/batch_probe.py --reps 30 --n 134217728 --q 131072 --inflight $inf 2>&1 | grep -E 'ms/call|phases' | tr '\n' ' ')" >> $OUT/ab.txt || return 1
  done
  echo "$L cfg2: $(timeout -k 10 120 env "$@" python tools/batch_probe.py --reps 30 2>&1 | grep -E 'ms/call|phases' | tr '\n' ' ')" >> $OUT/ab.txt || return 1
  for S in 1000 20; do
    W=$([ $S = 20 ] && echo 5 || echo 100)
    echo "$L bench S=$S: $(timeout -k 10 200 env "$@" python bench.py --no-cpu --no-extra --no-scan --steps $S --warmup $W 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1e3,2), 'us/step lat', round(d.get('latency_ms_per_batch',0)*1e3,1), 'F', [round(x*1e3,1) for x in d['roofline']['kernels_ms'].values()])")" >> $OUT/ab.txt || return 1
  done
}
for rep in 1 2; do
  run ring2 B=1 && run ring3 DHTGPU_LIB=opendht_amd/ab/ring3.so && run ring4 DHTGPU_LIB=opendht_amd/ab/ring4.so || exit 1
done
cat $OUT/ab.txt
