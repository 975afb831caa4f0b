# cfg-2 period vs in-flight depth and F4's quiet grid (1,000 steps, rotated twice)
set -o pipefail
OUT=gpurun_out/knobs1; mkdir -p $OUT
run() { local tag=$1; shift; timeout -k 10 200 env "$@" python bench.py --no-cpu --no-extra --no-scan --steps 1000 --warmup 100 --verify 0 $XA 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['ms_per_step']*1e3,2), 'us/step lat', round(d.get('latency_ms_per_batch',0)*1e3,1))"; }
for i in 1 2; do
  XA="" run base X=1 && XA="--inflight 4" run inflight4 X=1 && XA="--inflight 2" run inflight2 X=1 &&
  XA="" run f4q64 DHTGPU_F4QUIET=64 && XA="" run f4q32 DHTGPU_F4QUIET=32 && XA="" run f4q192 DHTGPU_F4QUIET=192 || exit 1
done | tee $OUT/knobs.txt
