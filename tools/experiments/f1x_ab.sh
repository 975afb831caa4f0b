# Is F1 on the cfg-2 step's critical path?  DHTGPU_F1X variants (1: plain bitmap stores -- wrong
# results, same work downstream; 8: slot atomic first; 16: +1 us per F1 wave), --verify 0.
set -o pipefail
OUT=gpurun_out/f1x; mkdir -p $OUT
b() { timeout -k 10 200 env $1 python bench.py --no-cpu --no-extra --no-scan --verify 0 --steps $2 --warmup $3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 S=$2', round(d['ms_per_step']*1e3,2), 'us/step lat', round(d.get('latency_ms_per_batch',0)*1e3,1), 'F', [round(x*1e3,1) for x in d['roofline']['kernels_ms'].values()])"; }
for i in 1 2; do
  for v in A=1 DHTGPU_F1X=1 DHTGPU_F1X=8 DHTGPU_F1X=16; do b $v 1000 100 || exit 1; done
  for v in A=1 DHTGPU_F1X=1; do b $v 20 5 || exit 1; done
done | tee $OUT/ab.txt
