# F2 / F3 CU sharing at 1 / 2 / 3 batches in flight (residency log), then the headline at 1,000
# steps (needs opendht_amd/ab/reslog.so: build_variant.sh reslog "-DDHT_RESLOG")
set -o pipefail
OUT=gpurun_out/${1:-res}; mkdir -p $OUT
for f in 3 2 1; do
  DHTGPU_LIB=opendht_amd/ab/reslog.so timeout -k 10 180 python tools/experiments/residency_probe.py --inflight $f > $OUT/res_inflight$f.json 2> $OUT/res_inflight$f.err || { tail -20 $OUT/res_inflight$f.err; exit 1; }
  cat $OUT/res_inflight$f.json
done
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu --no-extra --no-scan > $OUT/bench1000.json 2> $OUT/bench1000.err || { tail -20 $OUT/bench1000.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench1000.json')); print('bench1000', round(d['ms_per_step']*1e3,2), 'us/step', {k: round(v*1e3,1) for k,v in d['roofline']['kernels_ms'].items()})"
echo all-ok
