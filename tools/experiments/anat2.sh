set -o pipefail
OUT=gpurun_out/anat2; mkdir -p $OUT
run() { local tag=$1; shift; timeout -k 10 200 env "$@" python bench.py --no-cpu --no-extra --no-scan --steps 1000 --warmup 100 --verify 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['ms_per_step']*1e3,2), 'us/step lat', round(d.get('latency_ms_per_batch',0)*1e3,1), 'F', [round(x*1e3,1) for x in d['roofline']['kernels_ms'].values()])"; }
for i in 1 2; do
  run full X=1 && run f4min DHTGPU_LIB=opendht_amd/ab/measure.so DHTGPU_F4MIN_MEASURE=1 && run f12 DHTGPU_DBG=1 || exit 1
done | tee $OUT/ab.txt
