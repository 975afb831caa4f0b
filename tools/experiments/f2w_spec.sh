# F2 batched run writes (tree vs prev) and F3's speculative gather sizes (env knob) on the cfg-2 period
set -o pipefail
OUT=gpurun_out/f2w; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_scale.py > $OUT/tests.log 2>&1; tail -1 $OUT/tests.log
grep -q "passed" $OUT/tests.log && ! grep -q "failed" $OUT/tests.log || exit 1
run() { local tag=$1; shift; timeout -k 10 200 env "$@" python bench.py --no-cpu --no-extra --no-scan --steps 1000 --warmup 100 --verify 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['ms_per_step']*1e3,2), 'us/step lat', round(d.get('latency_ms_per_batch',0)*1e3,1), 'F', [round(x*1e3,1) for x in d['roofline']['kernels_ms'].values()])"; }
for i in 1 2; do
  run prev DHTGPU_LIB=opendht_amd/ab/prev.so && run tree X=1 && run spec256 DHTGPU_F3SPEC=256 && run spec320 DHTGPU_F3SPEC=320 || exit 1
done | tee $OUT/ab.txt
