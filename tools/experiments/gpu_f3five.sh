# five F3 workgroups per CU: parity through each variant, then the headline A/B (1,000 and 20 steps)
set -o pipefail
OUT=gpurun_out/${1:-f3five}; mkdir -p $OUT
for v in f3five55 f3five48; do
  DHTGPU_LIB=opendht_amd/ab/$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "batch" > $OUT/tests_$v.log 2>&1 || { tail -30 $OUT/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/tests_$v.log)"
done
b() { timeout -k 10 200 env "$@" python bench.py --no-cpu --no-extra --no-scan --steps $S --warmup $W 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 S=$S', round(d['ms_per_step']*1e3,2), 'us/step lat', round(d.get('latency_ms_per_batch',0)*1e3,1), 'F', [round(x*1e3,1) for x in d['roofline']['kernels_ms'].values()], 'fb', d.get('fallback_targets'))"; }
for i in 1 2; do
  S=1000 W=100 b X=1 && S=1000 W=100 b DHTGPU_LIB=opendht_amd/ab/f3five55.so && S=1000 W=100 b DHTGPU_LIB=opendht_amd/ab/f3five48.so && S=20 W=5 b X=1 && S=20 W=5 b DHTGPU_LIB=opendht_amd/ab/f3five55.so || exit 1
done | tee $OUT/ab.txt
echo all-ok
