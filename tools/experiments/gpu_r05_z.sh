# Round 5, pass z: the idle F4 grid at 32 / 16 / 8 workgroups (fallback tests with 8 first).
set -o pipefail
OUT=gpurun_out/r05z; mkdir -p $OUT
for v in f4g8; do
  lib=""; [ $v != tree ] && lib=opendht_amd/ab/$v.so
  DHTGPU_LIB=$lib timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k "fallback or clustered or batch or records" > $OUT/tests_$v.log 2>&1 || { tail -30 $OUT/tests_$v.log; exit 1; }
  echo "$v $(tail -1 $OUT/tests_$v.log)"
done
b() { timeout -k 10 200 env "$@" python bench.py --no-cpu --no-extra --no-scan --steps $S --warmup $W 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 S=$S', round(d['ms_per_step']*1e3,2), 'us/step lat', round(d.get('latency_ms_per_batch',0)*1e3,1), 'F', [round(x*1e3,1) for x in d['roofline']['kernels_ms'].values()])"; }
for i in 1 2; do
  for v in f4g32 f4g16 f4g8; do
    lib=X=1; [ $v != tree ] && lib=DHTGPU_LIB=opendht_amd/ab/$v.so
    S=1000 W=100 b $lib && S=20 W=5 b $lib || exit 1
  done
done | tee $OUT/ab.txt
echo all-ok
