set -o pipefail
OUT=gpurun_out/ksf; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1; tail -1 $OUT/gpu_tests.log
grep -q "passed" $OUT/gpu_tests.log && ! grep -q "failed" $OUT/gpu_tests.log || { tail -30 $OUT/gpu_tests.log; exit 1; }
for v in prev tree prev tree; do
  lib=""; [ $v != tree ] && lib="DHTGPU_LIB=opendht_amd/ab/$v.so"
  timeout -k 10 300 env $lib X=1 python bench.py --no-cpu --no-scan --steps 20 --warmup 5 --verify 0 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read()); sb=d['small_batch']
print('$v', ' '.join('%s %.2f' % (q, sb[q]['batch']['latency_ms']*1e3) for q in ('q1','q8','q32','q64')), 'S1', [round(sb[q]['kernels_ms']['k_s1_filter']*1e3,2) for q in ('q1','q8','q32','q64')])" || exit 1
done | tee $OUT/ks.txt
