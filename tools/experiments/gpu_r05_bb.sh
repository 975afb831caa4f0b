# Round 5, pass bb: F2 with 2x / 4x more (shorter) workgroups than CUs, and the verified
# 1,000-step world-of-one collective line.
set -o pipefail
OUT=gpurun_out/r05bb; mkdir -p $OUT
timeout -k 10 400 python bench.py --sharded --steps 1000 --warmup 100 --no-extra --verify 64 > $OUT/sharded_1000.json 2> $OUT/sharded_1000.err || { tail -20 $OUT/sharded_1000.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$OUT/sharded_1000.json') if l.startswith('{')][-1]); print('sharded 1000', round(d['ms_per_step']*1e3,2), d.get('verified_exact'), d.get('verified_targets'))"
for v in f2x2 f2x4; do
  DHTGPU_LIB=opendht_amd/ab/$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "batch" > $OUT/tests_$v.log 2>&1 || { tail -30 $OUT/tests_$v.log; exit 1; }
  echo "$v $(tail -1 $OUT/tests_$v.log)"
done
b() { timeout -k 10 200 env "$@" python bench.py --no-cpu --no-extra --no-scan --steps $S --warmup $W 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 S=$S', round(d['ms_per_step']*1e3,2), 'us/step lat', round(d.get('latency_ms_per_batch',0)*1e3,1), 'F', [round(x*1e3,1) for x in d['roofline']['kernels_ms'].values()])"; }
for i in 1 2; do
  for v in tree f2x2 f2x4; do
    lib=X=1; [ $v != tree ] && lib=DHTGPU_LIB=opendht_amd/ab/$v.so
    S=1000 W=100 b $lib && S=20 W=5 b $lib || exit 1
  done
done | tee $OUT/ab.txt
echo all-ok
