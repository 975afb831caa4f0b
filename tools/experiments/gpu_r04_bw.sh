# F2's four bitmap words read before any is tested (one LDS wait instead of four serialized
# read-wait pairs, as the compiler had scheduled them): B = opendht_amd/ab/bw/libdhtgpu.so, A = in-tree
# HEAD.  GPU parity + fuzz suites on B first, then alternating benches, probes, the cfg-3 shard.
set -o pipefail
OUT=gpurun_out/r04bw; mkdir -p $OUT
B=opendht_amd/ab/bw/libdhtgpu.so
timeout -k 10 600 env DHTGPU_LIB=$B python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fuzz.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
b() { timeout -k 10 200 env "$@" python bench.py --no-cpu --no-extra --no-scan --steps $S --warmup $W 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 S=$S', round(d['ms_per_step']*1e3,2), 'us/step lat', round(d.get('latency_ms_per_batch',0)*1e3,1), 'F', [round(x*1e3,1) for x in d['roofline']['kernels_ms'].values()])"; }
for i in 1 2; do
  S=1000 W=100 b A=1 && S=1000 W=100 b DHTGPU_LIB=$B && S=20 W=5 b A=1 && S=20 W=5 b DHTGPU_LIB=$B || exit 1
done | tee $OUT/ab.txt
for L in A B; do
  E=$([ $L = B ] && echo DHTGPU_LIB=$B || echo A=1)
  for inf in 1 2; do
    timeout -k 10 200 env $E python tools/batch_probe.py --reps 30 --n 134217728 --q 131072 --inflight $inf > $OUT/cfg3_${L}_$inf.log 2>&1 || exit 1
  done
  timeout -k 10 120 env $E python tools/batch_probe.py --reps 10 > $OUT/probe_$L.log 2>&1 &&
  timeout -k 10 120 env DHTGPU_DBG=256 $E python tools/batch_probe.py --reps 2 --n 134217728 --q 131072 > $OUT/stamps3_$L.log 2>&1 || exit 1
done
grep -H "phases\|ms/call" $OUT/probe_*.log $OUT/cfg3_*.log
for f in $OUT/stamps3_*.log; do echo "== $f"; grep -E "F2 (stream|end)" $f | tail -2; done
