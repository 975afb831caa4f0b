# cfg-3 shard: F2 on half the CUs (sub-partitioned calls) and/or a 4-deep non-temporal ring, one and two calls in flight
set -o pipefail
OUT=gpurun_out/r04f2h; mkdir -p $OUT
DHTGPU_LIB=opendht_amd/ab/f2_d2r4.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_scale.py -k "subpart or shard or cfg3" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  for v in tree d2r4 d2r2 d1r4; do
    lib=""; [ $v != tree ] && lib="DHTGPU_LIB=opendht_amd/ab/f2_$v.so"
    for inf in 1 2; do
      echo -n "$v inflight $inf: "
      timeout -k 10 120 env $lib X=1 python tools/batch_probe.py --reps 30 --n 134217728 --q 131072 --inflight $inf 2>/dev/null | grep -E "ms/call|phases" | tr '\n' ' ' || exit 1
      echo
    done
  done
done | tee $OUT/ab.txt
