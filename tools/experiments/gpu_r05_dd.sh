# Round 5, pass dd: the cfg-3 shard's F4 grid after a clean call (256 / 128 / 64 workgroups),
# two in flight, indices and handles; the sub-partition tests with 64 first.
set -o pipefail
OUT=gpurun_out/r05dd; mkdir -p $OUT
DHTGPU_LIB=opendht_amd/ab/f4s64.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py -k "sub or cfg3_shard" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  for v in tree f4s128 f4s64; do
    lib=""; [ $v != tree ] && lib=opendht_amd/ab/$v.so
    for h in "" --handles; do
      echo -n "$v ${h:-indices} "; DHTGPU_LIB=$lib timeout -k 10 200 python tools/batch_probe.py --reps 30 --n 134217728 --q 131072 --inflight 2 $h 2>&1 | grep -E "ms/call|phases" | tr '\n' ' ' || exit 1; echo
    done
  done
done | tee $OUT/cfg3_f4grid.txt
echo all-ok
