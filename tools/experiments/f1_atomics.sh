# F1 anatomy: what bounds k_f1_targets?  DHTGPU_DBG bits 24..26 (results wrong, F1 + F2 only):
# 1 plain bitmap store instead of the memory-side OR, 2 no returning slot atomic, 4 load only.
set -o pipefail
OUT=gpurun_out/f1at; mkdir -p $OUT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "small_batch_prefix_shard" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for d in 0 16777216 33554432 50331648 67108864; do
  for cfg in "--n 16777216 --q 65536" "--n 134217728 --q 131072"; do
    timeout -k 10 200 env DHTGPU_DBG=$d python tools/batch_probe.py --reps 10 $cfg > $OUT/p.log 2>&1 || { tail $OUT/p.log; exit 1; }
    echo "dbg $((d >> 24)) $cfg: $(grep phases $OUT/p.log)"
  done
done | tee $OUT/f1.txt
