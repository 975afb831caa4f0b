# cfg-3 shard A/B: F2's segment flushes staggered per workgroup (default) against all at one id
# offset (DHTGPU_DBG bit 24), one and two calls in flight; then the F2 phase stamps of each
set -o pipefail
OUT=gpurun_out/r04stag; mkdir -p $OUT
for rep in 1 2; do
  for dbg in 0 16777216; do
    for inf in 1 2; do
      echo "dbg $dbg inflight $inf" >> $OUT/ab.txt
      DHTGPU_DBG=$dbg timeout -k 10 120 python tools/batch_probe.py --reps 30 --n 134217728 --q 131072 --inflight $inf >> $OUT/ab.txt 2>&1 || exit 1
    done
  done
done
DHTGPU_DBG=256 timeout -k 10 120 python3 tools/batch_probe.py --reps 1 --n 134217728 --q 131072 > $OUT/stamps_new.log 2>&1 &&
DHTGPU_DBG=$((256 + 16777216)) timeout -k 10 120 python3 tools/batch_probe.py --reps 1 --n 134217728 --q 131072 > $OUT/stamps_old.log 2>&1 || exit 1
echo ok
