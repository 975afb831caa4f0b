# cfg-3 shard F2 decomposition at HEAD: full F2, F2 with no flush (DHTGPU_DBG 128), the bare
# stream of F2's shape (64: loads and an XOR only, no filter, no stage)
set -o pipefail
OUT=gpurun_out/r04abl; mkdir -p $OUT
for dbg in 0 128 64 0 128 64; do
  echo "dbg $dbg" >> $OUT/abl.txt
  DHTGPU_DBG=$dbg timeout -k 10 120 python tools/batch_probe.py --reps 30 --n 134217728 --q 131072 >> $OUT/abl.txt 2>&1 || exit 1
done
echo ok
