set -o pipefail
OUT=gpurun_out/r04x1; mkdir -p $OUT
for inf in 1 2 3 1 2; do
  echo "inflight $inf" >> $OUT/cfg3_inflight.txt
  timeout -k 10 120 python tools/batch_probe.py --reps 30 --n 134217728 --q 131072 --inflight $inf >> $OUT/cfg3_inflight.txt 2>&1 || exit 1
done
echo ok
