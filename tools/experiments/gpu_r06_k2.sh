# K2 (cfg 4) with several builds, alternating.  usage: bash ... tag lib...
set -o pipefail
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for i in 1 2; do
for b in "$@"; do
  e=""; [ $b != tree ] && e="DHTGPU_LIB=opendht_amd/ab/$b.so"
  timeout -k 10 200 env $e X=1 python tools/classify_probe.py --reps 20 > $OUT/k2_${b}_$i.log 2>&1 || { tail -5 $OUT/k2_${b}_$i.log; exit 1; }
  echo "k2 $b $i: $(tail -2 $OUT/k2_${b}_$i.log | tr '\n' ' ')"
done
done
