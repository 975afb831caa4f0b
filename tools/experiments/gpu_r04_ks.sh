# KS A/B: the small-batch tests on the in-tree build, then S1/S2 per q for builds name=path (rotated x3),
# on the cfg-2 set and the 2^26 set.   usage: bash tools/experiments/gpu_r04_ks.sh tag name=path ...
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "small or kat" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2 3; do
  for nv in "$@"; do
    p=${nv#*=}; lib=""; [ "$p" != tree ] && lib="DHTGPU_LIB=$p"
    for n in 16777216 67108864; do
      echo -n "${nv%%=*} n=$n "; timeout -k 10 120 env $lib X=1 python tools/small_probe.py --q 1 8 32 64 --reps 10 --n $n 2>/dev/null | tr '\n' ' ' || exit 1; echo
    done
  done
done | tee $OUT/ks.txt
