# K2 (cfg 4 classify, 10^8 ids) across library builds: name=path pairs ("tree" = in-tree),
# classify_probe.py three times each, rotated.   usage: bash tools/experiments/gpu_k2_libs.sh <tag> name=path ...
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in 1 2 3; do
  for nv in "$@"; do
    p=${nv#*=}; lib=""; [ "$p" != tree ] && lib="DHTGPU_LIB=$p"
    echo -n "${nv%%=*} "; timeout -k 10 120 env $lib X=1 python tools/classify_probe.py --reps 10 2>/dev/null | grep K2 || exit 1
  done
done | tee $OUT/k2.txt
