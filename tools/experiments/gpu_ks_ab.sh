# KS S1/S2 per q for the in-tree build and variant libraries (opendht_amd/ab/<name>.so), twice.
# usage: bash tools/experiments/gpu_ks_ab.sh <out-tag> <variant>...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in 1 2; do
  echo "== head" && timeout -k 10 120 python tools/small_probe.py --q 1 8 32 64 --reps 10 2>&1 | grep S1 || exit 1
  for v in "$@"; do
    echo "== $v" && DHTGPU_LIB=opendht_amd/ab/$v.so timeout -k 10 120 python tools/small_probe.py --q 1 8 32 64 --reps 10 2>&1 | grep S1 || exit 1
  done
done | tee $OUT/ks_ab.txt
echo all-ok
