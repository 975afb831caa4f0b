# KS S2 anatomy (measurement builds, results incomplete): m1 = prefix workgroups stop before answering, m2 = no scan roles, m3 = both
set -o pipefail
OUT=gpurun_out/r04s2; mkdir -p $OUT
for v in tree m1 m2 m3; do
  lib=""; [ $v != tree ] && lib="DHTGPU_LIB=opendht_amd/ab/s2$v.so"
  echo "== $v"; timeout -k 10 120 env $lib X=1 python tools/small_probe.py --q 1 2 4 8 64 --reps 20 2>/dev/null || exit 1
done | tee $OUT/s2.txt
