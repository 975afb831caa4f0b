# KS S2 stamps (measurement build with device printf): c, targets per prefix, load+sync and answer times
set -o pipefail
OUT=gpurun_out/r04s2p; mkdir -p $OUT
DHTGPU_LIB=opendht_amd/ab/s2m4.so timeout -k 10 120 python tools/small_probe.py --q 1 2 8 --reps 3 > $OUT/s2p.txt 2>&1 || { tail -20 $OUT/s2p.txt; exit 1; }
grep -c S2 $OUT/s2p.txt
