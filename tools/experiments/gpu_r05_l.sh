set -o pipefail
OUT=gpurun_out/r05l; mkdir -p $OUT
DHTGPU_DBG=256 timeout -k 10 120 python tools/batch_probe.py --reps 5 > $OUT/tree.log 2>&1 || { tail $OUT/tree.log; exit 1; }
DHTGPU_DBG=256 DHTGPU_LIB=opendht_amd/ab/noties.so timeout -k 10 120 python tools/batch_probe.py --reps 5 > $OUT/noties.log 2>&1 || { tail $OUT/noties.log; exit 1; }
grep -E "phase|ms/call|F2 " $OUT/tree.log | tail -30
echo ====
grep -E "phase|ms/call|F2 " $OUT/noties.log | tail -30
