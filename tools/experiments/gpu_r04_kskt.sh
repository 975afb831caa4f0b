# KS kernel trace: S1 / S2 durations and the gap between them at q = 1 and q = 8
set -o pipefail
OUT=gpurun_out/r04kskt; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 tools/small_probe.py --q 1 8 --reps 20 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
tail -5 $OUT/kt.log
