# Kernel-trace of the K6 probe: per-kernel average durations (rocprofv3 --stats) and the gaps
# between consecutive dispatches.  usage: bash tools/gpu_kt_probe.sh <out-tag> [probe args...]
set -o pipefail
OUT=gpurun_out/${1:-ktp}; shift; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 tools/batch_probe.py --reps 50 "$@" > $OUT/kt.log 2>&1 &&
python3 tools/kt_gaps.py $OUT/kt
