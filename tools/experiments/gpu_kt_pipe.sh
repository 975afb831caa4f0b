# Kernel trace of the pipelined bench (2 batches in flight): overlap between K6 kernels.
# usage: bash tools/gpu_kt_pipe.sh <out-tag> [bench args...]
set -o pipefail
OUT=gpurun_out/${1:-ktpipe}; shift; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT/kt -o run --output-format csv -- python3 bench.py --no-scan --no-cpu --steps 100 "$@" > $OUT/bench.log 2>&1 &&
python3 tools/kt_overlap.py $OUT/kt
