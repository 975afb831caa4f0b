# Pipelined K6 timeline at HEAD: a rocprofv3 kernel trace of the cfg-2 bench (3 batches in
# flight), its steady-state window and overlap summary, and the F2 / F3 phase stamps of a
# serial call (DHTGPU_DBG=256).   usage: bash tools/gpu_timeline.sh <out-tag> [VAR=value ...]
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 env "${@:-A=1}" rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --steps 400 --warmup 50 --no-cpu --no-extra --no-scan > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 tools/experiments/kt_timeline.py $OUT/kt 300 6 > $OUT/timeline.txt 2>&1
python3 tools/experiments/kt_overlap.py $OUT/kt > $OUT/overlap.txt 2>&1
head -40 $OUT/timeline.txt; head -30 $OUT/overlap.txt
timeout -k 10 120 env DHTGPU_DBG=256 "${@:-A=1}" python3 tools/batch_probe.py --reps 3 > $OUT/stamps.log 2>&1 || { tail -20 $OUT/stamps.log; exit 1; }
tail -40 $OUT/stamps.log
echo done
