set -o pipefail
OUT=gpurun_out/r01l; mkdir -p $OUT
export TMPDIR=/tmp
for g in 1 2 8; do
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt$g -o run --output-format csv -- python3 bench.py --simulate-world $g --simulate-rank 0 --no-scan --no-cpu --steps 10 --warmup 2 > $OUT/kt$g.log 2>&1 || exit 1; echo kt$g-ok; done
