# F3 ablations (DHTGPU_DBG bits, see batch.hip): 32 = stop after target tables, 16 = stop
# after the survivor sort.
set -o pipefail
OUT=gpurun_out/${1:-ablate}; mkdir -p $OUT
for d in ${DBGS:-0 32 16}; do DHTGPU_DBG=$d timeout -k 10 120 python tools/batch_probe.py --reps 20 > $OUT/probe$d.log 2>&1 || exit 1; echo "dbg=$d"; tail -2 $OUT/probe$d.log; done
