# Per-kernel SQ counters of the K6 probe (one pass per counter group), summarised per kernel.
# usage: bash tools/gpu_pmc_probe.sh <out-tag> [probe args...]
set -o pipefail
OUT=gpurun_out/${1:-pmcp}; shift; mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d $OUT/p1 -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 "$@" > $OUT/p1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $OUT/p2 -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 "$@" > $OUT/p2.log 2>&1 &&
python3 tools/pmc_kernels.py $OUT p1 p2 > $OUT/summary.txt && cat $OUT/summary.txt
