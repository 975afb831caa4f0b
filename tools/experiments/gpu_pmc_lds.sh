# LDS counters per kernel on the K6 probe (one pass).  usage: bash tools/gpu_pmc_lds.sh <out-tag>
set -o pipefail
OUT=gpurun_out/${1:-pmcl}; mkdir -p $OUT
export TMPDIR=/tmp
(rocprofv3 -L > $OUT/counters.txt 2>&1 || true)
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES -d $OUT/p1 -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 > $OUT/p1.log 2>&1 &&
python3 tools/pmc_kernels.py $OUT p1 | grep -A9 -E "k_f2_filter|k_f3_answer"
