# F3 VALU/SALU/LDS instruction counts per ablation (DHTGPU_DBG bits), one SQ pass each.
set -o pipefail
OUT=gpurun_out/${1:-pmca}; mkdir -p $OUT
export TMPDIR=/tmp
for d in ${DBGS:-32 16 512 0}; do
  DHTGPU_DBG=$d timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d $OUT/d$d -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 > $OUT/d$d.log 2>&1 || exit 1
  echo "== dbg=$d"; python3 tools/pmc_kernels.py $OUT d$d | grep -A8 k_f3_answer | grep -E "VALU|SALU|INSTS_LDS|WAVE_CYCLES|WAIT_INST_ANY"
done
