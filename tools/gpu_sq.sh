# SQ counters (two passes, 8 / 6 SQ counters + GRBM) for K6 at cfg 2, KS at q = 1 and K2
set -o pipefail
OUT=gpurun_out/${1:-sq}; mkdir -p $OUT
export TMPDIR=/tmp
A=GRBM_GUI_ACTIVE,SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES
B=SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_LDS,SQ_INSTS_BRANCH
for w in cfg2 ks1 k2; do
  case $w in cfg2) cmd="python3 tools/batch_probe.py --reps 3";; ks1) cmd="python3 tools/small_probe.py --q 1 --reps 5";; k2) cmd="python3 tools/classify_probe.py --reps 3";; esac
  timeout -s KILL 120 rocprofv3 --pmc $(echo $A | tr ',' ' ') -d $OUT/${w}_a -o run --output-format csv -- $cmd > $OUT/${w}_a.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc $(echo $B | tr ',' ' ') -d $OUT/${w}_b -o run --output-format csv -- $cmd > $OUT/${w}_b.log 2>&1 || { tail -5 $OUT/${w}_a.log $OUT/${w}_b.log; exit 1; }
  python3 tools/pmc_sq_summary.py $OUT/${w}_a $OUT/${w}_b > $OUT/${w}_summary.txt
done
cat $OUT/*_summary.txt | grep -E "^k_|->"
