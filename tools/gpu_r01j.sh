set -o pipefail
OUT=gpurun_out/r01j; mkdir -p $OUT
export TMPDIR=/tmp
A="--simulate-world 8 --simulate-rank 0 --no-scan --no-cpu --steps 3 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_WAIT_INST_ANY -d $OUT/pmc1 -o run --output-format csv -- python3 bench.py $A > $OUT/pmc1.log 2>&1 && echo pmc1-ok &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM -d $OUT/pmc2 -o run --output-format csv -- python3 bench.py $A > $OUT/pmc2.log 2>&1 && echo pmc2-ok &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py $A > $OUT/kt.log 2>&1 && echo kt-ok
