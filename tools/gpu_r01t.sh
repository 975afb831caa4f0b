set -o pipefail
OUT=gpurun_out/r01t; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | cut -c1-400 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --no-cpu --no-scan --steps 20 --warmup 2 > $OUT/kt.log 2>&1 && echo kt-ok &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 > $OUT/pmc_fetch.log 2>&1 && echo fetch-ok &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 tools/batch_probe.py --reps 3 > $OUT/pmc_write.log 2>&1 && echo write-ok &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM -d $OUT/pmc1 -o run --output-format csv -- python3 tools/batch_probe.py --reps 2 > $OUT/pmc1.log 2>&1 && echo pmc1-ok &&
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $OUT/pmc2 -o run --output-format csv -- python3 tools/batch_probe.py --reps 2 > $OUT/pmc2.log 2>&1 && echo pmc2-ok
