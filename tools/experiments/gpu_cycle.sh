# usage: bash tools/gpu_cycle.sh TAG [bench args...]  -- tests, bench, kernel trace, 2 PMC passes
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench.py --steps 5 --warmup 1 "$@" > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu "$@" > $OUT/kt.log 2>&1 && echo kt-ok &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d $OUT/pmc1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu "$@" > $OUT/pmc1.log 2>&1 && echo pmc1-ok &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH -d $OUT/pmc2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu "$@" > $OUT/pmc2.log 2>&1 && echo pmc2-ok
