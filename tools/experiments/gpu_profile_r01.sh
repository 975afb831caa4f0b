set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 60 ./tools/valu_peak > gpurun_out/valu_peak.log 2>&1 && cat gpurun_out/valu_peak.log &&
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/bench2.log 2>&1 && tail -1 gpurun_out/bench2.log &&
(rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true) &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_kt.log 2>&1 && echo kt-ok &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d gpurun_out/prof/pmc1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_pmc1.log 2>&1 && echo pmc1-ok &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH -d gpurun_out/prof/pmc2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_pmc2.log 2>&1 && echo pmc2-ok
