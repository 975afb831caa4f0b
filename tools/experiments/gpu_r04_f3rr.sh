# F3 groups dealt round-robin over the waves for every G: stamps, parity, cfg-2 A/B against HEAD
set -o pipefail
OUT=gpurun_out/r04f3rr; mkdir -p $OUT
DHTGPU_DBG=256 timeout -k 10 120 python3 tools/batch_probe.py --reps 1 > $OUT/stamps_cfg2.log 2>&1 || { tail $OUT/stamps_cfg2.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_fuzz.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/experiments/gpu_ab_libs.sh r04f3rr none tree=tree prev=opendht_amd/ab/prev.so
