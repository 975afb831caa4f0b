# F2 stage writes without per-word branches (per-lane trash slots) and the four bitmap reads issued together: parity, stamps, cfg-2 A/B, shard
set -o pipefail
OUT=gpurun_out/r04f2bf; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_fuzz.py tests/test_gpu_scale.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
DHTGPU_DBG=256 timeout -k 10 120 python3 tools/batch_probe.py --reps 1 > $OUT/stamps.log 2>&1 || exit 1
bash tools/experiments/gpu_ab_libs.sh r04f2bf none tree=tree prev=opendht_amd/ab/prev.so
