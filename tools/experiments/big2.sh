set -o pipefail
OUT=gpurun_out/big2; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1; tail -1 $OUT/gpu_tests.log
grep -q "passed" $OUT/gpu_tests.log && ! grep -q "failed" $OUT/gpu_tests.log || exit 1
bash tools/experiments/gpu_ab_libs.sh big2ab none prev=opendht_amd/ab/prev.so tree=tree || exit 1
timeout -k 10 120 python tools/batch_probe.py --reps 10 > $OUT/probe.log 2>&1; grep phases $OUT/probe.log
bash tools/experiments/gpu_k2_libs.sh k2b tree=tree k16_0=opendht_amd/ab/k2_16_0.so k32_0=opendht_amd/ab/k2_32_0.so k64_0=opendht_amd/ab/k2_64_0.so k16_1=opendht_amd/ab/k2_16_1.so k32_1=opendht_amd/ab/k2_32_1.so
