set -o pipefail
OUT=gpurun_out/big1; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1; tail -1 $OUT/gpu_tests.log
DHTGPU_LIB=opendht_amd/ab/prev.so timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread -m gpu tests/test_gpu_scale.py::test_subpartitions_k_sequence_fresh_context > $OUT/descfix_prev.log 2>&1; tail -1 $OUT/descfix_prev.log
grep -q "passed" $OUT/gpu_tests.log && ! grep -q "failed" $OUT/gpu_tests.log || exit 1
bash tools/experiments/gpu_ab_libs.sh big1ab none prev=opendht_amd/ab/prev.so tree=tree || exit 1
bash tools/experiments/gpu_k2_libs.sh k2a tree=tree k81=opendht_amd/ab/k2_8_1.so k80=opendht_amd/ab/k2_8_0.so k21=opendht_amd/ab/k2_2_1.so k160=opendht_amd/ab/k2_16_0.so
