# K2 register path: classify parity tests, then A/B against the cell-table build (4 and 8 workgroups per CU)
set -o pipefail
OUT=gpurun_out/r04x7; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k classify tests/test_gpu_kat.py tests/test_gpu_scale.py::test_cfg4_classify_1e8 > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/experiments/gpu_k2_libs.sh r04x7 tree=tree v3p8=opendht_amd/ab/k2_v3p8.so w5=opendht_amd/ab/k2_w5.so w6=opendht_amd/ab/k2_w6.so w8=opendht_amd/ab/k2_w8.so > /dev/null || exit 1
echo ok
