# F2 direct placement (DHT_F2_DIRECT=1 build): K6 parity under that build, then the cfg-2 A/B
set -o pipefail
OUT=gpurun_out/r04f2d; mkdir -p $OUT
DHTGPU_LIB=opendht_amd/ab/f2_direct.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_kat.py -k "topk or k6 or batch or subpart" > $OUT/tests_direct.log 2>&1 || { tail -30 $OUT/tests_direct.log; exit 1; }
tail -1 $OUT/tests_direct.log
bash tools/experiments/gpu_ab_libs.sh r04f2d none tree=tree direct=opendht_amd/ab/f2_direct.so
