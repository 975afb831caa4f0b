# Owner-form F1 (DHT_F1_OWNER=1 builds, 16 / 64 owners per sub-partition): K6 parity under each build, then the cfg-2 A/B and the cfg-3 shard
set -o pipefail
OUT=gpurun_out/r04f1o2; mkdir -p $OUT
for v in own16 own64; do
  DHTGPU_LIB=opendht_amd/ab/f1_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_scale.py -k "topk or k6 or batch or subpart or shard or cfg3" > $OUT/tests_$v.log 2>&1 || { tail -30 $OUT/tests_$v.log; exit 1; }
  tail -1 $OUT/tests_$v.log
done
bash tools/experiments/gpu_ab_libs.sh r04f1o2 none tree=tree own16=opendht_amd/ab/f1_own16.so own64=opendht_amd/ab/f1_own64.so
