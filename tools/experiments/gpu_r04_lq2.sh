# F3 sorting two bits below the mark level (Lq = Lm + 2): parity, stamps, cfg-2 A/B, cfg-3 shard
set -o pipefail
OUT=gpurun_out/r04lq2; mkdir -p $OUT
for v in lq2; do
  DHTGPU_LIB=opendht_amd/ab/$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_scale.py -k "k6 or batch or topk or subpart or shard or cfg3" > $OUT/tests_$v.log 2>&1 || { tail -30 $OUT/tests_$v.log; exit 1; }
  tail -1 $OUT/tests_$v.log
  DHTGPU_LIB=opendht_amd/ab/$v.so DHTGPU_DBG=256 timeout -k 10 120 python3 tools/batch_probe.py --reps 1 > $OUT/stamps_$v.log 2>&1 || exit 1
done
bash tools/experiments/gpu_ab_libs.sh r04lq2 none tree=tree lq2=opendht_amd/ab/lq2.so
