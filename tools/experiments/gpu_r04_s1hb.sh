# KS S1 filter width: 2^16 (tree) against 2^17 / 2^18 bitmap bits; small-batch parity under hb18, then S1/S2 medians
set -o pipefail
OUT=gpurun_out/r04s1hb; mkdir -p $OUT
DHTGPU_LIB=opendht_amd/ab/hb18.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_kat.py -k "small or ks or batch" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do for v in tree hb17 hb18; do
  lib=""; [ $v != tree ] && lib="DHTGPU_LIB=opendht_amd/ab/$v.so"
  echo "== $v"; timeout -k 10 120 env $lib X=1 python tools/small_probe.py --q 2 8 32 64 --reps 20 2>/dev/null || exit 1
done; done | tee $OUT/s1.txt
# F3 with 512-thread workgroups (G = 4 up to 128 targets per chunk): parity, stamps, cfg-2 A/B
DHTGPU_LIB=opendht_amd/ab/f3t512.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_kat.py -k "k6 or batch or topk or subpart or shard or cfg3 or kat" > $OUT/tests_f3t512.log 2>&1 || { tail -30 $OUT/tests_f3t512.log; exit 1; }
tail -1 $OUT/tests_f3t512.log
DHTGPU_LIB=opendht_amd/ab/f3t512.so DHTGPU_DBG=256 timeout -k 10 120 python3 tools/batch_probe.py --reps 1 > $OUT/stamps_f3t512.log 2>&1 || exit 1
bash tools/experiments/gpu_ab_libs.sh r04s1hb none tree=tree f3t512=opendht_amd/ab/f3t512.so
