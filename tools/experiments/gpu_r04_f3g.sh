# F3 group size for 65..128 targets per chunk: G = 2 (tree) against G = 1 (g1.so); stamps of the g1 build, then the cfg-2 A/B
set -o pipefail
OUT=gpurun_out/r04f3g; mkdir -p $OUT
DHTGPU_LIB=opendht_amd/ab/g1.so DHTGPU_DBG=256 timeout -k 10 120 python3 tools/batch_probe.py --reps 1 > $OUT/stamps_g1.log 2>&1 || { tail $OUT/stamps_g1.log; exit 1; }
DHTGPU_LIB=opendht_amd/ab/g1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "k6 or batch or topk" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/experiments/gpu_ab_libs.sh r04f3g none tree=tree g1=opendht_amd/ab/g1.so
