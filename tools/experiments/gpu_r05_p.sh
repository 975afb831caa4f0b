# Round 5, pass o: w0 ties answered inline by the detecting wave (opendht_amd/ab/tieinline2.so):
# K6 parity with that build, then the cfg-2 A/B and its F3 phase stamps.
set -o pipefail
OUT=gpurun_out/r05p; mkdir -p $OUT
V=opendht_amd/ab/tieinline2.so
DHTGPU_LIB=$V timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_kat.py -k "batch or fuzz or record or kat or cfg2 or clustered or fallback or w0" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
DHTGPU_DBG=256 DHTGPU_LIB=$V timeout -k 10 120 python tools/batch_probe.py --reps 5 > $OUT/stamps.log 2>&1 || { tail $OUT/stamps.log; exit 1; }
grep -E "phase [0-9]|phase A|phases ms" $OUT/stamps.log | tail -12
bash tools/experiments/gpu_ab_pair.sh r05p $V
