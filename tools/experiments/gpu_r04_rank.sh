# branch-free wave rank (wave_rank64): GPU parity (K6 / KS / KAT incl. duplicate ids and w0 ties), then cfg-2 A/B and KS
set -o pipefail
OUT=gpurun_out/r04rank; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_fuzz.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in tree prev tree prev; do
  lib=""; [ $v != tree ] && lib="DHTGPU_LIB=opendht_amd/ab/$v.so"
  echo "== $v"; timeout -k 10 120 env $lib X=1 python tools/small_probe.py --q 1 2 8 64 --reps 20 2>/dev/null || exit 1
done | tee $OUT/ks.txt
bash tools/experiments/gpu_ab_libs.sh r04rank none tree=tree prev=opendht_amd/ab/prev.so
