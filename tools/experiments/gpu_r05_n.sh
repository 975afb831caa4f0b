# Round 5, pass n: every w0 tie answered inside F3 (phase B wave path) instead of deferred to F4,
# against the in-tree build: phase stamps (DHTGPU_DBG=256) and the cfg-2 benches.
set -o pipefail
OUT=gpurun_out/r05n; mkdir -p $OUT
for v in tree tieinplace; do
  lib=""; [ $v != tree ] && lib=opendht_amd/ab/$v.so
  DHTGPU_DBG=256 DHTGPU_LIB=$lib timeout -k 10 120 python tools/batch_probe.py --reps 5 > $OUT/$v.log 2>&1 || { tail $OUT/$v.log; exit 1; }
  echo "== $v"; grep -E "phase [0-9]|phase A|phases ms" $OUT/$v.log; grep "slow block" $OUT/$v.log | head -3 | cut -c1-220
done
bash tools/experiments/gpu_ab_pair.sh r05n opendht_amd/ab/tieinplace.so
