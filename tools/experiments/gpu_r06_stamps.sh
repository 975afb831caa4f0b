# F2 phase stamps (DHTGPU_DBG=256: per-workgroup s_memrealtime phases, printed per call) of the cfg-3
# per-rank probes, for the in-tree build and a baseline build.   usage: bash tools/experiments/gpu_r06_stamps.sh tag base.so
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
for r in ${ROUTES:-prefix broadcast}; do
  timeout -k 10 300 env DHTGPU_DBG=256 python tools/batch_probe.py --reps 2 --cfg3 $r > $OUT/stamps_${r}_tree.log 2>&1 || { tail -5 $OUT/stamps_${r}_tree.log; exit 1; }
  timeout -k 10 300 env DHTGPU_DBG=256 DHTGPU_LIB=$2 python tools/batch_probe.py --reps 2 --cfg3 $r > $OUT/stamps_${r}_base.log 2>&1 || { tail -5 $OUT/stamps_${r}_base.log; exit 1; }
  for b in tree base; do echo "== $r $b"; grep -E "F2 " $OUT/stamps_${r}_$b.log | tail -7; done
done
