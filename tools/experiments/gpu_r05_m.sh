# Round 5, pass m: where F3's deferred-tie cost goes (phase stamps, DHTGPU_DBG=256): in-tree, ties
# never deferred, ties detected but not deferred, ties deferred without the candidate copy.
set -o pipefail
OUT=gpurun_out/r05m; mkdir -p $OUT
for v in tree noties tiedet tienocopy; do
  lib=""; [ $v != tree ] && lib=opendht_amd/ab/$v.so
  DHTGPU_DBG=256 DHTGPU_LIB=$lib timeout -k 10 120 python tools/batch_probe.py --reps 5 > $OUT/$v.log 2>&1 || { tail $OUT/$v.log; exit 1; }
  echo "== $v"; grep -E "phase A|phases ms" $OUT/$v.log; grep "slow block" $OUT/$v.log | head -3
done
