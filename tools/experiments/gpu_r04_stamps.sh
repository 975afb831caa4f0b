# per-block phase stamps of F2 / F3 at HEAD (DHTGPU_DBG=256, one call), cfg 2 and the cfg-3 shard
set -o pipefail
OUT=gpurun_out/r04stamps; mkdir -p $OUT
DHTGPU_DBG=256 timeout -k 10 120 python3 tools/batch_probe.py --reps 1 > $OUT/cfg2.log 2>&1 &&
DHTGPU_DBG=256 timeout -k 10 120 python3 tools/batch_probe.py --reps 1 --n 134217728 --q 131072 > $OUT/cfg3.log 2>&1 || exit 1
echo ok
