set -o pipefail
OUT=gpurun_out/${1:-r06s}; mkdir -p $OUT
timeout -k 10 300 env DHTGPU_DBG=256 python tools/batch_probe.py --reps 2 --cfg3 prefix > $OUT/stamps_prefix.log 2>&1 || { tail -5 $OUT/stamps_prefix.log; exit 1; }
grep -E "F2 " $OUT/stamps_prefix.log | tail -11
