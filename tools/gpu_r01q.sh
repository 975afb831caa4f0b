set -o pipefail
OUT=gpurun_out/r01q12; mkdir -p $OUT
for d in 64 65 1; do DHTGPU_DBG=$d timeout -k 10 120 python tools/batch_probe.py > $OUT/probe$d.log 2>&1 || exit 1; echo "dbg=$d"; tail -1 $OUT/probe$d.log; done
