set -o pipefail
O=gpurun_out/stage; mkdir -p $O
P="python tools/batch_probe.py --n 134217728 --q 131072 --reps 1"
DHTGPU_DBG=64 timeout -k 10 60 $P > $O/s64.log 2>&1 && DHTGPU_DBG=4 timeout -k 10 60 $P > $O/s4.log 2>&1 && timeout -k 10 60 $P > $O/s0.log 2>&1
