# K6 iteration loop on the GPU box: probe timings (production + streaming ablation), then the
# K6-relevant GPU parity tests.  usage: bash tools/gpu_probe.sh <out-tag>
set -o pipefail
OUT=gpurun_out/${1:-probe}; mkdir -p $OUT
for d in 0 64; do DHTGPU_DBG=$d timeout -k 10 120 python tools/batch_probe.py --reps 20 > $OUT/probe$d.log 2>&1 || exit 1; echo "dbg=$d"; tail -2 $OUT/probe$d.log; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "batch or topk_sizes or clustered or adversarial or 2p24 or duplicates or prefix or weak" > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; exit $rc
