set -o pipefail
O=gpurun_out/pipe; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "2p24 or full_batch or cluster" > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
DHTGPU_DBG=256 timeout -k 10 120 python3 tools/batch_probe.py --reps 1 > $O/stamps.log 2>&1 || exit 1
sed -n '/first call/,$p' $O/stamps.log | head -16
ABDBG=4194304 bash tools/gpu_ab.sh notest
