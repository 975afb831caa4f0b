set -o pipefail
O=gpurun_out/split; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
DHTGPU_DBG=4194304 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "2p24 or full_batch or cluster or batch" > $O/gpu_tests_split.log 2>&1 || { tail -30 $O/gpu_tests_split.log; exit 1; }
tail -1 $O/gpu_tests_split.log
DHTGPU_DBG=4194560 timeout -k 10 120 python3 tools/batch_probe.py --reps 1 > $O/stamps_split.log 2>&1 || exit 1
sed -n '/first call/,$p' $O/stamps_split.log | head -8
bash tools/gpu_ab2.sh 0 8388608 12582912
(cd old_r02 && timeout -k 10 120 python bench.py --no-cpu --no-extra --no-scan) > $O/old.log 2>&1 && tail -1 $O/old.log | cut -c 1-300
