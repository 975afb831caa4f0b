set -o pipefail
O=gpurun_out/fb; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for n in 268435456 1000000000; do timeout -k 10 200 python tools/batch_probe.py --n $n --q 1048576 --reps 3 2>&1 | grep "ms/call\|phases"; done
