# GPU suite + two default cfg-2 bench runs (the hint-sized F4 grid)
set -o pipefail
O=gpurun_out/fbh; rm -rf $O; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for i in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu --no-extra --no-scan > $O/b_$i.log 2>&1 || exit 1
  tail -1 $O/b_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('step', d['ms_per_step'], 'lat', d['latency_ms_per_batch'], 'f4', d['roofline']['kernels_ms']['k_f4_fallback'])"
done
