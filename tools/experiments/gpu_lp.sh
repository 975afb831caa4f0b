set -o pipefail
O=gpurun_out/lp; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for i in 1 2; do for v in 1 0; do
  DHTGPU_F4LP=$v timeout -k 10 120 python bench.py --no-cpu --no-extra --no-scan > $O/lp${v}_$i.log 2>&1 || exit 1
done; (cd old_r02 && timeout -k 10 120 python bench.py --no-cpu --no-extra --no-scan) > $O/old_$i.log 2>&1 || exit 1; done
for f in $O/*_*.log; do echo $f $(tail -1 $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['ms_per_step']*1e3,2),'us/step lat',round(d['latency_ms_per_batch']*1e3,1),{k:round(v*1e3,1) for k,v in d['roofline']['kernels_ms'].items()})"); done
