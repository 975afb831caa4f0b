# GPU parity suite, then an A/B of the cfg-2 bench step: HEAD (and HEAD with DHTGPU_DBG=$ABDBG) vs
# the worktree in old_r02 (same box)
set -o pipefail
O=gpurun_out/ab; rm -rf $O; mkdir -p $O
if [ "$1" != "notest" ]; then
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
fi
for i in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu --no-extra --no-scan > $O/head$i.log 2>&1 || exit 1
  if [ -n "$ABDBG" ]; then DHTGPU_DBG=$ABDBG timeout -k 10 120 python bench.py --no-cpu --no-extra --no-scan > $O/dbg$i.log 2>&1 || exit 1; fi
  (cd old_r02 && timeout -k 10 120 python bench.py --no-cpu --no-extra --no-scan) > $O/old$i.log 2>&1 || exit 1
done
for f in $O/*.log; do case $f in *gpu_tests*) continue;; esac; echo $f $(tail -1 $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['ms_per_step']*1e3,2),'us/step lat',round(d['latency_ms_per_batch']*1e3,1),{k:round(v*1e3,1) for k,v in d['roofline']['kernels_ms'].items()}, d['verified_exact'] if 'verified_exact' in d else '')"); done
