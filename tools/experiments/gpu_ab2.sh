# A/B of DHTGPU_DBG values on the cfg-2 bench (same box): $@ = dbg values (0 = production build path)
set -o pipefail
O=gpurun_out/ab2; rm -rf $O; mkdir -p $O
for i in 1 2; do for v in "$@"; do
  DHTGPU_DBG=$v timeout -k 10 120 python bench.py --no-cpu --no-extra --no-scan > $O/d${v}_$i.log 2>&1 || exit 1
done; done
for f in $O/*.log; do echo $f $(tail -1 $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['ms_per_step']*1e3,2),'us/step lat',round(d['latency_ms_per_batch']*1e3,1),{k:round(v*1e3,1) for k,v in d['roofline']['kernels_ms'].items()})"); done
