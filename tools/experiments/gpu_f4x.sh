set -o pipefail
O=gpurun_out/f4x; rm -rf $O; mkdir -p $O
for i in 1 2; do for g in 0 999; do
  DHTGPU_F4GRID=$g timeout -k 10 120 python bench.py --no-cpu --no-extra --no-scan --verify 0 > $O/g${g}_$i.log 2>&1 || exit 1
done; done
for f in $O/*.log; do echo $f $(tail -1 $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['ms_per_step']*1e3,2),'us/step',{k:round(v*1e3,1) for k,v in d['roofline']['kernels_ms'].items()})"); done
