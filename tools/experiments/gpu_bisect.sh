# cfg-2 bench step of several worktree builds on one box (bisection)
set -o pipefail
O=gpurun_out/bis; rm -rf $O; mkdir -p $O
for i in 1 2; do for d in . old_r02 wt_0f1fcf9 wt_e8a3322 wt_16c9cf3; do
  (cd $d && timeout -k 10 120 python bench.py --no-cpu --no-extra --no-scan) > $O/$(basename $d)_$i.log 2>&1 || exit 1
done; done
for f in $O/*.log; do echo $f $(tail -1 $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['ms_per_step']*1e3,2),'us/step',{k:round(v*1e3,1) for k,v in d['roofline']['kernels_ms'].items()})"); done
