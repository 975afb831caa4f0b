# pipelined segmented F2 flush: GPU parity suite (the cfg-3 shard tests take the segmented path),
# cfg-3 shard timing, stamps, and the forced-segment cfg-2 A/B
set -o pipefail
O=gpurun_out/seg; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
DHTGPU_F2SEG=32768 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "2p24 or full_batch or cluster or batch" > $O/gpu_tests_seg.log 2>&1 || { tail -30 $O/gpu_tests_seg.log; exit 1; }
tail -1 $O/gpu_tests_seg.log
timeout -k 10 120 python tools/batch_probe.py --n 134217728 --q 131072 --reps 20 > $O/cfg3.log 2>&1 || exit 1
grep "ms/call\|phases" $O/cfg3.log
DHTGPU_DBG=256 timeout -k 10 120 python tools/batch_probe.py --n 134217728 --q 131072 --reps 1 > $O/stamps_cfg3.log 2>&1 || exit 1
sed -n "/first call/,/F2 end/p" $O/stamps_cfg3.log
DHTGPU_F2SEG=32768 timeout -k 10 120 python bench.py --no-cpu --no-extra --no-scan > $O/bench_seg.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --no-cpu --no-extra --no-scan > $O/bench.log 2>&1 || exit 1
for f in $O/bench*.log; do echo $f $(tail -1 $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['ms_per_step']*1e3,2),'us/step',{k:round(v*1e3,1) for k,v in d['roofline']['kernels_ms'].items()})"); done
