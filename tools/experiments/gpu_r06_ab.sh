# Round-6 A/B of libdhtgpu builds on the cfg-3 per-rank shapes (bench.py's cfg3_<route>_rank inputs
# via tools/batch_probe.py --cfg3) and the cfg-2 headline, after the GPU tests named by SEL.
# usage: bash tools/experiments/gpu_r06_ab.sh <out-tag> "<pytest -k expr | none>" name=path [name=path ...]
set -o pipefail
TAG=$1; SEL=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ "$SEL" != none ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu -k "$SEL" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
for i in 1 2; do
  for nv in "$@"; do
    p=${nv#*=}; lib=""; [ "$p" != tree ] && lib="DHTGPU_LIB=$p"
    for r in ${ROUTES:-broadcast prefix}; do
      timeout -k 10 300 env $lib X=1 python tools/batch_probe.py --reps 20 --inflight 2 --cfg3 $r > $OUT/${r}_${nv%%=*}_$i.log 2>&1 || { tail -5 $OUT/${r}_${nv%%=*}_$i.log; exit 1; }
      echo "$r ${nv%%=*} $i: $(grep -h 'ms/call' $OUT/${r}_${nv%%=*}_$i.log) | $(grep -h phases $OUT/${r}_${nv%%=*}_$i.log)"
    done
    if [ -n "$CFG2" ]; then
      timeout -k 10 200 env $lib X=1 python bench.py --no-cpu --no-extra --no-scan --steps 1000 --warmup 100 --verify 0 2>/dev/null |
        python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg2 ${nv%%=*}', round(d['ms_per_step']*1e3,2), 'us/step lat', round(d.get('latency_ms_per_batch',0)*1e3,1), 'F', [round(x*1e3,1) for x in d['roofline']['kernels_ms'].values()])" || exit 1
    fi
  done
done | tee $OUT/ab.txt
echo done
