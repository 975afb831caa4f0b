# Compare several builds of libdhtgpu on the cfg-2 headline (1,000- and 20-step benches, rotated
# twice) and the cfg-3 shard probe.  Builds: name=path pairs ("tree" = the in-tree build).
# usage: bash tools/experiments/gpu_ab_libs.sh <out-tag> "<tests | none>" name=path [name=path ...]
set -o pipefail
TAG=$1; SEL=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ "$SEL" != none ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $SEL > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
run() {  # name path steps warmup
  local lib=""; [ "$2" != tree ] && lib="DHTGPU_LIB=$2"
  timeout -k 10 200 env $lib X=1 python bench.py --no-cpu --no-extra --no-scan --steps $3 --warmup $4 --verify 0 2>/dev/null |
    python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 S=$3', round(d['ms_per_step']*1e3,2), 'us/step lat', round(d.get('latency_ms_per_batch',0)*1e3,1), 'F', [round(x*1e3,1) for x in d['roofline']['kernels_ms'].values()])"
}
for i in 1 2; do
  for nv in "$@"; do run ${nv%%=*} ${nv#*=} 1000 100 || exit 1; done
  for nv in "$@"; do run ${nv%%=*} ${nv#*=} 20 5 || exit 1; done
done | tee $OUT/ab.txt
for nv in "$@"; do
  p=${nv#*=}; lib=""; [ "$p" != tree ] && lib="DHTGPU_LIB=$p"
  timeout -k 10 200 env $lib X=1 python tools/batch_probe.py --reps 10 --n 134217728 --q 131072 > $OUT/cfg3_${nv%%=*}.log 2>&1 || exit 1
done
grep -H "phases\|ms/call" $OUT/cfg3_*.log
echo done
