# Anatomy of the cfg-2 pipelined period: the same 1,000-step bench (3 batches in flight) with
#   A   opendht_amd/ab/prev.so (an earlier commit)
#   B   the in-tree build
#   F12 the in-tree build with DHTGPU_DBG=1: F1 + F2 only (measurement)
# then the cfg-3 shard probe on A and B.   usage: bash tools/experiments/gpu_anatomy.sh <tag> [tests]
set -o pipefail
TAG=$1; SEL=${2:-none}
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ "$SEL" != none ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $SEL > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
b() { local tag=$1; shift; timeout -k 10 200 env "$@" python bench.py --no-cpu --no-extra --no-scan --steps $S --warmup $W --verify 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag S=$S', round(d['ms_per_step']*1e3,2), 'us/step lat', round(d.get('latency_ms_per_batch',0)*1e3,1), 'F', [round(x*1e3,1) for x in d['roofline']['kernels_ms'].values()])"; }
for i in 1 2; do
  S=1000 W=100 b A DHTGPU_LIB=opendht_amd/ab/prev.so && S=1000 W=100 b B X=1 &&
  S=1000 W=100 b F12 DHTGPU_DBG=1 &&
  S=20 W=5 b A DHTGPU_LIB=opendht_amd/ab/prev.so && S=20 W=5 b B X=1 || exit 1
done | tee $OUT/ab.txt
timeout -k 10 200 python tools/batch_probe.py --reps 10 --n 134217728 --q 131072 > $OUT/cfg3_B.log 2>&1 && timeout -k 10 200 env DHTGPU_LIB=opendht_amd/ab/prev.so python tools/batch_probe.py --reps 10 --n 134217728 --q 131072 > $OUT/cfg3_A.log 2>&1 || exit 1
grep -H "phases\|ms/call" $OUT/cfg3_*.log
echo done
