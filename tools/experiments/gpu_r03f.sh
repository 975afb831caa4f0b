# Round-3 pass F: counter evidence and the short-window study.
#  1. bench windows: the driver's 20 steps / 5 warmup (x3), 20 / 200, 200 / 5 (no CPU, no extra legs)
#  2. PMC HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes): KS at q = 1 / 8 / 32, K6 at cfg 2
#     (warm, Infinity-Cache evicted), the 2^27-id cfg-3 shard, K2 at 10^8 ids
#  3. rocprofv3 kernel traces: cfg-3 shard, K2, the bench's 20-step run
# usage: bash tools/experiments/gpu_r03f.sh [out-tag]
set -o pipefail
TAG=${1:-r03f}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
b() { timeout -k 10 200 python bench.py --no-cpu --no-extra --no-scan "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', round(d['ms_per_step']*1e3,2), 'us/step')"; }
{ b --steps 20 --warmup 5 && b --steps 20 --warmup 5 && b --steps 20 --warmup 5 && b --steps 20 --warmup 200 && b --steps 200 --warmup 5 && b --steps 1000 --warmup 100; } > $OUT/windows.txt 2>&1 || { cat $OUT/windows.txt; exit 1; }
cat $OUT/windows.txt
pmc() {  # name, workload key, probe command...
  local name=$1 key=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/${name}_fetch -o run --output-format csv -- "$@" > $OUT/${name}_fetch.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/${name}_write -o run --output-format csv -- "$@" > $OUT/${name}_write.log 2>&1 &&
  python3 tools/pmc_traffic.py $OUT/${name}_fetch $OUT/${name}_write $OUT/pmc_traffic.json "$key" > $OUT/${name}_pmc.txt
}
for q in 1 8 32; do
  pmc ks_q$q "ks:16777216x${q}x8" python3 tools/small_probe.py --q $q --reps 10 || exit 1
done
pmc cfg2 "cfg2:16777216x65536x8" python3 tools/batch_probe.py --reps 3 &&
pmc cfg2cold "cfg2:16777216x65536x8:cold" python3 tools/batch_probe.py --reps 3 --evict &&
pmc cfg3 "cfg3shard:134217728x131072x8" python3 tools/batch_probe.py --reps 3 --n 134217728 --q 131072 &&
pmc k2 "cfg4:100000000" python3 tools/classify_probe.py --reps 3 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_cfg3 -o run --output-format csv -- python3 tools/batch_probe.py --reps 20 --n 134217728 --q 131072 > $OUT/kt_cfg3.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_k2 -o run --output-format csv -- python3 tools/classify_probe.py --reps 20 > $OUT/kt_k2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_small -o run --output-format csv -- python3 tools/small_probe.py --q 1 8 32 64 --reps 20 > $OUT/kt_small.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_bench -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-extra --no-scan > $OUT/kt_bench.log 2>&1 || exit 1
echo all-ok
