# Round-3 pass B: the whole GPU parity suite, KS timings, and the counter evidence:
# PMC HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes) for KS at q = 1 / 8 / 32, K6 at
# cfg 2 (warm and Infinity-Cache-evicted) and the 2^27-id cfg-3 shard, plus a rocprofv3 kernel
# trace of the cfg-3 shard.   usage: bash tools/experiments/gpu_r03b.sh <out-tag> [skip-tests]
set -o pipefail
TAG=${1:-r03b}; OUT=gpurun_out/$TAG; mkdir -p $OUT profiles/r03
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
  tail -2 $OUT/gpu_tests.log
fi
timeout -k 10 120 python tools/small_probe.py --q 1 8 32 64 > $OUT/small_probe.log 2>&1 || { cat $OUT/small_probe.log; exit 1; }
cat $OUT/small_probe.log
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
pmc cfg3 "cfg3shard:134217728x131072x8" python3 tools/batch_probe.py --reps 3 --n 134217728 --q 131072 || exit 1
cp $OUT/pmc_traffic.json profiles/r03/pmc_traffic.json
grep -h -A3 '"k_s1_filter"\|"k_s2_answer"\|"k_f3_answer"\|"k_f2_filter"' $OUT/*_pmc.txt | head -80
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_cfg3 -o run --output-format csv -- python3 tools/batch_probe.py --reps 20 --n 134217728 --q 131072 > $OUT/kt_cfg3.log 2>&1 || exit 1
echo all-ok
