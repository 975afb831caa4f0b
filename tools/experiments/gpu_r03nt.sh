# Round-3 pass NT: counters and kernel traces after the non-temporal stream loads (S1; F2 on
# sub-partitioned sets past the Infinity Cache): PMC HBM traffic of KS q = 1 / 8 / 32 and the
# cfg-3 shard (merged into a copy of profiles/r03/pmc_traffic.json), rocprofv3 kernel traces of
# the cfg-3 shard and KS.   usage: bash tools/experiments/gpu_r03nt.sh [out-tag]
set -o pipefail
TAG=${1:-r03nt}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cp profiles/r03/pmc_traffic.json $OUT/pmc_traffic.json
pmc() {  # name, workload key, probe command...
  local name=$1 key=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/${name}_fetch -o run --output-format csv -- "$@" > $OUT/${name}_fetch.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/${name}_write -o run --output-format csv -- "$@" > $OUT/${name}_write.log 2>&1 &&
  python3 tools/pmc_traffic.py $OUT/${name}_fetch $OUT/${name}_write $OUT/pmc_traffic.json "$key" > $OUT/${name}_pmc.txt
}
for q in 1 8 32; do
  pmc ks_q$q "ks:16777216x${q}x8" python3 tools/small_probe.py --q $q --reps 10 || exit 1
done
pmc cfg3 "cfg3shard:134217728x131072x8" python3 tools/batch_probe.py --reps 3 --n 134217728 --q 131072 || exit 1
cat $OUT/*_pmc.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_cfg3 -o run --output-format csv -- python3 tools/batch_probe.py --reps 20 --n 134217728 --q 131072 > $OUT/kt_cfg3.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_small -o run --output-format csv -- python3 tools/small_probe.py --q 1 8 32 64 --reps 20 > $OUT/kt_small.log 2>&1 || exit 1
grep -h "phases\|ms/call" $OUT/kt_cfg3.log; grep -h "S1/S2" $OUT/kt_small.log
echo all-ok
