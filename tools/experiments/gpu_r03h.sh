# Round-3 evidence pass H (HEAD): whole GPU suite, the driver-shaped bench (20 steps, every leg,
# CPU baseline), the 1,000-step headline, KS S1 measurement builds, PMC traffic (cfg 2 warm /
# cold, cfg-3 shard, K2) and kernel traces (the 20-step bench, cfg-3 shard, K2).
set -o pipefail
OUT=gpurun_out/${1:-r03h}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
timeout -k 10 400 python bench.py --steps 1000 --warmup 100 --no-cpu > $OUT/bench1000.json 2> $OUT/bench1000.err || { tail -20 $OUT/bench1000.err; exit 1; }
for v in tree s1_NOTAIL s1_NOFILTER tree; do
  lib=""; [ $v != tree ] && lib="DHTGPU_LIB=opendht_amd/ab/$v.so"
  echo -n "$v "; timeout -k 10 120 env $lib X=1 python tools/small_probe.py --q 1 8 64 --reps 20 2>/dev/null | tr '\n' ' '; echo
done | tee $OUT/s1_measure.txt
pmc() {  # name, workload key, probe command...
  local name=$1 key=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/${name}_fetch -o run --output-format csv -- "$@" > $OUT/${name}_fetch.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/${name}_write -o run --output-format csv -- "$@" > $OUT/${name}_write.log 2>&1 &&
  python3 tools/pmc_traffic.py $OUT/${name}_fetch $OUT/${name}_write $OUT/pmc_traffic.json "$key" > $OUT/${name}_pmc.txt
}
cp profiles/r03/pmc_traffic.json $OUT/pmc_traffic.json
pmc cfg2 "cfg2:16777216x65536x8" python3 tools/batch_probe.py --reps 3 &&
pmc cfg2cold "cfg2:16777216x65536x8:cold" python3 tools/batch_probe.py --reps 3 --evict &&
pmc cfg3 "cfg3shard:134217728x131072x8" python3 tools/batch_probe.py --reps 3 --n 134217728 --q 131072 &&
pmc k2 "cfg4:100000000" python3 tools/classify_probe.py --reps 3 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_bench -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-extra --no-scan > $OUT/kt_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_cfg3 -o run --output-format csv -- python3 tools/batch_probe.py --reps 20 --n 134217728 --q 131072 > $OUT/kt_cfg3.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_k2 -o run --output-format csv -- python3 tools/classify_probe.py --reps 20 > $OUT/kt_k2.log 2>&1 || exit 1
echo all-ok
