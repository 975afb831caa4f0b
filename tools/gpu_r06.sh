# Round-6 GPU passes.   usage: PART=<a|b|c> bash tools/gpu_r06.sh [tag]
#   a: the whole GPU suite + smoke, the driver's bench (20 steps, every leg, CPU baseline, the new
#      cfg-3 per-rank legs), the 1,000-step headline
#   b: rocprofv3 kernel traces (driver-shaped bench, the cfg-3 per-rank legs' probes) and PMC
#      FETCH/WRITE passes of the cfg-3 per-rank shapes, cfg 2 warm / cold, the cfg-3 shard, K2
#   c: rehearsals of the N > 1 paths on one GPU (2 ranks over gloo, RCCL world of one, cfg 3 at
#      10^9 ids as a world of one)
set -o pipefail
OUT=gpurun_out/${1:-r06}; mkdir -p $OUT
export TMPDIR=/tmp
PART=${PART:-a}
if [ "$PART" = a ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=12 > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu --no-extra > $OUT/bench1000.json 2> $OUT/bench1000.err || { tail -20 $OUT/bench1000.err; exit 1; }
python3 tools/summarize_bench.py $OUT/bench_driver.json $OUT/bench1000.json
echo all-ok
exit 0
fi
if [ "$PART" = b ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_bench20 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-extra --no-scan > $OUT/kt_bench20.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_cfg3prefix -o run --output-format csv -- python3 tools/batch_probe.py --reps 20 --inflight 2 --cfg3 prefix > $OUT/kt_cfg3prefix.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_cfg3broadcast -o run --output-format csv -- python3 tools/batch_probe.py --reps 20 --inflight 2 --cfg3 broadcast > $OUT/kt_cfg3broadcast.log 2>&1 || exit 1
pmc() {  # name, workload key, probe command...
  local name=$1 key=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/${name}_fetch -o run --output-format csv -- "$@" > $OUT/${name}_fetch.log 2>&1 &&
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/${name}_write -o run --output-format csv -- "$@" > $OUT/${name}_write.log 2>&1 &&
  python3 tools/pmc_traffic.py $OUT/${name}_fetch $OUT/${name}_write $OUT/pmc_traffic.json "$key" > $OUT/${name}_pmc.txt
}
cp profiles/r06/pmc_traffic.json $OUT/pmc_traffic.json
pmc cfg3prefix "@$OUT/cfg3prefix.key" python3 tools/batch_probe.py --reps 3 --cfg3 prefix --key-file $OUT/cfg3prefix.key &&
pmc cfg3broadcast "@$OUT/cfg3broadcast.key" python3 tools/batch_probe.py --reps 3 --cfg3 broadcast --key-file $OUT/cfg3broadcast.key &&
pmc cfg2 "cfg2:16777216x65536x8" python3 tools/batch_probe.py --reps 3 &&
pmc cfg2cold "cfg2:16777216x65536x8:cold" python3 tools/batch_probe.py --reps 3 --evict &&
pmc cfg3 "cfg3shard:134217728x131072x8" python3 tools/batch_probe.py --reps 3 --n 134217728 --q 131072 &&
pmc k2 "cfg4:100000000" python3 tools/classify_probe.py --reps 3 || exit 1
python3 - $OUT <<'PY'
import csv, glob, sys
o = sys.argv[1]
for k in ("kt_bench20", "kt_cfg3prefix", "kt_cfg3broadcast"):
    f = glob.glob(f"{o}/{k}/**/*kernel_stats.csv", recursive=True)[0]
    for row in csv.DictReader(open(f)):
        if "dhtgpu" in row["Name"]:
            nm = row["Name"].replace("void ", "").replace("(anonymous namespace)::", "").replace("dhtgpu::", "")
            print(k, nm.split("(")[0][:40], row["Calls"], round(float(row["AverageNs"]) / 1e3, 2), "us")
PY
echo all-ok
exit 0
fi
timeout -k 10 400 python bench.py --gpus 2 --rehearse-one-gpu --steps 20 --warmup 5 > $OUT/rehearse_2ranks.json 2> $OUT/rehearse_2ranks.err || { tail -20 $OUT/rehearse_2ranks.err; exit 1; }
timeout -k 10 300 python bench.py --sharded --steps 20 --warmup 5 --verify 64 > $OUT/sharded_allgather.json 2> $OUT/sharded_allgather.err || { tail -20 $OUT/sharded_allgather.err; exit 1; }
timeout -k 10 300 python bench.py --sharded --steps 1000 --warmup 100 --no-extra --verify 64 > $OUT/sharded_1000.json 2> $OUT/sharded_1000.err || { tail -20 $OUT/sharded_1000.err; exit 1; }
timeout -k 10 500 python tools/experiments/rehearse_cfg3.py > $OUT/rehearse_cfg3.json 2> $OUT/rehearse_cfg3.err || { tail -20 $OUT/rehearse_cfg3.err; exit 1; }
python3 tools/summarize_bench.py $OUT/sharded_allgather.json $OUT/sharded_1000.json
echo all-ok
