# Round-4 pass A: the whole GPU suite + smoke, the driver-shaped bench (20 steps, every leg, CPU
# baseline; small batches now warm / cold / past the Infinity Cache), a 2-rank rehearsal of the new
# N > 1 default (broadcast route, strong scaling of cfg 2) on one GPU, PMC traffic for the small-batch
# cold / 2^26 rows and the per-rank cfg-2 shards (N = 2, 4, 8).   usage: bash tools/experiments/gpu_r04a.sh [out-tag]
set -o pipefail
OUT=gpurun_out/${1:-r04a}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
timeout -k 10 300 python bench.py --gpus 2 --rehearse-one-gpu --steps 20 --warmup 5 > $OUT/rehearse_2ranks.json 2> $OUT/rehearse_2ranks.err || { tail -20 $OUT/rehearse_2ranks.err; exit 1; }
pmc() {  # name, workload key, probe command...
  local name=$1 key=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/${name}_fetch -o run --output-format csv -- "$@" > $OUT/${name}_fetch.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/${name}_write -o run --output-format csv -- "$@" > $OUT/${name}_write.log 2>&1 &&
  python3 tools/pmc_traffic.py $OUT/${name}_fetch $OUT/${name}_write $OUT/pmc_traffic.json "$key" > $OUT/${name}_pmc.txt
}
cp profiles/r04/pmc_traffic.json $OUT/pmc_traffic.json
for q in 1 8 32 64; do
  pmc ks_cold_q$q "ks:16777216x${q}x8:cold" python3 tools/small_probe.py --q $q --reps 5 --evict || exit 1
done
for q in 1 64; do
  pmc ks_big_q$q "ks:67108864x${q}x8" python3 tools/small_probe.py --q $q --reps 5 --n 67108864 --seed 2054 &&
  pmc ks_bigcold_q$q "ks:67108864x${q}x8:cold" python3 tools/small_probe.py --q $q --reps 5 --n 67108864 --seed 2054 --evict || exit 1
done
for n in 8388608 4194304 2097152; do
  pmc shard_$n "cfg2:${n}x65536x8" python3 tools/batch_probe.py --reps 3 --n $n || exit 1
done
python - "$OUT" <<'PY'
import json, sys
o = sys.argv[1]
d = json.load(open(f"{o}/bench_driver.json"))
print("driver", round(d["ms_per_step"] * 1e3, 2), "us/step", round(d["value"] / 1e9, 4), "G q/s, F2 frac",
      round(d["roofline"]["frac"], 3), "lat", d["latency_ms_per_batch"])
sb = d.get("small_batch", {})
for q in (1, 8, 32, 64):
    r = sb.get(f"q{q}", {})
    b = sb.get(f"big_q{q}", {})
    print(q, "warm", round(r.get("batch", {}).get("latency_ms", 0) * 1e3, 1), "cold", round(r.get("cold", {}).get("latency_ms", 0) * 1e3, 1),
          "cold s1_frac", round(r.get("cold", {}).get("s1_frac", 0), 3), "big cold s1_frac", round(b.get("cold", {}).get("s1_frac", 0), 3))
r = [json.loads(l) for l in open(f"{o}/rehearse_2ranks.json") if l.startswith("{")]
print("rehearsal", [(x.get("n_gpus"), x["config"]["route"], x["config"]["n_ids"], x["scaling"], round(x.get("ms_per_step", 0) * 1e3, 2), x.get("verified_exact")) for x in r])
PY
echo all-ok
