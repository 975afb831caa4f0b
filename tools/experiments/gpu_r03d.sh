# Round-3 pass D: parity suite after the F3 exact-gather default, F3's plan-sized stage and
# F4's paired ties; cfg-3 shard phases; the bench with its extra legs (no CPU baseline); K2.
set -o pipefail
OUT=gpurun_out/r03d; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for i in 1 2; do
  timeout -k 10 200 python tools/batch_probe.py --reps 10 --n 134217728 --q 131072 > $OUT/cfg3_$i.log 2>&1 || exit 1
done
grep -H "ms/call\|phases" $OUT/cfg3_*.log
timeout -k 10 120 python tools/classify_probe.py > $OUT/k2.log 2>&1 && timeout -k 10 120 python tools/classify_probe.py --no-buckets >> $OUT/k2.log 2>&1 || exit 1
grep K2 $OUT/k2.log
timeout -k 10 400 python bench.py --steps 1000 --warmup 100 --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r03d/bench.json"))
print("cfg2 step us", round(d["ms_per_step"] * 1e3, 2), "latency us", round(d["latency_ms_per_batch"] * 1e3, 1), "F-kernels", d["roofline"]["kernels_ms"])
c = d["cfg3_shard"]; print("cfg3 shard ms", round(c["ms_per_step"], 4), c["kernels_ms"], "f2 frac", round(c["roofline_f2"]["frac"], 3))
print("cfg4", d["cfg4"]["ms"], d["cfg4"]["roofline"]["frac"])
for q in ("q1", "q8", "q32", "q64"): print(q, round(d["small_batch"][q]["batch"]["latency_ms"] * 1e3, 2), d["small_batch"][q]["kernels_ms"])
PY
echo done
