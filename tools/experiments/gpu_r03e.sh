# Round-3 evidence pass E (HEAD after the re-entry): the whole GPU parity suite, the bench as
# the driver runs it (20 steps, every leg, CPU baseline), the 1,000-step headline without the
# CPU leg, the cfg-3 shard phases and K2.   Output: gpurun_out/r03e/
set -o pipefail
OUT=gpurun_out/${1:-r03e}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
timeout -k 10 400 python bench.py --steps 1000 --warmup 100 --no-cpu > $OUT/bench1000.json 2> $OUT/bench1000.err || { tail -20 $OUT/bench1000.err; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python tools/batch_probe.py --reps 10 --n 134217728 --q 131072 > $OUT/cfg3_$i.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/classify_probe.py > $OUT/k2.log 2>&1 || exit 1
OUT=$OUT python - <<'PY'
import json, os
OUT = os.environ["OUT"]
for f in ("bench_driver", "bench1000"):
    d = json.load(open(f"{OUT}/{f}.json"))
    print(f, "step us", round(d["ms_per_step"] * 1e3, 2), "value", round(d["value"] / 1e9, 4), "G q/s; kernels", d["roofline"].get("kernels_ms"), "frac", round(d["roofline"]["frac"], 3))
    if "cfg3_shard" in d:
        c = d["cfg3_shard"]; print(" cfg3 shard ms", round(c["ms_per_step"], 4), c.get("kernels_ms"))
    if "cfg4" in d: print(" cfg4", d["cfg4"]["ms"], d["cfg4"]["roofline"]["frac"])
    if "small_batch" in d:
        for q in ("q1", "q8", "q32", "q64"):
            s = d["small_batch"].get(q)
            if s: print(" ", q, round(s["batch"]["latency_ms"] * 1e3, 2), s.get("kernels_ms"))
    cb = d.get("cpu_baseline")
    if cb: print(" cpu", cb["value"], cb["cores"], cb.get("host_cpus"), [k for k in cb])
PY
grep -H "ms/call\|phases" $OUT/cfg3_*.log
grep K2 $OUT/k2.log
echo done
