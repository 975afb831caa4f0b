# Round-3 final evidence at HEAD: the whole GPU suite and smoke(), the driver's bench (20 steps,
# every leg, CPU baseline), the 1,000-step headline, a 2-rank rehearsal of the N > 1 path on one
# GPU (bench.py --gpus 2 starting its ranks itself; gloo: RCCL refuses two ranks on one GPU),
# F2/F3 phase stamps.   usage: bash tools/experiments/gpu_r03_final.sh [out-tag]
set -o pipefail
OUT=gpurun_out/${1:-r03final}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
timeout -k 10 400 python bench.py --steps 1000 --warmup 100 --no-cpu > $OUT/bench1000.json 2> $OUT/bench1000.err || { tail -20 $OUT/bench1000.err; exit 1; }
timeout -k 10 300 python bench.py --gpus 2 --rehearse-one-gpu --steps 20 --warmup 5 --no-cpu --no-extra > $OUT/rehearse_2ranks.json 2> $OUT/rehearse_2ranks.err || { tail -20 $OUT/rehearse_2ranks.err; exit 1; }
DHTGPU_DBG=256 timeout -k 10 120 python tools/batch_probe.py --reps 3 > $OUT/stamps.log 2>&1 || exit 1
python - "$OUT" <<'PY'
import json, sys
o = sys.argv[1]
for f in ("bench_driver", "bench1000"):
    d = json.load(open(f"{o}/{f}.json"))
    print(f, round(d["ms_per_step"] * 1e3, 2), "us/step", round(d["value"] / 1e9, 4), "G q/s, F2 frac", round(d["roofline"]["frac"], 3))
r = [json.loads(l) for l in open(f"{o}/rehearse_2ranks.json") if l.startswith("{")]
print("rehearsal", [(x.get("n_gpus"), round(x.get("ms_per_step", 0) * 1e3, 2), x.get("verified_exact")) for x in r])
PY
echo all-ok
