# Round-5 GPU pass: the GPU suite (new tests first), smoke, the driver-shaped bench, the
# world-of-one collective path and the one-GPU rehearsal of the cfg-3 leg over RCCL.
# usage: bash tools/gpu_r05.sh <tag> [quick]   (quick: skip the 1,000-step bench and the rehearsal)
set -o pipefail
OUT=gpurun_out/${1:-r05}; mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -q --timeout 300 --timeout-method thread --durations=8"
timeout -k 10 600 $T tests -m gpu -x -k "merge or records or cfg3 or tie" > $OUT/gpu_new.log 2>&1 || { tail -60 $OUT/gpu_new.log; exit 1; }
tail -1 $OUT/gpu_new.log
timeout -k 10 900 $T tests -m gpu --maxfail=3 -k "not (merge or records or cfg3 or tie)" > $OUT/gpu_tests.log 2>&1 || { tail -60 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
timeout -k 10 300 python bench.py --sharded --steps 20 --warmup 5 --verify 64 > $OUT/sharded_allgather.json 2> $OUT/sharded_allgather.err || { tail -20 $OUT/sharded_allgather.err; exit 1; }
timeout -k 10 300 python bench.py --sharded --steps 1000 --warmup 100 --no-extra --verify 64 > $OUT/sharded_1000.json 2> $OUT/sharded_1000.err || { tail -20 $OUT/sharded_1000.err; exit 1; }
if [ "$2" != quick ]; then
  timeout -k 10 400 python bench.py --steps 1000 --warmup 100 --no-cpu --no-extra > $OUT/bench1000.json 2> $OUT/bench1000.err || { tail -20 $OUT/bench1000.err; exit 1; }
  timeout -k 10 400 python tools/experiments/rehearse_cfg3.py > $OUT/rehearse_cfg3.json 2> $OUT/rehearse_cfg3.err || { tail -20 $OUT/rehearse_cfg3.err; exit 1; }
fi
python3 - $OUT <<'PY'
import json, os, sys
o = sys.argv[1]
for f in ("bench_driver", "bench1000", "sharded_allgather", "sharded_1000"):
    if not os.path.exists(f"{o}/{f}.json"):
        continue
    d = json.loads([l for l in open(f"{o}/{f}.json") if l.startswith("{")][0])
    print(f, round(d["ms_per_step"] * 1e3, 2), "us/step", round(d["value"] / 1e9, 4), "G q/s, F2 frac",
          round(d["roofline"]["frac"], 3), "lat", round(d["latency_ms_per_batch"] * 1e3, 1), "verified", d.get("verified_exact"),
          "kernels", {k: round(v * 1e3, 1) for k, v in d["roofline"]["kernels_ms"].items()})
PY
echo all-ok
