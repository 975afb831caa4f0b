# Round 5, pass g: K6 record form with every writer storing records (no conversion pass), the
# collective step's host trims.   usage: bash tools/experiments/gpu_r05_g.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-r05g}; mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -q --timeout 300 --timeout-method thread --durations=6"
timeout -k 10 900 $T tests -m gpu -x -k "records or merge or tie or fallback or cfg3 or fuzz or sharded" > $OUT/gpu_rec.log 2>&1 || { tail -60 $OUT/gpu_rec.log; exit 1; }
tail -1 $OUT/gpu_rec.log
timeout -k 10 200 python tools/shard_probe.py --steps 300 > $OUT/probe.json 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/probe.json'):
    d = json.loads(l)
    if 'N' in d: print('N', d['N'], 'rec', round(d['ms_per_step_records']*1e3, 1), 'idx', round(d['ms_per_step_indices']*1e3, 1), {k: round(v*1e3, 1) for k, v in d['kernels_ms_serial'].items()})
"
timeout -k 10 200 python tools/experiments/host_profile.py > $OUT/host_profile.json 2> $OUT/host_profile.err || { tail -20 $OUT/host_profile.err; exit 1; }
grep piece $OUT/host_profile.json
timeout -k 10 300 python bench.py --sharded --steps 1000 --warmup 100 --no-cpu --no-extra > $OUT/sh1000.json 2> $OUT/sh1000.err || { tail -20 $OUT/sh1000.err; exit 1; }
timeout -k 10 300 python bench.py --sharded --steps 20 --warmup 5 --no-extra --verify 64 > $OUT/sh20.json 2> $OUT/sh20.err || { tail -20 $OUT/sh20.err; exit 1; }
python3 - $OUT <<'PY'
import json, sys
o = sys.argv[1]
for f in ("sh1000", "sh20"):
    d = json.loads([l for l in open(f"{o}/{f}.json") if l.startswith("{")][-1])
    print(f, round(d["ms_per_step"] * 1e3, 2), "us/step; enq", round(d["host_enqueue_ms_per_step"] * 1e3, 1), "win",
          round(d["gpu_window_ms_per_step"] * 1e3, 1), "lat", round(d["latency_ms_per_batch"] * 1e3, 1),
          "verified", d.get("verified_exact"), {k: round(v * 1e3, 1) for k, v in d["roofline"]["kernels_ms"].items()})
PY
echo all-ok
