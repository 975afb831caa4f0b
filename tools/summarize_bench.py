"""One line per bench.py JSON result (the headline, its roofline, the cfg-3 legs): usage
python tools/summarize_bench.py FILE..."""
import json
import sys


def r(x, n=3):
    return None if x is None else round(x, n)


for f in sys.argv[1:]:
    lines = [l for l in open(f) if l.startswith("{")]
    if not lines:
        print(f, "no JSON line")
        continue
    d = json.loads(lines[-1])
    ro = d.get("roofline", {})
    print(f"{f}: {d['ms_per_step'] * 1e3:.2f} us/step {d['value'] / 1e9:.4f} G q/s  F2 frac {r(ro.get('frac'))} "
          f"step_frac {r(ro.get('step_hbm_frac'))} lat {r(d.get('latency_ms_per_batch', 0) * 1e3, 1)} us "
          f"verified {d.get('verified_exact')} hbm-cold {r(d.get('roofline_hbm', {}).get('frac'))}")
    for leg in ("cfg3_prefix_rank", "cfg3_broadcast_rank", "cfg3_shard", "cfg4"):
        x = d.get(leg)
        if not x:
            continue
        if "error" in x:
            print(f"  {leg}: ERROR {x['error']}")
            continue
        rf = x.get("roofline") or x.get("roofline_f2") or {}
        km = {k: r(v * 1e3, 1) for k, v in (x.get("kernels_ms") or {}).items() if v is not None}
        print(f"  {leg}: {r(x.get('ms_per_step', x.get('ms')), 4)} ms  frac {r(rf.get('frac'))} step_frac "
              f"{r(rf.get('step_frac'))} verified {x.get('verified_exact')} kernels_us {km}")
    sb = d.get("small_batch", {})
    if sb:
        print("  small_batch q1/8/32/64 us:", [r(sb[f"q{q}"]["batch"]["latency_ms"] * 1e3, 1) for q in (1, 8, 32, 64)
                                              if f"q{q}" in sb])
    cb = d.get("cpu_baseline")
    if cb:
        print(f"  cpu_baseline {r(cb['value'], 1)} q/s on {cb['cores']} cores ({cb['kind']})")
