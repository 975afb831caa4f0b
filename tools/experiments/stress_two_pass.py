"""Repeat the two-pass F1 clustered-target case (tests/test_gpu_scale.py::test_f1_two_pass_clustered_targets)
and plain shapes several times on one context, K6 against the K1 scan; prints every mismatch with the
rows' results.   usage: python tools/experiments/stress_two_pass.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import opendht_amd  # noqa: E402
import oracle as O  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4


def clustered(q, seed):
    tg = O.gen_ids(seed, q)
    a = q // 4
    tg[:a, 0] = 0xA7
    tg[:a, 1] = (tg[:a, 1] & 0x0F) | 0x30
    lo = a
    for g, pre in zip((96, 256, 700, 2048), (0x1C44, 0x5B12, 0x9E60, 0xD301)):
        tg[lo:lo + g, 0] = pre >> 8
        tg[lo:lo + g, 1] = pre & 0xFF
        tg[lo:lo + g, 2] = (tg[lo:lo + g, 2] & 0x03) | 0x98
        lo += g
    return tg


ctx = opendht_amd.Context(0)
bad_total = 0
for n, q, kind in ((1 << 22, 1 << 18, "clustered"), (1 << 22, 1 << 18, "uniform"), (1 << 22, 1 << 17, "clustered")):
    ctx.gen_ids(3737, n)
    tg = clustered(q, 3738) if kind == "clustered" else O.gen_ids(3738, q)
    sc, scnt = ctx.topk(tg, 8)
    for r in range(reps):
        got, cnt = ctx.batch_topk(tg, 8)
        bad = np.nonzero((got != sc).any(axis=1) | (cnt != scnt))[0]
        bad_total += bad.size
        print(f"n={n} q={q} {kind} rep {r}: {bad.size} rows differ", flush=True)
        for b in bad[:4]:
            print("   row", b, "target", tg[b][:4].tobytes().hex(), "k6", got[b].tolist(), cnt[b], "k1", sc[b].tolist(), scnt[b])
ctx.close()
print("total differing rows", bad_total)
