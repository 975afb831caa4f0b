"""K6 kernel times (F1..F4, HIP events on the kernels' own dispatches) of the cfg-3 per-rank shapes in
index form and in record form, serial calls on one stream.   usage: python tools/experiments/rec_vs_idx.py [broadcast|prefix]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import opendht_amd  # noqa: E402

route = sys.argv[1] if len(sys.argv) > 1 else "broadcast"
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
st = torch.cuda.Stream(dev)
s = st.cuda_stream
L = opendht_amd.lib()
ctx, tp, ts, q, _, lo = bench.cfg3_rank_setup(2024, route, L, dev, s)
k = 8
oi = torch.empty((q, k), dtype=torch.int32, device=dev)
oc = torch.empty(q, dtype=torch.int32, device=dev)
rec = torch.empty((q, k, 3), dtype=torch.int32, device=dev)


def idx(ev=None):
    if ev:
        ev.arm(ctx)
    ctx.batch_topk_dev(tp.data_ptr(), ts, q, k, oi.data_ptr(), oc.data_ptr(), None, 0, s)


def recf(ev=None):
    if ev:
        ev.arm(ctx)
    ctx.batch_topk_dev(tp.data_ptr(), ts, q, k, None, None, rec.data_ptr(), lo, s)


for name, fn in (("index", idx), ("record", recf), ("index", idx), ("record", recf)):
    for _ in range(3):
        fn()
    ev = bench.EvSets(10, st)
    for _ in range(10):
        fn(ev)
    print(route, name, "F1..F4 us:", [round(x * 1e3, 1) for x in ev.mean_ms()], flush=True)
ctx.close()
