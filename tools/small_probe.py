"""KS (small-batch path) driver for profiling: the cfg-2 id set (2^24 splitmix ids in HBM), q
targets per call.  --reps stream-ordered calls of dhtgpu_batch_topk_dev (for rocprofv3 kernel
traces / PMC passes), then the per-kernel event times (median of 20 timed calls) per q."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import opendht_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--q", type=int, nargs="+", default=[1, 8, 64])
ap.add_argument("--k", type=int, default=8)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--n", type=int, default=1 << 24, help="ids (2^24: the cfg-2 set; 2^26: past the Infinity Cache)")
ap.add_argument("--seed", type=int, default=2024)
ap.add_argument("--evict", action="store_true", help="read 512 MiB before every call (Infinity Cache evicted)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
s = st.cuda_stream
L = opendht_amd.lib()
ctx = opendht_amd.Context(0)
ctx.gen_ids(a.seed, a.n)
ebuf = torch.zeros(128 << 20, dtype=torch.int32, device=dev) if a.evict else None
ts = 64
tp = torch.empty(5 * ts, dtype=torch.int32, device=dev)
assert L.dhtgpu_gen_dev(2025, 0, 64, tp.data_ptr(), ts, s) == 0
oi = torch.empty((64, a.k), dtype=torch.int32, device=dev)
oc = torch.empty(64, dtype=torch.int32, device=dev)
for q in a.q:
    for _ in range(a.reps):
        if ebuf is not None:
            ebuf.sum()
        ctx.batch_topk_dev(tp.data_ptr(), ts, q, a.k, oi.data_ptr(), oc.data_ptr(), None, 0, s)
    torch.cuda.synchronize()
    res = [ctx.batch_topk_timed(tp.data_ptr(), ts, q, a.k, oi.data_ptr(), oc.data_ptr(), s)[0] for _ in range(20)]
    m = np.median(np.array(res), axis=0)
    print(f"q={q} k={a.k} S1/S2 us (median of 20):", [round(x * 1e3, 2) for x in m[1:3]], flush=True)
ctx.close()
