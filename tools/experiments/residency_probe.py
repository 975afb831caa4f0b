"""Do F2 and F3 of different batches in flight share CUs?  (measurement, DHTGPU_DBG bit 2^24)

Runs the cfg-2 headline shape (2^24 ids, 65,536 targets, k = 8) with --inflight batches
alternating over as many streams, with the library's workgroup residency log on: thread 0 of
every F2 and F3 workgroup appends {kernel | phase, HW_ID | XCC_ID << 32, s_memrealtime,
blockIdx} at its start and end.  Pairs each workgroup's start and end on its CU and reports, per
kernel, how much of its workgroups' time another kernel's workgroup was resident on the same CU.
F3 runs its Diag instantiation under the log (the stamp build: same VGPR granule).  The log's code
is compiled only into a measurement build:
    bash tools/experiments/build_variant.sh reslog "-DDHT_RESLOG"
    DHTGPU_LIB=opendht_amd/ab/reslog.so python tools/experiments/residency_probe.py --inflight 3
The log holds the first ~38 calls (98,303 records)."""
import argparse
import ctypes
import json
import os
import sys
from collections import defaultdict

os.environ["DHTGPU_DBG"] = str(1 << 24)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import opendht_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1 << 24)
ap.add_argument("--q", type=int, default=65536)
ap.add_argument("--k", type=int, default=8)
ap.add_argument("--inflight", type=int, default=3)
ap.add_argument("--calls", type=int, default=38)
a = ap.parse_args()

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
L = opendht_amd.lib()
ctx = opendht_amd.Context(0)
ctx.gen_ids(2024, a.n)
streams = [torch.cuda.Stream(dev) for _ in range(a.inflight)]
ts = a.q
tp = torch.empty(5 * ts, dtype=torch.int32, device=dev)
assert L.dhtgpu_gen_dev(2025, 0, a.q, tp.data_ptr(), ts, streams[0].cuda_stream) == 0
outs = [(torch.empty((a.q, a.k), dtype=torch.int32, device=dev), torch.empty(a.q, dtype=torch.int32, device=dev))
        for _ in range(a.inflight)]
torch.cuda.synchronize()
for i in range(a.calls):
    oi, oc = outs[i % a.inflight]
    ctx.batch_topk_dev(tp.data_ptr(), ts, a.q, a.k, oi.data_ptr(), oc.data_ptr(), None, 0, streams[i % a.inflight].cuda_stream)
torch.cuda.synchronize()

fn = L.dhtgpu_debug_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64)]
ptr, nbytes = ctypes.c_void_p(), ctypes.c_uint64()
assert fn(ctx._h, ctypes.byref(ptr), ctypes.byref(nbytes)) == 0 and ptr.value
host = np.zeros(nbytes.value // 8, dtype=np.uint64)
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
assert hip.hipMemcpy(host.ctypes.data, ptr.value, nbytes.value, 2) == 0
cnt = int(host[0])
recs = host[4: 4 + 4 * min(cnt, (host.size - 4) // 4)].reshape(-1, 4)

# pair start / end per (kernel, workgroup, wave slot): the same wave logs both
open_ = {}
iv = defaultdict(list)   # kernel -> [(cu, t0, t1)]
for tag, hw, t, blk in sorted(recs.tolist(), key=lambda r: r[2]):
    kern, phase = tag >> 4, tag & 1
    h = hw & 0xFFFFFFFF
    cu = (hw >> 32, (h >> 13) & 7, (h >> 12) & 1, (h >> 8) & 15)
    key = (kern, blk, h, hw >> 32)
    if phase == 0:
        open_[key] = t
    elif key in open_:
        iv[kern].append((cu, open_.pop(key), t))

by_cu = defaultdict(lambda: defaultdict(list))
for kern, lst in iv.items():
    for cu, t0, t1 in lst:
        by_cu[cu][kern].append((t0, t1))


def overlap(mine, other):
    """time of `mine` intervals during which at least one `other` interval is open"""
    if not other:
        return 0
    other = sorted(other)
    merged = []
    for s, e in other:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    tot = 0
    for s, e in mine:
        for ms, me in merged:
            if me <= s:
                continue
            if ms >= e:
                break
            tot += min(e, me) - max(s, ms)
    return tot


res = {"records": cnt, "cus_seen": len(by_cu), "calls": a.calls, "inflight": a.inflight}
for kern, other in ((2, 3), (3, 2)):
    busy = sum(t1 - t0 for cu in by_cu for t0, t1 in by_cu[cu][kern])
    shared = sum(overlap(by_cu[cu][kern], by_cu[cu][other]) for cu in by_cu)
    res[f"F{kern}"] = {"workgroups": len(iv[kern]), "busy_us": busy / 100.0, "with_F%d_on_same_cu_us" % other: shared / 100.0,
                       "shared_frac": shared / busy if busy else None,
                       "median_wg_us": float(np.median([t1 - t0 for _, t0, t1 in iv[kern]])) / 100.0 if iv[kern] else None}
# how many F3 workgroups of one CU overlap at once (LDS: 4 alone) -- peak per CU
peak = []
for cu in by_cu:
    ev = sorted([(t0, 1) for t0, _ in by_cu[cu][3]] + [(t1, -1) for _, t1 in by_cu[cu][3]])
    c = m = 0
    for _, d in ev:
        c += d
        m = max(m, c)
    peak.append(m)
res["F3_peak_per_cu"] = {str(v): peak.count(v) for v in sorted(set(peak))}
print(json.dumps(res))
ctx.close()
