"""Per-rank K6 in record form at the N = 1/2/4/8 range-shard sizes of the metric's workload
(2^24 / N ids, all 65,536 targets on every rank: the broadcast route's per-rank step), on ONE GPU
(single-GPU data to read the driver's scaling curve against; not a scaling run).
Per size: steps rotating over three streams (as bench.py --inflight 3), ms per step; the same
with final indices instead of records; per-kernel event times of serial calls; the record and
exchange bytes per rank at that N.   usage: python tools/shard_probe.py [--steps 200]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import opendht_amd  # noqa: E402
from opendht_amd import sharding  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--q", type=int, default=65536)
ap.add_argument("--k", type=int, default=8)
a = ap.parse_args()
sys.argv = [sys.argv[0]]
import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
st0 = torch.cuda.Stream(dev)
torch.cuda.set_stream(st0)
L = opendht_amd.lib()
q, k = a.q, a.k
tp, ts = bench.gen_targets(L, 2025, q, dev, st0.cuda_stream)
streams = [st0] + [torch.cuda.Stream(dev) for _ in range(2)]
out = {"workload": f"{q} targets x 2^24 / N ids per rank, k={k}", "rows": []}
for world in (1, 2, 4, 8):
    lo, hi = sharding.shard_range(1 << 24, world, 0)
    c = opendht_amd.Context(0)
    c.gen_ids(2024, hi - lo, start=lo)
    recs = [torch.empty((q, k, sharding.REC_WORDS), dtype=torch.int32, device=dev) for _ in range(3)]
    idx = [(torch.empty((q, k), dtype=torch.int32, device=dev), torch.empty(q, dtype=torch.int32, device=dev))
           for _ in range(3)]
    row = {"N": world, "ids_per_rank": hi - lo}
    for mode in ("records", "indices"):
        def step(i):
            s = streams[i % 3].cuda_stream
            if mode == "records":
                c.batch_topk_dev(tp.data_ptr(), ts, q, k, None, None, recs[i % 3].data_ptr(), lo, s)
            else:
                c.batch_topk_dev(tp.data_ptr(), ts, q, k, idx[i % 3][0].data_ptr(), idx[i % 3][1].data_ptr(), None, 0, s)
        for i in range(30):
            step(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st0)
        for i in range(a.steps):
            step(i)
        for s in streams[1:]:
            st0.wait_stream(s)
        e1.record(st0)
        torch.cuda.synchronize()
        row[f"ms_per_step_{mode}"] = e0.elapsed_time(e1) / a.steps
    ev = bench.EvSets(10, st0)
    for _ in range(10):
        ev.arm(c)
        c.batch_topk_dev(tp.data_ptr(), ts, q, k, None, None, recs[0].data_ptr(), lo, st0.cuda_stream)
    row["kernels_ms_serial"] = dict(zip(["F1", "F2", "F3", "F4"], ev.mean_ms()))
    row["record_bytes_per_rank"] = q * k * 4 * sharding.REC_WORDS
    row["allgather_bytes_in_per_gpu"] = world * q * k * 4 * sharding.REC_WORDS
    row["alltoall_bytes_in_per_gpu"] = q * k * 4 * sharding.REC_WORDS
    out["rows"].append(row)
    print(json.dumps(row), flush=True)
    c.close()
print(json.dumps(out))
