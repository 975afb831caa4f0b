"""Host-side cost of each piece of the world-of-one collective step (bench.py --sharded): K6 in
record form, the stream context, the RCCL all-gather, K3 through ctypes.  Each piece is enqueued
`--reps` times back to back and timed on the host (perf_counter), GPU work synchronised only at
the end of each piece.   usage: python tools/experiments/host_profile.py [--reps 300]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import opendht_amd  # noqa: E402
from opendht_amd import sharding  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=300)
a = ap.parse_args()
sys.argv = [sys.argv[0]]
import bench  # noqa: E402

dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
st0 = torch.cuda.Stream(dev)
torch.cuda.set_stream(st0)
s = st0.cuda_stream
L = opendht_amd.lib()
q, k = 65536, 8
tp, ts = bench.gen_targets(L, 2025, q, dev, s)
ctx = opendht_amd.Context(0)
ctx.gen_ids(2024, 1 << 24)
rec = torch.empty((q, k, 3), dtype=torch.int32, device=dev)
xb = torch.empty((q, k, 3), dtype=torch.int32, device=dev)
oi = torch.empty((q, k), dtype=torch.int32, device=dev)
oc = torch.empty(q, dtype=torch.int32, device=dev)
tx = sharding.TieExchange(1, k, dev)
ops = sharding.LibOps(L, ctx, tp.data_ptr(), ts)
torch.cuda.synchronize()


def timed(name, fn, reps=a.reps):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    r = {"piece": name, "host_us": (t1 - t0) * 1e6 / reps, "wall_us": (t2 - t0) * 1e6 / reps}
    print(json.dumps(r), flush=True)
    return r


rows = []
rows.append(timed("k6_records", lambda: ctx.batch_topk_dev(tp.data_ptr(), ts, q, k, None, None, rec.data_ptr(), 0, s)))
rows.append(timed("k6_indices", lambda: ctx.batch_topk_dev(tp.data_ptr(), ts, q, k, oi.data_ptr(), oc.data_ptr(), None, 0, s)))


def ctxm():
    with torch.cuda.stream(st0):
        pass


rows.append(timed("stream_context", ctxm))
rows.append(timed("set_stream", lambda: torch.cuda.set_stream(st0)))
rows.append(timed("ctypes_num_ids", lambda: L.dhtgpu_num_ids(ctx._h)))
rows.append(timed("all_gather_into_tensor", lambda: dist.all_gather_into_tensor(xb, rec)))
rows.append(timed("gather_records", lambda: sharding.gather_records(rec, out=xb)))
g = xb.view(1, q, k, 3)
rows.append(timed("k3_merge", lambda: ops.merge(g, 0, k, oi, oc, None, s)))
rows.append(timed("merge_allgather", lambda: sharding.merge_allgather(ops, rec, g, k, oi, oc, tx, 0, s)))


def full():
    with torch.cuda.stream(st0):
        ctx.batch_topk_dev(tp.data_ptr(), ts, q, k, None, None, rec.data_ptr(), 0, s)
        gg = sharding.gather_records(rec, out=xb)
        sharding.merge_allgather(ops, rec, gg, k, oi, oc, tx, 0, s)


rows.append(timed("full_step_one_stream", full))


def full_ss():
    torch.cuda.set_stream(st0)
    ctx.batch_topk_dev(tp.data_ptr(), ts, q, k, None, None, rec.data_ptr(), 0, s)
    dist.all_gather_into_tensor(xb, rec)
    ops.merge(g, 0, k, oi, oc, None, s)


rows.append(timed("full_step_set_stream_direct", full_ss))
print(json.dumps({"rows": rows}))
ctx.close()
dist.destroy_process_group()
