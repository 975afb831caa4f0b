"""Quick K6 driver for profiling: cfg-2 shaped inputs generated in HBM, `reps` stream-ordered
calls of dhtgpu_batch_topk_dev, then the per-kernel event times of one timed call."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import opendht_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1 << 24)
ap.add_argument("--q", type=int, default=65536)
ap.add_argument("--k", type=int, default=8)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--algo", default="batch")
ap.add_argument("--prefix", type=int, default=0, help="prefix shard: keep ids with top PREFIX bits == 0 of 2^PREFIX x n")
ap.add_argument("--evict", action="store_true", help="write 512 MiB before every call (Infinity Cache evicted)")
ap.add_argument("--inflight", type=int, default=1, help="calls alternate over this many streams")
ap.add_argument("--handles", action="store_true", help="sub-partitioned calls return sub-partition handles")
ap.add_argument("--cfg3", choices=["prefix", "broadcast"], default=None,
                help="bench.py's cfg3_<route>_rank inputs (one rank of cfg 3 at N = 8; broadcast: record form + K3)")
ap.add_argument("--key-file", default=None, help="--cfg3: write the PMC workload key bench.py looks up here")
a = ap.parse_args()
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
s = st.cuda_stream
L = opendht_amd.lib()
rec_out = None
if a.cfg3:
    import bench
    ctx, tp, ts, a.q, _, idx_lo = bench.cfg3_rank_setup(2024, a.cfg3, L, dev, s)
    a.n = ctx.num_ids
    if a.key_file:
        open(a.key_file, "w").write(f"cfg3{a.cfg3}:{a.n}x{a.q}x{a.k}")
    if a.cfg3 == "broadcast":
        rec_out = torch.empty((a.q, a.k, 3), dtype=torch.int32, device=dev)
else:
    ctx = opendht_amd.Context(0)
if a.cfg3:
    pass
elif a.prefix:
    ctx.gen_ids_prefix(2024, a.n << a.prefix, a.prefix, 0)
else:
    ctx.gen_ids(2024, a.n)
print("ids", ctx.num_ids, flush=True)
if a.handles:
    ctx.set_sub_handles(True)
if not a.cfg3:
    ts = (a.q + 63) // 64 * 64
    tp = torch.empty(5 * ts, dtype=torch.int32, device=dev)
    assert L.dhtgpu_gen_dev(2025, 0, a.q, tp.data_ptr(), ts, s) == 0
oi = torch.empty((a.q, a.k), dtype=torch.int32, device=dev)
oc = torch.empty(a.q, dtype=torch.int32, device=dev)


ebuf = torch.zeros(128 << 20, dtype=torch.int32, device=dev) if a.evict else None


streams = [st] + [torch.cuda.Stream(dev) for _ in range(a.inflight - 1)]
outs = [(oi, oc)] + [(torch.empty_like(oi), torch.empty_like(oc)) for _ in range(a.inflight - 1)]
ncall = [0]


def call():
    if ebuf is not None:
        ebuf.sum()
    i = ncall[0] % a.inflight
    ncall[0] += 1
    if rec_out is not None:   # cfg 3 broadcast rank: K6 in record form, then K3 over the one list
        ctx.batch_topk_dev(tp.data_ptr(), ts, a.q, a.k, None, None, rec_out.data_ptr(), idx_lo, streams[i].cuda_stream)
        assert L.dhtgpu_merge_dev(rec_out.data_ptr(), 1, a.q, a.k, tp.data_ptr(), ts, a.k, outs[i][0].data_ptr(),
                                  outs[i][1].data_ptr(), None, 0, streams[i].cuda_stream) == 0
    elif a.algo == "batch":
        ctx.batch_topk_dev(tp.data_ptr(), ts, a.q, a.k, outs[i][0].data_ptr(), outs[i][1].data_ptr(), None, 0,
                           streams[i].cuda_stream)
    else:
        ctx.index_build(s)
        ctx.index_topk_dev(tp.data_ptr(), ts, a.q, a.k, oi.data_ptr(), oc.data_ptr(), None, 0, s)


t0 = time.perf_counter()
call()
torch.cuda.synchronize()
print(f"first call {time.perf_counter() - t0:.3f} s", flush=True)
for _ in range(2 * a.inflight):   # every stream's workspace slot set up before the timed calls
    call()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.reps):
    call()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / a.reps
print(f"{a.algo} n={a.n} q={a.q} k={a.k}: {dt * 1e3:.4f} ms/call  {a.q / dt / 1e6:.1f} M q/s")
if a.algo == "batch":
    ms, fb, surv, slow = ctx.batch_topk_timed(tp.data_ptr(), ts, a.q, a.k, oi.data_ptr(), oc.data_ptr(), s)
    print("phases ms (F1,F2,F3,F4):", [round(x, 4) for x in ms], "fallback", fb, "survivors", surv, "wave-path", slow)
ctx.close()
