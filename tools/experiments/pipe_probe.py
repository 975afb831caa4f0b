"""Throughput of K6 with batches in flight: ONE context (its round-robin workspace slots) called
on D streams round-robin, so one batch's latency-bound F3/F4 overlaps the next batch's
HBM-bound F2.  Prints per-batch wall time for D = 1, 2, 3 and checks the outputs agree."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import opendht_amd  # noqa: E402

n, q, k, reps = 1 << 24, 65536, 8, 200
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
L = opendht_amd.lib()
ts = (q + 63) // 64 * 64
tp = torch.empty(5 * ts, dtype=torch.int32, device=dev)
assert L.dhtgpu_gen_dev(2025, 0, q, tp.data_ptr(), ts, None) == 0
ctx = opendht_amd.Context(0)
ctx.gen_ids(2024, n)
for D in (1, 2, 3):
    streams = [torch.cuda.Stream(dev) for _ in range(D)]
    outs = [(torch.empty((q, k), dtype=torch.int32, device=dev), torch.empty(q, dtype=torch.int32, device=dev))
            for _ in range(D)]
    torch.cuda.synchronize()

    def call(i):
        s, (oi, oc) = streams[i % D], outs[i % D]
        ctx.batch_topk_dev(tp.data_ptr(), ts, q, k, oi.data_ptr(), oc.data_ptr(), None, 0, s.cuda_stream)

    for i in range(10):
        call(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        call(i)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    ok = all(torch.equal(outs[0][0], o[0]) for o in outs[1:])
    print(f"D={D}: {dt * 1e6:.1f} us per batch, {q / dt / 1e9:.3f} G q/s, outputs agree: {ok}", flush=True)
ctx.close()
