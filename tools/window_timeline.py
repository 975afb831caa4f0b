"""Where a short timed window's extra time goes: the bench's cfg-2 stepping (three batches in
flight on three streams), a 20-call window from a synchronised start, a HIP event recorded on
each call's stream after the call; prints each call's completion time from the window's first
event (GPU clock) and the interval between completions.  Same library calls as bench.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import opendht_amd  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
n, q, k, fl, W = 1 << 24, 65536, 8, 3, 20
st = [torch.cuda.Stream(dev) for _ in range(fl)]
torch.cuda.set_stream(st[0])
L = opendht_amd.lib()
ctx = opendht_amd.Context(0)
ctx.gen_ids(2024, n)
ts = (q + 63) // 64 * 64
tp = torch.empty(5 * ts, dtype=torch.int32, device=dev)
assert L.dhtgpu_gen_dev(2025, 0, q, tp.data_ptr(), ts, st[0].cuda_stream) == 0
outs = [(torch.empty((q, k), dtype=torch.int32, device=dev), torch.empty(q, dtype=torch.int32, device=dev)) for _ in range(fl)]
i_call = [0]


def call():
    i = i_call[0] % fl
    i_call[0] += 1
    ctx.batch_topk_dev(tp.data_ptr(), ts, q, k, outs[i][0].data_ptr(), outs[i][1].data_ptr(), None, 0, st[i].cuda_stream)
    return i


for rep in range(4):
    for _ in range(5):   # the driver's warmup
        call()
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True)
    t0.record(st[i_call[0] % fl])
    evs = []
    for _ in range(W):
        i = call()
        e = torch.cuda.Event(enable_timing=True)
        e.record(st[i])
        evs.append(e)
    torch.cuda.synchronize()
    done = [t0.elapsed_time(e) * 1e3 for e in evs]
    gaps = [done[0]] + [done[j] - done[j - 1] for j in range(1, W)]
    print(f"window {rep}: total {max(done):.1f} us ({max(done) / W:.2f} us/call); completions:",
          " ".join(f"{d:.0f}" for d in done), flush=True)
    print("  intervals:", " ".join(f"{g:.1f}" for g in gaps), flush=True)
ctx.close()
