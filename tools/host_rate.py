"""Host enqueue rate of K6 calls vs the GPU period: is the pipelined cfg-2 step host-bound?
usage: python tools/host_rate.py [dir-with-opendht_amd]"""
import os
import sys
import time

sys.path.insert(0, sys.argv[1] if len(sys.argv) > 1 else os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import opendht_amd  # noqa: E402

dev = torch.device("cuda", 0)
L = opendht_amd.lib()
ctx = opendht_amd.Context(0)
ctx.gen_ids(2024, 1 << 24)
q, k = 65536, 8
ts = q
tp = torch.empty(5 * ts, dtype=torch.int32, device=dev)
st = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
assert L.dhtgpu_gen_dev(2025, 0, q, tp.data_ptr(), ts, st[0].cuda_stream) == 0
outs = [(torch.empty((q, k), dtype=torch.int32, device=dev), torch.empty(q, dtype=torch.int32, device=dev)) for _ in range(2)]
for i in range(200):
    ctx.batch_topk_dev(tp.data_ptr(), ts, q, k, outs[i % 2][0].data_ptr(), outs[i % 2][1].data_ptr(), None, 0, st[i % 2].cuda_stream)
torch.cuda.synchronize()
n = 2000
t0 = time.perf_counter()
for i in range(n):
    ctx.batch_topk_dev(tp.data_ptr(), ts, q, k, outs[i % 2][0].data_ptr(), outs[i % 2][1].data_ptr(), None, 0, st[i % 2].cuda_stream)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"enqueue {1e6 * (t1 - t0) / n:.2f} us/call, total {1e6 * (t2 - t0) / n:.2f} us/call")
