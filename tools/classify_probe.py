"""K2 (findBucket + commonBits classification, cfg 4) driver for profiling: 10^8 splitmix ids
in HBM, the bucket firsts of a table grown by onNewNode from 10^5 ids (bench.cfg4_firsts),
--reps stream-ordered calls, then the mean event time of 10 calls and the HBM fraction
(5 B/id algorithmic: word 0 in + the 1-B bucket out; SURVEY's contract counts 20 + 1)."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import opendht_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=100_000_000)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--no-buckets", action="store_true")
a = ap.parse_args()
sys.argv = [sys.argv[0]]
import bench  # noqa: E402  (the cfg-4 table generator)

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
s = st.cuda_stream
L = opendht_amd.lib()
myid, firsts = bench.cfg4_firsts(2024 + 5)
c = opendht_amd.Context(0)
c.gen_ids(2024 + 6, a.n)
planes, stride = c.ids_dev()
fp = torch.from_numpy(firsts.view(">u4").reshape(-1, 5).astype(np.uint32).T.copy().reshape(-1).view(np.int32)).to(dev)
my = np.frombuffer(myid.tobytes(), dtype=">u4").astype(np.uint32)
my_c = (ctypes.c_uint32 * 5)(*[int(x) for x in my])
bucket = torch.empty(a.n, dtype=torch.uint8, device=dev)
hist = torch.zeros(161, dtype=torch.int64, device=dev)


def call():
    assert L.dhtgpu_classify_dev(planes, stride, a.n, firsts.shape[0], fp.data_ptr(), my_c,
                                 None if a.no_buckets else bucket.data_ptr(), hist.data_ptr(), s) == 0


for _ in range(a.reps):
    call()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st)
for _ in range(10):
    call()
e1.record(st)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 10
b = (4 + (0 if a.no_buckets else 1)) * a.n   # word 0 streamed + the 1-B bucket (K2 reads words 1..4 only on word-0 ties)
print(f"K2 n={a.n} buckets={firsts.shape[0]}: {ms:.4f} ms  {b / ms / 1e6:.0f} GB/s  frac {b / ms / 1e6 / 8000:.3f}", flush=True)
c.close()
