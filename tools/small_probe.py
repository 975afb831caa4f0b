import sys, os, json
sys.path.insert(0, os.getcwd())
import torch, opendht_amd
dev = torch.device("cuda", 0); torch.cuda.set_device(0)
st = torch.cuda.Stream(dev); torch.cuda.set_stream(st); s = st.cuda_stream
L = opendht_amd.lib(); ctx = opendht_amd.Context(0); ctx.gen_ids(2024, 1 << 24)
q = 64; ts = 64
tp = torch.empty(5 * ts, dtype=torch.int32, device=dev)
assert L.dhtgpu_gen_dev(2025, 0, q, tp.data_ptr(), ts, s) == 0
oi = torch.empty((q, 8), dtype=torch.int32, device=dev); oc = torch.empty(q, dtype=torch.int32, device=dev)
for qq in (1, 8, 64):
    res = []
    for _ in range(20):
        ms, fb, surv, slow = ctx.batch_topk_timed(tp.data_ptr(), ts, qq, 8, oi.data_ptr(), oc.data_ptr(), s)
        res.append(ms)
    import numpy as np
    m = np.median(np.array(res), axis=0)
    print(os.environ.get("DHTGPU_S1", "0"), qq, [round(x * 1e3, 2) for x in m])
