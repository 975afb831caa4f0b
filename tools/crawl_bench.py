"""BASELINE.json configs[4]: dhtscanner-style crawl replay over a synthetic network.

Network: --n node ids generated in HBM (splitmix64 stream), a seeded fraction
--dead of nodes that never answer, implicit k-bucket routing tables (crawl model,
opendht_amd/csrc/crawl.hip).  Reports, as one JSON line:
  * the full dhtscanner crawl (tools/dhtscanner.cpp recursion, one batched search call per
    generation): steps, find_node requests, nodes found, wall time;
  * search-refresh throughput: --q independent iterative searches in one device call
    (searches/s, rounds and requests per search);
  * cpu_baseline: the oracle restatement of the same searches on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import opendht_amd  # noqa: E402
from opendht_amd import crawl  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=50_000_000)
ap.add_argument("--dead", type=float, default=0.1)
ap.add_argument("--q", type=int, default=65536)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--seed", type=int, default=2024)
ap.add_argument("--cpu-sample", type=int, default=1024)
ap.add_argument("--no-cpu", action="store_true")
a = ap.parse_args()

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
L = opendht_amd.lib()
ctx = opendht_amd.Context(0)
t0 = time.perf_counter()
ctx.gen_ids(a.seed, a.n)
dead = (np.random.default_rng(a.seed).random(a.n) < a.dead).astype(np.uint8)
ctx.net_prepare(dead, table_seed=a.seed)
setup_s = time.perf_counter() - t0

# host copy of the node ids, for the scanner's commonBits(first, last)
ids_cache = {}


def node_ids(ix):
    out = np.empty((len(ix), 20), np.uint8)
    for j, i in enumerate(ix):
        i = int(i)
        if i not in ids_cache:
            ids_cache[i] = ctx.get_ids(i, 1)[0]
        out[j] = ids_cache[i]
    return out


scanner = 12345 % a.n
t0 = time.perf_counter()
res = crawl.crawl(lambda t, s, r: ctx.search_batch(t, s, r), node_ids, scanner)
crawl_s = time.perf_counter() - t0

# refresh throughput: q random targets, searchers spread over the network, device buffers
q = a.q
ts = (q + 63) // 64 * 64
tp = torch.empty(5 * ts, dtype=torch.int32, device=dev)
assert L.dhtgpu_gen_dev(a.seed + 7, 0, q, tp.data_ptr(), ts, None) == 0
sr = torch.from_numpy(((np.arange(q, dtype=np.uint64) * 2654435761) % a.n).astype(np.uint32).view(np.int32)).to(dev)
o_idx = torch.empty((q, 64), dtype=torch.int32, device=dev)
o_fl = torch.empty((q, 64), dtype=torch.uint8, device=dev)
o_len, o_rd, o_qs = (torch.empty(q, dtype=torch.int32, device=dev) for _ in range(3))
args = (tp.data_ptr(), ts, q, sr.data_ptr(), 64, o_idx.data_ptr(), o_fl.data_ptr(), o_len.data_ptr(),
        o_rd.data_ptr(), o_qs.data_ptr(), None)
assert L.dhtgpu_search_batch_dev(ctx._h, *args) == 0
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.reps):
    assert L.dhtgpu_search_batch_dev(ctx._h, *args) == 0
torch.cuda.synchronize()
ref_s = (time.perf_counter() - t0) / a.reps
rounds = o_rd.cpu().numpy()
reqs = o_qs.cpu().numpy()

out = {"metric": "iterative searches/s (crawl-model find_node rounds, SEARCH_NODES=14, 4 requests/round)",
       "value": q / ref_s, "unit": "searches/s", "n_gpus": 1, "higher_is_better": True,
       "config": {"workload": f"cfg5 crawl replay: {a.n} nodes ({a.dead:.0%} dead), {q} searches", "n_nodes": a.n,
                  "dead_frac": a.dead, "searches": q},
       "ms_per_batch": ref_s * 1e3, "rounds_mean": float(rounds.mean()), "rounds_max": int(rounds.max()),
       "requests_mean": float(reqs.mean()), "setup_s": setup_s,
       "crawl": {"steps": res["steps"], "generations": res["generations"], "requests": res["queries"],
                 "nodes_found": int(res["found"].size), "wall_s": crawl_s},
       "data": "synthetic: splitmix64 node ids in HBM, seeded dead mask"}

if not a.no_cpu:
    import oracle as O
    m = min(a.cpu_sample, q)
    ids = O.gen_ids(a.seed, a.n)
    tg = O.gen_ids(a.seed + 7, m)
    srh = sr[:m].cpu().numpy().view(np.uint32)
    t0 = time.perf_counter()
    O.search_batch(ids, dead, a.seed, tg[:1], srh[:1], 64, threads=16)     # node sort + 1 search
    sort_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    w = O.search_batch(ids, dead, a.seed, tg, srh, 64, threads=16)
    cpu_s = time.perf_counter() - t0
    out["cpu_baseline"] = {"value": m / max(cpu_s - sort_s, 1e-9), "unit": "searches/s", "cores": 16, "kind": "port",
                           "sample": f"{m} searches over the same {a.n}-node network, {cpu_s:.2f} s wall of which "
                                     f"{sort_s:.2f} s node sort (excluded from value)"}
    g = [x[:m] for x in (o_idx.cpu().numpy().view(np.uint32), o_fl.cpu().numpy(), o_len.cpu().numpy().view(np.uint32),
                         o_rd.cpu().numpy().view(np.uint32), o_qs.cpu().numpy().view(np.uint32))]
    out["verified_searches"] = m
    out["verified_exact"] = bool(all(np.array_equal(x, y) for x, y in zip(g, w)))
print(json.dumps(out), flush=True)
ctx.close()
