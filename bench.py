"""bench.py -- batched k=8 XOR-closest lookup (OpenDHT's findClosestNodes ordering)
on MI355X through libdhtgpu.

Workload (BASELINE.json configs[1]): 65,536 random target hashes x 2^24 random 160-bit
node ids, k = 8, exact (bit-identical to std::partial_sort over InfoHash::xorCmp).
One step = one batched lookup of all targets against the whole id set.  Ids and
targets are generated in HBM before timing (synthetic splitmix64 stream).

Algorithms (--algo):
  batch  K6 per-batch target-prefix filter (default): every step streams the raw id word
         plane w0 once, keeps the ids sharing a level-Lm prefix with some target of the
         batch, and answers each target exactly from its complete prefix subtree in LDS
  index  K4 bucket-index build + K5 trie-descent query; the index is REBUILT from the raw
         id planes inside every timed step
  scan   K1 brute-force streaming scan (the north-star kernel design)
Nothing is cached between steps in any algorithm.

Multi-GPU (one process per GPU, torch.distributed over RCCL; --route):
  prefix     (default for a power-of-two world) ids AND targets are partitioned by their
             top log2(N) bits; each rank answers only its own targets from its own shard.
             If every shard holds >= k ids, a target's top-k provably lies in its own
             prefix subtree, so the data path needs no collective; the setup checks the
             minimum shard size with one all-reduce and refuses otherwise.
  broadcast  ids range-sharded, all targets on every rank, per-rank candidate records
             exchanged by one RCCL all-gather, merged by K3 (SURVEY §8(e) north-star scheme).
Scaling (--scaling): "weak" (default with the prefix route: the path partitions into
independent prefix shards, so every rank keeps the one-GPU workload -- --n ids and --q
targets per GPU out of a global problem N times as large; value = all ranks' targets / the
slowest rank's time) or "strong" (--n and --q are the global totals, split across ranks).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# Two batches in flight (--inflight) need their streams on different hardware queues; HIP's
# default of 4 queues per process is shared round-robin by every stream the process creates
# (torch's, the context's), so ask for 8 before the runtime starts.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import opendht_amd  # noqa: E402
from opendht_amd import sharding  # noqa: E402

METRIC = "queries/sec, k=8 XOR-NN over 16M 160-bit IDs; % HBM roofline at 1/2/4/8 GPUs"
# int32 VALU peak: a wave64 integer VALU op issues every 4 cycles per SIMD on gfx950
# (16 lanes/clk/SIMD): 1024 SIMDs x 16 x 2.4 GHz = 39.3 T lane-ops/s; tools/valu_peak
# measures 40.1 T on the box (profiles/r01_valu_peak.log).
VALU_PEAK_TOPS = 1024 * 16 * 2.4e9 / 1e12
HBM_PEAK_GBS = 8000.0
# Algorithmic VALU work per (id, target) pair in K1: the XOR distance and the running-min
# select, done two pairs at a time on packed top-16-bit words (v_xor_b32 + v_pk_min_u16
# per two pairs) = 1 lane-op per pair.  (SURVEY 8(d)'s contract assumed 3 ops/pair on a
# 64-bit lane; the packed prefilter is an algorithmic win, so frac here is measured
# against the op count the kernel actually needs and cannot exceed 1.)
OPS_PER_PAIR = 1.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)   # ~41 ms timed: steady state, not ramp-up
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--n", type=int, default=1 << 24, help="node ids (total over all ranks)")
    ap.add_argument("--q", type=int, default=65536, help="targets per step (total over all ranks)")
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--algo", choices=["batch", "index", "scan"], default="batch")
    ap.add_argument("--route", choices=["auto", "prefix", "broadcast"], default="auto")
    ap.add_argument("--sub-shards", type=int, default=0,
                    help="prefix route: split each rank's shard into this many prefix sub-shards (one "
                         "K6 context each, calls spread over the in-flight streams); 0 = auto, the "
                         "smallest power of two with <= 2^24 ids per sub-shard")
    ap.add_argument("--shard-index", choices=["local", "global"], default="local",
                    help="prefix shards: results as shard-local node indices (the rank owns its shard's "
                         "node table) or mapped to global stream indices (one gather per result)")
    ap.add_argument("--scaling", choices=["auto", "weak", "strong"], default="auto",
                    help="weak: --n/--q per GPU (global problem grows with N); strong: --n/--q global. "
                         "auto = weak for the prefix route, strong for broadcast")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="multi-rank correctness rehearsal on a one-GPU box: every rank on cuda:0, gloo "
                         "process group (timings are contended; not a scaling measurement)")
    ap.add_argument("--sharded", action="store_true",
                    help="use the multi-GPU code path (and its collectives) even with one rank")
    ap.add_argument("--simulate-world", type=int, default=0,
                    help="prefix route only: run rank --simulate-rank of a world of this size on one GPU")
    ap.add_argument("--simulate-rank", type=int, default=0)
    ap.add_argument("--cpu-targets", type=int, default=256, help="cpu_baseline sample (targets)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-scan", action="store_true", help="skip the reference K1 scan measurement (index algo)")
    ap.add_argument("--verify", type=int, default=16, help="targets re-checked against the oracle (rank 0)")
    ap.add_argument("--inflight", type=int, default=2,
                    help="batch algo: consecutive steps alternate over this many streams, so one step's "
                         "latency-bound F3/F4 overlaps the next step's HBM-bound F2 (1 = strictly serial)")
    return ap.parse_args()


PMC_FILE = "profiles/r01_batch/pmc_traffic.json"


def pmc_traffic(kernel, n, q, k):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 FETCH_SIZE/WRITE_SIZE passes
    (tools/pmc_traffic.py; gfx950 FETCH correction applied there), when they were taken on this
    workload (cfg 2 shape); None otherwise."""
    try:
        d = json.load(open(os.path.join(ROOT, PMC_FILE)))
    except (OSError, ValueError):
        return None
    if d.get("workload") != [n, q, k]:
        return None
    return d["kernels"].get(kernel, {}).get("traffic_bytes")


def oracle():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    return O


def cpu_baseline(ids, tg, k, threads):
    """Oracle (std::partial_sort with the restated InfoHash::xorCmp) on the host cores,
    over a bounded target sample of the same workload."""
    O = oracle()
    t0 = time.perf_counter()
    out, _ = O.topk(ids, tg, k, threads=threads)
    dt = time.perf_counter() - t0
    return {"value": tg.shape[0] / dt, "unit": "queries/s", "cores": threads, "kind": "port",
            "sample": f"{tg.shape[0]} targets x {ids.shape[0]} ids, k={k}, std::partial_sort(xorCmp) per target, "
                      f"{threads} threads, {dt:.2f} s wall"}, out


T_START = time.perf_counter()


def progress(msg):
    """Progress line on stderr (long setups and verifications keep the job visibly alive)."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench {time.perf_counter() - T_START:7.1f}s] {msg}", file=sys.stderr, flush=True)


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.rehearse_one_gpu:
        local = 0
    pow2 = lambda g: g > 0 and (g & (g - 1)) == 0
    route = a.route
    if route == "auto":
        route = "prefix" if (a.algo in ("index", "batch") and pow2(world)) else "broadcast"
    if a.simulate_world:
        assert world == 1 and route == "prefix" and pow2(a.simulate_world)
    scaling = a.scaling if a.scaling != "auto" else ("weak" if route == "prefix" else "strong")
    G_eff = a.simulate_world if a.simulate_world else world
    if scaling == "weak":   # --n / --q are per GPU: the global problem is G times larger
        a.n_total, a.q_total = a.n * G_eff, a.q * G_eff
    else:
        a.n_total, a.q_total = a.n, a.q
    use_dist = world > 1 or a.sharded
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        if a.rehearse_one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    tstream = torch.cuda.Stream(dev)              # every kernel and event of the bench runs here
    torch.cuda.set_stream(tstream)
    stream = tstream.cuda_stream
    L = opendht_amd.lib()
    ctx = opendht_amd.Context(local)

    G, R = (a.simulate_world, a.simulate_rank) if a.simulate_world else (world, rank)
    pbits = G.bit_length() - 1 if route == "prefix" else 0
    ts_all = (a.q_total + 63) // 64 * 64
    tp_all = torch.empty(5 * ts_all, dtype=torch.int32, device=dev)
    assert L.dhtgpu_gen_dev(a.seed + 1, 0, a.q_total, tp_all.data_ptr(), ts_all, stream) == 0
    S, sbits = 1, 0
    if route == "prefix":
        S = a.sub_shards
        if S <= 0:   # auto: K6 plans for <= 2^24 ids per context (n >> 2^24 has 256-id subtrees)
            S = 1
            while a.n_total // (G * S) > (1 << 24) and a.algo == "batch":
                S *= 2
        assert S & (S - 1) == 0, "--sub-shards must be a power of two"
        sbits = pbits + S.bit_length() - 1
        shards = []
        for s_i in range(S):
            c = ctx if s_i == 0 else opendht_amd.Context(local)
            if sbits:
                pv = R * S + s_i
                c.gen_ids_prefix(a.seed, a.n_total, sbits, pv)       # this (sub-)shard's ids
                c.set_global_indices(a.shard_index == "global")
                tps = torch.empty_like(tp_all)
                tg_s = torch.empty(ts_all, dtype=torch.int32, device=dev)
                q_s = c.select_prefix_dev(tp_all.data_ptr(), ts_all, a.q_total, sbits, pv, tps.data_ptr(), ts_all,
                                          tg_s.data_ptr(), stream)
            else:                                                 # one shard: the whole set
                c.gen_ids(a.seed, a.n_total)
                tps, q_s, tg_s = tp_all, a.q_total, None
            shards.append({"ctx": c, "tp": tps, "q": q_s, "tgidx": tg_s, "n": c.num_ids})
            progress(f"sub-shard {s_i}: {c.num_ids} ids, {q_s} targets")
        ts = ts_all
        shard_min = torch.tensor([min(sh["n"] for sh in shards)], dtype=torch.int64, device=dev)
        if use_dist:
            dist.all_reduce(shard_min, op=dist.ReduceOp.MIN)
        if int(shard_min.item()) < a.k:
            raise SystemExit("prefix route needs >= k ids per shard; rerun with --route broadcast")
        tp, q_local, tgidx = shards[0]["tp"], sum(sh["q"] for sh in shards), shards[0]["tgidx"]
        n_local = sum(sh["n"] for sh in shards)
        lo = 0
    else:
        lo, hi = sharding.shard_range(a.n_total, world, rank)
        ctx.gen_ids(a.seed, hi - lo, start=lo)      # this rank's contiguous slice of the global id stream
        tp, ts, q_local, tgidx = tp_all, ts_all, a.q_total, None
        n_local = hi - lo
        shards = [{"ctx": ctx, "tp": tp, "q": q_local, "tgidx": None, "n": n_local}]
    # the per-kernel diagnostics below time one K6 call on sub-shard 0
    q0, n0 = shards[0]["q"], shards[0]["n"]
    collective = use_dist and route == "broadcast"
    qk = max(q0, 1)
    out_idx = torch.empty((qk, a.k), dtype=torch.int32, device=dev)
    out_cnt = torch.empty(qk, dtype=torch.int32, device=dev)
    rec = torch.empty((a.q_total, a.k, 6), dtype=torch.int32, device=dev) if collective else None
    gathered = torch.empty((world * a.q_total, a.k, 6), dtype=torch.int32, device=dev) if collective else None

    def local_lookup(out_i, out_c, out_r, base, stream=stream, sh=None):
        sh = sh or shards[0]
        c, tps, qs = sh["ctx"], sh["tp"].data_ptr(), sh["q"]
        if a.algo == "batch":
            c.batch_topk_dev(tps, ts, qs, a.k, out_i, out_c, out_r, base, stream)
        elif a.algo == "index":
            c.index_build(stream)          # the index is rebuilt from the raw id planes every step
            c.index_topk_dev(tps, ts, qs, a.k, out_i, out_c, out_r, base, stream)
        else:
            c.topk_dev(tps, ts, qs, a.k, out_i, out_c, out_r, base, stream)

    # in-flight calls: call j (step i, sub-shard s: j = i * S + s) runs on stream j % D with
    # its own output buffers
    D = max(1, a.inflight) if (a.algo == "batch" and not collective) else 1
    streams = [tstream] + [torch.cuda.Stream(dev) for _ in range(D - 1)]
    outs = [[(out_idx, out_cnt) if (si == 0 and d == 0) else
             (torch.empty((max(sh["q"], 1), a.k), dtype=torch.int32, device=dev),
              torch.empty(max(sh["q"], 1), dtype=torch.int32, device=dev)) for d in range(D)]
            for si, sh in enumerate(shards)]
    step_no = [0]

    def step():
        i = step_no[0]
        step_no[0] += 1
        if not collective:
            for si, sh in enumerate(shards):
                j = i * len(shards) + si
                oi, oc = outs[si][j % D]
                local_lookup(oi.data_ptr(), oc.data_ptr(), None, 0, streams[j % D].cuda_stream, sh)
        else:
            local_lookup(None, None, rec.data_ptr(), lo)
            sharding.gather_records(rec, out=gathered)
            assert L.dhtgpu_merge_dev(gathered.data_ptr(), world, a.q_total, a.k, tp.data_ptr(), ts, a.k,
                                      out_idx.data_ptr(), out_cnt.data_ptr(), stream) == 0

    progress(f"setup done: {n_local} ids, {q_local} targets on this rank; warmup")
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(a.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ev_ms = ev0.elapsed_time(ev1) / a.steps
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if use_dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall = float(t.item())
    ms_per_step = wall * 1e3 / a.steps
    # outputs of the last timed step (for the verification below), per sub-shard
    got = []
    for si, sh in enumerate(shards):
        j = (step_no[0] - 1) * len(shards) + si
        gi = outs[si][j % D][0][:sh["q"]].cpu().numpy().view(np.uint32).copy()
        gt = sh["tgidx"][:sh["q"]].cpu().numpy().view(np.uint32).copy() if sh["tgidx"] is not None \
            else np.arange(sh["q"])
        got.append((gi, gt))

    def ev_time(fn, reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    progress(f"timed {a.steps} steps: {ms_per_step:.4f} ms/step; diagnostics")
    reps = max(3, min(a.steps, 20))
    # single-batch latency: the same step strictly serial on one stream
    lat_ms = ev_time(lambda: local_lookup(out_idx.data_ptr(), out_cnt.data_ptr(), None, 0), reps) \
        if not collective else None
    lat_global_ms = None
    if route == "prefix" and sbits and a.shard_index == "local":
        # the same batch with results mapped to global stream indices (for comparison)
        ctx.set_global_indices(True)
        lat_global_ms = ev_time(lambda: local_lookup(out_idx.data_ptr(), out_cnt.data_ptr(), None, 0), reps)
        ctx.set_global_indices(False)
    if a.algo == "batch":
        # per-kernel device times (HIP events between F1..F4 on the bench stream)
        runs = [ctx.batch_topk_timed(tp.data_ptr(), ts, q0, a.k, out_idx.data_ptr(), out_cnt.data_ptr(), stream)
                for _ in range(reps)]
        ph = [sum(r[0][i] for r in runs) / reps for i in range(4)]
        n_fb, surv, n_slow = runs[-1][1], runs[-1][2], runs[-1][3]
        kern = {"k_f1_targets": (ph[0], 12 * q0),
                "k_f2_filter": (ph[1], 4 * n0 + 8 * surv),
                "k_f3_answer": (ph[2], 8 * surv + q0 * (8 + 16 + 4 * a.k + 4)),
                "k_f4_fallback": (ph[3], 0)}
        dom = max(kern, key=lambda k: kern[k][0])
        dom_ms, dom_bytes = kern[dom]
        step_bytes = sum(v[1] for v in kern.values()) * len(shards)   # sub-shard 0's bytes x S
        tb = pmc_traffic(dom, n0, q0, a.k)
        roof = {"bound": "hbm", "achieved": dom_bytes / (dom_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": dom_bytes / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "traffic": tb / (dom_ms * 1e-3) / 1e9 if tb else None,
                "traffic_bytes_per_launch": tb, "traffic_source": PMC_FILE if tb else None,
                "kernel": dom, "kernel_ms": dom_ms, "alg_bytes_per_launch": dom_bytes,
                "kernels_ms": {k: v[0] for k, v in kern.items()},
                "step_alg_bytes": step_bytes,
                "step_hbm_frac": step_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                # SURVEY 8(d) contract bytes (every id read whole, 20 B) and their time at peak
                "contract_bytes": n_local * 20 + q_local * 20 + q_local * a.k * 4,
                "contract_floor_ms": (n_local * 20 + q_local * 20 + q_local * a.k * 4) / HBM_PEAK_GBS / 1e6}
        extra = {"survivors": surv, "survivor_frac": surv / max(n0, 1), "fallback_targets": n_fb,
                 "wave_path_targets": n_slow}
    elif a.algo == "index":
        # per-kernel device times of the index build (HIP events between its kernels, on
        # the bench stream) and of the query kernel alone
        phases = [ctx.index_build_timed(stream) for _ in range(reps)]
        ph = [sum(p[i] for p in phases) / reps for i in range(4)]
        q_ms = ev_time(lambda: ctx.index_topk_dev(tp.data_ptr(), ts, q0, a.k, out_idx.data_ptr(),
                                                  out_cnt.data_ptr(), None, 0, stream), reps)
        kern = {"k_p0_hist": (ph[0], 4 * n0), "k_p0_scans": (ph[1], 0),
                "k_p1_scatter": (ph[2], 12 * n0), "k_p2_buckets": (ph[3], 16 * n0),
                "k_query": (q_ms, q0 * (20 + a.k * 4))}
        dom = max(kern, key=lambda k: kern[k][0])
        dom_ms, dom_bytes = kern[dom]
        step_bytes = n0 * (4 + 8) + q0 * (20 + a.k * 4)
        roof = {"bound": "hbm", "achieved": dom_bytes / (dom_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": dom_bytes / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": None,
                "kernel": dom, "kernel_ms": dom_ms, "alg_bytes_per_launch": dom_bytes,
                "kernels_ms": {k: v[0] for k, v in kern.items()},
                "step_alg_bytes": step_bytes,
                "step_hbm_frac": step_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS}
        extra = {"query_only_qps_per_gpu": q0 / (q_ms * 1e-3), "index_build_ms": sum(ph)}
    else:
        kern_ms = ev_ms
        if collective:
            kern_ms = ev_time(lambda: local_lookup(None, None, rec.data_ptr(), lo), reps)
        pairs = q0 * n0
        achieved = OPS_PER_PAIR * pairs / (kern_ms * 1e-3) / 1e12
        roof = {"bound": "valu", "achieved": achieved, "peak": VALU_PEAK_TOPS, "unit": "TOP/s",
                "frac": achieved / VALU_PEAK_TOPS, "traffic": None,
                "kernel": "k_scan (K1 xor_topk_scan)", "kernel_ms": kern_ms,
                "ops_per_pair": OPS_PER_PAIR, "pairs_per_launch": pairs,
                "hbm_alg_bytes_per_launch": n0 * 20 + q0 * 20 + q0 * a.k * 4}
        extra = {}
    if a.algo != "scan" and not a.no_scan and world == 1 and not a.simulate_world:
        # the north-star brute-force scan (K1) on the same inputs, for reference
        sc_ms = ev_time(lambda: ctx.topk_dev(tp.data_ptr(), ts, q0, a.k, out_idx.data_ptr(),
                                             out_cnt.data_ptr(), None, 0, stream), 3)
        ach = OPS_PER_PAIR * q0 * n0 / (sc_ms * 1e-3) / 1e12
        extra["scan_k1"] = {"qps": q0 / (sc_ms * 1e-3), "kernel_ms": sc_ms, "bound": "valu",
                            "achieved_TOPs": ach, "peak_TOPs": VALU_PEAK_TOPS, "frac": ach / VALU_PEAK_TOPS}

    if rank == 0:
        par = {"prefix": f"prefix-routed shards x{G} (top {pbits} id bits"
                         + (f", {len(shards)} prefix sub-shards per GPU" if len(shards) > 1 else "")
                         + "; no data-path collective)",
               "broadcast": f"id-range shards x{world}" + (" + RCCL all-gather + K3 merge" if collective else "")}[route]
        res = {
            "metric": METRIC,
            "value": (a.q_total if not a.simulate_world else q_local) / (ms_per_step * 1e-3),
            "unit": "queries/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: splitmix64 ids and targets generated in HBM (SURVEY 8(d) spec)",
            "config": {"workload": ("cfg2" if (a.n, a.q) == (1 << 24, 65536) else "custom") + f" batched k-NN: {a.q} targets x {a.n} ids (2^{a.n.bit_length()-1}), k={a.k}"
                                   + (f" per GPU ({a.q_total} x {a.n_total} over {G_eff} GPUs)" if scaling == "weak" and G_eff > 1
                                      else ""),
                       "n_ids": a.n_total, "n_targets": a.q_total, "k": a.k, "algo": a.algo, "route": route,
                       "ids_per_gpu": n_local, "targets_per_gpu": q_local, "parallelism": par,
                       "inflight": D, "sub_shards": len(shards),
                       "result_indices": ("shard-local" if a.shard_index == "local" else "global")
                       if route == "prefix" and sbits else "global"},
            "latency_ms_per_batch": lat_ms,
            "roofline": roof,
        }
        if len(shards) > 1:
            res["sub_shard_note"] = (f"each rank's shard is split into {len(shards)} prefix sub-shards (one K6 context "
                                     f"each); kernels_ms / latency time one call on sub-shard 0 "
                                     f"({n0} ids, {q0} targets)")
        if lat_global_ms is not None:
            res["latency_ms_per_batch_global_indices"] = lat_global_ms
        if a.simulate_world:
            res["simulated"] = f"rank {R} of {G} on one GPU; value = this rank's targets / its step time"
        res.update(extra)
        # spot check of this run's output against the oracle (rank 0), and the cpu_baseline
        # leg (rank 0, N = 1 only)
        if not a.no_cpu and (a.verify or world == 1):
            progress("verifying against the oracle")
            O = oracle()
            nv = min(q_local, max(a.verify, a.cpu_targets if world == 1 else 0))
            tg_all = O.gen_ids(a.seed + 1, a.q_total)
            local_ix = route == "prefix" and sbits and a.shard_index == "local"
            ok, nver = True, 0
            if not local_ix:
                ids_all = O.gen_ids(a.seed, a.n_total)
            for si, sh in enumerate(shards):
                gi, gt = got[si]
                ns = min(sh["q"], max(1, nv // len(shards)))
                tg = tg_all[gt[:ns]]
                # shard-local results: the oracle over this (sub-)shard's own ids, read back
                # from the device -- the set the call answers from, same index space
                ids = sh["ctx"].get_ids() if local_ix else ids_all
                if si == 0 and world == 1 and not a.simulate_world:
                    cb, want = cpu_baseline(ids, tg, a.k, a.cpu_threads)
                    res["cpu_baseline"] = cb
                else:
                    want, _ = O.topk(ids, tg, a.k, threads=a.cpu_threads)
                ok = ok and bool(np.array_equal(gi[:ns], want))
                nver += ns
                del ids
            res["verified_targets"] = int(nver)
            res["verified_exact"] = ok
            progress("verified")
        print(json.dumps(res), flush=True)
    ctx.close()
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
