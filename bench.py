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
No result or intermediate of a step is reused by the next one.  Persistent per-set state (built
once per id set, outside the timed steps): the w0..w4 planes (20 B/id) and, for sets
one K6 plan cannot serve (the cfg-3 shard), their prefix sub-partitions (28 B/id).

Multi-GPU (one process per GPU, torch.distributed over RCCL; --route):
  broadcast  (default for N > 1; SURVEY §8(e) north-star scheme) the metric's own workload,
             strong scaling: the 2^24 cfg-2 ids range-sharded over the ranks, all 65,536 targets
             on every rank, K6 in record mode per rank (k candidate records of 12 B per target),
             one RCCL exchange (--exchange allgather: all_gather_into_tensor, every rank merges
             every target; alltoall: all_to_all_single by target slice, each rank merges its
             q / N targets), K3 merge.  value = the 65,536 targets / the slowest rank's step.
             Consecutive steps rotate over --inflight streams, so one step's exchange overlaps
             the next step's K6.  The other exchange and the prefix route are measured beside
             it (extra: broadcast_<exchange>, prefix_strong -- the same problem on the prefix
             route -- and prefix_weak), each labelled.
  prefix     ids AND targets are partitioned by their top log2(N) bits; each rank answers only
             its own targets from its own shard.  If every shard holds >= k ids, a target's
             top-k provably lies in its own prefix subtree, so the data path needs no
             collective; the setup checks the minimum shard size with one all-reduce.
Scaling (--scaling): "strong" (default with the broadcast route: --n and --q are global
totals) or "weak" (default with the prefix route: every rank keeps the one-GPU workload --
--n ids and --q targets per GPU out of a global problem N times as large; value = all ranks'
targets / the slowest rank's time).  N = 1 runs the one-GPU K6 over the whole set.

Beside the headline (`value`) the line carries, measured in the same run:
  roofline        F2 (the dominant K6 kernel) timed by events its own dispatches record over
                  serial calls after the timed steps; roofline_hbm: the same kernel with the Infinity Cache
                  evicted before each call (the cfg-2 working set otherwise stays in L3)
  small_batch     Q = 1 / 8 / 32 / 64 targets over the same ids (HBM-bound latency mode, KS path)
  find_closest    RoutingTable::findClosestNodes drop-in on a cfg-1-shaped table
  cfg3_shard      one GPU's shard of BASELINE cfg 3 (2^27 ids, 131,072 targets; the library
                  splits it into prefix sub-partitions) -- its w0 planes (537 MB) exceed L3;
                  `handles`: the same calls returning sub-partition handles
  cfg4 / cfg5     classification of 10^8 ids; iterative searches over 5*10^7 nodes
  cfg3 (N > 1)    BASELINE cfg 3 itself over the ranks: 10^9 ids, 2^20 targets, both routes
  cpu_baseline    the oracle port on the host cores (rank 0, N = 1): every host CPU and 1 core;
                  cfg 1 (findClosestNodes on an onNewNode-grown table), cfg 2 (partial_sort),
                  cfg 4 (findBucket + commonBits), getCachedNodes
Prints ONE JSON line on rank 0.
"""
import argparse
import bisect
import ctypes
import json
import os
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); N > 1 outside torch.distributed.run re-launches itself under it")
    ap.add_argument("--dry-run", action="store_true", help="print the launch plan and exit (no GPU)")
    ap.add_argument("--dry-run-ranks", action="store_true",
                    help="launch the ranks for real; each prints its identity and exits (no GPU)")
    ap.add_argument("--steps", type=int, default=1000)   # ~40 ms timed: steady state, not ramp-up
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--n", type=int, default=1 << 24, help="node ids (per GPU with weak scaling)")
    ap.add_argument("--q", type=int, default=65536, help="targets per step (per GPU with weak scaling)")
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--algo", choices=["batch", "index", "scan"], default="batch")
    ap.add_argument("--route", choices=["auto", "prefix", "broadcast"], default="auto",
                    help="auto = broadcast for N > 1 (the metric's workload, strong scaling), the whole set at N = 1")
    ap.add_argument("--exchange", choices=["allgather", "alltoall"], default="allgather",
                    help="broadcast route: RCCL all-gather of the candidate records (north star) or all-to-all by "
                         "target slice")
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
    ap.add_argument("--cpu-targets", type=int, default=256, help="cpu_baseline sample (targets, all host threads)")
    ap.add_argument("--cpu-threads", type=int, default=os.cpu_count() or 1,
                    help="cpu_baseline threads (default: every host CPU, nproc; the rate at the job's cgroup CPU "
                         "quota and the single-core figures are reported too)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the extra legs (small batch, cfg 1/3/4/5)")
    ap.add_argument("--no-scan", action="store_true", help="skip the reference K1 scan measurement")
    ap.add_argument("--verify", type=int, default=16, help="targets re-checked against the oracle (rank 0)")
    ap.add_argument("--inflight", type=int, default=3,
                    help="batch algo: consecutive steps rotate over this many streams, so one step's "
                         "latency-bound F3/F4 overlaps the other steps' HBM-bound F2 (1 = strictly serial; "
                         "3 measured best: 2 leaves each stream's F1-F4 chain exposed, 4 over-subscribes F2); "
                         "broadcast route: one step's exchange + merge overlap the next step's K6")
    return ap.parse_args(argv)


def run_plan(a, world):
    """The workload a run measures (pure: tests/test_bench_launch.py asserts the defaults).
    N > 1 defaults to the metric's own workload -- 2^24 ids and 65,536 targets in TOTAL -- on
    the broadcast route (SURVEY §8(e) north star) with strong scaling; N = 1 is the one-GPU K6
    over the whole set (one range shard, no collective): the first point of the same strong-scaling
    series."""
    pow2 = lambda g: g > 0 and (g & (g - 1)) == 0
    route = a.route
    if route == "auto":   # N = 1: one range shard = the whole set, no collective
        route = "broadcast"
    if route == "prefix" and not pow2(a.simulate_world or world):
        raise SystemExit("the prefix route needs a power-of-two world")
    scaling = a.scaling if a.scaling != "auto" else ("weak" if route == "prefix" else "strong")
    G = a.simulate_world if a.simulate_world else world
    n_total, q_total = (a.n * G, a.q * G) if scaling == "weak" else (a.n, a.q)
    return {"route": route, "scaling": scaling, "world": G, "n_total": n_total, "q_total": q_total,
            "exchange": a.exchange if route == "broadcast" and (world > 1 or a.sharded) else None}


def launcher_cmd(gpus, argv):
    """`python bench.py --gpus N` (N > 1) started as ONE process: the command that runs it as N
    ranks, one per GPU (torch.distributed.run, 127.0.0.1 rendezvous on a free port).  Built and
    started before anything touches the GPU (this process never initialises HIP)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def maybe_launch(argv):
    """--gpus N > 1 without a torch.distributed environment: start the N-rank job as a child
    process and return its exit code (None: this process is a rank, or N == 1).  --dry-run
    prints what would run (the launcher command, or this rank's identity) and exits;
    --dry-run-ranks starts the N ranks for real and each prints its identity (no GPU)."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=1)
    pre.add_argument("--dry-run", action="store_true")
    pre.add_argument("--dry-run-ranks", action="store_true")
    a, _ = pre.parse_known_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if a.gpus > 1 and env_world is None:
        cmd = launcher_cmd(a.gpus, argv)
        if a.dry_run and not a.dry_run_ranks:
            print(json.dumps({"mode": "launcher", "gpus": a.gpus, "cmd": cmd,
                              "env": {k: os.environ.get(k) for k in ("HSA_ENABLE_IPC_MODE_LEGACY",)}}))
            return 0
        print(f"[bench] --gpus {a.gpus}: launching {a.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
        return subprocess.call(cmd)
    if a.dry_run or a.dry_run_ranks:
        # one write of line + newline: the ranks share the launcher's stdout pipe, and a write
        # under PIPE_BUF bytes is atomic there (print's separate newline write could interleave)
        world = int(env_world or 1)
        line = json.dumps({"mode": "rank" if env_world is not None else "single", "gpus": a.gpus,
                           "world_size": world, "rank": int(os.environ.get("RANK", "0")),
                           "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                           "plan": run_plan(parse(argv), world)}) + "\n"
        os.write(sys.stdout.fileno(), line.encode())
        return 0
    return None


if __name__ == "__main__":
    _rc = maybe_launch(sys.argv[1:])
    if _rc is not None:
        sys.exit(_rc)
# Hardware queues: HIP's default (4 per process, shared round-robin by the streams) is kept.
# Measured: 8 queues leave the cfg-2 step unchanged (40.6-41.0 vs 40.8-40.9 us) and make the
# sub-partitioned cfg-3 shard 1.7x slower (0.60 vs 0.35 ms per call with two calls in flight).
# DHT_BENCH_HW_QUEUES overrides it for experiments.
if os.environ.get("DHT_BENCH_HW_QUEUES"):
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ["DHT_BENCH_HW_QUEUES"]

import numpy as np  # noqa: E402

_RESULT_FD = 1   # the JSON line's descriptor (the original stdout when run as a script)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import opendht_amd  # noqa: E402
from opendht_amd import sharding  # noqa: E402

METRIC = "queries/sec, k=8 XOR-NN over 16M 160-bit IDs; % HBM roofline at 1/2/4/8 GPUs"
# int32 VALU peak: a wave64 integer VALU op issues every 4 cycles per SIMD on gfx950
# (16 lanes/clk/SIMD): 1024 SIMDs x 16 x 2.4 GHz = 39.3 T lane-ops/s; tools/experiments/valu_peak
# measures 40.1 T on the box (profiles/r01_valu_peak.log).
VALU_PEAK_TOPS = 1024 * 16 * 2.4e9 / 1e12
HBM_PEAK_GBS = 8000.0
# Algorithmic VALU work per (id, target) pair in K1: the XOR distance and the running-min
# select, done two pairs at a time on packed top-16-bit words (v_xor_b32 + v_pk_min_u16
# per two pairs) = 1 lane-op per pair.  SURVEY 8(d)'s contract counts 3 ops/pair on a
# 64-bit lane; both fractions are reported (the packed prefilter is an algorithmic win).
OPS_PER_PAIR = 1.0
SURVEY_OPS_PER_PAIR = 3.0
PMC_FILE = "profiles/r06/pmc_traffic.json"


def oracle():
    """The CPU restatement (test infrastructure): only the verification and cpu_baseline legs."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    return O


T_START = time.perf_counter()


def progress(msg):
    """Progress line on stderr (long setups and verifications keep the job visibly alive)."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench {time.perf_counter() - T_START:7.1f}s] {msg}", file=sys.stderr, flush=True)


def pmc_traffic(workload, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 FETCH_SIZE/WRITE_SIZE passes
    (tools/pmc_traffic.py, gfx950 FETCH correction applied there) for `workload`; None if absent."""
    try:
        d = json.load(open(os.path.join(ROOT, PMC_FILE)))
    except (OSError, ValueError):
        return None
    w = d.get("workloads", {}).get(workload)
    if w is None:
        return None
    # a K6 phase's kernels: F1 is k_f1_targets or (batches >= 2^18) k_f1_coarse + k_f1_fine; F2 is
    # k_f2_filter or (prefix-sorted sub-partitions) k_f2_direct
    parts = K6_PHASE_KERNELS.get(kernel, (kernel,))
    got = [w[kn]["traffic_bytes"] for kn in parts if kn in w]
    return sum(got) if got else None


K6_PHASE_KERNELS = {"k_f1_targets": ("k_f1_targets", "k_f1_coarse", "k_f1_fine"),
                    "k_f2_filter": ("k_f2_filter", "k_f2_direct")}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def usable_cpus():
    """CPUs this process can keep busy: its affinity set, capped by the cgroup CPU quota (a GPU
    box's job gets 16 CPUs of time on a 256-CPU host: 256 threads there only time-slice)."""
    sh = cpu_share()
    n = sh.get("affinity_cpus") or os.cpu_count() or 1
    q = sh.get("cgroup_cpu_quota")
    return max(1, min(n, int(q + 0.5))) if q else n


def cpu_share():
    """The CPUs this process may actually run on: its affinity set and the cgroup CPU quota
    (a GPU box shares the host; os.cpu_count() reports the whole machine)."""
    out = {}
    try:
        out["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        out["cgroup_cpu_quota"] = None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    return out


class EvSets:
    """Per-call kernel timing: 8 events (F1..F4 start/stop) armed on a K6 call, recorded by the
    kernels' own dispatches (no synchronisation inside the timed region)."""

    def __init__(self, count, stream):   # stream: a torch.cuda.Stream
        self.sets = [[torch.cuda.Event(enable_timing=True) for _ in range(8)] for _ in range(count)]
        for s in self.sets:   # materialise the HIP events
            for e in s:
                e.record(stream)
        self.used = 0

    def arm(self, ctx):
        ctx.batch_events(self.sets[self.used])
        self.used += 1

    def mean_ms(self):
        """mean duration of F1..F4 over the armed calls (synchronises)."""
        torch.cuda.synchronize()
        acc = [0.0] * 4
        for s in self.sets[: self.used]:
            for i in range(4):
                acc[i] += s[2 * i].elapsed_time(s[2 * i + 1])
        return [a / max(self.used, 1) for a in acc]

    def median_ms(self):
        """median duration of F1..F4 over the armed calls (synchronises)."""
        torch.cuda.synchronize()
        return [float(np.median([s[2 * i].elapsed_time(s[2 * i + 1]) for s in self.sets[: self.used]]))
                for i in range(4)]


def ev_time(fn, reps, stream=None):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def gen_targets(L, seed, q, dev, stream):
    ts = (q + 63) // 64 * 64
    tp = torch.empty(5 * ts, dtype=torch.int32, device=dev)
    assert L.dhtgpu_gen_dev(seed, 0, q, tp.data_ptr(), ts, stream) == 0
    return tp, ts


def k6_kernels(ms, n, q, k, surv):
    """Algorithmic bytes per launch of the four K6 kernels."""
    return {"k_f1_targets": (ms[0], 12 * q), "k_f2_filter": (ms[1], 4 * n + 8 * surv),
            "k_f3_answer": (ms[2], 8 * surv + q * (8 + 16 + 4 * k + 4)), "k_f4_fallback": (ms[3], 0)}


def grow_table(myid, ids):
    """The RoutingTable a node with id `myid` holds after learning `ids` in order: onNewNode
    (src/routing_table.cpp:204-262) with every node good -- insert into findBucket's bucket
    (:153-166) while it holds < TARGET_NODES = 8, else split it (:169-200, depth :100-107) if it
    contains myid and retry, else drop the node.  Node order inside a bucket follows the
    reference's std::list splices (emplace_front on insert, splice-to-front on split).  The
    bench's workload generator (host logic on the input side); returns the snapshot the C ABI
    takes: bucket firsts (nb, 20), bucket offsets (nb + 1), node ids (m, 20)."""
    me = int.from_bytes(bytes(myid), "big")
    firsts, nodes = [0], [[]]
    lowbit = lambda x: 160 - (x & -x).bit_length() if x else -1      # infohash.h:132-143
    for row in ids:
        x = int.from_bytes(bytes(row), "big")
        while True:
            b = bisect.bisect_right(firsts, x) - 1
            if x in nodes[b]:
                break
            if len(nodes[b]) < 8:
                nodes[b].insert(0, x)
                break
            nxt = firsts[b + 1] if b + 1 < len(firsts) else None
            if not (firsts[b] <= me and (nxt is None or me < nxt)):
                break                                   # not my bucket: the node is cached away
            bit = max(lowbit(firsts[b]), lowbit(nxt) if nxt is not None else -1) + 1
            if bit >= 160:
                break
            firsts.insert(b + 1, firsts[b] | (1 << (159 - bit)))
            moved, nodes[b] = nodes[b], []
            nodes.insert(b + 1, [])
            for v in moved:                              # splice each to the front of its bucket
                nodes[bisect.bisect_right(firsts, v) - 1].insert(0, v)
    off = np.zeros(len(firsts) + 1, np.uint32)
    off[1:] = np.cumsum([len(v) for v in nodes])
    to_u8 = lambda vals: np.frombuffer(b"".join(v.to_bytes(20, "big") for v in vals) or b"",
                                       dtype=np.uint8).reshape(-1, 20).copy()
    return to_u8(firsts), off, to_u8([v for bn in nodes for v in bn])


def cfg1_table(seed):
    """BASELINE cfg 1's table: 10,000 random ids learned by one node."""
    rng = np.random.default_rng(seed)
    myid = np.frombuffer(rng.bytes(20), dtype=np.uint8).copy()
    ids = np.frombuffer(rng.bytes(20 * 10000), dtype=np.uint8).reshape(-1, 20)
    return (myid,) + grow_table(myid, ids)


def cfg4_firsts(seed):
    """The bucket firsts of a table grown from 10^5 random ids (SURVEY 8(d) cfg 4)."""
    rng = np.random.default_rng(seed)
    myid = np.frombuffer(rng.bytes(20), dtype=np.uint8).copy()
    firsts, _, _ = grow_table(myid, np.frombuffer(rng.bytes(20 * 100000), dtype=np.uint8).reshape(-1, 20))
    return myid, firsts


def l3_evict(buf):
    """Read 512 MiB (twice the Infinity Cache; a read leaves no dirty lines to write back during
    the next kernel): the next kernel reads the id set from HBM."""
    return buf.sum()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.rehearse_one_gpu:
        local = 0
    if a.simulate_world:
        assert world == 1 and a.route == "prefix", "--simulate-world runs one rank of the prefix route"
    plan = run_plan(a, world)
    route, scaling, G_eff = plan["route"], plan["scaling"], plan["world"]
    a.n_total, a.q_total = plan["n_total"], plan["q_total"]
    use_dist = world > 1 or a.sharded
    if use_dist:
        os.environ["NCCL_DEBUG"] = os.environ.get("DHT_BENCH_NCCL_DEBUG", "WARN")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        if a.rehearse_one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if use_dist and not a.rehearse_one_gpu:
        world = dist.get_world_size()          # the RCCL communicator's own count
    if world != a.gpus and not a.rehearse_one_gpu:
        progress(f"note: --gpus {a.gpus} but the process group has {world} ranks; n_gpus reports {world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    tstream = torch.cuda.Stream(dev)              # every kernel and event of the bench runs here
    torch.cuda.set_stream(tstream)
    stream = tstream.cuda_stream
    L = opendht_amd.lib()
    ctx = opendht_amd.Context(local)

    G, R = (a.simulate_world, a.simulate_rank) if a.simulate_world else (world, rank)
    pbits = G.bit_length() - 1 if route == "prefix" else 0
    tp_all, ts = gen_targets(L, a.seed + 1, a.q_total, dev, stream)
    if route == "prefix":
        if pbits:
            ctx.gen_ids_prefix(a.seed, a.n_total, pbits, R)       # this rank's prefix shard
            ctx.set_global_indices(a.shard_index == "global")
            tp = torch.empty_like(tp_all)
            tgidx = torch.empty(ts, dtype=torch.int32, device=dev)
            q_local = ctx.select_prefix_dev(tp_all.data_ptr(), ts, a.q_total, pbits, R, tp.data_ptr(), ts,
                                            tgidx.data_ptr(), stream)
        else:
            ctx.gen_ids(a.seed, a.n_total)
            tp, q_local, tgidx = tp_all, a.q_total, None
        n_local = ctx.num_ids
        shard_min = torch.tensor([n_local], dtype=torch.int64, device=dev)
        if use_dist:
            dist.all_reduce(shard_min, op=dist.ReduceOp.MIN)
        if int(shard_min.item()) < a.k:
            raise SystemExit("prefix route needs >= k ids per shard; rerun with --route broadcast")
        lo = 0
    else:
        lo, hi = sharding.shard_range(a.n_total, world, rank)
        ctx.gen_ids(a.seed, hi - lo, start=lo)      # this rank's contiguous slice of the global id stream
        tp, q_local, tgidx = tp_all, a.q_total, None
        n_local = hi - lo
    collective = use_dist and route == "broadcast"
    a2a = collective and plan["exchange"] == "alltoall"
    # alltoall: this rank merges (and owns the results of) targets [tlo, thi)
    tlo, thi = sharding.shard_range(a.q_total, world, rank) if a2a else (0, a.q_total)
    q_out = thi - tlo if collective else q_local
    qk = max(q_out, 1)

    def local_lookup(out_i, out_c, out_r, base, s=stream):
        if a.algo == "batch":
            ctx.batch_topk_dev(tp.data_ptr(), ts, q_local, a.k, out_i, out_c, out_r, base, s)
        elif a.algo == "index":
            ctx.index_build(s)          # the index is rebuilt from the raw id planes every step
            ctx.index_topk_dev(tp.data_ptr(), ts, q_local, a.k, out_i, out_c, out_r, base, s)
        else:
            ctx.topk_dev(tp.data_ptr(), ts, q_local, a.k, out_i, out_c, out_r, base, s)

    # in-flight calls: step i runs on stream i % D with its own buffers (broadcast route: K6 of
    # step i + 1 runs while step i's records cross xGMI -- RCCL orders its collectives on its own
    # stream after each step's K6, and the merge waits for its collective)
    D = max(1, a.inflight) if a.algo == "batch" else 1
    streams = [tstream] + [torch.cuda.Stream(dev) for _ in range(D - 1)]
    outs = [(torch.empty((qk, a.k), dtype=torch.int32, device=dev), torch.empty(qk, dtype=torch.int32, device=dev))
            for _ in range(D)]
    out_idx, out_cnt = outs[0]
    # the diagnostics' one-rank calls answer all q_local targets (alltoall: more rows than q_out)
    dg_idx, dg_cnt = (out_idx, out_cnt) if q_out >= q_local else \
        (torch.empty((max(q_local, 1), a.k), dtype=torch.int32, device=dev),
         torch.empty(max(q_local, 1), dtype=torch.int32, device=dev))
    RW = sharding.REC_WORDS
    recs = [torch.empty((a.q_total, a.k, RW), dtype=torch.int32, device=dev) for _ in range(D)] if collective else None
    rec = recs[0] if collective else None
    xbufs = [torch.empty((world * q_out, a.k, RW), dtype=torch.int32, device=dev) for _ in range(D)] \
        if collective else None
    txs = [sharding.TieExchange(world, a.k, dev) for _ in range(D)] if collective else None
    ops = sharding.LibOps(L, ctx, tp.data_ptr(), ts)
    step_no = [0]

    def exchange_merge(r, xb, oi, oc, s, tx):
        """the records of every rank for this rank's merged targets, then K3 and the tie exchange
        (words 2..4 of the candidates in rows whose records tie on 64 bits; same stream)"""
        if a2a:
            ex = sharding.exchange_records(r, out=xb)
            sharding.merge_alltoall(ops, r, ex, a.k, tlo, oi, oc, tx, lo, s)
        else:
            g = sharding.gather_records(r, out=xb)
            sharding.merge_allgather(ops, r, g, a.k, oi, oc, tx, lo, s)

    def settle(r, xb, oi, oc, s, tx):
        """after a sync: the every-row settlement if more rows tied than one tie exchange takes"""
        if a2a:
            ex = xb.view(world, q_out, a.k, RW)
            return sharding.settle_overflow_alltoall(ops, r, ex, a.k, tlo, oi, oc, tx, lo, s)
        g = xb.view(world, a.q_total, a.k, RW)
        return sharding.settle_overflow_allgather(ops, r, g, a.k, oi, oc, tx, lo, s)

    def step():
        i = step_no[0]
        step_no[0] += 1
        oi, oc = outs[i % D]
        st_ = streams[i % D]
        if not collective:
            local_lookup(oi.data_ptr(), oc.data_ptr(), None, 0, st_.cuda_stream)
        else:
            # the collective runs after this stream's K6 (RCCL orders itself after the current
            # stream; set directly: the stream context manager costs ~6 us of host time per step)
            torch.cuda.set_stream(st_)
            local_lookup(None, None, recs[i % D].data_ptr(), lo, st_.cuda_stream)
            exchange_merge(recs[i % D], xbufs[i % D], oi, oc, st_.cuda_stream, txs[i % D])

    progress(f"setup done: {n_local} ids, {q_local} targets on this rank; warmup")
    for _ in range(a.warmup):
        step()
    torch.cuda.set_stream(tstream)
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    # diagnostic: the same window on the GPU's clock (first kernel enqueued .. last stream done),
    # against which the host wall below adds the launch of the first step and the wake-up of
    # the final synchronize
    w_beg, w_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    w_beg.record(streams[0])
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    t_enq = time.perf_counter() - t0   # host time to enqueue the K steps (diagnostic)
    torch.cuda.set_stream(tstream)
    for st_ in streams[1:]:
        streams[0].wait_stream(st_)
    w_end.record(streams[0])
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if use_dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall = float(t.item())
    ms_per_step = wall * 1e3 / a.steps
    last = (step_no[0] - 1) % D
    tie_rows = None
    if collective:   # every in-flight slot's last step: rows the tie exchange settled (the same inputs every step)
        tie_rows = []
        for d in range(min(D, step_no[0])):
            torch.cuda.set_stream(streams[d])   # the settlement's collectives order after its stream
            tie_rows.append(settle(recs[d], xbufs[d], outs[d][0], outs[d][1], streams[d].cuda_stream, txs[d]))
        torch.cuda.set_stream(tstream)
        torch.cuda.synchronize()
    got_idx = outs[last][0][:q_out].cpu().numpy().view(np.uint32).copy()
    got_tg = tgidx[:q_local].cpu().numpy().view(np.uint32).copy() if tgidx is not None \
        else np.arange(tlo, tlo + q_out)
    progress(f"timed {a.steps} steps: {ms_per_step:.4f} ms/step; diagnostics")
    reps = max(3, min(a.steps, 20))
    res = {}
    extra = {}
    # single-batch latency: the same step strictly serial on one stream (broadcast route: K6 in
    # record mode + the exchange + K3 on every rank)
    if collective:
        if use_dist:
            dist.barrier()
        lat_ms = ev_time(lambda: (local_lookup(None, None, rec.data_ptr(), lo),
                                  exchange_merge(rec, xbufs[0], out_idx, out_cnt, stream, txs[0])), reps, tstream)
    else:
        lat_ms = ev_time(lambda: local_lookup(out_idx.data_ptr(), out_cnt.data_ptr(), None, 0), reps, tstream)
    if route == "prefix" and pbits and a.shard_index == "local":
        ctx.set_global_indices(True)
        extra["latency_ms_per_batch_global_indices"] = ev_time(
            lambda: local_lookup(dg_idx.data_ptr(), dg_cnt.data_ptr(), None, 0), reps, tstream)
        ctx.set_global_indices(False)
    if a.algo == "batch":
        # per-kernel device time: HIP events recorded by the kernels' own dispatches
        # (hipExtLaunchKernel) on the bench stream, averaged over `reps` serial calls of the timed
        # step right after the timed window (arming events on every in-flight step perturbs the
        # step: +8-15 us); the rocprofv3 kernel-trace average of the bench (profiles/r02) agrees
        kt = EvSets(reps, tstream)
        for _ in range(reps):
            kt.arm(ctx)
            local_lookup(dg_idx.data_ptr(), dg_cnt.data_ptr(), rec.data_ptr() if collective else None, lo)
        live = kt.mean_ms()
        tms, n_fb, surv, n_slow = ctx.batch_topk_timed(tp.data_ptr(), ts, q_local, a.k, dg_idx.data_ptr(),
                                                       dg_cnt.data_ptr(), stream)
        kern = k6_kernels(live, n_local, q_local, a.k, surv)
        dom = "k_f2_filter"
        dom_ms, dom_bytes = kern[dom]
        step_bytes = sum(v[1] for v in kern.values())
        wl = f"cfg2:{n_local}x{q_local}x{a.k}"
        tb = pmc_traffic(wl, dom)
        working = 4 * n_local + 16 * surv + q_local * (12 + 8 + 4 * a.k)
        roof = {"bound": "hbm", "achieved": dom_bytes / (dom_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": dom_bytes / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "traffic": tb / (dom_ms * 1e-3) / 1e9 if tb else None,
                "traffic_bytes_per_launch": tb, "traffic_source": PMC_FILE if tb else None,
                "kernel": dom, "kernel_ms": dom_ms, "alg_bytes_per_launch": dom_bytes,
                "kernel_timing": f"mean of {reps} serial calls of the timed step on the bench stream, HIP events "
                                 f"recorded by the kernels' own dispatches (hipExtLaunchKernel)",
                "kernels_ms": {k: v[0] for k, v in kern.items()},
                "step_alg_bytes": step_bytes,
                "step_hbm_frac": step_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "working_set_bytes": working,
                "served_from": "Infinity Cache: the cfg-2 working set (w0 plane + survivor buckets) stays "
                               "resident in the 256 MiB L3 across steps; see roofline_hbm for the HBM figure",
                # SURVEY 8(d) contract bytes (every id read whole, 20 B) and their time at peak
                "contract_bytes": n_local * 20 + q_local * 20 + q_local * a.k * 4,
                "contract_floor_ms": (n_local * 20 + q_local * 20 + q_local * a.k * 4) / HBM_PEAK_GBS / 1e6}
        extra.update({"survivors": surv, "survivor_frac": surv / max(n_local, 1), "fallback_targets": n_fb,
                      "wave_path_targets": n_slow})
        if use_dist:
            # aggregate over the ranks: every rank's F2 bytes / the slowest rank's F2 time, against
            # world x the one-GPU peak (each rank streams its own shard from its own HBM)
            # traffic: every rank's PMC bytes for its own shard workload (committed rocprofv3 passes
            # keyed by the per-rank shard, tools/batch_probe.py --n n_local); None if a rank has none
            agg = torch.tensor([float(dom_bytes), float(step_bytes), float(tb or 0.0), 0.0 if tb else 1.0],
                               dtype=torch.float64, device=dev)
            slow = torch.tensor([dom_ms], dtype=torch.float64, device=dev)
            dist.all_reduce(agg, op=dist.ReduceOp.SUM)
            dist.all_reduce(slow, op=dist.ReduceOp.MAX)
            ab, sb, sm = float(agg[0].item()), float(agg[1].item()), float(slow.item())
            tball = float(agg[2].item()) if float(agg[3].item()) == 0.0 else None
            roof["aggregate"] = {"ranks": world, "alg_bytes_all_ranks": ab, "slowest_rank_kernel_ms": sm,
                                 "achieved": ab / (sm * 1e-3) / 1e9, "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
                                 "frac": ab / (sm * 1e-3) / 1e9 / (HBM_PEAK_GBS * world),
                                 "traffic": tball / (sm * 1e-3) / 1e9 if tball else None,
                                 "traffic_bytes_all_ranks": tball,
                                 "traffic_source": f"{PMC_FILE} workloads[{wl!r}] per rank" if tball else None,
                                 "step_frac": sb / (ms_per_step * 1e-3) / 1e9 / (HBM_PEAK_GBS * world),
                                 "how": "sum of the ranks' F2 algorithmic bytes / the slowest rank's F2 time / "
                                        "(ranks x 8 TB/s); step_frac: all four kernels' bytes over the timed step"}
        # the same kernel with the Infinity Cache evicted before every call (HBM-bound figure)
        ebuf = torch.zeros(128 << 20, dtype=torch.int32, device=dev)
        cold = EvSets(8, tstream)
        for _ in range(8):
            l3_evict(ebuf)
            cold.arm(ctx)
            local_lookup(dg_idx.data_ptr(), dg_cnt.data_ptr(), None, 0)
        cms = cold.mean_ms()
        del ebuf
        ckern = k6_kernels(cms, n_local, q_local, a.k, surv)
        res["roofline_hbm"] = {"bound": "hbm", "kernel": dom, "kernel_ms": ckern[dom][0],
                               "achieved": dom_bytes / (ckern[dom][0] * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": dom_bytes / (ckern[dom][0] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                               "kernels_ms": {k: v[0] for k, v in ckern.items()},
                               "traffic_bytes_per_launch": pmc_traffic(wl + ":cold", dom),
                               "how": "512 MiB read between calls (2x the Infinity Cache), 8 serial calls, events "
                                      "of the kernels' dispatches"}
    elif a.algo == "index":
        phases = [ctx.index_build_timed(stream) for _ in range(reps)]
        ph = [sum(p[i] for p in phases) / reps for i in range(4)]
        q_ms = ev_time(lambda: ctx.index_topk_dev(tp.data_ptr(), ts, q_local, a.k, dg_idx.data_ptr(),
                                                  dg_cnt.data_ptr(), None, 0, stream), reps, tstream)
        kern = {"k_p0_hist": (ph[0], 4 * n_local), "k_p0_scans": (ph[1], 0),
                "k_p1_scatter": (ph[2], 12 * n_local), "k_p2_buckets": (ph[3], 16 * n_local),
                "k_query": (q_ms, q_local * (20 + a.k * 4))}
        dom = max(kern, key=lambda k: kern[k][0])
        dom_ms, dom_bytes = kern[dom]
        roof = {"bound": "hbm", "achieved": dom_bytes / (dom_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": dom_bytes / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": None,
                "kernel": dom, "kernel_ms": dom_ms, "alg_bytes_per_launch": dom_bytes,
                "kernels_ms": {k: v[0] for k, v in kern.items()}}
        extra.update({"query_only_qps_per_gpu": q_local / (q_ms * 1e-3), "index_build_ms": sum(ph)})
    else:
        kern_ms = ev_time(lambda: local_lookup(dg_idx.data_ptr(), dg_cnt.data_ptr(),
                                               rec.data_ptr() if collective else None, lo), reps, tstream)
        pairs = q_local * n_local
        achieved = OPS_PER_PAIR * pairs / (kern_ms * 1e-3) / 1e12
        roof = {"bound": "valu", "achieved": achieved, "peak": VALU_PEAK_TOPS, "unit": "TOP/s",
                "frac": achieved / VALU_PEAK_TOPS, "traffic": None,
                "kernel": "k_scan (K1 xor_topk_scan)", "kernel_ms": kern_ms,
                "ops_per_pair": OPS_PER_PAIR, "pairs_per_launch": pairs,
                "frac_survey_3op": SURVEY_OPS_PER_PAIR * pairs / (kern_ms * 1e-3) / 1e12 / VALU_PEAK_TOPS,
                "hbm_alg_bytes_per_launch": n_local * 20 + q_local * 20 + q_local * a.k * 4}

    if a.algo != "scan" and not a.no_scan and world == 1 and not a.simulate_world:
        # the north-star brute-force scan (K1) on the same inputs, for reference
        sc_ms = ev_time(lambda: ctx.topk_dev(tp.data_ptr(), ts, q_local, a.k, out_idx.data_ptr(),
                                             out_cnt.data_ptr(), None, 0, stream), 3, tstream)
        pairs = q_local * n_local
        ach = OPS_PER_PAIR * pairs / (sc_ms * 1e-3) / 1e12
        extra["scan_k1"] = {"qps": q_local / (sc_ms * 1e-3), "kernel_ms": sc_ms, "bound": "valu",
                            "achieved_TOPs": ach, "peak_TOPs": VALU_PEAK_TOPS, "frac": ach / VALU_PEAK_TOPS,
                            "ops_per_pair": OPS_PER_PAIR,
                            "frac_survey_3op": SURVEY_OPS_PER_PAIR * pairs / (sc_ms * 1e-3) / 1e12 / VALU_PEAK_TOPS,
                            "note": "frac counts the packed kernel's 1 lane-op per pair; frac_survey_3op counts "
                                    "SURVEY 8(d)'s 3 ops per pair (> 1 means the packed prefilter beats it)"}

    single = world == 1 and not a.simulate_world and not a.no_extra and a.algo == "batch"
    if single:
        progress("small-batch and table legs")
        extra["small_batch"] = small_batch_leg(ctx, tp, ts, n_local, a.k, stream, tstream, dev, a.seed)
        extra["find_closest"] = find_closest_leg(ctx, a, dev)
        ctx.close()   # the cfg-2 set is no longer needed: free HBM for the size legs
        ctx = None
        for name, fn in (("cfg3_prefix_rank", lambda *x: cfg3_rank_leg(*x, route="prefix")),
                         ("cfg3_broadcast_rank", lambda *x: cfg3_rank_leg(*x, route="broadcast")),
                         ("cfg3_shard", cfg3_shard_leg), ("cfg4", cfg4_leg), ("cfg5", cfg5_leg)):
            progress(f"{name} leg")
            try:
                extra[name] = fn(a, L, dev, stream, tstream)
            except Exception as e:  # noqa: BLE001 -- an extra leg must not cost the headline
                extra[name] = {"error": repr(e)}
    if world > 1 and not a.no_extra and a.algo == "batch" and route == "broadcast" and not a.simulate_world:
        # the same cfg-2 problem with the other exchange and on the prefix route (strong), and the
        # prefix route with weak scaling, each labelled; measured after the headline, on fresh contexts
        progress("N > 1 legs: the other exchange, the prefix route")
        other = "alltoall" if plan["exchange"] == "allgather" else "allgather"
        try:
            extra[f"broadcast_{other}"] = broadcast_leg(a, L, dev, world, rank, other, tp_all, ts, ctx, lo,
                                                        got_idx.reshape(-1, a.k), tlo)
        except Exception as e:  # noqa: BLE001 -- an extra leg must not cost the headline
            extra[f"broadcast_{other}"] = {"error": repr(e)}
        for name, strong in (("prefix_strong", True), ("prefix_weak", False)):
            try:
                if (world & (world - 1)) == 0:
                    extra[name] = prefix_leg(a, L, dev, world, rank, strong)
            except Exception as e:  # noqa: BLE001
                extra[name] = {"error": repr(e)}
    if world > 1 and not a.no_extra and a.algo == "batch" and not a.rehearse_one_gpu:
        progress("cfg3 leg over the ranks")
        try:
            if ctx is not None:
                ctx.close()
                ctx = None
            extra["cfg3"] = cfg3_multi_leg(a, L, dev, stream, tstream, world, rank)
        except Exception as e:  # noqa: BLE001
            extra["cfg3"] = {"error": repr(e)}

    if rank == 0:
        par = {"prefix": f"prefix-routed shards x{G} (top {pbits} id bits; no data-path collective)",
               "broadcast": f"id-range shards x{world}" + ((" + RCCL all-to-all by target slice + K3 merge" if a2a else
                                                             " + RCCL all-gather + K3 merge") if collective else "")}[route]
        res = {
            "metric": METRIC,
            "value": (a.q_total if not a.simulate_world else q_local) / (ms_per_step * 1e-3),
            "unit": "queries/s",
            "n_gpus": world,
            "dist_world_size": dist.get_world_size() if use_dist else 1,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_per_step,
            "host_enqueue_ms_per_step": t_enq * 1e3 / a.steps,   # rank 0's host time to enqueue a step
            "gpu_window_ms_per_step": w_beg.elapsed_time(w_end) / a.steps,   # rank 0, GPU clock (diagnostic)
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: splitmix64 ids and targets generated in HBM (SURVEY 8(d) spec)",
            "config": {"workload": ("cfg2" if (a.n, a.q) == (1 << 24, 65536) else "custom")
                                   + f" batched k-NN: {a.q} targets x {a.n} ids (2^{a.n.bit_length()-1}), k={a.k}"
                                   + (f" per GPU ({a.q_total} x {a.n_total} over {G_eff} GPUs)"
                                      if scaling == "weak" and G_eff > 1 else ""),
                       "n_ids": a.n_total, "n_targets": a.q_total, "k": a.k, "algo": a.algo, "route": route,
                       "ids_per_gpu": n_local, "targets_per_gpu": q_local, "parallelism": par,
                       "inflight": D, "exchange": plan["exchange"],
                       "results_on_this_rank": f"targets [{tlo}, {tlo + q_out})" if collective else None,
                       "result_indices": ("shard-local" if a.shard_index == "local" else "global")
                       if route == "prefix" and pbits else "global"},
            "latency_ms_per_batch": lat_ms,
            "roofline": roof,
            **res,
        }
        if a.simulate_world:
            res["simulated"] = f"rank {R} of {G} on one GPU; value = this rank's targets / its step time"
        res.update(extra)
        if collective:
            recb = sharding.REC_WORDS * 4
            rows_in = world * (q_out if a2a else a.q_total)
            res["exchange"] = {
                "record": "{w0, w1, global idx}", "record_bytes": recb,
                "record_bytes_per_rank": a.q_total * a.k * recb,
                "exchange_bytes_in_per_gpu": rows_in * a.k * recb,
                "exchange_bytes_over_xgmi_per_gpu": (world - 1) * (q_out if a2a else a.q_total) * a.k * recb,
                "tie_exchange_bytes_in_per_gpu": (world * sharding.TIE_CAP * a.k * 12
                                                  + (world * (1 + sharding.TIE_CAP) * 4 if a2a else 0))
                if world > 1 else 0,
                "tie_rows_settled": tie_rows,
                "note": "K3 orders candidates by their first 64 bits and the global index; rows where two lists' "
                        "candidates agree on those bits are settled by a second, fixed-size exchange of words 2..4 "
                        f"(at most {sharding.TIE_CAP} rows per step; more: an every-row settlement after the sync); "
                        "none with one rank"}
        if not a.no_cpu and (a.verify or world == 1):
            progress("verifying against the oracle")
            O = oracle()
            nv = min(q_out, max(a.verify, a.cpu_targets if world == 1 else 0))
            tg_all = O.gen_ids(a.seed + 1, a.q_total)
            tg = tg_all[got_tg[:nv]]
            local_ix = route == "prefix" and pbits and a.shard_index == "local"
            if local_ix:   # shard-local results: the oracle over this shard's own ids, in shard order
                top = O.gen_ids(a.seed, a.n_total)
                top = top[(top[:, 0] >> (8 - pbits)) == R]
                ids = top
            else:
                ids = O.gen_ids(a.seed, a.n_total)
            if world == 1 and not a.simulate_world:
                cb, want = cpu_baseline(O, ids, tg, a)
                res["cpu_baseline"] = cb
            else:
                want, _ = O.topk(ids, tg, a.k, threads=usable_cpus())
            res["verified_targets"] = int(nv)
            res["verified_exact"] = bool(np.array_equal(got_idx[:nv], want))
            progress("verified")
        os.write(_RESULT_FD, (json.dumps(res) + "\n").encode())
    if ctx is not None:
        ctx.close()
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


def small_batch_leg(ctx, tp, ts, n, k, stream, tstream, dev, seed=2024):
    """Q = 1 / 8 / 32 / 64 targets -- the reference's real call pattern is one target per request
    (src/dht.cpp:2128-2138 -> findClosestNodes): latency per call and the bytes the call has to
    stream (4 B/id of the w0 plane; SURVEY's contract counts 20 B/id).  The library's batch entry
    point takes the small-batch path (KS: S1 one pass over w0, S2 one workgroup per target prefix
    beside the scan roles that answer short subtrees -- none here) for q <= 64; K1 is the plain
    scan beside it.  Three regimes per q:
      warm  the cfg-2 set (67 MB w0 plane) stays in the 256 MiB Infinity Cache between calls
      cold  the same set with the Infinity Cache evicted before every call (512 MiB read): S1
            streams HBM
      big   a 2^26-id set (268 MB w0 plane, past the Infinity Cache), warm and cold"""
    out = {}
    oi = torch.empty((64, k), dtype=torch.int32, device=dev)
    oc = torch.empty(64, dtype=torch.int32, device=dev)
    ebuf = torch.zeros(128 << 20, dtype=torch.int32, device=dev)

    def cold_rows(c, nn, q, reps=9):
        """per call: evict, then events around the call and its kernels' own dispatches"""
        lat, s1, s2 = [], [], []
        for _ in range(reps):
            l3_evict(ebuf)
            ev = EvSets(1, tstream)
            ev.arm(c)
            c.batch_topk_dev(tp.data_ptr(), ts, q, k, oi.data_ptr(), oc.data_ptr(), None, 0, stream)
            m = ev.mean_ms()
            # S1's dispatch start to S2's end (an event recorded on the stream after the eviction
            # read is stamped before that kernel's tail drains: it overstated the call by ~35 us)
            lat.append(ev.sets[0][2].elapsed_time(ev.sets[0][5]))
            s1.append(m[1])
            s2.append(m[2])
        ms, s1m, s2m = float(np.median(lat)), float(np.median(s1)), float(np.median(s2))
        return {"latency_ms": ms, "qps": q / (ms * 1e-3), "kernels_ms": {"k_s1_filter": s1m, "k_s2_answer": s2m},
                "w0_frac": 4 * nn / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "s1_frac": 4 * nn / (s1m * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "timing": f"median of {reps} calls, each after a 512 MiB read (Infinity Cache evicted); latency = "
                          "S1 dispatch start to S2 end (events recorded by the kernels' own dispatches)",
                "pmc_traffic_bytes_per_launch": {kn: pmc_traffic(f"ks:{nn}x{q}x{k}:cold", kn)
                                                 for kn in ("k_s1_filter", "k_s2_answer")}}

    def warm_rows(c, nn, q, with_k1):
        row = {}
        fns = (("batch", c.batch_topk_dev), ("k1", c.topk_dev)) if with_k1 else (("batch", c.batch_topk_dev),)
        for name, fn in fns:
            call = lambda: fn(tp.data_ptr(), ts, q, k, oi.data_ptr(), oc.data_ptr(), None, 0, stream)
            call()
            ms = ev_time(call, 20 if name == "batch" else 3, tstream)
            row[name] = {"latency_ms": ms, "qps": q / (ms * 1e-3),
                         "w0_GBps": 4 * nn / (ms * 1e-3) / 1e9, "w0_frac": 4 * nn / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "contract_GBps": (20 * nn + 24 * q + 4 * k * q) / (ms * 1e-3) / 1e9}
        ev = EvSets(9, tstream)
        for _ in range(9):   # serial calls, median per kernel
            ev.arm(c)
            c.batch_topk_dev(tp.data_ptr(), ts, q, k, oi.data_ptr(), oc.data_ptr(), None, 0, stream)
        kms = ev.median_ms()
        row["kernels_ms"] = {"k_s1_filter": kms[1], "k_s2_answer (prefix answers + fallback scan roles)": kms[2]}
        row["kernel_timing"] = "median of 9 serial calls (events on the kernels' own dispatches)"
        row["s1_frac"] = 4 * nn / (kms[1] * 1e-3) / 1e9 / HBM_PEAK_GBS
        # rocprofv3 FETCH_SIZE (x2, gfx950) + WRITE_SIZE passes of tools/small_probe.py (profiles/r0x)
        row["pmc_traffic_bytes_per_launch"] = {kn: pmc_traffic(f"ks:{nn}x{q}x{k}", kn) for kn in ("k_s1_filter", "k_s2_answer")}
        return row

    for q in (1, 8, 32, 64):
        row = warm_rows(ctx, n, q, True)
        row["cold"] = cold_rows(ctx, n, q)
        out[f"q{q}"] = row
    nb = 1 << 26
    big = opendht_amd.Context(dev.index)
    try:
        big.gen_ids(seed + 30, nb)
        for q in (1, 8, 32, 64):
            out[f"big_q{q}"] = {"warm": warm_rows(big, nb, q, False), "cold": cold_rows(big, nb, q)}
    finally:
        big.close()
        del ebuf
        torch.cuda.synchronize()
    out["note"] = ("q<N>: the cfg-2 set (2^24 ids; warm rows L3-resident, .cold with the Infinity Cache evicted before "
                   "each call); big_q<N>: a 2^26-id set (268 MB w0 plane > 256 MiB L3). w0_frac = the 4 B/id w0 stream "
                   "over the whole call's time; s1_frac = the same bytes over the S1 kernel alone")
    return out


def find_closest_leg(ctx, a, dev):
    """RoutingTable::findClosestNodes (dhtgpu_find_closest, K1r) on a cfg-1-shaped table: one
    target per call (the reference's call pattern; host pointers, PCIe included) and one
    65,536-target batch."""
    myid, firsts, off, nodes = cfg1_table(a.seed)
    good = np.ones(nodes.shape[0], np.uint8)
    tg = np.frombuffer(np.random.default_rng(a.seed + 1).bytes(20 * 65536), dtype=np.uint8).reshape(-1, 20).copy()
    ctx.find_closest(firsts, off, nodes, good, tg[:1], 8)
    t0 = time.perf_counter()
    for i in range(200):
        ctx.find_closest(firsts, off, nodes, good, tg[i:i + 1], 8)
    single = (time.perf_counter() - t0) / 200
    ctx.find_closest(firsts, off, nodes, good, tg, 8)
    t0 = time.perf_counter()
    for _ in range(5):
        ctx.find_closest(firsts, off, nodes, good, tg, 8)
    batch = (time.perf_counter() - t0) / 5
    return {"table": f"{firsts.shape[0]} buckets, {nodes.shape[0]} nodes: onNewNode-grown from 10,000 random ids (cfg 1)",
            "single_target_us": single * 1e6, "batch_65536_ms": batch * 1e3, "batch_qps": 65536 / batch,
            "note": "host API per call: snapshot + targets uploaded, results downloaded (PCIe included)"}


CFG3_N, CFG3_Q, CFG3_WORLD = 1_000_000_000, 1 << 20, 8


def cfg3_rank_setup(seed, route, L, dev, stream, rank=0, world=CFG3_WORLD):
    """One rank's inputs of BASELINE cfg 3 (10^9 ids, 2^20 targets over `world` GPUs), exactly as the
    N-rank job builds them (cfg3_multi_leg's seeds): the prefix route's rank holds the ids of the
    10^9 stream whose top log2(world) bits equal its rank (gen_ids_prefix: ~1.25e8) and answers the
    ~2^20 / world targets of that prefix, with GLOBAL stream indices; the broadcast route's rank holds
    the id range shard_range(10^9, world, rank) and answers all 2^20 targets.
    Returns (ctx, target planes, stride, q on this rank, target rows' global index or None, idx base)."""
    c = opendht_amd.Context(dev.index)
    tp_all, ts = gen_targets(L, seed + 11, CFG3_Q, dev, stream)
    if route == "prefix":
        pbits = world.bit_length() - 1
        c.gen_ids_prefix(seed + 10, CFG3_N, pbits, rank)
        c.set_global_indices(True)
        tp = torch.empty_like(tp_all)
        tgidx = torch.empty(ts, dtype=torch.int32, device=dev)
        ql = c.select_prefix_dev(tp_all.data_ptr(), ts, CFG3_Q, pbits, rank, tp.data_ptr(), ts, tgidx.data_ptr(), stream)
        return c, tp, ts, ql, tgidx, 0
    lo, hi = sharding.shard_range(CFG3_N, world, rank)
    c.gen_ids(seed + 10, hi - lo, start=lo)
    return c, tp_all, ts, CFG3_Q, None, lo


def k6_step_bytes(n, q, k, surv, record=False, mapped=False):
    """Algorithmic bytes of one K6 call, per kernel: F1 12 B/target; F2
    4 B/id (w0) + 8 B/survivor; F3 8 B/survivor + 36 B/target (bucket entry, target words, count)
    + per result: 4 B written (index form) or 12 B written + 4 B of word 1 read (record form), + 4 B
    of the index map read when results are mapped to global indices through a sub-partition map."""
    per_res = (16 if record else 4) + (4 if mapped else 0)
    return {"k_f1_targets": 12 * q, "k_f2_filter": 4 * n + 8 * surv,
            "k_f3_answer": 8 * surv + q * (8 + 16 + 4) + q * k * per_res, "k_f4_fallback": 0}


def cfg3_rank_leg(a, L, dev, stream, tstream, route):
    """One rank of BASELINE cfg 3 at the exact N = 8 per-rank shape, on this one GPU:
      prefix     ~1.25e8 ids (the 10^9 stream's prefix-0 shard) x ~2^17 targets (those of prefix 0),
                 global indices -- what each rank of the prefix route does, no collective;
      broadcast  1.25e8 ids (shard_range(10^9, 8, 0)) x all 2^20 targets, K6 in record form then K3
                 over the one list -- each rank's work on the north-star route minus the all-gather
                 (K3 merges 8 lists there).
    Two calls in flight (one call's F3 / F4 / K3 beside the next call's F2).  roofline: F2 and the
    whole step against 8 TB/s, algorithmic bytes per k6_step_bytes; PMC traffic from the committed
    rocprofv3 passes of tools/batch_probe.py --cfg3 <route>.  Verified on >= 32 targets against the
    generator-fed oracle (orc_topk_gen: std::partial_sort semantics over the 10^9-id stream or the
    shard's range)."""
    k = a.k
    c, tp, ts, q, tgidx, lo = cfg3_rank_setup(a.seed, route, L, dev, stream)
    try:
        n = c.num_ids
        record = route == "broadcast"
        RW = sharding.REC_WORDS
        st2 = [tstream, torch.cuda.Stream(dev)]
        outs = [(torch.empty((q, k), dtype=torch.int32, device=dev), torch.empty(q, dtype=torch.int32, device=dev),
                 torch.empty((q, k, RW), dtype=torch.int32, device=dev) if record else None) for _ in range(2)]

        def call(i, s, ev=None):
            oi, oc, rec = outs[i]
            if ev is not None:
                ev.arm(c)
            if record:
                c.batch_topk_dev(tp.data_ptr(), ts, q, k, None, None, rec.data_ptr(), lo, s)
                assert L.dhtgpu_merge_dev(rec.data_ptr(), 1, q, k, tp.data_ptr(), ts, k, oi.data_ptr(), oc.data_ptr(),
                                          None, 0, s) == 0
            else:
                c.batch_topk_dev(tp.data_ptr(), ts, q, k, oi.data_ptr(), oc.data_ptr(), None, 0, s)
        t0 = time.perf_counter()
        call(0, stream)
        torch.cuda.synchronize()
        first_s = time.perf_counter() - t0
        for i in range(4):   # both streams' workspace slots set up before the timed windows
            call(i % 2, st2[i % 2].cuda_stream)
        steps = 20

        def window(nst):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(steps):
                call(i % 2, st2[i % nst].cuda_stream)
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) * 1e3 / steps
        ms1 = window(1)
        ms = window(2)
        got = outs[(steps - 1) % 2][0].clone()
        reps = 8   # kernel times: serial calls after the timed windows
        ev = EvSets(reps, tstream)
        for _ in range(reps):
            call(0, tstream.cuda_stream, ev)
        kms = ev.mean_ms()
        k3_ms = None
        if record:
            k3_ms = ev_time(lambda: L.dhtgpu_merge_dev(outs[0][2].data_ptr(), 1, q, k, tp.data_ptr(), ts, k,
                                                       outs[0][0].data_ptr(), outs[0][1].data_ptr(), None, 0, stream),
                            reps, tstream)
        _, fb, surv, slow = c.batch_topk_timed(tp.data_ptr(), ts, q, k, outs[0][0].data_ptr(), outs[0][1].data_ptr(),
                                               stream)
        alg = k6_step_bytes(n, q, k, surv, record=record, mapped=not record)
        names = list(alg)
        kern_ms = dict(zip(names, kms))
        if record:   # K3 over the one list: records + target words 0..1 in, indices + counts out
            alg["k_merge3"] = q * k * 12 + q * 8 + q * k * 4 + q * 4
            kern_ms["k_merge3"] = k3_ms
        step_bytes = sum(alg.values())
        f2b, f2ms = alg["k_f2_filter"], kern_ms["k_f2_filter"]
        key = f"cfg3{route}:{n}x{q}x{k}"
        tb = pmc_traffic(key, "k_f2_filter")
        tstep = None
        try:
            d = json.load(open(os.path.join(ROOT, PMC_FILE))).get("workloads", {}).get(key, {})
            step_k = ("k_f1_targets", "k_f1_coarse", "k_f1_fine", "k_f2_filter", "k_f2_direct", "k_f3_answer", "k_f4",
                      "k_merge3")   # the step's kernels only
            tstep = sum(d[kn]["traffic_bytes"] for kn in step_k if kn in d) or None
        except (OSError, ValueError):
            pass
        res = {"route": route,
               "workload": (f"rank 0 of the prefix route at N = {CFG3_WORLD}: {n} ids (the 10^9 stream's prefix-0 shard) x "
                            f"{q} targets (prefix 0 of {CFG3_Q}), k={k}, global indices" if route == "prefix" else
                            f"rank 0 of the broadcast route at N = {CFG3_WORLD}: {n} ids (shard_range(10^9, 8, 0)) x {q} "
                            f"targets, k={k}: K6 in record form + K3 over the one list (no all-gather)"),
               "ms_per_step": ms, "qps": q / (ms * 1e-3), "inflight": 2, "ms_per_step_one_stream": ms1,
               "setup_first_call_s": first_s, "kernels_ms": kern_ms,
               "kernel_timing": f"{reps} serial calls after the timed windows (events on the kernels' own dispatches)",
               "alg_bytes_per_launch": alg, "survivors": surv, "fallback": fb, "wave_path": slow,
               "roofline": {"bound": "hbm", "kernel": "k_f2_filter", "achieved": f2b / (f2ms * 1e-3) / 1e9,
                            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": f2b / (f2ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                            "kernel_ms": f2ms, "alg_bytes_per_launch": f2b,
                            "traffic": tb / (f2ms * 1e-3) / 1e9 if tb else None, "traffic_bytes_per_launch": tb,
                            "traffic_source": f"{PMC_FILE} workloads[{key!r}]" if tb else None,
                            "step_alg_bytes": step_bytes,
                            "step_frac": step_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                            "step_traffic_bytes": tstep,
                            "served_from": f"HBM: the w0 planes ({4 * n / 1e6:.0f} MB) exceed the 256 MiB L3",
                            "how": "frac: F2's algorithmic bytes / its mean event time; step_frac: every kernel's "
                                   "algorithmic bytes / the 2-in-flight step time; peak 8 TB/s",
                            "kernels": "phases as dispatched: F1 = k_f1_targets, or k_f1_coarse + k_f1_fine at >= 2^18 "
                                       "targets; F2 = k_f2_filter, or k_f2_direct over prefix-sorted sub-partitions; "
                                       "PMC traffic summed over a phase's kernels"}}
        if not a.no_cpu:
            O = oracle()
            rows = np.linspace(0, q - 1, 32).astype(np.int64)
            g = got.cpu().numpy().view(np.uint32)[rows]
            tgt_all = O.gen_ids(a.seed + 11, CFG3_Q)
            if route == "prefix":
                gi = tgidx[:q].cpu().numpy().view(np.uint32)[rows].astype(np.int64)
                want, _ = O.topk_gen(a.seed + 10, CFG3_N, tgt_all[gi], k, threads=usable_cpus())
            else:
                want, _ = O.topk_gen(a.seed + 10, n, tgt_all[rows], k, start=lo, threads=usable_cpus())
            res["verified_targets"] = int(rows.size)
            res["verified_exact"] = bool(np.array_equal(g, want))
            res["verified_against"] = ("orc_topk_gen over the whole 10^9-id stream (global indices)" if route == "prefix"
                                       else f"orc_topk_gen over the shard's ids [{lo}, {lo + n}) of the stream")
        return res
    finally:
        c.close()
        torch.cuda.synchronize()


def cfg3_shard_leg(a, L, dev, stream, tstream):
    """A 2^27-id set (~10^9 / 8, the prefix route's per-rank size rounded to a power of two) with
    131,072 targets spread over every prefix: the prefix route's per-rank shape (VERDICT r4 item 2's
    benchmark; cfg3_prefix_rank is the exact rank).  The library splits the set once into 8 prefix
    sub-partitions of 2^24 (setup, not timed) and serves all of them with ONE K6 launch sequence;
    their w0 planes (537 MB) exceed the Infinity Cache, so F2 streams HBM."""
    n, q, k = 1 << 27, 131072, a.k
    c = opendht_amd.Context(dev.index)
    try:
        c.gen_ids(a.seed + 3, n)
        tp, ts = gen_targets(L, a.seed + 4, q, dev, stream)
        outs = [(torch.empty((q, k), dtype=torch.int32, device=dev), torch.empty(q, dtype=torch.int32, device=dev))
                for _ in range(2)]
        t0 = time.perf_counter()
        c.batch_topk_dev(tp.data_ptr(), ts, q, k, outs[0][0].data_ptr(), outs[0][1].data_ptr(), None, 0, stream)
        torch.cuda.synchronize()
        first_s = time.perf_counter() - t0
        st2 = [tstream, torch.cuda.Stream(dev)]
        for i in range(4):   # both streams' workspace slots set up before the timed windows
            c.batch_topk_dev(tp.data_ptr(), ts, q, k, outs[i % 2][0].data_ptr(), outs[i % 2][1].data_ptr(), None, 0,
                             st2[i % 2].cuda_stream)
        steps = 20

        def window(nst):
            # back-to-back calls over nst streams (two in flight: one call's F3 / F4 run beside the
            # next call's F2), no events in the timed loop
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(steps):
                c.batch_topk_dev(tp.data_ptr(), ts, q, k, outs[i % 2][0].data_ptr(), outs[i % 2][1].data_ptr(), None,
                                 0, st2[i % nst].cuda_stream)
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) * 1e3 / steps
        ms1 = window(1)
        ms = window(2)
        reps = 8   # kernel times: serial calls after the timed window
        ev = EvSets(reps, tstream)
        for i in range(reps):
            ev.arm(c)
            c.batch_topk_dev(tp.data_ptr(), ts, q, k, outs[0][0].data_ptr(), outs[0][1].data_ptr(), None, 0,
                             tstream.cuda_stream)
        torch.cuda.synchronize()
        kms = ev.mean_ms()
        iso, fb, surv, slow = c.batch_topk_timed(tp.data_ptr(), ts, q, k, outs[0][0].data_ptr(), outs[0][1].data_ptr(),
                                                stream)
        kern = k6_kernels(kms, n, q, k, surv)
        f2ms, f2b = kern["k_f2_filter"]
        res = {"workload": f"{q} targets x {n} ids (2^27), k={k}: 8 prefix sub-partitions of ~2^24, one launch",
               "ms_per_step": ms, "qps": q / (ms * 1e-3), "inflight": 2,
               "ms_per_step_one_stream": ms1, "setup_first_call_s": first_s,
               "kernels_ms": {kk: v[0] for kk, v in kern.items()},
               "kernel_timing": "the fused launch's kernels (all 8 sub-partitions), 8 serial calls after the "
                                "timed window (events)",
               "kernels_ms_isolated": dict(zip(["k_f1_targets", "k_f2_filter", "k_f3_answer", "k_f4_fallback"],
                                               list(iso))),
               "roofline_f2_isolated_frac": f2b / (iso[1] * 1e-3) / 1e9 / HBM_PEAK_GBS,
               "roofline_f2": {"bound": "hbm", "achieved": f2b / (f2ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": f2b / (f2ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                               "alg_bytes_per_launch": f2b, "kernel_ms": f2ms,
                               "traffic_bytes_per_launch": pmc_traffic(f"cfg3shard:{n}x{q}x{k}", "k_f2_filter"),
                               "served_from": "HBM: 8 sub-partition w0 planes = 537 MB per step > 256 MiB L3"},
               "survivors": surv, "fallback": fb, "wave_path": slow,
               "persistent_state": "the 8 prefix sub-partitions (compacted copies with their shifted word-0 planes "
                                   "and index maps, 28 B/id) are built by the first call (setup_first_call_s) and kept "
                                   "across calls; every timed call streams all 2^27 word-0 entries"}
        got_idx = outs[(steps - 1) % 2][0].clone()
        # the same calls returning sub-partition handles (dhtgpu_set_sub_handles: no index-map read
        # per result), mapped back to global indices after the window for the check
        c.set_sub_handles(True)
        for i in range(4):
            c.batch_topk_dev(tp.data_ptr(), ts, q, k, outs[i % 2][0].data_ptr(), outs[i % 2][1].data_ptr(), None, 0,
                             st2[i % 2].cuda_stream)
        ms_h = window(2)
        evh = EvSets(reps, tstream)
        for i in range(reps):
            evh.arm(c)
            c.batch_topk_dev(tp.data_ptr(), ts, q, k, outs[0][0].data_ptr(), outs[0][1].data_ptr(), None, 0,
                             tstream.cuda_stream)
        torch.cuda.synchronize()
        hk = evh.mean_ms()
        mapped = torch.empty_like(outs[0][0])
        c.handles_to_indices_dev(outs[0][0].data_ptr(), q * k, mapped.data_ptr(), 0, stream)
        torch.cuda.synchronize()
        c.set_sub_handles(False)
        f3alg = kern["k_f3_answer"][1]
        res["handles"] = {"ms_per_step": ms_h, "qps": q / (ms_h * 1e-3), "inflight": 2,
                          "kernels_ms": dict(zip(["k_f1_targets", "k_f2_filter", "k_f3_answer", "k_f4_fallback"], hk)),
                          "f3_alg_bytes_per_launch": f3alg,
                          "f3_traffic_bytes_per_launch": pmc_traffic(f"cfg3shard:{n}x{q}x{k}:handles", "k_f3_answer"),
                          "f3_traffic_bytes_per_launch_indices": pmc_traffic(f"cfg3shard:{n}x{q}x{k}", "k_f3_answer"),
                          "mapped_equal_indices": bool(torch.equal(mapped, got_idx)),
                          "note": "results as sub-partition handles (offset of the id's sub-partition + its place "
                                  "there), mapped to global indices on request (dhtgpu_handles_to_indices_dev); "
                                  "ms_per_step above returns indices"}
        if not a.no_cpu:
            O = oracle()
            rows = np.arange(0, q, q // 16)
            got = got_idx.cpu().numpy().view(np.uint32)[rows]
            want, _ = O.topk(O.gen_ids(a.seed + 3, n), O.gen_ids(a.seed + 4, q)[rows], k, threads=usable_cpus())
            res["verified_targets"] = int(rows.size)
            res["verified_exact"] = bool(np.array_equal(got, want))
        return res
    finally:
        c.close()
        torch.cuda.synchronize()


def cfg4_leg(a, L, dev, stream, tstream):
    """BASELINE cfg 4: findBucket + commonBits classification of 10^8 ids vs a local id (K2),
    bucket firsts of a table grown by onNewNode from 10^5 ids.  K2 streams word 0 (4 B/id) and writes
    the 1-B bucket: 5 B/id algorithmic (words 1..4 are read only for ids whose word 0 ties a first's or
    myid's -- none here); SURVEY 8(d)'s contract counts every id whole, 21 B/id."""
    n = 100_000_000
    myid, firsts = cfg4_firsts(a.seed + 5)
    c = opendht_amd.Context(dev.index)
    try:
        c.gen_ids(a.seed + 6, n)
        planes, stride = c.ids_dev()
        fp = torch.from_numpy(firsts.view(">u4").reshape(-1, 5).astype(np.uint32).T.copy().reshape(-1).view(np.int32)).to(dev)
        my = np.frombuffer(myid.tobytes(), dtype=">u4").astype(np.uint32)
        my_c = (ctypes.c_uint32 * 5)(*[int(x) for x in my])
        bucket = torch.empty(n, dtype=torch.uint8, device=dev)
        hist = torch.zeros(161, dtype=torch.int64, device=dev)
        nb = firsts.shape[0]

        def call():   # dhtgpu_classify_dev accumulates into hist (the caller zeroes it)
            assert L.dhtgpu_classify_dev(planes, stride, n, nb, fp.data_ptr(), my_c, bucket.data_ptr(), hist.data_ptr(),
                                         stream) == 0
        call()
        hist.zero_()
        # K2 launches back to back (the histogram accumulating over them: 10 n in total); the
        # caller's zero fill stays outside the timed launches
        ms = ev_time(call, 10, tstream)
        b = 5 * n
        return {"workload": f"{n} ids vs one local id, {nb} routing buckets", "ms": ms, "ids_per_s": n / (ms * 1e-3),
                "roofline": {"bound": "hbm", "achieved": b / (ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "alg_bytes": b,
                             "alg_bytes_per_id": "4 (word 0 streamed) + 1 (bucket written)",
                             "traffic": pmc_traffic(f"cfg4:{n}", "k_classify"),
                             "contract_bytes": 21 * n, "contract_floor_ms": 21 * n / HBM_PEAK_GBS / 1e6},
                "hist_total_per_call": int(hist.sum().item()) // 10, "hist_total_ok": int(hist.sum().item()) == 10 * n}
    finally:
        c.close()
        torch.cuda.synchronize()


def cfg5_leg(a, L, dev, stream, tstream):
    """BASELINE cfg 5: iterative searches (Search::insertNode rounds) over a 5*10^7-node synthetic
    network with 10 % dead nodes (crawl model, crawl.hip), at the reference's 4 requests per round
    (MAX_REQUESTED_SEARCH_NODES, include/opendht/dht.h:321) and at the 3-way alpha BASELINE states."""
    n, q = 50_000_000, 65536
    c = opendht_amd.Context(dev.index)
    try:
        c.gen_ids(a.seed + 7, n)
        dead = (np.random.default_rng(a.seed + 7).random(n) < 0.1).astype(np.uint8)
        t0 = time.perf_counter()
        c.net_prepare(dead, table_seed=a.seed + 7)
        prep = time.perf_counter() - t0
        tp, ts = gen_targets(L, a.seed + 8, q, dev, stream)
        sr = torch.from_numpy(((np.arange(q, dtype=np.uint64) * 2654435761) % n).astype(np.uint32).view(np.int32)).to(dev)
        o_idx = torch.empty((q, 64), dtype=torch.int32, device=dev)
        o_fl = torch.empty((q, 64), dtype=torch.uint8, device=dev)
        o_len, o_rd, o_qs = (torch.empty(q, dtype=torch.int32, device=dev) for _ in range(3))
        args = (tp.data_ptr(), ts, q, sr.data_ptr(), 64, o_idx.data_ptr(), o_fl.data_ptr(), o_len.data_ptr(),
                o_rd.data_ptr(), o_qs.data_ptr(), stream)
        call = lambda: L.dhtgpu_search_batch_dev(c._h, *args)
        out = {"workload": f"{q} searches over {n} nodes (10% dead)", "net_prepare_s": prep}
        for alpha in (4, 3):
            c.set_search_alpha(alpha)
            call()
            ms = ev_time(call, 3, tstream)
            row = {"alpha": alpha, "ms_per_batch": ms, "searches_per_s": q / (ms * 1e-3),
                   "rounds_mean": float(o_rd.float().mean().item()), "requests_mean": float(o_qs.float().mean().item())}
            if alpha == 4:
                out.update(row)   # the reference's alpha: the leg's headline figures
            else:
                out["alpha3"] = row
        c.set_search_alpha(4)
        return out
    finally:
        c.close()
        torch.cuda.synchronize()


def timed_steps(step, steps, warmup, dev):
    """warmup, then `steps` timed calls of step() between barrier + synchronize pairs; the max
    over ranks of the wall time, ms per step"""
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    tm = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(tm, op=dist.ReduceOp.MAX)
    return float(tm.item()) * 1e3 / steps


def broadcast_leg(a, L, dev, world, rank, exchange, tp, ts, ctx, lo, ref_idx, ref_lo):
    """The headline's cfg-2 broadcast problem (same shard, same targets) with the other RCCL
    exchange; steps rotate over --inflight streams as in the headline.  Checked equal to the
    headline exchange on this rank's targets."""
    q, k = a.q_total, a.k
    D = max(1, a.inflight)
    streams = [torch.cuda.Stream(dev) for _ in range(D)]
    tlo, thi = sharding.shard_range(q, world, rank) if exchange == "alltoall" else (0, q)
    qo = thi - tlo
    RW = sharding.REC_WORDS
    recs = [torch.empty((q, k, RW), dtype=torch.int32, device=dev) for _ in range(D)]
    xb = [torch.empty((world * qo, k, RW), dtype=torch.int32, device=dev) for _ in range(D)]
    outs = [(torch.empty((max(qo, 1), k), dtype=torch.int32, device=dev),
             torch.empty(max(qo, 1), dtype=torch.int32, device=dev)) for _ in range(D)]
    txs = [sharding.TieExchange(world, k, dev) for _ in range(D)]
    ops = sharding.LibOps(L, ctx, tp.data_ptr(), ts)
    n_call = [0]

    def step():
        i = n_call[0] % D
        n_call[0] += 1
        st = streams[i]
        with torch.cuda.stream(st):
            ctx.batch_topk_dev(tp.data_ptr(), ts, q, k, None, None, recs[i].data_ptr(), lo, st.cuda_stream)
            if exchange == "alltoall":
                ex = sharding.exchange_records(recs[i], out=xb[i])
                sharding.merge_alltoall(ops, recs[i], ex, k, tlo, outs[i][0], outs[i][1], txs[i], lo, st.cuda_stream)
            else:
                g = sharding.gather_records(recs[i], out=xb[i])
                sharding.merge_allgather(ops, recs[i], g, k, outs[i][0], outs[i][1], txs[i], lo, st.cuda_stream)
    ms = timed_steps(step, a.steps, a.warmup, dev)
    last = (n_call[0] - 1) % D
    with torch.cuda.stream(streams[last]):
        if exchange == "alltoall":
            sharding.settle_overflow_alltoall(ops, recs[last], xb[last].view(world, qo, k, RW), k, tlo, outs[last][0],
                                              outs[last][1], txs[last], lo, streams[last].cuda_stream)
        else:
            sharding.settle_overflow_allgather(ops, recs[last], xb[last].view(world, q, k, RW), k, outs[last][0],
                                               outs[last][1], txs[last], lo, streams[last].cuda_stream)
    torch.cuda.synchronize()
    got = outs[last][0][:qo].cpu().numpy().view(np.uint32)
    # the rows both runs answered on this rank must agree (same shard, same targets)
    a0, a1 = max(tlo, ref_lo), min(thi, ref_lo + ref_idx.shape[0])
    same = bool(np.array_equal(got[a0 - tlo:a1 - tlo], ref_idx[a0 - ref_lo:a1 - ref_lo])) if a1 > a0 else None
    return {"exchange": exchange, "ms_per_step": ms, "value": q / (ms * 1e-3), "unit": "queries/s",
            "scaling": "strong (the headline's global batch)",
            "exchange_bytes_in_per_gpu": (world * q if exchange == "allgather" else world * qo) * k * 12,
            "results_on_this_rank": f"targets [{tlo}, {thi})",
            "equals_headline_rank0": same, "rows_compared_rank0": max(0, a1 - a0)}


def prefix_leg(a, L, dev, world, rank, strong):
    """The prefix route beside the headline (labelled; SURVEY 8(e)'s "better scheme"): ids and
    targets routed by their top log2(N) bits, no collective on the data path, shard-local result
    indices.  weak: every rank keeps the one-GPU workload (--n ids and --q targets per GPU);
    strong: the headline's own problem (--n ids and --q targets in total, every target on every
    rank as on the broadcast route, each rank answering those of its prefix from its 1/N of the
    ids) -- exact like the broadcast route (a target's top-k lies in its own prefix subtree when
    every shard holds >= k ids), with 1/N of its work and no exchange."""
    pbits = world.bit_length() - 1
    n_tot, q_tot = (a.n, a.q) if strong else (a.n * world, a.q * world)
    c = opendht_amd.Context(dev.index)
    try:
        c.gen_ids_prefix(a.seed + 20, n_tot, pbits, rank)
        c.set_global_indices(False)
        s = torch.cuda.current_stream(dev).cuda_stream
        tp_all, ts = gen_targets(L, a.seed + 21, q_tot, dev, s)
        tp = torch.empty_like(tp_all)
        ql = c.select_prefix_dev(tp_all.data_ptr(), ts, q_tot, pbits, rank, tp.data_ptr(), ts, None, s)
        D = max(1, a.inflight)
        streams = [torch.cuda.Stream(dev) for _ in range(D)]
        outs = [(torch.empty((max(ql, 1), a.k), dtype=torch.int32, device=dev),
                 torch.empty(max(ql, 1), dtype=torch.int32, device=dev)) for _ in range(D)]
        n_call = [0]

        def step():
            i = n_call[0] % D
            n_call[0] += 1
            c.batch_topk_dev(tp.data_ptr(), ts, ql, a.k, outs[i][0].data_ptr(), outs[i][1].data_ptr(), None, 0,
                             streams[i].cuda_stream)
        ms = timed_steps(step, a.steps, a.warmup, dev)
        if strong:
            return {"route": "prefix", "scaling": "strong", "ms_per_step": ms, "value": q_tot / (ms * 1e-3),
                    "unit": "queries/s", "workload": f"{q_tot} targets x {n_tot} ids in total over {world} (the headline's)",
                    "ids_rank": c.num_ids, "targets_rank": ql,
                    "note": "the headline's problem on the prefix route: each rank answers its own prefix's targets "
                            "from its prefix shard; no data-path collective (results stay on the owning rank)"}
        return {"route": "prefix", "scaling": "weak", "ms_per_step": ms, "value": q_tot / (ms * 1e-3),
                "unit": "queries/s", "workload": f"{a.q} targets x {a.n} ids per GPU ({q_tot} x {n_tot} over {world})",
                "ids_rank": c.num_ids, "targets_rank": ql,
                "note": "a different (N times larger) problem than the headline's; no data-path collective"}
    finally:
        c.close()
        torch.cuda.synchronize()


def cfg3_multi_leg(a, L, dev, stream, tstream, world, rank):
    """BASELINE cfg 3 over the ranks: 10^9 ids, 2^20 targets, k = 8, each route timed with two steps
    in flight (one step's exchange + merge, or F3 / F4, beside the next step's K6):
      broadcast  SURVEY 8(e) north star: id-range shards, every target on every rank, K6 record form,
                 one RCCL all-gather of q*k*12 B, K3 over the world's lists + the tie exchange; beside
                 it the same route with an all-to-all by target slice;
      prefix     ids and targets routed by their top log2(N) bits, no collective on the data path,
                 global indices.
    Each route carries an aggregate roofline (every rank's F2 / step algorithmic bytes over the slowest
    rank's time, against N x 8 TB/s; per-rank inputs = cfg3_rank_setup, the shapes the one-GPU
    cfg3_<route>_rank legs measure) and rank 0's rows are verified against the generator-fed oracle
    over the 10^9-id stream (32 targets)."""
    q, k = CFG3_Q, a.k
    out = {"workload": f"{q} targets x {CFG3_N} ids over {world} GPUs, k={k}", "inflight": 2}
    steps = 10
    D = 2
    RW = sharding.REC_WORDS

    def timed(step):
        for i in range(2 * D):
            step(i)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            step(i)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        tm = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        return float(tm.item()) * 1e3 / steps

    def aggregate(c, tp, ts, ql, ms, record, mapped, route):
        """every rank's F2 and step algorithmic bytes over the slowest rank's times (serial calls)"""
        ev = EvSets(6, tstream)
        oi = torch.empty((max(ql, 1), k), dtype=torch.int32, device=dev)
        oc = torch.empty(max(ql, 1), dtype=torch.int32, device=dev)
        torch.cuda.set_stream(tstream)
        for _ in range(6):
            ev.arm(c)
            c.batch_topk_dev(tp.data_ptr(), ts, ql, k, oi.data_ptr(), oc.data_ptr(), None, 0, stream)
        kms = ev.mean_ms()
        _, _, surv, _ = c.batch_topk_timed(tp.data_ptr(), ts, ql, k, oi.data_ptr(), oc.data_ptr(), stream)
        alg = k6_step_bytes(c.num_ids, ql, k, surv, record=record, mapped=mapped)
        tb = pmc_traffic(f"cfg3{route}:{c.num_ids}x{ql}x{k}", "k_f2_filter")
        v = torch.tensor([float(alg["k_f2_filter"]), float(sum(alg.values())), float(tb or 0.0), 0.0 if tb else 1.0],
                         dtype=torch.float64, device=dev)
        slow = torch.tensor([kms[1]], dtype=torch.float64, device=dev)
        dist.all_reduce(v, op=dist.ReduceOp.SUM)
        dist.all_reduce(slow, op=dist.ReduceOp.MAX)
        f2b, sb, sm = float(v[0].item()), float(v[1].item()), float(slow.item())
        tball = float(v[2].item()) if float(v[3].item()) == 0.0 else None
        peak = HBM_PEAK_GBS * world
        return {"ranks": world, "kernel": "k_f2_filter", "alg_bytes_all_ranks": f2b, "slowest_rank_kernel_ms": sm,
                "achieved": f2b / (sm * 1e-3) / 1e9, "peak": peak, "unit": "GB/s",
                "frac": f2b / (sm * 1e-3) / 1e9 / peak,
                "traffic": tball / (sm * 1e-3) / 1e9 if tball else None, "traffic_bytes_all_ranks": tball,
                "step_alg_bytes_all_ranks": sb, "step_frac": sb / (ms * 1e-3) / 1e9 / peak,
                "how": "sum over ranks of the algorithmic bytes (k6_step_bytes) / the slowest rank's F2 event time "
                       "(frac) or the timed step (step_frac) / (ranks x 8 TB/s); traffic: the ranks' PMC bytes "
                       "when every rank's shape has a committed pass"}

    def verify(rows_idx, tgi):
        """rank 0: rows vs orc_topk_gen over the whole 10^9-id stream (global indices)"""
        O = oracle()
        tg = O.gen_ids(a.seed + 11, q)[tgi]
        want, _ = O.topk_gen(a.seed + 10, CFG3_N, tg, k, threads=usable_cpus())
        return {"verified_targets": int(len(tgi)), "verified_exact": bool(np.array_equal(rows_idx, want))}

    # broadcast route: all-gather (north star), then the all-to-all beside it
    c, tp, ts, ql, _, lo = cfg3_rank_setup(a.seed, "broadcast", L, dev, stream, rank, world)
    try:
        sts = [tstream, torch.cuda.Stream(dev)]
        recs = [torch.empty((q, k, RW), dtype=torch.int32, device=dev) for _ in range(D)]
        gath = [torch.empty((world * q, k, RW), dtype=torch.int32, device=dev) for _ in range(D)]
        ois = [torch.empty((q, k), dtype=torch.int32, device=dev) for _ in range(D)]
        ocs = [torch.empty(q, dtype=torch.int32, device=dev) for _ in range(D)]
        txs = [sharding.TieExchange(world, k, dev) for _ in range(D)]
        ops = sharding.LibOps(L, c, tp.data_ptr(), ts)

        def bstep(i):
            d = i % D
            torch.cuda.set_stream(sts[d])
            c.batch_topk_dev(tp.data_ptr(), ts, q, k, None, None, recs[d].data_ptr(), lo, sts[d].cuda_stream)
            g = sharding.gather_records(recs[d], out=gath[d])
            sharding.merge_allgather(ops, recs[d], g, k, ois[d], ocs[d], txs[d], lo, sts[d].cuda_stream)
        ms = timed(bstep)
        nt = []
        for d in range(D):
            torch.cuda.set_stream(sts[d])
            nt.append(sharding.settle_overflow_allgather(ops, recs[d], gath[d].view(world, q, k, RW), k, ois[d],
                                                         ocs[d], txs[d], lo, sts[d].cuda_stream))
        torch.cuda.set_stream(tstream)
        torch.cuda.synchronize()
        row = {"ms_per_step": ms, "qps": q / (ms * 1e-3), "ids_per_gpu": c.num_ids, "record_bytes_per_gpu": q * k * 12,
               "allgather_bytes_in_per_gpu": world * q * k * 12, "tie_rows": nt, "scaling": "strong (one global batch)"}
        row["roofline"] = {"aggregate": aggregate(c, tp, ts, q, ms, True, False, "broadcast")}
        ref = ois[(steps + 2 * D - 1) % D]
        if rank == 0 and not a.no_cpu:
            rows = np.linspace(0, q - 1, 32).astype(np.int64)
            row.update(verify(ref.cpu().numpy().view(np.uint32)[rows], rows))
        out["broadcast"] = row
        # the all-to-all by target slice: each rank receives and merges only its own q / world targets
        tlo, thi = sharding.shard_range(q, world, rank)
        qm = thi - tlo
        exs = [torch.empty((world * qm, k, RW), dtype=torch.int32, device=dev) for _ in range(D)]
        oms = [torch.empty((max(qm, 1), k), dtype=torch.int32, device=dev) for _ in range(D)]
        ocms = [torch.empty(max(qm, 1), dtype=torch.int32, device=dev) for _ in range(D)]
        txa = [sharding.TieExchange(world, k, dev) for _ in range(D)]

        def astep(i):
            d = i % D
            torch.cuda.set_stream(sts[d])
            c.batch_topk_dev(tp.data_ptr(), ts, q, k, None, None, recs[d].data_ptr(), lo, sts[d].cuda_stream)
            ex = sharding.exchange_records(recs[d], out=exs[d])
            sharding.merge_alltoall(ops, recs[d], ex, k, tlo, oms[d], ocms[d], txa[d], lo, sts[d].cuda_stream)
        ms = timed(astep)
        for d in range(D):
            torch.cuda.set_stream(sts[d])
            sharding.settle_overflow_alltoall(ops, recs[d], exs[d].view(world, qm, k, RW), k, tlo, oms[d], ocms[d],
                                              txa[d], lo, sts[d].cuda_stream)
        torch.cuda.set_stream(tstream)
        torch.cuda.synchronize()
        last = (steps + 2 * D - 1) % D
        agree = bool(torch.equal(oms[last][:qm], ref[tlo:thi])) if qm else True
        out["broadcast_alltoall"] = {"ms_per_step": ms, "qps": q / (ms * 1e-3), "ids_per_gpu": c.num_ids,
                                     "exchange_bytes_in_per_gpu": world * qm * k * 12,
                                     "equals_allgather_route": agree,
                                     "results": "distributed by target slice (shard_range(q, world, rank))",
                                     "scaling": "strong (one global batch)"}
    finally:
        torch.cuda.set_stream(tstream)
        c.close()
        torch.cuda.synchronize()
    # prefix route (global indices)
    c, tp, ts, ql, tgidx, _ = cfg3_rank_setup(a.seed, "prefix", L, dev, stream, rank, world)
    try:
        sts = [tstream, torch.cuda.Stream(dev)]
        ois = [torch.empty((max(ql, 1), k), dtype=torch.int32, device=dev) for _ in range(D)]
        ocs = [torch.empty(max(ql, 1), dtype=torch.int32, device=dev) for _ in range(D)]

        def pstep(i):
            d = i % D
            c.batch_topk_dev(tp.data_ptr(), ts, ql, k, ois[d].data_ptr(), ocs[d].data_ptr(), None, 0, sts[d].cuda_stream)
        ms = timed(pstep)
        row = {"ms_per_step": ms, "qps": q / (ms * 1e-3), "ids_per_gpu_rank0": c.num_ids, "targets_rank0": ql,
               "result_indices": "global", "scaling": "strong (one global batch, routed by prefix)"}
        row["roofline"] = {"aggregate": aggregate(c, tp, ts, ql, ms, False, True, "prefix")}
        if rank == 0 and not a.no_cpu and ql:
            rows = np.linspace(0, ql - 1, 32).astype(np.int64)
            got = ois[(steps + 2 * D - 1) % D].cpu().numpy().view(np.uint32)[rows]
            row.update(verify(got, tgidx[:ql].cpu().numpy().view(np.uint32)[rows].astype(np.int64)))
        out["prefix"] = row
    finally:
        c.close()
        torch.cuda.synchronize()
    return out


def cpu_baseline(O, ids, tg, a):
    """Oracle port on the host cores (rank 0, N = 1): std::partial_sort(xorCmp) over the cfg-2
    set on a bounded target sample, built g++ -O2 (the reference's Release flags) and -O3
    -march=native, each at --cpu-threads (default: every host CPU, nproc) and at the CPUs the job
    may run at once (affinity capped by the cgroup quota), and on 1 core; `value` is the BEST of
    these rates, with its build and thread count.  Plus the reference's own
    RoutingTable::findClosestNodes call pattern (cfg 1), the cfg-4 findBucket + commonBits loop and
    NodeCache::getCachedNodes."""
    m1 = min(24, tg.shape[0])
    uq = usable_cpus()
    thread_counts = sorted({a.cpu_threads, uq})
    rows, want = [], None

    def run(build):
        nonlocal want
        for th in thread_counts:
            t0 = time.perf_counter()
            got, _ = O.topk(ids, tg, a.k, threads=th)
            dt = time.perf_counter() - t0
            if want is None:
                want = got
            rows.append({"build": build, "cores": th, "value": tg.shape[0] / dt, "wall_s": dt,
                         "same_results": bool(np.array_equal(got, want))})
        t0 = time.perf_counter()
        O.topk(ids, tg[:m1], a.k, threads=1)
        d1 = time.perf_counter() - t0
        rows.append({"build": build, "cores": 1, "value": m1 / d1, "wall_s": d1, "targets": m1})
    run("g++ -O2 (the reference's Release)")
    try:
        with O.native():
            run("g++ -O3 -march=native")
    except (OSError, subprocess.CalledProcessError) as e:
        rows.append({"build": "g++ -O3 -march=native", "error": str(e)[:200]})
    best = max((r for r in rows if "value" in r and r.get("targets") is None), key=lambda r: r["value"])
    cb = {"value": best["value"], "unit": "queries/s", "cores": best["cores"], "kind": "port",
          "compiler": best["build"],
          "sample": f"{tg.shape[0]} targets x {ids.shape[0]} ids, k={a.k}, std::partial_sort(xorCmp) per target; "
                    f"value = the best of the rows below ({best['build']}, {best['cores']} threads)",
          "rows": rows, "cpu_model": cpu_model(), "host_cpus": os.cpu_count(), **cpu_share(),
          "one_core": max((r for r in rows if r.get("cores") == 1 and "value" in r), key=lambda r: r["value"])}
    # cfg 1: findClosestNodes per target over the onNewNode-grown 10k-id table; the oracle grows
    # the same table from the same ids (its restated onNewNode) and must agree
    myid, firsts, off, nodes = cfg1_table(a.seed)
    rng = np.random.default_rng(a.seed)
    rng.bytes(20)
    of, oo, on = O.Table(myid).grow(np.frombuffer(rng.bytes(20 * 10000), dtype=np.uint8).reshape(-1, 20)).export()
    same_table = bool(np.array_equal(of, firsts) and np.array_equal(oo, off) and np.array_equal(on, nodes))
    good = np.ones(nodes.shape[0], np.uint8)
    tq = np.frombuffer(np.random.default_rng(a.seed + 1).bytes(20 * 1_000_000), dtype=np.uint8).reshape(-1, 20).copy()
    fc = {}
    for th in (1, a.cpu_threads):
        O.find_closest_batch(firsts, off, nodes, good, tq[:1000], 8, threads=th)
        t0 = time.perf_counter()
        O.find_closest_batch(firsts, off, nodes, good, tq, 8, threads=th)
        d = time.perf_counter() - t0
        fc[f"threads_{th}"] = {"queries_per_s": tq.shape[0] / d, "us_per_query_per_core": d * th / tq.shape[0] * 1e6}
    cb["cfg1_find_closest"] = {"table": f"{firsts.shape[0]} buckets, {nodes.shape[0]} nodes, onNewNode-grown from "
                                        f"10,000 ids", "table_equals_oracle_onNewNode": same_table,
                               "targets": tq.shape[0], **fc,
                               "kind": "port (RoutingTable::findClosestNodes, src/routing_table.cpp:110-150, restated "
                                       "over the table snapshot)"}
    # cfg 4: findBucket + commonBits per id (src/routing_table.cpp:153-166, infohash.h:154-176)
    m4, f4 = cfg4_firsts(a.seed + 5)
    ids4 = O.gen_ids(a.seed + 6, 20_000_000)
    c4 = {}
    for th, n4 in ((1, 2_000_000), (a.cpu_threads, ids4.shape[0])):
        O.classify(f4, m4, ids4[:100_000], threads=th)
        t0 = time.perf_counter()
        O.classify(f4, m4, ids4[:n4], threads=th)
        d = time.perf_counter() - t0
        c4[f"threads_{th}"] = {"ids_per_s": n4 / d, "ns_per_id_per_core": d * th / n4 * 1e9, "ids": n4}
    cb["cfg4_classify"] = {"table": f"{f4.shape[0]} buckets (onNewNode-grown from 10^5 ids)", **c4,
                           "kind": "port (findBucket linear walk + commonBits, per id)"}
    del ids4
    # NodeCache::getCachedNodes over a 10^6-node cache
    cache = O.gen_ids(a.seed + 9, 1_000_000)
    cache = cache[np.lexsort(cache.T[::-1])]
    acc = np.ones(cache.shape[0], np.uint8)
    gc = {}
    for th in (1, a.cpu_threads):
        t0 = time.perf_counter()
        O.cached_nodes_batch(cache, acc, tq[:200_000], 14, threads=th)
        d = time.perf_counter() - t0
        gc[f"threads_{th}"] = {"queries_per_s": 200_000 / d}
    cb["get_cached_nodes"] = {"cache": "10^6 nodes, count 14", **gc, "kind": "port"}
    return cb, want


if __name__ == "__main__":
    # stdout carries the one JSON line only: everything else written to fd 1 from here on (RCCL's
    # version banner and warnings, HIP runtime messages, stray prints) goes to stderr instead
    _RESULT_FD = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    main()
