"""GPU parity at BASELINE.json's full sizes (cfg 3 shard, cfg 4, cfg 5) and for the paths
that only large or non-uniform sets reach: K6 over prefix sub-partitions, sub-partitions
with fewer than k ids, the clustered-id fallback scan, two contexts on two host threads.
Checked against the CPU oracle on target samples, and on whole batches against the
independent K1 scan (a size-independent cross-check).  Marked gpu."""
import threading
import time

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import opendht_amd
    c = opendht_amd.Context(0)
    yield c
    c.close()


def sample_rows(q, m):
    return np.unique(np.r_[np.linspace(0, q - 1, m).astype(np.int64), [0, q - 1]])


def test_cfg3_shard_2p27(ctx):
    """The per-GPU shard of cfg 3 (1e9 ids over 8 GPUs ~ 2^27 ids) with 131,072 targets: one
    K6 plan cannot cover it, so the library splits the set into 8 prefix sub-partitions of 2^24
    and answers every target from its own (was DHTGPU_ERANGE).  Whole batch == K1 scan, a
    sample == std::partial_sort(xorCmp); the record form + K3 merge gives the same answer."""
    import torch
    import opendht_amd
    n, q, k = 1 << 27, 131072, 8
    ctx.gen_ids(777, n)
    tg = O.gen_ids(778, q)
    got, cnt = ctx.batch_topk(tg, k)
    assert np.all(cnt == k)
    sc, scnt = ctx.topk(tg, k)
    assert np.array_equal(cnt, scnt)
    bad = np.nonzero((got != sc).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} targets differ from the K1 scan, first {bad[:5]}"
    rows = sample_rows(q, 48)
    ids = O.gen_ids(777, n)
    want, wcnt = O.topk(ids, tg[rows], k, threads=16)
    assert np.array_equal(got[rows], want) and np.array_equal(cnt[rows], wcnt)
    # device form with candidate records, merged by K3 (the broadcast route's building block)
    dev = torch.device("cuda", 0)
    ts = (q + 63) // 64 * 64
    tp = torch.zeros(5 * ts, dtype=torch.int32, device=dev)
    L = opendht_amd.lib()
    tb = torch.from_numpy(tg.reshape(-1)).to(dev)
    rec = torch.empty((q, k, 3), dtype=torch.int32, device=dev)
    out = torch.empty((q, k), dtype=torch.int32, device=dev)
    oc = torch.empty(q, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    s = ctx.stream   # every launch below on the context's stream (stream-ordered)
    assert L.dhtgpu_pack_dev(tb.data_ptr(), q, tp.data_ptr(), ts, s) == 0
    ctx.batch_topk_dev(tp.data_ptr(), ts, q, k, None, None, rec.data_ptr(), 0, s)
    assert L.dhtgpu_merge_dev(rec.data_ptr(), 1, q, k, tp.data_ptr(), ts, k, out.data_ptr(), oc.data_ptr(), None, 0,
                              s) == 0
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), got)
    r = rec.cpu().numpy().view(np.uint32)
    assert np.array_equal(r[..., 2], got)
    w = ids[got[rows].astype(np.int64)].view(">u4").reshape(rows.size, k, 5)
    assert np.array_equal(r[rows, :, :2], w[..., :2].astype(np.uint32))


def test_cfg3_full_1e9_range_shards():
    """BASELINE cfg 3 at its stated size: 10^9 ids as the 8 range shards of
    sharding.shard_range(10^9, 8, r), each generated on its own context (one at a time: one GPU's
    share), 2^20 targets.  Per shard: K6 in record form with idx_base = lo (the library splits each
    1.25*10^8-id shard into 8 prefix sub-partitions); the 8 record lists concatenated exactly as the
    all-gather delivers them; K3 with lists = 8.  Checks: every count is 8; no row ties on 64 bits
    (hash ids; the tie exchange then settles nothing); the whole merged batch == one independent
    exact route, a single sub-partitioned K6 over all 10^9 ids (64 prefix sub-partitions); 40
    strided targets == std::partial_sort(xorCmp) over the 10^9-id stream (the generator-fed oracle:
    no 20-GB host array).  Reference: include/opendht/infohash.h:179-194; SURVEY 8(e)."""
    import torch
    import opendht_amd
    from opendht_amd import sharding
    n, q, k, world, seed = 10**9, 1 << 20, 8, 8, 1010
    L = opendht_amd.lib()
    dev = torch.device("cuda", 0)
    tg = O.gen_ids(1011, q)
    ts = q
    tp = torch.zeros(5 * ts, dtype=torch.int32, device=dev)
    assert L.dhtgpu_pack_dev(torch.from_numpy(tg.reshape(-1)).to(dev).data_ptr(), q, tp.data_ptr(), ts, None) == 0
    rec = torch.empty((world, q, k, 3), dtype=torch.int32, device=dev)
    t0 = time.perf_counter()
    with opendht_amd.Context(0) as c:
        for r in range(world):
            lo, hi = sharding.shard_range(n, world, r)
            c.gen_ids(seed, hi - lo, start=lo)
            c.batch_topk_dev(tp.data_ptr(), ts, q, k, None, None, rec[r].data_ptr(), lo, c.stream)
            torch.cuda.synchronize()
    t_shards = time.perf_counter() - t0
    out = torch.empty((q, k), dtype=torch.int32, device=dev)
    cnt = torch.empty(q, dtype=torch.int32, device=dev)
    ties = torch.zeros(1 + sharding.TIE_CAP, dtype=torch.int32, device=dev)
    assert L.dhtgpu_merge_dev(rec.data_ptr(), world, q, k, tp.data_ptr(), ts, k, out.data_ptr(), cnt.data_ptr(),
                              ties.data_ptr(), sharding.TIE_CAP, None) == 0
    torch.cuda.synchronize()
    assert int(ties[0].item()) == 0
    got = out.cpu().numpy().view(np.uint32)
    gcnt = cnt.cpu().numpy().view(np.uint32)
    del rec, out, cnt
    assert np.all(gcnt == k)
    t0 = time.perf_counter()
    with opendht_amd.Context(0) as c:
        c.gen_ids(seed, n)
        one, ocnt = c.batch_topk(tg, k)
    t_one = time.perf_counter() - t0
    assert np.array_equal(ocnt, gcnt)
    bad = np.nonzero((one != got).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} targets differ between the routes, first {bad[:5]}"
    rows = sample_rows(q, 40)
    t0 = time.perf_counter()
    want, wcnt = O.topk_gen(seed, n, tg[rows], k, threads=16)
    print(f"cfg3 full: 8 shards {t_shards:.1f} s, one-set route {t_one:.1f} s, oracle {time.perf_counter() - t0:.1f} s")
    assert np.array_equal(got[rows], want) and np.array_equal(gcnt[rows], wcnt)


def test_subpartition_with_fewer_than_k_ids(ctx):
    """2^26 ids whose prefix-11 quarter is emptied down to 5 ids, 2^18 targets (K6 plans this
    over 4 sub-partitions): targets with prefix 11 must take ids from outside their
    sub-partition, so the library routes them to the K1 scan over the whole set."""
    n, q, k = 1 << 26, 1 << 18, 8
    ids = O.gen_ids(2626, n)
    top = ids[:, 0] >> 6
    move = np.nonzero(top == 3)[0][5:]
    ids[move, 0] &= 0x7F                     # prefix 11 -> 01: sub-partition 3 keeps 5 ids
    ctx.set_ids(ids)
    tg = O.gen_ids(2627, q)
    got, cnt = ctx.batch_topk(tg, k)
    sc, scnt = ctx.topk(tg, k)
    assert np.array_equal(cnt, scnt) and np.array_equal(got, sc)
    rows = np.r_[sample_rows(q, 24), np.nonzero((tg[:, 0] >> 6) == 3)[0][:24]]
    want, wcnt = O.topk(ids, tg[rows], k, threads=16)
    assert np.array_equal(got[rows], want) and np.array_equal(cnt[rows], wcnt)


def test_subpartitions_k_sequence_fresh_context():
    """Sub-partition descriptor tables after a change of k on the same workspace: their offsets
    in the workspace move with k (they sit after the k-sized fallback records), and a call that
    reused the cached table signature without re-uploading read stale descriptors (a fault, once
    the workspace was large enough not to be reallocated).  k = 32 first (the largest workspace),
    then smaller k on the same context: every call == K1 scan."""
    import opendht_amd
    n, q = 1 << 25, 1 << 18   # q large enough that one plan cannot serve: 2 sub-partitions
    c = opendht_amd.Context(0)
    try:
        c.gen_ids(3131, n)
        tg = O.gen_ids(3132, q)
        for k in (32, 1, 3, 8, 16, 3):
            got, cnt = c.batch_topk(tg, k)
            sc, scnt = c.topk(tg, k)
            assert np.array_equal(cnt, scnt) and np.array_equal(got, sc), k
    finally:
        c.close()


@pytest.mark.parametrize("k", [1, 3, 16, 32])
def test_subpartitions_larger_k(ctx, k):
    """2^26 ids, 2^18 targets (4 prefix sub-partitions, one K6 launch sequence) at k = 1, 3, 16
    and 32 (k < 4: many empty mark-level subtrees, so the fallback scan's per-target form runs
    with its split cap): whole batch == K1 scan, a sample == std::partial_sort(xorCmp)."""
    n, q = 1 << 26, 1 << 18
    ctx.gen_ids(2929, n)
    tg = O.gen_ids(2930, q)
    got, cnt = ctx.batch_topk(tg, k)
    sc, scnt = ctx.topk(tg, k)
    assert np.array_equal(cnt, scnt) and np.array_equal(got, sc)
    rows = sample_rows(q, 16)
    want, wcnt = O.topk(O.gen_ids(2929, n), tg[rows], k, threads=16)
    assert np.array_equal(got[rows], want) and np.array_equal(cnt[rows], wcnt)


def test_subpartition_deficient_subtree_targets(ctx):
    """Sub-partitioned call (2^26 ids, 2^18 targets: 4 sub-partitions) where two targets' own
    level-18 subtrees (bits 2..19 after the 2 sub-partition bits; the mark level is 18 or 19)
    are emptied down to 3 ids:
    F3 lists them for the fallback scan, which for so short a list scans each target's own
    sub-partition (it holds >= k ids, so their top-k lies inside it).  Whole batch == K1 scan,
    the two targets == std::partial_sort(xorCmp)."""
    n, q, k = 1 << 26, 1 << 18, 8
    ids = O.gen_ids(2828, n)
    tg = O.gen_ids(2829, q)
    key = lambda a: ((a[:, 0].astype(np.uint32) << 16) | (a[:, 1].astype(np.uint32) << 8) | a[:, 2]) >> 4
    tk, ik = key(tg), key(ids)
    picks = [101, 202]
    for t in picks:
        inside = np.nonzero(ik == tk[t])[0][3:]
        ids[inside, 2] ^= 0x10           # bit 19: into the sibling subtree, same sub-partition
        ik = key(ids)
    ctx.set_ids(ids)
    got, cnt = ctx.batch_topk(tg, k)
    sc, scnt = ctx.topk(tg, k)
    assert np.array_equal(cnt, scnt) and np.array_equal(got, sc)
    want, wcnt = O.topk(ids, tg[picks], k, threads=16)
    assert np.array_equal(got[picks], want) and np.array_equal(cnt[picks], wcnt)


@pytest.mark.parametrize("q", [65536, 262144])
def test_subpartition_sibling_marking(ctx, q):
    """Sibling marking (round 6): 31.25 M ids = 2 prefix sub-partitions of ~1.56e7 with 65,536
    targets plan one level finer than the 4k rule (level-19 cells of ~30 ids) because the
    sub-partitions carry their level-19 cell counts: a target whose own cell holds < k ids marks the
    sibling cell too and answers from the complete pair.  Crafted: 48 targets' cells emptied down
    to 3 ids (moved into the sibling: the pair keeps them all), 16 targets' whole pairs emptied
    down to 2 + 2 ids (the pair is short: F3's fallback scan of the sub-partition).  Whole batch
    == K1 scan; the crafted targets and a sample == std::partial_sort(xorCmp).  q = 262,144: the
    survivors are dense (~22 %), so the sub-partitions are built prefix-sorted and F2 runs its
    bitmap window (the cfg-3 broadcast rank's route)."""
    n, k = 31_250_000, 8
    ids = O.gen_ids(3434, n)
    tg = O.gen_ids(3435, q)
    key = lambda a: ((a[:, 0].astype(np.uint32) << 12) | (a[:, 1].astype(np.uint32) << 4) | (a[:, 2] >> 4))
    ik, tk = key(ids), key(tg)
    rng = np.random.default_rng(3436)
    picks = rng.choice(q, 64, replace=False)
    for j, t in enumerate(picks):
        cell = tk[t]
        if j < 48:   # the cell keeps 3 ids, the rest move to the sibling cell (bit 19)
            inside = np.nonzero(ik == cell)[0][3:]
            ids[inside, 2] ^= 0x10
        else:        # cell and sibling keep 2 ids each, the rest move to the other pair (bit 18)
            for c_ in (cell, cell ^ 1):
                inside = np.nonzero(ik == c_)[0][2:]
                ids[inside, 2] ^= 0x20
        ik = key(ids)
    assert len(np.unique(ids, axis=0)) == n
    ctx.set_ids(ids)
    got, cnt = ctx.batch_topk(tg, k)
    sc, scnt = ctx.topk(tg, k)
    assert np.array_equal(cnt, scnt)
    bad = np.nonzero((got != sc).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} targets differ from the K1 scan, first {bad[:5]}"
    rows = np.r_[picks, sample_rows(q, 16)]
    want, wcnt = O.topk(ids, tg[rows], k, threads=16)
    assert np.array_equal(got[rows], want) and np.array_equal(cnt[rows], wcnt)


@pytest.mark.parametrize("n,q", [(1 << 22, 1 << 17), (1 << 25, 1 << 18)])
def test_f1_two_pass_clustered_targets(ctx, n, q):
    """F1's two-pass form (batches of >= 2^17 targets, round 6: coarse bins by workgroup-level
    reservations, then one workgroup per bin marking the bitmap and ranking the partitions in LDS):
    a quarter of the targets share their top 12 bits (their coarse bin overflows: those targets
    spill to the fallback scan from the first pass), and groups of 96, 256, 700 and 2,048 targets
    each share a 22-bit prefix (one partition's bucket overflows in the second pass, or the bin in
    the first, by size); one set and 2 sub-partitions.  Whole batch == K1 scan, a sample of each
    group == std::partial_sort(xorCmp)."""
    k = 8
    ctx.gen_ids(3737, n)
    tg = O.gen_ids(3738, q)
    a = q // 4
    tg[:a, 0] = 0xA7
    tg[:a, 1] = (tg[:a, 1] & 0x0F) | 0x30
    rows = [np.arange(0, a, a // 8)]
    lo = a
    for g, pre in zip((96, 256, 700, 2048), (0x1C44, 0x5B12, 0x9E60, 0xD301)):
        tg[lo:lo + g, 0] = pre >> 8
        tg[lo:lo + g, 1] = pre & 0xFF
        tg[lo:lo + g, 2] = (tg[lo:lo + g, 2] & 0x03) | 0x98
        rows.append(np.arange(lo, lo + g, g // 4))
        lo += g
    got, cnt = ctx.batch_topk(tg, k)
    sc, scnt = ctx.topk(tg, k)
    bad = np.nonzero((got != sc).any(axis=1) | (cnt != scnt))[0]
    if bad.size:   # which route is wrong: the oracle on the differing rows
        w, wc = O.topk(O.gen_ids(3737, n), tg[bad[:8]], k, threads=16)
        info = [(int(b), tg[b][:4].tobytes().hex(), got[b].tolist(), sc[b].tolist(), w[j].tolist())
                for j, b in enumerate(bad[:8])]
        pytest.fail(f"{bad.size} targets differ between K6 and the K1 scan: (row, target, K6, K1, oracle) {info}")
    rows = np.r_[np.concatenate(rows), sample_rows(q, 8)]
    want, wcnt = O.topk(O.gen_ids(3737, n), tg[rows], k, threads=16)
    assert np.array_equal(got[rows], want) and np.array_equal(cnt[rows], wcnt)


@pytest.mark.parametrize("k", [8, 32])
def test_clustered_ids_fallback_scan(ctx, k):
    """Verdict item 4: 2^24 ids of which 25 % share one 24-bit prefix, and targets inside the
    cluster.  The cluster's partition overflows K6's LDS stage, so its targets go to the K1
    fallback scan inside the same call (was: a 64-workgroup brute force per target).  Whole
    batch == K1 scan; oracle on a sample; the call costs no more than the plain K1 scan."""
    import opendht_amd  # noqa: F401
    n, q = 1 << 24, 65536
    ids = O.gen_ids(2424, n)
    ids[: n // 4, :3] = np.array([0x5A, 0xC3, 0x0F], np.uint8)
    ctx.set_ids(ids)
    tg = O.gen_ids(2425, q)
    tg[: q // 4, :3] = np.array([0x5A, 0xC3, 0x0F], np.uint8)
    ctx.batch_topk(tg[:256], k)          # warm-up (workspaces)
    t0 = time.perf_counter()
    got, cnt = ctx.batch_topk(tg, k)
    t_batch = time.perf_counter() - t0
    t0 = time.perf_counter()
    sc, scnt = ctx.topk(tg, k)
    t_scan = time.perf_counter() - t0
    print(f"clustered k={k}: K6 {t_batch * 1e3:.1f} ms, K1 {t_scan * 1e3:.1f} ms (host wall incl. transfers)")
    assert np.array_equal(cnt, scnt) and np.array_equal(got, sc)
    rows = np.r_[np.arange(0, q // 4, 997), np.arange(q // 4, q, 4999)]
    want, wcnt = O.topk(ids, tg[rows], k, threads=16)
    assert np.array_equal(got[rows], want) and np.array_equal(cnt[rows], wcnt)
    assert t_batch <= t_scan * 1.5 + 0.05


def test_cfg4_classify_1e8(ctx):
    """BASELINE cfg 4: bucket classification + commonBits histogram of 10^8 ids against a
    routing table grown from 10^5 ids: the whole histogram and every bucket index equal the
    oracle's findBucket + commonBits restatement."""
    n = 100_000_000
    myid = O.gen_ids(404, 1)[0]
    firsts, _, _ = O.Table(myid).grow(O.gen_ids(405, 100_000)).export()
    ctx.gen_ids(406, n)
    b, hist = ctx.classify(firsts, myid)
    ids = O.gen_ids(406, n)
    wb, wh = O.classify(firsts, myid, ids)
    assert int(hist.sum()) == n
    assert np.array_equal(hist, wh)
    assert np.array_equal(b, wb)


def test_cfg5_search_5e7(ctx):
    """BASELINE cfg 5: iterative searches over a 5*10^7-node network (10 % dead); 1,024
    searches equal the oracle's crawl model list for list."""
    n, m = 50_000_000, 1024
    ctx.gen_ids(2024, n)
    dead = (np.random.default_rng(2024).random(n) < 0.1).astype(np.uint8)
    ctx.net_prepare(dead, table_seed=2024)
    tg = O.gen_ids(2031, m)
    sr = ((np.arange(m, dtype=np.uint64) * 2654435761) % n).astype(np.uint32)
    got = ctx.search_batch(tg, sr)
    want = O.search_batch(O.gen_ids(2024, n), dead, 2024, tg, sr, 64, threads=16)
    for g, w, nm in zip(got, want, ["idx", "flags", "len", "rounds", "queries"]):
        bad = np.nonzero((g != w).reshape(g.shape[0], -1).any(axis=1))[0]
        assert bad.size == 0, f"{nm}: {bad.size} searches differ, first {bad[:5]}"


def test_two_contexts_two_threads():
    """One context per thread (the documented contract): two host threads drive K6 on two
    contexts of device 0 concurrently; every call matches the single-threaded answer."""
    import opendht_amd
    ids = [O.gen_ids(5150 + i, 200_000) for i in range(2)]
    tgs = [O.gen_ids(5160 + i, 4000) for i in range(2)]
    want = []
    with opendht_amd.Context(0) as c:
        for i in range(2):
            c.set_ids(ids[i])
            want.append(c.batch_topk(tgs[i], 8))
    errors = []

    def worker(i):
        try:
            with opendht_amd.Context(0) as c:
                c.set_ids(ids[i])
                for _ in range(25):
                    got = c.batch_topk(tgs[i], 8)
                    if not (np.array_equal(got[0], want[i][0]) and np.array_equal(got[1], want[i][1])):
                        errors.append(i)
                        return
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=100)
    assert not errors, errors


_TWO_THREAD_INDEX = r"""
import sys, threading
import numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/tests")
import opendht_amd, oracle as O
ids = [O.gen_ids(6150 + i, 300_000) for i in range(2)]
tgs = [O.gen_ids(6160 + i, 3000) for i in range(2)]
want = [O.topk(ids[i], tgs[i], 8, threads=8) for i in range(2)]
sr = (np.arange(500, dtype=np.uint64) * 7919 % 300_000).astype(np.uint32)
crawl_want = [O.search_batch(ids[i], None, 9 + i, tgs[i][:500], sr, threads=8) for i in range(2)]
errors, go = [], threading.Barrier(2)
def worker(i):
    try:
        with opendht_amd.Context(0) as c:
            c.set_ids(ids[i])
            go.wait()                      # both threads reach the first K4/K5 launch together
            for _ in range(6):
                got = c.index_topk(tgs[i], 8)
                if not (np.array_equal(got[0], want[i][0]) and np.array_equal(got[1], want[i][1])):
                    errors.append(("index", i)); return
            c.net_prepare(None, table_seed=9 + i)   # builds its order with the K4 index kernels
            got = c.search_batch(tgs[i][:500], sr)
            if not all(np.array_equal(g, w) for g, w in zip(got, crawl_want[i])):
                errors.append(("crawl", i))
    except Exception as e:
        errors.append(repr(e))
th = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
[t.start() for t in th]; [t.join(timeout=90) for t in th]
print("ERRORS", errors); sys.exit(1 if errors or any(t.is_alive() for t in th) else 0)
"""


def test_index_two_threads_fresh_process():
    """K4/K5 (index_topk) and the crawl network's order (net_prepare, built with the K4 kernels)
    driven from two host threads in a FRESH process, so both threads hit the first launch -- and
    the per-device once-only LDS attribute setup -- together (a plain static
    flag there raced).  Both threads' answers == the oracle."""
    import subprocess
    import sys
    root = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _TWO_THREAD_INDEX, root], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


def test_batches_over_three_streams(ctx):
    """Nine calls issued back to back over three streams without a synchronisation between them
    (the bench's --inflight 3: each stream keeps its own workspace slot), then the same batches
    one by one on the context's stream (every slot then changes streams: the cross-stream wait):
    the results agree, and a sample == std::partial_sort(xorCmp)."""
    import torch
    import opendht_amd
    n, q, k = 1 << 22, 16384, 8
    ctx.gen_ids(3131, n)
    dev = torch.device("cuda", 0)
    L = opendht_amd.lib()
    ts = (q + 63) // 64 * 64
    tgs = [O.gen_ids(3200 + i, q) for i in range(9)]
    tps = []
    for tg in tgs:
        tp = torch.zeros(5 * ts, dtype=torch.int32, device=dev)
        tb = torch.from_numpy(tg.reshape(-1)).to(dev)
        torch.cuda.synchronize()
        assert L.dhtgpu_pack_dev(tb.data_ptr(), q, tp.data_ptr(), ts, ctx.stream) == 0
        tps.append(tp)
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(dev) for _ in range(3)]
    outs = [(torch.empty((q, k), dtype=torch.int32, device=dev), torch.empty(q, dtype=torch.int32, device=dev))
            for _ in tgs]
    for i, tp in enumerate(tps):
        ctx.batch_topk_dev(tp.data_ptr(), ts, q, k, outs[i][0].data_ptr(), outs[i][1].data_ptr(), None, 0,
                           streams[i % 3].cuda_stream)
    torch.cuda.synchronize()
    for i, tg in enumerate(tgs):
        got, cnt = ctx.batch_topk(tg, k)
        assert np.array_equal(outs[i][0].cpu().numpy().view(np.uint32), got), f"batch {i}"
        assert np.array_equal(outs[i][1].cpu().numpy().view(np.uint32), cnt), f"batch {i}"
    rows = sample_rows(q, 16)
    want, wcnt = O.topk(O.gen_ids(3131, n), tgs[4][rows], k, threads=16)
    assert np.array_equal(outs[4][0].cpu().numpy().view(np.uint32)[rows], want)


def _handles_vs_indices(c, tg, k, base=0):
    """The same call with and without sub-partition handles; the handles mapped back on the
    device (dhtgpu_handles_to_indices_dev) must equal the indices, row for row."""
    import torch
    c.set_sub_handles(False)
    want, wcnt = c.batch_topk(tg, k)
    c.set_sub_handles(True)
    try:
        assert c.sub_handles_active(tg.shape[0], k)
        h, hcnt = c.batch_topk(tg, k)
    finally:
        c.set_sub_handles(False)
    assert np.array_equal(hcnt, wcnt)
    n = c.num_ids
    valid = h != 0xFFFFFFFF
    assert (h[valid] < n).all()
    dev = torch.device("cuda", 0)
    hd = torch.from_numpy(h.reshape(-1).view(np.int32)).to(dev)
    out = torch.empty_like(hd)
    c.handles_to_indices_dev(hd.data_ptr(), hd.numel(), out.data_ptr(), base, None)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32).reshape(h.shape)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} rows differ, first {bad[:4]}: {got[bad[0]]} vs {want[bad[0]]}"
    return h


@pytest.mark.parametrize("k", [8, 1, 3, 32])
def test_sub_handles_map_back(ctx, k):
    """Sub-partition handles (round 5, VERDICT r4 #2: no index-map read per result): 2^26 ids
    over 4 sub-partitions, 2^18 targets; every handle maps back to the index the call returns
    without handles (k < 4: the fallback scan's split merge), handles are a bijection onto [0, n)
    (two different ids never share one)."""
    n, q = 1 << 26, 1 << 18
    ctx.gen_ids(3737, n)
    tg = O.gen_ids(3738, q)
    h = _handles_vs_indices(ctx, tg, k)
    for row in h[:2000]:   # distinct ids within a row -> distinct handles
        r = row[row != 0xFFFFFFFF]
        assert np.unique(r).size == r.size


def test_sub_handles_whole_set_fallback(ctx):
    """Handles when targets fall back to the whole set (a sub-partition emptied below k ids:
    F4 scans the context's planes and converts its rows to handles by a binary search in the
    sub-partitions' index maps); and the prefix-shard form (global stream indices on the way
    back)."""
    n, q, k = 1 << 26, 1 << 18, 8
    ids = O.gen_ids(2626, n)
    top = ids[:, 0] >> 6
    move = np.nonzero(top == 3)[0][5:]
    ids[move, 0] &= 0x7F                     # prefix 11 -> 01: sub-partition 3 keeps 5 ids
    ctx.set_ids(ids)
    tg = O.gen_ids(2627, q)
    _handles_vs_indices(ctx, tg, k)
    import opendht_amd
    with opendht_amd.Context(0) as c:
        c.gen_ids_prefix(3939, 1 << 27, 1, 1)   # a 2^26-id prefix shard of a 2^27 stream
        _handles_vs_indices(c, O.gen_ids(3940, q), k)


def test_sub_handles_record_form_unaffected(ctx):
    """Record form ignores handles (records carry global indices for the cross-rank merge)."""
    import torch
    import opendht_amd
    n, q, k = 1 << 26, 1 << 18, 8
    ctx.gen_ids(3737, n)
    tg = O.gen_ids(3738, q)
    dev = torch.device("cuda", 0)
    ts = (q + 63) // 64 * 64
    tp = torch.zeros(5 * ts, dtype=torch.int32, device=dev)
    L = opendht_amd.lib()
    assert L.dhtgpu_pack_dev(torch.from_numpy(tg.reshape(-1)).to(dev).data_ptr(), q, tp.data_ptr(), ts, None) == 0
    recs = []
    for on in (False, True):
        ctx.set_sub_handles(on)
        r = torch.full((q, k, 3), -5, dtype=torch.int32, device=dev)
        ctx.batch_topk_dev(tp.data_ptr(), ts, q, k, None, None, r.data_ptr(), 7, ctx.stream)
        torch.cuda.synchronize()
        recs.append(r.cpu().numpy())
    ctx.set_sub_handles(False)
    assert np.array_equal(recs[0], recs[1])
