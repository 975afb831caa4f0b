"""Randomised GPU parity sweep: seeded random shapes (n from 1 to 2^21 ids, q from 1 to 4,096
targets, k from 1 to 32) and id distributions the fixed cases do not combine -- uniform, a few
shared 16-bit prefixes (clustered subtrees), a small pool drawn with replacement (equal ids:
ties break by the lower index, `xorCmp` + `partial_sort` order), low-entropy ids (only the last
bytes vary: w0 ties everywhere) -- with targets that are partly ids of the set.  K1 (scan),
K4/K5 (bucket index) and K6 (batch prefix filter, and its small-batch path for q <= 64) are all
compared with std::partial_sort(xorCmp) over every target.  Marked gpu."""
import numpy as np
import pytest

import merge_util as MU
import oracle as O
from test_gpu_parity import check_topk

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import opendht_amd
    c = opendht_amd.Context(0)
    yield c
    c.close()


def make_case(seed):
    rng = np.random.default_rng(seed)
    n = int(np.exp(rng.uniform(0, np.log(1 << 20))))
    q = int(rng.choice([1, 7, 64, 65, int(rng.integers(1, 3001))]))
    if seed >= 24:   # K6's full-batch plans: 2^20..2^21 ids, 1,024..4,096 targets
        n = int(rng.integers(1 << 20, (1 << 21) + 1))
        q = int(rng.integers(1024, 4097))
    k = int(rng.choice([1, 3, 8, 8, 16, 20, 32]))
    kind = ("uniform", "clustered", "pool", "lowentropy")[seed % 4]
    ids = rng.integers(0, 256, size=(n, 20), dtype=np.uint8)
    if kind == "clustered":
        heads = rng.integers(0, 256, size=(int(rng.integers(1, 9)), 2), dtype=np.uint8)
        ids[:, :2] = heads[rng.integers(0, len(heads), n)]
    elif kind == "pool":
        pool = rng.integers(0, 256, size=(max(1, n // 3), 20), dtype=np.uint8)
        ids = pool[rng.integers(0, len(pool), n)]
    elif kind == "lowentropy":
        ids[:, :17] = rng.integers(0, 256, size=17, dtype=np.uint8)
    tg = rng.integers(0, 256, size=(q, 20), dtype=np.uint8)
    if kind != "uniform":   # targets from the ids' distribution: inside the dense subtrees
        take = rng.random(q) < 0.5
        tg[take] = ids[rng.integers(0, n, int(take.sum()))]
        tg[take, 19] ^= rng.integers(0, 256, int(take.sum()), dtype=np.uint8)
    return np.ascontiguousarray(ids), np.ascontiguousarray(tg), k, kind


@pytest.mark.parametrize("seed", range(32))
def test_random_shapes(ctx, seed):
    ids, tg, k, kind = make_case(seed)
    check_topk(ctx, ids, tg, k)


def make_edge_case(seed):
    """Boundary shapes: n at or next to a power of two (plan levels flip there), n < k, q
    around the small-batch limit (64 / 65) and K6's target-bucket sizes, exact-hit targets
    (distance 0), ids sorted by key (F2 blocks see one prefix range each)."""
    rng = np.random.default_rng(10_000 + seed)
    p = int(rng.integers(0, 22))
    n = max(1, (1 << p) + int(rng.choice([-1, 0, 1, 3])))
    q = int(rng.choice([1, 2, 63, 64, 65, 66, 255, 256, 257, int(rng.integers(1, 2049))]))
    k = int(rng.integers(1, 33))
    ids = rng.integers(0, 256, size=(n, 20), dtype=np.uint8)
    if seed % 3 == 1:   # sorted by the full key
        ids = ids[np.lexsort(ids.T[::-1])]
    tg = rng.integers(0, 256, size=(q, 20), dtype=np.uint8)
    hit = rng.random(q) < 0.3
    tg[hit] = ids[rng.integers(0, n, int(hit.sum()))]   # exact hits
    return np.ascontiguousarray(ids), np.ascontiguousarray(tg), k


@pytest.mark.parametrize("seed", range(48))
def test_edge_shapes(ctx, seed):
    ids, tg, k = make_edge_case(seed)
    check_topk(ctx, ids, tg, k)


@pytest.mark.parametrize("seed", range(16))
def test_find_closest_random_tables(ctx, seed):
    """RoutingTable::findClosestNodes (K1r) on random tables: node count, expired fraction,
    a cluster near myid (deep buckets), count from 1 to 32; every target vs the oracle."""
    rng = np.random.default_rng(20_000 + seed)
    myid = rng.integers(0, 256, size=20, dtype=np.uint8)
    ids = rng.integers(0, 256, size=(int(rng.integers(1, 20001)), 20), dtype=np.uint8)
    if seed % 2:
        m = int(rng.integers(1, 10))
        ids[: ids.shape[0] // 2, :m] = myid[:m]
    firsts, off, nodes = O.Table(myid).grow(ids).export()
    good = (rng.random(nodes.shape[0]) >= rng.uniform(0, 0.9)).astype(np.uint8)
    tg = rng.integers(0, 256, size=(int(rng.integers(1, 300)), 20), dtype=np.uint8)
    if nodes.shape[0]:
        tg = np.concatenate([tg, nodes[rng.integers(0, nodes.shape[0], 8)]])
    count = int(rng.integers(1, 33))
    got, cnt = ctx.find_closest(firsts, off, nodes, good, tg, count)
    for qi in range(tg.shape[0]):
        want = O.find_closest(firsts, off, nodes, good, tg[qi], count)
        assert cnt[qi] == len(want) and list(got[qi, : cnt[qi]]) == list(want), (seed, qi)


@pytest.mark.parametrize("seed", range(16))
def test_cached_nodes_random(ctx, seed):
    """NodeCache::getCachedNodes (a8) on random sorted caches: size, accept fraction, count,
    targets on and between cached ids; every target vs the oracle."""
    rng = np.random.default_rng(30_000 + seed)
    n = int(rng.integers(1, 60001))
    ids = rng.integers(0, 256, size=(n, 20), dtype=np.uint8)
    if seed % 3 == 2:
        ids[: n // 2, :6] = ids[0, :6]
    s = np.unique(ids, axis=0)   # a std::map: unique keys, sorted
    acc = (rng.random(s.shape[0]) < rng.uniform(0.05, 1.0)).astype(np.uint8)
    ctx.set_ids(np.ascontiguousarray(s))
    tg = np.concatenate([rng.integers(0, 256, size=(int(rng.integers(1, 200)), 20), dtype=np.uint8),
                         s[rng.integers(0, s.shape[0], 6)], s[:1], s[-1:]])
    count = int(rng.integers(1, 33))
    got, cnt = ctx.cached_nodes(tg, count, acc)
    for qi in range(tg.shape[0]):
        want = O.cached_nodes(s, acc, tg[qi], count)
        assert list(got[qi, : cnt[qi]]) == list(want), (seed, qi)


@pytest.mark.parametrize("seed", range(12))
def test_prefix_shards_random(ctx, seed):
    """Prefix shards (SURVEY 8(e) routing) of random streams: pbits 1..8, random pval and k;
    the shard's own targets get the full set's answer in global stream indices, foreign
    targets the shard's own top-k (K1, K4/K5 and K6 where they apply)."""
    rng = np.random.default_rng(40_000 + seed)
    n = int(rng.integers(1000, (1 << 20) + 1))
    pbits = int(rng.integers(1, 9))
    pval = int(rng.integers(0, 1 << pbits))
    k = int(rng.integers(1, 33))
    sd = 50 + seed
    ids = O.gen_ids(sd, n)
    top = lambda a: a[:, 0].astype(np.uint32) >> (8 - pbits)
    ctx.gen_ids_prefix(sd, n, pbits, pval)
    shard = ids[top(ids) == pval]
    assert ctx.num_ids == shard.shape[0]
    tg = rng.integers(0, 256, size=(int(rng.integers(1, 1500)), 20), dtype=np.uint8)
    own = tg.copy()
    own[:, 0] = (own[:, 0] & (0xFF >> pbits)) | (pval << (8 - pbits))
    if shard.shape[0] >= k:   # the full set's top-k of an own-prefix target lies in the shard
        want, wcnt = O.topk(ids, own, k)
        for name, fn in (("scan", ctx.topk), ("index", ctx.index_topk), ("batch", ctx.batch_topk)):
            got, cnt = fn(own, k)
            assert np.array_equal(cnt, wcnt) and np.array_equal(got, want), (seed, name)
    gl = np.nonzero(top(ids) == pval)[0].astype(np.uint32)
    w2, c2 = O.topk(shard, tg, k)
    w2 = np.where(w2 == 0xFFFFFFFF, w2, gl[np.minimum(w2, max(gl.size - 1, 0))] if gl.size else w2)
    for name, fn in (("scan", ctx.topk), ("batch", ctx.batch_topk)):
        got, cnt = fn(tg, k)
        assert np.array_equal(cnt, c2) and np.array_equal(got, w2), (seed, name)


@pytest.mark.parametrize("seed", range(10))
def test_record_shards_merge_random(ctx, seed):
    """The broadcast route's building block at random shapes: the id set cut into 1..5 range
    shards at random bounds (one context each, idx_base = the shard's start), every shard
    answering the whole batch in record form (K6 or K1 alternately), K3 merging the shard
    records: == one flat top-k of the whole set."""
    import torch
    import opendht_amd
    rng = np.random.default_rng(50_000 + seed)
    n = int(rng.integers(50, 300_001))
    q = int(rng.integers(1, 1500))
    k = int(rng.integers(1, 33))
    ids = rng.integers(0, 256, size=(n, 20), dtype=np.uint8)
    if seed % 2:
        ids[: n // 3, :3] = ids[0, :3]
    tg = rng.integers(0, 256, size=(q, 20), dtype=np.uint8)
    nsh = int(rng.integers(1, 6))
    bounds = [0] + sorted(int(x) for x in rng.integers(0, n + 1, nsh - 1)) + [n]
    dev = torch.device("cuda", 0)
    ts = (q + 63) // 64 * 64
    tp = torch.zeros(5 * ts, dtype=torch.int32, device=dev)
    L = opendht_amd.lib()
    tb = torch.from_numpy(tg.reshape(-1)).to(dev)
    torch.cuda.synchronize()
    assert L.dhtgpu_pack_dev(tb.data_ptr(), q, tp.data_ptr(), ts, None) == 0
    torch.cuda.synchronize()
    rec = torch.empty((nsh, q, k, 3), dtype=torch.int32, device=dev)
    for s in range(nsh):
        c = opendht_amd.Context(0)
        c.set_ids(np.ascontiguousarray(ids[bounds[s]:bounds[s + 1]]))
        fn = c.batch_topk_dev if (s + seed) % 2 == 0 else c.topk_dev
        fn(tp.data_ptr(), ts, q, k, None, None, rec[s].data_ptr(), bounds[s], c.stream)
        torch.cuda.synchronize()
        c.close()
    out, cnt, _ = MU.merge(L, rec, tp, ts, k, ("host", MU.host_words_fn(ids, rec.cpu().numpy().view(np.uint32))))
    want, wcnt = O.topk(ids, tg, k)
    assert np.array_equal(cnt, wcnt), seed
    assert np.array_equal(out, want), seed


@pytest.mark.parametrize("seed", range(4))
def test_subpartitioned_random(ctx, seed):
    """Sets past one K6 plan at random shapes (n in (2^24, 2^26], q in [2^14, 2^17], random k):
    the library sub-partitions them; whole batch == K1 scan, a sample == the oracle."""
    rng = np.random.default_rng(60_000 + seed)
    n = int(rng.integers((1 << 24) + 1, (1 << 26) + 1))
    q = int(rng.integers(1 << 14, (1 << 17) + 1))
    k = int(rng.integers(1, 33))
    ctx.gen_ids(700 + seed, n)
    tg = rng.integers(0, 256, size=(q, 20), dtype=np.uint8)
    got, cnt = ctx.batch_topk(tg, k)
    sc, scnt = ctx.topk(tg, k)
    assert np.array_equal(cnt, scnt) and np.array_equal(got, sc), (seed, n, q, k)
    rows = np.unique(np.r_[rng.integers(0, q, 6), [0, q - 1]])
    want, wcnt = O.topk(O.gen_ids(700 + seed, n), tg[rows], k, threads=16)
    assert np.array_equal(got[rows], want) and np.array_equal(cnt[rows], wcnt)


def test_subpartition_overfull():
    """2^25 ids (two prefix sub-partitions by the top bit) with 75 % of them moved into
    sub-partition 0 (~2^24.6 ids: more than one K6 plan serves): the call must still be exact
    (K6 == K1 scan on the whole batch, a sample == the oracle)."""
    import opendht_amd
    n, q, k = 1 << 25, 1 << 17, 8
    ids = O.gen_ids(8080, n)
    ids[: 3 * n // 4, 0] &= 0x7F
    tg = O.gen_ids(8081, q)
    c = opendht_amd.Context(0)
    try:
        c.set_ids(ids)
        got, cnt = c.batch_topk(tg, k)
        sc, scnt = c.topk(tg, k)
        assert np.array_equal(cnt, scnt) and np.array_equal(got, sc)
        rows = np.r_[np.arange(0, q, q // 8), [q - 1]]
        want, wcnt = O.topk(ids, tg[rows], k, threads=16)
        assert np.array_equal(got[rows], want) and np.array_equal(cnt[rows], wcnt)
    finally:
        c.close()


@pytest.mark.parametrize("seed", range(8))
def test_search_batch_random(ctx, seed):
    """Crawl-model searches on random networks: size from 20 to 200,000 nodes, dead fraction up
    to 0.7, clustered ids on odd seeds, random max_rounds; list for list vs the oracle model."""
    rng = np.random.default_rng(70_000 + seed)
    n = int(np.exp(rng.uniform(np.log(20), np.log(200_000))))
    ids = rng.integers(0, 256, size=(n, 20), dtype=np.uint8)
    if seed % 2:
        ids[: n // 2, :2] = ids[0, :2]
    ids = np.unique(ids, axis=0)
    ids = ids[rng.permutation(ids.shape[0])]
    n = ids.shape[0]
    dead = (rng.random(n) < rng.uniform(0, 0.7)).astype(np.uint8) if seed % 4 else None
    q = int(rng.integers(1, 600))
    tg = rng.integers(0, 256, size=(q, 20), dtype=np.uint8)
    hit = rng.random(q) < 0.2
    tg[hit] = ids[rng.integers(0, n, int(hit.sum()))]
    sr = rng.integers(0, n, q).astype(np.uint32)
    rounds = int(rng.choice([1, 3, 8, 64]))
    ctx.set_ids(np.ascontiguousarray(ids))
    ctx.net_prepare(dead, table_seed=seed + 1)
    got = ctx.search_batch(tg, sr, rounds)
    want = O.search_batch(ids, dead, seed + 1, tg, sr, rounds)
    for g, w, nm in zip(got, want, ["idx", "flags", "len", "rounds", "queries"]):
        bad = np.nonzero((g != w).reshape(g.shape[0], -1).any(axis=1))[0]
        assert bad.size == 0, f"seed {seed} {nm}: {bad.size} searches differ, first {bad[:5]}"


@pytest.mark.parametrize("seed", range(3))
def test_subpartitioned_random_handles(ctx, seed):
    """Random sub-partitioned shapes with sub-partition handles on: when the call returns handles,
    mapping them back (dhtgpu_handles_to_indices_dev) gives exactly the K1 scan's indices."""
    import torch
    rng = np.random.default_rng(61_000 + seed)
    n = int(rng.integers((1 << 25) + 1, (1 << 26) + 1))
    q = int(rng.integers(1 << 17, (1 << 18) + 1))
    k = int(rng.integers(1, 33))
    ctx.gen_ids(710 + seed, n)
    tg = rng.integers(0, 256, size=(q, 20), dtype=np.uint8)
    sc, scnt = ctx.topk(tg, k)
    ctx.set_sub_handles(True)
    try:
        active = ctx.sub_handles_active(q, k)
        h, cnt = ctx.batch_topk(tg, k)
    finally:
        ctx.set_sub_handles(False)
    assert np.array_equal(cnt, scnt), (seed, n, q, k)
    if not active:   # one K6 plan served it: ordinary indices
        assert np.array_equal(h, sc)
        return
    dev = torch.device("cuda", 0)
    hd = torch.from_numpy(h.reshape(-1).view(np.int32)).to(dev)
    out = torch.empty_like(hd)
    ctx.handles_to_indices_dev(hd.data_ptr(), hd.numel(), out.data_ptr(), 0, None)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32).reshape(h.shape)
    bad = np.nonzero((got != sc).any(axis=1))[0]
    assert bad.size == 0, (seed, n, q, k, bad[:4])
