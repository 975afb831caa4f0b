"""GPU parity: libdhtgpu (HIP, gfx950) against the CPU oracle, bit-exact.
All calls go through the C ABI (ctypes).  Marked gpu: run on the MI355X box."""
import numpy as np
import pytest

import merge_util as MU
import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import opendht_amd
    c = opendht_amd.Context(0)
    yield c
    c.close()


def check_topk(ctx, ids, targets, k):
    """K1 (scan), K4/K5 (bucket index) and K6 (batch prefix filter) all bit-exact vs
    std::partial_sort(xorCmp)."""
    ctx.set_ids(ids)
    want, wcnt = O.topk(ids, targets, k)
    for name, fn in (("scan", ctx.topk), ("index", ctx.index_topk), ("batch", ctx.batch_topk)):
        got, gcnt = fn(targets, k)
        assert np.array_equal(gcnt, wcnt), name
        bad = np.nonzero((got != want).any(axis=1))[0]
        assert bad.size == 0, f"{name}: {bad.size} mismatching targets, first {bad[:5]}: got {got[bad[0]]} want {want[bad[0]]}"


def test_gen_matches_oracle(ctx):
    ctx.gen_ids(123, 10007, start=5)
    assert np.array_equal(ctx.get_ids(), O.gen_ids(123, 10007, start=5))


def test_set_get_roundtrip(ctx):
    ids = O.gen_ids(5, 4099)
    ctx.set_ids(ids)
    assert ctx.num_ids == 4099
    assert np.array_equal(ctx.get_ids(), ids)
    assert np.array_equal(ctx.get_ids(4000, 99), ids[4000:])


@pytest.mark.parametrize("n", [1, 7, 8, 9, 100, 4096, 5000, 70001])
@pytest.mark.parametrize("k", [1, 8, 14, 32])
def test_topk_sizes(ctx, n, k):
    check_topk(ctx, O.gen_ids(1000 + n, n), O.gen_ids(77, 150), k)


@pytest.mark.parametrize("q", [1, 2, 127, 128, 129, 1000, 4097])
def test_topk_batch_shapes(ctx, q):
    check_topk(ctx, O.gen_ids(31, 20000), O.gen_ids(32, q), 8)


def test_topk_targets_are_members(ctx):
    ids = O.gen_ids(41, 30000)
    check_topk(ctx, ids, ids[::997], 8)


def test_topk_clustered_w0_ties(ctx):
    """Many ids share their top 32 (even 64) bits with each other and with the
    targets: exercises the full 160-bit tie path of the scan."""
    ids = O.gen_ids(51, 40000)
    ids[:20000, :4] = ids[0, :4]
    ids[:5000, 4:8] = ids[0, 4:8]
    ids[20000:30000, :3] = 0
    tg = O.gen_ids(52, 300)
    tg[:100, :4] = ids[0, :4]
    tg[100:150, :8] = ids[0, :8]
    tg[150:200, :3] = 0
    check_topk(ctx, ids, tg, 8)
    check_topk(ctx, ids, tg, 32)


def test_index_adversarial_clusters(ctx):
    """Huge buckets (tens of thousands of ids sharing 40+ leading bits), a lone far id,
    targets inside/outside the clusters: exercises the index's take-child-and-descend
    iteration and its large-range selection."""
    ids = O.gen_ids(81, 60000)
    ids[:30000, :5] = 0x5A            # one big cluster (40 shared bits)
    ids[30000:45000, :3] = 0x00       # a second, 24-bit cluster
    ids[45000:45003, :6] = 0x5A       # 3 ids deeper inside the first cluster
    tg = O.gen_ids(82, 400)
    tg[:100, :5] = 0x5A
    tg[100:150, :7] = 0x5A
    tg[150:200, :2] = 0x00
    tg[200:220, 0] = 0x5B
    check_topk(ctx, ids, tg, 8)
    check_topk(ctx, ids, tg, 32)
    check_topk(ctx, ids[:5], tg, 8)


def test_topk_duplicates_tiebreak_by_index(ctx):
    base = O.gen_ids(61, 3000)
    ids = np.concatenate([base, base[::-1], base[:100]])
    tg = np.concatenate([base[:50], O.gen_ids(62, 50)])
    check_topk(ctx, ids, tg, 16)


def test_topk_empty_set(ctx):
    ctx.set_ids(np.zeros((0, 20), np.uint8))
    idx, cnt = ctx.topk(O.gen_ids(1, 5), 8)
    assert np.all(cnt == 0) and np.all(idx == 0xFFFFFFFF)


def test_topk_2p24_sample(ctx):
    """Cfg 2 set size (N = 2^24) with a target sample vs std::partial_sort(xorCmp)."""
    n = 1 << 24
    ctx.gen_ids(2024, n)
    tg = O.gen_ids(2025, 48)
    want, wcnt = O.topk(O.gen_ids(2024, n), tg, 8)
    for fn in (ctx.topk, ctx.index_topk, ctx.batch_topk):
        got, cnt = fn(tg, 8)
        assert np.array_equal(cnt, wcnt) and np.array_equal(got, want)


def test_index_vs_scan_full_batch(ctx):
    """Full cfg-2 batch (65,536 targets x 2^24 ids): the two independent GPU algorithms
    agree on every target (a size-independent cross-check; the oracle covers samples)."""
    ctx.gen_ids(2024, 1 << 24)
    tg = O.gen_ids(2025, 65536)
    a, ca = ctx.topk(tg, 8)
    b, cb = ctx.index_topk(tg, 8)
    assert np.array_equal(ca, cb) and np.array_equal(a, b)
    assert np.all(ca == 8)
    c, cc = ctx.batch_topk(tg, 8)
    assert np.array_equal(ca, cc) and np.array_equal(a, c)


def test_k6_cfg2_full_batch_vs_oracle(ctx):
    """The headline kernel at the headline size, pinned DIRECTLY to std::partial_sort(xorCmp)
    (VERDICT r2 weak #1): 2^24 ids, the whole 65,536-target batch through batch_topk (q > 64 ->
    the K6 path, not KS), 16 targets replaced by set members (exact hits, distance 0).  The oracle
    checks a strided sample, every exact hit, and every target whose top-9 holds two ids with equal
    word-0 distance (the w0 ties F3 defers to the exact wave path -- found with K1 at k = 9).
    The whole batch also == the K1 scan."""
    n, q, k = 1 << 24, 65536, 8
    ids = O.gen_ids(2024, n)
    ctx.gen_ids(2024, n)
    tg = O.gen_ids(2025, q)
    hits = np.arange(7, q, 4099)[:16]
    tg[hits] = ids[(hits * 977) % n]
    got, cnt = ctx.batch_topk(tg, k)
    assert np.all(cnt == k)
    sc, scnt = ctx.topk(tg, k)
    assert np.array_equal(cnt, scnt)
    bad = np.nonzero((got != sc).any(axis=1))[0]
    assert bad.size == 0, f"K6 vs K1: {bad.size} targets differ, first {bad[:5]}"
    assert np.array_equal(got[hits, 0], (hits * 977) % n)          # an exact hit is its own closest
    k9, _ = ctx.topk(tg, k + 1)
    w0 = ids[:, :4].view(">u4").reshape(-1).astype(np.uint32)
    t0 = tg[:, :4].view(">u4").reshape(-1).astype(np.uint32)
    d0 = w0[k9.astype(np.int64)] ^ t0[:, None]
    tie_rows = np.nonzero((d0[:, 1:] == d0[:, :-1]).any(axis=1))[0]
    assert tie_rows.size > 100, "a 2^24 uniform set has ~1,000 w0-tie targets per 65,536"
    rows = np.unique(np.r_[np.linspace(0, q - 1, 512).astype(np.int64), hits, tie_rows[:1024]])
    want, wcnt = O.topk(ids, tg[rows], k)
    assert np.array_equal(cnt[rows], wcnt)
    bad = np.nonzero((got[rows] != want).any(axis=1))[0]
    assert bad.size == 0, f"K6 vs oracle: {bad.size} of {rows.size} sampled targets differ, rows {rows[bad[:5]]}"


@pytest.mark.parametrize("expired,cluster", [(0.0, False), (0.3, False), (0.6, False), (0.3, True)])
def test_find_closest_vs_oracle(ctx, expired, cluster):
    myid = O.gen_ids(99, 1)[0]
    ids = O.gen_ids(100, 10000)
    if cluster:
        ids[:5000, :3] = myid[:3]
    firsts, off, nodes = O.Table(myid).grow(ids).export()
    rng = np.random.default_rng(7)
    good = (rng.random(nodes.shape[0]) >= expired).astype(np.uint8)
    tg = np.concatenate([O.gen_ids(101, 500), nodes[:40]])
    for count in (1, 8, 14, 32):
        got, cnt = ctx.find_closest(firsts, off, nodes, good, tg, count)
        for qi in range(tg.shape[0]):
            want = O.find_closest(firsts, off, nodes, good, tg[qi], count)
            assert cnt[qi] == len(want), (count, qi)
            assert list(got[qi, : cnt[qi]]) == list(want), (count, qi)
            assert np.all(got[qi, cnt[qi]:] == 0xFFFFFFFF)


def test_find_closest_empty_and_single_bucket(ctx):
    tg = O.gen_ids(5, 3)
    idx, cnt = ctx.find_closest(np.zeros((0, 20), np.uint8), np.zeros(1, np.uint32), [], [], tg, 8)
    assert np.all(cnt == 0)
    firsts, off, nodes = O.Table(O.gen_ids(6, 1)[0]).grow(O.gen_ids(7, 5)).export()
    good = np.ones(nodes.shape[0], np.uint8)
    idx, cnt = ctx.find_closest(firsts, off, nodes, good, tg, 8)
    for qi in range(3):
        assert list(idx[qi, : cnt[qi]]) == list(O.find_closest(firsts, off, nodes, good, tg[qi], 8))


def test_classify_vs_oracle(ctx):
    myid = O.gen_ids(1, 1)[0]
    firsts, _, _ = O.Table(myid).grow(O.gen_ids(2, 20000)).export()
    ids = O.gen_ids(3, 100003)
    ids[:50, :6] = myid[:6]      # populate deep commonBits bins
    ctx.set_ids(ids)
    b, hist = ctx.classify(firsts, myid)
    wb, wh = O.classify(firsts, myid, ids)
    assert np.array_equal(b, wb)
    assert np.array_equal(hist, wh)


@pytest.mark.parametrize("n,nb,seed", [(1, 1, 1), (5, 3, 2), (100003, 200, 3), (262147, 256, 4), (4099, 17, 5)])
def test_classify_word0_ties_and_flagged_cells(ctx, n, nb, seed):
    """K2 streams word 0 and loads words 1..4 only where word 0 cannot decide: ids whose word 0
    equals a bucket first's (findBucket's full-key tie) or myid's (commonBits past 32 bits), ids
    in cells of the word-0 cell table that hold a bucket boundary (random firsts: most cells),
    ids equal to a first, a ragged tail -- every bucket and the whole histogram equal the oracle."""
    rng = np.random.default_rng(seed)
    firsts = O.gen_ids(seed + 100, nb)
    firsts[0] = 0                                     # bucket 0 starts at the all-zero hash
    firsts = firsts[np.lexsort(firsts.T[::-1])]
    firsts = np.unique(firsts, axis=0)
    myid = O.gen_ids(seed + 200, 1)[0]
    ids = O.gen_ids(seed + 300, n)
    m = n // 8
    if m:
        pick = rng.integers(0, firsts.shape[0], size=m)
        ids[:m, :4] = firsts[pick, :4]                # word-0 ties with firsts
        ids[m:m + m // 2] = firsts[pick[: m // 2]]    # ids equal to a first
        ids[2 * m:3 * m, :4] = myid[:4]               # word 0 of myid: commonBits >= 32
        ids[3 * m:3 * m + 5] = myid                   # myid itself: 160
        ids[4 * m:5 * m, :3] = myid[:3]               # deep bins 8..31
    ctx.set_ids(ids)
    b, hist = ctx.classify(firsts, myid)
    wb, wh = O.classify(firsts, myid, ids)
    assert np.array_equal(hist, wh)
    bad = np.nonzero(b != wb)[0]
    assert bad.size == 0, f"{bad.size} buckets differ, first {bad[:5]}"


@pytest.mark.parametrize("shape", ["grown", "grown_deep", "one_bucket", "my_cell_0", "my_cell_last",
                                   "far_split", "far_split_mid_cell"])
def test_classify_register_path_shapes(ctx, shape):
    """K2's register path (bucket and bin from clz(word 0 ^ myid's word 0), no table read) is taken
    only when every cell but myid's maps to the bucket of its commonBits: routing tables grown by
    the reference's rule (onNewNode splits myid's bucket), a one-bucket table, myid in the first /
    last cell. A far bucket split (a boundary off myid's prefix, at a cell edge or inside a cell)
    must send the workgroups to the cell-table path. Every shape: buckets and histogram = oracle."""
    rng = np.random.default_rng(sum(map(ord, shape)))
    myid = O.gen_ids(11, 1)[0]
    if shape == "my_cell_0":
        myid[:4] = 0
    elif shape == "my_cell_last":
        myid[:4] = 0xFF
    if shape == "one_bucket":
        firsts = np.zeros((1, 20), np.uint8)
    else:
        grow = 200000 if shape == "grown_deep" else 20000
        firsts, _, _ = O.Table(myid).grow(O.gen_ids(12, grow)).export()
    if shape.startswith("far_split"):
        far = firsts[1].copy() if firsts.shape[0] > 1 else np.zeros(20, np.uint8)
        far[:] = 0
        far[0] = (~myid[0]) & 0x80 | 0x20               # off myid's first bit: a far bucket
        if shape == "far_split_mid_cell":
            far[1] = 0x11                                # inside its 10-bit cell
        firsts = np.concatenate([firsts, far[None, :]])
        firsts = np.unique(firsts[np.lexsort(firsts.T[::-1])], axis=0)
    ids = O.gen_ids(13, 65539)
    m = 4096
    ids[:m, :2] = myid[:2]                               # myid's cell and deep bins
    ids[m:2 * m, 0] = myid[0] ^ (1 << rng.integers(0, 8, m)).astype(np.uint8)   # every bin 0..7
    ids[2 * m:2 * m + 64] = myid
    pick = rng.integers(0, firsts.shape[0], 64)
    ids[3 * m:3 * m + 64] = firsts[pick]                 # ids equal to a first
    ctx.set_ids(ids)
    b, hist = ctx.classify(firsts, myid)
    wb, wh = O.classify(firsts, myid, ids)
    assert np.array_equal(hist, wh)
    bad = np.nonzero(b != wb)[0]
    assert bad.size == 0, f"{bad.size} buckets differ, first {bad[:5]}"


def test_classify_register_path_every_bin(ctx):
    """K2's register path takes commonBits c < 15 from clz(word 0 ^ myid's word 0) and sends
    c >= 15 to the exact path: ids with every commonBits 0..40 (myid with bit c flipped, random
    bits below), on a grown routing table, bucket and whole histogram = oracle."""
    rng = np.random.default_rng(4242)
    myid = O.gen_ids(21, 1)[0]
    firsts, _, _ = O.Table(myid).grow(O.gen_ids(22, 50000)).export()
    per = 257
    ids = O.gen_ids(23, 41 * per)
    bits = np.unpackbits(myid)
    for c in range(41):
        blk = np.unpackbits(ids[c * per:(c + 1) * per], axis=1)
        blk[:, :c] = bits[:c]
        blk[:, c] = 1 - bits[c]
        ids[c * per:(c + 1) * per] = np.packbits(blk, axis=1)
    ids = ids[rng.permutation(ids.shape[0])]
    ctx.set_ids(ids)
    b, hist = ctx.classify(firsts, myid)
    wb, wh = O.classify(firsts, myid, ids)
    assert np.array_equal(hist, wh)
    assert all(int(hist[c]) == per for c in range(41))
    assert np.array_equal(b, wb)


def test_cached_nodes_vs_oracle(ctx):
    ids = O.gen_ids(21, 50000)
    s = ids[np.lexsort(ids.T[::-1])]
    rng = np.random.default_rng(3)
    acc = (rng.random(s.shape[0]) < 0.7).astype(np.uint8)
    ctx.set_ids(s)
    tg = np.concatenate([O.gen_ids(22, 400), s[:10], s[-3:]])
    for count in (1, 8, 14):
        got, cnt = ctx.cached_nodes(tg, count, acc)
        for qi in range(tg.shape[0]):
            want = O.cached_nodes(s, acc, tg[qi], count)
            assert list(got[qi, : cnt[qi]]) == list(want)


def test_cached_nodes_unsorted_upload(ctx):
    """f2: an id set uploaded in arbitrary order is sorted on the device (LSD radix over the
    160-bit keys) and walked like NodeCache's std::map; indices refer to the caller's order.
    Duplicates are refused (a map has unique keys)."""
    import opendht_amd
    ids = O.gen_ids(24, 30000)
    ids[:3000, :8] = ids[0, :8]           # equal (w0, w1): the full 160-bit sort path
    rng = np.random.default_rng(4)
    perm = rng.permutation(ids.shape[0])
    shuffled = ids[perm]
    order = np.lexsort(shuffled.T[::-1])
    srt = shuffled[order]
    acc = (rng.random(ids.shape[0]) < 0.8).astype(np.uint8)   # caller order
    ctx.set_ids(shuffled)
    tg = np.concatenate([O.gen_ids(25, 300), shuffled[:20], ids[:10]])
    got, cnt = ctx.cached_nodes(tg, 14, acc)
    for qi in range(tg.shape[0]):
        want = O.cached_nodes(srt, acc[order], tg[qi], 14)
        assert list(got[qi, : cnt[qi]]) == list(order[want]), qi
    ctx.set_ids(np.concatenate([ids[:100], ids[50:51]]))
    with pytest.raises(opendht_amd.DhtGpuError) as ei:
        ctx.cached_nodes(O.gen_ids(1, 2), 8)
    assert ei.value.code == -5


def test_cache_mirror_1e6(ctx):
    """The NodeCache mirror at 10^6 entries uploaded unsorted: its device sort equals the host
    lexicographic order, getCachedNodes equals the oracle walk, the k-NN id set of the same
    context is untouched, and a repeated version skips the upload."""
    n = 1_000_000
    keys = O.gen_ids(31337, n)
    rng = np.random.default_rng(9)
    keys = keys[rng.permutation(n)]
    ctx.set_ids(O.gen_ids(4, 5000))
    before, _ = ctx.topk(O.gen_ids(5, 50), 8)
    ctx.cache_set(keys, version=3)
    order = np.lexsort(keys.T[::-1])
    assert np.array_equal(ctx.cache_sorted(), order.astype(np.uint32))
    acc = (rng.random(n) < 0.75).astype(np.uint8)
    tg = np.concatenate([O.gen_ids(31338, 500), keys[:12]])
    got, cnt = ctx.cache_nodes(tg, 14, acc)
    srt = keys[order]
    for qi in range(tg.shape[0]):
        want = O.cached_nodes(srt, acc[order], tg[qi], 14)
        assert list(got[qi, : cnt[qi]]) == list(order[want]), qi
    ctx.cache_set(keys[:10], version=3)   # same version, different n: uploaded
    assert ctx.cache_sorted().size == 10
    after, _ = ctx.topk(O.gen_ids(5, 50), 8)
    assert np.array_equal(before, after)


def test_sharded_records_merge(ctx):
    """K1 record mode + K3 merge over 3 shards == one flat top-k (the multi-GPU path
    on one device)."""
    import torch
    import opendht_amd
    ids = O.gen_ids(71, 30000)
    tg = O.gen_ids(72, 500)
    k = 8
    dev = torch.device("cuda", 0)
    tb = torch.from_numpy(tg.reshape(-1)).to(dev)
    ts = 512
    tp = torch.zeros(5 * ts, dtype=torch.int32, device=dev)
    L = opendht_amd.lib()
    assert L.dhtgpu_pack_dev(tb.data_ptr(), 500, tp.data_ptr(), ts, None) == 0
    bounds = [0, 7000, 19000, 30000]
    rec = torch.empty((3, 500, k, 3), dtype=torch.int32, device=dev)
    shards = []
    for s in range(3):
        c = opendht_amd.Context(0)
        c.set_ids(ids[bounds[s]:bounds[s + 1]])
        c.topk_dev(tp.data_ptr(), ts, 500, k, None, None, rec[s].data_ptr(), bounds[s], c.stream)
        torch.cuda.synchronize()
        shards.append(c)
    # the compact records are {w0, w1, global idx} of each shard's ascending top-k
    words = ids.view(">u4").reshape(-1, 5).astype(np.uint32)
    r0 = rec[1].cpu().numpy().view(np.uint32)
    li, _ = O.topk(ids[7000:19000], tg, k)
    assert np.array_equal(r0[..., 2], li + 7000) and np.array_equal(r0[..., :2], words[li + 7000, :2])
    out, cnt, nties = MU.merge(L, rec, tp, ts, k, ("ctx", MU.ctx_words_fn(L, shards, rec, bounds, k)))
    want, wcnt = O.topk(ids, tg, k)
    assert nties == 0
    assert np.array_equal(out, want) and np.array_equal(cnt, wcnt)
    for c in shards:
        c.close()


def test_cpp_adapter_on_gpu(tmp_path):
    """The C++11 drop-in adapter (include/dhtgpu.hpp) over reference-shaped types returns
    the same nodes, in the same order, as the oracle restatements."""
    import subprocess
    from test_abi import build_adapter_check
    exe = build_adapter_check(str(tmp_path / "adapter_check"))
    out = subprocess.run([exe, "--run"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 mismatches" in out.stdout


@pytest.mark.parametrize("pbits,pval", [(0, 0), (1, 1), (3, 5)])
def test_prefix_shard_matches_global_topk(ctx, pbits, pval):
    """Prefix routing: a shard holding the ids with top-pbits == pval answers
    every target carrying that prefix exactly like the full set, with global indices."""
    n = 120000
    ids = O.gen_ids(91, n)
    tg = O.gen_ids(92, 3000)
    top = lambda a: (a[:, 0].astype(np.uint32) >> (8 - pbits)) if pbits else np.zeros(a.shape[0], np.uint32)
    mine = tg[top(tg) == pval]
    assert mine.shape[0] > 0
    ctx.gen_ids_prefix(91, n, pbits, pval)
    shard = ids[top(ids) == pval]
    assert ctx.num_ids == shard.shape[0]
    assert np.array_equal(ctx.get_ids(), shard)
    want, wcnt = O.topk(ids, mine, 8)
    for fn in (ctx.topk, ctx.index_topk, ctx.batch_topk):
        got, cnt = fn(mine, 8)
        assert np.array_equal(cnt, wcnt) and np.array_equal(got, want)
    if pbits:
        # targets of other prefixes: the shard's own top-k (K6 answers them in the shifted
        # word-0 space like its own targets), alone and mixed into one batch with its own
        other = tg[top(tg) != pval][:200]
        gl = np.nonzero(top(ids) == pval)[0].astype(np.uint32)
        for tset in (other, tg):
            w2, c2 = O.topk(shard, tset, 8)
            w2 = np.where(w2 == 0xFFFFFFFF, w2, gl[np.minimum(w2, gl.size - 1)])
            for fn in (ctx.topk, ctx.batch_topk):
                got, cnt = fn(tset, 8)
                assert np.array_equal(cnt, c2) and np.array_equal(got, w2)


@pytest.mark.parametrize("pbits,pval", [(1, 0), (3, 6)])
def test_prefix_shard_weak_shape(ctx, pbits, pval):
    """The weak-scaling bench shape: rank pval of 2^pbits holds its prefix shard of a 2^24
    id stream (just under 2^(24 - pbits) ids: K6 marks at the finer level) and answers its
    own targets plus foreign ones; K6 == K1 scan on the whole batch, oracle on a sample."""
    n = 1 << 24
    ctx.gen_ids_prefix(4242, n, pbits, pval)
    m = ctx.num_ids
    tg = O.gen_ids(4243, 65536 >> pbits)
    tg[: tg.shape[0] - 64, 0] = (tg[: tg.shape[0] - 64, 0] & (0xFF >> pbits)) | (pval << (8 - pbits))
    got, cnt = ctx.batch_topk(tg, 8)
    sc, scnt = ctx.topk(tg, 8)
    assert np.array_equal(cnt, scnt) and np.array_equal(got, sc)
    assert np.all(cnt == 8)
    ids = O.gen_ids(4242, n)
    top = ids[:, 0].astype(np.uint32) >> (8 - pbits)
    gl = np.nonzero(top == pval)[0].astype(np.uint32)
    assert gl.size == m
    sample = np.r_[np.arange(0, tg.shape[0] - 64, 997), np.arange(tg.shape[0] - 64, tg.shape[0])]
    want, wcnt = O.topk(ids[gl], tg[sample], 8)
    assert np.array_equal(cnt[sample], wcnt) and np.array_equal(got[sample], gl[want])
    # shard-local result indices (what a rank owning its shard's node table keeps)
    ctx.set_global_indices(False)
    try:
        loc, lcnt = ctx.batch_topk(tg, 8)
        sl, slcnt = ctx.topk(tg, 8)
    finally:
        ctx.set_global_indices(True)
    assert np.array_equal(lcnt, cnt) and np.array_equal(slcnt, cnt)
    assert np.array_equal(gl[loc], got) and np.array_equal(sl, loc)


def test_topk_k32_many_splits(ctx):
    """K1 with a small batch over 2^20 ids at k = 32: the id-range splits are capped so that
    K3 can stage every split's 32 records in LDS (was: 256 splits, LDS overflow)."""
    ids = O.gen_ids(3232, 1 << 20)
    tg = O.gen_ids(3233, 16)
    ctx.set_ids(ids)
    want, wcnt = O.topk(ids, tg, 32)
    got, cnt = ctx.topk(tg, 32)
    assert np.array_equal(cnt, wcnt) and np.array_equal(got, want)


def test_select_prefix_dev(ctx):
    import torch
    n, stride = 50000, 50048
    dev = torch.device("cuda", 0)
    planes = torch.empty(5 * stride, dtype=torch.int32, device=dev)
    import opendht_amd
    assert opendht_amd.lib().dhtgpu_gen_dev(5, 0, n, planes.data_ptr(), stride, None) == 0
    out = torch.empty(5 * stride, dtype=torch.int32, device=dev)
    gidx = torch.empty(stride, dtype=torch.int32, device=dev)
    m = ctx.select_prefix_dev(planes.data_ptr(), stride, n, 2, 3, out.data_ptr(), stride, gidx.data_ptr())
    ids = O.gen_ids(5, n)
    sel = np.nonzero((ids[:, 0] >> 6) == 3)[0]
    assert m == sel.size
    assert np.array_equal(gidx[:m].cpu().numpy().view(np.uint32), sel.astype(np.uint32))
    words = out.view(5, stride)[:, :m].cpu().numpy().view(np.uint32).T
    assert np.array_equal(words, ids[sel].view(">u4").reshape(-1, 5).astype(np.uint32))


@pytest.mark.parametrize("n,q", [(20000, 200000), (300000, 64), (1 << 20, 70000)])
def test_batch_filter_regimes(ctx, n, q):
    """K6 across its regimes: nearly every id survives the filter (q >> 2^Lm), very few
    survive (q small), and the cfg-2 shape scaled down; checked on a target sample vs the
    oracle and on the whole batch vs the K1 scan."""
    ids = O.gen_ids(300 + q, n)
    tg = O.gen_ids(301 + q, q)
    ctx.set_ids(ids)
    got, cnt = ctx.batch_topk(tg, 8)
    sc, scnt = ctx.topk(tg, 8)
    assert np.array_equal(cnt, scnt) and np.array_equal(got, sc)
    sample = np.arange(0, q, max(1, q // 300))
    want, wcnt = O.topk(ids, tg[sample], 8)
    assert np.array_equal(got[sample], want) and np.array_equal(cnt[sample], wcnt)


def test_batch_clustered_targets_and_fallback(ctx):
    """All targets inside one prefix partition; sparse subtrees that force the exact
    brute-force fallback (subtree smaller than k); repeated calls (the prefix bitmap
    must be all-zero again after every call)."""
    ids = O.gen_ids(401, 50000)
    tg = O.gen_ids(402, 3000)
    tg[:, :2] = 0xA7                     # 16 shared leading bits: one partition
    ctx.set_ids(ids)
    for k in (8, 32):
        got, cnt = ctx.batch_topk(tg, k)
        want, wcnt = O.topk(ids, tg, k)
        assert np.array_equal(cnt, wcnt) and np.array_equal(got, want)
    # ids confined to a narrow prefix: most targets' level-Lm subtrees are empty
    ids2 = O.gen_ids(403, 40000)
    ids2[:, 0] = 0x3C
    tg2 = np.concatenate([O.gen_ids(404, 200), ids2[:50]])
    check_topk(ctx, ids2, tg2, 8)
    check_topk(ctx, ids, tg[:100], 14)    # a different batch on the first set again


@pytest.mark.parametrize("lists,k,seed,cap", [(1, 8, 1, 256), (2, 8, 2, 256), (3, 14, 3, 256), (8, 8, 4, 256),
                                              (8, 32, 5, 256), (13, 1, 6, 256), (64, 8, 7, 256), (5, 32, 9, 256),
                                              (4, 8, 10, 4), (64, 3, 11, 16)])
def test_merge_heads_ties_duplicates(ctx, lists, k, seed, cap):
    """K3 over compact records of id-range shards whose ids tie on their first 64 bits across
    shards (the records cannot order them: the rows are listed and settled by the second
    exchange of words 2..4 -- cap 4 / 16: more tie rows than one exchange takes, so the every-row
    settlement runs too), duplicated ids in different shards (global index decides), shards
    shorter than k and empty shards == one flat top-k of all ids."""
    import torch
    import opendht_amd
    rng = np.random.default_rng(seed)
    n, q = 4000, 300
    ids = O.gen_ids(600 + seed, n)
    ids[: n // 3, :8] = ids[0, :8]                 # 64-bit prefix cluster, spread over the shards
    ids[n // 2: n // 2 + 40] = ids[10:50]          # duplicates of cluster ids (other shards)
    ids = ids[rng.permutation(n)]
    tg = O.gen_ids(700 + seed, q)
    tg[: q // 2, :8] = O.gen_ids(600 + seed, 1)[0, :8]   # targets inside the cluster's prefix
    cuts = np.sort(rng.integers(0, n, size=lists - 1))
    if lists > 2:
        cuts[0] = cuts[1]                          # one empty shard
    bounds = [0] + [int(c) for c in cuts] + [n]
    rec = MU.host_records(ids, bounds, tg, k, O)
    dev = torch.device("cuda", 0)
    ts = (q + 63) // 64 * 64
    tp = torch.zeros(5 * ts, dtype=torch.int32, device=dev)
    L = opendht_amd.lib()
    assert L.dhtgpu_pack_dev(torch.from_numpy(tg.reshape(-1)).to(dev).data_ptr(), q, tp.data_ptr(), ts, None) == 0
    rd = torch.from_numpy(rec.view(np.int32)).to(dev)
    got, gcnt, nties = MU.merge(L, rd, tp, ts, k, ("host", MU.host_words_fn(ids, rec)), tie_cap=cap)
    want, wcnt = O.topk(ids, tg, k)
    assert np.array_equal(gcnt, wcnt)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} targets differ, first {bad[:3]}: {got[bad[0]]} vs {want[bad[0]]}"
    if lists > 1:
        assert nties > 0, "the 64-bit cluster must produce tie rows"
        if cap < 64:
            assert nties > cap
    if lists == 64:   # more lists than one merge takes
        assert L.dhtgpu_merge_dev(rd.data_ptr(), 65, 1, k, tp.data_ptr(), ts, k, rd.data_ptr(), rd.data_ptr(),
                                  rd.data_ptr(), cap, None) == opendht_amd.ERANGE


def test_merge_colliding_indices(ctx):
    """lists built with colliding index bases (every shard's records numbered from 0):
    different ids that share an index are both kept, ordered by distance; the same id sent by two
    lists under the same index is one candidate.  Checked against a host merge of (distance,
    index) with exact duplicates removed."""
    import torch
    import opendht_amd
    n, q, k = 3000, 200, 8
    ids = O.gen_ids(808, n)
    ids[1000:1040] = ids[0:40]                     # list 1's first 40 ids == list 0's (same local index)
    ids[:20, :8] = ids[2000, :8]                   # and 64-bit prefix ties across lists
    tg = O.gen_ids(809, q)
    tg[:50, :8] = ids[2000, :8]
    bounds = [0, 1000, 2000, 3000]
    rec = MU.host_records(ids, bounds, tg, k, O)
    for s in range(3):                             # local indices: every list counts from 0
        m = rec[s, ..., 2] != MU.NONE
        rec[s, ..., 2][m] -= bounds[s]
    dev = torch.device("cuda", 0)
    ts = (q + 63) // 64 * 64
    tp = torch.zeros(5 * ts, dtype=torch.int32, device=dev)
    L = opendht_amd.lib()
    assert L.dhtgpu_pack_dev(torch.from_numpy(tg.reshape(-1)).to(dev).data_ptr(), q, tp.data_ptr(), ts, None) == 0
    words = ids.view(">u4").reshape(-1, 5).astype(np.uint32)

    def wfn(j, rows, out):
        g = rec[j][rows][..., 2]
        w = np.full(g.shape + (3,), MU.NONE, np.uint32)
        ok = g != MU.NONE
        w[ok] = words[g[ok].astype(np.int64) + bounds[j], 2:5]
        return w
    got, gcnt, nties = MU.merge(L, torch.from_numpy(rec.view(np.int32)).to(dev), tp, ts, k, ("host", wfn))
    assert nties > 0
    tw = tg.view(">u4").reshape(-1, 5).astype(np.uint32)
    for i in range(q):
        cand = set()
        for s in range(3):
            for r in range(k):
                g = int(rec[s, i, r, 2])
                if g != MU.NONE:
                    cand.add(tuple(int(x) for x in (words[g + bounds[s]] ^ tw[i])) + (g,))
        order = sorted(cand)[:k]
        assert int(gcnt[i]) == len(order)
        assert list(got[i, :len(order)]) == [c[-1] for c in order], i


def test_batch_records_merge(ctx):
    """K6 record mode over 3 id shards + K3 merge == one flat top-k."""
    import torch
    import opendht_amd
    ids = O.gen_ids(501, 90000)
    q, k = 700, 8
    tg = O.gen_ids(502, q)
    dev = torch.device("cuda", 0)
    ts = 704
    tp = torch.zeros(5 * ts, dtype=torch.int32, device=dev)
    L = opendht_amd.lib()
    assert L.dhtgpu_pack_dev(torch.from_numpy(tg.reshape(-1)).to(dev).data_ptr(), q, tp.data_ptr(), ts, None) == 0
    bounds = [0, 20000, 61000, 90000]
    rec = torch.empty((3, q, k, 3), dtype=torch.int32, device=dev)
    shards = []
    for s in range(3):
        c = opendht_amd.Context(0)
        c.set_ids(ids[bounds[s]:bounds[s + 1]])
        c.batch_topk_dev(tp.data_ptr(), ts, q, k, None, None, rec[s].data_ptr(), bounds[s], c.stream)
        torch.cuda.synchronize()
        shards.append(c)
    out, cnt, nties = MU.merge(L, rec, tp, ts, k, ("ctx", MU.ctx_words_fn(L, shards, rec, bounds, k)))
    want, wcnt = O.topk(ids, tg, k)
    assert nties == 0 and np.array_equal(out, want) and np.array_equal(cnt, wcnt)
    for c in shards:
        c.close()


def _want_records(ids, gidx, tg, k):
    """(q, k, 3) compact records {w0, w1, global idx} of the exact top-k over `ids` (global index
    of local i = gidx[i]), NONE-padded."""
    q = tg.shape[0]
    words = ids.view(">u4").reshape(-1, 5).astype(np.uint32)
    idx, cnt = O.topk(ids, tg, k, threads=16)
    rec = np.full((q, k, 3), MU.NONE, dtype=np.uint32)
    for i in range(q):
        c = int(cnt[i])
        li = idx[i, :c].astype(np.int64)
        rec[i, :c, :2] = words[li, :2]
        rec[i, :c, 2] = gidx[li]
    return rec


def _ctx_records(c, tg, k, base):
    import torch
    import opendht_amd
    dev = torch.device("cuda", 0)
    q = tg.shape[0]
    ts = (q + 63) // 64 * 64
    tp = torch.zeros(5 * ts, dtype=torch.int32, device=dev)
    L = opendht_amd.lib()
    assert L.dhtgpu_pack_dev(torch.from_numpy(tg.reshape(-1)).to(dev).data_ptr(), q, tp.data_ptr(), ts, None) == 0
    rec = torch.full((q, k, 3), -7, dtype=torch.int32, device=dev)
    c.batch_topk_dev(tp.data_ptr(), ts, q, k, None, None, rec.data_ptr(), base, c.stream)
    torch.cuda.synchronize()
    return rec.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("case", ["uniform", "w0_ties", "fallback_split", "fallback_list", "prefix_shard"])
@pytest.mark.parametrize("k", [8, 14, 32])
def test_batch_records_every_writer(case, k):
    """K6 in record form stores every row's records from its own writer (round 5: no conversion
    pass): F3's fast path (uniform), F3's and F4's wave paths (ids pairing on word 0: deferred ties
    and wave-path targets), F4's fallback scan through its split merge (a short list) and as one
    split per group (a long list), and a prefix shard (shifted word-0 stage: word 0 read back).
    Every row == the records of the exact top-k, with the index base."""
    import opendht_amd
    base = 1000
    with opendht_amd.Context(0) as c:
        if case == "prefix_shard":
            n = 300000
            allids = O.gen_ids(611, n)
            c.gen_ids_prefix(611, n, 2, 1)
            sel = np.nonzero((allids[:, 0] >> 6) == 1)[0]
            ids, gidx = allids[sel], sel.astype(np.int64)
            tg = O.gen_ids(612, 1500)
            base = 0
        else:
            n = {"uniform": 200000, "w0_ties": 120000, "fallback_split": 40000, "fallback_list": 30000}[case]
            ids = O.gen_ids(600 + len(case), n)
            q = {"fallback_list": 40000}.get(case, 2000)
            tg = O.gen_ids(650 + len(case), q)
            if case == "w0_ties":
                ids[1::4, :4] = ids[0::4, :4]          # pairs sharing word 0
                tg[::3] = ids[5::7][: tg[::3].shape[0]]   # targets among them
            elif case.startswith("fallback"):
                ids[:, 0] = 0x3C                       # ids in one narrow prefix: most subtrees empty
                tg[:50] = ids[:50]
            c.set_ids(ids)
            gidx = np.arange(n, dtype=np.int64) + base
        got = _ctx_records(c, tg, k, base)
    want = _want_records(ids, gidx, tg, k)
    bad = np.nonzero((got != want).any(axis=(1, 2)))[0]
    assert bad.size == 0, f"{case} k={k}: {bad.size} rows differ, first {bad[:5]}: {got[bad[0]]} vs {want[bad[0]]}"


def test_batch_records_tie_words_from_contexts(ctx):
    """The second exchange's payload from live shard contexts (dhtgpu_tie_words_dev: global index ->
    the context's own planes; a prefix shard maps it back through its index map): K6 record mode
    over 3 id-range shards and 2 prefix shards whose ids share their first 64 bits across shards,
    K3 + tie exchange == one flat top-k (every row settled: cap 2)."""
    import torch
    import opendht_amd
    n, q, k = 60000, 600, 8
    ids = O.gen_ids(511, n)
    ids[::3, :8] = ids[1, :8]                      # a third of the ids share 64 bits
    tg = O.gen_ids(512, q)
    tg[::2, :8] = ids[1, :8]
    dev = torch.device("cuda", 0)
    ts = (q + 63) // 64 * 64
    tp = torch.zeros(5 * ts, dtype=torch.int32, device=dev)
    L = opendht_amd.lib()
    assert L.dhtgpu_pack_dev(torch.from_numpy(tg.reshape(-1)).to(dev).data_ptr(), q, tp.data_ptr(), ts, None) == 0
    bounds = [0, 11000, 40000, n]
    rec = torch.empty((3, q, k, 3), dtype=torch.int32, device=dev)
    shards = []
    for s in range(3):
        c = opendht_amd.Context(0)
        c.set_ids(ids[bounds[s]:bounds[s + 1]])
        c.batch_topk_dev(tp.data_ptr(), ts, q, k, None, None, rec[s].data_ptr(), bounds[s], c.stream)
        shards.append(c)
    torch.cuda.synchronize()
    want, wcnt = O.topk(ids, tg, k)
    for cap in (256, 2):
        out, cnt, nties = MU.merge(L, rec, tp, ts, k, ("ctx", MU.ctx_words_fn(L, shards, rec, bounds, k)),
                                   tie_cap=cap)
        assert nties > 2 and np.array_equal(out, want) and np.array_equal(cnt, wcnt), cap
    for c in shards:
        c.close()
    # prefix shards (global indices through the shard's index map) of the generated stream
    n2 = 200000
    ids2 = O.gen_ids(513, n2)
    tg2 = O.gen_ids(514, q)
    rec2 = torch.empty((2, q, k, 3), dtype=torch.int32, device=dev)
    tp2 = torch.zeros(5 * ts, dtype=torch.int32, device=dev)
    assert L.dhtgpu_pack_dev(torch.from_numpy(tg2.reshape(-1)).to(dev).data_ptr(), q, tp2.data_ptr(), ts, None) == 0
    shards = []
    for s in range(2):
        c = opendht_amd.Context(0)
        c.gen_ids_prefix(513, n2, 1, s)
        c.batch_topk_dev(tp2.data_ptr(), ts, q, k, None, None, rec2[s].data_ptr(), 0, c.stream)
        shards.append(c)
    torch.cuda.synchronize()
    out, cnt, _ = MU.merge(L, rec2, tp2, ts, k, ("ctx", MU.ctx_words_fn(L, shards, rec2, [0, 0], k)),
                           force_all=True)
    want, wcnt = O.topk(ids2, tg2, k)
    assert np.array_equal(out, want) and np.array_equal(cnt, wcnt)
    for c in shards:
        c.close()


@pytest.mark.parametrize("af", [4, 6])
def test_buffer_nodes_vs_oracle(ctx, af):
    """bufferNodes on the device: per target, its k-NN result (and shuffled / padded / short
    candidate lists) packed into 26 / 38-byte records, byte-identical to the oracle."""
    rng = np.random.default_rng(20 + af)
    alen = 4 if af == 4 else 16
    ids = O.gen_ids(950 + af, 5000)
    ids[:50, :4] = ids[0, :4]
    tail = O.special_addrs(rng, 5000, af)
    ctx.set_ids(ids)
    tg = O.gen_ids(960 + af, 400)
    tg[:30, :4] = ids[0, :4]
    knn, _ = ctx.topk(tg, 14)
    cand = knn.copy()
    for i in range(0, 400, 3):
        rng.shuffle(cand[i])
    cand[::5, 9:] = 0xFFFFFFFF
    cand[7, :] = 0xFFFFFFFF
    out, ln = ctx.buffer_nodes(tail, af, tg, cand)
    for i in range(400):
        want = O.buffer_nodes(ids, tail, alen, tg[i], cand[i])
        assert ln[i] == want.size, i
        assert np.array_equal(out[i, : ln[i]], want), i


def test_buffer_nodes_ids_and_bounds(ctx):
    """bufferNodes over the caller's own nodes leaves the context's id set alone; a candidate
    index past the node set is refused (EINVAL) instead of read out of bounds."""
    import opendht_amd
    rng = np.random.default_rng(77)
    nodes = O.gen_ids(980, 700)
    tail = O.special_addrs(rng, 700, 4)
    tg = O.gen_ids(981, 50)
    cand = rng.integers(0, 700, size=(50, 12)).astype(np.uint32)
    cand[::7, 10:] = 0xFFFFFFFF
    kset = O.gen_ids(982, 3000)
    ctx.set_ids(kset)
    out, ln = ctx.buffer_nodes_ids(nodes, tail, 4, tg, cand)
    for i in range(50):
        want = O.buffer_nodes(nodes, tail, 4, tg[i], cand[i])
        assert ln[i] == want.size and np.array_equal(out[i, : ln[i]], want), i
    assert np.array_equal(ctx.get_ids(), kset)
    bad = cand.copy()
    bad[3, 2] = 700
    with pytest.raises(opendht_amd.DhtGpuError) as ei:
        ctx.buffer_nodes_ids(nodes, tail, 4, tg, bad)
    assert ei.value.code == -1
    with pytest.raises(opendht_amd.DhtGpuError):
        ctx.buffer_nodes(O.special_addrs(rng, 3000, 4), 4, tg, np.full((50, 4), 3000, np.uint32))


@pytest.mark.parametrize("af", [4, 6])
def test_deserialize_nodes_vs_oracle(ctx, af):
    rng = np.random.default_rng(30 + af)
    alen = 4 if af == 4 else 16
    rec = 22 + alen
    myid = O.gen_ids(970, 1)[0]
    ids = O.gen_ids(971, 3000)
    ids[::41] = myid
    tail = O.special_addrs(rng, 3000, af)
    recs = np.concatenate([ids, tail], axis=1)
    blobs, from_af, from_addr, expect = [], [], [], []
    pos = 0
    for m in range(300):
        k = int(rng.integers(0, 9))
        b = recs[pos:pos + k].reshape(-1)
        pos += k
        if m % 17 == 0:
            b = np.concatenate([b, np.zeros(3, np.uint8)])     # not a whole number of records
        blobs.append(b.tobytes())
        from_af.append([0, 4, 6][m % 3])
        from_addr.append(rng.integers(0, 256, size=16, dtype=np.uint8))
    gids, gtail, gst, gms = ctx.deserialize_nodes(af, myid, blobs, np.array(from_af, np.uint8),
                                                  np.stack(from_addr))
    r = 0
    for m, b in enumerate(blobs):
        bad = len(b) % rec != 0
        assert gms[m] == (1 if bad else 0), m
        if bad:
            continue
        for j in range(len(b) // rec):
            one = np.frombuffer(b[j * rec:(j + 1) * rec], dtype=np.uint8)
            st, out = O.deserialize_node(one, af, myid, from_af[m], from_addr[m])
            assert gst[r] == st, (m, j)
            assert np.array_equal(gids[r], one[:20])
            if st != 1:                       # own id: the reference skips the record
                assert np.array_equal(gtail[r], out), (m, j)
            r += 1
    assert r == gids.shape[0]



@pytest.mark.parametrize("n,dead_frac,seed,alpha", [(3000, 0.0, 1, 4), (100000, 0.2, 2, 4), (40000, 0.5, 3, 4),
                                                    (100000, 0.2, 4, 3), (40000, 0.3, 5, 1), (20000, 0.1, 6, 8)])
def test_search_batch_vs_oracle(ctx, n, dead_frac, seed, alpha):
    """Crawl-replay search kernel == the oracle's model, list for list (indices, flags,
    lengths, rounds, requests); alpha = requests per round: the reference's 4
    (MAX_REQUESTED_SEARCH_NODES, include/opendht/dht.h:321), BASELINE cfg 5's 3, and 1 / 8."""
    ids = O.gen_ids(1000 + seed, n)
    dead = (np.random.default_rng(seed).random(n) < dead_frac).astype(np.uint8) if dead_frac else None
    tg = O.gen_ids(2000 + seed, 700)
    tg[:40] = ids[:40]                     # targets that are network nodes
    sr = ((np.arange(700, dtype=np.uint64) * 7919) % n).astype(np.uint32)
    ctx.set_ids(ids)
    ctx.net_prepare(dead, table_seed=seed)
    got = ctx.search_batch(tg, sr, alpha=alpha)
    ctx.set_search_alpha(4)
    want = O.search_batch(ids, dead, seed, tg, sr, alpha=alpha)
    names = ["idx", "flags", "len", "rounds", "queries"]
    for g, w, nm in zip(got, want, names):
        bad = np.nonzero((g != w).reshape(g.shape[0], -1).any(axis=1))[0]
        assert bad.size == 0, f"{nm}: {bad.size} searches differ, first {bad[:5]}"


def test_crawl_gpu_vs_oracle(ctx):
    """The dhtscanner crawl over the GPU search kernel visits the same steps and finds the
    same nodes as over the oracle model."""
    from opendht_amd import crawl
    ids = O.gen_ids(555, 200000)
    dead = (np.random.default_rng(5).random(200000) < 0.15).astype(np.uint8)
    ctx.set_ids(ids)
    ctx.net_prepare(dead, table_seed=31)
    g = crawl.crawl(lambda t, s, r: ctx.search_batch(t, s, r), lambda ix: ids[ix], 4321)
    o = crawl.crawl(lambda t, s, r: O.search_batch(ids, dead, 31, t, s, r), lambda ix: ids[ix], 4321)
    assert g["steps"] == o["steps"] and g["queries"] == o["queries"] and g["rounds"] == o["rounds"]
    assert np.array_equal(g["found"], o["found"])


def _search_case(seed, nn, q, cap, maxins, pre_len=0):
    rng = np.random.default_rng(seed)
    ids = O.gen_ids(seed, nn)
    ids[: nn // 8, :4] = ids[0, :4]                     # a cluster: long common prefixes
    state = rng.choice([0, 0, 0, 0, 1, 2, 3], size=nn).astype(np.uint8)
    tg = O.gen_ids(seed + 1, q)
    tg[: q // 4, :4] = ids[0, :4]
    lists = np.full((q, cap), 0xFFFFFFFF, np.uint32)
    flags = np.zeros((q, cap), np.uint8)
    lens = np.zeros(q, np.uint32)
    expired = (rng.random(q) < 0.2).astype(np.uint8)
    if pre_len:   # searches that already hold lists (built by the oracle itself)
        off0 = (np.arange(q + 1, dtype=np.uint64) * pre_len)
        n0 = rng.integers(0, nn, size=q * pre_len).astype(np.uint32)
        t0 = (rng.random(n0.size) < 0.5).astype(np.uint8)
        lists, flags, lens, expired, _ = O.search_insert(ids, state, tg, lists, flags, lens, expired, off0, n0, t0)
    counts = rng.integers(0, maxins, size=q)
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    node = rng.integers(0, nn, size=int(off[-1])).astype(np.uint32)
    node[::7] = node[::7] % 64                          # repeats of the same nodes
    tok = (rng.random(node.size) < 0.3).astype(np.uint8)
    return ids, state, tg, lists, flags, lens, expired, off, node, tok


@pytest.mark.parametrize("seed,nn,q,maxins,pre", [(31, 500, 3000, 40, 0), (32, 20000, 10000, 60, 20),
                                                  (33, 64, 700, 200, 5)])
def test_search_insert_matches_oracle(ctx, seed, nn, q, maxins, pre):
    """a10: batched Search::insertNode (search.h:636-722 + removeExpiredNode :541-551) over
    random insertion sequences -- expired and removable nodes, candidates, token replies,
    expired searches, repeated nodes, clustered ids -- equals the oracle list for list."""
    case = _search_case(seed, nn, q, 64, maxins, pre)
    got = ctx.search_insert(*case)
    want = O.search_insert(*case)
    for g, w, nm in zip(got, want, ["lists", "flags", "lens", "expired", "added"]):
        bad = np.nonzero((g != w).reshape(g.shape[0], -1).any(axis=1))[0] if g.ndim > 1 else np.nonzero(g != w)[0]
        assert bad.size == 0, f"{nm}: {bad.size} rows differ, first {bad[:5]}"


def test_search_insert_overflow_and_bounds(ctx):
    """A row too small for the list is reported (ERANGE), and node indices outside the node
    table are refused before any launch (EINVAL)."""
    import opendht_amd
    ids, state, tg, lists, flags, lens, expired, off, node, tok = _search_case(40, 300, 50, 4, 40)
    state[:] = 1                                        # every node bad: lists grow past 14
    with pytest.raises(opendht_amd.DhtGpuError) as e:
        ctx.search_insert(ids, state, tg, lists, flags, lens, expired, off, node, tok)
    assert e.value.code == opendht_amd.ERANGE
    node2 = node.copy()
    node2[0] = 300
    with pytest.raises(opendht_amd.DhtGpuError) as e:
        ctx.search_insert(ids, np.zeros(300, np.uint8), tg, np.full((50, 64), 0xFFFFFFFF, np.uint32),
                          np.zeros((50, 64), np.uint8), lens * 0, expired, off, node2, tok)
    assert e.value.code == opendht_amd.EINVAL


def test_table_stats_lowbit_depth(ctx):
    """a4/a6: InfoHash::lowbit of every bucket's first id and RoutingTable::depth of every
    bucket computed on the device equal the oracle on grown tables (and on a one-bucket table)."""
    for seed, n in [(71, 50_000), (72, 3), (73, 400_000)]:
        myid = O.gen_ids(seed, 1)[0]
        firsts, _, _ = O.Table(myid).grow(O.gen_ids(seed + 1, n)).export()
        lb, dp = ctx.table_stats(firsts)
        assert list(lb) == [O.lowbit(f) for f in firsts]
        assert list(dp) == [O.depth(firsts, b) for b in range(firsts.shape[0])]


@pytest.mark.parametrize("n", [1, 7, 9, 100, 5000, 70001])
@pytest.mark.parametrize("k", [1, 8, 14, 32])
@pytest.mark.parametrize("q", [1, 5, 8, 13, 64])
def test_small_batch_path(ctx, n, k, q):
    """Batches of <= 64 targets take the small-batch path (one pass over word 0 + one
    workgroup per target prefix, the K1 scan for short subtrees): bit-exact like K6.  q = 1 runs
    S1's register prefix check, q > 1 its LDS bitmap."""
    ids = O.gen_ids(3000 + n, n)
    tg = O.gen_ids(3100 + q, q)
    ctx.set_ids(ids)
    want, wcnt = O.topk(ids, tg, k)
    got, cnt = ctx.batch_topk(tg, k)
    assert np.array_equal(cnt, wcnt)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} targets differ, first {bad[:5]}"


@pytest.mark.parametrize("rows", [slice(0, 64), slice(0, 8), slice(14, 15), slice(8, 16), slice(40, 41)])
def test_small_batch_clusters_duplicates_fallback(ctx, rows):
    """Small batches over clustered ids (w0 ties, buckets past their capacity, subtrees short
    of k ids: the K1 fallback), targets sharing a prefix (one bucket, several targets) and
    duplicated ids; the whole batch and sub-batches of 8 and 1 (q = 1: S1's register prefix check)."""
    ids = O.gen_ids(51, 40000)
    ids[:20000, :4] = ids[0, :4]          # 20,000 ids in one 32-bit prefix: bucket overflow
    ids[:5000, 4:8] = ids[0, 4:8]
    ids[20000:20003, :3] = 0              # 3 ids under a 24-bit prefix: short of k
    ids = np.concatenate([ids, ids[30000:30050]])   # duplicates
    tg = O.gen_ids(52, 64)
    tg[:10, :4] = ids[0, :4]
    tg[10:14, :8] = ids[0, :8]
    tg[14:20, :3] = 0
    tg[20:30] = tg[30:40]                 # repeated targets
    tg[40:45] = ids[30000:30005]          # targets that are (duplicated) members
    tg = np.ascontiguousarray(tg[rows])
    ctx.set_ids(ids)
    for k in (8, 32):
        want, wcnt = O.topk(ids, tg, k)
        got, cnt = ctx.batch_topk(tg, k)
        assert np.array_equal(cnt, wcnt) and np.array_equal(got, want), k


@pytest.mark.parametrize("q", [40, 1])
@pytest.mark.parametrize("pbits,pval", [(1, 1), (3, 5)])
def test_small_batch_prefix_shard(ctx, pbits, pval, q):
    """Small batches on a prefix shard (the shifted word-0 plane), own and foreign targets,
    global and shard-local indices; q = 1 takes S1's register prefix check."""
    n = 120000
    ids = O.gen_ids(91, n)
    top = lambda a: a[:, 0].astype(np.uint32) >> (8 - pbits)
    ctx.gen_ids_prefix(91, n, pbits, pval)
    gl = np.nonzero(top(ids) == pval)[0].astype(np.uint32)
    tg = O.gen_ids(95, 40)
    tg[:30, 0] = (tg[:30, 0] & (0xFF >> pbits)) | (pval << (8 - pbits))
    tg = np.ascontiguousarray(tg[:q] if q > 1 else tg[3:4])
    w, wc = O.topk(ids[gl], tg, 8)
    got, cnt = ctx.batch_topk(tg, 8)
    assert np.array_equal(cnt, wc) and np.array_equal(got, gl[w])
    ctx.set_global_indices(False)
    try:
        loc, lcnt = ctx.batch_topk(tg, 8)
    finally:
        ctx.set_global_indices(True)
    assert np.array_equal(lcnt, wc) and np.array_equal(loc, w)


@pytest.mark.parametrize("k", [1, 2, 3])
def test_fallback_scan_small_k(ctx, k):
    """k < 4 with targets whose level-Lm subtree is empty (about 80 of 2,790 here at k = 1): F4's
    fallback scan may use up to 256 / k id-range splits, but its merge walks one split list per
    lane, so the splits are capped at 64 (lists past lane 63 were dropped: found by the
    randomised sweep, tests/test_gpu_fuzz.py seed 24)."""
    ids = O.gen_ids(2401, 1871338)
    tg = O.gen_ids(2402, 2790)
    ctx.set_ids(ids)
    want, wcnt = O.topk(ids, tg, k, threads=16)
    got, cnt = ctx.batch_topk(tg, k)
    assert np.array_equal(cnt, wcnt)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} targets differ, first {bad[:5]}"


def test_small_batch_alternating_fallback_fresh_context():
    """KS on a fresh context, calls alternating between batches whose buckets are all complete
    and batches with short or overflowing buckets (the scan roles inside S2 answer those):
    S2 reads one of two counter sets per call while it zeroes the other for the next call, so
    every call in the sequence must match std::partial_sort(xorCmp), for k = 1, 8, 32."""
    import opendht_amd
    ids = O.gen_ids(4401, 60000)
    ids[:9000, :4] = ids[0, :4]               # one 32-bit cluster: its bucket overflows
    ids[9000:9002, :3] = 0                    # a 24-bit prefix holding 2 ids: short of k
    uni = O.gen_ids(4402, 64)
    bad_tg = O.gen_ids(4403, 50)
    bad_tg[:5, :4] = ids[0, :4]
    bad_tg[5:9, :3] = 0
    with opendht_amd.Context(0) as c:
        c.set_ids(ids)
        for i, k in enumerate((8, 8, 1, 1, 32, 32, 8, 8)):
            tg = bad_tg if i % 2 else uni[: 1 + 9 * i]
            want, wcnt = O.topk(ids, tg, k)
            got, cnt = c.batch_topk(tg, k)
            assert np.array_equal(cnt, wcnt), (i, k)
            assert np.array_equal(got, want), (i, k)


def test_f4_half_grid_then_fallback_list():
    """K6's fallback scan runs at half its grid while the context's last completed call listed
    no fallback target: on a fresh context, a uniform batch (empty list, synchronised
    so the hint is 0), then batches whose targets' level-Lm subtrees are short of k ids -- the
    first of them starts from the half-size grid -- each == the oracle, k in {1, 8, 32}."""
    import opendht_amd
    n = 1 << 21
    ids = O.gen_ids(4501, n)
    tg_uni = O.gen_ids(4502, 4096)
    tg = O.gen_ids(4503, 4096)
    # empty the level-15 subtrees of 40 targets down to 2 ids each (the mark level is >= 15 here:
    # their top-k lies outside, so F3 lists them for the fallback scan)
    key = lambda a: ((a[:, 0].astype(np.uint32) << 16) | (a[:, 1].astype(np.uint32) << 8) | a[:, 2]) >> 9
    ik, tk = key(ids), key(tg)
    for t in range(0, 400, 10):
        inside = np.nonzero(ik == tk[t])[0][2:]
        ids[inside, 0] ^= 0x80
        ik = key(ids)
    with opendht_amd.Context(0) as c:
        c.set_ids(ids)
        for k in (1, 8, 32):
            got, cnt = c.batch_topk(tg_uni, k)          # synchronous: the hint is now 0
            want, wcnt = O.topk(ids, tg_uni[:64], k)
            assert np.array_equal(got[:64], want) and np.array_equal(cnt[:64], wcnt)
            got, cnt = c.batch_topk(tg, k)
            want, wcnt = O.topk(ids, tg, k)
            assert np.array_equal(cnt, wcnt), k
            bad = np.nonzero((got != want).any(axis=1))[0]
            assert bad.size == 0, f"k={k}: {bad.size} targets differ, first {bad[:5]}"


def test_dbg_bits_leave_results_unchanged(monkeypatch):
    """DHTGPU_DBG with every bit set (the variable is read at context creation and masked to the
    diagnostics bits; tests/test_abi.py pins the mask): K6, KS (here: K6 on small batches, bit 2^23)
    and the sub-partitioned route return exactly the oracle's nodes."""
    import opendht_amd
    monkeypatch.setenv("DHTGPU_DBG", str(0xFFFFFFFF & ~256))   # 256 (stamps) prints to stderr: left out
    ids = O.gen_ids(4242, 1 << 20)
    with opendht_amd.Context(0) as c:
        c.set_ids(ids)
        for q in (5, 64, 3000):
            tg = O.gen_ids(4243 + q, q)
            want, wcnt = O.topk(ids, tg, 8)
            got, cnt = c.batch_topk(tg, 8)
            assert np.array_equal(cnt, wcnt) and np.array_equal(got, want), q
