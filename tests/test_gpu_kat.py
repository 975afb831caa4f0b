"""The reference's own known answers (tests/infohashtester.cpp:76-138, transcribed as data in
tests/golden/infohash_kat.json) run through the HIP kernels themselves, not only through the
CPU oracle: the device comparator (every top-k path), commonBits (K2 classify's histogram),
lowbit (table_stats) and the lexicographic order (the NodeCache mirror's device radix sort).
Marked gpu: run on the MI355X box."""
import json
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "infohash_kat.json")


@pytest.fixture(scope="module")
def kat():
    with open(GOLD) as f:
        k = json.load(f)
    names = list(k["hashes"])
    k["names"] = names
    k["ids"] = np.stack([O.h(k["hashes"][nm]) for nm in names])
    k["pos"] = {nm: i for i, nm in enumerate(names)}
    return k


@pytest.fixture(scope="module")
def ctx():
    import opendht_amd
    c = opendht_amd.Context(0)
    yield c
    c.close()


def _order_rows(kat, got, targets):
    """the id names of each result row (-1 padding dropped)"""
    out = []
    for r in range(targets.shape[0]):
        out.append([kat["names"][i] for i in got[r] if i != 0xFFFFFFFF])
    return out


@pytest.mark.parametrize("path", ["scan", "index", "batch_small", "batch_k6"])
def test_kat_xor_cmp_through_topk(ctx, kat, path):
    """xor_cmp KATs (infohashtester.cpp:124-138), incl. the 'circular' max.xorCmp(null, min) = -1:
    with the five KAT hashes as the id set, every KAT hash as a target, the ascending XOR order each
    kernel returns puts a before b exactly when the reference's xorCmp(t, a, b) is -1."""
    ids = kat["ids"]
    ctx.set_ids(ids)
    n = ids.shape[0]
    tnames = kat["names"]
    targets = ids.copy()
    if path == "batch_k6":   # past the small-batch bound (q <= 64): the K6 pipeline F1..F4
        reps = 80 // n + 1
        targets = np.concatenate([ids] * reps)
        tnames = tnames * reps
    fn = {"scan": ctx.topk, "index": ctx.index_topk, "batch_small": ctx.batch_topk, "batch_k6": ctx.batch_topk}[path]
    got, cnt = fn(targets, n)
    assert np.all(cnt == n)
    want, _ = O.topk(ids, targets, n)
    assert np.array_equal(got, want), path
    rows = _order_rows(kat, got, targets)
    checked = 0
    for r, tn in enumerate(tnames):
        where = {nm: i for i, nm in enumerate(rows[r])}
        assert rows[r][0] == tn, (path, tn, rows[r])   # distance 0 first
        for t, a, b, w in kat["xor_cmp"]:
            if t != tn:
                continue
            assert (where[a] < where[b]) == (w == -1), (path, t, a, b, w, rows[r])
            checked += 1
    assert checked >= len(kat["xor_cmp"])


@pytest.mark.parametrize("k", [1, 3])
def test_kat_xor_cmp_small_k(ctx, kat, k):
    """the same ordering at k < n (the top-k cut itself): {null, min, max} only, k = 1 and 3"""
    sel = [kat["pos"][nm] for nm in ("null", "min", "max")]
    ids = kat["ids"][sel]
    ctx.set_ids(ids)
    want, wcnt = O.topk(ids, ids, k)
    for fn in (ctx.topk, ctx.index_topk, ctx.batch_topk):
        got, cnt = fn(ids, k)
        assert np.array_equal(cnt, wcnt) and np.array_equal(got, want)
    # max.xorCmp(null, min) = -1: from max, null is the closer of the two
    got, _ = ctx.topk(ids[2:3], 3)
    assert list(got[0]) == [2, 0, 1]


def test_kat_common_bits_through_classify(ctx, kat):
    """commonBits KATs (infohashtester.cpp:113-122) through K2's 161-bin histogram: the id set
    holds one hash, myid the other, so the histogram has exactly one count, at the KAT value."""
    H = {nm: kat["ids"][kat["pos"][nm]] for nm in kat["names"]}
    firsts = H["null"][None, :]   # one bucket covering everything
    for a, b, want in kat["common_bits"]:
        ctx.set_ids(H[b][None, :])
        bucket, hist = ctx.classify(firsts, H[a])
        assert int(hist.sum()) == 1 and int(hist[want]) == 1, (a, b, want, np.nonzero(hist)[0])
        assert int(bucket[0]) == 0


def test_kat_lowbit_through_table_stats(ctx, kat):
    """lowbit KATs (infohashtester.cpp:103-111) through the device's per-bucket table statistics"""
    names = [nm for nm, _ in kat["lowbit"]]
    firsts = np.stack([kat["ids"][kat["pos"][nm]] for nm in names])
    order = np.lexsort(firsts.T[::-1])   # bucket firsts ascend
    lb, _ = ctx.table_stats(firsts[order])
    for j, i in enumerate(order):
        assert int(lb[j]) == kat["lowbit"][i][1], names[i]


def test_kat_less_through_device_sort(ctx, kat):
    """operator< KATs (infohashtester.cpp:76-101) through the device radix sort of the NodeCache
    mirror: the sorted order puts a before b exactly when the reference's a < b."""
    ids = kat["ids"]
    ctx.cache_set(ids, version=0)
    perm = ctx.cache_sorted()
    rank = {kat["names"][int(i)]: r for r, i in enumerate(perm)}
    for a, b, want in kat["less"]:
        if a == b:
            continue
        assert (rank[a] < rank[b]) == want, (a, b)
