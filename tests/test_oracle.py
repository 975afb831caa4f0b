"""The oracle (CPU restatement) pinned against the reference's own known answers
(tests/infohashtester.cpp:76-138) and cross-checked against an independent
pure-Python restatement.  CPU only."""
import json
import os

import numpy as np
import pytest

import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "infohash_kat.json")


@pytest.fixture(scope="module")
def kat():
    with open(GOLD) as f:
        k = json.load(f)
    k["H"] = {name: O.h(v) for name, v in k["hashes"].items()}
    return k


def test_kat_less(kat):
    H = kat["H"]
    for a, b, want in kat["less"]:
        assert (O.cmp(H[a], H[b]) < 0) == want, (a, b)


def test_kat_lowbit(kat):
    H = kat["H"]
    for a, want in kat["lowbit"]:
        assert O.lowbit(H[a]) == want, a


def test_kat_common_bits(kat):
    H = kat["H"]
    for a, b, want in kat["common_bits"]:
        assert O.common_bits(H[a], H[b]) == want, (a, b)


def test_kat_xor_cmp(kat):
    H = kat["H"]
    for t, a, b, want in kat["xor_cmp"]:
        assert O.xor_cmp(H[t], H[a], H[b]) == want, (t, a, b)


def test_generator_deterministic_unique():
    a = O.gen_ids(7, 5000)
    b = O.gen_ids(7, 5000)
    assert np.array_equal(a, b)
    c = O.gen_ids(7, 100, start=4900)
    assert np.array_equal(a[4900:], c)
    assert len({bytes(r) for r in a}) == 5000


def test_xor_cmp_matches_bigint():
    rng = np.random.default_rng(1)
    for _ in range(3000):
        t, a, b = (rng.integers(0, 256, 20, dtype=np.uint8) for _ in range(3))
        if rng.random() < 0.3:
            m = int(rng.integers(0, 21))
            b[:m] = a[:m]
        da, db = O.py_dist(t, a), O.py_dist(t, b)
        want = -1 if da < db else (1 if da > db else 0)
        assert O.xor_cmp(t, a, b) == want


def test_common_bits_lowbit_bigint():
    rng = np.random.default_rng(2)
    for _ in range(3000):
        a = rng.integers(0, 256, 20, dtype=np.uint8)
        b = a.copy()
        nb = int(rng.integers(0, 161))
        if nb < 160:
            b[nb // 8] ^= 0x80 >> (nb % 8)
            b[nb // 8 + 1:] = rng.integers(0, 256, 20 - nb // 8 - 1, dtype=np.uint8)
        x = O.py_dist(a, b)
        assert O.common_bits(a, b) == (160 if x == 0 else 160 - x.bit_length())
        v = int.from_bytes(bytes(a), "big")
        want = -1 if v == 0 else 159 - ((v & -v).bit_length() - 1)
        assert O.lowbit(a) == want


@pytest.mark.parametrize("n,k", [(1, 8), (7, 8), (100, 8), (1000, 14), (3000, 32)])
def test_topk_vs_bigint(n, k):
    ids = O.gen_ids(11, n)
    tg = O.gen_ids(12, 16)
    out, cnt = O.topk(ids, tg, k)
    for qi in range(16):
        want = O.py_topk(ids, tg[qi], k)
        assert cnt[qi] == len(want)
        assert list(out[qi, :cnt[qi]]) == want
        assert np.all(out[qi, cnt[qi]:] == 0xFFFFFFFF)


def test_topk_duplicates_tie_by_index():
    base = O.gen_ids(3, 50)
    ids = np.concatenate([base, base[::-1], base[:5]])
    tg = np.concatenate([base[:4], O.gen_ids(4, 4)])
    out, cnt = O.topk(ids, tg, 16)
    for qi in range(tg.shape[0]):
        assert list(out[qi]) == O.py_topk(ids, tg[qi], 16)


def _py_find_closest_slice(firsts, off, ids, good, target, count):
    """SURVEY §8(a) a7 semantics as a slice: contiguous bucket range grown outward
    from findBucket(target) until >= count good nodes, then exact XOR top-count."""
    nb = firsts.shape[0]
    if nb == 0:
        return []
    j = O.find_bucket(firsts, target)
    g = [int(good[off[b]:off[b + 1]].sum()) for b in range(nb)]
    c, itn, itp = 0, j, j - 1
    while c < count and (itn < nb or itp >= 0):
        if itn < nb:
            c += g[itn]; itn += 1
        if itp >= 0:
            c += g[itp]; itp -= 1
    lo, hi = off[itp + 1], off[itn]
    cand = [(O.py_dist(target, ids[i]), i) for i in range(lo, hi) if good[i]]
    cand.sort()
    return [i for _, i in cand[:count]]


@pytest.mark.parametrize("n_grow,expired,cluster", [(2000, 0.0, False), (10000, 0.3, False),
                                                     (5000, 0.6, False), (3000, 0.3, True)])
def test_find_closest_restatement_vs_slice(n_grow, expired, cluster):
    myid = O.gen_ids(99, 1)[0]
    ids = O.gen_ids(100, n_grow)
    if cluster:
        ids[: n_grow // 2, :3] = myid[:3]
    tab = O.Table(myid).grow(ids)
    firsts, off, nodes = tab.export()
    assert firsts.shape[0] > 1 and nodes.shape[0] > 8
    rng = np.random.default_rng(5)
    good = (rng.random(nodes.shape[0]) >= expired).astype(np.uint8)
    targets = np.concatenate([O.gen_ids(101, 300), nodes[:50]])
    if cluster:
        targets[:100, :3] = myid[:3]
    for t in targets:
        for count in (8, 14):
            got = list(O.find_closest(firsts, off, nodes, good, t, count))
            assert got == _py_find_closest_slice(firsts, off, nodes, good, t, count)


def test_table_shape_cfg1():
    """Cfg 1: a table grown from 10k random ids (SURVEY: 12 buckets / ~91 nodes with the
    reference's own PRNG stream; our generator gives a similar shape)."""
    tab = O.Table(O.gen_ids(1, 1)[0]).grow(O.gen_ids(2, 10000))
    firsts, off, nodes = tab.export()
    assert 8 <= firsts.shape[0] <= 20
    assert 60 <= nodes.shape[0] <= 160
    assert np.all(np.diff(off) <= 8)
    # buckets are lexicographically sorted ranges containing their nodes
    for b in range(firsts.shape[0]):
        for i in range(off[b], off[b + 1]):
            assert O.find_bucket(firsts, nodes[i]) == b


def test_depth_and_classify():
    myid = O.gen_ids(1, 1)[0]
    firsts, off, nodes = O.Table(myid).grow(O.gen_ids(2, 4000)).export()
    ids = O.gen_ids(3, 2000)
    b, hist = O.classify(firsts, myid, ids)
    for i in range(0, 2000, 37):
        assert b[i] == O.find_bucket(firsts, ids[i])
    want = np.zeros(161, dtype=np.uint64)
    for r in ids:
        want[O.common_bits(r, myid)] += 1
    assert np.array_equal(hist, want)
    d = [O.depth(firsts, i) for i in range(firsts.shape[0])]
    assert max(d) >= 3


def _py_cached(sorted_ids, accept, target, count):
    keys = [bytes(r) for r in sorted_ids]
    import bisect
    n = len(keys)
    lo = bisect.bisect_left(keys, bytes(target))
    p, nx, out = lo - 1, lo, []
    while len(out) < count and (nx < n or p >= 0):
        if p < 0:
            it = nx; nx += 1
        elif nx >= n:
            it = p; p -= 1
        elif O.py_dist(target, sorted_ids[p]) < O.py_dist(target, sorted_ids[nx]):
            it = p; p -= 1
        else:
            it = nx; nx += 1
        if accept[it]:
            out.append(it)
    return out


@pytest.mark.parametrize("n", [0, 1, 5, 1000])
def test_cached_nodes_restatement(n):
    ids = O.gen_ids(21, max(n, 1))[:n]
    order = sorted(range(n), key=lambda i: bytes(ids[i]))
    s = ids[order] if n else ids
    rng = np.random.default_rng(9)
    accept = (rng.random(n) < 0.7).astype(np.uint8)
    for t in np.concatenate([O.gen_ids(22, 60), s[:5]]):
        for count in (1, 8, 14):
            assert list(O.cached_nodes(s, accept, t, count)) == _py_cached(s, accept, t, count)
