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


@pytest.mark.parametrize("n,k,start", [(5, 8, 0), (20000, 8, 0), (20000, 1, 3), (150000, 32, 10**6)])
def test_topk_gen_equals_topk(n, k, start):
    """The generator-fed entry (cfg 3's 10^9-id checker: ids made on the fly, per-thread bounded
    lists merged) == the array form, on stream indices; targets include exact hits and a target
    sharing 40 leading bits with an id (word-1 ties)."""
    ids = O.gen_ids(21, n, start=start)
    tg = O.gen_ids(22, 24)
    tg[:3] = ids[[0, n // 2, n - 1]]
    tg[3, :5] = ids[n // 3, :5]
    want, wcnt = O.topk(ids, tg, k, threads=4)
    got, gcnt = O.topk_gen(21, n, tg, k, start=start, threads=3)
    want = np.where(want == 0xFFFFFFFF, want, want + start)
    assert np.array_equal(got, want) and np.array_equal(gcnt, wcnt)
    assert list(got[5, :gcnt[5]]) == [start + i for i in O.py_topk(ids, tg[5], k)]


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


@pytest.mark.parametrize("af", [4, 6])
def test_buffer_nodes_oracle_vs_python(af):
    """bufferNodes restatement (C) == big-integer restatement, incl. absent candidates and
    fewer than 8 nodes."""
    rng = np.random.default_rng(af)
    ids = O.gen_ids(700 + af, 300)
    ids[:20, :4] = ids[0, :4]                 # shared w0 words: full-key ordering
    alen = 4 if af == 4 else 16
    tail = O.special_addrs(rng, 300, af)
    for trial in range(200):
        t = O.gen_ids(800 + trial, 1)[0]
        if trial % 3 == 0:
            t[:4] = ids[0, :4]
        c = int(rng.integers(0, 33))
        cand = rng.choice(300, size=c, replace=False).astype(np.uint32)
        if c > 2 and trial % 2:
            cand[rng.integers(0, c)] = 0xFFFFFFFF
        got = O.buffer_nodes(ids, tail, alen, t, cand)
        want = O.py_buffer_nodes(ids, tail, t, cand)
        assert np.array_equal(got, want), trial
        assert got.size % (22 + alen) == 0 and got.size <= 8 * (22 + alen)


@pytest.mark.parametrize("af", [4, 6])
def test_deserialize_node_oracle_vs_python(af):
    rng = np.random.default_rng(10 + af)
    alen = 4 if af == 4 else 16
    myid = O.gen_ids(901, 1)[0]
    ids = O.gen_ids(902, 500)
    ids[::37] = myid
    tail = O.special_addrs(rng, 500, af)
    for i in range(500):
        rec = np.concatenate([ids[i], tail[i]])
        from_af = [0, 4, 6][i % 3]
        from_addr = rng.integers(0, 256, size=16, dtype=np.uint8)
        st, out = O.deserialize_node(rec, af, myid, from_af, from_addr)
        wst, wout = O.py_deserialize_node(rec, af, myid, from_af, from_addr)
        assert st == wst, i
        if st != 1:
            assert np.array_equal(out, wout), i


def test_ipv4_record_layout_known_answer():
    """A hand-built 26-byte record (id || sin_addr || sin_port, network order) decodes to
    itself; 127.0.0.1 from an IPv4 sender takes the sender's address and keeps its port."""
    myid = O.h("00" * 20)
    rid = O.h("0123456789abcdef0123456789abcdef01234567")
    rec = np.concatenate([rid, O.h("c0a80001"), O.h("1f90")])          # 192.168.0.1:8080
    st, out = O.deserialize_node(rec, 4, myid, 4, np.zeros(16, np.uint8))
    assert st == 0 and bytes(out) == bytes.fromhex("c0a800011f90")
    rec2 = np.concatenate([rid, O.h("7f000001"), O.h("1f90")])         # 127.0.0.1:8080
    frm = np.concatenate([O.h("0a000002"), np.zeros(12, np.uint8)])     # from 10.0.0.2
    st, out = O.deserialize_node(rec2, 4, myid, 4, frm)
    assert st == 0 and bytes(out) == bytes.fromhex("0a0000021f90")
    st, _ = O.deserialize_node(np.concatenate([rid, O.h("e0000001"), O.h("1f90")]), 4, myid, 4, frm)
    assert st == 2                                                      # 224.0.0.1: martian


def test_crawl_driver_on_oracle_model():
    """dhtscanner restatement (opendht_amd/crawl.py) over the oracle's search model: the
    scan stays within the 2^8 prefix steps of tools/dhtscanner.cpp and finds nodes close
    to every probed prefix."""
    from opendht_amd import crawl
    ids = O.gen_ids(4242, 20000)
    dead = (np.random.default_rng(1).random(20000) < 0.1).astype(np.uint8)
    res = crawl.crawl(lambda t, s, r: O.search_batch(ids, dead, 99, t, s, r), lambda ix: ids[ix], 17)
    assert 1 <= res["steps"] <= 256
    assert res["found"].size > 100
    assert res["queries"] > 0
    # bit numbering of setBit: bit 159 is the last byte's lowest bit
    assert crawl.set_bit(np.zeros(20, np.uint8), 159)[19] == 1
    assert crawl.set_bit(np.zeros(20, np.uint8), 0)[0] == 0x80


def test_search_model_converges_to_exact_topk():
    """Size-independent property of the crawl model: with no dead nodes, nearly every
    search ends with the exact 8 XOR-closest nodes of the network at the head of its list."""
    ids = O.gen_ids(77, 50000)
    tg = O.gen_ids(78, 200)
    sr = (np.arange(200, dtype=np.uint32) * 211) % 50000
    idx, fl, ln, rd, qs = O.search_batch(ids, None, 5, tg, sr)
    want, _ = O.topk(ids, tg, 8)
    exact = sum(list(idx[i, :8]) == list(want[i]) for i in range(200))
    assert exact >= 190, exact
    assert np.all(ln >= 8) and np.all(rd <= 64)


def py_insert_node(ids, state, target, lst, fl, expired, x, token):
    """Search::insertNode (src/search.h:636-722) restated in Python on big integers, independent
    of the C oracle: lst/fl are Python lists (modified), returns (added, expired)."""
    dist = lambda i: int.from_bytes(bytes(ids[i]), "big") ^ int.from_bytes(bytes(target), "big")
    bad = lambda j: bool(state[lst[j]] & 1) or bool(fl[j] & 1)
    n = len(lst)
    found = False
    while n:
        n -= 1
        if lst[n] == x:
            found = True
            break
        if dist(x) > dist(lst[n]):
            n += 1
            break
    added = False
    if not found:
        t, nb, full = len(lst), 0, False
        if expired:
            if len(lst) >= 14:
                full, t = True, 14
        else:
            nb = sum(bad(j) for j in range(len(lst)))
            full = len(lst) - nb >= 14
            while t - nb > 14:
                t -= 1
                nb -= bad(t)
        if full:
            del lst[t:]
            del fl[t:]
            if n >= t:
                return False, expired
        lst.insert(n, x)
        fl.insert(n, 0)
        added = True
        if state[x] & 1:
            if not expired:
                nb += 1
        elif expired:
            nb, expired = len(lst) - 1, False
        while len(lst) - nb > 14:
            if not expired and bad(len(lst) - 1):
                nb -= 1
            lst.pop()
            fl.pop()
    if token and n < len(lst) and lst[n] == x:
        fl[n] = (fl[n] & ~1) | 2
        expired = False
    if added:
        for e in range(len(lst) - 1, -1, -1):
            if state[lst[e]] & 2:
                del lst[e]
                del fl[e]
                break
    return added, expired


def test_search_insert_oracle_vs_python():
    """The C restatement of Search::insertNode equals an independent Python restatement over
    random insertion sequences (expired / removable nodes, candidates, tokens, expired searches)."""
    rng = np.random.default_rng(11)
    nn, q, cap = 400, 60, 64
    ids = O.gen_ids(9, nn)
    ids[:40, :4] = ids[0, :4]
    state = rng.choice([0, 0, 0, 1, 3], size=nn).astype(np.uint8)
    tg = O.gen_ids(10, q)
    lists = np.full((q, cap), 0xFFFFFFFF, np.uint32)
    flags = np.zeros((q, cap), np.uint8)
    lens = np.zeros(q, np.uint32)
    expired = (rng.random(q) < 0.2).astype(np.uint8)
    counts = rng.integers(0, 40, size=q)
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    node = rng.integers(0, nn, size=int(off[-1])).astype(np.uint32)
    tok = (rng.random(node.size) < 0.3).astype(np.uint8)
    got = O.search_insert(ids, state, tg, lists, flags, lens, expired, off, node, tok)
    for s in range(q):
        lst, fl, ex = [], [], bool(expired[s])
        adds = []
        for i in range(int(off[s]), int(off[s + 1])):
            a, ex = py_insert_node(ids, state, tg[s], lst, fl, ex, int(node[i]), bool(tok[i]))
            adds.append(int(a))
        assert got[2][s] == len(lst), s
        assert list(got[0][s, : len(lst)]) == lst and list(got[1][s, : len(lst)]) == fl, s
        assert bool(got[3][s]) == ex and list(got[4][int(off[s]):int(off[s + 1])]) == adds, s
