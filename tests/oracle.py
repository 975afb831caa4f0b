"""ctypes wrapper around oracle/liboracle.so -- the CPU restatement used as the
parity CHECKER.  Test infrastructure only: imported by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg; never by the opendht_amd product path."""
import contextlib
import ctypes
import os
import subprocess
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_LIB = os.path.join(ROOT, "oracle", "liboracle.so")
_lib = None

u8p = ctypes.POINTER(ctypes.c_uint8)
u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)


def build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        _lib = _load(_LIB)
    return _lib


_native = None


@contextlib.contextmanager
def native():
    """The same restatement compiled here with g++ -O3 -march=native (SURVEY 8(d)(ii)'s second
    CPU-baseline build), active inside the with-block.  Built on first use into a temp dir on
    the host that runs it (march=native must be this host's CPU)."""
    global _lib, _native
    if _native is None:
        d = tempfile.mkdtemp(prefix="oracle_native_")
        so = os.path.join(d, "liboracle_native.so")
        src = [os.path.join(ROOT, "oracle", f) for f in ("dht_oracle.cpp", "crawl_oracle.cpp")]
        subprocess.check_call(["g++", "-O3", "-march=native", "-std=c++11", "-fPIC", "-pthread", "-shared",
                               "-o", so] + src)
        _native = _load(so)
    saved = lib()
    _lib = _native
    try:
        yield
    finally:
        _lib = saved


def _load(path):
    L = ctypes.CDLL(path)
    L.orc_gen_ids.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, u8p]
    L.orc_xor_cmp.argtypes = [u8p, u8p, u8p]
    L.orc_xor_cmp.restype = ctypes.c_int
    L.orc_common_bits.argtypes = [u8p, u8p]
    L.orc_common_bits.restype = ctypes.c_uint
    L.orc_lowbit.argtypes = [u8p]
    L.orc_lowbit.restype = ctypes.c_int
    L.orc_cmp.argtypes = [u8p, u8p]
    L.orc_cmp.restype = ctypes.c_int
    L.orc_topk.argtypes = [u8p, ctypes.c_uint64, u8p, ctypes.c_uint32, ctypes.c_uint32,
                           u32p, u32p, ctypes.c_int]
    L.orc_topk_gen.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, u8p, ctypes.c_uint32,
                               ctypes.c_uint32, u32p, u32p, ctypes.c_int]
    L.orc_table_new.argtypes = [u8p, ctypes.c_int]
    L.orc_table_new.restype = ctypes.c_void_p
    L.orc_table_free.argtypes = [ctypes.c_void_p]
    L.orc_table_insert.argtypes = [ctypes.c_void_p, u8p]
    L.orc_table_insert.restype = ctypes.c_int
    L.orc_table_nbuckets.argtypes = [ctypes.c_void_p]
    L.orc_table_nbuckets.restype = ctypes.c_uint32
    L.orc_table_nnodes.argtypes = [ctypes.c_void_p]
    L.orc_table_nnodes.restype = ctypes.c_uint32
    L.orc_table_export.argtypes = [ctypes.c_void_p, u8p, u32p, u8p]
    L.orc_find_bucket.argtypes = [ctypes.c_uint32, u8p, u8p]
    L.orc_find_bucket.restype = ctypes.c_int
    L.orc_depth.argtypes = [ctypes.c_uint32, u8p, ctypes.c_uint32]
    L.orc_depth.restype = ctypes.c_uint
    L.orc_find_closest.argtypes = [ctypes.c_uint32, u8p, u32p, u8p, u8p, u8p, ctypes.c_uint32, u32p]
    L.orc_find_closest.restype = ctypes.c_uint32
    L.orc_classify.argtypes = [ctypes.c_uint32, u8p, u8p, u8p, ctypes.c_uint64, u8p, u64p]
    L.orc_classify_mt.argtypes = [ctypes.c_uint32, u8p, u8p, u8p, ctypes.c_uint64, u8p, u64p, ctypes.c_int]
    L.orc_search_insert.argtypes = [u8p, u8p, u8p, ctypes.c_uint32, ctypes.c_uint32, u32p, u8p, u32p, u8p, u64p,
                                    u32p, u8p, u8p, ctypes.c_int]
    L.orc_find_closest_batch.argtypes = [ctypes.c_uint32, u8p, u32p, u8p, u8p, u8p, ctypes.c_uint32,
                                         ctypes.c_uint32, u32p, u32p, ctypes.c_int]
    L.orc_cached_nodes_batch.argtypes = [u8p, ctypes.c_uint64, u8p, u8p, ctypes.c_uint32, ctypes.c_uint32,
                                         u32p, u32p, ctypes.c_int]
    L.orc_cached_nodes.argtypes = [u8p, ctypes.c_uint64, u8p, u8p, ctypes.c_uint32, u32p]
    L.orc_cached_nodes.restype = ctypes.c_uint32
    L.orc_buffer_nodes.argtypes = [u8p, u8p, ctypes.c_uint32, u8p, u32p, ctypes.c_uint32, u8p]
    L.orc_buffer_nodes.restype = ctypes.c_uint32
    L.orc_deserialize_node.argtypes = [u8p, ctypes.c_uint32, u8p, ctypes.c_uint32, u8p, u8p]
    L.orc_deserialize_node.restype = ctypes.c_int
    L.orc_search_batch.argtypes = [u8p, ctypes.c_uint64, u8p, ctypes.c_uint64, u8p, u32p, ctypes.c_uint32,
                                   ctypes.c_uint32, u32p, u8p, u32p, u32p, u32p, ctypes.c_int, ctypes.c_uint32]
    return L


def _p(a, t):
    return a.ctypes.data_as(t)


def h(hexstr):
    return np.frombuffer(bytes.fromhex(hexstr), dtype=np.uint8).copy()


def gen_ids(seed, n, start=0):
    out = np.empty((n, 20), dtype=np.uint8)
    lib().orc_gen_ids(seed, start, n, _p(out, u8p))
    return out


def xor_cmp(t, a, b):
    return lib().orc_xor_cmp(_p(t, u8p), _p(a, u8p), _p(b, u8p))


def common_bits(a, b):
    return lib().orc_common_bits(_p(a, u8p), _p(b, u8p))


def lowbit(a):
    return lib().orc_lowbit(_p(a, u8p))


def cmp(a, b):
    return lib().orc_cmp(_p(a, u8p), _p(b, u8p))


def default_threads():
    """Worker threads when the caller names none: the host's CPUs, at most 16 (a GPU box's CPU
    share; os.cpu_count() there reports the whole machine).  An explicit count is used as given
    (bench.py's cpu_baseline runs at every host CPU)."""
    return min(os.cpu_count() or 1, 16)


def topk(ids, targets, k, threads=None):
    ids = np.ascontiguousarray(ids, dtype=np.uint8)
    targets = np.ascontiguousarray(targets, dtype=np.uint8)
    q = targets.shape[0]
    out = np.empty((q, k), dtype=np.uint32)
    cnt = np.empty(q, dtype=np.uint32)
    lib().orc_topk(_p(ids, u8p), ids.shape[0], _p(targets, u8p), q, k, _p(out, u32p), _p(cnt, u32p),
                   int(threads or default_threads()))
    return out, cnt


def topk_gen(seed, n, targets, k, start=0, threads=None):
    """topk() over the gen_ids(seed, n, start) stream generated on the fly (no id array: BASELINE
    cfg 3's 10^9 ids); indices are stream indices start + i."""
    targets = np.ascontiguousarray(targets, dtype=np.uint8)
    q = targets.shape[0]
    out = np.empty((q, k), dtype=np.uint32)
    cnt = np.empty(q, dtype=np.uint32)
    lib().orc_topk_gen(seed, start, n, _p(targets, u8p), q, k, _p(out, u32p), _p(cnt, u32p),
                       int(threads or default_threads()))
    return out, cnt


class Table:
    """A RoutingTable grown with onNewNode (src/routing_table.cpp:204-262)."""

    def __init__(self, myid, is_client=False):
        self.myid = np.ascontiguousarray(myid, dtype=np.uint8)
        self._t = lib().orc_table_new(_p(self.myid, u8p), int(is_client))

    def __del__(self):
        if getattr(self, "_t", None):
            lib().orc_table_free(self._t)
            self._t = None

    def insert(self, id20):
        id20 = np.ascontiguousarray(id20, dtype=np.uint8)
        return lib().orc_table_insert(self._t, _p(id20, u8p))

    def grow(self, ids):
        for row in np.ascontiguousarray(ids, dtype=np.uint8):
            self.insert(row)
        return self

    def export(self):
        nb = lib().orc_table_nbuckets(self._t)
        nn = lib().orc_table_nnodes(self._t)
        firsts = np.zeros((nb, 20), dtype=np.uint8)
        off = np.zeros(nb + 1, dtype=np.uint32)
        ids = np.zeros((max(nn, 1), 20), dtype=np.uint8)
        lib().orc_table_export(self._t, _p(firsts, u8p), _p(off, u32p), _p(ids, u8p))
        return firsts, off, ids[:nn]


def find_bucket(firsts, id20):
    firsts = np.ascontiguousarray(firsts, dtype=np.uint8)
    return lib().orc_find_bucket(firsts.shape[0], _p(firsts, u8p), _p(np.ascontiguousarray(id20), u8p))


def depth(firsts, b):
    firsts = np.ascontiguousarray(firsts, dtype=np.uint8)
    return lib().orc_depth(firsts.shape[0], _p(firsts, u8p), b)


def find_closest(firsts, off, ids, good, target, count):
    firsts = np.ascontiguousarray(firsts, dtype=np.uint8)
    ids = np.ascontiguousarray(ids, dtype=np.uint8)
    good = np.ascontiguousarray(good, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint32)
    target = np.ascontiguousarray(target, dtype=np.uint8)
    out = np.empty(max(count, 1), dtype=np.uint32)
    c = lib().orc_find_closest(firsts.shape[0], _p(firsts, u8p), _p(off, u32p), _p(ids, u8p),
                               _p(good, u8p), _p(target, u8p), count, _p(out, u32p))
    return out[:c].copy()


def find_closest_batch(firsts, off, ids, good, targets, count, threads=1):
    """findClosestNodes for every target: ((q, count) indices, UINT32_MAX padded; (q,) counts)."""
    firsts = np.ascontiguousarray(firsts, dtype=np.uint8)
    ids = np.ascontiguousarray(ids, dtype=np.uint8)
    good = np.ascontiguousarray(good, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint32)
    targets = np.ascontiguousarray(targets, dtype=np.uint8)
    q = targets.shape[0]
    out = np.full((q, count), 0xFFFFFFFF, dtype=np.uint32)
    cnt = np.zeros(q, dtype=np.uint32)
    lib().orc_find_closest_batch(firsts.shape[0], _p(firsts, u8p), _p(off, u32p), _p(ids, u8p), _p(good, u8p),
                                 _p(targets, u8p), q, count, _p(out, u32p), _p(cnt, u32p), threads)
    return out, cnt


def cached_nodes_batch(sorted_ids, accept, targets, count, threads=1):
    sorted_ids = np.ascontiguousarray(sorted_ids, dtype=np.uint8)
    accept = np.ascontiguousarray(accept, dtype=np.uint8)
    targets = np.ascontiguousarray(targets, dtype=np.uint8)
    q = targets.shape[0]
    out = np.full((q, count), 0xFFFFFFFF, dtype=np.uint32)
    cnt = np.zeros(q, dtype=np.uint32)
    lib().orc_cached_nodes_batch(_p(sorted_ids, u8p), sorted_ids.shape[0], _p(accept, u8p), _p(targets, u8p), q,
                                 count, _p(out, u32p), _p(cnt, u32p), threads)
    return out, cnt


def search_insert(node_ids, node_state, targets, lists, flags, lens, expired, ins_off, ins_node, ins_token):
    """Search::insertNode restatement, batched (same contract as libdhtgpu's search_insert)."""
    node_ids = np.ascontiguousarray(node_ids, dtype=np.uint8)
    st = np.ascontiguousarray(node_state, dtype=np.uint8)
    targets = np.ascontiguousarray(targets, dtype=np.uint8)
    lists = np.ascontiguousarray(lists, dtype=np.uint32).copy()
    flags = np.ascontiguousarray(flags, dtype=np.uint8).copy()
    lens = np.ascontiguousarray(lens, dtype=np.uint32).copy()
    expired = np.ascontiguousarray(expired, dtype=np.uint8).copy()
    off = np.ascontiguousarray(ins_off, dtype=np.uint64)
    node = np.ascontiguousarray(ins_node, dtype=np.uint32)
    tok = np.ascontiguousarray(ins_token, dtype=np.uint8)
    added = np.zeros(max(node.size, 1), np.uint8)
    lib().orc_search_insert(_p(node_ids, u8p), _p(st, u8p), _p(targets, u8p), targets.shape[0], lists.shape[1],
                            _p(lists, u32p), _p(flags, u8p), _p(lens, u32p), _p(expired, u8p), _p(off, u64p),
                            _p(node, u32p), _p(tok, u8p), _p(added, u8p), 4)
    return lists, flags, lens, expired, added[: node.size]


def classify(firsts, myid, ids, threads=1):
    """findBucket + commonBits per id (src/routing_table.cpp:153-166, infohash.h:154-176)."""
    firsts = np.ascontiguousarray(firsts, dtype=np.uint8)
    ids = np.ascontiguousarray(ids, dtype=np.uint8)
    myid = np.ascontiguousarray(myid, dtype=np.uint8)
    n = ids.shape[0]
    out = np.empty(max(n, 1), dtype=np.uint8)
    hist = np.zeros(161, dtype=np.uint64)
    if threads > 1:
        lib().orc_classify_mt(firsts.shape[0], _p(firsts, u8p), _p(myid, u8p), _p(ids, u8p), n,
                              _p(out, u8p), _p(hist, u64p), threads)
    else:
        lib().orc_classify(firsts.shape[0], _p(firsts, u8p), _p(myid, u8p), _p(ids, u8p), n,
                           _p(out, u8p), _p(hist, u64p))
    return out[:n].copy(), hist


def cached_nodes(sorted_ids, accept, target, count):
    sorted_ids = np.ascontiguousarray(sorted_ids, dtype=np.uint8)
    accept = np.ascontiguousarray(accept, dtype=np.uint8)
    target = np.ascontiguousarray(target, dtype=np.uint8)
    out = np.empty(max(count, 1), dtype=np.uint32)
    c = lib().orc_cached_nodes(_p(sorted_ids, u8p), sorted_ids.shape[0], _p(accept, u8p),
                               _p(target, u8p), count, _p(out, u32p))
    return out[:c].copy()


def buffer_nodes(ids, tail, alen, target, cand):
    """NetworkEngine::bufferNodes restatement: blob bytes."""
    ids = np.ascontiguousarray(ids, dtype=np.uint8)
    tail = np.ascontiguousarray(tail, dtype=np.uint8)
    target = np.ascontiguousarray(target, dtype=np.uint8)
    cand = np.ascontiguousarray(cand, dtype=np.uint32)
    out = np.zeros(8 * (22 + alen), dtype=np.uint8)
    n = lib().orc_buffer_nodes(_p(ids, u8p), _p(tail, u8p), alen, _p(target, u8p), _p(cand, u32p), cand.shape[0],
                               _p(out, u8p))
    return out[:n].copy()


def deserialize_node(rec, af, myid, from_af, from_addr):
    """NetworkEngine::deserializeNodes for one record: (status, address || port bytes)."""
    alen = 4 if af == 4 else 16
    rec = np.ascontiguousarray(rec, dtype=np.uint8)
    myid = np.ascontiguousarray(myid, dtype=np.uint8)
    fa = np.ascontiguousarray(from_addr, dtype=np.uint8).reshape(16)
    out = np.zeros(alen + 2, dtype=np.uint8)
    st = lib().orc_deserialize_node(_p(rec, u8p), af, _p(myid, u8p), from_af, _p(fa, u8p), _p(out, u8p))
    return st, out


def search_batch(ids, dead, table_seed, targets, searchers, max_rounds=64, threads=None, alpha=4):
    """Crawl-replay model (oracle/crawl_oracle.cpp): (idx, flags, len, rounds, queries); alpha =
    requests per round (4 = MAX_REQUESTED_SEARCH_NODES, include/opendht/dht.h:321)."""
    ids = np.ascontiguousarray(ids, dtype=np.uint8)
    targets = np.ascontiguousarray(targets, dtype=np.uint8)
    q = targets.shape[0]
    sr = np.ascontiguousarray(searchers, dtype=np.uint32)
    d = np.ascontiguousarray(dead, dtype=np.uint8) if dead is not None else None
    idx = np.empty((q, 64), np.uint32)
    fl = np.empty((q, 64), np.uint8)
    ln, rd, qs = (np.empty(q, np.uint32) for _ in range(3))
    lib().orc_search_batch(_p(ids, u8p), ids.shape[0], _p(d, u8p) if d is not None else None, table_seed,
                           _p(targets, u8p), _p(sr, u32p), q, max_rounds, _p(idx, u32p), _p(fl, u8p),
                           _p(ln, u32p), _p(rd, u32p), _p(qs, u32p), int(threads or default_threads()), int(alpha))
    return idx, fl, ln, rd, qs


# ---- independent pure-Python restatement (big integers) used to cross-check the C oracle ----
def py_dist(t, a):
    return int.from_bytes(bytes(t), "big") ^ int.from_bytes(bytes(a), "big")


def py_topk(ids, target, k):
    d = [(py_dist(target, row), i) for i, row in enumerate(ids)]
    d.sort()
    return [i for _, i in d[:k]]


def py_buffer_nodes(ids, tail, target, cand):
    """bufferNodes restated with big integers (stable order for equal ids)."""
    c = [int(x) for x in cand if x != 0xFFFFFFFF]
    c.sort(key=lambda i: py_dist(target, ids[i]))
    out = b""
    for i in c[:8]:
        out += bytes(ids[i]) + bytes(tail[i])
    return np.frombuffer(out, dtype=np.uint8)


def py_deserialize_node(rec, af, myid, from_af, from_addr):
    """deserializeNodes + isMartian restated from src/network_engine.cpp:362-386, :831-887."""
    alen = 4 if af == 4 else 16
    rec = bytes(rec)
    if rec[:20] == bytes(myid):
        return 1, None
    a = bytearray(rec[20:20 + alen])
    port = rec[20 + alen:22 + alen]
    loop = (a[0] == 127) if af == 4 else (bytes(a) == bytes(15) + b"\x01")
    if loop and from_af == af:
        a = bytearray(bytes(from_addr)[:alen])
    tailb = np.frombuffer(bytes(a) + port, dtype=np.uint8)
    if port == b"\0\0":
        return 2, tailb
    if af == 4:
        return (2 if a[0] == 0 or (a[0] & 0xE0) == 0xE0 else 0), tailb
    m = a[0] == 0xFF or (a[0] == 0xFE and (a[1] & 0xC0) == 0x80) or bytes(a) == bytes(16) or \
        bytes(a[:12]) == bytes(10) + b"\xff\xff"
    return (2 if m else 0), tailb


def special_addrs(rng, n, af):
    """Address || port tails mixing ordinary, loopback, martian and port-0 cases."""
    alen = 4 if af == 4 else 16
    t = rng.integers(0, 256, size=(n, alen + 2), dtype=np.uint8)
    k = rng.integers(0, 8, size=n)
    for i in range(n):
        if k[i] == 0:
            t[i, alen:] = 0                                   # port 0
        elif k[i] == 1:
            if af == 4:
                t[i, 0] = 127                                 # loopback
            else:
                t[i, :16] = 0
                t[i, 15] = 1
        elif k[i] == 2:
            if af == 4:
                t[i, 0] = 0
            else:
                t[i, 0] = 0xFF                                # multicast
        elif k[i] == 3:
            if af == 4:
                t[i, 0] = 0xE0 | (t[i, 0] & 0x1F)              # class D/E
            else:
                t[i, 0], t[i, 1] = 0xFE, 0x80 | (t[i, 1] & 0x3F)   # link-local
        elif k[i] == 4 and af == 6:
            t[i, :10] = 0
            t[i, 10:12] = 0xFF                                # v4-mapped
        elif k[i] == 5 and af == 6:
            t[i, :16] = 0                                     # unspecified
    return t
