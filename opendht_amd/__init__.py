"""opendht_amd -- Python host binding for libdhtgpu, the MI355X engine behind
OpenDHT's XOR-closest-node lookup.

This is a thin ctypes layer over the C ABI declared in include/dhtgpu.h; every
compute call runs the hand-written HIP kernels in opendht_amd/libdhtgpu.so.  There is
no CPU fallback: if the native library is missing or cannot be loaded, import of the
compute API raises.

Reference interfaces mirrored (OpenDHT tree paths):
  Context.topk            std::partial_sort(.., InfoHash::xorCmp)  (include/opendht/infohash.h:179-194)
  Context.find_closest    RoutingTable::findClosestNodes            (src/routing_table.cpp:110-150)
  Context.cached_nodes    NodeCache::getCachedNodes                 (src/node_cache.cpp:42-74)
  Context.cache_set/_nodes  the NodeCache mirror: unsorted keys sorted on the device (node_cache.h:43)
  Context.classify        RoutingTable::findBucket + InfoHash::commonBits
"""
import ctypes
import os

import numpy as np

__all__ = ["Context", "DhtGpuError", "NONE", "MAX_K", "lib", "LIB_PATH", "id_words"]

# DHTGPU_LIB: another build of the same library (A/B experiments, tools/experiments/gpu_ab_lib.sh)
LIB_PATH = os.environ.get("DHTGPU_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libdhtgpu.so")
NONE = 0xFFFFFFFF
MAX_K = 32
# status codes (include/dhtgpu.h)
EINVAL, ENOMEM, EDEVICE, ENOIDS, EUNSORTED, ERANGE = -1, -2, -3, -4, -5, -6

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p
_lib = None


class DhtGpuError(RuntimeError):
    def __init__(self, code, what=""):
        msg = _lib.dhtgpu_strerror(code).decode() if _lib is not None else str(code)
        super().__init__(f"libdhtgpu: {what}: {msg} ({code})")
        self.code = code


def _check(code, what):
    if code != 0:
        raise DhtGpuError(code, what)


def lib():
    """Load libdhtgpu.so (raises if absent: there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libdhtgpu.so not built at {LIB_PATH}: run `python -c 'import __graft_entry__ as g; g.build()'`")
    try:  # share the HIP runtime with torch when both live in the process
        import torch  # noqa: F401
    except Exception:
        pass
    L = ctypes.CDLL(LIB_PATH)
    sig = {
        "dhtgpu_strerror": ([ctypes.c_int], ctypes.c_char_p),
        "dhtgpu_device_count": ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        "dhtgpu_ctx_create": ([ctypes.c_int, ctypes.POINTER(_vp)], ctypes.c_int),
        "dhtgpu_ctx_destroy": ([_vp], None),
        "dhtgpu_ctx_stream": ([_vp], _vp),
        "dhtgpu_set_ids": ([_vp, _u8p, ctypes.c_uint64], ctypes.c_int),
        "dhtgpu_gen_ids": ([_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64], ctypes.c_int),
        "dhtgpu_num_ids": ([_vp], ctypes.c_uint64),
        "dhtgpu_set_global_indices": ([_vp, ctypes.c_int], ctypes.c_int),
        "dhtgpu_set_sub_handles": ([_vp, ctypes.c_int], ctypes.c_int),
        "dhtgpu_sub_handles_active": ([_vp, ctypes.c_uint32, ctypes.c_uint32], ctypes.c_int),
        "dhtgpu_handles_to_indices_dev": ([_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint32, _vp], ctypes.c_int),
        "dhtgpu_set_search_alpha": ([_vp, ctypes.c_uint32], ctypes.c_int),
        "dhtgpu_get_ids": ([_vp, ctypes.c_uint64, ctypes.c_uint64, _u8p], ctypes.c_int),
        "dhtgpu_ids_dev": ([_vp, ctypes.POINTER(_vp), ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
        "dhtgpu_topk": ([_vp, _u8p, ctypes.c_uint32, ctypes.c_uint32, _u32p, _u32p], ctypes.c_int),
        "dhtgpu_topk_dev": ([_vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, _vp,
                             ctypes.c_uint32, _vp], ctypes.c_int),
        "dhtgpu_merge_dev": ([_vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _vp, ctypes.c_uint64,
                              ctypes.c_uint32, _vp, _vp, _vp, ctypes.c_uint32, _vp], ctypes.c_int),
        "dhtgpu_tie_words_dev": ([_vp, _vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _vp, ctypes.c_uint32,
                                  ctypes.c_uint32, _vp, _vp], ctypes.c_int),
        "dhtgpu_merge_ties_dev": ([_vp, _vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _vp, ctypes.c_uint64,
                                   ctypes.c_uint32, _vp, ctypes.c_uint32, _vp, _vp, _vp], ctypes.c_int),
        "dhtgpu_pack_dev": ([_vp, ctypes.c_uint64, _vp, ctypes.c_uint64, _vp], ctypes.c_int),
        "dhtgpu_gen_dev": ([ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, _vp, ctypes.c_uint64, _vp],
                           ctypes.c_int),
        "dhtgpu_find_closest": ([_vp, ctypes.c_uint32, _u8p, _u32p, _u8p, _u8p, _u8p, ctypes.c_uint32,
                                 ctypes.c_uint32, _u32p, _u32p], ctypes.c_int),
        "dhtgpu_classify": ([_vp, ctypes.c_uint32, _u8p, _u8p, _u8p, _u64p], ctypes.c_int),
        "dhtgpu_classify_dev": ([_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, _vp, _u32p, _vp, _vp,
                                 _vp], ctypes.c_int),
        "dhtgpu_cached_nodes": ([_vp, _u8p, _u8p, ctypes.c_uint32, ctypes.c_uint32, _u32p, _u32p],
                                ctypes.c_int),
        "dhtgpu_cache_set": ([_vp, _u8p, ctypes.c_uint64, ctypes.c_uint64], ctypes.c_int),
        "dhtgpu_batch_events": ([_vp, ctypes.POINTER(_vp)], ctypes.c_int),
        "dhtgpu_search_insert": ([_vp, _u8p, _u8p, ctypes.c_uint32, _u8p, ctypes.c_uint32, ctypes.c_uint32, _u32p, _u8p,
                                  _u32p, _u8p, _u64p, _u32p, _u8p, _u8p], ctypes.c_int),
        "dhtgpu_table_stats": ([_vp, ctypes.c_uint32, _u8p, ctypes.POINTER(ctypes.c_int32), _u32p], ctypes.c_int),
        "dhtgpu_cache_nodes": ([_vp, _u8p, _u8p, ctypes.c_uint32, ctypes.c_uint32, _u32p, _u32p], ctypes.c_int),
        "dhtgpu_cache_sorted": ([_vp, _u32p], ctypes.c_int),
        "dhtgpu_buffer_nodes_ids": ([_vp, _u8p, _u8p, ctypes.c_uint32, ctypes.c_uint32, _u8p, ctypes.c_uint32, _u32p,
                                     ctypes.c_uint32, _u8p, _u32p], ctypes.c_int),
        "dhtgpu_index_build": ([_vp, _vp], ctypes.c_int),
        "dhtgpu_index_topk_dev": ([_vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, _vp,
                                   ctypes.c_uint32, _vp], ctypes.c_int),
        "dhtgpu_index_topk": ([_vp, _u8p, ctypes.c_uint32, ctypes.c_uint32, _u32p, _u32p], ctypes.c_int),
        "dhtgpu_index_build_timed": ([_vp, _vp, ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
        "dhtgpu_gen_ids_prefix": ([_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                   ctypes.c_uint32], ctypes.c_int),
        "dhtgpu_select_prefix_dev": ([_vp, _vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                      _vp, ctypes.c_uint64, _vp, _u64p, _vp], ctypes.c_int),
        "dhtgpu_batch_topk_dev": ([_vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, _vp,
                                   ctypes.c_uint32, _vp], ctypes.c_int),
        "dhtgpu_batch_topk_timed": ([_vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, _vp,
                                     ctypes.POINTER(ctypes.c_float), _u32p], ctypes.c_int),
        "dhtgpu_batch_topk": ([_vp, _u8p, ctypes.c_uint32, ctypes.c_uint32, _u32p, _u32p], ctypes.c_int),
        "dhtgpu_table_depth": ([ctypes.c_uint32, _u8p, ctypes.c_uint32, _u32p], ctypes.c_int),
        "dhtgpu_buffer_nodes_dev": ([_vp, _vp, ctypes.c_uint32, _vp, ctypes.c_uint64, ctypes.c_uint32, _vp,
                                     ctypes.c_uint32, _vp, _vp, _vp], ctypes.c_int),
        "dhtgpu_buffer_nodes": ([_vp, _u8p, ctypes.c_uint32, _u8p, ctypes.c_uint32, _u32p, ctypes.c_uint32, _u8p,
                                 _u32p], ctypes.c_int),
        "dhtgpu_deserialize_nodes": ([_vp, ctypes.c_uint32, _u8p, _u8p, _u64p, ctypes.c_uint32, _u8p, _u8p, _u8p,
                                      _u8p, _u8p, _u8p, _u32p], ctypes.c_int),
        "dhtgpu_net_prepare": ([_vp, _u8p, ctypes.c_uint64], ctypes.c_int),
        "dhtgpu_search_batch": ([_vp, _u8p, ctypes.c_uint32, _u32p, ctypes.c_uint32, _u32p, _u8p, _u32p, _u32p,
                                 _u32p], ctypes.c_int),
        "dhtgpu_search_batch_dev": ([_vp, _vp, ctypes.c_uint64, ctypes.c_uint32, _vp, ctypes.c_uint32, _vp, _vp,
                                     _vp, _vp, _vp, _vp], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def exported_symbols():
    """Names of every entry point declared in include/dhtgpu.h (for the ABI test)."""
    return ["dhtgpu_strerror", "dhtgpu_device_count", "dhtgpu_ctx_create", "dhtgpu_ctx_destroy",
            "dhtgpu_ctx_stream", "dhtgpu_set_ids", "dhtgpu_gen_ids", "dhtgpu_num_ids", "dhtgpu_get_ids",
            "dhtgpu_ids_dev", "dhtgpu_topk", "dhtgpu_topk_dev", "dhtgpu_merge_dev", "dhtgpu_tie_words_dev",
            "dhtgpu_merge_ties_dev", "dhtgpu_pack_dev",
            "dhtgpu_gen_dev", "dhtgpu_find_closest", "dhtgpu_classify", "dhtgpu_classify_dev",
            "dhtgpu_cached_nodes", "dhtgpu_index_build", "dhtgpu_index_topk_dev", "dhtgpu_index_topk",
            "dhtgpu_index_build_timed", "dhtgpu_gen_ids_prefix", "dhtgpu_select_prefix_dev",
            "dhtgpu_batch_topk_dev", "dhtgpu_batch_topk_timed", "dhtgpu_batch_topk", "dhtgpu_table_depth",
            "dhtgpu_buffer_nodes_dev", "dhtgpu_buffer_nodes", "dhtgpu_deserialize_nodes", "dhtgpu_net_prepare",
            "dhtgpu_search_batch", "dhtgpu_search_batch_dev", "dhtgpu_set_global_indices", "dhtgpu_set_sub_handles",
            "dhtgpu_sub_handles_active", "dhtgpu_handles_to_indices_dev", "dhtgpu_set_search_alpha", "dhtgpu_cache_set",
            "dhtgpu_cache_nodes", "dhtgpu_cache_sorted", "dhtgpu_buffer_nodes_ids", "dhtgpu_batch_events",
            "dhtgpu_search_insert", "dhtgpu_table_stats"]


def _ids(a, name="ids"):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    if a.ndim == 1:
        a = a.reshape(-1, 20)
    if a.ndim != 2 or a.shape[1] != 20:
        raise ValueError(f"{name}: expected (n, 20) uint8 big-endian InfoHash bytes, got {a.shape}")
    return a


def _p(a, t):
    return a.ctypes.data_as(t)


def id_words(ids):
    """(n,20) big-endian bytes -> (5, n) uint32 word planes (the device layout)."""
    ids = _ids(ids)
    return ids.view(">u4").reshape(-1, 5).astype(np.uint32).T.copy()


class Context:
    """One device context (mirrors the reference's single dht_thread ownership:
    not thread-safe, calls are synchronous)."""

    def __init__(self, device=0):
        L = lib()
        h = _vp()
        _check(L.dhtgpu_ctx_create(int(device), ctypes.byref(h)), "ctx_create")
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            lib().dhtgpu_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def stream(self):
        return lib().dhtgpu_ctx_stream(self._h)

    # ---- id set -------------------------------------------------------------
    def set_ids(self, ids):
        ids = _ids(ids)
        _check(lib().dhtgpu_set_ids(self._h, _p(ids, _u8p), ids.shape[0]), "set_ids")

    def gen_ids(self, seed, n, start=0):
        _check(lib().dhtgpu_gen_ids(self._h, seed, start, n), "gen_ids")

    def gen_ids_prefix(self, seed, n, pbits, pval, start=0):
        """Keep the ids of the stream [start, start+n) whose top pbits bits == pval
        (a prefix shard); result indices refer to the global stream."""
        _check(lib().dhtgpu_gen_ids_prefix(self._h, seed, start, n, pbits, pval), "gen_ids_prefix")

    def set_global_indices(self, on):
        """Prefix shards: results as global stream indices (True, default) or shard-local."""
        _check(lib().dhtgpu_set_global_indices(self._h, int(bool(on))), "set_global_indices")

    def set_sub_handles(self, on):
        """Sub-partitioned calls (sets one K6 plan cannot serve) return sub-partition handles
        instead of indices (no per-result index-map read); see include/dhtgpu.h."""
        _check(lib().dhtgpu_set_sub_handles(self._h, int(bool(on))), "set_sub_handles")

    def sub_handles_active(self, q, k):
        """True when a call of q targets at k returns handles."""
        return bool(lib().dhtgpu_sub_handles_active(self._h, q, k))

    def handles_to_indices_dev(self, handles_ptr, m, out_ptr, idx_base=0, stream=None):
        """m handles -> the indices the call would have returned (device pointers)."""
        _check(lib().dhtgpu_handles_to_indices_dev(self._h, handles_ptr, m, out_ptr, idx_base, stream),
               "handles_to_indices_dev")

    def select_prefix_dev(self, planes_ptr, stride, n, pbits, pval, out_planes_ptr, out_stride, out_gidx_ptr=None,
                          stream=None):
        cnt = ctypes.c_uint64()
        _check(lib().dhtgpu_select_prefix_dev(self._h, planes_ptr, stride, n, pbits, pval, out_planes_ptr, out_stride,
                                              out_gidx_ptr, ctypes.byref(cnt), stream), "select_prefix_dev")
        return cnt.value

    @property
    def num_ids(self):
        return int(lib().dhtgpu_num_ids(self._h))

    def get_ids(self, first=0, n=None):
        if n is None:
            n = self.num_ids - first
        out = np.empty((n, 20), dtype=np.uint8)
        _check(lib().dhtgpu_get_ids(self._h, first, n, _p(out, _u8p)), "get_ids")
        return out

    def ids_dev(self):
        p, s = _vp(), ctypes.c_uint64()
        _check(lib().dhtgpu_ids_dev(self._h, ctypes.byref(p), ctypes.byref(s)), "ids_dev")
        return p.value, s.value

    # ---- K1: flat exact top-k ---------------------------------------------------
    def topk(self, targets, k=8):
        """findClosestNodesBatch(targets[], k): (q,k) uint32 indices (NONE padded), (q,) counts."""
        t = _ids(targets, "targets")
        q = t.shape[0]
        out = np.empty((q, k), dtype=np.uint32)
        cnt = np.empty(q, dtype=np.uint32)
        _check(lib().dhtgpu_topk(self._h, _p(t, _u8p), q, k, _p(out, _u32p), _p(cnt, _u32p)), "topk")
        return out, cnt

    def index_topk(self, targets, k=8):
        """Same result as topk() through the K4/K5 bucket index (built on first use)."""
        t = _ids(targets, "targets")
        q = t.shape[0]
        out = np.empty((q, k), dtype=np.uint32)
        cnt = np.empty(q, dtype=np.uint32)
        _check(lib().dhtgpu_index_topk(self._h, _p(t, _u8p), q, k, _p(out, _u32p), _p(cnt, _u32p)), "index_topk")
        return out, cnt

    def index_build(self, stream=None):
        _check(lib().dhtgpu_index_build(self._h, stream), "index_build")

    def index_build_timed(self, stream=None):
        """Build with HIP events between kernels; returns device ms per phase:
        (P0 histogram, P0 scans, P1 partition scatter, P2 bucket gather)."""
        ms = (ctypes.c_float * 4)()
        _check(lib().dhtgpu_index_build_timed(self._h, stream, ms), "index_build_timed")
        return tuple(ms)

    def index_topk_dev(self, t_planes_ptr, t_stride, q, k, out_idx_ptr=None, out_cnt_ptr=None, out_rec_ptr=None,
                       idx_base=0, stream=None):
        _check(lib().dhtgpu_index_topk_dev(self._h, t_planes_ptr, t_stride, q, k, out_idx_ptr, out_cnt_ptr,
                                           out_rec_ptr, idx_base, stream), "index_topk_dev")

    def batch_topk(self, targets, k=8):
        """Same result as topk() through the K6 per-batch target-prefix filter."""
        t = _ids(targets, "targets")
        q = t.shape[0]
        out = np.empty((q, k), dtype=np.uint32)
        cnt = np.empty(q, dtype=np.uint32)
        _check(lib().dhtgpu_batch_topk(self._h, _p(t, _u8p), q, k, _p(out, _u32p), _p(cnt, _u32p)), "batch_topk")
        return out, cnt

    def batch_topk_dev(self, t_planes_ptr, t_stride, q, k, out_idx_ptr=None, out_cnt_ptr=None, out_rec_ptr=None,
                       idx_base=0, stream=None):
        _check(lib().dhtgpu_batch_topk_dev(self._h, t_planes_ptr, t_stride, q, k, out_idx_ptr, out_cnt_ptr,
                                           out_rec_ptr, idx_base, stream), "batch_topk_dev")

    def batch_topk_timed(self, t_planes_ptr, t_stride, q, k, out_idx_ptr, out_cnt_ptr, stream=None):
        """One K6 call with HIP events between its kernels; returns (device ms per phase
        (F1 mark targets, F2 filter ids, F3 answer, F4 fallback), fallback targets, survivors,
        targets answered by F3's exact wave path)."""
        ms = (ctypes.c_float * 4)()
        st = (ctypes.c_uint32 * 4)()
        _check(lib().dhtgpu_batch_topk_timed(self._h, t_planes_ptr, t_stride, q, k, out_idx_ptr, out_cnt_ptr,
                                             stream, ms, st), "batch_topk_timed")
        return tuple(ms), int(st[0]), int(st[1]), int(st[2])

    def batch_events(self, events):
        """Arm per-kernel timing of the next K6 call: `events` = 8 torch.cuda.Event(enable_timing=True)
        (F1..F4 start/stop, recorded by the kernels' own dispatches; no synchronisation)."""
        arr = (_vp * 8)(*[e.cuda_event for e in events])
        _check(lib().dhtgpu_batch_events(self._h, arr), "batch_events")

    def tie_words_dev(self, rec_ptr, q, k, idx_base, ties_ptr, tie_cap, row_base, out_words_ptr, stream=None):
        """Words 2..4 of this context's candidates (its own q x k compact records) in the rows a merge
        listed as 64-bit ties (ties_ptr None: every row) -- the second exchange's payload."""
        _check(lib().dhtgpu_tie_words_dev(self._h, rec_ptr, q, k, idx_base, ties_ptr, tie_cap, row_base,
                                          out_words_ptr, stream), "tie_words_dev")

    def topk_dev(self, t_planes_ptr, t_stride, q, k, out_idx_ptr=None, out_cnt_ptr=None, out_rec_ptr=None,
                 idx_base=0, stream=None):
        _check(lib().dhtgpu_topk_dev(self._h, t_planes_ptr, t_stride, q, k, out_idx_ptr, out_cnt_ptr,
                                     out_rec_ptr, idx_base, stream), "topk_dev")

    # ---- K1r: RoutingTable::findClosestNodes -------------------------------------
    def find_closest(self, firsts, bucket_off, node_ids, good, targets, count=8):
        firsts = _ids(firsts, "firsts") if len(firsts) else np.zeros((0, 20), np.uint8)
        off = np.ascontiguousarray(bucket_off, dtype=np.uint32)
        nodes = _ids(node_ids, "node_ids") if len(node_ids) else np.zeros((1, 20), np.uint8)
        good = np.ascontiguousarray(good, dtype=np.uint8) if len(good) else np.zeros(1, np.uint8)
        t = _ids(targets, "targets")
        q = t.shape[0]
        out = np.empty((q, count), dtype=np.uint32)
        cnt = np.empty(q, dtype=np.uint32)
        _check(lib().dhtgpu_find_closest(self._h, firsts.shape[0], _p(firsts, _u8p), _p(off, _u32p),
                                         _p(nodes, _u8p), _p(good, _u8p), _p(t, _u8p), q, count,
                                         _p(out, _u32p), _p(cnt, _u32p)), "find_closest")
        return out, cnt

    # ---- a11 / f4: compact node wire format ---------------------------------------
    def buffer_nodes(self, node_tail, af, targets, cand):
        """NetworkEngine::bufferNodes, batched: (q, 8*rec) uint8 blobs and (q,) byte lengths."""
        t = _ids(targets, "targets")
        q = t.shape[0]
        cand = np.ascontiguousarray(cand, dtype=np.uint32).reshape(q, -1)
        alen = 4 if af == 4 else 16
        tail = np.ascontiguousarray(node_tail, dtype=np.uint8).reshape(-1, alen + 2)
        rec = 20 + alen + 2
        out = np.zeros((q, 8 * rec), dtype=np.uint8)
        ln = np.zeros(q, dtype=np.uint32)
        _check(lib().dhtgpu_buffer_nodes(self._h, _p(tail, _u8p), af, _p(t, _u8p), q, _p(cand, _u32p),
                                         cand.shape[1], _p(out, _u8p), _p(ln, _u32p)), "buffer_nodes")
        return out, ln

    def deserialize_nodes(self, af, myid, blobs, from_af, from_addr):
        """NetworkEngine::deserializeNodes over a list of received blobs: returns
        (ids (r,20), tails (r, alen+2), status (r,), msg_status (m,))."""
        alen = 4 if af == 4 else 16
        m = len(blobs)
        off = np.zeros(m + 1, dtype=np.uint64)
        for i, b in enumerate(blobs):
            off[i + 1] = off[i] + len(b)
        blob = np.frombuffer(b"".join(bytes(b) for b in blobs) or b"\0", dtype=np.uint8).copy()
        fa = np.ascontiguousarray(from_af, dtype=np.uint8).reshape(m) if m else np.zeros(1, np.uint8)
        fad = np.ascontiguousarray(from_addr, dtype=np.uint8).reshape(m, 16) if m else np.zeros((1, 16), np.uint8)
        cap = max(1, int(off[-1]) // (20 + alen + 2))
        ids = np.zeros((cap, 20), np.uint8)
        tail = np.zeros((cap, alen + 2), np.uint8)
        st = np.zeros(cap, np.uint8)
        ms = np.zeros(max(m, 1), np.uint8)
        nrec = ctypes.c_uint32()
        my = np.ascontiguousarray(myid, dtype=np.uint8).reshape(20)
        _check(lib().dhtgpu_deserialize_nodes(self._h, af, _p(my, _u8p), _p(blob, _u8p), _p(off, _u64p), m,
                                              _p(fa, _u8p), _p(fad, _u8p), _p(ids, _u8p), _p(tail, _u8p),
                                              _p(st, _u8p), _p(ms, _u8p), ctypes.byref(nrec)), "deserialize_nodes")
        r = nrec.value
        return ids[:r], tail[:r], st[:r], ms[:m]

    # ---- f3: crawl replay ------------------------------------------------------------
    def net_prepare(self, dead=None, table_seed=0x5EED):
        """Turn the uploaded id set into the crawl-model network (dead: (n,) bool/uint8)."""
        d = None
        if dead is not None:
            d = np.ascontiguousarray(dead, dtype=np.uint8)
            if d.shape[0] != self.num_ids:
                raise ValueError("dead mask must have one byte per id")
        _check(lib().dhtgpu_net_prepare(self._h, _p(d, _u8p) if d is not None else None, table_seed), "net_prepare")

    def set_search_alpha(self, alpha):
        """Requests per search round for later search_batch calls (default 4 =
        MAX_REQUESTED_SEARCH_NODES, include/opendht/dht.h:321)."""
        _check(lib().dhtgpu_set_search_alpha(self._h, int(alpha)), "set_search_alpha")
        self._alpha = int(alpha)

    def search_batch(self, targets, searchers, max_rounds=64, alpha=None):
        """Iterative searches: (idx (q,64), flags (q,64), len (q,), rounds (q,), queries (q,)).
        alpha (optional): requests per round for THIS call only (the context's setting,
        set_search_alpha, default 4 = MAX_REQUESTED_SEARCH_NODES, is restored afterwards)."""
        t = _ids(targets, "targets")
        q = t.shape[0]
        sr = np.ascontiguousarray(searchers, dtype=np.uint32).reshape(q)
        idx = np.empty((q, 64), np.uint32)
        fl = np.empty((q, 64), np.uint8)
        ln, rd, qs = (np.empty(q, np.uint32) for _ in range(3))
        saved = getattr(self, "_alpha", 4)
        if alpha is not None:
            _check(lib().dhtgpu_set_search_alpha(self._h, int(alpha)), "set_search_alpha")
        try:
            _check(lib().dhtgpu_search_batch(self._h, _p(t, _u8p), q, _p(sr, _u32p), max_rounds, _p(idx, _u32p),
                                             _p(fl, _u8p), _p(ln, _u32p), _p(rd, _u32p), _p(qs, _u32p)),
                   "search_batch")
        finally:
            if alpha is not None:
                _check(lib().dhtgpu_set_search_alpha(self._h, int(saved)), "set_search_alpha")
        return idx, fl, ln, rd, qs

    # ---- K2: classification -------------------------------------------------------
    def classify(self, firsts, myid, buckets=True):
        firsts = _ids(firsts, "firsts")
        myid = np.ascontiguousarray(myid, dtype=np.uint8).reshape(20)
        hist = np.zeros(161, dtype=np.uint64)
        out = np.empty(max(self.num_ids, 1), dtype=np.uint8) if buckets else None
        _check(lib().dhtgpu_classify(self._h, firsts.shape[0], _p(firsts, _u8p), _p(myid, _u8p),
                                     _p(out, _u8p) if buckets else None, _p(hist, _u64p)), "classify")
        return (out[: self.num_ids] if buckets else None), hist

    # ---- a8: NodeCache::getCachedNodes ------------------------------------------------
    def cached_nodes(self, targets, count=14, accept=None):
        t = _ids(targets, "targets")
        q = t.shape[0]
        out = np.empty((q, count), dtype=np.uint32)
        cnt = np.empty(q, dtype=np.uint32)
        acc = None
        if accept is not None:
            acc = np.ascontiguousarray(accept, dtype=np.uint8)
            if acc.shape[0] != self.num_ids:
                raise ValueError("accept mask must have one byte per id")
        _check(lib().dhtgpu_cached_nodes(self._h, _p(acc, _u8p) if acc is not None else None, _p(t, _u8p), q,
                                         count, _p(out, _u32p), _p(cnt, _u32p)), "cached_nodes")
        return out, cnt


    # ---- f2: the NodeCache mirror (a second id set, sorted on the device) ----------------
    def cache_set(self, ids, version=0):
        """Upload NodeCache map keys in any order (unique); version != 0 equal to the last
        upload's skips the upload."""
        ids = _ids(ids)
        _check(lib().dhtgpu_cache_set(self._h, _p(ids, _u8p), ids.shape[0], int(version)), "cache_set")
        self._cache_n = ids.shape[0]

    def cache_nodes(self, targets, count=14, accept=None):
        """getCachedNodes over the mirror: (q, count) caller-order indices (NONE padded), (q,) counts."""
        t = _ids(targets, "targets")
        q = t.shape[0]
        out = np.empty((q, count), dtype=np.uint32)
        cnt = np.empty(q, dtype=np.uint32)
        acc = None
        if accept is not None:
            acc = np.ascontiguousarray(accept, dtype=np.uint8)
            if acc.shape[0] != getattr(self, "_cache_n", acc.shape[0]):
                raise ValueError("accept mask must have one byte per cache key")
        _check(lib().dhtgpu_cache_nodes(self._h, _p(acc, _u8p) if acc is not None else None, _p(t, _u8p), q, count,
                                        _p(out, _u32p), _p(cnt, _u32p)), "cache_nodes")
        return out, cnt

    def cache_sorted(self):
        """The mirror's lexicographic order as caller indices."""
        perm = np.empty(max(getattr(self, "_cache_n", 0), 1), dtype=np.uint32)
        _check(lib().dhtgpu_cache_sorted(self._h, _p(perm, _u32p)), "cache_sorted")
        return perm[: getattr(self, "_cache_n", 0)]

    def buffer_nodes_ids(self, node_ids, node_tail, af, targets, cand):
        """bufferNodes over the caller's own nodes (the context's id set is not used)."""
        t = _ids(targets, "targets")
        q = t.shape[0]
        nodes = _ids(node_ids, "node_ids")
        cand = np.ascontiguousarray(cand, dtype=np.uint32).reshape(q, -1)
        alen = 4 if af == 4 else 16
        tail = np.ascontiguousarray(node_tail, dtype=np.uint8).reshape(-1, alen + 2)
        rec = 20 + alen + 2
        out = np.zeros((q, 8 * rec), dtype=np.uint8)
        ln = np.zeros(q, dtype=np.uint32)
        _check(lib().dhtgpu_buffer_nodes_ids(self._h, _p(nodes, _u8p), _p(tail, _u8p), nodes.shape[0], af,
                                             _p(t, _u8p), q, _p(cand, _u32p), cand.shape[1], _p(out, _u8p),
                                             _p(ln, _u32p)), "buffer_nodes_ids")
        return out, ln


    # ---- a10: Search::insertNode, batched -----------------------------------------------------
    def search_insert(self, node_ids, node_state, targets, lists, flags, lens, expired, ins_off, ins_node,
                      ins_token):
        """Apply insertions (CSR ins_off over searches) to the search lists in place-copies:
        returns (lists, flags, lens, expired, added)."""
        nodes = _ids(node_ids, "node_ids")
        st = np.ascontiguousarray(node_state, dtype=np.uint8)
        t = _ids(targets, "targets")
        q = t.shape[0]
        lists = np.ascontiguousarray(lists, dtype=np.uint32).copy()
        cap = lists.shape[1]
        flags = np.ascontiguousarray(flags, dtype=np.uint8).copy()
        lens = np.ascontiguousarray(lens, dtype=np.uint32).copy()
        expired = np.ascontiguousarray(expired, dtype=np.uint8).copy()
        off = np.ascontiguousarray(ins_off, dtype=np.uint64)
        node = np.ascontiguousarray(ins_node, dtype=np.uint32)
        tok = np.ascontiguousarray(ins_token, dtype=np.uint8)
        added = np.zeros(max(node.size, 1), np.uint8)
        _check(lib().dhtgpu_search_insert(self._h, _p(nodes, _u8p), _p(st, _u8p), nodes.shape[0], _p(t, _u8p), q, cap,
                                          _p(lists, _u32p), _p(flags, _u8p), _p(lens, _u32p), _p(expired, _u8p),
                                          _p(off, _u64p), _p(node, _u32p) if node.size else None,
                                          _p(tok, _u8p) if tok.size else None, _p(added, _u8p)), "search_insert")
        return lists, flags, lens, expired, added[: node.size]

    def table_stats(self, firsts):
        """(lowbit, depth) of every bucket of a table snapshot, computed on the device."""
        f = _ids(firsts, "firsts")
        nb = f.shape[0]
        lb = np.zeros(max(nb, 1), np.int32)
        dp = np.zeros(max(nb, 1), np.uint32)
        _check(lib().dhtgpu_table_stats(self._h, nb, _p(f, _u8p), lb.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                        _p(dp, _u32p)), "table_stats")
        return lb[:nb], dp[:nb]


def table_depth(firsts, b):
    """RoutingTable::depth of bucket b of a table snapshot (src/routing_table.cpp:100-107)."""
    f = _ids(firsts, "firsts") if len(firsts) else np.zeros((0, 20), np.uint8)
    d = ctypes.c_uint32()
    _check(lib().dhtgpu_table_depth(f.shape[0], _p(f, _u8p), b, ctypes.byref(d)), "table_depth")
    return d.value


def device_count():
    n = ctypes.c_int()
    _check(lib().dhtgpu_device_count(ctypes.byref(n)), "device_count")
    return n.value
