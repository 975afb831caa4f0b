"""Test helpers for the compact-record merge (K3 + the tie exchange) on one device: the protocol
opendht_amd.sharding runs over RCCL, with the lists' producers in one process.  Test
infrastructure (imported by the -m gpu tests only)."""
import numpy as np

NONE = 0xFFFFFFFF


def host_records(ids, bounds, tg, k, O):
    """(lists, q, k, 3) compact records {w0, w1, global idx} of each id-range shard's exact top-k
    (the oracle's, ascending, NONE-padded like every producer in the library)."""
    q = tg.shape[0]
    words = ids.view(">u4").reshape(-1, 5).astype(np.uint32)
    rec = np.full((len(bounds) - 1, q, k, 3), NONE, dtype=np.uint32)
    for s in range(len(bounds) - 1):
        lo, hi = bounds[s], bounds[s + 1]
        if hi == lo:
            continue
        idx, cnt = O.topk(ids[lo:hi], tg, k)
        for i in range(q):
            c = int(cnt[i])
            g = lo + idx[i, :c].astype(np.int64)
            rec[s, i, :c, :2] = words[g, :2]
            rec[s, i, :c, 2] = g
    return rec


def host_words_fn(ids, rec_host):
    """words_fn for host-made records: words 2..4 of the ids the records name (global index)."""
    words = ids.view(">u4").reshape(-1, 5).astype(np.uint32)

    def fn(j, rows, out):
        r = rec_host[j][rows]                      # (m, k, 3)
        g = r[..., 2]
        w = np.full(g.shape + (3,), NONE, np.uint32)
        ok = g != NONE
        w[ok] = words[g[ok].astype(np.int64), 2:5]
        return w
    return fn


def ctx_words_fn(L, ctxs, rec, bases, k, stream=None):
    """words_fn over live shard contexts: dhtgpu_tie_words_dev on each list's own records, on the
    stream of the merge (torch's current stream when none is given: K3 and the tie words must be
    ordered on one stream -- the contexts' own streams do not wait for it)."""
    import torch

    def fn(j, ties, out, cap):
        q = rec.shape[1]
        s = stream if stream is not None else torch.cuda.current_stream(rec.device).cuda_stream
        ctxs[j].tie_words_dev(rec[j].data_ptr(), q, k, bases[j], ties.data_ptr() if ties is not None else None,
                              cap, 0, out.data_ptr(), s)
    return fn


def merge(L, rec, tp, ts, k, words, tie_cap=256, force_all=False):
    """K3 over rec (lists, q, k_in, 3) device records, then the fixed-size tie exchange (always
    issued when lists > 1, as sharding.merge_allgather does) and, after a sync, the every-row
    settlement when more than tie_cap rows tied.  words: ("ctx", fn(j, ties|None, out, cap)) for
    live contexts or ("host", fn(j, rows, out) -> (m, k, 3) array).  force_all: run the every-row
    settlement whatever the count.  Returns (idx, cnt, tie count)."""
    import torch
    lists, q, kin = rec.shape[0], rec.shape[1], rec.shape[2]
    dev = rec.device
    s = torch.cuda.current_stream(dev).cuda_stream   # K3, the tie words and the settlement: one stream
    out = torch.empty((q, k), dtype=torch.int32, device=dev)
    cnt = torch.empty(q, dtype=torch.int32, device=dev)
    ties = torch.full((1 + tie_cap,), -1, dtype=torch.int32, device=dev)   # merge_dev zeroes the count
    assert L.dhtgpu_merge_dev(rec.data_ptr(), lists, q, kin, tp.data_ptr(), ts, k, out.data_ptr(), cnt.data_ptr(),
                              ties.data_ptr() if lists > 1 else None, tie_cap, s) == 0
    count = 0
    if lists > 1:
        kind, fn = words

        def fill(rows_all):
            m = q if rows_all else tie_cap
            w = torch.full((lists, m, kin, 3), -1, dtype=torch.int32, device=dev)
            for j in range(lists):
                if kind == "ctx":
                    fn(j, None if rows_all else ties, w[j], tie_cap)
                else:
                    torch.cuda.synchronize()
                    c = min(int(ties[0].item()), tie_cap)
                    rows = np.arange(q) if rows_all else ties[1:1 + c].cpu().numpy().astype(np.int64)
                    hw = fn(j, rows, None)
                    if hw.shape[0]:
                        w[j, :hw.shape[0]] = torch.from_numpy(hw.view(np.int32)).to(dev)
            torch.cuda.synchronize()
            return w
        if tie_cap:
            w = fill(False)
            assert L.dhtgpu_merge_ties_dev(rec.data_ptr(), w.data_ptr(), lists, q, kin, tp.data_ptr(), ts, k,
                                           ties.data_ptr(), tie_cap, out.data_ptr(), cnt.data_ptr(), s) == 0
        torch.cuda.synchronize()
        count = int(ties[0].item())
        if count > tie_cap or force_all:
            w = fill(True)
            assert L.dhtgpu_merge_ties_dev(rec.data_ptr(), w.data_ptr(), lists, q, kin, tp.data_ptr(), ts, k, None,
                                           0, out.data_ptr(), cnt.data_ptr(), s) == 0
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32).copy(), cnt.cpu().numpy().view(np.uint32).copy(), count
