"""Multi-rank sharded lookup on CPU (gloo, world_size 2 and 3): id-range shards, per-rank
compact candidate records {w0, w1, global idx}, all-gather or all-to-all, merge, and the tie
exchange of words 2..4 for rows whose candidates share 64 bits.  The per-rank scan and the device
steps are stood in by the oracle and host code (test infrastructure) -- what is under test here is
the sharding and exchange logic of opendht_amd.sharding that bench.py runs over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from opendht_amd import sharding


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_partitions():
    for n in (0, 1, 7, 100, 12345):
        for w in (1, 2, 3, 8):
            parts = [sharding.shard_range(n, w, r) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in parts) - min(b - a for a, b in parts) <= 1


NONE = 0xFFFFFFFF


def records_from(ids_shard, lo, idx, cnt):
    """(q, k, 3) int32 compact records {w0, w1, global idx} like the library's record form."""
    q, k = idx.shape
    rec = np.full((q, k, 3), NONE, dtype=np.uint32)
    words = ids_shard.view(">u4").reshape(-1, 5).astype(np.uint32)
    for i in range(q):
        c = int(cnt[i])
        rec[i, :c, :2] = words[idx[i, :c], :2]
        rec[i, :c, 2] = idx[i, :c] + lo
    return torch.from_numpy(rec.view(np.int32))


class HostOps:
    """Host stand-ins for the protocol's three device steps (sharding.LibOps): the heads merge of
    K3 on (w0, w1, idx) listing rows where two lists' heads agree on 64 bits, this rank's words
    2..4 from its OWN shard only, and the full-key heads merge of the listed rows.  What is under
    test is the exchange logic of opendht_amd.sharding around them (gloo)."""

    def __init__(self, ids_shard, lo, targets):
        self.words = ids_shard.view(">u4").reshape(-1, 5).astype(np.uint32)
        self.lo = lo
        self.tw = targets.view(">u4").reshape(-1, 5).astype(np.uint32)

    def _heads(self, g, rows, t0, k, key):
        """k-way merge of the lists' heads per row; key(j, i, r) -> tuple or None"""
        world, _, kin = g.shape[0], g.shape[1], g.shape[2]
        outs, ties = {}, set()
        for i in rows:
            p = [0] * world
            res = []
            while len(res) < k:
                heads = [(key(j, i, p[j]), j) for j in range(world) if p[j] < kin and key(j, i, p[j]) is not None]
                if not heads:
                    break
                m = min(heads)[0]
                if sum(1 for h, _ in heads if h[:2] == m[:2]) > 1:
                    ties.add(i)
                res.append(m[-1])
                for h, j in heads:
                    if h == m:
                        p[j] += 1
            outs[i] = res
        return outs, ties

    def merge(self, g, t0, k, out_idx, out_cnt, ties, stream):
        gn = g.numpy().view(np.uint32)

        def key(j, i, r):
            c = gn[j, i, r]
            if c[2] == NONE:
                return None
            return (int(c[0] ^ self.tw[t0 + i, 0]), int(c[1] ^ self.tw[t0 + i, 1]), int(c[2]))
        outs, tied = self._heads(gn, range(gn.shape[1]), t0, k, key)
        self._write(outs, out_idx, out_cnt, k)
        if ties is not None:
            ties.zero_()
            tl = sorted(tied)
            ties[0] = len(tl)
            for s_, i in enumerate(tl[:sharding.TIE_CAP]):
                ties[1 + s_] = i

    def tie_words(self, rec, idx_base, ties, row_base, out, stream):
        rn = rec.numpy().view(np.uint32)
        q, k = rn.shape[0], rn.shape[1]
        rows = range(q) if ties is None else [int(ties[1 + s_]) + row_base
                                               for s_ in range(min(int(ties[0]), sharding.TIE_CAP))]
        on = out.numpy().view(np.uint32)
        for s_, i in enumerate(rows):
            for r in range(k):
                gi = rn[i, r, 2]
                on[s_, r] = NONE if gi == NONE else self.words[gi - idx_base, 2:5]

    def merge_ties(self, g, words, t0, k, ties, out_idx, out_cnt, stream):
        gn = g.numpy().view(np.uint32)
        wn = words.numpy().view(np.uint32).reshape(gn.shape[0], -1, gn.shape[2], 3)
        if ties is None:
            rows, slot = list(range(gn.shape[1])), {i: i for i in range(gn.shape[1])}
        else:
            rows = [int(ties[1 + s_]) for s_ in range(min(int(ties[0]), sharding.TIE_CAP))]
            slot = {i: s_ for s_, i in enumerate(rows)}

        def key(j, i, r):
            c = gn[j, i, r]
            if c[2] == NONE:
                return None
            full = np.r_[c[:2], wn[j, slot[i], r]] ^ self.tw[t0 + i]
            return tuple(int(x) for x in full) + (int(c[2]),)
        outs, _ = self._heads(gn, rows, t0, k, key)
        self._write(outs, out_idx, out_cnt, k)

    @staticmethod
    def _write(outs, out_idx, out_cnt, k):
        for i, res in outs.items():
            row = np.full(k, NONE, np.uint32)
            row[:len(res)] = res
            out_idx[i] = torch.from_numpy(row.view(np.int32))
            out_cnt[i] = len(res)


def _crafted(n, q, seed):
    """ids and targets where a quarter of the ids share their first 64 bits (cross-shard tie rows)"""
    import oracle as O
    ids = O.gen_ids(seed, n)
    tg = O.gen_ids(seed + 1, q)
    ids[::4, :8] = ids[1, :8]
    tg[::2, :8] = ids[1, :8]
    return ids, tg


def _worker_proto(rank, world, port, n, q, k, exchange, cap, ret, settle=True):
    """The whole protocol (records -> exchange -> K3 -> tie exchange -> overflow settlement) with
    host stand-ins for the device steps."""
    import oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sharding.TIE_CAP = cap
    ids, tg = _crafted(n, q, 31)
    lo, hi = sharding.shard_range(n, world, rank)
    idx, cnt = O.topk(ids[lo:hi], tg, k, threads=2)
    rec = records_from(ids[lo:hi], lo, idx, cnt)
    ops = HostOps(ids[lo:hi], lo, tg)
    tx = sharding.TieExchange(world, k, "cpu")
    if exchange == "allgather":
        tlo, thi = 0, q
        g = sharding.gather_records(rec)
        oi, oc = torch.empty((q, k), dtype=torch.int32), torch.empty(q, dtype=torch.int32)
        sharding.merge_allgather(ops, rec, g, k, oi, oc, tx, lo)
        flagged = bool(sharding.unsettled(tx))
        nt = sharding.settle_overflow_allgather(ops, rec, g, k, oi, oc, tx, lo) if settle else int(tx.ties[0])
    else:
        tlo, thi = sharding.shard_range(q, world, rank)
        ex = sharding.exchange_records(rec)
        oi, oc = torch.empty((max(thi - tlo, 1), k), dtype=torch.int32), torch.empty(max(thi - tlo, 1), dtype=torch.int32)
        sharding.merge_alltoall(ops, rec, ex, k, tlo, oi, oc, tx, lo)
        flagged = bool(sharding.unsettled(tx))
        nt = sharding.settle_overflow_alltoall(ops, rec, ex, k, tlo, oi, oc, tx, lo) if settle else int(tx.ties[0])
    want, wcnt = O.topk(ids, tg[tlo:thi], k, threads=2)
    got = oi.numpy().view(np.uint32)[:thi - tlo]
    ret[rank] = (bool(np.array_equal(got, want) and np.array_equal(oc.numpy()[:thi - tlo].astype(np.uint32), wcnt)),
                 nt, flagged)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,exchange,cap", [(2, "allgather", 256), (3, "allgather", 3), (2, "alltoall", 256),
                                                (3, "alltoall", 2)])
def test_tie_protocol_gloo(world, exchange, cap):
    """Compact records whose ids share 64 bits across shards: K3 lists the rows, the second exchange
    brings words 2..4 from the owning ranks (all-gather: every rank lists the same rows; all-to-all:
    each owner's own rows, tie lists all-gathered), cap 2 / 3: more rows than one exchange takes,
    so the every-row settlement runs too; every rank's results == one flat top-k."""
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker_proto, args=(world, _free_port(), 1500, 60, 8, exchange, cap, ret), nprocs=world, join=True)
    assert all(ret[r][0] for r in range(world)), dict(ret)
    assert max(ret[r][1] for r in range(world)) > 0
    # the overflow flag is raised exactly where more rows tied than one exchange settles
    assert all(ret[r][2] == (ret[r][1] > cap) for r in range(world)), dict(ret)


def test_tie_overflow_flagged_when_not_settled():
    """More than TIE_CAP rows tie (cap 2) and the caller skips settle_overflow_*: the rows past the
    cap are provisional, and unsettled(tx) says so on every rank that holds them -- a
    pipelined caller reads the flag instead of silently taking inexact rows.  Rows of a rank whose
    flag is down are exact."""
    world = 2
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker_proto, args=(world, _free_port(), 1500, 60, 8, "allgather", 2, ret, False), nprocs=world,
             join=True)
    for r in range(world):
        exact, count, flagged = ret[r]
        assert flagged == (count > 2), dict(ret)
        assert flagged or exact, dict(ret)
    assert any(ret[r][2] for r in range(world)), dict(ret)


def merge_records(gathered, targets, k):
    """Reference merge: order all candidates by (first 64 bits of the xor distance, global idx);
    exact for these hash ids (no two candidates share 64 bits)."""
    g = gathered.numpy().view(np.uint32)
    tw = targets.view(">u4").reshape(-1, 5).astype(np.uint32)
    world, q, kin, _ = g.shape
    out = np.full((q, k), NONE, dtype=np.uint32)
    cnt = np.zeros(q, dtype=np.uint32)
    for i in range(q):
        c = g[:, i].reshape(-1, 3)
        c = c[c[:, 2] != NONE]
        keys = [tuple(int(x) for x in (c[j, :2] ^ tw[i, :2])) + (int(c[j, 2]),) for j in range(c.shape[0])]
        order = sorted(range(len(keys)), key=lambda j: keys[j])[:k]
        out[i, :len(order)] = c[order, 2]
        cnt[i] = len(order)
    return out, cnt


def _worker_a2a(rank, world, port, n, q, k, ret):
    """The all-to-all route: each rank merges only the targets it owns."""
    import oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ids = O.gen_ids(7, n)
    tg = O.gen_ids(8, q)
    lo, hi = sharding.shard_range(n, world, rank)
    idx, cnt = O.topk(ids[lo:hi], tg, k, threads=2)
    got = sharding.exchange_records(records_from(ids[lo:hi], lo, idx, cnt))
    tlo, thi = sharding.shard_range(q, world, rank)
    assert got.shape[:2] == (world, thi - tlo)
    out, ocnt = merge_records(got, tg[tlo:thi], k)
    want, wcnt = O.topk(ids, tg[tlo:thi], k, threads=2)
    ret[rank] = bool(np.array_equal(out, want) and np.array_equal(ocnt, wcnt))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,q", [(2, 3001, 41), (3, 500, 40), (3, 20, 2)])
def test_exchange_records_gloo(world, n, q):
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker_a2a, args=(world, _free_port(), n, q, 8, ret), nprocs=world, join=True)
    assert all(ret[r] for r in range(world)), dict(ret)


def _worker(rank, world, port, n, q, k, ret):
    import oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ids = O.gen_ids(5, n)
    tg = O.gen_ids(6, q)
    lo, hi = sharding.shard_range(n, world, rank)

    def local():
        idx, cnt = O.topk(ids[lo:hi], tg, k, threads=2)
        return records_from(ids[lo:hi], lo, idx, cnt)

    out, cnt = sharding.sharded_topk(local, lambda g: merge_records(g, tg, k))
    want, wcnt = O.topk(ids, tg, k, threads=2)
    ret[rank] = bool(np.array_equal(out, want) and np.array_equal(cnt, wcnt))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 3001), (3, 20), (2, 5)])
def test_sharded_topk_gloo(world, n):
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), n, 40, 8, ret), nprocs=world, join=True)
    assert all(ret[r] for r in range(world)), dict(ret)
