"""Multi-rank sharded lookup on CPU (gloo, world_size 2 and 3): id-range shards, per-rank
candidate records {w0..w4, global idx}, all-gather, merge.  The per-rank scan and the
merge are stood in by the oracle (test infrastructure) -- what is under test here is the
sharding and exchange logic of opendht_amd.sharding that bench.py runs over RCCL."""
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


def records_from(ids_shard, lo, idx, cnt):
    """(q, k, 6) int32 records {w0..w4, global idx} like K1's record mode."""
    q, k = idx.shape
    rec = np.full((q, k, 6), 0xFFFFFFFF, dtype=np.uint32)
    words = ids_shard.view(">u4").reshape(-1, 5).astype(np.uint32)
    for i in range(q):
        for r in range(cnt[i]):
            rec[i, r, :5] = words[idx[i, r]]
            rec[i, r, 5] = idx[i, r] + lo
    return torch.from_numpy(rec.view(np.int32))


def merge_records(gathered, targets, k):
    """Reference merge: order all candidates by (xor distance words, global idx)."""
    g = gathered.numpy().view(np.uint32)
    tw = targets.view(">u4").reshape(-1, 5).astype(np.uint32)
    world, q, kin, _ = g.shape
    out = np.full((q, k), 0xFFFFFFFF, dtype=np.uint32)
    cnt = np.zeros(q, dtype=np.uint32)
    for i in range(q):
        c = g[:, i].reshape(-1, 6)
        c = c[c[:, 5] != 0xFFFFFFFF]
        keys = [tuple(int(x) for x in (c[j, :5] ^ tw[i])) + (int(c[j, 5]),) for j in range(c.shape[0])]
        order = sorted(range(len(keys)), key=lambda j: keys[j])[:k]
        out[i, :len(order)] = c[order, 5]
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
