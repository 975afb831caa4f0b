"""Multi-GPU sharding of the id set (north-star scheme).

The N ids are split into contiguous ranges, one per rank.  Every rank scans its range
for all targets and emits candidate records {w0..w4, global idx} (24 B, k per target);
the records are exchanged over RCCL (xGMI on MI355X, gloo in CPU tests) and K3 merges
world*k candidates per target into the exact global top-k.  Bit-exactness holds because
the merge uses the same total order (XOR distance, then global index).

Two exchanges: `gather_records` (all-gather: every rank merges every target -- world x the
records arrive at each GPU) and `exchange_records` (all-to-all by target slice: rank r
receives only the records of the targets it owns, shard_range(q, world, r), and merges
those -- q*k*24 B arrive per GPU whatever the world size, so xGMI carries 1/world of the
all-gather's bytes; the results stay distributed by target slice).
"""
import torch
import torch.distributed as dist

REC_WORDS = 6


def shard_range(n, world, rank):
    """Contiguous [lo, hi) share of n ids for `rank` (first n % world ranks get one more)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _host_staged(group, *ts):
    """gloo moves host tensors only: device tensors are staged through host copies (the
    one-GPU multi-rank rehearsal); RCCL takes device tensors as they are"""
    return dist.get_backend(group) == "gloo" and any(t.is_cuda for t in ts)


def gather_records(rec, group=None, out=None):
    """All-gather this rank's (q, k, 6) int32 candidate records -> (world, q, k, 6).
    `out` may be a preallocated (world*q, k, 6) buffer (the concatenated form every
    backend accepts); list l of the result is rank l's shard."""
    world = dist.get_world_size(group)
    if out is None:
        out = torch.empty((world * rec.shape[0],) + tuple(rec.shape[1:]), dtype=rec.dtype, device=rec.device)
    if _host_staged(group, rec, out):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(h, rec.contiguous().cpu(), group=group)
        out.copy_(h)
    else:
        dist.all_gather_into_tensor(out, rec.contiguous(), group=group)
    return out.view((world,) + tuple(rec.shape))


def exchange_records(rec, group=None, out=None):
    """All-to-all of this rank's (q, k, 6) records by target slice -> (world, q_r, k, 6): list
    s holds rank s's candidates for this rank's targets shard_range(q, world, rank)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    q = rec.shape[0]
    sizes = [b - a for a, b in (shard_range(q, world, r) for r in range(world))]
    mine = sizes[rank]
    if out is None:
        out = torch.empty((world * mine,) + tuple(rec.shape[1:]), dtype=rec.dtype, device=rec.device)
    if _host_staged(group, rec, out):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(h, rec.contiguous().cpu(), output_split_sizes=[mine] * world,
                               input_split_sizes=sizes, group=group)
        out.copy_(h)
    else:
        dist.all_to_all_single(out, rec.contiguous(), output_split_sizes=[mine] * world, input_split_sizes=sizes,
                               group=group)
    return out.view((world, mine) + tuple(rec.shape[1:]))


def sharded_topk(local_records, merge, group=None):
    """One sharded lookup: local_records() -> (q, k, 6) records of this rank's shard;
    merge(gathered (world, q, k, 6)) -> final (idx, cnt)."""
    return merge(gather_records(local_records(), group))
