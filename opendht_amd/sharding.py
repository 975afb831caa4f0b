"""Multi-GPU sharding of the id set (north-star scheme).

The N ids are split into contiguous ranges, one per rank.  Every rank answers all targets from
its range in record form: k compact candidate records {w0, w1, global idx} (12 B) per target; the
records are exchanged over RCCL (xGMI on MI355X, gloo in CPU tests) and K3 merges world*k
candidates per target into the exact global top-k (XOR distance, then global index).

The records carry 64 of an id's 160 bits.  Two candidates of one target that agree on them (ids
sharing their first 64 bits: never among the candidates of hash-distributed ids, but possible
for crafted ones) cannot be ordered by the records alone: K3 lists such rows (`ties` = {count,
rows[TIE_CAP]}), and a second, small exchange carries words 2..4 of every rank's candidates in
those rows only (TIE_CAP x k x 12 B per rank), after which the listed rows are merged again on
the full keys.  The exchange is always issued (fixed size, stream-ordered, no host sync); when
more than TIE_CAP rows tie, `settle_overflow_*` (after a synchronisation) repeats it for every
row.  With one rank there is nothing to tie across and no second exchange.

Per-step contract (a pipelined caller): a step's results are final once its stream has run
merge_* AND `unsettled(tx)` is false (a device flag, no host sync); when it is true -- more than
TIE_CAP rows tied, crafted ids only -- the caller synchronises and calls settle_overflow_* before
reading the rows.  merge_* never returns such a step's rows as final silently: the flag is the tie
count itself, written by K3 on the step's stream.

Streams: every device step of one lookup (K3, the tie words, the full-key settlement) runs on ONE
stream -- the caller's, or torch's current stream when the caller passes none -- and that stream
must be torch's current stream, because RCCL orders the collectives after it.

Two exchanges: the all-gather (`gather_records`, the north star's: every rank merges every
target, so every rank holds the same tie rows) and the all-to-all by target slice
(`exchange_records`: rank r receives only the records of the targets it owns, shard_range(q,
world, r), q*k*12 B per GPU whatever the world size; its tie rows are its own, so the tie lists
are all-gathered and each rank returns the words each owner asked for).
"""
import torch
import torch.distributed as dist

REC_WORDS = 3      # compact candidate record {w0, w1, global idx} (include/dhtgpu.h DHTGPU_REC_WORDS)
TIE_CAP = 256      # rows one fixed-size tie exchange settles


def shard_range(n, world, rank):
    """Contiguous [lo, hi) share of n ids for `rank` (first n % world ranks get one more)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


_GROUPS = {}   # resolved process group -> (its backend is gloo, world size): looked up once per group


def _group_info(group):
    """(gloo?, world size) of `group` (None = the default group, resolved to its current object, so
    a destroyed and re-created default group -- another backend -- is looked up afresh)"""
    g = group if group is not None else dist.group.WORLD
    info = _GROUPS.get(g)
    if info is None:
        if len(_GROUPS) > 64:
            _GROUPS.clear()
        info = _GROUPS[g] = (dist.get_backend(group) == "gloo", dist.get_world_size(group))
    return info


def _host_staged(group, *ts):
    """gloo moves host tensors only: device tensors are staged through host copies (the
    one-GPU multi-rank rehearsal); RCCL takes device tensors as they are"""
    return _group_info(group)[0] and any(t.is_cuda for t in ts)


def _stream(stream, t):
    """The one stream of a lookup's device steps: the caller's, else torch's current stream on
    t's device (RCCL orders the collectives after the current stream, so a caller's stream must be
    that one).  None for host tensors (the CPU tests' stand-in ops)."""
    if not t.is_cuda:
        return stream
    cur = torch.cuda.current_stream(t.device).cuda_stream
    if stream is None:
        return cur
    if stream != cur:
        raise ValueError("sharding: the lookup's stream must be torch's current stream (RCCL orders the "
                         "collectives after it); set it with torch.cuda.set_stream first")
    return stream


def gather_records(rec, group=None, out=None):
    """All-gather this rank's (q, k, W) int32 records -> (world, q, k, W).  `out` may be a
    preallocated (world*q, k, W) buffer (the concatenated form every backend accepts); list l of
    the result is rank l's shard.  Also moves the tie words ((TIE_CAP, k, 3) per rank)."""
    world = _group_info(group)[1]
    if out is None:
        out = torch.empty((world * rec.shape[0],) + tuple(rec.shape[1:]), dtype=rec.dtype, device=rec.device)
    elif tuple(out.shape) != (world * rec.shape[0],) + tuple(rec.shape[1:]):
        raise ValueError(f"gather_records: out {tuple(out.shape)} is not (world * q, ...) for world {world} and "
                         f"records {tuple(rec.shape)}")
    if _host_staged(group, rec, out):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(h, rec.contiguous().cpu(), group=group)
        out.copy_(h)
    else:
        dist.all_gather_into_tensor(out, rec.contiguous(), group=group)
    return out.view((world,) + tuple(rec.shape))


def exchange_records(rec, group=None, out=None):
    """All-to-all of this rank's (q, k, W) records by target slice -> (world, q_r, k, W): list s
    holds rank s's candidates for this rank's targets shard_range(q, world, rank)."""
    world = _group_info(group)[1]
    rank = dist.get_rank(group)
    q = rec.shape[0]
    sizes = [b - a for a, b in (shard_range(q, world, r) for r in range(world))]
    mine = sizes[rank]
    if out is None:
        out = torch.empty((world * mine,) + tuple(rec.shape[1:]), dtype=rec.dtype, device=rec.device)
    _all_to_all(out, rec.contiguous(), [mine] * world, sizes, group)
    return out.view((world, mine) + tuple(rec.shape[1:]))


def _all_to_all(out, inp, out_sizes, in_sizes, group):
    if _host_staged(group, inp, out):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(h, inp.cpu(), output_split_sizes=out_sizes, input_split_sizes=in_sizes, group=group)
        out.copy_(h)
    else:
        dist.all_to_all_single(out, inp, output_split_sizes=out_sizes, input_split_sizes=in_sizes, group=group)


def sharded_topk(local_records, merge, group=None):
    """One sharded lookup: local_records() -> (q, k, W) records of this rank's shard;
    merge(gathered (world, q, k, W)) -> final (idx, cnt)."""
    return merge(gather_records(local_records(), group))


class TieExchange:
    """Device buffers of the second exchange for one in-flight lookup: the tie list, this rank's
    words for it, and what arrives from every rank."""

    def __init__(self, world, k, device):
        self.world, self.k = world, k
        self.ties = torch.zeros(1 + TIE_CAP, dtype=torch.int32, device=device)
        self.ties_all = torch.zeros((world, 1 + TIE_CAP), dtype=torch.int32, device=device)
        self.words = torch.empty((world, TIE_CAP, k, 3), dtype=torch.int32, device=device)   # out (a2a: per owner)
        self.words_in = torch.empty((world, TIE_CAP, k, 3), dtype=torch.int32, device=device)


def unsettled(tx):
    """Device flag (0-dim bool tensor, no host sync): the last merge_* through `tx` listed more tie
    rows than one tie exchange settles, so its rows are final only after settle_overflow_*."""
    return tx.ties[0] > TIE_CAP


def _check(code, what):
    if code != 0:
        raise RuntimeError(f"libdhtgpu: {what} failed ({code})")


class LibOps:
    """The protocol's three device steps through libdhtgpu: K3 (dhtgpu_merge_dev), this rank's tie
    words (dhtgpu_tie_words_dev on its context) and the full-key settlement
    (dhtgpu_merge_ties_dev).  tp / ts: the target planes (row t0 of a slice = tp + 4 * t0)."""

    def __init__(self, L, ctx, tp, ts):
        self.L, self.ctx, self.tp, self.ts = L, ctx, tp, ts

    def merge(self, g, t0, k, out_idx, out_cnt, ties, stream):
        _check(self.L.dhtgpu_merge_dev(g.data_ptr(), g.shape[0], g.shape[1], g.shape[2], self.tp + 4 * t0, self.ts,
                                       k, out_idx.data_ptr(), out_cnt.data_ptr(),
                                       None if ties is None else ties.data_ptr(), TIE_CAP, stream), "merge_dev")

    def tie_words(self, rec, idx_base, ties, row_base, out, stream):
        self.ctx.tie_words_dev(rec.data_ptr(), rec.shape[0], rec.shape[1], idx_base,
                               None if ties is None else ties.data_ptr(), TIE_CAP, row_base, out.data_ptr(), stream)

    def merge_ties(self, g, words, t0, k, ties, out_idx, out_cnt, stream):
        _check(self.L.dhtgpu_merge_ties_dev(g.data_ptr(), words.data_ptr(), g.shape[0], g.shape[1], g.shape[2],
                                            self.tp + 4 * t0, self.ts, k, None if ties is None else ties.data_ptr(),
                                            TIE_CAP if ties is not None else 0, out_idx.data_ptr(), out_cnt.data_ptr(),
                                            stream), "merge_ties_dev")


def merge_allgather(ops, rec, gathered, k, out_idx, out_cnt, tx, idx_base, stream=None, group=None):
    """K3 over the all-gathered records (every rank merges every target) + the tie exchange.
    rec: this rank's own (q, k, 3) records (the tie words come from its own id set); gathered:
    (world, q, k, 3).  Stream-ordered, no host sync."""
    world = gathered.shape[0]
    stream = _stream(stream, rec)
    ops.merge(gathered, 0, k, out_idx, out_cnt, tx.ties if world > 1 else None, stream)
    if world == 1:
        return
    ops.tie_words(rec, idx_base, tx.ties, 0, tx.words[0], stream)
    gather_records(tx.words[0], group, out=tx.words_in.view(world * TIE_CAP, k, 3))
    ops.merge_ties(gathered, tx.words_in, 0, k, tx.ties, out_idx, out_cnt, stream)


def merge_alltoall(ops, rec, exch, k, tlo, out_idx, out_cnt, tx, idx_base, stream=None, group=None):
    """K3 over this rank's target slice [tlo, tlo + q_r) (exch: (world, q_r, k, 3) from
    exchange_records) + the tie exchange: the ranks' tie lists are all-gathered, each rank
    writes words 2..4 of its candidates for every owner's tie rows and an all-to-all returns
    them to the owners."""
    world, qr = exch.shape[0], exch.shape[1]
    q = rec.shape[0]
    stream = _stream(stream, rec)
    if qr:
        ops.merge(exch, tlo, k, out_idx, out_cnt, tx.ties if world > 1 else None, stream)
    else:
        tx.ties.zero_()
    if world == 1:
        return
    gather_records(tx.ties, group, out=tx.ties_all.view(-1))
    for s in range(world):
        slo, _ = shard_range(q, world, s)
        ops.tie_words(rec, idx_base, tx.ties_all[s], slo, tx.words[s], stream)
    n = TIE_CAP * k * 3
    _all_to_all(tx.words_in.view(-1), tx.words.view(-1), [n] * world, [n] * world, group)
    if qr:
        ops.merge_ties(exch, tx.words_in, tlo, k, tx.ties, out_idx, out_cnt, stream)


def settle_overflow_allgather(ops, rec, gathered, k, out_idx, out_cnt, tx, idx_base, stream=None, group=None):
    """After a synchronisation: when more rows tied than one tie exchange settles (the same count
    on every rank of the all-gather route), every row is merged again on the full keys.  Returns
    the tie count."""
    world, q = gathered.shape[0], gathered.shape[1]
    stream = _stream(stream, rec)
    count = int(tx.ties[0].item()) if world > 1 else 0
    if count > TIE_CAP:
        words = torch.empty((q, k, 3), dtype=torch.int32, device=rec.device)
        ops.tie_words(rec, idx_base, None, 0, words, stream)
        allw = gather_records(words, group)
        ops.merge_ties(gathered, allw, 0, k, None, out_idx, out_cnt, stream)
    return count


def settle_overflow_alltoall(ops, rec, exch, k, tlo, out_idx, out_cnt, tx, idx_base, stream=None, group=None):
    """The all-to-all route's overflow settlement (after a synchronisation; the ranks agree on
    it by an all-reduce of their tie counts): words 2..4 of every candidate go to the target's
    owner like the records did, and the owner merges its whole slice on the full keys.  Returns
    this rank's tie count."""
    world, qr = exch.shape[0], exch.shape[1]
    if world == 1:
        return 0
    stream = _stream(stream, rec)
    mine = int(tx.ties[0].item()) if qr else 0
    top = torch.tensor([mine], dtype=torch.int64)
    if not _group_info(group)[0]:
        top = top.to(rec.device)
    dist.all_reduce(top, op=dist.ReduceOp.MAX, group=group)
    if int(top.item()) > TIE_CAP:
        words = torch.empty((rec.shape[0], k, 3), dtype=torch.int32, device=rec.device)
        ops.tie_words(rec, idx_base, None, 0, words, stream)
        allw = exchange_records(words, group)
        if qr:
            ops.merge_ties(exch, allw, tlo, k, None, out_idx, out_cnt, stream)
    return mine
