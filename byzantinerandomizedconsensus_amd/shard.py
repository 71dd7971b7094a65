"""Instance sharding across ranks.

Instances are independent, so a run of ``total`` instances gives each rank a contiguous range of
GLOBAL instance ids.  Every Philox draw is keyed by the global id, so an instance computes the
same thing whichever rank runs it and however many ranks there are.  There is no data-path
exchange.  The one collective is ``reduce_stats``: an all-reduce of the statistics at the end
(RCCL over xGMI with the ``nccl`` backend on MI355X, gloo in the CPU tests).
"""

SUM_KEYS = ("instances", "running", "done", "quiescent", "stepcap", "overflow", "decided", "msgs_sent",
            "arrivals", "cell_steps", "deliveries", "decide_rounds_sum", "events_dropped", "lane_loads",
            # Engine.decisions(): first decided value per honest replica, and disagreeing instances
            "dec_-1", "dec_0", "dec_1", "dec_3", "dec_undecided", "disagreements")
MAX_KEYS = ("max_t",)


def shard_range(total, world, rank):
    """[first, first + count) of the global instance ids owned by ``rank``.  The first
    ``total % world`` ranks take one extra instance."""
    if not 0 <= rank < world:
        raise ValueError("rank %d outside world %d" % (rank, world))
    base, extra = divmod(total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def reduce_stats(stats, dist=None, device="cpu", hist=None):
    """All-reduce one rank's ``Engine.stats()`` dict (and optional round histogram list).

    Sums the counters, takes the max of ``max_t``; returns (stats, hist) for the whole job.  With
    ``dist`` None (single process) the inputs are returned unchanged."""
    if dist is None:
        return dict(stats), (list(hist) if hist is not None else None)
    import torch
    sums = torch.tensor([int(stats.get(k, 0)) for k in SUM_KEYS], dtype=torch.int64, device=device)
    dist.all_reduce(sums)
    maxs = torch.tensor([int(stats.get(k, 0)) for k in MAX_KEYS], dtype=torch.int64, device=device)
    dist.all_reduce(maxs, op=dist.ReduceOp.MAX)
    out = dict(stats)
    out.update({k: int(v) for k, v in zip(SUM_KEYS, sums.tolist())})
    out.update({k: int(v) for k, v in zip(MAX_KEYS, maxs.tolist())})
    h = None
    if hist is not None:
        ht = torch.tensor([int(x) for x in hist], dtype=torch.int64, device=device)
        dist.all_reduce(ht)
        h = [int(x) for x in ht.tolist()]
    return out, h


def max_over_ranks(value, dist=None, device="cpu"):
    """Max of a float over ranks (the bench's wall time)."""
    if dist is None:
        return value
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
