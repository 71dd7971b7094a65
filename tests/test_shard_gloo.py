"""Multi-rank path on CPU (gloo, world_size 2): instance sharding + the statistics all-reduce.

Each rank runs its shard of global instance ids through the C oracle (a stand-in for the
engine: test infrastructure only) and reduces with ``shard.reduce_stats``.  The job totals must
equal a single-process run over every instance: the invariance the bench's weak scaling rests
on (Philox keyed by global ids, no data-path exchange)."""
import json
import os
import socket

import pytest

from byzantinerandomizedconsensus_amd import shard

N, F, SEED, MODEL, DMAX, TOTAL, RCAP = 7, 2, 0xA11, 1, 4, 13, 2


def test_shard_range_partitions():
    for total in (0, 1, 7, 13, 1 << 20):
        for world in (1, 2, 3, 8):
            spans = [shard.shard_range(total, world, r) for r in range(world)]
            assert sum(c for _, c in spans) == total
            assert spans[0][0] == 0
            for (a, ca), (b, _) in zip(spans, spans[1:]):
                assert a + ca == b
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
    with pytest.raises(ValueError):
        shard.shard_range(10, 2, 2)


def _instance_stats(first, count):
    from oracle import oracle
    from tests.golden import specs as S
    st = {k: 0 for k in shard.SUM_KEYS}
    st["max_t"] = 0
    hist = [0] * 8
    for g in range(first, first + count):
        r = oracle.run(S.cons_spec(N, F, SEED, MODEL, DMAX, g, round_cap=RCAP))
        st["instances"] += 1
        st["done"] += r["status"] == "done"
        st["quiescent"] += r["status"] == "quiescent"
        st["msgs_sent"] += r["msgs_sent"]
        st["arrivals"] += r["arrivals"]
        st["deliveries"] += len(r["events"]["deliver"])
        st["max_t"] = max(st["max_t"], r["t_stop"])
        first_round = {}
        for (_t, node, rnd, _v) in r["events"]["decide"]:
            first_round.setdefault(node, rnd)
        st["decided"] += len(first_round) == N
        st["decide_rounds_sum"] += sum(first_round.values())
        for rnd in first_round.values():
            hist[min(rnd, 7)] += 1
    return st, hist


def _worker(rank, world, port, outdir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, count = shard.shard_range(TOTAL, world, rank)
    st, hist = _instance_stats(first, count)
    tot, h = shard.reduce_stats(st, dist, hist=hist)
    wall = shard.max_over_ranks(float(rank + 1), dist)
    with open(os.path.join(outdir, "rank%d.json" % rank), "w") as fh:
        json.dump({"stats": tot, "hist": h, "wall": wall}, fh)
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_two_rank_gloo_totals_equal_single_process(tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    single, hist = _instance_stats(0, TOTAL)
    for r in range(world):
        got = json.load(open(tmp_path / ("rank%d.json" % r)))
        assert got["stats"] == single
        assert got["hist"] == hist
        assert got["wall"] == float(world)
    assert single["instances"] == TOTAL and single["done"] + single["quiescent"] == TOTAL
