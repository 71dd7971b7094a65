"""Full-size GPU runs of BASELINE.json's configurations, checked through properties that do not
depend on the size: instances drawn from the full batch equal the C oracle run alone on their
global id (bit-exact status / last step / message counts / decide rounds), results do not depend
on how the instances are sharded across engines (multi-GPU invariance), and a
checksum over every instance is identical across shardings.

cfg2: 10,000 instances n=4 f=1, honest, uniform delays [1,4] (one GPU).
cfg3: one rank's shard of the 1M-instance n=16 f=5 run: 125,000 instances at global offset
      3 x 125,000, Byzantine {11..15} equivocating.
cfg4: the bench batch, 131,072 instances n=64 f=21, slow-set delays D=8 (reference and SPEC).
cfg4 at 2^20: the bench batches themselves, 257 (reference) / 129 (SPEC) ids sampled across the range.
cfg5: n=256 f=85, 512 instances per delay model (SPEC), 16 oracle-sampled ids per model.
"""
import hashlib
import random

import pytest

from oracle import oracle
from tests.golden import specs as S

VID = {v: i for i, v in enumerate(S.VALUES)}     # the oracle reports decided values as strings

pytestmark = pytest.mark.gpu


def _engine(**kw):
    from byzantinerandomizedconsensus_amd.engine import Engine
    return Engine(**kw)


def _L():
    from byzantinerandomizedconsensus_amd import _lib as L
    return L


KEYS = ("status", "t_stop", "msgs_sent", "arrivals", "cell_steps")   # cell_steps: the roofline unit


def _run(kw, first, count, ids=()):
    """Run [first, first + count); return every instance's result and the replicas of `ids`."""
    with _engine(instance_offset=first, instances=count, **kw) as eng:
        eng.run()
        res = eng.instances_result()
        reps = {i: eng.replicas(i, 1)[0] for i in ids}
    return res, reps


def _digest(res):
    h = hashlib.sha256()
    for r in res:
        h.update(repr(tuple(r[k] for k in KEYS)).encode())
    return h.hexdigest()


def _check_sample(res, reps, kw, base, ids, make_spec):
    for i in ids:
        sp = make_spec(base + i)
        exp = oracle.run(sp)
        for k in KEYS:
            assert res[i][k] == exp[k], "instance %d %s: engine %r oracle %r" % (base + i, k, res[i][k], exp[k])
        if i in reps:
            first = {}
            for t, node, rnd, val in sorted(exp["events"]["decide"]):
                first.setdefault(node, (rnd, t, VID[val]))
            for d, rep in enumerate(reps[i]):
                if d in sp.get("byzantine", []):
                    continue
                if d in first:
                    got = (rep["first_decide_round"], rep["first_decide_t"], rep["first_decide_value"])
                    assert got == first[d], (base + i, d, got, first[d])
                else:
                    assert rep["decide_count"] == 0, (base + i, d)


def _sharding_invariant(kw, first, count, full):
    half = count // 2
    a, _ = _run(kw, first, half)
    b, _ = _run(kw, first + half, count - half)
    assert _digest(a + b) == _digest(full)


def test_cfg2_full_size():
    L = _L()
    N = 10000
    kw = dict(n=4, f=1, protocol="consensus", seed=0x5EED0002, delay_model=L.DELAY_UNIFORM, delay_max=4,
              round_cap=2, step_cap=4000, key_window=8, proposals=L.PROPOSALS_PHILOX)
    ids = random.Random(2).sample(range(N), 64)
    res, reps = _run(kw, 0, N, ids)
    assert all(r["status"] in ("done", "quiescent") for r in res)
    _check_sample(res, reps, kw, 0, ids, lambda g: S.cons_spec(4, 1, 0x5EED0002, 1, 4, g, round_cap=2))
    _sharding_invariant(kw, 0, N, res)


def test_cfg3_rank_shard_full_size():
    L = _L()
    per, rank = 125000, 3
    byz = list(range(11, 16))
    kw = dict(n=16, f=5, protocol="consensus", seed=0x5EED0003, delay_model=L.DELAY_UNIFORM, delay_max=4,
              round_cap=1, step_cap=4000, key_window=4, variants=2, proposals=L.PROPOSALS_PHILOX,
              byz_pattern=L.BYZ_EQUIVOCATE, byzantine=byz)
    first = rank * per
    ids = random.Random(3).sample(range(per), 24)
    res, reps = _run(kw, first, per, ids)
    assert not any(r["status"] in ("overflow", "bad_injection", "running") for r in res)
    make = lambda g: S.cons_spec(16, 5, 0x5EED0003, 1, 4, g, round_cap=1, byzantine=byz, nv=2,  # noqa: E731
                                 extra=S.equivocation_actions(16, byz))
    _check_sample(res, reps, kw, first, ids, make)
    _sharding_invariant(kw, first, per, res)


@pytest.mark.parametrize("mode", ["reference", "spec"])
def test_cfg4_bench_batch_full_size(mode):
    L = _L()
    N = 131072
    spec = mode == "spec"
    kw = dict(n=64, f=21, protocol="consensus", seed=0x5EED0004, delay_model=L.DELAY_SLOWSET, delay_max=8,
              round_cap=1, step_cap=4000, key_window=8 if spec else 4, proposals=L.PROPOSALS_PHILOX,
              mode=L.MODE_SPEC if spec else L.MODE_REFERENCE, coin_seed=0xC017C017)
    with _engine(instance_offset=0, instances=N, **kw) as eng:
        eng.run()
        res = eng.instances_result()
        hist = eng.round_histogram(66)
        reps = eng.replicas(0, 8) + eng.replicas(N - 8, 8)
    assert hist[0] == 0 and sum(hist) == N, "every instance decided"
    if spec:
        make = lambda g: S.spec_cons_spec(64, 21, 0x5EED0004, 2, 8, g, round_cap=1, window=8,  # noqa: E731
                                          coin_seed=0xC017C017)
    else:
        make = lambda g: S.cons_spec(64, 21, 0x5EED0004, 2, 8, g, round_cap=1)  # noqa: E731
    sub = res[:8] + res[N - 8:]
    ids = list(range(8)) + list(range(N - 8, N))
    for j, g in enumerate(ids):
        exp = oracle.run(make(g))
        for k in KEYS:
            assert sub[j][k] == exp[k], (g, k)
        first = {}
        for t, node, rnd, val in sorted(exp["events"]["decide"]):
            first.setdefault(node, (rnd, t, VID[val]))
        got = [(r["first_decide_round"], r["first_decide_t"], r["first_decide_value"]) for r in reps[j]]
        assert got == [first[d] for d in range(64)], g


def _cfg5_cases():
    import json
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cfg5_oracle.json")
    with open(path) as fh:
        return json.load(fh)["cases"]


@pytest.mark.parametrize("model,dmax", [(0, 1), (1, 4), (3, 16)])
def test_cfg5_n256_full_size(model, dmax):
    """The 512-instance batch of each delay model; sampled ids equal the C oracle's results
    (tests/golden/cfg5_oracle.json, made by tests/golden/make_cfg5_oracle.py: an n = 256 oracle
    run takes about a minute) -- counters and every honest replica's first decision."""
    L = _L()
    N = 512
    kw = dict(n=256, f=85, protocol="consensus", seed=0x5EED0005, delay_model=model, delay_max=dmax,
              round_cap=1, step_cap=4000, key_window=8, proposals=L.PROPOSALS_PHILOX, mode=L.MODE_SPEC,
              coin_seed=0xC017C017)
    cases = [c for c in _cfg5_cases() if c["model"] == model and c["dmax"] == dmax]
    assert cases
    with _engine(instance_offset=0, instances=N, **kw) as eng:
        eng.run()
        res = eng.instances_result()
        hist = eng.round_histogram(66)
        reps = {c["g"]: eng.replicas(c["g"], 1)[0] for c in cases}
    assert hist[0] == 0 and sum(hist) == N
    assert all(r["status"] == "done" for r in res)
    for c in cases:
        g = c["g"]
        for k in KEYS:
            assert res[g][k] == c[k], (model, g, k)
        for d, (rep, exp) in enumerate(zip(reps[g], c["first_decide"])):
            assert exp is not None, (g, d)
            got = (rep["first_decide_round"], rep["first_decide_t"], rep["first_decide_value"])
            assert got == (exp[0], exp[1], VID[exp[2]]), (model, g, d)


@pytest.mark.parametrize("mode", ["reference", "spec"])
def test_cfg4_bench_batch_2p20_sampled(mode):
    """The bench's own batches (2^20 instances in one launch: the reference protocol, and SPEC with
    Q = 8 on 4-byte cells): instances sampled across the whole id range equal the oracle run alone
    on their global id."""
    L = _L()
    N = 1 << 20
    spec = mode == "spec"
    kw = dict(n=64, f=21, protocol="consensus", seed=0x5EED0004, delay_model=L.DELAY_SLOWSET, delay_max=8,
              round_cap=1, step_cap=4000, key_window=8 if spec else 4, proposals=L.PROPOSALS_PHILOX,
              mode=L.MODE_SPEC if spec else L.MODE_REFERENCE, coin_seed=0xC017C017)
    ids = sorted(random.Random(20).sample(range(N - 1), 128 if spec else 256)) + [N - 1]
    with _engine(instance_offset=0, instances=N, **kw) as eng:
        eng.run()
        hist = eng.round_histogram(66)
        vals, disagreements = eng.decisions()
        res = {i: eng.instances_result(i, 1)[0] for i in ids}
        reps = {i: eng.replicas(i, 1)[0] for i in ids}
    assert hist[0] == 0 and sum(hist) == N, "every instance decided"
    assert disagreements == 0 and vals["undecided"] == 0
    assert sum(vals.values()) == N * 64, "one first decision per honest replica"
    sampled = {}
    if spec:
        specs = [S.spec_cons_spec(64, 21, 0x5EED0004, 2, 8, g, round_cap=1, window=8, coin_seed=0xC017C017) for g in ids]
    else:
        specs = [S.cons_spec(64, 21, 0x5EED0004, 2, 8, g, round_cap=1) for g in ids]
    for g, (exp, first, _last, _count) in zip(ids, _oracle_first_last(specs)):
        for k in KEYS:
            assert res[g][k] == exp[k], (g, k)
        got = [(r["first_decide_round"], r["first_decide_t"], r["first_decide_value"]) for r in reps[g]]
        assert got == [first[d] for d in range(64)], g
        for d in range(64):
            sampled[first[d][2]] = sampled.get(first[d][2], 0) + 1
    # the decided-value histogram the bench reports: every sampled value occurs in it, and in SPEC
    # mode (coin rounds) both binary values appear, in the reference protocol "-1" (id 0)
    names = {0: "-1", 1: "0", 2: "1", 3: "3"}
    for v in sampled:
        assert vals[names[v]] > 0, (v, vals)
    if spec:
        assert vals["0"] > 0 and vals["1"] > 0 and vals["-1"] == 0
    else:
        assert vals["-1"] == N * 64, vals


def _oracle_first_last(specs):
    """The oracle on several specs at once (threads: ctypes releases the GIL in the C run): per
    spec the result and every replica's (first decision, last value, decide count)."""
    import concurrent.futures
    with concurrent.futures.ThreadPoolExecutor(min(8, len(specs))) as ex:
        outs = list(ex.map(lambda sp: oracle.run(sp, kinds=("decide",)), specs))
    per = []
    for exp in outs:
        first, last, count = {}, {}, {}
        for t, node, rnd, val in sorted(exp["events"]["decide"]):
            first.setdefault(node, (rnd, t, VID[val]))
            last[node] = VID[val]
            count[node] = count.get(node, 0) + 1
        per.append((exp, first, last, count))
    return per


@pytest.mark.parametrize("mode", ["reference", "spec"])
def test_cfg4_long_consensus_many_rounds(mode):
    """Long-running consensus (the reference re-proposes forever, core/byzantinerandomizedconsensus.py:
    96-106) on the cfg4 slow-set schedule (D = 8).  Reference protocol: SURVEY cfg4's round cap 64.
    Its phase leakage (:57-61, :71-78: deliveries of any phase count toward the current one) lets
    fast replicas end several phases per step, so by round 64 up to 127 phase indices of one origin
    are in flight and ~7,600 keys of one instance are live at once (oracle-measured): it
    runs with a key window of 128 on the key-lifetime kernel, which keeps no cells (2^14 instances:
    its key slots take 115 KB of LDS per wave).  SPEC: round cap 8 with its window of 8 at 2^17.
    Sampled instances equal the oracle (counters incl. cell-steps, and every replica's first and
    last decision, values included)."""
    L = _L()
    spec = mode == "spec"
    N, CAP = (1 << 17, 8) if spec else (1 << 14, 64)
    kw = dict(n=64, f=21, protocol="consensus", seed=0x5EED0004, delay_model=L.DELAY_SLOWSET, delay_max=8,
              round_cap=CAP, step_cap=4000, key_window=8 if spec else 128, proposals=L.PROPOSALS_PHILOX,
              mode=L.MODE_SPEC if spec else L.MODE_REFERENCE, coin_seed=0xC017C017)
    ids = sorted(random.Random(8).sample(range(N), 5)) + [N - 1]
    with _engine(instance_offset=0, instances=N, **kw) as eng:
        eng.run()
        assert eng.last_kernel() == "life"              # two-class form (SPEC too, round 6)
        st = eng.stats()
        hist = eng.round_histogram(66)
        res = {i: eng.instances_result(i, 1)[0] for i in ids}
        reps = {i: eng.replicas(i, 1)[0] for i in ids}
    assert st["done"] == N and st["overflow"] == 0       # no BRC_OVERFLOW anywhere in the batch
    assert hist[0] == 0 and sum(hist) == N
    if spec:
        specs = [S.spec_cons_spec(64, 21, 0x5EED0004, 2, 8, g, round_cap=CAP, window=8, coin_seed=0xC017C017)
                 for g in ids]
    else:
        specs = [S.cons_spec(64, 21, 0x5EED0004, 2, 8, g, round_cap=CAP) for g in ids]
    for g, (exp, first, last, count) in zip(ids, _oracle_first_last(specs)):
        for k in KEYS:
            assert res[g][k] == exp[k], (g, k)
        for d, r in enumerate(reps[g]):
            assert (r["first_decide_round"], r["first_decide_t"], r["first_decide_value"]) == first[d], (g, d)
            assert r["last_decide_value"] == last[d] and r["decide_count"] == count[d] >= CAP, (g, d)


def test_cfg4_many_rounds_2p20_one_launch():
    """The bench's many-round leg: the reference protocol to round cap 8 on the cfg4 schedule at the
    full 2^20 instances in ONE launch.  By round 8 ~1,000 keys of one instance are live at once
    (oracle-measured), so any cell store would need >= 1,025 x 64 x 4 B per instance = 275 GB: the
    engine picks the key-lifetime kernel (no cells; key window 32).  Sampled ids equal the oracle."""
    L = _L()
    N, CAP = 1 << 20, 8
    kw = dict(n=64, f=21, protocol="consensus", seed=0x5EED0004, delay_model=L.DELAY_SLOWSET, delay_max=8,
              round_cap=CAP, step_cap=4000, key_window=32, proposals=L.PROPOSALS_PHILOX)
    ids = sorted(random.Random(64).sample(range(N - 1), 31)) + [N - 1]
    with _engine(instance_offset=0, instances=N, **kw) as eng:
        eng.run()
        assert eng.last_kernel() == "life"
        st = eng.stats()
        vals, dis = eng.decisions()
        res = {i: eng.instances_result(i, 1)[0] for i in ids}
        reps = {i: eng.replicas(i, 1)[0] for i in ids}
    assert st["done"] == N and st["overflow"] == 0 and dis == 0
    specs = [S.cons_spec(64, 21, 0x5EED0004, 2, 8, g, round_cap=CAP) for g in ids]
    for g, (exp, first, last, count) in zip(ids, _oracle_first_last(specs)):
        for k in KEYS:
            assert res[g][k] == exp[k], (g, k)
        for d, r in enumerate(reps[g]):
            assert (r["first_decide_round"], r["first_decide_t"], r["first_decide_value"]) == first[d], (g, d)
            assert r["last_decide_value"] == last[d] and r["decide_count"] == count[d] >= CAP, (g, d)


@pytest.mark.parametrize("leg", ["long", "spec64"])
def test_cfg4_round_cap_64_2p20_bench_legs(leg):
    """bench.py's long and spec64 legs at their timed size: SURVEY cfg4's round cap 64 at the full 2^20
    instances per GPU, one launch each.  long: the reference protocol (the re-proposal loop
    core/byzantinerandomizedconsensus.py:96-106; by round 64 ~7,600 keys of one instance are live at
    once, so the key-lifetime kernel with a key window of 128, its slot metadata in HBM).  spec64: the
    intended protocol with the common coin (:88-92 made reachable), window 8, on the same kernel.
    Sampled ids equal the oracle (counters incl. cell-steps, every replica's first and last decision
    and its decide count)."""
    L = _L()
    N, CAP = 1 << 20, 64
    spec = leg == "spec64"
    kw = dict(n=64, f=21, protocol="consensus", seed=0x5EED0004, delay_model=L.DELAY_SLOWSET, delay_max=8,
              round_cap=CAP, step_cap=4000, key_window=8 if spec else 128, proposals=L.PROPOSALS_PHILOX,
              mode=L.MODE_SPEC if spec else L.MODE_REFERENCE, coin_seed=0xC017C017)
    ids = sorted(random.Random(6464 + spec).sample(range(N - 1), 5)) + [N - 1]
    with _engine(instance_offset=0, instances=N, **kw) as eng:
        eng.run()
        assert eng.last_kernel() == "life"              # two-class form (SPEC too, round 6)
        st = eng.stats()
        vals, dis = eng.decisions()
        res = {i: eng.instances_result(i, 1)[0] for i in ids}
        reps = {i: eng.replicas(i, 1)[0] for i in ids}
    assert st["done"] == N and st["overflow"] == 0 and dis == 0
    if spec:
        specs = [S.spec_cons_spec(64, 21, 0x5EED0004, 2, 8, g, round_cap=CAP, window=8, coin_seed=0xC017C017)
                 for g in ids]
    else:
        specs = [S.cons_spec(64, 21, 0x5EED0004, 2, 8, g, round_cap=CAP) for g in ids]
    for g, (exp, first, last, count) in zip(ids, _oracle_first_last(specs)):
        for k in KEYS:
            assert res[g][k] == exp[k], (g, k)
        for d, r in enumerate(reps[g]):
            assert (r["first_decide_round"], r["first_decide_t"], r["first_decide_value"]) == first[d], (g, d)
            assert r["last_decide_value"] == last[d] and r["decide_count"] == count[d] >= CAP, (g, d)


@pytest.mark.parametrize("model,dmax", [("slowset", 8), ("uniform", 2), ("uniform", 4), ("geometric", 16)])
def test_cfg4_connection_peers_2p20_sampled(model, dmax):
    """cfg4 with connection-identity peers -- what the shipped reference runs
    (core/brbroadcast.py:69) -- at the bench's full 2^20 instances in one launch (the key-lifetime
    kernel, csrc/brc_life.h; its two-class form under the slow set, its per-link form under uniform
    delays and under cfg5's geometric delays capped at 16, whose keys live up to 64 steps: the
    64-row ring): instances sampled across the range equal the oracle run alone on their global id,
    decided values included.  (Uniform D = 4 stalls every instance before its first decision in the
    reference protocol -- the oracle agrees -- so that case checks counters and silence.)"""
    L = _L()
    N = 1 << 20
    dm = {"slowset": L.DELAY_SLOWSET, "uniform": L.DELAY_UNIFORM, "geometric": L.DELAY_GEOMETRIC}[model]
    kw = dict(n=64, f=21, protocol="consensus", seed=0x5EED0004, delay_model=dm, delay_max=dmax,
              round_cap=1, step_cap=4000, key_window=4, proposals=L.PROPOSALS_PHILOX, peer_mode=L.PEER_CONNECTION)
    ids = sorted(random.Random(21).sample(range(N - 1), 47)) + [N - 1]
    with _engine(instance_offset=0, instances=N, **kw) as eng:
        eng.run()
        assert eng.last_kernel() == "life"
        hist = eng.round_histogram(66)
        vals, disagreements = eng.decisions()
        res = {i: eng.instances_result(i, 1)[0] for i in ids}
        reps = {i: eng.replicas(i, 1)[0] for i in ids}
        ovf = eng.stats()["overflow"]
    assert sum(hist) == N and disagreements == 0 and ovf == 0
    if model == "slowset":
        assert hist[0] == 0
    decided = 0
    specs = [S.cons_spec(64, 21, 0x5EED0004, dm, dmax, g, round_cap=1, peer_mode="connection") for g in ids]
    for g, (exp, first, _last, _count) in zip(ids, _oracle_first_last(specs)):
        for k in KEYS:
            assert res[g][k] == exp[k], (g, k)
        for d, r in enumerate(reps[g]):
            if d in first:
                assert (r["first_decide_round"], r["first_decide_t"], r["first_decide_value"]) == first[d], (g, d)
                decided += 1
            else:
                assert r["decide_count"] == 0, (g, d)
    if (model, dmax) in (("slowset", 8), ("uniform", 2)):     # uniform[1,4] stalls all; geometric most
        assert decided > 0


def _batch_digest(eng, chunk=1 << 16):
    """sha256 over every instance's (status, t_stop, msgs, arrivals, cell_steps, deliveries,
    decided) and every replica's consensus record (round, phase, value_count, decide_count, first
    decision round / step / value, last value), read in bulk (numpy) chunk by chunk."""
    import numpy as np
    h = hashlib.sha256()
    ikeys = ("status", "t_stop", "msgs_sent", "arrivals", "cell_steps", "deliveries", "decided")
    for first in range(0, eng.instances, chunk):
        cnt = min(chunk, eng.instances - first)
        ia = eng.instances_array(first, cnt)
        ra = eng.replicas_array(first, cnt)
        for k in ikeys:
            h.update(np.ascontiguousarray(ia[k]).tobytes())
        for k in ra.dtype.names:
            h.update(np.ascontiguousarray(ra[k]).tobytes())
    return h.hexdigest()


def test_cfg4_2p20_step_kernel_equals_lifetime_kernel():
    """The bench's whole 2^20 sender-peer cfg4 batch on both kernels (BRC_KERNEL=step: the step
    kernel's cell store; BRC_KERNEL=life: the key-lifetime kernel the headline runs, cells in registers): a digest
    of every instance's counters (cell-steps included: the roofline's unit) and every replica's
    consensus record is identical -- not a sample, the whole batch (reference:
    core/brbroadcast.py:60-119, core/byzantinerandomizedconsensus.py:53-106)."""
    import os
    L = _L()
    N = 1 << 20
    kw = dict(n=64, f=21, protocol="consensus", seed=0x5EED0004, delay_model=L.DELAY_SLOWSET, delay_max=8,
              round_cap=1, step_cap=4000, key_window=4, proposals=L.PROPOSALS_PHILOX)
    digests, stats = {}, {}
    for kernel in ("step", "life"):
        old = os.environ.get("BRC_KERNEL")
        os.environ["BRC_KERNEL"] = kernel
        try:
            eng = _engine(instance_offset=0, instances=N, **kw)
        finally:
            if old is None:
                os.environ.pop("BRC_KERNEL", None)
            else:
                os.environ["BRC_KERNEL"] = old
        with eng:
            eng.run()
            assert eng.last_kernel() == kernel
            digests[kernel] = _batch_digest(eng)
            stats[kernel] = eng.stats()
    assert stats["step"]["done"] == N and stats["step"]["overflow"] == 0
    for k in ("decided", "msgs_sent", "arrivals", "cell_steps", "deliveries", "decide_rounds_sum"):
        assert stats["step"][k] == stats["life"][k], k
    assert digests["step"] == digests["life"]
