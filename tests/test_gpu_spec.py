"""GPU parity of BRC_MODE_SPEC (Bracha-correct broadcast, consensus with per-phase
windows and a reachable common coin) against the C oracle, which tests/test_spec_model.py pins to
an independent pure-Python model.  Bar: bit-exact statuses, counts and ordered events."""
import random

import pytest

from oracle import oracle
from tests import golden_io
from tests.golden import specs as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def runner():
    from tests import engine_runner
    return engine_runner


def _compare(runner, specs):
    got = runner.run_specs(specs)
    for sp, r in zip(specs, got):
        exp = oracle.run(sp)
        exp["events"] = golden_io.canonical_events(exp["events"])
        for k in ("status", "t_stop", "msgs_sent", "arrivals", "cell_steps"):
            assert r[k] == exp[k], "%s %s: %r vs oracle %r" % (sp["name"], k, r[k], exp[k])
        for k in ("deliver", "decide", "send"):
            assert r["events"][k] == exp["events"][k], "%s: %s events differ" % (sp["name"], k)
    return got


@pytest.mark.parametrize("n,f,model,dmax,window,rcap", [
    (4, 1, 1, 4, 4, 3), (7, 2, 2, 3, 4, 2), (10, 3, 3, 5, 8, 2), (16, 5, 2, 8, 8, 1), (16, 5, 1, 4, 2, 2),
    (31, 10, 0, 1, 4, 3), (64, 21, 2, 8, 8, 1), (64, 21, 2, 8, 8, 4), (64, 21, 3, 16, 4, 2), (100, 33, 1, 4, 4, 1),
    (256, 85, 2, 8, 8, 1), (256, 42, 3, 16, 8, 1)])
def test_spec_consensus_vs_oracle(runner, n, f, model, dmax, window, rcap):
    count = 24 if n <= 16 else (8 if n <= 64 else 1)
    specs = []
    for g in range(count):
        sp = S.spec_cons_spec(n, f, 0x5EC0 + n, model, dmax, 300 + g, round_cap=rcap, window=window,
                              coin_seed=0xC0FFEE + n)
        sp["name"] = "spec%d/%d" % (n, g)
        specs.append(sp)
    got = _compare(runner, specs)
    assert any(r["status"] == "done" for r in got)


def test_spec_coin_and_split_votes_vs_oracle(runner):
    """Evenly split proposals: phase-2 tallies at or below f, so coin rounds run."""
    specs = []
    for g in range(32):
        sp = S.spec_cons_spec(7, 2, 0xC0, 2, 3, g, round_cap=2, window=4, coin_seed=99,
                              proposals=[1, 2, 1, 2, 1, 2, 1])
        sp["name"] = "coin/%d" % g
        specs.append(sp)
    got = _compare(runner, specs)
    assert max(d[2] for r in got for d in r["events"]["decide"]) > 1


def test_spec_byzantine_equivocation_and_staggered_vs_oracle(runner):
    rng = random.Random(3)
    byz = list(range(11, 16))
    specs = []
    for g in range(16):
        sp = S.spec_cons_spec(16, 5, 0x5EED0003, 1, 4, 3000 + g, round_cap=2, window=4, coin_seed=7,
                              byzantine=byz, nv=2, extra=S.equivocation_actions(16, byz),
                              starts=[rng.choice([0, 0, rng.randint(1, 6)]) for _ in range(16)])
        sp["name"] = "specbyz/%d" % g
        specs.append(sp)
    _compare(runner, specs)


@pytest.mark.parametrize("n,f,model,dmax", [(4, 1, 1, 4), (13, 4, 3, 6), (64, 21, 2, 8), (200, 66, 1, 3)])
def test_spec_brb_vs_oracle(runner, n, f, model, dmax):
    rng = random.Random(n)
    specs = []
    for g in range(8 if n <= 64 else 2):
        origins = rng.sample(range(n), min(n, 5))
        sends = [(rng.randint(0, 5), o, q) for o in origins for q in range(rng.randint(1, 2))]
        sp = S.spec_brb_spec(n, f, 0xB0B + n, model, dmax, 60 + g, sends, window=4)
        sp["name"] = "specbrb%d/%d" % (n, g)
        specs.append(sp)
    _compare(runner, specs)


def test_round_histogram_vs_oracle():
    """brc_read_round_histogram (cfg5's per-GPU histogram) against decide rounds from the oracle."""
    from byzantinerandomizedconsensus_amd import _lib as L
    from byzantinerandomizedconsensus_amd.engine import Engine
    n, f, count, bins = 7, 2, 96, 6
    specs = [S.spec_cons_spec(n, f, 0xC1, 2, 3, g, round_cap=1, window=4, coin_seed=5,
                              proposals=[1, 2, 1, 2, 1, 2, 1]) for g in range(count)]
    exp = [0] * bins
    for sp in specs:
        r = oracle.run(sp)
        first = {}
        for t, node, rnd, _ in sorted(r["events"]["decide"]):
            first.setdefault(node, rnd)
        exp[min(max(first.values()), bins - 1) if len(first) == n else 0] += 1
    with Engine(n=n, f=f, instances=count, protocol="consensus", seed=0xC1, delay_model=L.DELAY_SLOWSET,
                delay_max=3, round_cap=1, step_cap=10000, key_window=4, proposals=L.PROPOSALS_LOADED,
                mode=L.MODE_SPEC, coin_seed=5) as eng:
        eng.load_proposals([[1, 2, 1, 2, 1, 2, 1]] * count)
        eng.run()
        got = eng.round_histogram(bins)
    assert got == exp
    assert sum(exp[2:]) > 0, "some instance needed a coin round"


@pytest.mark.parametrize("n,f", [(70, 23), (100, 33), (48, 15)])
def test_spec_late_replica_completes_buffered_phases_at_once(runner, n, f):
    """A replica that proposes late finds Q phases' deliveries buffered and completes them in ONE
    step: up to Q = 8 SENDs by one replica in one step (the wide kernel queues them until the step's
    last key pass).  Start steps 14 / 18 give 5 / 7 such SENDs (checked below); at 22 the
    eighth would reuse the slot of the replica's own phase-0 key, which the engine's phase window
    reports as BRC_OVERFLOW."""
    import collections
    specs = []
    for j, ts in enumerate((14, 18)):
        starts = [0] * n
        starts[n - 1] = ts
        sp = S.spec_cons_spec(n, f, 0x5EED0106, 0, 1, j, round_cap=3, window=8, coin_seed=0xC017C017,
                              starts=starts)
        sp["name"] = "speclate%d/%d" % (n, ts)
        specs.append(sp)
    got = _compare(runner, specs)
    bursts = [max(collections.Counter((t, src) for t, src, typ, _kp, _s in r["events"]["send"] if typ == 1).values())
              for r in got]
    assert max(bursts) >= 7 and all(r["status"] == "done" for r in got), bursts
