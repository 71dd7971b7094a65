"""SPEC modes: the C oracle's restatement (oracle/brc_oracle.c) against the independent pure-Python
model (tests/spec_model.py) on random small workloads -- honest runs, coin rounds, Byzantine
silence and equivocation, staggered starts, every delay model and key window.  The reference
cannot run these modes, so this agreement is what pins their parity."""
import random

import pytest

from oracle import oracle
from tests import golden_io, spec_model
from tests.golden import specs as S


def _check(sp):
    exp = spec_model.run(sp)
    got = oracle.run(sp)
    for k in ("status", "t_stop", "msgs_sent", "arrivals"):
        assert got[k] == exp[k], "%s %s: oracle %r model %r" % (sp["name"], k, got[k], exp[k])
    a, b = golden_io.canonical_events(got["events"]), golden_io.canonical_events(exp["events"])
    for k in ("deliver", "decide", "send"):
        assert a[k] == b[k], "%s: %s events differ" % (sp["name"], k)
    return got


def _random_specs(seed, count):
    rng = random.Random(seed)
    out = []
    for i in range(count):
        n = rng.choice([4, 5, 6, 7, 8, 10, 13])
        f = rng.randint(0, (n - 1) // 3)
        model = rng.randint(0, 3)
        dmax = rng.randint(1, 6) if model else 1
        window = rng.choice([2, 4, 8])
        g = rng.getrandbits(20)
        if rng.random() < 0.25:
            sends = [(rng.randint(0, 5), o, q) for o in range(n) for q in range(rng.randint(0, 2))]
            sp = S.spec_brb_spec(n, f, rng.getrandbits(40), model, dmax, g, sends, window=window)
        else:
            byz = rng.sample(range(n), rng.randint(0, f))
            extra = []
            if byz and rng.random() < 0.5:
                extra = S.equivocation_actions(n, byz)
            starts = None if rng.random() < 0.6 else [rng.choice([0, 0, rng.randint(1, 8)]) for _ in range(n)]
            sp = S.spec_cons_spec(n, f, rng.getrandbits(40), model, dmax, g, round_cap=rng.randint(1, 4),
                                  window=window, coin_seed=rng.getrandbits(40), byzantine=byz,
                                  nv=2 if extra else 1, extra=extra, starts=starts, step_cap=3000)
        sp["name"] = "specfuzz/%d" % i
        out.append(sp)
    return out


@pytest.mark.parametrize("chunk", range(4))
def test_oracle_spec_matches_model(chunk):
    for sp in _random_specs(1000 + chunk, 40):
        _check(sp)


def test_spec_coin_rounds_happen():
    """With an even split the phase-2 tallies stay at or below f, so the common coin decides the
    next estimate; every honest replica still decides, and all decide the same value."""
    seen_coin = False
    for g in range(20):
        sp = S.spec_cons_spec(7, 2, 0xC0, 2, 3, g, round_cap=1, window=4, coin_seed=99,
                              proposals=[1, 2, 1, 2, 1, 2, 1])
        sp["name"] = "coin/%d" % g
        r = _check(sp)
        assert r["status"] == "done"
        dec = r["events"]["decide"]
        assert len({d[3] for d in dec}) == 1, "agreement"
        seen_coin |= max(d[2] for d in dec) > 1
    assert seen_coin, "no instance needed a coin round"


def test_oracle_beb_matches_model():
    """Best-effort broadcast: the C oracle's beb_on_message against the model."""
    rng = random.Random(44)
    for i in range(60):
        n = rng.choice([3, 4, 7, 10, 16])
        model = rng.randint(0, 3)
        dmax = rng.randint(1, 6) if model else 1
        sends = [(rng.randint(0, 6), o, q) for o in range(n) for q in range(rng.randint(0, 2))]
        byz = rng.sample(range(n), rng.randint(0, n // 3))
        sp = S.beb_spec(n, rng.getrandbits(40), model, dmax, rng.getrandbits(20),
                        [x for x in sends if x[1] not in byz], byzantine=byz)
        sp["name"] = "beb/%d" % i
        r = _check(sp)
        honest = n - len(byz)
        assert len(r["events"]["deliver"]) == honest * len([x for x in sends if x[1] not in byz])
