"""GPU parity: the HIP engine (through the C-ABI) against the reference's golden fixtures and
against the C oracle on fresh seeded workloads.  Bar: bit-exact (status, last active step,
message counts and every ordered delivery / decide / send event)."""
import random

import pytest

from oracle import oracle
from tests import golden_io
from tests.golden import specs as S

pytestmark = pytest.mark.gpu

GROUPS = golden_io.groups()


@pytest.fixture(scope="module")
def runner():
    from tests import engine_runner
    return engine_runner


@pytest.mark.parametrize("group", sorted(GROUPS))
def test_engine_matches_reference_fixtures(runner, group):
    cases = GROUPS[group]
    got = runner.run_specs([c["spec"] for c in cases])
    for i, (c, r) in enumerate(zip(cases, got)):
        golden_io.assert_matches(c["result"], r, "%s[%d]" % (group, i))
        # the roofline's unit: cell-steps equal the oracle's on the reference-pinned schedule
        assert r["cell_steps"] == golden_io.cell_steps(group, i), (group, i, r["cell_steps"])


def _compare_with_oracle(runner, specs):
    got = runner.run_specs(specs)
    for sp, r in zip(specs, got):
        exp = oracle.run(sp)
        exp["events"] = golden_io.canonical_events(exp["events"])
        for k in ("status", "t_stop", "msgs_sent", "arrivals", "cell_steps"):
            assert r[k] == exp[k], "%s %s: %r vs oracle %r" % (sp["name"], k, r[k], exp[k])
        for k in ("deliver", "decide", "send"):
            assert r["events"][k] == exp["events"][k], "%s: %s events differ" % (sp["name"], k)
    return got


@pytest.mark.parametrize("n,f,model,dmax", [(4, 1, 1, 4), (7, 2, 3, 6), (16, 5, 1, 4), (13, 4, 2, 5)])
def test_brb_random_vs_oracle(runner, n, f, model, dmax):
    rng = random.Random(n * 1000 + dmax)
    specs = []
    for g in range(48):
        sends = [(rng.randint(0, 5), o, q) for o in range(n) for q in range(rng.randint(0, 2))]
        sp = S.brb_spec(n, f, 0xBEEF + n, model, dmax, 1000 + g, sends)
        sp["name"] = "brb%d/%d" % (n, g)
        specs.append(sp)
    _compare_with_oracle(runner, specs)


@pytest.mark.parametrize("n,f,model,dmax,rcap", [(4, 1, 1, 4, 3), (6, 1, 1, 3, 2), (7, 2, 2, 4, 3),
                                                  (10, 3, 3, 5, 2), (16, 5, 2, 8, 2), (16, 3, 1, 2, 2),
                                                  (31, 10, 2, 6, 1), (33, 10, 1, 3, 1)])
def test_consensus_random_vs_oracle(runner, n, f, model, dmax, rcap):
    specs = []
    for g in range(32):
        sp = S.cons_spec(n, f, 0xC0DE + n, model, dmax, 500 + g, round_cap=rcap)
        sp["name"] = "cons%d/%d" % (n, g)
        specs.append(sp)
    _compare_with_oracle(runner, specs)


def test_consensus_n64_slowset_vs_oracle(runner):
    specs = []
    for g in range(6):
        sp = S.cons_spec(64, 21, 0x5EED0004, 2, 8, 77 + g, round_cap=1)
        sp["name"] = "cfg4/%d" % g
        specs.append(sp)
    _compare_with_oracle(runner, specs)


def test_equivocation_vs_oracle(runner):
    byz = list(range(11, 16))
    specs = []
    for g in range(16):
        sp = S.cons_spec(16, 5, 0x5EED0003, 1, 4, 3000 + g, round_cap=1, byzantine=byz, nv=2,
                         extra=S.equivocation_actions(16, byz))
        sp["name"] = "cfg3/%d" % g
        specs.append(sp)
    _compare_with_oracle(runner, specs)


def test_staggered_starts_vs_oracle(runner):
    rng = random.Random(5)
    specs = []
    for g in range(24):
        sp = S.cons_spec(6, 1, 99, 1, 3, 9000 + g, round_cap=2,
                         starts=[rng.choice([0, 0, rng.randint(1, 12)]) for _ in range(6)])
        sp["name"] = "stag/%d" % g
        specs.append(sp)
    _compare_with_oracle(runner, specs)


# ---- connection-identity peers (core/brbroadcast.py:69) ----
@pytest.mark.parametrize("n,f,model,dmax", [(4, 1, 1, 4), (7, 2, 3, 6), (16, 5, 2, 8), (33, 10, 1, 3), (64, 21, 2, 8),
                                             (16, 5, 3, 16), (64, 21, 1, 12),                 # D up to 16
                                             (100, 33, 1, 4), (128, 42, 2, 8), (256, 85, 3, 16), (256, 85, 0, 3)])
def test_connection_brb_floods_vs_oracle(runner, n, f, model, dmax):
    """Honest broadcasts plus Byzantine nodes that re-send ECHO / READY of honest keys at several
    steps: every copy is a new peer, so the counts (and K4 re-fires) differ from sender mode."""
    rng = random.Random(n * 31 + dmax)
    allm = (1 << n) - 1
    specs = []
    for g in range(24 if n <= 16 else 6 if n <= 64 else 3):
        byz = rng.sample(range(n), f)
        honest = [o for o in range(n) if o not in byz]
        sends = [(rng.randint(0, 3), o, 0) for o in rng.sample(honest, min(len(honest), 4))]
        extra = []
        for (t0, o, q) in sends:
            for b in rng.sample(byz, min(len(byz), 3)):
                for _ in range(rng.randint(1, 3)):
                    extra.append(dict(t=t0 + rng.randint(0, 6), kind="byz", src=b, type=rng.choice([2, 3]),
                                      kp=o, s=q, dst=allm))
        sp = S.brb_spec(n, f, 0xC0 + n, model, dmax, 900 + g, sends, byzantine=byz, extra=extra,
                        peer_mode="connection")
        sp["name"] = "connbrb%d/%d" % (n, g)
        specs.append(sp)
    _compare_with_oracle(runner, specs)


@pytest.mark.parametrize("n,f,model,dmax,rcap", [(4, 1, 1, 4, 3), (7, 2, 2, 4, 2), (10, 3, 3, 5, 2),
                                                  (16, 5, 2, 8, 2), (64, 21, 2, 8, 1), (10, 3, 3, 14, 2),
                                                  (100, 33, 1, 4, 1), (128, 42, 2, 8, 1)])
def test_connection_consensus_vs_oracle(runner, n, f, model, dmax, rcap):
    specs = []
    for g in range(24 if n <= 16 else 4 if n <= 64 else 1):
        sp = S.cons_spec(n, f, 0xC0C0 + n, model, dmax, 40 + g, round_cap=rcap, peer_mode="connection")
        sp["name"] = "conncons%d/%d" % (n, g)
        specs.append(sp)
    _compare_with_oracle(runner, specs)


def test_connection_equivocation_vs_oracle(runner):
    byz = list(range(11, 16))
    specs = []
    for g in range(16):
        sp = S.cons_spec(16, 5, 0x5EED0003, 1, 4, 3100 + g, round_cap=1, byzantine=byz, nv=2,
                         extra=S.equivocation_actions(16, byz), peer_mode="connection")
        sp["name"] = "conncfg3/%d" % g
        specs.append(sp)
    _compare_with_oracle(runner, specs)


@pytest.mark.parametrize("n,f,dmax", [(16, 5, 4), (100, 33, 4)])
def test_connection_many_copies_vs_oracle(runner, n, f, dmax):
    """Byzantine replicas re-send one READY / ECHO up to 255 times in one step (one-byte send
    counts, 8 count planes): the arrival counts and the :119 re-fires they trigger match the
    oracle."""
    allm = (1 << n) - 1
    byz = list(range(n - f, n))
    specs = []
    for g, copies in enumerate((40, 200, 255)):
        extra = [dict(t=1, kind="byz", src=byz[0], type=3, kp=0, s=0, dst=allm) for _ in range(copies)]
        extra += [dict(t=2, kind="byz", src=byz[1], type=2, kp=1, s=0, dst=allm) for _ in range(copies // 2)]
        sp = S.brb_spec(n, f, 0xC0F0 + n, 1, dmax, 70 + g, [(0, 0, 0), (0, 1, 0)], byzantine=byz, extra=extra,
                        peer_mode="connection")
        sp["name"] = "copies%d/%d" % (n, copies)
        specs.append(sp)
    _compare_with_oracle(runner, specs)


def test_connection_copy_count_ceiling_is_reported(runner):
    """256 copies of one type from one replica in one step exceed the one-byte count: the
    instance stops with bad_injection instead of miscounting."""
    n, f = 16, 5
    allm = (1 << n) - 1
    extra = [dict(t=1, kind="byz", src=15, type=3, kp=0, s=0, dst=allm) for _ in range(256)]
    sp = S.brb_spec(n, f, 0xC0F1, 1, 4, 5, [(0, 0, 0)], byzantine=[15], extra=extra, peer_mode="connection")
    sp["name"] = "copies-ceiling"
    assert runner.run_specs([sp])[0]["status"] == "bad_injection"
