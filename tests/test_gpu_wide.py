"""GPU parity of the large-committee kernel (n in (64, 256], csrc/brc_step_wide.h; SURVEY §8(d)
cfg5) against the C oracle on fresh seeded workloads.  Same bar as test_gpu_parity.py: status,
last active step, message counts and every ordered delivery / decide / send event, bit-exact.
The reference's own fixtures at n = 70, 100 and 256 run in test_gpu_parity.py (tests/golden)."""
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


def _compare(runner, specs, **kw):
    got = runner.run_specs(specs, **kw)
    for sp, r in zip(specs, got):
        exp = oracle.run(sp)
        exp["events"] = golden_io.canonical_events(exp["events"])
        for k in ("status", "t_stop", "msgs_sent", "arrivals", "cell_steps"):
            assert r[k] == exp[k], "%s %s: %r vs oracle %r" % (sp["name"], k, r[k], exp[k])
        for k in ("deliver", "decide", "send"):
            assert r["events"][k] == exp["events"][k], "%s: %s events differ" % (sp["name"], k)
    return got


@pytest.mark.parametrize("n,f,model,dmax", [(65, 21, 1, 4), (100, 33, 3, 16), (128, 42, 2, 8), (129, 40, 0, 1),
                                            (200, 66, 1, 3), (256, 85, 3, 16), (256, 85, 2, 8)])
def test_wide_brb_vs_oracle(runner, n, f, model, dmax):
    rng = random.Random(n * 7 + dmax)
    specs = []
    for g in range(6):
        origins = rng.sample(range(n), 3)
        sends = [(rng.randint(0, 4), o, q) for o in origins for q in range(rng.randint(1, 2))]
        sp = S.brb_spec(n, f, 0xB1DE + n, model, dmax, 40 + g, sends, dconst=1)
        sp["name"] = "wbrb%d/%d" % (n, g)
        specs.append(sp)
    _compare(runner, specs)


@pytest.mark.parametrize("n,f,model,dmax,rcap,count", [(65, 21, 2, 8, 1, 4), (96, 31, 1, 4, 2, 3),
                                                        (130, 43, 3, 6, 1, 2), (256, 85, 2, 8, 1, 1)])
def test_wide_consensus_vs_oracle(runner, n, f, model, dmax, rcap, count):
    specs = []
    for g in range(count):
        sp = S.cons_spec(n, f, 0xC0DE + n, model, dmax, 700 + g, round_cap=rcap)
        sp["name"] = "wcons%d/%d" % (n, g)
        specs.append(sp)
    _compare(runner, specs)


def test_wide_byzantine_and_staggered_vs_oracle(runner):
    """Byzantine replicas above 64 (mask words 1..3) and staggered proposals."""
    n, f = 160, 31
    byz = [3, 70, 128, 150]
    rng = random.Random(11)
    specs = []
    for g in range(3):
        sp = S.cons_spec(n, f, 0x5EED, 1, 3, 50 + g, round_cap=1, byzantine=byz,
                         starts=[rng.choice([0, 0, rng.randint(1, 6)]) for _ in range(n)])
        sp["name"] = "wbyz/%d" % g
        specs.append(sp)
    _compare(runner, specs)


def test_wide_scripted_byzantine_messages_vs_oracle(runner):
    """A Byzantine origin above 64 declares a key, SENDs it to everyone, and Byzantine peers ECHO
    and READY it (every-peer destinations, the only kind the wide engine takes)."""
    n, f = 100, 20
    allm = (1 << n) - 1
    byz = list(range(80, 100))
    specs = []
    for g in range(2):
        extra = [dict(t=0, kind="byz_key", kp=90, s=0, value=2),
                 dict(t=0, kind="byz", src=90, type=S.SEND, kp=90, s=0, dst=allm)]
        extra += [dict(t=1 + (b % 3), kind="byz", src=b, type=S.ECHO, kp=90, s=0, dst=allm) for b in byz]
        extra += [dict(t=2 + (b % 4), kind="byz", src=b, type=S.READY, kp=90, s=0, dst=allm) for b in byz[:12]]
        sp = S.brb_spec(n, f, 0xFACE, 1, 4, 5 + g, [(0, 1, 0), (1, 65, 0)], byzantine=byz, extra=extra)
        sp["name"] = "wscript/%d" % g
        specs.append(sp)
    _compare(runner, specs)
