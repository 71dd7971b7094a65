"""Workload shapes at the edges of what the engine expresses.

Supported, checked against the C oracle on the same seeded inputs:
  * restricted-destination SENDs at n > 64 (destination masks up to 256 bits, ABI v4
    brc_injection.dst_mask_hi) -- a Byzantine origin SENDs its key to a subset of the peers;
  * the equivocation pattern at n > 64 (SURVEY §8(d) cfg3's Byzantine behaviour on a large
    committee), as explicit injections and as the engine's built-in byz_pattern.
Rejected with a documented error code (include/brc.h), asserted here:
  * a restricted ECHO / READY injection (BRC_E_UNSUPPORTED): the engine keeps one "sent" time per
    (replica, key, type), so an ECHO that reached only some peers has no representation;
  * value ids past the kernel's width (BRC_E_INVALID): three bits on the narrow kernels (n <= 32,
    connection peers), two on the others; the class API maps at most seven (three) distinct
    proposal strings besides "-1" (network.ValueTable, tested on the CPU);
  * a second SEND of one key on the lean (n in 33..64, sender peers) and wide (n > 64) kernels
    (BRC_E_UNSUPPORTED) -- the ABI form of one payload string SENT by two origins
    (core/brbroadcast.py:76-79 keys its dicts by payload); the other narrow kernels take it as an
    extra SEND (reference fixtures brb_multisend_*); the class API raises EngineError for it
    before any engine call on the former (tests/test_api_shim.py).
"""
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


@pytest.mark.parametrize("n,f,model,dmax,peer_mode", [(100, 33, 0, 1, "sender"), (256, 85, 2, 8, "sender"),
                                                      (128, 42, 3, 16, "connection")])
def test_restricted_sends_wide_vs_oracle(runner, n, f, model, dmax, peer_mode):
    """Byzantine origins SEND their keys to random subsets (some above replica 64); honest keys
    flood.  Receivers outside a subset see no SEND, so their ECHO waits for the others' ECHOes."""
    rng = random.Random(n + dmax)
    specs = []
    for g in range(3):
        byz = rng.sample(range(n), 4)          # few silent replicas: honest keys can deliver
        honest = [o for o in range(n) if o not in byz]
        extra = []
        for j, b in enumerate(rng.sample(byz, 3)):
            dst = sum(1 << d for d in range(n) if rng.random() < 0.6)
            extra.append(dict(t=0, kind="byz_key", kp=b, s=0, value=0, payload="BYZ %d" % b))
            extra.append(dict(t=j, kind="byz", src=b, type=1, kp=b, s=0, dst=dst))
        sends = [(rng.randint(0, 2), o, 0) for o in rng.sample(honest, 2)]
        sp = S.brb_spec(n, f, 0xD570 + n, model, dmax, 300 + g, sends, byzantine=byz, extra=extra,
                        peer_mode=peer_mode)
        sp["name"] = "restricted%d/%d" % (n, g)
        specs.append(sp)
    got = _compare(runner, specs)
    assert any(r["events"]["deliver"] for r in got)


@pytest.mark.parametrize("n,f,model,dmax", [(16, 3, 1, 4), (8, 2, 2, 3), (13, 2, 3, 8)])
def test_record_runs_per_segment_vs_oracle(runner, n, f, model, dmax):
    """Narrow kernels that pack several instances into one wave (n <= 16: 4 or 8 per item) apply a
    step's run of SEND / KEY records per instance, all instances at once (brc_step.h do_actions).
    Consecutive instances with different numbers of declared and (restricted) SENT Byzantine keys
    at the same steps -- some none, some several -- each equal the oracle run alone."""
    rng = random.Random(1000 + n)
    byz = list(range(n - f, n))
    specs = []
    for g in range(12):
        extra = []
        for b in rng.sample(byz, rng.randint(0, len(byz))):
            dst = sum(1 << d for d in range(n) if rng.random() < 0.7)
            t = rng.randint(0, 1)
            extra.append(dict(t=t, kind="byz_key", kp=b, s=0, value=0, payload="BYZ %d" % b))
            if rng.random() < 0.8:
                extra.append(dict(t=t, kind="byz", src=b, type=1, kp=b, s=0, dst=dst))
        sends = [(rng.randint(0, 1), o, 0) for o in rng.sample(range(n - f), 2)]
        sp = S.brb_spec(n, f, 0xA11 + n, model, dmax, 700 + g, sends, byzantine=byz, extra=extra)
        sp["name"] = "records%d/%d" % (n, g)
        specs.append(sp)
    got = _compare(runner, specs)
    assert any(r["events"]["deliver"] for r in got)


@pytest.mark.parametrize("n,f,model,dmax", [(100, 33, 1, 4), (128, 42, 2, 8)])
def test_equivocation_wide_vs_oracle(runner, n, f, model, dmax):
    """SURVEY §8(d) cfg3's equivocation on a large committee: every Byzantine replica SENDs "0"
    to even and "1" to odd replicas, then ECHOes and READYs both."""
    byz = list(range(n - f, n))
    specs = []
    for g in range(2 if n <= 100 else 1):
        sp = S.cons_spec(n, f, 0xE0C0 + n, model, dmax, 50 + g, round_cap=1, byzantine=byz, nv=2,
                         extra=S.equivocation_actions(n, byz))
        sp["name"] = "equiv%d/%d" % (n, g)
        specs.append(sp)
    _compare(runner, specs)


def test_equivocation_pattern_wide_matches_oracle():
    """The engine's built-in pattern (byz_pattern = BRC_BYZ_EQUIVOCATE) at n = 100: sampled
    instances of a 256-instance batch equal the oracle given the same pattern as injections."""
    from byzantinerandomizedconsensus_amd import _lib as L
    from byzantinerandomizedconsensus_amd.engine import Engine
    n, f, N = 100, 33, 256
    byz = list(range(n - f, n))
    with Engine(n=n, f=f, instances=N, protocol="consensus", seed=0x5EED0006, delay_model=L.DELAY_UNIFORM,
                delay_max=4, round_cap=1, step_cap=4000, key_window=4, variants=2, proposals=L.PROPOSALS_PHILOX,
                byz_pattern=L.BYZ_EQUIVOCATE, byzantine=byz) as eng:
        eng.run()
        res = eng.instances_result()
    assert not any(r["status"] in ("overflow", "bad_injection", "running") for r in res)
    for g in (0, 77, N - 1):
        exp = oracle.run(S.cons_spec(n, f, 0x5EED0006, 1, 4, g, round_cap=1, byzantine=byz, nv=2,
                                     extra=S.equivocation_actions(n, byz)))
        for k in ("status", "t_stop", "msgs_sent", "arrivals", "cell_steps"):
            assert res[g][k] == exp[k], (g, k)


def _engine(n, **kw):
    from byzantinerandomizedconsensus_amd import _lib as L
    from byzantinerandomizedconsensus_amd.engine import Engine
    args = dict(n=n, f=(n - 1) // 3, instances=2, protocol="brb", seed=1, delay_model=L.DELAY_UNIFORM, delay_max=4,
                key_window=4)
    args.update(kw)
    return Engine(**args)


@pytest.mark.parametrize("n", [16, 40, 100])
def test_rejections_are_documented_error_codes(n):
    from byzantinerandomizedconsensus_amd import _lib as L
    allm = (1 << n) - 1
    with _engine(n) as eng:
        eng.inject([dict(t=0, kind=L.INJ_SEND, node=0, kp=0, s=0, dst=allm)])
        # restricted ECHO: E_UNSUPPORTED
        with pytest.raises(L.EngineError) as ei:
            eng.inject([dict(t=1, kind=L.INJ_MSG, type=L.ECHO, node=1, kp=0, s=0, dst=allm & ~2)])
        assert ei.value.code == L.E_UNSUPPORTED
        # a second SEND of the same key (one payload, two origins): an extra SEND at n <= 32,
        # E_UNSUPPORTED on the lean (n = 40) and wide (n = 100) kernels
        if n <= 32:
            eng.inject([dict(t=0, kind=L.INJ_SEND, node=1, kp=0, s=0, dst=allm)])
        else:
            with pytest.raises(L.EngineError) as ei:
                eng.inject([dict(t=0, kind=L.INJ_SEND, node=1, kp=0, s=0, dst=allm)])
            assert ei.value.code == L.E_UNSUPPORTED
    with _engine(n, protocol="consensus", round_cap=1) as eng:
        # value ids: three bits on the narrow kernel (n = 16), two on the wide one (n = 100); E_INVALID past them
        if n <= 32:
            eng.inject([dict(t=0, kind=L.INJ_PROPOSE, node=0, value=7)])
        with pytest.raises(L.EngineError) as ei:
            eng.inject([dict(t=0, kind=L.INJ_PROPOSE, node=1, value=8 if n <= 32 else 4)])
        assert ei.value.code == L.E_INVALID


@pytest.mark.parametrize("n,f,model,dmax", [(7, 1, 1, 3), (100, 19, 0, 1), (128, 25, 2, 4)])
def test_direct_deliver_vs_oracle(runner, n, f, model, dmax):
    """ByzantineRandomizedConsensus.deliver() called directly (BRC_INJ_DELIVER) on the narrow and
    the wide kernel: random hosts and values, before and after the replicas' own proposals."""
    specs = []
    for g in range(2):
        sp = S.cons_spec(n, f, 0xDE40 + n, model, dmax, 10 + g, round_cap=2,
                         starts=[(d * 7 + g) % 4 for d in range(n)],
                         extra=S.deliver_actions(n, 0xDE40 + n + g, count=3 * n))
        sp["name"] = "deliver%d/%d" % (n, g)
        specs.append(sp)
    _compare(runner, specs)
