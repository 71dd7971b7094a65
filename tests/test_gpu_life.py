"""The key-lifetime kernel (csrc/brc_life.h) against the step kernel and the C oracle.

The engine runs a fresh, eligible configuration (n in 33..64, consensus, constant or slow-set
delays (two-class form) or uniform / geometric delays (per-link form) with D <= 8, no events, no
injections; include/brc.h brc_last_kernel) on the lifetime
kernel: by default, except sender peers under per-link delays (there only when BRC_KERNEL=life).  The
step kernel is pinned to the reference fixtures (test_gpu_parity.py), so each workload here runs on
both kernels (BRC_KERNEL=life / step at engine creation) and every output must match: per-instance status, last active
step, message / arrival / cell-step / delivery counters, every replica's consensus record, the
round and decided-value histograms.  Sampled instances are also checked against the oracle
directly, decided values included.  Workloads cover all three protocol modes, both delay models,
several committee sizes, silent Byzantine replicas, loaded proposals, key variants, multi-round
runs, and the stalls the reference protocol produces (quiescent instances).
"""
import os
import random

import numpy as np
import pytest

from oracle import oracle
from tests.golden import specs as S

pytestmark = pytest.mark.gpu

COIN = 0xC017C017


def _L():
    from byzantinerandomizedconsensus_amd import _lib as L
    return L


def _workloads():
    L = _L()
    base = dict(protocol="consensus", step_cap=4000, proposals=L.PROPOSALS_PHILOX)
    W = {
        "ref-slow64": dict(base, n=64, f=21, seed=0x5EED0004, delay_model=L.DELAY_SLOWSET, delay_max=8, round_cap=1,
                           key_window=4),
        "ref-slow64-r3": dict(base, n=64, f=21, seed=0x5EED0014, delay_model=L.DELAY_SLOWSET, delay_max=8,
                              round_cap=3, key_window=8),
        # reference consensus with delay 1 everywhere advances several phases per step: the phase
        # window overflows (both kernels stop with BRC_OVERFLOW at the same step)
        "ref-const64-cap30-ovf": dict(base, n=64, f=21, seed=0x5EED0034, delay_model=L.DELAY_CONST, delay_max=1,
                                      delay_const=1, round_cap=0, key_window=8, step_cap=30),
        # ... which a key window of 32 covers (up to 27 phase indices of one origin in flight)
        "ref-const64-cap30-q32": dict(base, n=64, f=21, seed=0x5EED0034, delay_model=L.DELAY_CONST, delay_max=1,
                                      delay_const=1, round_cap=0, key_window=32, step_cap=30),
        "ref-slow64-r6-q32": dict(base, n=64, f=21, seed=0x5EED0036, delay_model=L.DELAY_SLOWSET, delay_max=8,
                                  round_cap=6, key_window=32),
        "ref-const64-r4": dict(base, n=64, f=21, seed=0x5EED0015, delay_model=L.DELAY_CONST, delay_max=2, delay_const=2,
                               round_cap=4, key_window=8),
        "spec-slow64": dict(base, n=64, f=21, seed=0x5EED0004, delay_model=L.DELAY_SLOWSET, delay_max=8, round_cap=2,
                            key_window=8, mode=L.MODE_SPEC, coin_seed=COIN),
        "beb-slow64": dict(base, n=64, f=21, seed=0x5EED0024, delay_model=L.DELAY_SLOWSET, delay_max=8, round_cap=1,
                           key_window=8, mode=L.MODE_BEB),
        "ref-const50": dict(base, n=50, f=16, seed=0xC0115, delay_model=L.DELAY_CONST, delay_max=3, delay_const=3,
                            round_cap=2, key_window=4),
        "ref-byz-slow64": dict(base, n=64, f=21, seed=0xB1250, delay_model=L.DELAY_SLOWSET, delay_max=5, round_cap=2,
                               key_window=4, byzantine=[3, 40, 63]),
        "spec-const37": dict(base, n=37, f=12, seed=0x37, delay_model=L.DELAY_CONST, delay_max=1, delay_const=1,
                             round_cap=3, key_window=4, mode=L.MODE_SPEC, coin_seed=COIN),
        "ref-slowD1-40": dict(base, n=40, f=13, seed=0xD1, delay_model=L.DELAY_SLOWSET, delay_max=1, round_cap=2,
                              key_window=4),
        "spec-nv2-slow48": dict(base, n=48, f=15, seed=0x4802, delay_model=L.DELAY_SLOWSET, delay_max=4, round_cap=2,
                                key_window=4, variants=2, mode=L.MODE_SPEC, coin_seed=COIN),
        # round_cap 0: consensus runs on until the step cap (statistics truncated at step 30, while keys
        # created before it still have arrivals past it)
        "ref-slow64-cap30": dict(base, n=64, f=21, seed=0x5EED0034, delay_model=L.DELAY_SLOWSET, delay_max=8,
                                 round_cap=0, key_window=8, step_cap=30),
        # connection-identity peers (core/brbroadcast.py:69): the kernel's default use
        "conn-slow64": dict(base, n=64, f=21, seed=0x5EED0004, delay_model=L.DELAY_SLOWSET, delay_max=8, round_cap=1,
                            key_window=4, peer_mode=L.PEER_CONNECTION),
        "conn-const64-r3": dict(base, n=64, f=21, seed=0xC0AA64, delay_model=L.DELAY_CONST, delay_max=2,
                                delay_const=2, round_cap=3, key_window=8, peer_mode=L.PEER_CONNECTION),
        "conn-const45-byz": dict(base, n=45, f=14, seed=0xC0AB45, delay_model=L.DELAY_CONST, delay_max=2, delay_const=2,
                                 round_cap=2, key_window=4, byzantine=[0, 44], peer_mode=L.PEER_CONNECTION),
        "conn-slow56-r2": dict(base, n=56, f=18, seed=0xC0AC56, delay_model=L.DELAY_SLOWSET, delay_max=5, round_cap=2,
                               key_window=8, peer_mode=L.PEER_CONNECTION),
        # per-link delays (the kernel's per-link form): uniform / geometric, every protocol mode
        "conn-unif64": dict(base, n=64, f=21, seed=0x5EED0004, delay_model=L.DELAY_UNIFORM, delay_max=4, round_cap=1,
                            key_window=4, peer_mode=L.PEER_CONNECTION),
        "conn-unif64-d2-r3": dict(base, n=64, f=21, seed=0xC0DE02, delay_model=L.DELAY_UNIFORM, delay_max=2,
                                  round_cap=3, key_window=8, peer_mode=L.PEER_CONNECTION),
        "conn-geo64": dict(base, n=64, f=21, seed=0x6E0064, delay_model=L.DELAY_GEOMETRIC, delay_max=8, round_cap=1,
                           key_window=4, peer_mode=L.PEER_CONNECTION),
        # delays up to 16 (cfg5's geometric cap): the per-link form's 64-row ring
        "conn-geo64-d16": dict(base, n=64, f=21, seed=0x6E1664, delay_model=L.DELAY_GEOMETRIC, delay_max=16,
                               round_cap=1, key_window=4, peer_mode=L.PEER_CONNECTION),
        "conn-unif50-d12-r2": dict(base, n=50, f=16, seed=0xC0D12, delay_model=L.DELAY_UNIFORM, delay_max=12,
                                   round_cap=2, key_window=8, peer_mode=L.PEER_CONNECTION),
        "ref-geo64-d16-cap40": dict(base, n=64, f=21, seed=0x5EED1664, delay_model=L.DELAY_GEOMETRIC, delay_max=16,
                                    round_cap=0, key_window=16, step_cap=40),
        "conn-unif45-byz": dict(base, n=45, f=14, seed=0xC0AD45, delay_model=L.DELAY_UNIFORM, delay_max=3, round_cap=2,
                                key_window=8, byzantine=[1, 30], peer_mode=L.PEER_CONNECTION),
        "ref-unif64-d2-r3": dict(base, n=64, f=21, seed=0x5EED0044, delay_model=L.DELAY_UNIFORM, delay_max=2,
                                 round_cap=3, key_window=8),
        "ref-geo64-cap30": dict(base, n=64, f=21, seed=0x5EED0054, delay_model=L.DELAY_GEOMETRIC, delay_max=6,
                                round_cap=0, key_window=32, step_cap=30),
        "spec-unif64": dict(base, n=64, f=21, seed=0x5EED0064, delay_model=L.DELAY_UNIFORM, delay_max=4, round_cap=2,
                            key_window=8, mode=L.MODE_SPEC, coin_seed=COIN),
        "beb-geo48": dict(base, n=48, f=15, seed=0x5EED0074, delay_model=L.DELAY_GEOMETRIC, delay_max=5, round_cap=1,
                          key_window=8, mode=L.MODE_BEB),
        "ref-loaded-slow48": dict(base, n=48, f=15, seed=0x4803, delay_model=L.DELAY_SLOWSET, delay_max=6, round_cap=1,
                                  key_window=4, proposals=L.PROPOSALS_LOADED),
    }
    return W


def _oracle_spec(kw, g, props=None):
    L = _L()
    n, f = kw["n"], kw["f"]
    model, dmax = kw["delay_model"], kw["delay_max"]
    extra = dict(byzantine=kw.get("byzantine", ()), dconst=kw.get("delay_const", 1), nv=kw.get("variants", 1),
                 step_cap=kw["step_cap"])
    if kw.get("peer_mode") == L.PEER_CONNECTION:
        extra["peer_mode"] = "connection"
    if props is not None:
        extra["proposals"] = list(props)
    mode = kw.get("mode", L.MODE_REFERENCE)
    if mode == L.MODE_SPEC:
        return S.spec_cons_spec(n, f, kw["seed"], model, dmax, g, round_cap=kw["round_cap"], window=kw["key_window"],
                                coin_seed=COIN, **extra)
    if mode == L.MODE_BEB:
        return S.beb_cons_spec(n, f, kw["seed"], model, dmax, g, round_cap=kw["round_cap"], **extra)
    return S.cons_spec(n, f, kw["seed"], model, dmax, g, round_cap=kw["round_cap"], **extra)


def _run(kw, count, offset, kernel, props=None):
    from byzantinerandomizedconsensus_amd.engine import Engine
    old = os.environ.pop("BRC_KERNEL", None)
    os.environ["BRC_KERNEL"] = kernel
    try:
        eng = Engine(instances=count, instance_offset=offset, **kw)
    finally:
        os.environ.pop("BRC_KERNEL", None)
        if old is not None:
            os.environ["BRC_KERNEL"] = old
    with eng:
        if props is not None:
            eng.load_proposals(props)
        eng.run()
        used = eng.last_kernel()
        out = {"inst": eng.instances_result(), "reps": eng.replicas(), "hist": eng.round_histogram(66),
               "dec": eng.decisions(), "stats": eng.stats()}
    assert used == kernel, (kernel, used)
    return out


@pytest.mark.parametrize("name", sorted(_workloads()))
def test_lifetime_kernel_equals_step_kernel_and_oracle(name):
    kw = _workloads()[name]
    L = _L()
    count, offset = 1024, 777
    props = None
    if kw.get("proposals") == L.PROPOSALS_LOADED:
        props = np.random.RandomState(5).randint(0, 4, size=(count, kw["n"])).astype(np.int8)
    life = _run(kw, count, offset, "life", props)
    step = _run(kw, count, offset, "step", props)
    for i, (a, b) in enumerate(zip(life["inst"], step["inst"])):
        for k in ("status", "t_stop", "msgs_sent", "arrivals", "cell_steps", "deliveries", "decided"):
            assert a[k] == b[k], (name, i, k, a[k], b[k])
    for i, (a, b) in enumerate(zip(life["reps"], step["reps"])):
        assert a == b, (name, i)
    assert life["hist"] == step["hist"] and life["dec"] == step["dec"]
    for k, v in step["stats"].items():
        if k not in ("lane_loads", "max_t"):
            assert life["stats"][k] == v, (name, k)
    assert life["stats"]["running"] == 0
    if name.endswith("-ovf"):
        assert life["stats"]["overflow"] > 0          # the engine's phase window, not the protocol
        return
    assert life["stats"]["overflow"] == 0
    # sampled ids against the oracle, decided values included
    for i in random.Random(len(name)).sample(range(count), 6):
        exp = oracle.run(_oracle_spec(kw, offset + i, None if props is None else props[i]))
        r = life["inst"][i]
        for k in ("status", "t_stop", "msgs_sent", "arrivals", "cell_steps"):
            assert r[k] == exp[k], (name, i, k, r[k], exp[k])
        first = {}
        for t, node, rnd, val in sorted(exp["events"]["decide"]):
            first.setdefault(node, (rnd, t, S.VALUES.index(val)))
        for d, rep in enumerate(life["reps"][i]):
            if d in kw.get("byzantine", ()):
                continue
            if d in first:
                assert (rep["first_decide_round"], rep["first_decide_t"], rep["first_decide_value"]) == first[d], (name, i, d)
            else:
                assert rep["decide_count"] == 0, (name, i, d)


def test_lifetime_only_engine_rejects_injections_up_front():
    """A sender-peer engine with a key window above 32 at n = 64 runs on the key-lifetime kernel only
    (brc.h brc_last_kernel): the choice is fixed at brc_create (configuration and device model, not free
    memory), brc_last_kernel reports it before any run, and brc_inject refuses at once
    (BRC_E_UNSUPPORTED) instead of succeeding and failing the later run; so does a stepped run."""
    from byzantinerandomizedconsensus_amd.engine import Engine
    L = _L()
    kw = dict(n=64, f=21, protocol="consensus", seed=0x5EED0004, delay_model=L.DELAY_SLOWSET, delay_max=8,
              round_cap=2, step_cap=4000, key_window=64, proposals=L.PROPOSALS_PHILOX)
    with Engine(instances=4, **kw) as eng:
        assert eng.last_kernel() == "life"
        with pytest.raises(L.EngineError) as ei:
            eng.inject([dict(t=0, kind=L.INJ_PROPOSE, instance=0, node=0, value=1)])
        assert ei.value.code == L.E_UNSUPPORTED
        with pytest.raises(L.EngineError) as ei:
            eng.run(5)
        assert ei.value.code == L.E_UNSUPPORTED
        eng.run()
        assert eng.last_kernel() == "life"
        assert all(r["status"] == "done" for r in eng.instances_result())
    with Engine(instances=4, **dict(kw, key_window=8)) as eng:
        # a window the step kernel takes: the lifetime kernel by default, and an injection moves the run
        # to the step kernel instead of being refused
        assert eng.last_kernel() == "life"
        eng.inject([dict(t=0, kind=L.INJ_PROPOSE, instance=0, node=0, value=1)])
        eng.run()
        assert eng.last_kernel() == "step"


def test_kernel_choice():
    """Default choice: eligible configurations run on the lifetime kernel, except sender peers under
    per-link delays (step kernel, faster there); event logs, injections, stepped runs and two-class delays
    past 8 stay on the step kernel; a lifetime-run instance cannot be re-opened by an injection."""
    from byzantinerandomizedconsensus_amd.engine import Engine
    L = _L()
    assert "BRC_KERNEL" not in os.environ
    kw = _workloads()["conn-slow64"]
    with Engine(instances=4, **kw) as eng:
        eng.run()
        assert eng.last_kernel() == "life"
        st = eng.instances_result()
    with Engine(instances=4, **_workloads()["ref-slow64"]) as eng:
        eng.run()
        assert eng.last_kernel() == "life"                # sender peers, two-class form
    with Engine(instances=4, **_workloads()["ref-unif64-d2-r3"]) as eng:
        eng.run()
        assert eng.last_kernel() == "step"                # sender peers, per-link delays
    with Engine(instances=4, event_capacity=1 << 16, **kw) as eng:
        eng.run()
        assert eng.last_kernel() == "step"
    with Engine(instances=4, **kw) as eng:
        eng.run(5)
        assert eng.last_kernel() == "step"
    with Engine(instances=4, **dict(kw, delay_model=L.DELAY_UNIFORM, delay_max=4)) as eng:
        eng.run()
        assert eng.last_kernel() == "life"                # per-link form
    with Engine(instances=4, **dict(kw, delay_model=L.DELAY_GEOMETRIC, delay_max=16)) as eng:
        eng.run()
        assert eng.last_kernel() == "life"                # per-link form, delays up to 16 (64-row ring)
    with Engine(instances=4, **dict(kw, delay_max=12)) as eng:
        eng.run()
        assert eng.last_kernel() == "step"                # two-class form: D <= 8
    with Engine(instances=4, **kw) as eng:
        eng.inject([dict(t=0, kind=L.INJ_PROPOSE, instance=0, node=0, value=1)])
        eng.run()
        assert eng.last_kernel() == "step"
        eng.reset()
        eng.run()
        assert eng.last_kernel() == "life"
        assert [r["status"] for r in eng.instances_result()] == [r["status"] for r in st]
    with Engine(instances=2, **dict(kw, round_cap=200, step_cap=20)) as eng:
        eng.run()
        assert eng.last_kernel() == "life"
        if eng.instances_result(0, 1)[0]["status"] == "quiescent":
            with pytest.raises(L.EngineError):
                eng.inject([dict(t=30, kind=L.INJ_PROPOSE, instance=0, node=0, value=1)])


def test_per_link_rerun_after_reset():
    """The per-link form leaves its HBM delivery-bitmap ring zero (rows of steps a stopped instance
    never reached are cleared at exit): a reset engine's second lifetime run equals its first."""
    from byzantinerandomizedconsensus_amd.engine import Engine
    kw = _workloads()["ref-geo64-cap30"]
    os.environ["BRC_KERNEL"] = "life"
    try:
        eng = Engine(instances=512, **kw)
    finally:
        os.environ.pop("BRC_KERNEL", None)
    with eng:
        eng.run()
        a = (eng.instances_result(), eng.replicas())
        eng.reset()
        eng.run()
        assert eng.last_kernel() == "life"
        b = (eng.instances_result(), eng.replicas())
    assert a == b
