"""GPU parity of best-effort broadcast (BRC_MODE_BEB, SURVEY §8 F4: core/bebroadcast.py as
intended) against the C oracle, which tests/test_spec_model.py pins to the pure-Python model: the
broadcast alone, and the reference's consensus running over it (its consensus_instance.deliver,
core/bebroadcast.py:42).  Plus the reference-shaped class API (``BEBroadcast``)."""
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


@pytest.mark.parametrize("n,model,dmax", [(4, 1, 4), (7, 3, 6), (16, 2, 8), (64, 1, 3), (100, 3, 16)])
def test_beb_vs_oracle(runner, n, model, dmax):
    rng = random.Random(n + dmax)
    specs = []
    for g in range(12 if n <= 64 else 2):
        origins = rng.sample(range(n), min(n, 6))
        sends = [(rng.randint(0, 5), o, q) for o in origins for q in range(rng.randint(1, 2))]
        sp = S.beb_spec(n, 0xBEB + n, model, dmax, 20 + g, sends)
        sp["name"] = "beb%d/%d" % (n, g)
        specs.append(sp)
    _compare(runner, specs)


@pytest.mark.parametrize("n,f,model,dmax,rcap", [(4, 1, 1, 4, 3), (7, 2, 2, 3, 2), (16, 5, 0, 1, 3),
                                                  (64, 21, 2, 8, 2), (96, 31, 1, 4, 1)])
def test_consensus_over_beb_vs_oracle(runner, n, f, model, dmax, rcap):
    specs = []
    for g in range(16 if n <= 16 else 2):
        sp = S.beb_cons_spec(n, f, 0xBEBC + n, model, dmax, 40 + g, round_cap=rcap)
        sp["name"] = "bebc%d/%d" % (n, g)
        specs.append(sp)
    got = _compare(runner, specs)
    assert any(r["status"] == "done" for r in got)


def test_beb_class_api_delivers_every_payload():
    """BEBroadcast(host_port, peer_list, consensus_instance) as the reference declares it: every
    node hands every broadcast payload to its consensus_instance.deliver."""
    from byzantinerandomizedconsensus_amd import network
    from byzantinerandomizedconsensus_amd.core.bebroadcast import BEBroadcast
    network.reset()
    peers = [("localhost", 9100 + i) for i in range(5)]

    class Sink:
        def __init__(self):
            self.got = []

        def deliver(self, message):
            self.got.append(message)

    sinks = [Sink() for _ in peers]
    nodes = [BEBroadcast(p[1], peers, s) for p, s in zip(peers, sinks)]
    for nd in nodes:
        nd.broadcast_listener()
    for i, nd in enumerate(nodes):
        nd.broadcast(BEBroadcast.MessageType.SEND, "BEB %d" % i)
    network.run_all()
    for s in sinks:
        assert s.got == ["BEB %d" % i for i in range(5)]
    network.reset()
