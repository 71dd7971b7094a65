"""The reference's class API on top of the engine.

CPU: import paths, constructor contracts and host-side bookkeeping (no engine launch).
GPU: reference-style drivers run unchanged and print exactly what the reference's golden
fixtures say the reference delivers / decides, in the reference's per-step order."""
import os
import subprocess
import sys

import pytest

from byzantinerandomizedconsensus_amd import _lib as L
from byzantinerandomizedconsensus_amd import network
from tests import golden_io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GROUPS = golden_io.groups()


@pytest.fixture(autouse=True)
def fresh_network():
    network.reset()
    saved = network.settings()
    yield
    network.reset()
    network.configure(**saved)


def test_reference_import_paths():
    import byzantinerandomizedconsensus  # noqa: F401
    from byzantinerandomizedconsensus.base.broadcast import Broadcast, IBroadcastHandler
    from byzantinerandomizedconsensus.base.consensus import Consensus, IConsensusHandler
    from byzantinerandomizedconsensus.core.brbroadcast import BRBroadcast
    from byzantinerandomizedconsensus.core.byzantinerandomizedconsensus import ByzantineRandomizedConsensus
    assert (BRBroadcast.SEND, BRBroadcast.ECHO, BRBroadcast.READY) == (1, 2, 3)
    assert issubclass(BRBroadcast, Broadcast) and Broadcast.BUFFER_SIZE == 1024
    assert issubclass(ByzantineRandomizedConsensus, Consensus)
    assert issubclass(ByzantineRandomizedConsensus, IBroadcastHandler)
    assert (ByzantineRandomizedConsensus.NONE, ByzantineRandomizedConsensus.PHASE1,
            ByzantineRandomizedConsensus.PHASE2) == (-1, 1, 2)
    for iface in (IBroadcastHandler, IConsensusHandler, Consensus):
        with pytest.raises(TypeError):
            iface()


def test_reference_path_bebroadcast_shares_the_cluster_registry():
    # reference path core/bebroadcast.py:9; its relative `from .. import network` must land on the
    # one network module, or a second cluster registry would split the peers
    from byzantinerandomizedconsensus.core.bebroadcast import BEBroadcast
    import byzantinerandomizedconsensus.network as alias_net
    from byzantinerandomizedconsensus_amd.core import bebroadcast
    assert BEBroadcast is bebroadcast.BEBroadcast
    assert alias_net is network
    peers = _peers(4, 6300)

    class H:
        def deliver(self, message):
            pass

    nodes = [BEBroadcast(p[1], peers, H()) for p in peers]
    assert len({id(nd.cluster) for nd in nodes}) == 1
    assert nodes[0].cluster is network.cluster_for(peers)


def _peers(n, port=6000):
    return [("localhost", port + i) for i in range(n)]


def test_constructor_asserts_like_reference():
    from byzantinerandomizedconsensus_amd.core.brbroadcast import BRBroadcast
    from byzantinerandomizedconsensus_amd.core.byzantinerandomizedconsensus import ByzantineRandomizedConsensus
    with pytest.raises(AssertionError):
        BRBroadcast(3, 1, ("localhost", 6000), _peers(3), None)            # core/brbroadcast.py:29
    with pytest.raises(AssertionError):
        ByzantineRandomizedConsensus(5, 1, _peers(5, 6100), ("localhost", 6100), None)   # :20


def test_brb_sends_become_injections():
    from byzantinerandomizedconsensus_amd.core.brbroadcast import BRBroadcast
    peers = _peers(4)
    nodes = [BRBroadcast(4, 1, p, peers, None) for p in peers]
    for nd in nodes:
        nd.broadcast_listener()
    nodes[2].broadcast(BRBroadcast.SEND, "A")
    nodes[2].broadcast(BRBroadcast.SEND, "A")      # the same message again: every link carries it again
    nodes[2].broadcast(BRBroadcast.SEND, "B")
    c = nodes[0].cluster
    assert all(nd.cluster is c for nd in nodes)
    assert [(a["node"], a["kp"], a["s"], a["t"]) for a in c.actions] == [(2, 2, 0, 0), (2, 2, 0, 0), (2, 2, 1, 0)]
    assert c.key_payload == {(2, 0): "A", (2, 1): "B"}
    nodes[1].broadcast(BRBroadcast.SEND, "A")      # one reference key, a second origin: an extra SEND
    assert (c.actions[-1]["node"], c.actions[-1]["kp"], c.actions[-1]["s"]) == (1, 2, 0)
    del c.actions[-1]
    del c.actions[1]
    # user-issued ECHO / READY (base/broadcast.py:17): the payload's key, every peer addressed;
    # a payload nobody SENT is declared first under the caller's next sequence number
    nodes[1].broadcast(BRBroadcast.ECHO, "A")
    nodes[3].broadcast(BRBroadcast.READY, "C")
    nodes[3].broadcast(BRBroadcast.SEND, "C")
    acts = [(a["kind"], a.get("type", 0), a["node"], a["kp"], a["s"]) for a in c.actions[2:]]
    assert acts == [(L.INJ_MSG, BRBroadcast.ECHO, 1, 2, 0), (L.INJ_KEY, 0, 3, 3, 0),
                    (L.INJ_MSG, BRBroadcast.READY, 3, 3, 0), (L.INJ_SEND, 0, 3, 3, 0)]
    assert all(a["dst"] == 15 for a in c.actions if a["kind"] != L.INJ_KEY)
    nodes[0].broadcast(BRBroadcast.SEND, "C")      # declared by node 3, SENT by 3 and now by 0
    assert (c.actions[-1]["kind"], c.actions[-1]["node"], c.actions[-1]["kp"]) == (L.INJ_SEND, 0, 3)
    with pytest.raises(L.EngineError):
        nodes[0].broadcast(7, "D")                 # the engine carries SEND / ECHO / READY only
    with pytest.raises(ValueError):
        BRBroadcast(4, 1, ("localhost", 1), peers, None)


def test_consensus_values_and_proposals(capsys):
    from byzantinerandomizedconsensus_amd.core.byzantinerandomizedconsensus import ByzantineRandomizedConsensus
    peers = _peers(6, 6200)
    nodes = [ByzantineRandomizedConsensus(6, 1, peers, p, None) for p in peers]
    for i, nd in enumerate(nodes):
        nd.message_queue.put_nowait(i % 2)
        nd.start()
    out = capsys.readouterr().out.splitlines()
    assert out[0] == "Consensus started on ('localhost', 6200)" and out[1] == "Proposal sent on ('localhost', 6200)"
    c = nodes[0].brb.cluster
    assert c.mode == "consensus"
    assert [(a["node"], a["value"]) for a in c.actions] == [(i, 1 + i % 2) for i in range(6)]
    assert c.values.strings == ["-1", "0", "1"]
    assert nodes[3].round == 1 and nodes[3].phase == 1


def test_peer_mode_setting():
    # the shipped reference identifies peers by connection (core/brbroadcast.py:69)
    assert network.settings()["peer_mode"] == "connection"
    network.configure(peer_mode="sender")
    assert network.settings()["peer_mode"] == "sender"
    with pytest.raises(ValueError):
        network.configure(peer_mode="tcp")


def test_direct_deliver_becomes_an_injection():
    import json
    from byzantinerandomizedconsensus_amd.core.byzantinerandomizedconsensus import ByzantineRandomizedConsensus
    peers = _peers(6, 6500)
    nodes = [ByzantineRandomizedConsensus(6, 1, peers, p, None) for p in peers]
    msg = {"host": list(peers[4]), "round": 1, "phase": 1, "message": "1"}      # :48-49 layout
    nodes[2].deliver(json.dumps(msg))
    c = nodes[0].brb.cluster
    assert [(a["kind"], a["node"], a["kp"], c.values.string(a["value"])) for a in c.actions] == \
        [(L.INJ_DELIVER, 2, 4, "1")]
    with pytest.raises(L.EngineError):
        nodes[2].deliver(json.dumps(dict(msg, host=["elsewhere", 1])))
    with pytest.raises(L.EngineError):                   # the reference keys 1 and "1" apart
        nodes[2].deliver(json.dumps(dict(msg, message=1)))
    assert len(c.actions) == 1


def test_value_table_limits():
    vt = network.ValueTable()                            # three-bit ids: seven strings besides "-1"
    assert [vt.id_of(x) for x in ("-1", "a", 3, "a", "3", "b", "c", "d", "e", "f")] == [0, 1, 2, 1, 2, 3, 4, 5, 6, 7]
    with pytest.raises(L.EngineError):
        vt.id_of("g")
    vt = network.ValueTable(4)                           # two-bit ids (n in 33..64 sender peers, n > 64)
    assert [vt.id_of(x) for x in ("-1", "a", 3, "a", "3", "b")] == [0, 1, 2, 1, 2, 3]
    with pytest.raises(L.EngineError):
        vt.id_of("c")


def test_cluster_value_table_width():
    """Clusters get three-bit value ids where their kernel keeps them (include/brc.h)."""
    network.reset()
    try:
        for n, pm, cap in ((7, "connection", 8), (16, "sender", 8), (40, "connection", 8), (40, "sender", 8),
                           (70, "connection", 4)):
            c = network.Cluster(tuple(("localhost", 9000 + i) for i in range(n)), dict(network.settings(), peer_mode=pm))
            assert c.values.cap == cap, (n, pm)
    finally:
        network.reset()


def test_repeat_send_on_general_and_wide_clusters():
    """33..64 nodes with sender peers run the narrow kernel's general form (brc.h BRC_FLAG_GENERAL_KEYS):
    a payload SENT again by its node or by a second origin is one key with extra SENDs, as on <= 32
    nodes (the engine drops a sender's repeat on every link it used, as the reference network does).
    Above 64 nodes (the wide kernel: one SEND per key) a repeat is refused."""
    from byzantinerandomizedconsensus_amd.core.brbroadcast import BRBroadcast
    network.reset()
    try:
        network.configure(peer_mode="sender")
        peers = _peers(40, 7100)
        nodes = [BRBroadcast(40, 13, p, peers, None) for p in peers]
        nodes[5].broadcast(BRBroadcast.SEND, "A")
        nodes[5].broadcast(BRBroadcast.SEND, "A")        # the same node again: an extra SEND, dropped by the engine
        nodes[6].broadcast(BRBroadcast.SEND, "A")        # a second origin: one key, two SENDs
        c = nodes[0].cluster
        assert [(a["node"], a["kp"], a["s"]) for a in c.actions] == [(5, 5, 0), (5, 5, 0), (6, 5, 0)]
        network.reset()
        network.configure(peer_mode="connection")        # connection peers: a repeat travels again
        peers = _peers(70, 7200)
        nodes = [BRBroadcast(70, 23, p, peers, None) for p in peers]
        nodes[5].broadcast(BRBroadcast.SEND, "A")
        with pytest.raises(L.EngineError):
            nodes[5].broadcast(BRBroadcast.SEND, "A")    # the wide kernel models one SEND per key
    finally:
        network.configure(peer_mode="connection")
        network.reset()


def test_step_event_order():
    evs = [(L.EV_DELIVER, 2, 0, 0), (L.EV_DELIVER, 0, 3, 0), (L.EV_DELIVER, 0, 1, 1), (L.EV_DELIVER, 0, 1, 0)]
    assert network.order_step_events(evs) == [(1, 0, 1, 0), (1, 0, 1, 1), (1, 0, 3, 0), (1, 2, 0, 0)]


# ---------------------------------------------------------------------------------- GPU
def _run_driver(name):
    env = dict(os.environ, PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "drivers", name)], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    return out.stdout.splitlines()


@pytest.mark.gpu
def test_brb_driver_unchanged_matches_reference():
    # FIFO n=4 f=1, every node SENDs at once -> 16 deliveries (connection peers,
    # as the shipped reference runs the driver)
    case = GROUPS["conn_brb_fifo_n4"][0]
    exp = ["TEST %d" % (kp + 1) for (_t, _node, kp, _s) in case["result"]["raw_order"]["deliver"]]
    assert _run_driver("brb_driver.py") == exp


@pytest.mark.gpu
def test_brc_driver_unchanged_matches_reference():
    case = GROUPS["conn_cons_brc_test_n6"][0]
    head = []
    for i in range(6):
        head += ["Consensus started on ('localhost', %d)" % (5555 + i), "Proposal sent on ('localhost', %d)" % (5555 + i)]
    exp = head + ["Consensus protocol decided on message: " + v for (_t, _n, _r, v) in case["result"]["raw_order"]["decide"]]
    assert _run_driver("brc_driver.py") == exp


@pytest.mark.gpu
@pytest.mark.parametrize("group", ["brb_uniform_n10", "conn_brb_uniform_n10"])
def test_upcall_order_and_steps_match_reference(group):
    """Every upcall at the step and in the per-step order the reference produces (uniform
    random delays: deliveries of several keys interleave across steps), with sender and with
    connection peer identity."""
    from byzantinerandomizedconsensus_amd.base.broadcast import IBroadcastHandler
    from byzantinerandomizedconsensus_amd.core.brbroadcast import BRBroadcast
    for case in GROUPS[group][:3]:
        sp = case["spec"]
        network.reset()
        network.configure(delay_model=sp["delay_model"], delay_max=sp["dmax"], seed=sp["seed"],
                          instance_id=sp["g"], peer_mode=sp.get("peer_mode", "sender"))
        got = []

        class H(IBroadcastHandler):
            def __init__(self, i):
                self.i = i

            def deliver(self, message):
                got.append([cluster.t, self.i, message])

        peers = _peers(sp["n"], 6300)
        nodes = [BRBroadcast(sp["n"], sp["f"], p, peers, H(i)) for i, p in enumerate(peers)]
        cluster = nodes[0].cluster
        for a in sp["actions"]:
            assert a["kind"] == "brb_send" and a["t"] == 0
            nodes[a["node"]].broadcast(BRBroadcast.SEND, a["payload"])
        cluster.run()
        # the reference's own upcall order (raw_order, recorded as it happened), not a sorted list
        exp = [[t, node, "TEST %d.%d" % (kp + 1, s)] for (t, node, kp, s) in case["result"]["raw_order"]["deliver"]]
        assert got == exp


@pytest.mark.gpu
def test_direct_deliver_calls_match_oracle():
    """ByzantineRandomizedConsensus.deliver(message) called by the program (the reference's :53
    entry point used directly): the decide upcalls equal the oracle's run of the same calls."""
    import json
    from byzantinerandomizedconsensus_amd.base.consensus import IConsensusHandler
    from byzantinerandomizedconsensus_amd.core.byzantinerandomizedconsensus import ByzantineRandomizedConsensus
    from oracle import oracle
    from tests.golden import specs as S
    props = [1, 2, 1, 2, 1, 3]
    for g in range(3):
        acts = [dict(t=0, kind="deliver", node=(i * 5 + g) % 6, kp=(3 * i + g + 1) % 6, value=(i + g) % 4)
                for i in range(9)]
        sp = S.cons_spec(6, 1, 0xDE30, 0, 1, g, round_cap=2, proposals=props, extra=acts)
        exp = oracle.run(sp)
        network.reset()
        network.configure(delay_model="const", delay_max=1, seed=sp["seed"], instance_id=g, round_cap=2)
        got = []

        class U(IConsensusHandler):
            def __init__(self, i):
                self.i = i

            def decide(self, message):
                got.append([cluster.t, self.i, message])

        peers = _peers(6, 6600)
        nodes = [ByzantineRandomizedConsensus(6, 1, peers, p, U(i)) for i, p in enumerate(peers)]
        cluster = nodes[0].brb.cluster
        for i, nd in enumerate(nodes):
            nd.message_queue.put_nowait(S.VALUES[props[i]])
            nd.start()
        for a in acts:
            nodes[a["node"]].deliver(json.dumps({"host": list(peers[a["kp"]]), "round": 1, "phase": 1,
                                                 "message": S.VALUES[a["value"]]}))
        cluster.run()
        assert got == [[t, node, v] for (t, node, _r, v) in sorted(exp["events"]["decide"])], g


@pytest.mark.gpu
@pytest.mark.parametrize("group", ["brb_usermsg_n7", "conn_brb_usermsg_n7", "brb_multisend_n40"])
def test_user_echo_ready_broadcasts_match_reference(group):
    """Honest nodes' user code issues ECHO / READY broadcasts (base/broadcast.py:17): an early ECHO
    of a SENT payload, ECHO / READY of payloads nobody SENDs (f + 1 READYs -> amplification ->
    delivery without a SEND), a READY that blocks a node's own (K3).  Upcalls at the steps and in
    the order the reference issued them, in both peer modes."""
    from byzantinerandomizedconsensus_amd.base.broadcast import IBroadcastHandler
    from byzantinerandomizedconsensus_amd.core.brbroadcast import BRBroadcast
    for case in GROUPS[group]:
        sp = case["spec"]
        network.reset()
        network.configure(delay_model=sp["delay_model"], delay_max=sp["dmax"], seed=sp["seed"],
                          instance_id=sp["g"], peer_mode=sp.get("peer_mode", "sender"))
        got = []

        class H(IBroadcastHandler):
            def __init__(self, i):
                self.i = i

            def deliver(self, message):
                got.append([cluster.t, self.i, message])

        peers = _peers(sp["n"], 6700)
        nodes = [BRBroadcast(sp["n"], sp["f"], p, peers, H(i)) for i, p in enumerate(peers)]
        cluster = nodes[0].cluster
        payload = {}
        for a in sp["actions"]:
            assert a["t"] == 0
            payload[(a["kp"], a["s"])] = a["payload"]
            nodes[a["node"]].broadcast(BRBroadcast.SEND if a["kind"] == "brb_send" else a["type"], a["payload"])
        assert {v: k for k, v in payload.items()} == cluster.payload_key     # the spec's keys are the API's
        cluster.run()
        exp = [[t, node, payload[(kp, s)]] for (t, node, kp, s) in case["result"]["raw_order"]["deliver"]]
        assert got == exp, sp["name"]


@pytest.mark.gpu
@pytest.mark.parametrize("group", ["cons_values_n7", "conn_cons_values_n7", "cons_values_n40"])
def test_more_than_three_proposal_strings_match_reference(group):
    """Seven proposal strings besides "-1" (three-bit value ids): the decide upcalls equal the
    reference's (tests/golden/<group>.json, made by the reference classes), both peer modes; five
    strings at n = 40 with sender peers (the general form, brc.h BRC_FLAG_GENERAL_KEYS)."""
    from byzantinerandomizedconsensus_amd.base.consensus import IConsensusHandler
    from byzantinerandomizedconsensus_amd.core.byzantinerandomizedconsensus import ByzantineRandomizedConsensus
    for case in GROUPS[group]:
        sp = case["spec"]
        network.reset()
        network.configure(delay_model=sp["delay_model"], delay_max=sp["dmax"], seed=sp["seed"], instance_id=sp["g"],
                          round_cap=sp["round_cap"], peer_mode=sp.get("peer_mode", "sender"))
        got = []

        class U(IConsensusHandler):
            def __init__(self, i):
                self.i = i

            def decide(self, message):
                got.append([cluster.t, self.i, message])

        n = sp["n"]
        peers = _peers(n, 6700)
        nodes = [ByzantineRandomizedConsensus(n, sp["f"], peers, p, U(i)) for i, p in enumerate(peers)]
        cluster = nodes[0].brb.cluster
        for a in sp["actions"]:
            assert a["kind"] == "propose" and a["t"] == 0
            nodes[a["node"]].message_queue.put_nowait(sp["values"][a["value"]])
        for nd in nodes:
            nd.start()
        status = cluster.run()
        assert status == case["result"]["status"], sp["name"]
        assert got == [[t, node, v] for (t, node, _r, v) in sorted(case["result"]["events"]["decide"])], sp["name"]


def test_repeated_send_refused_where_the_kernel_keeps_one_send_per_key():
    """Clusters above 64 nodes (wide kernel) model one SEND per key: a payload SENT again, or by a
    second node, raises before any engine call; up to 64 nodes it is an extra SEND."""
    from byzantinerandomizedconsensus_amd.core.brbroadcast import BRBroadcast
    for n, pm, ok in ((40, "sender", True), (40, "connection", True), (70, "connection", False), (16, "sender", True)):
        network.reset()
        network.configure(peer_mode=pm)
        try:
            peers = _peers(n, 7000)
            nodes = [BRBroadcast(n, (n - 1) // 3, p, peers, None) for p in peers[:3]]
            nodes[0].broadcast(BRBroadcast.SEND, "P")
            if ok:
                nodes[1].broadcast(BRBroadcast.SEND, "P")
                assert len(nodes[0].cluster.actions) == 2
            else:
                with pytest.raises(L.EngineError):
                    nodes[1].broadcast(BRBroadcast.SEND, "P")
        finally:
            network.reset()
            network.configure(peer_mode="connection")
