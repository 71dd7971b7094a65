"""Workload specs shared by the golden generator, the oracle tests and the GPU parity tests.

A spec is a plain dict (JSON-able):

    n, f, mode ('brb' | 'consensus'), nv (key variants per origin), seed, delay_model
    (0 const, 1 uniform, 2 slow-set, 3 geometric), dmax, dconst, g (global instance id),
    byzantine (replica ids that run no code), values (value id -> string, id 0 == "-1"),
    round_cap, step_cap, actions.

actions (each performed after step ``t`` is processed, messages stamped ``t``):
    {"kind": "propose",  "t", "node", "value"}                 ByzantineRandomizedConsensus.start()
    {"kind": "brb_send", "t", "node", "kp", "s", "payload"}     BRBroadcast.broadcast(SEND, payload)
    {"kind": "byz_key",  "t", "kp", "s", "value"[, "payload"]}   declare a Byzantine key
    {"kind": "byz",      "t", "src", "type", "kp", "s", "dst"}   raw Byzantine message(s)
    {"kind": "brb_msg",  "t", "node", "type", "kp", "s", "payload"}
                                      an honest node's own BRBroadcast.broadcast(ECHO | READY, payload)
                                      (base/broadcast.py:17): the key is declared on first use
"""
import copy
import random

VALUES = ["-1", "0", "1", "3"]
# seven proposal strings besides "-1": the three-bit value ids of the narrow kernels (include/brc.h
# brc_injection.value); the reference keys its value table by these strings
# (core/byzantinerandomizedconsensus.py:57-60)
VALUES8 = ["-1", "0", "1", "3", "alpha", "beta", "gamma", "delta"]
SEND, ECHO, READY = 1, 2, 3


def _sched(n, f, seed, model, dmax, dconst=1):
    from oracle.schedule import Schedule
    return Schedule(n, f, seed, model, dmax, dconst)


def brb_spec(n, f, seed, model, dmax, g, sends, dconst=1, byzantine=(), extra=(), step_cap=10000,
             peer_mode="sender"):
    """sends: list of (t, origin, seq)."""
    acts = [dict(t=t, kind="brb_send", node=o, kp=o, s=q, payload="TEST %d.%d" % (o + 1, q))
            for (t, o, q) in sends]
    acts += list(extra)
    return dict(n=n, f=f, mode="brb", nv=1, seed=seed, delay_model=model, dmax=dmax, dconst=dconst,
                g=g, byzantine=list(byzantine), values=VALUES, round_cap=0, step_cap=step_cap,
                actions=acts, peer_mode=peer_mode)


def cons_spec(n, f, seed, model, dmax, g, round_cap=2, proposals=None, byzantine=(), nv=1,
              starts=None, dconst=1, extra=(), step_cap=4000, peer_mode="sender"):
    """proposals: None -> Philox Bernoulli(1/2) value ids; or a list of value ids.
    starts: None -> every honest replica proposes at t=0; or a list of start times."""
    sch = _sched(n, f, seed, model, dmax, dconst)
    acts = []
    for i in range(n):
        if i in byzantine:
            continue
        v = sch.proposal_id(g, i) if proposals is None else proposals[i]
        acts.append(dict(t=0 if starts is None else starts[i], kind="propose", node=i, value=v))
    acts += list(extra)
    return dict(n=n, f=f, mode="consensus", nv=nv, seed=seed, delay_model=model, dmax=dmax,
                dconst=dconst, g=g, byzantine=list(byzantine), values=VALUES, round_cap=round_cap,
                step_cap=step_cap, actions=acts, peer_mode=peer_mode)


def spec_cons_spec(n, f, seed, model, dmax, g, round_cap=1, window=4, coin_seed=0xC01D, **kw):
    """BRC_MODE_SPEC consensus (tests/spec_model.py): the intended protocol, common coin keyed
    (coin_seed, g, round); ``window`` = phase indices a replica buffers (the engine's key window)."""
    sp = cons_spec(n, f, seed, model, dmax, g, round_cap=round_cap, **kw)
    sp.update(mode="spec", window=window, coin_seed=coin_seed)
    return sp


def spec_brb_spec(n, f, seed, model, dmax, g, sends, window=4, **kw):
    """BRC_MODE_SPEC broadcast only (Bracha-correct BRB)."""
    sp = brb_spec(n, f, seed, model, dmax, g, sends, **kw)
    sp.update(mode="spec_brb", window=window, coin_seed=0)
    return sp


def beb_spec(n, seed, model, dmax, g, sends, **kw):
    """Best-effort broadcast only (core/bebroadcast.py as intended; BRC_MODE_BEB)."""
    sp = brb_spec(n, 0, seed, model, dmax, g, sends, **kw)
    sp.update(mode="beb")
    return sp


def beb_cons_spec(n, f, seed, model, dmax, g, round_cap=1, **kw):
    """The reference's consensus over best-effort broadcast (its consensus_instance.deliver)."""
    sp = cons_spec(n, f, seed, model, dmax, g, round_cap=round_cap, **kw)
    sp.update(mode="beb_consensus")
    return sp


def user_msg_actions():
    """Honest nodes issue ECHO / READY broadcasts from user code (base/broadcast.py:17 accepts any
    type): an early ECHO of a SENT payload, an ECHO of a payload nobody SENDs, READYs of a fresh
    payload from f + 1 nodes (amplification, then delivery without any SEND), and a READY of a SENT
    payload.  Keys follow the class API's allocation: a payload's key is (first user, that node's
    next sequence number)."""
    E, R = ECHO, READY
    return [dict(t=0, kind="brb_msg", node=5, type=E, kp=0, s=0, payload="TEST 1.0"),
            dict(t=0, kind="brb_msg", node=4, type=E, kp=4, s=0, payload="USER E"),
            dict(t=0, kind="brb_msg", node=4, type=R, kp=4, s=1, payload="USER R"),
            dict(t=0, kind="brb_msg", node=5, type=R, kp=4, s=1, payload="USER R"),
            dict(t=0, kind="brb_msg", node=6, type=R, kp=4, s=1, payload="USER R"),
            dict(t=0, kind="brb_msg", node=6, type=R, kp=1, s=0, payload="TEST 2.0")]


def equivocation_actions(n, byzantine, nv=2, t_send=0, t_er=1):
    """SURVEY §8(d) cfg3 pattern: each Byzantine replica b SENDs value "0" to even
    destinations and "1" to odd ones, then ECHOes and READYs both keys to everyone."""
    even = sum(1 << d for d in range(0, n, 2))
    odd = sum(1 << d for d in range(1, n, 2))
    allm = (1 << n) - 1
    acts = []
    for b in byzantine:
        for v in range(2):
            acts.append(dict(t=t_send, kind="byz_key", kp=b * nv + v, s=0, value=1 + v))
        acts.append(dict(t=t_send, kind="byz", src=b, type=SEND, kp=b * nv, s=0, dst=even))
        acts.append(dict(t=t_send, kind="byz", src=b, type=SEND, kp=b * nv + 1, s=0, dst=odd))
        for v in range(2):
            acts.append(dict(t=t_er, kind="byz", src=b, type=ECHO, kp=b * nv + v, s=0, dst=allm))
            acts.append(dict(t=t_er, kind="byz", src=b, type=READY, kp=b * nv + v, s=0, dst=allm))
    return acts


def deliver_actions(n, seed, count=None, nval=4):
    """Direct deliver() calls: replica `node` is handed host `kp`'s message with value id `value`
    (0 .. nval-1) at step t (an action: after step t's messages)."""
    rng = random.Random(seed)
    return [dict(t=rng.randint(0, 8), kind="deliver", node=rng.randrange(n), kp=rng.randrange(n),
                 value=rng.randint(0, nval - 1)) for _ in range(count or 2 * n)]


def values8_specs():
    """More than three distinct proposal strings (VALUES8): majorities of one new string, splits
    that end in "-1", and direct deliver() calls carrying every id, in both peer modes."""
    G = {}
    pats = [[4, 4, 4, 4, 4, 5, 6], [7, 7, 7, 7, 7, 6, 5], [4, 5, 6, 7, 4, 5, 6], [6, 6, 6, 6, 6, 6, 4],
            [5, 5, 5, 5, 5, 7, 7], [7] * 7]
    models = ((0, 1), (1, 3), (2, 4), (0, 2), (0, 1), (3, 5))
    for pm, pre in (("sender", ""), ("connection", "conn_")):
        G[pre + "cons_values_n7"] = [dict(cons_spec(7, 1, 0x7A10 + g, m, d, g, round_cap=2, proposals=pats[g],
                                                    peer_mode=pm), values=VALUES8)
                                     for g, (m, d) in enumerate(models)]
    rng = random.Random(0x7A16)
    G["cons_values_deliver_n16"] = [dict(cons_spec(16, 3, 0x7A20 + g, m, d, g, round_cap=2,
                                                   proposals=[rng.choice((4, 5, 6, 7, 4, 4)) for _ in range(16)],
                                                   extra=deliver_actions(16, 0x7A30 + g, nval=8)), values=VALUES8)
                                    for g, (m, d) in enumerate(((0, 1), (0, 2), (1, 4), (2, 3)))]
    return G


def _kat(n, f, seq, byz_nodes, key=(1, 0), name=""):
    """Known-answer scenario: scripted Byzantine peers feed one honest node (node 0)
    the message sequence `seq` = [(t, type, src[, dst_mask])...] for one BRB key."""
    allm = (1 << n) - 1
    kp, s = key
    acts = [dict(t=0, kind="byz_key", kp=kp, s=s, value=0, payload="KAT %s" % name)]
    for item in seq:
        t, typ, src = item[:3]
        dst = item[3] if len(item) > 3 else allm
        acts.append(dict(t=t, kind="byz", src=src, type=typ, kp=kp, s=s, dst=dst))
    return dict(n=n, f=f, mode="brb", nv=1, seed=0, delay_model=0, dmax=1, dconst=1, g=0,
                byzantine=list(byz_nodes), values=VALUES, round_cap=0, step_cap=200, actions=acts)


def kat_specs():
    """SURVEY §4 K1-K7, K12 restated as scripted scenarios (node 0 honest, delay 1)."""
    S, E, R = SEND, ECHO, READY
    k = {}
    # K1: S, E1, E2, E3, R1, R2, R3 one per step
    k["K1"] = _kat(4, 1, [(0, S, 1, 1), (1, E, 1), (2, E, 2), (3, E, 3), (4, R, 1), (5, R, 2), (6, R, 3)],
                   [1, 2, 3], name="K1")
    # K2: ECHO before SEND: the SEND is then ignored (no ECHO from node 0)
    k["K2"] = _kat(4, 1, [(0, E, 1), (1, S, 1, 1), (2, E, 2), (3, E, 3), (4, R, 1), (5, R, 2), (6, R, 3)],
                   [1, 2, 3], name="K2")
    # K3: READY before the echo quorum blocks node 0's own READY
    k["K3"] = _kat(4, 1, [(0, S, 1, 1), (1, R, 1), (2, E, 1), (3, E, 2), (4, E, 3), (5, R, 2), (6, R, 3)],
                   [1, 2, 3], name="K3")
    # K4 (n=7, f=2): READYs only -> amplification, then delivery
    k["K4"] = _kat(7, 2, [(0, R, 1), (1, R, 2), (2, R, 3), (3, R, 4), (4, R, 5), (5, R, 6)],
                   [1, 2, 3, 4, 5, 6], name="K4")
    # K5: duplicate ECHOs from one sender change nothing (dropped by the network)
    k["K5"] = _kat(4, 1, [(0, S, 1, 1), (1, E, 1), (2, E, 1), (3, E, 1), (4, E, 2)], [1, 2, 3], name="K5")
    # K7: after DELIVER everything is ignored (fresh ECHO/READY from node 4 arrive afterwards).
    # (A second SEND of one key from another sender is not modelled by the engine: brc_inject
    # rejects it with BRC_E_UNSUPPORTED; honest nodes never send it.)
    k["K7"] = _kat(5, 1, [(0, S, 1, 1), (1, E, 1), (1, E, 2), (1, E, 3), (2, R, 1), (2, R, 2), (2, R, 3),
                          (5, E, 4), (6, R, 4)], [1, 2, 3, 4], name="K7")
    # K12 (n=7, f=2): three READYs then silence: node 0 amplifies; its own READY returns
    k["K12"] = _kat(7, 2, [(0, R, 1), (1, R, 2), (2, R, 3)], [1, 2, 3, 4, 5, 6], name="K12")
    # same-step mix: S, E and R for one key arriving together
    k["MIX"] = _kat(4, 1, [(0, S, 1), (0, E, 1), (0, E, 2), (0, E, 3), (1, R, 1), (1, R, 2), (1, R, 3)],
                    [1, 2, 3], name="MIX")
    # K6: two payloads from one origin are two independent keys (equivocation undetected)
    k6 = _kat(4, 1, [(0, S, 1, 1), (1, E, 2), (2, E, 3)], [1, 2, 3], key=(1, 0), name="K6a")
    k6["actions"] += [dict(t=0, kind="byz_key", kp=1, s=1, value=0, payload="KAT K6b"),
                      dict(t=0, kind="byz", src=1, type=SEND, kp=1, s=1, dst=1),
                      dict(t=1, kind="byz", src=2, type=ECHO, kp=1, s=1, dst=15),
                      dict(t=2, kind="byz", src=3, type=ECHO, kp=1, s=1, dst=15)]
    k["K6"] = k6
    for name, sp in k.items():
        sp["name"] = name
    return k


def cons_kat_specs():
    """K8-K11: consensus windows fed by scripted (Byzantine-origin) keys."""
    out = {}
    n, f = 6, 1
    allm = (1 << n) - 1

    def deliver_key(acts, b, variant, s, value, t, nv):
        # a key that every node delivers: Byzantine origin b, SEND + ECHO + READY from the
        # Byzantine coalition (nodes 2..5), enough to pass every threshold.
        kp = b * nv + variant
        acts.append(dict(t=t, kind="byz_key", kp=kp, s=s, value=value))
        acts.append(dict(t=t, kind="byz", src=b, type=SEND, kp=kp, s=s, dst=allm))
        for src in (2, 3, 4, 5):
            acts.append(dict(t=t, kind="byz", src=src, type=ECHO, kp=kp, s=s, dst=allm))
        for src in (2, 3, 4, 5):
            acts.append(dict(t=t + 1, kind="byz", src=src, type=READY, kp=kp, s=s, dst=allm))

    # K10: six deliveries all claiming host 2 -> value_count counts deliveries, hosts dedup
    acts = []
    for j in range(6):
        deliver_key(acts, 2, j % 2, j // 2, 1 + (j % 2), 0, 2)
    sp = cons_spec(n, f, 0, 0, 1, 0, round_cap=1, proposals=[1, 1, 1, 1, 1, 1], byzantine=[2, 3, 4, 5],
                   nv=2, extra=acts, step_cap=60)
    sp["name"] = "K10"
    out["K10"] = sp
    # K11: round 99 / phase 2 keys count in the current window (round/phase fields ignored)
    acts = []
    for j, b in enumerate((2, 3, 4, 5)):
        deliver_key(acts, b, 0, 2 * 98 + 1, 2, 0, 1)
    sp = cons_spec(n, f, 0, 0, 1, 0, round_cap=1, proposals=[1, 1, 1, 1, 1, 1], byzantine=[2, 3, 4, 5],
                   nv=1, extra=acts, step_cap=60)
    sp["name"] = "K11"
    out["K11"] = sp
    return out


def scenario_groups():
    """name -> list of specs.  Sizes chosen so the reference harness finishes in seconds."""
    G = {}
    allsends4 = [(0, i, 0) for i in range(4)]
    G["brb_fifo_n4"] = [brb_spec(4, 1, 1, 0, 1, 0, allsends4)]
    G["brb_uniform_n4"] = [brb_spec(4, 1, 0x5EED0002, 1, 4, g, allsends4) for g in range(30)]
    G["brb_geometric_n7"] = [brb_spec(7, 2, 77, 3, 6, g, [(0, i, 0) for i in range(7)]) for g in range(8)]
    G["brb_uniform_n10"] = [brb_spec(10, 3, 1010, 1, 3, g, [(0, i, 0) for i in range(10)]) for g in range(6)]
    G["brb_slowset_n16"] = [brb_spec(16, 5, 0x5EED0004, 2, 8, g, [(0, i, 0) for i in range(16)])
                            for g in range(3)]
    G["brb_staggered_n5"] = [brb_spec(5, 1, 55, 1, 3, g, [(0, 0, 0), (2, 1, 0), (2, 0, 1), (7, 3, 0), (9, 4, 0),
                                                         (9, 0, 2), (30, 2, 0)]) for g in range(8)]
    G["brb_byz_n7"] = [brb_spec(7, 2, 99, 1, 4, g, [(0, i, 0) for i in range(5)], byzantine=[5, 6],
                                extra=[dict(t=0, kind="byz_key", kp=5, s=0, value=0, payload="BYZ 5"),
                                       dict(t=0, kind="byz", src=5, type=SEND, kp=5, s=0, dst=0b0010101),
                                       dict(t=1, kind="byz", src=5, type=ECHO, kp=5, s=0, dst=127),
                                       dict(t=1, kind="byz", src=6, type=ECHO, kp=5, s=0, dst=127),
                                       dict(t=2, kind="byz", src=6, type=READY, kp=5, s=0, dst=127),
                                       dict(t=1, kind="byz", src=6, type=READY, kp=0, s=0, dst=127)])
                       for g in range(8)]
    G["kat"] = list(kat_specs().values()) + list(cons_kat_specs().values())
    G["cons_brc_test_n6"] = [cons_spec(6, 1, 3, 0, 1, 0, round_cap=3, proposals=[3] * 6)]
    G["cons_staggered_n6"] = [cons_spec(6, 1, 6, 1, 3, g, round_cap=2, proposals=[3] * 6,
                                        starts=[0, 5, 5, 12, 20, 21]) for g in range(4)]
    G["cons_uniform_n4"] = [cons_spec(4, 1, 0x5EED0002, 1, 4, g, round_cap=2) for g in range(20)]
    G["cons_const_n6"] = [cons_spec(6, 1, 16, 0, 1, g, round_cap=3) for g in range(6)]
    G["cons_uniform_n6"] = [cons_spec(6, 1, 61, 1, 4, g, round_cap=2) for g in range(16)]
    G["cons_slowset_n7"] = [cons_spec(7, 2, 71, 2, 4, g, round_cap=3) for g in range(8)]
    G["cons_geometric_n10"] = [cons_spec(10, 3, 103, 3, 5, g, round_cap=2) for g in range(6)]
    byz16 = list(range(11, 16))
    G["cons_equivocate_n16"] = [cons_spec(16, 5, 0x5EED0003, m, d, g, round_cap=1, byzantine=byz16, nv=2,
                                          extra=equivocation_actions(16, byz16))
                                for (m, d) in ((1, 4), (2, 4), (0, 1)) for g in range(2)]
    G["cons_slowset_n16"] = [cons_spec(16, 5, 0x5EED0004, 2, 8, g, round_cap=2) for g in range(3)]
    # many rounds of the reference protocol under the slow-set schedule: its phase leakage keeps up
    # to 13 phase indices of one origin in flight by round 8 (key_window: the engine window to use)
    G["cons_slowset_n16_r8"] = [dict(cons_spec(16, 5, 0x5EED0004, 2, 8, g, round_cap=8), key_window=16)
                                for g in range(3)]
    # SURVEY cfg4's round cap 64 (at n = 16): by round 64 up to 99 phase indices of one origin are in
    # flight (oracle-measured), so the engine runs it with a key window of 128
    G["cons_slowset_n16_r64"] = [dict(cons_spec(16, 5, 0x5EED0004, 2, 8, g, round_cap=64), key_window=128)
                                 for g in range(2)]
    G["cons_slowset_n64"] = [cons_spec(64, 21, 0x5EED0004, 2, 8, g, round_cap=1) for g in range(1)]
    # large committees (the wide kernel, n > 64)
    G["brb_uniform_n100"] = [brb_spec(100, 33, 0x5EED0005, 1, 4, g, [(0, 0, 0), (0, 57, 0), (3, 99, 0), (5, 0, 1)])
                             for g in range(2)]
    G["brb_geometric_n256"] = [brb_spec(256, 85, 0x5EED0005, 3, 16, g, [(0, 7, 0), (2, 200, 0)]) for g in range(1)]
    G["brb_slowset_n256"] = [brb_spec(256, 85, 0x5EED0005, 2, 8, g, [(0, 130, 0)]) for g in range(1)]
    G["cons_uniform_n70"] = [cons_spec(70, 23, 0x5EED0005, 1, 4, g, round_cap=1) for g in range(1)]
    G["cons_slowset_n70"] = [cons_spec(70, 23, 0x5EED0005, 2, 8, g, round_cap=1) for g in range(1)]
    # reference-protocol consensus on the wide kernel's committees (SURVEY §8(d) cfg5 sizes)
    G["cons_slowset_n128"] = [cons_spec(128, 42, 0x5EED0005, 2, 8, g, round_cap=1) for g in range(1)]
    G["cons_slowset_n256"] = [dict(cons_spec(256, 85, 0x5EED0005, 2, 8, g, round_cap=1), keep_wire=False)
                              for g in range(1)]
    # connection-identity peers (core/brbroadcast.py:69, the reference's local-test mode)
    G["conn_kat"] = [clone(sp, peer_mode="connection", name=sp["name"] + "-conn")
                     for sp in kat_specs().values()]
    G["conn_brb_slowset_n7"] = [brb_spec(7, 2, 0xC0AA, 2, 5, g, [(0, i, 0) for i in range(7)], peer_mode="connection")
                                for g in range(4)]
    G["conn_cons_slowset_n7"] = [cons_spec(7, 2, 0xC0AB, 2, 4, g, round_cap=2, peer_mode="connection")
                                 for g in range(6)]
    G["conn_cons_uniform_n6"] = [cons_spec(6, 1, 0xC0AC, 1, 3, g, round_cap=2, peer_mode="connection")
                                 for g in range(8)]
    G["conn_cons_byz_n16"] = [cons_spec(16, 5, 0x5EED0003, m, d, g, round_cap=1, byzantine=list(range(11, 16)), nv=2,
                                        extra=equivocation_actions(16, list(range(11, 16))), peer_mode="connection")
                              for (m, d) in ((1, 4), (2, 4)) for g in range(2)]
    # ByzantineRandomizedConsensus.deliver(message) called directly (core/byzantinerandomizedconsensus.py:53):
    # extra values from chosen hosts, some before the replica's own proposal (phase 0: counted only)
    G["cons_deliver_n6"] = [cons_spec(6, 1, 0xDE10, m, d, g, round_cap=2, starts=[0, 0, 0, 3, 0, 6],
                                      extra=deliver_actions(6, 0xDE10 + g)) for (m, d) in ((0, 1), (1, 3)) for g in range(3)]
    G["cons_deliver_n16"] = [cons_spec(16, 3, 0xDE20, 2, 4, g, round_cap=1, extra=deliver_actions(16, 0xDE20 + g))
                             for g in range(2)]
    # ECHO / READY broadcasts issued by honest nodes' user code (base/broadcast.py:17), both peer modes
    G["brb_usermsg_n7"] = [brb_spec(7, 2, 0x05E1, m, d, g, [(0, i, 0) for i in range(4)], extra=user_msg_actions())
                           for (m, d) in ((0, 1), (1, 3)) for g in range(3)]
    G["conn_brb_usermsg_n7"] = [clone(sp, peer_mode="connection", name="conn_brb_usermsg_n7/%d" % i)
                                for i, sp in enumerate(G["brb_usermsg_n7"])]
    # the reference's own drivers (test/brb_test.py, test/brc_test.py) as they run: connection peers
    G["conn_brb_fifo_n4"] = [clone(G["brb_fifo_n4"][0], peer_mode="connection", name="conn_brb_fifo_n4/0")]
    G["conn_cons_brc_test_n6"] = [clone(G["cons_brc_test_n6"][0], peer_mode="connection",
                                        name="conn_cons_brc_test_n6/0")]
    G["conn_brb_uniform_n10"] = [brb_spec(10, 3, 1010, 1, 3, g, [(0, i, 0) for i in range(10)], peer_mode="connection")
                                 for g in range(3)]
    # ... on the wide kernel (n > 64) and with delays up to D = 16
    G["conn_brb_uniform_n100"] = [brb_spec(100, 33, 0xC0AD, 1, 4, g, [(0, 0, 0), (0, 57, 0), (3, 99, 0)],
                                           peer_mode="connection") for g in range(2)]
    G["conn_brb_geometric_n128"] = [brb_spec(128, 42, 0xC0AE, 3, 16, g, [(0, 5, 0), (2, 100, 0)],
                                             peer_mode="connection") for g in range(1)]
    G["conn_brb_geometric_n16"] = [brb_spec(16, 5, 0xC0AF, 3, 12, g, [(0, i, 0) for i in range(0, 16, 3)],
                                            peer_mode="connection") for g in range(3)]
    G["conn_cons_geometric_n10"] = [cons_spec(10, 3, 0xC0B0, 3, 14, g, round_cap=2, peer_mode="connection")
                                    for g in range(4)]
    G["conn_cons_uniform_n100"] = [cons_spec(100, 33, 0xC0B1, 1, 4, g, round_cap=1, peer_mode="connection")
                                   for g in range(1)]
    G.update(values8_specs())
    G.update(multisend_specs())
    G.update(general_keys_specs())
    for name, specs in G.items():
        for i, sp in enumerate(specs):
            sp.setdefault("name", "%s/%d" % (name, i))
    return G


def multisend_specs():
    """One payload string SENT by several nodes, and SENT again by its own node (the reference keys
    BRB state by payload, core/brbroadcast.py:38-44, :76-82): one key, extra SENDs, both peer modes."""
    G = {}
    extra = [dict(t=0, kind="brb_send", node=3, kp=0, s=0, payload="TEST 1.0"),
             dict(t=1, kind="brb_send", node=4, kp=0, s=0, payload="TEST 1.0"),
             dict(t=3, kind="brb_send", node=1, kp=1, s=0, payload="TEST 2.0"),
             dict(t=2, kind="brb_send", node=5, kp=2, s=0, payload="TEST 3.0"),
             dict(t=2, kind="brb_send", node=6, kp=2, s=0, payload="TEST 3.0")]
    models = ((0, 1), (1, 3), (2, 4), (3, 5))
    for pm, pre in (("sender", ""), ("connection", "conn_")):
        G[pre + "brb_multisend_n7"] = [
            brb_spec(7, 2, 0x3A10 + g, m, d, g, [(0, 0, 0), (0, 1, 0), (2, 2, 0)], extra=extra, peer_mode=pm)
            for g, (m, d) in enumerate(models)]
    # payloads SENT by every node at once, and one SENT only by others after its origin crashed
    crash = [dict(t=0, kind="brb_send", node=o, kp=0, s=0, payload="TEST 1.0") for o in range(1, 16)]
    G["brb_multisend_n16"] = [brb_spec(16, 5, 0x3A20 + g, m, d, g, [(0, 0, 0), (1, 7, 0)], byzantine=[15],
                                       extra=crash[:14] + [dict(t=2, kind="brb_send", node=3, kp=7, s=0,
                                                                payload="TEST 8.0")])
                              for g, (m, d) in enumerate(((1, 4), (2, 8), (3, 6)))]
    return G


def general_keys_specs():
    """33..64 nodes with sender peers and what the reference keys by the payload string (core/brbroadcast.py:
    74-79, core/byzantinerandomizedconsensus.py:57-60): five proposal strings, one payload SENT by two origins
    and again by its own.  The engine runs them on the narrow kernel's general form (brc.h
    BRC_FLAG_GENERAL_KEYS; the lean kernel keeps 2-bit value ids and one SEND per key): general_keys."""
    G = {}
    extra = [dict(t=0, kind="brb_send", node=9, kp=0, s=0, payload="TEST 1.0"),      # a second origin
             dict(t=0, kind="brb_send", node=0, kp=0, s=0, payload="TEST 1.0"),      # its own origin again
             dict(t=0, kind="brb_send", node=21, kp=2, s=0, payload="TEST 3.0")]
    G["brb_multisend_n40"] = [dict(brb_spec(40, 13, 0x4A10 + g, m, d, g, [(0, 0, 0), (0, 1, 0), (0, 2, 0)],
                                            extra=extra), general_keys=True)
                              for g, (m, d) in enumerate(((0, 1), (1, 3), (2, 4)))]
    # ids 1..5 = "0", "1", "3", "alpha", "beta": a majority of a new string, a five-way split ("-1"), a
    # majority of "beta" with every other string present
    pats = [[4] * 30 + [1, 2, 3, 5] * 2 + [5, 5],
            [1, 2, 3, 4, 5] * 8,
            [5] * 29 + [1, 2, 3, 4] * 2 + [4, 3, 2]]
    G["cons_values_n40"] = [dict(cons_spec(40, 7, 0x4A20 + g, m, d, g, round_cap=2, proposals=pats[g]),
                                 values=VALUES8, general_keys=True)
                            for g, (m, d) in enumerate(((0, 1), (1, 3), (2, 4)))]
    return G


def clone(spec, **kw):
    sp = copy.deepcopy(spec)
    sp.update(kw)
    return sp
