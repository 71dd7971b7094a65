"""Independent pure-Python model of the SPEC protocol modes and of best-effort broadcast
(TEST INFRASTRUCTURE ONLY).

The reference never runs the protocol it intends: its broadcast echoes on an ECHO-created entry
(core/brbroadcast.py:76-98) and its consensus coin branch is dead (:89-92 of
core/byzantinerandomizedconsensus.py).  BRC_MODE_SPEC restates the intended protocol:

* Bracha broadcast -- ECHO on the first SEND of a key; ONE READY per key, sent at the echo quorum
  (|E| > (n+f)/2) or at f+1 READYs; DELIVER at 2f+1 READYs; nothing after DELIVER matters;
* consensus -- a phase ends once n-f DISTINCT origins delivered a key of that phase (keys of later
  phases are buffered, at most ``window`` phase indices ahead, earlier ones dropped); phase 1
  proposes a value carried by more than (n+f)/2 of those deliveries (:73), phase 2 decides above
  2f (:88), adopts above f, and otherwise takes the common coin of (instance, round) (:90-92).

Nothing from the reference can pin these modes, so parity is pinned by two restatements written
independently: the C oracle (``oracle/brc_oracle.c``, brb_on_message_spec / spec_deliver /
spec_advance) and this model, which keeps sets and dicts where the C code keeps bitsets and a
ring.  ``tests/test_spec_model.py`` checks they agree; the GPU tests then compare the engine with
the C oracle.  Only small instances are meant to run here (pure-Python loops).
"""
from collections import defaultdict

from oracle.schedule import PURPOSE_COIN, Schedule, _draw

SEND, ECHO, READY = 1, 2, 3


def coin_id(coin_seed, g, rnd):
    return 1 + (_draw(coin_seed, g, rnd, PURPOSE_COIN, 0)[0] & 1)


def run(spec):
    n, f, nv = spec["n"], spec["f"], spec.get("nv", 1)
    mode, window, g = spec["mode"], spec.get("window", 4), spec["g"]
    assert mode in ("spec", "spec_brb", "beb")
    sch = Schedule(n, f, spec["seed"], spec["delay_model"], spec["dmax"], spec.get("dconst", 1))
    byz = set(spec.get("byzantine", []))
    values = spec.get("values")
    st = {"t": 0, "msgs": 0, "arrivals": 0, "overflow": False}
    keys = {}
    sent, first = set(), set()
    inflight = defaultdict(list)
    cells = {}
    cons = [{"round": 0, "phase": 0, "win": {}, "decides": 0} for _ in range(n)]
    ev = {"deliver": [], "decide": [], "send": []}

    def send(src, dst, typ, kp, s):
        if (kp, s, typ, src, dst) in sent:
            return
        sent.add((kp, s, typ, src, dst))
        st["msgs"] += 1
        if (kp, s, typ, src) not in first:
            first.add((kp, s, typ, src))
            ev["send"].append([st["t"], src, typ, kp, s])
        if dst not in byz:
            inflight[st["t"] + sch.delay(g, src, dst)].append((dst, kp, s, typ, src))

    def bcast(src, typ, kp, s):
        for dst in range(n):
            send(src, dst, typ, kp, s)

    def declare(kp, s, v):
        assert keys.setdefault((kp, s), v) == v, "one payload per key"

    def send_key(node, s, v):
        declare(node * nv, s, v)
        bcast(node, SEND, node * nv, s)

    def advance(i):
        c = cons[i]
        while c["round"] > 0:
            s = 2 * (c["round"] - 1) + c["phase"] - 1
            w = c["win"].get(s)
            if w is None or len(w["hosts"]) < n - f:
                return
            del c["win"][s]
            n0, n1 = w["n0"], w["n1"]
            if c["phase"] == 1:
                prop = 1 if 2 * n0 > n + f else (2 if 2 * n1 > n + f else 0)
                c["phase"] = 2
                send_key(i, s + 1, prop)
            else:
                vmax, cmax = (2, n1) if n1 > n0 else (1, n0)
                if cmax > 2 * f:
                    ev["decide"].append([st["t"], i, c["round"], values[vmax] if values else vmax])
                    c["decides"] += 1
                    est = vmax
                elif cmax > f:
                    est = vmax
                else:
                    est = coin_id(spec["coin_seed"], g, c["round"])
                c["round"] += 1
                c["phase"] = 1
                send_key(i, s + 1, est)

    def deliver(i, kp, s):
        c = cons[i]
        cur = 2 * (c["round"] - 1) + c["phase"] - 1 if c["round"] else 0
        if s < cur:
            return
        if s >= cur + window:
            st["overflow"] = True
            return
        w = c["win"].setdefault(s, {"hosts": set(), "n0": 0, "n1": 0})
        host = kp // nv
        if host in w["hosts"]:
            return
        w["hosts"].add(host)
        v = keys[(kp, s)]
        if v == 1:
            w["n0"] += 1
        elif v == 2:
            w["n1"] += 1
        advance(i)

    def on_message(dst, kp, s, typ, src):
        st["arrivals"] += 1
        c = cells.setdefault((dst, kp, s), {"E": set(), "R": set(), "es": False, "rs": False, "dl": False})
        if c["dl"]:
            return
        if mode == "beb":               # best-effort broadcast: a SEND delivers, nothing is echoed
            if typ == SEND:
                c["dl"] = True
                ev["deliver"].append([st["t"], dst, kp, s])
            return
        if typ == SEND:
            if not c["es"]:
                c["es"] = True
                bcast(dst, ECHO, kp, s)
        elif typ == ECHO:
            c["E"].add(src)
            if 2 * len(c["E"]) > n + f and not c["rs"]:
                c["rs"] = True
                bcast(dst, READY, kp, s)
        elif typ == READY:
            c["R"].add(src)
            if len(c["R"]) > f and not c["rs"]:
                c["rs"] = True
                bcast(dst, READY, kp, s)
            if len(c["R"]) > 2 * f:
                c["dl"] = True
                ev["deliver"].append([st["t"], dst, kp, s])
                if mode == "spec":
                    deliver(dst, kp, s)

    def act(a):
        k = a["kind"]
        if k == "propose":
            c = cons[a["node"]]
            c["round"], c["phase"] = 1, 1
            send_key(a["node"], 0, a["value"])
            if mode == "spec":
                advance(a["node"])
        elif k == "brb_send":
            declare(a["kp"], a["s"], a.get("value", 0))
            bcast(a["node"], SEND, a["kp"], a["s"])
        elif k == "byz_key":
            declare(a["kp"], a["s"], a.get("value", 0))
        elif k == "byz":
            assert (a["kp"], a["s"]) in keys
            for dst in range(n):
                if (a["dst"] >> dst) & 1:
                    send(a["src"], dst, a["type"], a["kp"], a["s"])
        else:
            raise ValueError(k)

    acts = sorted(spec.get("actions", []), key=lambda a: a["t"])
    ai = 0
    while ai < len(acts) and acts[ai]["t"] == 0:
        act(acts[ai])
        ai += 1
    last_active = 0
    rcap = spec.get("round_cap", 0)
    while True:
        pending = [x for x in inflight if x > st["t"] and inflight[x]]
        nt = min(pending) if pending else None
        if ai < len(acts) and (nt is None or acts[ai]["t"] < nt):
            nt = acts[ai]["t"]
        if nt is None:
            status = "quiescent"
            break
        if nt > spec.get("step_cap", 10000):
            status = "stepcap"
            break
        st["t"] = nt
        msgs = sorted(inflight.pop(nt, []))
        if msgs or (ai < len(acts) and acts[ai]["t"] == nt):
            last_active = nt
        for m in msgs:
            on_message(*m)
        while ai < len(acts) and acts[ai]["t"] == nt:
            act(acts[ai])
            ai += 1
        if st["overflow"]:
            status = "overflow"
            break
        if mode == "spec" and rcap > 0 and all(cons[i]["decides"] >= rcap for i in range(n) if i not in byz):
            status = "done"
            break
    return {"status": status, "t_stop": last_active, "msgs_sent": st["msgs"], "arrivals": st["arrivals"],
            "events": ev}
