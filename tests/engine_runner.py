"""Run harness-format specs (tests/golden/specs.py) on the HIP engine and return results in
the same format as the reference harness / oracle, with every event list sorted canonically.

Specs that share a configuration and have consecutive global instance ids run as ONE batch
(one engine, one launch): the instance's global id is ``instance_offset + local index``.
"""
from collections import defaultdict

from byzantinerandomizedconsensus_amd import _lib as L
from byzantinerandomizedconsensus_amd.engine import Engine
from oracle.oracle import expand_actions

KIND = {"propose": L.INJ_PROPOSE, "brb_send": L.INJ_SEND, "byz_key": L.INJ_KEY}


def sort_result(res):
    ev = res["events"]
    out = dict(res)
    out["events"] = {k: sorted(map(list, ev[k]), key=lambda r: [str(x) if isinstance(x, str) else x for x in r])
                     if k in ev else None for k in ("deliver", "decide", "send")}
    return out


def _cfg_key(sp):
    return (sp["n"], sp["f"], sp["mode"], sp.get("nv", 1), sp["seed"], sp["delay_model"], sp["dmax"],
            sp.get("dconst", 1), sp.get("round_cap", 0), sp.get("step_cap", 10000),
            tuple(sorted(sp.get("byzantine", []))), sp.get("window"), sp.get("coin_seed"), sp.get("peer_mode", "sender"),
            sp.get("key_window"), sp.get("general_keys", False))


def _injections(sp, local):
    n, nv = sp["n"], sp.get("nv", 1)
    allm = (1 << n) - 1
    values = {}
    out = []
    for a in expand_actions(sp.get("actions", []), n):
        k = a["kind"]
        if k == "propose":
            out.append(dict(t=a["t"], kind=L.INJ_PROPOSE, instance=local, node=a["node"], value=a["value"]))
        elif k == "brb_send":
            out.append(dict(t=a["t"], kind=L.INJ_SEND, instance=local, node=a["node"], kp=a["kp"], s=a["s"],
                            value=a.get("value", 0), dst=allm))
        elif k == "deliver":               # ByzantineRandomizedConsensus.deliver() called directly
            out.append(dict(t=a["t"], kind=L.INJ_DELIVER, instance=local, node=a["node"], kp=a["kp"],
                            value=a["value"]))
        elif k == "byz_key":
            values[(a["kp"], a["s"])] = a.get("value", 0)
            out.append(dict(t=a["t"], kind=L.INJ_KEY, instance=local, node=a["kp"] // nv, kp=a["kp"], s=a["s"],
                            value=a.get("value", 0)))
        elif k == "byz":
            v = values.get((a["kp"], a["s"]), 0)
            if a["type"] == L.SEND:
                out.append(dict(t=a["t"], kind=L.INJ_SEND, instance=local, node=a["src"], kp=a["kp"], s=a["s"],
                                value=v, dst=a["dst"]))
            else:
                out.append(dict(t=a["t"], kind=L.INJ_MSG, type=a["type"], instance=local, node=a["src"],
                                kp=a["kp"], s=a["s"], value=v, dst=a["dst"]))
        else:
            raise ValueError(k)
    return out


def run_batch(specs, key_window=None, event_capacity=1 << 21, device=0):
    """specs share _cfg_key and have consecutive g.  The key window defaults to the spec's
    "key_window" (reference-protocol runs of many rounds keep more phases of one origin in flight),
    else 8 // nv."""
    sp0 = specs[0]
    spec_mode = sp0["mode"] in ("spec", "spec_brb")
    if spec_mode:
        key_window = sp0["window"]          # the SPEC buffering window IS the engine's key window
    elif key_window is None:
        key_window = sp0.get("key_window") or 8 // sp0.get("nv", 1)
    protocol = {"spec": "consensus", "spec_brb": "brb", "beb": "brb", "beb_consensus": "consensus"}.get(
        sp0["mode"], sp0["mode"])
    mode = L.MODE_SPEC if spec_mode else (L.MODE_BEB if sp0["mode"].startswith("beb") else L.MODE_REFERENCE)
    eng = Engine(n=sp0["n"], f=sp0["f"], instances=len(specs), protocol=protocol, seed=sp0["seed"],
                 delay_model=sp0["delay_model"], delay_max=sp0["dmax"], delay_const=sp0.get("dconst", 1),
                 round_cap=sp0.get("round_cap", 0), step_cap=sp0.get("step_cap", 10000), key_window=key_window,
                 variants=sp0.get("nv", 1), byzantine=sp0.get("byzantine", ()), event_capacity=event_capacity,
                 instance_offset=sp0["g"], device=device, mode=mode,
                 peer_mode=L.PEER_CONNECTION if sp0.get("peer_mode") == "connection" else L.PEER_SENDER,
                 coin_seed=sp0.get("coin_seed", 0), general_keys=sp0.get("general_keys", False))
    try:
        inj = []
        for i, sp in enumerate(specs):
            inj += _injections(sp, i)
        eng.inject(inj)
        eng.run()
        res = eng.instances_result()
        evs = eng.events()
    finally:
        eng.close()
    per = [{"deliver": [], "decide": [], "send": []} for _ in specs]
    for (inst, t, kind, node, typ, a, b, _v) in evs:
        if kind == L.EV_DELIVER:
            per[inst]["deliver"].append([t, node, a, b])
        elif kind == L.EV_DECIDE:
            per[inst]["decide"].append([t, node, a, specs[inst]["values"][b]])
        elif kind == L.EV_SEND:                # first broadcasts (copies: L.EV_COPY, wire export only)
            per[inst]["send"].append([t, node, typ, a, b])
    out = []
    for i, sp in enumerate(specs):
        r = res[i]
        out.append(sort_result({"status": r["status"], "t_stop": r["t_stop"], "msgs_sent": r["msgs_sent"],
                                "arrivals": r["arrivals"], "events": per[i], "cell_steps": r["cell_steps"]}))
    return out


def run_specs(specs, **kw):
    """Run any list of specs, batching compatible ones; results in input order."""
    groups = defaultdict(list)
    for idx, sp in enumerate(specs):
        groups[_cfg_key(sp)].append(idx)
    results = [None] * len(specs)
    for key, idxs in groups.items():
        idxs.sort(key=lambda i: specs[i]["g"])
        run = [idxs[0]]
        runs = []
        for i in idxs[1:]:
            if specs[i]["g"] == specs[run[-1]]["g"] + 1:
                run.append(i)
            else:
                runs.append(run)
                run = [i]
        runs.append(run)
        for r in runs:
            for i, res in zip(r, run_batch([specs[j] for j in r], **kw)):
                results[i] = res
    return results
