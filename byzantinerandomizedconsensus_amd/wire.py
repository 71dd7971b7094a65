"""The reference's wire format: engine traces <-> the bytes reference nodes exchange.

A reference node puts one JSON envelope on each TCP connection (``base/broadcast.py:37-38``):

    {"peer": <sender ip>, "type": <1 SEND | 2 ECHO | 3 READY>, "message": <payload>}

and ECHO/READY carry the payload of the SEND they answer (``core/brbroadcast.py:82,98,119``).
Consensus payloads are themselves JSON (``core/byzantinerandomizedconsensus.py:48-49, 80-81,
102-103``):

    {"host": [ip, port], "round": r, "phase": p, "message": "<value>"}

``Codec`` maps between that text and the engine's keys: key ``(kp, s)`` of origin ``kp // nv``
at phase index ``s = 2 (round - 1) + (phase - 1)`` with a value id (``"-1"``, ``"0"``, ``"1"``,
...).  ``export`` turns an engine event log (``Engine.events()``) into the envelopes the
reference would have sent, byte for byte (``json.dumps`` with its default separators, as the
reference calls it); ``to_injections`` turns envelopes captured from reference nodes (or written
by hand) into ``Engine.inject`` records.  Pure host code: no engine calls.
"""
import json

SEND, ECHO, READY = 1, 2, 3
EV_SEND, EV_COPY = 3, 4
DEFAULT_VALUES = ("-1", "0", "1", "3")


def default_addrs(n):
    """The addresses the golden harness gives nodes (``tests/golden/refharness.py``)."""
    return [("localhost", 7000 + i) for i in range(n)]


def envelope(peer_ip, mtype, payload):
    """base/broadcast.py:37-38"""
    return json.dumps({"peer": peer_ip, "type": mtype, "message": payload})


def consensus_payload(host, rnd, phase, value):
    """core/byzantinerandomizedconsensus.py:48-49 (same key order, so the same bytes)"""
    return json.dumps({"host": list(host), "round": rnd, "phase": phase, "message": value})


class Codec:
    """Payload text <-> engine keys for one instance.

    mode: "consensus" (payloads are consensus JSON, derived from the key) or "brb" (payloads come
    from ``payloads``, a {(kp, s): text} table, e.g. the strings given to ``broadcast``).
    """

    def __init__(self, n, mode="consensus", nv=1, addrs=None, values=DEFAULT_VALUES, payloads=None,
                 peer_mode="sender"):
        if peer_mode not in ("sender", "connection"):
            raise ValueError("peer_mode must be 'sender' or 'connection'")
        self.n, self.mode, self.nv, self.peer_mode = n, mode, nv, peer_mode
        self.addrs = [tuple(a) for a in (addrs or default_addrs(n))]
        self.index = {a: i for i, a in enumerate(self.addrs)}
        self.values = list(values)
        self.value_id = {v: i for i, v in enumerate(self.values)}
        self.payloads = dict(payloads or {})
        self.keys = {p: k for k, p in self.payloads.items()}

    # ------------------------------------------------------------------ payloads
    def payload(self, kp, s, value_id):
        text = self.payloads.get((kp, s))
        if text is not None:
            return text
        if self.mode != "consensus":
            raise KeyError("no payload registered for BRB key %r" % ((kp, s),))
        origin = kp // self.nv
        return consensus_payload(self.addrs[origin], s // 2 + 1, s % 2 + 1, self.values[value_id])

    def key(self, payload):
        """(kp, s, value id) of a payload text."""
        k = self.keys.get(payload)
        if k is not None:
            return k[0], k[1], 0
        if self.mode != "consensus":
            raise KeyError("unknown BRB payload %r" % payload)
        d = json.loads(payload)
        origin = self.index[tuple(d["host"])]
        s = 2 * (d["round"] - 1) + (d["phase"] - 1)
        if d["message"] not in self.value_id:
            raise ValueError("value %r outside the value table %r" % (d["message"], self.values))
        return origin * self.nv, s, self.value_id[d["message"]]

    # ------------------------------------------------------------------ engine -> wire
    def export(self, events, instance=0, dst_masks=None):
        """[t, src, dst, envelope] for every message the run put on the wire, sorted.

        events: ``Engine.events()`` tuples (instance, t, kind, node, type, kp, s, value id).
        dst_masks: {(t, node, type, kp, s): destination bit mask} for sends that did not go to
        every peer (the Byzantine injections that were restricted); everything else went to all.
        Connection-identity peers (core/brbroadcast.py:69) put every broadcast on the wire, the
        :119 READY re-fires included: the engine logs each one after the first as an EV_COPY
        event, and each becomes one more envelope per peer.
        """
        allm = (1 << self.n) - 1
        kinds = (EV_SEND, EV_COPY) if self.peer_mode == "connection" else (EV_SEND,)
        out = []
        for (inst, t, kind, node, typ, kp, s, value) in events:
            if inst != instance or kind not in kinds:
                continue
            env = envelope(self.addrs[node][0], typ, self.payload(kp, s, value))
            mask = (dst_masks or {}).get((t, node, typ, kp, s), allm)
            out.extend([t, node, dst, env] for dst in range(self.n) if (mask >> dst) & 1)
        return sorted(out)

    # ------------------------------------------------------------------ wire -> engine
    def decode(self, src, env):
        """One envelope sent by node ``src``: dict(type, payload, kp, s, value)."""
        d = json.loads(env)
        if d.get("peer") != self.addrs[src][0]:
            raise ValueError("envelope peer %r is not node %d's host" % (d.get("peer"), src))
        kp, s, v = self.key(d["message"])
        return {"type": d["type"], "payload": d["message"], "kp": kp, "s": s, "value": v}

    def to_injections(self, wire, instance=0):
        """Engine injections replaying captured wire messages [t, src, dst, envelope] (from
        Byzantine or external nodes): each key whose origin is one of the captured senders is
        declared once (keys of other origins belong to simulated honest nodes, which create
        them), then its SENDs (with their destination masks) and its ECHO / READY broadcasts."""
        from . import _lib as L
        allm = (1 << self.n) - 1
        groups, declared, out = {}, set(), []
        senders = {w[1] for w in wire}
        for t, src, dst, env in sorted(wire):
            m = self.decode(src, env)
            g = groups.setdefault((t, src, m["type"], m["kp"], m["s"]), {"mask": 0, "value": m["value"]})
            g["mask"] |= 1 << dst
        for (t, src, typ, kp, s), g in sorted(groups.items()):
            if kp // self.nv in senders and (kp, s) not in declared:
                declared.add((kp, s))
                out.append(dict(t=t, kind=L.INJ_KEY, instance=instance, node=kp // self.nv, kp=kp, s=s,
                                value=g["value"]))
            if typ == SEND:
                out.append(dict(t=t, kind=L.INJ_SEND, instance=instance, node=src, kp=kp, s=s, value=g["value"],
                                dst=g["mask"]))
            else:
                if g["mask"] != allm:
                    raise ValueError("ECHO/READY to a subset of the peers is not modelled (core/brbroadcast.py "
                                     "broadcasts them to every peer)")
                out.append(dict(t=t, kind=L.INJ_MSG, type=typ, instance=instance, node=src, kp=kp, s=s,
                                value=g["value"], dst=allm))
        return out
