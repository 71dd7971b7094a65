"""ctypes front-end of the C oracle (TEST INFRASTRUCTURE ONLY).

Imported only by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg,
always as the CHECKER or the CPU baseline -- never as a product path.  The spec format is
the one the golden harness (``tests/golden/refharness.py``) consumes, so a fixture, the
oracle and the HIP engine can all be fed the same workload.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")

ACT = {"propose": 1, "brb_send": 2, "byz_key": 3, "byz": 4, "deliver": 5}
STATUS = {1: "done", 2: "quiescent", 3: "stepcap", 4: "overflow"}
PEER_MODES = {"sender": 0, "connection": 1}
MODES = {"brb": 0, "consensus": 1, "spec": 2, "spec_brb": 3, "beb": 4, "beb_consensus": 5}


class _Action(ctypes.Structure):
    _fields_ = [("t", ctypes.c_uint32), ("kind", ctypes.c_uint32), ("node", ctypes.c_uint32),
                ("type", ctypes.c_uint32), ("kp", ctypes.c_uint32), ("s", ctypes.c_uint32),
                ("value", ctypes.c_int32), ("pad", ctypes.c_uint32), ("dst", ctypes.c_uint64 * 4)]


class _Spec(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("f", ctypes.c_uint32), ("mode", ctypes.c_uint32),
                ("nv", ctypes.c_uint32), ("seed", ctypes.c_uint64), ("delay_model", ctypes.c_uint32),
                ("dmax", ctypes.c_uint32), ("dconst", ctypes.c_uint32), ("round_cap", ctypes.c_uint32),
                ("g", ctypes.c_uint64), ("step_cap", ctypes.c_uint32), ("n_actions", ctypes.c_uint32),
                ("byz", ctypes.c_uint64 * 4), ("actions", ctypes.POINTER(_Action)),
                ("coin_seed", ctypes.c_uint64), ("window", ctypes.c_uint32), ("peer_mode", ctypes.c_uint32)]


class _Result(ctypes.Structure):
    _fields_ = [("status", ctypes.c_uint32), ("t_stop", ctypes.c_uint32),
                ("msgs_sent", ctypes.c_uint64), ("arrivals", ctypes.c_uint64),
                ("deliver", ctypes.POINTER(ctypes.c_uint32)), ("deliver_cap", ctypes.c_size_t),
                ("n_deliver", ctypes.c_size_t),
                ("decide", ctypes.POINTER(ctypes.c_uint32)), ("decide_cap", ctypes.c_size_t),
                ("n_decide", ctypes.c_size_t),
                ("sends", ctypes.POINTER(ctypes.c_uint32)), ("send_cap", ctypes.c_size_t),
                ("n_send", ctypes.c_size_t), ("cell_steps", ctypes.c_uint64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle library missing: build it with `make -C oracle`")
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_run.argtypes = [ctypes.POINTER(_Spec), ctypes.POINTER(_Result)]
        L.oracle_run.restype = ctypes.c_int
        L.oracle_delay.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                   ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                   ctypes.c_uint32]
        L.oracle_delay.restype = ctypes.c_uint32
        L.oracle_proposal_id.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
        L.oracle_proposal_id.restype = ctypes.c_uint32
        L.oracle_coin_id.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
        L.oracle_coin_id.restype = ctypes.c_uint32
        L.oracle_philox.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                    ctypes.POINTER(ctypes.c_uint32)]
        L.oracle_philox.restype = None
        _lib = L
    return _lib


def _mask4(m):
    return (ctypes.c_uint64 * 4)(*[(m >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)])


def philox(ctr, key):
    out = (ctypes.c_uint32 * 4)()
    lib().oracle_philox((ctypes.c_uint32 * 4)(*ctr), (ctypes.c_uint32 * 2)(*key), out)
    return tuple(out)


def expand_actions(actions, n):
    """Harness actions with every "brb_msg" (an honest node's own ECHO / READY broadcast,
    base/broadcast.py:17) restated as the raw message it puts on every link: a key declaration on
    the payload's first use ("byz_key") and a "byz" message from the node to all peers.  Stable in
    time order; the list order within a step is kept."""
    declared = set()
    out = []
    for a in sorted(actions, key=lambda a: a["t"]):
        if a["kind"] in ("brb_send", "byz_key"):
            declared.add((a["kp"], a["s"]))
        if a["kind"] != "brb_msg":
            out.append(a)
            continue
        key = (a["kp"], a["s"])
        if key not in declared:
            declared.add(key)
            out.append(dict(t=a["t"], kind="byz_key", kp=a["kp"], s=a["s"], value=a.get("value", 0)))
        out.append(dict(t=a["t"], kind="byz", src=a["node"], type=a["type"], kp=a["kp"], s=a["s"],
                        dst=(1 << n) - 1))
    return out


def run(spec, light=False, kinds=("deliver", "decide", "send")):
    """Run one instance of ``spec`` (harness format) and return the harness result format.
    ``light``: status and counters only (no event lists; one C call, no Python conversion).
    ``kinds``: the event lists to return (the others come back empty; their counts are exact)."""
    acts = expand_actions(spec.get("actions", []), spec["n"])
    arr = (_Action * max(1, len(acts)))()
    for i, a in enumerate(acts):
        x = arr[i]
        x.t, x.kind = a["t"], ACT[a["kind"]]
        x.node = a.get("node", a.get("src", 0))
        x.type = a.get("type", 0)
        x.kp, x.s = a.get("kp", 0), a.get("s", 0)
        x.value = a.get("value", 0)
        x.dst = _mask4(a.get("dst", 0))
    byz = 0
    for b in spec.get("byzantine", []):
        byz |= 1 << b
    sp = _Spec(n=spec["n"], f=spec["f"], mode=MODES[spec["mode"]],
               nv=spec.get("nv", 1), seed=spec["seed"], delay_model=spec["delay_model"],
               dmax=spec["dmax"], dconst=spec.get("dconst", 1), round_cap=spec.get("round_cap", 0),
               g=spec["g"], step_cap=spec.get("step_cap", 10000), n_actions=len(acts),
               byz=_mask4(byz), actions=arr, coin_seed=spec.get("coin_seed", 0), window=spec.get("window", 0),
               peer_mode=PEER_MODES[spec.get("peer_mode", "sender")])
    names = ("deliver", "decide", "send")
    caps = [0 if light or k not in kinds else 65536 for k in names]
    while True:
        bufs = [(ctypes.c_uint32 * (c * w))() for c, w in zip(caps, (4, 4, 5))]
        res = _Result(deliver=bufs[0], deliver_cap=caps[0], decide=bufs[1], decide_cap=caps[1],
                      sends=bufs[2], send_cap=caps[2])
        rc = lib().oracle_run(ctypes.byref(sp), ctypes.byref(res))
        if rc != 0:
            raise RuntimeError("oracle_run failed: %d" % rc)
        got = (res.n_deliver, res.n_decide, res.n_send)
        if light or all(k not in kinds or n <= c for k, n, c in zip(names, got, caps)):
            break
        caps = [2 * n if k in kinds and n > c else c for k, n, c in zip(names, got, caps)]

    if light:
        return {"status": STATUS.get(res.status), "t_stop": res.t_stop, "msgs_sent": res.msgs_sent,
                "arrivals": res.arrivals, "cell_steps": res.cell_steps,
                "counts": {"deliver": res.n_deliver, "decide": res.n_decide, "send": res.n_send}}

    def rows(buf, cnt, w, k):
        return [list(buf[i * w:(i + 1) * w]) for i in range(cnt)] if k in kinds else []

    dec = rows(bufs[1], res.n_decide, 4, "decide")
    values = spec.get("values")
    if values is not None:
        dec = [[t, nd, r, values[v]] for t, nd, r, v in dec]
    return {"status": STATUS.get(res.status), "t_stop": res.t_stop, "msgs_sent": res.msgs_sent,
            "arrivals": res.arrivals, "cell_steps": res.cell_steps,
            "events": {"deliver": rows(bufs[0], res.n_deliver, 4, "deliver"), "decide": dec,
                       "send": rows(bufs[2], res.n_send, 5, "send")}}
