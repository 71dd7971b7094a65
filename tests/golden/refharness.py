"""Lock-step harness that drives the UNMODIFIED reference classes (golden-vector generator).

Runs only in the build container, where ``/root/reference`` exists; never on the GPU box
and never from a test.  ``make_golden.py`` calls it and commits the resulting JSON
fixtures under ``tests/golden/``.  Nothing of the reference is copied: it is imported from
``/root/reference`` at generation time and exercised through its public classes.

How the reference is driven
---------------------------
* The module attribute ``socket`` of ``base/broadcast.py`` and ``core/brbroadcast.py`` is
  replaced by a fake module.  Client sockets (``base/broadcast.py:30-35``) hand each
  ``sendall`` to the simulated network; the sender is found by walking the caller frames
  up to ``Broadcast.broadcast`` (its ``self.host``).  The server socket
  (``core/brbroadcast.py:55-62``) blocks in ``accept()`` until the scheduler hands it ONE
  message, and returns ``(sender_name, port)`` as the peer address.  Sender-identity peers
  (``spec["peer_mode"] == "sender"``, the default): ``port`` is 0, so the reference's
  ``peer_address`` (``core/brbroadcast.py:69``) is the stable sender identity and the network
  drops duplicates.  Connection-identity peers (``"connection"``, the reference's local-test
  behaviour): ``port`` is a fresh number per message, as an ephemeral TCP port is, and nothing
  is dropped.
* ``threading`` stays real: every node runs its own listener thread
  (``core/brbroadcast.py:121-128``).  The scheduler hands over one message, then waits until
  that node is back in ``accept()`` -- so exactly one message is in processing at any time
  and the run is deterministic.
* Time, delays, canonical order and duplicate suppression follow ``oracle/schedule.py``.
* Consensus runs need ``python -O`` when ``N <= 5f`` (``core/byzantinerandomizedconsensus.py:20``).
"""
import json
import sys
import threading
from collections import defaultdict

REFERENCE = "/root/reference"

SEND, ECHO, READY = 1, 2, 3


class HarnessError(RuntimeError):
    pass




def _import_reference():
    sys.dont_write_bytecode = True     # the reference tree is read-only: no __pycache__ there
    if REFERENCE not in sys.path:
        sys.path.insert(0, REFERENCE)
    import byzantinerandomizedconsensus.base.broadcast as bmod
    import byzantinerandomizedconsensus.core.brbroadcast as brbmod
    import byzantinerandomizedconsensus.core.byzantinerandomizedconsensus as brcmod
    return bmod, brbmod, brcmod


def _caller_host():
    """Host address of the Broadcast object whose broadcast() is on the stack."""
    fr = sys._getframe(2)
    while fr is not None:
        if fr.f_code.co_name == "broadcast" and "self" in fr.f_locals:
            obj = fr.f_locals["self"]
            if hasattr(obj, "host") and hasattr(obj, "peers"):
                return tuple(obj.host)
        fr = fr.f_back
    raise HarnessError("send outside Broadcast.broadcast")


class _Conn:
    def __init__(self, data):
        self._data = data

    def recv(self, bufsize):
        # core/brbroadcast.py:62 -- one recv of BUFFER_SIZE bytes
        return self._data[:bufsize]

    def close(self):
        pass


class _FakeSocket:
    def __init__(self, net):
        self.net = net
        self.dst = None
        self.server = None

    # client side (base/broadcast.py:31-35)
    def connect(self, addr):
        self.dst = tuple(addr)
        self.src = _caller_host()

    def sendall(self, data):
        self.net.wire_send(self.src, self.dst, data)

    def shutdown(self, how):
        pass

    def close(self):
        pass

    # server side (core/brbroadcast.py:55-61)
    def bind(self, addr):
        self.server = self.net.register_server(tuple(addr))

    def listen(self, backlog):
        pass

    def accept(self):
        return self.server.accept()


class _FakeSocketModule:
    AF_INET = 2
    SOCK_STREAM = 1
    SHUT_RD = 0

    def __init__(self, net):
        self.net = net

    def socket(self, *args, **kw):
        return _FakeSocket(self.net)


class _Server:
    """One node's listening socket: a lock-step mailbox of size one."""

    def __init__(self, net, addr):
        self.net = net
        self.addr = addr
        self.cv = threading.Condition()
        self.item = None
        self.idle = False
        self.failed = None

    def accept(self):
        with self.cv:
            self.idle = True
            self.cv.notify_all()
            while self.item is None:
                self.cv.wait()
            item, self.item = self.item, None
            self.idle = False
        if item == "shutdown":
            raise SystemExit()   # ends the listener thread silently
        data, sender_name, port = item
        return _Conn(data), (sender_name, port)

    def hand(self, data, sender_name, port=0, timeout=30.0):
        with self.cv:
            if not self.idle:
                raise HarnessError("node %r not idle" % (self.addr,))
            self.item = (data, sender_name, port)
            self.idle = False
            self.cv.notify_all()
            ok = self.cv.wait_for(lambda: self.idle or self.failed, timeout)
            if not ok or self.failed:
                raise HarnessError("node %r did not return to accept()" % (self.addr,))

    def wait_idle(self, timeout=30.0):
        with self.cv:
            if not self.cv.wait_for(lambda: self.idle, timeout):
                raise HarnessError("node %r never reached accept()" % (self.addr,))

    def stop(self):
        with self.cv:
            self.item = "shutdown"
            self.cv.notify_all()


def consensus_payload(host, rnd, phase, value):
    # same dict/key order the reference builds (core/byzantinerandomizedconsensus.py:48-49)
    return json.dumps({"host": list(host), "round": rnd, "phase": phase, "message": value})


class Run:
    """One simulated instance.

    spec keys: n, f, mode ('brb'|'consensus'), nv, seed, delay_model, dmax, dconst,
    byzantine (list), values (value-id -> string, id 0 == "-1"), round_cap, step_cap,
    actions (list of injection actions, see make_golden.py), g (global instance id).
    """

    def __init__(self, spec, schedule):
        self.spec = spec
        self.sched = schedule
        self.n = spec["n"]
        self.f = spec["f"]
        self.nv = spec.get("nv", 1)
        self.g = spec["g"]
        self.mode = spec["mode"]
        self.connection = spec.get("peer_mode", "sender") == "connection"
        self.ports = 0
        self.byz = set(spec.get("byzantine", []))
        self.honest = [i for i in range(self.n) if i not in self.byz]
        self.values = spec["values"]
        self.addrs = [("localhost", 7000 + i) for i in range(self.n)]
        self.index = {a: i for i, a in enumerate(self.addrs)}
        self.servers = {}
        self.t = 0
        self.arrivals = defaultdict(list)
        self.sent = defaultdict(int)    # (src, type, kp, s) -> destinations already sent to (bit mask)
        self.keep_wire = spec.get("keep_wire", True)   # large runs: no per-message wire log
        self.first_sends = set()
        self.key_of_payload = {}
        self.payload_of_key = {}
        self.events = {"deliver": [], "decide": [], "send": []}
        self.wire = []                  # [t, src, dst, envelope] of every message the network carries
        self.msgs_sent = 0
        self.arrivals_processed = 0
        self.last_active = 0
        self.decides = defaultdict(int)

    # ------------------------------------------------------------------ network
    def register_server(self, addr):
        srv = _Server(self, addr)
        self.servers[self.index[addr]] = srv
        return srv

    def key_for(self, payload):
        k = self.key_of_payload.get(payload)
        if k is not None:
            return k
        if self.mode != "consensus":
            raise HarnessError("unregistered BRB payload %r" % payload)
        d = json.loads(payload)
        origin = self.index[tuple(d["host"])]
        if origin in self.byz:
            raise HarnessError("unregistered Byzantine payload %r" % payload)
        s = 2 * (d["round"] - 1) + (d["phase"] - 1)
        k = (origin * self.nv, s)
        self.register(payload, k)
        return k

    def register(self, payload, key):
        if self.key_of_payload.get(payload, key) != key or self.payload_of_key.get(key, payload) != payload:
            raise HarnessError("key collision %r %r" % (payload, key))
        self.key_of_payload[payload] = key
        self.payload_of_key[key] = payload

    def wire_send(self, src_addr, dst_addr, data):
        self.raw_send(self.index[src_addr], self.index[dst_addr], data)

    def raw_send(self, src, dst, data):
        env = json.loads(data.decode("utf-8"))
        payload, mtype = env["message"], env["type"]
        kp, s = self.key_for(payload)
        if not self.connection:
            ident = (src, mtype, kp, s)  # one payload per key (register() checks)
            if (self.sent[ident] >> dst) & 1:   # duplicate-suppressing network (sender-identity peers)
                return
            self.sent[ident] |= 1 << dst
        self.msgs_sent += 1
        if self.keep_wire:
            self.wire.append([self.t, src, dst, data.decode("utf-8")])
        fs = (src, mtype, payload)
        if fs not in self.first_sends:
            self.first_sends.add(fs)
            self.events["send"].append([self.t, src, mtype, kp, s])
        if dst in self.byz:             # counted as sent; a Byzantine node runs no code
            return
        t_arr = self.t + self.sched.delay(self.g, src, dst)
        self.arrivals[t_arr].append(((kp, s, mtype, src), dst, data, src))

    def byz_send(self, src, mtype, key, dst_mask):
        payload = self.payload_of_key[key]
        env = json.dumps({"peer": self.addrs[src][0], "type": mtype, "message": payload})
        data = env.encode("utf-8")
        for dst in range(self.n):
            if (dst_mask >> dst) & 1:
                self.raw_send(src, dst, data)

    # ------------------------------------------------------------------ nodes
    def build(self, refmods):
        bmod, brbmod, brcmod = refmods
        fake = _FakeSocketModule(self)
        bmod.socket = fake
        brbmod.socket = fake
        run = self

        class _BRBUser(bmod.IBroadcastHandler):
            def __init__(self, node):
                self.node = node

            def deliver(self, message):
                kp, s = run.key_for(message)
                run.events["deliver"].append([run.t, self.node, kp, s])

        from byzantinerandomizedconsensus.base.consensus import IConsensusHandler

        class _User(IConsensusHandler):
            def __init__(self, node):
                self.node = node
                self.obj = None

            def decide(self, message):
                run.events["decide"].append([run.t, self.node, self.obj.round, message])
                run.decides[self.node] += 1

        class _Tap:
            def __init__(self, node, inner):
                self.node, self.inner = node, inner

            def deliver(self, message):
                kp, s = run.key_for(message)
                run.events["deliver"].append([run.t, self.node, kp, s])
                return self.inner.deliver(message)

        self.nodes = {}
        for i in self.honest:
            if self.mode == "brb":
                node = brbmod.BRBroadcast(self.n, self.f, self.addrs[i], list(self.addrs), _BRBUser(i))
                node.broadcast_listener()
            else:
                user = _User(i)
                node = brcmod.ByzantineRandomizedConsensus(self.n, self.f, list(self.addrs),
                                                           self.addrs[i], user)
                user.obj = node
                node.brb.consensus = _Tap(i, node)
            self.nodes[i] = node
        for i in self.honest:
            while i not in self.servers:
                threading.Event().wait(0.001)
            self.servers[i].wait_idle()

    # ------------------------------------------------------------------ actions
    def act(self, a):
        kind = a["kind"]
        if kind == "propose":
            node = self.nodes[a["node"]]
            node.message_queue.put_nowait(self.values[a["value"]])
            node.start()                  # core/byzantinerandomizedconsensus.py:38-50
        elif kind == "brb_send":
            key = (a["kp"], a["s"])
            self.register(a["payload"], key)
            self.nodes[a["node"]].broadcast(SEND, a["payload"])   # base/broadcast.py:17
        elif kind == "brb_msg":       # an honest node's user code broadcasts ECHO / READY
            self.register(a["payload"], (a["kp"], a["s"]))
            self.nodes[a["node"]].broadcast(a["type"], a["payload"])   # base/broadcast.py:17
        elif kind == "byz_key":       # declare a Byzantine key and its payload
            key = (a["kp"], a["s"])
            if self.mode == "consensus":
                origin = a["kp"] // self.nv
                rnd, ph = a["s"] // 2 + 1, a["s"] % 2 + 1
                payload = consensus_payload(self.addrs[origin], rnd, ph, self.values[a["value"]])
            else:
                payload = a["payload"]
            self.register(payload, key)
        elif kind == "byz":
            self.byz_send(a["src"], a["type"], (a["kp"], a["s"]), a["dst"])
        elif kind == "deliver":       # ByzantineRandomizedConsensus.deliver(message) called directly
            msg = consensus_payload(self.addrs[a["kp"]], a.get("round", 1), a.get("phase", 1), self.values[a["value"]])
            self.nodes[a["node"]].deliver(msg)
        else:
            raise HarnessError("unknown action %r" % kind)

    # ------------------------------------------------------------------ run
    def run(self, refmods):
        import io
        import contextlib
        actions = defaultdict(list)
        for a in self.spec.get("actions", []):
            actions[a["t"]].append(a)
        rcap = self.spec.get("round_cap", 0)
        tcap = self.spec.get("step_cap", 10000)
        sink = io.StringIO()
        status = None
        try:
            with contextlib.redirect_stdout(sink):
                self.build(refmods)
                self.t = 0
                for a in actions.pop(0, []):
                    self.act(a)
                while True:
                    pending = [x for x in self.arrivals if x > self.t] + [x for x in actions if x > self.t]
                    if not pending:
                        status = "quiescent"
                        break
                    nt = min(pending)
                    if nt > tcap:
                        status = "stepcap"
                        break
                    self.t = nt
                    msgs = self.arrivals.pop(nt, [])
                    if msgs or nt in actions:
                        self.last_active = nt
                    msgs.sort(key=lambda m: (m[1], m[0]))
                    for order, dst, data, src in msgs:
                        if dst in self.servers:
                            self.arrivals_processed += 1
                            self.ports += 1
                            self.servers[dst].hand(data, "n%d" % src, self.ports if self.connection else 0)
                    for a in actions.pop(nt, []):
                        self.act(a)
                    if self.mode == "consensus" and rcap > 0 and all(
                            self.decides[i] >= rcap for i in self.honest):
                        status = "done"
                        break
        finally:
            for srv in self.servers.values():
                srv.stop()
        return {
            "status": status,
            "t_stop": self.last_active,
            "msgs_sent": self.msgs_sent,
            "arrivals": self.arrivals_processed,
            "events": self.events,
            "wire": self.wire,
        }


def run_spec(spec, schedule_cls):
    refmods = _import_reference()
    sch = schedule_cls(spec["n"], spec["f"], spec["seed"], spec["delay_model"], spec["dmax"],
                       spec.get("dconst", 1))
    return Run(spec, sch).run(refmods)
