"""The simulated network under the reference's class API.

The reference's transport is one TCP connection per message (``base/broadcast.py:26-40``)
and one listener thread per node (``core/brbroadcast.py:121-128``).  Here the nodes that
share a ``peer_list`` form a ``Cluster``: one single-instance HIP engine (``engine.Engine``,
the same kernels the batched runs use) whose lock-step network replaces the sockets.

* ``Broadcast.broadcast(SEND, m)`` and ``ByzantineRandomizedConsensus.propose(v)`` become
  injections stamped with the cluster's current step.
* ``Cluster.run()`` advances the engine ONE simulated step per launch and replays that step's
  DELIVER / DECIDE events into the user's ``deliver`` / ``decide`` handlers.  The order is
  the reference's processing order for a step: receiver ascending, then key, then (for
  decides) round.  A handler that broadcasts is injected at the same step, so it takes effect
  after that step's messages.
* Nothing runs until the program calls ``run()`` or the interpreter exits (an ``atexit``
  hook), so every ``start()``/``broadcast()`` a driver issues up front lands at step 0.  The
  golden harness fixes the same convention for the reference.

Deviations from the reference, all reported by exceptions and never silent:

* Consensus has no stop in the reference (it re-proposes forever,
  ``core/byzantinerandomizedconsensus.py:102-106``).  Clusters stop once every node has
  decided ``round_cap`` times (``configure``).
* At most seven distinct proposal strings besides ``"-1"`` (three-bit value ids) -- three on
  clusters above 64 nodes (and best-effort broadcast above 32), whose kernels keep two-bit ids.
* A payload SENT by two different origins (or SENT again) is one key in the reference (its
  dicts are keyed by the payload string); the engine models it as one key with extra SENDs
  (brc_step.h extra-SEND records: up to 16 per wave item, shared by the instances packed into
  it) on clusters up to 64 nodes (33..64 nodes with sender peers run the narrow kernel's general
  form for this, brc.h BRC_FLAG_GENERAL_KEYS); above 64 nodes a second origin raises
  ``EngineError``.  A node that SENDs its own payload again with sender peers is a no-op
  everywhere: the network drops a duplicate on every link (tests/golden/refharness.py).
* ``broadcast(type, m)`` takes SEND, ECHO and READY (the reference also puts other types on
  the wire, which its handler then ignores): other types raise ``EngineError``.
* Peer addresses in ``peer_list`` without a constructed node in this process are silent
  (crashed) replicas.
* A direct ``deliver()`` call (``core/byzantinerandomizedconsensus.py:53-60``) must carry a
  string ``"message"`` from a ``"host"`` in the peer list.  The reference keys its value table
  by the raw JSON value (so ``0`` and ``"0"`` are two values there) and adds an unknown host as
  one more origin; the engine's value ids and origin bits cover neither, so both raise
  ``EngineError``.

Peers are identified as the shipped reference identifies them: by connection
(``core/brbroadcast.py:69``; ``configure(peer_mode="sender")`` selects the commented-out :71
line).  Best-effort broadcast keeps no peer sets, so its clusters ignore the setting.
"""
import atexit
import threading

from . import _lib as L

_SETTINGS = {"delay_model": L.DELAY_CONST, "delay_max": 1, "delay_const": 1, "seed": 0,
             "round_cap": 3, "step_cap": 4000, "device": 0, "event_capacity": 1 << 20,
             "instance_id": 0, "peer_mode": "connection"}
_CLUSTERS = {}
_LOCK = threading.Lock()
_ATEXIT = [False]

DELAY_MODELS = {"const": L.DELAY_CONST, "uniform": L.DELAY_UNIFORM, "slowset": L.DELAY_SLOWSET,
                "geometric": L.DELAY_GEOMETRIC}
PEER_MODES = {"connection": L.PEER_CONNECTION, "sender": L.PEER_SENDER}


def configure(**kw):
    """Schedule and stop settings for clusters created afterwards.

    delay_model ('const' | 'uniform' | 'slowset' | 'geometric' or a BRC_DELAY_* id), delay_max,
    delay_const, seed, round_cap, step_cap, device, event_capacity, instance_id (the global
    instance id that keys the Philox schedule draws), peer_mode ('connection', the default:
    how the reference as shipped identifies peers, core/brbroadcast.py:69 -- every message is
    its own connection, nothing is deduplicated and the :119 READY amplification re-fires; or
    'sender', the commented-out :71 line)."""
    for k, v in kw.items():
        if k not in _SETTINGS:
            raise TypeError("unknown network setting %r" % k)
        if k == "peer_mode" and v not in PEER_MODES:
            raise ValueError("peer_mode must be 'connection' or 'sender', not %r" % (v,))
        if k == "delay_model" and isinstance(v, str):
            v = DELAY_MODELS[v]
        _SETTINGS[k] = v


def settings():
    return dict(_SETTINGS)


def _addr(a):
    return tuple(a) if isinstance(a, (list, tuple)) else a


def cluster_for(peer_list):
    key = tuple(_addr(a) for a in peer_list)
    with _LOCK:
        c = _CLUSTERS.get(key)
        if c is None or c.finished:
            c = _CLUSTERS[key] = Cluster(key, dict(_SETTINGS))
        if not _ATEXIT[0]:
            atexit.register(run_all)
            _ATEXIT[0] = True
    return c


def run_all():
    """Run every cluster that has pending work (the atexit hook)."""
    for c in list(_CLUSTERS.values()):
        if c.pending_work():
            c.run()


def reset():
    """Forget every cluster (tests)."""
    with _LOCK:
        for c in _CLUSTERS.values():
            c.close()
        _CLUSTERS.clear()


class ValueTable:
    """Consensus payload strings <-> value ids; id 0 is str(NONE) == "-1"
    (core/byzantinerandomizedconsensus.py:68).  `cap` ids: 8 (three-bit ids) or 4 (include/brc.h
    brc_injection.value)."""

    def __init__(self, cap=8):
        self.strings = ["-1"]
        self.cap = cap

    def id_of(self, s):
        s = str(s)
        if s in self.strings:
            return self.strings.index(s)
        if len(self.strings) == self.cap:
            raise L.EngineError(L.E_UNSUPPORTED, "more than %d distinct proposal values: %r"
                                % (self.cap - 1, self.strings[1:] + [s]))
        self.strings.append(s)
        return len(self.strings) - 1

    def string(self, vid):
        return self.strings[vid]


def order_step_events(events):
    """One step's (kind, node, a, b) events in the reference's processing order: receiver
    ascending (the canonical per-step order of oracle/schedule.py), then key slot / round."""
    return sorted(events, key=lambda e: (e[1], e[2], e[3], e[0]))


class Cluster:
    """All nodes of one peer list, simulated as one engine instance."""

    def __init__(self, peers, cfg):
        self.peers = peers
        self.index = {a: i for i, a in enumerate(peers)}
        self.cfg = cfg
        self.nodes = {}            # replica id -> BRBroadcast
        self.cons = {}             # replica id -> ByzantineRandomizedConsensus
        self.N = self.f = None
        self.t = 0
        self.actions = []          # injections not yet handed to the engine
        self.payload_key = {}      # BRB payload -> (origin, seq)
        self.key_payload = {}      # (origin, seq) -> payload
        self.seq = {}
        self.sent = set()          # keys SENT (a payload may be declared first by an ECHO / READY)
        # three-bit value ids on the narrow kernels that keep them (include/brc.h brc_injection.value)
        n = len(peers)
        # the wide kernel (> 64 nodes): two-bit value ids, one SEND per key.  33..64 nodes with sender peers
        # run the narrow kernel's general form (BRC_FLAG_GENERAL_KEYS), which keeps what n <= 32 keeps
        self.lean_or_wide = n > 64
        self.values = ValueTable(4 if self.lean_or_wide else 8)
        self.engine = None
        self.seen_events = 0
        self.finished = False
        self.status = None
        self.beb = False           # best-effort broadcast nodes (core/bebroadcast.py)

    # ------------------------------------------------------------------ registration
    def node_id(self, host):
        h = _addr(host)
        if h not in self.index:
            raise ValueError("host address %r is not in its own peer_list" % (h,))
        return self.index[h]

    def add_brb(self, node, N, f):
        i = self.node_id(node.host)
        if self.engine is not None:
            raise L.EngineError(L.E_STATE, "node added after the cluster started running")
        if self.beb:
            raise ValueError("BEBroadcast and BRBroadcast nodes cannot share a peer list")
        if self.N is None:
            self.N, self.f = N, f
        elif (self.N, self.f) != (N, f):
            raise ValueError("nodes of one peer list disagree on (N, f)")
        self.nodes[i] = node
        return i

    def add_beb(self, node):
        """A best-effort broadcast node (core/bebroadcast.py): no thresholds, f = 0."""
        i = self.node_id(node.host)
        if self.engine is not None:
            raise L.EngineError(L.E_STATE, "node added after the cluster started running")
        if self.N is not None and not self.beb:
            raise ValueError("BEBroadcast and BRBroadcast nodes cannot share a peer list")
        self.beb = True
        self.N, self.f = len(self.peers), 0
        if self.N > 32:               # best-effort broadcast runs sender peers: two-bit ids past 32 nodes
            if len(self.values.strings) > 4:
                raise L.EngineError(L.E_UNSUPPORTED, "more than 3 distinct proposal values on %d nodes" % self.N)
            self.values.cap = 4
            self.lean_or_wide = True
        self.nodes[i] = node
        return i

    def add_consensus(self, node, i):
        self.cons[i] = node

    @property
    def mode(self):
        return "consensus" if self.cons else "brb"

    def pending_work(self):
        return not self.finished and bool(self.actions)

    # ------------------------------------------------------------------ actions
    def _key_of(self, i, payload):
        """The payload's key; a payload new to the cluster gets the key (i, i's next sequence
        number).  The reference keys its dicts by the payload string (core/brbroadcast.py:38-44)."""
        key = self.payload_key.get(payload)
        if key is None:
            s = self.seq.get(i, 0)
            self.seq[i] = s + 1
            key = (i, s)
            self.payload_key[payload] = key
            self.key_payload[key] = payload
        return key

    def brb_send(self, i, payload):
        """BRBroadcast.broadcast(SEND, payload) by replica i (base/broadcast.py:17-40)."""
        if self.cons:
            raise L.EngineError(L.E_UNSUPPORTED, "raw BRB SENDs on a consensus cluster")
        payload = str(payload)
        key = self._key_of(i, payload)
        sender_peers = self.beb or self.cfg["peer_mode"] == "sender"
        if key[0] == i and key in self.sent and sender_peers and self.lean_or_wide:
            return            # the same node's repeat: a duplicate on every link, nothing travels
        if (key[0] != i or key in self.sent) and self.lean_or_wide:
            raise L.EngineError(L.E_UNSUPPORTED, "payload %r SENT twice (one reference key) on a %d-node cluster "
                                "with %s peers" % (payload, len(self.peers), self.cfg["peer_mode"]))
        self.sent.add(key)
        self.actions.append(dict(t=self.t, kind=L.INJ_SEND, node=i, kp=key[0], s=key[1], value=0,
                                 dst=(1 << len(self.peers)) - 1))

    def brb_msg(self, i, message_type, payload):
        """BRBroadcast.broadcast(ECHO | READY, payload) issued by replica i's own code
        (base/broadcast.py:17 accepts any type): the message goes to every peer, self included,
        exactly as the handler's own ECHO / READY broadcasts do (core/brbroadcast.py:82, :98,
        :119).  A payload nobody has SENT gets a key of its own (declared, never SENT)."""
        if self.cons:
            raise L.EngineError(L.E_UNSUPPORTED, "raw BRB messages on a consensus cluster")
        payload = str(payload)
        new = payload not in self.payload_key
        key = self._key_of(i, payload)
        if new:
            self.actions.append(dict(t=self.t, kind=L.INJ_KEY, node=i, kp=i, s=key[1], value=0))
        self.actions.append(dict(t=self.t, kind=L.INJ_MSG, type=message_type, node=i, kp=key[0], s=key[1],
                                 value=0, dst=(1 << len(self.peers)) - 1))

    def propose(self, i, message):
        """ByzantineRandomizedConsensus.propose (core/byzantinerandomizedconsensus.py:43-50)."""
        self.actions.append(dict(t=self.t, kind=L.INJ_PROPOSE, node=i, value=self.values.id_of(message)))

    def deliver(self, i, host, message):
        """ByzantineRandomizedConsensus.deliver called directly on replica i with a message of
        `host` (a peer address) carrying `message` (core/byzantinerandomizedconsensus.py:53-106):
        the replica's consensus state takes it at the current step, without BRB traffic."""
        if not isinstance(message, str):
            raise L.EngineError(L.E_UNSUPPORTED, "deliver(): message %r is not a string (the engine "
                                "keys values by their string)" % (message,))
        h = _addr(host)
        if h not in self.index:
            raise L.EngineError(L.E_UNSUPPORTED, "deliver(): host %r is not in the peer list" % (h,))
        self.actions.append(dict(t=self.t, kind=L.INJ_DELIVER, node=i, kp=self.index[h],
                                 value=self.values.id_of(message)))

    # ------------------------------------------------------------------ execution
    def _create_engine(self):
        from .engine import Engine
        n = len(self.peers)
        if self.N != n:
            raise ValueError("total_nodes=%d but the peer list has %d addresses" % (self.N, n))
        silent = [i for i in range(n) if i not in self.nodes]
        c = self.cfg
        self.engine = Engine(n=n, f=self.f, instances=1, protocol=self.mode, seed=c["seed"],
                             delay_model=c["delay_model"], delay_max=c["delay_max"],
                             delay_const=c["delay_const"],
                             round_cap=c["round_cap"] if self.cons else 0, step_cap=c["step_cap"],
                             key_window=8, variants=1, byzantine=silent,
                             event_capacity=c["event_capacity"], instance_offset=c["instance_id"],
                             device=c["device"], mode=L.MODE_BEB if self.beb else L.MODE_REFERENCE,
                             peer_mode=L.PEER_SENDER if self.beb else PEER_MODES[c["peer_mode"]],
                             general_keys=not self.beb)

    def _flush(self):
        if self.actions:
            acts, self.actions = self.actions, []
            self.engine.inject(acts)

    def run(self, max_steps=None):
        """Advance until the cluster is quiescent (or done / capped), dispatching upcalls."""
        if self.finished:
            return self.status
        if self.N is None:
            return None
        if self.engine is None:
            self._create_engine()
        steps = 0
        while max_steps is None or steps < max_steps:
            self._flush()
            left = self.engine.run(1)
            steps += 1
            now = self.engine.instances_result(0, 1)[0]
            self._dispatch()
            self.t = max(self.t, now["t_now"])
            if left == 0 and not self.actions:
                break
        self.status = self.engine.instances_result(0, 1)[0]["status"]
        if self.status in ("overflow", "bad_injection"):
            raise L.EngineError(L.E_UNSUPPORTED, "engine stopped with status %s" % self.status)
        if self.status in ("done", "stepcap"):
            self.finished = True
        return self.status

    def _dispatch(self):
        new, self.seen_events = self.engine.events_since(self.seen_events)   # only the new events
        by_t = {}
        for (_inst, t, kind, node, _typ, a, b, _v) in new:
            if kind in (L.EV_DELIVER, L.EV_DECIDE):
                by_t.setdefault(t, []).append((kind, node, a, b))
        for t in sorted(by_t):
            self.t = t
            for kind, node, a, b in order_step_events(by_t[t]):
                if kind == L.EV_DELIVER and not self.cons:
                    # core/brbroadcast.py:115 -> IBroadcastHandler.deliver(payload)
                    self.nodes[node].consensus.deliver(self.key_payload[(a, b)])
                elif kind == L.EV_DECIDE and node in self.cons:
                    # core/byzantinerandomizedconsensus.py:94 -> IConsensusHandler.decide(value)
                    self.cons[node].consensus_user.decide(self.values.string(b))

    def close(self):
        if self.engine is not None:
            self.engine.close()
            self.engine = None
        self.finished = True
