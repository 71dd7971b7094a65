"""Batched engine: Python front-end of the C-ABI (include/brc.h).

``Engine`` owns one device-resident batch of independent consensus instances.  It is the
object the reference-compatible classes (``base/``, ``core/``) and ``bench.py`` drive.
"""
import ctypes

import numpy as np

from . import _lib as L

M64 = (1 << 64) - 1


def _check(lib, handle, rc):
    if rc != L.OK:
        msg = lib.brc_last_error(handle) if handle else b""
        raise L.EngineError(rc, (msg or b"").decode(errors="replace"))


class Engine:
    """One device-resident batch.

    Parameters mirror ``brc_config``; ``byzantine`` is a list of replica ids that run no code.
    """

    def __init__(self, n, f, instances, protocol="consensus", seed=0, delay_model=L.DELAY_CONST,
                 delay_max=1, delay_const=1, round_cap=1, step_cap=4000, key_window=4, variants=1,
                 proposals=L.PROPOSALS_NONE, byz_pattern=L.BYZ_NONE, byzantine=(), event_capacity=0,
                 instance_offset=0, device=0, mode=L.MODE_REFERENCE, coin_seed=0, peer_mode=L.PEER_SENDER,
                 general_keys=False):
        self._lib = L.load()
        self._h = ctypes.c_void_p()
        mask = 0
        for b in byzantine:
            mask |= 1 << int(b)
        proto = {"brb": L.PROTO_BRB, "consensus": L.PROTO_CONSENSUS}.get(protocol, protocol)
        self.cfg = L.Config(n=n, f=f, protocol=proto, peer_mode=peer_mode, instances=instances,
                            instance_offset=instance_offset, seed=seed, delay_model=delay_model,
                            delay_max=delay_max, delay_const=delay_const, round_cap=round_cap,
                            step_cap=step_cap, key_window=key_window, variants=variants,
                            proposals=proposals, byz_pattern=byz_pattern, event_capacity=event_capacity,
                            byzantine_mask=mask & M64, device=device, mode=mode, coin_seed=coin_seed,
                            flags=L.FLAG_GENERAL_KEYS if general_keys else 0)
        for w in range(3):
            self.cfg.byzantine_mask_hi[w] = (mask >> (64 * (w + 1))) & M64
        rc = self._lib.brc_create(ctypes.byref(self.cfg), ctypes.byref(self._h))
        if rc != L.OK:
            why = self._lib.brc_last_error(None) or b""
            raise L.EngineError(rc, "brc_create: %s" % why.decode(errors="replace"))
        self.n, self.f, self.instances = n, f, instances

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if self._h:
            self._lib.brc_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _chk(self, rc):
        _check(self._lib, self._h, rc)

    # ------------------------------------------------------------------ inputs
    def load_proposals(self, proposals):
        arr = np.ascontiguousarray(proposals, dtype=np.int8).reshape(self.instances, self.n)
        self._chk(self._lib.brc_load_proposals(self._h, arr.ctypes.data_as(ctypes.c_void_p)))

    def load_byzantine(self, masks):
        """masks: [instances] (n <= 64) or [instances][(n + 63) // 64] uint64 words (bit d of word
        w = replica 64 w + d is Byzantine)."""
        arr = np.ascontiguousarray(masks, dtype=np.uint64).reshape(self.instances, (self.n + 63) // 64)
        self._chk(self._lib.brc_load_byzantine(self._h, arr.ctypes.data_as(ctypes.c_void_p)))

    def inject(self, items):
        """items: iterable of dicts with keys t, kind, instance, node, kp, s, value, type, dst."""
        items = list(items)
        if not items:
            return
        arr = (L.Injection * len(items))()
        for i, x in enumerate(items):
            a = arr[i]
            a.t = x["t"]
            a.kind = x["kind"]
            a.type = x.get("type", 0)
            a.instance = x.get("instance", 0)
            a.node = x.get("node", 0)
            a.kp = x.get("kp", 0)
            a.s = x.get("s", 0)
            a.value = x.get("value", 0)
            dst = x.get("dst", 0)                  # bit d = replica d (n up to 256)
            a.dst_mask = dst & M64
            for w in range(3):
                a.dst_mask_hi[w] = (dst >> (64 * (w + 1))) & M64
        self._chk(self._lib.brc_inject(self._h, arr, len(items)))

    # ------------------------------------------------------------------ execution
    def run(self, max_steps=0):
        left = ctypes.c_uint32(0)
        self._chk(self._lib.brc_run(self._h, max_steps, ctypes.byref(left)))
        return left.value

    def reset(self):
        self._chk(self._lib.brc_reset(self._h))

    def reset_at(self, instance_offset):
        """Reset and re-key the engine to global instances [instance_offset, +instances) (tiles a
        range larger than one engine's footprint; results equal one engine over the range)."""
        self._chk(self._lib.brc_reset_at(self._h, instance_offset))
        self.cfg.instance_offset = instance_offset

    def last_kernel_ms(self):
        ms = ctypes.c_float(0)
        self._chk(self._lib.brc_last_kernel_ms(self._h, ctypes.byref(ms)))
        return ms.value

    def last_kernel(self):
        """"step" or "life": the kernel the last run() launched (include/brc.h brc_last_kernel)."""
        k = ctypes.c_uint32(0)
        self._chk(self._lib.brc_last_kernel(self._h, ctypes.byref(k)))
        return "life" if k.value == L.KERNEL_LIFE else "step"

    # ------------------------------------------------------------------ outputs
    def instances_result(self, first=0, count=None):
        count = self.instances - first if count is None else count
        arr = (L.InstanceResult * count)()
        self._chk(self._lib.brc_read_instances(self._h, first, count, arr))
        return [{"status": L.STATUS_NAMES.get(r.status, r.status), "t_stop": r.t_stop, "t_now": r.t_now,
                 "decided": bool(r.decided), "msgs_sent": r.msgs_sent, "arrivals": r.arrivals,
                 "cell_steps": r.cell_steps, "deliveries": r.deliveries} for r in arr]

    def replicas(self, first=0, count=None):
        count = self.instances - first if count is None else count
        arr = (L.ReplicaResult * (count * self.n))()
        self._chk(self._lib.brc_read_replicas(self._h, first, count, arr))
        out = []
        for i in range(count):
            out.append([{k: getattr(arr[i * self.n + d], k) for k, _ in L.ReplicaResult._fields_}
                        for d in range(self.n)])
        return out

    def instances_array(self, first=0, count=None):
        """instances_result() as one numpy structured array (brc_instance_result fields, status as
        its numeric code): the bulk read for batches of millions of instances."""
        count = self.instances - first if count is None else count
        arr = (L.InstanceResult * count)()
        self._chk(self._lib.brc_read_instances(self._h, first, count, arr))
        return np.ctypeslib.as_array(arr).copy()

    def replicas_array(self, first=0, count=None):
        """replicas() as one numpy structured array of shape [count, n] (brc_replica_result fields)."""
        count = self.instances - first if count is None else count
        arr = (L.ReplicaResult * (count * self.n))()
        self._chk(self._lib.brc_read_replicas(self._h, first, count, arr))
        return np.ctypeslib.as_array(arr).reshape(count, self.n).copy()

    def events(self):
        """Event log: (instance, t, kind, node, type, a, b, value id) tuples, in device order."""
        cnt = ctypes.c_size_t(0)
        self._chk(self._lib.brc_read_events(self._h, None, 0, ctypes.byref(cnt)))
        cap = min(cnt.value, self.cfg.event_capacity)
        arr = (L.Event * max(1, cap))()
        self._chk(self._lib.brc_read_events(self._h, arr, cap, ctypes.byref(cnt)))
        if cnt.value > self.cfg.event_capacity:
            raise L.EngineError(L.E_STATE, "event log overflow: %d events, capacity %d"
                                % (cnt.value, self.cfg.event_capacity))
        return [(e.instance, e.t, e.kind, e.node, e.type, e.a, e.b, e.value) for e in arr[:cap]]

    def events_since(self, first):
        """Events first .. end of the log, and the new total: incremental draining (the log keeps
        every event since the last reset)."""
        total = ctypes.c_size_t(0)
        self._chk(self._lib.brc_read_events_range(self._h, first, None, 0, ctypes.byref(total)))
        if total.value > self.cfg.event_capacity:
            raise L.EngineError(L.E_STATE, "event log overflow: %d events, capacity %d"
                                % (total.value, self.cfg.event_capacity))
        cap = total.value - first if total.value > first else 0
        arr = (L.Event * max(1, cap))()
        if cap:
            self._chk(self._lib.brc_read_events_range(self._h, first, arr, cap, ctypes.byref(total)))
        return [(e.instance, e.t, e.kind, e.node, e.type, e.a, e.b, e.value) for e in arr[:cap]], total.value

    def decisions(self, labels=("-1", "0", "1", "3")):
        """First decisions of the honest replicas: ({label of value id v: c, "undecided": c},
        instances whose honest replicas decided different values).  labels[v] is the string value
        id v stands for (1 to 8 of them; id 0 is "-1").  The default labels are the wire codec's
        value table (Philox proposals); pass the strings your value ids stand for (e.g. a
        Cluster's value table) to label loaded proposals.  A decided id past the labels raises."""
        labels = tuple(labels)
        if not 1 <= len(labels) <= 8 or len(set(labels)) != len(labels) or "undecided" in labels:
            raise ValueError("labels: 1 to 8 distinct value strings, not 'undecided'")
        arr = np.zeros(9, dtype=np.uint64)
        dis = ctypes.c_uint64(0)
        self._chk(self._lib.brc_read_value_decisions(self._h, arr.ctypes.data_as(ctypes.c_void_p), ctypes.byref(dis)))
        if any(int(x) for x in arr[len(labels):8]):
            raise ValueError("value ids past the %d labels were decided: %s" % (len(labels), [int(x) for x in arr[:8]]))
        out = {labels[v]: int(arr[v]) for v in range(len(labels))}
        out["undecided"] = int(arr[8])
        return out, dis.value

    def round_histogram(self, bins=66):
        """hist[r] = instances whose honest replicas had all decided by round r; hist[0] =
        instances with an undecided honest replica; the last bin holds rounds >= bins - 1."""
        arr = np.zeros(bins, dtype=np.uint64)
        self._chk(self._lib.brc_read_round_histogram(self._h, arr.ctypes.data_as(ctypes.c_void_p), bins))
        return [int(x) for x in arr]

    def stats(self):
        s = L.Stats()
        self._chk(self._lib.brc_read_stats(self._h, ctypes.byref(s)))
        return {k: getattr(s, k) for k, _ in L.Stats._fields_}
