"""ctypes binding of ``libbrc_hip.so`` (the C-ABI declared in ``include/brc.h``).

There is deliberately no fallback: if the HIP library is missing or cannot be loaded the
import of any engine-backed class raises ``EngineUnavailable``.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libbrc_hip.so"
LIB_PATH = os.environ.get("BRC_LIB") or os.path.join(_HERE, LIB_NAME)   # BRC_LIB: dev A/B builds only

ABI_VERSION = 7

OK, E_INVALID, E_NOMEM, E_HIP, E_UNSUPPORTED, E_STATE = 0, -1, -2, -3, -4, -5
ERRORS = {E_INVALID: "invalid argument", E_NOMEM: "out of memory", E_HIP: "HIP error",
          E_UNSUPPORTED: "unsupported workload feature", E_STATE: "invalid engine state"}

PROTO_BRB, PROTO_CONSENSUS = 0, 1
MODE_REFERENCE, MODE_SPEC, MODE_BEB = 0, 1, 2
FLAG_GENERAL_KEYS = 1       # brc.h BRC_FLAG_GENERAL_KEYS (ABI v7)
PEER_SENDER, PEER_CONNECTION = 0, 1
DELAY_CONST, DELAY_UNIFORM, DELAY_SLOWSET, DELAY_GEOMETRIC = 0, 1, 2, 3
PROPOSALS_NONE, PROPOSALS_PHILOX, PROPOSALS_LOADED = 0, 1, 2
BYZ_NONE, BYZ_EQUIVOCATE = 0, 1
SEND, ECHO, READY = 1, 2, 3
INJ_PROPOSE, INJ_SEND, INJ_KEY, INJ_MSG, INJ_DELIVER = 1, 2, 3, 4, 5
RUNNING, DONE, QUIESCENT, STEPCAP, OVERFLOW, BADINJ = 0, 1, 2, 3, 4, 5
STATUS_NAMES = {RUNNING: "running", DONE: "done", QUIESCENT: "quiescent", STEPCAP: "stepcap",
                OVERFLOW: "overflow", BADINJ: "bad_injection"}
EV_DELIVER, EV_DECIDE, EV_SEND, EV_COPY = 1, 2, 3, 4
KERNEL_STEP, KERNEL_LIFE = 0, 1

EXPORTS = ["brc_create", "brc_load_proposals", "brc_load_byzantine", "brc_inject", "brc_run",
           "brc_reset", "brc_read_instances", "brc_read_replicas", "brc_read_events",
           "brc_read_stats", "brc_read_round_histogram", "brc_read_decisions", "brc_read_value_decisions", "brc_reset_at",
           "brc_read_events_range", "brc_last_kernel_ms", "brc_last_kernel", "brc_device_count", "brc_last_error",
           "brc_destroy", "brc_abi_version"]


class EngineUnavailable(RuntimeError):
    pass


class EngineError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (%d): %s" % (ERRORS.get(code, "error"), code, msg))
        self.code = code
        self.code = code


class Config(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("f", ctypes.c_uint32), ("protocol", ctypes.c_uint32),
                ("peer_mode", ctypes.c_uint32), ("instances", ctypes.c_uint64),
                ("instance_offset", ctypes.c_uint64), ("seed", ctypes.c_uint64),
                ("delay_model", ctypes.c_uint32), ("delay_max", ctypes.c_uint32),
                ("delay_const", ctypes.c_uint32), ("round_cap", ctypes.c_uint32),
                ("step_cap", ctypes.c_uint32), ("key_window", ctypes.c_uint32),
                ("variants", ctypes.c_uint32), ("proposals", ctypes.c_uint32),
                ("byz_pattern", ctypes.c_uint32), ("event_capacity", ctypes.c_uint32),
                ("byzantine_mask", ctypes.c_uint64), ("device", ctypes.c_int32),
                ("mode", ctypes.c_uint32), ("coin_seed", ctypes.c_uint64),
                ("byzantine_mask_hi", ctypes.c_uint64 * 3), ("flags", ctypes.c_uint32), ("reserved", ctypes.c_uint32 * 3)]


class Injection(ctypes.Structure):
    _fields_ = [("t", ctypes.c_uint32), ("kind", ctypes.c_uint16), ("type", ctypes.c_uint16),
                ("instance", ctypes.c_uint64), ("node", ctypes.c_uint32), ("kp", ctypes.c_uint32),
                ("s", ctypes.c_uint32), ("value", ctypes.c_int32), ("dst_mask", ctypes.c_uint64),
                ("dst_mask_hi", ctypes.c_uint64 * 3)]


class InstanceResult(ctypes.Structure):
    _fields_ = [("status", ctypes.c_uint32), ("t_stop", ctypes.c_uint32), ("t_now", ctypes.c_uint32),
                ("decided", ctypes.c_uint32), ("msgs_sent", ctypes.c_uint64),
                ("arrivals", ctypes.c_uint64), ("cell_steps", ctypes.c_uint64),
                ("deliveries", ctypes.c_uint64)]


class ReplicaResult(ctypes.Structure):
    _fields_ = [("round", ctypes.c_uint32), ("phase", ctypes.c_uint32), ("value_count", ctypes.c_uint32),
                ("decide_count", ctypes.c_uint32), ("first_decide_round", ctypes.c_uint32),
                ("first_decide_t", ctypes.c_uint32), ("first_decide_value", ctypes.c_int32),
                ("last_decide_value", ctypes.c_int32)]


class Event(ctypes.Structure):
    _fields_ = [("instance", ctypes.c_uint64), ("t", ctypes.c_uint32), ("kind", ctypes.c_uint8),
                ("node", ctypes.c_uint8), ("type", ctypes.c_uint8), ("value", ctypes.c_uint8),
                ("a", ctypes.c_uint32), ("b", ctypes.c_uint32)]


class Stats(ctypes.Structure):
    _fields_ = [(name, ctypes.c_uint64) for name in (
        "instances", "running", "done", "quiescent", "stepcap", "overflow", "decided",
        "msgs_sent", "arrivals", "cell_steps", "deliveries", "decide_rounds_sum", "max_t",
        "events_dropped", "lane_loads")]


_lib = None


def load():
    """Load the HIP library (raises EngineUnavailable if it is absent or broken)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EngineUnavailable("%s not built (run __graft_entry__.build())" % LIB_PATH)
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as exc:
        raise EngineUnavailable("cannot load %s: %s" % (LIB_PATH, exc))
    vp = ctypes.c_void_p
    sig = {
        "brc_create": ([ctypes.POINTER(Config), ctypes.POINTER(vp)], ctypes.c_int),
        "brc_load_proposals": ([vp, ctypes.c_void_p], ctypes.c_int),
        "brc_load_byzantine": ([vp, ctypes.c_void_p], ctypes.c_int),
        "brc_inject": ([vp, ctypes.POINTER(Injection), ctypes.c_size_t], ctypes.c_int),
        "brc_run": ([vp, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
        "brc_reset": ([vp], ctypes.c_int),
        "brc_read_instances": ([vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(InstanceResult)], ctypes.c_int),
        "brc_read_replicas": ([vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ReplicaResult)], ctypes.c_int),
        "brc_read_events": ([vp, ctypes.POINTER(Event), ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
        "brc_read_stats": ([vp, ctypes.POINTER(Stats)], ctypes.c_int),
        "brc_read_round_histogram": ([vp, ctypes.c_void_p, ctypes.c_uint32], ctypes.c_int),
        "brc_read_decisions": ([vp, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
        "brc_read_value_decisions": ([vp, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
        "brc_reset_at": ([vp, ctypes.c_uint64], ctypes.c_int),
        "brc_read_events_range": ([vp, ctypes.c_size_t, ctypes.POINTER(Event), ctypes.c_size_t,
                                   ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
        "brc_last_kernel_ms": ([vp, ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
        "brc_last_kernel": ([vp, ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
        "brc_device_count": ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        "brc_last_error": ([vp], ctypes.c_char_p),
        "brc_destroy": ([vp], None),
        "brc_abi_version": ([], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    if L.brc_abi_version() != ABI_VERSION:
        raise EngineUnavailable("ABI version mismatch: library %d, bindings %d" % (L.brc_abi_version(), ABI_VERSION))
    _lib = L
    return L


def device_count():
    c = ctypes.c_int(0)
    load().brc_device_count(ctypes.byref(c))
    return c.value
