"""MI355X-native batched simulator of sithu/ByzantineRandomizedConsensus's hot path.

Bracha reliable broadcast (core/brbroadcast.py) and the two-phase randomized-consensus round
(core/byzantinerandomizedconsensus.py) run as hand-written CDNA4 HIP kernels over millions of
independent instances (``csrc/brc_engine.hip``), reached through the C-ABI of
``include/brc.h`` (``libbrc_hip.so``, bound with ctypes in ``_lib.py``).

* ``Engine``                 -- batched device-resident instances (bench / parity tests)
* ``base`` / ``core``        -- the reference's class API (Broadcast, IBroadcastHandler,
                                Consensus, IConsensusHandler, BRBroadcast,
                                ByzantineRandomizedConsensus) on top of the engine
"""
from ._lib import EngineError, EngineUnavailable  # noqa: F401

__all__ = ["Engine", "EngineError", "EngineUnavailable"]


def __getattr__(name):
    if name == "Engine":
        from .engine import Engine
        return Engine
    raise AttributeError(name)
