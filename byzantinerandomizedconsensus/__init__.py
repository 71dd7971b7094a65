"""Import alias: ``byzantinerandomizedconsensus.{base,core}`` -> ``byzantinerandomizedconsensus_amd``.

Put this repository on ``PYTHONPATH`` in place of the reference and drivers written against the
reference (``from byzantinerandomizedconsensus.core.brbroadcast import BRBroadcast`` ...) run
unchanged on the MI355X engine.
"""
import importlib
import sys

# network first: the core modules import it relatively (``from .. import network``), and every
# alias must resolve to the one module object so all of them share one cluster registry
_MODULES = ["network", "base", "base.broadcast", "base.consensus", "core", "core.brbroadcast",
            "core.byzantinerandomizedconsensus", "core.bebroadcast"]

for _m in _MODULES:
    sys.modules[__name__ + "." + _m] = importlib.import_module("byzantinerandomizedconsensus_amd." + _m)
base = sys.modules[__name__ + ".base"]
core = sys.modules[__name__ + ".core"]
