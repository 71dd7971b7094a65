"""Import alias: ``byzantinerandomizedconsensus.{base,core}`` -> ``byzantinerandomizedconsensus_amd``.

Put this repository on ``PYTHONPATH`` in place of the reference and drivers written against the
reference (``from byzantinerandomizedconsensus.core.brbroadcast import BRBroadcast`` ...) run
unchanged on the MI355X engine.
"""
import importlib
import sys

_MODULES = ["base", "base.broadcast", "base.consensus", "core", "core.brbroadcast",
            "core.byzantinerandomizedconsensus"]

for _m in _MODULES:
    sys.modules[__name__ + "." + _m] = importlib.import_module("byzantinerandomizedconsensus_amd." + _m)
base = sys.modules[__name__ + ".base"]
core = sys.modules[__name__ + ".core"]
