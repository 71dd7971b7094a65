#!/usr/bin/env python3
"""Dev-only: per-section cycle split of the narrow (or, n > 128, the wide) step kernel.
Needs a variant built with -DBRC_STAMPS (tools/variant.py stamps -DBRC_STAMPS); run with
BRC_LIB=exp/stamps/libbrc_hip.so python tools/stamps.py [instances] [reference|spec|<configs.py workload>] [life]
(life: the key-lifetime kernel's sections, e.g. `tools/stamps.py 262144 cfg4-ref-r64 life`)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from byzantinerandomizedconsensus_amd import _lib as L  # noqa: E402
from byzantinerandomizedconsensus_amd.engine import Engine  # noqa: E402

inst = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
which = sys.argv[2] if len(sys.argv) > 2 else "reference"
life = len(sys.argv) > 3 and sys.argv[3] == "life"
os.environ["BRC_KERNEL"] = "life" if life else "step"
if which in ("reference", "spec"):
    spec = which == "spec"
    eng = Engine(n=64, f=21, instances=inst, protocol="consensus", seed=0x5EED0004, delay_model=L.DELAY_SLOWSET,
                 delay_max=8, round_cap=1, step_cap=4000, key_window=8 if spec else 4, variants=1,
                 proposals=L.PROPOSALS_PHILOX, mode=L.MODE_SPEC if spec else L.MODE_REFERENCE, coin_seed=0xC017C017)
else:
    import configs
    _size, _per, kw = configs.workloads(L)[which]
    kw = {k: v for k, v in kw.items() if k != "kernel"}
    eng = Engine(instances=inst, **kw)
lib = ctypes.CDLL(os.environ["BRC_LIB"])
out = (ctypes.c_ulonglong * 12)()
dbg = lib.brc_dbg_stamps_life if life else lib.brc_dbg_stamps16 if eng.n <= 16 else lib.brc_dbg_stamps256 if eng.n > 128 else lib.brc_dbg_stamps   # per unit
eng.reset(); eng.run()
dbg(out)
eng.reset(); eng.run()
dbg(out)
tot = sum(out[:8])
wide = eng.n > 128
names = ["step head", "class-code reads (HM)", "consensus words", "sends + stop checks", "lifetime simulation"] if life else ["step head + key list", "ballots", "barrier + next fetch", "arrival counts", "pass end + consensus",
         "sends, actions, stop", "cell update + store", "ring marks / t_quiet"] if wide else ["step head + key list", "key loop (BRB cells)", "consensus words", "actions", "stop checks",
         "consensus snapshot", "consensus row clears", "key-loop tail (ring rows)"]
for nm, v in zip(names, out[:8]):
    print("%-24s %6.1f %%  (%.3g ticks)" % (nm, 100.0 * v / tot, v))
kn = ["key-steps processed", "  no arrivals", "  only delivered cells", "  updated"]
for nm, v in zip(kn if not (wide or life) else [], out[8:]):
    print("%-24s %.4g  (%.1f %%)" % (nm, v, 100.0 * v / max(1, out[8])))
print("kernel ms %.2f" % eng.last_kernel_ms())
