#!/usr/bin/env python3
"""Cell-step counts of every reference fixture, from the C oracle (oracle_cell_steps.json).

    python tests/golden/make_cell_steps.py

A cell-step is a (receiver, key) cell with at least one message landing on it in a step
(DESIGN §4): the unit the rooflines are priced in.  The reference has no such counter, so the
counts come from the C oracle, which reproduces every fixture's events, counters and raw upcall
order (tests/test_oracle_golden.py) -- the counts are the oracle's on schedules pinned by the
reference.  test_oracle_golden.py re-derives them; the GPU parity tests compare the engine's
per-instance cell_steps with them.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle  # noqa: E402
from tests import golden_io  # noqa: E402


def main():
    out = {}
    for group, cases in sorted(golden_io.groups().items()):
        out[group] = [oracle.run(c["spec"], light=True)["cell_steps"] for c in cases]
        print(group, out[group][:4], flush=True)
    with open(os.path.join(HERE, "oracle_cell_steps.json"), "w") as fh:
        json.dump({"group": "oracle_cell_steps", "cases": out,
                   "note": "C-oracle cell-step counts of the reference fixtures (make_cell_steps.py)"},
                  fh, indent=0, sort_keys=True)


if __name__ == "__main__":
    main()
