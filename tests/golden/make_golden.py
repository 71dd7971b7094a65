#!/usr/bin/env python3
"""Generate the golden fixtures from the REAL reference (build container only).

    python -O tests/golden/make_golden.py            # writes tests/golden/*.json
    python -O tests/golden/make_golden.py --fuzz 300 # extra random oracle-vs-reference check

Every spec of ``specs.scenario_groups()`` is run through the unmodified reference classes by
``refharness.py`` (lock-step fake-socket transport) and, as a generation-time cross-check,
through the C oracle; the two must agree exactly.  The fixtures hold only inputs (the spec)
and the reference's outputs (status, message counts, ordered delivery/decide/send events).
``-O`` is required because the consensus configs violate the reference's ``N > 5f`` assert
(``core/byzantinerandomizedconsensus.py:20``); asserts guard nothing else it runs.
"""
import argparse
import hashlib
import json
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.schedule import Schedule  # noqa: E402
from oracle import oracle  # noqa: E402
from tests.golden import specs as S  # noqa: E402
from tests.golden.refharness import run_spec  # noqa: E402

FULL_EVENT_LIMIT = 6000


def digest(rows):
    return hashlib.sha256(json.dumps(rows, separators=(",", ":")).encode()).hexdigest()


def canonical(result):
    """Event lists in canonical sorted order (the engine reports events per step, not in the
    reference's processing order; within a (step, node) both orders are (kp, s))."""
    ev = result["events"]
    key = lambda r: [str(x) if isinstance(x, str) else x for x in r]  # noqa: E731
    out = dict(result)
    out["events"] = {k: sorted(map(list, ev[k]), key=key) for k in ("deliver", "decide", "send")}
    return out


def compact(result):
    raw = result["events"]
    result = canonical(result)
    ev = result["events"]
    out = {k: result[k] for k in ("status", "t_stop", "msgs_sent", "arrivals")}
    out["counts"] = {k: len(v) for k, v in ev.items()}
    out["digest"] = {k: digest(v) for k, v in ev.items()}
    total = sum(len(v) for v in ev.values())
    out["events"] = ev if total <= FULL_EVENT_LIMIT else {"decide": ev["decide"]}
    # the upcalls in the order the reference issued them (each kind on its own), for small runs:
    # pins the per-step order the class API replays, not only the canonical sort
    if total <= FULL_EVENT_LIMIT:
        out["raw_order"] = {k: [list(r) for r in raw[k]] for k in ("deliver", "decide")}
    return out


def same(a, b):
    return all(a[k] == b[k] for k in ("status", "t_stop", "msgs_sent", "arrivals")) and a["events"] == b["events"]


def fuzz_specs(count, rng):
    out = []
    for i in range(count):
        mode = rng.choice(["brb", "consensus"])
        n = rng.choice([4, 5, 6, 7, 8, 10, 13])
        f = rng.randint(0, (n - 1) // 3)
        model = rng.randint(0, 3)
        dmax = rng.randint(1, 6) if model else 1
        seed = rng.getrandbits(40)
        g = rng.getrandbits(20)
        if mode == "brb":
            sends = [(rng.randint(0, 6), o, q) for o in range(n) for q in range(rng.randint(0, 2))]
            sp = S.brb_spec(n, f, seed, model, dmax, g, sends)
        else:
            sp = S.cons_spec(n, f, seed, model, dmax, g, round_cap=rng.randint(1, 3),
                             starts=[rng.choice([0, 0, 0, rng.randint(1, 8)]) for _ in range(n)])
        sp["name"] = "fuzz/%d" % i
        out.append(sp)
    return out


def wire_specs():
    """Small runs whose every wire message (the bytes base/broadcast.py:37-38 puts on a TCP
    connection) is kept: BRB, consensus, and a Byzantine equivocator."""
    G = S.scenario_groups()
    K = {sp["name"]: sp for sp in G["conn_kat"]}
    # connection-identity peers (core/brbroadcast.py:69): every broadcast is on the wire, the :119
    # READY re-fires (K4, K12) and repeated Byzantine messages (K5) included
    return [G["brb_fifo_n4"][0], G["cons_brc_test_n6"][0], G["cons_uniform_n4"][0], G["brb_byz_n7"][0],
            G["conn_brb_fifo_n4"][0], G["conn_cons_brc_test_n6"][0], K["K4-conn"], K["K5-conn"], K["K12-conn"],
            G["conn_brb_usermsg_n7"][1]]


def write_wire():
    cases = []
    for sp in wire_specs():
        ref = run_spec(sp, Schedule)
        wire = sorted(ref["wire"])
        cases.append({"spec": sp, "wire": wire, "result": compact(ref)})
        print("%-24s %6d wire messages" % (sp["name"], len(wire)))
    with open(os.path.join(HERE, "wire.json"), "w") as fh:
        json.dump({"group": "wire", "generator": "tests/golden/make_golden.py --wire",
                   "source": "unmodified reference classes via tests/golden/refharness.py; addresses "
                             "('localhost', 7000 + node)", "cases": cases}, fh, separators=(",", ":"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fuzz", type=int, default=0)
    ap.add_argument("--only", default=None)
    ap.add_argument("--wire", action="store_true", help="write tests/golden/wire.json (SURVEY F2)")
    args = ap.parse_args()
    if __debug__:
        sys.exit("run with python -O (the reference asserts N > 5f)")
    if args.fuzz:
        rng = random.Random(20261015)
        bad = 0
        t0 = time.time()
        for sp in fuzz_specs(args.fuzz, rng):
            ref = run_spec(sp, Schedule)
            orc = oracle.run(sp)
            if not same(ref, orc):
                bad += 1
                print("MISMATCH", sp["name"], json.dumps(sp)[:300])
        print("fuzz: %d specs, %d mismatches, %.1fs" % (args.fuzz, bad, time.time() - t0))
        sys.exit(1 if bad else 0)
    if args.wire:
        write_wire()
        return
    groups = S.scenario_groups()
    for name, specs in groups.items():
        if args.only and name != args.only:
            continue
        t0 = time.time()
        cases = []
        for sp in specs:
            ref = run_spec(sp, Schedule)
            orc = oracle.run(sp)
            if not same(ref, orc):
                print("ORACLE MISMATCH in", sp["name"])
                for k in ("status", "t_stop", "msgs_sent", "arrivals"):
                    print("  ", k, ref[k], orc[k])
                for k in ref["events"]:
                    if ref["events"][k] != orc["events"][k]:
                        print("  events", k, len(ref["events"][k]), len(orc["events"][k]))
                sys.exit(1)
            cases.append({"spec": sp, "result": compact(ref)})
        path = os.path.join(HERE, name + ".json")
        with open(path, "w") as fh:
            json.dump({"group": name, "generator": "tests/golden/make_golden.py",
                       "source": "unmodified reference classes via tests/golden/refharness.py",
                       "cases": cases}, fh, separators=(",", ":"))
        print("%-24s %3d cases  %6.1fs  %s" % (name, len(cases), time.time() - t0,
                                              [c["result"]["status"] for c in cases][:6]))


if __name__ == "__main__":
    main()
