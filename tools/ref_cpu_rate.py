#!/usr/bin/env python3
"""Time the reference's OWN Python path on the bench workload (build container only).

    python -O tools/ref_cpu_rate.py [instances] [processes]   -> profiles/ref_cpu_rate.json

Each instance of SURVEY §8(d) cfg4 (n=64, f=21, slow-set delays D=8, Philox proposals, reference
protocol to the first decision -- exactly bench.py's reference leg) is run through the UNMODIFIED
reference classes by tests/golden/refharness.py (lock-step fake-socket transport; every message
goes through the reference's JSON encode, listener loop and consensus deliver).  Instances run
in separate processes, one per core; the harness is GIL-bound, so one instance uses one core.
Reported: decided instances/s and replica-message-steps/s (messages processed by honest
replicas, the reference's accept-loop iterations core/brbroadcast.py:60-119), with the core
count.  `-O` strips the reference's N > 5f assert (core/byzantinerandomizedconsensus.py:20).

The reference exists only in this container: never on the GPU box, never in bench.py.
"""
import json
import multiprocessing as mp
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.dont_write_bytecode = True          # nothing is written into the reference tree


def one(g):
    from oracle.schedule import Schedule
    from tests.golden import specs as S
    from tests.golden.refharness import run_spec
    sp = S.cons_spec(64, 21, 0x5EED0004, 2, 8, g, round_cap=1)
    t0 = time.perf_counter()
    r = run_spec(sp, Schedule)
    return g, r["status"], r["arrivals"], time.perf_counter() - t0


def main():
    if not os.path.isdir("/root/reference"):
        sys.exit("the reference is not present here (build container only)")
    if __debug__:
        sys.exit("run with python -O (the cfg4 consensus violates the reference's N > 5f assert)")
    count = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    procs = int(sys.argv[2]) if len(sys.argv) > 2 else min(count, os.cpu_count() or 1)
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(procs) as pool:
        rows = pool.map(one, range(count))
    wall = time.perf_counter() - t0
    busy = sum(r[3] for r in rows)
    arrivals = sum(r[2] for r in rows)
    decided = sum(r[1] == "done" for r in rows)
    out = {
        "what": "reference Python path (unmodified classes via tests/golden/refharness.py), cfg4 reference "
                "protocol to first decision, global ids 0..%d" % (count - 1),
        "instances": count, "decided": decided, "processes": procs, "wall_s": wall,
        "per_core_instances_per_s": decided / busy,
        "per_core_replica_message_steps_per_s": arrivals / busy,
        "node_instances_per_s": decided / wall,
        "arrivals_per_instance": arrivals / count,
        "cpu": platform.processor() or platform.machine(), "cpus_visible": os.cpu_count(),
        "python": platform.python_version(),
        "per_instance_s": [round(r[3], 2) for r in rows],
    }
    path = os.path.join(ROOT, "profiles", "ref_cpu_rate.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
