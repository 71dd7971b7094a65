#!/usr/bin/env python3
"""Oracle-sampled expectations for the cfg5 sweep over f (BASELINE.json configs[4]):
tests/golden/sweep_oracle.json -- n = 256, SPEC protocol, uniform[1,4] delays, f in {0, 42}, 4
sampled global ids of a 512-instance batch per f.

    python tests/golden/make_sweep_oracle.py [processes]

Same format and purpose as make_cfg5_oracle.py (which covers f = 85 under three delay models): the
C oracle (oracle/brc_oracle.c, the checker -- never the product) runs once per sampled id here, and
tests/test_gpu_sweep.py compares the engine's batch with these ids.  Not a reference fixture (its
group name starts with "oracle_").
"""
import json
import multiprocessing as mp
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

N, SEED, COIN, COUNT = 256, 0x5EED0005, 0xC017C017, 512     # sweep.py's seed / coin / BINS-independent
MODEL, DMAX = 1, 4                                            # uniform [1, 4] (sweep.py MODELS["uniform"])
FS = (0, 42)
PER_F = 4


def sample_ids(f):
    return sorted(random.Random(7000 + f).sample(range(COUNT), PER_F))


def one(job):
    from oracle import oracle
    from tests.golden import specs as S
    f, g = job
    sp = S.spec_cons_spec(N, f, SEED, MODEL, DMAX, g, round_cap=1, window=8, coin_seed=COIN)
    r = oracle.run(sp)
    first = {}
    for t, node, rnd, val in sorted(r["events"]["decide"]):
        first.setdefault(node, [rnd, t, val])
    return {"f": f, "g": g, "status": r["status"], "t_stop": r["t_stop"], "msgs_sent": r["msgs_sent"],
            "arrivals": r["arrivals"], "cell_steps": r["cell_steps"], "first_decide": [first.get(d) for d in range(N)]}


def main():
    procs = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    jobs = [(f, g) for f in FS for g in sample_ids(f)]
    with mp.get_context("fork").Pool(procs) as pool:
        cases = pool.map(one, jobs)
    out = {"group": "oracle_sweep_n256", "what": __doc__.strip().splitlines()[0], "n": N, "seed": SEED,
           "coin_seed": COIN, "delay_model": MODEL, "delay_max": DMAX, "instances": COUNT, "cases": cases}
    path = os.path.join(ROOT, "tests", "golden", "sweep_oracle.json")
    with open(path, "w") as fh:
        json.dump(out, fh, separators=(",", ":"))
    print("wrote", path, len(cases), "cases")


if __name__ == "__main__":
    main()
