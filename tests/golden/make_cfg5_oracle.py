#!/usr/bin/env python3
"""Oracle-sampled expectations for BASELINE.json cfg5 (n=256 f=85, SPEC protocol, 512 instances
per delay model): tests/golden/cfg5_oracle.json.

    python tests/golden/make_cfg5_oracle.py [processes]

An n = 256 oracle run takes 40-90 s, too long to repeat inside a GPU test per instance, so the C
oracle (oracle/brc_oracle.c, the checker -- never the product) is run here once per sampled
global id and its results are committed: status, last step, message counts, and every honest
replica's first decision (round, step, value).  tests/test_gpu_fullsize.py compares the HIP
engine's full 512-instance batch with these ids.  The file is not a reference fixture (its group
name starts with "oracle_", and golden_io.groups() leaves such files out).
"""
import json
import multiprocessing as mp
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

N, F, SEED, COIN, COUNT = 256, 85, 0x5EED0005, 0xC017C017, 512
MODELS = [(0, 1), (1, 4), (3, 16)]          # const D=1, uniform [1,4], geometric cap 16 (configs.py cfg5)
PER_MODEL = 16


def sample_ids(model):
    return sorted(random.Random(5000 + model).sample(range(COUNT), PER_MODEL))


def one(job):
    from oracle import oracle
    from tests.golden import specs as S
    model, dmax, g = job
    sp = S.spec_cons_spec(N, F, SEED, model, dmax, g, round_cap=1, window=8, coin_seed=COIN)
    r = oracle.run(sp)
    first = {}
    for t, node, rnd, val in sorted(r["events"]["decide"]):
        first.setdefault(node, [rnd, t, val])
    return {"model": model, "dmax": dmax, "g": g, "status": r["status"], "t_stop": r["t_stop"],
            "msgs_sent": r["msgs_sent"], "arrivals": r["arrivals"], "cell_steps": r["cell_steps"],
            "first_decide": [first.get(d) for d in range(N)]}


def main():
    procs = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    jobs = [(m, d, g) for m, d in MODELS for g in sample_ids(m)]
    with mp.get_context("fork").Pool(procs) as pool:
        cases = pool.map(one, jobs)
    out = {"group": "oracle_cfg5_n256", "what": __doc__.strip().splitlines()[0],
           "n": N, "f": F, "seed": SEED, "coin_seed": COIN, "instances": COUNT, "cases": cases}
    path = os.path.join(ROOT, "tests", "golden", "cfg5_oracle.json")
    with open(path, "w") as fh:
        json.dump(out, fh, separators=(",", ":"))
    print("wrote", path, len(cases), "cases")


if __name__ == "__main__":
    main()
