"""cfg5's sweep over f (BASELINE.json configs[4]) through the RCCL path.

sweep.py runs under torch.distributed.run with one rank on GPU 0 and the nccl backend (RCCL: the
histogram all-reduce is the collective an 8-GPU node uses), over f in {0, 42, 85}.  Its round
histograms and counters must equal the plain single-process run (the all-reduce of one rank is
the identity, and the sharding keeps global ids).  At f = 0 and f = 42 four sampled global ids of
the 512-instance batch must equal the C oracle (tests/golden/sweep_oracle.json, made by
tests/golden/make_sweep_oracle.py -- an n = 256 oracle run takes about a minute, so the oracle is
run once there): counters and every honest replica's first decision.

torchrun and the plain sweep run as child processes before this process touches the GPU.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from tests.golden import specs as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VID = {v: i for i, v in enumerate(S.VALUES)}
SWEEP = ["--f", "0,42,85", "--models", "uniform", "--instances", "512"]
SAME = ("instances", "decided", "statuses", "round_hist", "mean_decide_round", "max_decide_round", "msgs_sent",
        "arrivals", "cell_steps")

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _lines(cmd, timeout):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, "rc %d\n%s\n%s" % (p.returncode, p.stdout[-3000:], p.stderr[-3000:])
    out = [json.loads(x) for x in p.stdout.splitlines() if x.strip().startswith("{")]
    assert out, p.stdout[-2000:]
    return {(d["delay"], d["f"]): d for d in out}


def test_sweep_rccl_rank_equals_plain_run():
    dist = _lines([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
                   "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "sweep.py", "--dist"] + SWEEP,
                  600)
    plain = _lines([sys.executable, "sweep.py"] + SWEEP, 600)
    assert sorted(dist) == sorted(plain) == [("uniform", 0), ("uniform", 42), ("uniform", 85)]
    for key, d in dist.items():
        assert d["collective"] == "nccl all-reduce of the histograms", d["collective"]
        assert plain[key]["collective"] is None
        for k in SAME:
            assert d[k] == plain[key][k], (key, k)
        assert d["statuses"]["done"] == 512 and sum(d["round_hist"].values()) == 512
        r = d["roofline"]
        assert r["kernel"] == "brc_step_wide" and r["bytes_per_unit"] == 16 and 0 < r["frac"] < 1


@pytest.mark.parametrize("f", [0, 42])
def test_sweep_batch_matches_oracle_samples(f):
    from byzantinerandomizedconsensus_amd import _lib as L
    from byzantinerandomizedconsensus_amd.engine import Engine
    with open(os.path.join(ROOT, "tests", "golden", "sweep_oracle.json")) as fh:
        g = json.load(fh)
    cases = [c for c in g["cases"] if c["f"] == f]
    assert len(cases) == 4
    # sweep.py's engine for (uniform, f), rank 0 of one
    kw = dict(n=256, f=f, instances=g["instances"], protocol="consensus", seed=g["seed"],
              delay_model=g["delay_model"], delay_max=g["delay_max"], delay_const=1, round_cap=1, step_cap=4000,
              key_window=8, variants=1, proposals=L.PROPOSALS_PHILOX, instance_offset=0, mode=L.MODE_SPEC,
              coin_seed=g["coin_seed"])
    with Engine(**kw) as eng:
        eng.run()
        res = eng.instances_result()
        reps = {c["g"]: eng.replicas(c["g"], 1)[0] for c in cases}
    for c in cases:
        for k in ("status", "t_stop", "msgs_sent", "arrivals", "cell_steps"):
            assert res[c["g"]][k] == c[k], (f, c["g"], k)
        for d, (rep, exp) in enumerate(zip(reps[c["g"]], c["first_decide"])):
            assert exp is not None, (c["g"], d)
            got = (rep["first_decide_round"], rep["first_decide_t"], rep["first_decide_value"])
            assert got == (exp[0], exp[1], VID[exp[2]]), (f, c["g"], d)
