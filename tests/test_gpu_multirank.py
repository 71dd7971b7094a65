"""The engine's multi-rank path on the GPU: bench.py under torch.distributed.run, 2 ranks.

Both ranks share GPU 0 and reduce over gloo (rehearsal backend: the RCCL all-reduce is the same
`shard.reduce_stats` call with backend "nccl" on an 8-GPU node).  Each rank runs its contiguous
shard of global instance ids through the HIP engine -- the code path the driver's multi-GPU bench
takes -- and the all-reduced totals must equal ONE rank running every id: Philox draws use global
ids, so the job's results do not depend on the rank count (weak scaling, no
data-path exchange).  Three legs (reference protocol, SPEC coin rounds, the reference protocol to
round cap 8) are checked.

torchrun and the single-rank bench are started as child processes before this process touches
the GPU in this test; nothing replaces a GPU process image.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PER_RANK, WORLD = 4096, 2
KEYS = ("decided_fraction", "decide_round_hist", "decided_value_hist", "agreement_violations", "counts")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _last_json(out):
    for line in reversed(out.strip().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            return json.loads(line)
    raise AssertionError("no JSON line in bench output:\n" + out[-2000:])


def _run(cmd, timeout):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, "rc %d\n%s\n%s" % (p.returncode, p.stdout[-3000:], p.stderr[-3000:])
    return _last_json(p.stdout)


def _legs(d):
    out = {"reference": {k: d[k] for k in KEYS}}
    for leg in ("spec", "many", "long", "spec64", "ref2c", "spec2c"):
        if leg + "_leg" in d:
            out[leg] = {k: d[leg + "_leg"][k] for k in KEYS}
    return out


@pytest.mark.gpu
def test_two_ranks_equal_one_rank_over_the_same_global_ids():
    bench_args = ["--steps", "1", "--warmup", "0", "--no-cpu", "--legs", "reference,spec,many,long,spec64,ref2c,spec2c"]
    multi = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(WORLD),
                  "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
                  "--gpus", str(WORLD), "--backend", "gloo", "--instances", str(PER_RANK)] + bench_args, 300)
    single = _run([sys.executable, "bench.py", "--instances", str(PER_RANK * WORLD)] + bench_args, 300)
    assert multi["n_gpus"] == WORLD and single["n_gpus"] == 1
    assert multi["config"]["instances_per_gpu"] * WORLD == single["config"]["instances_per_gpu"]
    m, s = _legs(multi), _legs(single)
    for leg in ("reference", "spec", "many", "long", "spec64", "ref2c", "spec2c"):
        assert m[leg]["counts"]["instances"] == PER_RANK * WORLD
        assert m[leg]["counts"]["decided"] > 0
        assert m[leg] == s[leg], leg
    # the two-class lifetime legs run the step-kernel legs' workloads: the same results (lane_loads and max_t
    # are kernel-specific: the step kernel's row loads and last touched step)
    for a, b in (("reference", "ref2c"), ("spec", "spec2c")):
        ca = {k: v for k, v in s[a]["counts"].items() if k not in ("lane_loads", "max_t")}
        cb = {k: v for k, v in s[b]["counts"].items() if k not in ("lane_loads", "max_t")}
        assert ca == cb and {k: v for k, v in s[a].items() if k != "counts"} == \
            {k: v for k, v in s[b].items() if k != "counts"}, (a, b)


@pytest.mark.gpu
def test_rccl_rank_equals_plain_run():
    """One rank under torch.distributed.run with the nccl backend (= RCCL on ROCm), process group
    bound to the GPU (`device_id`): the statistics go through the device all-reduce of
    `shard.reduce_stats` / `max_over_ranks` -- the 8-GPU path's collective, run on the one leased
    GPU -- and must equal the plain single-process run over the same global ids."""
    bench_args = ["--steps", "1", "--warmup", "0", "--no-cpu", "--legs", "reference,spec,many",
                  "--instances", str(PER_RANK * WORLD)]
    rccl = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
                 "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
                 "--gpus", "1", "--backend", "nccl", "--dist"] + bench_args, 300)
    single = _run([sys.executable, "bench.py"] + bench_args, 300)
    assert rccl["collective"] == "nccl all-reduce of the statistics"
    assert single["collective"] is None
    r, s = _legs(rccl), _legs(single)
    for leg in ("reference", "spec", "many"):
        assert r[leg]["counts"]["decided"] > 0
        assert r[leg] == s[leg], leg
