"""bench.py / configs.py leg definitions (CPU): the headline and its SPEC leg pin the step kernel (the
general per-receiver path), the two-class lifetime legs run the same workloads on the key-lifetime
kernel, and every leg's workload string names the kernel form it measures."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import configs  # noqa: E402


def test_headline_legs_pin_the_step_kernel():
    assert bench.LEGS["reference"][5] == "step" and bench.LEGS["spec"][5] == "step"
    assert bench.LEGS["spec64"][5] == "step"
    # the many-round and connection-peer legs take the engine's own choice (the lifetime kernel)
    for leg in ("conn", "connu", "many", "long"):
        assert bench.LEGS[leg][5] is None


def test_two_class_legs_mirror_their_step_kernel_legs():
    for a, b in (("reference", "ref2c"), ("spec", "spec2c")):
        assert bench.LEGS[a][:5] == bench.LEGS[b][:5]
        assert bench.LEGS[b][5] == "life"
        assert "two-class" in bench.workload_name(b, 1, 1 << 20)
        assert "step kernel" in bench.workload_name(a, 1, 1 << 20)
    # the headline is the first leg of the default run
    old = sys.argv
    try:
        sys.argv = ["bench.py"]
        args = bench.parse()
    finally:
        sys.argv = old
    assert args.legs[0] == "reference" and {"ref2c", "spec2c"} <= set(args.legs)


def test_configs_two_class_rows_mirror_their_step_rows():
    class L:                         # the constants configs.workloads reads (no HIP library needed)
        DELAY_UNIFORM, DELAY_SLOWSET = 1, 2
        PROPOSALS_PHILOX = 1
        MODE_SPEC, MODE_BEB = 1, 2
        BYZ_EQUIVOCATE = 1
        PEER_CONNECTION = 1
    W = configs.workloads(L)
    for base in ("cfg4-ref", "cfg4-spec", "cfg4-beb", "cfg4-spec-r64"):
        sz, per, kw = W[base]
        sz2, per2, kw2 = W[base + "-2c"]
        assert kw["kernel"] == "step" and kw2["kernel"] == "life"
        assert (sz, per) == (sz2, per2)
        assert {k: v for k, v in kw.items() if k != "kernel"} == {k: v for k, v in kw2.items() if k != "kernel"}
    assert configs.BENCH_LEGS["cfg4-ref-2c"] == "ref2c" and configs.BENCH_LEGS["cfg4-spec-2c"] == "spec2c"
