"""GPU: the engine's event log, exported through the wire codec, is byte for
byte the traffic the unmodified reference put on its TCP connections (tests/golden/wire.json),
and captured Byzantine traffic replayed through ``Codec.to_injections`` reproduces the run."""
import pytest

from tests import engine_runner, golden_io
from tests.test_wire import CASES, codec_for, dst_masks

pytestmark = pytest.mark.gpu


def run_events(spec, injections):
    from byzantinerandomizedconsensus_amd import _lib as L
    from byzantinerandomizedconsensus_amd.engine import Engine
    with Engine(n=spec["n"], f=spec["f"], instances=1, protocol=spec["mode"], seed=spec["seed"],
                delay_model=spec["delay_model"], delay_max=spec["dmax"], delay_const=spec.get("dconst", 1),
                round_cap=spec.get("round_cap", 0), step_cap=spec.get("step_cap", 10000),
                key_window=8 // spec.get("nv", 1), variants=spec.get("nv", 1),
                byzantine=spec.get("byzantine", ()), event_capacity=1 << 20, instance_offset=spec["g"],
                peer_mode=L.PEER_CONNECTION if spec.get("peer_mode") == "connection" else L.PEER_SENDER) as eng:
        eng.inject(injections)
        eng.run()
        return eng.events(), eng.instances_result()[0]


@pytest.mark.parametrize("idx", range(len(CASES)), ids=[c["spec"]["name"] for c in CASES])
def test_exported_wire_equals_reference_bytes(idx):
    case = CASES[idx]
    spec = case["spec"]
    events, res = run_events(spec, engine_runner._injections(spec, 0))
    got = codec_for(spec).export(events, dst_masks=dst_masks(spec))
    assert len(got) == res["msgs_sent"] == len(case["wire"])
    assert got == case["wire"]


def test_replayed_byzantine_capture_reproduces_run():
    case = next(c for c in CASES if c["spec"]["name"].startswith("brb_byz_n7"))
    spec = case["spec"]
    byz = set(spec["byzantine"])
    codec = codec_for(spec)
    honest = [x for x in engine_runner._injections(spec, 0) if x["node"] not in byz or x["kind"] == 1]
    replay = codec.to_injections([w for w in case["wire"] if w[1] in byz])
    events, res = run_events(spec, honest + replay)
    assert codec.export(events, dst_masks=dst_masks(spec)) == case["wire"]
    for k in ("status", "t_stop", "msgs_sent", "arrivals"):
        assert res[k] == case["result"][k], k
    assert golden_io.digest(golden_io.canonical_events(
        {"deliver": [[t, nd, a, b] for (_i, t, kd, nd, _ty, a, b, _v) in events if kd == 1],
         "decide": [], "send": []})["deliver"]) == case["result"]["digest"]["deliver"]
