"""Wire format against bytes captured from the unmodified reference
(tests/golden/wire.json, written by ``make_golden.py --wire``): the codec reproduces every
envelope byte for byte, and captured Byzantine traffic turns back into the injections that
produced it.  The engine-side export is checked on the GPU (test_gpu_wire)."""
import json
import os

import pytest

from byzantinerandomizedconsensus_amd import wire
from tests import engine_runner

HERE = os.path.dirname(os.path.abspath(__file__))


def load_cases():
    with open(os.path.join(HERE, "golden", "wire.json")) as fh:
        return json.load(fh)["cases"]


CASES = load_cases()


def codec_for(spec):
    payloads = {(a["kp"], a["s"]): a["payload"] for a in spec["actions"] if "payload" in a}
    return wire.Codec(spec["n"], mode=spec["mode"], nv=spec.get("nv", 1), values=spec["values"],
                      payloads=payloads, peer_mode=spec.get("peer_mode", "sender"))


def dst_masks(spec):
    """Destinations of the spec's restricted (Byzantine) SENDs, keyed like export() wants."""
    out = {}
    for a in spec["actions"]:
        if a["kind"] == "byz" and a["type"] == wire.SEND:
            out[(a["t"], a["src"], wire.SEND, a["kp"], a["s"])] = a["dst"]
    return out


@pytest.mark.parametrize("idx", range(len(CASES)), ids=[c["spec"]["name"] for c in CASES])
def test_envelopes_round_trip_byte_exact(idx):
    case = CASES[idx]
    codec = codec_for(case["spec"])
    for t, src, dst, env in case["wire"]:
        m = codec.decode(src, env)
        assert wire.envelope(codec.addrs[src][0], m["type"], codec.payload(m["kp"], m["s"], m["value"])) == env


def test_message_count_matches_reference():
    for case in CASES:
        assert len(case["wire"]) == case["result"]["msgs_sent"], case["spec"]["name"]


def test_byzantine_traffic_becomes_its_injections():
    case = next(c for c in CASES if c["spec"]["name"].startswith("brb_byz_n7"))
    spec = case["spec"]
    byz = set(spec["byzantine"])
    codec = codec_for(spec)
    got = codec.to_injections([w for w in case["wire"] if w[1] in byz])
    want = [x for x in engine_runner._injections(spec, 0) if x["kind"] != 1 and x["node"] in byz]
    norm = lambda xs: sorted(tuple(sorted((k, v) for k, v in x.items() if k != "value")) for x in xs)  # noqa: E731
    # declared keys carry no payload value in a BRB run; everything else must agree
    assert norm(got) == norm(want)


def test_connection_export_counts_every_broadcast():
    # connection-identity peers (core/brbroadcast.py:69): a READY re-fire (:119) is logged as a COPY
    # event and exported as one more envelope per peer; sender peers never carry copies
    c = wire.Codec(4, peer_mode="connection")
    evs = [(0, 1, wire.EV_SEND, 2, wire.READY, 0, 0, 1), (0, 2, wire.EV_COPY, 2, wire.READY, 0, 0, 1),
           (0, 2, wire.EV_COPY, 2, wire.READY, 0, 0, 1)]
    assert len(c.export(evs)) == 12
    assert len(wire.Codec(4).export(evs)) == 4
    with pytest.raises(ValueError):
        wire.Codec(4, peer_mode="tcp")


def test_connection_cases_carry_refires():
    # the connection-identity fixtures hold more envelopes than first broadcasts x peers: re-fires
    conn = [c for c in CASES if c["spec"].get("peer_mode") == "connection"]
    assert len(conn) >= 4
    firsts = {c["spec"]["name"]: c["result"]["counts"]["send"] * c["spec"]["n"] for c in conn}
    assert any(len(c["wire"]) > firsts[c["spec"]["name"]] for c in conn)
