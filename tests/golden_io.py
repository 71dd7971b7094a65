"""Loading and comparing the golden fixtures (tests/golden/*.json)."""
import glob
import hashlib
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def groups():
    out = {}
    for path in sorted(glob.glob(os.path.join(GOLDEN, "*.json"))):
        with open(path) as fh:
            data = json.load(fh)
        if data["group"].startswith("oracle_"):      # oracle-made expectations, not reference fixtures
            continue
        out[data["group"]] = data["cases"]
    return out


_CELL_STEPS = None


def cell_steps(group, idx):
    """The oracle's cell-step count of fixture case (group, idx) (tests/golden/make_cell_steps.py)."""
    global _CELL_STEPS
    if _CELL_STEPS is None:
        with open(os.path.join(GOLDEN, "oracle_cell_steps.json")) as fh:
            _CELL_STEPS = json.load(fh)["cases"]
    return _CELL_STEPS[group][idx]


def digest(rows):
    return hashlib.sha256(json.dumps(rows, separators=(",", ":")).encode()).hexdigest()


def canonical_events(ev):
    key = lambda r: [str(x) if isinstance(x, str) else x for x in r]  # noqa: E731
    return {k: sorted(map(list, ev[k]), key=key) for k in ("deliver", "decide", "send")}


def assert_matches(expected, got, label=""):
    """expected: fixture 'result' (compact form); got: result with canonical event lists."""
    for k in ("status", "t_stop", "msgs_sent", "arrivals"):
        assert got[k] == expected[k], "%s: %s differs: got %r expected %r" % (label, k, got[k], expected[k])
    ev = canonical_events(got["events"])
    for k in ("deliver", "decide", "send"):
        assert len(ev[k]) == expected["counts"][k], "%s: %d %s events, expected %d" % (
            label, len(ev[k]), k, expected["counts"][k])
        if k in expected["events"]:
            assert ev[k] == expected["events"][k], "%s: %s events differ" % (label, k)
        assert digest(ev[k]) == expected["digest"][k], "%s: %s digest differs" % (label, k)
