"""The C oracle reproduces every golden fixture generated from the unmodified reference."""
import pytest

from oracle import oracle
from tests import golden_io

GROUPS = golden_io.groups()
LARGE = ("cons_slowset_n64", "cons_slowset_n256")      # ~10 s / ~30 s oracle runs: tests of their own
CASES = [(g, i) for g, cases in GROUPS.items() for i in range(len(cases)) if g not in LARGE]


@pytest.mark.parametrize("group,idx", CASES, ids=["%s-%d" % c for c in CASES])
def test_oracle_matches_reference(group, idx):
    case = GROUPS[group][idx]
    got = oracle.run(case["spec"])
    golden_io.assert_matches(case["result"], got, "%s[%d]" % (group, idx))


@pytest.mark.slow
@pytest.mark.parametrize("group", LARGE)
def test_oracle_matches_reference_large(group):
    """n = 64 and n = 256 (SURVEY §8(d) cfg4 / cfg5 committees): reference-protocol consensus to the
    first decision under slow-set delays, generated from the unmodified reference."""
    case = GROUPS[group][0]
    got = oracle.run(case["spec"])
    golden_io.assert_matches(case["result"], got, group)


def test_fixture_inventory():
    # every SURVEY §4 known-answer scenario has a fixture
    names = {c["spec"]["name"] for c in GROUPS["kat"]}
    assert {"K1", "K2", "K3", "K4", "K5", "K6", "K7", "K10", "K11", "K12", "MIX"} <= names
    assert GROUPS["brb_fifo_n4"][0]["result"]["msgs_sent"] == 144
    assert GROUPS["brb_fifo_n4"][0]["result"]["counts"]["deliver"] == 16
