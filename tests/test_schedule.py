"""Philox4x32-10 and the schedule draws: Python restatement vs C oracle vs Random123 KATs."""
import random

import pytest

from oracle import oracle, schedule

# Random123 kat_vectors, philox4x32_10
KAT = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
       ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
       ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
        (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]


@pytest.mark.parametrize("ctr,key,out", KAT)
def test_philox_kat_python(ctr, key, out):
    assert schedule.philox4x32_10(ctr, key) == out


@pytest.mark.parametrize("ctr,key,out", KAT)
def test_philox_kat_c(ctr, key, out):
    assert oracle.philox(ctr, key) == out


@pytest.mark.parametrize("model,dmax", [(0, 1), (1, 4), (1, 7), (2, 8), (3, 16), (3, 5)])
def test_delay_python_matches_c(model, dmax):
    rng = random.Random(model * 100 + dmax)
    lib = oracle.lib()
    for _ in range(400):
        n = rng.randint(1, 64)
        f = rng.randint(0, max(0, (n - 1) // 3))
        seed, g = rng.getrandbits(64), rng.getrandbits(40)
        sch = schedule.Schedule(n, f, seed, model, dmax, 1)
        src, dst = rng.randrange(n), rng.randrange(n)
        d = sch.delay(g, src, dst)
        assert 1 <= d <= dmax
        assert d == lib.oracle_delay(n, f, seed, model, dmax, 1, g, src, dst)
        assert sch.proposal_id(g, src) == lib.oracle_proposal_id(seed, g, src)


def test_slowset_has_f_members():
    sch = schedule.Schedule(64, 21, 0x5EED0004, schedule.DELAY_SLOWSET, 8)
    for g in range(20):
        assert sum(sch.is_slow(g, x) for x in range(64)) == 21


def test_uniform_delay_covers_range():
    sch = schedule.Schedule(16, 5, 7, schedule.DELAY_UNIFORM, 4)
    seen = {sch.delay(g, s, d) for g in range(4) for s in range(16) for d in range(16)}
    assert seen == {1, 2, 3, 4}
