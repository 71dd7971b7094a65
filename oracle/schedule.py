"""Deterministic schedule specification, pure Python (TEST INFRASTRUCTURE ONLY).

This module is part of the oracle: it is imported by ``tests/``, by the golden-vector
harness (``tests/golden/make_golden.py``) and by nothing in the product path.  The HIP
engine computes the same functions on the device (``csrc/schedule.h``) and the C oracle
restates them in ``oracle/brc_oracle.c``; ``tests/test_schedule.py`` pins all three to
the Random123 Philox4x32-10 known-answer vectors and to each other.

The reference has no schedule at all: its transport is one TCP connection per message
(``byzantinerandomizedconsensus/base/broadcast.py:26-40``) and delivery order is whatever
the OS does.  The simulator replaces that transport with a lock-step network:

* time is an integer step; a message sent while step ``t`` is processed (or by an
  injection action stamped ``t``) reaches ``dst`` at ``t + delay(g, src, dst)``, with
  ``1 <= delay <= D``;
* a receiver processes the messages of one step in the canonical order
  ``(kp, s, type, sender)`` (key slot, phase index, SEND<ECHO<READY, sender id);
* the network is duplicate-suppressing: a message identical to one already sent on the
  same link ``(src, dst, type, payload)`` is dropped.

All random quantities are counter-based Philox4x32-10 draws keyed by the run seed, so
every instance is reproducible from ``(seed, global instance id)`` alone.
"""

M0 = 0xD2511F53
M1 = 0xCD9E8D57
W0 = 0x9E3779B9
W1 = 0xBB67AE85
MASK32 = 0xFFFFFFFF

PURPOSE_DELAY = 1
PURPOSE_PROPOSAL = 2
PURPOSE_SLOWSET = 3
PURPOSE_COIN = 4

DELAY_CONST = 0
DELAY_UNIFORM = 1
DELAY_SLOWSET = 2
DELAY_GEOMETRIC = 3


def philox4x32_10(ctr, key):
    """Philox4x32 with 10 rounds (Salmon et al., SC'11; Random123 reference)."""
    c0, c1, c2, c3 = (x & MASK32 for x in ctr)
    k0, k1 = (x & MASK32 for x in key)
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> 32, p0 & MASK32
        hi1, lo1 = p1 >> 32, p1 & MASK32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & MASK32, lo1, (hi0 ^ c3 ^ k1) & MASK32, lo0
        k0 = (k0 + W0) & MASK32
        k1 = (k1 + W1) & MASK32
    return (c0, c1, c2, c3)


def _draw(seed, g, a, purpose, b):
    return philox4x32_10((g & MASK32, (g >> 32) & MASK32, a & MASK32,
                          ((purpose & 0xFF) << 24) | (b & 0xFFFFFF)),
                         (seed & MASK32, (seed >> 32) & MASK32))


class Schedule:
    """Delay/proposal model of one run.  ``g`` is the GLOBAL instance id."""

    def __init__(self, n, f, seed, model=DELAY_CONST, dmax=1, dconst=1):
        assert 1 <= dmax <= 16, "delay_max must be in [1, 16]"
        assert 1 <= dconst <= dmax or model != DELAY_CONST
        self.n, self.f, self.seed = n, f, seed
        self.model, self.dmax, self.dconst = model, dmax, dconst
        self._slow_cache = {}

    def slow_offset(self, g):
        return _draw(self.seed, g, 0, PURPOSE_SLOWSET, 0)[0] % self.n

    def is_slow(self, g, x):
        off = self._slow_cache.get(g)
        if off is None:
            off = self._slow_cache[g] = self.slow_offset(g)
        return ((x - off) % self.n) < self.f

    def delay(self, g, src, dst):
        m = self.model
        if m == DELAY_CONST:
            return self.dconst
        if m == DELAY_SLOWSET:
            return self.dmax if (self.is_slow(g, src) or self.is_slow(g, dst)) else 1
        w = _draw(self.seed, g, dst, PURPOSE_DELAY, src >> 2)[src & 3]
        if m == DELAY_UNIFORM:
            return 1 + ((w * self.dmax) >> 32)
        if m == DELAY_GEOMETRIC:
            ones = 0
            while ones < 32 and (w >> ones) & 1:
                ones += 1
            return min(1 + ones, self.dmax)
        raise ValueError("unknown delay model %r" % m)

    def proposal_id(self, g, i):
        """Value id of replica i's Bernoulli(1/2) proposal: 1 -> "0", 2 -> "1"."""
        return 1 + (_draw(self.seed, g, i, PURPOSE_PROPOSAL, 0)[0] & 1)

    def coin(self, g, rnd):
        return _draw(self.seed, g, rnd, PURPOSE_COIN, 0)[0] & 1
