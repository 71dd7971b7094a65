"""Host check of the lean kernels' packed key-pair cell update (brc_step.h, BRC_PK): the v_pk_*_u16
formulas, restated here on uint32 words with 16-bit lane arithmetic, equal the per-key integer form
(brb_cell_update / brb_cell_update_spec as brc_step.h writes them) on every field of the new cell word
and on the ECHO / READY / DELIVER outputs, over random cell states, arrival counts and thresholds.
The GPU parity suite checks the kernel itself; this pins the algebra (no cross-half carries or shifts).
"""
import numpy as np


def test_packed_pair_update_matches_per_key_form():
    rng = np.random.default_rng(1)
    N = 400_000
    M32 = np.uint64(0xFFFFFFFF)
    def u(x): return np.asarray(x, dtype=np.uint64) & M32
    def half_op(a, b, f):
        lo = f(a & 0xFFFF, b & 0xFFFF) & 0xFFFF
        hi = f(a >> 16, b >> 16) & 0xFFFF
        return u(lo | (hi << 16))
    pk_add = lambda a, b: half_op(a, b, lambda x, y: x + y)
    pk_sub = lambda a, b: half_op(a, b, lambda x, y: (x - y) & 0xFFFF)
    pk_min = lambda a, b: half_op(a, b, np.minimum)
    pk_max = lambda a, b: half_op(a, b, np.maximum)
    pk_ge = lambda a, b: (u(~pk_sub(a, b)) >> 15) & 0x10001
    pk2 = lambda x: u(x | (x << 16))
    nz = lambda x: (u(x + 0x007F007F) >> 7) & 0x10001
    T_echo, T_amp, T_del = 43, 22, 43
    for SPEC in (False, True):
      for (Te, Ta, Td) in ((43, 22, 43), (33, 17, 33), (3, 2, 3)):
        fl = rng.integers(0, 32, (2, N)).astype(np.uint64); ec = rng.integers(0, 64, (2, N)).astype(np.uint64)
        rc = rng.integers(0, 64, (2, N)).astype(np.uint64)
        ea = rng.integers(0, 65, (2, N)).astype(np.uint64); ra = rng.integers(0, 65, (2, N)).astype(np.uint64)
        sa = rng.integers(0, 2, (2, N)).astype(np.uint64); opn = rng.integers(0, 2, (2, N)).astype(bool)
        ea[:, rng.random(N) < .3] = 0; ra[:, rng.random(N) < .3] = 0
        # scalar reference (brc_step.h per-key code)
        ge = lambda a, b: ((u(a - b) >> 31) ^ 1)
        F, EC_, RC_ = fl.copy(), ec.copy(), rc.copy(); es = np.zeros_like(F); rs = np.zeros_like(F); dl = np.zeros_like(F)
        if SPEC:
            es = np.where(opn, sa, 0) & u(~(F >> 3)) & 1; F |= es << 3
            EC_ = EC_ + np.where(opn, ea, 0); RC_ = RC_ + np.where(opn, ra, 0)
            rs = opn.astype(np.uint64) & u(~(F >> 4)) & (ge(EC_, Te) | ge(RC_, Ta)); F |= rs << 4
            dl = opn.astype(np.uint64) & ge(RC_, Td); F |= dl << 2
        else:
            est = np.where(opn, sa, 0) & u(~F) & 1; es = est & u(~(F >> 3)); F |= est | (est << 3)
            e = np.where(opn, ea, 0); eon = np.minimum(e, 1); chk = np.minimum(e + (F & 1) - eon, 1); F |= eon; EC_ = EC_ + e
            r1 = eon & chk & ge(EC_, Te) & (u(~F) >> 1) & 1; rs = r1 & u(~(F >> 4)); F |= (r1 << 1) | (r1 << 4)
            r = np.where(opn, ra, 0); ron = np.minimum(r, 1); rexm = u(0 - ((F >> 1) & 1))
            rlo = u(2 + (u(RC_ - 1) & rexm)); rhi = u(r + (RC_ & rexm)); F |= ron << 1; RC_ = RC_ + r
            any_ = ron & ge(rhi, rlo); alo = np.maximum(rlo, Ta); ahi = np.minimum(rhi, Td - 1)
            r2 = any_ & u(~F) & u(~(F >> 4)) & ge(ahi, alo) & 1; F |= r2 << 4; dl = any_ & ge(rhi, Td); F |= dl << 2; rs |= r2
        # packed
        lo = fl | (ec << 5) | (rc << 11)
        P0 = u((lo[0] & 0xFFFF) | (lo[1] << 16)); P1 = u(((lo[0] >> 8) & 0xFFFF) | ((lo[1] >> 8) << 16))
        FL = P0 & 0x001F001F; EC = (P0 >> 5) & 0x003F003F; RC = (P1 >> 3) & 0x003F003F
        ONM = u(np.where(opn[0], 0xFFFF, 0) | np.where(opn[1], 0xFFFF0000, 0)); ON = ONM & 0x10001
        SA = u(sa[0] | (sa[1] << 16)) & ONM; E = u(ea[0] | (ea[1] << 16)) & ONM; R = u(ra[0] | (ra[1] << 16)) & ONM
        ES = RS = DL = u(0)
        if SPEC:
            ES = SA & u(~(FL >> 3)) & 0x10001; FL |= ES << 3
            EC = pk_add(EC, E); RC = pk_add(RC, R)
            RS = ON & u(~(FL >> 4)) & (pk_ge(EC, pk2(Te)) | pk_ge(RC, pk2(Ta))); FL |= RS << 4
            DL = ON & pk_ge(RC, pk2(Td)); FL |= DL << 2
        else:
            est = SA & u(~FL) & 0x10001; ES = est & u(~(FL >> 3)); FL |= est | (est << 3)
            eon = nz(E); chk = nz(u(E + (FL & 0x10001) - eon)); FL |= eon; EC = pk_add(EC, E)
            r1 = eon & chk & pk_ge(EC, pk2(Te)) & (u(~FL) >> 1) & 0x10001; RS = r1 & u(~(FL >> 4)); FL |= u((r1 << 1) | (r1 << 4))
            ron = nz(R); rexm = pk_sub(u(0), (FL >> 1) & 0x10001)
            rlo = pk_add(pk_sub(RC, 0x10001) & rexm, 0x20002); rhi = pk_add(R, RC & rexm); FL |= u(ron << 1); RC = pk_add(RC, R)
            any_ = ron & pk_ge(rhi, rlo); alo = pk_max(rlo, pk2(Ta)); ahi = pk_min(rhi, pk2(Td - 1))
            r2 = any_ & u(~FL) & u(~(FL >> 4)) & pk_ge(ahi, alo) & 0x10001; FL |= u(r2 << 4); DL = any_ & pk_ge(rhi, pk2(Td)); FL |= u(DL << 2); RS |= r2
        PL = u(FL | (pk_min(EC, 0x003F003F) << 5)); PR = pk_min(RC, 0x003F003F)
        for i in range(2):
            got = ((PL >> (16 * i)) & 0xFFFF) | (((PR >> (16 * i)) & 0xFFFF) << 11)
            want = F[i] | (np.minimum(EC_[i], 63) << 5) | (np.minimum(RC_[i], 63) << 11)
            w = opn[i]
            assert np.array_equal(got[w], want[w]), (SPEC, i, np.argmax(got[w] != want[w]))
            for nm, P, S in (("es", ES, es), ("rs", RS, rs), ("dl", DL, dl)):
                g = (P >> (16 * i)) & 1
                assert np.array_equal(g[w], S[i][w]), (nm, SPEC, i)
        pass
