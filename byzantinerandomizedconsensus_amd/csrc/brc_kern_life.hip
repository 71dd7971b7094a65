// brc_kern_life.hip -- instantiations of the key-lifetime kernel (brc_life.h), one per protocol mode (and connection peers)
// and delay family (two-class / per-link);
// own translation unit so the build compiles it beside the step kernels.
#include "brc_life.h"

namespace brc {
template <bool PL, int DLX>
static int launch_life_pl(int mode, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P) {
    if (mode == BRC_MODE_SPEC) return launch_life_one<BRC_MODE_SPEC, PL, DLX>(blocks, lds, s, P);
    if (mode == BRC_MODE_BEB) return launch_life_one<BRC_MODE_BEB, PL, DLX>(blocks, lds, s, P);
    if (mode == BRC_MODE_REFERENCE) return launch_life_one<BRC_MODE_REFERENCE, PL, DLX>(blocks, lds, s, P);
    if (mode == KMODE_CONN) return launch_life_one<KMODE_CONN, PL, DLX>(blocks, lds, s, P);
    return BRC_E_INVALID;
}
// perlink: uniform / geometric delays (per-receiver delay masks, HBM delivery bitmaps); dm16: delays up
// to 16 (the per-link form's 64-row ring); qbig: key windows of 64 / 128 (two-class form, not SPEC)
int launch_life(int mode, bool perlink, bool dm16, bool qbig, bool hm, uint32_t blocks, uint32_t lds, hipStream_t s,
                const Params* P) {
    if (hm && !qbig) {
        // key window 32, two-class form: the slot metadata in HBM (brc_internal.h life_hbm_meta)
        if (perlink || mode == BRC_MODE_SPEC) return BRC_E_INVALID;
        if (mode == BRC_MODE_BEB) return launch_life_one<BRC_MODE_BEB, false, 8, false, true>(blocks, lds, s, P);
        if (mode == BRC_MODE_REFERENCE) return launch_life_one<BRC_MODE_REFERENCE, false, 8, false, true>(blocks, lds, s, P);
        if (mode == KMODE_CONN) return launch_life_one<KMODE_CONN, false, 8, false, true>(blocks, lds, s, P);
        return BRC_E_INVALID;
    }
    if (qbig) {
        if (!hm) return BRC_E_INVALID;
        if (perlink || mode == BRC_MODE_SPEC) return BRC_E_INVALID;
        if (mode == BRC_MODE_BEB) return launch_life_one<BRC_MODE_BEB, false, 8, true>(blocks, lds, s, P);
        if (mode == BRC_MODE_REFERENCE) return launch_life_one<BRC_MODE_REFERENCE, false, 8, true>(blocks, lds, s, P);
        if (mode == KMODE_CONN) return launch_life_one<KMODE_CONN, false, 8, true>(blocks, lds, s, P);
        return BRC_E_INVALID;
    }
    if (perlink && dm16) return launch_life_pl<true, 16>(mode, blocks, lds, s, P);
    return perlink ? launch_life_pl<true, 8>(mode, blocks, lds, s, P) : launch_life_pl<false, 8>(mode, blocks, lds, s, P);
}
}  // namespace brc

#ifdef BRC_STAMPS
// dev-only: the lifetime kernel's section timers (tools/stamps.py)
extern "C" int brc_dbg_stamps_life(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(brc::brc_stamps), BRC_NSTAMPS * sizeof(unsigned long long)) != hipSuccess) return -1;
    unsigned long long z[BRC_NSTAMPS] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(brc::brc_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
