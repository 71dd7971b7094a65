// brc_kern_64r.hip -- lean step-kernel instantiations for NPAD = 64 with register-resident link-delay
// masks (NLR = 2: constant and slow-set delay models); own translation unit so the build compiles
// it beside brc_kern_64.hip (see brc_step.h).
#include "brc_step.h"

namespace brc {
// Lean kernels with register-resident delay masks (NLR = 2): NPAD = 64, sender peers, at most two
// distinct link delays (constant or slow-set models).
static int launch_step_regmask(int dm, bool events, int mode, uint32_t blocks, uint32_t lds, hipStream_t s,
                               const Params* P) {
    if (mode == KMODE_CONN) return BRC_E_INVALID;
#define BRC_CASE(DMX)                                                                                  \
    if (dm == DMX) {                                                                                   \
        if (mode == BRC_MODE_SPEC) return events ? launch_one<64, DMX, true, BRC_MODE_SPEC, 2>(blocks, lds, s, P) : launch_one<64, DMX, false, BRC_MODE_SPEC, 2>(blocks, lds, s, P); \
        if (mode == BRC_MODE_BEB) return events ? launch_one<64, DMX, true, BRC_MODE_BEB, 2>(blocks, lds, s, P) : launch_one<64, DMX, false, BRC_MODE_BEB, 2>(blocks, lds, s, P); \
        return events ? launch_one<64, DMX, true, BRC_MODE_REFERENCE, 2>(blocks, lds, s, P) : launch_one<64, DMX, false, BRC_MODE_REFERENCE, 2>(blocks, lds, s, P); \
    }
#ifdef BRC_ONLY_DM8
    BRC_CASE(8)
#else
    BRC_CASE(4) BRC_CASE(8) BRC_CASE(16)
#endif
#undef BRC_CASE
    return BRC_E_INVALID;
}


int launch_step_64r(int dm, bool events, int mode, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P) {
    return launch_step_regmask(dm, events, mode, blocks, lds, s, P);
}
}  // namespace brc

#ifdef BRC_STAMPS
// dev-only: read and clear the section timers of the lean NPAD = 64 kernels (tools/stamps.py)
extern "C" int brc_dbg_stamps(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(brc::brc_stamps), BRC_NSTAMPS * sizeof(unsigned long long)) != hipSuccess) return -1;
    const unsigned long long z[BRC_NSTAMPS] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(brc::brc_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
