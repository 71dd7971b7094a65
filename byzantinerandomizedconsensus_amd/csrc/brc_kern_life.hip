// brc_kern_life.hip -- instantiations of the key-lifetime kernel (brc_life.h), one per protocol mode (and connection peers)
// and delay family (two-class / per-link);
// own translation unit so the build compiles it beside the step kernels.
#include "brc_life.h"

namespace brc {
template <bool PL>
static int launch_life_pl(int mode, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P) {
    if (mode == BRC_MODE_SPEC) return launch_life_one<BRC_MODE_SPEC, PL>(blocks, lds, s, P);
    if (mode == BRC_MODE_BEB) return launch_life_one<BRC_MODE_BEB, PL>(blocks, lds, s, P);
    if (mode == BRC_MODE_REFERENCE) return launch_life_one<BRC_MODE_REFERENCE, PL>(blocks, lds, s, P);
    if (mode == KMODE_CONN) return launch_life_one<KMODE_CONN, PL>(blocks, lds, s, P);
    return BRC_E_INVALID;
}
// perlink: uniform / geometric delays (per-receiver delay masks, HBM delivery bitmaps)
int launch_life(int mode, bool perlink, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P) {
    return perlink ? launch_life_pl<true>(mode, blocks, lds, s, P) : launch_life_pl<false>(mode, blocks, lds, s, P);
}
}  // namespace brc
