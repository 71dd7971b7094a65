// brc_kern_64r.hip -- lean step-kernel instantiations for NPAD = 64 with register-resident link-delay
// masks (NLR = 2: constant and slow-set delay models); own translation unit so the build compiles
// it beside brc_kern_64.hip (see brc_step.h).
#include "brc_step.h"

namespace brc {
int launch_step_64r(int dm, bool events, int mode, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P) {
    return launch_step_regmask(dm, events, mode, blocks, lds, s, P);
}
}  // namespace brc

#ifdef BRC_STAMPS
// dev-only: read and clear the section timers of the lean NPAD = 64 kernels (tools/stamps.py)
extern "C" int brc_dbg_stamps(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(brc::brc_stamps), 4 * sizeof(unsigned long long)) != hipSuccess) return -1;
    const unsigned long long z[4] = {0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(brc::brc_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
