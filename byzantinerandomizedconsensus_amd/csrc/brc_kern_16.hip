// brc_kern_16.hip -- step-kernel instantiations for replica sets padded to NPAD = 16 lanes
// (one translation unit per width so the build compiles them in parallel; see brc_step.h).
#include "brc_step.h"

namespace brc {
int launch_step_16(int dm, bool events, int mode, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P) {
    return launch_step<16>(dm, events, mode, blocks, lds, s, P);
}
}  // namespace brc

#ifdef BRC_STAMPS
// dev-only: the section timers of this unit's kernels (tools/stamps.py, NPAD = 16 workloads)
extern "C" int brc_dbg_stamps16(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(brc::brc_stamps), BRC_NSTAMPS * sizeof(unsigned long long)) != hipSuccess) return -1;
    const unsigned long long z[BRC_NSTAMPS] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(brc::brc_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
