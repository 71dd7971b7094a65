// brc_kern_256.hip -- wide step-kernel instantiations for committees padded to NPAD = 256 replicas
// (one workgroup of 4 waves per instance; see brc_step_wide.h).
#include "brc_step_wide.h"

namespace brc {
int launch_step_256(int dm, bool events, int mode, bool wv4, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P) {
    return launch_step_wide<256>(dm, events, mode, wv4, blocks, lds, s, P);
}
}  // namespace brc

#ifdef BRC_STAMPS
// dev-only: the section timers of this unit's kernels (tools/stamps.py, NPAD = 256 workloads)
extern "C" int brc_dbg_stamps256(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(brc::brc_stamps), BRC_NSTAMPS * sizeof(unsigned long long)) != hipSuccess) return -1;
    const unsigned long long z[BRC_NSTAMPS] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(brc::brc_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
