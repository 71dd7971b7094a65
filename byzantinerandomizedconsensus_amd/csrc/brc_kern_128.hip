// brc_kern_128.hip -- wide step-kernel instantiations for committees padded to NPAD = 128 replicas
// (one workgroup of 2 waves per instance; see brc_step_wide.h).
#include "brc_step_wide.h"

namespace brc {
int launch_step_128(int dm, bool events, int mode, bool wv4, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P) {
    return launch_step_wide<128>(dm, events, mode, wv4, blocks, lds, s, P);
}
}  // namespace brc
