// brc_kern_32.hip -- step-kernel instantiations for replica sets padded to NPAD = 32 lanes
// (one translation unit per width so the build compiles them in parallel; see brc_step.h).
#include "brc_step.h"

namespace brc {
int launch_step_32(int dm, bool events, int mode, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P) {
    return launch_step<32>(dm, events, mode, blocks, lds, s, P);
}
}  // namespace brc
