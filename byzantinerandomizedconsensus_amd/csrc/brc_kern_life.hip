// brc_kern_life.hip -- instantiations of the key-lifetime kernel (brc_life.h), one per protocol mode (and connection peers);
// own translation unit so the build compiles it beside the step kernels.
#include "brc_life.h"

namespace brc {
int launch_life(int mode, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P) {
    if (mode == BRC_MODE_SPEC) return launch_life_one<BRC_MODE_SPEC>(blocks, lds, s, P);
    if (mode == BRC_MODE_BEB) return launch_life_one<BRC_MODE_BEB>(blocks, lds, s, P);
    if (mode == BRC_MODE_REFERENCE) return launch_life_one<BRC_MODE_REFERENCE>(blocks, lds, s, P);
    if (mode == KMODE_CONN) return launch_life_one<KMODE_CONN>(blocks, lds, s, P);
    return BRC_E_INVALID;
}
}  // namespace brc
