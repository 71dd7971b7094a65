// schedule.h -- counter-based schedule draws (Philox4x32-10), host + device.
//
// The reference has no schedule: its transport is one TCP connection per message
// (base/broadcast.py:26-40) and ordering is whatever the OS does.  The engine replaces it with
// a lock-step network whose every random quantity is a Philox4x32-10 draw keyed by the run
// seed and counted by (global instance id, purpose, a, b).  oracle/schedule.py and
// oracle/brc_oracle.c restate these functions; tests/test_schedule.py pins all three to the
// Random123 known-answer vectors.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace brc {

enum : uint32_t { PURPOSE_DELAY = 1, PURPOSE_PROPOSAL = 2, PURPOSE_SLOWSET = 3, PURPOSE_COIN = 4 };

struct u32x4 { uint32_t x, y, z, w; };

__host__ __device__ inline u32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                               uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0; c1 = lo1; c2 = hi0 ^ c3 ^ k1; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return {c0, c1, c2, c3};
}

// counter (g_lo, g_hi, a, purpose << 24 | b), key (seed_lo, seed_hi)
__host__ __device__ inline u32x4 draw(uint64_t seed, uint64_t g, uint32_t a, uint32_t purpose, uint32_t b) {
    return philox4x32_10((uint32_t)g, (uint32_t)(g >> 32), a, (purpose << 24) | (b & 0xFFFFFFu),
                         (uint32_t)seed, (uint32_t)(seed >> 32));
}

__host__ __device__ inline uint32_t uniform_delay(uint32_t w, uint32_t dmax) {
    return 1u + (uint32_t)(((uint64_t)w * dmax) >> 32);
}

__host__ __device__ inline uint32_t geometric_delay(uint32_t w, uint32_t dmax) {
    // 1 + number of trailing one bits, capped at dmax: P(delay = k) = 2^-k below the cap
    const uint32_t ones = (w == 0xFFFFFFFFu) ? 32u : (uint32_t)__builtin_ctz(~w);
    return (1u + ones < dmax) ? 1u + ones : dmax;
}

__host__ __device__ inline uint32_t slow_offset(uint64_t seed, uint64_t g, uint32_t n) {
    return draw(seed, g, 0, PURPOSE_SLOWSET, 0).x % n;
}

__host__ __device__ inline uint32_t proposal_id(uint64_t seed, uint64_t g, uint32_t i) {
    return 1u + (draw(seed, g, i, PURPOSE_PROPOSAL, 0).x & 1u);
}

// BRC_MODE_SPEC common coin of (instance, round): value id 1 ("0") or 2 ("1")
__host__ __device__ inline uint32_t coin_id(uint64_t coin_seed, uint64_t g, uint32_t round) {
    return 1u + (draw(coin_seed, g, round, PURPOSE_COIN, 0).x & 1u);
}

}  // namespace brc
