// brc_step.h -- the MI355X (gfx950) step kernel: batched Bracha broadcast + randomized consensus.
//
// One 64-lane wavefront simulates an "item": IPW = 64 / NPAD independent instances, lane =
// (instance segment, replica).  Lane d is at once receiver d (its BRB cells), sender d (its
// send steps are read back by every receiver through __ballot) and consensus replica d.  A
// wave runs its item from the current step to completion in ONE launch: instances are
// independent, so no inter-wave communication exists at all.  Workgroups hold WPB such waves
// that never synchronise with each other (LDS is partitioned per wave).
//
// Hot path replaced (reference = sithu/ByzantineRandomizedConsensus):
//   brb_cell_update()  <- core/brbroadcast.py:60-119  (per-message handler, batched per step)
//   consensus pass     <- core/byzantinerandomizedconsensus.py:53-106 (deliver / get_max_val)
//   send_key()         <- core/byzantinerandomizedconsensus.py:43-51, base/broadcast.py:17-40
//
// Cell = (receiver, key).  The network suppresses duplicates (oracle/schedule.py), so every
// ECHO/READY that reaches a cell comes from a new sender: the reference's sets
// (core/brbroadcast.py:38-41) only ever matter through their sizes, and a cell is one word:
//   bits  0- 4 flags  (entry in echo_sent_list, entry in ready_sent_list, delivered,
//                      ECHO sent, READY sent)
//   bits  5-11 |echo set|      bits 12-18 |ready set|     bits 19-31 allocation generation
//   bits 32-47 step this lane SENT its ECHO of the key     bits 48-63 ... its READY (0xFFFF: never)
// A cell whose generation differs from its key slot's is stale in every field, send steps
// included, so recycling a slot (or a whole batch, brc_reset) never touches the cells.
// HBM (lane-contiguous => every access is one coalesced 512-B wave access):
//   cells [item][NK + 1][64] u64 -- row NK is a trash row: the key loop runs whole chunks, and the
//   padding slots of the last chunk load and store it, so no load or store is conditional and the
//   compiler can wait for exactly the loads a chunk needs while the next chunk's are in flight
// per instance key slots (copied to LDS for the launch): meta [inst][NK] u64 (s+1 | t_send |
//   t_quiet | sender | value), mgen [inst][NK] u32 (generation | restricted-SEND flag),
//   kdst [inst][NK] u64 (SEND destinations, read only for restricted SENDs)
// per item: act [item][32][nkw] u64 (key slots that may have arrivals at step t mod 32)
// per lane: cons0/cons1 [item][64] u64, hmask [item][4][64] T (consensus state)
#pragma once
#include "brc_internal.h"
#include "schedule.h"

namespace brc {

constexpr uint32_t NOKEY = 0xFFFFFFFFu;
// lean key-list entries (u32): key slot (< 2^12) | the message types that can land on it this step << TB_SH
// | for a SEND landing now: its sender << KL_SND_SH, its link delay - 1 << KL_DT_SH, KL_RESTR for a
// restricted SEND -- everything the key loop needs from the slot's metadata
constexpr uint32_t TB_S = 1, TB_E = 2, TB_R = 4, TB_SH = 12, TB_KEY = (1u << TB_SH) - 1u;
constexpr uint32_t KL_SND_SH = 15, KL_DT_SH = 21, KL_RESTR = 1u << 25;

template <int NPAD> struct MaskOf { using type = uint64_t; };
template <> struct MaskOf<4> { using type = uint8_t; };
template <> struct MaskOf<8> { using type = uint8_t; };
template <> struct MaskOf<16> { using type = uint16_t; };
template <> struct MaskOf<32> { using type = uint32_t; };

template <typename T> __device__ __forceinline__ uint32_t popc(T x) { return (uint32_t)__popcll((uint64_t)x); }


// Whole-wave reductions (NPAD = 64) through DPP row operations and four lane reads: each 16-lane
// row reduces with quad_perm xor 1 and xor 2, row_half_mirror and row_mirror, and the four row
// results combine in scalar registers -- no LDS round trip and no shuffle-address registers.  Every
// lane must be active (the step loop's reductions run in wave-uniform control flow); otherwise the
// shuffle form below is used.
__device__ __forceinline__ uint32_t dpp_row_or(uint32_t x) {
    x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);    // quad_perm [1,0,3,2]
    x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true);    // quad_perm [2,3,0,1]
    x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, true);   // row_half_mirror
    x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, true);   // row_mirror
    return x;
}
__device__ __forceinline__ uint32_t dpp_row_max(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true));
    x = max(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true));
    x = max(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, true));
    x = max(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, true));
    return x;
}
__device__ __forceinline__ bool full_exec() { return __builtin_amdgcn_read_exec() == ~0ull; }
__device__ __forceinline__ uint32_t rl(uint32_t x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }

// OR / max over every lane, called with every lane active (wave-uniform control flow)
__device__ __forceinline__ uint32_t wave_or_all(uint32_t x) {
    const uint32_t r = dpp_row_or(x);
    return rl(r, 0) | rl(r, 16) | rl(r, 32) | rl(r, 48);
}
__device__ __forceinline__ uint32_t wave_max_all(uint32_t x) {
    const uint32_t r = dpp_row_max(x);
    return max(max(rl(r, 0), rl(r, 16)), max(rl(r, 32), rl(r, 48)));
}
// OR of every lane's x (the same value in every lane)
__device__ __forceinline__ uint32_t wave_or(uint32_t x) {
    if (full_exec()) {
        const uint32_t r = dpp_row_or(x);
        return rl(r, 0) | rl(r, 16) | rl(r, 32) | rl(r, 48);
    }
#pragma unroll
    for (int o = 32; o; o >>= 1) x |= (uint32_t)__shfl_xor((int)x, o);
    return x;
}

template <int NPAD> __device__ __forceinline__ uint32_t seg_max(uint32_t x) {
    if constexpr (NPAD == 64) {
        if (full_exec()) {
            const uint32_t r = dpp_row_max(x);
            return max(max(rl(r, 0), rl(r, 16)), max(rl(r, 32), rl(r, 48)));
        }
    }
#pragma unroll
    for (int o = NPAD / 2; o; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o));
    return x;
}

template <int NPAD, typename T> __device__ __forceinline__ T seg_or(T x) {
#pragma unroll
    for (int o = NPAD / 2; o; o >>= 1) x |= (T)__shfl_xor((unsigned long long)x, o);
    return x;
}

__device__ __forceinline__ uint32_t hibit(uint32_t x) { return x ? 32u - (uint32_t)__clz(x) : 0u; }

// Slot groups of G in {2, 4, 8, 16, 32} consecutive bits of a 64-bit key word: fold_groups leaves bit
// G*i set iff group i has a set bit; compress_groups packs those bits (multiples of G) to bits 0 .. 64/G - 1.
__device__ __forceinline__ uint64_t fold_groups(uint64_t x, uint32_t G) {
    if (G == 2) return (x | (x >> 1)) & 0x5555555555555555ull;
    if (G == 4) return (x | (x >> 1) | (x >> 2) | (x >> 3)) & 0x1111111111111111ull;
    x |= x >> 1; x |= x >> 2; x |= x >> 4;
    if (G == 8) return x & 0x0101010101010101ull;
    x |= x >> 8;
    if (G == 16) return x & 0x0001000100010001ull;
    x |= x >> 16;
    return x & 0x0000000100000001ull;
}
__device__ __forceinline__ uint64_t compress_groups(uint64_t x, uint32_t G) {
    if (G == 2) {
        x = (x | (x >> 1)) & 0x3333333333333333ull; x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
        x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull; x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
        return (x | (x >> 16)) & 0xFFFFFFFFull;
    }
    if (G == 4) {
        x = (x | (x >> 3)) & 0x0303030303030303ull; x = (x | (x >> 6)) & 0x000F000F000F000Full;
        x = (x | (x >> 12)) & 0x000000FF000000FFull;
        return (x | (x >> 24)) & 0xFFFFull;
    }
    if (G == 8) {
        x = (x | (x >> 7)) & 0x0003000300030003ull; x = (x | (x >> 14)) & 0x0000000F0000000Full;
        return (x | (x >> 28)) & 0xFFull;
    }
    if (G == 16) {
        x = (x | (x >> 15)) & 0x0000000300000003ull;
        return (x | (x >> 30)) & 0xFull;
    }
    return (x | (x >> 31)) & 0x3ull;
}

// compile-time unrolled loop: f(IC<0>{}), ..., f(IC<N-1>{}) (register arrays stay statically indexed)
template <int I> struct IC { static constexpr int value = I; };
template <int N> struct Unrolled {
    template <typename F> __device__ __forceinline__ static void run(F&& f) {
        Unrolled<N - 1>::run(f);
        f(IC<N - 1>{});
    }
};
template <> struct Unrolled<0> {
    template <typename F> __device__ __forceinline__ static void run(F&&) {}
};

// wave-uniform value -> scalar registers (valid only when every lane holds the same value)
__device__ __forceinline__ uint32_t uni32(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    return (uint64_t)uni32((uint32_t)x) | ((uint64_t)uni32((uint32_t)(x >> 32)) << 32);
}
__device__ __forceinline__ uint64_t readlane64(uint64_t x, int l) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l) << 32);
}

// Pointers read from device memory are generic (flat) to the compiler; flat accesses count in
// both vmcnt and lgkmcnt, so every LDS wait would also wait for them.  gp() marks a pointer as
// global memory (address space 1) so accesses compile to global_load/store.
template <typename T> using gptr_t = __attribute__((address_space(1))) T*;
template <typename T> __device__ __forceinline__ gptr_t<T> gp(T* p) { return (gptr_t<T>)p; }

// one 24-B injection record through global (not flat) loads
// the first 24 B of a record (everything but dst_hi, which only the wide kernel reads)
__device__ __forceinline__ InjDev load_inj(const InjDev* p) {
    const gptr_t<const uint64_t> q = gp((const uint64_t*)p);
    const uint64_t w[3] = {q[0], q[1], q[2]};
    InjDev r;
    __builtin_memcpy(&r, w, 24);
    r.dst_hi[0] = r.dst_hi[1] = r.dst_hi[2] = 0;
    return r;
}

// packed LDS/HBM key metadata
__device__ __forceinline__ uint32_t m_s1(uint64_t m) { return (uint32_t)(m & 0xFFFF); }
__device__ __forceinline__ uint32_t m_tsend(uint64_t m) { return (uint32_t)((m >> 16) & 0xFFFF); }
__device__ __forceinline__ uint32_t m_tquiet(uint64_t m) { return (uint32_t)((m >> 32) & 0xFFFF); }
__device__ __forceinline__ uint32_t m_sender(uint64_t m) { return (uint32_t)((m >> 48) & 0xFF); }
__device__ __forceinline__ uint32_t m_value(uint64_t m) { return (uint32_t)((m >> 56) & 0x7F); }
// lean kernels: the LDS copy of a restricted-SEND key's metadata carries this bit (value ids are < 4)
constexpr uint64_t M_RESTRICTED = 1ull << 63;
__device__ __forceinline__ uint64_t m_pack(uint32_t s1, uint32_t tsend, uint32_t tquiet, uint32_t sender, uint32_t value) {
    return (uint64_t)(s1 & 0xFFFF) | ((uint64_t)(tsend & 0xFFFF) << 16) | ((uint64_t)(tquiet & 0xFFFF) << 32) |
           ((uint64_t)(sender & 0xFF) << 48) | ((uint64_t)(value & 0xFF) << 56);
}
__device__ __forceinline__ uint64_t m_with_tquiet(uint64_t m, uint32_t q) {
    return (m & ~(0xFFFFull << 32)) | ((uint64_t)(q & 0xFFFF) << 32);
}

// core/brbroadcast.py:60-119 for ONE (receiver, key) cell and every message reaching it in one
// step, in the canonical order SEND, ECHO by sender ascending, READY by sender ascending.  All
// arrivals grow their set (duplicates are suppressed), so the sequential threshold crossings
// have closed forms in the set sizes:
//   ECHO  : the first ECHO of a missing entry creates it WITHOUT the quorum check (:87-89);
//           every later one is checked (:92-98), the last checked size is |E| after the step.
//   READY : same creation quirk (:103-105); checked sizes run lo..hi; DELIVER at the first size
//           >= 2f+1 (:111-115); amplification (:118-119) fires for checked sizes in [f+1, 2f]
//           while no ECHO entry exists -- only its first firing leaves the node (duplicates).
// Branch-free (selects only): the wave evaluates it for all 64 receivers of a key at once.
__device__ __forceinline__ void brb_cell_update(uint32_t& fl, uint32_t& ec, uint32_t& rc, bool s_arr,
                                                uint32_t ea, uint32_t ra, uint32_t T_echo, uint32_t T_amp,
                                                uint32_t T_del, bool& echo_send, bool& ready_send, bool& deliver) {
    const bool open = !(fl & F_DEL);                                        // :74
    // a send the node already made (a user-issued ECHO / READY, base/broadcast.py:17) is a duplicate
    // on every link: the state changes, the sender-identity network carries nothing new
    const bool es_st = open && s_arr && !(fl & F_EEX);                      // :76-82
    echo_send = es_st && !(fl & F_ES);
    fl |= es_st ? (F_EEX | F_ES) : 0u;
    const bool e_on = open && ea != 0;
    const uint32_t checked = (fl & F_EEX) ? ea : ea - 1u;                   // :87-89
    fl |= e_on ? F_EEX : 0u;
    ec += e_on ? ea : 0u;                                                   // :89/:92
    const bool r1s = e_on && checked != 0 && ec >= T_echo && !(fl & F_REX); // :95-98
    const bool r1 = r1s && !(fl & F_RS);
    fl |= r1s ? (F_REX | F_RS) : 0u;
    const bool r_on = open && ra != 0;
    const bool rex = (fl & F_REX) != 0;
    const uint32_t lo = rex ? rc + 1u : 2u, hi = rex ? rc + ra : ra;       // :103-108
    fl |= r_on ? F_REX : 0u;
    rc += r_on ? ra : 0u;
    const bool any = r_on && hi >= lo;
    const uint32_t alo = max(lo, T_amp), ahi = min(hi, T_del - 1u);
    const bool r2 = any & !(fl & F_EEX) & (alo <= ahi) & !(fl & F_RS);      // :118-119
    fl |= r2 ? F_RS : 0u;
    deliver = any && hi >= T_del;                                           // :111-115
    fl |= deliver ? F_DEL : 0u;
    ready_send = r1 || r2;
}

// Bracha's broadcast as core/brbroadcast.py:60-119 intends it (BRC_MODE_SPEC; oracle
// brb_on_message_spec): ECHO on the first SEND of a key, ONE READY per key -- at the echo quorum or
// at f+1 READYs --, DELIVER at 2f+1 READYs, everything after DELIVER ignored.  All ECHOs of a step
// precede its READYs, so the sequential checks reduce to the step's final set sizes.
__device__ __forceinline__ void brb_cell_update_spec(uint32_t& fl, uint32_t& ec, uint32_t& rc, bool s_arr,
                                                     uint32_t ea, uint32_t ra, uint32_t T_echo, uint32_t T_amp,
                                                     uint32_t T_del, bool& echo_send, bool& ready_send, bool& deliver) {
    const bool open = !(fl & F_DEL);
    echo_send = open && s_arr && !(fl & F_ES);
    fl |= echo_send ? F_ES : 0u;
    ec += open ? ea : 0u;
    rc += open ? ra : 0u;
    ready_send = open && !(fl & F_RS) && (ec >= T_echo || rc >= T_amp);
    fl |= ready_send ? F_RS : 0u;
    deliver = open && rc >= T_del;
    fl |= deliver ? F_DEL : 0u;
}

// Best-effort broadcast (BRC_MODE_BEB; core/bebroadcast.py:30-42 as intended -- its constructor
// raises TypeError): a SEND delivers at its arrival, nothing is echoed.  The network suppresses
// duplicates, so each (origin, key) SEND reaches a receiver once.
__device__ __forceinline__ void brb_cell_update_beb(uint32_t& fl, bool s_arr, bool& echo_send, bool& ready_send,
                                                    bool& deliver) {
    deliver = s_arr && !(fl & F_DEL);
    fl |= deliver ? F_DEL : 0u;
    echo_send = ready_send = false;
}

// core/brbroadcast.py:60-119 with CONNECTION-identity peers (:69, the reference's local-test mode;
// SURVEY F1): every message is a new peer address, so the closed form of brb_cell_update holds
// with ea / ra counting MESSAGES, and the :118-119 amplification re-fires once per qualifying
// READY -- nothing suppresses the duplicates.  n_ready = READY broadcasts of the cell this step
// (the :98 one, or the re-fires); F_RS is left to the caller (it marks "has broadcast READY").
__device__ __forceinline__ void brb_cell_update_conn(uint32_t& fl, uint32_t& ec, uint32_t& rc, bool s_arr,
                                                     uint32_t ea, uint32_t ra, uint32_t T_echo, uint32_t T_amp,
                                                     uint32_t T_del, bool& echo_send, uint32_t& n_ready,
                                                     bool& deliver) {
    const bool open = !(fl & F_DEL);                                        // :74
    echo_send = open && s_arr && !(fl & F_EEX);                             // :76-82
    fl |= echo_send ? (F_EEX | F_ES) : 0u;
    const bool e_on = open && ea != 0;
    const uint32_t checked = (fl & F_EEX) ? ea : ea - 1u;                   // :87-89
    fl |= e_on ? F_EEX : 0u;
    ec += e_on ? ea : 0u;
    const bool r1 = e_on && checked != 0 && ec >= T_echo && !(fl & F_REX); // :95-98
    fl |= r1 ? F_REX : 0u;
    const bool r_on = open && ra != 0;
    const bool rex = (fl & F_REX) != 0;
    const uint32_t lo = rex ? rc + 1u : 2u, hi = rex ? rc + ra : ra;       // :103-108
    fl |= r_on ? F_REX : 0u;
    rc += r_on ? ra : 0u;
    const bool any = r_on && hi >= lo;
    const uint32_t alo = max(lo, T_amp), ahi = min(hi, T_del - 1u);
    const uint32_t fires = (any && !(fl & F_EEX) && alo <= ahi) ? ahi - alo + 1u : 0u;   // :118-119, each
    deliver = any && hi >= T_del;                                           // :111-115
    fl |= deliver ? F_DEL : 0u;
    n_ready = (r1 ? 1u : 0u) + fires;
}

// CONNECTION peers: a lane's send counts of one type over the last 16 steps, one byte per step
// (slot = step mod 16; slots 0-7 in `lo`, 8-15 in `hi`); `tl` = the last step with a send (NEVER:
// none).  Valid because a send reaches its receiver within D <= 16 steps and a cell is read before
// it is written in a step.  A count saturates nowhere below 255: one lane sends at most f + 1
// READY copies of a key in one step (brb_cell_update_conn), and injections past 255 are refused.
struct Ring16 { uint64_t lo, hi; };
constexpr uint32_t RING_MAX = 255u;
__device__ __forceinline__ uint32_t ring_count(const Ring16& r, uint32_t tl, uint32_t s) {
    if (tl == NEVER || s > tl || tl - s >= 16u) return 0u;
    // half select in arithmetic form: a ?: of the two fields becomes a scratch round trip
    const uint64_t w = r.lo ^ ((r.lo ^ r.hi) & (0ull - (uint64_t)((s >> 3) & 1u)));
    return (uint32_t)(w >> (8u * (s & 7u))) & 0xFFu;
}
__device__ __forceinline__ Ring16 ring_put(Ring16 r, uint32_t tl, uint32_t t, uint32_t c) {
    if (tl == NEVER || t - tl >= 16u) {
        r.lo = r.hi = 0;
    } else {
        for (uint32_t s = tl + 1u; s != t + 1u; ++s) {  // clear the slots of steps tl+1 .. t
            const uint64_t m = ~(0xFFull << (8u * (s & 7u)));
            if (s & 8u) r.hi &= m; else r.lo &= m;
        }
    }
    const uint64_t v = (uint64_t)min(c, RING_MAX) << (8u * (t & 7u)), m = ~(0xFFull << (8u * (t & 7u)));
    if (t & 8u) r.hi = (r.hi & m) | v; else r.lo = (r.lo & m) | v;
    return r;
}

#ifndef BRC_NL_MSTORE
#define BRC_NL_MSTORE 1      // non-lean kernels: exec-masked cell stores (0: whole-wave stores)
#endif
#ifndef BRC_LPK
#define BRC_LPK 1            // non-lean kernels: narrow delay masks packed in a register (0: read from LDS)
#endif
#ifndef BRC_MIN_WAVES
#define BRC_MIN_WAVES 4      // waves per SIMD the register allocation must allow
#endif
#ifndef BRC_MIN_WAVES_LEAN
#define BRC_MIN_WAVES_LEAN 4 // ... for the one-instance-per-wave (lean) instantiations: 128 VGPRs, no spills
#endif                       // (A/B round 4: 162.7 ms vs 168.1 ms at 5 waves, which spill 32 VGPRs)
#ifndef BRC_MIN_WAVES_LEAN_SPEC
#define BRC_MIN_WAVES_LEAN_SPEC 4 // lean SPEC: its LDS (9.2 KB per wave) bounds residency near 17 waves per CU
#endif                            // anyway (A/B round 4: 295 ms at 4 vs 309 ms at 5 waves/SIMD)
#ifndef BRC_SPEC_MULTI
#define BRC_SPEC_MULTI 1     // lean SPEC consensus: a key word's deliveries at once per distinct phase index
#endif
#ifndef BRC_PERKEY_CNT
#define BRC_PERKEY_CNT 1     // lean kernels: arrival counts per key of a pair only where that key's entry has the type (A/B: -0.8 %)
#endif
#ifndef BRC_BRANCHLESS
#define BRC_BRANCHLESS 0     // lean kernels: ECHO / READY stages of a pair evaluated whether or not they can land
#endif
#ifndef BRC_NOEARLY
#define BRC_NOEARLY 0        // lean kernels: no early exit for pairs that reach no open cell
#endif
#ifndef BRC_LCHUNK_SPEC
#define BRC_LCHUNK_SPEC 4    // lean SPEC: key slots in flight per chunk (8 spills two VGPRs there)
#endif
#ifndef BRC_DACC
#define BRC_DACC 1           // lean REFERENCE: deliveries collected per key word in a register (0: LDS atomics)
#endif
#ifndef BRC_OOBST
#define BRC_OOBST 1          // lean kernels: the key loop's cell stores unconditional, kept words dropped out of range
#endif
#ifndef BRC_PK
#define BRC_PK 1             // lean kernels: a key pair's cell updates in the two 16-bit halves of a register
#endif

// Two u16 lanes per register (v_pk_*_u16): the lean kernels update the cells of a key PAIR with one
// instruction per operation.  Every operand stays below 2^15 (set sizes <= 127, thresholds <= 65),
// so pk_ge's sign test is exact in each half; results are 0/1 in bits 0 and 16.
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) + __builtin_bit_cast(u16x2, b));
}
__device__ __forceinline__ uint32_t pk_sub(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) - __builtin_bit_cast(u16x2, b));
}
__device__ __forceinline__ uint32_t pk_min(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t pk_ge(uint32_t a, uint32_t b) { return (~pk_sub(a, b) >> 15) & 0x10001u; }
__device__ __forceinline__ uint32_t pk2(uint32_t x) { return x | (x << 16); }   // x < 2^16 in both halves

// Lean instantiations: one instance per wave (NPAD = 64, IPW = 1) with sender-identity peers.
// Every key-slot field is then wave-uniform, so the per-key work runs on scalar key ids,
// metadata read once per chunk, exec-masked cell stores and (NLR = 2) link-delay masks held in
// registers -- the headline configuration has exactly two link delays.
#ifdef BRC_STAMPS
#define BRC_NSTAMPS 12
// dev-only: [0..7] section timers (s_memtime ticks): step head + key list, key loop, consensus
// words, actions, stop checks, consensus snapshot, consensus row clears, key-loop tail (ring rows);
// [8..11] lean key-steps: processed, without arrivals, reaching only delivered cells, fully updated
__device__ unsigned long long brc_stamps[BRC_NSTAMPS];
#endif
template <int NPAD, int MODE> constexpr bool lean_kernel() { return NPAD == 64 && MODE != KMODE_CONN && MODE != KMODE_XREF; }

// Event-log instantiations (EV) run the class API's single-instance clusters and the parity tests' small
// batches, never a bandwidth workload: they take BRC_MIN_WAVES_EV waves per SIMD (256 VGPRs) so the event
// code spills nothing (at 128 VGPRs the n = 4 connection-peer kernel spilled 126 VGPRs to scratch)
#ifndef BRC_MIN_WAVES_EV
#define BRC_MIN_WAVES_EV 2
#endif
template <int NPAD, int DM, bool EV, int MODE, int NLR>
__global__ __launch_bounds__(64 * WPB, (EV ? BRC_MIN_WAVES_EV
                                           : lean_kernel<NPAD, MODE>() ? (MODE == BRC_MODE_SPEC ? BRC_MIN_WAVES_LEAN_SPEC
                                                                                              : BRC_MIN_WAVES_LEAN)
                                                                       : BRC_MIN_WAVES))
void brc_step(const Params* __restrict__ pp) {
    // Parameters live in device memory, not in kernarg: the loop's global stores may alias
    // them, so the compiler re-reads cold fields (scalar loads) where they are used instead of
    // pinning ~60 of them in SGPRs across the hot loop.  Hot fields are copied to locals below.
    const Params& P = *pp;
    constexpr bool SPEC = MODE == BRC_MODE_SPEC, BEB = MODE == BRC_MODE_BEB, CONN = MODE == KMODE_CONN;
    constexpr bool LEAN = lean_kernel<NPAD, MODE>();
    static_assert(NLR == 0 || (LEAN && NLR == 2), "register delay masks: lean kernels, two delays");
    constexpr uint32_t CW = CONN ? 5 : 1;        // u64 words per cell (CONN: + ECHO and READY send rings)
    using T = typename MaskOf<NPAD>::type;
    constexpr uint32_t RS = ring_steps(DM);      // activity-ring rows (> the largest delay)
    constexpr int IPW = 64 / NPAD;
    // activity-ring words per (row, key word): lean, one per message type; else one per instance of the item
    constexpr uint32_t AT = act_types(LEAN, IPW);
    constexpr bool PSEG = BRC_PSEG && !LEAN && IPW > 1;   // each instance walks its own key list
    // consensus value ids (brc_internal.h value_ids): VB bits each, NVAL of them; VREP has a 1 in
    // the low bit of every VB-bit field of `order`
    constexpr uint32_t NVAL = value_ids(!LEAN), VB = LEAN ? 2u : 3u, VMASK = NVAL - 1u;
    constexpr uint32_t VREP = LEAN ? 0x55u : 0x249249u;
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];

    // wid via readfirstlane: the item (and every address derived from it) is then provably wave-uniform
    const int wid = (int)uni32(threadIdx.x / 64), lane = threadIdx.x % 64;
    const uint64_t item = (uint64_t)blockIdx.x * WPB + wid;
    if (item >= P.nitems) return;               // whole wave exits; waves never synchronise
    const uint32_t n = P.n, NK = P.NK, Q = P.Q, NV = P.NV, D = P.D, nkw = P.nkw;
    const uint32_t T_echo = P.T_echo, T_amp = P.T_amp, T_del = P.T_del;
    // Q (phase window) and NV (key variants) are powers of two (brc_create): shifts, not divisions
    const uint32_t qsh = (uint32_t)__ffs(Q) - 1u, Qm = Q - 1u, ksh = qsh + (uint32_t)__ffs(NV) - 1u;
    // per-wave LDS carve (lds_bytes_per_wave): meta[IPW*NK] u64 | act[TS][nkw] u64 |
    //     dbits[nkw][64] u64 | consensus area | L[nL][64] T | mgen[IPW*NK] u16 | klist[NK + 2 CHUNK] u16
    // consensus area: REFERENCE hm[NVAL][64] T;  SPEC seen[Q][64] T, cnt[Q][64] u32
    const uint32_t nL = NLR ? 0u : P.nL;        // NLR: the masks live in registers, not in LDS
    const uint32_t h_words = cons_words(SPEC, (uint32_t)sizeof(T), Q, NV, NVAL);
    const bool seen_on = NV > 1;                 // SPEC: host sets needed only with key variants
    const uint32_t l_words = (nL * 64 * (uint32_t)sizeof(T) + 7) / 8;
    uint64_t* s_meta = smem + (size_t)wid * (lds_bytes_per_wave(NPAD, NK, nkw, nL, SPEC, Q, NV, RS, LEAN) / 8);
    uint64_t* s_act = s_meta + IPW * NK;
    // this step's deliveries, per lane: LDS, or (DBG: lean SPEC, whose LDS limits residency) one
    // HBM row per wave written once per key word from a register (dacc) -- no LDS at all
    constexpr bool DBG = LEAN && SPEC;
    const uint32_t dbw = DBG ? 0u : 64u * nkw;    // LDS u64 words of the delivery bitmap
    uint64_t* s_dbits = s_act + RS * nkw * AT;
    T* s_hm = (T*)(s_dbits + dbw);               // s_hm[v*64 + lane]: hosts that delivered value v
    T* s_seen = s_hm;                            // SPEC, NV > 1: s_seen[q*64 + lane]: hosts delivered for phase slot q
    // SPEC: s_cnt[q*64 + lane] = #origins | #"0" << 10 | #"1" << 20 for phase slot q
    uint32_t* s_cnt = (uint32_t*)(s_seen + (seen_on ? Q * 64 : 0u));
    T* s_L = (T*)(s_dbits + dbw + h_words);      // s_L[j*64 + lane]: senders at the j-th delay of dset
    // gen | GEN16_RESTRICTED (lean kernels keep no generations: no area)
    uint16_t* s_gen = (uint16_t*)(s_dbits + dbw + h_words + l_words);
    uint16_t* s_klist = s_gen + (LEAN ? 0u : ((IPW * NK + 3) & ~3u));        // this step's active key slots
    const uint32_t KLS = NK + 2 * KPAD;          // PSEG: entries per instance list (list seg at seg * KLS)
    // lean REFERENCE / BEB: u32 entries (KL_*); lean SPEC keeps u16 entries (its LDS bounds its residency)
    constexpr bool KL32 = LEAN && (!SPEC || BRC_KL32_SPEC);
    uint32_t* s_klist32 = (uint32_t*)s_klist;
    // non-lean kernels: a window of the item's injection records, staged in LDS (INJ_CACHE at a time)
    uint64_t* s_injc = (uint64_t*)(s_klist + ((KLS * (PSEG ? IPW : 1u) + 3) & ~3u));

    const int seg = lane / NPAD, d = lane % NPAD, segbase = seg * NPAD;
    const uint64_t inst = item * IPW + seg;
    const bool iex = inst < P.instances;
    const uint64_t g = P.inst_offset + inst;
    const uint64_t all64 = (n >= 64) ? ~0ull : ((1ull << n) - 1);
    const T allm = (T)all64;
    const uint64_t segbits = (NPAD == 64) ? ~0ull : (((1ull << NPAD) - 1) << segbase);
    const uint32_t mbase = seg * NK;             // this lane's instance in the LDS meta arrays

    ItemState its = P.items[item];
    uint32_t t = LEAN ? uni32(its.t) : its.t, inj_pos = LEAN ? uni32(its.inj_pos) : its.inj_pos;   // lean: wave-uniform
    uint32_t ep = LEAN ? uni32(its.epoch) : 0u;  // lean: compact-cell send steps are offsets from ep
    const uint32_t inj_off = gp(P.inj_off)[item], inj_cnt = gp(P.inj_cnt)[item];
    // injection record `pos` of this item: lean kernels load it directly (their workloads carry few);
    // the others keep INJ_CACHE records staged in LDS and refill the window with one coalesced load
    uint32_t injc_base = 0x80000000u;           // no window yet: pos - injc_base >= INJ_CACHE for any pos
    auto inj_at = [&](uint32_t pos) -> InjDev {
        if constexpr (LEAN) {
            return load_inj(P.inj + inj_off + pos);
        } else {
            if (pos - injc_base >= INJ_CACHE) {
                injc_base = pos;
                const uint32_t i = pos + (uint32_t)lane / 3u;
                if ((uint32_t)lane < 3 * INJ_CACHE && i < inj_cnt)
                    s_injc[lane] = gp((const uint64_t*)(P.inj + inj_off + i))[lane % 3];
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            }
            const uint32_t o = 3 * (pos - injc_base);
            const uint64_t w[3] = {s_injc[o], s_injc[o + 1], s_injc[o + 2]};
            InjDev r;
            __builtin_memcpy(&r, w, 24);
            r.dst_hi[0] = r.dst_hi[1] = r.dst_hi[2] = 0;
            return r;
        }
    };
    {
        const uint64_t mb = item * IPW * (uint64_t)NK;
        for (uint32_t i = lane; i < IPW * NK; i += 64) {
            const bool ok = item * IPW + i / NK < P.instances;
            const uint32_t g32 = ok ? gp(P.mgen)[mb + i] : 0u;
            s_meta[i] = ok ? gp(P.meta)[mb + i] | ((LEAN && (g32 & GEN_RESTRICTED)) ? M_RESTRICTED : 0ull) : 0ull;
            if (!LEAN) s_gen[i] = gen16(g32);
        }
        for (uint32_t i = lane; i < RS * nkw * AT; i += 64) s_act[i] = gp(P.act)[item * RS * nkw * AT + i];
        if (!DBG) for (uint32_t w = 0; w < nkw; ++w) s_dbits[w * 64 + lane] = 0;
    }
    uint32_t any_rows = uni32(gp(P.actany)[item]);   // ring rows holding any marked key (wave-uniform)
    uint32_t lane_rows = 0;                      // rows marked by per-lane sends, merged per step

    uint32_t status = BRC_DONE, t_stop = 0, q_until = 0;
    if (iex) {
        const uint64_t w0 = *(const gptr_t<uint64_t>)&gp(P.inst)[inst];     // status | t_stop | q_until | flags
        status = w0 & 0xFFFF; t_stop = (w0 >> 16) & 0xFFFF; q_until = (w0 >> 32) & 0xFFFF;
    }
    const uint64_t byzm = iex ? gp(P.byz)[inst] : ~0ull;
    const bool real = iex && (uint32_t)d < n;
    const bool honest = real && !((byzm >> d) & 1ull);
    // lane masks: a wave-uniform 64-bit mask turns back into a per-lane predicate at no cost
    // (inverse ballot: the SGPR pair is the lane mask), where a bool kept across blocks is
    // re-materialised with a select and a compare at every ballot
    const uint64_t hon_mask = uni64(__ballot(honest));
    auto lane_in = [](uint64_t mask) -> bool { return __builtin_amdgcn_inverse_ballot_w64(mask); };

    // ---- link-delay masks: L[i] = senders j whose link j -> d has delay i+1 (schedule.h)
    T L[DM];
#pragma unroll
    for (int i = 0; i < DM; ++i) L[i] = 0;
    if (real) {
        if (P.delay_model == BRC_DELAY_CONST) {
#pragma unroll
            for (int i = 0; i < DM; ++i) if ((uint32_t)i + 1 == P.dconst) L[i] = allm;
        } else if (P.delay_model == BRC_DELAY_SLOWSET) {
            const uint32_t off = slow_offset(P.seed, g, n);
            const bool me_slow = ((uint32_t)d + n - off) % n < P.f;
            // the slow set of this lane's instance: its segment's lanes with me_slow
            const T slowm = (T)(__ballot(me_slow) >> segbase);
#pragma unroll
            for (int i = 0; i < DM; ++i) {
                if ((uint32_t)i + 1 == D) L[i] |= me_slow ? allm : slowm;
                if (i == 0) L[i] |= me_slow ? (T)0 : (T)(allm & ~slowm);
            }
        } else {
            for (uint32_t j4 = 0; j4 < (n + 3) / 4; ++j4) {
                const u32x4 w = draw(P.seed, g, (uint32_t)d, PURPOSE_DELAY, j4);
                const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t j = 4 * j4 + q;
                    if (j >= n) break;
                    const uint32_t dl = (P.delay_model == BRC_DELAY_UNIFORM) ? uniform_delay(ws[q], D)
                                                                             : geometric_delay(ws[q], D);
#pragma unroll
                    for (int i = 0; i < DM; ++i) if ((uint32_t)i + 1 == dl) L[i] |= (T)((T)1 << j);
                }
            }
        }
    }
    bool ovf = false, badinj = false;
    // outset: delays (bit i <=> delay i+1) from THIS lane, as a sender, to honest receivers;
    // outv (lane i): the senders of the wave with a delay-(i+1) link to an honest receiver
    uint32_t outset = 0;
    uint64_t outv = 0;
#pragma unroll
    for (int i = 0; i < DM; ++i) {
        const T m = seg_or<NPAD, T>(honest ? L[i] : (T)0);
        const bool has_i = real && ((m >> d) & 1);
        if (has_i) outset |= 1u << i;
        const uint64_t b = __ballot(has_i);
        if (lane == i) outv = b;
    }
    const uint32_t maxout = hibit(outset);
    const uint32_t dset = wave_or_all(outset);       // every delay some link of this wave has
    // dlist: the delays present, minus one, 4 bits each in ascending order; ndl of them
    uint64_t dlist = 0;
    uint32_t ndl = 0;
    for (uint32_t ds = dset; ds; ds &= ds - 1) dlist |= (uint64_t)(__ffs(ds) - 1) << (4 * ndl++);
    dlist = uni64(dlist); ndl = uni32(ndl);
    // compact delay masks: the j-th delay present in the wave -> s_L[j]; every nonzero L[i] of an
    // honest receiver is in dset (its sender's outset has bit i)
    // NLR: the (at most two) delays present -> registers: RL0/RL1 = masks, dly0/dly1 = delays,
    // OV0/OV1 = the wave's senders with such a link (wave-uniform)
    T RL0 = 0, RL1 = 0;
    // LPK (narrow masks, few delays: NPAD = 16 at D <= 4, NPAD <= 8 at D <= 8): every compact mask
    // packed into one u64 register, read by a shift instead of an LDS round trip per key
    constexpr bool LPK = NLR == 0 && BRC_LPK && sizeof(T) * DM <= 8;
    uint64_t Lpk = 0;
    uint32_t dly0 = 0, dly1 = 0;
    uint64_t OV0 = 0, OV1 = 0;
    if constexpr (NLR != 0) {
        if (ndl > 2) ovf = true;                     // cannot happen: the host picks NLR for <= 2 delays
        dly0 = ndl > 0 ? (uint32_t)(dlist & 15) + 1u : 0u;
        dly1 = ndl > 1 ? (uint32_t)((dlist >> 4) & 15) + 1u : 0u;
#pragma unroll
        for (int i = 0; i < DM; ++i) {
            if ((uint32_t)i + 1 == dly0) RL0 = L[i];
            if ((uint32_t)i + 1 == dly1) RL1 = L[i];
        }
        if (ndl > 0) OV0 = uni64(readlane64(outv, (int)dly0 - 1));
        if (ndl > 1) OV1 = uni64(readlane64(outv, (int)dly1 - 1));
    } else {
        uint32_t j = 0;
#pragma unroll
        for (int i = 0; i < DM; ++i)
            if ((dset >> i) & 1) {
                if (j < nL) s_L[j * 64 + lane] = L[i];
                if constexpr (LPK) Lpk |= (uint64_t)L[i] << ((j * 8 * sizeof(T)) & 63);
                ++j;
            }
        if (j > nL) ovf = true;                      // cannot happen: delay_values() bounds dset
    }
    // lean ring marks (process_pair): lane L < 8 marks for delay class L & 1
    const uint64_t mk_ov = (lane & 1) ? OV1 : OV0;
    // the j-th delay mask present in the wave (j < ndl)
    auto Lmask = [&](uint32_t j) -> T {
        if constexpr (NLR != 0) return j == 0 ? RL0 : RL1;
        else if constexpr (LPK) return (T)(Lpk >> ((j * 8 * sizeof(T)) & 63));
        else return s_L[j * 64 + lane];
    };
    // cell (k, lane) at [k * CW * 64] (CONN send rings: ECHO at + 64, + 128, READY at + 192, + 256)
    const gptr_t<uint64_t> mycells = gp(P.cells) + item * (uint64_t)(NK + 1) * CW * 64 + lane;
    // lean SPEC: this wave's HBM delivery-bitmap row, word w at [w * 64]
    const gptr_t<uint64_t> gdbits = gp(P.dbits) + item * (uint64_t)nkw * 64 + lane;
    // lean kernels: compact u32 cells (brc_internal.h C32_*), row k at [k * 64].  Accessed through a
    // buffer resource over the item's rows (base and size in SGPRs): a row access is one
    // buffer_load/store_dword with voffset = 4 lane (a constant VGPR) and soffset = 256 k (an SGPR),
    // no per-lane 64-bit address arithmetic; a row index past the item's rows reads 0 and drops stores
    const __amdgpu_buffer_rsrc_t crs =
        __builtin_amdgcn_make_buffer_rsrc((void*)((uint32_t*)P.cells + item * (uint64_t)(NK + 1) * 64), (short)0,
                                          (int)((NK + 1) * 256u), 0x00020000);
    const uint32_t lv4 = (uint32_t)lane * 4u;
    auto cld = [&](uint32_t k) -> uint32_t { return __builtin_amdgcn_raw_buffer_load_b32(crs, lv4, k * 256u, 0); };
    auto cst = [&](uint32_t k, uint32_t v) { __builtin_amdgcn_raw_buffer_store_b32(v, crs, lv4, k * 256u, 0); };
    // the key loop's cell store as ONE unconditional instruction: lanes that keep their word get a
    // voffset past the resource's range, whose stores the buffer unit drops.  A store skipped by an
    // exec branch instead leaves the compiler unsure how many vector-memory ops are outstanding, and
    // its vmcnt waits then assume the fewest -- each pair waited for more cell loads than it reads
    auto cst_if = [&](uint32_t k, uint32_t v, bool wr) {
        if constexpr (BRC_OOBST) __builtin_amdgcn_raw_buffer_store_b32(v, crs, wr ? lv4 : 0x80000000u, k * 256u, 0);
        else if (wr) cst(k, v);
    };
    // lean: this lane's own key slots (bit s mod Q) allocated since the last flush; the wave
    // rewrites those rows fresh (flush_clears) before anything reads them
    uint32_t clr = 0;
    auto flush_clears = [&]() {
        if constexpr (LEAN) {
            for (uint64_t b = __ballot(clr != 0); b; b &= b - 1) {
                const int L = __ffsll((unsigned long long)b) - 1;
                for (uint32_t cm = uni32((uint32_t)__builtin_amdgcn_readlane((int)clr, L)); cm; cm &= cm - 1) {
                    const uint32_t k = ((uint32_t)L * NV) * Q + (uint32_t)__ffs(cm) - 1u;
                    cst(k, C32_FRESH);
                }
            }
            clr = 0;
        }
    };
    // lean: move the epoch to t - C32_KEEP when t is too far past it for a 7-bit offset.  Sends
    // before the new epoch are more than DM steps old and can no longer arrive: they become
    // C32_OLD (still "sent").  Only rows of slots holding a key.
    auto rebase = [&]() {
        if constexpr (LEAN) {
            const uint32_t nep = t - C32_KEEP, delta = nep - ep;
            for (uint32_t k = 0; k < NK; ++k) {
                if (m_s1(uni64(s_meta[k])) == 0) continue;
                const uint32_t c = cld(k);
                uint32_t oE = (c >> C32_OE_SH) & 127u, oR = c >> C32_OR_SH;
                if (oE < C32_OLD) oE = oE >= delta ? oE - delta : C32_OLD;
                if (oR < C32_OLD) oR = oR >= delta ? oR - delta : C32_OLD;
                cst(k, (c & ((1u << C32_OE_SH) - 1u)) | (oE << C32_OE_SH) | (oR << C32_OR_SH));
            }
            ep = nep;
        }
    };

    // ---- consensus state (core/byzantinerandomizedconsensus.py:25-29)
    uint64_t c0 = 0, c1 = 0;
    const size_t li = item * 64 + lane;
    const bool cons_lane = honest && P.protocol == BRC_PROTO_CONSENSUS;
    if (cons_lane) { c0 = gp(P.cons0)[li]; c1 = gp(P.cons1)[li]; }
    if constexpr (SPEC) {
        const T* gseen = (const T*)P.hmask;
        const uint32_t* gcnt = (const uint32_t*)((const char*)P.hmask + (seen_on ? P.nitems * Q * 64 * sizeof(T) : 0));
        for (uint32_t q = 0; q < Q; ++q) {
            if (seen_on) s_seen[q * 64 + lane] = cons_lane ? gp(gseen)[(item * Q + q) * 64 + lane] : (T)0;
            s_cnt[q * 64 + lane] = cons_lane ? gp(gcnt)[(item * Q + q) * 64 + lane] : 0u;
        }
    } else {
        for (uint32_t v = 0; v < NVAL; ++v)
            s_hm[v * 64 + lane] = cons_lane ? gp((const T*)P.hmask)[(item * NVAL + v) * 64 + lane] : (T)0;
    }
    uint32_t round = c0 & 0xFFFF, phase = (c0 >> 16) & 0xF, nvals = (c0 >> 20) & 0xF;   // cons0_pack
    uint32_t order = (c0 >> 24) & 0xFFFFFF, vcount = (c0 >> 48) & 0xFFFF;
    uint32_t dcount = c1 & 0xFFFF, frnd = (c1 >> 16) & 0xFFFF, ft = (c1 >> 32) & 0xFFFF;
    uint32_t fval = (c1 >> 48) & 0xFF, lval = (c1 >> 56) & 0xFF;

    // Extra SENDs of a key already SENT (one payload string SENT by several origins, or again: the
    // reference keys its BRB state by payload, core/brbroadcast.py:38-44, :76-82), non-lean kernels:
    // per item XSEND_MAX records {k | t << 16 | seg << 40, sender mask, dst mask} in HBM (P.xsend,
    // written by brc_inject), xs_n in use (P.xsn).  Sender j of a record lands on receiver d at
    // t + delay(j -> d), as the key's own SEND; SENDs of one key at one step to one destination set
    // share a record.  (Sender peers: brc_inject has removed the links a sender used before.)
    uint32_t xs_n = LEAN ? 0u : uni32(gp(P.xsn)[item]);
    auto xs_ld = [&](uint32_t i) -> uint64_t { return uni64(gp(P.xsend)[item * (uint64_t)(3 * XSEND_MAX) + i]); };

    uint32_t st_msgs = 0, st_arr = 0, st_cells = 0, st_del = 0, st_loads = 0, st_smax = 0;
    uint32_t st_bcast = 0;                       // lean path: ECHO/READY broadcasts (n messages each)
    // lean path, wave-uniform: key list entries (nk_lean) minus empty slots among them (nk_skip)
    uint32_t nk_lean = 0, nk_skip = 0;

    auto log_ev = [&](uint32_t kind, uint32_t node, uint32_t type, uint32_t a, uint32_t b, uint32_t v) {
        if (EV) {
            const unsigned long long i = atomicAdd(P.event_count, 1ull);
            if (i < P.event_cap) {
                brc_event e;
                e.instance = inst; e.t = t; e.kind = (uint8_t)kind; e.node = (uint8_t)node;
                e.type = (uint8_t)type; e.value = (uint8_t)v; e.a = a; e.b = b;
                P.events[i] = e;
            }
        }
    };
    // key k may have arrivals of message type ty (BRC_SEND / BRC_ECHO / BRC_READY) at t + i + 1 for
    // every bit i of ds (called by individual lanes).  Lean kernels: typed rows (ECHO row, READY row);
    // a SEND leaves no key mark there (the key list finds SEND arrivals from the key metadata), only
    // the row bit that makes the step loop visit that step.
    auto mark_lane = [&](uint32_t k, uint32_t ds, uint32_t ty) {
        while (ds) {
            const uint32_t i = __ffs(ds) - 1; ds &= ds - 1;
            const uint32_t row = (t + i + 1) & (RS - 1);
            if (!LEAN || ty != BRC_SEND)
                atomicOr((unsigned long long*)&s_act[(row * AT + (LEAN ? ty - BRC_ECHO : PSEG ? (uint32_t)seg : 0u)) * nkw + (k >> 6)],
                         1ull << (k & 63));
            lane_rows |= 1u << row;
        }
    };
    // lean kernels: does key slot k still have ECHO / READY arrivals pending?  Every ring row but the
    // current one holds only future marks (a marked row is always visited and cleared), so the key
    // loop keeps no per-key t_quiet for them; t_quiet in the metadata covers the SEND alone.
    auto ring_busy = [&](uint32_t k) -> bool {
        const uint32_t kw = k >> 6, cur = t & (RS - 1);
        uint64_t acc = 0;
#pragma unroll 1
        for (uint32_t r = 0; r < RS; ++r)
            if (r != cur) acc |= s_act[(r * AT + 0) * nkw + kw] | s_act[(r * AT + 1) * nkw + kw];
        return (acc >> (k & 63)) & 1ull;
    };
    // honest origin d broadcasts SEND for its key (d, s) with value v
    // (core/byzantinerandomizedconsensus.py:48-50 / :80-83 / :102-106, base/broadcast.py:30-35)
    auto send_key_now = [&](uint32_t s, uint32_t v) {
        const uint32_t k = (d * NV) * Q + (s & Qm);
        const uint64_t m = s_meta[mbase + k];
        // a busy slot, or a phase index past this run's generation budget (brc_run): overflow
        if ((m_s1(m) != 0 && (t < m_tquiet(m) || (LEAN && ring_busy(k)))) || s >= P.s_limit) { ovf = true; return; }
        if (!LEAN) s_gen[mbase + k] = (uint16_t)(((s_gen[mbase + k] & GEN_MASK) + 1) & GEN_MASK);
        if (LEAN) clr |= 1u << (s & Qm);                 // compact cells: the row is rewritten fresh
        s_meta[mbase + k] = m_pack(s + 1, t, t + maxout, d, v);
        mark_lane(k, outset, BRC_SEND);
        q_until = max(q_until, t + maxout);
        st_msgs += n;
        st_smax = max(st_smax, s);
        log_ev(BRC_EV_SEND, d, BRC_SEND, d * NV, s, v);
    };
    // During the consensus pass a replica's SENDs are queued and performed after the pass
    // (flush_sends): a phase change reallocates the replica's own slot, while another replica may
    // still have to count a delivery of the slot's old key from this same step -- deferring keeps
    // every slot's metadata as the BRB phase left it for the whole pass (no snapshot needed).  The
    // SENDs of one replica in one pass have consecutive phase indices (each phase change advances
    // the index by one): the queue keeps the first index and a VB-bit value id per SEND.
    bool defer_sends = false;
    uint32_t sq_s = 0, sq_n = 0;
    SendQ<VB> sq_v;
    sq_v.clear();
    auto send_key = [&](uint32_t s, uint32_t v) {
        if (defer_sends) {
            if (sq_n == 0) sq_s = s;
            if (s == sq_s + sq_n && sq_n < SENDQ_MAX) { sq_v.put(sq_n, v & VMASK); ++sq_n; }
            else ovf = true;                                 // consecutive indices; past SENDQ_MAX: overflow
            return;
        }
        send_key_now(s, v);
    };
    auto flush_sends = [&]() {
        for (uint32_t i = 0; i < sq_n; ++i) send_key_now(sq_s + i, sq_v.get(i) & VMASK);
        sq_n = 0; sq_v.clear();
    };
    auto get_max_val = [&](uint32_t bound2) -> uint32_t {          // :64-68
        for (uint32_t i = 0; i < nvals; ++i) {
            const uint32_t v = (order >> (VB * i)) & VMASK;
            if (2 * popc(s_hm[v * 64 + lane]) > bound2) return v;
        }
        return 0;                                                    // str(NONE) == "-1"
    };
    auto cons_reset = [&]() {
        vcount = 0; nvals = 0; order = 0;
        for (uint32_t v = 0; v < NVAL; ++v) s_hm[v * 64 + lane] = 0;
    };
    // :71-106: the phase ends a delivery may complete (value_count has just grown)
    auto cons_after = [&]() {
        if (vcount >= P.T_cnt && phase == 1) {                       // :71
            const uint32_t prop = get_max_val(P.bound_p1);           // :73
            phase = 2; cons_reset();                                 // :75-78
            send_key(2 * (round - 1) + 1, prop);                     // :80-83
        }
        if (vcount >= P.T_cnt && phase == 2) {                       // :86
            const uint32_t dec = get_max_val(P.bound_p2);            // :88
            // :89 compares str with int: never equal -> decide() always runs (:94)
            ++dcount;
            if (dcount == 1) { frnd = round; ft = t; fval = dec; }
            lval = dec;
            log_ev(BRC_EV_DECIDE, d, 0, round, dec, dec);
            ++round; phase = 1; cons_reset();                        // :96-100
            send_key(2 * (round - 1), dec);                          // :102-106
        }
    };
    // :53-106 for a message of `host` carrying value id v (a BRB delivery, or BRC_INJ_DELIVER)
    auto cons_deliver_vh = [&](uint32_t v, uint32_t host) {
        // v already inserted? compare it with every VB-bit field of `order` at once (nvals <= NVAL)
        const uint32_t x = order ^ (v * VREP);                       // a field is 0 where it equals v
        const uint32_t valid = (1u << (VB * nvals)) - 1u;             // fields in use
        const bool found = (~(x | (x >> 1) | (VB == 3 ? x >> 2 : 0u)) & VREP & valid) != 0;
        if (!found) { order |= v << (VB * nvals); ++nvals; }        // :57-58
        s_hm[v * 64 + lane] |= (T)((T)1 << host);                   // :60
        ++vcount;                                                    // :61
        cons_after();
    };
    auto cons_deliver = [&](uint32_t k) {
        cons_deliver_vh(m_value(s_meta[mbase + k]) & VMASK, k >> ksh); // metadata as the BRB phase left it
    };

    // ---- SPEC consensus (oracle spec_advance / spec_deliver): the protocol
    // core/byzantinerandomizedconsensus.py:53-106 intends -- a phase ends once n-f DISTINCT origins
    // delivered a key of THAT phase (deliveries of later phases are buffered in slot s % Q, earlier
    // ones dropped); phase 1 proposes a value carried by more than (n+f)/2 of them (:73), phase 2
    // decides above 2f (:88), adopts above f and otherwise takes the common coin (:90-92, reachable
    // here), then the next round starts.
    auto spec_advance = [&]() {
        while (round > 0) {
            const uint32_t s = 2 * (round - 1) + (phase - 1), q = s & Qm;
            const uint32_t cc = s_cnt[q * 64 + lane], n0 = (cc >> 10) & 0x3FF, n1 = cc >> 20;
            if ((seen_on ? popc(s_seen[q * 64 + lane]) : (cc & 0x3FF)) < n - P.f) return;
            if (seen_on) s_seen[q * 64 + lane] = 0;
            s_cnt[q * 64 + lane] = 0;
            if (phase == 1) {
                const uint32_t prop = (2 * n0 > n + P.f) ? 1u : (2 * n1 > n + P.f) ? 2u : 0u;
                phase = 2;
                send_key(s + 1, prop);
            } else {
                const uint32_t vmax = n1 > n0 ? 2u : 1u, cmax = max(n0, n1);
                uint32_t est;
                if (cmax > 2 * P.f) {
                    ++dcount;
                    if (dcount == 1) { frnd = round; ft = t; fval = vmax; }
                    lval = vmax;
                    log_ev(BRC_EV_DECIDE, d, 0, round, vmax, vmax);
                    est = vmax;
                } else if (cmax > P.f) {
                    est = vmax;
                } else {
                    est = coin_id(P.coin_seed, g, round);
                }
                ++round; phase = 1;
                send_key(s + 1, est);
            }
        }
    };
    auto spec_deliver = [&](uint32_t k) {
        const uint64_t mk = s_meta[mbase + k];                      // as the BRB phase left it (send_key)
        const uint32_t s = m_s1(mk) - 1u, v = m_value(mk) & 3u, host = k >> ksh;
        const uint32_t cur = round ? 2 * (round - 1) + (phase - 1) : 0u;
        if (s < cur) return;
        if (s >= cur + Q) { ovf = true; return; }
        const uint32_t q = s & Qm;
        if (seen_on) {
            if ((s_seen[q * 64 + lane] >> host) & 1) return;
            s_seen[q * 64 + lane] |= (T)((T)1 << host);
        }
        s_cnt[q * 64 + lane] += 1u + (v == 1 ? 1u << 10 : 0u) + (v == 2 ? 1u << 20 : 0u);
        spec_advance();
    };

    // BRC_INJ_MSG: this lane (the record's node) broadcasts ECHO / READY of key r.slot; true if the
    // message travels (sender peers: not a duplicate; connection peers: always)
    auto msg_cell = [&](const InjDev& r) -> bool {
        const uint32_t k = LEAN ? uni32(r.slot) : r.slot;   // lean: records are wave-uniform (IPW = 1)
        bool sent = false;
        const uint64_t m = s_meta[mbase + k];
        if (m_s1(m) != r.s + 1u) {
            badinj = true;
        } else if constexpr (LEAN) {
            // compact cell: F_ES / F_RS and the send-step offset
            const uint32_t wv = cld(k);
            const uint32_t bit = (r.type == BRC_ECHO) ? F_ES : F_RS;
            const uint32_t sh = (r.type == BRC_ECHO) ? C32_OE_SH : C32_OR_SH;
            if (!(wv & bit)) {
                sent = true;
                cst(k, ((wv | bit) & ~(127u << sh)) | ((t - ep) << sh));
                st_msgs += n;
                log_ev(BRC_EV_SEND, d, r.type, (k >> qsh), r.s, m_value(m));
            }
        } else {
            const uint32_t gen = s_gen[mbase + k] & GEN_MASK;
            uint64_t wv = mycells[(size_t)k * (CW * 64)];
            const bool stale = ((wv >> 19) & GEN_MASK) != gen;
            if (stale) wv = TIMES_NEVER | ((uint64_t)gen << 19);
            const uint32_t bit = (r.type == BRC_ECHO) ? F_ES : F_RS;
            const int sh = (r.type == BRC_ECHO) ? 32 : 48;
            if constexpr (CONN) {
                // every injected broadcast travels: one more send of this type at step t
                const size_t ri = (size_t)k * (CW * 64) + ((r.type == BRC_ECHO) ? 64 : 192);
                const uint32_t tl = (uint32_t)(wv >> sh) & 0xFFFF;
                Ring16 ring = {mycells[ri], mycells[ri + 64]};
                const uint32_t c = ring_count(ring, tl, t) + 1u;
                if (c > RING_MAX) {
                    badinj = true;                      // beyond the one-byte count
                } else {
                    sent = true;
                    ring = ring_put(ring, tl, t, c);
                    mycells[ri] = ring.lo;
                    mycells[ri + 64] = ring.hi;
                    // the first broadcast of (node, type, key) is a SEND event, every later copy a COPY
                    log_ev((wv & bit) ? BRC_EV_COPY : BRC_EV_SEND, d, r.type, (k >> qsh), r.s, m_value(m));
                    wv = ((wv | bit) & ~(0xFFFFull << sh)) | ((uint64_t)t << sh);
                    mycells[(size_t)k * (CW * 64)] = wv;
                    st_msgs += n;
                }
            } else if (!(wv & bit)) {
                sent = true;
                wv |= bit;
                wv = (wv & ~(0xFFFFull << sh)) | ((uint64_t)t << sh);
                mycells[(size_t)k * (CW * 64)] = wv;
                st_msgs += n;
                log_ev(BRC_EV_SEND, d, r.type, (k >> qsh), r.s, m_value(m));
            }
        }
        return sent;
    };
    // ... and its wave-level effects: ring marks at t + the senders' link delays, the key's t_quiet
    auto msg_marks = [&](const InjDev& r, bool mine, bool sent) {
        const uint32_t k = r.slot;
        const uint32_t os = wave_or(sent ? outset : 0u);
        if (os) {
            if (lane == 0) mark_lane(k, os, r.type);
            const uint32_t myq = seg_max<NPAD>(sent ? t + maxout : 0u);
            if (mine && myq) {
                if (d == 0) {
                    const uint64_t m = s_meta[mbase + k];
                    if (myq > m_tquiet(m)) s_meta[mbase + k] = m_with_tquiet(m, myq);
                }
                q_until = max(q_until, myq);
            }
        }
    };

    // a SEND / KEY record of this lane's instance (the caller's `mine`): the slot's metadata (lane d = 0),
    // and for a SEND its destinations, ring marks at the delays in os and its message count.  Returns
    // whether the slot was (re)allocated (lean: a fresh row)
    auto send_rec = [&](const InjDev& r, const uint32_t os) -> bool {
        const bool is_send = r.kind == BRC_INJ_SEND;
        const uint32_t k = r.slot;
        bool fresh = false;
        if (d == 0) {
            uint64_t m = s_meta[mbase + k];
            uint32_t gen = LEAN ? 0u : s_gen[mbase + k] & GEN_MASK;
            const bool declared = m_s1(m) == r.s + 1u && m_tsend(m) == NEVER && is_send;
            if ((!declared && m_s1(m) != 0 && (t < m_tquiet(m) || (LEAN && ring_busy(k)))) || r.s >= P.s_limit) {
                ovf = true;
            } else {
                uint32_t tq = m_tquiet(m);
                // a declared key holds its slot at least until the next step
                if (!declared) { gen = (gen + 1) & GEN_MASK; tq = t + 1; fresh = true; }
                if (is_send) tq = max(tq, t + hibit(os));
                m = m_pack(r.s + 1, is_send ? t : NEVER, tq, r.node, (uint32_t)(uint8_t)r.value);
                s_meta[mbase + k] = m;
                const bool restricted = is_send && (r.dst & all64) != all64;
                if (!LEAN) s_gen[mbase + k] = (uint16_t)(gen | (restricted ? GEN16_RESTRICTED : 0u));
                if (LEAN && restricted) s_meta[mbase + k] = m | M_RESTRICTED;
                st_smax = max(st_smax, (uint32_t)r.s);
                if (is_send) {
                    gp(P.kdst)[inst * NK + k] = r.dst;
                    mark_lane(k, os, BRC_SEND);
                    st_msgs += __popcll(r.dst & all64);
                    log_ev(BRC_EV_SEND, r.node, BRC_SEND, (k >> qsh), r.s, (uint32_t)(uint8_t)r.value);
                }
            }
        }
        return fresh;
    };
    // the delays at which this lane (an honest destination of SEND r) hears the SEND's origin
    auto send_delay_set = [&](const InjDev& r, const bool mine) -> uint32_t {
        uint32_t myset = 0;
        if (r.kind == BRC_INJ_SEND && mine && honest && ((r.dst >> d) & 1ull)) {
            uint32_t j = 0;
            for (uint32_t ds = dset; ds; ds &= ds - 1, ++j)
                if ((Lmask(j) >> r.node) & 1) myset = 1u << (__ffs(ds) - 1);
        }
        return myset;
    };

    // ---- actions stamped t (performed after step t's messages)
    auto do_actions = [&]() -> bool {
        bool mine_any = false;
        const bool running = status == BRC_RUNNING;
        if (its.initialized == 0 && t == 0) {
            if (P.protocol == BRC_PROTO_CONSENSUS && P.proposals != BRC_PROPOSALS_NONE && honest && running) {
                const uint32_t v = (P.proposals == BRC_PROPOSALS_PHILOX) ? proposal_id(P.seed, g, d)
                                                                         : (uint32_t)gp(P.prop)[inst * n + d];
                round = 1; phase = 1;                                 // :43-47
                send_key(0, v & (SPEC ? 3u : VMASK));
                if constexpr (SPEC) spec_advance();                   // phase 0 may be buffered
            }
            flush_clears();
        }
        while (inj_pos < inj_cnt) {
            const InjDev r = inj_at(inj_pos);
            if (r.t != t) break;
            ++inj_pos;
            const bool mine = running && seg == (int)r.seg;
            mine_any |= mine;
            if (r.kind == BRC_INJ_PROPOSE) {
                if (mine && honest && d == r.node) {
                    round = 1; phase = 1; send_key(0, (uint32_t)r.value & (SPEC ? 3u : VMASK));
                    if constexpr (SPEC) spec_advance();
                }
            } else if (r.kind == BRC_INJ_DELIVER) {
                // a direct deliver() call (brc_inject refuses it for SPEC): host in r.slot
                if constexpr (!SPEC) {
                    if (mine && honest && d == r.node) cons_deliver_vh((uint32_t)r.value & VMASK, r.slot);
                }
            } else if (!LEAN && IPW > 1 && (r.kind == BRC_INJ_SEND || r.kind == BRC_INJ_KEY) && !(r.type & 2u)) {
                // a run of SEND / KEY records at this step (within the staged window, no extra SEND):
                // the item's instances are independent, so every segment applies its own records, in
                // order, all segments at once (cfg3's equivocation pattern: 40 such records per wave)
                const uint32_t p0 = inj_pos - 1;
                uint32_t p1 = inj_pos;
                while (p1 < inj_cnt && p1 - injc_base < INJ_CACHE) {
                    const InjDev q = inj_at(p1);
                    if (q.t != t || (q.kind != BRC_INJ_SEND && q.kind != BRC_INJ_KEY) || (q.type & 2u)) break;
                    ++p1;
                }
                inj_pos = p1;
                uint32_t myrecs = 0;
                for (uint32_t p = p0; p < p1; ++p)
                    if (seg == (int)inj_at(p).seg) myrecs |= 1u << (p - p0);
                while (__any(myrecs != 0)) {
                    InjDev q = r;
                    const bool has = myrecs != 0;
                    if (has) {
                        const uint32_t i = (uint32_t)__ffs(myrecs) - 1u;
                        myrecs &= myrecs - 1;
                        q = inj_at(p0 + i);              // inside the staged window: no refill
                    }
                    const bool mq = has && running;
                    mine_any |= mq;
                    const uint32_t os = seg_or<NPAD, uint32_t>(send_delay_set(q, mq));
                    if (mq) {
                        send_rec(q, os);
                        q_until = max(q_until, t + hibit(os));
                    }
                }
            } else if (r.kind == BRC_INJ_SEND || r.kind == BRC_INJ_KEY) {
                // KEY declares a (Byzantine) key without sending; SEND sends it, allocating the
                // slot first unless that key was declared and not yet sent
                const uint32_t os = wave_or(send_delay_set(r, mine));
                // a SEND of a key already SENT (another origin or again, one payload): brc_inject has
                // put it in the item's extra-SEND records (r.type bit 1; bit 0: a repeat of this node's)
                if (!LEAN && (r.type & 2u)) {
                    if (mine && d == 0) {
                        const uint32_t k = r.slot;
                        const uint64_t m = s_meta[mbase + k];
                        if (m_s1(m) != r.s + 1u || m_tsend(m) == NEVER) {
                            badinj = true;                   // the key is not the SENT one brc_inject saw
                        } else {
                            if (t + hibit(os) > m_tquiet(m)) s_meta[mbase + k] = m_with_tquiet(m, t + hibit(os));
                            mark_lane(k, os, BRC_SEND);
                            st_msgs += __popcll(r.dst & all64);
                            // a node's first SEND of the key is a SEND event; a repeat is a COPY event with
                            // connection peers and none with sender peers (as for any duplicate)
                            if (!(r.type & 1u)) log_ev(BRC_EV_SEND, r.node, BRC_SEND, (k >> qsh), r.s, m_value(m));
                            else if (CONN) log_ev(BRC_EV_COPY, r.node, BRC_SEND, (k >> qsh), r.s, m_value(m));
                        }
                    }
                    if (mine) q_until = max(q_until, t + hibit(os));
                } else if (mine) {
                    const bool fresh = send_rec(r, os);
                    if constexpr (LEAN) {
                        if (__ballot(fresh)) cst(uni32((uint32_t)r.slot), C32_FRESH);
                    }
                    q_until = max(q_until, t + hibit(os));
                }
            } else if (r.kind == BRC_INJ_MSG) {
                if constexpr (!LEAN) {
                    // a run of MSG records at this step (within the staged window): every lane applies
                    // its own records at once, so their cell loads overlap (cfg3's equivocation pattern
                    // is 80 such records per wave at step 1)
                    const uint32_t p0 = inj_pos - 1;
                    uint32_t p1 = inj_pos;
                    while (p1 < inj_cnt && p1 - injc_base < INJ_CACHE) {
                        const InjDev q = inj_at(p1);
                        if (q.t != t || q.kind != BRC_INJ_MSG) break;
                        ++p1;
                    }
                    inj_pos = p1;
                    uint32_t myrecs = 0;
                    for (uint32_t p = p0; p < p1; ++p) {
                        const InjDev q = inj_at(p);
                        const bool mq = running && seg == (int)q.seg;
                        mine_any |= mq;
                        if (mq && d == q.node) myrecs |= 1u << (p - p0);
                    }
                    // the wave-level effects of a record reduce to its one sending lane: ring marks
                    // at t + its link delays, its q_until, and the key's t_quiet (an LDS CAS: lanes
                    // of other records may raise the same key's t_quiet)
                    while (__any(myrecs != 0)) {
                        if (myrecs) {
                            const uint32_t i = (uint32_t)__ffs(myrecs) - 1u;
                            myrecs &= myrecs - 1;
                            const InjDev q = inj_at(p0 + i);
                            if (msg_cell(q) && outset) {
                                mark_lane(q.slot, outset, q.type);
                                const uint32_t myq = t + maxout;
                                q_until = max(q_until, myq);
                                unsigned long long* mp = (unsigned long long*)&s_meta[mbase + q.slot];
                                unsigned long long cur = *mp;
                                while (m_tquiet(cur) < myq) {
                                    const unsigned long long prev = atomicCAS(mp, cur, (unsigned long long)m_with_tquiet(cur, myq));
                                    if (prev == cur) break;
                                    cur = prev;
                                }
                            }
                        }
                    }
                } else {
                    msg_marks(r, mine, (mine && d == r.node) ? msg_cell(r) : false);
                }
            }
            flush_clears();                          // PROPOSE / DELIVER may have started a key
        }
        its.initialized = 1;
        return mine_any;
    };

    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (its.initialized == 0 && t == 0) {
        do_actions();
        q_until = NPAD == 64 ? wave_max_all(q_until) : seg_max<NPAD>(q_until);
        any_rows |= wave_or_all(lane_rows);
        lane_rows = 0;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }

#ifdef BRC_STAMPS
    uint64_t stamp_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t kcount[4] = {0, 0, 0, 0};
    uint64_t stamp_prev = __builtin_amdgcn_s_memtime();
#define BRC_STAMP(i) do { const uint64_t _n = __builtin_amdgcn_s_memtime(); stamp_acc[i] += _n - stamp_prev; stamp_prev = _n; } while (0)
#define BRC_KCOUNT(i) (++kcount[i])
#else
#define BRC_STAMP(i) do {} while (0)
#define BRC_KCOUNT(i) do {} while (0)
#endif
    for (uint32_t it = 0; it < P.max_steps; ++it) {
        const bool running0 = status == BRC_RUNNING;
        if (!__any(running0)) break;
        const bool running = IPW == 1 || running0;       // one instance per wave: it is running
        const bool hon_run = honest && running, real_run = real && running;
        // next step with possible arrivals (activity ring) or a pending action
        const uint32_t rot = (t + 1) & (RS - 1);
        const uint32_t rr = (rot ? ((any_rows >> rot) | (any_rows << (RS - rot))) : any_rows) &
                            (RS == 32 ? ~0u : ((1u << RS) - 1u));
        uint32_t next = rr ? t + (uint32_t)__ffs(rr) : 0xFFFFFFFFu;
        if (inj_pos < inj_cnt) next = min(next, inj_at(inj_pos).t);
        if (next == 0xFFFFFFFFu) { if (running) status = BRC_QUIESCENT; break; }
        if (next > P.step_cap) { if (running) status = BRC_STEPCAP; break; }
        t = LEAN ? uni32(next) : next;
        const uint32_t row = t & (RS - 1);
        if (LEAN && t - ep > C32_REBASE) rebase();

        // ================= BRB: the step's active key slots; one (receiver, key) cell per lane.
        // The ring row becomes a key list (marks made now land on other rows, so it is fixed);
        // keys come CHUNK at a time and the next chunk's cell words load while one is processed.
        const uint32_t cells0 = st_cells;
        // lean: this step's deliveries are collected per key word in a register (dacc, word dcur) and
        // stored once when the next word starts: LDS, or (DBG) the wave's HBM row; dwm = words written
        uint64_t dacc = 0;
        uint32_t dcur = NOKEY, dwm = 0;
        auto flush_dacc = [&](uint32_t wk, uint64_t v) {
            if constexpr (DBG) gdbits[wk * 64] = v;
            else s_dbits[wk * 64 + lane] = v;
            dwm |= 1u << wk;
        };
        uint32_t nkeys = 0, nks = 0;                // PSEG: nks = this instance's list length
        if constexpr (LEAN) {
            // typed marks: ECHO / READY rows; SEND arrivals from the slot's metadata -- the SEND of slot
            // k lands now at some receiver iff t - t_send is a delay of its sender's outset (reading the
            // next key word ahead measured no gain: A/B round 4)
            for (uint32_t w = 0; w < nkw; ++w) {
                const uint64_t mE = uni64(s_act[(row * AT + 0) * nkw + w]), mR = uni64(s_act[(row * AT + 1) * nkw + w]);
                const uint64_t m = s_meta[w * 64 + lane];
                const uint32_t dt = t - m_tsend(m);                        // the delay of a SEND landing now
                bool sl;
                if constexpr (NLR != 0) {
                    // OV0 / OV1: the senders with a link of delay dly0 / dly1 to an honest receiver
                    const uint32_t snd = m_sender(m) & 63u;
                    sl = m_s1(m) != 0 && ((dt == dly0 && ((OV0 >> snd) & 1ull)) || (dt == dly1 && ((OV1 >> snd) & 1ull)));
                } else {
                    const uint32_t dt1 = dt - 1u;
                    const uint32_t os = (uint32_t)__shfl((int)outset, (int)m_sender(m));
                    sl = m_s1(m) != 0 && dt1 < 32u && ((os >> (dt1 & 31u)) & 1u);
                }
                const uint32_t tb = (sl ? TB_S : 0u) | ((uint32_t)(mE >> lane) & 1u) * TB_E | ((uint32_t)(mR >> lane) & 1u) * TB_R;
                const uint64_t bits = __ballot(tb != 0);
                const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(bits >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)bits, 0u));
                if (tb != 0) {
                    if constexpr (KL32) {
                        const uint32_t sx = (tb & TB_S) ? (((m_sender(m) & 63u) << KL_SND_SH) | (((dt - 1u) & 15u) << KL_DT_SH) |
                                                           ((m & M_RESTRICTED) ? KL_RESTR : 0u)) : 0u;
                        s_klist32[nkeys + below] = (w * 64 + lane) | (tb << TB_SH) | sx;
                    } else {
                        s_klist[nkeys + below] = (uint16_t)((w * 64 + lane) | (tb << TB_SH));
                    }
                }
                nkeys += (uint32_t)__popcll(bits);
            }
        } else if constexpr (PSEG) {
            // one key list per instance (segment): the segment's lanes list its marked slots, NPAD bits
            // of a ring word at a time; nks = this segment's length, nkeys = the longest list
            for (uint32_t w = 0; w < nkw; ++w) {
                const uint64_t bits = s_act[(row * AT + (uint32_t)seg) * nkw + w];
                for (uint32_t b0 = 0; b0 < 64; b0 += NPAD) {
                    const uint32_t b = b0 + (uint32_t)d;
                    if ((bits >> b) & 1ull)
                        s_klist[(uint32_t)seg * KLS + nks + (uint32_t)__popcll(bits & ((1ull << b) - 1ull))] = (uint16_t)(w * 64 + b);
                }
                nks += (uint32_t)__popcll(bits);
            }
            nkeys = wave_max_all(nks);
        } else {
            for (uint32_t w = 0; w < nkw; ++w) {
                const uint64_t bits = uni64(s_act[row * nkw + w]);
                const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(bits >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)bits, 0u));
                if ((bits >> lane) & 1) s_klist[nkeys + below] = (uint16_t)(w * 64 + lane);
                nkeys += (uint32_t)__popcll(bits);
            }
        }
        if (!PSEG && lane < 2 * KPAD) {                           // chunk padding -> the trash row
            if constexpr (KL32) s_klist32[nkeys + lane] = NK;
            else s_klist[nkeys + lane] = (uint16_t)NK;
        }
        if constexpr (LEAN) nk_lean += nkeys;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        BRC_STAMP(0);
        // p < nkeys + CHUNK: padded list.  The key ids stay in SGPRs with the words they address,
        // so processing a key does not wait on another LDS round trip for its id.
        auto fetch = [&](uint32_t p, uint64_t (&ww)[CHUNK], uint32_t (&kk)[CHUNK]) {
            Unrolled<CHUNK>::run([&](auto ci) {
                constexpr int c = decltype(ci)::value;
                if constexpr (PSEG) {
                    // this instance's own list (past its end: the trash row), one key per segment
                    kk[c] = p + c < nks ? (uint32_t)s_klist[(uint32_t)seg * KLS + p + c] : NK;
                } else {
                    kk[c] = uni32(s_klist[p + c]);
                }
                ww[c] = mycells[(size_t)kk[c] * (CW * 64)];
            });
        };
        // ---- lean path (IPW == 1): k, m (meta), gw (generation) are wave-uniform; wd = this lane's
        // cell word.  Same transitions as process() below, with the per-key work cut down:
        // arrivals are matched against precomputed t - delay, the delay masks are registers
        // (NLR), and only lanes whose cell changes store (exec-masked).
        // send steps are offsets from the epoch: ts = t - ep <= C32_REBASE, and t - delay - ep
        // wraps to a huge value (matching no 7-bit offset) for a delay reaching before the epoch
        const uint32_t ts = t - ep;
        const uint32_t tm0 = ts - dly0, tm1 = ndl > 1 ? ts - dly1 : 0x10000u;   // 0x10000: no 7-bit offset
        // A key-list entry carries the message types that can land on its key this step (TB_*): only
        // those are evaluated.  Keys go in PAIRS: the scalar work (type dispatch, early exits, ring
        // marks) is shared by two keys, while each key's per-lane work is its own -- the CU's scalar
        // unit, not the SIMDs, bounds this loop.  The loop carries little state from key to key:
        // ring rows and q_until are derived from the ring once per step (below), the cell statistics
        // st_cells, st_del and st_bcast are wave-uniform popcounts of ballots, st_arr is per lane.
        // NLR: the ring word lane L < 8 marks for a pair (key word added per key): the row at t + delay
        // of class L & 1, type (L >> 1) & 1; mk_ov = the senders with a link of that class
        const uint32_t mk_row = ((t + ((lane & 1) ? dly1 : dly0)) & (RS - 1)) * AT * nkw + ((lane >> 1) & 1) * nkw;
        // senders whose message of one type, sent at offset tx, lands on this receiver now
        auto count = [&](uint32_t tx) -> uint32_t {
            if constexpr (NLR != 0) {
                // for an honest receiver the delay classes partition the real senders (RL1 = real &
                // ~RL0; with one delay tm1 matches nothing): ONE popcount of a bitfield merge
                const uint64_t b0 = __ballot(tx == tm0), b1 = __ballot(tx == tm1);
                return popc(b1 ^ ((b0 ^ b1) & RL0));
            } else {
                const uint32_t dx = ts - tx;                     // C32_OLD / C32_NEVER: no delay
                uint32_t c = 0;
                Unrolled<DM>::run([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    if ((uint32_t)j < ndl) {
                        const uint64_t b = __ballot(dx == ((dlist >> (4 * j)) & 15u) + 1u);
                        if (b) c += popc(b & s_L[j * 64 + lane]);
                    }
                });
                return c;
            }
        };
        // mk_a / mk_v (NLR): this lane's ring mark for the pair (LDS word, bit; mk_a = NOKEY: none), issued
        // by the caller after the next chunk's key ids are read, so that read never waits for the mark
        auto process_pair = [&](const uint32_t (&ent)[2], const uint64_t (&m)[2], const uint32_t (&lo)[2],
                                uint32_t (&nw)[2], bool (&wr)[2], uint32_t& mk_a, uint64_t& mk_v) {
            uint32_t k[2], tb[2], tE[2], tR[2], ea[2] = {0u, 0u}, ra[2] = {0u, 0u}, sa[2] = {0u, 0u};
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                k[i] = ent[i] & TB_KEY; tb[i] = (ent[i] >> TB_SH) & 7u;
                // lanes that are not real replicas and Byzantine lanes never update their cells here, so
                // their words keep the fresh row's "never sent" unless an injection sent for them
                tE[i] = (lo[i] >> C32_OE_SH) & 127u; tR[i] = lo[i] >> C32_OR_SH;   // offsets: SENT ECHO / READY
            }
            BRC_KCOUNT(0);
            // a type that cannot land on one key of the pair counts zero there: exact either way.
            // BRC_BRANCHLESS: ECHO and READY are always evaluated (a stage without arrivals is the
            // identity), so a pair is one basic block the scheduler can interleave
            const uint32_t tbu = (tb[0] | tb[1]) | (BRC_BRANCHLESS ? (TB_E | TB_R) : 0u);
            if constexpr (BRC_PERKEY_CNT) {
                // a key's count only where its own entry has that type (the pair's stages still run
                // for both keys: zero arrivals are the identity)
                if (tb[0] & TB_E) ea[0] = count(tE[0]);
                if (tb[1] & TB_E) ea[1] = count(tE[1]);
                if (tb[0] & TB_R) ra[0] = count(tR[0]);
                if (tb[1] & TB_R) ra[1] = count(tR[1]);
            } else {
                if (tbu & TB_E) { ea[0] = count(tE[0]); ea[1] = count(tE[1]); }
                if (tbu & TB_R) { ra[0] = count(tR[0]); ra[1] = count(tR[1]); }
            }
            if (tbu & TB_S) {
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    if (tb[i] & TB_S) {
                        // SEND from the key's origin: lands on d iff delay(origin -> d) == t - t_send, and
                        // the key list holds the key now only for such a delay of the origin's outset
                        // sender, delay and restriction of the SEND: from the key-list entry (KL32) or
                        // the key's metadata (the row is wave-uniform)
                        const uint64_t mi = KL32 ? 0ull : uni64(m[i]);
                        const uint32_t dt = KL32 ? ((ent[i] >> KL_DT_SH) & 15u) + 1u : t - m_tsend(mi);
                        const uint32_t snd = KL32 ? (ent[i] >> KL_SND_SH) & 63u : m_sender(mi);
                        const bool restr = KL32 ? (ent[i] & KL_RESTR) != 0 : (mi & M_RESTRICTED) != 0;
                        bool hit;
                        if constexpr (NLR != 0) {
                            hit = (((RL0 >> snd) & 1) != 0) == (dt == dly0);
                        } else {
                            const uint32_t sj = popc(dset & ((1u << ((dt - 1u) & 31)) - 1u));
                            hit = (s_L[sj * 64 + lane] >> snd) & 1;
                        }
                        uint64_t hm = __ballot(hit) & hon_mask;
                        if (restr) hm &= __ballot((gp(P.kdst)[inst * NK + k[i]] >> d) & 1ull);
                        sa[i] = lane_in(hm) ? 1u : 0u;
                    }
                }
            }
            uint64_t ob[2];
            uint32_t arr2 = 0;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const uint32_t arr = ea[i] + ra[i] + sa[i];
                const uint64_t hb = __ballot(arr != 0) & hon_mask;   // receivers with arrivals
                arr2 += arr;
                st_cells += popc(hb);
                // a delivered cell ignores everything (core/brbroadcast.py:74): only open cells change
                ob[i] = hb & ~__ballot((lo[i] & F_DEL) != 0);
            }
            st_arr += arr2;                                      // non-honest lanes are dropped at the end
            if (!BRC_NOEARLY && !(ob[0] | ob[1])) return;       // no open cell receives anything now
            BRC_KCOUNT(3);
            // Per-lane work below is branch-free integer arithmetic on 0/1 flags; a stage runs only
            // when its message type can land (a stage without arrivals is the identity).
            auto ge = [](uint32_t a, uint32_t b) -> uint32_t { return ((a - b) >> 31) ^ 1u; };   // a >= b (< 2^31)
            uint32_t fl[2], ec[2], rc[2], es[2] = {0u, 0u}, rs[2] = {0u, 0u}, dl[2] = {0u, 0u};
            bool opn[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                opn[i] = lane_in(ob[i]);
                fl[i] = lo[i] & 31u; ec[i] = (lo[i] >> C32_EC_SH) & 63u; rc[i] = (lo[i] >> C32_RC_SH) & 63u;
            }
            constexpr bool PK = BRC_PK && !BEB;
            uint32_t FL = 0, EC = 0, RC = 0;     // PK: key 0 in bits 0-15, key 1 in bits 16-31
            if constexpr (PK) {
                // the same transitions as the per-key code below (brb_cell_update / _spec), both keys at once
                const uint32_t P0 = (lo[0] & 0xFFFFu) | (lo[1] << 16);              // flags + |E|
                const uint32_t P1 = ((lo[0] >> 8) & 0xFFFFu) | ((lo[1] >> 8) << 16); // |R| at bits 3-8
                FL = P0 & 0x001F001Fu;
                EC = (P0 >> C32_EC_SH) & 0x003F003Fu;
                RC = (P1 >> (C32_RC_SH - 8)) & 0x003F003Fu;
                const uint32_t ONM = (opn[0] ? 0xFFFFu : 0u) | (opn[1] ? 0xFFFF0000u : 0u), ON = ONM & 0x10001u;
                const uint32_t SA = (sa[0] | (sa[1] << 16)) & ONM;
                const uint32_t E = (ea[0] | (ea[1] << 16)) & ONM, R = (ra[0] | (ra[1] << 16)) & ONM;
                // x != 0 per half for halves <= 128 (min(x, 1) is split per half by the compiler)
                auto nz = [](uint32_t x) -> uint32_t { return ((x + 0x007F007Fu) >> 7) & 0x10001u; };
                uint32_t ES = 0, RS = 0, DL = 0;
                if constexpr (SPEC) {
                    if (tbu & TB_S) { ES = SA & ~(FL >> 3) & 0x10001u; FL |= ES << 3; }        // !F_ES
                    if (tbu & (TB_E | TB_R)) {
                        EC = pk_add(EC, E);
                        RC = pk_add(RC, R);
                        RS = ON & ~(FL >> 4) & (pk_ge(EC, pk2(T_echo)) | pk_ge(RC, pk2(T_amp)));  // !F_RS
                        FL |= RS << 4;
                        DL = ON & pk_ge(RC, pk2(T_del));
                        FL |= DL << 2;
                    }
                } else {
                    if (tbu & TB_S) {                                                   // :76-82
                        const uint32_t est = SA & ~FL & 0x10001u;                       // SEND, no ECHO entry
                        ES = est & ~(FL >> 3);                                          // not sent already
                        FL |= est | (est << 3);                                         // F_EEX | F_ES
                    }
                    if (tbu & TB_E) {                                                   // :84-98
                        const uint32_t eon = nz(E);
                        const uint32_t chk = nz(E + (FL & 0x10001u) - eon);             // a checked ECHO (:87-89)
                        FL |= eon;
                        EC = pk_add(EC, E);
                        const uint32_t r1 = eon & chk & pk_ge(EC, pk2(T_echo)) & (~FL >> 1) & 0x10001u;  // !F_REX (:95)
                        RS = r1 & ~(FL >> 4);
                        FL |= (r1 << 1) | (r1 << 4);
                    }
                    if (tbu & TB_R) {                                                   // :100-119
                        const uint32_t ron = nz(R);
                        const uint32_t rexm = pk_sub(0u, (FL >> 1) & 0x10001u);        // 0xFFFF per half iff F_REX
                        const uint32_t rlo = pk_add(pk_sub(RC, 0x10001u) & rexm, 0x20002u), rhi = pk_add(R, RC & rexm);
                        FL |= ron << 1;
                        RC = pk_add(RC, R);
                        const uint32_t any = ron & pk_ge(rhi, rlo);
                        const uint32_t alo = pk_max(rlo, pk2(T_amp)), ahi = pk_min(rhi, pk2(T_del - 1u));
                        const uint32_t r2 = any & ~FL & ~(FL >> 4) & pk_ge(ahi, alo) & 0x10001u;   // !F_EEX, !F_RS
                        FL |= r2 << 4;
                        DL = any & pk_ge(rhi, pk2(T_del));
                        FL |= DL << 2;
                        RS |= r2;
                    }
                }
                es[0] = ES & 1u; es[1] = ES >> 16;
                rs[0] = RS & 1u; rs[1] = RS >> 16;
                dl[0] = DL & 1u; dl[1] = DL >> 16;
            } else if constexpr (BEB) {
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    dl[i] = (opn[i] && sa[i]) ? 1u : 0u;         // brb_cell_update_beb
                    fl[i] |= dl[i] << 2;
                }
            } else if constexpr (SPEC) {
                // brb_cell_update_spec: ECHO on the first SEND, one READY (echo quorum or f+1 READYs),
                // DELIVER at 2f+1 READYs; only a growing set can newly pass a threshold
                if (tbu & TB_S) {
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        es[i] = (opn[i] ? sa[i] : 0u) & ~(fl[i] >> 3) & 1u;   // !F_ES
                        fl[i] |= es[i] << 3;
                    }
                }
                if (tbu & (TB_E | TB_R)) {
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        ec[i] += opn[i] ? ea[i] : 0u;
                        rc[i] += opn[i] ? ra[i] : 0u;
                        rs[i] = (opn[i] ? 1u : 0u) & ~(fl[i] >> 4) & (ge(ec[i], T_echo) | ge(rc[i], T_amp));   // !F_RS
                        fl[i] |= rs[i] << 4;
                        dl[i] = (opn[i] ? 1u : 0u) & ge(rc[i], T_del);
                        fl[i] |= dl[i] << 2;
                    }
                }
            } else {
                // brb_cell_update in integer form.  F_EEX = bit 0, F_REX = 1, F_DEL = 2, F_ES = 3, F_RS = 4.
                if (tbu & TB_S) {                                                // :76-82
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const uint32_t est = (opn[i] ? sa[i] : 0u) & ~fl[i] & 1u;  // SEND, no ECHO entry
                        es[i] = est & ~(fl[i] >> 3);                             // not sent already (user ECHO)
                        fl[i] |= est | (est << 3);                               // F_EEX | F_ES
                    }
                }
                if (tbu & TB_E) {                                                // :84-98
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const uint32_t e = opn[i] ? ea[i] : 0u;
                        const uint32_t eon = min(e, 1u);
                        const uint32_t chk = min(e + (fl[i] & 1u) - eon, 1u);    // a checked ECHO (:87-89)
                        fl[i] |= eon;                                            // F_EEX
                        ec[i] += e;
                        const uint32_t r1 = eon & chk & ge(ec[i], T_echo) & (~fl[i] >> 1) & 1u;   // !F_REX (:95)
                        rs[i] = r1 & ~(fl[i] >> 4);                              // not sent already (user READY)
                        fl[i] |= (r1 << 1) | (r1 << 4);                          // F_REX | F_RS
                    }
                }
                if (tbu & TB_R) {                                                // :100-119
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const uint32_t r = opn[i] ? ra[i] : 0u;
                        const uint32_t ron = min(r, 1u);
                        const uint32_t rexm = 0u - ((fl[i] >> 1) & 1u);          // all ones iff F_REX
                        const uint32_t rlo = 2u + ((rc[i] - 1u) & rexm), rhi = r + (rc[i] & rexm);   // checked sizes
                        fl[i] |= ron << 1;                                       // F_REX
                        rc[i] += r;
                        const uint32_t any = ron & ge(rhi, rlo);
                        const uint32_t alo = max(rlo, T_amp), ahi = min(rhi, T_del - 1u);
                        const uint32_t r2 = any & ~fl[i] & ~(fl[i] >> 4) & ge(ahi, alo) & 1u;   // !F_EEX, !F_RS
                        fl[i] |= r2 << 4;                                        // F_RS
                        dl[i] = any & ge(rhi, T_del);
                        fl[i] |= dl[i] << 2;                                     // F_DEL
                        rs[i] |= r2;
                    }
                }
            }
            uint64_t eb[2], rb[2], db[2];
            // PK: flags and |E| of both keys, |R| apart (its field crosses bit 16)
            const uint32_t PL = FL | (pk_min(EC, 0x003F003Fu) << C32_EC_SH), PR = pk_min(RC, 0x003F003Fu);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                // new word for open cells; the others keep theirs.  A count reaches 64 only when every
                // sender's message of that type has arrived, so none is compared again: the stored
                // counts saturate at 63 without changing any later transition
                const uint32_t sends = ((es[i] ? ts : tE[i]) << C32_OE_SH) | ((rs[i] ? ts : tR[i]) << C32_OR_SH);
                if constexpr (PK)
                    nw[i] = ((PL >> (16 * i)) & 0xFFFFu) | (((PR >> (16 * i)) & 0xFFFFu) << C32_RC_SH) | sends;
                else
                    nw[i] = fl[i] | (min(ec[i], 63u) << C32_EC_SH) | (min(rc[i], 63u) << C32_RC_SH) | sends;
                wr[i] = opn[i];
                eb[i] = __ballot(es[i] != 0); rb[i] = __ballot(rs[i] != 0); db[i] = __ballot(dl[i] != 0);
            }
            st_bcast += popc(eb[0]) + popc(rb[0]) + popc(eb[1]) + popc(rb[1]);
            st_del += popc(db[0]) + popc(db[1]);
            if (db[0] | db[1]) {
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    if (db[i]) {
                        if constexpr (LEAN && (DBG || BRC_DACC)) {
                            // keys come in ascending slot order: a word is complete when the next word starts
                            const uint32_t wk = k[i] >> 6;
                            if (wk != dcur) {
                                if (dcur != NOKEY) flush_dacc(dcur, dacc);
                                dacc = 0; dcur = wk;
                            }
                            dacc |= (uint64_t)dl[i] << (k[i] & 63);
                        } else {
                            atomicOr((unsigned long long*)&s_dbits[(k[i] >> 6) * 64 + lane], (uint64_t)dl[i] << (k[i] & 63));
                        }
                    }
                }
            }
            if (EV) {
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const uint64_t mi = uni64(m[i]);
                    const uint32_t kp = (k[i] >> qsh), s = m_s1(mi) - 1u;
                    if (es[i]) log_ev(BRC_EV_SEND, d, BRC_ECHO, kp, s, m_value(mi));
                    if (rs[i]) log_ev(BRC_EV_SEND, d, BRC_READY, kp, s, m_value(mi));
                    if (dl[i]) log_ev(BRC_EV_DELIVER, d, 0, kp, s, m_value(mi));
                }
            }
            // sends: typed ring marks at t + every delay some sending lane has (the step's ring rows,
            // q_until and the keys' pending arrivals follow from the ring itself)
            if (eb[0] | rb[0] | eb[1] | rb[1]) {
                if constexpr (NLR != 0) {
                    // one LDS op for the pair: lane L < 8 marks key L >> 2, type (L >> 1) & 1 (ECHO,
                    // READY), delay class L & 1 -- iff a sender of that type has a link of that class
                    const bool lk1 = lane_in(0xF0F0F0F0F0F0F0F0ull), lty = lane_in(0xCCCCCCCCCCCCCCCCull);
                    const uint64_t sm = (lk1 ? (lty ? rb[1] : eb[1]) : (lty ? rb[0] : eb[0])) & mk_ov;
                    const uint32_t kx = lk1 ? k[1] : k[0];
                    if (lane < 8 && sm != 0) { mk_a = mk_row + (kx >> 6); mk_v = 1ull << (kx & 63); }
                } else {
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        uint32_t osE = 0, osR = 0;
                        for (uint32_t ds = dset; ds; ds &= ds - 1) {
                            const uint32_t j = (uint32_t)__ffs(ds) - 1;
                            const uint64_t ov = readlane64(outv, (int)j);
                            if (eb[i] & ov) osE |= 1u << j;
                            if (rb[i] & ov) osR |= 1u << j;
                        }
                        const uint64_t kbit = 1ull << (k[i] & 63);
                        for (uint32_t x = osE | (osR << 16); x; x &= x - 1) {
                            const uint32_t b = (uint32_t)__ffs(x) - 1;
                            const uint32_t r = (t + (b & 15u) + 1u) & (RS - 1);
                            if (lane == 0) atomicOr((unsigned long long*)&s_act[(r * AT + (b >> 4)) * nkw + (k[i] >> 6)], kbit);
                        }
                    }
                }
            }
        };
        // xsa: this lane's extra-SEND arrivals of key k (the pre-pass below; 0 in the key loop)
        // always inlined: an outlined call (the event-log instantiations' choice) keeps every variable it
        // captures by reference in scratch memory
        auto process = [&](const uint32_t k, const uint64_t wd, const uint32_t xsa) __attribute__((always_inline)) {
            // both LDS reads issue before either is waited on (k == NK, the trash row: junk, unused)
            const uint64_t m_raw = s_meta[mbase + k];
            const uint32_t gw_raw = s_gen[mbase + k];
            uint64_t m = m_raw;
            uint32_t gw = gw_raw;
            if (IPW == 1) { m = uni64(m); gw = uni32(gw); }      // one instance per wave
            const uint32_t gen = gw & GEN_MASK;
            // the slot holds a key (not one the extra-SEND pre-pass processed this step)
            const bool kl = k < NK && m_s1(m) != 0 && (LEAN || !(gw & GEN16_XDONE));
            const bool live = kl && running;
            const bool cur = kl && real_run && (((uint32_t)wd >> 19) & GEN_MASK) == gen;
            const uint64_t word = cur ? wd : TIMES_NEVER;
            const uint32_t tE = (uint32_t)(word >> 32) & 0xFFFF, tR = (uint32_t)(word >> 48);
            const uint32_t dE = t - tE, dR = t - tR;             // steps since this lane sent
            uint32_t ea = 0, ra = 0;
            Ring16 ringE = {0, 0}, ringR = {0, 0};               // CONN: this lane's send counts
            if constexpr (CONN) {
                ringE = {mycells[(size_t)k * (CW * 64) + 64], mycells[(size_t)k * (CW * 64) + 128]};
                ringR = {mycells[(size_t)k * (CW * 64) + 192], mycells[(size_t)k * (CW * 64) + 256]};
                uint32_t j = 0;
                for (uint32_t ds = dset; ds; ds &= ds - 1, ++j) {
                    const uint32_t dly = (uint32_t)__ffs(ds);
                    const uint32_t ce = ring_count(ringE, tE, t - dly), cr = ring_count(ringR, tR, t - dly);
                    if (__ballot((ce | cr) != 0)) {               // arrivals = sum over senders of counts:
                        const T Lj = s_L[j * 64 + lane];         // one ballot per count bit
#pragma unroll
                        for (int b = 0; b < 8; ++b) {
                            const uint64_t be = __ballot((ce >> b) & 1u), br = __ballot((cr >> b) & 1u);
                            ea += popc((T)(be >> segbase) & Lj) << b;
                            ra += popc((T)(br >> segbase) & Lj) << b;
                        }
                    }
                }
            } else {
                // the j-th delay present in the wave, precomputed (dlist), unrolled, and no test for
                // empty ballots: a branch per delay cost more than the popcounts it skipped (r1 A/B)
                Unrolled<DM>::run([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    if ((uint32_t)j < ndl) {
                        const uint32_t dly = (dlist >> (4 * j)) & 15u;
                        const uint64_t be = __ballot(dE == dly + 1u), br = __ballot(dR == dly + 1u);
                        const T Lj = Lmask(j);
                        ea += popc((T)(be >> segbase) & Lj);
                        ra += popc((T)(br >> segbase) & Lj);
                    }
                });
            }
            // SEND from the key's origin: arrives at t_send + delay(origin -> d)
            bool s_arr = false;
            const uint32_t dt = t - m_tsend(m);
            const uint32_t bit = 1u << ((dt - 1u) & 31);
            const bool s_win = kl && dt - 1u < D && (dset & bit) != 0;     // uniform if IPW == 1
            if (IPW == 1 ? s_win : __any(s_win)) {
                bool hit = (Lmask(popc(dset & (bit - 1u))) >> m_sender(m)) & 1;
                // a restricted SEND lands only on its destinations (kdst); per lane -- the lanes of an item hold
                // different instances, each its own key (and padding lanes, whose slot fields are junk)
                const bool restr = s_win && (gw & GEN16_RESTRICTED) != 0;
                if (IPW == 1 ? restr : __any(restr))
                    if (restr) hit = hit && ((gp(P.kdst)[inst * NK + k] >> d) & 1ull);
                s_arr = s_win && hon_run && hit;
            }
            const uint32_t sa = (LEAN ? 0u : xsa) + (s_arr ? 1u : 0u);   // SEND arrivals (extra SENDs: several)
            s_arr = sa != 0;
            const bool has = kl && hon_run && (s_arr || ea || ra);
            st_loads += (kl && real_run) ? 1u : 0u;
            uint32_t fl = (uint32_t)word & 31, ec = (uint32_t)(word >> 5) & 127, rc = (uint32_t)(word >> 12) & 127;
            bool es, rs, dl;
            uint32_t n_ready = 0;                                // CONN: READY broadcasts this step
            bool first_ready = false;
            const bool had_es = (fl & F_ES) != 0;                // a user-issued ECHO was logged already
            if constexpr (CONN) {
                brb_cell_update_conn(fl, ec, rc, s_arr, has ? ea : 0u, has ? ra : 0u, T_echo, T_amp, T_del, es, n_ready, dl);
                rs = n_ready != 0;
                first_ready = rs && !(fl & F_RS);
                fl |= rs ? F_RS : 0u;
                ec = min(ec, 127u); rc = min(rc, 127u);
                if (es) ringE = ring_put(ringE, tE, t, 1u);
                if (rs) ringR = ring_put(ringR, tR, t, n_ready);
                if (es) {
                    mycells[(size_t)k * (CW * 64) + 64] = ringE.lo;
                    mycells[(size_t)k * (CW * 64) + 128] = ringE.hi;
                }
                if (rs) {
                    mycells[(size_t)k * (CW * 64) + 192] = ringR.lo;
                    mycells[(size_t)k * (CW * 64) + 256] = ringR.hi;
                }
            } else if constexpr (BEB) brb_cell_update_beb(fl, s_arr, es, rs, dl);
            else if constexpr (SPEC) brb_cell_update_spec(fl, ec, rc, s_arr, has ? ea : 0u, has ? ra : 0u, T_echo, T_amp, T_del, es, rs, dl);
            else brb_cell_update(fl, ec, rc, s_arr, has ? ea : 0u, has ? ra : 0u, T_echo, T_amp, T_del, es, rs, dl);
            {
                const uint32_t tEn = es ? t : tE, tRn = rs ? t : tR;
                const uint64_t nw = (uint64_t)fl | ((uint64_t)ec << 5) | ((uint64_t)rc << 12) |
                                    ((uint64_t)gen << 19) | ((uint64_t)tEn << 32) | ((uint64_t)tRn << 48);
#if BRC_NL_MSTORE
                if (has) mycells[(size_t)k * (CW * 64)] = nw;   // only cells with arrivals change
#else
                mycells[(size_t)k * (CW * 64)] = has ? nw : wd;  // whole-wave store (unchanged words back)
#endif
            }
            st_arr += has ? ea + ra + sa : 0u;
            st_cells += has ? 1u : 0u;
            st_msgs += ((es ? 1u : 0u) + (CONN ? n_ready : (rs ? 1u : 0u))) * n;
            st_del += dl ? 1u : 0u;
            if (__ballot(dl))
                atomicOr((unsigned long long*)&s_dbits[(k >> 6) * 64 + lane], dl ? (1ull << (k & 63)) : 0ull);
            if (EV) {
                const uint32_t kp = (k >> qsh), s = m_s1(m) - 1u;
                if (es) log_ev(had_es ? BRC_EV_COPY : BRC_EV_SEND, d, BRC_ECHO, kp, s, m_value(m));
                if constexpr (CONN) {
                    // connection peers: every READY broadcast travels; the first of the key is a SEND
                    // event, the :119 re-fires after it COPY events (one per broadcast)
                    for (uint32_t c = 0; c < n_ready; ++c)
                        log_ev((c == 0 && first_ready) ? BRC_EV_SEND : BRC_EV_COPY, d, BRC_READY, kp, s, m_value(m));
                } else if (rs) {
                    log_ev(BRC_EV_SEND, d, BRC_READY, kp, s, m_value(m));
                }
                if (dl) log_ev(BRC_EV_DELIVER, d, 0, kp, s, m_value(m));
            }
            // sends: ring marks at t + every delay some sending lane has; t_quiet of the key
            const uint64_t sb = __ballot(es || rs);
            if (sb) {
                uint32_t os = 0, oss = 0;
                for (uint32_t ds = dset; ds; ds &= ds - 1) {
                    const uint32_t i = (uint32_t)__ffs(ds) - 1;
                    const uint64_t x = sb & readlane64(outv, (int)i);
                    if (x) os |= 1u << i;
                    if (IPW > 1 && ((x & segbits) != 0)) oss |= 1u << i;
                }
                if (IPW == 1) oss = os;
                if constexpr (PSEG) {
                    // the key is this segment's (keys differ across segments): its own senders' delays
                    for (uint32_t x = oss; x; x &= x - 1) {
                        const uint32_t r = (t + (uint32_t)__ffs(x)) & (RS - 1);
                        if (d == 0) atomicOr((unsigned long long*)&s_act[(r * AT + (uint32_t)seg) * nkw + (k >> 6)], 1ull << (k & 63));
                        lane_rows |= 1u << r;
                    }
                } else {
                    for (uint32_t x = os; x; x &= x - 1) {
                        const uint32_t r = (t + (uint32_t)__ffs(x)) & (RS - 1);
                        if (lane == 0) atomicOr((unsigned long long*)&s_act[r * nkw + (k >> 6)], 1ull << (k & 63));
                        any_rows |= 1u << r;
                    }
                }
                const uint32_t myq = oss ? t + hibit(oss) : 0u;
                if (live && myq) {
                    if ((IPW == 1 || d == 0) && myq > m_tquiet(m)) s_meta[mbase + k] = m_with_tquiet(m, myq);
                    q_until = max(q_until, myq);
                }
            }
        };
        // lean key pipeline registers (LC key slots in flight: lean SPEC keeps 4, which needs no spill at 4 waves/SIMD)
        constexpr int LC = SPEC ? BRC_LCHUNK_SPEC : LCHUNK;
        uint32_t w[LC];                  // lean: compact cell words in flight
        uint32_t kk[LC];
        if constexpr (LEAN) {
            // software pipeline, unrolled by LC so the in-flight cell words never move between
            // registers: slot c holds key p + c; right after it is processed, slot c loads key
            // p + c + LC, so LC cell loads stay in flight.  The chunk's key metadata is read
            // at its start (a key's t_quiet update touches only its own slot, so reading ahead is
            // exact).  Slots past the list load the trash row NK and are not processed.
            auto kid = [&](uint32_t p) { return uni32(KL32 ? s_klist32[p] : (uint32_t)s_klist[p]); };
            auto cell = [&](uint32_t e) { return cld(e & TB_KEY); };
            // prologue loads pinned in slot order (the scheduler would otherwise reorder them and
            // the compiler's wait for slot 0 would then drain every load)
            Unrolled<LC>::run([&](auto ci) {
                constexpr int c = decltype(ci)::value;
                // OOBST: the loop's order (two stores, then two loads, per pair) from the start, with
                // stores that write nothing, so the loop entry's count of outstanding ops is the loop's own
                if constexpr (BRC_OOBST && (c % 2 == 0)) {
                    __builtin_amdgcn_raw_buffer_store_b32(0u, crs, 0x80000000u, 0u, 0);
                    __builtin_amdgcn_raw_buffer_store_b32(0u, crs, 0x80000000u, 256u, 0);
                }
                kk[c] = kid(c);
                w[c] = cell(kk[c]);
                __builtin_amdgcn_sched_barrier(0);
            });
            for (uint32_t p = 0; p < nkeys; p += LC) {
                uint64_t mm[LC];
                Unrolled<LC>::run([&](auto ci) {
                    constexpr int c = decltype(ci)::value;
                    // KL32: only the event log needs the key's metadata (phase index and value)
                    mm[c] = (EV || !KL32) ? s_meta[kk[c] & TB_KEY] : 0ull;
                });
                // the refill entries p + LC .. p + 2 LC - 1 in 8-B reads (p % 4 == 0 and s_klist
                // is 8-B aligned), so a refill never waits on an LDS round trip of its own
                static_assert(LC == 4 || LC == 8 || LC == 16, "four, eight or sixteen key-list entries per refill");
                uint64_t knext[LC / 2];           // entries 2i | 2i + 1 << 32
                Unrolled<LC / 4>::run([&](auto qi) {
                    constexpr int q = decltype(qi)::value;
                    if constexpr (KL32) {
                        knext[2 * q] = *(const uint64_t*)&s_klist32[p + LC + 4 * q];
                        knext[2 * q + 1] = *(const uint64_t*)&s_klist32[p + LC + 4 * q + 2];
                    } else {
                        const uint64_t k4 = *(const uint64_t*)&s_klist[p + LC + 4 * q];
                        knext[2 * q] = (k4 & 0xFFFFull) | ((k4 & 0xFFFF0000ull) << 16);
                        knext[2 * q + 1] = ((k4 >> 32) & 0xFFFFull) | ((k4 >> 48) << 32);
                    }
                });
                Unrolled<LC / 2>::run([&](auto ci) {
                    constexpr int c = 2 * decltype(ci)::value;
                    // a pair past the list is skipped; the second key of a pair at the list's end is
                    // the padding entry (the trash row, no message type): it changes nothing
                    const uint32_t ent[2] = {kk[c], kk[c + 1]};
                    const uint64_t mp[2] = {mm[c], mm[c + 1]};
                    const uint32_t lo[2] = {w[c], w[c + 1]};
                    uint32_t nw[2] = {w[c], w[c + 1]};
                    bool wr[2] = {false, false};
                    uint32_t mk_a = NOKEY;
                    uint64_t mk_v = 0;
                    if (p + c < nkeys) process_pair(ent, mp, lo, nw, wr, mk_a, mk_v);
                    cst_if(kk[c] & TB_KEY, nw[0], wr[0]);
                    cst_if(kk[c + 1] & TB_KEY, nw[1], wr[1]);
                    // refill (none after the last chunk: no load is left in flight past the loop, so the
                    // code after it neither waits for one nor keeps its registers)
                    if constexpr (BRC_OOBST) {
                        // unconditional too (a skipped load is the same uncertainty as a skipped store):
                        // after the last chunk the loads fall out of range, return 0 and touch no memory
                        const uint32_t rv = (p + LC < nkeys) ? lv4 : 0x80000000u;
                        kk[c] = uni32((uint32_t)knext[c / 2]);
                        w[c] = __builtin_amdgcn_raw_buffer_load_b32(crs, rv, (kk[c] & TB_KEY) * 256u, 0);
                        kk[c + 1] = uni32((uint32_t)(knext[c / 2] >> 32));
                        w[c + 1] = __builtin_amdgcn_raw_buffer_load_b32(crs, rv, (kk[c + 1] & TB_KEY) * 256u, 0);
                    } else if (p + LC < nkeys) {
                        kk[c] = uni32((uint32_t)knext[c / 2]);
                        w[c] = cell(kk[c]);
                        kk[c + 1] = uni32((uint32_t)(knext[c / 2] >> 32));
                        w[c + 1] = cell(kk[c + 1]);
                    }
                    if (mk_a != NOKEY) atomicOr((unsigned long long*)&s_act[mk_a], mk_v);
                });
            }
        } else {
            // Extra-SEND pre-pass (records of keys SENT again, rare): a key with extra SEND arrivals
            // now is processed here, whole (its SENDs ahead of its ECHO / READY, the canonical
            // order), with the arrival count summed over its records; the key loop then skips it
            // (GEN16_XDONE, cleared after the loop).  No code of this is in the key loop's process().
            auto xs_active = [&](uint64_t w0) -> bool {
                const uint32_t dt2 = t - ((uint32_t)(w0 >> 16) & 0xFFFFu);
                return dt2 - 1u < D && ((dset >> ((dt2 - 1u) & 31)) & 1u);
            };
            if (xs_n) {
                for (uint32_t i = 0; i < xs_n; ++i) {
                    const uint64_t w0 = xs_ld(3 * i);
                    const uint32_t k = (uint32_t)(w0 & 0xFFFFu);
                    if (!xs_active(w0)) continue;
                    bool seen = false;                   // an earlier active record of this slot
                    for (uint32_t j = 0; j < i; ++j) {
                        const uint64_t v0 = xs_ld(3 * j);
                        seen = seen || ((uint32_t)(v0 & 0xFFFFu) == k && xs_active(v0));
                    }
                    if (seen) continue;
                    uint32_t xsa = 0;
                    for (uint32_t j = i; j < xs_n; ++j) {
                        const uint64_t v0 = xs_ld(3 * j);
                        if ((uint32_t)(v0 & 0xFFFFu) != k || !xs_active(v0)) continue;
                        const uint32_t dt2 = t - ((uint32_t)(v0 >> 16) & 0xFFFFu), b2 = 1u << (dt2 - 1u);
                        const uint64_t snd = xs_ld(3 * j + 1), dst2 = xs_ld(3 * j + 2);
                        const bool mine2 = hon_run && seg == (int)((v0 >> 40) & 0xFF) && ((dst2 >> d) & 1ull);
                        xsa += mine2 ? popc((T)(Lmask(popc(dset & (b2 - 1u))) & (T)snd)) : 0u;
                    }
                    process(k, mycells[(size_t)k * (CW * 64)], xsa);
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    if (d == 0) s_gen[mbase + k] |= GEN16_XDONE;
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                }
            }
            uint64_t wA[CHUNK];
            uint32_t kA[CHUNK];
            fetch(0, wA, kA);
            for (uint32_t p = 0; p < nkeys; p += CHUNK) {
                uint64_t wB[CHUNK];
                uint32_t kB[CHUNK];
                fetch(p + CHUNK, wB, kB);
                Unrolled<CHUNK>::run([&](auto ci) {
                    constexpr int c = decltype(ci)::value;
                    process(kA[c], wA[c], 0u);                   // padding slots: the trash row
                });
                Unrolled<CHUNK>::run([&](auto ci) {
                    constexpr int c = decltype(ci)::value;
                    wA[c] = wB[c];
                    kA[c] = kB[c];
                });
            }
            if (xs_n) {
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                for (uint32_t i = 0; i < xs_n; ++i) {
                    const uint64_t w0 = xs_ld(3 * i);
                    if (xs_active(w0) && d == 0) s_gen[mbase + (uint32_t)(w0 & 0xFFFFu)] &= (uint16_t)~GEN16_XDONE;
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            }
        }
        BRC_STAMP(1);
        if constexpr (LEAN) {
            if (dcur != NOKEY) flush_dacc(dcur, dacc);
            // ring rows the key loop marked (every row but the current one, which it consumes), and
            // q_until = the furthest of them: the same values per-key tracking would have produced
            uint32_t rb = 0;
            {
                const uint32_t rsh = (uint32_t)__ffs(AT * nkw) - 1u;      // AT * nkw is a power of two
                for (uint32_t i = lane; i < RS * AT * nkw; i += 64)
                    if (s_act[i] != 0) rb |= 1u << (i >> rsh);
                rb = wave_or_all(rb) & ~(1u << row);
            }
            if (rb) {
                any_rows |= rb;
                const uint32_t rel = (row ? ((rb >> row) | (rb << (RS - row))) : rb) & (RS == 32 ? ~0u : ((1u << RS) - 1u));
                q_until = max(q_until, t + hibit(rel) - 1u);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        BRC_STAMP(7);

        // ================= consensus: this step's deliveries in canonical (kp, s) order; SENDs deferred
        defer_sends = true;
        BRC_STAMP(5);
        {
            const uint64_t gm0 = (Q >= 64) ? ~0ull : ((1ull << Q) - 1);
            const bool cons = P.protocol == BRC_PROTO_CONSENSUS && honest && running;
            if (!LEAN && !SPEC && Q >= 64) {
                // key windows of 64 / 128 (the reference protocol's many-round runs; brc_create
                // keeps the lean and SPEC kernels at <= 32): a key prefix spans Q / 64 whole words; its
                // deliveries of one step go one at a time, smallest phase index first (canonical (kp, s))
                const uint32_t wpg = Q > 64 ? Q / 64 : 1u;
#pragma unroll 1
                for (uint32_t w = 0; w < nkw; w += wpg) {
                    uint64_t gb[2] = {0ull, 0ull};
                    for (uint32_t j = 0; j < wpg; ++j) {
                        gb[j] = cons ? s_dbits[(w + j) * 64 + lane] : 0ull;
                        s_dbits[(w + j) * 64 + lane] = 0;
                    }
                    while (gb[0] | gb[1]) {
                        uint32_t bs = 0xFFFFFFFFu, bk = 0;
                        for (uint32_t j = 0; j < wpg; ++j)
                            for (uint64_t x = gb[j]; x; x &= x - 1) {
                                const uint32_t kk = (w + j) * 64 + (uint32_t)__ffsll((unsigned long long)x) - 1u;
                                const uint32_t s1 = m_s1(s_meta[mbase + kk]);
                                if (s1 < bs) { bs = s1; bk = kk; }
                            }
                        gb[(bk >> 6) - w] &= ~(1ull << (bk & 63));
                        cons_deliver(bk);
                    }
                }
            } else {
            // the deliveries of key word w (bits: this lane's), in slot order
            auto cons_word = [&](const uint32_t w, uint64_t bits) {
                if (!cons) bits = 0;
                if constexpr (LEAN && SPEC) {
                    // SPEC (one key variant per origin): when every lane with deliveries in this word is
                    // at the same phase index c0, the slots' phase indices classify against c0 with
                    // ballots (lane = slot). A lane whose current-phase deliveries cannot complete the
                    // phase (spec_advance acts only at n - f origins) adds the word's deliveries to its
                    // phase-slot counts at once; the others go one by one.
                    const uint64_t hb = __ballot(bits != 0);
                    if (!seen_on && hb) {
                        const uint32_t cur = round ? 2 * (round - 1) + (phase - 1) : 0u;
                        const uint64_t sm = s_meta[w * 64 + lane];
                        const uint32_t ss = m_s1(sm) - 1u, sv = m_value(sm) & 3u;   // slot w*64+lane
                        const uint64_t v1 = __ballot(sv == 1), v2 = __ballot(sv == 2);
                        // one pass per distinct phase index c0 among the delivering lanes (one, or two at a
                        // phase boundary; BRC_SPEC_MULTI = 0: only words whose lanes share one index)
                        uint64_t pend = hb;
                        while (pend) {
                            const uint32_t c0 = uni32((uint32_t)__builtin_amdgcn_readlane((int)cur, __ffsll((unsigned long long)pend) - 1));
                            const bool at = bits != 0 && cur == c0;
                            const uint64_t bat = __ballot(at);
                            if (!BRC_SPEC_MULTI && bat != pend) break;
                            pend &= ~bat;
                            const uint64_t inw = __ballot(ss >= c0 && ss - c0 < Q), atc = __ballot(ss == c0);
                            const uint64_t past = __ballot(ss != 0xFFFFFFFFu && ss >= c0 && ss - c0 >= Q);
                            const uint32_t ncur = (uint32_t)__popcll(bits & atc);
                            const uint32_t qc = c0 & Qm;
                            if (at && (round == 0 || (s_cnt[qc * 64 + lane] & 0x3FFu) + ncur < n - P.f)) {
                                if (bits & past) ovf = true;                  // beyond the window (spec_deliver)
                                const uint64_t b = bits & inw;
                                // slots of phase slot q (slot mod Q == q): bit q of every Q-bit group
                                const uint64_t g0 = Q == 2 ? 0x5555555555555555ull : Q == 4 ? 0x1111111111111111ull
                                                                                    : 0x0101010101010101ull;
                                for (uint32_t q = 0; q < Q; ++q) {
                                    const uint64_t bq = b & (g0 << q);
                                    if (bq) atomicAdd(&s_cnt[q * 64 + lane], (uint32_t)__popcll(bq) + ((uint32_t)__popcll(bq & v1) << 10) +
                                                                     ((uint32_t)__popcll(bq & v2) << 20));
                                }
                                bits = 0;
                            }
                        }
                    }
                }
                if constexpr (LEAN && !SPEC) {
                    // A lane whose deliveries in this word can change no phase (fewer than T_cnt - vcount
                    // of them, or not in phase 1 / 2) and hit each key prefix at most once takes them all
                    // at once: the value sets gain the hosts (an origin is Q * NV consecutive slots),
                    // vcount the count, and values new to `order` enter by first slot (= delivery order).
                    // The others (a phase change, or two phases of one key in one step) go one by one.
                    // A phase change inside the word splits it: the prefix (in delivery order) that
                    // completes the phase goes at once, then the phase ends (cons_after), then the rest.
                    if (__ballot(bits != 0)) {
                        const uint32_t sv = m_value(s_meta[w * 64 + lane]) & 3u;     // slot w*64+lane's value
                        const uint64_t vm[4] = {__ballot(sv == 0), __ballot(sv == 1), __ballot(sv == 2), __ballot(sv == 3)};
                        uint32_t nb = (uint32_t)__popcll(bits);
                        const bool oneper = (uint32_t)__popcll(fold_groups(bits, Q)) == nb;
                        // the deliveries of `part` (a subset of this word's, one per key prefix) at once
                        auto bulk = [&](uint64_t part) {
                            const uint32_t G = Q * NV, opw = 64u / G;
                            uint32_t first[4];
#pragma unroll
                            for (int v = 0; v < 4; ++v) {
                                const uint64_t dv = part & vm[v];
                                first[v] = dv ? (uint32_t)__ffsll((unsigned long long)dv) - 1u : 64u;
                                if (dv) s_hm[v * 64 + lane] |= (T)(compress_groups(fold_groups(dv, G), G) << (w * opw));
                                // already inserted? (the field test of cons_deliver_vh)
                                const uint32_t xo = order ^ ((uint32_t)v * 0x55u);
                                if (((~(xo | (xo >> 1)) & 0x55u & ((1u << (2 * nvals)) - 1u)) != 0)) first[v] = 64u;
                            }
                            for (int r = 0; r < 4; ++r) {       // new values, by first delivery
                                uint32_t bv = 0, bp = 64u;
#pragma unroll
                                for (int v = 0; v < 4; ++v) if (first[v] < bp) { bp = first[v]; bv = (uint32_t)v; }
                                if (bp == 64u) break;
                                order |= bv << (2 * nvals); ++nvals;
#pragma unroll
                                for (int v = 0; v < 4; ++v) if ((uint32_t)v == bv) first[v] = 64u;   // static indices
                            }
                        };
                        while (nb && oneper) {
                            if ((phase != 1 && phase != 2) || vcount + nb < P.T_cnt) {
                                bulk(bits);
                                vcount += nb;
                                bits = 0;
                                break;
                            }
                            // the deliveries up to the one that completes the phase: the lowest `need` bits
                            const uint32_t need = vcount >= P.T_cnt ? 1u : P.T_cnt - vcount;
                            uint64_t x = bits;
                            uint32_t kth = need, pos = 0;
#pragma unroll
                            for (uint32_t sh = 32; sh; sh >>= 1) {      // position of the need-th set bit
                                const uint32_t c = (uint32_t)__popcll(x & ((1ull << sh) - 1ull));
                                if (kth > c) { kth -= c; x >>= sh; pos += sh; }
                            }
                            const uint64_t pre = bits & (pos >= 63 ? ~0ull : ((2ull << pos) - 1ull));
                            bulk(pre);
                            vcount += need;
                            bits &= ~pre;
                            nb -= need;
                            cons_after();                                 // :71-106
                        }
                    }
                }
                // one delivery per iteration, ascending slot = ascending (origin, variant); the slots
                // of one key prefix hold its phase indices mod Q, so when several of them deliver in
                // the same step (rare) the smallest phase index goes first
                while (bits) {
                    uint32_t best = __ffsll((unsigned long long)bits) - 1;
                    const uint64_t grp = bits & (gm0 << (best & ~Qm));
                    if (grp & (grp - 1)) {
                        uint32_t bs = 0xFFFFFFFFu;
                        for (uint64_t x = grp; x; x &= x - 1) {
                            const uint32_t bb = __ffsll((unsigned long long)x) - 1;
                            const uint32_t s1 = m_s1(s_meta[mbase + w * 64 + bb]);
                            if (s1 < bs) { bs = s1; best = bb; }
                        }
                    }
                    bits &= ~(1ull << best);
                    if constexpr (SPEC) spec_deliver(w * 64 + best);
                    else cons_deliver(w * 64 + best);
                }
            };
            if constexpr (DBG) {
                // HBM delivery words (lean SPEC): only the words written this step, their loads issued
                // together (up to 8 at a time) instead of one round trip per word before its pass
                uint32_t wm = dwm;                                  // uniform: the word passes ballot over slots (lanes)
#pragma unroll 1
                while (wm) {
                    uint64_t bv[8];
                    uint64_t wv = 0;                                // word ids, 5 bits each (nkw <= 32)
                    uint32_t nw = 0;
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        bv[i] = 0;
                        if (wm) {
                            const uint32_t w = (uint32_t)__ffs(wm) - 1u;
                            wm &= wm - 1u;
                            bv[i] = gdbits[w * 64];
                            wv |= (uint64_t)w << (5 * i);
                            ++nw;
                        }
                    }
#pragma unroll 1
                    for (uint32_t i = 0; i < nw; ++i) {
                        uint64_t b = bv[0];
#pragma unroll
                        for (int j = 1; j < 8; ++j) b = i == (uint32_t)j ? bv[j] : b;
                        cons_word((uint32_t)(wv >> (5 * i)) & 31u, b);
                    }
                }
            } else {
#pragma unroll 1
                for (uint32_t w = 0; w < nkw; ++w) {
                    const uint64_t bits = s_dbits[w * 64 + lane];
                    s_dbits[w * 64 + lane] = 0;
                    cons_word(w, bits);
                }
            }
            }
        }
        BRC_STAMP(2);
        defer_sends = false;
        flush_sends();                                   // the SENDs the consensus started this step
        flush_clears();                                  // ... and their fresh rows
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        BRC_STAMP(6);

        // ================= actions stamped t
        const bool inj_mine = do_actions();
        any_rows |= wave_or_all(lane_rows);
        lane_rows = 0;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        BRC_STAMP(3);

        // ================= per-instance stop conditions
        q_until = NPAD == 64 ? wave_max_all(q_until) : seg_max<NPAD>(q_until);
        const uint64_t b_act = __ballot(st_cells != cells0 || inj_mine) & segbits;
        const uint64_t b_ovf = __ballot(ovf) & segbits;
        const uint64_t b_bad = __ballot(badinj) & segbits;
        const uint64_t b_und = __ballot(honest && dcount < P.round_cap) & segbits;
        // segments with injections still to come (scanned by the whole wave: the record window is
        // refilled with every lane active)
        uint32_t seg_pending = 0;
        if (__any(running && q_until <= t && inj_pos < inj_cnt))
            for (uint32_t p = inj_pos; p < inj_cnt; ++p) seg_pending |= 1u << inj_at(p).seg;
        if (running) {
            if (b_act) t_stop = t;
            if (b_bad) status = BRC_BADINJ;
            else if (b_ovf) status = BRC_OVERFLOW;
            else if (P.protocol == BRC_PROTO_CONSENSUS && P.round_cap > 0 && !b_und) status = BRC_DONE;
            else if (q_until <= t && !((seg_pending >> seg) & 1u)) status = BRC_QUIESCENT;
        }
        for (uint32_t i = lane; i < nkw * AT; i += 64) s_act[row * nkw * AT + i] = 0;
        any_rows &= ~(1u << row);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        BRC_STAMP(4);
    }

#ifdef BRC_STAMPS
    if (lane == 0) for (int i = 0; i < 8; ++i) atomicAdd(&brc_stamps[i], (unsigned long long)stamp_acc[i]);
    if (lane == 0) for (int i = 0; i < 4; ++i) atomicAdd(&brc_stamps[8 + i], (unsigned long long)kcount[i]);
#endif
#undef BRC_STAMP
    // ---- write back
    {
        const uint64_t mb = item * IPW * (uint64_t)NK;
        for (uint32_t i = lane; i < IPW * NK; i += 64) {
            if (item * IPW + i / NK < P.instances) {
                gp(P.meta)[mb + i] = s_meta[i] & ~M_RESTRICTED;
                gp(P.mgen)[mb + i] = LEAN ? ((s_meta[i] & M_RESTRICTED) ? GEN_RESTRICTED : 0u) : gen32(s_gen[i]);
            }
        }
        for (uint32_t i = lane; i < RS * nkw * AT; i += 64) gp(P.act)[item * RS * nkw * AT + i] = s_act[i];
    }
    if (lane == 0) {
        gp(P.actany)[item] = any_rows;
        ItemState o = {t, inj_pos, 1u, ep};
        P.items[item] = o;
    }
    if (honest && P.protocol == BRC_PROTO_CONSENSUS) {
        gp(P.cons0)[li] = cons0_pack(round, phase, nvals, order, vcount);
        gp(P.cons1)[li] = (uint64_t)(dcount & 0xFFFF) | ((uint64_t)(frnd & 0xFFFF) << 16) | ((uint64_t)(ft & 0xFFFF) << 32) |
                      ((uint64_t)(fval & 0xFF) << 48) | ((uint64_t)(lval & 0xFF) << 56);
        if constexpr (SPEC) {
            T* gseen = (T*)P.hmask;
            uint32_t* gcnt = (uint32_t*)((char*)P.hmask + (seen_on ? P.nitems * Q * 64 * sizeof(T) : 0));
            for (uint32_t q = 0; q < Q; ++q) {
                if (seen_on) gp(gseen)[(item * Q + q) * 64 + lane] = s_seen[q * 64 + lane];
                gp(gcnt)[(item * Q + q) * 64 + lane] = s_cnt[q * 64 + lane];
            }
        } else {
            for (uint32_t v = 0; v < NVAL; ++v) gp((T*)P.hmask)[(item * NVAL + v) * 64 + lane] = s_hm[v * 64 + lane];
        }
    }
    if (LEAN && lane != 0) { st_cells = 0; st_del = 0; st_bcast = 0; }   // lean: wave-uniform counts
    if (LEAN && !honest) st_arr = 0;             // lean: arrivals were summed on every lane
    st_msgs += st_bcast * n;
    if (LEAN && real) st_loads += nk_lean - nk_skip;
    // statistics: reduce over the segment, its leader writes the instance row
    uint32_t sums[4] = {st_msgs, st_arr, st_cells, st_del};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int o = NPAD / 2; o; o >>= 1) sums[q] += (uint32_t)__shfl_xor((int)sums[q], o);
    }
    if (iex && d == 0) {
        gptr_t<uint64_t> ip = (gptr_t<uint64_t>)&gp(P.inst)[inst];
        *ip = (*ip & 0xFFFF000000000000ull) | (uint64_t)(status & 0xFFFF) | ((uint64_t)(t_stop & 0xFFFF) << 16) |
              ((uint64_t)(q_until & 0xFFFF) << 32);
        gp(P.istats)[inst * 4 + 0] += sums[0];
        gp(P.istats)[inst * 4 + 1] += sums[1];
        gp(P.istats)[inst * 4 + 2] += sums[2];
        gp(P.istats)[inst * 4 + 3] += sums[3];
    }
    uint64_t w6[5] = {st_cells, st_arr, st_msgs, st_del, st_loads};
#pragma unroll
    for (int q = 0; q < 5; ++q) {
#pragma unroll
        for (int o = 32; o; o >>= 1) w6[q] += (uint64_t)__shfl_xor((unsigned long long)w6[q], o);
    }
    uint32_t smax = st_smax;
#pragma unroll
    for (int o = 32; o; o >>= 1) smax = max(smax, (uint32_t)__shfl_xor((int)smax, o));
    const uint32_t nrun = popc(__ballot(iex && d == 0 && status == BRC_RUNNING));
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < 5; ++q) if (w6[q]) atomicAdd(&P.gcount[q], (unsigned long long)w6[q]);
        if (smax) atomicMax(&P.gcount[5], (unsigned long long)smax);
        if (nrun) atomicAdd(&P.gcount[6], (unsigned long long)nrun);
    }
}

// Launch one (DM, EV, MODE, NLR) instantiation of the step kernel for a fixed NPAD.
template <int NPAD, int DMX, bool EV, int MODE, int NLR = 0>
int launch_one(uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P) {
    auto kern = brc_step<NPAD, DMX, EV, MODE, NLR>;
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return BRC_E_HIP;
    kern<<<dim3(blocks), dim3(64 * WPB), lds, s>>>(P);
    return hipGetLastError() == hipSuccess ? 0 : BRC_E_HIP;
}

template <int NPAD>
int launch_step(int dm, bool events, int mode, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P) {
    // connection-identity peers: reference protocol, D <= 16 (brc_create)
    if (mode == KMODE_CONN && dm == 4) return events ? launch_one<NPAD, 4, true, KMODE_CONN>(blocks, lds, s, P)
                                                     : launch_one<NPAD, 4, false, KMODE_CONN>(blocks, lds, s, P);
    if (mode == KMODE_CONN && dm == 8) return events ? launch_one<NPAD, 8, true, KMODE_CONN>(blocks, lds, s, P)
                                                     : launch_one<NPAD, 8, false, KMODE_CONN>(blocks, lds, s, P);
    if (mode == KMODE_CONN && dm == 16) return events ? launch_one<NPAD, 16, true, KMODE_CONN>(blocks, lds, s, P)
                                                      : launch_one<NPAD, 16, false, KMODE_CONN>(blocks, lds, s, P);
    if constexpr (NPAD == 64) {
        // BRC_FLAG_GENERAL_KEYS: the reference protocol with sender peers on the general (non-lean) form
        if (mode == KMODE_XREF && dm == 4) return events ? launch_one<NPAD, 4, true, KMODE_XREF>(blocks, lds, s, P)
                                                         : launch_one<NPAD, 4, false, KMODE_XREF>(blocks, lds, s, P);
        if (mode == KMODE_XREF && dm == 8) return events ? launch_one<NPAD, 8, true, KMODE_XREF>(blocks, lds, s, P)
                                                         : launch_one<NPAD, 8, false, KMODE_XREF>(blocks, lds, s, P);
        if (mode == KMODE_XREF && dm == 16) return events ? launch_one<NPAD, 16, true, KMODE_XREF>(blocks, lds, s, P)
                                                          : launch_one<NPAD, 16, false, KMODE_XREF>(blocks, lds, s, P);
    }
    if (mode == KMODE_XREF) return BRC_E_INVALID;
#define BRC_CASE(DMX)                                                                                  \
    if (dm == DMX) {                                                                                   \
        if (mode == BRC_MODE_SPEC) return events ? launch_one<NPAD, DMX, true, BRC_MODE_SPEC>(blocks, lds, s, P) : launch_one<NPAD, DMX, false, BRC_MODE_SPEC>(blocks, lds, s, P); \
        if (mode == BRC_MODE_BEB) return events ? launch_one<NPAD, DMX, true, BRC_MODE_BEB>(blocks, lds, s, P) : launch_one<NPAD, DMX, false, BRC_MODE_BEB>(blocks, lds, s, P); \
        return events ? launch_one<NPAD, DMX, true, BRC_MODE_REFERENCE>(blocks, lds, s, P) : launch_one<NPAD, DMX, false, BRC_MODE_REFERENCE>(blocks, lds, s, P); \
    }
#ifdef BRC_ONLY_DM8
    BRC_CASE(8)
#else
    BRC_CASE(4) BRC_CASE(8) BRC_CASE(16)
#endif
#undef BRC_CASE
    return BRC_E_INVALID;
}

}  // namespace brc
