// brc_internal.h -- types shared by the engine's host code (brc_engine.hip) and the step-kernel
// translation units (brc_kern_<NPAD>.hip).  Not part of the public ABI (include/brc.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/brc.h"

namespace brc {

constexpr int TS = 32;            // activity ring (steps) at the largest DM; > max delay (ring_steps(dm) per kernel)
#ifndef BRC_WPB
#define BRC_WPB 1
#endif
constexpr int WPB = BRC_WPB;      // independent waves per workgroup (narrow kernel); 1 measured best:
                                  // LDS-bound SPEC runs pack more waves per CU (exp/ab.sh, r1)
constexpr uint32_t NEVER = 0xFFFFu;
constexpr uint64_t TIMES_NEVER = 0xFFFFFFFF00000000ull;
constexpr uint32_t F_EEX = 1, F_REX = 2, F_DEL = 4, F_ES = 8, F_RS = 16;
constexpr uint32_t GEN_MASK = 0x1FFF;
constexpr uint32_t GEN_RESTRICTED = 0x80000000u;
constexpr uint32_t GEN16_RESTRICTED = 0x8000u;  // the narrow kernel's 16-bit LDS copy of mgen
constexpr uint32_t GEN16_XDONE = 0x4000u;       // ... key processed by this step's extra-SEND pre-pass (brc_step.h)
__host__ __device__ inline uint16_t gen16(uint32_t g) {
    return (uint16_t)((g & GEN_MASK) | ((g & GEN_RESTRICTED) ? GEN16_RESTRICTED : 0u));
}
__host__ __device__ inline uint32_t gen32(uint16_t g) {
    return (g & GEN_MASK) | ((g & GEN16_RESTRICTED) ? GEN_RESTRICTED : 0u);
}
// activity-ring rows of the narrow kernel: a power of two above the largest delay (D <= DM)
__host__ __device__ constexpr uint32_t ring_steps(int dm) { return dm <= 8 ? 16u : 32u; }
constexpr uint32_t STEP_LIMIT = 60000;
constexpr uint32_t GEN_FULL_CLEAR = 6000;   // host forces a full clear before tags can wrap
#ifndef BRC_CHUNK_W
#define BRC_CHUNK_W 4
#endif
constexpr int CHUNK_W = BRC_CHUNK_W;                // wide kernel: keys whose ballots are exchanged per barrier
#ifndef BRC_WIDE_DCW
#define BRC_WIDE_DCW 2     // 128 key-list positions per pass: keeps cfg5 at <= 40 KB (4 workgroups per CU)
#endif
// wide kernel: delivery-bitmap words per receiver = key-list positions per pass / 64
__host__ __device__ inline uint32_t dpos_words_wide(uint32_t nkw) { return nkw < BRC_WIDE_DCW ? nkw : BRC_WIDE_DCW; }
// The consensus pass's deferred-SEND queue (brc_step.h, brc_life.h send_key): the SENDs one replica starts in
// one step's pass -- one per phase end, consecutive phase indices -- at most SENDQ_MAX of them, else
// BRC_OVERFLOW.  One bound for every kernel, so the step and key-lifetime kernels overflow at the same
// point; the queue keeps 2-bit value ids in one 64-bit word, 3-bit ones one per nibble of two.  Measured with the oracle: at
// most 17 phase ends of
// one replica in one step (cfg4, n = 64, round cap 64: bench.py's long leg, whose 2^20-instance GPU test sees
// no overflow), 12 on the reference-pinned round-cap-64 fixture (tests/test_oracle_golden.py pins it); with
// every link at delay 1 up to 27 (tests/test_gpu_life.py ref-const64-cap30-q32).
constexpr uint32_t SENDQ_MAX = 32;
template <uint32_t VB> struct SendQ {      // the queued SENDs' VB-bit value ids (VB = 3: entry i in nibble i % 16 of word i / 16)
    uint64_t w[VB == 2 ? 1 : 2];
    __device__ __forceinline__ void clear() { for (auto& x : w) x = 0; }
    __device__ __forceinline__ void put(uint32_t i, uint32_t v) {
        if constexpr (VB == 2) { w[0] |= (uint64_t)(v & 3u) << (2 * i); return; }
        const uint64_t x = (uint64_t)(v & 15u) << (4 * (i & 15u));
        if (i < 16) w[0] |= x; else w[VB == 2 ? 0 : 1] |= x;
    }
    __device__ __forceinline__ uint32_t get(uint32_t i) const {
        if constexpr (VB == 2) return (uint32_t)(w[0] >> (2 * i)) & 3u;
        return (uint32_t)((i < 16 ? w[0] : w[VB == 2 ? 0 : 1]) >> (4 * (i & 15u))) & 15u;
    }
};
constexpr int KMODE_CONN = 3;               // kernel mode: reference protocol, connection-identity peers
constexpr int KMODE_XREF = 4;               // ... reference protocol, sender peers, NPAD = 64 in the general
                                            // (non-lean) form: BRC_FLAG_GENERAL_KEYS
#ifndef BRC_CHUNK
#define BRC_CHUNK 4
#endif
constexpr int CHUNK = BRC_CHUNK;            // narrow kernel: key slots whose cell loads are in flight together
#ifndef BRC_LCHUNK
#define BRC_LCHUNK 8
#endif
constexpr int LCHUNK = BRC_LCHUNK;          // ... on the lean kernels (4 or 8; A/B round 4: 8 is 0.9 % faster)
constexpr int KPAD = CHUNK > LCHUNK ? CHUNK : LCHUNK;   // key-list padding entries: 2 KPAD
#ifndef BRC_KL32_SPEC
#define BRC_KL32_SPEC 0     // lean SPEC with u32 key-list entries too (1 KB more LDS per wave at Q = 8)
#endif

struct InjDev {       // 48 B, per item CSR, sorted by t
    uint32_t t;
    uint16_t slot, s;
    uint8_t kind, type, seg, node;
    int8_t value;
    uint8_t restricted;   // SEND to a strict subset of the peers (set by the host for n > 64)
    uint8_t pad[2];
    uint64_t dst;         // destinations 0..63 (the narrow kernel reads the first 24 B only)
    uint64_t dst_hi[3];   // destinations 64..255 (wide kernel)
};

// epoch: the lean kernels' send-step base (compact cells below); 0 elsewhere
struct ItemState { uint32_t t, inj_pos, initialized, epoch; };

// Compact cell of the lean kernels (NPAD = 64, sender peers: brc_step.h), one u32:
//   bits 0-4 flags F_EEX, F_REX, F_DEL, F_ES, F_RS
//   bits 5-10 |echo set|, 11-16 |ready set| (both saturate at 63)
//   bits 17-23 / 24-30: step this lane SENT its ECHO / READY, as an offset from the item's epoch;
//   C32_OLD = sent more than DM steps before the epoch, C32_NEVER = not sent
// No generation tag: a slot's row is rewritten fresh whenever the slot is (re)allocated.
constexpr uint32_t C32_EC_SH = 5, C32_RC_SH = 11, C32_OE_SH = 17, C32_OR_SH = 24;
constexpr uint32_t C32_NEVER = 127, C32_OLD = 126;
constexpr uint32_t C32_FRESH = (C32_NEVER << C32_OE_SH) | (C32_NEVER << C32_OR_SH);
constexpr uint32_t C32_REBASE = 100;   // a step more than this past the epoch moves the epoch first
constexpr uint32_t C32_KEEP = 17;      // ... to t - C32_KEEP: sends in the last 16 steps keep their step

struct InstState { uint16_t status, t_stop, q_until, flags; uint32_t pad0, pad1; };

struct Params {
    uint32_t n, f, D, Q, NV, NK, nkw;
    uint32_t protocol, delay_model, dconst, round_cap, step_cap, proposals;
    uint32_t T_echo, T_amp, T_del, T_cnt, bound_p1, bound_p2;
    uint64_t seed, inst_offset, instances, nitems;
    uint32_t max_steps, nL;   // nL: delay_values() of the run
    uint32_t mode;            // BRC_MODE_*
    uint32_t s_limit;         // phase indices >= s_limit overflow: the slot generation tags must not wrap
    uint64_t coin_seed;
    uint64_t event_cap;
    uint64_t* cells;
    uint64_t* meta; uint32_t* mgen; uint64_t* kdst;
    uint64_t* act; uint32_t* actany; ItemState* items; InstState* inst; uint64_t* istats;
    uint64_t* cons0; uint64_t* cons1; void* hmask;
    const InjDev* inj; const uint32_t* inj_off; const uint32_t* inj_cnt;
    const uint64_t* byz; const int8_t* prop;
    brc_event* events; unsigned long long* event_count;
    uint64_t* dbits;              // lean SPEC: per-wave delivery bitmaps [item][nkw][64] (brc_step.h DBG)
    uint64_t* dring;              // per-link key-lifetime kernel: delivery bitmap ring [item][LIFE_RW or LIFE_RW16][nkw][64] (brc_life.h)
    uint32_t* lmeta;              // key-lifetime kernel, key windows >= 32: key-slot metadata + class delivery steps
                                  // [item][2][NK] u32 in HBM (brc_life.h)
    uint64_t* xsend;              // non-lean step kernels: extra-SEND records [item][XSEND_MAX][3] (brc_step.h)
    uint32_t* xsn;                // ... records in use per item
    unsigned long long* gcount;   // [0] cell_steps [1] arrivals [2] msgs [3] deliveries [4] lane loads [5] max s
                                  // [6] instances still running after the launch
};

// Distinct link delays a delay model can produce (bounds the compact delay-mask table in LDS).
__host__ __device__ inline uint32_t delay_values(uint32_t model, uint32_t dmax) {
    return model == BRC_DELAY_CONST ? 1u : model == BRC_DELAY_SLOWSET ? (dmax > 1 ? 2u : 1u) : dmax;
}

// Extra-SEND records per item (a payload SENT by several origins; brc_step.h): live at once
constexpr uint32_t XSEND_MAX = 16;

// Consensus value ids (core/byzantinerandomizedconsensus.py:57-60 keys its tables by payload string;
// id 0 is str(NONE) == "-1"): 2 bits (3 strings + "-1") on the lean, wide and key-lifetime kernels,
// 3 bits (7 strings + "-1") on the other narrow kernels (NPAD <= 32, and connection peers).
__host__ __device__ constexpr uint32_t value_ids(bool narrow_full) { return narrow_full ? 8u : 4u; }

// Consensus record word 0 (cons0): round [0,16) | phase [16,20) | nvals [20,24) | order [24,48) (the
// value ids in insertion order, 2 or 3 bits each) | value_count [48,64)
__host__ __device__ inline uint64_t cons0_pack(uint32_t round, uint32_t phase, uint32_t nvals, uint32_t order,
                                               uint32_t vcount) {
    return (uint64_t)(round & 0xFFFF) | ((uint64_t)(phase & 0xF) << 16) | ((uint64_t)(nvals & 0xF) << 20) |
           ((uint64_t)(order & 0xFFFFFF) << 24) | ((uint64_t)(vcount & 0xFFFF) << 48);
}

// u64 words of a wave's consensus LDS area: REFERENCE hm[nval][64] T; SPEC [seen[Q][64] T +] cnt[Q][64] u32
__host__ __device__ inline uint32_t cons_words(bool spec, uint32_t msize, uint32_t Q, uint32_t nv, uint32_t nval = 4) {
    // SPEC with one key variant per origin: a replica delivers each (origin, phase) key at most
    // once, so the origin count needs no host set (seen masks only when nv > 1)
    return spec ? (Q * 64 * (nv > 1 ? msize : 0u) + Q * 64 * 4 + 7) / 8 : (nval * 64 * msize + 7) / 8;
}

// Activity-ring words per (row, key word): the lean kernels keep one ECHO and one READY row (typed
// marks: a key step evaluates only the message types that can land; SEND arrivals are found from the
// key metadata), the others one untyped row for the wave item.  BRC_PSEG=1 (experimental) gives the
// non-lean kernels one row and key list per instance of the item (IPW = 64 / NPAD of them), so a key
// step loads only the instances with arrivals on it: measured SLOWER on cfg2 / cfg3 / cfg3-spec /
// cfg2-spec (per-lane key ids turn the key dispatch into vector work; round-5 A/B), so off by default.
#ifndef BRC_PSEG
#define BRC_PSEG 0
#endif
__host__ __device__ constexpr uint32_t act_types(bool lean, uint32_t ipw = 1) { return lean ? 2u : BRC_PSEG ? ipw : 1u; }

// Injection records the non-lean narrow kernels stage in LDS at a time (one memory round trip per
// INJ_CACHE records instead of one per record: cfg3's equivocation pattern is 120 records per wave)
constexpr uint32_t INJ_CACHE = 16;

// Bytes of dynamic LDS one wave of the step kernel needs (must match the kernel's carve):
// meta[IPW*NK] u64 | act[RS][act_types][nkw] u64 | dbits[nkw][64] u64 (not on lean SPEC) | consensus area | L[nL][64] T |
// mgen[IPW*NK] u16 (not on the lean kernels) | klist[NK + 2 KPAD] u16 (tail padded with the trash row NK;
// u32 entries on the lean REFERENCE / BEB kernels; BRC_PSEG: one list per instance on the others) |
// injc[INJ_CACHE][3] u64 (not on the lean kernels)
__host__ __device__ inline uint32_t lds_bytes_per_wave(int npad, uint32_t NK, uint32_t nkw, uint32_t nL, bool spec,
                                                       uint32_t Q, uint32_t nv, uint32_t rs, bool lean) {
    const uint32_t ipw = 64 / (uint32_t)npad;
    const uint32_t msize = npad <= 8 ? 1 : (uint32_t)npad / 8;
    const uint32_t h_words = cons_words(spec, msize, Q, nv, value_ids(!lean));
    const uint32_t l_words = (nL * 64 * msize + 7) / 8;
    // (lean REFERENCE / BEB kernels: u32 entries, brc_step.h KL_*)
    const uint32_t klist_u16 = (NK + 2 * KPAD) * ((lean && (!spec || BRC_KL32_SPEC)) ? 2u : lean ? 1u : act_types(false, ipw));
    const uint32_t gen_words = lean ? 0u : (ipw * NK + 3) / 4;   // lean kernels keep no slot generations
    const uint32_t dbits_words = (lean && spec) ? 0u : 64 * nkw;   // lean SPEC keeps them in HBM
    const uint32_t injc_words = lean ? 0u : 3 * INJ_CACHE;
    return 8 * (ipw * NK + rs * nkw * act_types(lean, ipw) + dbits_words + h_words + l_words + gen_words + (klist_u16 + 3) / 4 +
                injc_words);
}

// Bytes of dynamic LDS one workgroup of the wide kernel needs (brc_step_wide.h carve):
// meta[NK] u64 | act[rs][nkw] u64 (rs = ring_steps(dm)) | dpos[DCW][NPAD] u64 | consensus area |
// xb[2][CHUNK_W][nL][2][NW] u64 | outm[16][NW] u64 | sq[Q][NPAD] u8 | fresh[nkw] u64 | klist[NK] u16 |
// red[12] u32 | pmw[2][CHUNK_W][NW] u32
// consensus area: REFERENCE hm[4][NW][NPAD] u64;  SPEC cnt[Q][NPAD] u32 (one key variant per origin)
__host__ __device__ inline uint32_t cons_words_wide(bool spec, uint32_t npad, uint32_t Q) {
    const uint32_t nw = npad / 64;
    return spec ? (Q * npad + 1) / 2 : 4 * nw * npad;
}
// Wide kernel: link-delay code bit planes per DM (delay - 1 in NPL bits), and the u64 words one
// wave publishes per (key, message type) in the ballot exchange: one per link delay present
// (constant, slow-set), or -- uniform / geometric delays -- the NPL bit planes of "steps since
// this lane sent, minus one" plus the mask of lanes whose send lies inside the 2^NPL window.
__host__ __device__ constexpr int npl_of(int dm) { return dm == 4 ? 2 : dm == 8 ? 3 : 4; }
__host__ __device__ inline bool plane_model(uint32_t model) {
    return model == BRC_DELAY_UNIFORM || model == BRC_DELAY_GEOMETRIC;
}
__host__ __device__ inline uint32_t xwords_wide(uint32_t model, uint32_t dmax, int dm) {
    return plane_model(model) ? (uint32_t)npl_of(dm) + 1u : delay_values(model, dmax);
}

__host__ __device__ inline uint32_t lds_bytes_wide(int npad, uint32_t NK, uint32_t nkw, uint32_t nL, bool spec, uint32_t Q,
                                                    uint32_t rs) {
    const uint32_t nw = (uint32_t)npad / 64;
    return 8 * (NK + rs * nkw + dpos_words_wide(nkw) * (uint32_t)npad + cons_words_wide(spec, (uint32_t)npad, Q) +
                2 * CHUNK_W * nL * 2 * nw + 16 * nw) +
           Q * (uint32_t)npad + 8 * nkw + 2 * NK + 4 * (12 + 2 * CHUNK_W * nw);
}

// Bytes of the global consensus-set buffer (hmask) per item: REFERENCE host masks [4][lanes] of
// n bits; SPEC phase windows seen[Q][lanes] (n bits; narrow kernel only) + cnt[Q][lanes] u32.
inline uint64_t cons_bytes_per_item(bool spec, bool wide, uint32_t lanes, uint32_t msize, uint32_t Q, uint32_t nv,
                                    uint32_t nval = 4) {
    return spec ? (uint64_t)Q * lanes * ((wide || nv == 1 ? 0 : msize) + 4) : (uint64_t)nval * lanes * msize;
}

// Key-lifetime kernel (brc_life.h): ring steps (> 4 Dd - 1 for Dd <= 8) and LDS bytes of one wave
// (must match the kernel's carve):
//   meta[NK] u32 | two-class form: dA[NK], dB[NK] u8 (each receiver class's delivery step of the key,
//   0x80 | step mod 128) | (8-B aligned) consensus area (cons_words at NPAD = 64)
constexpr uint32_t LIFE_RW = 32;
// Key windows >= 32 in the two-class form (life_hbm_meta): the slot metadata lives in HBM (P.lmeta) and
// LDS keeps only the class delivery steps plus a 128-word snapshot of the metadata of the key words a
// consensus pass reads (their own instantiations, brc_life<..., HMT>).
#ifndef BRC_LIFE_HM_Q
#define BRC_LIFE_HM_Q 32
#endif
__host__ __device__ inline bool life_hbm_meta(uint32_t Q, bool perlink) { return !perlink && Q >= BRC_LIFE_HM_Q; }
// Their class delivery steps live in HBM too (one u32 per slot beside the metadata: 8 B per slot in
// P.lmeta); LDS keeps, per ring step, the key words with a delivery then (LIFE_RW rows x 128 bits) and the
// consumed words' class bitmaps (16 B per key word).
__host__ __device__ inline uint32_t lds_bytes_life(uint32_t NK, bool spec, uint32_t Q, uint32_t nv, bool perlink) {
    if (life_hbm_meta(Q, perlink))
        return 4u * 128u + 16u * 32u + 16u * ((NK + 63) / 64) + 8 * cons_words(spec, 8, Q, nv);
    return ((4u * NK + (perlink ? 0u : 2 * NK) + 7) & ~7u) + 8 * cons_words(spec, 8, Q, nv);
}
// Launch the key-lifetime kernel (brc_kern_life.hip): one 64-lane workgroup per instance
// (perlink: uniform / geometric delays, delivery bitmaps in P.dring; dm16: delays up to 16, whose
// keys live up to 64 steps: P.dring has LIFE_RW16 rows)
constexpr uint32_t LIFE_RW16 = 64;
// qbig: key windows of 64 / 128 (two-class form, not SPEC)
// hm: the slot metadata in HBM (life_hbm_meta)
int launch_life(int mode, bool perlink, bool dm16, bool qbig, bool hm, uint32_t blocks, uint32_t lds, hipStream_t s,
                const Params* P);

// Step-kernel launchers, one translation unit per replica-set width NPAD (brc_kern_<NPAD>.hip).
// Return 0 on success, BRC_E_INVALID when no instantiation matches (dm), BRC_E_HIP on a launch error.
int launch_step_4(int dm, bool events, int mode, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P);
int launch_step_8(int dm, bool events, int mode, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P);
int launch_step_16(int dm, bool events, int mode, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P);
int launch_step_32(int dm, bool events, int mode, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P);
int launch_step_64(int dm, bool events, int mode, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P);
// NPAD = 64 lean kernels with the (at most two) link-delay masks in registers (brc_kern_64r.hip)
int launch_step_64r(int dm, bool events, int mode, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P);
// wide kernel (brc_step_wide.h): one workgroup of NPAD threads per instance
// wv4: the 4-waves-per-SIMD instantiation (wide_waves4: DM <= 8, no link-delay planes, sender peers)
int launch_step_128(int dm, bool events, int mode, bool wv4, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P);
int launch_step_256(int dm, bool events, int mode, bool wv4, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P);

}  // namespace brc
