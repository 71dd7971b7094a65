// brc_engine.hip -- MI355X (gfx950) batched Bracha-broadcast + randomized-consensus engine.
//
// One 64-lane wavefront simulates an "item": IPW = 64 / NPAD independent instances, lane =
// (instance segment, replica).  Lane d is at once receiver d (its BRB cells), sender d (its
// send steps are read back by every receiver through __ballot) and consensus replica d.  A
// wave runs its item from the current step to completion in ONE launch: instances are
// independent, so no inter-wave communication exists at all.  Workgroups hold 4 such waves
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
// HBM (lane-contiguous => every access is one coalesced 512-B wave access):
//   cells [item][NK][64] u64
// per instance key slots (copied to LDS for the launch): meta [inst][NK] u64 (s+1 | t_send |
//   t_quiet | sender | value), mgen [inst][NK] u32 (generation | restricted-SEND flag),
//   kdst [inst][NK] u64 (SEND destinations, read only for restricted SENDs)
// per item: act [item][32][nkw] u64 (key slots that may have arrivals at step t mod 32)
// per lane: cons0/cons1 [item][64] u64, hmask [item][4][64] T (consensus state)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/brc.h"
#include "schedule.h"

namespace {

constexpr int TS = 32;            // activity ring (steps); > max delay
constexpr int WPB = 4;            // independent waves per workgroup
#ifndef BRC_CHUNK
#define BRC_CHUNK 8
#endif
constexpr int CHUNK = BRC_CHUNK;  // key slots processed together (memory-level parallelism)
constexpr uint32_t NEVER = 0xFFFFu;
constexpr uint64_t TIMES_NEVER = 0xFFFFFFFF00000000ull;
constexpr uint32_t F_EEX = 1, F_REX = 2, F_DEL = 4, F_ES = 8, F_RS = 16;
constexpr uint32_t GEN_MASK = 0x1FFF;
constexpr uint32_t GEN_RESTRICTED = 0x80000000u;
constexpr uint32_t STEP_LIMIT = 60000;
constexpr uint32_t GEN_FULL_CLEAR = 6000;   // host forces a full clear before tags can wrap

struct InjDev {       // 24 B, per item CSR, sorted by t
    uint32_t t;
    uint16_t slot, s;
    uint8_t kind, type, seg, node;
    int8_t value;
    uint8_t pad[3];
    uint64_t dst;
};

struct ItemState { uint32_t t, inj_pos, initialized, pad; };

struct InstState { uint16_t status, t_stop, q_until, flags; uint32_t pad0, pad1; };

struct Params {
    uint32_t n, f, D, Q, NV, NK, nkw;
    uint32_t protocol, delay_model, dconst, round_cap, step_cap, proposals;
    uint32_t T_echo, T_amp, T_del, T_cnt, bound_p1, bound_p2;
    uint64_t seed, inst_offset, instances, nitems;
    uint32_t max_steps, pad;
    uint64_t event_cap;
    uint64_t* cells;
    uint64_t* meta; uint32_t* mgen; uint64_t* kdst;
    uint64_t* act; uint32_t* actany; ItemState* items; InstState* inst; uint64_t* istats;
    uint64_t* cons0; uint64_t* cons1; void* hmask;
    const InjDev* inj; const uint32_t* inj_off; const uint32_t* inj_cnt;
    const uint64_t* byz; const int8_t* prop;
    brc_event* events; unsigned long long* event_count;
    unsigned long long* gcount;   // [0] cell_steps [1] arrivals [2] msgs [3] deliveries [4] lane loads [5] max s
};

template <int NPAD> struct MaskOf { using type = uint64_t; };
template <> struct MaskOf<4> { using type = uint8_t; };
template <> struct MaskOf<8> { using type = uint8_t; };
template <> struct MaskOf<16> { using type = uint16_t; };
template <> struct MaskOf<32> { using type = uint32_t; };

template <int NPAD> constexpr int nkw_of() { return NPAD / 8 < 1 ? 1 : NPAD / 8; }   // NK <= 8 * NPAD

template <typename T> __device__ __forceinline__ uint32_t popc(T x) { return (uint32_t)__popcll((uint64_t)x); }

__device__ __forceinline__ uint32_t wave_or(uint32_t x) {
#pragma unroll
    for (int o = 32; o; o >>= 1) x |= (uint32_t)__shfl_xor((int)x, o);
    return x;
}

template <int NPAD> __device__ __forceinline__ uint32_t seg_max(uint32_t x) {
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

// packed LDS/HBM key metadata
__device__ __forceinline__ uint32_t m_s1(uint64_t m) { return (uint32_t)(m & 0xFFFF); }
__device__ __forceinline__ uint32_t m_tsend(uint64_t m) { return (uint32_t)((m >> 16) & 0xFFFF); }
__device__ __forceinline__ uint32_t m_tquiet(uint64_t m) { return (uint32_t)((m >> 32) & 0xFFFF); }
__device__ __forceinline__ uint32_t m_sender(uint64_t m) { return (uint32_t)((m >> 48) & 0xFF); }
__device__ __forceinline__ uint32_t m_value(uint64_t m) { return (uint32_t)((m >> 56) & 0xFF); }
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
__device__ __forceinline__ void brb_cell_update(uint32_t& fl, uint32_t& ec, uint32_t& rc, bool s_arr,
                                                uint32_t ea, uint32_t ra, uint32_t T_echo, uint32_t T_amp,
                                                uint32_t T_del, bool& echo_send, bool& ready_send, bool& deliver) {
    echo_send = ready_send = deliver = false;
    if (fl & F_DEL) return;                                              // :74
    if (s_arr && !(fl & F_EEX)) { fl |= F_EEX | F_ES; echo_send = true; }   // :76-82
    if (ea) {
        uint32_t checked = ea;
        if (!(fl & F_EEX)) { fl |= F_EEX; checked = ea - 1; }           // :87-89
        ec += ea;                                                        // :89/:92
        if (checked && ec >= T_echo && !(fl & F_REX)) { fl |= F_REX | F_RS; ready_send = true; }   // :95-98
    }
    if (ra) {
        uint32_t lo, hi;
        if (!(fl & F_REX)) { fl |= F_REX; lo = 2; hi = ra; }            // :103-105
        else { lo = rc + 1; hi = rc + ra; }                              // :108
        rc += ra;
        if (hi >= lo) {
            if (!(fl & F_EEX)) {                                         // :118
                const uint32_t alo = max(lo, T_amp), ahi = min(hi, T_del - 1);
                if (alo <= ahi && !(fl & F_RS)) { fl |= F_RS; ready_send = true; }   // :119
            }
            if (hi >= T_del) { fl |= F_DEL; deliver = true; }            // :111-115
        }
    }
}

#ifndef BRC_MIN_WAVES
#define BRC_MIN_WAVES 4      // waves per SIMD the register allocation must allow
#endif

template <int NPAD, int DM>
__global__ __launch_bounds__(64 * WPB, BRC_MIN_WAVES) void brc_kernel(Params P) {
    using T = typename MaskOf<NPAD>::type;
    constexpr int IPW = 64 / NPAD;
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];

    const int wid = threadIdx.x / 64, lane = threadIdx.x % 64;
    const uint64_t item = (uint64_t)blockIdx.x * WPB + wid;
    if (item >= P.nitems) return;               // whole wave exits; waves never synchronise
    const uint32_t n = P.n, NK = P.NK, Q = P.Q, NV = P.NV, D = P.D, nkw = P.nkw;
    // per-wave LDS carve: meta[IPW*NK] u64 | act[TS][nkw] u64 | dbits[nkw][64] u64 |
    //                     L[DM][64] T | hm[4][64] T | mgen[IPW*NK] u32 | any u32
    const uint32_t l_words = (DM * 64 * (uint32_t)sizeof(T) + 7) / 8;
    const uint32_t h_words = (4 * 64 * (uint32_t)sizeof(T) + 7) / 8;
    const uint32_t per_wave_words = IPW * NK + TS * nkw + 64 * nkw + l_words + h_words + (IPW * NK + 2) / 2 + 1;
    uint64_t* s_meta = smem + (size_t)wid * per_wave_words;
    uint64_t* s_act = s_meta + IPW * NK;
    uint64_t* s_dbits = s_act + TS * nkw;        // this step's deliveries, per lane
    T* s_L = (T*)(s_dbits + 64 * nkw);           // s_L[i*64 + lane]: senders at delay i+1
    T* s_hm = (T*)(s_dbits + 64 * nkw + l_words);   // s_hm[v*64 + lane]: hosts that delivered value v
    uint32_t* s_gen = (uint32_t*)(s_dbits + 64 * nkw + l_words + h_words);
    uint32_t* s_any = s_gen + IPW * NK;

    const int seg = lane / NPAD, d = lane % NPAD, segbase = seg * NPAD;
    const uint64_t inst = item * IPW + seg;
    const bool iex = inst < P.instances;
    const uint64_t g = P.inst_offset + inst;
    const uint64_t all64 = (n >= 64) ? ~0ull : ((1ull << n) - 1);
    const T allm = (T)all64;
    const uint64_t segbits = (NPAD == 64) ? ~0ull : (((1ull << NPAD) - 1) << segbase);
    const uint32_t mbase = seg * NK;             // this lane's instance in the LDS meta arrays

    ItemState its = P.items[item];
    uint32_t t = its.t, inj_pos = its.inj_pos;
    const uint32_t inj_off = P.inj_off[item], inj_cnt = P.inj_cnt[item];
    {
        const uint64_t mb = item * IPW * (uint64_t)NK;
        for (uint32_t i = lane; i < IPW * NK; i += 64) {
            const bool ok = item * IPW + i / NK < P.instances;
            s_meta[i] = ok ? P.meta[mb + i] : 0ull;
            s_gen[i] = ok ? P.mgen[mb + i] : 0u;
        }
        for (uint32_t i = lane; i < TS * nkw; i += 64) s_act[i] = P.act[item * TS * nkw + i];
        for (uint32_t w = 0; w < nkw; ++w) s_dbits[w * 64 + lane] = 0;
        if (lane == 0) *s_any = P.actany[item];
    }

    uint32_t status = BRC_DONE, t_stop = 0, q_until = 0;
    if (iex) {
        const uint64_t w0 = *(const uint64_t*)&P.inst[inst];     // status | t_stop | q_until | flags
        status = w0 & 0xFFFF; t_stop = (w0 >> 16) & 0xFFFF; q_until = (w0 >> 32) & 0xFFFF;
    }
    const uint64_t byzm = iex ? P.byz[inst] : ~0ull;
    const bool real = iex && (uint32_t)d < n;
    const bool honest = real && !((byzm >> d) & 1ull);

    // ---- link-delay masks: L[i] = senders j whose link j -> d has delay i+1 (schedule.h)
    T L[DM];
#pragma unroll
    for (int i = 0; i < DM; ++i) L[i] = 0;
    if (real) {
        if (P.delay_model == BRC_DELAY_CONST) {
#pragma unroll
            for (int i = 0; i < DM; ++i) if ((uint32_t)i + 1 == P.dconst) L[i] = allm;
        } else if (P.delay_model == BRC_DELAY_SLOWSET) {
            const uint32_t off = brc::slow_offset(P.seed, g, n);
            T slowm = 0;
            for (uint32_t j = 0; j < n; ++j) if (((j + n - off) % n) < P.f) slowm |= (T)((T)1 << j);
            const bool me_slow = ((uint32_t)d + n - off) % n < P.f;
#pragma unroll
            for (int i = 0; i < DM; ++i) {
                if ((uint32_t)i + 1 == D) L[i] |= me_slow ? allm : slowm;
                if (i == 0) L[i] |= me_slow ? (T)0 : (T)(allm & ~slowm);
            }
        } else {
            for (uint32_t j4 = 0; j4 < (n + 3) / 4; ++j4) {
                const brc::u32x4 w = brc::draw(P.seed, g, (uint32_t)d, brc::PURPOSE_DELAY, j4);
                const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t j = 4 * j4 + q;
                    if (j >= n) break;
                    const uint32_t dl = (P.delay_model == BRC_DELAY_UNIFORM) ? brc::uniform_delay(ws[q], D)
                                                                             : brc::geometric_delay(ws[q], D);
#pragma unroll
                    for (int i = 0; i < DM; ++i) if ((uint32_t)i + 1 == dl) L[i] |= (T)((T)1 << j);
                }
            }
        }
    }
    // outset: delays (bit i <=> delay i+1) from THIS lane, as a sender, to honest receivers
    uint32_t outset = 0;
#pragma unroll
    for (int i = 0; i < DM; ++i) {
        const T m = seg_or<NPAD, T>(honest ? L[i] : (T)0);
        if (real && ((m >> d) & 1)) outset |= 1u << i;
        s_L[i * 64 + lane] = L[i];
    }
    const uint32_t maxout = hibit(outset);
    const uint32_t dset = uni32(wave_or(outset));    // every delay some link of this wave has
    uint64_t* const mycells = P.cells + item * (uint64_t)NK * 64 + lane;   // cell (k, lane) at [k * 64]

    // ---- consensus state (core/byzantinerandomizedconsensus.py:25-29)
    uint64_t c0 = 0, c1 = 0;
    const size_t li = item * 64 + lane;
    const bool cons_lane = honest && P.protocol == BRC_PROTO_CONSENSUS;
    if (cons_lane) { c0 = P.cons0[li]; c1 = P.cons1[li]; }
    for (int v = 0; v < 4; ++v) s_hm[v * 64 + lane] = cons_lane ? ((const T*)P.hmask)[(item * 4 + v) * 64 + lane] : (T)0;
    uint32_t round = c0 & 0xFFFF, phase = (c0 >> 16) & 0xFF, nvals = (c0 >> 24) & 0xFF;
    uint32_t order = (c0 >> 32) & 0xFF, vcount = (c0 >> 48) & 0xFFFF;
    uint32_t dcount = c1 & 0xFFFF, frnd = (c1 >> 16) & 0xFFFF, ft = (c1 >> 32) & 0xFFFF;
    uint32_t fval = (c1 >> 48) & 0xFF, lval = (c1 >> 56) & 0xFF;

    uint32_t st_msgs = 0, st_arr = 0, st_cells = 0, st_del = 0, st_loads = 0, st_smax = 0;
    bool ovf = false, badinj = false;

    auto log_ev = [&](uint32_t kind, uint32_t node, uint32_t type, uint32_t a, uint32_t b) {
        if (P.event_cap) {
            const unsigned long long i = atomicAdd(P.event_count, 1ull);
            if (i < P.event_cap) {
                brc_event e;
                e.instance = inst; e.t = t; e.kind = (uint8_t)kind; e.node = (uint8_t)node;
                e.type = (uint8_t)type; e.pad = 0; e.a = a; e.b = b;
                P.events[i] = e;
            }
        }
    };
    auto mark = [&](uint32_t k, uint32_t dset) {   // key k may have arrivals at t + delay
        while (dset) {
            const uint32_t i = __ffs(dset) - 1; dset &= dset - 1;
            const uint32_t row = (t + i + 1) & (TS - 1);
            atomicOr((unsigned long long*)&s_act[row * nkw + (k >> 6)], 1ull << (k & 63));
            atomicOr(s_any, 1u << row);
        }
    };
    // honest origin d broadcasts SEND for its key (d, s) with value v
    // (core/byzantinerandomizedconsensus.py:48-50 / :80-83 / :102-106, base/broadcast.py:30-35)
    auto send_key = [&](uint32_t s, uint32_t v) {
        const uint32_t k = (d * NV) * Q + (s % Q);
        const uint64_t m = s_meta[mbase + k];
        if (m_s1(m) != 0 && t < m_tquiet(m)) { ovf = true; return; }
        s_gen[mbase + k] = ((s_gen[mbase + k] & GEN_MASK) + 1) & GEN_MASK;
        s_meta[mbase + k] = m_pack(s + 1, t, t + maxout, d, v);
        mark(k, outset);
        q_until = max(q_until, t + maxout);
        st_msgs += n;
        st_smax = max(st_smax, s);
        log_ev(BRC_EV_SEND, d, BRC_SEND, d * NV, s);
    };
    auto get_max_val = [&](uint32_t bound2) -> uint32_t {          // :64-68
        for (uint32_t i = 0; i < nvals; ++i) {
            const uint32_t v = (order >> (2 * i)) & 3;
            if (2 * popc(s_hm[v * 64 + lane]) > bound2) return v;
        }
        return 0;                                                    // str(NONE) == "-1"
    };
    auto cons_reset = [&]() {
        vcount = 0; nvals = 0; order = 0;
        for (int v = 0; v < 4; ++v) s_hm[v * 64 + lane] = 0;
    };
    auto cons_deliver = [&](uint32_t k) {                            // :53-106
        const uint32_t v = m_value(s_meta[mbase + k]) & 3, host = (k / Q) / NV;
        bool found = false;
        for (uint32_t i = 0; i < nvals; ++i) found |= ((order >> (2 * i)) & 3) == v;
        if (!found) { order |= v << (2 * nvals); ++nvals; }         // :57-58
        s_hm[v * 64 + lane] |= (T)((T)1 << host);                   // :60
        ++vcount;                                                    // :61
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
            log_ev(BRC_EV_DECIDE, d, 0, round, dec);
            ++round; phase = 1; cons_reset();                        // :96-100
            send_key(2 * (round - 1), dec);                          // :102-106
        }
    };

    // ---- actions stamped t (performed after step t's messages)
    auto do_actions = [&]() -> bool {
        bool mine_any = false;
        const bool running = status == BRC_RUNNING;
        if (its.initialized == 0 && t == 0) {
            if (P.protocol == BRC_PROTO_CONSENSUS && P.proposals != BRC_PROPOSALS_NONE && honest && running) {
                const uint32_t v = (P.proposals == BRC_PROPOSALS_PHILOX) ? brc::proposal_id(P.seed, g, d)
                                                                         : (uint32_t)P.prop[inst * n + d];
                round = 1; phase = 1;                                 // :43-47
                send_key(0, v & 3);
            }
        }
        while (inj_pos < inj_cnt) {
            const InjDev r = P.inj[inj_off + inj_pos];
            if (r.t != t) break;
            ++inj_pos;
            const bool mine = running && seg == (int)r.seg;
            mine_any |= mine;
            if (r.kind == BRC_INJ_PROPOSE) {
                if (mine && honest && d == r.node) { round = 1; phase = 1; send_key(0, (uint32_t)r.value & 3); }
            } else if (r.kind == BRC_INJ_SEND || r.kind == BRC_INJ_KEY) {
                // KEY declares a (Byzantine) key without sending; SEND sends it, allocating the
                // slot first unless that key was declared and not yet sent
                const bool is_send = r.kind == BRC_INJ_SEND;
                uint32_t myset = 0;
                if (is_send && mine && honest && ((r.dst >> d) & 1ull)) {
                    for (uint32_t i = 0; i < D; ++i) if ((s_L[i * 64 + lane] >> r.node) & 1) myset = 1u << i;
                }
                const uint32_t os = wave_or(myset);
                if (mine) {
                    const uint32_t k = r.slot;
                    if (d == 0) {
                        uint64_t m = s_meta[mbase + k];
                        uint32_t gen = s_gen[mbase + k] & GEN_MASK;
                        const bool declared = m_s1(m) == r.s + 1u && m_tsend(m) == NEVER && is_send;
                        if (!declared && m_s1(m) != 0 && t < m_tquiet(m)) {
                            ovf = true;
                        } else {
                            uint32_t tq = m_tquiet(m);
                            // a declared key holds its slot at least until the next step
                            if (!declared) { gen = (gen + 1) & GEN_MASK; tq = t + 1; }
                            if (is_send) tq = max(tq, t + hibit(os));
                            m = m_pack(r.s + 1, is_send ? t : NEVER, tq, r.node, (uint32_t)(uint8_t)r.value);
                            s_meta[mbase + k] = m;
                            const bool restricted = is_send && (r.dst & all64) != all64;
                            s_gen[mbase + k] = gen | (restricted ? GEN_RESTRICTED : 0u);
                            st_smax = max(st_smax, (uint32_t)r.s);
                            if (is_send) {
                                P.kdst[inst * NK + k] = r.dst;
                                mark(k, os);
                                st_msgs += __popcll(r.dst & all64);
                                log_ev(BRC_EV_SEND, r.node, BRC_SEND, k / Q, r.s);
                            }
                        }
                    }
                    q_until = max(q_until, t + hibit(os));
                }
            } else if (r.kind == BRC_INJ_MSG) {
                const uint32_t k = r.slot;
                bool sent = false;
                if (mine && d == r.node) {
                    const uint64_t m = s_meta[mbase + k];
                    if (m_s1(m) != r.s + 1u) {
                        badinj = true;
                    } else {
                        const uint32_t gen = s_gen[mbase + k] & GEN_MASK;
                        const size_t ci = ((size_t)item * NK + k) * 64 + lane;
                        uint64_t wv = P.cells[ci];
                        if (((wv >> 19) & GEN_MASK) != gen) wv = TIMES_NEVER | ((uint64_t)gen << 19);
                        const uint32_t bit = (r.type == BRC_ECHO) ? F_ES : F_RS;
                        if (!(wv & bit)) {
                            sent = true;
                            wv |= bit;
                            const int sh = (r.type == BRC_ECHO) ? 32 : 48;
                            wv = (wv & ~(0xFFFFull << sh)) | ((uint64_t)t << sh);
                            P.cells[ci] = wv;
                            st_msgs += n;
                            log_ev(BRC_EV_SEND, d, r.type, k / Q, r.s);
                        }
                    }
                }
                const uint32_t os = wave_or(sent ? outset : 0u);
                if (os) {
                    if (lane == 0) mark(k, os);
                    const uint32_t myq = seg_max<NPAD>(sent ? t + maxout : 0u);
                    if (mine && myq) {
                        if (d == 0) {
                            const uint64_t m = s_meta[mbase + k];
                            if (myq > m_tquiet(m)) s_meta[mbase + k] = m_with_tquiet(m, myq);
                        }
                        q_until = max(q_until, myq);
                    }
                }
            }
        }
        its.initialized = 1;
        return mine_any;
    };

    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (its.initialized == 0 && t == 0) {
        do_actions();
        q_until = seg_max<NPAD>(q_until);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }

    for (uint32_t it = 0; it < P.max_steps; ++it) {
        const bool running = status == BRC_RUNNING;
        if (!__any(running)) break;
        // next step with possible arrivals (activity ring) or a pending action
        const uint32_t any = *s_any;
        const uint32_t rot = (t + 1) & (TS - 1);
        const uint32_t rr = rot ? ((any >> rot) | (any << (TS - rot))) : any;
        uint32_t next = rr ? t + (uint32_t)__ffs(rr) : 0xFFFFFFFFu;
        if (inj_pos < inj_cnt) next = min(next, P.inj[inj_off + inj_pos].t);
        if (next == 0xFFFFFFFFu) { if (running) status = BRC_QUIESCENT; break; }
        if (next > P.step_cap) { if (running) status = BRC_STEPCAP; break; }
        t = next;
        const uint32_t row = t & (TS - 1);

        // ================= BRB: active key slots in chunks; one (receiver, key) cell per lane
        bool lane_active = false, any_del = false;
#pragma unroll 1
        for (uint32_t w = 0; w < nkw; ++w) {
            uint64_t rem = uni64(s_act[row * nkw + w]);
            while (rem) {
                uint32_t kc[CHUNK];
                bool vc[CHUNK];
                uint64_t wc[CHUNK];
                // phase A: every lane's cell word of CHUNK key slots, all loads in flight at once
                Unrolled<CHUNK>::run([&](auto ci) {
                    constexpr int c = decltype(ci)::value;
                    vc[c] = rem != 0;
                    kc[c] = w * 64 + (vc[c] ? (uint32_t)(__ffsll((unsigned long long)rem) - 1) : 0u);
                    rem &= rem - 1;
                    wc[c] = vc[c] ? mycells[(size_t)kc[c] * 64] : TIMES_NEVER;
                });
                // phase B: arrivals (ballots over senders), closed-form update, sends
                Unrolled<CHUNK>::run([&](auto ci) {
                    constexpr int c = decltype(ci)::value;
                    if (!vc[c]) return;
                    const uint32_t k = kc[c];
                    uint64_t m = s_meta[mbase + k];
                    uint32_t gw = s_gen[mbase + k];
                    if (IPW == 1) { m = uni64(m); gw = uni32(gw); }      // one instance per wave
                    const bool live = running && m_s1(m) != 0;
                    const uint64_t word = (live && real) ? wc[c] : TIMES_NEVER;
                    const uint32_t tE = (uint32_t)(word >> 32) & 0xFFFF, tR = (uint32_t)(word >> 48);
                    const uint32_t dE = t - tE, dR = t - tR;             // steps since this lane sent
                    uint32_t ea = 0, ra = 0;
                    for (uint32_t ds = dset; ds; ds &= ds - 1) {         // only delays some link has
                        const uint32_t i = __ffs(ds) - 1;
                        const uint64_t be = __ballot(dE == i + 1), br = __ballot(dR == i + 1);
                        if (be | br) {
                            const T Li = s_L[i * 64 + lane];
                            ea += popc((T)(be >> segbase) & Li);
                            ra += popc((T)(br >> segbase) & Li);
                        }
                    }
                    bool s_arr = false;
                    if (live && honest) {
                        const uint32_t dt = t - m_tsend(m);
                        if (dt >= 1 && dt <= D) {
                            const bool to_me = !(gw & GEN_RESTRICTED) || ((P.kdst[inst * NK + k] >> d) & 1ull);
                            s_arr = to_me && ((s_L[(dt - 1) * 64 + lane] >> m_sender(m)) & 1);
                        }
                    }
                    const bool has = live && honest && (s_arr || ea || ra);
                    bool echo_send = false, ready_send = false, deliver = false;
                    st_loads += (live && real) ? 1u : 0u;
                    if (has) {
                        const uint32_t gen = gw & GEN_MASK;
                        uint32_t fl = (uint32_t)word & 31, ec = (uint32_t)(word >> 5) & 127, rc = (uint32_t)(word >> 12) & 127;
                        uint32_t tEn = tE, tRn = tR;
                        if ((((uint32_t)word >> 19) & GEN_MASK) != gen) { fl = 0; ec = 0; rc = 0; tEn = NEVER; tRn = NEVER; }
                        brb_cell_update(fl, ec, rc, s_arr, ea, ra, P.T_echo, P.T_amp, P.T_del,
                                        echo_send, ready_send, deliver);
                        if (echo_send) tEn = t;
                        if (ready_send) tRn = t;
                        mycells[(size_t)k * 64] =
                            (uint64_t)fl | ((uint64_t)ec << 5) | ((uint64_t)rc << 12) | ((uint64_t)gen << 19) |
                            ((uint64_t)tEn << 32) | ((uint64_t)tRn << 48);
                        st_arr += ea + ra + (s_arr ? 1u : 0u);
                        st_cells += 1;
                        if (echo_send) st_msgs += n;
                        if (ready_send) st_msgs += n;
                        if (deliver) {
                            st_del += 1; any_del = true;
                            s_dbits[w * 64 + lane] |= 1ull << (k & 63);
                        }
                        if (P.event_cap) {
                            const uint32_t kp = k / Q, s = m_s1(m) - 1u;
                            if (echo_send) log_ev(BRC_EV_SEND, d, BRC_ECHO, kp, s);
                            if (ready_send) log_ev(BRC_EV_SEND, d, BRC_READY, kp, s);
                            if (deliver) log_ev(BRC_EV_DELIVER, d, 0, kp, s);
                        }
                    }
                    lane_active |= has;
                    const bool sent = echo_send || ready_send;
                    if (__ballot(sent)) {
                        const uint32_t os = wave_or(sent ? outset : 0u);
                        if (lane == 0) mark(k, os);
                        const uint32_t myq = seg_max<NPAD>(sent ? t + maxout : 0u);
                        if (live && myq) {
                            if (d == 0 && myq > m_tquiet(m)) s_meta[mbase + k] = m_with_tquiet(m, myq);
                            q_until = max(q_until, myq);
                        }
                    }
                });
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

        // ================= consensus: this step's deliveries in canonical (kp, s) order
        if (any_del) {
            const uint64_t gm0 = (Q >= 64) ? ~0ull : ((1ull << Q) - 1);
            const bool cons = P.protocol == BRC_PROTO_CONSENSUS && honest && running;
#pragma unroll 1
            for (uint32_t w = 0; w < nkw; ++w) {
                uint64_t bits = s_dbits[w * 64 + lane];
                s_dbits[w * 64 + lane] = 0;
                if (!cons) bits = 0;
                while (bits) {
                    const uint32_t b0 = __ffsll((unsigned long long)bits) - 1;
                    const uint32_t base = b0 - (b0 % Q);
                    uint64_t grp = bits & (gm0 << base);
                    bits &= ~(gm0 << base);
                    while (grp) {          // several phase indices of one origin: ascending s
                        uint32_t best = __ffsll((unsigned long long)grp) - 1;
                        if (grp & (grp - 1)) {
                            uint32_t bs = 0xFFFFFFFFu;
                            for (uint64_t x = grp; x; x &= x - 1) {
                                const uint32_t bb = __ffsll((unsigned long long)x) - 1;
                                const uint32_t s1 = m_s1(s_meta[mbase + w * 64 + bb]);
                                if (s1 < bs) { bs = s1; best = bb; }
                            }
                        }
                        grp &= ~(1ull << best);
                        cons_deliver(w * 64 + best);
                    }
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

        // ================= actions stamped t
        const bool inj_mine = do_actions();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

        // ================= per-instance stop conditions
        q_until = seg_max<NPAD>(q_until);
        const uint64_t b_act = __ballot(lane_active || inj_mine) & segbits;
        const uint64_t b_ovf = __ballot(ovf) & segbits;
        const uint64_t b_bad = __ballot(badinj) & segbits;
        const uint64_t b_und = __ballot(honest && dcount < P.round_cap) & segbits;
        if (running) {
            if (b_act) t_stop = t;
            if (b_bad) status = BRC_BADINJ;
            else if (b_ovf) status = BRC_OVERFLOW;
            else if (P.protocol == BRC_PROTO_CONSENSUS && P.round_cap > 0 && !b_und) status = BRC_DONE;
            else if (q_until <= t) {
                bool pending = false;
                for (uint32_t p = inj_pos; p < inj_cnt && !pending; ++p) pending = P.inj[inj_off + p].seg == (uint32_t)seg;
                if (!pending) status = BRC_QUIESCENT;
            }
        }
        if ((uint32_t)lane < nkw) s_act[row * nkw + lane] = 0;
        if (lane == 0) atomicAnd(s_any, ~(1u << row));
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }

    // ---- write back
    {
        const uint64_t mb = item * IPW * (uint64_t)NK;
        for (uint32_t i = lane; i < IPW * NK; i += 64) {
            if (item * IPW + i / NK < P.instances) { P.meta[mb + i] = s_meta[i]; P.mgen[mb + i] = s_gen[i]; }
        }
        for (uint32_t i = lane; i < TS * nkw; i += 64) P.act[item * TS * nkw + i] = s_act[i];
    }
    if (lane == 0) {
        P.actany[item] = *s_any;
        ItemState o = {t, inj_pos, 1u, 0u};
        P.items[item] = o;
    }
    if (honest && P.protocol == BRC_PROTO_CONSENSUS) {
        P.cons0[li] = (uint64_t)(round & 0xFFFF) | ((uint64_t)(phase & 0xFF) << 16) | ((uint64_t)(nvals & 0xFF) << 24) |
                      ((uint64_t)(order & 0xFF) << 32) | ((uint64_t)(vcount & 0xFFFF) << 48);
        P.cons1[li] = (uint64_t)(dcount & 0xFFFF) | ((uint64_t)(frnd & 0xFFFF) << 16) | ((uint64_t)(ft & 0xFFFF) << 32) |
                      ((uint64_t)(fval & 0xFF) << 48) | ((uint64_t)(lval & 0xFF) << 56);
        for (int v = 0; v < 4; ++v) ((T*)P.hmask)[(item * 4 + v) * 64 + lane] = s_hm[v * 64 + lane];
    }
    // statistics: reduce over the segment, its leader writes the instance row
    uint32_t sums[4] = {st_msgs, st_arr, st_cells, st_del};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int o = NPAD / 2; o; o >>= 1) sums[q] += (uint32_t)__shfl_xor((int)sums[q], o);
    }
    if (iex && d == 0) {
        uint64_t* ip = (uint64_t*)&P.inst[inst];
        *ip = (*ip & 0xFFFF000000000000ull) | (uint64_t)(status & 0xFFFF) | ((uint64_t)(t_stop & 0xFFFF) << 16) |
              ((uint64_t)(q_until & 0xFFFF) << 32);
        P.istats[inst * 4 + 0] += sums[0];
        P.istats[inst * 4 + 1] += sums[1];
        P.istats[inst * 4 + 2] += sums[2];
        P.istats[inst * 4 + 3] += sums[3];
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
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < 5; ++q) if (w6[q]) atomicAdd(&P.gcount[q], (unsigned long long)w6[q]);
        if (smax) atomicMax(&P.gcount[5], (unsigned long long)smax);
    }
}

// Byzantine equivocation pattern expanded straight into the CSR lists.
__global__ void expand_equivocate(InjDev* inj, uint32_t* off, uint32_t* cnt, const uint64_t* byz,
                                  uint64_t instances, uint64_t nitems, uint32_t ipw, uint32_t n, uint32_t nv,
                                  uint32_t Q, uint32_t per_item) {
    const uint64_t item = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (item >= nitems) return;
    InjDev* o = inj + item * per_item;
    uint32_t c = 0;
    uint64_t even = 0, odd = 0;
    for (uint32_t dd = 0; dd < n; ++dd) { if (dd & 1) odd |= 1ull << dd; else even |= 1ull << dd; }
    for (int pass = 0; pass < 2; ++pass) {
        for (uint32_t sgi = 0; sgi < ipw; ++sgi) {
            const uint64_t in = item * ipw + sgi;
            if (in >= instances) break;
            const uint64_t bm = byz[in];
            for (uint32_t b = 0; b < n; ++b) {
                if (!((bm >> b) & 1ull)) continue;
                for (uint32_t v = 0; v < 2; ++v) {
                    const uint32_t kp = b * nv + v;
                    InjDev r = {};
                    r.slot = (uint16_t)(kp * Q + 0); r.s = 0; r.seg = (uint8_t)sgi; r.node = (uint8_t)b;
                    r.value = (int8_t)(1 + v);
                    if (pass == 0) {
                        r.t = 0; r.kind = BRC_INJ_SEND; r.type = BRC_SEND; r.dst = v ? odd : even;
                        o[c++] = r;
                    } else {
                        r.t = 1; r.kind = BRC_INJ_MSG; r.dst = ~0ull;
                        r.type = BRC_ECHO; o[c++] = r;
                        r.type = BRC_READY; o[c++] = r;
                    }
                }
            }
        }
    }
    off[item] = (uint32_t)(item * per_item);
    cnt[item] = c;
}

// brc_reset: free every slot but keep its generation; drop every stored send step.
__global__ void reset_slots(uint64_t* meta, uint32_t* mgen, uint64_t keys, uint64_t* cells, uint64_t ncells) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < keys) { meta[i] = 0; mgen[i] &= GEN_MASK; }
    if (i < ncells) cells[i] = (cells[i] & 0xFFFFFFFFull) | TIMES_NEVER;
}

__global__ void fill_u64(uint64_t* p, uint64_t v, uint64_t count) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) p[i] = v;
}

// ------------------------------------------------------------------------------------ host
struct Engine {
    brc_config cfg;
    int npad = 0, dm = 0, ipw = 0, nkw_t = 0;
    uint32_t NK = 0, nkw = 0, msize = 0, lds_bytes = 0;
    uint64_t nitems = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    float last_ms = 0.f;
    std::string err;
    uint64_t* cells = nullptr;
    uint64_t* meta = nullptr; uint32_t* mgen = nullptr; uint64_t* kdst = nullptr;
    uint64_t* act = nullptr; uint32_t* actany = nullptr; ItemState* items = nullptr;
    InstState* inst = nullptr; uint64_t* istats = nullptr;
    uint64_t* cons0 = nullptr; uint64_t* cons1 = nullptr; void* hmask = nullptr;
    InjDev* inj = nullptr; uint32_t* inj_off = nullptr; uint32_t* inj_cnt = nullptr; size_t inj_capacity = 0;
    uint64_t* byz = nullptr; int8_t* prop = nullptr;
    brc_event* events = nullptr; unsigned long long* event_count = nullptr;
    unsigned long long* gcount = nullptr;
    std::vector<std::vector<InjDev>> pending;   // per item: uploaded-but-unconsumed + new
    bool inj_dirty = false, pattern_active = false;
    uint64_t gen_budget = 0;                     // generation advance bound since the last full clear
    std::vector<std::pair<uint64_t, uint32_t>> send_keys;   // (instance, kp<<16|s) of injected SENDs
};

#define HIPCHK(e, x)                                                                   \
    do {                                                                               \
        hipError_t _r = (x);                                                           \
        if (_r != hipSuccess) {                                                        \
            (e)->err = std::string(#x) + ": " + hipGetErrorString(_r);                 \
            return BRC_E_HIP;                                                          \
        }                                                                              \
    } while (0)

static int pick_npad(uint32_t n) {
    int p = 4;
    while ((uint32_t)p < n) p *= 2;
    return p;
}

static int pick_dm(uint32_t d) { return d <= 4 ? 4 : d <= 8 ? 8 : 16; }

template <typename F>
static int dispatch(int npad, int dm, F&& f) {
#define BRC_CASE(NP, DMX) if (npad == NP && dm == DMX) return f(brc_kernel<NP, DMX>);
#ifdef BRC_ONLY_64_8
    BRC_CASE(64, 8)
#else
    BRC_CASE(4, 4) BRC_CASE(4, 8) BRC_CASE(4, 16)
    BRC_CASE(8, 4) BRC_CASE(8, 8) BRC_CASE(8, 16)
    BRC_CASE(16, 4) BRC_CASE(16, 8) BRC_CASE(16, 16)
    BRC_CASE(32, 4) BRC_CASE(32, 8) BRC_CASE(32, 16)
    BRC_CASE(64, 4) BRC_CASE(64, 8) BRC_CASE(64, 16)
#endif
#undef BRC_CASE
    return BRC_E_INVALID;
}

static void free_all(Engine* e) {
    void* ps[] = {e->cells, e->meta, e->mgen, e->kdst, e->act, e->actany, e->items, e->inst, e->istats,
                  e->cons0, e->cons1, e->hmask, e->inj, e->inj_off, e->inj_cnt, e->byz, e->prop, e->events,
                  e->event_count, e->gcount};
    for (void* p : ps) if (p) (void)hipFree(p);
    if (e->ev0) (void)hipEventDestroy(e->ev0);
    if (e->ev1) (void)hipEventDestroy(e->ev1);
    if (e->stream) (void)hipStreamDestroy(e->stream);
}

static int clear_state(Engine* e, bool full) {
    const size_t cells = (size_t)e->nitems * e->NK * 64;
    const size_t keys = (size_t)e->cfg.instances * e->NK;
    if (full) {
        hipLaunchKernelGGL(fill_u64, dim3((uint32_t)((cells + 255) / 256)), dim3(256), 0, e->stream, e->cells,
                           TIMES_NEVER, (uint64_t)cells);
        HIPCHK(e, hipGetLastError());
        HIPCHK(e, hipMemsetAsync(e->meta, 0, keys * 8, e->stream));
        HIPCHK(e, hipMemsetAsync(e->mgen, 0, keys * 4, e->stream));
        e->gen_budget = 0;
    } else {
        // cells keep their generation tags; every slot keeps (and will bump) its own, so
        // every cell written before the reset reads as stale; send steps are dropped since
        // the step counter restarts at 0
        const size_t m = std::max(cells, keys);
        hipLaunchKernelGGL(reset_slots, dim3((uint32_t)((m + 255) / 256)), dim3(256), 0, e->stream, e->meta, e->mgen,
                           (uint64_t)keys, e->cells, (uint64_t)cells);
        HIPCHK(e, hipGetLastError());
    }
    HIPCHK(e, hipMemsetAsync(e->act, 0, (size_t)e->nitems * TS * e->nkw * 8, e->stream));
    HIPCHK(e, hipMemsetAsync(e->actany, 0, (size_t)e->nitems * 4, e->stream));
    HIPCHK(e, hipMemsetAsync(e->items, 0, (size_t)e->nitems * sizeof(ItemState), e->stream));
    HIPCHK(e, hipMemsetAsync(e->inst, 0, (size_t)e->cfg.instances * sizeof(InstState), e->stream));
    HIPCHK(e, hipMemsetAsync(e->istats, 0, (size_t)e->cfg.instances * 4 * 8, e->stream));
    HIPCHK(e, hipMemsetAsync(e->cons0, 0, (size_t)e->nitems * 64 * 8, e->stream));
    HIPCHK(e, hipMemsetAsync(e->cons1, 0, (size_t)e->nitems * 64 * 8, e->stream));
    HIPCHK(e, hipMemsetAsync(e->hmask, 0, (size_t)e->nitems * 4 * 64 * e->msize, e->stream));
    HIPCHK(e, hipMemsetAsync(e->gcount, 0, 8 * 8, e->stream));
    if (e->event_count) HIPCHK(e, hipMemsetAsync(e->event_count, 0, 8, e->stream));
    return BRC_OK;
}

static int upload_injections(Engine* e) {
    if (!e->inj_dirty) return BRC_OK;
    std::vector<ItemState> its(e->nitems);
    HIPCHK(e, hipMemcpyAsync(its.data(), e->items, e->nitems * sizeof(ItemState), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    size_t total = 0;
    std::vector<uint32_t> off(e->nitems), cnt(e->nitems);
    for (uint64_t i = 0; i < e->nitems; ++i) {
        auto& v = e->pending[i];
        const size_t consumed = std::min<size_t>(its[i].inj_pos, v.size());   // part of the last upload
        v.erase(v.begin(), v.begin() + consumed);
        std::stable_sort(v.begin(), v.end(), [](const InjDev& a, const InjDev& b) { return a.t < b.t; });
        off[i] = (uint32_t)total; cnt[i] = (uint32_t)v.size();
        total += v.size();
        its[i].inj_pos = 0;
    }
    if (total > e->inj_capacity) {
        if (e->inj) (void)hipFree(e->inj);
        e->inj = nullptr;
        HIPCHK(e, hipMalloc(&e->inj, std::max<size_t>(total, 1) * sizeof(InjDev)));
        e->inj_capacity = total;
    }
    std::vector<InjDev> flat;
    flat.reserve(total);
    for (auto& v : e->pending) flat.insert(flat.end(), v.begin(), v.end());
    if (total) HIPCHK(e, hipMemcpyAsync(e->inj, flat.data(), total * sizeof(InjDev), hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->inj_off, off.data(), e->nitems * 4, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->inj_cnt, cnt.data(), e->nitems * 4, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->items, its.data(), e->nitems * sizeof(ItemState), hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->inj_dirty = false;
    return BRC_OK;
}

static int apply_pattern(Engine* e) {
    if (e->cfg.byz_pattern != BRC_BYZ_EQUIVOCATE) return BRC_OK;
    const uint32_t cap = (uint32_t)e->ipw * 6u * e->cfg.n;   // worst case: every replica Byzantine
    const size_t total = (size_t)e->nitems * cap;
    if (total > e->inj_capacity) {
        if (e->inj) (void)hipFree(e->inj);
        e->inj = nullptr;
        HIPCHK(e, hipMalloc(&e->inj, total * sizeof(InjDev)));
        e->inj_capacity = total;
    }
    const uint32_t blocks = (uint32_t)((e->nitems + 127) / 128);
    hipLaunchKernelGGL(expand_equivocate, dim3(blocks), dim3(128), 0, e->stream, e->inj, e->inj_off, e->inj_cnt,
                       e->byz, e->cfg.instances, e->nitems, (uint32_t)e->ipw, e->cfg.n, e->cfg.variants,
                       e->cfg.key_window, cap);
    HIPCHK(e, hipGetLastError());
    e->pattern_active = true;
    return BRC_OK;
}

}  // namespace

extern "C" {

int brc_abi_version(void) { return BRC_ABI_VERSION; }

int brc_device_count(int* count) {
    if (!count) return BRC_E_INVALID;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *count = c;
    return BRC_OK;
}

const char* brc_last_error(void* h) {
    if (!h) return "null engine";
    return static_cast<Engine*>(h)->err.c_str();
}

int brc_create(const brc_config* cfg, void** out) {
    if (!cfg || !out) return BRC_E_INVALID;
    *out = nullptr;
    const brc_config& c = *cfg;
    if (c.n < 1 || c.n > 64 || c.instances == 0 || c.delay_max < 1 || c.delay_max > 16 ||
        c.step_cap > STEP_LIMIT || c.peer_mode != BRC_PEER_SENDER ||
        (c.protocol != BRC_PROTO_BRB && c.protocol != BRC_PROTO_CONSENSUS) || c.delay_model > BRC_DELAY_GEOMETRIC ||
        (c.delay_model == BRC_DELAY_CONST && (c.delay_const < 1 || c.delay_const > c.delay_max)) ||
        !(c.key_window == 2 || c.key_window == 4 || c.key_window == 8) ||
        !(c.variants == 1 || c.variants == 2 || c.variants == 4) || c.key_window * c.variants > 8 ||
        c.f >= c.n || (c.byz_pattern == BRC_BYZ_EQUIVOCATE && c.variants < 2) ||
        (c.byz_pattern != BRC_BYZ_NONE && c.byz_pattern != BRC_BYZ_EQUIVOCATE) ||
        c.proposals > BRC_PROPOSALS_LOADED)
        return BRC_E_INVALID;
    Engine* e = new Engine();
    e->cfg = c;
    e->npad = pick_npad(c.n);
    e->dm = pick_dm(c.delay_max);
    e->ipw = 64 / e->npad;
    e->nkw_t = e->npad / 8 < 1 ? 1 : e->npad / 8;
    e->NK = (uint32_t)e->npad * c.variants * c.key_window;
    e->nkw = (e->NK + 63) / 64;
    e->msize = e->npad <= 8 ? 1 : (uint32_t)e->npad / 8;
    e->nitems = (c.instances + e->ipw - 1) / e->ipw;
    const uint32_t l_words = ((uint32_t)e->dm * 64 * e->msize + 7) / 8;
    const uint32_t h_words = (4 * 64 * e->msize + 7) / 8;
    const uint32_t per_wave_words = e->ipw * e->NK + TS * e->nkw + 64 * e->nkw + l_words + h_words + (e->ipw * e->NK + 2) / 2 + 1;
    e->lds_bytes = per_wave_words * 8 * WPB;
    if (e->nkw > (uint32_t)e->nkw_t || e->nitems > 0x7FFFFFFFull * WPB || e->lds_bytes > 160 * 1024) { delete e; return BRC_E_INVALID; }
    auto fail = [&](int code) { free_all(e); delete e; return code; };
    if (hipSetDevice(c.device) != hipSuccess) { delete e; return BRC_E_HIP; }
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) return fail(BRC_E_HIP);
    if (hipEventCreate(&e->ev0) != hipSuccess || hipEventCreate(&e->ev1) != hipSuccess) return fail(BRC_E_HIP);
    const size_t cells = (size_t)e->nitems * e->NK * 64;
    const size_t keys = (size_t)c.instances * e->NK;
    struct A { void** p; size_t bytes; } allocs[] = {
        {(void**)&e->cells, cells * 8}, {(void**)&e->meta, keys * 8}, {(void**)&e->mgen, keys * 4},
        {(void**)&e->kdst, keys * 8}, {(void**)&e->act, (size_t)e->nitems * TS * e->nkw * 8},
        {(void**)&e->actany, (size_t)e->nitems * 4}, {(void**)&e->items, (size_t)e->nitems * sizeof(ItemState)},
        {(void**)&e->inst, c.instances * sizeof(InstState)}, {(void**)&e->istats, c.instances * 32},
        {(void**)&e->cons0, (size_t)e->nitems * 512}, {(void**)&e->cons1, (size_t)e->nitems * 512},
        {&e->hmask, (size_t)e->nitems * 256 * e->msize}, {(void**)&e->inj_off, (size_t)e->nitems * 4},
        {(void**)&e->inj_cnt, (size_t)e->nitems * 4}, {(void**)&e->byz, c.instances * 8}, {(void**)&e->gcount, 64},
    };
    for (auto& a : allocs)
        if (hipMalloc(a.p, std::max<size_t>(a.bytes, 8)) != hipSuccess) return fail(BRC_E_NOMEM);
    if (c.event_capacity) {
        if (hipMalloc(&e->events, (size_t)c.event_capacity * sizeof(brc_event)) != hipSuccess) return fail(BRC_E_NOMEM);
        if (hipMalloc(&e->event_count, 8) != hipSuccess) return fail(BRC_E_NOMEM);
    }
    if (hipMemsetAsync(e->inj_off, 0, (size_t)e->nitems * 4, e->stream) != hipSuccess) return fail(BRC_E_HIP);
    if (hipMemsetAsync(e->inj_cnt, 0, (size_t)e->nitems * 4, e->stream) != hipSuccess) return fail(BRC_E_HIP);
    if (hipMemsetAsync(e->kdst, 0, keys * 8, e->stream) != hipSuccess) return fail(BRC_E_HIP);
    {
        std::vector<uint64_t> bm(c.instances, c.byzantine_mask & ((c.n >= 64) ? ~0ull : ((1ull << c.n) - 1)));
        if (hipMemcpy(e->byz, bm.data(), c.instances * 8, hipMemcpyHostToDevice) != hipSuccess) return fail(BRC_E_HIP);
    }
    if (clear_state(e, true) != BRC_OK) return fail(BRC_E_HIP);
    e->pending.assign(e->nitems, {});
    if (apply_pattern(e) != BRC_OK) return fail(BRC_E_HIP);
    if (hipStreamSynchronize(e->stream) != hipSuccess) return fail(BRC_E_HIP);
    *out = e;
    return BRC_OK;
}

int brc_load_proposals(void* h, const int8_t* proposals) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || !proposals) return BRC_E_INVALID;
    if (e->cfg.proposals != BRC_PROPOSALS_LOADED) return BRC_E_STATE;
    const size_t bytes = e->cfg.instances * e->cfg.n;
    for (size_t i = 0; i < bytes; ++i)
        if (proposals[i] < 0 || proposals[i] > 3) { e->err = "proposal value ids must be in [0, 3]"; return BRC_E_INVALID; }
    if (!e->prop) HIPCHK(e, hipMalloc(&e->prop, bytes));
    HIPCHK(e, hipMemcpyAsync(e->prop, proposals, bytes, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return BRC_OK;
}

int brc_load_byzantine(void* h, const uint64_t* masks) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || !masks) return BRC_E_INVALID;
    const uint64_t lim = (e->cfg.n >= 64) ? ~0ull : ((1ull << e->cfg.n) - 1);
    std::vector<uint64_t> bm(masks, masks + e->cfg.instances);
    for (auto& m : bm) m &= lim;
    HIPCHK(e, hipMemcpyAsync(e->byz, bm.data(), e->cfg.instances * 8, hipMemcpyHostToDevice, e->stream));
    if (e->cfg.byz_pattern) { int rc = apply_pattern(e); if (rc) return rc; }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return BRC_OK;
}

int brc_inject(void* h, const brc_injection* list, size_t count) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || (!list && count)) return BRC_E_INVALID;
    if (e->pattern_active) { e->err = "explicit injections cannot be combined with byz_pattern"; return BRC_E_STATE; }
    const brc_config& c = e->cfg;
    const uint64_t all = (c.n >= 64) ? ~0ull : ((1ull << c.n) - 1);
    std::vector<ItemState> its;
    std::vector<InstState> ist;
    bool have_state = false;
    std::vector<uint64_t> reopen;
    std::vector<InjDev> staged;
    std::vector<uint64_t> staged_item;
    std::vector<std::pair<uint64_t, uint32_t>> new_sends;
    for (size_t i = 0; i < count; ++i) {
        const brc_injection& x = list[i];
        if (x.instance >= c.instances || x.node >= c.n || x.t > c.step_cap) { e->err = "injection out of range"; return BRC_E_INVALID; }
        if (x.value < 0 || x.value > 3 || x.s >= 0xFFFE) { e->err = "value id / phase index out of range"; return BRC_E_INVALID; }
        InjDev r = {};
        r.t = x.t; r.kind = (uint8_t)x.kind; r.type = (uint8_t)x.type; r.node = (uint8_t)x.node;
        r.seg = (uint8_t)(x.instance % e->ipw); r.value = (int8_t)x.value; r.s = (uint16_t)x.s;
        r.dst = x.dst_mask & all;
        if (x.kind == BRC_INJ_PROPOSE) {
            if (c.protocol != BRC_PROTO_CONSENSUS) { e->err = "PROPOSE needs the consensus protocol"; return BRC_E_INVALID; }
        } else if (x.kind == BRC_INJ_SEND || x.kind == BRC_INJ_MSG || x.kind == BRC_INJ_KEY) {
            if (x.kp >= c.n * c.variants) { e->err = "kp out of range"; return BRC_E_INVALID; }
            r.slot = (uint16_t)(x.kp * c.key_window + (x.s % c.key_window));
            if (x.kind == BRC_INJ_MSG) {
                if (x.type != BRC_ECHO && x.type != BRC_READY) { e->err = "MSG type must be ECHO or READY"; return BRC_E_INVALID; }
                if ((x.dst_mask & all) != all) { e->err = "ECHO/READY injections must address every peer"; return BRC_E_UNSUPPORTED; }
            } else if (x.kind == BRC_INJ_SEND) {
                // one SEND per key: a second SEND (other sender / destinations) is not modelled
                auto key = std::make_pair(x.instance, (uint32_t)(x.kp * 0x10000u + x.s));
                if (std::find(e->send_keys.begin(), e->send_keys.end(), key) != e->send_keys.end() ||
                    std::find(new_sends.begin(), new_sends.end(), key) != new_sends.end()) {
                    e->err = "a key can be SENT only once";
                    return BRC_E_UNSUPPORTED;
                }
                new_sends.push_back(key);
            }
        } else {
            e->err = "unknown injection kind";
            return BRC_E_INVALID;
        }
        if (!have_state) {
            its.resize(e->nitems); ist.resize(c.instances);
            HIPCHK(e, hipMemcpyAsync(its.data(), e->items, e->nitems * sizeof(ItemState), hipMemcpyDeviceToHost, e->stream));
            HIPCHK(e, hipMemcpyAsync(ist.data(), e->inst, c.instances * sizeof(InstState), hipMemcpyDeviceToHost, e->stream));
            HIPCHK(e, hipStreamSynchronize(e->stream));
            have_state = true;
        }
        const uint64_t item = x.instance / e->ipw;
        if (its[item].initialized != 0 && x.t < its[item].t) { e->err = "injection time is before the instance's current step"; return BRC_E_STATE; }
        if (ist[x.instance].status == BRC_QUIESCENT) reopen.push_back(x.instance);
        else if (ist[x.instance].status != BRC_RUNNING) { e->err = "instance already stopped"; return BRC_E_STATE; }
        staged.push_back(r);
        staged_item.push_back(item);
    }
    for (size_t i = 0; i < staged.size(); ++i) e->pending[staged_item[i]].push_back(staged[i]);
    e->send_keys.insert(e->send_keys.end(), new_sends.begin(), new_sends.end());
    for (uint64_t in : reopen) {
        ist[in].status = BRC_RUNNING;
        HIPCHK(e, hipMemcpyAsync(&e->inst[in], &ist[in], sizeof(InstState), hipMemcpyHostToDevice, e->stream));
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (count) e->inj_dirty = true;
    return BRC_OK;
}

int brc_run(void* h, uint32_t max_steps, uint32_t* running_left) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return BRC_E_INVALID;
    const brc_config& c = e->cfg;
    HIPCHK(e, hipSetDevice(c.device));
    if (c.protocol == BRC_PROTO_CONSENSUS && c.proposals == BRC_PROPOSALS_LOADED && !e->prop) {
        e->err = "proposals not loaded";
        return BRC_E_STATE;
    }
    int rc = upload_injections(e);
    if (rc) return rc;
    Params P;
    memset(&P, 0, sizeof(P));
    P.n = c.n; P.f = c.f; P.D = c.delay_max; P.Q = c.key_window; P.NV = c.variants; P.NK = e->NK; P.nkw = e->nkw;
    P.protocol = c.protocol; P.delay_model = c.delay_model; P.dconst = c.delay_const; P.round_cap = c.round_cap;
    P.step_cap = c.step_cap; P.proposals = c.proposals;
    P.T_echo = (c.n + c.f) / 2 + 1;     // len > (N+f)/2        core/brbroadcast.py:95
    P.T_amp = c.f + 1;                  // len > f              :118
    P.T_del = 2 * c.f + 1;              // len > 2f             :111
    P.T_cnt = c.n - c.f + 1;            // value_count > N-f    core/byzantinerandomizedconsensus.py:71,86
    P.bound_p1 = c.n + c.f;             // 2|hosts| > N+f       :73
    P.bound_p2 = 4 * c.f;               // 2|hosts| > 4f        :88
    P.seed = c.seed; P.inst_offset = c.instance_offset; P.instances = c.instances; P.nitems = e->nitems;
    P.max_steps = max_steps ? max_steps : 0xFFFFFFFFu;
    P.event_cap = c.event_capacity;
    P.cells = e->cells; P.meta = e->meta; P.mgen = e->mgen; P.kdst = e->kdst;
    P.act = e->act; P.actany = e->actany; P.items = e->items;
    P.inst = e->inst; P.istats = e->istats; P.cons0 = e->cons0; P.cons1 = e->cons1; P.hmask = e->hmask;
    P.inj = e->inj; P.inj_off = e->inj_off; P.inj_cnt = e->inj_cnt; P.byz = e->byz; P.prop = e->prop;
    P.events = e->events; P.event_count = e->event_count; P.gcount = e->gcount;
    HIPCHK(e, hipEventRecord(e->ev0, e->stream));
    const uint32_t blocks = (uint32_t)((e->nitems + WPB - 1) / WPB);
    rc = dispatch(e->npad, e->dm, [&](auto kern) {
        if (e->lds_bytes > 64 * 1024 &&
            hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)e->lds_bytes) != hipSuccess)
            return (int)BRC_E_HIP;
        kern<<<dim3(blocks), dim3(64 * WPB), e->lds_bytes, e->stream>>>(P);
        return 0;
    });
    if (rc) { e->err = "no kernel instantiation"; return rc; }
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipEventRecord(e->ev1, e->stream));
    HIPCHK(e, hipEventSynchronize(e->ev1));
    HIPCHK(e, hipEventElapsedTime(&e->last_ms, e->ev0, e->ev1));
    unsigned long long smax = 0;
    HIPCHK(e, hipMemcpy(&smax, e->gcount + 5, 8, hipMemcpyDeviceToHost));
    e->gen_budget += smax / c.key_window + 2;   // allocations of any one slot in this run
    if (running_left) {
        std::vector<InstState> ist(c.instances);
        HIPCHK(e, hipMemcpy(ist.data(), e->inst, c.instances * sizeof(InstState), hipMemcpyDeviceToHost));
        uint32_t r = 0;
        for (auto& s : ist) r += s.status == BRC_RUNNING;
        *running_left = r;
    }
    return BRC_OK;
}

int brc_reset(void* h) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return BRC_E_INVALID;
    HIPCHK(e, hipSetDevice(e->cfg.device));
    int rc = clear_state(e, e->gen_budget >= GEN_FULL_CLEAR);
    if (rc) return rc;
    for (auto& v : e->pending) v.clear();
    e->send_keys.clear();
    if (e->pattern_active) {
        e->pattern_active = false;
        rc = apply_pattern(e);
        if (rc) return rc;
    } else {
        HIPCHK(e, hipMemsetAsync(e->inj_off, 0, (size_t)e->nitems * 4, e->stream));
        HIPCHK(e, hipMemsetAsync(e->inj_cnt, 0, (size_t)e->nitems * 4, e->stream));
    }
    e->inj_dirty = false;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return BRC_OK;
}

int brc_read_instances(void* h, uint64_t first, uint64_t count, brc_instance_result* out) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || !out || first + count > e->cfg.instances) return BRC_E_INVALID;
    if (!count) return BRC_OK;
    const brc_config& c = e->cfg;
    std::vector<InstState> ist(count);
    std::vector<uint64_t> st(count * 4);
    HIPCHK(e, hipMemcpyAsync(ist.data(), e->inst + first, count * sizeof(InstState), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipMemcpyAsync(st.data(), e->istats + first * 4, count * 32, hipMemcpyDeviceToHost, e->stream));
    const uint64_t i0 = first / e->ipw, i1 = (first + count - 1) / e->ipw;
    std::vector<ItemState> its(i1 - i0 + 1);
    HIPCHK(e, hipMemcpyAsync(its.data(), e->items + i0, its.size() * sizeof(ItemState), hipMemcpyDeviceToHost, e->stream));
    std::vector<uint64_t> c1((i1 - i0 + 1) * 64);
    std::vector<uint64_t> bm(count);
    HIPCHK(e, hipMemcpyAsync(bm.data(), e->byz + first, count * 8, hipMemcpyDeviceToHost, e->stream));
    if (c.protocol == BRC_PROTO_CONSENSUS)
        HIPCHK(e, hipMemcpyAsync(c1.data(), e->cons1 + i0 * 64, c1.size() * 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    for (uint64_t i = 0; i < count; ++i) {
        const uint64_t in = first + i, item = in / e->ipw, seg = in % e->ipw;
        brc_instance_result& r = out[i];
        r.status = ist[i].status; r.t_stop = ist[i].t_stop; r.t_now = its[item - i0].t;
        r.msgs_sent = st[i * 4 + 0]; r.arrivals = st[i * 4 + 1]; r.cell_steps = st[i * 4 + 2]; r.deliveries = st[i * 4 + 3];
        uint32_t dec = c.protocol == BRC_PROTO_CONSENSUS ? 1u : 0u;
        if (dec)
            for (uint32_t dd = 0; dd < c.n; ++dd) {
                if ((bm[i] >> dd) & 1ull) continue;
                if ((c1[(item - i0) * 64 + seg * e->npad + dd] & 0xFFFF) == 0) { dec = 0; break; }
            }
        r.decided = dec;
    }
    return BRC_OK;
}

int brc_read_replicas(void* h, uint64_t first, uint64_t count, brc_replica_result* out) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || !out || first + count > e->cfg.instances) return BRC_E_INVALID;
    if (!count) return BRC_OK;
    const uint64_t i0 = first / e->ipw, i1 = (first + count - 1) / e->ipw;
    const size_t nl = (i1 - i0 + 1) * 64;
    std::vector<uint64_t> c0(nl), c1(nl);
    HIPCHK(e, hipMemcpyAsync(c0.data(), e->cons0 + i0 * 64, nl * 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipMemcpyAsync(c1.data(), e->cons1 + i0 * 64, nl * 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    for (uint64_t i = 0; i < count; ++i) {
        const uint64_t in = first + i, item = in / e->ipw, seg = in % e->ipw;
        for (uint32_t dd = 0; dd < e->cfg.n; ++dd) {
            const size_t l = (item - i0) * 64 + seg * e->npad + dd;
            brc_replica_result& r = out[i * e->cfg.n + dd];
            const uint64_t a = c0[l], b = c1[l];
            r.round = a & 0xFFFF; r.phase = (a >> 16) & 0xFF; r.value_count = (a >> 48) & 0xFFFF;
            r.decide_count = b & 0xFFFF; r.first_decide_round = (b >> 16) & 0xFFFF;
            r.first_decide_t = (b >> 32) & 0xFFFF;
            r.first_decide_value = r.decide_count ? (int32_t)((b >> 48) & 0xFF) : -1;
            r.last_decide_value = r.decide_count ? (int32_t)((b >> 56) & 0xFF) : -1;
        }
    }
    return BRC_OK;
}

int brc_read_events(void* h, brc_event* out, size_t cap, size_t* count) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || !count) return BRC_E_INVALID;
    if (!e->event_count) { *count = 0; return BRC_OK; }
    unsigned long long n = 0;
    HIPCHK(e, hipMemcpy(&n, e->event_count, 8, hipMemcpyDeviceToHost));
    *count = (size_t)n;
    const size_t avail = std::min<size_t>((size_t)n, e->cfg.event_capacity);
    if (out && cap) HIPCHK(e, hipMemcpy(out, e->events, std::min(avail, cap) * sizeof(brc_event), hipMemcpyDeviceToHost));
    return BRC_OK;
}

int brc_read_stats(void* h, brc_stats* out) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || !out) return BRC_E_INVALID;
    memset(out, 0, sizeof(*out));
    const uint64_t N = e->cfg.instances;
    std::vector<brc_instance_result> r(N);
    int rc = brc_read_instances(h, 0, N, r.data());
    if (rc) return rc;
    out->instances = N;
    for (auto& x : r) {
        out->running += x.status == BRC_RUNNING;
        out->done += x.status == BRC_DONE;
        out->quiescent += x.status == BRC_QUIESCENT;
        out->stepcap += x.status == BRC_STEPCAP;
        out->overflow += x.status == BRC_OVERFLOW || x.status == BRC_BADINJ;
        out->decided += x.decided;
        out->msgs_sent += x.msgs_sent; out->arrivals += x.arrivals; out->cell_steps += x.cell_steps;
        out->deliveries += x.deliveries;
        out->max_t = std::max<uint64_t>(out->max_t, x.t_now);
    }
    unsigned long long gc[8] = {0};
    HIPCHK(e, hipMemcpy(gc, e->gcount, 64, hipMemcpyDeviceToHost));
    out->lane_loads = gc[4];
    if (e->cfg.protocol == BRC_PROTO_CONSENSUS) {
        std::vector<uint64_t> c1((size_t)e->nitems * 64);
        std::vector<uint64_t> bm(N);
        HIPCHK(e, hipMemcpy(c1.data(), e->cons1, c1.size() * 8, hipMemcpyDeviceToHost));
        HIPCHK(e, hipMemcpy(bm.data(), e->byz, N * 8, hipMemcpyDeviceToHost));
        for (uint64_t in = 0; in < N; ++in) {
            const uint64_t item = in / e->ipw, seg = in % e->ipw;
            for (uint32_t dd = 0; dd < e->cfg.n; ++dd)
                if (!((bm[in] >> dd) & 1ull)) out->decide_rounds_sum += (c1[item * 64 + seg * e->npad + dd] >> 16) & 0xFFFF;
        }
    }
    if (e->event_count) {
        unsigned long long n = 0;
        HIPCHK(e, hipMemcpy(&n, e->event_count, 8, hipMemcpyDeviceToHost));
        out->events_dropped = n > e->cfg.event_capacity ? n - e->cfg.event_capacity : 0;
    }
    return BRC_OK;
}

int brc_last_kernel_ms(void* h, float* ms) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || !ms) return BRC_E_INVALID;
    *ms = e->last_ms;
    return BRC_OK;
}

void brc_destroy(void* h) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return;
    (void)hipSetDevice(e->cfg.device);
    (void)hipStreamSynchronize(e->stream);
    free_all(e);
    delete e;
}

}  // extern "C"
