// brc_step_wide.h -- the large-committee step kernel (gfx950): n in (64, 256], SURVEY §8(d) cfg5.
//
// Same protocol, same lock-step network and the same per-cell closed form as brc_step.h, but one
// instance no longer fits a wavefront: a workgroup of NW = NPAD / 64 waves simulates ONE
// instance, thread d = receiver d = sender d = consensus replica d.  What a 64-lane ballot did in
// the narrow kernel becomes a per-wave ballot plus an LDS exchange:
//   * arrivals of a key: every wave ballots "my ECHO/READY was sent `dly` steps ago" for each link
//     delay present, lane 0 writes the word to LDS (double-buffered per chunk of keys), one
//     workgroup barrier, then every receiver pops (ballot words & its link-delay masks);
//   * sends: each wave marks the activity ring for its own senders (idempotent LDS atomics), the
//     key's t_quiet is raised with a 64-bit LDS atomicMax on the packed metadata word (only that
//     field changes in the BRB phase, so the max of the words is the max of the t_quiet fields);
//   * per-step control (next step, status, rows of the ring) is reduced once per step through a
//     rotating set of LDS slots (one barrier per reduction).
// Link-delay masks do not fit LDS at n = 256 (16 delays x 256 receivers x 32 B), so each thread
// keeps its links' delay CODES as NPL bit planes in registers (n bits per plane) and rebuilds the
// mask of one delay with NPL ANDs per 64-bit word when a ballot word is non-zero.
//
// Cell word (one u64 per (receiver, key)): flags:5 | |E|:8 | |R|:8 | (unused):11 | t_echo_sent:16 |
// t_ready_sent:16.  |E| saturates at 255 (only |E| >= T_echo <= 171 is ever tested) and |R| is
// below T_del until the cell delivers, after which it is never read (core/brbroadcast.py:74).
//
// Hot path replaced (reference = sithu/ByzantineRandomizedConsensus): as brc_step.h --
//   brb_cell_update()  <- core/brbroadcast.py:60-119
//   consensus pass     <- core/byzantinerandomizedconsensus.py:53-106
//   send_key()         <- core/byzantinerandomizedconsensus.py:43-51, base/broadcast.py:17-40
#pragma once
#include "brc_step.h"

#ifndef BRC_WIDE_PLANE_FENCE
#define BRC_WIDE_PLANE_FENCE 0   // bit-plane matching: a scheduling barrier after each ballot word (A/B round 4:
#endif                               // 59 instead of 73 spills at DM = 16, but 368 vs 338 ms on cfg5 geometric)
#ifndef BRC_WIDE_WAVES16
#define BRC_WIDE_WAVES16 BRC_WIDE_WAVES   // waves per SIMD the DM = 16 (geometric) instantiations allow (2: no
#endif                                     // spills at 206 VGPRs, but 444 vs 338 ms -- occupancy wins, A/B round 4)
#ifndef BRC_WIDE_MSTORE
#define BRC_WIDE_MSTORE 1    // exec-masked cell stores (0: whole-row stores, unchanged words written back)
#endif

namespace brc {

// waves per SIMD the register allocation must allow (<= 168 VGPRs at 3): with generation-free cells
// and a byte-wide SEND queue a cfg5 workgroup takes 48-51 KB of LDS, so three fit a CU
#ifndef BRC_WIDE_WAVES
#define BRC_WIDE_WAVES 3
#endif


__device__ __forceinline__ uint64_t wave_or64(uint64_t x) {
#pragma unroll
    for (int o = 32; o; o >>= 1) x |= (uint64_t)__shfl_xor((unsigned long long)x, o);
    return x;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
#pragma unroll
    for (int o = 32; o; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o));
    return x;
}

// WV: waves per SIMD the register allocation must allow (0: BRC_WIDE_WAVES / BRC_WIDE_WAVES16).  4 is
// the instantiation for DM <= 8 under the constant / slow-set models (no delay-code planes in registers):
// 128 VGPRs, and with the DM-sized ring and 2-word delivery bitmaps a cfg5 workgroup fits 40 KB of LDS, so
// four workgroups share a CU (cfg5 const: 37.8 -> 31.9 ms, A/B round 5; uniform planes lose: 137.7 -> 139.8)
template <int NPAD, int DM, bool EV, int MODE, int WV = 0>
__global__ __launch_bounds__(NPAD, (EV ? BRC_MIN_WAVES_EV : WV ? WV : DM == 16 ? BRC_WIDE_WAVES16 : BRC_WIDE_WAVES)) void brc_step_wide(const Params* __restrict__ pp) {
    const Params& P = *pp;
    constexpr bool SPEC = MODE == BRC_MODE_SPEC, BEB = MODE == BRC_MODE_BEB, CONN = MODE == KMODE_CONN;
    // u64 words per cell: CONN adds the lane's ECHO and READY send-count rings (Ring16, brc_step.h)
    constexpr uint32_t CW = CONN ? 5 : 1;
    // DM > 8 (geometric): in a given wave most delays carry no send, so each wave publishes which
    // did (pmw) and the readers visit only those; with DM <= 8 that bookkeeping costs more than it
    // saves (measured cfg5: geometric -20% kernel time, const/uniform +5%)
    constexpr bool SPARSE_D = DM > 8;
    constexpr int NW = NPAD / 64;
    constexpr uint32_t TS = ring_steps(DM);              // activity-ring rows (> the largest delay)
    constexpr int NPL = npl_of(DM);                      // bit planes of a link's delay code
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];

    const int tid = threadIdx.x, wid = tid / 64, lane = tid % 64;
    const uint64_t inst = blockIdx.x;
    if (inst >= P.instances) return;            // whole workgroup exits
    const uint32_t n = P.n, NK = P.NK, Q = P.Q, NV = P.NV, D = P.D, nkw = P.nkw, nL = P.nL;
    const uint32_t T_echo = P.T_echo, T_amp = P.T_amp, T_del = P.T_del, model = P.delay_model;
    // Q and NV are powers of two (brc_create): shifts, not divisions
    const uint32_t qsh = (uint32_t)__ffs(Q) - 1u, Qm = Q - 1u, ksh = qsh + (uint32_t)__ffs(NV) - 1u;
    // uniform / geometric delays: arrivals are matched on delay-code bit planes (xwords_wide), so
    // the exchange and the receiver's test cost the same however many delays are present
    // CONN: a sender's copies of one type may span several send steps, so the exchange is per link
    // delay (compact index j) and carries the copy count as 8 bit planes (8 nL words, brc_create)
    const bool planes = !CONN && plane_model(model);
    const uint32_t nX = CONN ? 8u * nL : planes ? (uint32_t)NPL + 1u : nL;   // exchanged words per (key, type)
    // LDS carve (lds_bytes_wide): meta[NK] u64 | act[TS][nkw] u64 | dpos[DCW][NPAD] u64 |
    //   consensus area | xb[2][CHUNK_W][nX][2][NW] u64 | outm[16][NW] u64 | sq[Q][NPAD] u8 |
    //   fresh[nkw] u64 | klist[NK] u16 | red[3][4] u32 | pmw[2][CHUNK_W][NW] u32
    // dpos: this pass's deliveries, one bit per key-list POSITION (not per key slot): a step's keys
    // are processed in passes of at most 64 DCW keys, which bounds the delivery bitmap (a slot-
    // indexed one would take NK x NPAD bits and cap the CU at one workgroup)
    // consensus area: REFERENCE hm[4][NW][NPAD] u64;  SPEC cnt[Q][NPAD] u32
    uint64_t* s_meta = smem;
    uint64_t* s_act = s_meta + NK;
    const uint32_t DCW = dpos_words_wide(nkw);     // delivery-bitmap words per receiver
    uint64_t* s_dpos = s_act + TS * nkw;
    uint64_t* s_hm = s_dpos + (size_t)DCW * NPAD;
    // SPEC, per phase slot q = s % Q: #origins | #"0" << 10 | #"1" << 20.  The wide engine takes
    // one key variant per origin (brc_create), so a replica delivers each (origin, phase) key at
    // most once and the origin count needs no host set.
    uint32_t* s_cnt = (uint32_t*)s_hm;
    uint64_t* s_xb = s_hm + cons_words_wide(SPEC, NPAD, Q);
    uint64_t* s_outm = s_xb + 2 * CHUNK_W * nX * 2 * NW;
    uint8_t* s_sq = (uint8_t*)(s_outm + 16 * NW);      // deferred SENDs: values (phase indices consecutive)
    // key slots (re)allocated since the last clear: their rows are rewritten "never sent" before
    // anything reads them, so cells carry no generation tag (clear_fresh)
    uint64_t* s_fresh = (uint64_t*)(s_sq + Q * NPAD);
    uint16_t* s_klist = (uint16_t*)(s_fresh + nkw);    // key slots < 2^11
    uint32_t* s_red = (uint32_t*)(s_klist + NK);       // NK is a multiple of 64: 4-B aligned
    uint32_t* s_pmw = s_red + 12;                // per wave: delays (compact index) with any send
    const uint32_t d = (uint32_t)tid;
    const uint64_t g = P.inst_offset + inst;
    auto validw = [&](int w) -> uint64_t {     // senders < n in word w
        const uint32_t lo = 64u * (uint32_t)w;
        return n >= lo + 64 ? ~0ull : (n <= lo ? 0ull : ((1ull << (n - lo)) - 1));
    };

    ItemState its = P.items[inst];
    uint32_t t = its.t, inj_pos = its.inj_pos;
    const uint32_t inj_off = gp(P.inj_off)[inst], inj_cnt = gp(P.inj_cnt)[inst];
    for (uint32_t i = d; i < NK; i += NPAD)   // restricted-SEND flag in bit 63 of the LDS copy (value ids < 4)
        s_meta[i] = gp(P.meta)[inst * NK + i] | ((gp(P.mgen)[inst * NK + i] & GEN_RESTRICTED) ? M_RESTRICTED : 0ull);
    if (d < nkw) s_fresh[d] = 0;
    for (uint32_t i = d; i < TS * nkw; i += NPAD) s_act[i] = gp(P.act)[inst * TS * nkw + i];
    for (uint32_t w = 0; w < DCW; ++w) s_dpos[w * NPAD + d] = 0;
    for (uint32_t i = d; i < 16 * NW; i += NPAD) s_outm[i] = 0;
    if (d < 12) s_red[d] = 0;
    uint32_t any_rows = uni32(gp(P.actany)[inst]);
    uint32_t lane_rows = 0;

    uint32_t status, t_stop, q_until;
    {
        const uint64_t w0 = *(const gptr_t<uint64_t>)&gp(P.inst)[inst];
        status = w0 & 0xFFFF; t_stop = (w0 >> 16) & 0xFFFF; q_until = (w0 >> 32) & 0xFFFF;
    }
    const uint64_t byzw = gp(P.byz)[inst * NW + wid];
    const bool real = d < n;
    const bool honest = real && !((byzw >> lane) & 1ull);

    // ---- link delays j -> d as NPL bit planes of the delay code (schedule.h)
    uint64_t PL[NPL][NW];
#pragma unroll
    for (int b = 0; b < NPL; ++b)
#pragma unroll
        for (int w = 0; w < NW; ++w) PL[b][w] = 0;
    if (real) {
        if (model == BRC_DELAY_SLOWSET) {
            const uint32_t off = slow_offset(P.seed, g, n);
            const bool me_slow = (d + n - off) % n < P.f;
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                uint64_t sm = 0;
                for (uint32_t b = 0; b < 64; ++b) {
                    const uint32_t j = 64u * w + b;
                    if (j < n && (j + n - off) % n < P.f) sm |= 1ull << b;
                }
                PL[0][w] = me_slow ? validw(w) : sm;          // code 1 <=> delay D
            }
        } else if (model == BRC_DELAY_UNIFORM || model == BRC_DELAY_GEOMETRIC) {
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                for (uint32_t j4 = 0; j4 < 16; ++j4) {
                    const uint32_t j0 = 64u * w + 4 * j4;
                    if (j0 >= n) break;
                    const u32x4 r = draw(P.seed, g, d, PURPOSE_DELAY, j0 >> 2);
                    const uint32_t ws[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        if (j0 + q >= n) break;
                        const uint32_t dl = (model == BRC_DELAY_UNIFORM) ? uniform_delay(ws[q], D) : geometric_delay(ws[q], D);
#pragma unroll
                        for (int b = 0; b < NPL; ++b)
                            if (((dl - 1) >> b) & 1) PL[b][w] |= 1ull << (4 * j4 + q);
                    }
                }
            }
        }
    }
    // word w of L_dly = the senders whose link to this receiver has delay dly
    auto Lw = [&](uint32_t dly, auto wc) -> uint64_t {
        constexpr int w = decltype(wc)::value;
        if (!real) return 0ull;
        const uint64_t v = validw(w);
        if (model == BRC_DELAY_CONST) return dly == P.dconst ? v : 0ull;
        uint32_t code;
        if (model == BRC_DELAY_SLOWSET) {
            if (D == 1) return dly == 1 ? v : 0ull;
            if (dly == D) code = 1; else if (dly == 1) code = 0; else return 0ull;
            return code ? (v & PL[0][w]) : (v & ~PL[0][w]);
        }
        code = dly - 1;
        if (code >= (1u << NPL)) return 0ull;
        uint64_t x = v;
#pragma unroll
        for (int b = 0; b < NPL; ++b) x &= ((code >> b) & 1) ? PL[b][w] : ~PL[b][w];
        return x;
    };
    // delay of the link o -> d (o wave-uniform)
    auto link_delay = [&](uint32_t o) -> uint32_t {
        if (model == BRC_DELAY_CONST) return P.dconst;
        uint32_t code = 0;
        const uint32_t ow = o >> 6, ob = o & 63;
        Unrolled<NW>::run([&](auto wc) {
            constexpr int w = decltype(wc)::value;
            if ((uint32_t)w == ow) {
#pragma unroll
                for (int b = 0; b < NPL; ++b) code |= (uint32_t)((PL[b][w] >> ob) & 1ull) << b;
            }
        });
        if (model == BRC_DELAY_SLOWSET) return (D > 1 && (code & 1)) ? D : 1u;
        return code + 1;
    };

    // ---- outm[i][w]: senders with a delay-(i+1) link to some honest receiver; outset / dset
    auto outm_row = [&](int i) {
        Unrolled<NW>::run([&](auto wc) {
            constexpr int w = decltype(wc)::value;
            const uint64_t x = wave_or64(honest ? Lw((uint32_t)i + 1, wc) : 0ull);
            if (lane == 0 && x) atomicOr((unsigned long long*)&s_outm[i * NW + w], (unsigned long long)x);
        });
    };
    if constexpr (DM > 8) {
        // once-per-launch setup as a loop: unrolled, its 16 x NW wave reductions were most of the DM = 16
        // instantiations' scratch instructions (504 -> 84 on cfg5 geometric, same kernel time)
#pragma unroll 1
        for (int i = 0; i < DM; ++i) outm_row(i);
    } else {
#pragma unroll
        for (int i = 0; i < DM; ++i) outm_row(i);
    }
    __syncthreads();
    uint32_t outset = 0, dset = 0;
#pragma unroll
    for (int i = 0; i < DM; ++i) {
        uint64_t anyw = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) anyw |= s_outm[i * NW + w];
        if (anyw) dset |= 1u << i;
        if (real && ((s_outm[i * NW + wid] >> lane) & 1ull)) outset |= 1u << i;
    }
    dset = uni32(dset);
    // dlist: the delays present, minus one, 4 bits each in ascending order (compact index j)
    uint64_t dlist = 0;
    {
        uint32_t nd = 0;
        for (uint32_t ds = dset; ds; ds &= ds - 1) dlist |= (uint64_t)(__ffs(ds) - 1) << (4 * nd++);
    }
    dlist = uni64(dlist);
    const uint32_t maxout = hibit(outset);
    bool ovf = (uint32_t)__popc(dset) > nL, badinj = false;   // cannot happen: delay_values() bounds dset
    // cell (k, d) at [k * CW * NPAD]; CONN rings: ECHO at + NPAD, + 2 NPAD, READY at + 3 NPAD, + 4 NPAD
    const gptr_t<uint64_t> mycells = gp(P.cells) + inst * (uint64_t)NK * CW * NPAD + d;

    // ---- consensus state (core/byzantinerandomizedconsensus.py:25-29)
    uint64_t c0 = 0, c1 = 0;
    const size_t li = inst * NPAD + d;
    const bool cons_lane = honest && P.protocol == BRC_PROTO_CONSENSUS;
    if (cons_lane) { c0 = gp(P.cons0)[li]; c1 = gp(P.cons1)[li]; }
    auto hm = [&](uint32_t v, uint32_t w) -> uint64_t& { return s_hm[(v * NW + w) * NPAD + d]; };
    auto cnt = [&](uint32_t q) -> uint32_t& { return s_cnt[q * NPAD + d]; };
    const gptr_t<uint32_t> gcnt = gp((uint32_t*)P.hmask);
    if constexpr (SPEC) {
        for (uint32_t q = 0; q < Q; ++q) cnt(q) = cons_lane ? gcnt[(inst * Q + q) * NPAD + d] : 0u;
    } else {
        for (uint32_t v = 0; v < 4; ++v)
            for (uint32_t w = 0; w < NW; ++w)
                hm(v, w) = cons_lane ? gp((const uint64_t*)P.hmask)[((inst * 4 + v) * NW + w) * NPAD + d] : 0ull;
    }
    uint32_t round = c0 & 0xFFFF, phase = (c0 >> 16) & 0xF, nvals = (c0 >> 20) & 0xF;   // cons0_pack
    uint32_t order = (c0 >> 24) & 0xFFFFFF, vcount = (c0 >> 48) & 0xFFFF;
    uint32_t dcount = c1 & 0xFFFF, frnd = (c1 >> 16) & 0xFFFF, ft = (c1 >> 32) & 0xFFFF;
    uint32_t fval = (c1 >> 48) & 0xFF, lval = (c1 >> 56) & 0xFF;

    uint32_t st_msgs = 0, st_arr = 0, st_cells = 0, st_del = 0, st_loads = 0, st_smax = 0;

    // ---- block reductions: OR of a, OR of b, MAX of c over the workgroup (rotating LDS slots)
    uint32_t rctr = 0;
    auto block_red = [&](uint32_t& a, uint32_t& b, uint32_t& c) {
        uint32_t* cur = s_red + 4 * (rctr % 3);
        uint32_t* nxt = s_red + 4 * ((rctr + 1) % 3);
        ++rctr;
        const uint32_t wa = wave_or(a), wb = wave_or(b), wc = wave_max(c);
        if (lane == 0) {
            if (wa) atomicOr(&cur[0], wa);
            if (wb) atomicOr(&cur[1], wb);
            if (wc) atomicMax(&cur[2], wc);
        }
        if (tid == 0) { nxt[0] = 0; nxt[1] = 0; nxt[2] = 0; }
        __syncthreads();
        a = cur[0]; b = cur[1]; c = cur[2];
    };
    auto block_or = [&](uint32_t x) -> uint32_t {
        uint32_t b = 0, c = 0;
        block_red(x, b, c);
        return x;
    };

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
    bool fmark = false;          // this thread marked a slot row fresh since the last clear_fresh
    auto mark_lane = [&](uint32_t k, uint32_t ds) {
        while (ds) {
            const uint32_t i = __ffs(ds) - 1; ds &= ds - 1;
            const uint32_t row = (t + i + 1) & (TS - 1);
            atomicOr((unsigned long long*)&s_act[row * nkw + (k >> 6)], 1ull << (k & 63));
            lane_rows |= 1u << row;
        }
    };
    auto send_key = [&](uint32_t s, uint32_t v) {
        const uint32_t k = (d * NV) * Q + (s & Qm);
        const uint64_t m = s_meta[k];
        // a busy slot, or a phase index past this run's generation budget (brc_run): overflow
        if ((m_s1(m) != 0 && t < m_tquiet(m)) || s >= P.s_limit) { ovf = true; return; }
        atomicOr((unsigned long long*)&s_fresh[k >> 6], 1ull << (k & 63));   // the row is rewritten (clear_fresh)
        fmark = true;
        s_meta[k] = m_pack(s + 1, t, t + maxout, d, v);
        mark_lane(k, outset);
        q_until = max(q_until, t + maxout);
        st_msgs += n;
        st_smax = max(st_smax, s);
        log_ev(BRC_EV_SEND, d, BRC_SEND, d * NV, s, v);
    };
    // Consensus runs between key-list passes, so the SENDs it starts are queued and performed after
    // the step's last pass: every BRB message of the step (those of a key whose slot a new key
    // reuses included) is processed before any slot is reallocated, as the serial semantics have it.
    // One replica's SENDs of one step take distinct slots (phase index mod Q), so Q entries hold all
    // of them: a (Q+1)-th would find its slot busy and overflow in send_key as well (a replica that
    // starts late completes up to Q buffered SPEC phases at once).
    // The SENDs of one replica in one step have consecutive phase indices (each phase change
    // advances the index by one), so the queue keeps the first index and one value byte per SEND.
    uint32_t nsq = 0, sq_s = 0;
    auto send_later = [&](uint32_t s, uint32_t v) {
        if (nsq == 0) sq_s = s;
        if (nsq < Q && s == sq_s + nsq) s_sq[nsq++ * NPAD + d] = (uint8_t)v;
        else ovf = true;
    };
    auto flush_sends = [&]() {
        for (uint32_t i = 0; i < nsq; ++i) send_key(sq_s + i, s_sq[i * NPAD + d]);
        nsq = 0;
    };
    // rewrite the rows of the slots allocated since the last call to "never sent" (each thread its
    // own cell; the connection-peer send rings are ignored while the cell reads never sent)
    // One barrier (with the "any thread marked a row" vote) when no slot was allocated since the
    // last call: injection records that allocate nothing pay no row sweep.
    auto clear_fresh = [&]() {
        if (!__syncthreads_or(fmark ? 1 : 0)) return;
        fmark = false;
        for (uint32_t w = 0; w < nkw; ++w)
            for (uint64_t x = s_fresh[w]; x; x &= x - 1)
                mycells[(size_t)(w * 64 + (uint32_t)__builtin_ctzll(x)) * (CW * NPAD)] = TIMES_NEVER;
        __syncthreads();
        if (d < nkw) s_fresh[d] = 0;
        __syncthreads();
    };
    auto popc_hm = [&](uint32_t v) -> uint32_t {
        uint32_t c = 0;
        for (uint32_t w = 0; w < NW; ++w) c += (uint32_t)__popcll(hm(v, w));
        return c;
    };
    auto get_max_val = [&](uint32_t bound2) -> uint32_t {          // :64-68
        for (uint32_t i = 0; i < nvals; ++i) {
            const uint32_t v = (order >> (2 * i)) & 3;
            if (2 * popc_hm(v) > bound2) return v;
        }
        return 0;                                                    // str(NONE) == "-1"
    };
    auto cons_reset = [&]() {
        vcount = 0; nvals = 0; order = 0;
        for (uint32_t v = 0; v < 4; ++v)
            for (uint32_t w = 0; w < NW; ++w) hm(v, w) = 0;
    };
    // :53-106 for a message of `host` carrying value id v (a BRB delivery, or BRC_INJ_DELIVER)
    auto cons_deliver_vh = [&](uint32_t v, uint32_t host, bool defer) {
        // v already inserted? every 2-bit field of `order` compared at once (nvals <= 4)
        const uint32_t x = order ^ (v * 0x55u);
        const bool found = (~(x | (x >> 1)) & 0x55u & ((1u << (2 * nvals)) - 1u)) != 0;
        if (!found) { order |= v << (2 * nvals); ++nvals; }         // :57-58
        hm(v, host >> 6) |= 1ull << (host & 63);                     // :60
        ++vcount;                                                    // :61
        if (vcount >= P.T_cnt && phase == 1) {                       // :71
            const uint32_t prop = get_max_val(P.bound_p1);           // :73
            phase = 2; cons_reset();                                 // :75-78
            if (defer) send_later(2 * (round - 1) + 1, prop); else send_key(2 * (round - 1) + 1, prop);   // :80-83
        }
        if (vcount >= P.T_cnt && phase == 2) {                       // :86
            const uint32_t dec = get_max_val(P.bound_p2);            // :88
            ++dcount;                                                // :89 never equal -> :94
            if (dcount == 1) { frnd = round; ft = t; fval = dec; }
            lval = dec;
            log_ev(BRC_EV_DECIDE, d, 0, round, dec, dec);
            ++round; phase = 1; cons_reset();                        // :96-100
            if (defer) send_later(2 * (round - 1), dec); else send_key(2 * (round - 1), dec);   // :102-106
        }
    };
    auto cons_deliver = [&](uint32_t k) { cons_deliver_vh(m_value(s_meta[k]) & 3, k >> ksh, true); };

    // ---- SPEC consensus (as brc_step.h spec_advance / spec_deliver)
    auto spec_advance = [&](bool defer) {
        while (round > 0) {
            const uint32_t s = 2 * (round - 1) + (phase - 1), q = s & Qm;
            const uint32_t cc = cnt(q), n0 = (cc >> 10) & 0x3FF, n1 = cc >> 20;
            if ((cc & 0x3FF) < n - P.f) return;
            cnt(q) = 0;
            if (phase == 1) {
                const uint32_t prop = (2 * n0 > n + P.f) ? 1u : (2 * n1 > n + P.f) ? 2u : 0u;
                phase = 2;
                if (defer) send_later(s + 1, prop); else send_key(s + 1, prop);
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
                if (defer) send_later(s + 1, est); else send_key(s + 1, est);
            }
        }
    };
    auto spec_deliver = [&](uint32_t k) {
        const uint64_t m = s_meta[k];
        const uint32_t s = m_s1(m) - 1u, v = m_value(m);
        const uint32_t cur = round ? 2 * (round - 1) + (phase - 1) : 0u;
        if (s < cur) return;
        if (s >= cur + Q) { ovf = true; return; }
        cnt(s & Qm) += 1u + (v == 1 ? 1u << 10 : 0u) + (v == 2 ? 1u << 20 : 0u);
        spec_advance(true);
    };

    // ---- actions stamped t (performed after step t's messages); every branch is workgroup-uniform
    auto do_actions = [&]() -> bool {
        bool mine_any = false;
        const bool running = status == BRC_RUNNING;
        if (its.initialized == 0 && t == 0) {
            if (P.protocol == BRC_PROTO_CONSENSUS && P.proposals != BRC_PROPOSALS_NONE && honest && running) {
                const uint32_t v = (P.proposals == BRC_PROPOSALS_PHILOX) ? proposal_id(P.seed, g, d)
                                                                         : (uint32_t)gp(P.prop)[inst * n + d];
                round = 1; phase = 1;                                 // :43-47
                send_key(0, v & 3);
                if constexpr (SPEC) spec_advance(false);              // phase 0 may be buffered
            }
            clear_fresh();
        }
        while (inj_pos < inj_cnt) {
            const InjDev r = load_inj(P.inj + inj_off + inj_pos);
            if (r.t != t) break;
            ++inj_pos;
            const bool mine = running;
            mine_any |= mine;
            if (r.kind == BRC_INJ_PROPOSE) {
                if (mine && honest && d == r.node) {
                    round = 1; phase = 1; send_key(0, (uint32_t)r.value & 3);
                    if constexpr (SPEC) spec_advance(false);
                }
            } else if (r.kind == BRC_INJ_DELIVER) {
                // a direct deliver() call (brc_inject refuses it for SPEC): host in r.slot
                if constexpr (!SPEC) {
                    if (mine && honest && d == r.node) cons_deliver_vh((uint32_t)r.value & 3, r.slot, false);
                }
            } else if (r.kind == BRC_INJ_SEND || r.kind == BRC_INJ_KEY) {
                const bool is_send = r.kind == BRC_INJ_SEND;
                // restricted SEND (equivocation): this wave's word of the destination set, kept per
                // key in kdst for the arrival test; each wave writes and reads only its own word
                const bool restricted = is_send && r.restricted;
                const uint64_t dw = restricted ? gp((const uint64_t*)(P.inj + inj_off + inj_pos - 1))[2 + wid] : ~0ull;
                uint32_t myset = 0;
                if (is_send && mine && honest && ((dw >> lane) & 1ull)) myset = 1u << (link_delay(r.node) - 1);
                if (restricted && mine && lane == 0) gp(P.kdst)[(inst * NK + r.slot) * NW + wid] = dw;
                const uint32_t os = block_or(myset);
                if (mine) {
                    const uint32_t k = r.slot;
                    if (d == 0) {
                        uint64_t m = s_meta[k];
                        const bool declared = m_s1(m) == r.s + 1u && m_tsend(m) == NEVER && is_send;
                        if ((!declared && m_s1(m) != 0 && t < m_tquiet(m)) || r.s >= P.s_limit) {
                            ovf = true;
                        } else {
                            uint32_t tq = m_tquiet(m);
                            if (!declared) { tq = t + 1; s_fresh[k >> 6] |= 1ull << (k & 63); fmark = true; }
                            if (is_send) tq = max(tq, t + hibit(os));
                            m = m_pack(r.s + 1, is_send ? t : NEVER, tq, r.node, (uint32_t)(uint8_t)r.value);
                            s_meta[k] = m | (restricted ? M_RESTRICTED : 0ull);
                            st_smax = max(st_smax, (uint32_t)r.s);
                            if (is_send) {
                                mark_lane(k, os);
                                uint32_t nd = n;                 // links the SEND travels on
                                if (restricted) {
                                    const gptr_t<const uint64_t> rw = gp((const uint64_t*)(P.inj + inj_off + inj_pos - 1));
                                    nd = 0;
#pragma unroll
                                    for (int w = 0; w < NW; ++w) nd += (uint32_t)__popcll(rw[2 + w]);
                                }
                                st_msgs += nd;
                                log_ev(BRC_EV_SEND, r.node, BRC_SEND, (k >> qsh), r.s, (uint32_t)(uint8_t)r.value);
                            }
                        }
                    }
                    q_until = max(q_until, t + hibit(os));
                }
            } else if (r.kind == BRC_INJ_MSG) {
                const uint32_t k = r.slot;
                bool sent = false;
                if (mine && d == r.node) {
                    const uint64_t m = s_meta[k];
                    if (m_s1(m) != r.s + 1u) {
                        badinj = true;
                    } else {
                        uint64_t wv = mycells[(size_t)k * (CW * NPAD)];
                        const uint32_t bit = (r.type == BRC_ECHO) ? F_ES : F_RS;
                        const int sh = (r.type == BRC_ECHO) ? 32 : 48;
                        if constexpr (CONN) {
                            // every injected broadcast travels: one more send of this type at step t
                            const gptr_t<uint64_t> rp = mycells + (size_t)k * (CW * NPAD) + ((r.type == BRC_ECHO) ? NPAD : 3 * NPAD);
                            const uint32_t tl = (uint32_t)(wv >> sh) & 0xFFFF;
                            Ring16 ring = {rp[0], rp[NPAD]};
                            const uint32_t c = ring_count(ring, tl, t) + 1u;
                            if (c > RING_MAX) {
                                badinj = true;                      // beyond the one-byte count
                            } else {
                                sent = true;
                                ring = ring_put(ring, tl, t, c);
                                rp[0] = ring.lo;
                                rp[NPAD] = ring.hi;
                                // the first broadcast of (node, type, key) is a SEND event, every later copy a COPY
                                log_ev((wv & bit) ? BRC_EV_COPY : BRC_EV_SEND, d, r.type, (k >> qsh), r.s, m_value(m));
                                wv = ((wv | bit) & ~(0xFFFFull << sh)) | ((uint64_t)t << sh);
                                mycells[(size_t)k * (CW * NPAD)] = wv;
                                st_msgs += n;
                            }
                        } else if (!(wv & bit)) {
                            sent = true;
                            wv |= bit;
                            wv = (wv & ~(0xFFFFull << sh)) | ((uint64_t)t << sh);
                            mycells[(size_t)k * (CW * NPAD)] = wv;
                            st_msgs += n;
                            log_ev(BRC_EV_SEND, d, r.type, (k >> qsh), r.s, m_value(m));
                        }
                    }
                }
                const uint32_t os = block_or(sent ? outset : 0u);
                if (os) {
                    if (d == 0) mark_lane(k, os);
                    const uint32_t myq = t + hibit(os);
                    if (mine) {
                        if (d == 0 && myq > m_tquiet(s_meta[k])) s_meta[k] = m_with_tquiet(s_meta[k], myq);
                        q_until = max(q_until, myq);
                    }
                }
            }
            if (r.kind != BRC_INJ_MSG) clear_fresh();    // PROPOSE / DELIVER / SEND / KEY may allocate a slot
        }
        its.initialized = 1;
        return mine_any;
    };

    __syncthreads();
    if (its.initialized == 0 && t == 0) {
        do_actions();
        uint32_t a = 0;
        block_red(a, lane_rows, q_until);
        any_rows |= lane_rows;
        lane_rows = 0;
    }

#ifdef BRC_STAMPS
    // dev-only section timers (tools/stamps.py): per-wave s_memtime deltas, summed over the grid
    uint64_t stamp_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t stamp_prev = __builtin_amdgcn_s_memtime();
#define BRC_WSTAMP(i) do { const uint64_t _n = __builtin_amdgcn_s_memtime(); stamp_acc[i] += _n - stamp_prev; stamp_prev = _n; } while (0)
#else
#define BRC_WSTAMP(i) do {} while (0)
#endif
    for (uint32_t it = 0; it < P.max_steps; ++it) {
        if (status != BRC_RUNNING) break;                 // workgroup-uniform
        const uint32_t rot = (t + 1) & (TS - 1);
        const uint32_t rr = rot ? ((any_rows >> rot) | (any_rows << (TS - rot))) : any_rows;
        uint32_t next = rr ? t + (uint32_t)__ffs(rr) : 0xFFFFFFFFu;
        if (inj_pos < inj_cnt) next = min(next, gp(P.inj)[inj_off + inj_pos].t);
        if (next == 0xFFFFFFFFu) { status = BRC_QUIESCENT; break; }
        if (next > P.step_cap) { status = BRC_STEPCAP; break; }
        t = next;
        const uint32_t row = t & (TS - 1);

        // ================= BRB: this step's active key slots, as a key list in canonical (kp, s) order
        const uint32_t cells0 = st_cells;
        uint32_t nkeys = 0;
        for (uint32_t w = 0; w < nkw; ++w) {
            const uint64_t bits = uni64(s_act[row * nkw + w]);
            if (wid == 0) {
                const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(bits >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)bits, 0u));
                if ((bits >> lane) & 1) s_klist[nkeys + below] = (uint16_t)(w * 64 + lane);
            }
            nkeys += (uint32_t)__popcll(bits);
        }
        __syncthreads();
        {   // slot order is (kp, s mod Q): where one key prefix has several active slots (rare), order
            // them by phase index so that list positions follow the canonical (kp, s) order
            bool run = false;
            for (uint32_t p = d; p + 1 < nkeys; p += NPAD) run |= (s_klist[p] >> qsh) == (s_klist[p + 1] >> qsh);
            if (block_or(run ? 1u : 0u)) {
                if (tid == 0) {
                    for (uint32_t p = 1; p < nkeys; ++p) {          // insertion sort inside each prefix
                        const uint16_t k = s_klist[p];
                        const uint32_t s1 = m_s1(s_meta[k]);
                        uint32_t q = p;
                        while (q > 0 && (s_klist[q - 1] >> qsh) == (uint32_t)(k >> qsh) &&
                               m_s1(s_meta[s_klist[q - 1]]) > s1) {
                            s_klist[q] = s_klist[q - 1];
                            --q;
                        }
                        s_klist[q] = k;
                    }
                }
                __syncthreads();
            }
        }
        BRC_WSTAMP(0);

        // phase 1 of a chunk: ballot words "my ECHO / READY of key c was sent dly steps ago"
        // The key id, meta word and generation it reads stay in SGPRs for phase 2 (process): meta
        // changes in between only in t_quiet, through process's own atomicMax, which keeps the max.
        auto ballots = [&](uint32_t p, uint32_t buf, const uint64_t (&ww)[CHUNK_W], const uint32_t (&kk)[CHUNK_W],
                           uint64_t (&mm)[CHUNK_W]) {
            // the chunk's metadata words first, all in flight together (the ballot-word writes below
            // would otherwise order each key's read behind the previous key's writes)
            Unrolled<CHUNK_W>::run([&](auto ci) {
                constexpr int c = decltype(ci)::value;
                mm[c] = p + c < nkeys ? uni64(s_meta[kk[c]]) : 0ull;
            });
            Unrolled<CHUNK_W>::run([&](auto ci) {
                constexpr int c = decltype(ci)::value;
                if (p + c < nkeys) {
                    const uint32_t k = kk[c];
                    const uint64_t m = mm[c];
                    const bool cur = m_s1(m) != 0 && real;
                    const uint64_t word = cur ? ww[c] : TIMES_NEVER;
                    const uint32_t dE = t - ((uint32_t)(word >> 32) & 0xFFFF), dR = t - (uint32_t)(word >> 48);
                    uint64_t* xb = s_xb + ((buf * CHUNK_W + c) * nX) * 2 * NW;
                    if constexpr (CONN) {
                        // per delay present: the 8 bit planes of "copies I sent dly steps ago"
                        const gptr_t<uint64_t> rp = mycells + (size_t)k * (CW * NPAD);
                        const Ring16 rE = {rp[NPAD], rp[2 * NPAD]}, rR = {rp[3 * NPAD], rp[4 * NPAD]};
                        const uint32_t tE = (uint32_t)(word >> 32) & 0xFFFF, tR = (uint32_t)(word >> 48);
                        uint32_t j = 0, pm = 0;
                        for (uint32_t ds = dset; ds; ds &= ds - 1, ++j) {
                            const uint32_t dly = (uint32_t)__ffs(ds);
                            const uint32_t ce = ring_count(rE, tE, t - dly), cr = ring_count(rR, tR, t - dly);
                            if (__ballot((ce | cr) != 0)) {
                                pm |= 1u << j;
#pragma unroll
                                for (int b = 0; b < 8; ++b) {
                                    const uint64_t be = __ballot((ce >> b) & 1u), br = __ballot((cr >> b) & 1u);
                                    if (lane == 0) { xb[(j * 8 + b) * 2 * NW + wid] = be; xb[(j * 8 + b) * 2 * NW + NW + wid] = br; }
                                }
                            }
                        }
                        if (lane == 0) s_pmw[(buf * CHUNK_W + c) * NW + wid] = pm;
                        return;
                    }
                    if (planes) {
                        // code = steps since this lane sent - 1; a receiver matches it against the
                        // code of its link from this lane, plane by plane
                        const uint32_t cE = dE - 1u, cR = dR - 1u;
                        const uint64_t vE = __ballot(cE < (1u << NPL)), vR = __ballot(cR < (1u << NPL));
                        if (lane == 0) { xb[NPL * 2 * NW + wid] = vE; xb[NPL * 2 * NW + NW + wid] = vR; }
#pragma unroll
                        for (int b = 0; b < NPL; ++b) {
                            const uint64_t be = __ballot((cE >> b) & 1u), br = __ballot((cR >> b) & 1u);
                            if (lane == 0) { xb[b * 2 * NW + wid] = be; xb[b * 2 * NW + NW + wid] = br; }
                        }
                        return;
                    }
                    uint32_t j = 0, pm = 0;
                    for (uint32_t ds = dset; ds; ds &= ds - 1, ++j) {
                        const uint32_t dly = (uint32_t)__ffs(ds);
                        const uint64_t be = __ballot(dE == dly), br = __ballot(dR == dly);
                        if constexpr (SPARSE_D) {
                            if (be | br) {
                                pm |= 1u << j;
                                if (lane == 0) { xb[j * 2 * NW + wid] = be; xb[j * 2 * NW + NW + wid] = br; }
                            }
                        } else if (lane == 0) { xb[j * 2 * NW + wid] = be; xb[j * 2 * NW + NW + wid] = br; }
                    }
                    if constexpr (SPARSE_D) { if (lane == 0) s_pmw[(buf * CHUNK_W + c) * NW + wid] = pm; }
                }
            });
        };
        // the chunk's key ids in one LDS read per 4 (p is a multiple of CHUNK_W, the list 8-B aligned and
        // NK a multiple of 64, so the read stays inside it), then their cell words
        static_assert(CHUNK_W % 4 == 0, "key ids are read 4 at a time");
        auto fetch = [&](uint32_t p, uint64_t (&ww)[CHUNK_W], uint32_t (&kk)[CHUNK_W]) {
            uint64_t ids[CHUNK_W / 4];
#pragma unroll
            for (int g4 = 0; g4 < CHUNK_W / 4; ++g4)
                ids[g4] = p + 4 * g4 < nkeys ? uni64(*(const uint64_t*)(s_klist + p + 4 * g4)) : 0ull;
            Unrolled<CHUNK_W>::run([&](auto ci) {
                constexpr int c = decltype(ci)::value;
                ww[c] = TIMES_NEVER;
                kk[c] = 0;
                if (p + c < nkeys) {
                    kk[c] = (uint32_t)(ids[c / 4] >> (16 * (c % 4))) & 0xFFFFu;
                    ww[c] = mycells[(size_t)kk[c] * (CW * NPAD)];
                }
            });
        };
        // phase 2: one (receiver d, key k) cell
        auto process = [&](const uint32_t k, const uint64_t wd, const uint64_t m, uint32_t buf, int c,
                           uint32_t pos) __attribute__((always_inline)) {
            const bool kl = m_s1(m) != 0;                        // the slot holds a key
            const bool cur = kl && real;
            const uint64_t word = cur ? wd : TIMES_NEVER;
            const uint32_t tE = (uint32_t)(word >> 32) & 0xFFFF, tR = (uint32_t)(word >> 48);
            uint32_t ea = 0, ra = 0;
            {
                // only the delays at which some wave had a send (each wave's pmw word); a wave that
                // had none there did not write its ballot words, so they read as zero
                const uint64_t* xb = s_xb + ((buf * CHUNK_W + c) * nX) * 2 * NW;
                if constexpr (CONN) {
                    // arrivals = sum over senders of their copy counts (one popcount per bit plane)
                    uint32_t pwv[NW], pm = 0;
#pragma unroll
                    for (int w = 0; w < NW; ++w) { pwv[w] = uni32(s_pmw[(buf * CHUNK_W + c) * NW + w]); pm |= pwv[w]; }
                    for (; pm; pm &= pm - 1) {
                        const uint32_t j = (uint32_t)__ffs(pm) - 1, dly = (uint32_t)((dlist >> (4 * j)) & 15u) + 1u;
                        Unrolled<NW>::run([&](auto wc) {
                            constexpr int w = decltype(wc)::value;
                            if ((pwv[w] >> j) & 1u) {
                                const uint64_t L = Lw(dly, wc);
#pragma unroll
                                for (int b = 0; b < 8; ++b) {
                                    ea += (uint32_t)__popcll(xb[(j * 8 + b) * 2 * NW + w] & L) << b;
                                    ra += (uint32_t)__popcll(xb[(j * 8 + b) * 2 * NW + NW + w] & L) << b;
                                }
                            }
                        });
                    }
                } else if (planes) {
                    // senders whose send is `code + 1` steps old, where code is their link's delay
                    // code to this receiver: no plane differs (PL = 0 off the real receivers,
                    // whose counts are never used)
                    Unrolled<NW>::run([&](auto wc) {
                        constexpr int w = decltype(wc)::value;
                        // xe |= plane ^ PL, one 3-input bit op per plane and 32-bit half (v_bitop3 0xBE:
                        // (a ^ b) | c); a sender matches where no plane differs
                        uint32_t xe[2] = {0u, 0u}, xr[2] = {0u, 0u};
#pragma unroll
                        for (int b = 0; b < NPL; ++b) {
                            const uint64_t pe = xb[b * 2 * NW + w], pr = xb[b * 2 * NW + NW + w], pl = PL[b][w];
#pragma unroll
                            for (int h = 0; h < 2; ++h) {
                                xe[h] = __builtin_amdgcn_bitop3_b32((uint32_t)(pe >> (32 * h)), (uint32_t)(pl >> (32 * h)), xe[h], 0xBE);
                                xr[h] = __builtin_amdgcn_bitop3_b32((uint32_t)(pr >> (32 * h)), (uint32_t)(pl >> (32 * h)), xr[h], 0xBE);
                            }
                        }
                        const uint64_t ve = xb[NPL * 2 * NW + w], vr = xb[NPL * 2 * NW + NW + w];
                        ea += (uint32_t)__popc((uint32_t)ve & ~xe[0]) + (uint32_t)__popc((uint32_t)(ve >> 32) & ~xe[1]);
                        ra += (uint32_t)__popc((uint32_t)vr & ~xr[0]) + (uint32_t)__popc((uint32_t)(vr >> 32) & ~xr[1]);
                        // one word's planes at a time: hoisting every word's LDS reads spills (DM = 16)
                        if (BRC_WIDE_PLANE_FENCE) __builtin_amdgcn_sched_barrier(0);
                    });
                } else if constexpr (SPARSE_D) {
                    uint32_t pwv[NW], pm = 0;
#pragma unroll
                    for (int w = 0; w < NW; ++w) { pwv[w] = uni32(s_pmw[(buf * CHUNK_W + c) * NW + w]); pm |= pwv[w]; }
                    for (; pm; pm &= pm - 1) {
                        const uint32_t j = (uint32_t)__ffs(pm) - 1, dly = (uint32_t)((dlist >> (4 * j)) & 15u) + 1u;
                        Unrolled<NW>::run([&](auto wc) {
                            constexpr int w = decltype(wc)::value;
                            const bool wrote = (pwv[w] >> j) & 1u;
                            const uint64_t xe = wrote ? xb[j * 2 * NW + w] : 0ull, xr = wrote ? xb[j * 2 * NW + NW + w] : 0ull;
                            const uint64_t L = Lw(dly, wc);
                            ea += (uint32_t)__popcll(xe & L);
                            ra += (uint32_t)__popcll(xr & L);
                        });
                    }
                } else {
                    uint32_t j = 0;
                    for (uint32_t ds = dset; ds; ds &= ds - 1, ++j) {
                        const uint32_t dly = (uint32_t)__ffs(ds);
                        uint64_t xe[NW], xr[NW], any = 0;
#pragma unroll
                        for (int w = 0; w < NW; ++w) { xe[w] = xb[j * 2 * NW + w]; xr[w] = xb[j * 2 * NW + NW + w]; any |= xe[w] | xr[w]; }
                        if (any) {
                            Unrolled<NW>::run([&](auto wc) {
                                constexpr int w = decltype(wc)::value;
                                const uint64_t L = Lw(dly, wc);
                                ea += (uint32_t)__popcll(xe[w] & L);
                                ra += (uint32_t)__popcll(xr[w] & L);
                            });
                        }
                    }
                }
            }
            BRC_WSTAMP(3);
            // SEND from the key's origin: arrives at t_send + delay(origin -> d)
            bool s_arr = false;
            const uint32_t dt = t - m_tsend(m);
            const bool s_win = kl && dt - 1u < D && ((dset >> ((dt - 1u) & 31)) & 1u);   // uniform
            if (s_win) {
                bool hit = link_delay(m_sender(m)) == dt;
                if (m & M_RESTRICTED) hit = hit && ((gp(P.kdst)[(inst * NK + k) * NW + wid] >> lane) & 1ull);
                s_arr = honest && hit;
            }
            const bool has = kl && honest && (s_arr || ea || ra);
            st_loads += (kl && real) ? 1u : 0u;
            uint32_t fl = (uint32_t)word & 31, ec = (uint32_t)(word >> 5) & 255, rc = (uint32_t)(word >> 13) & 255;
            bool es, rs, dl;
            uint32_t n_ready = 0;                                // CONN: READY broadcasts this step
            bool first_ready = false;
            const bool had_es = (fl & F_ES) != 0;                // a user-issued ECHO was logged already
            if constexpr (CONN) {
                brb_cell_update_conn(fl, ec, rc, s_arr, has ? ea : 0u, has ? ra : 0u, T_echo, T_amp, T_del, es, n_ready, dl);
                rs = n_ready != 0;
                first_ready = rs && !(fl & F_RS);
                fl |= rs ? F_RS : 0u;
                const gptr_t<uint64_t> rp = mycells + (size_t)k * (CW * NPAD);
                if (es) {
                    const Ring16 r = ring_put(Ring16{rp[NPAD], rp[2 * NPAD]}, tE, t, 1u);
                    rp[NPAD] = r.lo; rp[2 * NPAD] = r.hi;
                }
                if (rs) {
                    const Ring16 r = ring_put(Ring16{rp[3 * NPAD], rp[4 * NPAD]}, tR, t, n_ready);
                    rp[3 * NPAD] = r.lo; rp[4 * NPAD] = r.hi;
                }
            } else if constexpr (BEB) brb_cell_update_beb(fl, s_arr, es, rs, dl);
            else if constexpr (SPEC) brb_cell_update_spec(fl, ec, rc, s_arr, has ? ea : 0u, has ? ra : 0u, T_echo, T_amp, T_del, es, rs, dl);
            else brb_cell_update(fl, ec, rc, s_arr, has ? ea : 0u, has ? ra : 0u, T_echo, T_amp, T_del, es, rs, dl);
            {
                const uint32_t tEn = es ? t : tE, tRn = rs ? t : tR;
                const uint64_t nw = (uint64_t)fl | ((uint64_t)min(ec, 255u) << 5) | ((uint64_t)min(rc, 255u) << 13) |
                                    ((uint64_t)tEn << 32) | ((uint64_t)tRn << 48);
#if BRC_WIDE_MSTORE
                if (has) mycells[(size_t)k * (CW * NPAD)] = nw;  // only cells with arrivals change (exec-masked)
#else
                mycells[(size_t)k * (CW * NPAD)] = has ? nw : wd;
#endif
            }
            st_arr += has ? ea + ra + (s_arr ? 1u : 0u) : 0u;
            st_cells += has ? 1u : 0u;
            st_msgs += ((es ? 1u : 0u) + (CONN ? n_ready : (rs ? 1u : 0u))) * n;
            st_del += dl ? 1u : 0u;
            if (dl) atomicOr((unsigned long long*)&s_dpos[(pos >> 6) * NPAD + d], 1ull << (pos & 63));   // pos: in this pass (no-return LDS OR)
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
            BRC_WSTAMP(6);
            // sends of this wave: ring marks at t + every delay its sending lanes have; t_quiet
            const uint64_t sb = __ballot(es || rs);
            if (sb) {
                // the delays some sending lane of this wave has to an honest receiver: a DPP OR of the
                // senders' outsets (no LDS round trip per delay)
                const uint32_t os = wave_or_all((es || rs) ? outset : 0u);
                for (uint32_t x = os; x; x &= x - 1) {
                    const uint32_t r = (t + (uint32_t)__ffs(x)) & (TS - 1);
                    if (lane == 0) atomicOr((unsigned long long*)&s_act[r * nkw + (k >> 6)], 1ull << (k & 63));
                    lane_rows |= 1u << r;
                }
                if (kl && os) {
                    const uint32_t myq = t + hibit(os);
                    if (lane == 0) atomicMax((unsigned long long*)&s_meta[k], (unsigned long long)m_with_tquiet(m, myq));
                    q_until = max(q_until, myq);
                }
            }
        };
        // passes of at most 64 DCW keys: BRB over the pass's keys, then the consensus over the pass's
        // deliveries in list (= canonical) order; SENDs started by the consensus wait for the last pass
        for (uint32_t base = 0; base < nkeys; base += 64 * DCW) {
            const uint32_t end = min(nkeys, base + 64 * DCW);
            {
                uint64_t wA[CHUNK_W];
                uint32_t kA[CHUNK_W];
                fetch(base, wA, kA);
                for (uint32_t p = base; p < end; p += CHUNK_W) {
                    const uint32_t buf = (p / CHUNK_W) & 1;
                    uint64_t mA[CHUNK_W];
                    ballots(p, buf, wA, kA, mA);
                    BRC_WSTAMP(1);
                    __syncthreads();
                    BRC_WSTAMP(2);
                    uint64_t wB[CHUNK_W];
                    uint32_t kB[CHUNK_W];
                    fetch(p + CHUNK_W, wB, kB);
                    BRC_WSTAMP(2);
                    Unrolled<CHUNK_W>::run([&](auto ci) {
                        constexpr int c = decltype(ci)::value;
                        if (p + c < end) process(kA[c], wA[c], mA[c], buf, c, p + c - base);
                    });
                    BRC_WSTAMP(7);
                    Unrolled<CHUNK_W>::run([&](auto ci) {
                        constexpr int c = decltype(ci)::value;
                        wA[c] = wB[c];
                        kA[c] = kB[c];
                    });
                }
            }
            __syncthreads();
            // ============= consensus: this pass's deliveries, ascending list position
            {
                const bool cons = P.protocol == BRC_PROTO_CONSENSUS && honest;
                const uint32_t words = (end - base + 63) / 64;
#pragma unroll 1
                for (uint32_t w = 0; w < words; ++w) {
                    uint64_t bits = s_dpos[w * NPAD + d];
                    s_dpos[w * NPAD + d] = 0;
                    if (!cons) bits = 0;
                    while (bits) {
                        const uint32_t b = __ffsll((unsigned long long)bits) - 1;
                        bits &= bits - 1;
                        const uint32_t k = s_klist[base + w * 64 + b];
                        if constexpr (SPEC) spec_deliver(k);
                        else cons_deliver(k);
                    }
                }
            }
            __syncthreads();
            BRC_WSTAMP(4);
        }
        flush_sends();
        clear_fresh();

        // ================= actions stamped t
        const bool inj_mine = do_actions();

        // ================= per-instance stop conditions (one workgroup reduction)
        uint32_t flags = ((st_cells != cells0 || inj_mine) ? 1u : 0u) | (ovf ? 2u : 0u) | (badinj ? 4u : 0u) |
                         ((honest && dcount < P.round_cap) ? 8u : 0u);
        block_red(flags, lane_rows, q_until);
        any_rows |= lane_rows;
        lane_rows = 0;
        if (flags & 1u) t_stop = t;
        if (flags & 4u) status = BRC_BADINJ;
        else if (flags & 2u) status = BRC_OVERFLOW;
        else if (P.protocol == BRC_PROTO_CONSENSUS && P.round_cap > 0 && !(flags & 8u)) status = BRC_DONE;
        else if (q_until <= t && inj_pos >= inj_cnt) status = BRC_QUIESCENT;
        if (d < nkw) s_act[row * nkw + d] = 0;
        any_rows &= ~(1u << row);
        BRC_WSTAMP(5);
    }
    __syncthreads();
#ifdef BRC_STAMPS
    if (lane == 0) for (int i = 0; i < 8; ++i) atomicAdd(&brc_stamps[i], (unsigned long long)stamp_acc[i]);
#endif
#undef BRC_WSTAMP

    // ---- write back
    for (uint32_t i = d; i < NK; i += NPAD) {
        gp(P.meta)[inst * NK + i] = s_meta[i] & ~M_RESTRICTED;
        gp(P.mgen)[inst * NK + i] = (s_meta[i] & M_RESTRICTED) ? GEN_RESTRICTED : 0u;
    }
    for (uint32_t i = d; i < TS * nkw; i += NPAD) gp(P.act)[inst * TS * nkw + i] = s_act[i];
    if (d == 0) {
        gp(P.actany)[inst] = any_rows;
        ItemState o = {t, inj_pos, 1u, 0u};
        P.items[inst] = o;
    }
    if (honest && P.protocol == BRC_PROTO_CONSENSUS) {
        gp(P.cons0)[li] = cons0_pack(round, phase, nvals, order, vcount);
        gp(P.cons1)[li] = (uint64_t)(dcount & 0xFFFF) | ((uint64_t)(frnd & 0xFFFF) << 16) | ((uint64_t)(ft & 0xFFFF) << 32) |
                          ((uint64_t)(fval & 0xFF) << 48) | ((uint64_t)(lval & 0xFF) << 56);
        if constexpr (SPEC) {
            for (uint32_t q = 0; q < Q; ++q) gcnt[(inst * Q + q) * NPAD + d] = cnt(q);
        } else {
            for (uint32_t v = 0; v < 4; ++v)
                for (uint32_t w = 0; w < NW; ++w) gp((uint64_t*)P.hmask)[((inst * 4 + v) * NW + w) * NPAD + d] = hm(v, w);
        }
    }
    // statistics: wave sums, then one atomic per wave and counter
    uint64_t w6[5] = {st_cells, st_arr, st_msgs, st_del, st_loads};
#pragma unroll
    for (int q = 0; q < 5; ++q) {
#pragma unroll
        for (int o = 32; o; o >>= 1) w6[q] += (uint64_t)__shfl_xor((unsigned long long)w6[q], o);
    }
    const uint32_t smax = wave_max(st_smax);
    if (lane == 0) {
        // istats row: msgs, arrivals, cell-steps, deliveries
        const uint64_t row4[4] = {w6[2], w6[1], w6[0], w6[3]};
#pragma unroll
        for (int q = 0; q < 4; ++q) if (row4[q]) atomicAdd((unsigned long long*)&P.istats[inst * 4 + q], (unsigned long long)row4[q]);
#pragma unroll
        for (int q = 0; q < 5; ++q) if (w6[q]) atomicAdd(&P.gcount[q], (unsigned long long)w6[q]);
        if (smax) atomicMax(&P.gcount[5], (unsigned long long)smax);
    }
    if (d == 0) {
        gptr_t<uint64_t> ip = (gptr_t<uint64_t>)&gp(P.inst)[inst];
        *ip = (*ip & 0xFFFF000000000000ull) | (uint64_t)(status & 0xFFFF) | ((uint64_t)(t_stop & 0xFFFF) << 16) |
              ((uint64_t)(q_until & 0xFFFF) << 32);
        if (status == BRC_RUNNING) atomicAdd(&P.gcount[6], 1ull);
    }
}

template <int NPAD, int DMX, bool EV, int MODE, int WV = 0>
int launch_wide_one(uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P) {
    auto kern = brc_step_wide<NPAD, DMX, EV, MODE, WV>;
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return BRC_E_HIP;
    kern<<<dim3(blocks), dim3(NPAD), lds, s>>>(P);
    return hipGetLastError() == hipSuccess ? 0 : BRC_E_HIP;
}

template <int NPAD>
int launch_step_wide(int dm, bool events, int mode, bool wv4, uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P) {
    // the 4-wave instantiations (host-chosen, wide_waves4): same LDS carve, so the event-log runs take the 3-wave ones
    if (wv4 && !events && dm <= 8 && mode != KMODE_CONN) {
        if (dm == 4) {
            if (mode == BRC_MODE_SPEC) return launch_wide_one<NPAD, 4, false, BRC_MODE_SPEC, 4>(blocks, lds, s, P);
            if (mode == BRC_MODE_BEB) return launch_wide_one<NPAD, 4, false, BRC_MODE_BEB, 4>(blocks, lds, s, P);
            return launch_wide_one<NPAD, 4, false, BRC_MODE_REFERENCE, 4>(blocks, lds, s, P);
        }
        if (mode == BRC_MODE_SPEC) return launch_wide_one<NPAD, 8, false, BRC_MODE_SPEC, 4>(blocks, lds, s, P);
        if (mode == BRC_MODE_BEB) return launch_wide_one<NPAD, 8, false, BRC_MODE_BEB, 4>(blocks, lds, s, P);
        return launch_wide_one<NPAD, 8, false, BRC_MODE_REFERENCE, 4>(blocks, lds, s, P);
    }
#define BRC_CASE(DMX)                                                                                  \
    if (dm == DMX) {                                                                                   \
        if (mode == BRC_MODE_SPEC) return events ? launch_wide_one<NPAD, DMX, true, BRC_MODE_SPEC>(blocks, lds, s, P) : launch_wide_one<NPAD, DMX, false, BRC_MODE_SPEC>(blocks, lds, s, P); \
        if (mode == BRC_MODE_BEB) return events ? launch_wide_one<NPAD, DMX, true, BRC_MODE_BEB>(blocks, lds, s, P) : launch_wide_one<NPAD, DMX, false, BRC_MODE_BEB>(blocks, lds, s, P); \
        if (mode == KMODE_CONN) return events ? launch_wide_one<NPAD, DMX, true, KMODE_CONN>(blocks, lds, s, P) : launch_wide_one<NPAD, DMX, false, KMODE_CONN>(blocks, lds, s, P); \
        return events ? launch_wide_one<NPAD, DMX, true, BRC_MODE_REFERENCE>(blocks, lds, s, P) : launch_wide_one<NPAD, DMX, false, BRC_MODE_REFERENCE>(blocks, lds, s, P); \
    }
    BRC_CASE(4) BRC_CASE(8) BRC_CASE(16)
#undef BRC_CASE
    return BRC_E_INVALID;
}

}  // namespace brc
