// brc_life.h -- the key-lifetime kernel: batched Bracha broadcast + randomized consensus for
// n <= 64 replicas (NPAD = 64, one instance per wavefront) under a two-class link-delay model.
//
// Why a second kernel.  The step kernel (brc_step.h) advances every live key one simulated step
// at a time: per (key, step) it loads the key's 64 receiver cells from HBM, applies the handler
// and stores them back, so a key costs one HBM round trip, a key-list entry and a metadata read
// per active step.  But the BRB state of one key never depends on any other key
// (core/brbroadcast.py:60-119 touches echo_sent_list[m], ready_sent_list[m] and the delivered
// flag of m only), and a key is created by a SEND whose whole future is fixed at that moment.  So
// this kernel simulates a key's ENTIRE lifetime -- every step at which one of its messages lands
// -- right when the key is created, with the 64 receiver cells in registers; nothing of the key
// goes to HBM.  What leaves the lifetime simulation is (a) for each future step, the keys some
// receivers deliver then (consumed by the consensus pass of that step, in canonical key order,
// exactly as the step kernel does) and (b) per-step statistics.  Both live in LDS rings indexed
// by step mod RW; the consensus step loop commits a step's statistics when it reaches it, so an
// instance that stops at step T counts exactly the events of steps <= T.
//
// Two-class delays.  Under the constant and slow-set models a link's delay
// is 1 when both ends are "fast" and Dd otherwise (constant: no fast class, Dd = the constant).
// Every receiver of a class therefore sees the same arrival counts, and receivers of one class
// evolve identically: a key's lifetime is two class states (honest fast receivers, honest slow
// ones), and its deliveries at a step are whole honest classes, which the consensus pass reads as
// two per-class key bitmaps per step.  So the keys created in a step are simulated one per lane
// (lane L: a key of origin L), each as its two class states, the arrival counts in closed form
// (simulate_batch; round 6: 4.6-5.4x on the many-round legs over one key per wave, which left the
// scalar unit saturated).  A key's messages all land within 4 Dd steps
// of its SEND (ECHO <= Dd, READY <= 3 Dd: a class READYs by quorum or is amplified by the other),
// so RW = 32 covers Dd <= 8; the host uses this kernel only there (brc_engine.hip).
//
// Connection-identity peers (core/brbroadcast.py:69, KMODE_CONN): sets count messages and the :119
// amplification re-fires, so a lane may send several READY copies at several steps; the copies
// landing at each relative step are summed per receiver class at send time into a per-key LDS ring
// (s_pr) instead of ballots over one send step per lane.
//
// Per-link delays (PL: uniform / geometric, D <= 8, SURVEY §8(d) cfg4 under cfg5's delay models).
// Every (sender, receiver) link has its own delay, so receivers no longer fall into two classes:
// each lane keeps the senders of each delay as a mask L[i] (bit j: link j -> lane has delay i+1,
// drawn exactly as the step kernel draws them) and counts its arrivals at relative step r as
// sum_i popc(ballot(sent at r - i - 1) & L[i]) -- READY copies (connection peers) through bit planes
// of the per-lane counts kept in a 16-step byte ring.  Deliveries are no longer whole classes, so a
// key's delivery at a future step is a bit in a per-lane HBM bitmap ring [item][RW][nkw][64]
// (P.dring, written with no-return atomics, read and cleared by the consensus pass of that step):
// 64 KB per instance at NK = 256 instead of the step kernel's 40-B connection cells.
//
// Scope (host-checked): sender- or connection-identity peers, consensus protocol with Philox or loaded
// proposals, constant or slow-set delays (two-class) or uniform / geometric delays (PL) with D <= 8,
// no injections, no event log, a fresh engine run to completion.  Everything else runs on the step kernel.  Results are identical to
// the step kernel's (tests/test_gpu_life.py checks both against the C oracle).
#pragma once
#include "brc_step.h"

namespace brc {

constexpr uint32_t LIFE_NEVER = 0xFFFFu;         // relative send step: not sent

// meta word of a key slot: low 16 bits = value << 14 | (s + 1) (the consensus snapshot format),
// high 16 bits = the last step with an arrival of the key at an honest receiver (slot busy before it)
__device__ __forceinline__ uint32_t lm_s1(uint32_t m) { return m & 0x3FFFu; }
__device__ __forceinline__ uint32_t lm_tend(uint32_t m) { return m >> 16; }

#ifndef BRC_LIFE_LANES
#define BRC_LIFE_LANES 1   // two-class form, sender peers: the new keys' lifetimes simulated one key per lane
#endif
#ifndef BRC_LIFE_QBULK
#define BRC_LIFE_QBULK 1   // key windows of 64 / 128: a lane's deliveries of one origin at once when no phase can end
#endif
#ifndef BRC_LIFE_SKIP
#define BRC_LIFE_SKIP 1   // LANES: a batch jumps to the next relative step some lane has pending
#endif
#ifndef BRC_LIFE_HSTAT
#define BRC_LIFE_HSTAT 1   // LANES, sender peers: one wave sum per batch step, the 0/1 statistics by ballots
#endif
#ifndef BRC_LIFE_BSTAT
#define BRC_LIFE_BSTAT 0   // LANES, sender peers: the batch's step statistics by ballot popcounts instead of wave sums
#endif
#ifndef BRC_LIFE_LANES_WAVES
#define BRC_LIFE_LANES_WAVES 8   // their waves per SIMD
#endif
#ifndef BRC_LIFE_PL_CONN_WAVES
#define BRC_LIFE_PL_CONN_WAVES 6   // per-link form, connection peers: waves per SIMD (A/B: 5 284.4, 6 273.2, 7 277.5 ms)
#endif
// DLX: per-link form's largest delay (8, or 16: cfg5's geometric cap), whose keys live up to 4 DLX steps:
// RW = 64 ring rows then (step statistics in 64 lanes, delivery bitmaps in a 64-row HBM ring).
// QBIG: key windows of 64 / 128 (the reference protocol's many-round runs), two-class form only.  Both
// are instantiations of their own, so the default ones keep their registers.
// HMT: the slot metadata in HBM (key windows >= 32, two-class form; QBIG implies it)
template <int MODE, bool PL, int DLX = 8, bool QBIG = false, bool HMT = false>
__global__ __launch_bounds__(64, PL ? (MODE == KMODE_CONN ? BRC_LIFE_PL_CONN_WAVES : 6) : (MODE != KMODE_CONN && BRC_LIFE_LANES) ? BRC_LIFE_LANES_WAVES : 8) void brc_life(const Params* __restrict__ pp) {
    const Params& P = *pp;
    constexpr bool SPEC = MODE == BRC_MODE_SPEC, BEB = MODE == BRC_MODE_BEB, CONN = MODE == KMODE_CONN;
    static_assert(DLX == 8 || (PL && DLX == 16), "delays up to 16: per-link form");
    static_assert(!(QBIG && (PL || MODE == BRC_MODE_SPEC)), "key windows above 32: two-class form, not SPEC");
    constexpr uint32_t RW = (PL && DLX > 8) ? 64u : LIFE_RW;     // ring rows (> the longest key lifetime)
    constexpr uint64_t RWM = RW == 64 ? ~0ull : ((1ull << RW) - 1ull);
    // pending-step masks: bit r - PB <=> relative step r.  RW = 32: PB = 0 (steps <= 32 plus a delay <= 8
    // stay inside 64 bits); RW = 64: PB = 1 (steps 1 .. 64), and a step past the ring is an overflow
    constexpr uint32_t PB = RW == 64 ? 1u : 0u;
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    const uint32_t lane = threadIdx.x;
    const uint64_t item = blockIdx.x;
    if (item >= P.nitems) return;
    const uint32_t n = P.n, NK = P.NK, Q = P.Q, NV = P.NV, nkw = P.nkw;
    const uint32_t T_echo = P.T_echo, T_amp = P.T_amp, T_del = P.T_del;
    const uint32_t qsh = (uint32_t)__ffs(Q) - 1u, Qm = Q - 1u, ksh = qsh + (uint32_t)__ffs(NV) - 1u;
    const bool seen_on = NV > 1;

    // ---- LDS carve (lds_bytes_life)
    // Key windows >= 32 (the reference protocol's many-round runs; NK = 8192 slots at n = 64 and Q = 128) keep
    // the slot metadata in HBM instead (P.lmeta, 32 KB per instance at Q = 128): in LDS it held 32 of the wave's
    // 50 KB and capped the CU at 3 such waves.  Its accesses are few per key (the SEND claims the slot, the
    // lifetime simulation stamps the slot's last step, the consensus pass reads a key word's values once into
    // s_sv), against a lifetime of ~20 simulated steps
    constexpr bool HM = QBIG || HMT;
    static_assert(!(HM && PL), "HBM slot metadata: two-class form");
    uint32_t* const g_meta = HM ? P.lmeta + item * (uint64_t)NK * 2 : nullptr;
    // HM: the class delivery steps too (below), one u32 per slot: class A's code | class B's << 8, written
    // whole when the key is simulated (a reused slot's old key is quiet, its deliveries all consumed)
    uint32_t* const g_dab = HM ? g_meta + NK : nullptr;
    uint32_t* s_meta = (uint32_t*)smem;
    uint32_t* s_sv = (uint32_t*)smem;             // HM: metadata snapshot of the key words being consumed [2][64]
    // HM: per ring step (t mod LIFE_RW) the key words with a class delivery then ([32][2] u64, bit w), and the
    // step's consumed class bitmaps of those words ([nkw][2] u64: class A, class B)
    uint64_t* const s_wsum = (uint64_t*)smem + 64;
    uint64_t* const s_kab = (uint64_t*)smem + 128;
    // two-class form: the step at which each receiver class delivers key slot k -- a class's honest
    // receivers evolve identically, so a class delivers a key once, at one step, whole.  One byte,
    // 0x80 | step mod 128 (0: none): a key's deliveries lie within 4 Dd <= 32 steps of its creation, and
    // the consensus pass clears the entries of the step it consumes (every entry's step is one it visits:
    // a delivery lands on an honest class, so its step has arrivals), so no stale entry aliases a later
    // step.  The per-link form keeps its deliveries in HBM (P.dring).
    uint8_t* s_dA = (uint8_t*)(s_meta + NK);     // (PL, HM: unused)
    uint8_t* s_dB = s_dA + NK;
    uint64_t* s_hm = HM ? s_kab + 2 * nkw                                   // REFERENCE / BEB: hosts per value [4][64]
                        : (uint64_t*)((char*)smem + ((4 * NK + (PL ? 0u : 2 * NK) + 7) & ~7u));
    // slot metadata word k: LDS, or (HM) this instance's HBM row through agent-scope relaxed atomics (L2-served,
    // in program order for one location, as the delivery ring P.dring is accessed)
    auto mld = [&](uint32_t k) -> uint32_t {
        if (HM) return __hip_atomic_load(g_meta + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return s_meta[k];
    };
    auto mst = [&](uint32_t k, uint32_t v) {
        if (HM) __hip_atomic_store(g_meta + k, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else s_meta[k] = v;
    };
    uint64_t* s_seen = s_hm;                      // SPEC, NV > 1: [Q][64]
    uint32_t* s_cnt = (uint32_t*)(s_seen + (seen_on ? Q * 64 : 0u));   // SPEC: [Q][64]

    const uint32_t d = lane;
    const uint64_t inst = item;                   // one instance per wave
    const uint64_t g = P.inst_offset + inst;
    const uint64_t byzm = gp(P.byz)[inst];
    const bool real = d < n;
    const bool honest = real && !((byzm >> d) & 1ull);
    const uint64_t real_mask = (n >= 64) ? ~0ull : ((1ull << n) - 1);
    const uint64_t hon_mask = uni64(__ballot(honest));
    auto lane_in = [](uint64_t mask) -> bool { return __builtin_amdgcn_inverse_ballot_w64(mask); };
    // wave sum through DPP row butterflies and four lane reads (VALU; the kernel is SALU-bound).
    // Every lane active (the kernel's wave-level code never diverges around it).
    auto wave_sum = [](uint32_t x) -> uint32_t {
        x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);    // quad_perm [1,0,3,2]
        x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true);    // quad_perm [2,3,0,1]
        x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, true);   // row_half_mirror
        x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, true);   // row_mirror
        return uni32(rl(x, 0) + rl(x, 16) + rl(x, 32) + rl(x, 48));
    };
    // per-row statistics of the step ring in lane registers (lane = row < RW): arrivals, messages,
    // cells, deliveries -- a select per key-step instead of an exec-masked LDS read-modify-write
    uint32_t rg_arr = 0, rg_msg = 0, rg_cell = 0, rg_del = 0;

    // ---- two delay classes: delay(j -> d) = 1 if j and d are both fast, Dd otherwise
    uint64_t Fm = 0;                               // real fast replicas (PL: none, Dd unused)
    uint32_t Dd = P.delay_model == BRC_DELAY_CONST ? P.dconst : P.D;
    if (PL) {
        Dd = 1;
    } else if (P.delay_model == BRC_DELAY_SLOWSET && P.D > 1) {
        const uint32_t off = slow_offset(P.seed, g, n);
        const bool slow = ((d + n - off) % n) < P.f;
        Fm = uni64(__ballot(real && !slow));
    } else if (P.delay_model == BRC_DELAY_SLOWSET) {
        Dd = 1;                                    // D = 1: every link has delay 1
    }
    Dd = uni32(Dd);
    const uint64_t Sm = real_mask & ~Fm;
    const uint64_t HF = Fm & hon_mask, HS = Sm & hon_mask;
    const uint32_t nHF = (uint32_t)__popcll(HF), nHS = (uint32_t)__popcll(HS);
    const bool laneF = lane_in(Fm);

    // ---- PL: per-link delay masks (brc_step.h link-delay masks, NPAD = 64): L[i] = senders j whose
    // link j -> d has delay i+1; OV[i] (wave-uniform) = senders with a delay-(i+1) link to an honest receiver
    constexpr int DL = PL ? DLX : 1;
    uint64_t L[DL], OV[DL];
#pragma unroll
    for (int i = 0; i < DL; ++i) L[i] = OV[i] = 0;
    if constexpr (PL) {
        if (real) {
            for (uint32_t j4 = 0; j4 < (n + 3) / 4; ++j4) {
                const u32x4 w = draw(P.seed, g, d, PURPOSE_DELAY, j4);
                const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t j = 4 * j4 + q;
                    if (j >= n) break;
                    const uint32_t dl = (P.delay_model == BRC_DELAY_UNIFORM) ? uniform_delay(ws[q], P.D)
                                                                             : geometric_delay(ws[q], P.D);
#pragma unroll
                    for (int i = 0; i < DL; ++i) if ((uint32_t)i + 1 == dl) L[i] |= 1ull << j;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < DL; ++i) OV[i] = uni64(seg_or<64, uint64_t>(honest ? L[i] : 0ull));
    }
    // PL: this lane's delays to honest receivers as a sender (bit i: delay i+1), for the pending steps
    uint32_t myout = 0;
    if constexpr (PL) {
#pragma unroll
        for (int i = 0; i < DL; ++i) myout |= (uint32_t)((OV[i] >> lane) & 1ull) << i;
    }
    // PL: this wave's delivery-bitmap ring in HBM, word (row, w) of this lane at [(row * nkw + w) * 64]
    uint64_t* const dring = PL ? P.dring + item * (uint64_t)RW * nkw * 64 + lane : nullptr;

    // ---- LDS init
    for (uint32_t i = lane; i < NK; i += 64) {
        mst(i, 0u);
        if (HM) __hip_atomic_store(g_dab + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else if (!PL) { s_dA[i] = 0; s_dB[i] = 0; }
    }
    if (HM) s_wsum[lane] = 0;
    if constexpr (SPEC) {
        for (uint32_t q = 0; q < Q; ++q) {
            if (seen_on) s_seen[q * 64 + lane] = 0;
            s_cnt[q * 64 + lane] = 0;
        }
    } else {
        for (int v = 0; v < 4; ++v) s_hm[v * 64 + lane] = 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

    uint32_t status = BRC_RUNNING, t_stop = 0, t = 0;
    bool ovf = false;
    // committed statistics (wave-uniform) and per-lane work counters
    // per-instance totals in one lane-distributed register (lane 0 messages, 1 arrivals, 2 cells,
    // 3 deliveries, 4 key-steps): VALU selects instead of five uniform 64-bit SGPR pairs live
    // through the kernel (it is SALU- and SGPR-bound)
    uint64_t acc = 0;
    auto acc_add = [&](uint32_t l, uint32_t v) { acc += (lane == l) ? (uint64_t)v : 0ull; };
    auto acc_get = [&](int l) -> uint64_t {
        return ((uint64_t)uni32(rl((uint32_t)(acc >> 32), l)) << 32) | uni32(rl((uint32_t)acc, l));
    };
    uint32_t st_smax = 0;
    using RowT = typename std::conditional<RW == 64, uint64_t, uint32_t>::type;
    RowT rows = 0;                                 // ring rows holding arrivals at honest receivers

    // ---- consensus state (core/byzantinerandomizedconsensus.py:25-29)
    const bool cons_lane = honest;                 // consensus protocol (host-checked)
    uint32_t round = 0, phase = 0, nvals = 0, order = 0, vcount = 0;
    uint32_t dcount = 0, frnd = 0, ft = 0, fval = 0, lval = 0;
    // this lane's keys created this step: bit s mod Q (Q <= 32), or (QBIG) phase indices clr_s .. clr_s +
    // clr_n - 1 (a replica's SENDs of one step have consecutive indices: each phase end advances it by one)
    uint32_t clr = 0, clr_s = 0, clr_n = 0;
    uint32_t msg_now = 0;                          // SEND messages sent this step (per lane, counted at once)

    // honest origin d broadcasts SEND for its key (d, s) with value v (core/byzantinerandomizedconsensus.py:48-50,
    // :80-83, :102-106): the slot is claimed now, its lifetime is simulated after the step (simulate below).
    // A reused slot's old delivery steps are <= now (reuse waits for its last arrival), so they match no
    // later step: nothing of the old key needs clearing.
    auto send_key_now = [&](uint32_t s, uint32_t v) {
        const uint32_t k = (d * NV) * Q + (s & Qm);
        const uint32_t m = mld(k);
        if ((lm_s1(m) != 0 && t < lm_tend(m)) || s >= 0x3FFEu) { ovf = true; return; }
        mst(k, ((t + 1u) << 16) | ((v & 3u) << 14) | (s + 1u));   // busy until simulated
        if constexpr (QBIG) {
            if (clr_n == 0) clr_s = s;
            ++clr_n;
        } else {
            clr |= 1u << (s & Qm);
        }
        msg_now += n;
        st_smax = max(st_smax, s);
    };
    // During the consensus pass a replica's SENDs are queued and made after it (as brc_step.h does): a phase
    // change reuses the replica's own slot while another replica may still count this step's delivery of
    // the slot's old key, so every slot's metadata stays as it was for the whole pass.  One replica's SENDs
    // of one pass have consecutive phase indices: the first index and a 2-bit value each.
    bool defer = false;
    uint32_t sq_s = 0, sq_n = 0;
    SendQ<2> sq_v;
    sq_v.clear();
    auto send_key = [&](uint32_t s, uint32_t v) {
        if (defer) {
            if (sq_n == 0) sq_s = s;
            if (s == sq_s + sq_n && sq_n < SENDQ_MAX) { sq_v.put(sq_n, v & 3u); ++sq_n; }
            else ovf = true;                             // consecutive indices; more than SENDQ_MAX in one step: overflow
            return;
        }
        send_key_now(s, v);
    };
    auto flush_sends = [&]() {
        for (uint32_t i = 0; i < sq_n; ++i) send_key_now(sq_s + i, sq_v.get(i) & 3u);
        sq_n = 0; sq_v.clear();
    };
    // a slot's consensus view: value << 14 | (s + 1), as the BRB phase left it
    // (HM: the consensus passes read it from their s_sv snapshot of the word being consumed, snap_w)
    auto snap = [&](uint32_t k) -> uint32_t { return mld(k) & 0xFFFFu; };
    auto snap_w = [&](uint32_t k) -> uint32_t { return HM ? s_sv[k & 63u] : s_meta[k] & 0xFFFFu; };
    auto get_max_val = [&](uint32_t bound2) -> uint32_t {          // :64-68
        for (uint32_t i = 0; i < nvals; ++i) {
            const uint32_t v = (order >> (2 * i)) & 3;
            if (2 * (uint32_t)__popcll(s_hm[v * 64 + lane]) > bound2) return v;
        }
        return 0;                                                    // str(NONE) == "-1"
    };
    auto cons_reset = [&]() {
        vcount = 0; nvals = 0; order = 0;
        for (int v = 0; v < 4; ++v) s_hm[v * 64 + lane] = 0;
    };
    auto cons_deliver_vh = [&](uint32_t v, uint32_t host) {          // :53-106
        const uint32_t x = order ^ (v * 0x55u);
        const uint32_t valid = (1u << (2 * nvals)) - 1u;
        const bool found = (~(x | (x >> 1)) & 0x55u & valid) != 0;
        if (!found) { order |= v << (2 * nvals); ++nvals; }         // :57-58
        s_hm[v * 64 + lane] |= 1ull << host;                        // :60
        ++vcount;                                                    // :61
        if (vcount >= P.T_cnt && phase == 1) {                       // :71
            const uint32_t prop = get_max_val(P.bound_p1);           // :73
            phase = 2; cons_reset();                                 // :75-78
            send_key(2 * (round - 1) + 1, prop);                     // :80-83
        }
        if (vcount >= P.T_cnt && phase == 2) {                       // :86
            const uint32_t dec = get_max_val(P.bound_p2);            // :88 (:89 is always False: decide runs)
            ++dcount;
            if (dcount == 1) { frnd = round; ft = t; fval = dec; }
            lval = dec;
            ++round; phase = 1; cons_reset();                        // :96-100
            send_key(2 * (round - 1), dec);                          // :102-106
        }
    };
    // SPEC consensus (oracle spec_advance / spec_deliver; brc_step.h)
    auto spec_advance = [&]() {
        while (round > 0) {
            const uint32_t s = 2 * (round - 1) + (phase - 1), q = s & Qm;
            const uint32_t cc = s_cnt[q * 64 + lane], n0 = (cc >> 10) & 0x3FF, n1 = cc >> 20;
            if ((seen_on ? (uint32_t)__popcll(s_seen[q * 64 + lane]) : (cc & 0x3FF)) < n - P.f) return;
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
        const uint32_t sn = snap(k);
        const uint32_t s = (sn & 0x3FFFu) - 1u, v = sn >> 14, host = k >> ksh;
        const uint32_t cur = round ? 2 * (round - 1) + (phase - 1) : 0u;
        if (s < cur) return;
        if (s >= cur + Q) { ovf = true; return; }
        const uint32_t q = s & Qm;
        if (seen_on) {
            if ((s_seen[q * 64 + lane] >> host) & 1) return;
            s_seen[q * 64 + lane] |= 1ull << host;
        }
        s_cnt[q * 64 + lane] += 1u + (v == 1 ? 1u << 10 : 0u) + (v == 2 ? 1u << 20 : 0u);
        spec_advance();
    };

    // the BRB cell handler of one receiver at one relative step, sender-identity peers (core/brbroadcast.py:60-119;
    // brc_step.h process_pair): opn = the cell is open and has arrivals, sa / ea / ra its SEND / ECHO / READY
    // arrivals, hS / hE / hR the key's message types landing now; es / rs / dl: ECHO / READY sent, delivered
    auto upd_cell = [&](uint32_t& fl, uint32_t& ec, uint32_t& rc, bool opn, uint32_t sa, uint32_t ea, uint32_t ra,
                        bool hS, bool hE, bool hR, uint32_t& es, uint32_t& rs, uint32_t& dl, uint32_t& nr) {
        auto ge = [](uint32_t x, uint32_t y) -> uint32_t { return ((x - y) >> 31) ^ 1u; };   // x >= y (< 2^31)
        if constexpr (CONN) {
            // core/brbroadcast.py:60-119 with connection-identity peers (brc_step.h brb_cell_update_conn):
            // sets count messages; the :119 amplification re-fires, nr READY copies this step.  In
            // integer form (0/1 words, VALU): the bool form's per-lane conditions became SGPR lane
            // masks combined with scalar ANDs, and this kernel is SALU-bound.
            const uint32_t o = opn ? 1u : 0u, om = 0u - o;
            es = o & sa & ~fl & 1u;                                   // :76-82 (F_EEX = bit 0)
            fl |= es | (es << 3);
            const uint32_t e = ea & om, eon = min(e, 1u);             // :84-98
            const uint32_t chk = min(e + (fl & 1u) - eon, 1u);
            fl |= eon;
            ec += e;
            const uint32_t r1 = eon & chk & ge(ec, T_echo) & (~fl >> 1) & 1u;
            fl |= r1 << 1;
            const uint32_t x = ra & om, ron = min(x, 1u);             // :100-119
            const uint32_t rexm = 0u - ((fl >> 1) & 1u);
            const uint32_t rlo = 2u + ((rc - 1u) & rexm), rhi = x + (rc & rexm);
            fl |= ron << 1;
            rc += x;
            const uint32_t any = ron & ge(rhi, rlo);
            const uint32_t alo = max(rlo, T_amp), ahi = min(rhi, T_del - 1u);
            const uint32_t fire = any & ~fl & ge(ahi, alo) & 1u;      // :118 (no F_RS test: re-fires)
            nr = r1 + ((ahi - alo + 1u) & (0u - fire));
            dl = any & ge(rhi, T_del);                                // :111-115
            fl |= dl << 2;
            rs = min(nr, 1u);
            fl |= rs << 4;
            return;
        }
        if constexpr (BEB) {
            dl = (opn && sa) ? 1u : 0u;                             // brb_cell_update_beb
            fl |= dl << 2;
        } else if constexpr (SPEC) {
            if (hS) { es = (opn ? sa : 0u) & ~(fl >> 3) & 1u; fl |= es << 3; }   // brb_cell_update_spec
            if (hE || hR) {
                ec += opn ? ea : 0u;
                rc += opn ? ra : 0u;
                rs = (opn ? 1u : 0u) & ~(fl >> 4) & (ge(ec, T_echo) | ge(rc, T_amp));
                fl |= rs << 4;
                dl = (opn ? 1u : 0u) & ge(rc, T_del);
                fl |= dl << 2;
            }
        } else {
            // brb_cell_update in integer form (brc_step.h process_pair).  F_EEX = bit 0, F_REX = 1,
            // F_DEL = 2, F_ES = 3, F_RS = 4.
            if (hS) {                                                // :76-82
                es = (opn ? sa : 0u) & ~fl & 1u;
                fl |= es | (es << 3);
            }
            if (hE) {                                                // :84-98
                const uint32_t e = opn ? ea : 0u;
                const uint32_t eon = min(e, 1u);
                const uint32_t chk = min(e + (fl & 1u) - eon, 1u);
                fl |= eon;
                ec += e;
                const uint32_t r1 = eon & chk & ge(ec, T_echo) & (~fl >> 1) & 1u;
                fl |= (r1 << 1) | (r1 << 4);
                rs = r1;
            }
            if (hR) {                                                // :100-119
                const uint32_t x = opn ? ra : 0u;
                const uint32_t ron = min(x, 1u);
                const uint32_t rexm = 0u - ((fl >> 1) & 1u);
                const uint32_t rlo = 2u + ((rc - 1u) & rexm), rhi = x + (rc & rexm);
                fl |= ron << 1;
                rc += x;
                const uint32_t any = ron & ge(rhi, rlo);
                const uint32_t alo = max(rlo, T_amp), ahi = min(rhi, T_del - 1u);
                const uint32_t r2 = any & ~fl & ~(fl >> 4) & ge(ahi, alo) & 1u;
                fl |= r2 << 4;
                dl = any & ge(rhi, T_del);
                fl |= dl << 2;
                rs |= r2;
            }
        }
        nr = rs;
    };
    // ---- the lifetime of key slot k created at step t (wave-uniform): every step at which one of
    // its messages lands on an honest receiver, in order; cells in registers (brc_step.h C32 fields
    // unpacked: flags, |echo set|, |ready set|, and the relative steps this lane SENT ECHO / READY)
    auto simulate = [&](uint32_t k) {
        const uint32_t o = k >> ksh;                  // origin
        const bool oF = (Fm >> o) & 1ull;
        const uint32_t t0 = t;
        // SEND arrivals: fast receivers at 1 if the origin is fast, everyone else at Dd
        uint32_t sdl = (oF && laneF) ? 1u : Dd;
        // relative steps with SEND / ECHO / READY arrivals: bit r - PB <=> step r
        uint64_t pendS = 0, pendE = 0, pendR = 0;
        if constexpr (PL) {
            sdl = 0;
#pragma unroll
            for (int i = 0; i < DL; ++i) {
                if ((L[i] >> o) & 1ull) sdl = (uint32_t)i + 1u;
                if ((OV[i] >> o) & 1ull) pendS |= (2ull >> PB) << i;
            }
        } else {
            if (oF && HF) pendS |= 2ull;
            if (HS || (!oF && HF)) pendS |= 1ull << Dd;
        }
        uint32_t fl = 0, ec = 0, rc = 0, rE = LIFE_NEVER, rR = LIFE_NEVER;
        Ring16 ringR = {0ull, 0ull};                  // PL connection peers: READY copies per step
        uint32_t last = t0;
        uint32_t prv = 0;                             // CONN two-class: READY copies landing at relative step = lane
        uint32_t dab = 0;                             // HM: the key's class delivery codes (A | B << 8)
        const uint32_t kw = k >> 6;
        const uint64_t kbit = 1ull << (k & 63);
        for (uint64_t pend = pendS; pend; pend = pendS | pendE | pendR) {
            const uint32_t r = (uint32_t)__builtin_ctzll(pend) + PB;
            const uint64_t rb = 1ull << (r - PB);
            const bool hS = (pendS & rb) != 0, hE = (pendE & rb) != 0, hR = (pendR & rb) != 0;
            pendS &= ~rb; pendE &= ~rb; pendR &= ~rb;
            if (r > RW) { ovf = true; break; }        // two-class: cannot happen for Dd <= 8 (lifetime <= 4 Dd)
            const uint32_t ts = t0 + r, row = ts & (RW - 1);
            acc_add(4u, 1u);
            // arrival counts per receiver class (fast: fast senders at r - 1, slow senders at r - Dd;
            // slow: every sender at r - Dd), then per lane
            const uint32_t c1 = r - 1u, cD = r >= Dd ? r - Dd : 0xFFFFFFFFu;
            uint32_t ea = 0, ra = 0, eA = 0, eB = 0, rA = 0, rB = 0;
            if constexpr (PL) {
                // per receiver: the senders of each delay i+1 that sent at r - i - 1
#pragma unroll
                for (int i = 0; i < DL; ++i) {
                    if (!OV[i] || r <= (uint32_t)i) continue;
                    const uint32_t sr = r - (uint32_t)i - 1u;
                    if (hE) {
                        const uint64_t x = __ballot(rE == sr);
                        if (x) ea += (uint32_t)__popcll(x & L[i]);
                    }
                    if (hR) {
                        if constexpr (CONN) {
                            const uint32_t c = ring_count(ringR, rR, sr);
                            const uint64_t x = __ballot(c != 0);
                            if (x) {
                                if (__ballot(c > 1u)) {
                                    // the count planes up to the wave's highest set bit (copies > 3 are rare)
                                    uint32_t np = 2;
                                    while (np < 8 && __ballot((c >> np) != 0u)) ++np;
                                    for (uint32_t b = 0; b < np; ++b) {
                                        const uint64_t pb = __ballot((c >> b) & 1u);
                                        ra += (uint32_t)__popcll(pb & L[i]) << b;
                                    }
                                } else {
                                    ra += (uint32_t)__popcll(x & L[i]);
                                }
                            }
                        } else {
                            const uint64_t x = __ballot(rR == sr);
                            if (x) ra += (uint32_t)__popcll(x & L[i]);
                        }
                    }
                }
            } else {
            if (hE) {
                const uint64_t x1 = __ballot(rE == c1), xD = __ballot(rE == cD);
                eA = (uint32_t)__popcll(x1 & Fm) + (uint32_t)__popcll(xD & Sm);
                eB = (uint32_t)__popcll(xD);
                ea = laneF ? eA : eB;
            }
            if (hR) {
                if constexpr (CONN) {
                    const uint32_t ab = uni32(rl(prv, (int)r));
                    rA = ab & 0xFFFFu; rB = ab >> 16;
                } else {
                    const uint64_t x1 = __ballot(rR == c1), xD = __ballot(rR == cD);
                    rA = (uint32_t)__popcll(x1 & Fm) + (uint32_t)__popcll(xD & Sm);
                    rB = (uint32_t)__popcll(xD);
                }
                ra = laneF ? rA : rB;
            }
            }
            const uint32_t sa = (hS && honest && r == sdl) ? 1u : 0u;
            const uint64_t sab = hS ? __ballot(sa != 0) : 0ull;
            const uint32_t a = ea + ra + sa;
            const uint64_t hb = __ballot(a != 0) & hon_mask;          // receivers with arrivals
            const uint32_t cells = (uint32_t)__popcll(hb);
            const uint32_t arr = PL ? wave_sum(honest ? ea + ra : 0u) + (uint32_t)__popcll(sab)
                                    : nHF * (eA + rA) + nHS * (eB + rB) + (uint32_t)__popcll(sab);
            // a delivered cell ignores everything (core/brbroadcast.py:74)
            const bool opn = lane_in(hb) && !(fl & F_DEL);
            uint32_t es = 0, rs = 0, dl = 0, nr = 0;
            upd_cell(fl, ec, rc, opn, sa, ea, ra, hS, hE, hR, es, rs, dl, nr);
            const uint64_t eb = __ballot(es != 0), rbm = __ballot(rs != 0), db = __ballot(dl != 0);
            if (es) rE = r;
            if (!CONN && rs) rR = r;
            if (PL && CONN && nr) { ringR = ring_put(ringR, rR, r, nr); rR = r; }
            // READY messages sent now by fast / slow senders (CONN: copies, a lane may send several)
            uint32_t cF = (uint32_t)__popcll(rbm & Fm), cS = (uint32_t)__popcll(rbm & Sm);
            if constexpr (CONN) {
                if (__ballot(nr > 1)) {                                  // per-class sums of the per-lane counts
                    const uint32_t pk = wave_sum(laneF ? nr : nr << 16);   // <= 64 x 255 per half
                    cF = pk & 0xFFFFu; cS = pk >> 16;
                }
            }
            const uint32_t msgs = n * ((uint32_t)__popcll(eb) + cF + cS);
            const uint32_t dels = (uint32_t)__popcll(db);
            if (PL && db) {
                // this lane delivers the key at step ts: its bit in the lane's bitmap of row ts
                if (dl) __hip_atomic_fetch_or(dring + (row * nkw + kw) * 64, kbit, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
            } else if (db) {
                // receivers of one class evolve identically: a delivery step takes whole honest classes
                const uint64_t dA = db & HF, dB = db & HS;
                if ((dA && dA != HF) || (dB && dB != HS)) ovf = true;
                if constexpr (HM) {
                    dab |= (dA ? (0x80u | (ts & 0x7Fu)) : 0u) | (dB ? (0x80u | (ts & 0x7Fu)) << 8 : 0u);
                    if (lane == 0)                           // a delivery of word kw at ts (no-return LDS OR: no wait)
                        atomicOr((unsigned long long*)&s_wsum[row * 2 + (kw >> 6)], 1ull << (kw & 63));
                } else {
                    if (dA && lane == 0) s_dA[k] = (uint8_t)(0x80u | (ts & 0x7Fu));
                    if (dB && lane == 0) s_dB[k] = (uint8_t)(0x80u | (ts & 0x7Fu));
                }
            }
            // the messages sent now land on fast receivers after 1 step (fast senders) and on every
            // other (sender, receiver) pair after Dd steps
            if (PL) {
                // a message sent now lands after every delay i+1 some link of its sender has to an honest
                // receiver: the senders' delay sets OR-ed over the wave (one DPP reduction, VALU)
                if (eb | rbm) {
                    uint32_t x = (es ? myout : 0u) | ((rs ? myout : 0u) << DL);
                    x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);
                    x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true);
                    x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, true);
                    x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, true);
                    x = uni32(rl(x, 0) | rl(x, 16) | rl(x, 32) | rl(x, 48));
                    // arrivals at r + i + 1 for every delay bit i: bit r + i + 1 - PB (RW = 64: a step past the
                    // ring is an overflow, never lost; RW = 32: r <= 32 and delays <= 8 fit the 64 bits)
                    constexpr uint32_t DM1 = (1u << DL) - 1u;
                    if (PB && (r + hibit(x & DM1) > RW || r + hibit(x >> DL) > RW)) ovf = true;
                    // a send at r = RW (RW = 64: a key past its 4 DLX-step lifetime bound) lands past the ring:
                    // overflow above, and no shift by 64 (undefined; the hardware would wrap it to 0)
                    if (r + 1u - PB < 64u) {
                        pendE |= (uint64_t)(x & DM1) << (r + 1u - PB);
                        pendR |= (uint64_t)(x >> DL) << (r + 1u - PB);
                    }
                }
            } else if (eb) {
                if ((eb & Fm) && HF) pendE |= rb << 1;
                if (HS || ((eb & Sm) && HF)) pendE |= rb << Dd;
            }
            if (!PL && rbm) {
                const bool at1 = cF && HF, atD = HS || (cS && HF);
                if (at1) pendR |= rb << 1;
                if (atD) pendR |= rb << Dd;
                if constexpr (CONN) {
                    if (at1) prv += lane == r + 1 ? cF : 0u;
                    if (atD) prv += lane == r + Dd ? cS + ((cF + cS) << 16) : 0u;
                }
            }
            {
                const bool mine = lane == row;
                rg_arr += mine ? arr : 0u; rg_msg += mine ? msgs : 0u;
                rg_cell += mine ? cells : 0u; rg_del += mine ? dels : 0u;
            }
            rows |= (RowT)1 << row;
            last = ts;
        }
        if (lane == 0) {
            mst(k, (mld(k) & 0xFFFFu) | (last << 16));
            if (HM) __hip_atomic_store(g_dab + k, dab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    // ---- two-class form, sender peers (LANES): the keys created this step simulated one per lane -- lane L
    // takes one key of origin L (a batch per key index of each origin).  A key's honest receivers of one
    // class evolve identically (above), so its lifetime is two class states, A (honest fast receivers) and
    // B (honest slow ones), advanced by upd_cell per relative step r; a class's arrival count is a
    // comparison of the class states' send steps times the class sizes (simulate()'s ballot popcounts in
    // closed form), and the step statistics are wave sums over the batch.  The keys are independent, so
    // this is simulate(k) for every key of the batch at once: the same slot stamps, class delivery steps,
    // ring statistics and overflows, in VALU instead of the scalar unit, which simulate() saturates.
    constexpr bool LANES = BRC_LIFE_LANES && !PL;
    auto simulate_batch = [&](const bool has, const uint32_t k) {
        const bool vA = HF != 0, vB = HS != 0;
        const bool oF = laneF;                        // the origin is this lane
        const uint32_t sdlA = oF ? 1u : Dd;           // SEND arrival step at class A (class B: Dd)
        // pending message types of the next steps, a window sliding with r: bit j of field S (bits 0-9),
        // E (10-19), R (20-29) <=> step r + j (a message lands at most Dd <= 8 steps after it is sent)
        uint32_t pend = 0;
        if (has) {
            if (oF && vA) pend |= 1u;
            if (vB || (!oF && vA)) pend |= 1u << (Dd - 1u);
        }
        uint32_t flA = 0, ecA = 0, rcA = 0, flB = 0, ecB = 0, rcB = 0;
        // the relative steps the classes SENT ECHO / READY, a byte each (0xFF: not sent): A's ECHO, A's READY,
        // B's ECHO, B's READY
        uint32_t sent = 0xFFFFFFFFu;
        uint32_t last = t, dab = 0;
        const uint32_t kw = k >> 6;
        // CONN: READY copies landing at steps r + j (j < 9): class A's in the low half, class B's in the high
        uint32_t win[9];
#pragma unroll
        for (int j = 0; j < 9; ++j) win[j] = 0;
        uint32_t rstep = 1;                           // SKIP: steps to the next one some lane has pending
#pragma unroll 1
        for (uint32_t r = 1; ; r += rstep) {
            if (!__ballot(pend != 0u)) break;
            const bool hS = (pend & 1u) != 0, hE = (pend & (1u << 10)) != 0, hR = (pend & (1u << 20)) != 0;
            bool act = hS || hE || hR;
            if (act && r > RW) {                      // past the ring: overflow (cannot happen for Dd <= 8)
                ovf = true; act = false;
                pend = 0;
            }
            const uint32_t ts = t + r, row = ts & (RW - 1);
            const uint32_t c1 = r - 1u, cD = r >= Dd ? r - Dd : 0x100u;   // 0x100: matches no byte
            // class arrivals: fast senders (class A) land on A after 1 step, every other pair after Dd
            uint32_t eA = 0, eB = 0, rA = 0, rB = 0;
            // which class sent now-landing messages: e1 / q1 A's ECHO / READY sent at r - 1, e3 / q3 at
            // r - Dd, e2 / q2 B's at r - Dd
            bool e1 = false, e2 = false, e3 = false, q1 = false, q2 = false, q3 = false;
            if (hE) {
                const uint32_t xA = sent & 0xFFu, xB = (sent >> 16) & 0xFFu;
                e1 = xA == c1; e2 = xB == cD; e3 = xA == cD;
                eA = (e1 ? nHF : 0u) + (e2 ? nHS : 0u);
                eB = (e3 ? nHF : 0u) + (e2 ? nHS : 0u);
            }
            if (hR) {
                if constexpr (CONN) {
                    rA = win[0] & 0xFFFFu; rB = win[0] >> 16;
                } else {
                    const uint32_t xA = (sent >> 8) & 0xFFu, xB = sent >> 24;
                    q1 = xA == c1; q2 = xB == cD; q3 = xA == cD;
                    rA = (q1 ? nHF : 0u) + (q2 ? nHS : 0u);
                    rB = (q3 ? nHF : 0u) + (q2 ? nHS : 0u);
                }
            }
            const uint32_t saA = (hS && r == sdlA) ? 1u : 0u, saB = (hS && r == Dd) ? 1u : 0u;
            const uint32_t aA = act ? eA + rA + saA : 0u, aB = act ? eB + rB + saB : 0u;
            // a delivered cell ignores everything (core/brbroadcast.py:74)
            const bool opnA = vA && aA != 0 && !(flA & F_DEL), opnB = vB && aB != 0 && !(flB & F_DEL);
            uint32_t esA = 0, rsA = 0, dlA = 0, esB = 0, rsB = 0, dlB = 0, nrA = 0, nrB = 0;
            if (act) {
                upd_cell(flA, ecA, rcA, opnA, saA, eA, rA, hS, hE, hR, esA, rsA, dlA, nrA);
                upd_cell(flB, ecB, rcB, opnB, saB, eB, rB, hS, hE, hR, esB, rsB, dlB, nrB);
            }
            if (CONN) rsA = rsB = 0;                  // CONN: READY copies go through win, not send steps
            if (esA | rsA | esB | rsB) {
                const uint32_t sm = (esA ? 0xFFu : 0u) | (rsA ? 0xFF00u : 0u) | (esB ? 0xFF0000u : 0u) | (rsB ? 0xFF000000u : 0u);
                sent = (sent & ~sm) | ((r * 0x01010101u) & sm);
            }
            // step statistics over the batch: arrivals nHF aA + nHS aB, messages n (nHF (esA + rsA) + nHS (esB +
            // rsB)), cells nHF [aA > 0] + nHS [aB > 0], deliveries nHF dlA + nHS dlB (simulate()'s popcounts)
            const uint64_t am = __ballot(act);
            if (am) {
                uint32_t arr, msgs, cells;
                if constexpr (CONN) {
                    // READY copies: a count may reach 64 x 64 per lane, so the sums take whole words
                    const uint32_t sA = wave_sum(aA), sB = wave_sum(aB);
                    const uint32_t s2 = wave_sum((esA + nrA) | ((esB + nrB) << 16));
                    arr = nHF * sA + nHS * sB;
                    msgs = n * (nHF * (s2 & 0xFFFFu) + nHS * (s2 >> 16));
                    cells = nHF * (uint32_t)__popcll(__ballot(aA != 0)) + nHS * (uint32_t)__popcll(__ballot(aB != 0));
                } else if constexpr (BRC_LIFE_BSTAT) {
                    // the sums as popcounts of ballots: a lane's class counts are class sizes times conditions
                    auto pc = [&](bool c) -> uint32_t { return (uint32_t)__popcll(__ballot(act && c)); };
                    const uint32_t n2 = pc(e2) + pc(q2);
                    const uint32_t sA = nHF * (pc(e1) + pc(q1)) + nHS * n2 + pc(saA != 0);
                    const uint32_t sB = nHF * (pc(e3) + pc(q3)) + nHS * n2 + pc(saB != 0);
                    arr = nHF * sA + nHS * sB;
                    msgs = n * (nHF * (pc(esA != 0) + pc(rsA != 0)) + nHS * (pc(esB != 0) + pc(rsB != 0)));
                    cells = nHF * pc(aA != 0) + nHS * pc(aB != 0);
                } else if constexpr (BRC_LIFE_HSTAT) {
                    // one wave sum (the arrival counts); the 0/1 terms as ballot popcounts
                    auto pc = [&](bool c) -> uint32_t { return (uint32_t)__popcll(__ballot(c)); };
                    const uint32_t s1 = wave_sum(aA | (aB << 16));
                    arr = nHF * (s1 & 0xFFFFu) + nHS * (s1 >> 16);
                    msgs = n * (nHF * (pc(esA != 0) + pc(rsA != 0)) + nHS * (pc(esB != 0) + pc(rsB != 0)));
                    cells = nHF * pc(aA != 0) + nHS * pc(aB != 0);
                } else {
                    const uint32_t s1 = wave_sum(aA | (aB << 16));
                    const uint32_t s2 = wave_sum((esA + rsA) | ((esB + rsB) << 8) | ((aA != 0 ? 1u : 0u) << 16) |
                                                 ((aB != 0 ? 1u : 0u) << 24));
                    arr = nHF * (s1 & 0xFFFFu) + nHS * (s1 >> 16);
                    msgs = n * (nHF * (s2 & 0xFFu) + nHS * ((s2 >> 8) & 0xFFu));
                    cells = nHF * ((s2 >> 16) & 0xFFu) + nHS * (s2 >> 24);
                }
                const uint32_t ndA = (uint32_t)__popcll(__ballot(dlA != 0)), ndB = (uint32_t)__popcll(__ballot(dlB != 0));
                const uint32_t dels = nHF * ndA + nHS * ndB;
                const bool mine = lane == row;
                rg_arr += mine ? arr : 0u; rg_msg += mine ? msgs : 0u;
                rg_cell += mine ? cells : 0u; rg_del += mine ? dels : 0u;
                acc_add(4u, (uint32_t)__popcll(am));
                rows |= (RowT)1 << row;
            }
            if (dlA || dlB) {
                // a class delivers the key at step ts, whole
                const uint32_t tc = 0x80u | (ts & 0x7Fu);
                if constexpr (HM) {
                    dab |= (dlA ? tc : 0u) | (dlB ? tc << 8 : 0u);
                    // a delivery of word kw at ts (no-return LDS OR)
                    atomicOr((unsigned long long*)&s_wsum[row * 2 + (kw >> 6)], 1ull << (kw & 63));
                } else {
                    if (dlA) s_dA[k] = (uint8_t)tc;
                    if (dlB) s_dB[k] = (uint8_t)tc;
                }
            }
            // the messages sent now land on class A after 1 step (fast senders) and on every other pair
            // after Dd steps
            if (esA || esB) {
                if (esA) pend |= 1u << 11;
                if (vB || esB) pend |= 1u << (10u + Dd);
            }
            if (rsA || rsB) {
                if (rsA) pend |= 1u << 21;
                if (vB || rsB) pend |= 1u << (20u + Dd);
            }
            if constexpr (CONN) {
                // copies sent now: class A's land on A after 1 step, every other pair's after Dd
                if (nrA || nrB) {
                    const uint32_t cF = nHF * nrA, cS = nHS * nrB;
                    win[1] += cF;
                    const uint32_t cd = cS + ((cF + cS) << 16);
#pragma unroll
                    for (int j = 1; j < 9; ++j) win[j] += (uint32_t)j == Dd ? cd : 0u;
                    if (nrA) pend |= 1u << 21;
                    if (vB) pend |= 1u << (20u + Dd);
                }
            }
            if (act) last = ts;
            if constexpr (BRC_LIFE_SKIP) {
                // step r consumed; the window moves to the next step any lane of the batch has pending (the
                // lowest offset over the three fields and the wave: no set bit crosses a field boundary)
                pend &= ~(1u | (1u << 10) | (1u << 20));
                uint32_t m = (pend | (pend >> 10) | (pend >> 20)) & 0x3FFu;
                m |= (uint32_t)__builtin_amdgcn_mov_dpp((int)m, 0xB1, 0xF, 0xF, true);
                m |= (uint32_t)__builtin_amdgcn_mov_dpp((int)m, 0x4E, 0xF, 0xF, true);
                m |= (uint32_t)__builtin_amdgcn_mov_dpp((int)m, 0x141, 0xF, 0xF, true);
                m |= (uint32_t)__builtin_amdgcn_mov_dpp((int)m, 0x140, 0xF, 0xF, true);
                m = uni32(rl(m, 0) | rl(m, 16) | rl(m, 32) | rl(m, 48));
                rstep = m ? (uint32_t)__builtin_ctz(m) : 1u;
                pend >>= rstep;
            } else {
                pend = (pend >> 1) & ~((1u << 9) | (1u << 19));   // step r consumed: the window moves to r + 1
            }
            if constexpr (CONN) {
                // the READY-copy window moves with it (rstep <= 9 steps: entries past it are zero)
#pragma unroll 1
                for (uint32_t q = 0; q < rstep; ++q) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) win[j] = win[j + 1];
                    win[8] = 0;
                }
            }
        }
        if (has) {
            mst(k, (mld(k) & 0xFFFFu) | (last << 16));
            if (HM) __hip_atomic_store(g_dab + k, dab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    // the keys created this step (every lane's clr_s .. clr_s + clr_n - 1), each simulated once
    auto simulate_new = [&]() {
        if constexpr (LANES) {
#pragma unroll 1
            for (;;) {
                bool has;
                uint32_t k = 0;
                if constexpr (QBIG) {
                    has = clr_n != 0;
                    if (has) { k = (lane * NV) * Q + (clr_s & Qm); ++clr_s; --clr_n; }
                } else {
                    has = clr != 0;
                    if (has) { k = (lane * NV) * Q + (uint32_t)__ffs(clr) - 1u; clr &= clr - 1u; }
                }
                if (!__ballot(has)) break;
                simulate_batch(has, k);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            }
            clr = 0; clr_n = 0;
            return;
        }
        if constexpr (QBIG) {
            for (uint64_t b = __ballot(clr_n != 0); b; b &= b - 1) {
                const int L = __ffsll((unsigned long long)b) - 1;
                const uint32_t s0 = uni32((uint32_t)__builtin_amdgcn_readlane((int)clr_s, L));
                const uint32_t cn = uni32((uint32_t)__builtin_amdgcn_readlane((int)clr_n, L));
                for (uint32_t i = 0; i < cn; ++i) {
                    const uint32_t k = ((uint32_t)L * NV) * Q + ((s0 + i) & Qm);
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    simulate(k);
                }
            }
            clr_n = 0;
        } else {
            for (uint64_t b = __ballot(clr != 0); b; b &= b - 1) {
                const int L = __ffsll((unsigned long long)b) - 1;
                for (uint32_t cm = uni32((uint32_t)__builtin_amdgcn_readlane((int)clr, L)); cm; cm &= cm - 1) {
                    const uint32_t k = ((uint32_t)L * NV) * Q + (uint32_t)__ffs(cm) - 1u;
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    simulate(k);
                }
            }
            clr = 0;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    };

    // ---- step 0: the proposals (actions stamped 0, core/byzantinerandomizedconsensus.py:38-50)
    if (honest) {
        const uint32_t v = (P.proposals == BRC_PROPOSALS_PHILOX) ? proposal_id(P.seed, g, d)
                                                                 : (uint32_t)gp(P.prop)[inst * n + d];
        round = 1; phase = 1;
        send_key(0, v & 3);
        if constexpr (SPEC) spec_advance();
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    acc_add(0u, wave_sum(msg_now));
    msg_now = 0;
    if (__ballot(ovf)) status = BRC_OVERFLOW;
    else simulate_new();

    const uint64_t gm0 = (Q >= 64) ? ~0ull : ((1ull << Q) - 1);
#ifdef BRC_STAMPS
    // dev-only section timers (tools/stamps.py life): step head, HM class-code reads, consensus words,
    // sends + stop checks, lifetime simulation of the new keys
    uint64_t stamp_acc[5] = {0, 0, 0, 0, 0};
    uint64_t stamp_prev = __builtin_amdgcn_s_memtime();
#define LIFE_STAMP(i) do { const uint64_t _n = __builtin_amdgcn_s_memtime(); stamp_acc[i] += _n - stamp_prev; stamp_prev = _n; } while (0)
#else
#define LIFE_STAMP(i) do {} while (0)
#endif
    while (status == BRC_RUNNING) {
        // next step with arrivals at an honest receiver
        const uint32_t rot = (t + 1) & (RW - 1);
        const RowT rr = (RowT)((rot ? ((rows >> rot) | (rows << (RW - rot))) : rows) & RWM);
        if (!rr) { status = BRC_QUIESCENT; break; }
        const uint32_t next = t + 1 + (uint32_t)__builtin_ctzll(rr);
        if (next > P.step_cap) { status = BRC_STEPCAP; break; }
        t = uni32(next);
        const uint32_t row = t & (RW - 1);
        // commit the step's statistics
        {
            const uint32_t a = uni32(rl(rg_arr, (int)row)), mg = uni32(rl(rg_msg, (int)row));
            const uint32_t ce = uni32(rl(rg_cell, (int)row)), de = uni32(rl(rg_del, (int)row));
            acc += lane == 0 ? (uint64_t)mg : lane == 1 ? (uint64_t)a : lane == 2 ? (uint64_t)ce : lane == 3 ? (uint64_t)de : 0ull;
            if (ce) t_stop = t;
        }
        // ================= consensus: this step's deliveries in canonical (kp, s) order
        defer = true;
        LIFE_STAMP(0);
        // HM: the key words the step's summary row flags -- their class codes read from HBM 8 words at a time,
        // consumed entries cleared, the two class bitmaps of each kept in LDS for dword()
        uint64_t fw[2] = {0ull, 0ull};
        if constexpr (HM) {
            const uint32_t tc = 0x80u | (t & 0x7Fu);
            fw[0] = uni64(s_wsum[row * 2]); fw[1] = uni64(s_wsum[row * 2 + 1]);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            if (lane < 2) s_wsum[row * 2 + lane] = 0;       // consumed: the row is free for step t + LIFE_RW
            uint64_t pend[2] = {fw[0], fw[1]};
#pragma unroll 1
            while (pend[0] | pend[1]) {
                uint32_t wl[8], x[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int h = pend[0] ? 0 : 1;
                    wl[i] = 0xFFFFFFFFu; x[i] = 0u;
                    if (pend[h]) {
                        wl[i] = 64u * (uint32_t)h + (uint32_t)__builtin_ctzll(pend[h]);
                        pend[h] &= pend[h] - 1;
                        x[i] = __hip_atomic_load(g_dab + wl[i] * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    if (wl[i] == 0xFFFFFFFFu) continue;
                    const bool a = (x[i] & 0xFFu) == tc, b = ((x[i] >> 8) & 0xFFu) == tc;
                    const uint64_t kA = __ballot(a), kB = __ballot(b);
                    if (lane == 0) { s_kab[2 * wl[i]] = kA; s_kab[2 * wl[i] + 1] = kB; }
                    if (a || b)                              // consumed: free the entries for step t + 128
                        __hip_atomic_store(g_dab + wl[i] * 64 + lane, x[i] & ~((a ? 0xFFu : 0u) | (b ? 0xFF00u : 0u)),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        LIFE_STAMP(1);
        // this step's delivery bits of key word w for this lane (read once: PL clears the ring word)
        auto dword = [&](uint32_t w) -> uint64_t {
            uint64_t bits;
            if constexpr (PL) {
                uint64_t* const dp = dring + (row * nkw + w) * 64;
                bits = __hip_atomic_load(dp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (bits) __hip_atomic_store(dp, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (!cons_lane) bits = 0;
            } else if constexpr (HM) {
                bits = 0;
                if (cons_lane && ((fw[w >> 6] >> (w & 63)) & 1ull)) bits = s_kab[2 * w + (laneF ? 0u : 1u)];
            } else {
                // the keys of word w whose delivery step for this lane's class is now
                const uint32_t kk = w * 64 + lane, tc = 0x80u | (t & 0x7Fu);
                const uint32_t eA = s_dA[kk], eB = s_dB[kk];
                const uint64_t kA = __ballot(eA == tc), kB = __ballot(eB == tc);
                if (kA | kB) {                            // consumed: free the entries for step t + 128
                    if (eA == tc) s_dA[kk] = 0;
                    if (eB == tc) s_dB[kk] = 0;
                }
                bits = cons_lane ? (laneF ? kA : kB) : 0ull;
            }
            return bits;
        };
        // HM: the next key word >= w the step's summary flags (NOKEY: none) -- the consensus passes visit only
        // those, and read each one's slot metadata one flagged word (group) AHEAD, so the HBM round trip of
        // the next word overlaps the deliveries of this one (no SEND changes the metadata during the pass)
        auto next_flagged = [&](uint32_t w) -> uint32_t {
            if (w < 64) { const uint64_t x = fw[0] & (~0ull << w); if (x) return (uint32_t)__builtin_ctzll(x); w = 64; }
            if (w < 128) { const uint64_t x = fw[1] & (~0ull << (w - 64)); if (x) return 64u + (uint32_t)__builtin_ctzll(x); }
            return NOKEY;
        };
        if constexpr (QBIG) {
            // key windows of 64 / 128 (the reference protocol's many-round runs): a key prefix
            // (origin, variant) spans Q / 64 whole words; its deliveries of one step (one origin) go one
            // at a time, smallest phase index first -- the canonical (kp, s) order
            const uint32_t wpg = Q > 64 ? Q / 64 : 1u;
            uint32_t gw = next_flagged(0);
            if (gw != NOKEY) gw &= ~(wpg - 1u);                       // the flagged word's group
            uint32_t pf0 = 0, pf1 = 0;                                // the group's metadata words, in flight
            if (gw != NOKEY) {
                pf0 = mld(gw * 64 + lane);
                if (wpg > 1) pf1 = mld((gw + 1) * 64 + lane);
            }
#pragma unroll 1
            while (gw != NOKEY) {
                const uint32_t w = gw, m0 = pf0, m1 = pf1;
                gw = next_flagged(w + wpg);
                if (gw != NOKEY) {
                    gw &= ~(wpg - 1u);
                    pf0 = mld(gw * 64 + lane);
                    if (wpg > 1) pf1 = mld((gw + 1) * 64 + lane);
                }
                uint64_t gb[2] = {dword(w), wpg > 1 ? dword(w + 1) : 0ull};
                if (!__ballot((gb[0] | gb[1]) != 0)) continue;
                s_sv[lane] = m0 & 0xFFFFu;
                if (wpg > 1) s_sv[64 + lane] = m1 & 0xFFFFu;
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                if constexpr (BRC_LIFE_QBULK) {
                    // a lane whose deliveries here (one origin: one host) can end no phase -- fewer than T_cnt -
                    // vcount of them, or not in phase 1 / 2 -- and bring at most one value new to `order` takes
                    // them at once: its host joins each value's set, vcount grows by their number (the
                    // one-by-one loop below would do exactly this; only the insertion order of two or more new
                    // values needs the phase order, so those go one by one)
                    const uint32_t nb = (uint32_t)(__popcll(gb[0]) + __popcll(gb[1]));
                    if (nb && ((phase != 1 && phase != 2) || vcount + nb < P.T_cnt)) {
                        uint32_t V = 0;                       // values among the deliveries (bit v)
                        for (uint32_t j = 0; j < wpg; ++j)
                            for (uint64_t x = gb[j]; x; x &= x - 1)
                                V |= 1u << (s_sv[j * 64 + (uint32_t)__builtin_ctzll(x)] >> 14);
                        uint32_t known = 0;                   // values already in `order`
                        for (uint32_t i = 0; i < nvals; ++i) known |= 1u << ((order >> (2 * i)) & 3u);
                        const uint32_t nv = V & ~known;
                        if ((nv & (nv - 1u)) == 0) {
                            if (nv) { order |= ((uint32_t)__builtin_ctz(nv)) << (2 * nvals); ++nvals; }
                            const uint64_t hb = 1ull << (w >> (ksh - 6));      // host = origin of the group
                            for (uint32_t v = 0; v < 4; ++v)
                                if ((V >> v) & 1u) s_hm[v * 64 + lane] |= hb;
                            vcount += nb;
                            gb[0] = gb[1] = 0;
                        }
                    }
                }
                while (gb[0] | gb[1]) {
                    uint32_t bs = 0xFFFFFFFFu, bk = 0;
                    for (uint32_t j = 0; j < wpg; ++j)
                        for (uint64_t x = gb[j]; x; x &= x - 1) {
                            const uint32_t kk = (w + j) * 64 + (uint32_t)__ffsll((unsigned long long)x) - 1u;
                            const uint32_t s1 = s_sv[kk - w * 64] & 0x3FFFu;
                            if (s1 < bs) { bs = s1; bk = kk; }
                        }
                    gb[(bk >> 6) - w] &= ~(1ull << (bk & 63));
                    static_assert(!(QBIG && SPEC), "QBIG: reference protocol");
                    cons_deliver_vh(s_sv[bk - w * 64] >> 14, bk >> ksh);
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            }
        } else {
        uint32_t pfw = NOKEY, pf = 0;                 // HM: the next flagged word and its metadata, in flight
        if (HM) {
            pfw = next_flagged(0);
            if (pfw != NOKEY) pf = mld(pfw * 64 + lane);
        }
#pragma unroll 1
        for (uint32_t w = HM ? pfw : 0u; w < nkw; w = HM ? pfw : w + 1u) {
            uint64_t bits = dword(w);
            if (HM) {
                const uint32_t m = pf;
                pfw = next_flagged(w + 1u);
                if (pfw != NOKEY) pf = mld(pfw * 64 + lane);
                if (__ballot(bits != 0)) {             // the word's slot metadata (read one flagged word ahead)
                    s_sv[lane] = m & 0xFFFFu;
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                }
            }
            if constexpr (SPEC) {
                // word at once when every delivering lane is at one phase index c0 and its current-phase
                // deliveries cannot complete the phase (brc_step.h, SPEC consensus pass)
                const uint64_t hb = __ballot(bits != 0);
                if (!seen_on && hb) {
                    const uint32_t cur = round ? 2 * (round - 1) + (phase - 1) : 0u;
                    const uint32_t c0 = uni32((uint32_t)__builtin_amdgcn_readlane((int)cur, __ffsll((unsigned long long)hb) - 1));
                    if (!__ballot(bits != 0 && cur != c0)) {
                        const uint32_t sn = snap(w * 64 + lane);
                        const uint32_t ss = (sn & 0x3FFFu) - 1u, sv = sn >> 14;
                        const uint64_t inw = __ballot(ss >= c0 && ss - c0 < Q), atc = __ballot(ss == c0);
                        const uint64_t past = __ballot(ss != 0xFFFFFFFFu && ss >= c0 && ss - c0 >= Q);
                        const uint64_t v1 = __ballot(sv == 1), v2 = __ballot(sv == 2);
                        const uint32_t ncur = (uint32_t)__popcll(bits & atc);
                        const uint32_t qc = c0 & Qm;
                        if (bits && (round == 0 || (s_cnt[qc * 64 + lane] & 0x3FFu) + ncur < n - P.f)) {
                            if (bits & past) ovf = true;
                            const uint64_t b = bits & inw;
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
            } else {
                // word at once when no phase can change (brc_step.h, REFERENCE consensus pass)
                if (__ballot(bits != 0)) {
                    const uint32_t sv = snap_w(w * 64 + lane) >> 14;
                    const uint64_t vm[4] = {__ballot(sv == 0), __ballot(sv == 1), __ballot(sv == 2), __ballot(sv == 3)};
                    const uint32_t nb = (uint32_t)__popcll(bits);
                    const bool oneper = (uint32_t)__popcll(fold_groups(bits, Q)) == nb;
                    if (nb && oneper && ((phase != 1 && phase != 2) || vcount + nb < P.T_cnt)) {
                        const uint32_t G = Q * NV, opw = 64u / G;
                        uint32_t first[4];
#pragma unroll
                        for (int v = 0; v < 4; ++v) {
                            const uint64_t dv = bits & vm[v];
                            first[v] = dv ? (uint32_t)__ffsll((unsigned long long)dv) - 1u : 64u;
                            if (dv) s_hm[v * 64 + lane] |= compress_groups(fold_groups(dv, G), G) << (w * opw);
                            const uint32_t xo = order ^ ((uint32_t)v * 0x55u);
                            if (((~(xo | (xo >> 1)) & 0x55u & ((1u << (2 * nvals)) - 1u)) != 0)) first[v] = 64u;
                        }
                        for (int r = 0; r < 4; ++r) {
                            uint32_t bv = 0, bp = 64u;
#pragma unroll
                            for (int v = 0; v < 4; ++v) if (first[v] < bp) { bp = first[v]; bv = (uint32_t)v; }
                            if (bp == 64u) break;
                            order |= bv << (2 * nvals); ++nvals;
#pragma unroll
                            for (int v = 0; v < 4; ++v) if ((uint32_t)v == bv) first[v] = 64u;
                        }
                        vcount += nb;
                        bits = 0;
                    }
                }
            }
            // one delivery at a time, ascending slot; several phases of one key prefix: smallest s first
            while (bits) {
                uint32_t best = __ffsll((unsigned long long)bits) - 1;
                const uint64_t grp = bits & (gm0 << (best & ~Qm));
                if (grp & (grp - 1)) {
                    uint32_t bs = 0xFFFFFFFFu;
                    for (uint64_t x = grp; x; x &= x - 1) {
                        const uint32_t bb = __ffsll((unsigned long long)x) - 1;
                        const uint32_t s1 = snap_w(w * 64 + bb) & 0x3FFFu;
                        if (s1 < bs) { bs = s1; best = bb; }
                    }
                }
                bits &= ~(1ull << best);
                if constexpr (SPEC) spec_deliver(w * 64 + best);
                else cons_deliver_vh(snap_w(w * 64 + best) >> 14, (w * 64 + best) >> ksh);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        LIFE_STAMP(2);
        defer = false;
        flush_sends();                                // the SENDs this step's consensus started
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        acc_add(0u, wave_sum(msg_now));
        msg_now = 0;
        // the step is consumed: its ring row is free for step t + RW
        if (lane == row) { rg_arr = 0; rg_msg = 0; rg_cell = 0; rg_del = 0; }
        rows &= ~((RowT)1 << row);
        // ================= per-instance stop conditions (brc_step.h)
        const uint64_t b_und = __ballot(honest && dcount < P.round_cap);
        if (__ballot(ovf)) status = BRC_OVERFLOW;
        else if (P.round_cap > 0 && !b_und) status = BRC_DONE;
        LIFE_STAMP(3);
        if (status == BRC_RUNNING) simulate_new();    // the keys this step's consensus created
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        LIFE_STAMP(4);
    }
#ifdef BRC_STAMPS
    if (lane == 0) for (int i = 0; i < 5; ++i) atomicAdd(&brc_stamps[i], (unsigned long long)stamp_acc[i]);
#endif
#undef LIFE_STAMP
    if (__ballot(ovf) && status != BRC_OVERFLOW) status = BRC_OVERFLOW;
    if constexpr (PL) {
        // rows of steps the instance did not reach: leave the bitmap ring zero for the next launch
        for (uint64_t rm = rows; rm; rm &= rm - 1) {
            const uint32_t row = (uint32_t)__builtin_ctzll(rm);
            for (uint32_t w = 0; w < nkw; ++w)
                __hip_atomic_store(dring + (row * nkw + w) * 64, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }

    // ---- write back (result readers: inst, istats, items, cons0/cons1, gcount)
    const uint64_t tot_msg = acc_get(0), tot_arr = acc_get(1), tot_cell = acc_get(2), tot_del = acc_get(3);
    const uint64_t key_steps = acc_get(4);
    if (lane == 0) {
        gptr_t<uint64_t> ip = (gptr_t<uint64_t>)&gp(P.inst)[inst];
        *ip = (uint64_t)(status & 0xFFFF) | ((uint64_t)(t_stop & 0xFFFF) << 16) | ((uint64_t)(t & 0xFFFF) << 32);
        gp(P.istats)[inst * 4 + 0] = tot_msg;
        gp(P.istats)[inst * 4 + 1] = tot_arr;
        gp(P.istats)[inst * 4 + 2] = tot_cell;
        gp(P.istats)[inst * 4 + 3] = tot_del;
        ItemState o = {t, 0u, 1u, 0u};
        P.items[item] = o;
        gp(P.actany)[item] = 0;
    }
    const size_t li = item * 64 + lane;
    if (honest) {
        gp(P.cons0)[li] = cons0_pack(round, phase, nvals, order, vcount);
        gp(P.cons1)[li] = (uint64_t)(dcount & 0xFFFF) | ((uint64_t)(frnd & 0xFFFF) << 16) | ((uint64_t)(ft & 0xFFFF) << 32) |
                          ((uint64_t)(fval & 0xFF) << 48) | ((uint64_t)(lval & 0xFF) << 56);
    }
    uint32_t smax = st_smax;
#pragma unroll
    for (int o2 = 32; o2; o2 >>= 1) smax = max(smax, (uint32_t)__shfl_xor((int)smax, o2));
    if (lane == 0) {
        const unsigned long long w6[5] = {tot_cell, tot_arr, tot_msg, tot_del, key_steps * 64ull};
#pragma unroll
        for (int q = 0; q < 5; ++q) if (w6[q]) atomicAdd(&P.gcount[q], w6[q]);
        if (smax) atomicMax(&P.gcount[5], (unsigned long long)smax);
    }
}

template <int MODE, bool PL, int DLX = 8, bool QBIG = false, bool HMT = false>
int launch_life_one(uint32_t blocks, uint32_t lds, hipStream_t s, const Params* P) {
    auto kern = brc_life<MODE, PL, DLX, QBIG, HMT>;
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return BRC_E_HIP;
    kern<<<dim3(blocks), dim3(64), lds, s>>>(P);
    return hipGetLastError() == hipSuccess ? 0 : BRC_E_HIP;
}

}  // namespace brc
