// brc_engine.hip -- host side of the MI355X batched consensus engine: the C-ABI of
// include/brc.h (brc_create ... brc_destroy), device memory, injection CSR upload, and the small
// helper kernels.  The step kernel itself is brc_step.h, instantiated per replica-set width in
// brc_kern_<NPAD>.hip.
//
// Reference boundary replaced (sithu/ByzantineRandomizedConsensus):
//   BRBroadcast / ByzantineRandomizedConsensus constructors  -> brc_create
//   the listener accept loop (core/brbroadcast.py:60-128)     -> brc_run (one step-kernel launch)
//   Broadcast.broadcast / Consensus.propose                   -> brc_inject / brc_load_proposals
//   deliver / decide upcalls                                  -> brc_read_events / brc_read_replicas
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>
#include <unordered_map>

#include "brc_internal.h"

namespace {

using namespace brc;

// Byzantine equivocation pattern expanded straight into the CSR lists.
// bw: Byzantine-mask words per instance (n > 64: one instance per item, ipw = 1)
__global__ void expand_equivocate(InjDev* inj, uint32_t* off, uint32_t* cnt, const uint64_t* byz,
                                  uint64_t instances, uint64_t nitems, uint32_t ipw, uint32_t n, uint32_t nv,
                                  uint32_t Q, uint32_t per_item, uint32_t bw) {
    const uint64_t item = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (item >= nitems) return;
    InjDev* o = inj + item * per_item;
    uint32_t c = 0;
    uint64_t even[4] = {0, 0, 0, 0}, odd[4] = {0, 0, 0, 0};   // 64 is even: bit parity = replica parity
    for (uint32_t dd = 0; dd < n; ++dd) {
        if (dd & 1) odd[dd >> 6] |= 1ull << (dd & 63); else even[dd >> 6] |= 1ull << (dd & 63);
    }
    for (int pass = 0; pass < 2; ++pass) {
        for (uint32_t sgi = 0; sgi < ipw; ++sgi) {
            const uint64_t in = item * ipw + sgi;
            if (in >= instances) break;
            for (uint32_t b = 0; b < n; ++b) {
                if (!((byz[in * bw + (b >> 6)] >> (b & 63)) & 1ull)) continue;
                for (uint32_t v = 0; v < 2; ++v) {
                    const uint32_t kp = b * nv + v;
                    InjDev r = {};
                    r.slot = (uint16_t)(kp * Q + 0); r.s = 0; r.seg = (uint8_t)sgi; r.node = (uint8_t)b;
                    r.value = (int8_t)(1 + v);
                    if (pass == 0) {
                        r.t = 0; r.kind = BRC_INJ_SEND; r.type = BRC_SEND; r.restricted = 1;
                        const uint64_t* dm = v ? odd : even;
                        r.dst = dm[0]; r.dst_hi[0] = dm[1]; r.dst_hi[1] = dm[2]; r.dst_hi[2] = dm[3];
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

// brc_reset: free every slot but keep its generation.  Cells are left alone: the next
// allocation of a slot bumps its generation, which makes every cell of the old key stale
// (send steps included, brc_step.h), so a reset costs O(keys), not O(cells).
__global__ void reset_slots(uint64_t* meta, uint32_t* mgen, uint64_t keys) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < keys) { meta[i] = 0; mgen[i] &= GEN_MASK; }
}

// Decide-round histogram: per instance, the round by which EVERY honest replica
// had decided (max of the first-decide rounds); bin 0 = some honest replica never decided; rounds
// >= bins-1 share the last bin.  One thread per instance; the bins are reduced in LDS first.
__global__ void round_histogram(const uint64_t* cons1, const uint64_t* byz, uint64_t instances, uint32_t ipw,
                                uint32_t lpi, uint32_t npad, uint32_t bw, uint32_t n, uint32_t bins,
                                unsigned long long* hist) {
    extern __shared__ unsigned long long sh[];
    for (uint32_t b = threadIdx.x; b < bins; b += blockDim.x) sh[b] = 0;
    __syncthreads();
    const uint64_t in = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (in < instances) {
        const uint64_t item = in / ipw, seg = in % ipw;
        uint32_t worst = 0;
        bool all = true;
        for (uint32_t d = 0; d < n; ++d) {
            if ((byz[in * bw + d / 64] >> (d % 64)) & 1ull) continue;
            const uint64_t c1 = cons1[item * lpi + seg * npad + d];
            if ((c1 & 0xFFFF) == 0) { all = false; break; }
            worst = max(worst, (uint32_t)((c1 >> 16) & 0xFFFF));
        }
        const uint32_t bin = all ? min(worst, bins - 1) : 0u;
        atomicAdd(&sh[bin], 1ull);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < bins; b += blockDim.x)
        if (sh[b]) atomicAdd(&hist[b], sh[b]);
}

// First decisions of the honest replicas (brc_read_value_decisions): per instance, count each honest
// replica's first decided value id (bin 8: never decided) and flag instances whose honest replicas
// decided different values.  One thread per instance; bins reduced in LDS first.
__global__ void decision_histogram(const uint64_t* cons1, const uint64_t* byz, uint64_t instances, uint32_t ipw,
                                   uint32_t lpi, uint32_t npad, uint32_t bw, uint32_t n,
                                   unsigned long long* out /* [10]: 9 value bins, disagreements */) {
    __shared__ unsigned long long sh[10];
    if (threadIdx.x < 10) sh[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t in = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (in < instances) {
        const uint64_t item = in / ipw, seg = in % ipw;
        uint32_t cnt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        uint32_t seen = 0;                       // value ids decided by some honest replica
        for (uint32_t d = 0; d < n; ++d) {
            if ((byz[in * bw + d / 64] >> (d % 64)) & 1ull) continue;
            const uint64_t c1 = cons1[item * lpi + seg * npad + d];
            if ((c1 & 0xFFFF) == 0) { ++cnt[8]; continue; }
            const uint32_t v = (uint32_t)(c1 >> 48) & 7u;      // first decided value id
            ++cnt[v];
            seen |= 1u << v;
        }
        for (int b = 0; b < 9; ++b) if (cnt[b]) atomicAdd(&sh[b], (unsigned long long)cnt[b]);
        if (seen & (seen - 1)) atomicAdd(&sh[9], 1ull);
    }
    __syncthreads();
    if (threadIdx.x < 10 && sh[threadIdx.x]) atomicAdd(&out[threadIdx.x], sh[threadIdx.x]);
}

// grid-stride fill: a dispatch holds < 2^32 work-items per dimension, and the cell array can
// exceed that (2^17 instances x 512 key slots x 64 lanes = 2^32 words at n = 64, Q = 8)
template <typename W> __global__ void fill_words(W* p, W v, uint64_t count) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) p[i] = v;
}

// ------------------------------------------------------------------------------------ host
struct Engine {
    brc_config cfg;
    int npad = 0, dm = 0, ipw = 0, nkw_t = 0;
    bool wide = false;                           // n > 64: one workgroup per instance (brc_step_wide.h)
    bool wide_wv4 = false;                       // wide: the 4-waves-per-SIMD instantiations (brc_step_wide.h WV)
    bool regmask = false;                        // NPAD = 64 lean kernel with register delay masks (NLR = 2)
    bool compact = false;                        // lean kernels (NPAD = 64, sender peers): u32 cells (C32_*)
    bool general = false;                        // BRC_FLAG_GENERAL_KEYS at NPAD = 64 (KMODE_XREF)
    uint32_t lpi = 64;                           // replica lanes per item (64, or NPAD when wide)
    uint32_t bw = 1;                             // Byzantine-mask words per instance
    uint32_t NK = 0, nkw = 0, msize = 0, lds_bytes = 0;
    uint32_t rows = 0;                           // cell rows per item
    uint32_t rs = TS;                            // activity-ring rows: ring_steps(dm)
    uint64_t cons_bytes = 0;                     // consensus-set buffer (hmask) bytes per item
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
    uint64_t* dbits = nullptr;                   // lean SPEC: per-wave delivery bitmaps (brc_step.h DBG)
    uint64_t* dring = nullptr;                   // per-link lifetime kernel: delivery bitmap ring (brc_life.h)
    uint32_t* lmeta = nullptr;                   // lifetime kernel, key windows >= 64: slot metadata in HBM
    uint64_t* xsend = nullptr; uint32_t* xsn = nullptr;   // extra-SEND records (non-lean step kernels)
    bool life_pl = false;                        // lifetime kernel in its per-link delay form
    uint32_t life_rw = LIFE_RW;                  // ... its delivery-ring rows (LIFE_RW16 for delays above 8)
    uint32_t nval = 4;                           // consensus value ids the step kernel keeps (value_ids)
    bool values_wide = false;                    // a loaded proposal uses a value id >= 4 (no lifetime kernel)
    Params* dparams = nullptr;                   // device copy of the launch parameters
    Params hparams;
    std::vector<std::vector<InjDev>> pending;   // per item: uploaded-but-unconsumed + new
    bool inj_dirty = false, pattern_active = false;
    // slot generation budget: reallocations of one key slot are bounded by max phase index / Q + 2
    // per epoch (brc_reset to brc_reset); gen_base sums the epochs since the last full clear
    uint64_t gen_base = 0, gen_cur = 0;
    // injected SENDs per key (instance << 32 | kp << 16 | s): how many, and each sender's destinations
    std::unordered_map<uint64_t, uint32_t> send_count;
    std::unordered_map<uint64_t, std::vector<std::pair<uint32_t, uint64_t>>> send_dst;
    struct XRec { uint32_t k, t, seg; uint64_t smask, dst; };
    std::unordered_map<uint64_t, std::vector<XRec>> xrec;   // item -> extra-SEND records (P.xsend)
    // key-lifetime kernel (brc_life.h): eligible configuration, engine fresh since create / reset,
    // and whether the last run used it (its instances are then final: no re-opening injections)
    bool life_cfg = false, fresh = true, life_done = false, last_life = false;
    // false: the step kernel cannot serve this engine (its cells would not fit, or a lean key window
    // above 32): only the key-lifetime kernel runs, and the step kernel's key-slot arrays are not allocated
    bool step_ok = true;
    bool cells_ready = false;                    // the step kernel's cell array (allocated on first use
                                                 // when the lifetime kernel may serve the engine)
    uint32_t life_lds = 0;
};

thread_local std::string g_create_err;    // brc_last_error(NULL): the last brc_create failure

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

// bits of replicas 64w .. 64w+63 that exist in an n-replica instance
static uint64_t word_mask(uint32_t n, uint32_t w) {
    const uint32_t lo = 64 * w;
    return n >= lo + 64 ? ~0ull : (n <= lo ? 0ull : ((1ull << (n - lo)) - 1));
}

static int pick_dm(uint32_t d) { return d <= 4 ? 4 : d <= 8 ? 8 : 16; }

static int launch_step(int npad, int dm, bool events, int mode, bool wv4, uint32_t blocks, uint32_t lds, hipStream_t st,
                       const Params* P) {
    switch (npad) {
    case 4: return launch_step_4(dm, events, mode, blocks, lds, st, P);
    case 8: return launch_step_8(dm, events, mode, blocks, lds, st, P);
    case 16: return launch_step_16(dm, events, mode, blocks, lds, st, P);
    case 32: return launch_step_32(dm, events, mode, blocks, lds, st, P);
    case 64: return launch_step_64(dm, events, mode, blocks, lds, st, P);
    case 128: return launch_step_128(dm, events, mode, wv4, blocks, lds, st, P);
    case 256: return launch_step_256(dm, events, mode, wv4, blocks, lds, st, P);
    default: return BRC_E_INVALID;
    }
}

static void free_all(Engine* e) {
    void* ps[] = {e->cells, e->meta, e->mgen, e->kdst, e->act, e->actany, e->items, e->inst, e->istats,
                  e->cons0, e->cons1, e->hmask, e->inj, e->inj_off, e->inj_cnt, e->byz, e->prop, e->events,
                  e->event_count, e->gcount, e->dbits, e->dring, e->lmeta, e->xsend, e->xsn, e->dparams};
    for (void* p : ps) if (p) (void)hipFree(p);
    if (e->ev0) (void)hipEventDestroy(e->ev0);
    if (e->ev1) (void)hipEventDestroy(e->ev1);
    if (e->stream) (void)hipStreamDestroy(e->stream);
}

static int fill_cells(Engine* e) {
    const size_t cells = (size_t)e->nitems * e->rows * e->lpi;
    const uint64_t fb = std::min<uint64_t>((cells + 255) / 256, 1u << 20);
    if (e->compact)
        hipLaunchKernelGGL(fill_words<uint32_t>, dim3((uint32_t)fb), dim3(256), 0, e->stream, (uint32_t*)e->cells,
                           C32_FRESH, (uint64_t)cells);
    else
        hipLaunchKernelGGL(fill_words<uint64_t>, dim3((uint32_t)fb), dim3(256), 0, e->stream, e->cells, TIMES_NEVER,
                           (uint64_t)cells);
    HIPCHK(e, hipGetLastError());
    return BRC_OK;
}

// the step kernel's cells, allocated at its first launch on an engine the lifetime kernel may serve
static int ensure_cells(Engine* e) {
    if (e->cells_ready) return BRC_OK;
    const size_t bytes = (size_t)e->nitems * e->rows * e->lpi * (e->compact ? 4 : 8);
    if (e->cells) (void)hipFree(e->cells);
    e->cells = nullptr;
    if (hipMalloc(&e->cells, std::max<size_t>(bytes, 8)) != hipSuccess) {
        (void)hipGetLastError();
        e->err = "device allocation of " + std::to_string(bytes) + " B of step-kernel cells failed";
        return BRC_E_NOMEM;
    }
    e->cells_ready = true;
    return fill_cells(e);
}

static int clear_state(Engine* e, bool full) {
    const size_t keys = (size_t)e->cfg.instances * e->NK;
    if (!e->step_ok) {
        // lifetime kernel only: it keeps key slots in LDS; no cells, key metadata or activity ring
    } else if (full) {
        if (e->cells_ready) {
            const int rc = fill_cells(e);
            if (rc) return rc;
        }
        HIPCHK(e, hipMemsetAsync(e->meta, 0, keys * 8, e->stream));
        HIPCHK(e, hipMemsetAsync(e->mgen, 0, keys * 4, e->stream));
        e->gen_base = 0;
        e->gen_cur = 0;
    } else {
        hipLaunchKernelGGL(reset_slots, dim3((uint32_t)((keys + 255) / 256)), dim3(256), 0, e->stream, e->meta, e->mgen,
                           (uint64_t)keys);
        HIPCHK(e, hipGetLastError());
    }
    if (e->step_ok)
        HIPCHK(e, hipMemsetAsync(e->act, 0, (size_t)e->nitems * e->rs * e->nkw * act_types(e->compact, e->ipw) * 8, e->stream));
    HIPCHK(e, hipMemsetAsync(e->actany, 0, (size_t)e->nitems * 4, e->stream));
    HIPCHK(e, hipMemsetAsync(e->items, 0, (size_t)e->nitems * sizeof(ItemState), e->stream));
    HIPCHK(e, hipMemsetAsync(e->inst, 0, (size_t)e->cfg.instances * sizeof(InstState), e->stream));
    HIPCHK(e, hipMemsetAsync(e->istats, 0, (size_t)e->cfg.instances * 4 * 8, e->stream));
    HIPCHK(e, hipMemsetAsync(e->cons0, 0, (size_t)e->nitems * e->lpi * 8, e->stream));
    HIPCHK(e, hipMemsetAsync(e->cons1, 0, (size_t)e->nitems * e->lpi * 8, e->stream));
    HIPCHK(e, hipMemsetAsync(e->hmask, 0, (size_t)e->nitems * e->cons_bytes, e->stream));
    HIPCHK(e, hipMemsetAsync(e->gcount, 0, 8 * 8, e->stream));
    if (!e->compact && !e->wide) HIPCHK(e, hipMemsetAsync(e->xsn, 0, (size_t)e->nitems * 4, e->stream));
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
                       e->cfg.key_window, cap, e->bw);
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
    if (!h) return g_create_err.c_str();   // why the last brc_create on this thread failed
    return static_cast<Engine*>(h)->err.c_str();
}

int brc_create(const brc_config* cfg, void** out) {
    g_create_err.clear();
    if (!cfg || !out) { g_create_err = "null argument"; return BRC_E_INVALID; }
    *out = nullptr;
    const brc_config& c = *cfg;
    if (c.n < 1 || c.n > 256 || c.instances == 0 || c.delay_max < 1 || c.delay_max > 16 ||
        c.step_cap > STEP_LIMIT || c.peer_mode > BRC_PEER_CONNECTION ||
        (c.peer_mode == BRC_PEER_CONNECTION && c.mode != BRC_MODE_REFERENCE) ||
        (c.protocol != BRC_PROTO_BRB && c.protocol != BRC_PROTO_CONSENSUS) || c.delay_model > BRC_DELAY_GEOMETRIC ||
        (c.delay_model == BRC_DELAY_CONST && (c.delay_const < 1 || c.delay_const > c.delay_max)) ||
        !(c.key_window == 2 || c.key_window == 4 || c.key_window == 8 || c.key_window == 16 || c.key_window == 32 ||
          c.key_window == 64 || c.key_window == 128) ||
        !(c.variants == 1 || c.variants == 2 || c.variants == 4) ||
        // more than 8 live phase indices per origin: reference / best-effort protocols on the narrow kernels
        // (up to 128: the reference protocol's many-round runs; the lean kernels take <= 32 and
        // leave larger windows to the key-lifetime kernel, below)
        c.key_window * c.variants > ((c.mode != BRC_MODE_SPEC && c.n <= 64) ? 128u : 8u) ||
        c.f >= c.n || (c.byz_pattern == BRC_BYZ_EQUIVOCATE && c.variants < 2) ||
        (c.byz_pattern != BRC_BYZ_NONE && c.byz_pattern != BRC_BYZ_EQUIVOCATE) ||
        c.proposals > BRC_PROPOSALS_LOADED || c.mode > BRC_MODE_BEB || (c.flags & ~(uint32_t)BRC_FLAG_GENERAL_KEYS) ||
        // the general form at NPAD = 64 with sender peers is the reference protocol's (KMODE_XREF)
        ((c.flags & BRC_FLAG_GENERAL_KEYS) && c.n > 32 && c.n <= 64 && c.peer_mode == BRC_PEER_SENDER &&
         c.mode != BRC_MODE_REFERENCE) ||
        (c.n > 64 && c.mode == BRC_MODE_SPEC && c.variants != 1))
    {
        g_create_err = "invalid configuration (see include/brc.h field ranges)";
        return BRC_E_INVALID;
    }
    Engine* e = new Engine();
    e->cfg = c;
    e->npad = pick_npad(c.n);
    e->dm = pick_dm(c.delay_max);
    e->rs = ring_steps(e->dm);
    e->wide = e->npad > 64;
    e->ipw = e->wide ? 1 : 64 / e->npad;
    e->lpi = e->wide ? (uint32_t)e->npad : 64u;
    e->bw = e->wide ? (uint32_t)e->npad / 64 : 1u;
    e->nkw_t = e->npad / 8 < 1 ? 1 : e->npad / 8;
    e->NK = (uint32_t)e->npad * c.variants * c.key_window;
    // narrow kernel: + the trash row (brc_step.h); connection peers: 5 words per cell (the cell word
    // and two 16-step send-count rings, brc_step.h Ring16)
    const uint32_t cw = c.peer_mode == BRC_PEER_CONNECTION ? 5u : 1u;
    e->rows = e->wide ? e->NK * cw : (e->NK + 1) * cw;
    e->nkw = (e->NK + 63) / 64;
    e->msize = e->npad <= 8 ? 1 : (uint32_t)e->npad / 8;
    e->nitems = (c.instances + e->ipw - 1) / e->ipw;
    const bool spec = c.mode == BRC_MODE_SPEC;
    const uint32_t nL = delay_values(c.delay_model, c.delay_max);
    // BRC_FLAG_GENERAL_KEYS: NPAD = 64 with sender peers on the general form (KMODE_XREF), not the lean one
    e->general = (c.flags & BRC_FLAG_GENERAL_KEYS) && e->npad == 64 && c.peer_mode == BRC_PEER_SENDER;
    e->regmask = e->npad == 64 && c.peer_mode == BRC_PEER_SENDER && nL <= 2 && !e->general;
    e->compact = e->npad == 64 && c.peer_mode == BRC_PEER_SENDER && !e->general;   // = lean_kernel<64, mode> (brc_step.h)
    // wide exchange words per (key, type): connection peers send 8 count planes per link delay
    const uint32_t xw = c.peer_mode == BRC_PEER_CONNECTION ? 8u * nL : xwords_wide(c.delay_model, c.delay_max, e->dm);
    e->lds_bytes = e->wide ? lds_bytes_wide(e->npad, e->NK, e->nkw, xw,
                                            spec, c.key_window, e->rs)
                           : lds_bytes_per_wave(e->npad, e->NK, e->nkw, e->regmask ? 0u : nL, spec, c.key_window,
                                                c.variants, e->rs, e->compact) * WPB;
    // wide kernel at 4 waves per SIMD (128 VGPRs): DM <= 8 without delay-code planes in registers (constant /
    // slow-set delays), sender peers, and LDS for four workgroups per CU
    e->wide_wv4 = e->wide && e->dm <= 8 && !plane_model(c.delay_model) && c.peer_mode == BRC_PEER_SENDER &&
                  e->lds_bytes <= 40u * 1024u;
    e->nval = value_ids(!e->compact && !e->wide);
    e->cons_bytes = cons_bytes_per_item(spec, e->wide, e->lpi, e->msize, c.key_window, c.variants, e->nval);
    // key-lifetime kernel (brc_life.h): NPAD = 64 consensus under a two-class delay model with D <= 8
    // or per-link (uniform / geometric) delays with D <= 8, proposals from Philox or loaded, no event
    // log, no Byzantine pattern.  BRC_KERNEL=step | life | auto (default): auto runs it whenever the
    // configuration is eligible, except sender peers under per-link delays (the step kernel is faster
    // there): since round 6 its two-class form simulates a step's new keys one per lane, 1.8-7x faster than
    // the step kernel on cfg4.  A run it cannot take (injections, an event log, a stepped run)
    // falls back to the step kernel.
    // The lifetime kernel keeps no cells, so it also runs sender peers whose step-kernel cell store
    // would not fit in the free device memory (the reference protocol's many-round runs: its phase
    // leakage keeps ~1,000 keys of one instance live by round 8 at n = 64) and the key
    // windows above 32 the lean step kernel does not take.
    {
        const char* kv = getenv("BRC_KERNEL");
        const bool force_step = kv && strcmp(kv, "step") == 0, force_life = kv && strcmp(kv, "life") == 0;
        e->life_pl = c.delay_model == BRC_DELAY_UNIFORM || c.delay_model == BRC_DELAY_GEOMETRIC;
        e->life_lds = lds_bytes_life(e->NK, spec, c.key_window, c.variants, e->life_pl);
        e->life_rw = (e->life_pl && c.delay_max > 8) ? LIFE_RW16 : LIFE_RW;
        const bool eligible = e->npad == 64 && c.protocol == BRC_PROTO_CONSENSUS && !e->general &&
                              c.proposals != BRC_PROPOSALS_NONE && c.event_capacity == 0 && c.byz_pattern == BRC_BYZ_NONE &&
                              c.delay_max <= (e->life_pl ? 16u : 8u) && e->life_lds <= 160 * 1024 &&
                              // per-link form: its HBM delivery ring is [RW][NK] bits per instance
                              !(e->life_pl && c.key_window * c.variants > 32);
        bool big = e->compact && c.key_window * c.variants > 32;          // the lean kernels take <= 32
        if (!big && e->compact && c.peer_mode == BRC_PEER_SENDER && hipSetDevice(c.device) == hipSuccess) {
            // the step kernel's whole per-instance state (cells, slot metadata / generations / destinations,
            // activity ring) against 90 % of the device's TOTAL memory: the choice depends on the
            // configuration and the device model only, never on what else holds memory at the time (an
            // engine whose state fits but cannot be allocated now fails brc_create with BRC_E_NOMEM)
            size_t fr = 0, tot = 0;
            const size_t keys = (size_t)c.instances * e->NK;
            const size_t need = (size_t)e->nitems * (e->NK + 1) * 64 * 4 + keys * (8 + 4 + 8) +
                                (size_t)e->nitems * e->rs * e->nkw * act_types(true, 1) * 8;
            if (hipMemGetInfo(&fr, &tot) == hipSuccess && need > tot / 10 * 9) big = true;
            (void)hipGetLastError();
        }
        const bool prefer_life = c.peer_mode == BRC_PEER_CONNECTION || !e->life_pl;
        e->life_cfg = eligible && !force_step && (force_life || prefer_life || big);
        e->step_ok = !big;
        if (big && !e->life_cfg) {
            g_create_err = c.key_window * c.variants > 32
                ? "key windows above 32 at n in 33..64 with sender peers run on the key-lifetime kernel only "
                  "(consensus, Philox / loaded proposals, delay_max <= 8, constant or slow-set delays, no event log)"
                : "the step kernel's cells do not fit in free device memory and the key-lifetime kernel cannot run "
                  "this configuration";
            delete e;
            return BRC_E_INVALID;
        }
    }
    if ((e->step_ok && ((e->wide && e->nkw > (uint32_t)e->nkw_t) ||
                        e->lds_bytes > 160 * 1024)) || e->nitems > 0x7FFFFFFFull * WPB) {
        g_create_err = "configuration exceeds the kernel's LDS / key-slot limits (lds " + std::to_string(e->lds_bytes) + " B)";
        delete e;
        return BRC_E_INVALID;
    }
    auto fail = [&](int code) {
        g_create_err = e->err.empty() ? std::string("brc_create: HIP call failed: ") + hipGetErrorString(hipGetLastError())
                                      : e->err;
        free_all(e); delete e; return code;
    };
    if (hipSetDevice(c.device) != hipSuccess) { g_create_err = "hipSetDevice failed"; delete e; return BRC_E_HIP; }
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) return fail(BRC_E_HIP);
    if (hipEventCreate(&e->ev0) != hipSuccess || hipEventCreate(&e->ev1) != hipSuccess) return fail(BRC_E_HIP);
    const size_t cells = (size_t)e->nitems * e->rows * e->lpi;
    const size_t keys = e->step_ok ? (size_t)c.instances * e->NK : 1;    // the step kernel's key-slot arrays
    struct A { void** p; size_t bytes; } allocs[] = {
        {(void**)&e->cells, e->life_cfg ? 8 : cells * (e->compact ? 4 : 8)}, {(void**)&e->meta, keys * 8}, {(void**)&e->mgen, keys * 4},
        {(void**)&e->kdst, keys * 8 * e->bw},
        {(void**)&e->act, e->step_ok ? (size_t)e->nitems * e->rs * e->nkw * act_types(e->compact, e->ipw) * 8 : 8},
        {(void**)&e->actany, (size_t)e->nitems * 4}, {(void**)&e->items, (size_t)e->nitems * sizeof(ItemState)},
        {(void**)&e->inst, c.instances * sizeof(InstState)}, {(void**)&e->istats, c.instances * 32},
        {(void**)&e->cons0, (size_t)e->nitems * e->lpi * 8}, {(void**)&e->cons1, (size_t)e->nitems * e->lpi * 8},
        {&e->hmask, (size_t)e->nitems * e->cons_bytes}, {(void**)&e->inj_off, (size_t)e->nitems * 4},
        {(void**)&e->inj_cnt, (size_t)e->nitems * 4}, {(void**)&e->byz, c.instances * e->bw * 8}, {(void**)&e->gcount, 64},
        {(void**)&e->dparams, sizeof(Params)},
        {(void**)&e->dbits, (e->compact && spec && e->step_ok) ? (size_t)e->nitems * e->nkw * 64 * 8 : 8},
        {(void**)&e->dring, (e->life_cfg && e->life_pl) ? (size_t)e->nitems * e->life_rw * e->nkw * 64 * 8 : 8},
        {(void**)&e->lmeta, (e->life_cfg && life_hbm_meta(c.key_window, e->life_pl)) ? (size_t)e->nitems * e->NK * 8 : 8},
        // extra-SEND records: the non-lean narrow kernels only (the lean and wide kernels refuse extra SENDs)
        {(void**)&e->xsend, (e->compact || e->wide) ? 8 : (size_t)e->nitems * XSEND_MAX * 24},
        {(void**)&e->xsn, (e->compact || e->wide) ? 8 : (size_t)e->nitems * 4},
    };
    for (auto& a : allocs)
        if (hipMalloc(a.p, std::max<size_t>(a.bytes, 8)) != hipSuccess) {
            e->err = "device allocation of " + std::to_string(a.bytes) + " B failed";
            return fail(BRC_E_NOMEM);
        }
    if (c.event_capacity) {
        if (hipMalloc(&e->events, (size_t)c.event_capacity * sizeof(brc_event)) != hipSuccess) return fail(BRC_E_NOMEM);
        if (hipMalloc(&e->event_count, 8) != hipSuccess) return fail(BRC_E_NOMEM);
    }
    e->cells_ready = !e->life_cfg;
    e->last_life = e->life_cfg;       // brc_last_kernel before the first run: the kernel a fresh run launches
    if (hipMemsetAsync(e->inj_off, 0, (size_t)e->nitems * 4, e->stream) != hipSuccess) return fail(BRC_E_HIP);
    if (hipMemsetAsync(e->inj_cnt, 0, (size_t)e->nitems * 4, e->stream) != hipSuccess) return fail(BRC_E_HIP);
    if (hipMemsetAsync(e->kdst, 0, keys * 8 * e->bw, e->stream) != hipSuccess) return fail(BRC_E_HIP);   // keys = 1: 8 B
    // the lifetime kernel leaves its bitmap ring zero at exit
    if (e->life_cfg && e->life_pl &&
        hipMemsetAsync(e->dring, 0, (size_t)e->nitems * e->life_rw * e->nkw * 64 * 8, e->stream) != hipSuccess)
        return fail(BRC_E_HIP);
    {
        std::vector<uint64_t> bm((size_t)c.instances * e->bw);
        for (uint64_t i = 0; i < c.instances; ++i)
            for (uint32_t w = 0; w < e->bw; ++w)
                bm[i * e->bw + w] = (w == 0 ? c.byzantine_mask : c.byzantine_mask_hi[w - 1]) & word_mask(c.n, w);
        if (hipMemcpy(e->byz, bm.data(), bm.size() * 8, hipMemcpyHostToDevice) != hipSuccess) return fail(BRC_E_HIP);
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
    const int vmax = e->cfg.mode == BRC_MODE_SPEC ? 3 : (int)e->nval - 1;
    bool wide_ids = false;
    for (size_t i = 0; i < bytes; ++i) {
        if (proposals[i] < 0 || proposals[i] > vmax) {
            e->err = "proposal value ids must be in [0, " + std::to_string(vmax) + "] on this kernel";
            return BRC_E_INVALID;
        }
        wide_ids = wide_ids || proposals[i] > 3;
    }
    e->values_wide = wide_ids;               // the lifetime kernel keeps 2-bit value ids
    if (!e->prop) HIPCHK(e, hipMalloc(&e->prop, bytes));
    HIPCHK(e, hipMemcpyAsync(e->prop, proposals, bytes, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return BRC_OK;
}

int brc_load_byzantine(void* h, const uint64_t* masks) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || !masks) return BRC_E_INVALID;
    const uint32_t words = (e->cfg.n + 63) / 64;
    std::vector<uint64_t> bm((size_t)e->cfg.instances * e->bw, 0);
    for (uint64_t i = 0; i < e->cfg.instances; ++i)
        for (uint32_t w = 0; w < words; ++w) bm[i * e->bw + w] = masks[i * words + w] & word_mask(e->cfg.n, w);
    HIPCHK(e, hipMemcpyAsync(e->byz, bm.data(), bm.size() * 8, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (e->cfg.byz_pattern) { int rc = apply_pattern(e); if (rc) return rc; }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return BRC_OK;
}

int brc_inject(void* h, const brc_injection* list, size_t count) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || (!list && count)) return BRC_E_INVALID;
    if (e->pattern_active) { e->err = "explicit injections cannot be combined with byz_pattern"; return BRC_E_STATE; }
    const brc_config& c = e->cfg;
    if (!e->step_ok && count) {
        e->err = "this engine runs on the key-lifetime kernel only (its step-kernel state does not fit the device, "
                 "or a key window above 32 at n in 33..64 with sender peers): no injections";
        return BRC_E_UNSUPPORTED;
    }
    const uint64_t all = (c.n >= 64) ? ~0ull : ((1ull << c.n) - 1);
    std::vector<ItemState> its;
    std::vector<InstState> ist;
    bool have_state = false;
    std::vector<uint64_t> reopen;
    std::vector<InjDev> staged;
    std::vector<uint64_t> staged_item;
    std::unordered_map<uint64_t, uint32_t> new_count;                                   // this batch's SENDs
    std::unordered_map<uint64_t, std::vector<std::pair<uint32_t, uint64_t>>> new_dst;
    for (size_t i = 0; i < count; ++i) {
        const brc_injection& x = list[i];
        if (x.instance >= c.instances || x.node >= c.n || x.t > c.step_cap) { e->err = "injection out of range"; return BRC_E_INVALID; }
        if (x.value < 0 || x.value >= (int)(c.mode == BRC_MODE_SPEC ? 4u : e->nval) || x.s >= 0xFFFE) {
            e->err = "value id / phase index out of range (value ids 4..7 need n <= 32 or connection peers, not SPEC)";
            return BRC_E_INVALID;
        }
        bool drop = false;                       // a repeated SEND carried on no link (sender peers)
        InjDev r = {};
        r.t = x.t; r.kind = (uint8_t)x.kind; r.type = (uint8_t)x.type; r.node = (uint8_t)x.node;
        r.seg = (uint8_t)(x.instance % e->ipw); r.value = (int8_t)x.value; r.s = (uint16_t)x.s;
        r.dst = x.dst_mask & all;
        bool full = (r.dst == word_mask(c.n, 0));
        for (uint32_t w = 1; w < e->bw; ++w) {
            r.dst_hi[w - 1] = x.dst_mask_hi[w - 1] & word_mask(c.n, w);
            full = full && r.dst_hi[w - 1] == word_mask(c.n, w);
        }
        r.restricted = (x.kind == BRC_INJ_SEND && !full) ? 1 : 0;
        if (x.kind == BRC_INJ_PROPOSE) {
            if (c.protocol != BRC_PROTO_CONSENSUS) { e->err = "PROPOSE needs the consensus protocol"; return BRC_E_INVALID; }
        } else if (x.kind == BRC_INJ_DELIVER) {
            if (c.protocol != BRC_PROTO_CONSENSUS) { e->err = "DELIVER needs the consensus protocol"; return BRC_E_INVALID; }
            if (c.mode == BRC_MODE_SPEC) { e->err = "DELIVER: SPEC consensus counts phase-indexed keys"; return BRC_E_UNSUPPORTED; }
            if (x.kp >= c.n) { e->err = "DELIVER host out of range"; return BRC_E_INVALID; }
            r.slot = (uint16_t)x.kp;               // the message's host
        } else if (x.kind == BRC_INJ_SEND || x.kind == BRC_INJ_MSG || x.kind == BRC_INJ_KEY) {
            if (x.kp >= c.n * c.variants) { e->err = "kp out of range"; return BRC_E_INVALID; }
            r.slot = (uint16_t)(x.kp * c.key_window + (x.s % c.key_window));
            if (x.kind == BRC_INJ_MSG) {
                if (x.type != BRC_ECHO && x.type != BRC_READY) { e->err = "MSG type must be ECHO or READY"; return BRC_E_INVALID; }
                if (!full) { e->err = "ECHO/READY injections must address every peer"; return BRC_E_UNSUPPORTED; }
            } else if (x.kind == BRC_INJ_SEND) {
                // a second SEND of a key (another origin or the same, one payload string SENT again):
                // an extra-SEND record on the non-lean step kernels; the lean and wide kernels model
                // one SEND per key
                const uint64_t k64 = (x.instance << 32) | (uint64_t)(x.kp * 0x10000u + x.s);
                auto it0 = e->send_count.find(k64);
                auto it1 = new_count.find(k64);
                const uint32_t before = (it0 != e->send_count.end() ? it0->second : 0u) +
                                        (it1 != new_count.end() ? it1->second : 0u);
                if ((e->compact || e->wide) && before) {
                    e->err = "a key can be SENT only once on this kernel (n in 33..64 with sender peers, or n > 64)";
                    return BRC_E_UNSUPPORTED;
                }
                ++new_count[k64];
                // this node's earlier SENDs of the key (this batch included): r.type = 1 marks a repeat
                // (brc_step.h: a COPY event with connection peers); sender peers carry a repeated
                // message on a link no further (the links it used are dropped from the record)
                uint64_t prev = 0;
                bool had = false;
                for (const auto* mp : {&e->send_dst, &new_dst}) {
                    auto it = mp->find(k64);
                    if (it != mp->end())
                        for (const auto& q : it->second)
                            if (q.first == x.node) { prev |= q.second; had = true; }
                }
                new_dst[k64].push_back({x.node, r.dst});
                // a key SENT before (by any node): an extra-SEND record (bit 1), bit 0 = this node's repeat
                const bool again = !(e->compact || e->wide) && before > 0;
                r.type = (again ? 2 : 0) | (had ? 1 : 0);
                if (c.peer_mode == BRC_PEER_SENDER) r.dst &= ~prev;
                drop = had && r.dst == 0;
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
        if (ist[x.instance].status == BRC_QUIESCENT && e->life_done) {
            e->err = "instance finished by the key-lifetime kernel (no step state to resume): brc_reset first";
            return BRC_E_STATE;
        }
        if (ist[x.instance].status != BRC_QUIESCENT && ist[x.instance].status != BRC_RUNNING) {
            e->err = "instance already stopped"; return BRC_E_STATE;
        }
        // a repeated SEND carried on no link (sender peers) changes no instance state: accepted, not staged
        // (after the stopped-instance checks: a stopped instance refuses it like every other injection)
        if (drop) continue;
        if (ist[x.instance].status == BRC_QUIESCENT) reopen.push_back(x.instance);
        staged.push_back(r);
        staged_item.push_back(item);
    }
    // extra-SEND records (r.type bit 1) into their items' tables: a record of the same key, step and
    // destinations without this sender takes it, else a new one (records whose arrivals all lie in
    // steps already run leave the table when it is rewritten); all-or-nothing (a batch that
    // overflows a table changes nothing)
    std::unordered_map<uint64_t, std::vector<Engine::XRec>> xnew;
    for (size_t i = 0; i < staged.size(); ++i) {
        const InjDev& r = staged[i];
        if (r.kind != BRC_INJ_SEND || !(r.type & 2)) continue;
        const uint64_t item = staged_item[i];
        if (!xnew.count(item)) {
            // the table is rewritten: records whose arrivals all lie in steps already run are
            // dropped, so the kernel's per-step scan covers live records only (xs_n shrinks)
            std::vector<Engine::XRec> v0;
            if (e->xrec.count(item))
                for (const auto& q : e->xrec[item])
                    if (!(its[item].initialized != 0 && q.t + c.delay_max < its[item].t)) v0.push_back(q);
            xnew[item] = v0;
        }
        auto& v = xnew[item];
        int slot = -1;
        for (size_t j = 0; j < v.size(); ++j) {
            if (v[j].k == r.slot && v[j].t == r.t && v[j].seg == r.seg && v[j].dst == r.dst && !((v[j].smask >> r.node) & 1ull)) {
                slot = (int)j;
                break;
            }
        }
        const Engine::XRec nr = {r.slot, r.t, r.seg, 1ull << r.node, r.dst};
        if (slot >= 0) v[slot].smask |= 1ull << r.node;
        else if (v.size() < XSEND_MAX) v.push_back(nr);
        else {
            e->err = "more than " + std::to_string(XSEND_MAX) + " extra-SEND records in flight in one item";
            return BRC_E_UNSUPPORTED;
        }
    }
    std::vector<uint64_t> xbuf;
    xbuf.reserve(xnew.size() * (3 * XSEND_MAX + 1));
    for (auto& kv : xnew) {
        e->xrec[kv.first] = kv.second;
        const size_t o = xbuf.size();
        xbuf.resize(o + 3 * XSEND_MAX + 1, 0);
        for (size_t j = 0; j < kv.second.size(); ++j) {
            const auto& q = kv.second[j];
            xbuf[o + 3 * j] = (uint64_t)q.k | ((uint64_t)q.t << 16) | ((uint64_t)q.seg << 40);
            xbuf[o + 3 * j + 1] = q.smask;
            xbuf[o + 3 * j + 2] = q.dst;
        }
        xbuf[o + 3 * XSEND_MAX] = kv.second.size();
        HIPCHK(e, hipMemcpyAsync(e->xsend + kv.first * 3 * XSEND_MAX, &xbuf[o], 3 * XSEND_MAX * 8, hipMemcpyHostToDevice,
                                 e->stream));
        HIPCHK(e, hipMemcpyAsync(e->xsn + kv.first, &xbuf[o + 3 * XSEND_MAX], 4, hipMemcpyHostToDevice, e->stream));
    }
    for (size_t i = 0; i < staged.size(); ++i) e->pending[staged_item[i]].push_back(staged[i]);
    for (const auto& kv : new_count) e->send_count[kv.first] += kv.second;
    for (auto& kv : new_dst) {
        auto& v = e->send_dst[kv.first];
        v.insert(v.end(), kv.second.begin(), kv.second.end());
    }
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
    // slot generations are 13-bit (wide kernel 11-bit) tags: past the budget a stale cell could
    // read as current.  brc_reset clears fully once the budget is spent; a run that keeps stepping
    // one simulation without resetting must stop here instead of risking the wrap.
    // The lean (compact-cell) kernels, the wide kernel and the lifetime kernel keep no generation tags:
    // a slot's row is rewritten at allocation, so only the 14-bit phase-index snapshot bounds them.
    const uint64_t gen_hard = GEN_MASK - 2;
    const bool genfree = e->compact || e->wide;    // no cell generation tags (rows rewritten at allocation)
    if (!genfree && e->gen_base + 2 >= gen_hard) {
        e->err = "slot generation budget exhausted: call brc_reset";
        return BRC_E_STATE;
    }
    int rc = upload_injections(e);
    if (rc) return rc;
    bool no_inj = true;
    for (const auto& v : e->pending) if (!v.empty()) { no_inj = false; break; }
    const bool life = e->life_cfg && e->fresh && no_inj && max_steps == 0 && !e->values_wide;
    if (!life && !e->step_ok) {
        e->err = "this engine runs on the key-lifetime kernel only (its step-kernel state does not fit, or a key "
                 "window above 32 at n in 33..64 with sender peers): a fresh run to completion, no injections, "
                 "max_steps = 0, value ids < 4 (brc_reset first)";
        return BRC_E_UNSUPPORTED;
    }
    if (!life) {
        rc = ensure_cells(e);
        if (rc) return rc;
    }
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
    P.nL = delay_values(c.delay_model, c.delay_max);
    P.event_cap = c.event_capacity;
    P.mode = c.mode; P.coin_seed = c.coin_seed;
    // a slot allocated for phase index s has been reallocated at most gen_base + s/Q + 1 times
    // (and phase indices stay below 2^14 - 1: the narrow kernel's consensus snapshot keeps s + 1 in 14 bits)
    P.s_limit = genfree ? 0x3FFEu : (uint32_t)std::min<uint64_t>(0x3FFEull, (gen_hard - 1 - e->gen_base) * c.key_window);
    P.cells = e->cells; P.meta = e->meta; P.mgen = e->mgen; P.kdst = e->kdst;
    P.act = e->act; P.actany = e->actany; P.items = e->items;
    P.inst = e->inst; P.istats = e->istats; P.cons0 = e->cons0; P.cons1 = e->cons1; P.hmask = e->hmask;
    P.inj = e->inj; P.inj_off = e->inj_off; P.inj_cnt = e->inj_cnt; P.byz = e->byz; P.prop = e->prop;
    P.events = e->events; P.event_count = e->event_count; P.gcount = e->gcount; P.dbits = e->dbits;
    P.dring = e->dring; P.lmeta = e->lmeta; P.xsend = e->xsend; P.xsn = e->xsn;
    const uint32_t blocks = e->wide ? (uint32_t)e->nitems : (uint32_t)((e->nitems + WPB - 1) / WPB);
    e->hparams = P;
    HIPCHK(e, hipMemcpyAsync(e->dparams, &e->hparams, sizeof(Params), hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemsetAsync(e->gcount + 6, 0, 8, e->stream));   // instances still running after this launch
    HIPCHK(e, hipEventRecord(e->ev0, e->stream));   // times the step kernel alone
    const int kmode = c.peer_mode == BRC_PEER_CONNECTION ? KMODE_CONN : e->general ? KMODE_XREF : (int)c.mode;
    e->fresh = false;
    e->last_life = life;
    if (life) {
        rc = launch_life(kmode, e->life_pl, e->life_rw == LIFE_RW16, c.key_window >= 64,
                         life_hbm_meta(c.key_window, e->life_pl), (uint32_t)e->nitems,
                         e->life_lds, e->stream, e->dparams);
        e->life_done = true;
    } else {
        rc = e->regmask ? launch_step_64r(e->dm, c.event_capacity != 0, kmode, blocks, e->lds_bytes, e->stream, e->dparams)
                        : launch_step(e->npad, e->dm, c.event_capacity != 0, kmode, e->wide_wv4, blocks, e->lds_bytes,
                                      e->stream, e->dparams);
    }
    if (rc == BRC_E_INVALID) { e->err = "no kernel instantiation"; return rc; }
    if (rc) { e->err = std::string("step kernel launch: ") + hipGetErrorString(hipGetLastError()); return rc; }
    HIPCHK(e, hipEventRecord(e->ev1, e->stream));
    HIPCHK(e, hipEventSynchronize(e->ev1));
    HIPCHK(e, hipEventElapsedTime(&e->last_ms, e->ev0, e->ev1));
    unsigned long long gc[8];
    HIPCHK(e, hipMemcpy(gc, e->gcount, sizeof(gc), hipMemcpyDeviceToHost));
    if (!genfree) e->gen_cur = std::max<uint64_t>(e->gen_cur, gc[5] / c.key_window + 2);   // gc[5]: max phase index
    if (running_left) *running_left = (uint32_t)gc[6];   // counted by the step kernel
    return BRC_OK;
}

int brc_reset(void* h) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return BRC_E_INVALID;
    HIPCHK(e, hipSetDevice(e->cfg.device));
    const bool full = e->gen_base + e->gen_cur >= GEN_FULL_CLEAR;
    if (!full) { e->gen_base += e->gen_cur; e->gen_cur = 0; }
    int rc = clear_state(e, full);   // full: gen_base = gen_cur = 0
    if (rc) return rc;
    for (auto& v : e->pending) v.clear();
    e->send_count.clear();
    e->send_dst.clear();
    e->xrec.clear();
    if (e->pattern_active) {
        e->pattern_active = false;
        rc = apply_pattern(e);
        if (rc) return rc;
    } else {
        HIPCHK(e, hipMemsetAsync(e->inj_off, 0, (size_t)e->nitems * 4, e->stream));
        HIPCHK(e, hipMemsetAsync(e->inj_cnt, 0, (size_t)e->nitems * 4, e->stream));
    }
    e->inj_dirty = false;
    e->fresh = true;
    e->life_done = false;
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
    std::vector<uint64_t> c1((i1 - i0 + 1) * e->lpi);
    std::vector<uint64_t> bm(count * e->bw);
    HIPCHK(e, hipMemcpyAsync(bm.data(), e->byz + first * e->bw, bm.size() * 8, hipMemcpyDeviceToHost, e->stream));
    if (c.protocol == BRC_PROTO_CONSENSUS)
        HIPCHK(e, hipMemcpyAsync(c1.data(), e->cons1 + i0 * e->lpi, c1.size() * 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    for (uint64_t i = 0; i < count; ++i) {
        const uint64_t in = first + i, item = in / e->ipw, seg = in % e->ipw;
        brc_instance_result& r = out[i];
        r.status = ist[i].status; r.t_stop = ist[i].t_stop; r.t_now = its[item - i0].t;
        r.msgs_sent = st[i * 4 + 0]; r.arrivals = st[i * 4 + 1]; r.cell_steps = st[i * 4 + 2]; r.deliveries = st[i * 4 + 3];
        uint32_t dec = c.protocol == BRC_PROTO_CONSENSUS ? 1u : 0u;
        if (dec)
            for (uint32_t dd = 0; dd < c.n; ++dd) {
                if ((bm[i * e->bw + dd / 64] >> (dd % 64)) & 1ull) continue;
                if ((c1[(item - i0) * e->lpi + seg * e->npad + dd] & 0xFFFF) == 0) { dec = 0; break; }
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
    const size_t nl = (i1 - i0 + 1) * e->lpi;
    std::vector<uint64_t> c0(nl), c1(nl);
    HIPCHK(e, hipMemcpyAsync(c0.data(), e->cons0 + i0 * e->lpi, nl * 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipMemcpyAsync(c1.data(), e->cons1 + i0 * e->lpi, nl * 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    for (uint64_t i = 0; i < count; ++i) {
        const uint64_t in = first + i, item = in / e->ipw, seg = in % e->ipw;
        for (uint32_t dd = 0; dd < e->cfg.n; ++dd) {
            const size_t l = (item - i0) * e->lpi + seg * e->npad + dd;
            brc_replica_result& r = out[i * e->cfg.n + dd];
            const uint64_t a = c0[l], b = c1[l];
            r.round = a & 0xFFFF; r.phase = (a >> 16) & 0xF; r.value_count = (a >> 48) & 0xFFFF;   // cons0_pack
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
        std::vector<uint64_t> c1((size_t)e->nitems * e->lpi);
        std::vector<uint64_t> bm(N * e->bw);
        HIPCHK(e, hipMemcpy(c1.data(), e->cons1, c1.size() * 8, hipMemcpyDeviceToHost));
        HIPCHK(e, hipMemcpy(bm.data(), e->byz, bm.size() * 8, hipMemcpyDeviceToHost));
        for (uint64_t in = 0; in < N; ++in) {
            const uint64_t item = in / e->ipw, seg = in % e->ipw;
            for (uint32_t dd = 0; dd < e->cfg.n; ++dd)
                if (!((bm[in * e->bw + dd / 64] >> (dd % 64)) & 1ull))
                    out->decide_rounds_sum += (c1[item * e->lpi + seg * e->npad + dd] >> 16) & 0xFFFF;
        }
    }
    if (e->event_count) {
        unsigned long long n = 0;
        HIPCHK(e, hipMemcpy(&n, e->event_count, 8, hipMemcpyDeviceToHost));
        out->events_dropped = n > e->cfg.event_capacity ? n - e->cfg.event_capacity : 0;
    }
    return BRC_OK;
}

int brc_read_round_histogram(void* h, uint64_t* hist, uint32_t bins) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || !hist || bins < 2 || bins > 4096) return BRC_E_INVALID;
    if (e->cfg.protocol != BRC_PROTO_CONSENSUS) { e->err = "round histogram needs the consensus protocol"; return BRC_E_STATE; }
    HIPCHK(e, hipSetDevice(e->cfg.device));
    unsigned long long* dh = nullptr;
    HIPCHK(e, hipMalloc(&dh, (size_t)bins * 8));
    if (hipMemsetAsync(dh, 0, (size_t)bins * 8, e->stream) != hipSuccess) { (void)hipFree(dh); return BRC_E_HIP; }
    const uint32_t tpb = 256;
    const uint32_t blocks = (uint32_t)((e->cfg.instances + tpb - 1) / tpb);
    hipLaunchKernelGGL(round_histogram, dim3(blocks), dim3(tpb), (size_t)bins * 8, e->stream, e->cons1, e->byz,
                       e->cfg.instances, (uint32_t)e->ipw, e->lpi, (uint32_t)e->npad, e->bw, e->cfg.n, bins, dh);
    hipError_t r = hipGetLastError();
    if (r == hipSuccess) r = hipMemcpyAsync(hist, dh, (size_t)bins * 8, hipMemcpyDeviceToHost, e->stream);
    if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
    (void)hipFree(dh);
    if (r != hipSuccess) { e->err = std::string("round histogram: ") + hipGetErrorString(r); return BRC_E_HIP; }
    return BRC_OK;
}

int brc_read_value_decisions(void* h, uint64_t* value_hist, uint64_t* disagreements) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || !value_hist || !disagreements) return BRC_E_INVALID;
    if (e->cfg.protocol != BRC_PROTO_CONSENSUS) { e->err = "decisions need the consensus protocol"; return BRC_E_STATE; }
    HIPCHK(e, hipSetDevice(e->cfg.device));
    unsigned long long* d = nullptr;
    HIPCHK(e, hipMalloc(&d, 10 * 8));
    hipError_t r = hipMemsetAsync(d, 0, 10 * 8, e->stream);
    if (r == hipSuccess) {
        const uint32_t tpb = 256;
        const uint32_t blocks = (uint32_t)((e->cfg.instances + tpb - 1) / tpb);
        hipLaunchKernelGGL(decision_histogram, dim3(blocks), dim3(tpb), 0, e->stream, e->cons1, e->byz,
                           e->cfg.instances, (uint32_t)e->ipw, e->lpi, (uint32_t)e->npad, e->bw, e->cfg.n, d);
        r = hipGetLastError();
    }
    unsigned long long hout[10] = {0};
    if (r == hipSuccess) r = hipMemcpyAsync(hout, d, sizeof(hout), hipMemcpyDeviceToHost, e->stream);
    if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
    (void)hipFree(d);
    if (r != hipSuccess) { e->err = std::string("decision histogram: ") + hipGetErrorString(r); return BRC_E_HIP; }
    for (int b = 0; b < 9; ++b) value_hist[b] = hout[b];
    *disagreements = hout[9];
    return BRC_OK;
}

int brc_read_decisions(void* h, uint64_t* value_hist, uint64_t* disagreements) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || !value_hist || !disagreements) return BRC_E_INVALID;
    uint64_t v9[9];
    const int rc = brc_read_value_decisions(h, v9, disagreements);
    if (rc) return rc;
    for (int b = 4; b < 8; ++b)
        if (v9[b]) { e->err = "value ids >= 4 were decided: use brc_read_value_decisions"; return BRC_E_STATE; }
    for (int b = 0; b < 4; ++b) value_hist[b] = v9[b];
    value_hist[4] = v9[8];
    return BRC_OK;
}

int brc_reset_at(void* h, uint64_t instance_offset) {
    Engine* e = static_cast<Engine*>(h);
    if (!e) return BRC_E_INVALID;
    e->cfg.instance_offset = instance_offset;
    return brc_reset(h);
}

int brc_read_events_range(void* h, size_t first, brc_event* out, size_t cap, size_t* total) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || !total) return BRC_E_INVALID;
    if (!e->event_count) { *total = 0; return BRC_OK; }
    unsigned long long n = 0;
    HIPCHK(e, hipMemcpy(&n, e->event_count, 8, hipMemcpyDeviceToHost));
    *total = (size_t)n;
    const size_t avail = std::min<size_t>((size_t)n, e->cfg.event_capacity);
    if (out && cap && first < avail)
        HIPCHK(e, hipMemcpy(out, e->events + first, std::min(avail - first, cap) * sizeof(brc_event),
                            hipMemcpyDeviceToHost));
    return BRC_OK;
}

int brc_last_kernel(void* h, uint32_t* kind) {
    Engine* e = static_cast<Engine*>(h);
    if (!e || !kind) return BRC_E_INVALID;
    *kind = e->last_life ? BRC_KERNEL_LIFE : BRC_KERNEL_STEP;
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
