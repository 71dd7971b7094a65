/*
 * brc.h -- C-ABI of the MI355X batched consensus engine (libbrc_hip.so).
 *
 * Drop-in boundary for the reference's hot path.  The reference exposes it as Python
 * classes; this ABI is what those classes (re-implemented in
 * byzantinerandomizedconsensus_amd/) bind through ctypes:
 *
 *   reference                                                   replaced by
 *   ---------------------------------------------------------   ----------------------------
 *   BRBroadcast.__init__ / ByzantineRandomizedConsensus.__init__ brc_create
 *     (core/brbroadcast.py:17-44, core/byzantinerandomizedconsensus.py:18-36)
 *   BRBroadcast.broadcast_listener (core/brbroadcast.py:121-128) brc_run (the accept loop,
 *     + the listener loop body (core/brbroadcast.py:60-119)       batched over instances)
 *   Broadcast.broadcast(SEND, m)     (base/broadcast.py:17-40)   brc_inject(BRC_INJ_SEND)
 *   ByzantineRandomizedConsensus.start/propose (:38-51)          brc_inject(BRC_INJ_PROPOSE) /
 *                                                                brc_load_proposals
 *   IBroadcastHandler.deliver upcall (base/broadcast.py:52-55)   brc_read_events (DELIVER)
 *   IConsensusHandler.decide upcall  (base/consensus.py:22-24)   brc_read_events (DECIDE),
 *                                                                brc_read_replicas
 *   (Byzantine peers: raw sends into the transport)              brc_inject(BRC_INJ_KEY/SEND/MSG),
 *                                                                brc_load_byzantine
 *
 * Conventions: every call returns 0 on success or a negative BRC_E_* code; host buffers
 * are caller-owned; device buffers are engine-owned; one host thread per engine; all work
 * is ordered on the engine's own HIP stream; no callbacks cross the ABI.
 */
#ifndef BRC_H
#define BRC_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BRC_ABI_VERSION 7

enum {
    BRC_OK = 0,
    BRC_E_INVALID = -1,      /* bad argument / unsupported configuration */
    BRC_E_NOMEM = -2,        /* device or host allocation failed */
    BRC_E_HIP = -3,          /* HIP runtime error (see brc_last_error) */
    BRC_E_UNSUPPORTED = -4,  /* a workload feature the engine does not model */
    BRC_E_STATE = -5         /* call not valid in the current engine state */
};

enum { BRC_PROTO_BRB = 0, BRC_PROTO_CONSENSUS = 1 };
/* BRC_MODE_REFERENCE: the protocol exactly as the reference runs it, quirks included (SURVEY §4
 * K1-K12).  BRC_MODE_SPEC: the protocol the reference intends (Bracha-correct broadcast; consensus
 * with per-phase windows and the core/byzantinerandomizedconsensus.py:88-92 coin made reachable as
 * a common Philox coin keyed (coin_seed, instance, round)). */
/* BRC_MODE_BEB: best-effort broadcast (core/bebroadcast.py as intended -- the reference's class
 * cannot be constructed): a SEND delivers at its arrival, no ECHO/READY; with BRC_PROTO_CONSENSUS
 * the reference's consensus runs on top of it (its consensus_instance.deliver, :42). */
enum { BRC_MODE_REFERENCE = 0, BRC_MODE_SPEC = 1, BRC_MODE_BEB = 2 };
/* Peer identity of core/brbroadcast.py:69-71.  SENDER (:71): sets hold sender ids and the
 * network drops a message identical to one already sent on the link.  CONNECTION (:69, the
 * reference's local-test mode): every message is its own connection -- a new peer -- so sets
 * count messages, nothing is dropped, and the :119 amplification re-fires on every qualifying READY.
 * CONNECTION needs BRC_MODE_REFERENCE (any n <= 256, delay_max <= 16); it keeps per-cell send
 * counts of one byte, so an injection of a 256th copy of one type by one replica in one step stops
 * the instance with BRC_BADINJ. */
enum { BRC_PEER_SENDER = 0, BRC_PEER_CONNECTION = 1 };
enum { BRC_DELAY_CONST = 0, BRC_DELAY_UNIFORM = 1, BRC_DELAY_SLOWSET = 2, BRC_DELAY_GEOMETRIC = 3 };
enum { BRC_PROPOSALS_NONE = 0, BRC_PROPOSALS_PHILOX = 1, BRC_PROPOSALS_LOADED = 2 };
enum { BRC_BYZ_NONE = 0, BRC_BYZ_EQUIVOCATE = 1 };
enum { BRC_SEND = 1, BRC_ECHO = 2, BRC_READY = 3 };
/* BRC_INJ_DELIVER: ByzantineRandomizedConsensus.deliver(message) called directly on replica `node`
 * (core/byzantinerandomizedconsensus.py:53) with a message of host `kp` (a replica id) carrying
 * value id `value` -- no BRB traffic; the consensus logic runs as on a BRB delivery.  Consensus
 * protocol, BRC_MODE_REFERENCE or BRC_MODE_BEB (BRC_MODE_SPEC counts phases: BRC_E_UNSUPPORTED). */
enum { BRC_INJ_PROPOSE = 1, BRC_INJ_SEND = 2, BRC_INJ_KEY = 3, BRC_INJ_MSG = 4, BRC_INJ_DELIVER = 5 };
enum { BRC_RUNNING = 0, BRC_DONE = 1, BRC_QUIESCENT = 2, BRC_STEPCAP = 3, BRC_OVERFLOW = 4, BRC_BADINJ = 5 };
/* BRC_EV_SEND: the first broadcast of (node, type, key) -- the reference harness's send log.
 * BRC_EV_COPY (connection-identity peers only): every later broadcast of it, one event each (the
 * :119 READY re-fires, repeated injected messages); with the SEND events they are the complete wire
 * traffic (wire.Codec.export).  Sender-identity peers suppress such duplicates on the network. */
enum { BRC_EV_DELIVER = 1, BRC_EV_DECIDE = 2, BRC_EV_SEND = 3, BRC_EV_COPY = 4 };

typedef struct {
    uint32_t n;               /* replicas per instance, self included (1..256) */
    uint32_t f;               /* fault bound: thresholds (n+f)/2, f+1, 2f+1, n-f+1 */
    uint32_t protocol;        /* BRC_PROTO_* */
    uint32_t peer_mode;       /* BRC_PEER_SENDER / BRC_PEER_CONNECTION (core/brbroadcast.py:69-71) */
    uint64_t instances;       /* instances owned by this engine */
    uint64_t instance_offset; /* global id of instance 0 (Philox counter; multi-GPU shard) */
    uint64_t seed;            /* schedule seed (delays, proposals, slow set) */
    uint32_t delay_model;     /* BRC_DELAY_* */
    uint32_t delay_max;       /* D, 1..16 */
    uint32_t delay_const;     /* BRC_DELAY_CONST value */
    uint32_t round_cap;       /* consensus: instance DONE when every honest replica decided this many times */
    uint32_t step_cap;        /* last simulated step (<= 60000) */
    uint32_t key_window;      /* Q: live phase indices per origin (2, 4, 8; 16 .. 128 with n <= 64 and the
                                 reference / best-effort protocols, whose phase leakage keeps up to ~17
                                 phases of one origin in flight by round 8 and 127 by round 64 under
                                 slow-set D = 8; above 32 at n in 33..64 with sender peers: the
                                 key-lifetime kernel only) */
    uint32_t variants;        /* NV: key variants per origin (1, 2 or 4; Q*NV <= 8, <= 128 where Q may be) */
    uint32_t proposals;       /* BRC_PROPOSALS_* (consensus) */
    uint32_t byz_pattern;     /* BRC_BYZ_* applied to every instance */
    uint32_t event_capacity;  /* 0: no event log */
    uint64_t byzantine_mask;  /* replicas 0..63 that run no code (all instances; see brc_load_byzantine) */
    int32_t device;           /* HIP device ordinal */
    uint32_t mode;            /* BRC_MODE_* */
    uint64_t coin_seed;       /* BRC_MODE_SPEC: common-coin key */
    uint64_t byzantine_mask_hi[3];  /* replicas 64..255 that run no code */
    uint32_t flags;           /* BRC_FLAG_* */
    uint32_t reserved[3];
} brc_config;
/* BRC_FLAG_GENERAL_KEYS (v7): at n in 33..64 with sender peers and the reference protocol, run the
 * narrow kernel's general form instead of the lean one -- 8-B cells with generation tags, 3-bit value
 * ids (7 proposal strings besides "-1") and extra SENDs of one key (one payload SENT by several
 * origins, core/brbroadcast.py:74-79 keys by the payload string) -- what n <= 32 and connection peers
 * always have.  For the class API's single-instance clusters; the batched workloads keep the lean
 * kernels (4-B cells, 2-bit ids). */
enum { BRC_FLAG_GENERAL_KEYS = 1 };

typedef struct {
    uint32_t t;               /* action time: performed after step t, messages stamped t */
    uint16_t kind;            /* BRC_INJ_* */
    uint16_t type;            /* BRC_INJ_MSG: BRC_ECHO / BRC_READY */
    uint64_t instance;        /* engine-local instance index */
    uint32_t node;            /* proposer / sender */
    uint32_t kp;              /* key slot: origin * variants + variant */
    uint32_t s;               /* phase index 2*(round-1)+(phase-1), or BRB sequence */
    int32_t value;            /* value id (0 == "-1"): 0..7 on the narrow kernels that keep 3-bit ids
                                 (n <= 32, or connection peers at n <= 64; not BRC_MODE_SPEC), 0..3 on
                                 the others (n in 33..64 with sender peers, n > 64, SPEC); larger:
                                 BRC_E_INVALID.  The same range holds for brc_load_proposals */
    uint64_t dst_mask;        /* BRC_INJ_SEND destinations 0..63; BRC_INJ_MSG must address all
                                 peers (a restricted ECHO / READY: BRC_E_UNSUPPORTED).  A second
                                 SEND of a key (another node, or the same again: one payload string
                                 SENT twice, one key in the reference) is an extra SEND on the
                                 narrow kernels that keep 3-bit value ids (up to 16 extra-SEND
                                 records in flight per wave item; it must not precede the key's
                                 first SEND); BRC_E_UNSUPPORTED on the others */
    uint64_t dst_mask_hi[3];  /* destinations 64..255 (n > 64), as byzantine_mask_hi */
} brc_injection;

typedef struct {
    uint32_t status;          /* BRC_RUNNING ... */
    uint32_t t_stop;          /* last step with an arrival at an honest replica or an action */
    uint32_t t_now;           /* engine time of the instance's wave */
    uint32_t decided;         /* every honest replica decided at least once */
    uint64_t msgs_sent;       /* link messages sent (duplicate-suppressed) */
    uint64_t arrivals;        /* messages processed by honest replicas (replica-message-steps) */
    uint64_t cell_steps;      /* (receiver, key) cells that had arrivals, summed over steps */
    uint64_t deliveries;
} brc_instance_result;

typedef struct {
    uint32_t round, phase, value_count, decide_count;
    uint32_t first_decide_round, first_decide_t;
    int32_t first_decide_value, last_decide_value;
} brc_replica_result;

typedef struct {
    uint64_t instance;
    uint32_t t;
    uint8_t kind, node, type;
    uint8_t value;            /* value id of the key's payload (DECIDE: the decided value) */
    uint32_t a, b;            /* DELIVER: kp, s   DECIDE: round, value   SEND: kp, s */
} brc_event;

typedef struct {
    uint64_t instances, running, done, quiescent, stepcap, overflow, decided;
    uint64_t msgs_sent, arrivals, cell_steps, deliveries;
    uint64_t decide_rounds_sum;   /* sum of first-decide rounds over honest replicas */
    uint64_t max_t;
    uint64_t events_dropped;
    uint64_t lane_loads;          /* cell words read (one per real lane per processed key-step) */
} brc_stats;

int brc_create(const brc_config* cfg, void** engine);
int brc_load_proposals(void* engine, const int8_t* proposals /* [instances][n] value ids */);
int brc_load_byzantine(void* engine, const uint64_t* byz_masks /* [instances][(n + 63) / 64] */);
int brc_inject(void* engine, const brc_injection* list, size_t count);
int brc_run(void* engine, uint32_t max_steps, uint32_t* running_left);
int brc_reset(void* engine);
int brc_read_instances(void* engine, uint64_t first, uint64_t count, brc_instance_result* out);
int brc_read_replicas(void* engine, uint64_t first, uint64_t count, brc_replica_result* out /* [count][n] */);
int brc_read_events(void* engine, brc_event* out, size_t cap, size_t* count);
int brc_read_stats(void* engine, brc_stats* out);
/* Decide-round histogram over instances (consensus): hist[r] = instances whose honest replicas
 * had ALL decided by round r (the max of their first-decide rounds), hist[0] = instances with an
 * undecided honest replica, rounds >= bins-1 in hist[bins-1].  bins in [2, 4096].  Per engine
 * (= per GPU shard); SURVEY §8(d) cfg5 all-reduces it over ranks (shard.reduce_stats). */
int brc_read_round_histogram(void* engine, uint64_t* hist, uint32_t bins);
/* Decisions of the honest replicas (consensus; the decide() upcall of
 * core/byzantinerandomizedconsensus.py:94): value_hist[v] for v = 0..3 counts replicas whose FIRST
 * decision carried value id v (0 is the reference's "-1"), value_hist[4] replicas that never
 * decided; *disagreements counts instances whose honest replicas' first decisions differ
 * (the agreement check of SURVEY §8(e)).  Per engine; shard.reduce_stats all-reduces them. */
int brc_read_decisions(void* engine, uint64_t* value_hist /* [5] */, uint64_t* disagreements);
/* The same over 3-bit value ids: value_hist[v] for v = 0..7, value_hist[8] never decided.
 * brc_read_decisions is BRC_E_STATE once a value id >= 4 was decided. */
int brc_read_value_decisions(void* engine, uint64_t* value_hist /* [9] */, uint64_t* disagreements);
/* brc_reset, then re-key the engine to the global instances [instance_offset, +instances): one
 * engine sweeps a range larger than its device footprint in tiles, with the results one engine
 * over the whole range would give (every Philox counter uses the global id).  Loaded proposals
 * and Byzantine masks are kept (they are indexed by engine-local instance). */
int brc_reset_at(void* engine, uint64_t instance_offset);
/* Events first .. first+cap-1 of the log (brc_read_events reads from 0); *total = events logged
 * since the last reset, dropped ones included.  Lets a caller drain the log incrementally. */
int brc_read_events_range(void* engine, size_t first, brc_event* out, size_t cap, size_t* total);
int brc_last_kernel_ms(void* engine, float* ms);
/* Which kernel the last brc_run launched.  BRC_KERNEL_LIFE (the key-lifetime kernel) runs a fresh
 * engine (after brc_create / brc_reset) to completion in one launch when the configuration allows:
 * n in 33..64, consensus with Philox or loaded proposals, constant / slow-set delays with
 * delay_max <= 8 (its two-class form) or uniform / geometric delays with delay_max <= 16 (its
 * per-link form, which keeps a delivery-bitmap ring in HBM: 64 KB per instance at NK = 256, 128 KB
 * for delays above 8), no event log, no byz_pattern, no injections, max_steps == 0.  By default it
 * runs every such configuration except sender peers under uniform / geometric delays (the step kernel
 * is faster there); a run it cannot take (injections, max_steps > 0) goes to the step kernel.  Sender
 * peers whose step-kernel state (cells, slot arrays, activity ring) would exceed 90 % of the device's
 * TOTAL memory -- a choice fixed by the configuration and device model, not by what else holds memory
 * -- or whose key window is above 32 are lifetime-kernel-only: brc_inject returns BRC_E_UNSUPPORTED
 * and so does a run with max_steps > 0.  Before the first brc_run, brc_last_kernel reports the kernel a fresh run to
 * completion would launch.  The environment variable
 * BRC_KERNEL (read by brc_create) = life uses it for every eligible engine, = step never.  Its
 * results equal the step kernel's; its instances end final, so a later injection that would
 * re-open a QUIESCENT instance is BRC_E_STATE until brc_reset. */
enum { BRC_KERNEL_STEP = 0, BRC_KERNEL_LIFE = 1 };
int brc_last_kernel(void* engine, uint32_t* kind);
int brc_device_count(int* count);
const char* brc_last_error(void* engine);   /* engine NULL: why the last brc_create on this thread failed */
void brc_destroy(void* engine);
int brc_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
