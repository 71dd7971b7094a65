/*
 * brc_oracle.c -- CPU oracle (TEST INFRASTRUCTURE ONLY; see brc_oracle.h).
 *
 * Event-by-event restatement of the reference under the lock-step schedule:
 *   - brb_on_message()      <- core/brbroadcast.py:60-119   (one accept-loop iteration)
 *   - net_broadcast()       <- base/broadcast.py:17-40      (fan-out to every peer, self included)
 *   - cons_deliver()        <- core/byzantinerandomizedconsensus.py:53-106
 *   - cons_propose()        <- core/byzantinerandomizedconsensus.py:43-51
 * Dicts keyed by payload strings become a (kp, s) key table; sets of peer addresses become
 * bitsets of sender ids (sender-identity peer mode, core/brbroadcast.py:69-71).
 * SPEC modes (see brc_oracle.h):
 *   - brb_on_message_spec() <- Bracha's broadcast as core/brbroadcast.py:60-119 intends it
 *   - spec_deliver()        <- core/byzantinerandomizedconsensus.py:53-106 with per-(round, phase)
 *                              windows and the :88-92 fallback reachable (common coin)
 */
#include "brc_oracle.h"
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ Philox / schedule */
#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

void oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)PHILOX_M0 * c0, p1 = (uint64_t)PHILOX_M1 * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0; c1 = lo1; c2 = hi0 ^ c3 ^ k1; c3 = lo0;
        k0 += PHILOX_W0; k1 += PHILOX_W1;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static void draw(uint64_t seed, uint64_t g, uint32_t a, uint32_t purpose, uint32_t b, uint32_t out[4]) {
    uint32_t ctr[4] = {(uint32_t)g, (uint32_t)(g >> 32), a, (purpose << 24) | (b & 0xFFFFFFu)};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    oracle_philox(ctr, key, out);
}

uint32_t oracle_delay(uint32_t n, uint32_t f, uint64_t seed, uint32_t model, uint32_t dmax,
                      uint32_t dconst, uint64_t g, uint32_t src, uint32_t dst) {
    uint32_t w[4];
    if (model == 0) return dconst;
    if (model == 2) {
        draw(seed, g, 0, 3, 0, w);
        uint32_t off = w[0] % n;
        int ss = ((src + n - off) % n) < f, ds = ((dst + n - off) % n) < f;
        return (ss || ds) ? dmax : 1;
    }
    draw(seed, g, dst, 1, src >> 2, w);
    uint32_t x = w[src & 3];
    if (model == 1) return 1 + (uint32_t)(((uint64_t)x * dmax) >> 32);
    uint32_t ones = 0;
    while (ones < 32 && ((x >> ones) & 1u)) ++ones;
    return (1 + ones < dmax) ? 1 + ones : dmax;
}

uint32_t oracle_proposal_id(uint64_t seed, uint64_t g, uint32_t i) {
    uint32_t w[4];
    draw(seed, g, i, 2, 0, w);
    return 1 + (w[0] & 1u);
}

/* common coin of (instance, round): value id 1 ("0") or 2 ("1") */
uint32_t oracle_coin_id(uint64_t coin_seed, uint64_t g, uint32_t round) {
    uint32_t w[4];
    draw(coin_seed, g, round, 4, 0, w);
    return 1 + (w[0] & 1u);
}

/* ------------------------------------------------------------------ bitsets */
typedef struct { uint64_t w[4]; } bits_t;
static inline void bset(bits_t* b, uint32_t i) { b->w[i >> 6] |= 1ull << (i & 63); }
static inline int btest(const bits_t* b, uint32_t i) { return (int)((b->w[i >> 6] >> (i & 63)) & 1ull); }
static inline uint32_t bcount(const bits_t* b) {
    return (uint32_t)(__builtin_popcountll(b->w[0]) + __builtin_popcountll(b->w[1]) +
                      __builtin_popcountll(b->w[2]) + __builtin_popcountll(b->w[3]));
}

/* ------------------------------------------------------------------ state */
typedef struct {
    uint8_t eex, rex, del;   /* echo_sent_list / ready_sent_list entry exists, delivered */
    uint8_t es, rs;          /* SPEC: ECHO sent, READY sent */
    bits_t e, r;             /* the two sets (core/brbroadcast.py:38-41), sender-identity peers */
    uint32_t ne, nr;         /* their sizes under connection-identity peers (one peer per message) */
} cell_t;

typedef struct {
    uint32_t kp, s;
    int32_t value;
    cell_t* cells;           /* [n] per receiver */
    bits_t* sent;            /* [3][n] destinations already sent to, per (type, src) */
} key_t_;

typedef struct {
    uint32_t dst, kp, s, type, src, key;
} msg_t;

typedef struct {
    msg_t* v; size_t n, cap;
} bucket_t;

#define NVAL 8
#define SPEC_RING 64
typedef struct {
    uint32_t round, phase, value_count, decides;
    uint32_t nvals;
    int32_t order[NVAL];     /* insertion order of message_values (dict order) */
    bits_t hosts[NVAL];
    /* SPEC: deliveries buffered per phase index s (ring slot s % window) */
    bits_t seen[SPEC_RING];
    uint32_t cnt[SPEC_RING][2];
} cons_t;

typedef struct {
    const oracle_spec* sp;
    oracle_result* res;
    uint32_t n, f, t, D;
    key_t_* keys; size_t nkeys, kcap;
    uint32_t* hkeys; size_t hcap;   /* open-addressing map (kp,s) -> key index+1 */
    bucket_t buckets[17];
    cons_t cons[OR_MAXN];
    uint8_t delay[OR_MAXN][OR_MAXN];
    int err, overflow;
} sim_t;

static uint64_t kh(uint32_t kp, uint32_t s) {
    uint64_t x = ((uint64_t)kp << 32) | s;
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

static int key_find(sim_t* S, uint32_t kp, uint32_t s) {
    if (!S->hcap) return -1;
    size_t m = S->hcap - 1, i = (size_t)kh(kp, s) & m;
    while (S->hkeys[i]) {
        key_t_* k = &S->keys[S->hkeys[i] - 1];
        if (k->kp == kp && k->s == s) return (int)(S->hkeys[i] - 1);
        i = (i + 1) & m;
    }
    return -1;
}

static void hash_insert(sim_t* S, uint32_t idx) {
    size_t m = S->hcap - 1, i = (size_t)kh(S->keys[idx].kp, S->keys[idx].s) & m;
    while (S->hkeys[i]) i = (i + 1) & m;
    S->hkeys[i] = idx + 1;
}

static int key_get(sim_t* S, uint32_t kp, uint32_t s, int32_t value) {
    int id = key_find(S, kp, s);
    if (id >= 0) {
        if (S->keys[id].value != value) S->err = -5;   /* one payload per (kp, s) */
        return id;
    }
    if (S->nkeys == S->kcap) {
        size_t nc = S->kcap ? S->kcap * 2 : 64;
        key_t_* nk = (key_t_*)realloc(S->keys, nc * sizeof(key_t_));
        if (!nk) { S->err = -2; return -1; }
        S->keys = nk; S->kcap = nc;
    }
    if ((S->nkeys + 1) * 2 > S->hcap) {
        size_t nh = S->hcap ? S->hcap * 2 : 256;
        while ((S->nkeys + 1) * 2 > nh) nh *= 2;
        free(S->hkeys);
        S->hkeys = (uint32_t*)calloc(nh, sizeof(uint32_t));
        if (!S->hkeys) { S->err = -2; return -1; }
        S->hcap = nh;
        for (size_t i = 0; i < S->nkeys; ++i) hash_insert(S, (uint32_t)i);
    }
    key_t_* k = &S->keys[S->nkeys];
    k->kp = kp; k->s = s; k->value = value;
    k->cells = (cell_t*)calloc(S->n, sizeof(cell_t));
    k->sent = (bits_t*)calloc(3 * (size_t)S->n, sizeof(bits_t));
    if (!k->cells || !k->sent) { S->err = -2; return -1; }
    hash_insert(S, (uint32_t)S->nkeys);
    return (int)(S->nkeys++);
}

static void push_event(uint32_t* buf, size_t cap, size_t* cnt, int words, const uint32_t* w) {
    if (*cnt < cap) memcpy(buf + (*cnt) * words, w, words * sizeof(uint32_t));
    (*cnt)++;
}

static int is_honest(const sim_t* S, uint32_t i) {
    return !((S->sp->byz[i >> 6] >> (i & 63)) & 1ull);
}

/* One link message.  Sender-identity peers: a duplicate-suppressing network (oracle/schedule.py
 * docstring).  Connection-identity peers: every message travels (each is its own connection). */
static void net_send(sim_t* S, uint32_t src, uint32_t dst, uint32_t type, int key) {
    key_t_* k = &S->keys[key];
    bits_t* sent = &k->sent[(type - 1) * S->n + src];
    if (S->sp->peer_mode != OR_PEER_CONNECTION && btest(sent, dst)) return;
    int first = !(sent->w[0] | sent->w[1] | sent->w[2] | sent->w[3]);
    bset(sent, dst);
    S->res->msgs_sent++;
    if (first) {
        uint32_t ev[5] = {S->t, src, type, k->kp, k->s};
        push_event(S->res->sends, S->res->send_cap, &S->res->n_send, 5, ev);
    }
    if (!is_honest(S, dst)) return;   /* counted as sent; Byzantine nodes run no code */
    uint32_t ta = S->t + S->delay[src][dst];
    bucket_t* b = &S->buckets[ta % (S->D + 1)];
    if (b->n == b->cap) {
        size_t nc = b->cap ? b->cap * 2 : 1024;
        msg_t* nv = (msg_t*)realloc(b->v, nc * sizeof(msg_t));
        if (!nv) { S->err = -2; return; }
        b->v = nv; b->cap = nc;
    }
    msg_t m = {dst, k->kp, k->s, type, src, (uint32_t)key};
    b->v[b->n++] = m;
}

/* base/broadcast.py:17-40: one message to every peer, self included (:30). */
static void net_broadcast(sim_t* S, uint32_t src, uint32_t type, int key) {
    for (uint32_t d = 0; d < S->n; ++d) net_send(S, src, d, type, key);
}

static void cons_send_key(sim_t* S, uint32_t node, uint32_t s, int32_t value) {
    int key = key_get(S, node * S->sp->nv, s, value);
    if (key >= 0) net_broadcast(S, node, OR_SEND, key);
}

/* core/byzantinerandomizedconsensus.py:64-68 get_max_val: first value (dict insertion
 * order) whose host set is larger than `bound`; `twice` compares 2|hosts| > bound2 so the
 * float bound (N+f)/2 (:73) is exact in integers. */
static int32_t get_max_val(const cons_t* c, uint32_t bound2) {
    for (uint32_t i = 0; i < c->nvals; ++i)
        if (2u * bcount(&c->hosts[c->order[i]]) > bound2) return c->order[i];
    return 0;   /* str(NONE) == "-1" */
}

static void cons_reset(cons_t* c) {
    c->value_count = 0;
    c->nvals = 0;
    memset(c->hosts, 0, sizeof(c->hosts));
}

/* core/byzantinerandomizedconsensus.py:53-106 */
/* core/byzantinerandomizedconsensus.py:53-106 at replica `node` for a message of `host` carrying
 * value id v (the BRB deliver upcall, or a direct deliver() call: OR_ACT_DELIVER) */
static void cons_deliver_vh(sim_t* S, uint32_t node, int32_t v, uint32_t host) {
    cons_t* c = &S->cons[node];
    if (v < 0 || v >= NVAL || host >= S->n) { S->err = -6; return; }
    uint32_t i;
    for (i = 0; i < c->nvals; ++i) if (c->order[i] == v) break;
    if (i == c->nvals) c->order[c->nvals++] = v;   /* :57-58 */
    bset(&c->hosts[v], host);                      /* :60 */
    c->value_count++;                              /* :61 */
    uint32_t n = S->n, f = S->f;
    if (c->value_count > n - f && c->phase == 1) { /* :71 */
        int32_t prop = get_max_val(c, n + f);      /* :73 */
        c->phase = 2;                              /* :75 */
        cons_reset(c);                             /* :76-78 */
        cons_send_key(S, node, 2 * (c->round - 1) + 1, prop);   /* :80-83 */
    }
    if (c->value_count > n - f && c->phase == 2) { /* :86 */
        int32_t dec = get_max_val(c, 4 * f);       /* :88  (|hosts| > 2f) */
        /* :89 compares the string decision with the int NONE: never equal, so the coin
         * branch (:90-92) is dead and decide() always runs (:94). */
        uint32_t ev[4] = {S->t, node, c->round, (uint32_t)dec};
        push_event(S->res->decide, S->res->decide_cap, &S->res->n_decide, 4, ev);
        c->decides++;
        c->round++;                                /* :96 */
        c->phase = 1;                              /* :97 */
        cons_reset(c);                             /* :98-100 */
        cons_send_key(S, node, 2 * (c->round - 1), dec);        /* :102-106 */
    }
}

static void cons_deliver(sim_t* S, uint32_t node, int key) {
    const key_t_* k = &S->keys[key];
    cons_deliver_vh(S, node, k->value, k->kp / S->sp->nv);   /* host: frozenset(dict["host"]) (:55) */
}

/* ------------------------------------------------------------------ SPEC consensus */
static uint32_t spec_window(const sim_t* S) {
    return (S->sp->window && S->sp->window < SPEC_RING) ? S->sp->window : SPEC_RING;
}

/* Phase ends of replica `node` while its current window holds n-f distinct origins
 * (core/byzantinerandomizedconsensus.py:71-106 as intended: thresholds of :73 and :88, the
 * :90 "> f" fallback, and the :92 coin made common and reachable). */
static void spec_advance(sim_t* S, uint32_t node) {
    cons_t* c = &S->cons[node];
    const uint32_t n = S->n, f = S->f, W = spec_window(S);
    while (c->round > 0) {
        const uint32_t s = 2 * (c->round - 1) + (c->phase - 1), q = s % W;
        if (bcount(&c->seen[q]) < n - f) return;
        const uint32_t c0 = c->cnt[q][0], c1 = c->cnt[q][1];
        memset(&c->seen[q], 0, sizeof(bits_t));
        c->cnt[q][0] = c->cnt[q][1] = 0;
        if (c->phase == 1) {
            /* :73 -- a value carried by more than (n+f)/2 of the phase's deliveries, else "-1" */
            const int32_t prop = (2 * c0 > n + f) ? 1 : (2 * c1 > n + f) ? 2 : 0;
            c->phase = 2;
            cons_send_key(S, node, s + 1, prop);
        } else {
            /* :88-92 -- the more frequent of "0"/"1" (tie: "0"): decide above 2f, adopt above f,
             * else the common coin of (instance, round) */
            const int32_t vmax = (c1 > c0) ? 2 : 1;
            const uint32_t cmax = (c1 > c0) ? c1 : c0;
            int32_t est;
            if (cmax > 2 * f) {
                uint32_t ev[4] = {S->t, node, c->round, (uint32_t)vmax};
                push_event(S->res->decide, S->res->decide_cap, &S->res->n_decide, 4, ev);
                c->decides++;
                est = vmax;
            } else if (cmax > f) {
                est = vmax;
            } else {
                est = (int32_t)oracle_coin_id(S->sp->coin_seed, S->sp->g, c->round);
            }
            c->round++;
            c->phase = 1;
            cons_send_key(S, node, s + 1, est);
        }
    }
}

/* one BRB delivery at replica `node` (SPEC): counted once per origin in the window of its
 * phase index; earlier phases are ignored, phases beyond the window overflow */
static void spec_deliver(sim_t* S, uint32_t node, int key) {
    cons_t* c = &S->cons[node];
    key_t_* k = &S->keys[key];
    const uint32_t W = spec_window(S), host = k->kp / S->sp->nv, s = k->s;
    const uint32_t cur = c->round ? 2 * (c->round - 1) + (c->phase - 1) : 0;
    if (s < cur) return;
    if (s >= cur + W) { S->overflow = 1; return; }
    const uint32_t q = s % W;
    if (btest(&c->seen[q], host)) return;
    bset(&c->seen[q], host);
    if (k->value == 1) c->cnt[q][0]++;
    else if (k->value == 2) c->cnt[q][1]++;
    spec_advance(S, node);
}

/* Bracha's broadcast (SPEC): ECHO on the first SEND of a key, one READY per key sent at the
 * echo quorum or at f+1 READYs, DELIVER at 2f+1 READYs; everything after DELIVER ignored. */
static void brb_on_message_spec(sim_t* S, const msg_t* m) {
    key_t_* k = &S->keys[m->key];
    cell_t* c = &k->cells[m->dst];
    uint32_t n = S->n, f = S->f;
    S->res->arrivals++;
    if (c->del) return;
    if (m->type == OR_SEND) {
        if (!c->es) { c->es = 1; net_broadcast(S, m->dst, OR_ECHO, (int)m->key); }
    } else if (m->type == OR_ECHO) {
        bset(&c->e, m->src);
        if (2u * bcount(&c->e) > n + f && !c->rs) { c->rs = 1; net_broadcast(S, m->dst, OR_READY, (int)m->key); }
    } else if (m->type == OR_READY) {
        bset(&c->r, m->src);
        if (bcount(&c->r) > f && !c->rs) { c->rs = 1; net_broadcast(S, m->dst, OR_READY, (int)m->key); }
        if (bcount(&c->r) > 2 * f) {
            c->del = 1;
            uint32_t ev[4] = {S->t, m->dst, k->kp, k->s};
            push_event(S->res->deliver, S->res->deliver_cap, &S->res->n_deliver, 4, ev);
            if (S->sp->mode == OR_MODE_SPEC) spec_deliver(S, m->dst, (int)m->key);
        }
    }
}

/* core/bebroadcast.py:30-42 as intended (its constructor passes the wrong arguments to
 * Broadcast.__init__ and raises): every received message is delivered -- to the consensus
 * instance in BEB_CONSENSUS mode (:42).  Only SENDs are ever sent; the network delivers each
 * (origin, key) SEND once. */
static void beb_on_message(sim_t* S, const msg_t* m) {
    key_t_* k = &S->keys[m->key];
    cell_t* c = &k->cells[m->dst];
    S->res->arrivals++;
    if (m->type != OR_SEND || c->del) return;
    c->del = 1;
    uint32_t ev[4] = {S->t, m->dst, k->kp, k->s};
    push_event(S->res->deliver, S->res->deliver_cap, &S->res->n_deliver, 4, ev);
    if (S->sp->mode == OR_MODE_BEB_CONSENSUS) cons_deliver(S, m->dst, (int)m->key);
}

/* set.add(peer_address) then len(set) (core/brbroadcast.py:69-71): a sender id, or a new
 * connection per message */
static uint32_t peer_add(const sim_t* S, bits_t* set, uint32_t* cnt, uint32_t src) {
    if (S->sp->peer_mode == OR_PEER_CONNECTION) return ++*cnt;
    bset(set, src);
    return bcount(set);
}

/* core/brbroadcast.py:60-119, one accept-loop iteration at node `dst`. */
static void brb_on_message(sim_t* S, const msg_t* m) {
    key_t_* k = &S->keys[m->key];
    cell_t* c = &k->cells[m->dst];
    uint32_t n = S->n, f = S->f;
    S->res->arrivals++;
    if (c->del) return;                                       /* :74 */
    if (m->type == OR_SEND) {
        if (!c->eex) {                                        /* :76 */
            c->eex = 1; memset(&c->e, 0, sizeof(bits_t)); c->ne = 0;   /* :79 */
            net_broadcast(S, m->dst, OR_ECHO, (int)m->key);   /* :82 */
        }
    } else if (m->type == OR_ECHO) {
        if (!c->eex) {                                        /* :87-89: no threshold check */
            c->eex = 1; memset(&c->e, 0, sizeof(bits_t)); c->ne = 0;
            peer_add(S, &c->e, &c->ne, m->src);
        } else {
            const uint32_t ne = peer_add(S, &c->e, &c->ne, m->src);   /* :92 */
            if (2u * ne > n + f && !c->rex) {                 /* :95 */
                c->rex = 1; memset(&c->r, 0, sizeof(bits_t)); c->nr = 0;   /* :96 */
                net_broadcast(S, m->dst, OR_READY, (int)m->key);  /* :98 */
            }
        }
    } else if (m->type == OR_READY) {
        if (!c->rex) {                                        /* :103-105: no check */
            c->rex = 1; memset(&c->r, 0, sizeof(bits_t)); c->nr = 0;
            peer_add(S, &c->r, &c->nr, m->src);
        } else {
            const uint32_t nr = peer_add(S, &c->r, &c->nr, m->src);   /* :108 */
            if (nr > 2 * f) {                                 /* :111 */
                c->del = 1;                                   /* :112 */
                uint32_t ev[4] = {S->t, m->dst, k->kp, k->s};
                push_event(S->res->deliver, S->res->deliver_cap, &S->res->n_deliver, 4, ev);
                if (S->sp->mode == OR_MODE_CONSENSUS) cons_deliver(S, m->dst, (int)m->key);  /* :115 */
            } else if (!c->eex && nr > f) {                   /* :118 */
                net_broadcast(S, m->dst, OR_READY, (int)m->key);  /* :119 (re-fires) */
            }
        }
    }
}

static int msg_cmp(const void* a, const void* b) {
    const msg_t* x = (const msg_t*)a; const msg_t* y = (const msg_t*)b;
    if (x->dst != y->dst) return x->dst < y->dst ? -1 : 1;
    if (x->kp != y->kp) return x->kp < y->kp ? -1 : 1;
    if (x->s != y->s) return x->s < y->s ? -1 : 1;
    if (x->type != y->type) return x->type < y->type ? -1 : 1;
    if (x->src != y->src) return x->src < y->src ? -1 : 1;
    return 0;
}

static void do_action(sim_t* S, const oracle_action* a) {
    switch (a->kind) {
    case OR_ACT_PROPOSE: {                    /* core/byzantinerandomizedconsensus.py:43-50 */
        cons_t* c = &S->cons[a->node];
        c->round = 1; c->phase = 1;           /* value_count is NOT reset (:44-46) */
        cons_send_key(S, a->node, 0, a->value);
        if (S->sp->mode == OR_MODE_SPEC) spec_advance(S, a->node);   /* phase 0 may be buffered */
        break;
    }
    case OR_ACT_BRB_SEND: {                   /* BRBroadcast.broadcast(SEND, msg) */
        int key = key_get(S, a->kp, a->s, a->value);
        if (key >= 0) net_broadcast(S, a->node, OR_SEND, key);
        break;
    }
    case OR_ACT_BYZ_KEY:
        key_get(S, a->kp, a->s, a->value);
        break;
    case OR_ACT_DELIVER:                      /* a direct deliver() call (:53): no BRB involved */
        if (a->node >= S->n || !is_honest(S, a->node) ||
            (S->sp->mode != OR_MODE_CONSENSUS && S->sp->mode != OR_MODE_BEB_CONSENSUS)) { S->err = -9; return; }
        cons_deliver_vh(S, a->node, a->value, a->kp);
        break;
    case OR_ACT_BYZ: {
        int key = key_find(S, a->kp, a->s);
        if (key < 0) { S->err = -7; return; }
        for (uint32_t d = 0; d < S->n; ++d)
            if ((a->dst[d >> 6] >> (d & 63)) & 1ull) net_send(S, a->node, d, a->type, key);
        break;
    }
    default:
        S->err = -8;
    }
}

int oracle_run(const oracle_spec* sp, oracle_result* res) {
    if (!sp || !res || sp->n == 0 || sp->n > OR_MAXN || sp->dmax < 1 || sp->dmax > 16 || sp->nv < 1)
        return -1;
    sim_t* S = (sim_t*)calloc(1, sizeof(sim_t));
    if (!S) return -2;
    S->sp = sp; S->res = res; S->n = sp->n; S->f = sp->f; S->D = sp->dmax;
    res->status = 0; res->t_stop = 0; res->msgs_sent = 0; res->arrivals = 0;
    res->n_deliver = res->n_decide = res->n_send = 0;
    res->cell_steps = 0;
    for (uint32_t s = 0; s < S->n; ++s)
        for (uint32_t d = 0; d < S->n; ++d)
            S->delay[s][d] = (uint8_t)oracle_delay(sp->n, sp->f, sp->seed, sp->delay_model, sp->dmax,
                                                   sp->dconst, sp->g, s, d);
    /* actions must be sorted by time */
    size_t ai = 0;
    S->t = 0;
    while (ai < sp->n_actions && sp->actions[ai].t == 0) do_action(S, &sp->actions[ai++]);
    uint32_t last_active = 0;
    for (;;) {
        if (S->err) break;
        /* next step with arrivals or actions */
        uint32_t nt = UINT32_MAX;
        for (uint32_t dt = 1; dt <= S->D; ++dt)
            if (S->buckets[(S->t + dt) % (S->D + 1)].n) { nt = S->t + dt; break; }
        if (ai < sp->n_actions && sp->actions[ai].t < nt) nt = sp->actions[ai].t;
        if (nt == UINT32_MAX) { res->status = OR_ST_QUIESCENT; break; }
        if (nt > sp->step_cap) { res->status = OR_ST_STEPCAP; break; }
        S->t = nt;
        bucket_t* b = &S->buckets[nt % (S->D + 1)];
        int active = b->n > 0 || (ai < sp->n_actions && sp->actions[ai].t == nt);
        if (active) last_active = nt;
        /* take the bucket (sends made now land at >= t+1, never in this bucket) */
        msg_t* v = b->v; size_t cnt = b->n;
        b->v = NULL; b->n = 0; b->cap = 0;
        qsort(v, cnt, sizeof(msg_t), msg_cmp);
        /* cell-steps: distinct (receiver, key) among the step's messages (sorted by dst, kp, s) */
        for (size_t i = 0; i < cnt; ++i)
            if (i == 0 || v[i].dst != v[i - 1].dst || v[i].key != v[i - 1].key) res->cell_steps++;
        const int spec = sp->mode == OR_MODE_SPEC || sp->mode == OR_MODE_SPEC_BRB;
        const int beb = sp->mode == OR_MODE_BEB || sp->mode == OR_MODE_BEB_CONSENSUS;
        for (size_t i = 0; i < cnt && !S->err; ++i) {
            if (spec) brb_on_message_spec(S, &v[i]);
            else if (beb) beb_on_message(S, &v[i]);
            else brb_on_message(S, &v[i]);
        }
        free(v);
        while (ai < sp->n_actions && sp->actions[ai].t == nt) do_action(S, &sp->actions[ai++]);
        if (S->overflow) { res->status = OR_ST_OVERFLOW; break; }
        if ((sp->mode == OR_MODE_CONSENSUS || sp->mode == OR_MODE_SPEC || sp->mode == OR_MODE_BEB_CONSENSUS) &&
            sp->round_cap > 0) {
            int all = 1;
            for (uint32_t i = 0; i < S->n; ++i)
                if (is_honest(S, i) && S->cons[i].decides < sp->round_cap) { all = 0; break; }
            if (all) { res->status = OR_ST_DONE; break; }
        }
    }
    res->t_stop = last_active;
    int err = S->err;
    for (size_t i = 0; i < S->nkeys; ++i) { free(S->keys[i].cells); free(S->keys[i].sent); }
    free(S->keys); free(S->hkeys);
    for (int i = 0; i < 17; ++i) free(S->buckets[i].v);
    free(S);
    return err;
}
