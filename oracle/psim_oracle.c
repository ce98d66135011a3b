/*
 * oracle/psim_oracle.c -- TEST INFRASTRUCTURE ONLY.  Not part of the product.
 *
 * A deliberately plain, single-threaded CPU restatement of partisan's
 * HyParView peer-service manager and Plumtree broadcast under the BSP round
 * model R0.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker.  The
 * product (libpartisan_gpu_sim.so) never links or calls it.
 *
 * Style: views are kept as lists in sets:to_list/1 order and every handler is
 * written as a transliteration of the Erlang clause it cites, with the
 * list operations (--, lists:usort, lists:sublist(shuffle(...))) spelled out.
 * The GPU engine (partisan_amd/csrc/psim_engine.hip) is an independent
 * data-oriented implementation of the same model; the parity tests compare the
 * two bit for bit.
 *
 * PARITY UNPINNED against the Erlang reference: /root/reference holds no
 * golden vectors for this path and no Erlang VM
 * exists in this image, so the reference cannot be run to produce any.  This
 * oracle is pinned only by the reference's behavioural invariants
 * (test/partisan_SUITE.erl:2044-2108 connectivity + symmetry,
 *  :2024-2041 crashed node leaves every view, :1955-1994 delivery), which
 * tests/test_oracle.py checks, and by line-by-line citation.
 *
 * Exported symbols mirror include/partisan_gpu_sim.h with an `orc_` prefix.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/partisan_gpu_sim.h"

/* ------------------------------------------------------------------ RNG -- */
/* Philox4x32-10 (Salmon et al. 2011).  key = seed, counter = (draw#, node,
 * stream).  One 58-bit value per draw, the width of OTP's exsplus
 * (partisan_config.erl:154-170 seeds exsplus; the harness installs a
 * Philox-backed rand alg handler with bits=58). */
static void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                   uint32_t k1, uint32_t out[4]) {
    for (int i = 0; i < 10; i++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0;
        c1 = (uint32_t)p1;
        c2 = n2;
        c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

#define STREAM_HYPARVIEW 0u
#define TWO58 ((uint64_t)1 << 58)

typedef struct node {
    uint32_t up, epoch, start_round, join_contact;
    uint64_t rng;
    uint32_t act[PSIM_ACTIVE_CAP]; uint32_t act_n;
    uint32_t pas[PSIM_PASSIVE_CAP]; uint32_t pas_n;
    uint32_t sent_peer[PSIM_IDMAP_CAP], sent_id[PSIM_IDMAP_CAP], sent_n, sent_head;
    uint32_t recv_peer[PSIM_IDMAP_CAP], recv_id[PSIM_IDMAP_CAP], recv_n, recv_head;
    uint32_t pt_all[PSIM_PT_MEMBERS_CAP], pt_all_n;
    uint32_t pt_common[PSIM_PT_MEMBERS_CAP], pt_common_n;
    /* eager_sets / lazy_sets (plumtree:76-84): one slot per root, PSIM_NONE = free */
    uint32_t rt_root[PSIM_PT_ROOTS];
    /* the sets of all slots share a pool of PSIM_PT_SET_POOL entries each */
    uint32_t rt_eag[PSIM_PT_ROOTS][PSIM_PT_SET_POOL], rt_eag_n[PSIM_PT_ROOTS];
    uint32_t rt_laz[PSIM_PT_ROOTS][PSIM_PT_SET_POOL], rt_laz_n[PSIM_PT_ROOTS];
    uint32_t out_peer[PSIM_PT_OUT_CAP], out_msg[PSIM_PT_OUT_CAP], out_round[PSIM_PT_OUT_CAP], out_n;
    uint64_t have;                  /* plumtree_backend ETS: bit (msg id mod PSIM_MSG_SLOTS) */
    uint32_t trk_round, trk_hop;
    /* the manager's connections (partisan_peer_service_connections) beyond
     * the active view: lingering peers, and | PSIM_CONN_DOWN the active
     * members without one; insertion order */
    uint32_t conn[PSIM_CONN_CAP], conn_n;
} node;

typedef struct omsg {
    uint32_t dst, src, seq;
    uint32_t type, ttl, nex;
    uint32_t a0, a1, a2, a3;        /* a3: record word 7 (X-BOT's DisconnectNode, else 0) */
    uint32_t ex[PSIM_EXCHANGE_CAP];
    uint32_t slot;                  /* full strategy: payload snapshot (not part of the record digest) */
} omsg;

/* pluggable manager + membership strategy state of a node */
typedef struct snode {
    uint32_t started;               /* has ever been started (full: no restarts) */
    uint32_t pending, hello_sent;   /* internal_join/3: Pending = [Contact] until the handshake */
    uint32_t last_ping;             /* scamp last_message_time as a round, PSIM_NONE = undefined */
    uint32_t view[PSIM_SVIEW_CAP], view_n;   /* scamp v1 membership / v2 partial_view */
    uint32_t view_slots;            /* scamp v1: active slots of the membership set (sets v1, >= 16) */
    uint32_t inv[PSIM_SVIEW_CAP], inv_n;     /* scamp v2 in_view */
    uint32_t leave_tgt;             /* leave/1 call of this round: target + 1, 0 = none */
} snode;

typedef struct msgvec { omsg *v; size_t n, cap; } msgvec;

struct psim_handle {
    psim_config cfg;
    uint32_t N;
    uint32_t lo, hi;                /* owned id range (sharded protocol) */
    node *nodes;
    uint8_t *part, *crashed_now;
    uint64_t round;
    msgvec inbox, out;              /* inbox sorted by (dst, src, seq) */
    size_t *in_beg;                 /* N+1 offsets into inbox */
    /* pending events */
    uint32_t *pend_crash; size_t pend_crash_n, pend_crash_cap;
    uint32_t *pend_join, *pend_contact; size_t pend_join_n, pend_join_cap;
    uint8_t *pend_join_mark;   /* ids in pend_join: a node starts at most once per round */
    uint32_t *pend_lv_a, *pend_lv_t; size_t pend_lv_n, pend_lv_cap;
    uint8_t *pend_part; int pend_part_set, pend_part_clear;
    /* broadcasts of the next round (psim_broadcast, in call order) */
    uint32_t pend_b_root[PSIM_MSG_SLOTS], pend_b_msg[PSIM_MSG_SLOTS]; uint32_t pend_b_n;
    /* message slots: the id owning slot k and its root (node_spec map identity) */
    uint32_t slot_msg[PSIM_MSG_SLOTS], slot_root[PSIM_MSG_SLOTS];
    uint32_t *origin;               /* per node: message id + 1 it originates this round, 0 = none */
    uint32_t tracked_msg;
    psim_round_stats *st;           /* stats of the round being executed */
    /* PLUGGABLE handles */
    snode *sn;
    uint32_t W;                     /* full: words per member bitset */
    uint32_t *fbits;                /* full: N rows of 2W words: the ORSet's adds, then its
                                       removes (tombstones); member = add & ~rmv */
    uint32_t *pay_in, *pay_out;     /* full: gossip payload snapshots of rounds r-1 and r */
    size_t pay_out_n, pay_out_cap, pay_in_cap;
    /* omission faults (interposition funs, pluggable:297-326): the pairs
     * (src << 32 | dst) of the installed {send_omission, Dst} funs at Src and
     * {receive_omission, Src} funs at Dst, and the generally omitting nodes;
     * nx_* are the next round's (the API edits them, round_begin adopts them) */
    struct fault_set { uint64_t *send, *recv; size_t send_n, recv_n; uint8_t *faulted; } flt, nx;
    int faults_dirty;
    uint8_t *btab;                  /* low 8 bits of erlang:phash(NodeSpec, 2^32) - 1 per node
                                       (orc_set_phash_table / orc_set_bucket_table), NULL = stand-in */
};

/* per-node execution context */
typedef struct ctx {
    struct psim_handle *h;
    node *s;
    uint32_t me;
    uint32_t seq;
    uint32_t snap;                  /* full: payload slot of the current state, PSIM_NONE */
    int dirty;                      /* full: state changed since that snapshot */
    int gossip_due;                 /* full, fanout > 0: a coalesced gossip is owed this round */
    int stop;                       /* the manager stopped in this round (leave, App. A Q12) */
    uint32_t nomit_send;            /* sends an omission fault dropped this round */
} ctx;

/* a fixed-table overflow of kind PSIM_OVF_* */
static void ovf(ctx *c, int kind) {
    c->h->st->overflow++;
    c->h->st->overflow_by[kind]++;
}

static uint64_t draw58(ctx *c) {
    uint32_t o[4];
    uint64_t k = c->s->rng++;
    philox((uint32_t)k, (uint32_t)(k >> 32), c->me, STREAM_HYPARVIEW, (uint32_t)c->h->cfg.seed,
           (uint32_t)(c->h->cfg.seed >> 32), o);
    return ((((uint64_t)o[1]) << 32) | o[0]) >> 6;
}

/* rand:uniform/1 for a 58-bit alg handler (OTP rand.erl ?uniform_range):
 * V < N -> V+1; else I = V rem N, accept when V - I =< 2^58 - N. */
static uint32_t uniform_n(ctx *c, uint32_t n) {
    for (;;) {
        uint64_t v = draw58(c);
        if (v < n) return (uint32_t)v + 1;
        uint64_t i = v % n;
        if (v - i <= TWO58 - n) return (uint32_t)i + 1;
    }
}

/* rand:uniform/0 as a sort key: (V bsr 5) * 2^-53 -- the 53-bit integer is an
 * order-preserving stand-in for the float. */
static uint64_t uniform_key(ctx *c) { return draw58(c) >> 5; }

/* ------------------------------------------------------- sets v1 order -- */
/* OTP sets (v1, stdlib sets.erl; the default `sets` before OTP 24 and the
 * one the reference's strategies use) is a linear hash table: `n` active
 * slots (16 at sets:new/0), MaxN the power of two >= n, an element's slot
 * get_slot/2 = phash(E, MaxN), or that minus MaxN/2 past n (the buddy slot).
 * add_element/2 prepends to the slot's bucket; past 5 n elements
 * maybe_expand/2 opens slot n + 1 and rehashes its buddy's bucket into the
 * two (order kept); del_element/2 below 3 n elements (n > 16) closes slot n
 * with maybe_contract/2, its bucket appended to its buddy's
 * (put_bucket_s(Segs0, Slot1, B1 ++ B2), B1 the buddy's bucket).
 * to_list/1 folds slot n..1, each bucket head first, prepending: slot 1..n,
 * oldest first within a slot.  Up to 80 elements that
 * is 16 buckets, erlang:phash(NodeSpec, 16) - 1.  The hash is
 * erlang:phash(NodeSpec, 2^32) - 1 from the handle's table (orc_set_phash_table,
 * e.g. exported by the in-BEAM harness; its low 8 bits: MaxN <= 256 covers
 * every set of <= 128 ids the engine holds); without one the stand-in below
 * (murmur3 fmix32 of the id): see DESIGN.md.  Restated from OTP's published
 * sets.erl; no OTP is present here, so the order past 80 is unpinned. */
static uint32_t phash_default(uint32_t id) {
    uint32_t h = id;
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
    return h;
}
static uint32_t bucket16_default(uint32_t id) { return phash_default(id) & 15u; }
static uint32_t phash8(const struct psim_handle *h, uint32_t id) {
    return h->btab ? h->btab[id] : (phash_default(id) & 255u);
}
static uint32_t set_maxn(uint32_t ns) {
    uint32_t m = 16;
    while (m < ns) m <<= 1;
    return m;
}
/* get_slot/2, 0-based */
static uint32_t set_slot(const struct psim_handle *h, uint32_t e, uint32_t ns) {
    uint32_t m = set_maxn(ns), x = phash8(h, e) & (m - 1);
    return x < ns ? x : x - m / 2;
}
/* the list re-ordered by slot under ns slots, stably: after a slot opens
 * (its entries, from the buddy slot, go to the end: rehash/4 keeps order).
 * `closing` (a slot index under ns + 1, or ~0u): the slot maybe_contract/2
 * just closed; its entries, at the list's end, go in front of the buddy
 * slot's own -- the merged bucket B1 ++ B2 read back by to_list's reversing
 * fold */
static void set_reslot(const struct psim_handle *h, uint32_t *l, uint32_t n, uint32_t ns, uint32_t closing) {
    for (uint32_t i = 1; i < n; i++) {
        uint32_t e = l[i], k = 2 * set_slot(h, e, ns) + (set_slot(h, e, ns + 1) == closing ? 0u : 1u);
        int j = (int)i - 1;
        while (j >= 0 && 2 * set_slot(h, l[j], ns) + (set_slot(h, l[j], ns + 1) == closing ? 0u : 1u) > k) {
            l[j + 1] = l[j];
            j--;
        }
        l[j + 1] = e;
    }
}

static int list_member(const uint32_t *l, uint32_t n, uint32_t e) {
    for (uint32_t i = 0; i < n; i++)
        if (l[i] == e) return 1;
    return 0;
}

/* sets:add_element/2 of a set with *ns active slots (NULL: 16, a set that
 * never grows past 80 elements -- every HyParView view) */
static void set_add(const struct psim_handle *h, uint32_t *l, uint32_t *n, uint32_t e, uint32_t *ns) {
    if (list_member(l, *n, e)) return;
    uint32_t slots = ns ? *ns : 16, b = set_slot(h, e, slots), pos = *n;
    for (uint32_t i = 0; i < *n; i++)
        if (set_slot(h, l[i], slots) > b) { pos = i; break; }
    for (uint32_t i = *n; i > pos; i--) l[i] = l[i - 1];
    l[pos] = e;
    (*n)++;
    if (ns && *n > 5 * *ns) {           /* maybe_expand/2: size + 1 > exp_size */
        (*ns)++;
        set_reslot(h, l, *n, *ns, ~0u);
    }
}

/* sets:del_element/2 of a set with *ns active slots: maybe_contract/2 below
 * 3 n elements */
static void set_del_slots(const struct psim_handle *h, uint32_t *l, uint32_t *n, uint32_t e, uint32_t *ns) {
    uint32_t j = 0;
    for (uint32_t i = 0; i < *n; i++)
        if (l[i] != e) l[j++] = l[i];
    if (j == *n) return;                /* Dc = 0 */
    for (uint32_t i = j; i < *n; i++) l[i] = 0;
    *n = j;
    if (*n < 3 * *ns && *ns > 16) {
        (*ns)--;
        set_reslot(h, l, *n, *ns, *ns);
    }
}

/* sets:del_element/2 of a set that never grew past 16 slots */
static void set_del(uint32_t *l, uint32_t *n, uint32_t e) {
    uint32_t j = 0;
    for (uint32_t i = 0; i < *n; i++)
        if (l[i] != e) l[j++] = l[i];
    for (uint32_t i = j; i < *n; i++) l[i] = 0;
    *n = j;
}

/* List -- Omit (elements unique, so a filter) */
static uint32_t list_subtract(const uint32_t *l, uint32_t n, const uint32_t *omit, uint32_t no,
                              uint32_t *out) {
    uint32_t k = 0;
    for (uint32_t i = 0; i < n; i++)
        if (!list_member(omit, no, l[i])) out[k++] = l[i];
    return k;
}

static int cmp_u32(const void *a, const void *b) {
    uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
    return x < y ? -1 : x > y;
}

/* lists:usort/1 over node ids (term order of the harness node_specs = id order) */
static uint32_t usort(uint32_t *l, uint32_t n) {
    if (n == 0) return 0;
    qsort(l, n, sizeof(uint32_t), cmp_u32);
    uint32_t k = 1;
    for (uint32_t i = 1; i < n; i++)
        if (l[i] != l[k - 1]) l[k++] = l[i];
    return k;
}

/* select_random/2, hyparview:1346-1356: index = rand:uniform(length(List)),
 * no draw when the list is empty (uniform(0) raises before drawing). */
static uint32_t select_random(ctx *c, const uint32_t *view, uint32_t n, const uint32_t *omit,
                              uint32_t no) {
    uint32_t tmp[PSIM_PASSIVE_CAP];
    uint32_t k = list_subtract(view, n, omit, no, tmp);
    if (k == 0) return PSIM_NONE;
    return tmp[uniform_n(c, k) - 1];
}

/* select_random_sublist/2 + shuffle/1, hyparview:1359-1361, :1586-1587:
 * one rand:uniform() key per element in to_list order, lists:sort of
 * {Key, Elem} tuples, then lists:sublist(.., K). */
static uint32_t select_random_sublist(ctx *c, const uint32_t *view, uint32_t n, uint32_t k,
                                      uint32_t *out) {
    uint64_t key[PSIM_PASSIVE_CAP];
    uint32_t el[PSIM_PASSIVE_CAP];
    for (uint32_t i = 0; i < n; i++) { key[i] = uniform_key(c); el[i] = view[i]; }
    for (uint32_t i = 1; i < n; i++) {       /* insertion sort by (key, elem) */
        uint64_t kk = key[i]; uint32_t ee = el[i]; int j = (int)i - 1;
        while (j >= 0 && (key[j] > kk || (key[j] == kk && el[j] > ee))) {
            key[j + 1] = key[j]; el[j + 1] = el[j]; j--;
        }
        key[j + 1] = kk; el[j + 1] = ee;
    }
    uint32_t m = n < k ? n : k;
    for (uint32_t i = 0; i < m; i++) out[i] = el[i];
    return m;
}

/* ------------------------------------------------------------ emission -- */
static uint64_t mix64(uint64_t z) {
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27; z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z;
}

/* Digest of one message: the sum over the 16 words of its 64-B record
 * image [dst, src, type|ttl<<8|nex<<16, seq, a0, a1, a2, a3, ex0..ex7] of
 * word_j * (0x9E3779B1 + 2j * 0x632BE5AB) mod 2^64 (odd multipliers).
 * Position-sensitive, order-free across messages (the round digest is a sum),
 * and one multiply-add per lane on the GPU. */
static uint64_t digest_mul(uint32_t j) { return (uint64_t)(uint32_t)(0x9E3779B1u + 2u * j * 0x632BE5ABu); }

static uint64_t msg_hash(const omsg *m) {
    uint32_t w[16] = {m->dst, m->src, m->type | (m->ttl << 8) | (m->nex << 16), m->seq,
                      m->a0, m->a1, m->a2, m->a3};
    for (uint32_t i = 0; i < m->nex; i++) w[8 + i] = m->ex[i];
    uint64_t h = 0;
    for (uint32_t j = 0; j < 16; j++) h += (uint64_t)w[j] * digest_mul(j);
    return h;
}

static void vec_push(msgvec *v, const omsg *m) {
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 1024;
        v->v = (omsg *)realloc(v->v, v->cap * sizeof(omsg));
    }
    v->v[v->n++] = *m;
}

static void emit4(ctx *c, uint32_t dst, uint32_t type, uint32_t ttl, uint32_t a0, uint32_t a1,
                  uint32_t a2, uint32_t a3, const uint32_t *ex, uint32_t nex) {
    omsg m;
    memset(&m, 0, sizeof m);
    m.dst = dst; m.src = c->me; m.seq = c->seq++;
    m.type = type; m.ttl = ttl; m.nex = nex;
    m.a0 = a0; m.a1 = a1; m.a2 = a2; m.a3 = a3;
    for (uint32_t i = 0; i < nex; i++) m.ex[i] = ex[i];
    vec_push(&c->h->out, &m);
    c->h->st->emitted[type]++;
    c->h->st->digest += msg_hash(&m);
}

static void emit(ctx *c, uint32_t dst, uint32_t type, uint32_t ttl, uint32_t a0, uint32_t a1,
                 uint32_t a2, const uint32_t *ex, uint32_t nex) {
    emit4(c, dst, type, ttl, a0, a1, a2, 0, ex, nex);
}

/* A connection attempt (partisan_util:maybe_connect/2, util.erl:75-134)
 * succeeds iff the peer's manager is running and no network partition
 * separates the two (partition model DESIGN.md). */
static int connect_ok(ctx *c, uint32_t dst) {
    struct psim_handle *h = c->h;
    if (dst >= h->N || dst == c->me) return 0;
    return h->nodes[dst].up && h->part[dst] == h->part[c->me];
}

/* ------------------------------------------------------ connections -- */
/* The Connections dict of the manager as the active view
 * plus the table of node.conn: a peer outside the active view is connected
 * iff it is in the table; an active member is connected unless the table
 * holds it | PSIM_CONN_DOWN.  maybe_connect/2 opens a connection before every
 * HyParView send; only disconnect/2 (hyparview:1237-1258) and the peer's
 * death (EXIT, :609-654) close one; leaving the active view always goes
 * through one of those. */
static int conn_find(const node *s, uint32_t e) {
    for (uint32_t i = 0; i < s->conn_n; i++)
        if (s->conn[i] == e) return (int)i;
    return -1;
}
static void conn_add(ctx *c, uint32_t e) {
    node *s = c->s;
    if (conn_find(s, e) >= 0) return;
    if (s->conn_n >= PSIM_CONN_CAP) { ovf(c, PSIM_OVF_CONN); return; }
    s->conn[s->conn_n++] = e;
}
static void conn_del(node *s, uint32_t e) {
    int i = conn_find(s, e);
    if (i < 0) return;
    for (uint32_t j = (uint32_t)i; j + 1 < s->conn_n; j++) s->conn[j] = s->conn[j + 1];
    s->conn[--s->conn_n] = 0;
}
/* X-BOT: the member's connection pid was stopped by a do_disconnect whose
 * state was discarded -- the dead pid is still in the dict (PSIM_CONN_CLOSING) */
static int conn_closing(const node *s, uint32_t p) { return s->conn_n && conn_find(s, p | PSIM_CONN_CLOSING) >= 0; }
/* partisan_peer_service_connections:find/2 succeeds over a live pid */
static int conn_has(ctx *c, uint32_t p) {
    node *s = c->s;
    if (list_member(s->act, s->act_n, p))
        return conn_find(s, p | PSIM_CONN_DOWN) < 0 && !conn_closing(s, p);
    return conn_find(s, p) >= 0;
}
/* partisan_util:maybe_connect/2: 1 iff connected afterwards (a dead pid in
 * the dict counts as found: maybe_connect opens nothing, util.erl:111-115) */
static int maybe_connect(ctx *c, uint32_t p) {
    if (conn_closing(c->s, p)) return 1;
    if (!connect_ok(c, p)) return 0;
    if (list_member(c->s->act, c->s->act_n, p)) conn_del(c->s, p | PSIM_CONN_DOWN);
    else conn_add(c, p);
    return 1;
}
/* disconnect/2 (hyparview:1237-1258).  X-BOT: stopping a pid that is already
 * dead (PSIM_CONN_CLOSING) raises noproc in gen_server:stop/1 and would take
 * the manager down; here the entry is pruned like a live one */
static void disconnect(ctx *c, uint32_t p) {
    if (conn_closing(c->s, p)) conn_del(c->s, p | PSIM_CONN_CLOSING);
    if (list_member(c->s->act, c->s->act_n, p)) conn_add(c, p | PSIM_CONN_DOWN);
    else conn_del(c->s, p);
}

/* maybe_connect, then do_send_message/3 (hyparview:1274-1343): on success
 * partisan_util:dispatch_pid/1 draws rand:uniform(1) (util:190-195).  Every
 * HyParView send of the reference is preceded by a maybe_connect of its
 * destination (:506, :594, :721, :743, :784, :830, :878, :906, :987, :1110,
 * :1127, :1493, :1701). */
static int hv_send(ctx *c, uint32_t dst, uint32_t type, uint32_t ttl, uint32_t a0, uint32_t a1,
                   const uint32_t *ex, uint32_t nex) {
    if (conn_closing(c->s, dst)) {                /* X-BOT: dispatch_pid draws, the call to the */
        (void)uniform_n(c, 1);                    /* dead pid fails (hyparview:1507-1514) */
        c->h->st->send_fail++;
        return 0;
    }
    if (!maybe_connect(c, dst)) { c->h->st->send_fail++; return 0; }
    (void)uniform_n(c, 1);
    emit(c, dst, type, ttl, a0, a1, 0, ex, nex);
    return 1;
}

/* ----------------------------------------------------- disconnect ids -- */
#define ID(e, n) (((uint32_t)(e) << 20) | (uint32_t)(n))
#define ID_E(id) ((id) >> 20)
#define ID_C(id) ((id) & 0xFFFFFu)

static int map_find(const uint32_t *peer, uint32_t n, uint32_t p) {
    for (uint32_t i = 0; i < n; i++)
        if (peer[i] == p) return (int)i;
    return -1;
}

/* dict:store/3 into a fixed table; when full the oldest slot is replaced
 * (counted as overflow). */
static void map_store(ctx *c, uint32_t *peer, uint32_t *id, uint32_t *n, uint32_t *head,
                      uint32_t p, uint32_t v) {
    int i = map_find(peer, *n, p);
    if (i >= 0) { id[i] = v; return; }
    if (*n < PSIM_IDMAP_CAP) { peer[*n] = p; id[*n] = v; (*n)++; return; }
    ovf(c, PSIM_OVF_IDMAP);
    peer[*head] = p; id[*head] = v;
    *head = (*head + 1) % PSIM_IDMAP_CAP;
}

/* get_current_id/2, hyparview:1622-1630 */
static uint32_t current_id(ctx *c, uint32_t p) {
    int i = map_find(c->s->recv_peer, c->s->recv_n, p);
    return i >= 0 ? c->s->recv_id[i] : ID(1, 0);
}

/* get_next_id/3, hyparview:1633-1639 */
static uint32_t next_id(ctx *c, uint32_t p) {
    int i = map_find(c->s->sent_peer, c->s->sent_n, p);
    if (i >= 0 && ID_E(c->s->sent_id[i]) == c->s->epoch) return c->s->sent_id[i] + 1;
    return ID(c->s->epoch, 1);
}

/* is_addable/3 integer-epoch clause, hyparview:1670-1676 */
static int addable_epoch(ctx *c, uint32_t pe, uint32_t p) {
    int i = map_find(c->s->sent_peer, c->s->sent_n, p);
    if (i < 0) return 1;
    return pe >= ID_E(c->s->sent_id[i]);
}

/* is_addable/3 disconnect-id clause, hyparview:1656-1669 */
static int addable_id(ctx *c, uint32_t d, uint32_t p) {
    int i = map_find(c->s->sent_peer, c->s->sent_n, p);
    if (i < 0) return 1;
    uint32_t e = ID_E(c->s->sent_id[i]), n = ID_C(c->s->sent_id[i]);
    if (ID_E(d) > e) return 1;
    if (ID_E(d) == e) return ID_C(d) >= n;
    return 0;
}

/* is_valid_disconnect/3, hyparview:1642-1653 */
static int valid_disconnect(ctx *c, uint32_t p, uint32_t d) {
    int i = map_find(c->s->recv_peer, c->s->recv_n, p);
    if (i < 0) return 1;
    uint32_t e = ID_E(c->s->recv_id[i]), n = ID_C(c->s->recv_id[i]);
    if (ID_E(d) > e) return 1;
    return ID_C(d) > n;
}

/* ------------------------------------------------------ view updates -- */
/* add_to_passive_view/2, hyparview:1423-1448 */
static void add_to_passive(ctx *c, uint32_t p) {
    node *s = c->s;
    if (p == c->me || list_member(s->act, s->act_n, p) || list_member(s->pas, s->pas_n, p)) return;
    if (s->pas_n >= c->h->cfg.max_passive_size) {
        uint32_t omit[1] = {c->me};
        uint32_t r = select_random(c, s->pas, s->pas_n, omit, 1);
        if (r != PSIM_NONE) set_del(s->pas, &s->pas_n, r);
    }
    set_add(c->h, s->pas, &s->pas_n, p, NULL);
}

/* drop_random_element_from_active_view/1, hyparview:1467-1512 (no reservations) */
static void drop_random_active(ctx *c) {
    node *s = c->s;
    uint32_t omit[1] = {c->me};
    uint32_t p = select_random(c, s->act, s->act_n, omit, 1);
    if (p == PSIM_NONE) return;
    set_del(s->act, &s->act_n, p);
    conn_del(s, p | PSIM_CONN_DOWN);
    add_to_passive(c, p);
    uint32_t nid = next_id(c, p);
    map_store(c, s->sent_peer, s->sent_id, &s->sent_n, &s->sent_head, p, nid);
    hv_send(c, p, PSIM_MSG_DISCONNECT, 0, nid, 0, NULL, 0);   /* maybe_connect (:1493), send */
    disconnect(c, p);                                         /* (:1506) */
}

/* add_to_active_view/3, hyparview:1371-1420 (tag/reserved ignored).  The
 * connection the caller opened (every caller but neighbor_accepted runs
 * maybe_connect first) moves with the peer into the active view; without one
 * the peer is an active member without a connection. */
static void add_to_active(ctx *c, uint32_t p) {
    node *s = c->s;
    if (p == c->me || list_member(s->act, s->act_n, p)) return;
    set_del(s->pas, &s->pas_n, p);
    if (s->act_n >= c->h->cfg.max_active_size) drop_random_active(c);
    int had = conn_find(s, p) >= 0;
    conn_del(s, p);
    set_add(c->h, s->act, &s->act_n, p, NULL);
    if (!had) conn_add(c, p | PSIM_CONN_DOWN);
}

/* [Myself] ++ select_random_sublist(Active, k_active) ++
 * select_random_sublist(Passive, k_passive), then lists:usort
 * (hyparview:577-586, :989-998, :1689-1698) */
static uint32_t build_exchange(ctx *c, uint32_t *ex) {
    node *s = c->s;
    uint32_t e[1 + PSIM_ACTIVE_CAP + PSIM_PASSIVE_CAP];
    uint32_t n = 0;
    e[n++] = c->me;
    n += select_random_sublist(c, s->act, s->act_n, c->h->cfg.k_active, e + n);
    n += select_random_sublist(c, s->pas, s->pas_n, c->h->cfg.k_passive, e + n);
    n = usort(e, n);
    for (uint32_t i = 0; i < n; i++) ex[i] = e[i];
    return n;
}

/* merge_exchange/2, hyparview:1590-1595 */
static void merge_exchange(ctx *c, const uint32_t *ex, uint32_t nex) {
    node *s = c->s;
    uint32_t omit[1 + PSIM_ACTIVE_CAP], add[PSIM_EXCHANGE_CAP];
    omit[0] = c->me;
    for (uint32_t i = 0; i < s->act_n; i++) omit[1 + i] = s->act[i];
    uint32_t k = list_subtract(ex, nex, omit, 1 + s->act_n, add);
    k = usort(add, k);
    for (uint32_t i = 0; i < k; i++) add_to_passive(c, add[i]);
}

/* move_peer_from_passive_to_active/2, hyparview:1679-1709 */
static void move_to_active(ctx *c, uint32_t p) {
    if (p == PSIM_NONE) return;
    uint32_t ex[PSIM_EXCHANGE_CAP];
    uint32_t nex = build_exchange(c, ex);
    hv_send(c, p, PSIM_MSG_NEIGHBOR_REQUEST, 0, current_id(c, p), 0, ex, nex);
}

/* ------------------------------------------------------------- X-BOT -- */
/* partisan_hyparview_xbot_peer_service_manager (xbot below): HyParView with
 * the X-BOT optimization rounds (xbot:586-606, :691-716, :1171-1346).  Round
 * model R0-X, DESIGN.md section 2c. */
static int is_xbot(const struct psim_handle *h) { return h->cfg.manager == PSIM_MANAGER_XBOT; }

/* the latency oracle: toroidal L1 distance on a 1024 x 1024 grid of
 * hash-placed nodes (psim_xbot_latency in include/partisan_gpu_sim.h) */
static uint32_t xb_coord(uint64_t seed, uint32_t id) {
    return (uint32_t)mix64(seed ^ ((uint64_t)id * 0x9E3779B97F4A7C15ull)) & 0xFFFFFu;
}
static uint32_t xb_axis(uint32_t a, uint32_t b) {
    uint32_t d = a > b ? a - b : b - a;
    return d < 1024u - d ? d : 1024u - d;
}
uint32_t orc_xbot_latency(uint64_t seed, uint32_t a, uint32_t b) {
    if (a == b) return 0;
    uint32_t p = xb_coord(seed, a), q = xb_coord(seed, b);
    return xb_axis(p & 1023u, q & 1023u) + xb_axis(p >> 10, q >> 10);
}

/* net_adm:ping/1 answers pong: the node runs (pings go over distributed
 * Erlang, not partisan: a partition does not stop them) */
static int xb_pong(ctx *c, uint32_t p) { return p == c->me || (p < c->h->N && c->h->nodes[p].up); }

/* is_better(latency, New, Old) at the deciding node (xbot:1318-1333) */
static int xb_better(ctx *c, uint32_t nw, uint32_t old) {
    if (!xb_pong(c, nw)) return 0;
    if (!xb_pong(c, old)) return 1;
    uint64_t sd = c->h->cfg.seed;
    return orc_xbot_latency(sd, c->me, nw) < orc_xbot_latency(sd, c->me, old);
}

/* select_disconnect_node/1 + select_worst_in_active_view/2 (xbot:1336-1346)
 * over sets:to_list(Active) */
static uint32_t xb_worst(ctx *c) {
    node *s = c->s;
    uint32_t worst = s->act[0];
    for (uint32_t i = 1; i < s->act_n; i++)
        if (!xb_better(c, s->act[i], worst)) worst = s->act[i];
    return worst;
}

/* do_send_message over the Connections of a maybe_connect whose result the
 * handler throws away (send_join/2 xbot:1349-1363, every optimization send):
 * the send goes out iff the peer can be reached; the dict is not changed */
static int xb_send(ctx *c, uint32_t dst, uint32_t type, uint32_t ttl, uint32_t a0, uint32_t a1,
                   uint32_t a2, uint32_t a3) {
    if (conn_closing(c->s, dst)) {                /* the dead pid: a draw, a failed call */
        (void)uniform_n(c, 1);
        c->h->st->send_fail++;
        return 0;
    }
    if (!connect_ok(c, dst)) { c->h->st->send_fail++; return 0; }
    (void)uniform_n(c, 1);
    emit4(c, dst, type, ttl, a0, a1, a2, a3, NULL, 0);
    return 1;
}
static void xb_join(ctx *c, uint32_t p) { xb_send(c, p, PSIM_MSG_JOIN, 0, c->s->epoch, 0, 0, 0); }

/* do_disconnect/2 (xbot:1367-1379) with its result discarded by every caller:
 * the passive add's eviction draw is consumed (the rand state lives in the
 * process dictionary) and a live connection's pid is stopped, but the
 * views and the dict stay as they were -- the pid's 'EXIT' removes the peer
 * next round (process_node) */
static void xb_do_disconnect(ctx *c, uint32_t p) {
    node *s = c->s;
    if (!list_member(s->act, s->act_n, p)) return;
    if (p != c->me && !list_member(s->pas, s->pas_n, p) && s->pas_n >= c->h->cfg.max_passive_size)
        (void)uniform_n(c, s->pas_n);             /* select_random(Passive, [Myself]) */
    if (conn_find(s, p | PSIM_CONN_DOWN) < 0 && !conn_closing(s, p)) conn_add(c, p | PSIM_CONN_CLOSING);
}

/* the optimization messages (xbot:1171-1314); a0 Old, a1 Initiator, a2
 * Candidate, a3 Disconnect (PSIM_NONE = undefined), ttl the answer */
static void xb_handle(ctx *c, const omsg *m) {
    node *s = c->s;
    uint32_t old = m->a0, ini = m->a1, cand = m->a2, dis = m->a3, ans = m->ttl;
    switch (m->type) {
    case PSIM_MSG_XBOT_OPTIMIZATION:              /* xbot:1205-1224 (at the candidate) */
        if (s->act_n < c->h->cfg.max_active_size) {
            xb_join(c, ini);
            xb_send(c, ini, PSIM_MSG_XBOT_OPTIMIZATION_REPLY, 1, old, ini, cand, PSIM_NONE);
        } else {
            uint32_t d = xb_worst(c);
            xb_send(c, d, PSIM_MSG_XBOT_REPLACE, 0, old, ini, cand, d);
        }
        break;
    case PSIM_MSG_XBOT_REPLACE:                   /* xbot:1252-1267 (at the disconnect node) */
        if (!xb_better(c, old, cand)) xb_send(c, cand, PSIM_MSG_XBOT_REPLACE_REPLY, 0, old, ini, cand, dis);
        else xb_send(c, old, PSIM_MSG_XBOT_SWITCH, 0, old, ini, cand, dis);
        break;
    case PSIM_MSG_XBOT_SWITCH:                    /* xbot:1295-1314 (at the old node) */
        if (list_member(s->act, s->act_n, ini)) {
            xb_do_disconnect(c, ini);
            xb_join(c, dis);
            xb_send(c, dis, PSIM_MSG_XBOT_SWITCH_REPLY, 1, old, ini, cand, dis);
        } else {
            xb_send(c, dis, PSIM_MSG_XBOT_SWITCH_REPLY, 0, old, ini, cand, dis);
        }
        break;
    case PSIM_MSG_XBOT_SWITCH_REPLY:              /* xbot:1270-1292 (at the disconnect node) */
        if (ans) {
            xb_do_disconnect(c, cand);
            xb_join(c, old);
        }
        xb_send(c, cand, PSIM_MSG_XBOT_REPLACE_REPLY, ans, old, ini, cand, dis);
        break;
    case PSIM_MSG_XBOT_REPLACE_REPLY:             /* xbot:1227-1249 (at the candidate) */
        if (ans) {
            xb_do_disconnect(c, dis);
            xb_join(c, ini);
        }
        xb_send(c, ini, PSIM_MSG_XBOT_OPTIMIZATION_REPLY, ans, old, ini, cand, dis);
        break;
    case PSIM_MSG_XBOT_OPTIMIZATION_REPLY:        /* xbot:1171-1202 (at the initiator) */
        if (!ans) break;
        if (dis != PSIM_NONE && list_member(s->act, s->act_n, old)) xb_do_disconnect(c, old);
        xb_join(c, cand);
        break;
    default:
        break;
    }
}

/* handle_info(xbot_execution) (xbot:587-606, :691-716): with a full active
 * view, two passive candidates, each checked against the active members in
 * to_list order; the first member it beats gets an optimization message */
static void xb_execute(ctx *c) {
    node *s = c->s;
    if (s->act_n < c->h->cfg.max_active_size) return;
    uint32_t cand[2], act[PSIM_ACTIVE_CAP], na = s->act_n;
    memcpy(act, s->act, sizeof act);
    uint32_t nc = select_random_sublist(c, s->pas, s->pas_n, 2, cand);
    for (uint32_t i = 0; i < nc; i++)
        for (uint32_t j = 0; j < na; j++)
            if (xb_better(c, cand[i], act[j])) {
                xb_send(c, cand[i], PSIM_MSG_XBOT_OPTIMIZATION, 0, act[j], c->me, cand[i], PSIM_NONE);
                break;
            }
}

/* --------------------------------------------------------- plumtree -- */
static void pt_set_add(uint32_t *l, uint32_t *n, uint32_t cap, uint32_t e, ctx *c) {
    uint32_t i = 0;
    while (i < *n && l[i] < e) i++;
    if (i < *n && l[i] == e) return;
    if (*n >= cap) { ovf(c, PSIM_OVF_PT); return; }
    for (uint32_t j = *n; j > i; j--) l[j] = l[j - 1];
    l[i] = e;
    (*n)++;
}

static void pt_set_del(uint32_t *l, uint32_t *n, uint32_t e) { set_del(l, n, e); }

static void rt_clear(node *s, int k) {
    s->rt_root[k] = PSIM_NONE;
    memset(s->rt_eag[k], 0, sizeof s->rt_eag[k]); s->rt_eag_n[k] = 0;
    memset(s->rt_laz[k], 0, sizeof s->rt_laz[k]); s->rt_laz_n[k] = 0;
}

/* the root slot of `root`, -1 if it has no per-root sets */
static int rt_find(const node *s, uint32_t root) {
    for (int k = 0; k < PSIM_PT_ROOTS; k++)
        if (s->rt_root[k] == root) return k;
    return -1;
}

/* notify/1 (hyparview:1598-1599) -> partisan_peer_service:decode/1
 * (peer_service.erl:117-119) -> plumtree update/1 -> handle_cast({update,..})
 * (plumtree:314-336), reset_peers/4 (:652-659), neighbors_down/2 (:404-423). */
static void notify(ctx *c) {
    node *s = c->s;
    if (!c->h->cfg.plumtree) return;
    uint32_t cur[PSIM_ACTIVE_CAP], ncur = s->act_n;
    for (uint32_t i = 0; i < ncur; i++) cur[i] = s->act[i];        /* atom names */
    ncur = usort(cur, ncur);
    uint32_t newm[PSIM_ACTIVE_CAP], rem[PSIM_PT_MEMBERS_CAP];
    uint32_t nnew = list_subtract(cur, ncur, s->pt_all, s->pt_all_n, newm);
    uint32_t nrem = list_subtract(s->pt_all, s->pt_all_n, cur, ncur, rem);
    if (nnew > 0) {
        /* EagerPeers = ordsets:union(EagerPeers0, New); reset_peers(Current, ..) */
        uint32_t u[PSIM_PT_MEMBERS_CAP + PSIM_ACTIVE_CAP], nu = 0;
        for (uint32_t i = 0; i < s->pt_common_n; i++) u[nu++] = s->pt_common[i];
        for (uint32_t i = 0; i < nnew; i++) u[nu++] = newm[i];
        nu = usort(u, nu);
        nu = list_subtract(u, nu, rem, nrem, u);   /* neighbors_down applied below anyway */
        memset(s->pt_common, 0, sizeof s->pt_common);
        for (uint32_t i = 0; i < nu; i++) s->pt_common[i] = u[i];
        s->pt_common_n = nu;
        /* del_element(myself(), ..) removes nothing: myself() is a map (Q6);
         * eager_sets = lazy_sets = orddict:new() (:656-657) */
        for (int k = 0; k < PSIM_PT_ROOTS; k++) rt_clear(s, k);
        memset(s->pt_all, 0, sizeof s->pt_all);
        for (uint32_t i = 0; i < ncur; i++) s->pt_all[i] = cur[i];
        s->pt_all_n = ncur;
    }
    /* neighbors_down(Removed, ..) */
    for (uint32_t i = 0; i < nrem; i++) {
        pt_set_del(s->pt_common, &s->pt_common_n, rem[i]);
        for (int k = 0; k < PSIM_PT_ROOTS; k++)        /* every root's sets (:410-413) */
            if (s->rt_root[k] != PSIM_NONE) {
                pt_set_del(s->rt_eag[k], &s->rt_eag_n[k], rem[i]);
                pt_set_del(s->rt_laz[k], &s->rt_laz_n[k], rem[i]);
            }
        uint32_t j = 0;
        for (uint32_t k = 0; k < s->out_n; k++)
            if (s->out_peer[k] != rem[i]) {
                s->out_peer[j] = s->out_peer[k]; s->out_msg[j] = s->out_msg[k];
                s->out_round[j] = s->out_round[k]; j++;
            }
        for (uint32_t k = j; k < s->out_n; k++) s->out_peer[k] = s->out_msg[k] = s->out_round[k] = 0;
        s->out_n = j;
    }
}

/* all_peers/3 (plumtree:627-631): the per-root set or the common default */
static void pt_get(ctx *c, uint32_t root, uint32_t *eg, uint32_t *ne, uint32_t *lz, uint32_t *nl) {
    node *s = c->s;
    int k = rt_find(s, root);
    if (k >= 0) {
        *ne = s->rt_eag_n[k]; memcpy(eg, s->rt_eag[k], sizeof s->rt_eag[k]);
        *nl = s->rt_laz_n[k]; memcpy(lz, s->rt_laz[k], sizeof s->rt_laz[k]);
    } else {
        memset(eg, 0, PSIM_PT_SET_POOL * 4); memset(lz, 0, PSIM_PT_SET_POOL * 4);
        *ne = s->pt_common_n;
        for (uint32_t i = 0; i < s->pt_common_n; i++) eg[i] = s->pt_common[i];
        *nl = 0;                                   /* common_lazys is always [] */
    }
}

/* entries of all slots of a pool */
static uint32_t pool_n(const uint32_t *n) {
    uint32_t t = 0;
    for (int k = 0; k < PSIM_PT_ROOTS; k++) t += n[k];
    return t;
}

/* ordsets:add_element into slot k of a pool: an add to a full pool is an
 * overflow */
static void pool_add(ctx *c, uint32_t (*set)[PSIM_PT_SET_POOL], uint32_t *n, int k, uint32_t e) {
    for (uint32_t i = 0; i < n[k]; i++)
        if (set[k][i] == e) return;
    if (pool_n(n) >= PSIM_PT_SET_POOL) { ovf(c, PSIM_OVF_PT); return; }
    pt_set_add(set[k], &n[k], PSIM_PT_SET_POOL, e, c);
}

/* update_peers/5 + set_peers/4 (plumtree:593-609): orddict:store(Root, ..)
 * into the root's slot; a new root takes the lowest free slot, its sets
 * starting as (common_eagers, []) -- with every slot taken, or the eager pool
 * too full for the common eagers, the store is an overflow (the sets stay
 * as they were) */
static void pt_update(ctx *c, uint32_t from, uint32_t root, int to_eager) {
    node *s = c->s;
    int k = rt_find(s, root);
    if (k < 0) {
        k = rt_find(s, PSIM_NONE);
        if (k < 0 || pool_n(s->rt_eag_n) + s->pt_common_n > PSIM_PT_SET_POOL) { ovf(c, PSIM_OVF_PT); return; }
        s->rt_root[k] = root;
        memcpy(s->rt_eag[k], s->pt_common, s->pt_common_n * 4); s->rt_eag_n[k] = s->pt_common_n;
        s->rt_laz_n[k] = 0;
    }
    if (to_eager) {
        pool_add(c, s->rt_eag, s->rt_eag_n, k, from);
        pt_set_del(s->rt_laz[k], &s->rt_laz_n[k], from);
    } else {
        pt_set_del(s->rt_eag[k], &s->rt_eag_n[k], from);
        pool_add(c, s->rt_laz, s->rt_laz_n, k, from);
    }
}

/* send/3 (plumtree:633-638) -> cast_message -> forward_message
 * (hyparview:441-460) -> do_send_message/4 without maybe_connect: succeeds
 * only over an existing connection of this node's manager -- an active member
 * or a lingering peer (App. A Q11) -- to a running peer in the same partition
 * group. */
static int pt_conn(ctx *c, uint32_t ident) {
    uint32_t id = ident & ~PSIM_MAP_BIT;
    return !(id == c->me || id >= c->h->N || !conn_has(c, id) || !c->h->nodes[id].up ||
             c->h->part[id] != c->h->part[c->me]);
}

static void pt_send(ctx *c, uint32_t ident, uint32_t type, uint32_t msg, uint32_t rnd,
                    uint32_t root) {
    if (!pt_conn(c, ident)) {
        c->h->st->send_fail++;
        return;
    }
    emit(c, ident & ~PSIM_MAP_BIT, type, 0, msg, rnd, root, NULL, 0);
}

/* add_outstanding/6 (plumtree:574-579): ordset keyed by peer, then {Id,..,Round,Root} */
static void pt_add_out(ctx *c, uint32_t peer, uint32_t msg, uint32_t rnd) {
    node *s = c->s;
    uint32_t i = 0;
    while (i < s->out_n &&
           (s->out_peer[i] < peer || (s->out_peer[i] == peer && s->out_msg[i] < msg) ||
            (s->out_peer[i] == peer && s->out_msg[i] == msg && s->out_round[i] < rnd)))
        i++;
    if (i < s->out_n && s->out_peer[i] == peer && s->out_msg[i] == msg && s->out_round[i] == rnd)
        return;
    if (s->out_n >= PSIM_PT_OUT_CAP) { ovf(c, PSIM_OVF_PT_OUT); return; }
    for (uint32_t j = s->out_n; j > i; j--) {
        s->out_peer[j] = s->out_peer[j - 1]; s->out_msg[j] = s->out_msg[j - 1];
        s->out_round[j] = s->out_round[j - 1];
    }
    s->out_peer[i] = peer; s->out_msg[i] = msg; s->out_round[i] = rnd;
    s->out_n++;
}

/* ack_outstanding/6 (plumtree:562-567) */
static void pt_ack_out(ctx *c, uint32_t peer, uint32_t msg, uint32_t rnd) {
    node *s = c->s;
    for (uint32_t i = 0; i < s->out_n; i++)
        if (s->out_peer[i] == peer && s->out_msg[i] == msg && s->out_round[i] == rnd) {
            for (uint32_t j = i; j + 1 < s->out_n; j++) {
                s->out_peer[j] = s->out_peer[j + 1]; s->out_msg[j] = s->out_msg[j + 1];
                s->out_round[j] = s->out_round[j + 1];
            }
            s->out_n--;
            s->out_peer[s->out_n] = s->out_msg[s->out_n] = s->out_round[s->out_n] = 0;
            return;
        }
}

/* plumtree_backend is_stale/1 (:101-104, :148-152) over the node's message
 * slots; a retired id (its slot taken by a newer broadcast) is an overflow
 * and answers stale */
static int pt_have(ctx *c, uint32_t msg) {
    uint32_t k = msg % PSIM_MSG_SLOTS;
    if (c->h->slot_msg[k] != msg) { ovf(c, PSIM_OVF_PT); return 1; }
    return (int)((c->s->have >> k) & 1u);
}

/* the root of a live message id (IHAVE of an outstanding entry); a retired
 * id is an overflow and PSIM_NONE */
static uint32_t msg_root(ctx *c, uint32_t msg) {
    uint32_t k = msg % PSIM_MSG_SLOTS;
    if (c->h->slot_msg[k] != msg) { ovf(c, PSIM_OVF_PT); return PSIM_NONE; }
    return c->h->slot_root[k];
}

/* eager_push/7 + schedule_lazy_push/6 (plumtree:428-441) */
static void pt_push(ctx *c, uint32_t msg, uint32_t rnd, uint32_t root, uint32_t from) {
    uint32_t eg[PSIM_PT_SET_POOL], lz[PSIM_PT_SET_POOL], ne, nl;
    pt_get(c, root, eg, &ne, lz, &nl);
    pt_set_del(eg, &ne, from);                    /* all_filtered_peers/4 */
    for (uint32_t i = 0; i < ne; i++) pt_send(c, eg[i], PSIM_MSG_PT_BROADCAST, msg, rnd, root);
    pt_get(c, root, eg, &ne, lz, &nl);
    pt_set_del(lz, &nl, from);
    for (uint32_t i = 0; i < nl; i++) pt_add_out(c, lz[i], msg, rnd);
}

static void pt_handle(ctx *c, const omsg *m) {
    node *s = c->s;
    uint32_t from = m->src | PSIM_MAP_BIT, root = m->a2, msg = m->a0, rnd = m->a1;
    switch (m->type) {
    case PSIM_MSG_PT_BROADCAST: {                 /* plumtree:288-293, :368-378 */
        int valid = !pt_have(c, msg);             /* plumtree_backend merge/2 :87-96 */
        if (valid) {
            s->have |= 1ull << (msg % PSIM_MSG_SLOTS);
            c->h->st->first_deliveries++;
            if (msg == c->h->tracked_msg) { s->trk_round = (uint32_t)c->h->round; s->trk_hop = rnd + 1; }
            pt_update(c, from, root, 1);
            pt_push(c, msg, rnd + 1, root, from);
        } else {
            pt_update(c, from, root, 0);
            pt_send(c, from, PSIM_MSG_PT_PRUNE, 0, 0, root);
        }
        break;
    }
    case PSIM_MSG_PT_PRUNE:                       /* plumtree:294-298 */
        pt_update(c, from, root, 0);
        break;
    case PSIM_MSG_PT_IHAVE:                       /* plumtree:299-303, :380-386 */
        if (pt_have(c, msg)) {
            pt_send(c, from, PSIM_MSG_PT_IGNORED_IHAVE, msg, rnd, root);
        } else {
            pt_send(c, from, PSIM_MSG_PT_GRAFT, msg, rnd, root);
            pt_update(c, from, root, 1);
        }
        break;
    case PSIM_MSG_PT_IGNORED_IHAVE:               /* plumtree:304-307 */
        pt_ack_out(c, from, msg, rnd);
        break;
    case PSIM_MSG_PT_GRAFT:                       /* plumtree:308-313, :388-402 */
        if (pt_have(c, msg)) {                    /* backend graft/1 :105-108, :153-159 */
            pt_update(c, from, root, 1);
            pt_send(c, from, PSIM_MSG_PT_BROADCAST, msg, rnd, root);
        }
        break;
    default:
        break;
    }
}

/* ------------------------------------------------------- hyparview -- */
static void hv_handle(ctx *c, const omsg *m) {
    struct psim_handle *h = c->h;
    node *s = c->s;
    uint32_t me = c->me;
    switch (m->type) {
    case PSIM_MSG_JOIN: {                         /* hyparview:703-771 */
        uint32_t p = m->src, pe = m->a0;
        if (addable_epoch(c, pe, p) && !list_member(s->act, s->act_n, p)) {
            if (maybe_connect(c, p)) {                /* :721-723 */
                add_to_active(c, p);
                hv_send(c, p, PSIM_MSG_NEIGHBOR, 0, current_id(c, p), 0, NULL, 0);
                uint32_t omit[2] = {me, p}, peers[PSIM_ACTIVE_CAP];
                uint32_t np = list_subtract(s->act, s->act_n, omit, 2, peers);
                for (uint32_t i = 0; i < np; i++)
                    if (is_xbot(h))                   /* xbot:765-786: the fold's connections are
                                                         dropped, State1 is kept */
                        xb_send(c, peers[i], PSIM_MSG_FORWARD_JOIN, h->cfg.arwl, p, pe, 0, 0);
                    else
                        hv_send(c, peers[i], PSIM_MSG_FORWARD_JOIN, h->cfg.arwl, p, pe, NULL, 0);
                notify(c);
            }
        }
        break;
    }
    case PSIM_MSG_NEIGHBOR: {                     /* hyparview:774-805 */
        uint32_t p = m->src;
        if (addable_id(c, m->a0, p) && maybe_connect(c, p)) add_to_active(c, p);   /* :784-786 */
        notify(c);
        break;
    }
    case PSIM_MSG_FORWARD_JOIN: {                 /* hyparview:808-923 */
        uint32_t p = m->a0, pe = m->a1, ttl = m->ttl, sender = m->src;
        if (ttl == 0 || s->act_n == 1) {
            if (addable_epoch(c, pe, p) && !list_member(s->act, s->act_n, p) && maybe_connect(c, p)) {
                add_to_active(c, p);
                hv_send(c, p, PSIM_MSG_NEIGHBOR, 0, current_id(c, p), 0, NULL, 0);
            }
        } else {
            uint32_t act0[PSIM_ACTIVE_CAP], n0 = s->act_n;
            memcpy(act0, s->act, sizeof act0);
            uint32_t pas0[PSIM_PASSIVE_CAP], np0 = s->pas_n;   /* State0's passive view */
            memcpy(pas0, s->pas, sizeof pas0);
            if (ttl == h->cfg.prwl) add_to_passive(c, p);   /* State2 (:859-866) */
            uint32_t omit[3] = {sender, me, p};
            uint32_t r = select_random(c, act0, n0, omit, 3);
            if (r == PSIM_NONE) {
                if (addable_epoch(c, pe, p) && !list_member(act0, n0, p)) {
                    if (maybe_connect(c, p)) {        /* :878-880 */
                        add_to_active(c, p);
                        hv_send(c, p, PSIM_MSG_NEIGHBOR, 0, current_id(c, p), 0, NULL, 0);
                    } else if (!is_xbot(h)) {
                        /* {error, not_found} -> State0 (:896-897): the passive
                         * insert is discarded; its eviction draw stays consumed
                         * (the rand state lives in the process dictionary).
                         * X-BOT keeps State2 (xbot:921-922) */
                        memcpy(s->pas, pas0, sizeof pas0);
                        s->pas_n = np0;
                    }
                }
            } else {
                hv_send(c, r, PSIM_MSG_FORWARD_JOIN, ttl - 1, p, pe, NULL, 0);
            }
        }
        notify(c);
        break;
    }
    case PSIM_MSG_DISCONNECT: {                   /* hyparview:926-972 */
        uint32_t p = m->src, d = m->a0;
        if (!valid_disconnect(c, p, d)) break;
        uint32_t pas0[PSIM_PASSIVE_CAP], np0 = s->pas_n;
        memcpy(pas0, s->pas, sizeof pas0);
        set_del(s->act, &s->act_n, p);
        conn_del(s, p | PSIM_CONN_DOWN);
        add_to_passive(c, p);
        map_store(c, s->recv_peer, s->recv_id, &s->recv_n, &s->recv_head, p, d);
        disconnect(c, p);                         /* :952 */
        if (s->act_n == 1) {
            uint32_t omit[2] = {me, p};
            move_to_active(c, select_random(c, pas0, np0, omit, 2));
        }
        break;
    }
    case PSIM_MSG_NEIGHBOR_REQUEST: {             /* hyparview:975-1053 */
        uint32_t p = m->src, d = m->a0;
        uint32_t ack[PSIM_EXCHANGE_CAP];
        int conn = maybe_connect(c, p);           /* :987, kept in both branches */
        uint32_t nack = build_exchange(c, ack);
        if (addable_id(c, d, p)) {               /* priority is always high (:1706) */
            if (conn || is_xbot(h)) {             /* X-BOT accepts without the find (xbot:1026-1045) */
                hv_send(c, p, PSIM_MSG_NEIGHBOR_ACCEPTED, 0, current_id(c, p), 0, ack, nack);
                add_to_active(c, p);
            }
        } else {
            hv_send(c, p, PSIM_MSG_NEIGHBOR_REJECTED, 0, 0, 0, ack, nack);
        }
        merge_exchange(c, m->ex, m->nex);
        notify(c);
        break;
    }
    case PSIM_MSG_NEIGHBOR_REJECTED:              /* hyparview:1056-1067 */
        disconnect(c, m->src);                    /* :1063 */
        merge_exchange(c, m->ex, m->nex);
        break;
    case PSIM_MSG_NEIGHBOR_ACCEPTED:              /* hyparview:1070-1089 */
        if (addable_id(c, m->a0, m->src)) add_to_active(c, m->src);
        merge_exchange(c, m->ex, m->nex);
        notify(c);
        break;
    case PSIM_MSG_SHUFFLE_REPLY:                  /* hyparview:1091-1093 */
        merge_exchange(c, m->ex, m->nex);
        break;
    case PSIM_MSG_SHUFFLE: {                      /* hyparview:1095-1136 */
        uint32_t ttl = m->ttl, sender = m->src;
        if (ttl > 0 && s->act_n > 1) {
            uint32_t omit[2] = {sender, me};
            uint32_t r = select_random(c, s->act, s->act_n, omit, 2);
            if (r != PSIM_NONE) hv_send(c, r, PSIM_MSG_SHUFFLE, ttl - 1, 0, 0, m->ex, m->nex);
        } else {
            uint32_t resp[PSIM_EXCHANGE_CAP];
            uint32_t nr = select_random_sublist(c, s->pas, s->pas_n, m->nex, resp);
            hv_send(c, sender, PSIM_MSG_SHUFFLE_REPLY, 0, 0, 0, resp, nr);
            merge_exchange(c, m->ex, m->nex);
        }
        break;
    }
    default:
        if (m->type >= PSIM_MSG_XBOT_OPTIMIZATION && is_xbot(h)) xb_handle(c, m);
        break;
    }
}

static int timer_due(uint32_t period, uint64_t r, uint32_t start) {
    return period > 0 && r > start && ((r - start) % period) == 0;
}

static void process_node(struct psim_handle *h, uint32_t n) {
    node *s = &h->nodes[n];
    ctx c = {h, s, n, 0, PSIM_NONE, 0, 0, 0, 0};
    uint64_t r = h->round;
    size_t b = h->in_beg[n], e = h->in_beg[n + 1];
    /* a fresh incarnation has no connections: traffic addressed to the
     * previous one is lost */
    if (s->start_round == r && e > b) { h->st->dropped += e - b; e = b; }
    int promo = h->cfg.random_promotion && timer_due(h->cfg.promotion_period, r, s->start_round);
    /* a due promotion timer is work only if it can act (hv:547-551) */
    int promo_work = promo && s->act_n < h->cfg.min_active_size;
    int shuf = timer_due(h->cfg.shuffle_period, r, s->start_round);
    int origin = h->origin[n] != 0 && h->cfg.plumtree;
    int lazy_due = h->cfg.plumtree && timer_due(h->cfg.lazy_tick_period, r, s->start_round);
    int lazy = lazy_due && s->out_n > 0;
    int xbot = is_xbot(h) && timer_due(h->cfg.xbot_period, r, s->start_round);
    /* X-BOT: the 'EXIT' of every connection pid a discarded do_disconnect
     * stopped last round (xbot:608-653), in table order */
    uint32_t closed[PSIM_CONN_CAP], nclosed = 0;
    for (uint32_t i = 0; i < s->conn_n; i++)
        if (s->conn[i] & PSIM_CONN_CLOSING) closed[nclosed++] = s->conn[i] & ~PSIM_CONN_CLOSING;
    /* EXIT at every holder of a connection to a peer that crashed this round
     * (App. A Q11): the connected active members in to_list order, then the
     * lingering peers in table order (their EXITs only edit the passive view
     * and the table) */
    uint32_t exits[PSIM_ACTIVE_CAP + PSIM_CONN_CAP], nexit = 0;
    for (uint32_t i = 0; i < s->act_n; i++)
        if (s->act[i] != n && h->crashed_now[s->act[i]] && conn_find(s, s->act[i] | PSIM_CONN_DOWN) < 0 &&
            !conn_closing(s, s->act[i]))
            exits[nexit++] = s->act[i];
    for (uint32_t i = 0; i < s->conn_n; i++)
        if (!(s->conn[i] & (PSIM_CONN_DOWN | PSIM_CONN_CLOSING)) && h->crashed_now[s->conn[i]])
            exits[nexit++] = s->conn[i];
    int joining = (s->start_round == r && s->join_contact != PSIM_NONE);
    if (!(e > b || joining || nexit || nclosed || promo_work || shuf || xbot || origin || lazy)) return;
    h->st->nodes_processed++;

    /* handle_cast({join, Peer}), hyparview:500-515 */
    if (joining) hv_send(&c, s->join_contact, PSIM_MSG_JOIN, 0, s->epoch, 0, NULL, 0);

    /* handle_info({'EXIT', ..}), hyparview:609-654: the connection is pruned,
     * the peer leaves the passive view, and the active view with a promotion */
    for (uint32_t i = 0; i < nclosed; i++) {       /* X-BOT: the stopped pids' EXITs first */
        uint32_t d = closed[i];
        h->st->exits++;
        conn_del(s, d | PSIM_CONN_CLOSING);
        if (list_member(s->pas, s->pas_n, d)) set_del(s->pas, &s->pas_n, d);
        if (list_member(s->act, s->act_n, d)) {
            set_del(s->act, &s->act_n, d);
            uint32_t omit[1] = {n};
            move_to_active(&c, select_random(&c, s->pas, s->pas_n, omit, 1));
        }
    }
    for (uint32_t i = 0; i < nexit; i++) {
        uint32_t d = exits[i];
        h->st->exits++;
        conn_del(s, d);
        if (list_member(s->pas, s->pas_n, d)) set_del(s->pas, &s->pas_n, d);
        if (list_member(s->act, s->act_n, d)) {
            set_del(s->act, &s->act_n, d);
            uint32_t omit[1] = {n};
            move_to_active(&c, select_random(&c, s->pas, s->pas_n, omit, 1));
        }
    }

    for (size_t i = b; i < e; i++)
        if (h->inbox.v[i].type < PSIM_MSG_PT_BROADCAST || h->inbox.v[i].type >= PSIM_MSG_XBOT_OPTIMIZATION) {
            h->st->delivered[h->inbox.v[i].type]++;
            hv_handle(&c, &h->inbox.v[i]);
        }

    if (promo && s->act_n < h->cfg.min_active_size) {   /* hyparview:542-561, :1718-1728 */
        uint32_t omit[1] = {n};
        move_to_active(&c, select_random(&c, s->pas, s->pas_n, omit, 1));
    }

    if (shuf) {                                          /* hyparview:572-607 */
        uint32_t ex[PSIM_EXCHANGE_CAP];
        uint32_t nex = build_exchange(&c, ex);
        uint32_t omit[1] = {n};
        uint32_t r2 = select_random(&c, s->act, s->act_n, omit, 1);
        if (r2 != PSIM_NONE) hv_send(&c, r2, PSIM_MSG_SHUFFLE, h->cfg.arwl, 0, 0, ex, nex);
    }

    if (xbot) xb_execute(&c);                     /* xbot:587-606 */

    if (!h->cfg.plumtree) return;
    for (size_t i = b; i < e; i++)
        if (h->inbox.v[i].type >= PSIM_MSG_PT_BROADCAST && h->inbox.v[i].type <= PSIM_MSG_PT_GRAFT) {
            h->st->delivered[h->inbox.v[i].type]++;
            pt_handle(&c, &h->inbox.v[i]);
        }

    if (origin) {                                  /* plumtree:282-287, backend:179-200 */
        uint32_t my = n | PSIM_MAP_BIT, msg = h->origin[n] - 1;
        s->have |= 1ull << (msg % PSIM_MSG_SLOTS);
        if (msg == h->tracked_msg) { s->trk_round = (uint32_t)r; s->trk_hop = 0; }
        pt_push(&c, msg, 0, my, my);
    }

    if (lazy_due) {                               /* plumtree:341-345, :443-453 */
        for (uint32_t i = 0; i < s->out_n; i++) {
            if (!pt_conn(&c, s->out_peer[i])) { h->st->send_fail++; continue; }
            emit(&c, s->out_peer[i] & ~PSIM_MAP_BIT, PSIM_MSG_PT_IHAVE, 0, s->out_msg[i], s->out_round[i],
                 msg_root(&c, s->out_msg[i]), NULL, 0);
        }
    }
}

/* ================================================== pluggable manager ==
 * partisan_pluggable_peer_service_manager driving one membership strategy
 * (round model R0-P):
 *   full      partisan_full_membership_strategy.erl   (ORSet of node_specs as
 *             an add bitset and a remove bitset: member = add & ~remove)
 *   scamp v1  partisan_scamp_v1_membership_strategy.erl
 *   scamp v2  partisan_scamp_v2_membership_strategy.erl
 * A join is internal_join/3 (pluggable:1423-1458): the joiner's client
 * connects and says hello, the contact's server answers with its
 * get_local_state/0 (peer_service_server:125-148), and the joiner's manager
 * runs Strategy:join/3 on {connected, ..} (pluggable:986-1044).  Strategy
 * messages go out through do_send_message/7 (pluggable:1309-1363). */

static int is_pl(const struct psim_handle *h) { return h->cfg.manager == PSIM_MANAGER_PLUGGABLE; }
static uint32_t *fb_row(struct psim_handle *h, uint32_t n) { return h->fbits + (size_t)n * 2 * h->W; }
/* word w of the member set of a [adds | removes] row */
static uint32_t fb_mem(const struct psim_handle *h, const uint32_t *b, uint32_t w) { return b[w] & ~b[h->W + w]; }

static uint32_t pl_member(ctx *c, uint32_t p) {
    struct psim_handle *h = c->h;
    if (h->cfg.strategy == PSIM_STRATEGY_FULL) return (fb_mem(h, fb_row(h, c->me), p >> 5) >> (p & 31u)) & 1u;
    snode *q = &h->sn[c->me];
    return (uint32_t)list_member(q->view, q->view_n, p);
}

static void pl_emit(ctx *c, uint32_t dst, uint32_t type, uint32_t a0, uint32_t slot) {
    emit(c, dst, type, 0, a0, 0, 0, NULL, 0);
    c->h->out.v[c->h->out.n - 1].slot = slot;
}

/* A strategy message to Peer: establish_connections/3 (pluggable:1096-1108)
 * keeps a connection to every member and pending node, so the send succeeds
 * iff Peer is one of them, runs and is not partitioned away; a successful
 * dispatch draws rand:uniform(1) (partisan_util:dispatch_pid/3 util:190-195). */
static int pair_in(const uint64_t *l, size_t n, uint32_t src, uint32_t dst) {
    uint64_t k = (uint64_t)src << 32 | dst;
    for (size_t i = 0; i < n; i++) if (l[i] == k) return 1;
    return 0;
}

/* the dict:fold of the interposition funs over a forwarded strategy message
 * (handle_cast({forward_message, ..}) pluggable:669-684): {send_omission, Dst}
 * (prop_partisan_crash_fault_model:166-177) and the `faulted` reader
 * (partisan_trace_orchestrator:623-637) turn it into `undefined` */
static int omit_send(ctx *c, uint32_t dst) {
    struct psim_handle *h = c->h;
    return h->flt.faulted[c->me] || pair_in(h->flt.send, h->flt.send_n, c->me, dst);
}

/* ... and over a received one (handle_cast({receive_message, ..}) :634-667):
 * {receive_omission, Src} (crash_fault_model:125-135), `faulted` (:638-650) */
static int omit_recv(ctx *c, uint32_t src) {
    struct psim_handle *h = c->h;
    return h->flt.faulted[c->me] || pair_in(h->flt.recv, h->flt.recv_n, src, c->me);
}

static int pl_send(ctx *c, uint32_t dst, uint32_t type, uint32_t a0, uint32_t slot) {
    /* forward_message's interposition fold runs first: an omitted message
     * is never looked up in the connections nor dispatched (pluggable:727-760) */
    if (omit_send(c, dst)) { c->h->st->omitted++; c->nomit_send++; return 0; }
    /* full: every target comes from the node's own member row, or is an old
     * member whose connection is still open (leave/1) */
    int full = c->h->cfg.strategy == PSIM_STRATEGY_FULL;
    if (!connect_ok(c, dst) || !(full || pl_member(c, dst) || dst == c->h->sn[c->me].pending)) {
        c->h->st->send_fail++;
        return 0;
    }
    (void)uniform_n(c, 1);
    pl_emit(c, dst, type, a0, slot);
    return 1;
}

/* --------------------------------------------------------------- full -- */
static uint32_t popcount32(uint32_t x) { return (uint32_t)__builtin_popcount(x); }

static uint32_t full_count(struct psim_handle *h, const uint32_t *b) {
    uint32_t k = 0;
    for (uint32_t w = 0; w < h->W; w++) k += popcount32(fb_mem(h, b, w));
    return k;
}

/* the k-th (0-based) member in id order */
static uint32_t full_nth(struct psim_handle *h, const uint32_t *b, uint32_t k) {
    for (uint32_t w = 0; w < h->W; w++) {
        uint32_t x = fb_mem(h, b, w), pc = popcount32(x);
        if (k < pc) {
            for (; k; k--) x &= x - 1;
            return w * 32 + (uint32_t)__builtin_ctz(x);
        }
        k -= pc;
    }
    return PSIM_NONE;
}

/* The Erlang message carries the state term of its moment: one snapshot per
 * distinct state a node gossips during the round. */
static uint32_t full_snapshot(ctx *c) {
    struct psim_handle *h = c->h;
    if (c->snap != PSIM_NONE && !c->dirty) return c->snap;
    if (h->pay_out_n == h->pay_out_cap) {
        h->pay_out_cap = h->pay_out_cap ? h->pay_out_cap * 2 : 64;
        h->pay_out = (uint32_t *)realloc(h->pay_out, h->pay_out_cap * 2 * h->W * sizeof(uint32_t));
    }
    memcpy(h->pay_out + h->pay_out_n * 2 * h->W, fb_row(h, c->me), 2 * h->W * sizeof(uint32_t));
    c->snap = (uint32_t)h->pay_out_n++;
    c->dirty = 0;
    return c->snap;
}

/* gossip_messages/1 (full:127-144): {membership_strategy, {Myself, State}} to
 * every member of membership_list/1 (fanout 0: the reference), or -- config
 * B's extension of the `fanout` key no strategy reads --
 * to `fanout` members, each drawn as rand:uniform(length(Members)).  The
 * whole list is built before the manager sends any of it.
 * With fanout > 0 the gossips a round owes (join, every non-equal merge,
 * periodic) are coalesced into one, sent after the node's inbox: the
 * reference's gossip-on-every-change multiplies the message count by the
 * fanout each round until the states agree. */
static void full_gossip(ctx *c) {
    struct psim_handle *h = c->h;
    const uint32_t *b = fb_row(h, c->me);
    uint32_t slot = full_snapshot(c), cnt = full_count(h, b);
    if (h->cfg.fanout == 0) {
        for (uint32_t w = 0; w < h->W; w++)
            for (uint32_t x = fb_mem(h, b, w); x; x &= x - 1)
                pl_send(c, w * 32 + (uint32_t)__builtin_ctz(x), PSIM_PL_GOSSIP, cnt, slot);
        return;
    }
    uint32_t tgt[PSIM_SVIEW_CAP];
    for (uint32_t i = 0; i < h->cfg.fanout; i++) tgt[i] = full_nth(h, b, uniform_n(c, cnt) - 1);
    for (uint32_t i = 0; i < h->cfg.fanout; i++) pl_send(c, tgt[i], PSIM_PL_GOSSIP, cnt, slot);
}

/* ?SET:merge/2 into the node's state; returns whether it was ?SET:equal/2 */
static int full_merge(ctx *c, const uint32_t *p) {
    struct psim_handle *h = c->h;
    uint32_t *b = fb_row(h, c->me);
    int equal = 1;
    for (uint32_t w = 0; w < 2 * h->W; w++) {     /* adds and removes */
        if (b[w] != p[w]) equal = 0;
        uint32_t m = b[w] | p[w];
        if (m != b[w]) { b[w] = m; c->dirty = 1; }
    }
    return equal;
}

/* -------------------------------------------------------------- scamp -- */
/* select_random_sublist/2 + shuffle/1 (scamp_v1:263-269, scamp_v2:345-350) */
static uint32_t sublist_view(ctx *c, const uint32_t *view, uint32_t n, uint32_t k, uint32_t *out) {
    uint64_t key[PSIM_SVIEW_CAP];
    uint32_t el[PSIM_SVIEW_CAP];
    for (uint32_t i = 0; i < n; i++) { key[i] = uniform_key(c); el[i] = view[i]; }
    for (uint32_t i = 1; i < n; i++) {
        uint64_t kk = key[i]; uint32_t ee = el[i]; int j = (int)i - 1;
        while (j >= 0 && (key[j] > kk || (key[j] == kk && el[j] > ee))) {
            key[j + 1] = key[j]; el[j + 1] = el[j]; j--;
        }
        key[j + 1] = kk; el[j + 1] = ee;
    }
    uint32_t m = n < k ? n : k;
    for (uint32_t i = 0; i < m; i++) out[i] = el[i];
    return m;
}

/* random_0_or_1/0 (scamp_v1:272-279): rand:uniform(10) >= 5 */
static uint32_t random_0_or_1(ctx *c) { return uniform_n(c, 10) >= 5 ? 1u : 0u; }

/* sets:add_element/2 (v1) or [Node | List] (v2) into a fixed table */
static void scamp_add(ctx *c, uint32_t *l, uint32_t *n, uint32_t e, int as_set) {
    if (as_set && list_member(l, *n, e)) return;
    if (*n >= PSIM_SVIEW_CAP) { ovf(c, PSIM_OVF_STRATEGY); return; }
    if (as_set) { set_add(c->h, l, n, e, &c->h->sn[c->me].view_slots); return; }
    for (uint32_t i = *n; i > 0; i--) l[i] = l[i - 1];
    l[0] = e;
    (*n)++;
}

/* Strategy:join/3 at the joiner (scamp_v1:52-99, scamp_v2:64-113): add the
 * contact; forward_subscription(Myself) to it, forward_subscription(Contact)
 * to every member known before (v1: sets:fold/3, the reverse of to_list;
 * v2: lists:foldl/3) and to C (v1) / C - 1 (v2) random ones of them. */
static void scamp_join(ctx *c, uint32_t contact) {
    snode *q = &c->h->sn[c->me];
    int v1 = c->h->cfg.strategy == PSIM_STRATEGY_SCAMP_V1;
    uint32_t m0[PSIM_SVIEW_CAP], n0 = q->view_n;
    memcpy(m0, q->view, sizeof m0);
    scamp_add(c, q->view, &q->view_n, contact, v1);
    uint32_t dst[1 + 2 * PSIM_SVIEW_CAP], arg[1 + 2 * PSIM_SVIEW_CAP], k = 0;
    dst[k] = contact; arg[k++] = c->me;
    for (uint32_t i = 0; i < n0; i++) { dst[k] = m0[v1 ? n0 - 1 - i : i]; arg[k++] = contact; }
    uint32_t sel[PSIM_SVIEW_CAP];
    uint32_t ns = sublist_view(c, m0, n0, v1 ? c->h->cfg.scamp_c : c->h->cfg.scamp_c - 1, sel);
    for (uint32_t i = 0; i < ns; i++) { dst[k] = sel[i]; arg[k++] = contact; }
    for (uint32_t i = 0; i < k; i++) pl_send(c, dst[i], PSIM_PL_FWD_SUB, arg[i], PSIM_NONE);
}

/* periodic/1 (scamp_v1:125-174, scamp_v2:130-178): "isolated" when a ping
 * was ever received and the last one is older than
 * ?PERIODIC_INTERVAL * ?SCAMP_MESSAGE_WINDOW = 100000 us (App. A Q12: in
 * rounds of 1 s, any earlier round) -> forward_subscription(Myself) to one
 * random member; then a ping to every member. */
static void scamp_periodic(ctx *c) {
    snode *q = &c->h->sn[c->me];
    uint32_t m[PSIM_SVIEW_CAP], n = q->view_n;
    memcpy(m, q->view, sizeof m);
    int isolated = q->last_ping != PSIM_NONE && (uint32_t)c->h->round > q->last_ping;
    uint32_t sel[1], ns = 0;
    if (isolated) ns = sublist_view(c, m, n, 1, sel);
    for (uint32_t i = 0; i < ns; i++) pl_send(c, sel[i], PSIM_PL_FWD_SUB, c->me, PSIM_NONE);
    for (uint32_t i = 0; i < n; i++) pl_send(c, m[i], PSIM_PL_PING, c->me, PSIM_NONE);
}

/* handle_message(.., {forward_subscription, Node}) (scamp_v1:212-252,
 * scamp_v2:284-327): Keep = trunc((size + 1) * random_0_or_1()), so the
 * subscription is kept iff the draw is 0 and Node is not a member yet (v2
 * then asks Node to keep us); otherwise it is forwarded to one random member */
static void scamp_fwd(ctx *c, uint32_t node) {
    snode *q = &c->h->sn[c->me];
    int v1 = c->h->cfg.strategy == PSIM_STRATEGY_SCAMP_V1;
    uint32_t rnd = random_0_or_1(c);
    if (rnd == 0 && !list_member(q->view, q->view_n, node)) {
        scamp_add(c, q->view, &q->view_n, node, v1);
        if (!v1) pl_send(c, node, PSIM_PL_KEEP_SUB, c->me, PSIM_NONE);
        return;
    }
    uint32_t sel[1];
    uint32_t m0[PSIM_SVIEW_CAP];
    memcpy(m0, q->view, sizeof m0);
    if (sublist_view(c, m0, q->view_n, 1, sel)) pl_send(c, sel[0], PSIM_PL_FWD_SUB, node, PSIM_NONE);
}

/* leave/1 at the actor, Node = t (handle_call({leave, Node}) pluggable:502-515
 * -> internal_leave/2 :1390-1420, not the actor itself):
 *   v1 leave/2 (scamp_v1:102-122): delete t from the membership, then
 *      {remove_subscription, t} to every member of the old list (to_list order);
 *   v2 leave/2 (scamp_v2:116-127): {bootstrap_remove_subscription, t} to every
 *      member of the partial view, no state change. */
static void scamp_leave(ctx *c, uint32_t t) {
    snode *q = &c->h->sn[c->me];
    uint32_t m0[PSIM_SVIEW_CAP], n0 = q->view_n;
    memcpy(m0, q->view, sizeof m0);
    int v1 = c->h->cfg.strategy == PSIM_STRATEGY_SCAMP_V1;
    /* the connections to the old members stay open (they close only on
     * 'EXIT', pluggable:971-984), so the sends are judged on the old view */
    for (uint32_t i = 0; i < n0; i++)
        pl_send(c, m0[i], v1 ? PSIM_PL_REMOVE_SUB : PSIM_PL_BOOT_REMOVE, t, PSIM_NONE);
    if (v1) set_del_slots(c->h, q->view, &q->view_n, t, &q->view_slots);   /* sets:del_element/2 (sv1:111) */
}

/* leave/1 of the full strategy at the actor, NameToRemove = t (full:58-89):
 * ?SET:mutate({rmv, N}) of t's spec if it is a member (its add is
 * tombstoned), then gossip_messages(State0, StateToGossip): the new state to
 * every member of the OLD list (t included).  fanout > 0 (config B's
 * extension): the coalesced gossip of the round instead. */
static void full_leave(ctx *c, uint32_t t) {
    struct psim_handle *h = c->h;
    uint32_t *b = fb_row(h, c->me);
    uint32_t was = (fb_mem(h, b, t >> 5) >> (t & 31u)) & 1u;
    if (was) { b[h->W + (t >> 5)] |= 1u << (t & 31u); c->dirty = 1; }
    if (h->cfg.fanout) { c->gossip_due = 1; return; }
    uint32_t slot = full_snapshot(c), cnt = full_count(h, b);
    for (uint32_t w = 0; w < h->W; w++) {
        uint32_t x = fb_mem(h, b, w);
        if (was && w == (t >> 5)) x |= 1u << (t & 31u);
        for (; x; x &= x - 1) pl_send(c, w * 32 + (uint32_t)__builtin_ctz(x), PSIM_PL_GOSSIP, cnt, slot);
    }
}

/* ------------------------------------------------------------- driver -- */
static void pl_handle(ctx *c, const omsg *m) {
    struct psim_handle *h = c->h;
    snode *q = &h->sn[c->me];
    int full = h->cfg.strategy == PSIM_STRATEGY_FULL;
    switch (m->type) {
    case PSIM_PL_HELLO:       /* the server's answer: {state, Tag, get_local_state()} */
        if (!connect_ok(c, m->src)) { h->st->send_fail++; break; }
        if (full) pl_emit(c, m->src, PSIM_PL_STATE, full_count(h, fb_row(h, c->me)), full_snapshot(c));
        else pl_emit(c, m->src, PSIM_PL_STATE, 0, PSIM_NONE);
        break;
    case PSIM_PL_STATE:       /* handle_info({connected, Node, _, RemoteState}) pluggable:986-1044 */
        if (q->pending != m->src) break;
        q->pending = PSIM_NONE;
        if (full) {           /* join/3 full:49-55: merge, then gossip */
            full_merge(c, h->pay_in + (size_t)m->slot * 2 * h->W);
            if (h->cfg.fanout) c->gossip_due = 1;
            else full_gossip(c);
        } else {
            scamp_join(c, m->src);
        }
        break;
    case PSIM_PL_GOSSIP:      /* handle_message/2 full:99-116 */
        if (!full) break;
        if (!full_merge(c, h->pay_in + (size_t)m->slot * 2 * h->W)) {
            /* a merged removal of ourselves: the manager stops
               (pluggable:1182-1188) before the gossip it cast goes out */
            if (!pl_member(c, c->me)) { c->stop = 1; break; }
            if (h->cfg.fanout) c->gossip_due = 1;
            else full_gossip(c);
        }
        break;
    case PSIM_PL_FWD_SUB:
        if (!full) scamp_fwd(c, m->a0);
        break;
    case PSIM_PL_PING:        /* scamp_v1:177-188, scamp_v2:181-191 */
        if (!full) q->last_ping = (uint32_t)h->round;
        break;
    case PSIM_PL_KEEP_SUB:    /* scamp_v2:328-338: InView = [Node | InView0] */
        if (h->cfg.strategy == PSIM_STRATEGY_SCAMP_V2) scamp_add(c, q->inv, &q->inv_n, m->a0, 0);
        break;
    case PSIM_PL_REMOVE_SUB:  /* scamp_v1:190-211: a member Node reaches
                                 sets:del_element(Membership0, Node) with its
                                 arguments swapped (App. A Q12): the manager crashes */
        if (h->cfg.strategy == PSIM_STRATEGY_SCAMP_V1 && list_member(q->view, q->view_n, m->a0)) c->stop = 1;
        break;
    case PSIM_PL_BOOT_REMOVE: /* scamp_v2:192-238: at Node itself every branch
                                 stops the manager before its casts go out --
                                 lists:nth(0, ..) (App. A Q12), or the reset
                                 partial view leaves it out of its own membership
                                 (pluggable:1182-1188) */
        if (h->cfg.strategy == PSIM_STRATEGY_SCAMP_V2 && m->a0 == c->me) c->stop = 1;
        break;
    default:
        break;
    }
}

int orc_crash(struct psim_handle *h, const uint32_t *nodes, size_t n);

static void pl_process_node(struct psim_handle *h, uint32_t n) {
    node *s = &h->nodes[n];
    snode *q = &h->sn[n];
    ctx c = {h, s, n, 0, PSIM_NONE, 0, 0, 0, 0};
    uint64_t r = h->round;
    size_t b = h->in_beg[n], e = h->in_beg[n + 1];
    if (s->start_round == r && e > b) { h->st->dropped += e - b; e = b; }
    int hello = q->pending != PSIM_NONE && !q->hello_sent;
    int periodic = timer_due(h->cfg.periodic_interval, r, s->start_round);
    uint32_t leave = q->leave_tgt;
    if (!(e > b || hello || periodic || leave)) return;
    h->st->nodes_processed++;
    /* a manager that stops this round sends nothing: its sends are casts to
     * itself (schedule_self_message_delivery/6 pluggable:1585-1609) */
    size_t out0 = h->out.n;
    uint64_t em0[PSIM_MSG_NTYPES], dig0 = h->st->digest, fail0 = h->st->send_fail;
    memcpy(em0, h->st->emitted, sizeof em0);
    if (leave) {              /* leave/1 (pluggable:502-515, :1390-1420) */
        q->leave_tgt = 0;
        if (h->cfg.strategy == PSIM_STRATEGY_FULL) full_leave(&c, leave - 1);
        else scamp_leave(&c, leave - 1);
    }
    if (hello) {              /* establish_connections -> client connect + hello */
        if (connect_ok(&c, q->pending)) { pl_emit(&c, q->pending, PSIM_PL_HELLO, 0, PSIM_NONE); q->hello_sent = 1; }
        else h->st->send_fail++;
    }
    for (size_t i = b; i < e && !c.stop; i++) {
        /* strategy messages pass the receive interposition; hello / state
         * are the client and server processes' */
        if (h->inbox.v[i].type >= PSIM_PL_GOSSIP && omit_recv(&c, h->inbox.v[i].src)) {
            h->st->omitted++;
            continue;
        }
        h->st->delivered[h->inbox.v[i].type]++;
        pl_handle(&c, &h->inbox.v[i]);
        if (c.stop) h->st->dropped += e - i - 1;
    }
    if (c.stop) {             /* down from the next round, as a crash */
        h->out.n = out0;
        memcpy(h->st->emitted, em0, sizeof em0);
        h->st->digest = dig0; h->st->send_fail = fail0;
        /* the receive-side omissions of the inbox before the stop stand;
         * the send-side ones were casts to itself that never ran */
        h->st->omitted -= c.nomit_send;
        orc_crash(h, &n, 1);
        return;
    }
    if (periodic) {           /* handle_info(periodic) pluggable:881-903 */
        if (h->cfg.strategy == PSIM_STRATEGY_FULL) c.gossip_due = 1;
        else scamp_periodic(&c);
    }
    if (c.gossip_due) full_gossip(&c);
}

static void pl_node_init(struct psim_handle *h, uint32_t n, uint32_t contact) {
    snode *q = &h->sn[n];
    memset(q, 0, sizeof *q);
    q->started = 1;
    q->pending = contact;
    q->last_ping = PSIM_NONE;
    q->view[0] = n; q->view_n = 1;               /* init/1: Myself only */
    q->view_slots = 16;                          /* sets:new/0 */
    if (h->cfg.strategy == PSIM_STRATEGY_FULL) {
        q->view_n = 0; q->view[0] = 0;
        uint32_t *b = fb_row(h, n);
        memset(b, 0, 2 * h->W * sizeof(uint32_t));
        b[n >> 5] |= 1u << (n & 31u);            /* new_state/1 full:171-175 */
    }
}

/* ---------------------------------------------------------- rounds -- */
static void node_init(struct psim_handle *h, uint32_t n, uint32_t contact) {
    node *s = &h->nodes[n];
    uint32_t ep = h->cfg.persist_epoch ? s->epoch + 1 : 1;
    memset(s, 0, sizeof *s);
    s->up = 1;
    s->epoch = ep;
    s->start_round = (uint32_t)h->round;
    s->join_contact = contact;
    s->act[0] = n; s->act_n = 1;                 /* sets:add_element(Myself, ..) :299 */
    s->pt_all[0] = n; s->pt_all_n = 1;           /* plumtree start_link/0 :127-144 */
    s->pt_common[0] = n; s->pt_common_n = 1;
    for (int k = 0; k < PSIM_PT_ROOTS; k++) s->rt_root[k] = PSIM_NONE;
    s->trk_round = PSIM_NONE;
    if (is_pl(h)) pl_node_init(h, n, contact);
}

static int cmp_dst(const void *a, const void *b) {
    const omsg *x = (const omsg *)a, *y = (const omsg *)b;
    if (x->dst != y->dst) return x->dst < y->dst ? -1 : 1;
    if (x->src != y->src) return x->src < y->src ? -1 : 1;
    return x->seq < y->seq ? -1 : x->seq > y->seq;
}

/* Round, first half: events (applied to every node: up/partition state is
 * replicated on every shard) and the handlers of the owned nodes; the
 * round's emissions are left in h->out in (src, seq) order. */
static void round_begin(struct psim_handle *h, psim_round_stats *st) {
    memset(st, 0, sizeof *st);
    st->round = h->round;
    h->st = st;
    for (size_t i = 0; i < h->pend_crash_n; i++) {
        uint32_t n = h->pend_crash[i];
        if (h->nodes[n].up) { h->nodes[n].up = 0; h->crashed_now[n] = 1; }
    }
    for (size_t i = 0; i < h->pend_join_n; i++) {
        node_init(h, h->pend_join[i], h->pend_contact[i]);
        h->pend_join_mark[h->pend_join[i]] = 0;
    }
    for (size_t i = 0; i < h->pend_lv_n; i++) h->sn[h->pend_lv_a[i]].leave_tgt = h->pend_lv_t[i] + 1;
    h->pend_lv_n = 0;
    if (h->pend_part_clear) memset(h->part, 0, h->N);
    if (h->pend_part_set) memcpy(h->part, h->pend_part, h->N);
    if (h->faults_dirty) {          /* interposition funs installed / removed */
        memcpy(h->flt.faulted, h->nx.faulted, h->N);
        h->flt.send = (uint64_t *)realloc(h->flt.send, (h->nx.send_n + 1) * 8);
        h->flt.recv = (uint64_t *)realloc(h->flt.recv, (h->nx.recv_n + 1) * 8);
        if (h->nx.send_n) memcpy(h->flt.send, h->nx.send, h->nx.send_n * 8);
        if (h->nx.recv_n) memcpy(h->flt.recv, h->nx.recv, h->nx.recv_n * 8);
        h->flt.send_n = h->nx.send_n; h->flt.recv_n = h->nx.recv_n;
        h->faults_dirty = 0;
    }
    /* broadcasts: each takes its message slot (the slot's previous id is
     * retired: its delivery bit cleared everywhere) and is originated this
     * round at its root if the root runs; the last one is the tracked one */
    for (uint32_t n = 0; n < h->N; n++) h->origin[n] = 0;
    if (h->pend_b_n) {
        uint64_t clear = 0;
        for (uint32_t i = 0; i < h->pend_b_n; i++) {
            uint32_t k = h->pend_b_msg[i] % PSIM_MSG_SLOTS;
            clear |= 1ull << k;
            h->slot_msg[k] = h->pend_b_msg[i];
            h->slot_root[k] = h->pend_b_root[i] | PSIM_MAP_BIT;
            if (h->nodes[h->pend_b_root[i]].up) h->origin[h->pend_b_root[i]] = h->pend_b_msg[i] + 1;
        }
        h->tracked_msg = h->pend_b_msg[h->pend_b_n - 1];
        for (uint32_t n = 0; n < h->N; n++) {
            h->nodes[n].have &= ~clear;
            h->nodes[n].trk_round = PSIM_NONE;
            h->nodes[n].trk_hop = 0;
        }
    }
    h->pend_crash_n = h->pend_join_n = 0;
    h->pend_part_set = h->pend_part_clear = 0;
    h->pend_b_n = 0;

    h->out.n = 0;
    for (uint32_t n = h->lo; n < h->hi; n++) {
        if (h->nodes[n].up) {
            st->nodes_up++;
            if (is_pl(h)) pl_process_node(h, n);
            else process_node(h, n);
        } else {
            st->dropped += h->in_beg[n + 1] - h->in_beg[n];
        }
    }
    memset(h->crashed_now, 0, h->N);
}

/* Round, second half: the messages addressed to the owned nodes (from every
 * shard) become the canonical inbox of round r+1, sorted by (dst, src, seq). */
static void round_end(struct psim_handle *h, msgvec *in) {
    qsort(in->v, in->n, sizeof(omsg), cmp_dst);
    if (h->fbits) {                 /* this round's snapshots are read next round */
        uint32_t *t = h->pay_in; h->pay_in = h->pay_out; h->pay_out = t;
        size_t tc = h->pay_in_cap; h->pay_in_cap = h->pay_out_cap; h->pay_out_cap = tc;
        h->pay_out_n = 0;
    }
    if (in != &h->inbox) {
        msgvec t = h->inbox; h->inbox = *in; *in = t;
    }
    size_t j = 0;
    for (uint32_t n = 0; n <= h->N; n++) {
        while (j < h->inbox.n && h->inbox.v[j].dst < n) j++;
        h->in_beg[n] = j;
    }
    h->round++;
}

static void run_round(struct psim_handle *h, psim_round_stats *st) {
    round_begin(h, st);
    round_end(h, &h->out);
}

/* ------------------------------------------------------------- ABI -- */
void orc_default_config(psim_config *cfg) {
    memset(cfg, 0, sizeof *cfg);
    cfg->abi_version = PSIM_ABI_VERSION;
    cfg->n_nodes = 32;
    cfg->seed = 1;
    cfg->max_active_size = 6; cfg->min_active_size = 3; cfg->max_passive_size = 30;
    cfg->arwl = 5; cfg->prwl = 30; cfg->k_active = 3; cfg->k_passive = 4;
    cfg->shuffle_period = 10; cfg->promotion_period = 5; cfg->random_promotion = 1;
    cfg->persist_epoch = 0; cfg->plumtree = 1; cfg->lazy_tick_period = 1;
    cfg->device = -1; cfg->n_shards = 1; cfg->shard_world = 1;
    cfg->manager = PSIM_MANAGER_HYPARVIEW; cfg->strategy = PSIM_STRATEGY_FULL;
    cfg->periodic_interval = 10; cfg->scamp_c = 5; cfg->fanout = 0;
    cfg->xbot_period = 35;
}

int orc_create(const psim_config *cfg, struct psim_handle **out) {
    if (!cfg || !out || cfg->abi_version != PSIM_ABI_VERSION || cfg->n_nodes == 0 ||
        cfg->n_nodes >= PSIM_MAP_BIT || cfg->max_active_size < 2 ||
        cfg->max_active_size > PSIM_ACTIVE_CAP || cfg->max_passive_size < 1 ||
        cfg->max_passive_size > 30 || 1 + cfg->k_active + cfg->k_passive > PSIM_EXCHANGE_CAP ||
        cfg->arwl > 255 || cfg->prwl > 255 || cfg->manager > PSIM_MANAGER_XBOT ||
        cfg->strategy > PSIM_STRATEGY_SCAMP_V2 || cfg->scamp_c < 1 || cfg->scamp_c > 64 ||
        cfg->fanout > 64 || cfg->strict > 1)
        return PSIM_EINVAL;
    int full = cfg->manager == PSIM_MANAGER_PLUGGABLE && cfg->strategy == PSIM_STRATEGY_FULL;
    if (full && cfg->shard_world > 1) return PSIM_EUNSUPPORTED;   /* payloads are shard-local */
    struct psim_handle *h = (struct psim_handle *)calloc(1, sizeof *h);
    if (!h) return PSIM_ENOMEM;
    h->cfg = *cfg;
    h->N = cfg->n_nodes;
    h->lo = 0; h->hi = h->N;
    if (cfg->shard_world > 1) {
        if (cfg->shard_rank >= cfg->shard_world || cfg->shard_world > h->N) { free(h); return PSIM_EINVAL; }
        uint32_t per = (h->N + cfg->shard_world - 1) / cfg->shard_world;
        h->lo = cfg->shard_rank * per < h->N ? cfg->shard_rank * per : h->N;
        h->hi = h->lo + per < h->N ? h->lo + per : h->N;
    }
    h->nodes = (node *)calloc(h->N, sizeof(node));
    h->part = (uint8_t *)calloc(h->N, 1);
    h->crashed_now = (uint8_t *)calloc(h->N, 1);
    h->in_beg = (size_t *)calloc((size_t)h->N + 1, sizeof(size_t));
    h->pend_part = (uint8_t *)calloc(h->N, 1);
    if (!h->nodes || !h->part || !h->crashed_now || !h->in_beg || !h->pend_part) return PSIM_ENOMEM;
    if (cfg->manager == PSIM_MANAGER_PLUGGABLE) {
        h->sn = (snode *)calloc(h->N, sizeof(snode));
        if (!h->sn) return PSIM_ENOMEM;
        if (full) {
            h->W = (h->N + 31) / 32;
            h->fbits = (uint32_t *)calloc((size_t)h->N * 2 * h->W, sizeof(uint32_t));
            if (!h->fbits) return PSIM_ENOMEM;
        }
    }
    h->origin = (uint32_t *)calloc(h->N, sizeof(uint32_t));
    h->flt.faulted = (uint8_t *)calloc(h->N, 1);
    h->nx.faulted = (uint8_t *)calloc(h->N, 1);
    if (!h->origin || !h->flt.faulted || !h->nx.faulted) return PSIM_ENOMEM;
    for (int k = 0; k < PSIM_MSG_SLOTS; k++) h->slot_msg[k] = h->slot_root[k] = PSIM_NONE;
    h->tracked_msg = PSIM_NONE;
    *out = h;
    return PSIM_OK;
}

void orc_destroy(struct psim_handle *h) {
    if (!h) return;
    free(h->nodes); free(h->part); free(h->crashed_now); free(h->in_beg); free(h->pend_part);
    free(h->inbox.v); free(h->out.v);
    free(h->pend_crash); free(h->pend_join); free(h->pend_contact); free(h->pend_join_mark); free(h->origin);
    free(h->pend_lv_a); free(h->pend_lv_t);
    free(h->sn); free(h->fbits); free(h->pay_in); free(h->pay_out);
    free(h->flt.send); free(h->flt.recv); free(h->flt.faulted);
    free(h->nx.send); free(h->nx.recv); free(h->nx.faulted);
    free(h->btab);
    free(h);
}

int orc_join(struct psim_handle *h, const uint32_t *nodes, const uint32_t *contacts, size_t n) {
    for (size_t i = 0; i < n; i++)
        if (nodes[i] >= h->N || (contacts[i] != PSIM_NONE && contacts[i] >= h->N)) return PSIM_ERANGE;
    if (!h->pend_join_mark && !(h->pend_join_mark = (uint8_t *)calloc(h->N, 1))) return PSIM_ENOMEM;
    for (size_t i = 0; i < n; i++) {
        if (h->pend_join_mark[nodes[i]]) {          /* a second start of the node this round */
            for (size_t j = 0; j < i; j++) h->pend_join_mark[nodes[j]] = 0;
            return PSIM_EINVAL;
        }
        h->pend_join_mark[nodes[i]] = 1;
    }
    if (h->fbits) {                 /* an ORSet re-add would need per-incarnation tokens */
        for (size_t i = 0; i < n; i++)
            if (h->sn[nodes[i]].started) {
                for (size_t j = 0; j < n; j++) h->pend_join_mark[nodes[j]] = 0;
                return PSIM_EUNSUPPORTED;
            }
        for (size_t i = 0; i < n; i++) h->sn[nodes[i]].started = 1;
    }
    if (h->pend_join_n + n > h->pend_join_cap) {
        h->pend_join_cap = (h->pend_join_n + n) * 2;
        h->pend_join = (uint32_t *)realloc(h->pend_join, h->pend_join_cap * 4);
        h->pend_contact = (uint32_t *)realloc(h->pend_contact, h->pend_join_cap * 4);
    }
    for (size_t i = 0; i < n; i++) {
        h->pend_join[h->pend_join_n] = nodes[i];
        h->pend_contact[h->pend_join_n++] = contacts[i];
    }
    return PSIM_OK;
}

/* psim_revive: a restart without a join (psim_join with no contact) */
int orc_revive(struct psim_handle *h, const uint32_t *nodes, size_t n) {
    uint32_t *none = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
    if (!none) return PSIM_ENOMEM;
    for (size_t i = 0; i < n; i++) none[i] = PSIM_NONE;
    int rc = orc_join(h, nodes, none, n);
    free(none);
    return rc;
}

int orc_crash(struct psim_handle *h, const uint32_t *nodes, size_t n) {
    for (size_t i = 0; i < n; i++)
        if (nodes[i] >= h->N) return PSIM_ERANGE;
    if (h->pend_crash_n + n > h->pend_crash_cap) {
        h->pend_crash_cap = (h->pend_crash_n + n) * 2;
        h->pend_crash = (uint32_t *)realloc(h->pend_crash, h->pend_crash_cap * 4);
    }
    for (size_t i = 0; i < n; i++) h->pend_crash[h->pend_crash_n++] = nodes[i];
    return PSIM_OK;
}

/* psim_leave: leave/0 under the pluggable manager stops the manager before
 * the Strategy:leave/2 messages it cast to itself go out
 * (pluggable:502-515, :1390-1420, :1585-1609) -- a crash; the HyParView
 * manager answers `error` (hyparview:363-364). */
int orc_leave(struct psim_handle *h, const uint32_t *nodes, size_t n) {
    if (!is_pl(h)) return PSIM_EUNSUPPORTED;
    return orc_crash(h, nodes, n);
}

/* psim_leave_node: leave/1 -- actors[i] removes targets[i]
 * (handle_call({leave, Node}) pluggable:502-515).  actor == target is
 * leave/0.  One call per actor and round; unsharded handles only (a stop is
 * known on its own shard). */
int orc_leave_node(struct psim_handle *h, const uint32_t *actors, const uint32_t *targets, size_t n) {
    if (!is_pl(h) || h->lo != 0 || h->hi != h->N) return PSIM_EUNSUPPORTED;
    for (size_t i = 0; i < n; i++) {
        if (actors[i] >= h->N || targets[i] >= h->N) return PSIM_ERANGE;
        for (size_t j = 0; j < h->pend_lv_n; j++) if (h->pend_lv_a[j] == actors[i]) return PSIM_EINVAL;
        for (size_t j = 0; j < i; j++) if (actors[j] == actors[i]) return PSIM_EINVAL;
    }
    for (size_t i = 0; i < n; i++) {
        if (actors[i] == targets[i]) {
            int rc = orc_crash(h, &actors[i], 1);
            if (rc) return rc;
            continue;
        }
        if (h->pend_lv_n == h->pend_lv_cap) {
            h->pend_lv_cap = h->pend_lv_cap ? 2 * h->pend_lv_cap : 64;
            h->pend_lv_a = (uint32_t *)realloc(h->pend_lv_a, h->pend_lv_cap * 4);
            h->pend_lv_t = (uint32_t *)realloc(h->pend_lv_t, h->pend_lv_cap * 4);
        }
        h->pend_lv_a[h->pend_lv_n] = actors[i];
        h->pend_lv_t[h->pend_lv_n++] = targets[i];
    }
    return PSIM_OK;
}

int orc_set_partition(struct psim_handle *h, const uint8_t *group, size_t n) {
    if (n != h->N) return PSIM_EINVAL;
    for (size_t i = 0; i < n; i++)
        if (group[i] > PSIM_PARTITION_MAX) return PSIM_EINVAL;
    memcpy(h->pend_part, group, n);
    h->pend_part_set = 1; h->pend_part_clear = 0;
    return PSIM_OK;
}

int orc_clear_partition(struct psim_handle *h) {
    h->pend_part_clear = 1; h->pend_part_set = 0;
    return PSIM_OK;
}

/* psim_set_omission: add_interposition_fun / remove_interposition_fun of
 * {send_omission, Dst} at Src or {receive_omission, Src} at Dst
 * (pluggable:297-310; prop_partisan_crash_fault_model:117-196).  The funs
 * are a dict keyed by name: a pair is installed at most once. */
int orc_set_omission(struct psim_handle *h, int kind, const uint32_t *src, const uint32_t *dst, size_t n, int on) {
    if (!is_pl(h)) return PSIM_EUNSUPPORTED;      /* the HyParView manager has no interposition */
    if (kind != PSIM_OMIT_SEND && kind != PSIM_OMIT_RECEIVE) return PSIM_EINVAL;
    for (size_t i = 0; i < n; i++) if (src[i] >= h->N || dst[i] >= h->N) return PSIM_ERANGE;
    uint64_t **l = kind == PSIM_OMIT_SEND ? &h->nx.send : &h->nx.recv;
    size_t *ln = kind == PSIM_OMIT_SEND ? &h->nx.send_n : &h->nx.recv_n;
    for (size_t i = 0; i < n; i++) {
        uint64_t k = (uint64_t)src[i] << 32 | dst[i];
        size_t j = 0;
        while (j < *ln && (*l)[j] != k) j++;
        if (on && j == *ln) {
            *l = (uint64_t *)realloc(*l, (*ln + 1) * 8);
            (*l)[(*ln)++] = k;
        } else if (!on && j < *ln) {
            (*l)[j] = (*l)[--(*ln)];
        }
    }
    h->faults_dirty = 1;
    return PSIM_OK;
}

/* psim_set_faulted: begin_omission / end_omission (crash_fault_model:93-114) */
int orc_set_faulted(struct psim_handle *h, const uint32_t *nodes, size_t n, int on) {
    if (!is_pl(h)) return PSIM_EUNSUPPORTED;
    for (size_t i = 0; i < n; i++) if (nodes[i] >= h->N) return PSIM_ERANGE;
    for (size_t i = 0; i < n; i++) h->nx.faulted[nodes[i]] = on ? 1 : 0;
    h->faults_dirty = 1;
    return PSIM_OK;
}

/* psim_clear_faults: resolve_all_faults_with_heal (crash_fault_model:198-229) */
int orc_clear_faults(struct psim_handle *h) {
    if (!is_pl(h)) return PSIM_EUNSUPPORTED;
    h->nx.send_n = h->nx.recv_n = 0;
    memset(h->nx.faulted, 0, h->N);
    h->faults_dirty = 1;
    return PSIM_OK;
}

int orc_broadcast(struct psim_handle *h, uint32_t root, uint32_t msg_id) {
    if (is_pl(h)) return PSIM_EUNSUPPORTED;      /* Plumtree runs over the HyParView manager */
    if (root >= h->N || msg_id > 0xFFFF) return PSIM_ERANGE;
    for (uint32_t i = 0; i < h->pend_b_n; i++)    /* one per root and per slot per round */
        if (h->pend_b_root[i] == root || h->pend_b_msg[i] % PSIM_MSG_SLOTS == msg_id % PSIM_MSG_SLOTS)
            return PSIM_EINVAL;
    h->pend_b_root[h->pend_b_n] = root;
    h->pend_b_msg[h->pend_b_n++] = msg_id;
    return PSIM_OK;
}

int orc_step(struct psim_handle *h, uint32_t n_rounds, psim_round_stats *stats) {
    psim_round_stats tmp;
    for (uint32_t i = 0; i < n_rounds; i++) {
        psim_round_stats *st = stats ? &stats[i] : &tmp;
        run_round(h, st);
        if (h->cfg.strict && st->overflow) return PSIM_ECAPACITY;   /* cfg.strict: fail loudly */
    }
    return PSIM_OK;
}

int orc_get_round(struct psim_handle *h, uint64_t *round) { *round = h->round; return PSIM_OK; }

int orc_get_nodes(struct psim_handle *h, uint32_t first, uint32_t count, psim_node_view *out) {
    if ((uint64_t)first + count > h->N) return PSIM_ERANGE;
    for (uint32_t k = 0; k < count; k++) {
        const node *s = &h->nodes[first + k];
        psim_node_view *v = &out[k];
        memset(v, 0, sizeof *v);
        v->up = s->up; v->epoch = s->epoch; v->start_round = s->start_round;
        v->rng_ctr = s->rng;
        v->act_n = s->act_n; v->pas_n = s->pas_n;
        memcpy(v->act, s->act, sizeof v->act); memcpy(v->pas, s->pas, sizeof v->pas);
        v->sent_n = s->sent_n; v->sent_head = s->sent_head; v->recv_n = s->recv_n; v->recv_head = s->recv_head;
        memcpy(v->sent_peer, s->sent_peer, sizeof v->sent_peer); memcpy(v->sent_id, s->sent_id, sizeof v->sent_id);
        memcpy(v->recv_peer, s->recv_peer, sizeof v->recv_peer); memcpy(v->recv_id, s->recv_id, sizeof v->recv_id);
        v->pt_all_n = s->pt_all_n; v->pt_common_n = s->pt_common_n;
        v->pt_out_n = s->out_n;
        memcpy(v->pt_all, s->pt_all, sizeof v->pt_all); memcpy(v->pt_common, s->pt_common, sizeof v->pt_common);
        for (int q = 0; q < PSIM_PT_ROOTS; q++) {
            v->pt_root[q] = s->rt_root[q]; v->pt_eager_n[q] = s->rt_eag_n[q]; v->pt_lazy_n[q] = s->rt_laz_n[q];
        }
        for (int q = 0, oe = 0, ol = 0; q < PSIM_PT_ROOTS; q++) {      /* pooled: slot by slot */
            memcpy(v->pt_eager + oe, s->rt_eag[q], s->rt_eag_n[q] * 4); oe += (int)s->rt_eag_n[q];
            memcpy(v->pt_lazy + ol, s->rt_laz[q], s->rt_laz_n[q] * 4); ol += (int)s->rt_laz_n[q];
        }
        memcpy(v->pt_out_peer, s->out_peer, sizeof v->pt_out_peer);
        memcpy(v->pt_out_msg, s->out_msg, sizeof v->pt_out_msg);
        memcpy(v->pt_out_round, s->out_round, sizeof v->pt_out_round);
        v->have = s->have; v->trk_round = s->trk_round; v->trk_hop = s->trk_hop;
        v->conn_n = s->conn_n;
        memcpy(v->conn, s->conn, sizeof v->conn);
    }
    return PSIM_OK;
}

/* psim_get_msg_slots: the live message slots (plumtree_backend's ETS set) */
int orc_get_msg_slots(struct psim_handle *h, uint32_t *ids, uint32_t *roots, size_t cap) {
    if (!h || !ids || !roots || cap < PSIM_MSG_SLOTS) return PSIM_EINVAL;
    for (int k = 0; k < PSIM_MSG_SLOTS; k++) { ids[k] = h->slot_msg[k]; roots[k] = h->slot_root[k]; }
    return PSIM_OK;
}

/* Delivery of the tracked broadcast (psim_get_delivery). */
int orc_get_delivery(struct psim_handle *h, uint32_t first, uint32_t count, uint8_t *have, uint32_t *round,
                     uint32_t *hop) {
    if ((uint64_t)first + count > h->N) return PSIM_ERANGE;
    uint64_t bit = h->tracked_msg == PSIM_NONE ? 0ull : 1ull << (h->tracked_msg % PSIM_MSG_SLOTS);
    for (uint32_t k = 0; k < count; k++) {
        const node *s = &h->nodes[first + k];
        have[k] = (s->have & bit) ? 1 : 0;
        round[k] = s->trk_round;
        hop[k] = s->trk_hop;
    }
    return PSIM_OK;
}

static uint32_t hbin(uint32_t v) { return v < PSIM_HIST_BINS ? v : PSIM_HIST_BINS - 1; }
static uint32_t uf_find(uint32_t *p, uint32_t x) {
    while (p[x] != x) { p[x] = p[p[x]]; x = p[x]; }
    return x;
}

/* Overlay statistics (psim_get_histograms), list-style over all nodes:
 * in-degrees counted link by link, symmetry by scanning the peer's view,
 * components by union-find over live active links. */
int orc_get_histograms(struct psim_handle *h, psim_histograms *out) {
    if (is_pl(h)) return PSIM_EUNSUPPORTED;
    memset(out, 0, sizeof *out);
    uint32_t N = h->N;
    uint32_t *ina = calloc(N, 4), *inp = calloc(N, 4), *par = malloc((size_t)N * 4), *sz = calloc(N, 4);
    if (!ina || !inp || !par || !sz) { free(ina); free(inp); free(par); free(sz); return PSIM_ENOMEM; }
    uint64_t bit = h->tracked_msg == PSIM_NONE ? 0ull : 1ull << (h->tracked_msg % PSIM_MSG_SLOTS);
    for (uint32_t i = 0; i < N; i++) par[i] = i;
    for (uint32_t i = 0; i < N; i++) {
        const node *s = &h->nodes[i];
        if (!s->up) continue;
        out->n_up++;
        uint32_t deg = 0;
        for (uint32_t k = 0; k < s->act_n; k++) {
            uint32_t p = s->act[k];
            if (p == i) continue;
            deg++;
            if (!h->nodes[p].up) continue;
            ina[p]++;
            out->active_links++;
            const node *q = &h->nodes[p];
            for (uint32_t j = 0; j < q->act_n; j++)
                if (q->act[j] == i) { out->symmetric_links++; break; }
            uint32_t a = uf_find(par, i), b = uf_find(par, p);
            if (a != b) par[a > b ? a : b] = a < b ? a : b;
        }
        for (uint32_t k = 0; k < s->pas_n; k++) {
            uint32_t p = s->pas[k];
            if (p != i && h->nodes[p].up) inp[p]++;
        }
        out->active_out[hbin(deg)]++;
        out->passive_fill[hbin(s->pas_n)]++;
        if (bit && (s->have & bit)) {
            out->delivered++;
            out->hop[hbin(s->trk_hop)]++;
            if (s->trk_round != PSIM_NONE && s->trk_round > out->last_round) out->last_round = s->trk_round;
        }
    }
    for (uint32_t i = 0; i < N; i++) {
        if (!h->nodes[i].up) continue;
        out->active_in[hbin(ina[i])]++;
        out->passive_in[hbin(inp[i])]++;
        uint32_t r = uf_find(par, i);
        if (r == i) out->components++;
        if (++sz[r] > out->largest_component) out->largest_component = sz[r];
    }
    free(ina); free(inp); free(par); free(sz);
    return PSIM_OK;
}

static uint64_t members_hash(struct psim_handle *h, const uint32_t *b) {
    uint64_t x = 0;
    for (uint32_t w = 0; w < h->W; w++)
        for (uint32_t v = fb_mem(h, b, w); v; v &= v - 1) x += mix64((uint64_t)(w * 32 + (uint32_t)__builtin_ctz(v)) + 1);
    return x;
}

int orc_get_strategy_nodes(struct psim_handle *h, uint32_t first, uint32_t count, psim_strategy_view *out) {
    if (!is_pl(h)) return PSIM_ESTATE;
    if ((uint64_t)first + count > h->N) return PSIM_ERANGE;
    for (uint32_t k = 0; k < count; k++) {
        uint32_t n = first + k;
        const node *s = &h->nodes[n];
        const snode *q = &h->sn[n];
        psim_strategy_view *v = &out[k];
        memset(v, 0, sizeof *v);
        v->up = s->up; v->start_round = s->start_round; v->rng_ctr = s->rng;
        v->pending = q->started ? q->pending : PSIM_NONE;
        v->last_ping = q->started ? q->last_ping : PSIM_NONE;
        v->view_n = q->view_n; v->in_n = q->inv_n;
        memcpy(v->view, q->view, sizeof v->view);
        memcpy(v->in_view, q->inv, sizeof v->in_view);
        if (h->cfg.strategy == PSIM_STRATEGY_SCAMP_V1 && q->view_n) v->view_slots = q->view_slots;
        if (h->fbits) {
            v->members = full_count(h, fb_row(h, n));
            v->members_hash = members_hash(h, fb_row(h, n));
        }
    }
    return PSIM_OK;
}

int orc_get_member_bits(struct psim_handle *h, uint32_t node, uint32_t *words, size_t n_words) {
    if (!h->fbits) return PSIM_ESTATE;
    if (node >= h->N) return PSIM_ERANGE;
    if (n_words < h->W) return PSIM_EINVAL;
    const uint32_t *b = fb_row(h, node);
    for (uint32_t w = 0; w < h->W; w++) words[w] = fb_mem(h, b, w);
    return PSIM_OK;
}

/* inbox of the next round, for message-level diffs in tests */
int orc_get_inbox(struct psim_handle *h, uint32_t *out, size_t cap, size_t *n) {
    *n = h->inbox.n;
    if (!out) return PSIM_OK;
    for (size_t i = 0; i < h->inbox.n && i < cap; i++) {
        const omsg *m = &h->inbox.v[i];
        uint32_t *o = out + i * 16;
        o[0] = m->dst; o[1] = m->src; o[2] = m->seq; o[3] = m->type | (m->ttl << 8) | (m->nex << 16);
        o[4] = m->a0; o[5] = m->a1; o[6] = m->a2; o[7] = m->a3;
        for (int k = 0; k < 8; k++) o[8 + k] = k < (int)m->nex ? m->ex[k] : 0;
    }
    return PSIM_OK;
}

/* exposed for RNG known-answer tests */
void orc_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                uint32_t out[4]) {
    philox(c0, c1, c2, c3, k0, k1, out);
}
uint32_t orc_bucket16(uint32_t id) { return bucket16_default(id); }

/* psim_set_bucket_table: the 16-slot bucket alone (the hash's bits 4-7 read as 0) */
int orc_set_bucket_table(struct psim_handle *h, const uint8_t *buckets, size_t n) {
    if (!h) return PSIM_EINVAL;
    if (h->round != 0) return PSIM_ESTATE;
    if (!buckets) { free(h->btab); h->btab = NULL; return PSIM_OK; }
    if (n != h->N) return PSIM_EINVAL;
    for (size_t i = 0; i < n; i++)
        if (buckets[i] > 15) return PSIM_EINVAL;
    if (!h->btab && !(h->btab = (uint8_t *)malloc(n))) return PSIM_ENOMEM;
    memcpy(h->btab, buckets, n);
    return PSIM_OK;
}

/* The sets v1 restatement alone (tests/test_strategies.py pins it against a
 * bucket-level model of OTP's sets.erl): ops[i] = e adds element e, ~e
 * deletes it, in a fresh set over the hash table `phash` (n entries); the
 * final sets:to_list/1 into out (cap >= its size), *out_n, *slots. */
int orc_sets_run(const uint32_t *phash, size_t n, const uint32_t *ops, size_t n_ops, uint32_t *out, size_t cap,
                 uint32_t *out_n, uint32_t *slots) {
    struct psim_handle h;
    memset(&h, 0, sizeof h);
    h.N = (uint32_t)n;
    uint8_t *tab = (uint8_t *)malloc(n ? n : 1);
    if (!tab) return PSIM_ENOMEM;
    for (size_t i = 0; i < n; i++) tab[i] = (uint8_t)phash[i];
    h.btab = tab;
    uint32_t *l = (uint32_t *)calloc(n_ops + 1, sizeof(uint32_t)), k = 0, ns = 16;
    if (!l) { free(tab); return PSIM_ENOMEM; }
    int rc = PSIM_OK;
    for (size_t i = 0; i < n_ops && !rc; i++) {
        uint32_t e = ops[i] >> 31 ? ~ops[i] : ops[i];
        if (e >= n) { rc = PSIM_ERANGE; break; }
        if (ops[i] >> 31) set_del_slots(&h, l, &k, e, &ns);
        else set_add(&h, l, &k, e, &ns);
    }
    if (!rc && cap < k) rc = PSIM_EINVAL;
    if (!rc) { memcpy(out, l, k * sizeof(uint32_t)); *out_n = k; *slots = ns; }
    free(l); free(tab);
    return rc;
}

/* psim_set_phash_table: erlang:phash(NodeSpec, 2^32) - 1 per node */
int orc_set_phash_table(struct psim_handle *h, const uint32_t *phash, size_t n) {
    if (!h) return PSIM_EINVAL;
    if (h->round != 0) return PSIM_ESTATE;
    if (!phash) { free(h->btab); h->btab = NULL; return PSIM_OK; }
    if (n != h->N) return PSIM_EINVAL;
    if (!h->btab && !(h->btab = (uint8_t *)malloc(n))) return PSIM_ENOMEM;
    for (size_t i = 0; i < n; i++) h->btab[i] = (uint8_t)phash[i];
    return PSIM_OK;
}

/* ---------------------------------------------- sharded protocol (tests) --
 * One oracle per rank owns [lo, hi); a round is orc_round_emit (events +
 * owned handlers; the emissions are read with orc_get_outbox in (src, seq)
 * order, packed like orc_get_inbox), the host exchanges messages by owner,
 * then orc_round_absorb with every message addressed to the owned range. */
static void pack(const omsg *m, uint32_t *o) {
    o[0] = m->dst; o[1] = m->src; o[2] = m->seq; o[3] = m->type | (m->ttl << 8) | (m->nex << 16);
    o[4] = m->a0; o[5] = m->a1; o[6] = m->a2; o[7] = m->a3;
    for (int k = 0; k < 8; k++) o[8 + k] = k < (int)m->nex ? m->ex[k] : 0;
}

int orc_round_emit(struct psim_handle *h, psim_round_stats *st) {
    round_begin(h, st);
    return PSIM_OK;
}

int orc_get_outbox(struct psim_handle *h, uint32_t *out, size_t cap, size_t *n) {
    *n = h->out.n;
    if (!out) return PSIM_OK;
    for (size_t i = 0; i < h->out.n && i < cap; i++) pack(&h->out.v[i], out + i * 16);
    return PSIM_OK;
}

int orc_round_absorb(struct psim_handle *h, const uint32_t *recs, size_t n) {
    msgvec in = {0, 0, 0};
    for (size_t i = 0; i < n; i++) {
        const uint32_t *o = recs + i * 16;
        omsg m;
        memset(&m, 0, sizeof m);
        m.dst = o[0]; m.src = o[1]; m.seq = o[2];
        m.type = o[3] & 0xFF; m.ttl = (o[3] >> 8) & 0xFF; m.nex = (o[3] >> 16) & 0xFF;
        m.a0 = o[4]; m.a1 = o[5]; m.a2 = o[6]; m.a3 = o[7];
        for (int k = 0; k < 8; k++) m.ex[k] = o[8 + k];
        if (m.dst < h->lo || m.dst >= h->hi) { free(in.v); return PSIM_ERANGE; }
        vec_push(&in, &m);
    }
    round_end(h, &in);
    free(in.v);
    return PSIM_OK;
}
