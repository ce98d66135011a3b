// psim_consume.hip -- the node-round kernel (K-consume + K-timer + K-emit).
//
// One 64-lane wave owns one node at a time (grid-stride over nodes).  The
// node's views are spread across lanes -- lane l holds active[l], passive[l],
// the l-th disconnect-id slot, the l-th Plumtree set entries -- so every list
// operation of the reference handlers (member, --, usort, select_random,
// sublist(shuffle(..)), ordsets add/del) becomes a handful of ballots and
// shuffles, and control flow is wave-uniform: no divergence between nodes
// and no scratch.  Messages are read and written as one coalesced 64-B record
// by lanes 0-15.
//
// k_consume runs the node's EXIT events, HyParView inbox and timers (and
// replays its notifies into the Plumtree state); k_pt then runs its Plumtree
// inbox, origin broadcast and lazy tick -- the fixed order of the round model
// R0.  k_relay, ahead of both, does the lone SHUFFLE
// relays and lazy ticks of a steady round in one lane per node and lists the
// rest for the two wave kernels.  Besides its own rows a wave reads only the
// flag/partition bytes of peers and the previous round's records.
//
// Reference handlers are cited as file:line under /root/reference:
//   hv = src/partisan_hyparview_peer_service_manager.erl
//   pt = src/partisan_plumtree_broadcast.erl
#include "psim_device.h"
#include "psim_kernels.h"
#include "psim_wave.h"

namespace psim {

#define ID_OF(e, n) (((uint32_t)(e) << 20) | (uint32_t)(n))
#define ID_E(id) ((id) >> 20)
#define ID_C(id) ((id)&0xFFFFFu)

constexpr int WAVES_PER_BLOCK = 4;
#ifndef PSIM_WAVES_PER_SIMD
#define PSIM_WAVES_PER_SIMD 4
#endif

// Diagnostic build only (-DPSIM_STAMPS): s_memtime between phase
// boundaries, summed per phase over all waves (psim::debug_stamps).
#ifdef PSIM_STAMPS
__device__ unsigned long long g_stamps[32];
__device__ unsigned long long g_stamps_lite[32];   // k_consume_lite's phases (profiles/stamps.py --lite)
#define STAMP(w, k)                                                                  \
    do {                                                                             \
        uint64_t t_ = __builtin_amdgcn_s_memtime();                                  \
        if (lane_id() == 0) (w).stl[(k)] += t_ - (w).t_last;                         \
        (w).t_last = t_;                                                             \
    } while (0)
// k_ptl (a lane per node, divergent): the first active lane adds the time
// since the wave's last stamp (both in LDS) to phase k -- the branches of a
// divergent handler run one after another, each charged its own time --
// into g_stamps_lite[16 + k] at the kernel's end
#define PTL_STAMP(k)                                                                 \
    do {                                                                             \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();                            \
        if (lane_id() == (uint32_t)__ffsll((long long)__builtin_amdgcn_read_exec()) - 1) { \
            ptl_st[(k)] += t_ - ptl_st[15];                                          \
            ptl_st[15] = t_;                                                         \
        }                                                                            \
    } while (0)
#else
#define STAMP(w, k) do { } while (0)
#define PTL_STAMP(k) do { } while (0)
#endif
constexpr uint32_t NONE = PSIM_NONE;

// ------------------------------------------------------------ the wave --
struct Wv {
    const RoundArgs* a;
    uint32_t* lds;       // 64 words of per-wave scratch
    uint32_t* nlog;      // notify log: NLOG snapshots x 8 ids + NLOG counts
    uint32_t nlog_n;
#ifdef PSIM_STAMPS
    uint64_t* stl;
    uint64_t t_last;
#endif
    uint64_t* st;        // block stats (LDS)
    uint32_t me, li, mypart, round;   // global id, local row index
    // the node's header fields (Hdr, psim_device.h)
    uint64_t rng;                     // the Philox draw counter
    uint32_t start_round, contact, epoch;
    uint32_t have, aux, trk_round, trk_hop;
    uint32_t vd;                      // views changed this round: 1 active, 2 passive
    uint32_t sx, rx, ox;              // id-map / outstanding extension rows + 1 (0: none)
    uint32_t act_n, pas_n, sent_n, sent_head, recv_n, recv_head;
    uint32_t all_n, com_n, out_n;
    uint32_t A, P, SP, SI, RP, RI, COM, EAG, LAZ;
    uint32_t AR;         // lanes 0-7: all_members; lanes RTB..: the root row -- lane RTB + k
                         // (k < PSIM_PT_ROOTS) root k (NONE = free), RTB + RT_EN / RT_LN the
                         // eager / lazy counts (byte k: slot k)
    const uint32_t* slots;   // the message slots in LDS (ids, then roots)
    uint64_t OUT;
    bool maps, pt, maps_dirty, pt_dirty;
    uint64_t obase;
    uint32_t seq;
    uint32_t CV, CF;     // connection cache: ids of Passive (lanes 0-31), Active (32-39)
                         // and the connection table (40-47) at node start; CF = flags |
                         // part << 8 of each
    uint32_t CN;         // the connection table (lanes 0 .. conn_n - 1): lingering peers, and
                         // | PSIM_CONN_DOWN the active members without a connection
    uint32_t conn_n, conn_dn;   // its entries, and those marked PSIM_CONN_DOWN
    uint32_t conn_cl;           // X-BOT: ... and those marked PSIM_CONN_CLOSING (stopped pids)
    bool cn_dirty;
    uint64_t digest;     // per-lane partial: lane j sums the hashes of record word j
    uint32_t SC;         // per-lane stats counter: lane k counts stats slot k (< NST)
    // draw cache: lane l holds the 58-bit draw of counter dc_base + l, filled
    // by one VALU Philox for 64 counters at once (dc_base = NONE64: empty)
    uint32_t DCL, DCH;
    uint64_t dc_base;
    // emissions are staged in LDS and written once per node (flush_recs), so
    // the body issues no global store: a later vmcnt wait never drains one
    uint32_t* srec;      // STAGE records x 16 words
    uint32_t* skey;      // their route keys
    uint32_t flushed;    // records already written for this node
    uint32_t fl;         // flag byte at node start (writeback)
    uint32_t KM;         // magic_lanes(): the exact-modulo multipliers
    bool work;           // the node had work this round
    bool lazy_quiet;     // its lazy tick ran and found no outstanding peer connected (flag_byte)
};
constexpr uint64_t NONE64 = ~0ull;
constexpr uint32_t STAGE = 16;
constexpr uint32_t RTB = PSIM_PT_MEMBERS_CAP;   // first lane of the root row in Wv::AR

// stats: lane k of SC holds slot k's count for this wave; flushed once per wave
DEV void st_add(Wv& w, int k, uint32_t v) { w.SC += lane_id() == (uint32_t)k ? v : 0u; }
// a fixed-table overflow of kind PSIM_OVF_*
DEV void ovf(Wv& w, int kind) {
    const uint32_t l = lane_id();
    w.SC += (l == (uint32_t)ST_OVF || l == (uint32_t)(ST_OVF_BY + kind)) ? 1u : 0u;
}
// this wave's counters and digest partials into the block's LDS stats
DEV void flush_wave_stats(const Wv& w, uint64_t* sst) {
    const uint32_t l = lane_id();
    if (l < NST && w.SC) atomicAdd((unsigned long long*)&sst[l], (unsigned long long)w.SC);
    uint64_t dg = w.digest;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) dg += shfl64(dg, (int)((l + off) & 63));
    if (l == 0 && dg) atomicAdd((unsigned long long*)&sst[ST_DIGEST], (unsigned long long)dg);
}

// compact the lanes of V selected by `keep` (uniform mask) to the front
DEV uint32_t compact(Wv& w, uint32_t V, uint64_t keep) {
    uint32_t l = lane_id();
    if ((keep >> l) & 1ull) w.lds[popc(keep & lt_mask())] = V;
    __builtin_amdgcn_wave_barrier();
    uint32_t m = popc(keep);
    uint32_t r = l < m ? w.lds[l] : 0u;
    __builtin_amdgcn_wave_barrier();
    return r;
}
DEV uint64_t compact64(Wv& w, uint64_t V, uint64_t keep) {
    uint32_t lo = compact(w, (uint32_t)V, keep);
    uint32_t hi = compact(w, (uint32_t)(V >> 32), keep);
    return ((uint64_t)hi << 32) | lo;
}

// lists:usort of the lanes of E selected by `valid` (uniform mask, lists
// of at most a few dozen entries): the first occurrence of each value is
// kept and lands at its rank among the kept values.  Returns the count; E
// holds the sorted unique values in lanes 0.., zeros above.
DEV uint32_t usort_mask(Wv& w, uint32_t& E, uint64_t valid) {
    uint32_t l = lane_id();
    bool dup = false;
    for (uint64_t m = valid; m; m &= m - 1) {             // drop later duplicates
        int j = ffs64(m);
        dup |= ((uint32_t)j < l) && rl(E, j) == E;
    }
    uint64_t keep = valid & ballot(!dup);
    uint32_t rank = 0;
    for (uint64_t m = keep; m; m &= m - 1) rank += rl(E, ffs64(m)) < E ? 1u : 0u;
    if ((keep >> l) & 1ull) w.lds[rank] = E;
    __builtin_amdgcn_wave_barrier();
    uint32_t c = popc(keep);
    E = l < c ? w.lds[l] : 0u;
    __builtin_amdgcn_wave_barrier();
    return c;
}
DEV uint32_t usort_lanes(Wv& w, uint32_t& E, uint32_t m) {
    return usort_mask(w, E, m >= 64 ? ~0ull : ((1ull << m) - 1ull));
}

DEV uint32_t hw_start(const Wv& w) { return w.start_round; }
DEV uint32_t hw_contact(const Wv& w) { return w.contact; }
DEV uint32_t hw_epoch(const Wv& w) { return w.epoch; }

// ----------------------------------------------------------------- RNG --
// The node's draws are consecutive Philox counters, so a cache line of 64
// of them costs one VALU Philox (every lane a counter) instead of 64 scalar
// ones; select_random and sublist both read it.
DEV void dc_fill(Wv& w, uint64_t base) {
    uint64_t v = draw58_at(base + lane_id(), w.me, kargs().seed);
    w.DCL = (uint32_t)v; w.DCH = (uint32_t)(v >> 32);
    w.dc_base = base;
}
DEV uint64_t draw(Wv& w) {
    uint64_t c = w.rng++;
    // (a single SALU Philox for a node's first draw measured 3 % slower)
    if (c < w.dc_base || c - w.dc_base >= 64) dc_fill(w, c);
    uint32_t i = (uint32_t)(c - w.dc_base);
    return ((uint64_t)rl(w.DCH, i) << 32) | rl(w.DCL, i);
}

// rand:uniform/1 with a 58-bit generator (OTP rand.erl ?uniform_range);
// here n <= 64 always (a count of lanes), so only the exact small modulo
// is compiled in
DEV uint32_t uniform_n(Wv& w, uint32_t n) {
    const uint64_t two58 = 1ull << 58;
    for (;;) {
        uint64_t v = draw(w);
        if (v < n) return (uint32_t)v + 1;
        uint64_t i = mod_small_m(v, n, rl(w.KM, n & 63));
        if (v - i <= two58 - n) return (uint32_t)i + 1;
    }
}

// select_random/2 (hv:1346-1356): rand:uniform(length(View -- Omit));
// nothing drawn when nothing is eligible
DEV uint32_t select_random(Wv& w, uint32_t V, uint32_t n, uint32_t o0, uint32_t o1, uint32_t o2) {
    uint32_t l = lane_id();
    uint64_t M = ballot(l < n && V != o0 && V != o1 && V != o2);
    uint32_t cnt = popc(M);
    if (cnt == 0) return NONE;
    uint32_t k = uniform_n(w, cnt) - 1;
    // the k-th set bit of M: the lane in M with k members of M below it
    return rl(V, ffs64(ballot(((M >> l) & 1ull) && popc(M & lt_mask()) == k)));
}

// lists:sublist(shuffle(to_list(View)), K) (hv:1359-1361, :1586-1587): one
// rand:uniform() key per element (element l draws counter rng + l); each lane
// counts the (key, element) pairs below its own -- its position in the sorted
// list -- and the first K positions are appended to OUT at lanes on..
DEV uint32_t sublist(Wv& w, uint32_t V, uint32_t n, uint32_t k, uint32_t& OUT, uint32_t on) {
    uint32_t l = lane_id();
    uint64_t base = w.rng;
    if (base < w.dc_base || base + n - w.dc_base > 64) dc_fill(w, base);   // must cover [base, base + n)
    uint32_t off = (uint32_t)(base - w.dc_base);
    uint32_t src = (l + off) & 63;
    uint32_t kl = shfl(w.DCL, (int)src), kh = shfl(w.DCH, (int)src);
    uint64_t key = l < n ? ((((uint64_t)kh) << 32) | kl) >> 5 : ~0ull;
    uint32_t m = n < k ? n : k;
    const uint32_t hi = (uint32_t)(key >> 21);
    // few of many (a passive view): the m smallest of the top 32 key bits,
    // one wave minimum each; a tie at a pick (about once in 10^7) falls
    // through to the exact path below
    if (n >= 3 * m) {
        uint32_t H = hi, O = OUT;
        bool tie = false;
        for (uint32_t i = 0; i < m && !tie; i++) {
            const uint32_t mn = wave_min(H);
            const uint64_t at = ballot(H == mn);
            tie = popc(at) > 1;
            const int j = ffs64(at);
            O = l == on + i ? rl(V, j) : O;
            H = l == (uint32_t)j ? 0xFFFFFFFFu : H;
        }
        if (!tie) {
            OUT = O;
            w.rng = base + n;
            return on + m;
        }
    }
    // rank on the top 32 of the 53 key bits; only when two of them tie (about
    // once in 10^7 sublists) is the full (key, element) order recounted
    uint32_t rank = 0, eq = 0;
    for (uint32_t j = 0; j < n; j++) {
        uint32_t hj = rl(hi, j);
        rank += hj < hi ? 1u : 0u;
        eq += hj == hi ? 1u : 0u;
    }
    if (ballot(l < n && eq > 1)) {
        rank = 0;
        for (uint32_t j = 0; j < n; j++) {
            uint64_t kj = rl64(key, j);
            uint32_t ej = rl(V, j);
            rank += (kj < key || (kj == key && ej < V)) ? 1u : 0u;
        }
    }
    if (l < n && rank < m) w.lds[rank] = V;
    __builtin_amdgcn_wave_barrier();
    uint32_t got = (l >= on && l < on + m) ? w.lds[(l - on) & 63] : 0u;
    __builtin_amdgcn_wave_barrier();
    OUT = (l >= on && l < on + m) ? got : OUT;
    w.rng = base + n;
    return on + m;
}

// ------------------------------------------------------------- emission --
DEV void flush_recs(Wv& w);
DEV void flush_full(Wv& w);

DEV void emit4(Wv& w, uint32_t dst, uint32_t type, uint32_t ttl, uint32_t a0, uint32_t a1,
               uint32_t a2, uint32_t a3, uint32_t EX, uint32_t nex) {
    uint32_t l = lane_id();
    uint32_t s = w.seq++;
    uint32_t k = s - w.flushed;                      // staging slot
    uint32_t tt = type | (ttl << 8) | (nex << 16);
    // lanes 8..15 take the exchange ids of lanes 0..7 (DPP row_shr:8)
    uint32_t exv = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)EX, 0x118, 0xF, 0xF, true);
    uint32_t word = l == 0 ? dst : l == 1 ? w.me : l == 2 ? tt : l == 3 ? s : l == 4 ? a0
                  : l == 5 ? a1 : l == 6 ? a2 : l == 7 ? a3 : (l - 8 < nex ? exv : 0u);
    if (l < 16) {
        w.srec[k * 16 + l] = word;
        w.digest += (uint64_t)word * digest_mul(l);   // the oracle's msg_hash, word l
    }
    if (l == 0) w.skey[k] = dst | (max_emit(type) << KEY_DST_BITS);
    st_add(w, ST_EMIT + type, 1);
    if (k + 1 == STAGE) flush_full(w);               // a node with > STAGE emissions
}
DEV void emit(Wv& w, uint32_t dst, uint32_t type, uint32_t ttl, uint32_t a0, uint32_t a1,
              uint32_t a2, uint32_t EX, uint32_t nex) {
    emit4(w, dst, type, ttl, a0, a1, a2, 0u, EX, nex);
}

// The staged records [flushed, seq) to outbox slots obase + flushed..: one
// 1-KiB store (lane l: 16-B piece l & 3 of record l >> 2) and one route-key
// store.  Both always run with every lane active -- lanes past the last
// record repeat it, and with nothing staged they rewrite the node's own
// first slot (reserved, and unused when ocnt says so) -- so every node issues
// the same number of vector memory operations and the compiler's vmcnt
// waits for later loads are exact instead of draining these stores.
DEV void flush_recs(Wv& w) {
    const uint32_t l = lane_id();
    const uint32_t cnt = w.seq - w.flushed;
    uint32_t j, g, jk, gk;                           // staging / outbox index (records, keys)
    if (cnt) {
        j = min(l >> 2, cnt - 1); g = w.flushed + j;
        jk = min(l, cnt - 1); gk = w.flushed + jk;
    } else {
        j = w.flushed ? STAGE - 1 : 0; g = w.flushed ? w.flushed - 1 : 0;
        jk = j; gk = g;
    }
    __builtin_amdgcn_wave_barrier();
    const uint4 piece = reinterpret_cast<const uint4*>(w.srec + j * 16)[l & 3];
    const uint32_t key = w.skey[jk];
    reinterpret_cast<uint4*>(kargs().rec_out + w.obase + g)[l & 3] = piece;
    kargs().okey[w.obase + gk] = key;
    __builtin_amdgcn_wave_barrier();
    w.flushed = w.seq;
}

// A full staging buffer from inside emit: lane l stores piece l of the 16
// records (record l >> 2, 16-B piece l & 3 -- i.e. uint4 l of the run) and
// lanes 0-15 their route keys.  Kept apart from flush_recs so the emit
// sites carry only these few temporaries (uniform bases, one index).
DEV void flush_full(Wv& w) {
    const uint32_t l = lane_id();
    __builtin_amdgcn_wave_barrier();
    const uint64_t r0 = w.obase + w.flushed;
    uint4* rb = reinterpret_cast<uint4*>(kargs().rec_out + r0);
    uint32_t* kb = kargs().okey + r0;
    rb[l] = reinterpret_cast<const uint4*>(w.srec)[l];
    kb[l & (STAGE - 1)] = w.skey[l & (STAGE - 1)];
    __builtin_amdgcn_wave_barrier();
    w.flushed = w.seq;
}

// maybe_connect + find (partisan_util.erl:75-134): the peer's manager runs
// and no partition separates the two
// F_UP and the partition of another node cannot change during k_consume,
// so the cache filled at node start answers exactly for its members
DEV bool connect_ok(const Wv& w, uint32_t dst) {
    if (dst >= kargs().n_nodes || dst == w.me) return false;
    uint64_t m = ballot(w.CV == dst);
    uint32_t v = m ? rl(w.CF, ffs64(m))
                   : ((uint32_t)kargs().flags[dst] | ((uint32_t)kargs().part[dst] << 8));
    return (v & F_UP) && (v >> 8) == w.mypart;
}

// -------------------------------------------------------- connections --
// The manager's Connections dict (the oracle's conn_*):
// the active view plus the table CN -- lingering peers outside the active
// view, and | PSIM_CONN_DOWN the active members without a connection.
// maybe_connect/2 opens one before every HyParView send; only disconnect/2
// (hv:1237-1258) and the peer's death (EXIT, hv:609-654) close one.
DEV int conn_find(const Wv& w, uint32_t e) { return idx_of(w.CN, w.conn_n, e); }
DEV void conn_add(Wv& w, uint32_t e) {
    if (conn_find(w, e) >= 0) return;
    if (w.conn_n >= PSIM_CONN_CAP) { ovf(w, PSIM_OVF_CONN); return; }
    w.CN = lane_id() == w.conn_n ? e : w.CN;
    w.conn_n++;
    w.conn_dn += (e & PSIM_CONN_DOWN) ? 1u : 0u;
    w.conn_cl += (e & PSIM_CONN_CLOSING) ? 1u : 0u;
    w.cn_dirty = true;
}
DEV void conn_del(Wv& w, uint32_t e) {
    const int k = conn_find(w, e);
    if (k < 0) return;
    vdel(w.CN, w.conn_n, (uint32_t)k);
    w.conn_dn -= (e & PSIM_CONN_DOWN) ? 1u : 0u;
    w.conn_cl -= (e & PSIM_CONN_CLOSING) ? 1u : 0u;
    w.cn_dirty = true;
}
// X-BOT: the member's connection pid was stopped by a do_disconnect whose
// state was discarded; the dead pid stays in the dict until its 'EXIT'
DEV bool conn_closing(const Wv& w, uint32_t p) { return w.conn_cl && conn_find(w, p | PSIM_CONN_CLOSING) >= 0; }
// partisan_peer_service_connections:find/2 succeeds over a live pid
DEV bool conn_has(const Wv& w, uint32_t p) {
    if (has(w.A, w.act_n, p))
        return (!w.conn_dn || conn_find(w, p | PSIM_CONN_DOWN) < 0) && !conn_closing(w, p);
    return w.conn_n && conn_find(w, p) >= 0;
}
// partisan_util:maybe_connect/2 (util.erl:75-134): connected afterwards (a
// dead pid in the dict counts as found: nothing is opened)
DEV bool maybe_connect(Wv& w, uint32_t p) {
    if (conn_closing(w, p)) return true;
    if (!connect_ok(w, p)) return false;
    if (has(w.A, w.act_n, p)) {
        if (w.conn_dn) conn_del(w, p | PSIM_CONN_DOWN);
    } else {
        conn_add(w, p);
    }
    return true;
}
// disconnect/2 (hv:1237-1258); X-BOT: a stopped pid is pruned like a live
// one (the reference's second gen_server:stop raises noproc)
DEV void disconnect(Wv& w, uint32_t p) {
    if (conn_closing(w, p)) conn_del(w, p | PSIM_CONN_CLOSING);
    if (has(w.A, w.act_n, p)) conn_add(w, p | PSIM_CONN_DOWN);
    else if (w.conn_n) conn_del(w, p);
}

// maybe_connect, then do_send_message/3 (hv:1274-1343); success draws
// rand:uniform(1) in partisan_util:dispatch_pid/1 (util:190-195), always
// exactly one value.  Every HyParView send of the reference is preceded by
// a maybe_connect of its destination.
DEV void hv_send(Wv& w, uint32_t dst, uint32_t type, uint32_t ttl, uint32_t a0, uint32_t a1,
                 uint32_t EX, uint32_t nex) {
    if (conn_closing(w, dst)) { w.rng++; st_add(w, ST_FAIL, 1); return; }   // X-BOT: a dead pid (draw, fail)
    if (!maybe_connect(w, dst)) { st_add(w, ST_FAIL, 1); return; }
    w.rng++;
    emit(w, dst, type, ttl, a0, a1, 0, EX, nex);
}

// ----------------------------------------------------------- id maps --
// The id maps, loaded on first use (most nodes of a round never touch
// them): lanes below IDMAP_IN hold the node's own entries, lanes above its
// extension row's -- one load per array either way.
DEV void load_maps(Wv& w) {
    if (w.maps) return;
    static_assert(PSIM_IDMAP_CAP == 64, "an id map is one entry per lane");
    KArgs& a = kargs();
    const uint32_t l = lane_id(), sx = w.sx, rx = w.rx;
    const bool own = l < IDMAP_IN;
    const size_t io = w.li * IDMAP_IN + (l & (IDMAP_IN - 1));
    const size_t so = sx ? (size_t)(sx - 1) * IDMAP_EXT + ((l - IDMAP_IN) & 63) : 0;
    const size_t ro = rx ? (size_t)(rx - 1) * IDMAP_EXT + ((l - IDMAP_IN) & 63) : 0;
    const uint64_t sv = *(own || !sx ? a.sentm + io : a.mapx + so);
    const uint64_t rv = *(own || !rx ? a.recvm + io : a.mapx + ro);
    const uint64_t s2 = own || sx ? sv : 0ull, r2 = own || rx ? rv : 0ull;
    w.SP = (uint32_t)s2; w.SI = (uint32_t)(s2 >> 32);
    w.RP = (uint32_t)r2; w.RI = (uint32_t)(r2 >> 32);
    w.maps = true;
}

DEV void map_store(Wv& w, uint32_t& PV, uint32_t& IV, uint32_t& n, uint32_t& head, uint32_t p,
                   uint32_t v) {
    uint32_t l = lane_id();
    w.maps_dirty = true;
    int i = idx_of(PV, n, p);
    if (i >= 0) { IV = l == (uint32_t)i ? v : IV; return; }
    if (n < PSIM_IDMAP_CAP) {
        PV = l == n ? p : PV; IV = l == n ? v : IV; n++;
        return;
    }
    ovf(w, PSIM_OVF_IDMAP);
    PV = l == head ? p : PV; IV = l == head ? v : IV;
    head = (head + 1) % PSIM_IDMAP_CAP;
}

DEV uint32_t current_id(Wv& w, uint32_t p) {             // hv:1622-1630
    int i = idx_of(w.RP, w.recv_n, p);
    return i >= 0 ? rl(w.RI, i) : ID_OF(1, 0);
}
DEV uint32_t next_id(Wv& w, uint32_t p) {                // hv:1633-1639
    int i = idx_of(w.SP, w.sent_n, p);
    if (i >= 0) {
        uint32_t s = rl(w.SI, i);
        if (ID_E(s) == hw_epoch(w)) return s + 1;
    }
    return ID_OF(hw_epoch(w), 1);
}
DEV bool addable_epoch(Wv& w, uint32_t pe, uint32_t p) { // hv:1670-1676
    int i = idx_of(w.SP, w.sent_n, p);
    return i < 0 || pe >= ID_E(rl(w.SI, i));
}
DEV bool addable_id(Wv& w, uint32_t d, uint32_t p) {     // hv:1656-1669
    int i = idx_of(w.SP, w.sent_n, p);
    if (i < 0) return true;
    uint32_t s = rl(w.SI, i);
    if (ID_E(d) != ID_E(s)) return ID_E(d) > ID_E(s);
    return ID_C(d) >= ID_C(s);
}
DEV bool valid_disconnect(Wv& w, uint32_t p, uint32_t d) { // hv:1642-1653
    int i = idx_of(w.RP, w.recv_n, p);
    if (i < 0) return true;
    uint32_t s = rl(w.RI, i);
    if (ID_E(d) > ID_E(s)) return true;
    return ID_C(d) > ID_C(s);
}

// ------------------------------------------------------- view updates --
DEV void add_to_passive(Wv& w, uint32_t p) {             // hv:1423-1448
    uint32_t l = lane_id();
    if (p == w.me || ballot((l < w.act_n && w.A == p) || (l < w.pas_n && w.P == p))) return;
    if (w.pas_n >= kargs().max_passive) {
        // select_random(Passive, [Myself]): Myself is never in Passive (no
        // path inserts it), so the index draw addresses Passive directly
        uint32_t k = uniform_n(w, w.pas_n) - 1;
        vdel(w.P, w.pas_n, k);
    }
    view_add(kargs().btab, w.P, w.pas_n, p);
    w.vd |= 2u;
}

DEV void drop_random_active(Wv& w) {                     // hv:1467-1512
    uint32_t p = select_random(w, w.A, w.act_n, w.me, w.me, w.me);
    if (p == NONE) return;
    vdel_val(w.A, w.act_n, p);
    if (w.conn_dn) conn_del(w, p | PSIM_CONN_DOWN);
    w.vd |= 1u;
    add_to_passive(w, p);
    uint32_t nid = next_id(w, p);
    map_store(w, w.SP, w.SI, w.sent_n, w.sent_head, p, nid);
    hv_send(w, p, PSIM_MSG_DISCONNECT, 0, nid, 0, 0, 0);   // maybe_connect (hv:1493), send
    disconnect(w, p);                                     // (hv:1506)
}

// (the connection the caller opened -- every caller but neighbor_accepted
// runs maybe_connect first -- moves with the peer into the active view;
// without one the peer is an active member without a connection)
DEV void add_to_active(Wv& w, uint32_t p) {              // hv:1371-1420
    if (p == w.me || has(w.A, w.act_n, p)) return;
    if (vdel_val(w.P, w.pas_n, p)) w.vd |= 2u;
    if (w.act_n >= kargs().max_active) drop_random_active(w);
    const bool had = w.conn_n && conn_find(w, p) >= 0;
    if (had) conn_del(w, p);
    view_add(kargs().btab, w.A, w.act_n, p);
    w.vd |= 1u;
    if (!had) conn_add(w, p | PSIM_CONN_DOWN);
}

// usort([Myself] ++ sublist(Active, k_active) ++ sublist(Passive, k_passive))
DEV uint32_t build_exchange(Wv& w, uint32_t& EX) {
    EX = lane_id() == 0 ? w.me : 0u;
    uint32_t m = 1;
    m = sublist(w, w.A, w.act_n, kargs().k_active, EX, m);
    m = sublist(w, w.P, w.pas_n, kargs().k_passive, EX, m);
    return usort_lanes(w, EX, m);
}

// merge_exchange/2 (hv:1590-1595): add_to_passive for each of
// usort(Exchange) -- Active -- [Myself], in order.  Every eviction draws
// rand:uniform(|Passive|) with |Passive| = max_passive_size, so the draws of
// up to mt evictions are taken in parallel (lane j: the j-th eviction's
// index); if any of them would be rejected by ?uniform_range (p ~ 2^-53)
// the sequential add_to_passive chain runs instead.  The passive entries'
// bucket tags are kept beside them for the to_list-order inserts.
DEV void merge_exchange(Wv& w, uint32_t EX, uint32_t nex) {
    const uint32_t l = lane_id();
    bool in_act = false;
    for (uint32_t j = 0; j < w.act_n; j++) in_act |= (EX == rl(w.A, j));
    uint32_t T = EX;
    const uint32_t mt = usort_mask(w, T, ballot(l < nex && EX != w.me && !in_act));
    if (!mt) return;
    const uint32_t maxp = kargs().max_passive;
    const uint64_t c0 = w.rng;
    if (c0 < w.dc_base || c0 + mt - w.dc_base > 64) dc_fill(w, c0);   // cover [c0, c0 + mt)
    const uint32_t off = (uint32_t)(c0 - w.dc_base);
    const uint32_t src = (off + l) & 63;
    const uint64_t v = ((uint64_t)shfl(w.DCH, (int)src) << 32) | shfl(w.DCL, (int)src);
    const uint32_t KI = mod_small_m(v, maxp, rl(w.KM, maxp & 63));
    const bool rej = v >= maxp && v - KI > (1ull << 58) - maxp;
    if (maxp > 64 || ballot(l < mt && rej)) {
        for (uint32_t i = 0; i < mt; i++) add_to_passive(w, rl(T, i));
        return;
    }
    const uint8_t* bt = kargs().btab;
    uint32_t PB = l < w.pas_n ? bucket16(bt, w.P) : 0u;
    uint32_t used = 0;
    for (uint32_t i = 0; i < mt; i++) {
        const uint32_t t = rl(T, i);
        if (ballot(l < w.pas_n && w.P == t)) continue;
        if (w.pas_n >= maxp) {                       // select_random(Passive, [Myself]) + remove
            const uint32_t k = rl(KI, used++);
            uint32_t n2 = w.pas_n;
            vdel(PB, n2, k);
            vdel(w.P, w.pas_n, k);
        }
        const uint32_t b = bucket16(bt, t);
        const uint32_t pos = popc(ballot(l < w.pas_n && PB <= b));
        uint32_t n2 = w.pas_n;
        vins(PB, n2, pos, b);
        vins(w.P, w.pas_n, pos, t);
        w.vd |= 2u;
    }
    w.rng = c0 + used;
}

DEV void move_to_active(Wv& w, uint32_t p) {             // hv:1679-1709
    if (p == NONE) return;
    uint32_t EX;
    uint32_t nex = build_exchange(w, EX);
    hv_send(w, p, PSIM_MSG_NEIGHBOR_REQUEST, 0, current_id(w, p), 0, EX, nex);
}

// ------------------------------------------------------------ plumtree --
DEV void ord_add(Wv& w, uint32_t& V, uint32_t& n, uint32_t cap, uint32_t e) {
    uint32_t l = lane_id();
    if (ballot(l < n && V == e)) return;
    if (n >= cap) { ovf(w, PSIM_OVF_PT); return; }
    vins(V, n, popc(ballot(l < n && V < e)), e);
}

// Per-root sets, pooled: the eager (lazy) entries of every slot in one
// 64-lane register -- slot 0's entries first, then slot 1's, ... -- with slot
// k's count in byte k of RT lane RT_EN (RT_LN), so its entries start at the
// sum of the counts below k.  Only the total over the slots is bounded.
DEV uint32_t rt_word(const Wv& w, uint32_t which) { return rl(w.AR, RTB + which); }
DEV uint32_t byte_sum(uint32_t c) { return (c * 0x01010101u) >> 24; }   // counts <= 64: no carry
DEV uint32_t rt_off(uint32_t cw, uint32_t k) { return k ? byte_sum(cw & (0xFFFFFFFFu >> (32 - 8 * k))) : 0u; }
DEV uint32_t rt_count(const Wv& w, uint32_t which, uint32_t k) { return (rt_word(w, which) >> (8 * k)) & 0xFFu; }
DEV void rt_set_count(Wv& w, uint32_t which, uint32_t k, uint32_t n) {
    const uint32_t l = lane_id();
    w.AR = l == RTB + which ? ((w.AR & ~(0xFFu << (8 * k))) | (n << (8 * k))) : w.AR;
}
DEV uint32_t rt_root(const Wv& w, uint32_t k) { return rl(w.AR, RTB + k); }
// the slot of `root`, -1 without per-root sets
DEV int rt_find(const Wv& w, uint32_t root) {
    const uint32_t l = lane_id();
    const int at = ffs64(ballot(l >= RTB && l < RTB + PSIM_PT_ROOTS && w.AR == root));
    return at < 0 ? -1 : at - (int)RTB;
}

// ordsets add_element / del_element within slot k of the pool V (which =
// RT_EN for the eager pool, RT_LN for the lazy one)
DEV void slot_add(Wv& w, uint32_t& V, uint32_t which, uint32_t k, uint32_t e) {
    const uint32_t l = lane_id(), cw = rt_word(w, which);
    const uint32_t n = (cw >> (8 * k)) & 0xFFu, b = rt_off(cw, k);
    const bool in = l >= b && l < b + n;
    if (ballot(in && V == e)) return;
    uint32_t T = byte_sum(cw);
    if (T >= PSIM_PT_SET_POOL) { ovf(w, PSIM_OVF_PT); return; }
    vins(V, T, b + popc(ballot(in && V < e)), e);
    rt_set_count(w, which, k, n + 1);
}
DEV void slot_del(Wv& w, uint32_t& V, uint32_t which, uint32_t k, uint32_t e) {
    const uint32_t l = lane_id(), cw = rt_word(w, which);
    const uint32_t n = (cw >> (8 * k)) & 0xFFu, b = rt_off(cw, k);
    const int at = ffs64(ballot(l >= b && l < b + n && V == e));
    if (at < 0) return;
    uint32_t T = byte_sum(cw);
    vdel(V, T, (uint32_t)at);
    rt_set_count(w, which, k, n - 1);
}

DEV uint32_t take_ext_row(Wv& w, uint32_t* top, uint32_t rows, int kind);

// The outstanding table's tail (entries OUT_HEAD.. of a table past one
// register, psim_device.h): lane l holds entry OUT_HEAD + l, in place in the
// extension row (a tail implies one: pt_add_out takes it before the first
// tail entry)
DEV uint64_t* out_tail(const Wv& w) {
    return kargs().outx + (size_t)(w.ox - 1) * OUT_EXT + OUT_TAIL_AT + lane_id();
}
DEV uint64_t load_out_tail(const Wv& w) {
    return lane_id() < w.out_n - OUT_HEAD ? *out_tail(w) : 0ull;
}

// neighbors_down/2's outstanding filter (pt:414-416): the entries to peer e
// leave, the order kept across the register and the tail
DEV void out_drop_peer(Wv& w, uint32_t e) {
    const uint32_t l = lane_id();
    const uint64_t keep = ballot(l < w.out_n && (uint32_t)(w.OUT >> 32) != e);
    if (w.out_n <= OUT_HEAD) {
        if (popc(keep) != w.out_n) {
            w.OUT = compact64(w, w.OUT, keep);
            w.out_n = popc(keep);
        }
        return;
    }
    const uint32_t nt = w.out_n - OUT_HEAD;
    uint64_t T = load_out_tail(w);
    const uint64_t kt = ballot(l < nt && (uint32_t)(T >> 32) != e);
    const uint32_t k1 = popc(keep), k2 = popc(kt);
    if (k1 + k2 == w.out_n) return;
    const uint64_t H = compact64(w, w.OUT, keep);
    T = compact64(w, T, kt);
    // the register: its k1 kept entries, then the tail's first 64 - k1
    const uint64_t up = shfl64(T, (int)((l - k1) & 63));
    w.OUT = l < k1 ? H : (l - k1 < k2 ? up : 0ull);
    const uint32_t sh = OUT_HEAD - k1;
    const uint64_t rest = shfl64(T, (int)((l + sh) & 63));
    T = l + sh < k2 ? rest : 0ull;
    w.out_n = k1 + k2;
    *out_tail(w) = T;                                 // (zeros past the table: a getter reads the row)
}

// notify/1 (hv:1598-1599) -> plumtree update/1 -> handle_cast({update, ..})
// (pt:314-336), reset_peers/4 (:652-659), neighbors_down/2 (:404-423)
DEV void apply_notify(Wv& w, uint32_t SNAP, uint32_t sn) {
    w.pt_dirty = true;
    uint32_t l = lane_id();
    uint32_t CUR = SNAP;
    uint32_t nc = usort_lanes(w, CUR, sn);
    bool in_all = false;
    for (uint32_t j = 0; j < w.all_n; j++) in_all |= (CUR == rl(w.AR, j));
    uint64_t newm = ballot(l < nc && !in_all);
    bool in_cur = false;
    for (uint32_t j = 0; j < nc; j++) in_cur |= (w.AR == rl(CUR, j));
    uint64_t remm = ballot(l < w.all_n && !in_cur);
    uint32_t REM = compact(w, w.AR, remm);
    uint32_t nr = popc(remm);
    if (newm) {
        for (uint64_t m = newm; m; m &= m - 1) {
            uint32_t e = rl(CUR, ffs64(m));
            if (has(w.COM, w.com_n, e)) continue;
            if (w.com_n >= PSIM_PT_MEMBERS_CAP) {
                bool made = false;
                for (uint32_t r = 0; r < nr && !made; r++) made = vdel_val(w.COM, w.com_n, rl(REM, r));
                if (!made) { ovf(w, PSIM_OVF_PT); continue; }
            }
            ord_add(w, w.COM, w.com_n, PSIM_PT_MEMBERS_CAP, e);
        }
        // eager_sets = lazy_sets = orddict:new() (pt:656-657)
        w.AR = l < RTB ? CUR : (l < RTB + PSIM_PT_ROOTS ? NONE : 0u);
        w.EAG = 0; w.LAZ = 0;
        w.all_n = nc;
    }
    for (uint32_t r = 0; r < nr; r++) {
        uint32_t e = rl(REM, r);
        vdel_val(w.COM, w.com_n, e);
        for (uint32_t k = 0; k < PSIM_PT_ROOTS; k++) {   // every root's sets (pt:410-413)
            if (rt_root(w, k) == NONE) continue;
            slot_del(w, w.EAG, RT_EN, k, e);
            slot_del(w, w.LAZ, RT_LN, k, e);
        }
        out_drop_peer(w, e);
    }
}

// notify/1 only ever feeds Plumtree state, which nothing reads during the
// HyParView phase, so each call logs the active view it would publish and the
// log is replayed, in order, before the Plumtree phase (one inlined copy of
// the update logic instead of one per call site).  A notify identical to the
// previous one is a no-op (New and Removed are both empty) and is not logged.
constexpr uint32_t NLOG = 16;
DEV void load_pt_rows(Wv& w);
DEV void replay_notifies(Wv& w) {
    if (!w.nlog_n) return;
    if (!w.pt) load_pt_rows(w);                  // the Plumtree rows, on the first replay only
    uint32_t l = lane_id();
    for (uint32_t i = 0; i < w.nlog_n; i++) {
        uint32_t V = l < PSIM_ACTIVE_CAP ? w.nlog[i * PSIM_ACTIVE_CAP + l] : 0u;
        uint32_t n = w.nlog[NLOG * PSIM_ACTIVE_CAP + i];
        __builtin_amdgcn_wave_barrier();
        apply_notify(w, V, n);
    }
    w.nlog_n = 0;
}
DEV void notify(Wv& w) {
    if (!kargs().plumtree) return;
    uint32_t l = lane_id();
    if (w.nlog_n) {
        uint32_t k = w.nlog_n - 1;
        uint32_t V = l < PSIM_ACTIVE_CAP ? w.nlog[k * PSIM_ACTIVE_CAP + l] : 0u;
        uint32_t n = w.nlog[NLOG * PSIM_ACTIVE_CAP + k];
        __builtin_amdgcn_wave_barrier();
        if (n == w.act_n && !ballot(l < PSIM_ACTIVE_CAP && V != w.A)) return;
    }
    if (w.nlog_n == NLOG) replay_notifies(w);
    if (l < PSIM_ACTIVE_CAP) w.nlog[w.nlog_n * PSIM_ACTIVE_CAP + l] = w.A;
    if (l == 0) w.nlog[NLOG * PSIM_ACTIVE_CAP + w.nlog_n] = w.act_n;
    __builtin_amdgcn_wave_barrier();
    w.nlog_n++;
}

// update_peers/5 + set_peers/4 (pt:593-609): the root's slot; a new root
// takes the lowest free slot, its sets starting as (common_eagers, []) at its
// place in the pools; with every slot taken, or no room in the eager pool
// for the common eagers, the store is an overflow
DEV void pt_update(Wv& w, uint32_t from, uint32_t root, bool to_eager) {
    w.pt_dirty = true;
    int k = rt_find(w, root);
    if (k < 0) {
        k = rt_find(w, NONE);
        const uint32_t cw = rt_word(w, RT_EN), m = w.com_n;
        if (k < 0 || byte_sum(cw) + m > PSIM_PT_SET_POOL) { ovf(w, PSIM_OVF_PT); return; }
        const uint32_t l = lane_id(), b = rt_off(cw, (uint32_t)k);
        const uint32_t c = shfl(w.COM, (int)((l - b) & 63)), up = shfl(w.EAG, (int)((l - m) & 63));
        w.EAG = l < b ? w.EAG : (l < b + m ? c : up);
        w.AR = l == RTB + (uint32_t)k ? root : w.AR;
        rt_set_count(w, RT_EN, k, m);
        rt_set_count(w, RT_LN, k, 0);
    }
    if (to_eager) {
        slot_add(w, w.EAG, RT_EN, k, from);
        slot_del(w, w.LAZ, RT_LN, k, from);
    } else {
        slot_del(w, w.EAG, RT_EN, k, from);
        slot_add(w, w.LAZ, RT_LN, k, from);
    }
}

// send/3 (pt:633-638) -> forward_message (hv:441-460) -> do_send_message
// without maybe_connect: only over an existing connection of the manager (an
// active member, or a lingering peer)
DEV bool pt_conn(const Wv& w, uint32_t ident) {
    uint32_t id = ident & ~PSIM_MAP_BIT;
    return id != w.me && conn_has(w, id) && connect_ok(w, id);
}
DEV void pt_send(Wv& w, uint32_t ident, uint32_t type, uint32_t msg, uint32_t rnd, uint32_t root) {
    if (!pt_conn(w, ident)) {
        st_add(w, ST_FAIL, 1);
        return;
    }
    emit(w, ident & ~PSIM_MAP_BIT, type, 0, msg, rnd, root, 0, 0);
}

// Batched sends of one handler: the lanes of `cand` (ascending = the
// reference's list order) each hold a peer identity; returns the lanes whose
// send/3 finds a connection -- the peer in the active view, running, same
// partition (k_pt's cache lanes 32-39 are its active view) -- and counts a
// send failure for each of the others.
DEV uint64_t pt_conn_mask(Wv& w, uint64_t cand, uint32_t IDENT) {
    const uint32_t l = lane_id(), id = IDENT & ~PSIM_MAP_BIT;
    uint32_t fl = 0;
    bool in = false;
    for (uint32_t j = 0; j < w.act_n; j++) {          // (has/3 + the cache lookup of connect_ok)
        const uint32_t aj = rl(w.A, j), cj = rl(w.CF, 32 + j);
        const bool hit = aj == id;
        in |= hit;
        fl = hit ? cj : fl;
    }
    // the connection table (cache lanes 40..: its entries at phase start,
    // unchanged in the Plumtree phase): an active member marked down has no
    // connection, a lingering peer has one
    for (uint32_t j = 0; j < w.conn_n; j++) {
        const uint32_t ej = rl(w.CN, j), cj = rl(w.CF, 40 + j);
        in = ej == (id | PSIM_CONN_DOWN) || ej == (id | PSIM_CONN_CLOSING) ? false : in;
        const bool hit = ej == id;
        in |= hit;
        fl = hit ? cj : fl;
    }
    const bool ok = ((cand >> l) & 1ull) && in && id != w.me && id < kargs().n_nodes && (fl & F_UP) &&
                    (fl >> 8) == w.mypart;
    const uint64_t m = ballot(ok);
    st_add(w, ST_FAIL, popc(cand) - popc(m));
    return m;
}

// emit() for the lanes of `m` at once, in ascending lane order: record k
// takes dst (and, PER_LANE, a0 / a1 / a2) from the k-th lane of m; four
// records per wave step through the staging buffer (same words, digest, keys
// and stats as k emit() calls)
template <bool PER_LANE>
DEV void emit_batch(Wv& w, uint64_t m, uint32_t type, uint32_t DST, uint32_t A0, uint32_t A1, uint32_t A2) {
    const uint32_t n = popc(m);
    if (!n) return;
    const uint32_t l = lane_id(), j = l & 15, r = l >> 4;
    for (uint64_t rem = m; rem;) {
        // the next (up to) four records: lanes s0..s3 of m
        int s[4];
        uint32_t c = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            s[q] = rem ? ffs64(rem) : s[q > 0 ? q - 1 : 0];
            c += rem ? 1u : 0u;
            rem &= rem - 1;
        }
        uint32_t staged = w.seq - w.flushed;
        if (staged + c > STAGE) { flush_recs(w); staged = 0; }
        const int src = r == 0 ? s[0] : r == 1 ? s[1] : r == 2 ? s[2] : s[3];
        const uint32_t dk = shfl(DST, src);
        const uint32_t b0 = PER_LANE ? shfl(A0, src) : A0, b1 = PER_LANE ? shfl(A1, src) : A1;
        const uint32_t b2 = PER_LANE ? shfl(A2, src) : A2;
        const uint32_t word = j == 0 ? dk : j == 1 ? w.me : j == 2 ? type : j == 3 ? w.seq + r
                            : j == 4 ? b0 : j == 5 ? b1 : j == 6 ? b2 : 0u;
        if (r < c) {
            w.srec[(staged + r) * 16 + j] = word;
            w.digest += (uint64_t)word * digest_mul(j);
            if (j == 0) w.skey[staged + r] = dk | (max_emit(type) << KEY_DST_BITS);
        }
        w.seq += c;
        if (staged + c == STAGE) flush_full(w);
    }
    st_add(w, ST_EMIT + type, n);
}

DEV void pt_add_out(Wv& w, uint32_t peer, uint32_t msg, uint32_t rnd) {   // pt:574-579
    uint32_t l = lane_id();
    uint64_t key = ((uint64_t)peer << 32) | (msg << 16) | (rnd & 0xFFFFu);
    w.pt_dirty = true;
    if (ballot(l < w.out_n && w.OUT == key)) return;
    if (w.out_n < OUT_HEAD) {
        vins64(w.OUT, w.out_n, popc(ballot(l < w.out_n && w.OUT < key)), key);
        return;
    }
    // a full register: the sorted order continues in the tail
    const uint32_t nt = w.out_n - OUT_HEAD;
    uint64_t T = nt ? load_out_tail(w) : 0ull;
    if (ballot(l < nt && T == key)) return;
    if (w.out_n >= PSIM_PT_OUT_CAP) { ovf(w, PSIM_OVF_PT_OUT); return; }
    if (!w.ox) {
        w.ox = take_ext_row(w, kargs().outx_top, kargs().outx_rows, PSIM_OVF_PT_OUT);
        if (!w.ox) return;
    }
    uint32_t pos = popc(ballot(w.OUT < key));
    uint64_t into = key;
    if (pos < OUT_HEAD) {                 // the register's last entry moves to the tail's front
        into = rl64(w.OUT, OUT_HEAD - 1);
        uint32_t n = OUT_HEAD - 1;
        vins64(w.OUT, n, pos, key);
        pos = 0;
    } else {
        pos = popc(ballot(l < nt && T < key));
    }
    uint32_t n = nt;
    vins64(T, n, pos, into);
    *out_tail(w) = T;
    w.out_n++;
}

DEV void pt_ack_out(Wv& w, uint32_t peer, uint32_t msg, uint32_t rnd) {   // pt:562-567
    const uint32_t l = lane_id();
    uint64_t key = ((uint64_t)peer << 32) | (msg << 16) | (rnd & 0xFFFFu);
    int k = ffs64(ballot(l < w.out_n && w.OUT == key));
    if (w.out_n <= OUT_HEAD) {
        if (k >= 0) { vdel64(w.OUT, w.out_n, (uint32_t)k); w.pt_dirty = true; }
        return;
    }
    uint32_t nt = w.out_n - OUT_HEAD;
    uint64_t T = load_out_tail(w);
    if (k >= 0) {                         // the tail's front moves up into the register
        const uint64_t t0 = rl64(T, 0);
        uint32_t n = OUT_HEAD;
        vdel64(w.OUT, n, (uint32_t)k);
        w.OUT = l == OUT_HEAD - 1 ? t0 : w.OUT;
        k = 0;
    } else {
        k = ffs64(ballot(l < nt && T == key));
        if (k < 0) return;
    }
    vdel64(T, nt, (uint32_t)k);
    *out_tail(w) = T;
    w.out_n--;
    w.pt_dirty = true;
}

// eager_push/7 + schedule_lazy_push/6 (pt:428-441) over all_peers/3: the
// root's slot, or the common eagers (and no lazys)
DEV void pt_push(Wv& w, uint32_t msg, uint32_t rnd, uint32_t root, uint32_t from) {
    const int k = rt_find(w, root);
    if (k >= 0) {
        const uint32_t ce = rt_word(w, RT_EN), cl = rt_word(w, RT_LN);
        const uint32_t be = rt_off(ce, (uint32_t)k), bl = rt_off(cl, (uint32_t)k);
        const uint32_t ne = (ce >> (8 * k)) & 0xFFu, nl = (cl >> (8 * k)) & 0xFFu;
        // the eager sends, batched (entries of the slot: lanes be .. be + ne)
        const uint32_t l = lane_id();
        const uint64_t cand = ballot(l >= be && l < be + ne && w.EAG != from);
        emit_batch<false>(w, pt_conn_mask(w, cand, w.EAG), PSIM_MSG_PT_BROADCAST, w.EAG & ~PSIM_MAP_BIT, msg, rnd, root);
        for (uint32_t i = 0; i < nl; i++) {
            uint32_t e = rl(w.LAZ, bl + i);
            if (e != from) pt_add_out(w, e, msg, rnd);
        }
    } else {
        const uint64_t cand = ballot(lane_id() < w.com_n && w.COM != from);
        emit_batch<false>(w, pt_conn_mask(w, cand, w.COM), PSIM_MSG_PT_BROADCAST, w.COM & ~PSIM_MAP_BIT, msg, rnd, root);
    }
}

// plumtree_backend is_stale/1 (:101-104, :148-152) over the message slots; a
// retired id (its slot taken by a newer broadcast) counts an overflow and
// answers stale
DEV bool pt_have(Wv& w, uint32_t msg) {
    const uint32_t k = msg % PSIM_MSG_SLOTS;
    if (w.slots[k] != msg) { ovf(w, PSIM_OVF_PT); return true; }
    return ((k < 32 ? w.have >> k : w.aux >> (k - 32)) & 1u) != 0;
}
DEV void pt_mark(Wv& w, uint32_t msg) {
    const uint32_t k = msg % PSIM_MSG_SLOTS;
    if (k < 32) w.have |= 1u << k; else w.aux |= 1u << (k - 32);
}
// the root of a live message id (an IHAVE of an outstanding entry); a
// retired id counts an overflow and is PSIM_NONE
DEV uint32_t msg_root(Wv& w, uint32_t msg) {
    const uint32_t k = msg % PSIM_MSG_SLOTS;
    if (w.slots[k] != msg) { ovf(w, PSIM_OVF_PT); return NONE; }
    return w.slots[PSIM_MSG_SLOTS + k];
}

DEV void pt_handle(Wv& w, uint32_t type, uint32_t src, uint32_t msg, uint32_t rnd, uint32_t root) {
    uint32_t from = src | PSIM_MAP_BIT;
    switch (type) {
    case PSIM_MSG_PT_BROADCAST:                        // pt:288-293, :368-378
        if (!pt_have(w, msg)) {                        // plumtree_backend merge/2
            pt_mark(w, msg);
            st_add(w, ST_FIRST, 1);
            if (msg == kargs().tracked_msg) { w.trk_round = w.round; w.trk_hop = rnd + 1; }
            pt_update(w, from, root, true);
            pt_push(w, msg, rnd + 1, root, from);
        } else {
            pt_update(w, from, root, false);
            pt_send(w, from, PSIM_MSG_PT_PRUNE, 0, 0, root);
        }
        break;
    case PSIM_MSG_PT_PRUNE:                            // pt:294-298
        pt_update(w, from, root, false);
        break;
    case PSIM_MSG_PT_IHAVE:                            // pt:299-303, :380-386
        if (pt_have(w, msg)) {
            pt_send(w, from, PSIM_MSG_PT_IGNORED_IHAVE, msg, rnd, root);
        } else {
            pt_send(w, from, PSIM_MSG_PT_GRAFT, msg, rnd, root);
            pt_update(w, from, root, true);
        }
        break;
    case PSIM_MSG_PT_IGNORED_IHAVE:                    // pt:304-307
        pt_ack_out(w, from, msg, rnd);
        break;
    case PSIM_MSG_PT_GRAFT:                            // pt:308-313, :388-402
        if (pt_have(w, msg)) {
            pt_update(w, from, root, true);
            pt_send(w, from, PSIM_MSG_PT_BROADCAST, msg, rnd, root);
        }
        break;
    default:
        break;
    }
}

// --------------------------------------------------------------- X-BOT --
// partisan_hyparview_xbot_peer_service_manager (xbot): HyParView plus the
// optimization rounds (xbot:586-606, :691-716, :1171-1346), round model R0-X
// (the oracle's xb_*).  Every X-BOT node with X-BOT work runs
// here, in k_consume.
// net_adm:ping/1 answers pong iff the node runs (pings go over distributed
// Erlang, so a partition does not stop them); F_UP of another node does not
// change during the phase
DEV bool xb_pong(const Wv& w, uint32_t p) {
    if (p == w.me) return true;
    if (p >= kargs().n_nodes) return false;
    const uint64_t m = ballot(w.CV == p);
    const uint32_t f = m ? rl(w.CF, ffs64(m)) : (uint32_t)kargs().flags[p];
    return (f & F_UP) != 0;
}
// is_better(latency, New, Old) at this node (xbot:1318-1333)
DEV bool xb_better(const Wv& w, uint32_t nw, uint32_t old) {
    if (!xb_pong(w, nw)) return false;
    if (!xb_pong(w, old)) return true;
    const uint64_t sd = kargs().seed;
    return xbot_latency(sd, w.me, nw) < xbot_latency(sd, w.me, old);
}
// select_disconnect_node/1 + select_worst_in_active_view/2 (xbot:1336-1346)
DEV uint32_t xb_worst(const Wv& w) {
    uint32_t worst = rl(w.A, 0);
    for (uint32_t i = 1; i < w.act_n; i++) {
        const uint32_t h = rl(w.A, i);
        if (!xb_better(w, h, worst)) worst = h;
    }
    return worst;
}
// do_send_message over a maybe_connect whose result the handler drops
// (send_join/2 xbot:1349-1363 and every optimization send): out iff the peer
// can be reached, the connection table unchanged
DEV void xb_send(Wv& w, uint32_t dst, uint32_t type, uint32_t ans, uint32_t a0, uint32_t a1, uint32_t a2,
                 uint32_t a3) {
    if (conn_closing(w, dst)) { w.rng++; st_add(w, ST_FAIL, 1); return; }
    if (!connect_ok(w, dst)) { st_add(w, ST_FAIL, 1); return; }
    w.rng++;
    emit4(w, dst, type, ans, a0, a1, a2, a3, 0, 0);
}
DEV void xb_join(Wv& w, uint32_t p) { xb_send(w, p, PSIM_MSG_JOIN, 0, hw_epoch(w), 0, 0, 0); }
// do_disconnect/2 (xbot:1367-1379), its state discarded by every caller: the
// passive add's eviction draw is consumed and a live connection's pid
// stopped (PSIM_CONN_CLOSING); its 'EXIT' removes the peer next round
DEV void xb_do_disconnect(Wv& w, uint32_t p) {
    if (!has(w.A, w.act_n, p)) return;
    if (p != w.me && !has(w.P, w.pas_n, p) && w.pas_n >= kargs().max_passive) (void)uniform_n(w, w.pas_n);
    if ((!w.conn_dn || conn_find(w, p | PSIM_CONN_DOWN) < 0) && !conn_closing(w, p)) conn_add(w, p | PSIM_CONN_CLOSING);
}
// the optimization messages: a0 Old, a1 Initiator, a2 Candidate, a3
// Disconnect (NONE = undefined), ttl the answer
DEV void xb_handle(Wv& w, uint32_t type, uint32_t ans, uint32_t old, uint32_t ini, uint32_t cand, uint32_t dis) {
    switch (type) {
    case PSIM_MSG_XBOT_OPTIMIZATION:                   // xbot:1205-1224, at the candidate
        if (w.act_n < kargs().max_active) {
            xb_join(w, ini);
            xb_send(w, ini, PSIM_MSG_XBOT_OPTIMIZATION_REPLY, 1, old, ini, cand, NONE);
        } else {
            const uint32_t d = xb_worst(w);
            xb_send(w, d, PSIM_MSG_XBOT_REPLACE, 0, old, ini, cand, d);
        }
        break;
    case PSIM_MSG_XBOT_REPLACE:                        // xbot:1252-1267, at the disconnect node
        if (!xb_better(w, old, cand)) xb_send(w, cand, PSIM_MSG_XBOT_REPLACE_REPLY, 0, old, ini, cand, dis);
        else xb_send(w, old, PSIM_MSG_XBOT_SWITCH, 0, old, ini, cand, dis);
        break;
    case PSIM_MSG_XBOT_SWITCH:                         // xbot:1295-1314, at the old node
        if (has(w.A, w.act_n, ini)) {
            xb_do_disconnect(w, ini);
            xb_join(w, dis);
            xb_send(w, dis, PSIM_MSG_XBOT_SWITCH_REPLY, 1, old, ini, cand, dis);
        } else {
            xb_send(w, dis, PSIM_MSG_XBOT_SWITCH_REPLY, 0, old, ini, cand, dis);
        }
        break;
    case PSIM_MSG_XBOT_SWITCH_REPLY:                   // xbot:1270-1292, at the disconnect node
        if (ans) {
            xb_do_disconnect(w, cand);
            xb_join(w, old);
        }
        xb_send(w, cand, PSIM_MSG_XBOT_REPLACE_REPLY, ans, old, ini, cand, dis);
        break;
    case PSIM_MSG_XBOT_REPLACE_REPLY:                  // xbot:1227-1249, at the candidate
        if (ans) {
            xb_do_disconnect(w, dis);
            xb_join(w, ini);
        }
        xb_send(w, ini, PSIM_MSG_XBOT_OPTIMIZATION_REPLY, ans, old, ini, cand, dis);
        break;
    case PSIM_MSG_XBOT_OPTIMIZATION_REPLY:             // xbot:1171-1202, at the initiator
        if (!ans) break;
        if (dis != NONE && has(w.A, w.act_n, old)) xb_do_disconnect(w, old);
        xb_join(w, cand);
        break;
    default:
        break;
    }
}
// handle_info(xbot_execution) (xbot:587-606, :691-716): with a full active
// view, two passive candidates, each checked against the active members in
// to_list order; the first one it beats gets an optimization message
DEV void xb_execute(Wv& w) {
    if (w.act_n < kargs().max_active) return;
    uint32_t C = 0;
    const uint32_t nc = sublist(w, w.P, w.pas_n, 2, C, 0);
    const uint32_t A0 = w.A, na = w.act_n;
    for (uint32_t i = 0; i < nc; i++) {
        const uint32_t c = rl(C, i);
        for (uint32_t j = 0; j < na; j++) {
            const uint32_t old = rl(A0, j);
            if (xb_better(w, c, old)) {
                xb_send(w, c, PSIM_MSG_XBOT_OPTIMIZATION, 0, old, w.me, c, NONE);
                break;
            }
        }
    }
}

// ----------------------------------------------------------- hyparview --
DEV void hv_handle(Wv& w, uint32_t type, uint32_t p, uint32_t ttl, uint32_t a0, uint32_t a1,
                   uint32_t a2, uint32_t a3, uint32_t EX, uint32_t nex) {
    KArgs& a = kargs();
    uint32_t me = w.me;
    switch (type) {
    case PSIM_MSG_JOIN:                                // hv:703-771
        if (addable_epoch(w, a0, p) && !has(w.A, w.act_n, p) && maybe_connect(w, p)) {   // :721-723
            add_to_active(w, p);
            hv_send(w, p, PSIM_MSG_NEIGHBOR, 0, current_id(w, p), 0, 0, 0);
            // (members(Active) -- [Myself]) -- [Peer], in to_list order
            for (uint32_t i = 0; i < w.act_n; i++) {
                uint32_t q = rl(w.A, i);
                if (q == me || q == p) continue;
                if (a.xbot) xb_send(w, q, PSIM_MSG_FORWARD_JOIN, a.arwl, p, a0, 0, 0);   // xbot:765-786:
                else hv_send(w, q, PSIM_MSG_FORWARD_JOIN, a.arwl, p, a0, 0, 0);          // the fold's dict dropped
            }
            notify(w);
        }
        break;
    case PSIM_MSG_NEIGHBOR:                            // hv:774-805
        if (addable_id(w, a0, p) && maybe_connect(w, p)) add_to_active(w, p);   // :784-786
        notify(w);
        break;
    case PSIM_MSG_FORWARD_JOIN: {                      // hv:808-923
        uint32_t q = a0, pe = a1, sender = p;
        if (ttl == 0 || w.act_n == 1) {
            if (addable_epoch(w, pe, q) && !has(w.A, w.act_n, q) && maybe_connect(w, q)) {
                add_to_active(w, q);
                hv_send(w, q, PSIM_MSG_NEIGHBOR, 0, current_id(w, q), 0, 0, 0);
            }
        } else {
            // the passive add at TTL == prwl never changes the active view,
            // so the live active row is Active0 for the select and the test
            const uint32_t P_s = w.P, np_s = w.pas_n;  // State0's passive view
            if (ttl == a.prwl) add_to_passive(w, q);    // State2 (hv:859-866)
            uint32_t r = select_random(w, w.A, w.act_n, sender, me, q);
            if (r == NONE) {
                if (addable_epoch(w, pe, q) && !has(w.A, w.act_n, q)) {
                    if (maybe_connect(w, q)) {                 // :878-880
                        add_to_active(w, q);
                        hv_send(w, q, PSIM_MSG_NEIGHBOR, 0, current_id(w, q), 0, 0, 0);
                    } else if (!a.xbot) {
                        // {error, not_found} -> State0 (hv:896-897): the insert
                        // is discarded, its eviction draw stays consumed
                        // (X-BOT keeps State2, xbot:921-922)
                        w.P = P_s; w.pas_n = np_s;
                    }
                }
            } else {
                hv_send(w, r, PSIM_MSG_FORWARD_JOIN, ttl - 1, q, pe, 0, 0);
            }
        }
        notify(w);
        break;
    }
    case PSIM_MSG_DISCONNECT: {                        // hv:926-972
        if (!valid_disconnect(w, p, a0)) break;
        vdel_val(w.A, w.act_n, p);
        if (w.conn_dn) conn_del(w, p | PSIM_CONN_DOWN);
        w.vd |= 1u;
        uint32_t P0 = w.P, np0 = w.pas_n;              // Passive before the add
        add_to_passive(w, p);
        map_store(w, w.RP, w.RI, w.recv_n, w.recv_head, p, a0);
        disconnect(w, p);                              // :952
        if (w.act_n == 1) move_to_active(w, select_random(w, P0, np0, me, p, me));
        break;
    }
    case PSIM_MSG_NEIGHBOR_REQUEST: {                  // hv:975-1053
        uint32_t ACK;
        const bool conn = maybe_connect(w, p);         // :987, kept in both branches
        uint32_t nack = build_exchange(w, ACK);
        if (addable_id(w, a0, p)) {                    // priority is always high (:1706)
            if (conn || a.xbot) {                      // (X-BOT: no find, xbot:1026-1045)
                hv_send(w, p, PSIM_MSG_NEIGHBOR_ACCEPTED, 0, current_id(w, p), 0, ACK, nack);
                add_to_active(w, p);
            }
        } else {
            hv_send(w, p, PSIM_MSG_NEIGHBOR_REJECTED, 0, 0, 0, ACK, nack);
        }
        merge_exchange(w, EX, nex);
        notify(w);
        break;
    }
    case PSIM_MSG_NEIGHBOR_REJECTED:                   // hv:1056-1067
        disconnect(w, p);                              // :1063
        merge_exchange(w, EX, nex);
        break;
    case PSIM_MSG_NEIGHBOR_ACCEPTED:                   // hv:1070-1089
        if (addable_id(w, a0, p)) add_to_active(w, p);
        merge_exchange(w, EX, nex);
        notify(w);
        break;
    case PSIM_MSG_SHUFFLE_REPLY:                       // hv:1091-1093
        merge_exchange(w, EX, nex);
        break;
    case PSIM_MSG_SHUFFLE:                             // hv:1095-1136
        if (ttl > 0 && w.act_n > 1) {
            uint32_t r = select_random(w, w.A, w.act_n, p, me, me);
            if (r != NONE) hv_send(w, r, PSIM_MSG_SHUFFLE, ttl - 1, 0, 0, EX, nex);
            STAMP(w, 25);
        } else {
            uint32_t RESP = 0;
            uint32_t nr = sublist(w, w.P, w.pas_n, nex, RESP, 0);
            STAMP(w, 26);
            hv_send(w, p, PSIM_MSG_SHUFFLE_REPLY, 0, 0, 0, RESP, nr);
            STAMP(w, 27);
            merge_exchange(w, EX, nex);
            STAMP(w, 28);
        }
        break;
    default:
        if (type >= PSIM_MSG_XBOT_OPTIMIZATION && a.xbot) xb_handle(w, type, ttl, a0, a1, a2, a3);
        break;
    }
}

DEV bool timer_due(uint32_t period, uint32_t r, uint32_t start) {
    return period > 0 && r > start && ((r - start) % period) == 0;
}

// Inbox chunk c (messages c..c+3 of the node's dense run): lane l loads
// word l&15 of message c + (l>>4), one 256-B load instruction per chunk.
DEV uint32_t load_chunk(KArgs& a, uint32_t ib, uint32_t ik, uint32_t c) {
    uint32_t l = lane_id();
    return (c + (l >> 4) < ik) ? reinterpret_cast<const uint32_t*>(a.rec_in + ib + c + (l >> 4))[l & 15]
                               : 0u;
}

// chunk c (a multiple of 4) of the node's inbox: the first from the first
// input stage, any later one loaded
DEV uint32_t inbox_chunk(const Wv& w, KArgs& a, uint32_t ib, uint32_t ik, uint32_t c, uint32_t R0) {
    return c == 0 ? R0 : load_chunk(a, ib, ik, c);
}

// The HyParView kernel's inputs arrive in two stages, each issued one step
// ahead with every lane loading (lanes beyond a row re-read an element of
// it), so every node issues the same vector memory operations:
//   NodeIn (rows, from the work descriptor): header, active and passive
//          views, the first inbox chunk, the node's flag and partition bytes;
//   NodeX  (needs the rows): flag/partition bytes of every view member (the
//          connection cache).
// The disconnect-id maps are loaded on first use (load_maps).
// The Plumtree rows are not staged: the Plumtree phase runs in k_pt; this
// kernel reads them only to replay notifies (load_pt_rows).
struct NodeIn {
    uint32_t n, ib, ik, ob, tf;    // tf: due timers (DESC_* bits, k_desc)
    bool maps;                     // DESC_MAPS_BIT (k_relay)
    bool xb;                       // DESC_XBOT_BIT: X-BOT's xbot_execution is due (k_desc)
    uint32_t H;                    // header word l & 15
    uint32_t A, P, R0;
    uint32_t CN;                   // connection-table entry l & 7 (k_consume_lite: 0)
    uint32_t fl, part;
};
struct NodeX {
    uint32_t CV, CF;               // view ids (passive 0-31, active 32-39, connection table
                                   // 40-47), their flags | part << 8
};

DEV uint32_t load_desc(KArgs& a, uint32_t k) {
    uint32_t l = lane_id();
    return reinterpret_cast<const uint32_t*>(a.desc + k)[l & 3];
}

template <bool CONN = true>
DEV NodeIn load_node(KArgs& a, uint32_t D) {
    uint32_t l = lane_id();
    NodeIn x;
    x.n = rl(D, 0); x.ib = rl(D, 1); x.ik = rl(D, 2) & DESC_CNT_MASK; x.tf = rl(D, 2) >> 28; x.ob = rl(D, 3);
    x.maps = (rl(D, 2) & DESC_MAPS_BIT) != 0;
    x.xb = (rl(D, 2) & DESC_XBOT_BIT) != 0;
    const size_t li = x.n - a.lo;
    x.H = reinterpret_cast<const uint32_t*>(a.hdr + li)[l & 15];
    x.A = a.act[li * PSIM_ACTIVE_CAP + (l & 7)];
    x.P = a.pas[li * PSIM_PASSIVE_CAP + (l & 31)];
    uint32_t m = x.ik ? min(l >> 4, x.ik - 1) : 0u;  // record ib exists (the inbox has one spare)
    x.R0 = reinterpret_cast<const uint32_t*>(a.rec_in + x.ib + m)[l & 15];
    x.CN = CONN ? a.conn[li * PSIM_CONN_CAP + (l & 7)] : 0u;
    x.fl = a.flags[x.n];
    x.part = a.part[x.n];
    return x;
}

// the connection-table entry in cache lane 40 + j (j < conn_n, else NONE):
// the peer of a lingering connection; NONE for a member marked down.  Every
// lane must call it (a shuffle reads lanes 0-7: a lane outside the exec
// mask reads as 0)
DEV uint32_t conn_cache_id(uint32_t CN, uint32_t H) {
    const uint32_t l = lane_id(), cn = rl(H, HW_CONN) & 0xFF;
    const uint32_t e = shfl(CN, (int)(l & 7));
    return l >= 40 && l < 48 && l - 40 < cn && !(e & (PSIM_CONN_DOWN | PSIM_CONN_CLOSING)) ? e : NONE;
}

// flag | partition << 8 of the view members in CV (the connection cache)
// (the passive lanes from the up-and-partition pairs, one read each
// instead of a flag byte and a partition byte, measured slower at 2^26: E
// 75.6 -> 76.1 ms a round with 2-B pairs, 75.0 -> 75.4 with 1-B pairs
// (k_consume -0.1 ms, k_pt +0.2); profiles/r05/ab_log.txt r5v, r5x)
DEV uint32_t cache_flags(KArgs& a, uint32_t cv, uint32_t me) {
    const uint32_t ca = cv < a.n_nodes ? cv : me;
    const uint32_t f = a.flags[ca], pt = a.part[ca];
    return cv < a.n_nodes ? (f | (pt << 8)) : 0u;
}

template <bool LITE = false>
DEV NodeX load_x(KArgs& a, const NodeIn& x) {
    uint32_t l = lane_id();
    NodeX y;
    const uint32_t hw9 = rl(x.H, 9);                 // act_n, pas_n, .. (Hdr word 9)
    const uint32_t act_n = hw9 & 0xFF, pas_n = (hw9 >> 8) & 0xFF;
    uint32_t av = shfl(x.A, (int)(l & 7));
    // (LITE: k_consume_lite's handlers only send to active members and to
    // senders -- no passive-member entries)
    uint32_t cv = l < 32 ? (!LITE && l < pas_n ? x.P : NONE) : (l < 40 && l - 32 < act_n ? av : NONE);
    if (!LITE) {                                     // (uniform: every lane runs the shuffle)
        const uint32_t cc = conn_cache_id(x.CN, x.H);
        cv = l >= 40 ? cc : cv;
    }
    y.CV = cv;
    y.CF = cache_flags(a, cv, x.n);
    return y;
}

// the Plumtree rows of the running node (all_members | common_eagers | root
// row, per-root eager and lazy sets, outstanding) into the wave's registers
DEV void load_pt_regs(Wv& w, uint32_t PA, uint32_t PG, uint32_t PL, uint64_t PO) {
    const uint32_t l = lane_id();
    const uint32_t c8 = shfl(PA, (int)((l + 8) & 63));   // lanes 0-7: com (8-15); lanes 8-15: the root row (16-23)
    w.AR = l < RTB ? PA : (l < RTB + RT_WORDS ? c8 : 0u);
    w.COM = l < PSIM_PT_MEMBERS_CAP ? c8 : 0u;
    w.EAG = PG; w.LAZ = PL;
    w.OUT = PO;
    w.pt = true;
}
// outstanding entry l of the node (its row, then its extension row: one
// 8-B load per lane either way)
DEV uint64_t load_po(KArgs& a, size_t li, uint32_t ox) {
    const uint32_t l = lane_id();
    const bool own = l < OUT_IN;
    const uint64_t* p = own || !ox ? a.pt_out + li * OUT_IN + (l & (OUT_IN - 1))
                                   : a.outx + (size_t)(ox - 1) * OUT_EXT + (l - OUT_IN);
    const uint64_t v = *p;
    return own || ox ? v : 0ull;
}
// lanes 0-7 pt_all, 8-15 pt_com, 16-23 the root row (and again above 24)
DEV uint32_t load_pa(KArgs& a, size_t li) {
    const uint32_t l = lane_id();
    return ((l & 31) < 8 ? a.pt_all + li * PSIM_PT_MEMBERS_CAP
                         : (l & 31) < 16 ? a.pt_com + li * PSIM_PT_MEMBERS_CAP : a.pt_rt + li * RT_WORDS)[l & 7];
}
DEV void load_pt_rows(Wv& w) {
    KArgs& a = kargs();
    const uint32_t l = lane_id();
    const size_t li = w.li;
    load_pt_regs(w, load_pa(a, li), a.pt_eag[li * RT_SET + l], a.pt_laz[li * RT_SET + l], load_po(a, li, w.ox));
}

// the header words of the node into the wave's scalars
DEV void begin_header(Wv& w, uint32_t H) {
    w.start_round = rl(H, 2); w.contact = rl(H, 3); w.epoch = rl(H, 4);
    w.rng = ((uint64_t)rl(H, 1) << 32) | rl(H, 0);
    w.aux = rl(H, 5); w.have = rl(H, 6); w.trk_round = rl(H, 7); w.trk_hop = rl(H, 8);
    const uint32_t w9 = rl(H, 9), w10 = rl(H, 10), w11 = rl(H, 11);
    w.act_n = w9 & 0xFF; w.pas_n = (w9 >> 8) & 0xFF; w.sent_n = (w9 >> 16) & 0xFF; w.sent_head = w9 >> 24;
    w.recv_n = w10 & 0xFF; w.recv_head = (w10 >> 8) & 0xFF; w.all_n = (w10 >> 16) & 0xFF; w.com_n = w10 >> 24;
    w.out_n = (w11 >> 16) & 0xFF;
    w.conn_n = w11 & 0xFF; w.conn_dn = (w11 >> 8) & 0xFF; w.conn_cl = w11 >> 24;
    w.sx = rl(H, HW_SENT_EXT); w.rx = rl(H, HW_RECV_EXT); w.ox = rl(H, HW_OUT_EXT);
}

// node state and the per-node scratch of the wave, from the staged inputs
DEV void begin_node(Wv& w, const NodeIn& x, const NodeX& y) {
    const uint32_t l = lane_id();
    w.li = x.n - kargs().lo;
    w.me = x.n;
    begin_header(w, x.H);
    w.vd = 0;
    w.A = l < PSIM_ACTIVE_CAP ? x.A : 0u;
    w.P = l < PSIM_PASSIVE_CAP ? x.P : 0u;
    w.fl = x.fl;
    w.obase = x.ob;
    w.mypart = x.part;
    w.CV = y.CV; w.CF = y.CF;
    w.CN = l < w.conn_n ? x.CN : 0u;
    w.cn_dirty = false;
    w.maps = false; w.pt = false; w.maps_dirty = false; w.pt_dirty = false;
    w.seq = 0; w.flushed = 0;
    w.nlog_n = 0;
    w.dc_base = NONE64;                                // the cache holds another node's stream
    w.work = false;
    w.lazy_quiet = false;
}

// The node's HyParView handlers in the order of round model R0, then the
// replay of its notifies into the Plumtree state.  No global store.  The
// Plumtree inbox, origin and lazy tick follow in k_pt.
DEV void body_hv(Wv& w, const NodeIn& x) {
    KArgs& a = kargs();
    const uint32_t r = a.round;
    const uint32_t l = lane_id();
    const uint32_t n = x.n;
    uint32_t ik = x.ik;
    const uint32_t ib = x.ib;
    const uint32_t R0 = x.R0;
    if (hw_start(w) == r && ik) {           // fresh incarnation: no connections yet
        st_add(w, ST_DROPPED, ik);
        ik = 0;
    }
    bool promo = (x.tf & DESC_PROMO) != 0;
    bool shuf = (x.tf & DESC_SHUFFLE) != 0;
    bool origin = (x.tf & DESC_ORIGIN) != 0;
    bool lazy = (x.tf & DESC_LAZY) != 0 && w.out_n > 0;
    bool joining = hw_start(w) == r && hw_contact(w) != NONE;
    // EXIT (hv:609-654) at every holder of a connection to a peer that
    // crashed this round (App. A Q11): the connected active members (cache
    // lanes 32-39, less those marked down), then the lingering peers (40-47)
    uint64_t exits = 0, lexits = 0;
    if (a.crash_round) {
        bool dead = l >= 32 && l < 40 && l - 32 < w.act_n && w.CV != n && (w.CF & F_CRASHED);
        for (uint32_t j = 0; j < w.conn_n && (w.conn_dn || w.conn_cl); j++)
            dead &= rl(w.CN, j) != (w.CV | PSIM_CONN_DOWN) && rl(w.CN, j) != (w.CV | PSIM_CONN_CLOSING);
        exits = (ballot(dead) >> 32) & 0xFFull;
        lexits = (ballot(l >= 40 && l < 48 && w.CV != NONE && (w.CF & F_CRASHED)) >> 40) & 0xFFull;
    }
    bool promo_work = promo && w.act_n < a.min_active;
    const uint32_t ncl = w.conn_cl;                   // X-BOT: connection pids stopped last round
    if (!(ik || joining || exits || lexits || ncl || promo_work || shuf || x.xb || origin || lazy)) { STAMP(w, 0); return; }
    w.work = true;
    st_add(w, ST_PROC, 1);
    if (x.maps) load_maps(w);                         // (k_relay: a handler here may use them)
    STAMP(w, 1);

    if (joining)                                      // hv:500-515
        hv_send(w, hw_contact(w), PSIM_MSG_JOIN, 0, hw_epoch(w), 0, 0, 0);

    if (ncl) {                                        // X-BOT: their 'EXIT's (xbot:608-653), table order
        const uint64_t cm = ballot(l < w.conn_n && (w.CN & PSIM_CONN_CLOSING));
        const uint32_t D = compact(w, w.CN & ~PSIM_CONN_CLOSING, cm);
        const uint32_t nd = popc(cm);
        for (uint32_t i = 0; i < nd; i++) {
            const uint32_t d = rl(D, i);
            st_add(w, ST_EXITS, 1);
            conn_del(w, d | PSIM_CONN_CLOSING);
            if (vdel_val(w.P, w.pas_n, d)) w.vd |= 2u;
            if (vdel_val(w.A, w.act_n, d)) {
                w.vd |= 1u;
                move_to_active(w, select_random(w, w.P, w.pas_n, n, n, n));
            }
        }
    }

    if (exits | lexits) {                             // hv:609-654
        // the crashed peers, listed before any handler runs: the active
        // members in to_list order, then the lingering peers in table order
        // (from the cache's copy of the active view at node start: the
        // X-BOT EXITs above may have shifted w.A)
        const uint32_t AV = shfl(w.CV, (int)((l + 32) & 63));
        uint32_t D = compact(w, AV, exits);
        const uint32_t na = popc(exits);
        const uint32_t LV = shfl(w.CV, (int)((l + 40) & 63));
        const uint32_t LD = compact(w, LV, lexits);
        const uint32_t LS = shfl(LD, (int)((l - na) & 63));   // (every lane: a lane outside
        D = l >= na ? LS : D;                                    //  the exec mask reads as 0)
        const uint32_t nd = na + popc(lexits);
        for (uint32_t i = 0; i < nd; i++) {
            uint32_t d = rl(D, i);
            st_add(w, ST_EXITS, 1);
            if (w.conn_n) conn_del(w, d);             // the connection is pruned
            if (vdel_val(w.P, w.pas_n, d)) w.vd |= 2u;
            if (vdel_val(w.A, w.act_n, d)) {
                w.vd |= 1u;
                move_to_active(w, select_random(w, w.P, w.pas_n, n, n, n));
            }
        }
    }

    STAMP(w, 2);
    for (uint32_t c = 0; c < ik; c += 4) {            // HyParView inbox, canonical order
        uint32_t R4 = inbox_chunk(w, a, ib, ik, c, R0);
        uint32_t cm = ik - c < 4 ? ik - c : 4;
        for (uint32_t q = 0; q < cm; q++) {
            uint32_t b = q * 16;
            uint32_t tt = rl(R4, b + 2), type = tt & 0xFF;
            if (type >= PSIM_MSG_PT_BROADCAST && type < PSIM_MSG_XBOT_OPTIMIZATION) continue;
            st_add(w, ST_DELIV + type, 1);
            uint32_t nex = (tt >> 16) & 0xFF;
            uint32_t ex = shfl(R4, (int)((b + 8 + l) & 63));
            ex = l < nex ? ex : 0u;
            STAMP(w, 3);
            hv_handle(w, type, rl(R4, b + 1), (tt >> 8) & 0xFF, rl(R4, b + 4), rl(R4, b + 5), rl(R4, b + 6),
                      rl(R4, b + 7), ex, nex);
            STAMP(w, 4 + type);
        }
    }

    STAMP(w, 3);
    if (promo && w.act_n < a.min_active)              // hv:542-561
        move_to_active(w, select_random(w, w.P, w.pas_n, n, n, n));
    STAMP(w, 13);
    if (shuf) {                                       // hv:572-607
        uint32_t EX;
        uint32_t nex = build_exchange(w, EX);
        uint32_t t = select_random(w, w.A, w.act_n, n, n, n);
        if (t != NONE) hv_send(w, t, PSIM_MSG_SHUFFLE, a.arwl, 0, 0, EX, nex);
    }
    if (x.xb) xb_execute(w);                          // xbot:587-606
    STAMP(w, 14);
    if (a.plumtree) replay_notifies(w);
    STAMP(w, 15);
}

// the header word l & 15 from the wave's scalars
DEV uint32_t header_word(const Wv& w, uint32_t k) {
    uint32_t v = 0;                                  // pad words: 0 on a HyParView handle
    v = k == 0 ? (uint32_t)w.rng : v;
    v = k == 1 ? (uint32_t)(w.rng >> 32) : v;
    v = k == 2 ? w.start_round : v;
    v = k == 3 ? w.contact : v;
    v = k == 4 ? w.epoch : v;
    v = k == 5 ? w.aux : v;
    v = k == 6 ? w.have : v;
    v = k == 7 ? w.trk_round : v;
    v = k == 8 ? w.trk_hop : v;
    v = k == 9 ? (w.act_n | (w.pas_n << 8) | (w.sent_n << 16) | (w.sent_head << 24)) : v;
    v = k == 10 ? (w.recv_n | (w.recv_head << 8) | (w.all_n << 16) | (w.com_n << 24)) : v;
    v = k == 11 ? (w.conn_n | (w.conn_dn << 8) | (w.out_n << 16) | (w.conn_cl << 24)) : v;
    v = k == HW_SENT_EXT ? w.sx : v;
    v = k == HW_RECV_EXT ? w.rx : v;
    v = k == HW_OUT_EXT ? w.ox : v;
    return v;
}

// the Plumtree rows of the wave back (a rare branch in the HyParView
// kernel: only after a notify replay)
DEV void store_pt_rows(Wv& w) {
    KArgs& a = kargs();
    const uint32_t l = lane_id();
    const size_t li = w.li;
    uint32_t all = shfl(w.AR, (int)(l & 7)), com = shfl(w.COM, (int)(l & 7)), rt = shfl(w.AR, (int)(RTB + (l & 7)));
    const uint32_t l31 = l & 31;
    uint32_t* p1 = (l31 < 8 ? a.pt_all + li * PSIM_PT_MEMBERS_CAP
                            : l31 < 16 ? a.pt_com + li * PSIM_PT_MEMBERS_CAP : a.pt_rt + li * RT_WORDS) + (l & 7);
    *p1 = l31 < 8 ? all : l31 < 16 ? com : rt;
    a.pt_eag[li * RT_SET + l] = w.EAG;
    a.pt_laz[li * RT_SET + l] = w.LAZ;
    // outstanding: own entries, the extension row (lanes without one
    // rewrite the header's draw counter)
    const bool own = l < OUT_IN;
    uint64_t* po = own ? a.pt_out + li * OUT_IN + l
                       : w.ox ? a.outx + (size_t)(w.ox - 1) * OUT_EXT + (l - OUT_IN)
                              : reinterpret_cast<uint64_t*>(a.hdr + li);
    *po = own || w.ox ? w.OUT : w.rng;
}

// an extension row (+ 1) of a pool; 0 with the pool exhausted (an overflow
// of `kind`: the table keeps its own entries)
DEV uint32_t take_ext_row(Wv& w, uint32_t* top, uint32_t rows, int kind) {
    uint32_t r = 0;
    if (lane_id() == 0) r = atomicAdd(top, 1u);
    r = uni(r);
    if (r >= rows) { ovf(w, kind); return 0; }
    return r + 1;
}
// the outstanding table outgrew its own row (the pool exhausted: the
// overflow is counted and the entries past the row are dropped)
DEV void out_ext(Wv& w) {
    if (w.pt_dirty && w.out_n > OUT_IN && !w.ox) {
        w.ox = take_ext_row(w, kargs().outx_top, kargs().outx_rows, PSIM_OVF_PT_OUT);
        if (!w.ox) w.out_n = OUT_IN;
    }
}

DEV uint8_t flag_byte(const Wv& w) {
    return (uint8_t)((w.fl & (F_UP | F_CRASHED)) | (w.out_n && !w.lazy_quiet ? F_LAZY : 0) |
                     (min(w.out_n, 15u) << F_OUTN_SHIFT) |
                     (w.act_n < kargs().min_active ? F_LOWACT : 0));
}

// Write back the node: a fixed set of full-wave stores (each lane past a
// row's end repeats one of its elements; a row that did not change is
// "stored" as a rewrite of header word 0 with its own value), then the
// staged records.  10 vector memory operations for every node, the Plumtree
// rows too after a notify replay.
DEV void writeback(Wv& w) {
    KArgs& a = kargs();
    const uint32_t l = lane_id();
    const size_t li = w.li;
    const uint32_t h0 = (uint32_t)w.rng;
    if (w.maps_dirty) {                               // a map outgrew its own rows
        if (w.sent_n > IDMAP_IN && !w.sx) w.sx = take_ext_row(w, a.mapx_top, a.mapx_rows, PSIM_OVF_IDMAP);
        if (w.recv_n > IDMAP_IN && !w.rx) w.rx = take_ext_row(w, a.mapx_top, a.mapx_rows, PSIM_OVF_IDMAP);
    }
    out_ext(w);
    uint32_t* hrow = reinterpret_cast<uint32_t*>(a.hdr + li);
    hrow[l & 15] = header_word(w, l & 15);
    {
        bool dirty = (w.vd & 1u) != 0;
        uint32_t x = shfl(w.A, (int)(l & 7));
        *(dirty ? a.act + li * PSIM_ACTIVE_CAP + (l & 7) : hrow) = dirty ? x : h0;
    }
    {
        bool dirty = (w.vd & 2u) != 0;
        uint32_t x = shfl(w.P, (int)(l & 31));
        *(dirty ? a.pas + li * PSIM_PASSIVE_CAP + (l & 31) : hrow) = dirty ? x : h0;
    }
    {
        // own entries, then the extension rows (lanes without a row: the
        // header's draw counter rewritten)
        const bool own = l < IDMAP_IN;
        const bool ds = w.maps_dirty && (own || w.sx), dr = w.maps_dirty && (own || w.rx);
        const size_t io = li * IDMAP_IN + (l & (IDMAP_IN - 1));
        const size_t so = w.sx ? (size_t)(w.sx - 1) * IDMAP_EXT + ((l - IDMAP_IN) & 63) : 0;
        const size_t ro = w.rx ? (size_t)(w.rx - 1) * IDMAP_EXT + ((l - IDMAP_IN) & 63) : 0;
        uint64_t* h64 = reinterpret_cast<uint64_t*>(hrow);   // (the draw counter, rewritten)
        *(ds ? (own ? a.sentm + io : a.mapx + so) : h64) = ds ? (((uint64_t)w.SI << 32) | w.SP) : w.rng;
        *(dr ? (own ? a.recvm + io : a.mapx + ro) : h64) = dr ? (((uint64_t)w.RI << 32) | w.RP) : w.rng;
    }
    {
        // the connection table (a fixed store: unchanged, it rewrites the
        // header's word 0)
        const uint32_t x = shfl(w.CN, (int)(l & 7));
        *(w.cn_dirty ? a.conn + li * PSIM_CONN_CAP + (l & 7) : hrow) = w.cn_dirty ? x : h0;
    }
    if (w.pt_dirty) store_pt_rows(w);
    a.ocnt[li] = w.seq;
    // (the next node's base, loaded here: in the input stages its register
    // cost more than the wait, measured)
    st_add(w, ST_BOUND, w.seq > a.obase[li + 1] - w.obase ? 1u : 0u);   // (checked by the engine)
    // only this wave writes its node's flag byte; peers read F_UP/F_CRASHED
    a.flags[w.me] = flag_byte(w);
    flush_recs(w);
    STAMP(w, 23);
}

// one HyParView-phase wave per node of the list (k_relay leaves here every
// node whose HyParView work is more than one SHUFFLE relay)
__global__ void __launch_bounds__(256, PSIM_WAVES_PER_SIMD) k_consume(RoundArgs args) {
    if (*kargs().ctl) return;                         // an aborted batch (run_batch)
    __shared__ uint64_t sst[NST];
    __shared__ uint32_t scratch[WAVES_PER_BLOCK][64];
    __shared__ uint32_t nlogs[WAVES_PER_BLOCK][NLOG * (PSIM_ACTIVE_CAP + 1)];
    __shared__ __attribute__((aligned(16))) uint32_t srecs[WAVES_PER_BLOCK][STAGE * 16];
    __shared__ uint32_t skeys[WAVES_PER_BLOCK][STAGE];
    for (int i = threadIdx.x; i < NST; i += blockDim.x) sst[i] = 0;
    __syncthreads();

    const uint32_t wid = threadIdx.x >> 6;
    const uint32_t gw = uni(blockIdx.x * WAVES_PER_BLOCK + wid);
    const uint32_t nw = gridDim.x * WAVES_PER_BLOCK;
    Wv w;
    w.a = &args;
    w.lds = scratch[wid];
    w.nlog = nlogs[wid];
    w.srec = srecs[wid];
    w.skey = skeys[wid];
    w.slots = nullptr;
#ifdef PSIM_STAMPS
    __shared__ uint64_t stamps[WAVES_PER_BLOCK][32];
    if ((threadIdx.x & 63) < 32) stamps[wid][threadIdx.x & 63] = 0;
    w.stl = stamps[wid];
    w.t_last = __builtin_amdgcn_s_memtime();
#endif
    w.st = sst;
    w.round = kargs().round;
    w.SC = 0;
    w.digest = 0;
    w.KM = magic_lanes();
    const uint32_t na = *kargs().n_alist;
    if (gw < na) {
        // Pipeline over this wave's nodes i, i + nw, ...: while node i is
        // processed, the rows of node i + nw are in flight; after its body the
        // second-stage loads of node i + nw go out, then node i's stores, then
        // the rows of node i + 2nw.  Every node issues the same loads and
        // stores, so each wait is for exactly the stage it needs.
        const uint32_t last = na - 1;
        NodeIn x = load_node(kargs(), load_desc(kargs(), gw));
        NodeX y = load_x(kargs(), x);
        NodeIn xn = load_node(kargs(), load_desc(kargs(), min(gw + nw, last)));
        uint32_t d = load_desc(kargs(), min(gw + 2 * nw, last));
        for (uint32_t i = gw; i < na; i += nw) {
            STAMP(w, 24);
            begin_node(w, x, y);
            body_hv(w, x);
            NodeX yn = load_x(kargs(), xn);
            writeback(w);
            NodeIn xnn = load_node(kargs(), d);
            d = load_desc(kargs(), min(i + 3 * nw, last));
            x = xn; y = yn; xn = xnn;
        }
    }
#ifdef PSIM_STAMPS
    if (lane_id() < 32) atomicAdd(&g_stamps[lane_id()], (unsigned long long)w.stl[lane_id()]);
#endif
    flush_wave_stats(w, sst);
    __syncthreads();
    for (int i = threadIdx.x; i < NST; i += blockDim.x)
        kargs().stat_part[(size_t)blockIdx.x * NST + i] = sst[i];
}

// ------------------------------------------------ shuffle-exchange phase --
// k_consume_lite: the same wave-per-node pipeline for the nodes k_relay
// finds whose HyParView phase is SHUFFLE walks and their replies only -- a
// SHUFFLE that ends here (hv:1095-1136 with TTL 0 or |active| = 1: the reply
// sublist(Passive, |Exchange|), then merge_exchange), a SHUFFLE_REPLY
// (hv:1091-1093: merge_exchange), any SHUFFLE relays among them, then a due
// shuffle start (hv:572-607) -- with nothing else (no join, EXIT, promotion,
// other message type).  These handlers change only the passive view and the
// draw counter, never the active view (no notify) or an id map, and send
// only to active members and to a message's sender, so the kernel carries
// a fraction of k_consume's live state and runs at twice its occupancy: in
// the rounds after a cohort's shuffle starts, most of k_consume's list was
// these nodes.  Same handlers (hv_handle), draws, records and stats.
DEV void body_lite(Wv& w, const NodeIn& x) {
    KArgs& a = kargs();
    const uint32_t l = lane_id();
    // (k_relay sends here only nodes with no active member marked down whose
    // walks end at a Sender in the active view: every send goes to an active
    // member over its connection, so the connection table is neither read
    // nor written -- nor is header word 11)
    w.conn_n = 0; w.conn_dn = 0; w.conn_cl = 0;
    w.work = true;
    st_add(w, ST_PROC, 1);
    STAMP(w, 1);
    for (uint32_t c = 0; c < x.ik; c += 4) {          // HyParView inbox, canonical order
        uint32_t R4 = inbox_chunk(w, a, x.ib, x.ik, c, x.R0);
        uint32_t cm = x.ik - c < 4 ? x.ik - c : 4;
        for (uint32_t q = 0; q < cm; q++) {
            uint32_t b = q * 16;
            uint32_t tt = rl(R4, b + 2), type = tt & 0xFF;
            if (type >= PSIM_MSG_PT_BROADCAST) continue;
            st_add(w, ST_DELIV + type, 1);
            uint32_t nex = (tt >> 16) & 0xFF;
            uint32_t ex = shfl(R4, (int)((b + 8 + l) & 63));
            ex = l < nex ? ex : 0u;
            const uint32_t p = rl(R4, b + 1), ttl = (tt >> 8) & 0xFF;
            STAMP(w, 2);
            if (type == PSIM_MSG_SHUFFLE_REPLY) {        // hv:1091-1093
                merge_exchange(w, ex, nex);
                STAMP(w, 3);
            } else if (ttl > 0 && w.act_n > 1) {         // hv:1095-1136: relay
                uint32_t r = select_random(w, w.A, w.act_n, p, w.me, w.me);
                if (r != NONE) hv_send(w, r, PSIM_MSG_SHUFFLE, ttl - 1, 0, 0, ex, nex);
                STAMP(w, 4);
            } else {                                     // the walk ends here
                uint32_t RESP = 0;
                uint32_t nr = sublist(w, w.P, w.pas_n, nex, RESP, 0);
                STAMP(w, 5);
                hv_send(w, p, PSIM_MSG_SHUFFLE_REPLY, 0, 0, 0, RESP, nr);
                STAMP(w, 6);
                merge_exchange(w, ex, nex);
                STAMP(w, 7);
            }
        }
    }
    STAMP(w, 2);
    if (x.tf & DESC_SHUFFLE) {                        // hv:572-607
        uint32_t EX;
        uint32_t nex = build_exchange(w, EX);
        uint32_t t = select_random(w, w.A, w.act_n, w.me, w.me, w.me);
        if (t != NONE) hv_send(w, t, PSIM_MSG_SHUFFLE, a.arwl, 0, 0, EX, nex);
        STAMP(w, 8);
    }
}

// the draw counter and passive size in the header, the passive row when it
// changed, the outbox count and the records (the flag byte, the active row,
// the id maps and the Plumtree rows are unchanged)
DEV void writeback_lite(Wv& w) {
    KArgs& a = kargs();
    const uint32_t l = lane_id();
    const size_t li = w.li;
    uint32_t* hrow = reinterpret_cast<uint32_t*>(a.hdr + li);
    const uint32_t k = l & 15;
    // words 0-1: the draw counter; word 9: act_n | pas_n << 8 | sent_n << 16 | sent_head << 24
    const uint32_t hw = k == 0 ? (uint32_t)w.rng : k == 1 ? (uint32_t)(w.rng >> 32)
                      : (w.act_n | (w.pas_n << 8) | (w.sent_n << 16) | (w.sent_head << 24));
    if (l < 16 && (k < 2 || k == 9)) hrow[k] = hw;
    {
        bool dirty = (w.vd & 2u) != 0;
        uint32_t x = shfl(w.P, (int)(l & 31));
        *(dirty ? a.pas + li * PSIM_PASSIVE_CAP + (l & 31) : hrow) = dirty ? x : (uint32_t)w.rng;
    }
    a.ocnt[li] = w.seq;
    st_add(w, ST_BOUND, w.seq > a.obase[li + 1] - w.obase ? 1u : 0u);
    flush_recs(w);
}

#ifndef PSIM_LITE_WAVES
#define PSIM_LITE_WAVES 7
#endif
#ifndef PSIM_LITE_WPB
#define PSIM_LITE_WPB 4
#endif
constexpr uint32_t LITE_WPB = PSIM_LITE_WPB;        // waves per k_consume_lite block
__global__ void __launch_bounds__(64 * PSIM_LITE_WPB, PSIM_LITE_WAVES) k_consume_lite(RoundArgs args) {
    if (*kargs().ctl) return;                         // an aborted batch (run_batch)
    __shared__ uint64_t sst[NST];
    __shared__ uint32_t scratch[LITE_WPB][64];
    __shared__ __attribute__((aligned(16))) uint32_t srecs[LITE_WPB][STAGE * 16];
    __shared__ uint32_t skeys[LITE_WPB][STAGE];
    for (int i = threadIdx.x; i < NST; i += blockDim.x) sst[i] = 0;
    __syncthreads();
    const uint32_t wid = threadIdx.x >> 6;
    const uint32_t gw = uni(blockIdx.x * LITE_WPB + wid);
    const uint32_t nw = gridDim.x * LITE_WPB;
    Wv w;
    w.a = &args;
    w.lds = scratch[wid];
    w.nlog = nullptr;
    w.srec = srecs[wid];
    w.skey = skeys[wid];
    w.slots = nullptr;
#ifdef PSIM_STAMPS
    __shared__ uint64_t stamps[LITE_WPB][32];
    if ((threadIdx.x & 63) < 32) stamps[wid][threadIdx.x & 63] = 0;
    w.stl = stamps[wid];
    w.t_last = __builtin_amdgcn_s_memtime();
#endif
    w.st = sst;
    w.round = kargs().round;
    w.SC = 0;
    w.digest = 0;
    w.KM = magic_lanes();
    uint32_t lc[4], na;
    lite_counts(kargs(), lc, na);
    if (gw < na) {
        const uint32_t last = na - 1;
        KArgs& a0 = kargs();
        NodeIn x = load_node<false>(a0, reinterpret_cast<const uint32_t*>(kargs().desc_lite + lite_at(a0, lc, gw))[lane_id() & 3]);
        NodeX y = load_x<true>(kargs(), x);
        NodeIn xn = load_node<false>(kargs(), reinterpret_cast<const uint32_t*>(kargs().desc_lite + lite_at(a0, lc, min(gw + nw, last)))[lane_id() & 3]);
        uint32_t d = reinterpret_cast<const uint32_t*>(kargs().desc_lite + lite_at(a0, lc, min(gw + 2 * nw, last)))[lane_id() & 3];
        for (uint32_t i = gw; i < na; i += nw) {
            STAMP(w, 0);
            begin_node(w, x, y);
            body_lite(w, x);
            NodeX yn = load_x<true>(kargs(), xn);
            STAMP(w, 9);
            writeback_lite(w);
            STAMP(w, 10);
            NodeIn xnn = load_node<false>(kargs(), d);
            d = reinterpret_cast<const uint32_t*>(kargs().desc_lite + lite_at(kargs(), lc, min(i + 3 * nw, last)))[lane_id() & 3];
            x = xn; y = yn; xn = xnn;
            STAMP(w, 11);
        }
    }
#ifdef PSIM_STAMPS
    if (lane_id() < 32) atomicAdd(&g_stamps_lite[lane_id()], (unsigned long long)w.stl[lane_id()]);
#endif
    flush_wave_stats(w, sst);
    __syncthreads();
    for (int i = threadIdx.x; i < NST; i += blockDim.x)
        kargs().stat_lite[(size_t)blockIdx.x * NST + i] = sst[i];
}

// ------------------------------------------------------- Plumtree phase --
// k_pt: one wave per node with Plumtree work (k_relay's second list), after
// the node's HyParView phase (k_relay's lane or k_consume): its Plumtree
// inbox in canonical order, its origin broadcast and its lazy tick
// (pt:282-313, :341-345, :443-453; round model R0 steps 2f-2h).  It reads
// the header, active view and outbox count the HyParView phase left and
// continues the node's emissions after them.  The same two-stage pipeline:
//   PtIn   header, active view, first inbox chunk, flag / partition bytes,
//          the outbox count so far
//   PtX    flag / partition bytes of the active members, the Plumtree rows
struct PtIn {
    uint32_t n, ib, ik, ob, tf;
    uint32_t H, A, R0, CN;
    uint32_t fl, part, oc;
};
struct PtX {
    uint32_t CF, PA, PG, PL;
    uint64_t PO;
};

DEV PtIn load_pt_node(KArgs& a, uint32_t D) {
    const uint32_t l = lane_id();
    PtIn x;
    x.n = rl(D, 0); x.ib = rl(D, 1); x.ik = rl(D, 2) & DESC_CNT_MASK; x.tf = rl(D, 2) >> 28; x.ob = rl(D, 3);
    const size_t li = x.n - a.lo;
    x.H = reinterpret_cast<const uint32_t*>(a.hdr + li)[l & 15];
    x.A = a.act[li * PSIM_ACTIVE_CAP + (l & 7)];
    const uint32_t m = x.ik ? min(l >> 4, x.ik - 1) : 0u;
    x.R0 = reinterpret_cast<const uint32_t*>(a.rec_in + x.ib + m)[l & 15];
    x.CN = a.conn[li * PSIM_CONN_CAP + (l & 7)];
    x.fl = a.flags[x.n];
    x.part = a.part[x.n];
    x.oc = a.ocnt[li];
    return x;
}

// the active members' ids in cache lanes 32-39 and the connection table's
// lingering peers in 40-47 (connect_ok, pt_conn_mask)
DEV uint32_t act_cache(const PtIn& x) {
    const uint32_t l = lane_id(), act_n = rl(x.H, 9) & 0xFF;
    const uint32_t av = shfl(x.A, (int)(l & 7));
    const uint32_t cc = conn_cache_id(x.CN, x.H);    // (every lane: it shuffles)
    return l >= 32 && l < 40 && l - 32 < act_n ? av : (l >= 40 ? cc : NONE);
}

DEV PtX load_pt_x(KArgs& a, const PtIn& x) {
    const uint32_t l = lane_id();
    PtX y;
    const size_t li = x.n - a.lo;
    y.CF = cache_flags(a, act_cache(x), x.n);
    y.PA = load_pa(a, li);
    y.PG = a.pt_eag[li * RT_SET + l];
    y.PL = a.pt_laz[li * RT_SET + l];
    y.PO = load_po(a, li, rl(x.H, HW_OUT_EXT));
    return y;
}

DEV void begin_pt(Wv& w, const PtIn& x, const PtX& y) {
    const uint32_t l = lane_id();
    w.li = x.n - kargs().lo;
    w.me = x.n;
    // only the header fields the Plumtree phase reads or writes live in
    // scalars (the rest go back from the loaded word)
    w.rng = ((uint64_t)rl(x.H, 1) << 32) | rl(x.H, 0);   // (store_pt_rows' fixed store rewrites it)
    w.start_round = rl(x.H, 2);
    w.aux = rl(x.H, 5); w.have = rl(x.H, 6); w.trk_round = rl(x.H, 7); w.trk_hop = rl(x.H, 8);
    const uint32_t w10 = rl(x.H, 10);
    w.act_n = rl(x.H, 9) & 0xFF; w.all_n = (w10 >> 16) & 0xFF; w.com_n = w10 >> 24;
    w.out_n = (rl(x.H, 11) >> 16) & 0xFF;
    w.ox = rl(x.H, HW_OUT_EXT);
    w.A = l < PSIM_ACTIVE_CAP ? x.A : 0u;
    w.fl = x.fl;
    w.obase = x.ob;
    w.mypart = x.part;
    w.CV = act_cache(x); w.CF = y.CF;
    const uint32_t w11 = rl(x.H, HW_CONN);
    w.conn_n = w11 & 0xFF; w.conn_dn = (w11 >> 8) & 0xFF; w.conn_cl = w11 >> 24;
    w.CN = l < w.conn_n ? x.CN : 0u;
    load_pt_regs(w, y.PA, y.PG, y.PL, y.PO);
    w.pt_dirty = false;
    w.lazy_quiet = false;
    w.seq = x.oc; w.flushed = x.oc;                  // after the HyParView phase's records
}

// the lazy tick's IHAVEs for the outstanding table's tail (entries
// OUT_HEAD.., after the register's: the table's order); the entries sent
DEV uint64_t lazy_tick_tail(Wv& w) {
    const uint32_t l = lane_id();
    const uint64_t T = load_out_tail(w);
    const uint32_t peer = (uint32_t)(T >> 32), msg = ((uint32_t)T >> 16) & 0xFFFFu;
    const uint64_t ok = pt_conn_mask(w, ballot(l < w.out_n - OUT_HEAD), peer);
    const uint32_t sk = msg % PSIM_MSG_SLOTS;
    const bool live = w.slots[sk] == msg;
    const uint32_t root = live ? w.slots[PSIM_MSG_SLOTS + sk] : NONE;
    const uint32_t dead = popc(ok & ballot(!live));
    st_add(w, ST_OVF, dead);
    st_add(w, ST_OVF_BY + PSIM_OVF_PT, dead);
    emit_batch<true>(w, ok, PSIM_MSG_PT_IHAVE, peer & ~PSIM_MAP_BIT, msg, (uint32_t)T & 0xFFFFu, root);
    return ok;
}

DEV void body_pt(Wv& w, const PtIn& x) {
    KArgs& a = kargs();
    const uint32_t r = a.round, n = x.n;
    // a fresh incarnation drops its inbox (counted by the HyParView phase)
    const uint32_t ik = hw_start(w) == r ? 0u : x.ik;
    for (uint32_t c = 0; c < ik; c += 4) {            // Plumtree inbox, canonical order
        uint32_t R4 = c == 0 ? x.R0 : load_chunk(a, x.ib, ik, c);
        uint32_t cm = ik - c < 4 ? ik - c : 4;
        for (uint32_t q = 0; q < cm; q++) {
            uint32_t b = q * 16;
            uint32_t type = rl(R4, b + 2) & 0xFF;
            if (type < PSIM_MSG_PT_BROADCAST || type > PSIM_MSG_PT_GRAFT) continue;
            st_add(w, ST_DELIV + type, 1);
            STAMP(w, 29);
            pt_handle(w, type, rl(R4, b + 1), rl(R4, b + 4), rl(R4, b + 5), rl(R4, b + 6));
            STAMP(w, 16 + type - PSIM_MSG_PT_BROADCAST);
        }
    }
    STAMP(w, 29);
    if (x.tf & DESC_ORIGIN) {                         // pt:282-287, backend:179-200
        const uint32_t my = n | PSIM_MAP_BIT, msg = uni(a.origin[n - a.lo]) - 1;
        pt_mark(w, msg);
        if (msg == a.tracked_msg) { w.trk_round = r; w.trk_hop = 0; }
        pt_push(w, msg, 0, my, my);
        STAMP(w, 21);
    }
    if ((x.tf & DESC_LAZY) && w.out_n > 0) {          // pt:341-345, :443-453
        // an IHAVE per outstanding entry (lane e: entry e), batched; the
        // root of a sent entry's id from its slot (a retired id: overflow,
        // PSIM_NONE)
        const uint32_t l = lane_id();
        const uint32_t peer = (uint32_t)(w.OUT >> 32), msg = ((uint32_t)w.OUT >> 16) & 0xFFFFu;
        const uint64_t ok = pt_conn_mask(w, ballot(l < w.out_n), peer);
        const uint32_t sk = msg % PSIM_MSG_SLOTS;
        const bool live = w.slots[sk] == msg;
        const uint32_t root = live ? w.slots[PSIM_MSG_SLOTS + sk] : NONE;
        const uint32_t dead = popc(ok & ballot(!live));
        st_add(w, ST_OVF, dead);
        st_add(w, ST_OVF_BY + PSIM_OVF_PT, dead);
        emit_batch<true>(w, ok, PSIM_MSG_PT_IHAVE, peer & ~PSIM_MAP_BIT, msg, (uint32_t)w.OUT & 0xFFFFu, root);
        const uint64_t ok_tail = w.out_n > OUT_HEAD ? lazy_tick_tail(w) : 0ull;
        // no entry's peer connected: the tick is the round's last handler, so
        // until a handler or a partition change connects one, every later
        // tick fails the same way (k_node_prep counts it without a wave)
        w.lazy_quiet = (ok | ok_tail) == 0;
        STAMP(w, 22);
    }
}

// H: the header word l & 15 as loaded (the words the Plumtree phase leaves
// alone are stored back from it)
DEV void writeback_pt(Wv& w, uint32_t H) {
    KArgs& a = kargs();
    const uint32_t l = lane_id();
    const size_t li = w.li;
    out_ext(w);
    {
        const uint32_t k = l & 15;
        uint32_t v = H;
        v = k == 5 ? w.aux : v;
        v = k == 6 ? w.have : v;
        v = k == 7 ? w.trk_round : v;
        v = k == 8 ? w.trk_hop : v;
        v = k == 10 ? ((v & 0xFFFFu) | (w.all_n << 16) | (w.com_n << 24)) : v;
        v = k == 11 ? ((v & ~0xFF0000u) | (w.out_n << 16)) : v;
        v = k == HW_OUT_EXT ? w.ox : v;
        reinterpret_cast<uint32_t*>(a.hdr + li)[k] = v;
    }
    if (w.pt_dirty) store_pt_rows(w);
    a.ocnt[li] = w.seq;
    st_add(w, ST_BOUND, w.seq > a.obase[li + 1] - w.obase ? 1u : 0u);
    a.flags[w.me] = flag_byte(w);
    if (w.seq != w.flushed) flush_recs(w);
}

#ifndef PSIM_PT_WAVES
#define PSIM_PT_WAVES 5
#endif
__global__ void __launch_bounds__(256, PSIM_PT_WAVES) k_pt(RoundArgs args) {
    if (*kargs().ctl) return;                         // an aborted batch (run_batch)
    __shared__ uint64_t sst[NST];
    __shared__ uint32_t scratch[WAVES_PER_BLOCK][64];
    __shared__ __attribute__((aligned(16))) uint32_t srecs[WAVES_PER_BLOCK][STAGE * 16];
    __shared__ uint32_t skeys[WAVES_PER_BLOCK][STAGE];
    __shared__ uint32_t sslots[2 * PSIM_MSG_SLOTS];
    for (int i = threadIdx.x; i < 2 * PSIM_MSG_SLOTS; i += blockDim.x) sslots[i] = kargs().slots[i];
    for (int i = threadIdx.x; i < NST; i += blockDim.x) sst[i] = 0;
    __syncthreads();
    const uint32_t wid = threadIdx.x >> 6;
    const uint32_t gw = uni(blockIdx.x * WAVES_PER_BLOCK + wid);
    const uint32_t nw = gridDim.x * WAVES_PER_BLOCK;
    Wv w;
    w.a = &args;
    w.lds = scratch[wid];
    w.nlog = nullptr;
    w.srec = srecs[wid];
    w.skey = skeys[wid];
    w.slots = sslots;
#ifdef PSIM_STAMPS
    __shared__ uint64_t stamps[WAVES_PER_BLOCK][32];
    if ((threadIdx.x & 63) < 32) stamps[wid][threadIdx.x & 63] = 0;
    w.stl = stamps[wid];
    w.t_last = __builtin_amdgcn_s_memtime();
#endif
    w.st = sst;
    w.round = kargs().round;
    w.SC = 0;
    w.digest = 0;
    const uint32_t na = *kargs().n_alist;
    if (gw < na) {
        const uint32_t last = na - 1;
        PtIn x = load_pt_node(kargs(), load_desc(kargs(), gw));
        PtX y = load_pt_x(kargs(), x);
        PtIn xn = load_pt_node(kargs(), load_desc(kargs(), min(gw + nw, last)));
        uint32_t d = load_desc(kargs(), min(gw + 2 * nw, last));
        for (uint32_t i = gw; i < na; i += nw) {
            STAMP(w, 31);
            begin_pt(w, x, y);
            STAMP(w, 29);
            body_pt(w, x);
            PtX yn = load_pt_x(kargs(), xn);
            writeback_pt(w, x.H);
            STAMP(w, 30);
            PtIn xnn = load_pt_node(kargs(), d);
            d = load_desc(kargs(), min(i + 3 * nw, last));
            x = xn; y = yn; xn = xnn;
        }
    }
#ifdef PSIM_STAMPS
    if (lane_id() < 32) atomicAdd(&g_stamps[lane_id()], (unsigned long long)w.stl[lane_id()]);
#endif
    flush_wave_stats(w, sst);
    __syncthreads();
    for (int i = threadIdx.x; i < NST; i += blockDim.x)
        kargs().stat_part[(size_t)blockIdx.x * NST + i] = sst[i];
}

// ------------------------------------------------ relays and lazy ticks --
// k_relay gives every node with work one lane and sorts it: most nodes with
// work in a steady-state round do little for HyParView -- at most relay the
// SHUFFLEs of their inbox (hv:1095-1136 with TTL > 0 and |active| > 1: a
// select_random over active -- [Sender, Myself], then do_send_message) --
// and such a lane does it here, exactly as k_consume's body and writeback
// would (the same draws, records, sequence numbers, digest and stats).  The
// other lists: a due shuffle start with nothing else heavy -> k_shuf (after
// the relays); SHUFFLE terminals / replies -> k_consume_lite; any other
// HyParView work (another message type, a promotion that can act, a join, a
// crashed active member) -> k_consume; Plumtree work (messages, a due lazy
// tick with entries outstanding) -> k_ptl, an origin -> k_pt, after the
// HyParView phase.  The order within a list does not matter (each node
// writes its own rows and outbox region; the stats and the digest are sums).
DEV uint64_t relay_emit(KArgs& a, uint64_t slot, uint32_t dst, uint32_t me, uint32_t tt, uint32_t seq,
                        uint32_t a0, uint32_t a1, uint32_t a2, const uint32_t (&X)[8]) {
    const uint32_t W[16] = {dst, me, tt, seq, a0, a1, a2, 0u, X[0], X[1], X[2], X[3], X[4], X[5], X[6], X[7]};
    uint64_t dg = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) dg += (uint64_t)W[j] * digest_mul(j);
    uint4* o = reinterpret_cast<uint4*>(a.rec_out + slot);
    o[0] = make_uint4(dst, me, tt, seq);
    o[1] = make_uint4(a0, a1, a2, 0u);
    if (!PSIM_SHORT_TAIL || ((tt >> 16) & 0xFFu)) {   // (a short record's tail: zeros, by the route)
        o[2] = make_uint4(X[0], X[1], X[2], X[3]);
        o[3] = make_uint4(X[4], X[5], X[6], X[7]);
    }
    a.okey[slot] = dst | (max_emit(tt & 0xFF) << KEY_DST_BITS);
    return dg;
}

// appends the lanes with `go` of this block step to list `desc` (counter
// `cnt`): wave counts, a block scan in LDS, one global atomic per block step
// (a same-address atomic per wave serialised at L2 and cost ~100 us per round)
DEV void block_append(bool go, const uint4& D, uint4* desc, uint32_t* cnt, uint32_t* wcnt) {
    const uint64_t m = ballot(go);
    const uint32_t wv = threadIdx.x >> 6;
    __syncthreads();                                  // the previous use's readers of wcnt are done
    if (lane_id() == 0) wcnt[wv] = popc(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t k = 0; k < (blockDim.x >> 6); k++) t += wcnt[k];
        wcnt[4] = t ? atomicAdd(cnt, t) : 0u;
    }
    __syncthreads();
    if (go) {
        uint32_t b0 = wcnt[4];
        for (uint32_t k = 0; k < wv; k++) b0 += wcnt[k];
        desc[b0 + popc(m & lt_mask())] = D;
    }
}

#ifndef PSIM_RELAY_WAVES       // (5: 95 VGPRs, no spills; 0.532 -> 0.527 ms a phase against 4, profiles/r04 ab6)
#define PSIM_RELAY_WAVES 5
#endif
#ifndef PSIM_RELAY_FJ         // FORWARD_JOIN relays on k_relay's lanes (0: k_consume's waves, for A/B)
#define PSIM_RELAY_FJ 1
#endif
#ifndef PSIM_PTL_BIN          // k_ptl's list binned by BROADCAST presence (0: one list, for A/B)
#define PSIM_PTL_BIN 1
#endif
#ifndef PSIM_LITE_BIN         // the lite list binned by SHUFFLE terminals (0: one list, for A/B)
#define PSIM_LITE_BIN 1
#endif
__global__ void __launch_bounds__(256, PSIM_RELAY_WAVES) k_relay(RoundArgs) {
    if (*kargs().ctl) return;                         // an aborted batch (run_batch)
    // the node-round phase starts here: its span's first stamp (the last is
    // taken by the first kernel after the phase, RoundArgs::ktime)
    if (blockIdx.x == 0 && threadIdx.x == 0) kargs().ktime[0] = __builtin_amdgcn_s_memrealtime();
    enum { R_PROC, R_DELIV, R_SHUF, R_FAIL, R_DIGEST, R_BOUND, R_DELIV_FJ, R_FJ, R_N };
    __shared__ unsigned long long sst[R_N];
    __shared__ uint32_t wc5[9][5];                    // per list: the wave counts, then the block's base
    if (threadIdx.x < R_N) sst[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t l = lane_id();
    const uint32_t na = *kargs().n_alist;
    const uint64_t two58 = 1ull << 58;
    unsigned long long v[R_N] = {};
    for (uint32_t base = blockIdx.x * blockDim.x; base < na; base += gridDim.x * blockDim.x) {
        KArgs& a = kargs();                           // (re-read per step, not held in SGPRs)
        const uint32_t P = base + threadIdx.x;
        uint4 D = make_uint4(0, 0, 0, 0);
        bool heavy = false, to_pt = false, relay = false, maps = false, shuf = false, lite = false, bcast = false, term = false,
             extra = false;
        Hdr h;
        uint32_t ik = 0, oend = 0;
        uint4 act0 = make_uint4(0, 0, 0, 0), act1 = act0;
        uint32_t me_part = 0;
        uint32_t hvm = 0;                             // the HyParView records among the first 32
        uint8_t fl0 = 0;                              // (the flag byte, read with the rows: read after
                                                      // the relays' stores, its wait drained them --
                                                      // gfx9 counts loads and stores in one in-order counter)
        if (P < na) {
            D = a.desc[P];
            const uint32_t id = D.x, tf = D.z >> 28;
            ik = D.z & DESC_CNT_MASK;
            // the header, the active row and the partition byte are
            // independent: issued together, waited once
            const size_t li = id - a.lo;
            h = a.hdr[li];
            oend = (uint32_t)a.obase[li + 1];
            const uint4* ar = reinterpret_cast<const uint4*>(a.act + li * PSIM_ACTIVE_CAP);
            act0 = ar[0];
            act1 = ar[1];
            me_part = a.part[id];
            fl0 = a.flags[id];
            // the inbox: how many HyParView messages, and whether each is a
            // SHUFFLE with TTL left (a relay while |active| > 1)
            uint32_t hvn = 0;
            hvm = 0;
            bool all_relay = true, all_shuf = true, term_out = false, fjn = false;
            bcast = false; term = false; extra = (tf & DESC_SHUFFLE) != 0;
            const uint32_t av[8] = {act0.x, act0.y, act0.z, act0.w, act1.x, act1.y, act1.z, act1.w};
            // (four records' first 16 B issued before any is waited on: a
            // loop of single loads waits one memory latency per record)
            for (uint32_t j = 0; j < ik; j += 4) {
                uint2 T[4];                                   // (src, type word)
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint4 r4 = j + q < ik ? *reinterpret_cast<const uint4*>(a.rec_in + D.y + j + q)
                                                : make_uint4(0, 0, (uint32_t)PSIM_MSG_PT_BROADCAST, 0);
                    T[q] = make_uint2(r4.y, r4.z);
                }
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t tt = T[q].y, type = tt & 0xFF;
                    bcast |= j + q < ik && type == PSIM_MSG_PT_BROADCAST;
                    if (type < PSIM_MSG_PT_BROADCAST || type >= PSIM_MSG_XBOT_OPTIMIZATION) {   // (X-BOT's: heavy)
                        hvn++;
                        hvm |= j + q < 32 ? 1u << (j + q) : 0u;
                        maps |= type <= PSIM_MSG_NEIGHBOR_ACCEPTED;   // id maps (hv:703-1089)
                        const uint32_t ttl = (tt >> 8) & 0xFF;
                        const bool relays = ttl > 0 && h.act_n > 1;
                        // a FORWARD_JOIN with TTL left, off the passive walk's
                        // step (TTL == PRWL adds the joiner to the passive
                        // view) and four active members or more (a pick
                        // whatever its three omits): a relay like a
                        // SHUFFLE's (hv:867-870, :899-906)
                        const bool fj = PSIM_RELAY_FJ && !a.xbot && type == PSIM_MSG_FORWARD_JOIN && ttl > 0 &&
                                        ttl != a.prwl && h.act_n >= 4;
                        fjn |= fj;
                        all_relay &= (type == PSIM_MSG_SHUFFLE && ttl > 0) || fj;
                        all_shuf &= type == PSIM_MSG_SHUFFLE || type == PSIM_MSG_SHUFFLE_REPLY;
                        // a walk that ends here replies to its Sender: maybe_connect
                        // (hv:1127) opens a lingering connection to a Sender outside
                        // the active view -- the connection table's path, k_consume
                        term |= type == PSIM_MSG_SHUFFLE && !relays;
                        extra |= type == PSIM_MSG_SHUFFLE && relays;
                        if (type == PSIM_MSG_SHUFFLE && !relays) {
                            bool in = false;
#pragma unroll
                            for (int k = 0; k < 8; k++) in |= (uint32_t)k < h.act_n && av[k] == T[q].x;
                            term_out |= !in;
                        }
                    }
                }
            }
            const bool fresh = h.start_round == a.round;
            bool exits = false;                       // a crashed peer held over a connection: EXIT events
            if (a.crash_round) {
                uint32_t cv[PSIM_CONN_CAP] = {};
                if (h.conn_n) {
                    const uint4* cr = reinterpret_cast<const uint4*>(a.conn + li * PSIM_CONN_CAP);
                    const uint4 c0 = cr[0], c1 = cr[1];
                    cv[0] = c0.x; cv[1] = c0.y; cv[2] = c0.z; cv[3] = c0.w;
                    cv[4] = c1.x; cv[5] = c1.y; cv[6] = c1.z; cv[7] = c1.w;
                }
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    bool down = false;
#pragma unroll
                    for (int k = 0; k < PSIM_CONN_CAP; k++) down |= (uint32_t)k < h.conn_n && cv[k] == (av[j] | PSIM_CONN_DOWN);
                    exits |= (uint32_t)j < h.act_n && av[j] != id && av[j] < a.n_nodes && !down &&
                             crashed_now(a, av[j]);
                }
#pragma unroll
                for (int k = 0; k < PSIM_CONN_CAP; k++)
                    exits |= (uint32_t)k < h.conn_n && !(cv[k] & PSIM_CONN_DOWN) && crashed_now(a, cv[k] & KEY_DST_MASK);
            }
            // an active member without a connection (conn_dn): the next send
            // to it reconnects (maybe_connect) -- the connection table's path
            const bool cdown = h.conn_dn != 0 && (hvn > 0 || (tf & DESC_SHUFFLE));
            // X-BOT: a due xbot_execution, or connection pids stopped last
            // round (their 'EXIT's): k_consume
            const bool xwork = a.xbot && (h.conn_cl || (D.z & DESC_XBOT_BIT));
            // (a FORWARD_JOIN relay ends in notify/1 (hv:921): a no-op only
            // while Plumtree's all_members is the active view -- else its
            // update belongs to k_consume)
            bool fj_ok = true;
            if (fjn && a.plumtree) {
                const uint4* pr = reinterpret_cast<const uint4*>(a.pt_all + li * PSIM_PT_MEMBERS_CAP);
                const uint4 p0 = pr[0], p1 = pr[1];
                const uint32_t pv[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
                fj_ok = h.all_n == h.act_n;
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    bool in = false;
#pragma unroll
                    for (int k = 0; k < 8; k++) in |= (uint32_t)k < h.all_n && pv[k] == av[j];
                    fj_ok &= (uint32_t)j >= h.act_n || in;
                }
            }
            heavy = exits || fresh || ((tf & DESC_PROMO) && h.act_n < a.min_active) ||
                    (hvn && !all_shuf && !(all_relay && fj_ok)) || term_out || cdown || xwork;
            // SHUFFLE terminals and replies (with whatever relays and shuffle
            // start come with them): k_consume_lite
            lite = !heavy && hvn && !(all_relay && h.act_n > 1);
            // a due shuffle with nothing else heavy: k_shuf, after the relays
            shuf = !heavy && !lite && (tf & DESC_SHUFFLE);
            maps = maps || exits || (tf & DESC_PROMO) || h.conn_cl;   // move_to_active: current_id
            relay = !heavy && !lite && hvn > 0;
            const bool pt_msgs = !fresh && ik > hvn, origin = (tf & DESC_ORIGIN) != 0;
            const bool lazy = (tf & DESC_LAZY) && h.out_n > 0;
            // the Plumtree phase (messages, an origin, a due lazy tick with
            // entries outstanding) runs after the HyParView phase: k_ptl, or
            // k_pt for an origin
            to_pt = a.plumtree && (pt_msgs || origin || lazy);
            // (k_consume and k_consume_lite count their own)
            if (!heavy && !lite && (relay || to_pt || shuf)) v[R_PROC]++;
        }
        // a relaying lane's members' up-and-partition pairs, issued before
        // the list appends' barriers so that their latency hides behind them
        // (read per relay, after its draw, they were one dependent load each)
        uint32_t upm[4] = {NONE, NONE, NONE, NONE};   // member j's pair in bits 16 (j & 1) of word j >> 1
        if (P < na && (relay || lite)) {
            const uint32_t av[8] = {act0.x, act0.y, act0.z, act0.w, act1.x, act1.y, act1.z, act1.w};
            KArgs& a = kargs();
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
                const uint32_t q0 = (uint32_t)j < h.act_n && av[j] < a.n_nodes ? av[j] : D.x;
                const uint32_t q1 = (uint32_t)j + 1 < h.act_n && av[j + 1] < a.n_nodes ? av[j + 1] : D.x;
                upm[j >> 1] = (uint32_t)a.upart[q0] | ((uint32_t)a.upart[q1] << 16);
            }
        }
        // (k_ptl takes the Plumtree phase of nodes without an origin, and
        // hands k_pt the ones that do not fit a lane)
        const bool origin_node = ((D.z >> 28) & DESC_ORIGIN) != 0;
        {
            // the seven lists at once: one barrier-separated count, the
            // block atomics from seven lanes of one instruction (one after
            // another they were serial L2 round trips per block step); k_ptl's
            // list as two, BROADCAST nodes from its front, the others from
            // its back (ptl_desc), and the lite list likewise by SHUFFLE
            // terminals (lite_at)
            const bool ptl = P < na && to_pt && !origin_node, lt = P < na && lite;
            const bool lt0 = lt && !(extra && PSIM_LITE_BIN), lt1 = lt && extra && PSIM_LITE_BIN;
            const bool tb = term || !PSIM_LITE_BIN;
            const bool g[9] = {P < na && heavy, P < na && to_pt && origin_node, ptl && (bcast || !PSIM_PTL_BIN),
                               P < na && shuf, lt0 && tb, ptl && !(bcast || !PSIM_PTL_BIN), lt0 && !tb,
                               lt1 && tb, lt1 && !tb};
            uint64_t m[9];
#pragma unroll
            for (int k = 0; k < 9; k++) m[k] = ballot(g[k]);
            const uint32_t wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
            __syncthreads();                          // the previous step's readers of wc5 are done
            if (l == 0)
#pragma unroll
                for (int k = 0; k < 9; k++) wc5[k][wv] = popc(m[k]);
            __syncthreads();
            if (threadIdx.x < 9) {
                const uint32_t k = threadIdx.x;
                uint32_t t = 0;
                for (uint32_t j = 0; j < nwv; j++) t += wc5[k][j];
                uint32_t* cnt = k == 0 ? a.n_slow : k == 1 ? a.n_pt : k == 2 ? a.n_ptl : k == 3 ? a.n_shuf
                              : k == 4 ? a.n_lite : k == 5 ? a.n_ptl + 1 : a.n_lite + (k - 5);
                wc5[k][4] = t ? atomicAdd(cnt, t) : 0u;
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < 9; k++)
                if (g[k]) {
                    uint32_t b0 = wc5[k][4];
                    for (uint32_t j = 0; j < wv; j++) b0 += wc5[k][j];
                    const uint32_t at = b0 + popc(m[k] & lt_mask());
                    uint4* desc = k == 0 ? a.desc_slow : k == 1 ? a.desc_pt : k == 2 || k == 5 ? a.desc_ptl
                                : k == 3 ? a.desc_shuf : a.desc_lite;
                    const uint32_t nl = a.n_local;
                    desc[k == 5 || k == 6 ? nl - 1 - at : k == 7 ? nl + at : k == 8 ? 2 * nl - 1 - at : at] =
                        k == 0 && maps ? make_uint4(D.x, D.y, D.z | DESC_MAPS_BIT, D.w) : D;
                }
        }
        if (P < na && lite && !heavy) {
            // the lite node's connection bits (k_lite_half's connect_ok)
            uint32_t cm = 0;
#pragma unroll
            for (int j = 0; j < 8; j++)
                cm |= ((upm[j >> 1] >> (16 * (j & 1))) & 0xFFFFu) == me_part ? 1u << j : 0u;
            kargs().lite_cm[D.x - kargs().lo] = (uint8_t)cm;
        }
        if (P >= na || heavy || lite) continue;
        const uint32_t id = D.x;
        const size_t li = id - a.lo;
        const uint32_t A[8] = {act0.x, act0.y, act0.z, act0.w, act1.x, act1.y, act1.z, act1.w};
        uint64_t rng = h.rng;
        uint32_t seq = 0;
        // the SHUFFLE / FORWARD_JOIN relays, in inbox order: a relay lane's
        // HyParView records (hvm; every record of an inbox past 32); a
        // Plumtree record's type word is not read again -- each such load
        // after a relay's stores waited for them (one in-order counter)
        const bool big = ik > 32;
        uint32_t rm = relay ? hvm : 0u;
        for (uint32_t jr = 0; relay && (big ? jr < ik : rm != 0); jr++) {
            if (!big) {
                jr = (uint32_t)__ffs(rm) - 1;
                rm &= rm - 1;
            }
            const Msg* rp = a.rec_in + D.y + jr;
            const uint32_t tt = rp->tt;
            if ((tt & 0xFF) >= PSIM_MSG_PT_BROADCAST) continue;
            const bool fj = (tt & 0xFF) == PSIM_MSG_FORWARD_JOIN;
            const uint32_t ttl = (tt >> 8) & 0xFF, nex = (tt >> 16) & 0xFF, src = rp->src;
            // (FORWARD_JOIN: the joiner and its epoch)
            const uint32_t jq = fj ? rp->a0 : NONE, jpe = fj ? rp->a1 : 0u;
            v[fj ? R_DELIV_FJ : R_DELIV]++;
            // select_random(Active, [Sender, Myself]) (hv:1346-1356); a
            // FORWARD_JOIN's omits the joiner too (hv:867-870)
            uint32_t elig = 0;
#pragma unroll
            for (int j = 0; j < 8; j++)
                elig |= (j < h.act_n && A[j] != src && A[j] != id && A[j] != jq) ? (1u << j) : 0u;
            const uint32_t cnt = __popc(elig);
            if (cnt) {
                uint32_t k;
                for (;;) {                                // rand:uniform(cnt) - 1 (?uniform_range)
                    const uint64_t x = draw58_at(rng++, id, a.seed);
                    if (x < cnt) { k = (uint32_t)x; break; }
                    const uint32_t i = mod_small(x, cnt);
                    if (x - i <= two58 - cnt) { k = i; break; }
                }
                uint32_t e = elig;
                for (uint32_t j = 0; j < k; j++) e &= e - 1;
                const uint32_t jr_ = (uint32_t)__ffs(e) - 1;
                const uint32_t r = A[jr_];
                uint32_t up = 0;
#pragma unroll
                for (int j = 0; j < 8; j++)
                    if ((uint32_t)j == jr_) up = (upm[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
                // do_send_message: maybe_connect + find, then the dispatch draw
                if (r < a.n_nodes && up == me_part) {
                    rng++;
                    uint32_t X[8] = {};
                    if (!fj) {
                        const uint4* ex = reinterpret_cast<const uint4*>(rp->ex);
                        const uint4 e0 = ex[0], e1 = ex[1];
                        const uint32_t E[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
#pragma unroll
                        for (int j = 0; j < 8; j++) X[j] = (uint32_t)j < nex ? E[j] : 0u;
                    }
                    v[R_DIGEST] += relay_emit(a, D.w + seq, r, id,
                                              fj ? PSIM_MSG_FORWARD_JOIN | ((ttl - 1) << 8)
                                                 : PSIM_MSG_SHUFFLE | ((ttl - 1) << 8) | (nex << 16),
                                              seq, fj ? jq : 0u, jpe, 0u, X);
                    seq++;
                    v[fj ? R_FJ : R_SHUF]++;
                } else {
                    v[R_FAIL]++;
                }
            }
        }
        if (rng != h.rng) a.hdr[li].rng = rng;
        a.ocnt[li] = seq;
        v[R_BOUND] += seq > oend - D.w ? 1u : 0u;
        if (!to_pt) {                                 // (k_ptl / k_pt write the byte of their nodes)
            a.flags[id] = (uint8_t)((fl0 & (F_UP | F_CRASHED)) | (h.out_n ? F_LAZY : 0) |
                                    (min((uint32_t)h.out_n, 15u) << F_OUTN_SHIFT) |
                                    (h.act_n < a.min_active ? F_LOWACT : 0));
        }
    }
    // wave sums, then one LDS atomic per wave and counter
#pragma unroll
    for (int k = 0; k < R_N; k++)
        for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o);
    if (l == 0)
        for (int k = 0; k < R_N; k++)
            if (v[k]) atomicAdd(&sst[k], v[k]);
    __syncthreads();
    uint64_t* row = kargs().stat_relay + (size_t)blockIdx.x * NST;
    for (uint32_t k = threadIdx.x; k < NST; k += blockDim.x)
        row[k] = k == ST_PROC ? sst[R_PROC] : k == ST_DELIV + PSIM_MSG_SHUFFLE ? sst[R_DELIV]
               : k == ST_EMIT + PSIM_MSG_SHUFFLE ? sst[R_SHUF] : k == ST_FAIL ? sst[R_FAIL]
               : k == ST_DELIV + PSIM_MSG_FORWARD_JOIN ? sst[R_DELIV_FJ] : k == ST_EMIT + PSIM_MSG_FORWARD_JOIN ? sst[R_FJ]
               : k == ST_DIGEST ? sst[R_DIGEST] : k == ST_BOUND ? sst[R_BOUND] : 0ull;
}

// ------------------------------------------------------ shuffle starts --
// k_shuf: one lane per node whose HyParView work this round is its due
// passive_view_maintenance timer (hv:572-607), after any SHUFFLE relays
// k_relay ran for it, with nothing else HyParView-heavy (k_relay's list).
// The exchange is usort([Myself] ++ sublist(Active, k_active) ++
// sublist(Passive, k_passive)) (hv:577-586): each sublist keys its
// elements with consecutive draws in to_list order and keeps the K smallest
// (key, element) pairs -- here a running top-K in registers, one element at
// a time, exact on the full 53-bit keys -- then select_random(Active,
// [Myself]) picks the target and do_send_message draws the dispatch value.
// The view rows are only read: a shuffle start changes nothing but the
// draw counter.  Same draws, record, sequence number, digest and stats as
// k_consume's body; the node's Plumtree phase (if any) follows in k_pt.
constexpr int SHUF_TOPK = PSIM_EXCHANGE_CAP - 1;   // k_active + k_passive <= 7

// keep the K smallest (key, element) pairs in ascending order (slots >= K
// hold ~0): the new pair enters at the end and bubbles up, unrolled
DEV void topk_insert(uint64_t (&K)[SHUF_TOPK], uint32_t (&E)[SHUF_TOPK], uint64_t key, uint32_t e) {
    uint64_t ck = key;
    uint32_t ce = e;
#pragma unroll
    for (int i = 0; i < SHUF_TOPK; i++) {
        const bool lt = ck < K[i] || (ck == K[i] && ce < E[i]);
        const uint64_t tk = lt ? K[i] : ck;
        const uint32_t te = lt ? E[i] : ce;
        K[i] = lt ? ck : K[i];
        E[i] = lt ? ce : E[i];
        ck = tk;
        ce = te;
    }
}

__global__ void __launch_bounds__(256) k_shuf(RoundArgs) {
    if (*kargs().ctl) return;                         // an aborted batch (run_batch)
    enum { S_SHUF, S_FAIL, S_DIGEST, S_BOUND, S_N };
    __shared__ unsigned long long sst[S_N];
    if (threadIdx.x < S_N) sst[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t l = lane_id();
    const uint32_t ns = *kargs().n_shuf;
    const uint64_t two58 = 1ull << 58;
    unsigned long long v[S_N] = {};
    for (uint32_t P = blockIdx.x * blockDim.x + threadIdx.x; P < ns; P += gridDim.x * blockDim.x) {
        KArgs& a = kargs();
        const uint4 D = a.desc_shuf[P];
        const uint32_t id = D.x;
        const size_t li = id - a.lo;
        const uint64_t rng0 = a.hdr[li].rng;
        const uint32_t cnts = reinterpret_cast<const uint32_t*>(a.hdr + li)[9];   // act_n, pas_n, ..
        const uint32_t act_n = cnts & 0xFF, pas_n = (cnts >> 8) & 0xFF;
        const uint4* ar = reinterpret_cast<const uint4*>(a.act + li * PSIM_ACTIVE_CAP);
        const uint4 a0 = ar[0], a1 = ar[1];
        const uint32_t A[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        uint32_t seq = a.ocnt[li];                    // after k_relay's relays
        const uint32_t oend = (uint32_t)a.obase[li + 1];
        const uint32_t me_part = a.part[id];
        uint64_t rng = rng0;
        // sublist(Active, k_active): keys rng .. rng + act_n - 1
        uint64_t K[SHUF_TOPK];
        uint32_t E[SHUF_TOPK];
#pragma unroll
        for (int i = 0; i < SHUF_TOPK; i++) { K[i] = ~0ull; E[i] = ~0u; }
#pragma unroll
        for (int j = 0; j < PSIM_ACTIVE_CAP; j++)
            if ((uint32_t)j < act_n) topk_insert(K, E, draw58_at(rng + j, id, a.seed) >> 5, A[j]);
        rng += act_n;
        const uint32_t ka = min(act_n, a.k_active), kp = min(pas_n, a.k_passive);
        uint32_t X[8];
        X[0] = id;
#pragma unroll
        for (int i = 0; i < SHUF_TOPK; i++) X[1 + i] = (uint32_t)i < ka ? E[i] : ~0u;
        // sublist(Passive, k_passive): keys rng .. rng + pas_n - 1, the
        // passive row streamed 16 B at a time
#pragma unroll
        for (int i = 0; i < SHUF_TOPK; i++) { K[i] = ~0ull; E[i] = ~0u; }
        const uint4* pr = reinterpret_cast<const uint4*>(a.pas + li * PSIM_PASSIVE_CAP);
        for (uint32_t j0 = 0; j0 < pas_n; j0 += 4) {
            const uint4 q = pr[j0 >> 2];
            const uint32_t Q[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int c = 0; c < 4; c++)
                if (j0 + c < pas_n) topk_insert(K, E, draw58_at(rng + j0 + c, id, a.seed) >> 5, Q[c]);
        }
        rng += pas_n;
        // [Myself] ++ the active picks ++ the passive picks (slots past the
        // picks hold ~0, which sorts last and is cut below)
#pragma unroll
        for (int i = 0; i < SHUF_TOPK; i++) {
            const uint32_t e = (uint32_t)i < kp ? E[i] : ~0u;
            // X[1 + ka + i] = e, as selects over the fixed slots
#pragma unroll
            for (int o = 1; o < 8; o++) X[o] = ((uint32_t)o == 1 + ka + (uint32_t)i) ? e : X[o];
        }
        // lists:usort/1: an 8-input sorting network, then the duplicates out
#define CSW(i, j) { const uint32_t lo_ = min(X[i], X[j]), hi_ = max(X[i], X[j]); X[i] = lo_; X[j] = hi_; }
        CSW(0, 1) CSW(2, 3) CSW(4, 5) CSW(6, 7)
        CSW(0, 2) CSW(1, 3) CSW(4, 6) CSW(5, 7)
        CSW(1, 2) CSW(5, 6) CSW(0, 4) CSW(3, 7)
        CSW(1, 5) CSW(2, 6)
        CSW(1, 4) CSW(3, 6)
        CSW(2, 4) CSW(3, 5)
        CSW(3, 4)
#undef CSW
        uint32_t U[8], nex = 0;
#pragma unroll
        for (int o = 0; o < 8; o++) U[o] = 0u;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const bool keep = X[i] != ~0u && (i == 0 || X[i] != X[i - 1]);
#pragma unroll
            for (int o = 0; o < 8; o++) U[o] = (keep && nex == (uint32_t)o) ? X[i] : U[o];
            nex += keep ? 1u : 0u;
        }
        // select_random(Active, [Myself]) (hv:1346-1356)
        uint32_t elig = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) elig |= ((uint32_t)j < act_n && A[j] != id) ? (1u << j) : 0u;
        const uint32_t cnt = __popc(elig);
        if (cnt) {
            uint32_t k;
            for (;;) {                                // rand:uniform(cnt) - 1 (?uniform_range)
                const uint64_t x = draw58_at(rng++, id, a.seed);
                if (x < cnt) { k = (uint32_t)x; break; }
                const uint32_t i = mod_small(x, cnt);
                if (x - i <= two58 - cnt) { k = i; break; }
            }
            uint32_t e = elig;
            for (uint32_t j = 0; j < k; j++) e &= e - 1;
            const uint32_t t = A[__ffs(e) - 1];
            // do_send_message: maybe_connect + find, then the dispatch draw
            if (t < a.n_nodes && a.upart[t] == me_part) {
                rng++;
                v[S_DIGEST] += relay_emit(a, D.w + seq, t, id, PSIM_MSG_SHUFFLE | (a.arwl << 8) | (nex << 16), seq,
                                          0u, 0u, 0u, U);
                seq++;
                v[S_SHUF]++;
            } else {
                v[S_FAIL]++;
            }
        }
        a.hdr[li].rng = rng;
        a.ocnt[li] = seq;
        v[S_BOUND] += seq > oend - D.w ? 1u : 0u;
    }
#pragma unroll
    for (int k = 0; k < S_N; k++)
        for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o);
    if (l == 0)
        for (int k = 0; k < S_N; k++)
            if (v[k]) atomicAdd(&sst[k], v[k]);
    __syncthreads();
    uint64_t* row = kargs().stat_shuf + (size_t)blockIdx.x * NST;
    for (uint32_t k = threadIdx.x; k < NST; k += blockDim.x)
        row[k] = k == ST_EMIT + PSIM_MSG_SHUFFLE ? sst[S_SHUF] : k == ST_FAIL ? sst[S_FAIL]
               : k == ST_DIGEST ? sst[S_DIGEST] : k == ST_BOUND ? sst[S_BOUND] : 0ull;
}

// ---------------------------------------------------- Plumtree lanes --
// k_ptl: one lane per node with Plumtree work (k_relay's list, origins
// aside), after its HyParView phase.  In config C's steady state a node keeps
// per-root sets for one root (the broadcaster) with a handful of eager and
// lazy peers and a few outstanding entries, and its Plumtree phase is a
// BROADCAST (first delivery: eager push + lazy adds; duplicate: PRUNE), some
// PRUNEs, IHAVE answers and acks, then the lazy tick.  A lane holds slot 0's
// eager and lazy sets (16 entries each) and the outstanding table (PTL_CAP
// entries) in LDS columns when the node's data fits that: no root in slots
// 1-3, every message's root slot 0's (or slot 0 free and one root), the sets
// and the table far enough below their capacity that this round's adds fit,
// no outstanding extension row.  Any other node is appended to k_pt's list
// and runs there (the wave path).  k_relay orders the list: nodes with a
// BROADCAST first, so most waves run one kind of node (ptl_desc).
// Same handlers as pt_handle / pt_push / the lazy tick (pt:288-313, :341-345,
// :368-453, :562-631): the same records, sequence numbers, digest, stats.
#ifndef PSIM_PTL_CAP          // (12: 14 KiB of LDS a block, 11 per CU; 16 took 16 KiB, 9 per CU --
#define PSIM_PTL_CAP 12       //  at 2^26 12 measured 0.8 ms a round faster, profiles/r04/ab3e)
#endif
#ifndef PSIM_PTL_SET_CAP
#define PSIM_PTL_SET_CAP 16
#endif
constexpr int PTL_CAP = PSIM_PTL_CAP;           // outstanding entries a lane holds
constexpr int PTL_SET = PSIM_PTL_SET_CAP;       // eager / lazy entries a lane holds

constexpr uint32_t PTL_BLK = PTL_BLOCK;   // k_ptl block: one wave, 14 KiB of per-lane tables

// A lane's tables in LDS, entry i of lane t at row i, column t (conflict-free):
// unrolled scans read fixed offsets, run-time indexing is one access
struct LdsCol {
    uint32_t* p;
    DEV uint32_t& operator[](uint32_t i) const { return p[i * PTL_BLK]; }
};
DEV bool col_has(const LdsCol& V, uint32_t n, uint32_t x) {
    bool r = false;
#pragma unroll
    for (int i = 0; i < PTL_SET; i++) r |= (uint32_t)i < n && V[i] == x;
    return r;
}
#ifndef PSIM_PTL_PF           // k_ptl's set / table loops read one entry ahead (0: A/B)
#define PSIM_PTL_PF 1
#endif
// ordsets:del_element/2: the search stops at the first entry >= x (the set
// is ascending), the entries after x move down one; each LDS read is issued
// an iteration ahead of its use
DEV void col_del(const LdsCol& V, uint32_t& n, uint32_t x) {
    uint32_t at = n, e = n ? V[0] : 0u;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t en = i + 1 < n ? V[i + 1] : 0u;
        if (e >= x) {
            if (e == x) at = i;
            break;
        }
        e = en;
    }
    if (at == n) return;
    uint32_t nx = at + 1 < n ? V[at + 1] : 0u;
    for (uint32_t i = at; i + 1 < n; i++) {
        const uint32_t m = nx;
        nx = i + 2 < n ? V[i + 2] : 0u;
        V[i] = m;
    }
    n--;
    V[n] = 0u;
}
// ordsets:add_element/2 (the caller guarantees room): from the back, the
// entries above x move up one -- one pass, no separate search -- and a
// member found below them moves them back (x already in the set)
DEV void col_add(const LdsCol& V, uint32_t& n, uint32_t x) {
    const uint32_t top = V[n];                        // (restored when x is a member)
    uint32_t i = n, e = n ? V[n - 1] : 0u;
    while (i && e > x) {
        const uint32_t e2 = i > 1 ? V[i - 2] : 0u;
        V[i] = e;
        i--;
        e = e2;
    }
    if (i && e == x) {
        for (uint32_t k = i; k < n; k++) V[k] = V[k + 1];
        V[n] = top;
        return;
    }
    V[i] = x;
    n++;
}

#ifndef PSIM_PTL_CONN         // k_ptl takes nodes with a connection table (0: k_pt does, for A/B)
#define PSIM_PTL_CONN 1
#endif
constexpr uint32_t PTL_CN = 4;  // ... of at most 4 entries (a lane's registers; more: k_pt)
struct PtLane {
    uint32_t id, me_part, act_n;
    uint32_t A[PSIM_ACTIVE_CAP];
    uint32_t cmask;                // bit j: A[j] is a live connection (ptl_conn's test, per member)
#if PSIM_PTL_CONN
    uint32_t L[PTL_CN];            // the connection table's lingering peers (entries without a flag)
    uint32_t lmask;                // bit k: L[k] is outside the active view, running, same partition
#endif
    uint32_t root0;                // slot 0's root (NONE = free)
    LdsCol EG, LZ, OL, OH;         // slot 0's eager / lazy sets; outstanding keys (low, high words)
    uint32_t ne, nl, on;
    uint64_t have;
    bool sets_dirty, out_dirty;
};

// send/3 (pt:633-638): over an existing connection -- the peer in the active
// view, running, same partition
// (the members' up-and-partition pairs are read once per node, all eight
// loads in flight together: read per send they were one dependent memory
// latency per send; no kernel of the phase changes them)
// (loading only the members a send of this node may go to -- the senders
// its answers go to, its lazy tick's peers -- measured slower at 2^20 and
// at 2^26: the loads then wait for the records and the table, and the
// random lines come from the MALL, profiles/r05/ab_log.txt r5k / r5l)
// (the pairs are loaded as soon as the active row arrives, before the
// node's precondition pass, whose work then covers their latency)
DEV void ptl_load_pairs(KArgs& a, const PtLane& n, uint16_t (&up)[PSIM_ACTIVE_CAP]) {
#pragma unroll
    for (int j = 0; j < PSIM_ACTIVE_CAP; j++) {
        const uint32_t q = (uint32_t)j < n.act_n && n.A[j] < a.n_nodes ? n.A[j] : n.id;
        up[j] = a.upart[q];
    }
}
DEV uint32_t ptl_conn_mask(KArgs& a, const PtLane& n, const uint16_t (&up)[PSIM_ACTIVE_CAP]) {
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < PSIM_ACTIVE_CAP; j++)
        m |= ((uint32_t)j < n.act_n && n.A[j] < a.n_nodes && n.A[j] != n.id && up[j] == n.me_part) ? 1u << j : 0u;
    return m;
}

DEV bool ptl_conn(KArgs& a, const PtLane& n, uint32_t ident) {
    const uint32_t p = ident & ~PSIM_MAP_BIT;
    bool c = false;
#pragma unroll
    for (int j = 0; j < PSIM_ACTIVE_CAP; j++) c |= ((n.cmask >> j) & 1u) && n.A[j] == p;
#if PSIM_PTL_CONN
    // conn_has: a lingering peer's connection (lmask holds none of the
    // active members: for those the active test alone decides)
#pragma unroll
    for (int k = 0; k < (int)PTL_CN; k++) c |= ((n.lmask >> k) & 1u) && n.L[k] == p;
#endif
    return c;
}

// update_peers/5 + set_peers/4 (pt:593-609) on slot 0 (a new root takes it
// with the common eagers, read here; the lane's preconditions leave no other
// case)
DEV void ptl_update(KArgs& a, PtLane& n, size_t li, uint32_t com_n, uint32_t from, uint32_t root, bool to_eager) {
    n.sets_dirty = true;
    if (n.root0 != root) {
        n.root0 = root;
        const uint4* cr = reinterpret_cast<const uint4*>(a.pt_com + li * PSIM_PT_MEMBERS_CAP);
        const uint4 c0 = cr[0], c1 = cr[1];
        const uint32_t C8[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
        for (int i = 0; i < PTL_SET; i++) { n.EG[i] = i < 8 && (uint32_t)i < com_n ? C8[i & 7] : 0u; n.LZ[i] = 0u; }
        n.ne = com_n; n.nl = 0;
    }
    // the set `from` joins and the one it leaves, selected per lane: every
    // lane of the wave runs the one add and the one delete together, whatever
    // its message (the two directions as branches ran one after the other)
    LdsCol A, D;
    A.p = to_eager ? n.EG.p : n.LZ.p;
    D.p = to_eager ? n.LZ.p : n.EG.p;
    uint32_t na = to_eager ? n.ne : n.nl, nd = to_eager ? n.nl : n.ne;
    col_add(A, na, from);
    col_del(D, nd, from);
    n.ne = to_eager ? na : nd;
    n.nl = to_eager ? nd : na;
}

DEV uint64_t out_at(const PtLane& n, uint32_t i) { return ((uint64_t)n.OH[i] << 32) | n.OL[i]; }
// add_outstanding/6 (pt:574-579), ack_outstanding/6 (pt:562-567): the table
// as sorted peer << 32 | msg << 16 | round keys
DEV void ptl_add_out(PtLane& n, uint64_t key) {
    uint32_t pos = 0;
    bool in = false;
    for (uint32_t i = 0; i < n.on; i++) {
        const uint64_t e = out_at(n, i);
        in |= e == key;
        pos += e < key ? 1u : 0u;
    }
    if (in) return;
    for (uint32_t i = n.on; i > pos; i--) { n.OL[i] = n.OL[i - 1]; n.OH[i] = n.OH[i - 1]; }
    n.OL[pos] = (uint32_t)key; n.OH[pos] = (uint32_t)(key >> 32);
    n.on++;
    n.out_dirty = true;
}
// schedule_lazy_push/6 over slot 0's lazy set (pt:368-378): the keys
// peer << 32 | lo of its members other than `from` -- ascending with the
// set -- merged into the ascending table: a forward pass counts the keys
// the table lacks, a backward pass moves the table's larger entries up and
// places the new keys (add_outstanding per member searched the whole table
// and shifted its tail for each key)
#ifndef PSIM_PTL_LAZYM        // (0: add_outstanding per member, for A/B)
#define PSIM_PTL_LAZYM 1
#endif
DEV void ptl_add_lazy(PtLane& n, uint32_t from, uint32_t lo) {
    uint32_t add = 0;
    for (uint32_t j = 0, i = 0; j < n.nl; j++) {
        const uint32_t e = n.LZ[j];
        if (e == from) continue;
        const uint64_t key = ((uint64_t)e << 32) | lo;
        while (i < n.on && out_at(n, i) < key) i++;
        add += (i < n.on && out_at(n, i) == key) ? 0u : 1u;
    }
    if (!add) return;
    int i = (int)n.on - 1, d = (int)(n.on + add) - 1;
    for (int j = (int)n.nl - 1; j >= 0; j--) {
        const uint32_t e = n.LZ[j];
        if (e == from) continue;
        const uint64_t key = ((uint64_t)e << 32) | lo;
        uint64_t t = i >= 0 ? out_at(n, i) : 0ull;
        while (i >= 0 && t > key) {
            n.OL[d] = (uint32_t)t; n.OH[d] = (uint32_t)(t >> 32);
            d--; i--;
            t = i >= 0 ? out_at(n, i) : 0ull;
        }
        if (i >= 0 && t == key) continue;             // (already outstanding)
        n.OL[d] = (uint32_t)key; n.OH[d] = e;
        d--;
    }
    n.on += add;
    n.out_dirty = true;
}
DEV void ptl_ack_out(PtLane& n, uint64_t key) {
    for (uint32_t i = 0; i < n.on; i++) {
        if (out_at(n, i) != key) continue;
        for (uint32_t j = i; j + 1 < n.on; j++) { n.OL[j] = n.OL[j + 1]; n.OH[j] = n.OH[j + 1]; }
        n.on--;
        n.OL[n.on] = 0u; n.OH[n.on] = 0u;
        n.out_dirty = true;
        return;
    }
}

#ifndef PSIM_PTL_BLOCKS_PER_CU
#define PSIM_PTL_BLOCKS_PER_CU 3
#endif
#ifndef PSIM_PTL_RREG
#define PSIM_PTL_RREG 6       // 4: 61.75, 6: 60.89 ms a phase at 2^26 (profiles/r04/ab_rreg.sh); 8 spills
#endif
// the first PTL_RREG Plumtree records of a k_ptl node, kept in registers from
// the precondition pass: a record load issued after the node's emissions
// waits for those stores too (one vector memory counter, in order), so the
// handler loop loads none of them
constexpr int PTL_RREG = PSIM_PTL_RREG;
struct PtlRecs {
    uint32_t src[PTL_RREG > 0 ? PTL_RREG : 1], tt[PTL_RREG > 0 ? PTL_RREG : 1], msg[PTL_RREG > 0 ? PTL_RREG : 1],
        rnd[PTL_RREG > 0 ? PTL_RREG : 1], root[PTL_RREG > 0 ? PTL_RREG : 1];
};
// record j's source, type word, message id, round and root
DEV void ptl_rec(const KArgs& a, const PtlRecs& R, uint32_t base, uint32_t j, uint32_t& src, uint32_t& tt,
                 uint32_t& msg, uint32_t& rnd, uint32_t& root) {
    if (j < (uint32_t)PTL_RREG) {
        src = R.src[0]; tt = R.tt[0]; msg = R.msg[0]; rnd = R.rnd[0]; root = R.root[0];
#pragma unroll
        for (int k = 1; k < PTL_RREG; k++)
            if (j == (uint32_t)k) { src = R.src[k]; tt = R.tt[k]; msg = R.msg[k]; rnd = R.rnd[k]; root = R.root[k]; }
    } else {
        const uint4* rq = reinterpret_cast<const uint4*>(a.rec_in + base + j);
        const uint4 q0 = rq[0], q1 = rq[1];
        src = q0.y; tt = q0.z; msg = q1.x; rnd = q1.y; root = q1.z;
    }
}
#ifdef PSIM_PTL_WPE      // (a waves-per-SIMD floor for the register allocator, for A/B builds)
#define PTL_BOUNDS __launch_bounds__(PTL_BLK) __attribute__((amdgpu_waves_per_eu(PSIM_PTL_WPE)))
#else
#define PTL_BOUNDS __launch_bounds__(PTL_BLK, PSIM_PTL_BLOCKS_PER_CU)
#endif
__global__ void PTL_BOUNDS k_ptl(RoundArgs) {
    if (*kargs().ctl) return;                         // an aborted batch (run_batch)
    enum { T_FIRST, T_FAIL, T_OVF, T_BOUND, T_DLV, T_EMT = T_DLV + 5, T_N = T_EMT + 5 };
    __shared__ unsigned long long sst[T_N + 1];       // (+ the digest)
    __shared__ uint32_t sslots[2 * PSIM_MSG_SLOTS];
    __shared__ uint32_t tabs[(2 * PTL_SET + 2 * PTL_CAP) * PTL_BLK];
    for (int i = threadIdx.x; i < 2 * PSIM_MSG_SLOTS; i += blockDim.x) sslots[i] = kargs().slots[i];
    if (threadIdx.x < T_N + 1) sst[threadIdx.x] = 0;
#ifdef PSIM_STAMPS
    __shared__ unsigned long long ptl_st[16];
    if (threadIdx.x < 16) ptl_st[threadIdx.x] = threadIdx.x == 15 ? __builtin_amdgcn_s_memtime() : 0ull;
#endif
    __syncthreads();
    const uint32_t l = lane_id();
    const uint32_t nq0 = kargs().n_ptl[0], nq = nq0 + kargs().n_ptl[1];
    uint32_t v[T_N] = {};
    uint64_t dig = 0;
    const uint32_t X0[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    PtLane n;
    n.EG.p = tabs + threadIdx.x;
    n.LZ.p = tabs + PTL_SET * PTL_BLK + threadIdx.x;
    n.OL.p = tabs + 2 * PTL_SET * PTL_BLK + threadIdx.x;
    n.OH.p = tabs + (2 * PTL_SET + PTL_CAP) * PTL_BLK + threadIdx.x;
    for (uint32_t base = blockIdx.x * blockDim.x; base < nq; base += gridDim.x * blockDim.x) {
        KArgs& a = kargs();
        const uint32_t P = base + threadIdx.x;
        bool go = false, fall = false;
        uint4 D = make_uint4(0, 0, 0, 0);
        PtlRecs R;
        uint32_t root0 = NONE, rtw4 = 0, rtw5 = 0, w10 = 0, w11 = 0, start = 0, act_n = 0, tmask = 0;
        uint16_t up[PSIM_ACTIVE_CAP];
        if (P < nq) {
            D = ptl_desc(a, nq0, P);
            const size_t li = D.x - a.lo;
            const uint32_t* hp = reinterpret_cast<const uint32_t*>(a.hdr + li);
            // (the active row and the partition byte with the node's rows:
            // loaded after its precondition pass, they and the members' pairs
            // were two more dependent memory waits before its handlers)
            const uint4* ar = reinterpret_cast<const uint4*>(a.act + li * PSIM_ACTIVE_CAP);
            const uint4 a0 = ar[0], a1 = ar[1];
            n.me_part = a.part[D.x];
            const uint4 hq1 = reinterpret_cast<const uint4*>(hp)[1], hq2 = reinterpret_cast<const uint4*>(hp)[2];
            start = hp[2];
            act_n = hq2.y & 0xFF;                     // word 9
            w10 = hq2.z; w11 = hq2.w;
            const uint4* rr = reinterpret_cast<const uint4*>(a.pt_rt + li * RT_WORDS);
            const uint4 r0 = rr[0], r1 = rr[1];
            root0 = r0.x; rtw4 = r1.x; rtw5 = r1.y;
            n.id = D.x;
            n.act_n = act_n;
            n.A[0] = a0.x; n.A[1] = a0.y; n.A[2] = a0.z; n.A[3] = a0.w;
            n.A[4] = a1.x; n.A[5] = a1.y; n.A[6] = a1.z; n.A[7] = a1.w;
            ptl_load_pairs(a, n, up);
            // the lane's preconditions over the inbox's Plumtree messages
            const uint32_t ik = start == a.round ? 0u : (D.z & DESC_CNT_MASK);
            // eager / lazy adds this inbox can make: a BROADCAST adds its
            // sender to one of them (first delivery: eager, else lazy), an
            // IHAVE of a missing id and a GRAFT to eager, a PRUNE to lazy
            // (plumtree:288-313; an IGNORED_I_HAVE to neither)
            uint32_t n_eg = 0, n_lz = 0, r0t = root0;
            uint64_t bm = 0;                          // message slots of the BROADCASTs
            // (an outstanding extension row taken earlier holds zeros while the
            // table fits its own row: this round's adds must fit that row)
            // (a connection table -- lingering peers, or active members
            // without a connection -- of at most PTL_CN entries is read below
            // for the sends' tests; a larger one, or X-BOT's closing entries,
            // go to k_pt: at the C line's broadcast peak every node k_pt took
            // held one, profiles/r05/ab_log.txt r6u)
            bool ok = r0.y == NONE && r0.z == NONE && r0.w == NONE &&
                      (PSIM_PTL_CONN ? (w11 >> 24) == 0 && (w11 & 0xFFu) <= PTL_CN : (w11 & 0xFFFFu) == 0) &&
                      (root0 == NONE || ((rtw4 >> 8) == 0 && (rtw5 >> 8) == 0));
#pragma unroll
            for (int j = 0; j < PTL_RREG; j++) {      // (all issued before the first is used)
                uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;
                if ((uint32_t)j < ik) {
                    const uint4* rq = reinterpret_cast<const uint4*>(a.rec_in + D.y + j);
                    q0 = rq[0]; q1 = rq[1];
                }
                R.src[j] = q0.y; R.tt[j] = q0.z; R.msg[j] = q1.x; R.rnd[j] = q1.y; R.root[j] = q1.z;
            }
            for (uint32_t j = 0; ok && j < ik; j++) {
                uint32_t src, tt, msg, rnd, root;
                ptl_rec(a, R, D.y, j, src, tt, msg, rnd, root);
                const uint32_t type = tt & 0xFF;
                if (type < PSIM_MSG_PT_BROADCAST || type > PSIM_MSG_PT_GRAFT) continue;
                n_eg += type == PSIM_MSG_PT_BROADCAST || type == PSIM_MSG_PT_IHAVE || type == PSIM_MSG_PT_GRAFT;
                n_lz += type == PSIM_MSG_PT_BROADCAST || type == PSIM_MSG_PT_PRUNE;
                tmask |= 1u << type;
                if (type == PSIM_MSG_PT_BROADCAST) bm |= 1ull << (msg % PSIM_MSG_SLOTS);
                if (type != PSIM_MSG_PT_IGNORED_IHAVE) {
                    if (r0t == NONE) r0t = root;      // the root a first update would store
                    ok &= root == r0t;
                }
            }
            // first deliveries (lazy adds): the BROADCASTs' slots not delivered yet
            const uint32_t nb = popc(bm & ~(((uint64_t)hq1.y << 32) | hq1.z));
            const uint32_t com_n = w10 >> 24, out_n = (w11 >> 16) & 0xFF;
            const uint32_t ne0 = root0 == NONE ? com_n : (rtw4 & 0xFF), nl0 = root0 == NONE ? 0u : (rtw5 & 0xFF);
            ok &= ne0 + n_eg <= (uint32_t)PTL_SET && nl0 + n_lz <= (uint32_t)PTL_SET &&
                  out_n + nb * (nl0 + n_lz) <= (uint32_t)PTL_CAP;
            go = ok;
            fall = !ok;
        }
        PTL_STAMP(0);
        // nodes that do not fit go to k_pt's list: one atomic a wave (a block
        // is one wave), its return waited for only where the list entries are
        // written, after the node's handlers
        const uint64_t fm = ballot(fall);
        uint32_t fbase = 0;
        if (fm && lane_id() == 0) fbase = atomicAdd(kargs().n_pt, (uint32_t)popc(fm));
        PTL_STAMP(1);
        if (go) {
        const uint32_t id = D.x;
        const size_t li = id - a.lo;
        n.cmask = ptl_conn_mask(a, n, up);
#if PSIM_PTL_CONN
        n.lmask = 0;
        {
            // the connection table (k_pt's conn_has, pt:633-638): an active
            // member marked PSIM_CONN_DOWN has no connection; an entry without
            // a flag is a lingering peer with one (no closing entries here:
            // X-BOT's go to k_pt)
            const uint32_t cn = w11 & 0xFFu;
            uint32_t CN[PTL_CN] = {};
            if (cn) {
                const uint4 c0 = *reinterpret_cast<const uint4*>(a.conn + li * PSIM_CONN_CAP);
                CN[0] = c0.x; CN[1] = c0.y; CN[2] = c0.z; CN[3] = c0.w;
            }
            uint32_t down = 0, inA = 0;
#pragma unroll
            for (int k = 0; k < (int)PTL_CN; k++) {
                const uint32_t e = CN[k];
                bool ina = false;
#pragma unroll
                for (int j = 0; j < PSIM_ACTIVE_CAP; j++) {
                    down |= ((uint32_t)k < cn && (uint32_t)j < act_n && e == (n.A[j] | PSIM_CONN_DOWN)) ? 1u << j : 0u;
                    ina |= (uint32_t)j < act_n && n.A[j] == e;
                }
                inA |= ina ? 1u << k : 0u;
            }
            n.cmask &= ~down;
            upart_t lup[PTL_CN];
#pragma unroll
            for (int k = 0; k < (int)PTL_CN; k++) {
                const bool lg = (uint32_t)k < cn && !(CN[k] & (PSIM_CONN_DOWN | PSIM_CONN_CLOSING)) && CN[k] < a.n_nodes;
                n.L[k] = lg ? CN[k] : NONE;
                lup[k] = lg ? a.upart[CN[k]] : UPART_DOWN;
            }
#pragma unroll
            for (int k = 0; k < (int)PTL_CN; k++)
                n.lmask |= (n.L[k] != NONE && n.L[k] != id && !((inA >> k) & 1u) && (uint32_t)lup[k] == n.me_part)
                               ? 1u << k : 0u;
        }
#endif
        PTL_STAMP(2);
        n.root0 = root0;
        n.ne = root0 == NONE ? 0u : (rtw4 & 0xFF);
        n.nl = root0 == NONE ? 0u : (rtw5 & 0xFF);
        // the sets only for messages that may update them, the table only for
        // lazy adds, acks or a lazy tick (the rest is never read, nor stored)
        const bool need_sets = (tmask & ((1u << PSIM_MSG_PT_BROADCAST) | (1u << PSIM_MSG_PT_PRUNE) |
                                         (1u << PSIM_MSG_PT_IHAVE) | (1u << PSIM_MSG_PT_GRAFT))) != 0;
        const bool need_out = (tmask & ((1u << PSIM_MSG_PT_BROADCAST) | (1u << PSIM_MSG_PT_IGNORED_IHAVE))) != 0 ||
                              (((D.z >> 28) & DESC_LAZY) && ((w11 >> 16) & 0xFF) > 0);
        if (need_sets) {
            const uint4* er = reinterpret_cast<const uint4*>(a.pt_eag + li * RT_SET);
            const uint4* lr = reinterpret_cast<const uint4*>(a.pt_laz + li * RT_SET);
#pragma unroll
            for (int q = 0; q < (PTL_SET + 3) / 4; q++) {  // (a capacity not a multiple of 4: the tail quad's first words)
                const uint4 e = er[q], z = lr[q];
                const uint32_t E4[4] = {e.x, e.y, e.z, e.w}, Z4[4] = {z.x, z.y, z.z, z.w};
#pragma unroll
                for (int k = 0; k < 4; k++)
                    if (4 * q + k < PTL_SET) { n.EG[4 * q + k] = E4[k]; n.LZ[4 * q + k] = Z4[k]; }
            }
        }
        if (need_out) {
            const uint4* orow = reinterpret_cast<const uint4*>(a.pt_out + li * OUT_IN);
#pragma unroll
            for (int q = 0; q < PTL_CAP / 2; q++) {
                const uint4 o = orow[q];
                n.OL[2 * q] = o.x; n.OH[2 * q] = o.y; n.OL[2 * q + 1] = o.z; n.OH[2 * q + 1] = o.w;
            }
        }
        const uint32_t com_n = w10 >> 24;
        const uint32_t* hp = reinterpret_cast<const uint32_t*>(a.hdr + li);
        n.on = (w11 >> 16) & 0xFF;
        n.have = ((uint64_t)hp[5] << 32) | hp[6];
        n.sets_dirty = false; n.out_dirty = false;
        uint32_t trk_round = hp[7], trk_hop = hp[8];
        const uint32_t hw4 = hp[4];
        const uint8_t fl0 = a.flags[id];              // (read before the emissions' stores: see PtlRecs)
        uint32_t seq = a.ocnt[li];
        const uint32_t oend = (uint32_t)a.obase[li + 1];
#ifdef PSIM_STAMPS
        {   // (the loads above waited for here, as the first handler would)
            volatile uint32_t sink_ = n.EG[0] + n.OL[0] + hw4 + fl0 + seq + oend;
            (void)sink_;
        }
#endif
        PTL_STAMP(3);
        const uint32_t ik = start == a.round ? 0u : (D.z & DESC_CNT_MASK);
        for (uint32_t j = 0; j < ik; j++) {           // the Plumtree inbox, canonical order
            uint32_t src, tt, msg, rnd, root;
            ptl_rec(a, R, D.y, j, src, tt, msg, rnd, root);
            const uint32_t type = tt & 0xFF;
            if (type < PSIM_MSG_PT_BROADCAST || type > PSIM_MSG_PT_GRAFT) continue;
            const uint32_t from = src | PSIM_MAP_BIT;
            v[T_DLV + type - PSIM_MSG_PT_BROADCAST]++;
            // plumtree_backend is_stale/1 over the slots (a retired id: overflow, stale)
            const uint32_t sk = msg % PSIM_MSG_SLOTS;
            const bool live = sslots[sk] == msg;
            const bool have = !live || ((n.have >> sk) & 1ull);
            if (type != PSIM_MSG_PT_PRUNE && type != PSIM_MSG_PT_IGNORED_IHAVE && !live) v[T_OVF]++;
            uint32_t sto = NONE, stt = 0, sa0 = 0, sa1 = 0;     // a single send of the handler
            // update_peers/5 (pt:593-609) at one call site for every message:
            // to eager -- a first delivery, an IHAVE of a missing id, a GRAFT
            // of a held one; to lazy -- a duplicate, a PRUNE (a wave whose
            // lanes hold different messages ran one update per branch)
            const bool first = type == PSIM_MSG_PT_BROADCAST && !have;
            const bool to_eager = first || (type == PSIM_MSG_PT_IHAVE && !have) || (type == PSIM_MSG_PT_GRAFT && have);
            const bool to_lazy = (type == PSIM_MSG_PT_BROADCAST && have) || type == PSIM_MSG_PT_PRUNE;
            if (to_eager || to_lazy) ptl_update(a, n, li, com_n, from, root, to_eager);
            PTL_STAMP(4);
            if (type == PSIM_MSG_PT_BROADCAST) {     // pt:288-293, :368-378
                if (!have) {
                    n.have |= 1ull << sk;
                    v[T_FIRST]++;
                    if (msg == a.tracked_msg) { trk_round = a.round; trk_hop = rnd + 1; }
                    // eager_push/7 + schedule_lazy_push/6 over slot 0's sets
                    // (each entry's LDS read issued an iteration ahead of its
                    // use: the loop waited one LDS latency per member)
#if PSIM_PTL_PF
                    uint32_t e_nx = n.EG[0];
#endif
                    for (uint32_t i = 0; i < n.ne; i++) {
#if PSIM_PTL_PF
                        const uint32_t e = e_nx;
                        e_nx = n.EG[(i + 1) % PTL_SET];
#else
                        const uint32_t e = n.EG[i];
#endif
                        if (e == from) continue;
                        if (ptl_conn(a, n, e)) {
                            dig += relay_emit(a, D.w + seq, e & ~PSIM_MAP_BIT, id, PSIM_MSG_PT_BROADCAST, seq, msg, rnd + 1,
                                              root, X0);
                            seq++;
                            v[T_EMT + 0]++;
                        } else {
                            v[T_FAIL]++;
                        }
                    }
#if PSIM_PTL_LAZYM
                    ptl_add_lazy(n, from, (msg << 16) | ((rnd + 1) & 0xFFFFu));
#else
#if PSIM_PTL_PF
                    uint32_t z_nx = n.LZ[0];
#endif
                    for (uint32_t i = 0; i < n.nl; i++) {
#if PSIM_PTL_PF
                        const uint32_t e = z_nx;
                        z_nx = n.LZ[(i + 1) % PTL_SET];
#else
                        const uint32_t e = n.LZ[i];
#endif
                        if (e != from) ptl_add_out(n, ((uint64_t)e << 32) | (msg << 16) | ((rnd + 1) & 0xFFFFu));
                    }
#endif
                    PTL_STAMP(5);
                } else {                             // a duplicate: PRUNE back
                    sto = from; stt = PSIM_MSG_PT_PRUNE;
                }
            } else if (type == PSIM_MSG_PT_IHAVE) {  // pt:299-303, :380-386
                sto = from; stt = have ? PSIM_MSG_PT_IGNORED_IHAVE : PSIM_MSG_PT_GRAFT; sa0 = msg; sa1 = rnd;
            } else if (type == PSIM_MSG_PT_IGNORED_IHAVE) {   // pt:304-307
                ptl_ack_out(n, ((uint64_t)from << 32) | (msg << 16) | (rnd & 0xFFFFu));
                PTL_STAMP(9);
            } else if (type == PSIM_MSG_PT_GRAFT && have) {   // pt:308-313, :388-402
                sto = from; stt = PSIM_MSG_PT_BROADCAST; sa0 = msg; sa1 = rnd;
            }                                        // (PRUNE pt:294-298: the update only)
            if (sto != NONE) {                        // (the IHAVE answer goes before the update in
                if (ptl_conn(a, n, sto)) {            //  the reference; the update sends nothing)
                    dig += relay_emit(a, D.w + seq, src, id, stt, seq, sa0, sa1, root, X0);
                    seq++;
                    v[T_EMT + stt - PSIM_MSG_PT_BROADCAST]++;
                } else {
                    v[T_FAIL]++;
                }
                PTL_STAMP(10);
            }
        }
        PTL_STAMP(11);
        bool quiet = false;                              // (flag_byte's lazy_quiet)
        if (((D.z >> 28) & DESC_LAZY) && n.on > 0) {   // the lazy tick (pt:341-345, :443-453)
            const uint32_t seq0 = seq;
#if PSIM_PTL_PF
            uint64_t o_nx = out_at(n, 0);
#endif
            for (uint32_t i = 0; i < n.on; i++) {
#if PSIM_PTL_PF
                const uint64_t o = o_nx;
                o_nx = out_at(n, (i + 1) % PTL_CAP);
#else
                const uint64_t o = out_at(n, i);
#endif
                const uint32_t peer = (uint32_t)(o >> 32);
                if (!ptl_conn(a, n, peer)) { v[T_FAIL]++; continue; }
                const uint32_t msg = (uint32_t)(o >> 16) & 0xFFFFu, sk = msg % PSIM_MSG_SLOTS;
                const bool live = sslots[sk] == msg;
                v[T_OVF] += live ? 0u : 1u;
                dig += relay_emit(a, D.w + seq, peer & ~PSIM_MAP_BIT, id, PSIM_MSG_PT_IHAVE, seq, msg,
                                  (uint32_t)o & 0xFFFFu, live ? sslots[PSIM_MSG_SLOTS + sk] : NONE, X0);
                seq++;
                v[T_EMT + 2]++;
            }
            quiet = seq == seq0;
        }
        PTL_STAMP(12);
        // write back: header words 5-8 and 11, the sets, the table, the flag byte
        uint32_t* hw = reinterpret_cast<uint32_t*>(a.hdr + li);
        reinterpret_cast<uint4*>(hw)[1] = make_uint4(hw4, (uint32_t)(n.have >> 32), (uint32_t)n.have, trk_round);
        hw[8] = trk_hop;
        hw[11] = (w11 & ~0xFF0000u) | (n.on << 16);
        if (n.sets_dirty) {
            // (slots 1-3 stay free, the count words hold slot 0's counts only)
            uint4* rr = reinterpret_cast<uint4*>(a.pt_rt + li * RT_WORDS);
            rr[0] = make_uint4(n.root0, NONE, NONE, NONE);
            rr[1].x = n.ne;
            rr[1].y = n.nl;
            uint4* er = reinterpret_cast<uint4*>(a.pt_eag + li * RT_SET);
            uint4* lr = reinterpret_cast<uint4*>(a.pt_laz + li * RT_SET);
#pragma unroll
            for (int q = 0; q < PTL_SET / 4; q++) {
                er[q] = make_uint4(n.EG[4 * q], n.EG[4 * q + 1], n.EG[4 * q + 2], n.EG[4 * q + 3]);
                lr[q] = make_uint4(n.LZ[4 * q], n.LZ[4 * q + 1], n.LZ[4 * q + 2], n.LZ[4 * q + 3]);
            }
#pragma unroll
            for (int i = PTL_SET & ~3; i < PTL_SET; i++) {     // (the rest of the row is left as it was)
                a.pt_eag[li * RT_SET + i] = n.EG[i];
                a.pt_laz[li * RT_SET + i] = n.LZ[i];
            }
        }
        if (n.out_dirty) {
            uint4* orow = reinterpret_cast<uint4*>(a.pt_out + li * OUT_IN);
#pragma unroll
            for (int q = 0; q < PTL_CAP / 2; q++)
                orow[q] = make_uint4(n.OL[2 * q], n.OH[2 * q], n.OL[2 * q + 1], n.OH[2 * q + 1]);
        }
        a.ocnt[li] = seq;
        v[T_BOUND] += seq > oend - D.w ? 1u : 0u;
        a.flags[id] = (uint8_t)((fl0 & (F_UP | F_CRASHED)) | (n.on && !quiet ? F_LAZY : 0) |
                                (min(n.on, 15u) << F_OUTN_SHIFT) |
                                (act_n < a.min_active ? F_LOWACT : 0));
        PTL_STAMP(13);
        }
        if (fm) {
            fbase = (uint32_t)__shfl((int)fbase, 0);
            if (fall) kargs().desc_pt[fbase + popc(fm & ((1ull << lane_id()) - 1ull))] = D;
        }
    }
#ifdef PSIM_STAMPS
    PTL_STAMP(14);
    if (threadIdx.x < 15) atomicAdd(&g_stamps_lite[16 + threadIdx.x], ptl_st[threadIdx.x]);
#endif
#pragma unroll
    for (int k = 0; k < T_N; k++)
        for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o);
    for (int o = 32; o > 0; o >>= 1) dig += shfl64(dig, (int)((l + o) & 63));
    if (l == 0) {
        for (int k = 0; k < T_N; k++)
            if (v[k]) atomicAdd(&sst[k], (unsigned long long)v[k]);
        if (dig) atomicAdd(&sst[T_N], (unsigned long long)dig);
    }
    __syncthreads();
    uint64_t* row = kargs().stat_ptl + (size_t)blockIdx.x * NST;
    for (uint32_t k = threadIdx.x; k < NST; k += blockDim.x) {
        uint64_t x = 0;
        if (k == ST_FIRST) x = sst[T_FIRST];
        else if (k == ST_FAIL) x = sst[T_FAIL];
        else if (k == ST_OVF || k == ST_OVF_BY + PSIM_OVF_PT) x = sst[T_OVF];
        else if (k == ST_DIGEST) x = sst[T_N];
        else if (k == ST_BOUND) x = sst[T_BOUND];
        else if (k >= ST_DELIV + PSIM_MSG_PT_BROADCAST && k <= ST_DELIV + PSIM_MSG_PT_GRAFT)
            x = sst[T_DLV + k - ST_DELIV - PSIM_MSG_PT_BROADCAST];
        else if (k >= ST_EMIT + PSIM_MSG_PT_BROADCAST && k <= ST_EMIT + PSIM_MSG_PT_GRAFT)
            x = sst[T_EMT + k - ST_EMIT - PSIM_MSG_PT_BROADCAST];
        row[k] = x;
    }
}

// one wave-slot per resident wave: the grid strides over the active list
// with no second generation of waves (a partial generation is a tail)
static uint32_t resident_grid(const void* k, int block = WAVES_PER_BLOCK * 64) {
    int dev = 0, nb = 0;
    hipDeviceProp_t p;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, block, 0) != hipSuccess || nb <= 0)
        return 1024;
    return (uint32_t)nb * (uint32_t)p.multiProcessorCount;
}
uint32_t consume_grid() { return resident_grid((const void*)k_consume); }
uint32_t lite_grid() { return resident_grid((const void*)k_consume_lite, 64 * LITE_WPB); }
uint32_t lite_block() { return 64 * LITE_WPB; }
uint32_t pt_grid() { return resident_grid((const void*)k_pt); }
uint32_t ptl_grid() { return resident_grid((const void*)k_ptl, PTL_BLK); }

#ifdef PSIM_STAMPS
int debug_stamps(unsigned long long* out) {
    // k_consume / k_pt phases in out[0..31], k_consume_lite's in out[32..63]
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 32) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out + 32, HIP_SYMBOL(g_stamps_lite), sizeof(unsigned long long) * 32) != hipSuccess)
        return -1;
    unsigned long long z[32] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof z) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps_lite), z, sizeof z) != hipSuccess) return -1;
    // k_lite_half's, when it ran (psim_lite.hip): 96 entries
    if (debug_stamps_half(out + 64) != 32) return -1;
    return 96;
}
#else
int debug_stamps(unsigned long long*) { return 0; }
#endif

// this TU's layout (psim_kernels.h layout_sig, checked by psim_create)
uint32_t layout_sig_consume() { return layout_sig(); }

}  // namespace psim
