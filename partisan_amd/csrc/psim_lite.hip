// psim_lite.hip -- k_lite_half: the SHUFFLE-exchange phase of k_relay's
// lite list (hv:1091-1136 terminals, replies and relays, then a due
// passive_view_maintenance start hv:572-607) with TWO nodes per wave.
//
// The wave-per-node kernel (k_consume_lite, psim_consume.hip) spent its time
// on one node's serial chain of dependent scalar and vector steps: 8.9 k SALU
// against 9.4 k VALU instructions per wave, issuing on 30 % of its cycles
// (profiles/r03/p38/sq_kernels.txt).  Every list here is at most 32 entries
// (passive <= 30, active <= 8, exchanges <= 8), so a 64-lane wave carries two
// nodes, one per 32-lane half, and every value that was wave-uniform -- a
// node's draw counter, view sizes, the element a step picks -- lives in a
// VGPR that holds the same value across its half.  List operations become
// per-half VALU work with no SALU decisions:
//   membership / count   the half's 32 ballot bits (hmask) and v_bcnt
//   element j            ds_bpermute within the half (hget)
//   insert in to_list    a per-lane prefix predicate on the bucket tags and
//     order              whole-wave DPP shifts (lane 32 never takes lane 31's)
//   sublist(shuffle)     one Philox draw per lane, each lane's rank among the
//                        half's keys (an exact recount on a top-32-bit tie)
// so one instruction stream advances two nodes.  Control flow diverges only
// between the halves (exec-masked), never inside one.  The handlers are the
// wave kernel's -- the same draws, records, sequence numbers, digest, stats
// and rows -- which the GPU parity tests check against the oracle; the wave
// kernel stays for A/B (PSIM_LITE_WAVE=1).
//
// Reference: hv = src/partisan_hyparview_peer_service_manager.erl
#include <utility>

#include "psim_device.h"
#include "psim_kernels.h"
#include "psim_wave.h"

namespace psim {

namespace {

constexpr uint32_t HSTAGE = 16;                 // staged records per half
#ifndef PSIM_HALF_WPB
#define PSIM_HALF_WPB 4
#endif
#ifndef PSIM_HALF_WAVES
#define PSIM_HALF_WAVES 4
#endif
constexpr uint32_t HWPB = PSIM_HALF_WPB;        // waves per block

// Diagnostic build only (-DPSIM_STAMPS, `make stamps`): s_memtime between
// phase boundaries, per half (slot half * 16 + phase), summed over all waves
// into g_stamps_half (debug_stamps_half; profiles/stamps.py).  A phase both
// halves run is charged to each; one only the other half runs goes to this
// half's next stamp.
#ifdef PSIM_STAMPS
__device__ unsigned long long g_stamps_half[32];
#define HSTAMP(w, k)                                                                 \
    do {                                                                             \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();                            \
        if (hl_id() == 0) (w).stl[(hb_id() >> 1) + (k)] += t_ - (w).t_last;          \
        (w).t_last = t_;                                                             \
    } while (0)
#else
#define HSTAMP(w, k) do { } while (0)
#endif

DEV uint32_t hl_id() { return __lane_id() & 31u; }
DEV uint32_t hb_id() { return __lane_id() & 32u; }

// the 32 ballot bits of this lane's half
DEV uint32_t hmask(bool p) {
    const uint64_t b = __ballot(p);
    return (__lane_id() & 32u) ? (uint32_t)(b >> 32) : (uint32_t)b;
}
DEV bool hany(bool p) { return hmask(p) != 0u; }
// lane j (< 32, per lane) of this lane's half
DEV uint32_t hget(uint32_t v, uint32_t j) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((hb_id() + (j & 31u)) << 2), (int)v);
}
DEV uint64_t hget64(uint64_t v, uint32_t j) {
    return ((uint64_t)hget((uint32_t)(v >> 32), j) << 32) | hget((uint32_t)v, j);
}
// lane J (a constant) of this lane's half: ds_swizzle in bitmask mode
// (and 0, or J: each 32-lane group reads its lane J) -- no address register,
// so the unrolled loops below keep no per-J constants live.
// Every cross-lane read (hget, hgetc, the DPP shifts) must run with the whole
// half active: a source lane outside the exec mask reads as 0.  So none of
// them sits on the right of a per-lane && or ?: -- each is its own statement.
template <int J>
DEV uint32_t hgetc(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, J << 5);
}
// f(J) for J = 0 .. N - 1, J a compile-time constant
template <class F, int... J>
DEV void unroll_seq(F&& f, std::integer_sequence<int, J...>) {
    (f(std::integral_constant<int, J>{}), ...);
}
template <int N, class F>
DEV void unroll(F&& f) {
    unroll_seq(f, std::make_integer_sequence<int, N>{});
}
// lane j of this lane's half for a j every active lane agrees on (a loop
// counter both halves step together): two v_readlane, no LDS round trip --
// the dependent chains below wait on this broadcast at every step
DEV uint32_t hget_u(uint32_t v, uint32_t j) {
    const uint32_t ju = __builtin_amdgcn_readfirstlane(j);
    const uint32_t a = __builtin_amdgcn_readlane(v, ju), b = __builtin_amdgcn_readlane(v, ju + 32);
    return hb_id() ? b : a;
}
// lane 0 of this lane's half
DEV uint32_t hget_c0(uint32_t v) {
    const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 32);
    return hb_id() ? b : a;
}
// order-preserving delete of entry k / insert of e at pos in a half's list of
// n entries (lanes >= n hold 0): the whole-wave DPP shifts of psim_wave.h --
// a half's lane 31 reads lane 32 only when n > 32, and lane 32 (its lane 0)
// never takes lane 31's value
DEV uint32_t hdel(uint32_t V, uint32_t n, uint32_t k) {
    const uint32_t l = hl_id(), nx = from_next(V);
    return l < k ? V : (l + 1 < n ? nx : 0u);
}

// one node per half: everything here is per lane, equal across the half
struct Hn {
    uint32_t me, ob, ib, ik;
    uint32_t fl;                     // the due timers (DESC_* bits, k_desc) | HF_PDIRTY | partition << 8
                                     // | header word 9's bytes 2-3 << 16 (kept for the writeback)
    uint32_t act_n, pas_n;
    uint64_t rng;                    // the Philox draw counter
    uint32_t A, P;                   // lane hl: active[hl] (hl < 8), passive[hl]
    uint32_t AF;                     // bit j: active member j is up in this node's group (k_relay's
                                     // RoundArgs::lite_cm); bits 8..: the outbox's slots,
                                     // obase[row + 1] - ob (out_cap), saturating at 2^24 - 1
    uint32_t seq, flushed;
    uint64_t dcb;                    // draw cache: lane hl holds the draw of counter dcb + hl
    uint32_t DCL, DCH;
};
constexpr uint32_t HF_PDIRTY = 16;  // Hn::fl: the passive view changed
DEV uint32_t local_row(const Hn& x) { return x.me - kargs().lo; }
// the node's outbox slots: no store goes past them (a record past the bound
// is not stored -- the engine fails the round on the bound check)
DEV uint32_t out_cap(const Hn& x) { return x.AF >> 8; }

// a node's counters (each half counts its own node's; lane 0 of the half
// adds them to the block's stats at the node's end), and the wave's digest
struct Hc {                           // (summed over the half's nodes: < 2^16 each)
    uint32_t dl;                     // SHUFFLE | SHUFFLE_REPLY << 16 delivered
    uint32_t em;                     // SHUFFLE | SHUFFLE_REPLY << 16 emitted
    uint32_t pb;                     // nodes | bound violations << 16
    uint32_t fail;
    uint64_t digest;                 // lane j < 16 of a half sums word j of its records
};

struct Hw {                          // the wave's LDS
    unsigned long long* sst;         // the block's stats (NST)
    uint32_t* srec;                  // 2 halves x HSTAGE records x 16 words
    uint32_t* skey;                  // 2 halves x HSTAGE route keys
    uint32_t* scr;                   // 2 halves x 32 words of scratch
    uint32_t KM;                     // lane hl: kMagic[hl] (exact modulo, n < 32)
#ifdef PSIM_STAMPS
    unsigned long long* stl;         // 2 halves x 16 phase sums (LDS)
    uint64_t t_last;
#endif
};

// ------------------------------------------------------------------ RNG --
DEV void dc_fill(Hn& x, uint64_t base) {
    const uint64_t v = draw58_at(base + hl_id(), x.me, kargs().seed);
    x.DCL = (uint32_t)v; x.DCH = (uint32_t)(v >> 32);
    x.dcb = base;
}
DEV uint64_t draw(Hn& x) {
    const uint64_t c = x.rng++;
    if (c < x.dcb || c - x.dcb >= 32) dc_fill(x, c);
    const uint32_t i = (uint32_t)(c - x.dcb);
    return ((uint64_t)hget(x.DCH, i) << 32) | hget(x.DCL, i);
}
// rand:uniform(n), n < 32 (OTP rand.erl ?uniform_range on 58-bit draws)
DEV uint32_t uniform_n(Hn& x, const Hw& w, uint32_t n) {
    const uint64_t two58 = 1ull << 58;
    const uint32_t M = hget(w.KM, n);
    for (;;) {
        const uint64_t v = draw(x);
        if (v < n) return (uint32_t)v + 1;
        const uint32_t i = mod_small_m(v, n, M);
        if (v - i <= two58 - n) return i + 1;
    }
}

// select_random/2 (hv:1346-1356): rand:uniform(length(View -- Omit)), no
// draw when nothing is eligible
DEV uint32_t select_random(Hn& x, const Hw& w, uint32_t V, uint32_t n, uint32_t o0, uint32_t o1) {
    const uint32_t l = hl_id();
    uint32_t M = hmask(l < n && V != o0 && V != o1);
    const uint32_t cnt = (uint32_t)__popc(M);
    if (cnt == 0) return PSIM_NONE;
    const uint32_t k = uniform_n(x, w, cnt) - 1;
    // the k-th eligible lane: the one with k eligible lanes below it (no
    // loop of up to k steps, whose count differs between the halves)
    const bool hit = ((M >> l) & 1u) && (uint32_t)__popc(M & ((1u << l) - 1u)) == k;
    return hget(V, (uint32_t)__ffs(hmask(hit)) - 1);
}

// lists:sublist(shuffle(to_list(View)), K) (hv:1359-1361, :1586-1587): one
// rand:uniform() key per element (element l draws counter rng + l), the K
// smallest (key, element) pairs in order, appended to OUT at lanes on..
template <int MAXN>
DEV uint32_t sublist(Hn& x, Hw& w, uint32_t V, uint32_t n, uint32_t k, uint32_t& OUT, uint32_t on) {
    const uint32_t l = hl_id();
    const uint64_t base = x.rng;
    if (base < x.dcb || base + n > x.dcb + 32) dc_fill(x, base);      // cover [base, base + n)
    const uint32_t src = (uint32_t)(base - x.dcb) + l;                // (lanes >= n: unused)
    const uint64_t v = ((uint64_t)hget(x.DCH, src) << 32) | hget(x.DCL, src);
    const uint64_t key = l < n ? v >> 5 : ~0ull;
    const uint32_t m = n < k ? n : k;
    const uint32_t hi = (uint32_t)(key >> 21);
    // rank on the top 32 of the 53 key bits (n <= MAXN: lanes >= n hold ~0
    // and count for no lane below n); two lanes of one rank -- a tie, about
    // once in 10^7 sublists -- show as a rank slot another lane took, and the
    // ranks are recounted exactly on (key, element)
    uint32_t rank = 0;
    unroll<MAXN>([&](auto J) {
        const uint32_t hj = hgetc<J>(hi);
        rank += hj < hi ? 1u : 0u;
        // (at most eight swizzles in flight: the scheduler would otherwise
        // issue all of them first and hold MAXN results in registers)
        if constexpr (J % 8 == 7) __builtin_amdgcn_sched_barrier(0);
    });
    uint32_t* s = w.scr + hb_id();
    if (l < n) s[rank] = l;
    __builtin_amdgcn_wave_barrier();
    const uint32_t owner = s[rank & 31];
    __builtin_amdgcn_wave_barrier();
    if (hany(l < n && owner != l)) {
        rank = 0;
        for (uint32_t j = 0; j < n; j++) {
            const uint64_t kj = hget64(key, j);
            const uint32_t ej = hget(V, j);
            rank += (kj < key || (kj == key && ej < V)) ? 1u : 0u;
        }
    }
    if (l < n && rank < m) s[rank] = V;
    __builtin_amdgcn_wave_barrier();
    const uint32_t got = s[(l - on) & 31];
    __builtin_amdgcn_wave_barrier();
    OUT = (l >= on && l < on + m) ? got : OUT;
    x.rng = base + n;
    return on + m;
}

// lists:usort of E's lanes with `valid` (at most 8: lanes 0-7): E gets the
// sorted distinct values in lanes 0.., zeros above; returns their count
DEV uint32_t husort(Hw& w, uint32_t& E, bool valid) {
    const uint32_t l = hl_id();
    const uint32_t v = valid ? E : PSIM_NONE;
    bool dup = false;
    unroll<8>([&](auto J) {
        const uint32_t vj = hgetc<J>(v);
        dup |= ((uint32_t)J < l) & (vj == v);
    });
    const uint32_t u = valid && !dup ? v : PSIM_NONE;                 // first occurrences
    uint32_t rank = 0;
    unroll<8>([&](auto J) { rank += hgetc<J>(u) < u ? 1u : 0u; });
    const uint32_t c = (uint32_t)__popc(hmask(u != PSIM_NONE));
    uint32_t* s = w.scr + hb_id();
    if (u != PSIM_NONE) s[rank] = u;
    __builtin_amdgcn_wave_barrier();
    const uint32_t got = s[l];
    __builtin_amdgcn_wave_barrier();
    E = l < c ? got : 0u;
    return c;
}

// ------------------------------------------------------------- emission --
DEV void flush(Hn& x, Hw& w) {
    const uint32_t l = hl_id(), h = hb_id() >> 5;
    const uint32_t cnt = x.seq - x.flushed;
    const uint32_t cap = out_cap(x);
    __builtin_amdgcn_wave_barrier();
    const uint32_t* sr = w.srec + h * (HSTAGE * 16);
    const uint32_t* sk = w.skey + h * HSTAGE;
    // 16-B piece l & 3 of record l >> 2, eight records a pass
    for (uint32_t j0 = 0; j0 < cnt; j0 += 8) {
        const uint32_t j = j0 + (l >> 2);
        if (j < cnt && x.flushed + j < cap)
            reinterpret_cast<uint4*>(kargs().rec_out + x.ob + x.flushed + j)[l & 3] =
                reinterpret_cast<const uint4*>(sr + j * 16)[l & 3];
    }
    if (l < cnt && x.flushed + l < cap) kargs().okey[x.ob + x.flushed + l] = sk[l];
    __builtin_amdgcn_wave_barrier();
    x.flushed = x.seq;
}

// one record (psim_device.h Msg) into the half's staging buffer: lanes 0-15
// of the half write its words, lanes 8-15 taking the exchange ids of lanes
// 0-7 (DPP row_shr:8, inside the half's first row)
DEV void emit(Hn& x, Hw& w, Hc& c, uint32_t dst, uint32_t type, uint32_t ttl, uint32_t EX, uint32_t nex) {
    const uint32_t l = hl_id(), h = hb_id() >> 5;
    const uint32_t k = x.seq - x.flushed;
    const uint32_t tt = type | (ttl << 8) | (nex << 16);
    const uint32_t exv = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)EX, 0x118, 0xF, 0xF, true);
    const uint32_t word = l == 0 ? dst : l == 1 ? x.me : l == 2 ? tt : l == 3 ? x.seq
                        : l < 8 ? 0u : (l - 8 < nex ? exv : 0u);
    if (l < 16) {
        w.srec[(h * HSTAGE + k) * 16 + l] = word;
        c.digest += (uint64_t)word * digest_mul(l);      // (l < 16: record word l's multiplier)
    }
    if (l == 0) w.skey[h * HSTAGE + k] = dst | (max_emit(type) << KEY_DST_BITS);
    x.seq++;
    c.em += type == PSIM_MSG_SHUFFLE ? 1u : 0x10000u;
    if (k + 1 == HSTAGE) flush(x, w);
}

// maybe_connect + find (partisan_util.erl:75-134): the peer runs and no
// partition separates the two.  Every lite send goes to an active member
// (k_relay sends a walk that ends at a Sender outside the active view to
// k_consume), read from the connection cache; others from the pair array.
DEV bool connect_ok(const Hn& x, uint32_t dst) {
    KArgs& a = kargs();
    if (dst >= a.n_nodes || dst == x.me) return false;
    const uint32_t m = hmask(hl_id() < x.act_n && x.A == dst);
    if (m) return (x.AF >> (__ffs(m) - 1)) & 1u;
    return (uint32_t)a.upart[dst] == ((x.fl >> 8) & 0xFFu);
}

// do_send_message/3 (hv:1274-1343) after maybe_connect: the dispatch draw of
// partisan_util:dispatch_pid/1 (util:190-195), then the record
DEV void hv_send(Hn& x, Hw& w, Hc& c, uint32_t dst, uint32_t type, uint32_t ttl, uint32_t EX, uint32_t nex) {
    if (!connect_ok(x, dst)) { c.fail++; return; }
    x.rng++;
    emit(x, w, c, dst, type, ttl, EX, nex);
}

// ------------------------------------------------------- view updates --
// the half's passive view P with its bucket tags PB (sets v1 order): t into
// to_list order -- after every entry whose bucket is <= t's
DEV void pas_insert(Hn& x, uint32_t& PB, uint32_t t, uint32_t b) {
    const uint32_t l = hl_id(), n = x.pas_n;
    const bool le = l < n && PB <= b;                 // a prefix of the half
    const uint32_t lep = from_prev(le ? 1u : 0u), pv = from_prev(x.P), pbv = from_prev(PB);
    const bool at = l <= n && (l == 0 || lep);        // the first lane past the prefix
    x.P = le ? x.P : at ? t : (l <= n ? pv : 0u);
    PB = le ? PB : at ? b : (l <= n ? pbv : 0u);
    x.pas_n = n + 1;
    x.fl |= HF_PDIRTY;
}

// merge_exchange/2 (hv:1590-1595): add_to_passive/2 (hv:1423-1448) for each
// of usort(Exchange) -- Active -- [Myself], in order.  A full passive view
// evicts select_random(Passive, [Myself]) first: rand:uniform(|Passive|),
// Myself never being in Passive.  With |Passive| = max_passive_size at every
// eviction the draws are taken together (lane i: the i-th eviction's index);
// one the ?uniform_range test would reject (p ~ 2^-53) sends the half down
// the step-by-step draws instead.
// sorted: EX is already usort'ed -- a SHUFFLE's exchange (hv:586: every
// shuffle start sends lists:usort(Exchange0), and relays pass it on
// unchanged) -- so the candidates are its valid lanes in order, compacted
// through LDS (no 8 x 8 swizzle rank: terminals are half of the merges)
#ifndef PSIM_MERGE_SORTED     // (0: every merge through husort, for A/B)
#define PSIM_MERGE_SORTED 1
#endif
DEV void merge_exchange(Hn& x, Hw& w, uint32_t EX, uint32_t nex, bool sorted) {
    KArgs& a = kargs();
    const uint32_t l = hl_id();
    bool in_act = false;
    unroll<8>([&](auto J) {
        const uint32_t aj = hgetc<J>(x.A);
        in_act |= ((uint32_t)J < x.act_n) & (aj == EX);
    });
    uint32_t T = EX;
    const bool valid = l < nex && EX != x.me && !in_act;
    uint32_t mt;
    if (PSIM_MERGE_SORTED && sorted) {
        const uint32_t vm = hmask(valid);
        uint32_t* sc = w.scr + hb_id();
        if (valid) sc[__popc(vm & ((1u << l) - 1u))] = EX;
        __builtin_amdgcn_wave_barrier();
        mt = (uint32_t)__popc(vm);
        const uint32_t got = sc[l];
        __builtin_amdgcn_wave_barrier();
        T = l < mt ? got : 0u;
    } else {
        mt = husort(w, T, valid);
    }
    if (!mt) return;
    const uint32_t maxp = a.max_passive;
    const uint8_t* bt = a.btab;
    uint32_t PB = l < x.pas_n ? bucket16(bt, x.P) : 0u;
    const uint32_t TB = l < mt ? bucket16(bt, T) : 0u;        // the candidates' buckets
    const uint64_t c0 = x.rng;
    if (c0 < x.dcb || c0 + mt > x.dcb + 32) dc_fill(x, c0);         // cover [c0, c0 + mt)
    const uint32_t src = (uint32_t)(c0 - x.dcb) + l;
    const uint64_t v = ((uint64_t)hget(x.DCH, src) << 32) | hget(x.DCL, src);
    const uint32_t KI = mod_small_m(v, maxp, hget(w.KM, maxp));
    const bool par = !hany(l < mt && v >= maxp && v - KI > (1ull << 58) - maxp);
    uint32_t used = 0;
    if (par) {
        // branch-free steps, unrolled: candidate I of the half (a no-op past
        // mt or when already a member) evicts the index in K's lane 0 when
        // the view is full, then goes in at its bucket's position.  An entry
        // and its bucket are one tag, bucket << 27 | id (ids < 2^27,
        // KEY_DST_MASK), lanes past the count hold TSENT: the entries of a
        // bucket <= t's are the tags <= t's bucket | 0x07FFFFFF (a prefix),
        // membership is tag equality (a candidate past mt is TSENT and
        // matches the empty lanes: a no-op), and eviction + insertion is one
        // select per lane among its own, its predecessor's and its
        // successor's tag and t's
        constexpr uint32_t TSENT = 0xFFFFFFFFu, IDM = (1u << 27) - 1;
        uint32_t PT = l < x.pas_n ? (PB << 27) | x.P : TSENT;
        const uint32_t TG = l < mt ? (TB << 27) | T : TSENT;
        uint32_t K = KI;                             // the next eviction's index in the half's lane 0
        uint32_t n = x.pas_n, dirty = 0;
        // every candidate's tag fetched up front: one LDS wait, not one a
        // step (the half's step chain waited on its swizzle each step;
        // phase 0.505 -> 0.502 ms, profiles/r05/ab_log.txt)
        uint32_t TT8[PSIM_EXCHANGE_CAP];
        unroll<PSIM_EXCHANGE_CAP>([&](auto I) { TT8[I] = hgetc<I>(TG); });
        __builtin_amdgcn_sched_barrier(0);
        unroll<PSIM_EXCHANGE_CAP>([&](auto I) {
            const uint32_t tt = TT8[I];
            const bool mem = hany(PT == tt);
            const bool ev = !mem && n >= maxp;       // select_random(Passive, [Myself]) + remove
            const uint32_t k = hget_c0(K);
            const uint32_t kn = from_next(K), pv = from_prev(PT), nx = from_next(PT);
            K = ev ? kn : K;
            used += ev ? 1u : 0u;
            // entries of a bucket <= t's, then t's position once lane k is gone
            const uint32_t c = (uint32_t)__popc(hmask(PT <= (tt | IDM)));
            const uint32_t p = c - ((ev && k < c) ? 1u : 0u);
            const bool gone = ev && l >= k, gone1 = ev && l >= k + 1;   // (l - 1 >= k)
            const uint32_t F = l < p ? (gone ? nx : PT) : l == p ? tt : (gone1 ? PT : pv);
            PT = mem ? PT : F;
            n += (mem ? 0u : 1u) - (ev ? 1u : 0u);
            dirty |= mem ? 0u : 1u;
        });
        x.pas_n = n;
        x.P = PT == TSENT ? 0u : PT & IDM;
        x.fl |= dirty ? HF_PDIRTY : 0u;
    } else {
        for (uint32_t i = 0; i < mt; i++) {          // step by step, with ?uniform_range redraws
            const uint32_t t = hget_u(T, i), tb = hget_u(TB, i);
            if (hany(l < x.pas_n && x.P == t)) continue;
            if (x.pas_n >= maxp) {                   // select_random(Passive, [Myself]) + remove
                x.rng = c0 + used;
                const uint32_t k = uniform_n(x, w, x.pas_n) - 1;
                used = (uint32_t)(x.rng - c0);
                PB = hdel(PB, x.pas_n, k);
                x.P = hdel(x.P, x.pas_n, k);
                x.pas_n--;
            }
            pas_insert(x, PB, t, tb);
        }
    }
    x.rng = c0 + used;
}

// ---------------------------------------------------------- the node --
// inputs of a half's node: its descriptor, header words, rows, the first
// inbox record (all lanes of a half load the same addresses, or their own
// element of a row)
struct HIn {
    uint4 D;
    uint32_t r0, r1, w9, A, P, part;
    uint32_t cm, oe;                 // k_relay's connection bits; obase[row + 1] (low word)
    uint32_t SRC, TT;                // lane hl: sender and type word of inbox record hl
    uint32_t EX4;                    // lane hl: exchange id hl & 7 of inbox record hl >> 3
};

// (the descriptor comes from a load issued before the previous node's
// writeback: issued after those stores, its wait drained them -- the memory
// counter is in order -- at every node)
DEV uint4 load_desc(KArgs& a, const uint32_t (&lc)[4], uint32_t i, bool live) {
    return live ? a.desc_lite[lite_at(a, lc, i)] : make_uint4(0, 0, 0, 0);
}
// the node's rows: header words, active and passive rows, partition byte
// (for the next node issued after this one's body, so that they are not
// held in registers across it)
DEV void load_rows(KArgs& a, HIn& in, bool live) {
    const uint32_t l = hl_id();
    const size_t li = live ? in.D.x - a.lo : 0;
    const uint32_t* hrow = reinterpret_cast<const uint32_t*>(a.hdr + li);
    in.r0 = hrow[0]; in.r1 = hrow[1]; in.w9 = hrow[9];
    in.A = l < PSIM_ACTIVE_CAP ? a.act[li * PSIM_ACTIVE_CAP + l] : 0u;
    in.P = a.pas[li * PSIM_PASSIVE_CAP + l];
    in.part = a.part[live ? in.D.x : 0];
    in.cm = a.lite_cm[li];
    in.oe = reinterpret_cast<const uint32_t*>(a.obase + li + 1)[0];   // (totals < 2^32 slots)
}
// the descriptor's inbox heads (issued a node ahead)
DEV HIn load_in(KArgs& a, const uint4& D) {
    const uint32_t l = hl_id();
    HIn in;
    in.D = D;
    in.r0 = in.r1 = in.w9 = in.A = in.P = in.part = in.cm = in.oe = 0;
    // the first 32 records' senders and type words, the first four's
    // exchanges (one load instruction each, issued a node ahead)
    const uint32_t ik = in.D.z & DESC_CNT_MASK;
    const Msg* r = a.rec_in + in.D.y + (l < ik ? l : 0u);      // (the inbox has a spare record)
    const uint2 st = *reinterpret_cast<const uint2*>(&r->src);
    in.SRC = l < ik ? st.x : 0u;
    in.TT = l < ik ? st.y : (uint32_t)PSIM_MSG_PT_BROADCAST;
    in.EX4 = a.rec_in[in.D.y + ((l >> 3) < ik ? (l >> 3) : 0u)].ex[l & 7];
    return in;
}

DEV void begin(Hn& x, const HIn& in) {
    const uint32_t l = hl_id();
    x.me = in.D.x; x.ib = in.D.y;
    x.ik = in.D.z & DESC_CNT_MASK; x.ob = in.D.w;
    x.fl = (in.D.z >> 28) | (in.part << 8) | (in.w9 & 0xFFFF0000u);
    x.rng = ((uint64_t)in.r1 << 32) | in.r0;
    x.act_n = in.w9 & 0xFF; x.pas_n = (in.w9 >> 8) & 0xFF;
    x.A = l < x.act_n ? in.A : 0u;
    x.P = l < x.pas_n ? in.P : 0u;
    x.seq = 0; x.flushed = 0;
    x.dcb = ~0ull;
}

// the HyParView phase of a lite node (psim_consume.hip body_lite)
DEV void body(Hn& x, Hw& w, Hc& c, const HIn& in) {
    KArgs& a = kargs();
    const uint32_t l = hl_id();
    // the inbox in canonical order, 32 records at a time: lane hl holds
    // record c + hl's sender and type word, and the loop visits the
    // HyParView records among them (Plumtree ones are k_ptl's)
    for (uint32_t cb = 0; cb < x.ik; cb += 32) {
      uint32_t SRC = in.SRC, TT = in.TT;
      if (cb) {
          const bool has = cb + l < x.ik;
          const uint2 st = *reinterpret_cast<const uint2*>(&a.rec_in[x.ib + (has ? cb + l : 0u)].src);
          SRC = has ? st.x : 0u;
          TT = has ? st.y : (uint32_t)PSIM_MSG_PT_BROADCAST;
      }
      uint32_t M = hmask((TT & 0xFF) < PSIM_MSG_PT_BROADCAST);
      while (M) {
        const uint32_t j = (uint32_t)__ffs(M) - 1;
        M &= M - 1;
        const uint32_t p = hget(SRC, j), tt = hget(TT, j);
        const uint32_t e4 = hget(in.EX4, (j << 3) | (l & 7));      // (records 0-3: prefetched)
        const uint32_t q = cb + j;
        uint32_t ex = q < 4 ? e4 : a.rec_in[x.ib + q].ex[l & 7];
        const uint32_t nex = (tt >> 16) & 0xFF, ttl = (tt >> 8) & 0xFF;
        const uint32_t type = tt & 0xFF;
        ex = l < nex ? ex : 0u;
        const bool reply = type == PSIM_MSG_SHUFFLE_REPLY;          // hv:1091-1093
        const bool relay = !reply && ttl > 0 && x.act_n > 1;         // hv:1095-1136
        c.dl += reply ? 0x10000u : 1u;
        HSTAMP(w, 6);
        if (relay) {
            const uint32_t r = select_random(x, w, x.A, x.act_n, p, x.me);
            if (r != PSIM_NONE) hv_send(x, w, c, r, PSIM_MSG_SHUFFLE, ttl - 1, ex, nex);
            HSTAMP(w, 1);
        } else {
            if (!reply) {                             // the walk ends here: reply to Sender
                uint32_t RESP = 0;
                const uint32_t nr = sublist<PSIM_PASSIVE_CAP - 2>(x, w, x.P, x.pas_n, nex, RESP, 0);
                HSTAMP(w, 2);
                hv_send(x, w, c, p, PSIM_MSG_SHUFFLE_REPLY, 0, RESP, nr);
                HSTAMP(w, 3);
            }
            merge_exchange(x, w, ex, nex, !reply);
            HSTAMP(w, 4);
        }
      }
    }
    if (x.fl & DESC_SHUFFLE) {                        // hv:572-607
        uint32_t EX = l == 0 ? x.me : 0u;
        uint32_t m = 1;
        m = sublist<PSIM_ACTIVE_CAP>(x, w, x.A, x.act_n, a.k_active, EX, m);
        m = sublist<PSIM_PASSIVE_CAP - 2>(x, w, x.P, x.pas_n, a.k_passive, EX, m);
        const uint32_t nex = husort(w, EX, l < m);
        const uint32_t t = select_random(x, w, x.A, x.act_n, x.me, x.me);
        if (t != PSIM_NONE) hv_send(x, w, c, t, PSIM_MSG_SHUFFLE, a.arwl, EX, nex);
        HSTAMP(w, 5);
    }
}

// a half's counters into the block's stats (once, at the kernel's end: the
// per-node LDS atomics cost a writeback's worth of issue slots)
DEV void count(Hw& w, const Hc& c) {
    if (hl_id() != 0) return;
    unsigned long long* st = w.sst;
    if (c.pb & 0xFFFFu) atomicAdd(&st[ST_PROC], (unsigned long long)(c.pb & 0xFFFFu));
    if (c.pb >> 16) atomicAdd(&st[ST_BOUND], (unsigned long long)(c.pb >> 16));
    if (c.dl & 0xFFFFu) atomicAdd(&st[ST_DELIV + PSIM_MSG_SHUFFLE], (unsigned long long)(c.dl & 0xFFFFu));
    if (c.dl >> 16) atomicAdd(&st[ST_DELIV + PSIM_MSG_SHUFFLE_REPLY], (unsigned long long)(c.dl >> 16));
    if (c.em & 0xFFFFu) atomicAdd(&st[ST_EMIT + PSIM_MSG_SHUFFLE], (unsigned long long)(c.em & 0xFFFFu));
    if (c.em >> 16) atomicAdd(&st[ST_EMIT + PSIM_MSG_SHUFFLE_REPLY], (unsigned long long)(c.em >> 16));
    if (c.fail) atomicAdd(&st[ST_FAIL], (unsigned long long)c.fail);
}

// the draw counter and passive size in the header, the passive row when it
// changed, the outbox count and the records (the flag byte, the active row,
// the id maps and the Plumtree rows are unchanged)
DEV void writeback(Hn& x, Hw& w, Hc& c) {
    KArgs& a = kargs();
    const uint32_t l = hl_id();
    const uint32_t li = local_row(x);
    uint32_t* hrow = reinterpret_cast<uint32_t*>(a.hdr + li);
    const uint32_t w9 = (x.fl & 0xFFFF0000u) | (x.pas_n << 8) | x.act_n;
    if (l < 3) hrow[l == 2 ? 9 : l] = l == 0 ? (uint32_t)x.rng : l == 1 ? (uint32_t)(x.rng >> 32) : w9;
    if (x.fl & HF_PDIRTY) a.pas[(size_t)li * PSIM_PASSIVE_CAP + l] = x.P;
    flush(x, w);
    if (l == 0) a.ocnt[li] = x.seq;
    c.pb += 1u + (x.seq > out_cap(x) ? 0x10000u : 0u);
    if ((c.dl | c.em | c.pb) & 0x80008000u) {        // (a 16-bit half past 2^15: flush early)
        count(w, c);
        c.dl = 0; c.em = 0; c.pb = 0; c.fail = 0;
    }
}


}  // namespace

__global__ void __launch_bounds__(64 * PSIM_HALF_WPB, PSIM_HALF_WAVES) k_lite_half(RoundArgs args) {
    if (*kargs().ctl) return;                         // an aborted batch (run_batch)
    __shared__ unsigned long long sst[NST];
    __shared__ __attribute__((aligned(16))) uint32_t srecs[HWPB][2 * HSTAGE * 16];
    __shared__ uint32_t skeys[HWPB][2 * HSTAGE];
    __shared__ uint32_t scrs[HWPB][64];
#ifdef PSIM_STAMPS
    __shared__ unsigned long long stls[HWPB][32];
    for (int i = threadIdx.x; i < (int)(HWPB * 32); i += blockDim.x) (&stls[0][0])[i] = 0;
#endif
    for (int i = threadIdx.x; i < NST; i += blockDim.x) sst[i] = 0;
    __syncthreads();
    const uint32_t wid = threadIdx.x >> 6, l = hl_id();
    Hw w;
    w.sst = sst; w.srec = srecs[wid]; w.skey = skeys[wid]; w.scr = scrs[wid];
    w.KM = kMagic[l == 0 ? 64 : l];
#ifdef PSIM_STAMPS
    w.stl = stls[wid];
    w.t_last = __builtin_amdgcn_s_memtime();
#endif
    Hc c = {};
    // half h of global wave gw takes list entries 2 gw + h, + 2 nw, ...
    const uint32_t nw = gridDim.x * HWPB;
    const uint32_t first = 2 * (blockIdx.x * HWPB + wid) + (hb_id() >> 5);
    uint32_t lc[4], na;
    lite_counts(kargs(), lc, na);
    if (first < na) {
        Hn x;
        HIn in = load_in(kargs(), load_desc(kargs(), lc, first, true));
        load_rows(kargs(), in, true);
        uint4 Dn = load_desc(kargs(), lc, first + 2 * nw < na ? first + 2 * nw : first, first + 2 * nw < na);
        for (uint32_t i = first; i < na; i += 2 * nw) {
            HSTAMP(w, 8);
            begin(x, in);
            // the connection bits and the outbox bound, loaded with the rows
            x.AF = in.cm | (min(in.oe - x.ob, 0xFFFFFFu) << 8);
            // the next node's inputs, in flight while this one runs
            const uint32_t nx = i + 2 * nw, nnx = i + 4 * nw;
            HIn inn = load_in(kargs(), Dn);
            HSTAMP(w, 0);
            body(x, w, c, in);
            HSTAMP(w, 9);
            Dn = load_desc(kargs(), lc, nnx < na ? nnx : i, nnx < na);
            load_rows(kargs(), inn, nx < na);
            writeback(x, w, c);
            HSTAMP(w, 7);
            in = inn;
        }
        count(w, c);
    }
    // the digest partials of every lane
    {
        uint64_t dg = c.digest;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) dg += __shfl_xor(dg, off);
        if (__lane_id() == 0 && dg) atomicAdd(&sst[ST_DIGEST], (unsigned long long)dg);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < NST; i += blockDim.x)
        kargs().stat_lite[(size_t)blockIdx.x * NST + i] = sst[i];
#ifdef PSIM_STAMPS
    if (threadIdx.x < 32) {
        unsigned long long t = 0;
        for (uint32_t k = 0; k < HWPB; k++) t += stls[k][threadIdx.x];
        if (t) atomicAdd(&g_stamps_half[threadIdx.x], t);
    }
#endif
}

static uint32_t half_resident_grid() {
    int dev = 0, nb = 0;
    hipDeviceProp_t p;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)k_lite_half, 64 * HWPB, 0) != hipSuccess ||
        nb <= 0)
        return 1024;
    return (uint32_t)nb * (uint32_t)p.multiProcessorCount;
}
uint32_t lite_half_grid() { return half_resident_grid(); }
uint32_t lite_half_block() { return 64 * HWPB; }

}  // namespace psim

namespace psim {
#ifdef PSIM_STAMPS
int debug_stamps_half(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps_half), sizeof(unsigned long long) * 32) != hipSuccess) return -1;
    unsigned long long z[32] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps_half), z, sizeof z) != hipSuccess) return -1;
    return 32;
}
#else
int debug_stamps_half(unsigned long long*) { return 0; }
#endif
// this TU's layout (psim_kernels.h layout_sig, checked by psim_create)
uint32_t layout_sig_lite() { return layout_sig(); }

}  // namespace psim
