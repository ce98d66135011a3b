// psim_strategy.hip -- the node-round kernel of a PLUGGABLE handle:
// partisan's pluggable peer-service manager driving one membership strategy
// (round model R0-P).
//
// One 64-lane wave per node with work, as in psim_consume.hip.  A SCAMP
// membership / partial view / in-view lives one id per lane, so the
// strategies' list operations (lists:member, [N | L], sets:add_element,
// sublist(shuffle(L), K)) are ballots, DPP lane shifts and one rank count.
// The full strategy's ORSet is the node's member bitset row, walked 1 KiB
// (64 lanes x 16 B) per step for merge / equal / count / k-th member; a
// gossip carries a snapshot of the row (the Erlang message carries the state
// term of its moment), written once into this round's payload arena and
// read by the receivers next round.
//
// Reference handlers are cited as file:line under /root/reference:
//   full = src/partisan_full_membership_strategy.erl
//   sv1  = src/partisan_scamp_v1_membership_strategy.erl
//   sv2  = src/partisan_scamp_v2_membership_strategy.erl
//   pl   = src/partisan_pluggable_peer_service_manager.erl
#include "psim_device.h"
#include "psim_kernels.h"
#include "psim_wave.h"

namespace psim {

namespace {

constexpr int PL_WAVES = 4;        // waves per block
constexpr uint32_t NONE = PSIM_NONE;
constexpr uint64_t NONE64 = ~0ull;

// A SCAMP list of up to PSIM_SVIEW_CAP = 128 ids in two registers: entry l
// in lane l of `a`, entry 64 + l in lane l of `b` (entries past the count 0)
static_assert(PSIM_SVIEW_CAP == 128, "a SCAMP list is two 64-lane registers");
struct L2 { uint32_t a, b; };
DEV bool has2(const L2& V, uint32_t n, uint32_t e) {
    const uint32_t l = lane_id();
    return (ballot(l < n && V.a == e) | ballot(64 + l < n && V.b == e)) != 0;
}
DEV uint32_t get2(const L2& V, uint32_t i) { return i < 64 ? rl(V.a, (int)i) : rl(V.b, (int)(i - 64)); }
// insert e at position pos (entries from pos move up one)
DEV void ins2(L2& V, uint32_t& n, uint32_t pos, uint32_t e) {
    const uint32_t l = lane_id();
    const uint32_t carry = rl(V.a, 63);
    const uint32_t pa = from_prev(V.a);
    uint32_t pb = from_prev(V.b);
    pb = l == 0 ? carry : pb;
    V.a = l < pos ? V.a : (l == pos ? e : (l <= n ? pa : 0u));
    const uint32_t j = 64 + l;
    V.b = j < pos ? V.b : (j == pos ? e : (j <= n ? pb : 0u));
    n++;
}
// every entry moves to its position: entry l of the list to PA (lane l),
// entry 64 + l to PB, through the wave's 128 scratch words
DEV void permute2(uint32_t* lds, L2& V, uint32_t n, uint32_t PA, uint32_t PB) {
    const uint32_t l = lane_id();
    if (l < n) lds[PA] = V.a;
    if (64 + l < n) lds[PB] = V.b;
    __builtin_amdgcn_wave_barrier();
    V.a = l < n ? lds[l] : 0u;
    V.b = 64 + l < n ? lds[64 + l] : 0u;
    __builtin_amdgcn_wave_barrier();
}

// A SCAMP v1 membership is an OTP sets v1 linear hash table (sets.erl) of
// `ns` active slots; the list holds sets:to_list/1 order: slot 0..ns-1,
// oldest first within a slot (an element is prepended to its bucket, and
// to_list's fold reverses it).  sets:add_element/2: after every entry of a
// slot <= e's; then maybe_expand/2 -- past 5 ns elements slot ns opens and
// the entries of its buddy slot ns - MaxN/2 whose phash(E, MaxN') is ns + 1
// move into it, order kept: to the list's end (MaxN doubles when ns reaches
// it).
DEV void add_set2(uint32_t* lds, L2& V, uint32_t& n, uint32_t e, uint32_t& ns) {
    const uint8_t* bt = kargs().btab;
    const uint32_t l = lane_id(), b = set_slot(bt, e, ns);
    const uint32_t pos = popc(ballot(l < n && set_slot(bt, V.a, ns) <= b)) +
                         popc(ballot(64 + l < n && set_slot(bt, V.b, ns) <= b));
    ins2(V, n, pos, e);
    if (n <= 5 * ns) return;
    ns++;                                       // maybe_expand/2: one slot more
    const bool ma = l < n && set_slot(bt, V.a, ns) == ns - 1;
    const bool mb = 64 + l < n && set_slot(bt, V.b, ns) == ns - 1;
    const uint64_t lt = (1ull << l) - 1;
    const uint64_t bma = ballot(ma), bmb = ballot(mb);
    const uint64_t sa = ballot(l < n && !ma), sb = ballot(64 + l < n && !mb);
    const uint32_t stay = popc(sa) + popc(sb);
    const uint32_t PA = ma ? stay + popc(bma & lt) : popc(sa & lt);
    const uint32_t PB = mb ? stay + popc(bma) + popc(bmb & lt) : popc(sa) + popc(sb & lt);
    permute2(lds, V, n, PA, PB);
}

// sets:del_element/2 of a member at list position i, then maybe_contract/2:
// below 3 ns elements (ns > 16) slot ns - 1 closes and its entries join its
// buddy slot ns - 1 - MaxN/2 as put_bucket_s(Segs0, Slot1, B1 ++ B2) stores
// them (B1 the buddy's bucket, B2 the closing slot's); to_list's reversing
// fold then yields the closing slot's entries first, then the buddy's own
DEV void del_set2(uint32_t* lds, L2& V, uint32_t& n, uint32_t e, uint32_t& ns) {
    const uint8_t* bt = kargs().btab;
    const uint32_t l = lane_id();
    const uint64_t lt = (1ull << l) - 1;
    {
        const bool ka = l < n && V.a != e, kb = 64 + l < n && V.b != e;
        const uint64_t ba = ballot(ka), bb = ballot(kb);
        const uint32_t k = popc(ba) + popc(bb);
        if (k == n) return;                     // not a member: Dc = 0
        permute2(lds, V, n, ka ? popc(ba & lt) : k, kb ? popc(ba) + popc(bb & lt) : k);
        V.a = l < k ? V.a : 0u;                 // (entries past the count are 0)
        V.b = 64 + l < k ? V.b : 0u;
        n = k;
    }
    if (!(n < 3 * ns && ns > 16)) return;
    const uint32_t top = ns - 1, to = top - set_maxn(ns) / 2;
    // the closing slot's entries (at the list's end) go after every entry of
    // a slot < `to`, in front of the buddy slot's own
    const bool ga = l < n && set_slot(bt, V.a, ns) == top, gb = 64 + l < n && set_slot(bt, V.b, ns) == top;
    const bool ea = l < n && !ga && set_slot(bt, V.a, ns) < to, eb = 64 + l < n && !gb && set_slot(bt, V.b, ns) < to;
    const uint64_t bga = ballot(ga), bgb = ballot(gb);
    const uint32_t p = popc(ballot(ea)) + popc(ballot(eb)), g = popc(bga) + popc(bgb);
    const uint64_t na = ballot(l < n && !ga), nb = ballot(64 + l < n && !gb);
    const uint32_t ra = popc(na & lt), rb = popc(na) + popc(nb & lt);
    const uint32_t PA = ga ? p + popc(bga & lt) : ra + (ra >= p ? g : 0u);
    const uint32_t PB = gb ? p + popc(bga) + popc(bgb & lt) : rb + (rb >= p ? g : 0u);
    permute2(lds, V, n, PA, PB);
    ns--;
}

// Hdr fields of a pluggable node (see RoundArgs): join_contact = pending
// contact, aux = round of the last ping, have = hello sent,
// act_n = view length, pas_n = in_view length, pad1[1] = SCAMP v1's set
// slots - 16 (sets v1 linear hashing, add_set2).
struct Pw {
    const RoundArgs* a;
    uint32_t* lds;                 // 128 words of per-wave scratch
    uint32_t me, li, mypart, round;
    Hdr h;
    L2 V, I;                       // scamp: view / in_view, entries l and 64 + l in lane l
    uint32_t vn, in_n;
    uint32_t vs;                   // scamp v1: the membership set's active slots (sets v1, 16..)
    L2 CV, CF;                     // connection cache: view ids at node start and
                                   // flags | part << 8 of each
    uint32_t seq;
    uint64_t obase;
    uint64_t digest;               // lane j sums the hashes of record word j
    uint32_t SC;                   // lane k counts stats slot k
    uint32_t DCL, DCH;             // draw cache: counters dc_base + lane
    uint64_t dc_base;
    uint32_t* row;                 // full: the node's member bitset
    uint32_t snap;                 // full: payload slot of the current state
    bool dirty, gossip_due;
    bool stop;                     // the manager stopped this round (leave, App. A Q12)
    uint32_t nfail;                // this node's failed sends this round (uniform)
    uint32_t nomit;                // ... and its sends an omission fault dropped
};

DEV void st_add(Pw& w, int k, uint32_t v) { w.SC += lane_id() == (uint32_t)k ? v : 0u; }
DEV void ovf(Pw& w, int kind) {                       // a fixed-table overflow of kind PSIM_OVF_*
    const uint32_t l = lane_id();
    w.SC += (l == (uint32_t)ST_OVF || l == (uint32_t)(ST_OVF_BY + kind)) ? 1u : 0u;
}

DEV uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off);
    return v;
}

// ----------------------------------------------------------------- RNG --
DEV void dc_fill(Pw& w, uint64_t base) {
    uint64_t v = draw58_at(base + lane_id(), w.me, kargs().seed);
    w.DCL = (uint32_t)v; w.DCH = (uint32_t)(v >> 32);
    w.dc_base = base;
}
DEV uint64_t draw(Pw& w) {
    uint64_t c = w.h.rng++;
    if (c < w.dc_base || c - w.dc_base >= 64) dc_fill(w, c);
    uint32_t i = (uint32_t)(c - w.dc_base);
    return ((uint64_t)rl(w.DCH, i) << 32) | rl(w.DCL, i);
}
// rand:uniform/1 with a 58-bit generator (OTP rand.erl ?uniform_range)
DEV uint32_t uniform_n(Pw& w, uint32_t n) {
    const uint64_t two58 = 1ull << 58;
    for (;;) {
        uint64_t v = draw(w);
        if (v < n) return (uint32_t)v + 1;
        uint64_t i = n <= 64 ? mod_small(v, n) : mod58(v, n);
        if (v - i <= two58 - n) return (uint32_t)i + 1;
    }
}

// lists:sublist(shuffle(L), K) (sv1:263-269, sv2:345-350) over a list of up
// to 128 ids: element j keys on counter rng + j (two draw-cache fills past 64
// entries); its rank among the (key, id) pairs is its position after
// lists:sort; the first K (<= 64) land in OUT lanes 0..
DEV uint32_t sublist(Pw& w, const L2& V, uint32_t n, uint32_t k, uint32_t& OUT) {
    const uint32_t l = lane_id();
    const uint64_t base = w.h.rng;
    dc_fill(w, base);
    const uint64_t ka = l < n ? ((((uint64_t)w.DCH) << 32) | w.DCL) >> 5 : ~0ull;
    uint64_t kb = ~0ull;
    if (n > 64) {
        dc_fill(w, base + 64);
        kb = 64 + l < n ? ((((uint64_t)w.DCH) << 32) | w.DCL) >> 5 : ~0ull;
    }
    const uint32_t m = n < k ? n : k;
    uint32_t ra = 0, rb = 0;
    for (uint32_t j = 0; j < n; j++) {
        const uint64_t kj = j < 64 ? rl64(ka, (int)j) : rl64(kb, (int)(j - 64));
        const uint32_t ej = get2(V, j);
        ra += (kj < ka || (kj == ka && ej < V.a)) ? 1u : 0u;
        rb += (kj < kb || (kj == kb && ej < V.b)) ? 1u : 0u;
    }
    if (l < n && ra < m) w.lds[ra] = V.a;
    if (64 + l < n && rb < m) w.lds[rb] = V.b;
    __builtin_amdgcn_wave_barrier();
    uint32_t got = l < m ? w.lds[l] : 0u;
    __builtin_amdgcn_wave_barrier();
    OUT = got;
    w.h.rng = base + n;
    return m;
}

// ------------------------------------------------------------ emission --
// record {dst, src, type, seq, a0, 0, 0, payload slot, 0 x 8}; the slot is
// an arena index, not part of the message, so it is hashed as 0
DEV void emit(Pw& w, uint32_t dst, uint32_t type, uint32_t a0, uint32_t slot) {
    uint32_t l = lane_id();
    uint32_t s = w.seq++;
    uint64_t at = w.obase + s;
    uint32_t word = l == 0 ? dst : l == 1 ? w.me : l == 2 ? type : l == 3 ? s : l == 4 ? a0
                  : l == 7 ? slot : 0u;
    if (l < 16) {
        reinterpret_cast<uint32_t*>(kargs().rec_out + at)[l] = word;
        uint32_t hw = l == 7 ? 0u : word;
        w.digest += (uint64_t)hw * digest_mul(l);
    }
    if (l == 0) kargs().okey[at] = dst;     // pluggable bounds come from k_node_prep
    st_add(w, ST_EMIT + type, 1);
}

// maybe_connect + find (partisan_util.erl:75-134): the peer runs and no
// partition separates the two; view members answer from the cache
DEV bool connect_ok(const Pw& w, uint32_t dst) {
    if (dst >= kargs().n_nodes || dst == w.me) return false;
    const uint64_t ma = ballot(w.CV.a == dst), mb = ballot(w.CV.b == dst);
    uint32_t v = ma ? rl(w.CF.a, ffs64(ma)) : mb ? rl(w.CF.b, ffs64(mb))
               : ((uint32_t)kargs().flags[dst] | ((uint32_t)kargs().part[dst] << 8));
    return (v & F_UP) && (v >> 8) == w.mypart;
}

// establish_connections/3 (pl:1096-1108) connects to members and the pending
// contact only.  The full strategy sends to members only (every target is
// read from its own member row), so only SCAMP needs the check.
DEV bool connected(const Pw& w, uint32_t p) {
    if (kargs().strategy == PSIM_STRATEGY_FULL) return true;
    return has2(w.V, w.vn, p) || p == w.h.join_contact;
}

// ---------------------------------------------------- omission faults --
// the installed interposition funs (pl:297-326) as sorted pair keys
// src << 32 | dst: a wave-uniform binary search
DEV bool pair_in(const uint64_t* l, uint32_t n, uint64_t k) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (l[m] < k) lo = m + 1;
        else hi = m;
    }
    return lo < n && l[lo] == k;
}
// the fold of handle_cast({forward_message, ..}) (pl:669-684) turns the
// message into `undefined`: {send_omission, Dst} at the sender
// (prop_partisan_crash_fault_model:166-177), the `faulted` reader
// (partisan_trace_orchestrator:623-637)
DEV bool omit_send(const Pw& w, uint32_t dst) {
    return kargs().faulted[w.me] || pair_in(kargs().omit, kargs().n_omit_s, (uint64_t)w.me << 32 | dst);
}
// ... and that of handle_cast({receive_message, ..}) (pl:634-667):
// {receive_omission, Src} at the receiver (crash_fault_model:125-135)
DEV bool omit_recv(const Pw& w, uint32_t src) {
    return kargs().faulted[w.me] ||
           pair_in(kargs().omit + kargs().n_omit_s, kargs().n_omit_r, (uint64_t)src << 32 | w.me);
}

// do_send_message/7 (pl:1309-1363); success draws rand:uniform(1) in
// partisan_util:dispatch_pid/3 (util:190-195).  The interposition fold runs
// first: an omitted message meets no connection lookup and no draw (pl:727-760)
DEV void pl_send(Pw& w, uint32_t dst, uint32_t type, uint32_t a0, uint32_t slot) {
    if (kargs().faults && omit_send(w, dst)) { st_add(w, ST_OMIT, 1); w.nomit++; return; }
    if (!connect_ok(w, dst) || !connected(w, dst)) { st_add(w, ST_FAIL, 1); w.nfail++; return; }
    w.h.rng++;
    emit(w, dst, type, a0, slot);
}

// ---------------------------------------------------------------- full --
// ?SET:merge/2 into the row (full:49-55, :99-116); returns ?SET:equal/2 of
// the two states before it
DEV bool full_merge(Pw& w, const uint32_t* p) {
    const uint32_t fw = kargs().tomb ? 2 * kargs().fw : kargs().fw;   // adds (+ removes)
    bool neq = false, chg = false;
    for (uint32_t base = 0; base < fw; base += 256) {
        uint32_t i = base + 4 * lane_id();
        if (i < fw) {
            uint4 o = *reinterpret_cast<const uint4*>(w.row + i);
            uint4 q = *reinterpret_cast<const uint4*>(p + i);
            neq |= (o.x != q.x) | (o.y != q.y) | (o.z != q.z) | (o.w != q.w);
            uint4 m = make_uint4(o.x | q.x, o.y | q.y, o.z | q.z, o.w | q.w);
            if (m.x != o.x || m.y != o.y || m.z != o.z || m.w != o.w) {
                *reinterpret_cast<uint4*>(w.row + i) = m;
                chg = true;
            }
        }
    }
    if (ballot(chg)) w.dirty = true;
    st_add(w, ST_BYTES, 8 * fw);
    return ballot(neq) == 0;
}

// four member words (add & ~remove) of the node's row at word i
DEV uint4 mem4(const Pw& w, uint32_t i) {
    uint4 o = *reinterpret_cast<const uint4*>(w.row + i);
    if (kargs().tomb) {
        const uint4 t = *reinterpret_cast<const uint4*>(w.row + kargs().fw + i);
        o = make_uint4(o.x & ~t.x, o.y & ~t.y, o.z & ~t.z, o.w & ~t.w);
    }
    return o;
}

DEV uint32_t full_count(const Pw& w) {
    const uint32_t fw = kargs().fw;
    uint32_t c = 0;
    for (uint32_t base = 0; base < fw; base += 256) {
        uint32_t i = base + 4 * lane_id();
        if (i < fw) {
            uint4 o = mem4(w, i);
            c += __popc(o.x) + __popc(o.y) + __popc(o.z) + __popc(o.w);
        }
    }
    st_add(const_cast<Pw&>(w), ST_BYTES, 4 * fw);
    return uni(wave_sum(c));
}

// the k-th (0-based) member in id order
DEV uint32_t full_nth(const Pw& w, uint32_t k) {
    const uint32_t fw = kargs().fw;
    const uint32_t l = lane_id();
    for (uint32_t base = 0; base < fw; base += 256) {
        uint32_t i = base + 4 * l;
        uint4 o = i < fw ? mem4(w, i) : make_uint4(0, 0, 0, 0);
        uint32_t inc = __popc(o.x) + __popc(o.y) + __popc(o.z) + __popc(o.w);
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            uint32_t t = (uint32_t)__shfl_up((int)inc, off);
            if (l >= (uint32_t)off) inc += t;
        }
        uint32_t tot = rl(inc, 63);
        st_add(const_cast<Pw&>(w), ST_BYTES, 1024);
        if (k < tot) {
            int L = ffs64(ballot(inc > k));
            uint32_t kk = k - (L ? rl(inc, L - 1) : 0u);
            uint32_t ws[4] = {rl(o.x, L), rl(o.y, L), rl(o.z, L), rl(o.w, L)};
            for (int j = 0; j < 4; j++) {
                uint32_t pc = __popc(ws[j]);
                if (kk < pc) {
                    uint32_t x = ws[j];
                    for (; kk; kk--) x &= x - 1;
                    return (base + 4 * (uint32_t)L + (uint32_t)j) * 32 + (uint32_t)(__ffs(x) - 1);
                }
                kk -= pc;
            }
        }
        k -= tot;
    }
    return NONE;
}

// a snapshot of the state for the messages of one gossip: one arena slot per
// distinct state the node sends this round
DEV uint32_t full_snapshot(Pw& w) {
    if (w.snap != NONE && !w.dirty) return w.snap;
    uint32_t s = 0;
    if (lane_id() == 0) s = atomicAdd(kargs().pay_top, 1u);
    s = rl(s, 0);
    if (s >= kargs().pay_cap) { ovf(w, PSIM_OVF_STRATEGY); s = kargs().pay_cap - 1; }
    const uint32_t fw = kargs().tomb ? 2 * kargs().fw : kargs().fw;   // adds (+ removes)
    uint32_t* dst = kargs().pay_out + (size_t)s * 2 * kargs().fw;
    for (uint32_t base = 0; base < fw; base += 256) {
        uint32_t i = base + 4 * lane_id();
        if (i < fw) *reinterpret_cast<uint4*>(dst + i) = *reinterpret_cast<const uint4*>(w.row + i);
    }
    w.snap = s;
    w.dirty = false;
    st_add(w, ST_BYTES, 8 * fw);
    return s;
}

// gossip_messages/1 (full:127-144) to every member (fanout 0), or to
// `fanout` members each drawn as rand:uniform(length(Members)) -- config B's
// extension, coalesced to one gossip per round.  The
// whole list is built before the manager sends any of it.
DEV void full_gossip(Pw& w, uint32_t extra = NONE) {
    uint32_t slot = full_snapshot(w), cnt = full_count(w);
    const uint32_t fw = kargs().fw;
    if (kargs().fanout == 0) {
        for (uint32_t base = 0; base < fw; base += 256) {
            uint32_t i = base + 4 * lane_id();
            uint4 o = i < fw ? mem4(w, i) : make_uint4(0, 0, 0, 0);
            if (extra != NONE && i == ((extra >> 5) & ~3u)) {    // an old member (leave/1)
                const uint32_t b = 1u << (extra & 31u), q = (extra >> 5) & 3u;
                o.x |= q == 0 ? b : 0u; o.y |= q == 1 ? b : 0u;
                o.z |= q == 2 ? b : 0u; o.w |= q == 3 ? b : 0u;
            }
            for (uint64_t nz = ballot((o.x | o.y | o.z | o.w) != 0); nz; nz &= nz - 1) {
                int L = ffs64(nz);
                uint32_t ws[4] = {rl(o.x, L), rl(o.y, L), rl(o.z, L), rl(o.w, L)};
                for (int j = 0; j < 4; j++)
                    for (uint32_t x = ws[j]; x; x &= x - 1)
                        pl_send(w, (base + 4 * (uint32_t)L + (uint32_t)j) * 32 + (uint32_t)(__ffs(x) - 1),
                                PSIM_PL_GOSSIP, cnt, slot);
            }
        }
        return;
    }
    uint32_t TG = 0;
    for (uint32_t i = 0; i < kargs().fanout; i++) {
        uint32_t t = full_nth(w, uniform_n(w, cnt) - 1);
        TG = lane_id() == i ? t : TG;
    }
    for (uint32_t i = 0; i < kargs().fanout; i++) pl_send(w, rl(TG, i), PSIM_PL_GOSSIP, cnt, slot);
}

// --------------------------------------------------------------- scamp --
// sets:add_element/2 (v1, sets:to_list order) or [E | L] (v2) into a fixed table
DEV void scamp_add(Pw& w, L2& L, uint32_t& n, uint32_t e, bool as_set) {
    if (as_set && has2(L, n, e)) return;
    if (n >= PSIM_SVIEW_CAP) { ovf(w, PSIM_OVF_STRATEGY); return; }
    if (as_set) add_set2(w.lds, L, n, e, w.vs);
    else ins2(L, n, 0, e);
}

// Strategy:join/3 at the joiner (sv1:52-99, sv2:64-113)
DEV void scamp_join(Pw& w, uint32_t contact) {
    const bool v1 = kargs().strategy == PSIM_STRATEGY_SCAMP_V1;
    const L2 M0 = w.V;
    const uint32_t n0 = w.vn;
    scamp_add(w, w.V, w.vn, contact, v1);
    uint32_t SEL = 0;
    uint32_t ns = sublist(w, M0, n0, v1 ? kargs().scamp_c : kargs().scamp_c - 1, SEL);
    pl_send(w, contact, PSIM_PL_FWD_SUB, w.me, NONE);
    for (uint32_t i = 0; i < n0; i++)            // v1: sets:fold/3 = reverse of to_list
        pl_send(w, get2(M0, v1 ? n0 - 1 - i : i), PSIM_PL_FWD_SUB, contact, NONE);
    for (uint32_t i = 0; i < ns; i++) pl_send(w, rl(SEL, i), PSIM_PL_FWD_SUB, contact, NONE);
}

// periodic/1 (sv1:125-174, sv2:130-178); "isolated" = a ping was received
// and not this round (App. A Q12: 100000 us against 1-s rounds)
DEV void scamp_periodic(Pw& w) {
    const L2 M = w.V;
    const uint32_t n = w.vn;
    const bool isolated = w.h.aux != NONE && w.round > w.h.aux;
    if (isolated) {
        uint32_t SEL = 0;
        if (sublist(w, M, n, 1, SEL)) pl_send(w, rl(SEL, 0), PSIM_PL_FWD_SUB, w.me, NONE);
    }
    for (uint32_t i = 0; i < n; i++) pl_send(w, get2(M, i), PSIM_PL_PING, w.me, NONE);
}

// handle_message(.., {forward_subscription, Node}) (sv1:212-252, sv2:284-327)
DEV void scamp_fwd(Pw& w, uint32_t node) {
    const bool v1 = kargs().strategy == PSIM_STRATEGY_SCAMP_V1;
    const uint32_t rnd = uniform_n(w, 10) >= 5 ? 1u : 0u;    // random_0_or_1/0 sv1:272-279
    if (rnd == 0 && !has2(w.V, w.vn, node)) {
        scamp_add(w, w.V, w.vn, node, v1);
        if (!v1) pl_send(w, node, PSIM_PL_KEEP_SUB, w.me, NONE);
        return;
    }
    uint32_t SEL = 0;
    if (sublist(w, w.V, w.vn, 1, SEL)) pl_send(w, rl(SEL, 0), PSIM_PL_FWD_SUB, node, NONE);
}

// leave/1 at the actor, Node = t (pl:502-515 -> internal_leave/2 :1390-1420):
// v1 leave/2 (sv1:102-122) deletes t and sends {remove_subscription, t} to
// the old membership; v2 leave/2 (sv2:116-127) sends
// {bootstrap_remove_subscription, t} to the partial view, state unchanged
DEV void scamp_leave(Pw& w, uint32_t t) {
    const bool v1 = kargs().strategy == PSIM_STRATEGY_SCAMP_V1;
    const L2 M0 = w.V;
    const uint32_t n0 = w.vn;
    // the connections to the old members stay open (closed only on 'EXIT',
    // pl:971-984): the sends are judged on the old view
    for (uint32_t i = 0; i < n0; i++)
        pl_send(w, get2(M0, i), v1 ? PSIM_PL_REMOVE_SUB : PSIM_PL_BOOT_REMOVE, t, NONE);
    if (v1) del_set2(w.lds, w.V, w.vn, t, w.vs);    // sets:del_element/2 (sv1:111)
}

// leave/1 of the full strategy at the actor (full:58-89): the target's add is
// tombstoned if it is a member, then the new state goes to every member of
// the OLD list (the target included); fanout > 0: the round's coalesced gossip
DEV void full_leave(Pw& w, uint32_t t) {
    const uint32_t wi = t >> 5, bit = 1u << (t & 31u);
    const bool was = (w.row[wi] & ~w.row[kargs().fw + wi] & bit) != 0;   // (tomb is on)
    __builtin_amdgcn_wave_barrier();
    if (was) {
        if (lane_id() == 0) w.row[kargs().fw + wi] |= bit;
        __builtin_amdgcn_wave_barrier();
        w.dirty = true;
    }
    if (kargs().fanout) { w.gossip_due = true; return; }
    full_gossip(w, was ? t : NONE);
}

// -------------------------------------------------------------- driver --
DEV void pl_handle(Pw& w, uint32_t type, uint32_t src, uint32_t a0, uint32_t slot) {
    const bool full = kargs().strategy == PSIM_STRATEGY_FULL;
    switch (type) {
    case PSIM_PL_HELLO:            // server: {state, Tag, get_local_state()} server:125-148
        if (!connect_ok(w, src)) { st_add(w, ST_FAIL, 1); w.nfail++; break; }
        if (full) {
            uint32_t cnt = full_count(w);
            emit(w, src, PSIM_PL_STATE, cnt, full_snapshot(w));
        } else {
            emit(w, src, PSIM_PL_STATE, 0, NONE);
        }
        break;
    case PSIM_PL_STATE:            // handle_info({connected, ..}) pl:986-1044
        if (w.h.join_contact != src) break;
        w.h.join_contact = NONE;
        if (full) {                // join/3 full:49-55
            full_merge(w, kargs().pay_in + (size_t)slot * 2 * kargs().fw);
            if (kargs().fanout) w.gossip_due = true;
            else full_gossip(w);
        } else {
            scamp_join(w, src);
        }
        break;
    case PSIM_PL_GOSSIP:           // handle_message/2 full:99-116
        if (!full) break;
        if (!full_merge(w, kargs().pay_in + (size_t)slot * 2 * kargs().fw)) {
            // a merged removal of ourselves: the manager stops (pl:1182-1188)
            // before the gossip it cast goes out
            if (kargs().tomb && ((w.row[kargs().fw + (w.me >> 5)] >> (w.me & 31u)) & 1u)) { w.stop = true; break; }
            if (kargs().fanout) w.gossip_due = true;
            else full_gossip(w);
        }
        break;
    case PSIM_PL_FWD_SUB:
        if (!full) scamp_fwd(w, a0);
        break;
    case PSIM_PL_PING:             // sv1:177-188, sv2:181-191
        if (!full) w.h.aux = w.round;
        break;
    case PSIM_PL_KEEP_SUB:         // sv2:328-338: InView = [Node | InView0]
        if (kargs().strategy == PSIM_STRATEGY_SCAMP_V2) scamp_add(w, w.I, w.in_n, a0, false);
        break;
    case PSIM_PL_REMOVE_SUB:       // sv1:190-211: a member Node hits the swapped
                                   // sets:del_element/2 arguments (App. A Q12): crash
        if (kargs().strategy == PSIM_STRATEGY_SCAMP_V1 && has2(w.V, w.vn, a0)) w.stop = true;
        break;
    case PSIM_PL_BOOT_REMOVE:      // sv2:192-238: Node itself stops before its casts
                                   // go out (lists:nth(0, ..), or the self-less reset, pl:1182-1188)
        if (kargs().strategy == PSIM_STRATEGY_SCAMP_V2 && a0 == w.me) w.stop = true;
        break;
    default:
        break;
    }
}

DEV uint32_t load_chunk(KArgs& a, uint32_t ib, uint32_t ik, uint32_t c) {
    uint32_t l = lane_id();
    return (c + (l >> 4) < ik) ? reinterpret_cast<const uint32_t*>(a.rec_in + ib + c + (l >> 4))[l & 15]
                               : 0u;
}

DEV void process_pl(Pw& w, uint32_t n, uint32_t ib, uint32_t ik, uint32_t ob) {
    KArgs& a = kargs();
    const uint32_t l = lane_id();
    const uint32_t li = n - a.lo;
    const uint32_t r = a.round;
    {
        uint32_t H = l < 16 ? reinterpret_cast<const uint32_t*>(a.hdr + li)[l] : 0u;
        uint32_t* hw = reinterpret_cast<uint32_t*>(&w.h);
#pragma unroll
        for (int k = 0; k < 16; k++) hw[k] = rl(H, k);
    }
    w.me = n; w.li = li;
    w.mypart = a.part[n];
    if (w.h.start_round == r && ik) { st_add(w, ST_DROPPED, ik); ik = 0; }
    const bool hello = w.h.join_contact != NONE && !w.h.have;
    const bool periodic = a.periodic > 0 && r > w.h.start_round && ((r - w.h.start_round) % a.periodic) == 0;
    const uint32_t leave = w.h.pad1[0];
    if (!(ik || hello || periodic || leave)) return;
    st_add(w, ST_PROC, 1);
    const bool full = a.strategy == PSIM_STRATEGY_FULL;
    w.vn = w.h.act_n; w.in_n = w.h.pas_n;
    w.vs = 16 + w.h.pad1[1];
    const uint32_t* vrow = a.sview + (size_t)li * PSIM_SVIEW_CAP;
    const uint32_t* irow = a.sinv + (size_t)li * PSIM_SVIEW_CAP;
    w.V.a = full ? 0u : vrow[l];
    w.V.b = full || w.vn <= 64 ? 0u : vrow[64 + l];
    const bool v2 = a.strategy == PSIM_STRATEGY_SCAMP_V2;
    w.I.a = v2 ? irow[l] : 0u;
    w.I.b = v2 && w.in_n > 64 ? irow[64 + l] : 0u;
    const L2 V0 = w.V, I0 = w.I;
    w.CV.a = l < w.vn ? w.V.a : NONE;
    w.CV.b = 64 + l < w.vn ? w.V.b : NONE;
    w.CF.a = w.CV.a < a.n_nodes ? ((uint32_t)a.flags[w.CV.a] | ((uint32_t)a.part[w.CV.a] << 8)) : 0u;
    w.CF.b = w.CV.b < a.n_nodes ? ((uint32_t)a.flags[w.CV.b] | ((uint32_t)a.part[w.CV.b] << 8)) : 0u;
    w.row = full ? a.fbits + (size_t)li * 2 * a.fw : nullptr;
    w.seq = 0; w.obase = ob;
    w.snap = NONE; w.dirty = false; w.gossip_due = false;
    w.dc_base = NONE64;
    w.stop = false;
    // a manager that stops this round sends nothing: its sends are casts to
    // itself (schedule_self_message_delivery/6 pl:1585-1609)
    w.nfail = 0; w.nomit = 0;

    if (leave) {                   // leave/1 (pl:502-515, :1390-1420)
        w.h.pad1[0] = 0;
        if (full) full_leave(w, leave - 1);
        else scamp_leave(w, leave - 1);
    }

    if (hello) {                   // internal_join/3 -> connect + hello (pl:1423-1458)
        if (connect_ok(w, w.h.join_contact)) {
            emit(w, w.h.join_contact, PSIM_PL_HELLO, 0, NONE);
            w.h.have = 1;
        } else {
            st_add(w, ST_FAIL, 1); w.nfail++;
        }
    }
    for (uint32_t c = 0; c < ik; c += 4) {
        uint32_t R4 = load_chunk(a, ib, ik, c);
        uint32_t cm = ik - c < 4 ? ik - c : 4;
        for (uint32_t q = 0; q < cm; q++) {
            uint32_t b = q * 16;
            uint32_t type = rl(R4, b + 2) & 0xFF;
            // strategy messages pass the receive interposition (hello /
            // state are the client and server processes')
            if (kargs().faults && type >= PSIM_PL_GOSSIP && omit_recv(w, rl(R4, b + 1))) {
                st_add(w, ST_OMIT, 1);
                continue;
            }
            st_add(w, ST_DELIV + type, 1);
            pl_handle(w, type, rl(R4, b + 1), rl(R4, b + 4), rl(R4, b + 7));
            if (w.stop) { st_add(w, ST_DROPPED, ik - (c + q) - 1); break; }
        }
        if (w.stop) break;
    }
    if (w.stop) {                  // down from the next round, as a crash
        // this node's sends and failures undone: the records it wrote are
        // read back (no per-node snapshot of the counters held in registers)
        const uint32_t l2 = lane_id();
        for (uint32_t k = 0; k < w.seq; k++) {
            const uint32_t word = l2 < 16 ? reinterpret_cast<const uint32_t*>(a.rec_out + w.obase + k)[l2] : 0u;
            w.digest -= (uint64_t)(l2 == 7 ? 0u : word) * digest_mul(l2);
            st_add(w, ST_EMIT + rl(word, 2), (uint32_t)-1);
        }
        st_add(w, ST_FAIL, (uint32_t)-w.nfail);
        st_add(w, ST_OMIT, (uint32_t)-w.nomit);   // (casts to itself that never ran)
        st_add(w, ST_STOP, 1);
        if (l2 == 0) a.stop_ids[atomicAdd(a.n_stop, 1u)] = n;
        w.seq = 0;
    }
    if (periodic && !w.stop) {                // handle_info(periodic) pl:881-903
        if (full) w.gossip_due = true;
        else scamp_periodic(w);
    }
    if (w.gossip_due && !w.stop) full_gossip(w);

    // ---- write back
    w.h.act_n = (uint8_t)w.vn; w.h.pas_n = (uint8_t)w.in_n;
    w.h.pad1[1] = w.vs - 16;
    if (!full && ballot(w.V.a != V0.a)) a.sview[(size_t)li * PSIM_SVIEW_CAP + l] = w.V.a;
    if (!full && ballot(w.V.b != V0.b)) a.sview[(size_t)li * PSIM_SVIEW_CAP + 64 + l] = w.V.b;
    if (v2 && ballot(w.I.a != I0.a)) a.sinv[(size_t)li * PSIM_SVIEW_CAP + l] = w.I.a;
    if (v2 && ballot(w.I.b != I0.b)) a.sinv[(size_t)li * PSIM_SVIEW_CAP + 64 + l] = w.I.b;
    {
        const uint32_t* hw = reinterpret_cast<const uint32_t*>(&w.h);
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < 16; k++) v = l == (uint32_t)k ? hw[k] : v;
        if (l < 16) reinterpret_cast<uint32_t*>(a.hdr + li)[l] = v;
    }
    if (l == 0) a.ocnt[li] = w.seq;
}

}  // namespace

__global__ void __launch_bounds__(256) k_consume_pl(RoundArgs args) {
    if (*kargs().ctl) return;                         // an aborted batch (run_batch)
    __shared__ uint64_t sst[NST];
    __shared__ uint32_t scratch[PL_WAVES][128];
    for (int i = threadIdx.x; i < NST; i += blockDim.x) sst[i] = 0;
    if (threadIdx.x == 0) atomicMin(&kargs().ktime[0], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    __syncthreads();
    const uint32_t wid = threadIdx.x >> 6;
    const uint32_t gw = uni(blockIdx.x * PL_WAVES + wid);
    const uint32_t nw = gridDim.x * PL_WAVES;
    Pw w;
    w.a = &args;
    w.lds = scratch[wid];
    w.round = kargs().round;
    w.SC = 0;
    w.digest = 0;
    const uint32_t na = *kargs().n_alist;
    for (uint32_t k = gw; k < na; k += nw) {
        const uint4 d = kargs().desc[k];
        process_pl(w, uni(d.x), uni(d.y), uni(d.z) & DESC_CNT_MASK, uni(d.w));
    }
    {
        uint32_t l = lane_id();
        if (l < NST && w.SC) atomicAdd((unsigned long long*)&sst[l], (unsigned long long)w.SC);
        uint64_t d = w.digest;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) d += shfl64(d, (int)((l + off) & 63));
        if (l == 0 && d) atomicAdd((unsigned long long*)&sst[ST_DIGEST], (unsigned long long)d);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < NST; i += blockDim.x)
        kargs().stat_part[(size_t)blockIdx.x * NST + i] = sst[i];
    if (threadIdx.x == 0) atomicMax(&kargs().ktime[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

// this TU's layout (psim_kernels.h layout_sig, checked by psim_create)
uint32_t layout_sig_strategy() { return layout_sig(); }

}  // namespace psim
