// psim_ptq.hip -- k_ptq: the Plumtree phase of k_relay's Plumtree list
// (nodes without an origin) with FOUR nodes per wave, one per 16-lane DPP
// row.
//
// k_ptl (psim_consume.hip) runs one node per lane: a lane's eager / lazy sets
// and outstanding table live in 256 B of LDS columns, so a CU holds ~9 of its
// waves (2.0 waves/SIMD at 2^26, profiles/r04/e26a), and every ordsets
// insert, delete and send is a per-lane loop whose trip counts differ across
// the 64 lanes -- 1.6 M SALU instructions per wave of exec-mask bookkeeping,
// 53 % of the cycles waiting on memory.  The lists of a node that k_ptl takes
// hold at most 16 entries (its preconditions), so here a node owns a row of
// 16 lanes and entry i of each list lives in lane i of that row, in VGPRs:
//   membership / rank        the row's 16 ballot bits (qmask) and v_bcnt
//   ordsets insert / delete   a rank, then one DPP row_shr:1 / row_shl:1
//   entry j, j constant       DPP row_newbcast:j (a VALU operand, no LDS)
//   entry j, j a loop index   ds_bpermute within the row (qget)
//   eager push, lazy tick    every lane sends its own entry's record at
//                             seq + (its rank among the sending lanes)
// No LDS tables: the waves' occupancy is set by VGPRs alone.  Control flow
// diverges only between rows (exec-masked), never inside one; every
// cross-lane read runs with its whole row active (a source lane outside the
// exec mask reads 0), so none sits on the right of a per-lane && or ?:.
// Same preconditions, handlers, records, sequence numbers, digest, stats and
// rows as k_ptl: pt_handle / pt_push / the lazy tick, pt:288-313, :341-345,
// :368-453, :562-631.  An A/B alternative (PSIM_PTL_QUARTER=1), not the
// default: parity-exact, but slower -- 0.602 against k_ptl's 0.584 ms a phase
// on the survey line and 79.3 against 68.1 ms at 2^26 (profiles/r04/pq2):
// a row runs each handler for 4 nodes where k_ptl's lanes run it for 64, and
// 5 waves/SIMD (96 VGPRs) do not make up for that.
//
// Reference: pt = src/partisan_plumtree_broadcast.erl
#include <utility>

#include "psim_device.h"
#include "psim_kernels.h"
#include "psim_wave.h"

namespace psim {

namespace {

#ifndef PSIM_PTQ_WPB
#define PSIM_PTQ_WPB 4
#endif
#ifndef PSIM_PTQ_WAVES
#define PSIM_PTQ_WAVES 5
#endif
constexpr uint32_t QWPB = PSIM_PTQ_WPB;          // waves per block
constexpr uint32_t QNODES = 4 * QWPB;            // nodes per block step
constexpr uint32_t QCAP = 16;                    // entries a row holds per list: one per lane
constexpr uint32_t NONE = PSIM_NONE;

DEV uint32_t ql() { return __lane_id() & 15u; }  // lane in the row
DEV uint32_t qb() { return __lane_id() & 48u; }  // the row's lane 0
// the 16 ballot bits of this lane's row
DEV uint32_t qmask(bool p) { return (uint32_t)(__ballot(p) >> qb()) & 0xFFFFu; }
DEV bool qany(bool p) { return qmask(p) != 0u; }
DEV uint32_t qcount(bool p) { return (uint32_t)__popc(qmask(p)); }
// lane j (per lane, < 16) of this lane's row
DEV uint32_t qget(uint32_t v, uint32_t j) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((qb() + (j & 15u)) << 2), (int)v);
}
// lane J (a constant) of this lane's row: DPP row_newbcast:J
template <int J>
DEV uint32_t qbc(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x150 + J, 0xF, 0xF, false);
}
// lane l - 1 / l + 1 of the row (0 past the row's ends): DPP row_shr:1 / row_shl:1
DEV uint32_t qprev(uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true); }
DEV uint32_t qnext(uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x101, 0xF, 0xF, true); }
// OR over the row, in every lane (row_shr 1, 2, 4, 8 leave the row's OR in
// lane 15; lanes without a source keep their own value)
DEV uint32_t qor(uint32_t v) {
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);
    return qbc<15>(v);
}
template <class F, int... J>
DEV void qunroll_seq(F&& f, std::integer_sequence<int, J...>) {
    (f(std::integral_constant<int, J>{}), ...);
}
template <int N, class F>
DEV void qunroll(F&& f) {
    qunroll_seq(f, std::make_integer_sequence<int, N>{});
}

// k_ptl's stats slots; a row counts slot k in its lane k (one register)
enum { T_FIRST, T_FAIL, T_OVF, T_BOUND, T_DLV, T_EMT = T_DLV + 5, T_N = T_EMT + 5 };
static_assert(T_N <= 16, "a row's lanes hold its counters");
DEV void qc(uint32_t& C, uint32_t k, uint32_t inc) { C += ql() == k ? inc : 0u; }

// one node per row: the hot scalars per lane, equal across the row; the
// cold ones one per lane of two registers (lane k holds field k, read by
// row_newbcast:k): the node's header words (H, lane k = word k: the tracked
// round and hop, the counts of words 9-11) and G below
struct Qn {
    uint32_t fl;                     // DESC due timers << 28 | QF_* bits
    uint32_t A;                      // lane j < 8: active[j]
    uint32_t root0, ne, nl, on;
    uint64_t have;
    uint32_t EG, LZ, OL, OH;         // lane i: eager[i], lazy[i], outstanding key i (low, high word)
    uint32_t seq;
    uint32_t H, G;
};
enum { G_ID, G_IB, G_IK, G_OW, G_OEND, G_CMASK };
enum { H_TRKR = 7, H_TRKH = 8, H_W9 = 9, H_W10 = 10, H_W11 = 11 };
template <int K> DEV uint32_t gf(const Qn& n) { return qbc<K>(n.G); }
template <int K> DEV uint32_t hf(const Qn& n) { return qbc<K>(n.H); }
DEV void setf(uint32_t& R, uint32_t k, uint32_t v) { R = ql() == k ? v : R; }
enum : uint32_t { QF_SETS = 1, QF_OUT = 2 };     // Qn::fl: the sets / the table changed

// send/3 (pt:633-638) of this lane's peer `e` (per lane): in the active view,
// running, same partition -- a compare against each member's lane
DEV bool qconn(const Qn& n, uint32_t e) {
    const uint32_t p = e & ~PSIM_MAP_BIT;
    const uint32_t cm = gf<G_CMASK>(n);
    bool c = false;
    qunroll<PSIM_ACTIVE_CAP>([&](auto J) {
        const uint32_t Aj = qbc<J>(n.A);
        c |= ((cm >> J) & 1u) && Aj == p;
    });
    return c;
}

// the record this lane sends (relay_emit, psim_consume.hip): a Plumtree
// record's ex words are 0; no store past the node's outbox (the engine fails
// the round on the bound check, stats T_BOUND).  The sender's id and outbox
// come in a Qe read with the whole row active: the emitting lanes are a
// per-lane subset, where a row_newbcast would read inactive lanes as 0.
struct Qe {
    uint32_t id, ow, oend;
};
DEV Qe qe(const Qn& n) { return Qe{gf<G_ID>(n), gf<G_OW>(n), gf<G_OEND>(n)}; }
DEV uint64_t qemit(KArgs& a, const Qe& e, uint32_t at, uint32_t dst, uint32_t tt, uint32_t a0, uint32_t a1,
                   uint32_t a2) {
    const uint32_t id = e.id, ow = e.ow, oend = e.oend;
    const uint32_t W[7] = {dst, id, tt, at, a0, a1, a2};
    uint64_t dg = 0;
#pragma unroll
    for (int j = 0; j < 7; j++) dg += (uint64_t)W[j] * digest_mul(j);
    const uint32_t slot = ow + at;
    if (slot < oend) {
        uint4* o = reinterpret_cast<uint4*>(a.rec_out + slot);
        o[0] = make_uint4(dst, id, tt, at);
        o[1] = make_uint4(a0, a1, a2, 0u);
        o[2] = make_uint4(0u, 0u, 0u, 0u);
        o[3] = make_uint4(0u, 0u, 0u, 0u);
        a.okey[slot] = dst | (max_emit(tt & 0xFF) << KEY_DST_BITS);
    }
    return dg;
}

// ordsets:add_element/2 / del_element/2 on a row list of n entries (lanes
// >= n hold 0; the caller guarantees room)
DEV void qadd(uint32_t& V, uint32_t& n, uint32_t x) {
    const uint32_t l = ql();
    const bool in = qany(l < n && V == x);
    const uint32_t pos = qcount(l < n && V < x);
    const uint32_t pv = qprev(V);
    if (in) return;
    V = l < pos ? V : l == pos ? x : l <= n ? pv : V;
    n++;
}
DEV void qdel(uint32_t& V, uint32_t& n, uint32_t x) {
    const uint32_t l = ql();
    const uint32_t m = qmask(l < n && V == x);
    const uint32_t nx = qnext(V);
    if (!m) return;
    const uint32_t at = (uint32_t)__builtin_ctz(m);
    V = l < at ? V : l + 1 < n ? nx : l + 1 == n ? 0u : V;
    n--;
}

// update_peers/5 + set_peers/4 (pt:593-609) on slot 0 (a new root takes it
// with the common eagers; the preconditions leave no other case)
DEV void qupdate(KArgs& a, Qn& n, uint32_t from, uint32_t root, bool to_eager) {
    n.fl |= QF_SETS;
    if (n.root0 != root) {
        n.root0 = root;
        const uint32_t l = ql();
        const uint32_t li = gf<G_ID>(n) - a.lo, com_n = hf<H_W10>(n) >> 24;
        const uint32_t c = l < 8u && l < com_n ? a.pt_com[(size_t)li * PSIM_PT_MEMBERS_CAP + l] : 0u;
        n.EG = c; n.LZ = 0u;
        n.ne = com_n; n.nl = 0;
    }
    if (to_eager) {
        qadd(n.EG, n.ne, from);
        qdel(n.LZ, n.nl, from);
    } else {
        qdel(n.EG, n.ne, from);
        qadd(n.LZ, n.nl, from);
    }
}

// add_outstanding/6 (pt:574-579), ack_outstanding/6 (pt:562-567): the table
// as sorted peer << 32 | msg << 16 | round keys, (OH, OL) per lane
DEV void qadd_out(Qn& n, uint32_t hi, uint32_t lo) {
    const uint32_t l = ql();
    const bool live = l < n.on;
    const bool in = qany(live && n.OH == hi && n.OL == lo);
    const uint32_t pos = qcount(live && (n.OH < hi || (n.OH == hi && n.OL < lo)));
    const uint32_t pl = qprev(n.OL), ph = qprev(n.OH);
    if (in) return;
    n.OL = l < pos ? n.OL : l == pos ? lo : l <= n.on ? pl : n.OL;
    n.OH = l < pos ? n.OH : l == pos ? hi : l <= n.on ? ph : n.OH;
    n.on++;
    n.fl |= QF_OUT;
}
DEV void qack_out(Qn& n, uint32_t hi, uint32_t lo) {
    const uint32_t l = ql();
    const uint32_t m = qmask(l < n.on && n.OH == hi && n.OL == lo);
    const uint32_t nl = qnext(n.OL), nh = qnext(n.OH);
    if (!m) return;
    const uint32_t at = (uint32_t)__builtin_ctz(m);
    n.OL = l < at ? n.OL : l + 1 < n.on ? nl : l + 1 == n.on ? 0u : n.OL;
    n.OH = l < at ? n.OH : l + 1 < n.on ? nh : l + 1 == n.on ? 0u : n.OH;
    n.on--;
    n.fl |= QF_OUT;
}

// appends the rows with `fall` (lane 0 of the row votes) to k_pt's list: wave
// counts, a block scan in LDS, one global atomic per block step
DEV void qappend(bool fall, const uint4& D, uint32_t* wcnt) {
    const uint64_t m = __ballot(fall && ql() == 0);
    const uint32_t wv = threadIdx.x >> 6;
    __syncthreads();
    if (__lane_id() == 0) wcnt[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t k = 0; k < QWPB; k++) t += wcnt[k];
        wcnt[QWPB] = t ? atomicAdd(kargs().n_pt, t) : 0u;
    }
    __syncthreads();
    if (fall && ql() == 0) {
        uint32_t b0 = wcnt[QWPB];
        for (uint32_t k = 0; k < wv; k++) b0 += wcnt[k];
        kargs().desc_pt[b0 + (uint32_t)__popcll(m & ((1ull << __lane_id()) - 1ull))] = D;
    }
}

}  // namespace

__global__ void __launch_bounds__(64 * QWPB) __attribute__((amdgpu_waves_per_eu(PSIM_PTQ_WAVES)))
k_ptq(RoundArgs) {
    if (*kargs().ctl) return;                         // an aborted batch (run_batch)
    __shared__ unsigned long long sst[T_N + 1];       // (+ the digest)
    __shared__ uint32_t sslots[2 * PSIM_MSG_SLOTS];
    __shared__ uint32_t wcnt[QWPB + 1];
    for (uint32_t i = threadIdx.x; i < 2 * PSIM_MSG_SLOTS; i += blockDim.x) sslots[i] = kargs().slots[i];
    if (threadIdx.x < T_N + 1) sst[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t l = ql();
    const uint32_t nq0 = kargs().n_ptl[0], nq = nq0 + kargs().n_ptl[1];
    uint32_t C = 0;                                   // lane k of a row: counter k of its nodes
    uint64_t dig = 0;
    const uint32_t row = (threadIdx.x >> 4);          // the block's row of this lane
    for (uint32_t base = blockIdx.x * QNODES; base < nq; base += gridDim.x * QNODES) {
        KArgs& a = kargs();
        const uint32_t P = base + row;
        Qn n;
        uint4 D = make_uint4(0, 0, 0, 0);
        bool valid = P < nq, ok = false;
        uint32_t tmask = 0, ik = 0;
        // the inbox's last chunk of 16 records (lane k: record 16 c + k), kept
        // for the handlers when it is the only chunk
        uint32_t qsrc = 0, qtype = 0, qmsg = 0, qrnd = 0, qroot = 0;
        if (valid) {
            D = ptl_desc(a, nq0, P);
            n.fl = (D.z >> 28) << 28;
            const uint32_t li = D.x - a.lo;
            // header word l, root-row word l (l < 8)
            n.H = reinterpret_cast<const uint32_t*>(a.hdr + li)[l];
            const uint32_t rw = l < RT_WORDS ? a.pt_rt[(size_t)li * RT_WORDS + l] : 0u;
            const uint32_t start = hf<2>(n), w5 = hf<5>(n), w6 = hf<6>(n), w11 = hf<H_W11>(n);
            const uint32_t r0 = qbc<0>(rw), r1 = qbc<1>(rw), r2 = qbc<2>(rw), r3 = qbc<3>(rw),
                           rtw4 = qbc<4>(rw), rtw5 = qbc<5>(rw);
            n.have = ((uint64_t)w5 << 32) | w6;
            n.on = (w11 >> 16) & 0xFF;
            n.root0 = r0;
            ik = start == a.round ? 0u : (D.z & DESC_CNT_MASK);
            n.G = l == G_ID ? D.x : l == G_IB ? D.y : l == G_IK ? ik : l == G_OW ? D.w : 0u;
            // the preconditions (k_ptl's): slot 0 only, no connection table,
            // every message's root slot 0's (or slot 0 free and one root), and
            // this inbox's adds fit 16 entries
            ok = r1 == NONE && r2 == NONE && r3 == NONE && (w11 & 0xFFFFu) == 0 &&
                 (r0 == NONE || ((rtw4 >> 8) == 0 && (rtw5 >> 8) == 0));
            uint32_t n_eg = 0, n_lz = 0, bml = 0, bmh = 0, r0t = r0;
            for (uint32_t c = 0; c < ik; c += QCAP) {
                const bool in = c + l < ik;
                uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;
                if (in) {
                    const uint4* rq = reinterpret_cast<const uint4*>(a.rec_in + D.y + c + l);
                    q0 = rq[0]; q1 = rq[1];
                }
                qsrc = q0.y; qtype = q0.z & 0xFF; qmsg = q1.x; qrnd = q1.y; qroot = q1.z;
                const bool pt = in && qtype >= PSIM_MSG_PT_BROADCAST && qtype <= PSIM_MSG_PT_GRAFT;
                n_eg += qcount(pt && (qtype == PSIM_MSG_PT_BROADCAST || qtype == PSIM_MSG_PT_IHAVE ||
                                      qtype == PSIM_MSG_PT_GRAFT));
                n_lz += qcount(pt && (qtype == PSIM_MSG_PT_BROADCAST || qtype == PSIM_MSG_PT_PRUNE));
                tmask |= qor(pt ? 1u << qtype : 0u);
                const bool bc = pt && qtype == PSIM_MSG_PT_BROADCAST;
                const uint32_t sk = qmsg % PSIM_MSG_SLOTS;
                bml |= qor(bc && sk < 32 ? 1u << sk : 0u);
                bmh |= qor(bc && sk >= 32 ? 1u << (sk - 32) : 0u);
                // the roots: the first message's (an IHAVE of a retired id
                // carries none) while slot 0 is free, then all equal to it
                const bool rs = pt && qtype != PSIM_MSG_PT_IGNORED_IHAVE;
                if (r0t == NONE) {
                    const uint32_t m = qmask(rs && qroot != NONE);
                    const uint32_t f = m ? (uint32_t)__builtin_ctz(m) : 16u;
                    const uint32_t rf = qget(qroot, f);
                    if (m) {
                        r0t = rf;
                        ok &= !qany(rs && l > f && qroot != r0t);
                    }
                } else {
                    ok &= !qany(rs && qroot != r0t);
                }
            }
            // first deliveries (lazy adds): the BROADCASTs' slots not delivered yet
            const uint32_t nb = (uint32_t)__popcll((((uint64_t)bmh << 32) | bml) & ~n.have);
            const uint32_t com_n = hf<H_W10>(n) >> 24;
            const uint32_t ne0 = r0 == NONE ? com_n : (rtw4 & 0xFF), nl0 = r0 == NONE ? 0u : (rtw5 & 0xFF);
            ok &= ne0 + n_eg <= QCAP && nl0 + n_lz <= QCAP && n.on + nb * (nl0 + n_lz) <= QCAP;
            n.ne = r0 == NONE ? 0u : (rtw4 & 0xFF);
            n.nl = r0 == NONE ? 0u : (rtw5 & 0xFF);
        }
        // nodes that do not fit go to k_pt's list (one atomic per block step)
        qappend(valid && !ok, D, wcnt);
        if (!(valid && ok)) continue;
        const uint32_t id = D.x;
        const size_t li = id - a.lo;
        {
            // the members' up and partition bytes, lane j < 8 member j's
            const uint32_t me_part = a.part[id], act_n = hf<H_W9>(n) & 0xFF;
            n.A = l < PSIM_ACTIVE_CAP ? a.act[li * PSIM_ACTIVE_CAP + l] : NONE;
            const bool mem = l < act_n && l < PSIM_ACTIVE_CAP && n.A < a.n_nodes;
            const uint32_t q = mem ? n.A : id;
            const uint32_t up = a.upart[q];
            setf(n.G, G_CMASK, qmask(mem && n.A != id && up == me_part));
        }
        // the sets only for messages that may update them, the table only for
        // lazy adds, acks or a lazy tick
        const bool need_sets = (tmask & ((1u << PSIM_MSG_PT_BROADCAST) | (1u << PSIM_MSG_PT_PRUNE) |
                                         (1u << PSIM_MSG_PT_IHAVE) | (1u << PSIM_MSG_PT_GRAFT))) != 0;
        const bool need_out = (tmask & ((1u << PSIM_MSG_PT_BROADCAST) | (1u << PSIM_MSG_PT_IGNORED_IHAVE))) != 0 ||
                              (((n.fl >> 28) & DESC_LAZY) && n.on > 0);
        n.EG = n.LZ = n.OL = n.OH = 0u;
        if (need_sets) {
            n.EG = a.pt_eag[li * RT_SET + l];
            n.LZ = a.pt_laz[li * RT_SET + l];
        }
        if (need_out) {
            const uint64_t o = a.pt_out[li * OUT_IN + l];
            n.OL = (uint32_t)o; n.OH = (uint32_t)(o >> 32);
        }
        n.seq = a.ocnt[li];
        setf(n.G, G_OEND, (uint32_t)a.obase[li + 1]);  // (the outbox's end slot)
        const bool one_chunk = ik <= QCAP;
        for (uint32_t c = 0; c < gf<G_IK>(n); c += QCAP) {   // the Plumtree inbox, canonical order
            const uint32_t ikc = gf<G_IK>(n), ib = gf<G_IB>(n);
            if (!one_chunk) {
                const bool in = c + l < ikc;
                uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;
                if (in) {
                    const uint4* rq = reinterpret_cast<const uint4*>(a.rec_in + ib + c + l);
                    q0 = rq[0]; q1 = rq[1];
                }
                qsrc = q0.y; qtype = q0.z & 0xFF; qmsg = q1.x; qrnd = q1.y; qroot = q1.z;
            }
            const uint32_t cn = min(QCAP, ikc - c);
            for (uint32_t j = 0; j < cn; j++) {
                const uint32_t type = qget(qtype, j);
                const uint32_t src = qget(qsrc, j), msg = qget(qmsg, j), rnd = qget(qrnd, j), root = qget(qroot, j);
                if (type < PSIM_MSG_PT_BROADCAST || type > PSIM_MSG_PT_GRAFT) continue;
                const uint32_t from = src | PSIM_MAP_BIT;
                qc(C, T_DLV + type - PSIM_MSG_PT_BROADCAST, 1);
                // plumtree_backend is_stale/1 over the slots (a retired id: overflow, stale)
                const uint32_t sk = msg % PSIM_MSG_SLOTS;
                const bool live = sslots[sk] == msg;
                const bool have = !live || ((n.have >> sk) & 1ull);
                if (type != PSIM_MSG_PT_PRUNE && type != PSIM_MSG_PT_IGNORED_IHAVE && !live) qc(C, T_OVF, 1);
                uint32_t sto = NONE, stt = 0, sa0 = 0, sa1 = 0;     // a single send of the handler
                if (type == PSIM_MSG_PT_BROADCAST) {     // pt:288-293, :368-378
                    if (!have) {
                        n.have |= 1ull << sk;
                        qc(C, T_FIRST, 1);
                        if (msg == a.tracked_msg) { setf(n.H, H_TRKR, a.round); setf(n.H, H_TRKH, rnd + 1); }
                        qupdate(a, n, from, root, true);
                        // eager_push/7: every eager entry but the sender, in
                        // set order, each lane its own record
                        const bool el = l < n.ne && n.EG != from;
                        const bool cn_ = qconn(n, n.EG);
                        const uint32_t okm = qmask(el && cn_);
                        qc(C, T_FAIL, qcount(el && !cn_));
                        const Qe e = qe(n);
                        if (el && cn_) {
                            const uint32_t at = n.seq + (uint32_t)__popc(okm & ((1u << l) - 1u));
                            dig += qemit(a, e, at, n.EG & ~PSIM_MAP_BIT, PSIM_MSG_PT_BROADCAST, msg, rnd + 1, root);
                        }
                        n.seq += (uint32_t)__popc(okm);
                        qc(C, T_EMT + 0, (uint32_t)__popc(okm));
                        // schedule_lazy_push/6: an outstanding entry per lazy peer
                        for (uint32_t i = 0; i < n.nl; i++) {
                            const uint32_t e = qget(n.LZ, i);
                            if (e != from) qadd_out(n, e, (msg << 16) | ((rnd + 1) & 0xFFFFu));
                        }
                    } else {
                        qupdate(a, n, from, root, false);
                        sto = from; stt = PSIM_MSG_PT_PRUNE;
                    }
                } else if (type == PSIM_MSG_PT_PRUNE) {  // pt:294-298
                    qupdate(a, n, from, root, false);
                } else if (type == PSIM_MSG_PT_IHAVE) {  // pt:299-303, :380-386
                    sto = from; stt = have ? PSIM_MSG_PT_IGNORED_IHAVE : PSIM_MSG_PT_GRAFT; sa0 = msg; sa1 = rnd;
                    if (!have) qupdate(a, n, from, root, true);
                } else if (type == PSIM_MSG_PT_IGNORED_IHAVE) {   // pt:304-307
                    qack_out(n, from, (msg << 16) | (rnd & 0xFFFFu));
                } else if (have) {                       // GRAFT pt:308-313, :388-402
                    qupdate(a, n, from, root, true);
                    sto = from; stt = PSIM_MSG_PT_BROADCAST; sa0 = msg; sa1 = rnd;
                }
                if (sto != NONE) {                        // (the IHAVE answer goes before the update in
                    const bool cs = qconn(n, sto);        //  the reference; the update sends nothing)
                    const Qe e = qe(n);
                    if (cs) {
                        if (l == 0) dig += qemit(a, e, n.seq, src, stt, sa0, sa1, root);
                        n.seq++;
                        qc(C, T_EMT + stt - PSIM_MSG_PT_BROADCAST, 1);
                    } else {
                        qc(C, T_FAIL, 1);
                    }
                }
            }
        }
        if (((n.fl >> 28) & DESC_LAZY) && n.on > 0) {   // the lazy tick (pt:341-345, :443-453)
            const bool el = l < n.on;
            const bool cs = qconn(n, n.OH);
            const uint32_t okm = qmask(el && cs);
            qc(C, T_FAIL, qcount(el && !cs));
            const uint32_t msg = (n.OL >> 16) & 0xFFFFu, sk = msg % PSIM_MSG_SLOTS;
            const bool live = sslots[sk] == msg;
            qc(C, T_OVF, qcount(el && cs && !live));
            const Qe e = qe(n);
            if (el && cs) {
                const uint32_t at = n.seq + (uint32_t)__popc(okm & ((1u << l) - 1u));
                dig += qemit(a, e, at, n.OH & ~PSIM_MAP_BIT, PSIM_MSG_PT_IHAVE, msg, n.OL & 0xFFFFu,
                             live ? sslots[PSIM_MSG_SLOTS + sk] : NONE);
            }
            n.seq += (uint32_t)__popc(okm);
            qc(C, T_EMT + 2, (uint32_t)__popc(okm));
        }
        // write back: header words 5-8 and 11, the sets, the table, the flag byte
        // (the row addresses recomputed from an opaque copy of the node id:
        // kept from the loads they held 10 VGPRs across the handlers)
        uint32_t idw = gf<G_ID>(n);
        asm volatile("" : "+v"(idw));
        const size_t lw = idw - a.lo;
        {
            uint32_t* hwp = reinterpret_cast<uint32_t*>(a.hdr + lw);
            const uint32_t v = l == 5 ? (uint32_t)(n.have >> 32) : l == 6 ? (uint32_t)n.have
                             : l == H_W11 ? (n.H & ~0xFF0000u) | (n.on << 16) : n.H;
            if ((l >= 5 && l <= 8) || l == H_W11) hwp[l] = v;
        }
        if (n.fl & QF_SETS) {
            // (slots 1-3 stay free, the count words hold slot 0's counts only)
            if (l < 6) {
                const uint32_t v = l == 0 ? n.root0 : l < 4 ? NONE : l == 4 ? n.ne : n.nl;
                a.pt_rt[lw * RT_WORDS + l] = v;
            }
            a.pt_eag[lw * RT_SET + l] = n.EG;
            a.pt_laz[lw * RT_SET + l] = n.LZ;
        }
        if (n.fl & QF_OUT) a.pt_out[lw * OUT_IN + l] = ((uint64_t)n.OH << 32) | n.OL;
        const uint32_t act_n = hf<H_W9>(n) & 0xFF, obound = gf<G_OEND>(n) - gf<G_OW>(n);
        if (l == 0) {
            a.ocnt[lw] = n.seq;
            const uint8_t fb = a.flags[idw];
            a.flags[idw] = (uint8_t)((fb & (F_UP | F_CRASHED)) | (n.on ? F_LAZY : 0) |
                                     (min(n.on, 15u) << F_OUTN_SHIFT) | (act_n < a.min_active ? F_LOWACT : 0));
        }
        qc(C, T_BOUND, n.seq > obound ? 1u : 0u);
    }
    // the rows' counters: lane k sums lane k of the four rows
    C += (uint32_t)__shfl_xor((int)C, 16);
    C += (uint32_t)__shfl_xor((int)C, 32);
    for (int o = 32; o > 0; o >>= 1) dig += shfl64(dig, (int)((__lane_id() + o) & 63));
    if (__lane_id() < T_N && C) atomicAdd(&sst[__lane_id()], (unsigned long long)C);
    if (__lane_id() == 0 && dig) atomicAdd(&sst[T_N], (unsigned long long)dig);
    __syncthreads();
    uint64_t* rowp = kargs().stat_ptl + (size_t)blockIdx.x * NST;
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
        rowp[k] = x;
    }
}

uint32_t ptq_block() { return 64 * QWPB; }
uint32_t ptq_nodes() { return QNODES; }
uint32_t ptq_grid() {
    int dev = 0, nb = 0;
    hipDeviceProp_t p;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)k_ptq, 64 * QWPB, 0) != hipSuccess || nb <= 0)
        return 1024;
    return (uint32_t)nb * (uint32_t)p.multiProcessorCount;
}

}  // namespace psim
