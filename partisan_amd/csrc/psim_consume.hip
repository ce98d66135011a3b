// psim_consume.hip -- the node-round kernel (K-consume + K-timer + K-emit).
//
// One lane owns one node for the whole round: it runs the node's EXIT events,
// its HyParView inbox, its timers, then its Plumtree inbox, origin broadcast
// and lazy tick, in the fixed order of the round model R0 (DESIGN.md section
// 2).  Everything the lane touches besides its own rows is read-only for the
// round (the flag/partition bytes of peers and the previous round's message
// records), so lanes never race.
//
// Reference handlers are cited as file:line under /root/reference:
//   hv = src/partisan_hyparview_peer_service_manager.erl
//   pt = src/partisan_plumtree_broadcast.erl
#include "psim_device.h"
#include "psim_kernels.h"

namespace psim {

#define ID_OF(e, n) (((uint32_t)(e) << 20) | (uint32_t)(n))
#define ID_E(id) ((id) >> 20)
#define ID_C(id) ((id)&0xFFFFFu)

struct Lane {
    const RoundArgs* a;
    uint32_t me;
    uint8_t mypart;
    Hdr h;
    uint32_t *act, *pas, *sentp, *senti, *recvp, *recvi, *all, *com, *eag, *laz;
    uint64_t* out;               // outstanding: peer << 32 | msg << 16 | round
    Msg* ob;                     // this node's outbox region
    uint32_t* okey;
    uint32_t seq;
    uint64_t* st;                // LDS stats of the block
};

__device__ __forceinline__ void st_add(Lane& L, int k, uint64_t v) {
    atomicAdd((unsigned long long*)&L.st[k], (unsigned long long)v);
}

// ---------------------------------------------------------------- RNG --
__device__ __forceinline__ uint64_t draw(Lane& L) { return draw58_at(L.h.rng++, L.me, L.a->seed); }

// rand:uniform/1 with a 58-bit generator (OTP rand.erl ?uniform_range)
__device__ uint32_t uniform_n(Lane& L, uint32_t n) {
    const uint64_t two58 = 1ull << 58;
    for (;;) {
        uint64_t v = draw(L);
        if (v < n) return (uint32_t)v + 1;
        uint64_t i = v % n;
        if (v - i <= two58 - n) return (uint32_t)i + 1;
    }
}

// ------------------------------------------------------- row primitives --
__device__ __forceinline__ int find(const uint32_t* row, uint32_t n, uint32_t e) {
    for (uint32_t i = 0; i < n; i++)
        if (row[i] == e) return (int)i;
    return -1;
}

// sets:add_element/2 keeping sets:to_list/1 order: (bucket, insertion seq)
__device__ void view_add(uint32_t* row, uint8_t& n, uint32_t e) {
    uint32_t b = bucket16(e);
    uint32_t i = n;
    while (i > 0 && bucket16(row[i - 1]) > b) { row[i] = row[i - 1]; i--; }
    row[i] = e;
    n++;
}

// sets:del_element/2 (order preserving); vacated slot zeroed
__device__ bool row_del(uint32_t* row, uint8_t& n, uint32_t e) {
    int k = find(row, n, e);
    if (k < 0) return false;
    for (uint32_t i = k; i + 1 < n; i++) row[i] = row[i + 1];
    n--;
    row[n] = 0;
    return true;
}

// ordsets:add_element/2 into a sorted row of capacity cap
__device__ bool ord_add(Lane& L, uint32_t* row, uint8_t& n, uint32_t cap, uint32_t e) {
    uint32_t i = n;
    while (i > 0 && row[i - 1] > e) i--;
    if (i > 0 && row[i - 1] == e) return true;
    if (n >= cap) { st_add(L, ST_OVF, 1); return false; }
    for (uint32_t j = n; j > i; j--) row[j] = row[j - 1];
    row[i] = e;
    n++;
    return true;
}

// select_random/2 (hv:1346-1356): uniform index over View -- Omit, no draw
// when nothing is eligible.  Up to three omitted elements.
__device__ uint32_t select_random(Lane& L, const uint32_t* row, uint32_t n, uint32_t o0,
                                  uint32_t o1, uint32_t o2) {
    uint32_t cnt = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint32_t e = row[i];
        cnt += (e != o0 && e != o1 && e != o2);
    }
    if (cnt == 0) return PSIM_NONE;
    uint32_t k = uniform_n(L, cnt) - 1;
    for (uint32_t i = 0; i < n; i++) {
        uint32_t e = row[i];
        if (e != o0 && e != o1 && e != o2) {
            if (k == 0) return e;
            k--;
        }
    }
    return PSIM_NONE;
}

// lists:sublist(shuffle(to_list(View)), K) (hv:1359-1361, :1586-1587).
// Element i's sort key is the counter-based draw at rng+i, so the k smallest
// (key, elem) pairs are found by k selection passes without storing keys.
__device__ uint32_t sublist(Lane& L, const uint32_t* row, uint32_t n, uint32_t k, uint32_t* out,
                            uint32_t on) {
    uint64_t base = L.h.rng;
    uint64_t pk = 0;
    uint32_t pe = 0;
    bool first = true;
    uint32_t m = n < k ? n : k;
    for (uint32_t j = 0; j < m; j++) {
        uint64_t bk = ~0ull;
        uint32_t be = 0xFFFFFFFFu;
        for (uint32_t i = 0; i < n; i++) {
            uint64_t kk = draw58_at(base + i, L.me, L.a->seed) >> 5;
            uint32_t e = row[i];
            bool after = first || kk > pk || (kk == pk && e > pe);
            bool better = kk < bk || (kk == bk && e < be);
            if (after && better) { bk = kk; be = e; }
        }
        out[on + j] = be;
        pk = bk; pe = be; first = false;
    }
    L.h.rng = base + n;
    return on + m;
}

// insertion-sort + dedupe (lists:usort/1 over ids)
__device__ uint32_t usort_small(uint32_t* v, uint32_t n) {
    for (uint32_t i = 1; i < n; i++) {
        uint32_t x = v[i];
        int j = (int)i - 1;
        while (j >= 0 && v[j] > x) { v[j + 1] = v[j]; j--; }
        v[j + 1] = x;
    }
    uint32_t k = n ? 1 : 0;
    for (uint32_t i = 1; i < n; i++)
        if (v[i] != v[k - 1]) v[k++] = v[i];
    return k;
}

// ------------------------------------------------------------- emission --
__device__ void emit(Lane& L, uint32_t dst, uint32_t type, uint32_t ttl, uint32_t a0, uint32_t a1,
                     uint32_t a2, const uint32_t* ex, uint32_t nex) {
    uint32_t s = L.seq++;
    Msg m;
    m.dst = dst; m.src = L.me; m.tt = type | (ttl << 8) | (nex << 16); m.seq = s;
    m.a0 = a0; m.a1 = a1; m.a2 = a2; m.pad = 0;
#pragma unroll
    for (int i = 0; i < PSIM_EXCHANGE_CAP; i++) m.ex[i] = (uint32_t)i < nex ? ex[i] : 0u;
    uint4* d = reinterpret_cast<uint4*>(&L.ob[s]);
    const uint4* q = reinterpret_cast<const uint4*>(&m);
    d[0] = q[0]; d[1] = q[1]; d[2] = q[2]; d[3] = q[3];
    L.okey[s] = dst | (max_emit(type) << KEY_DST_BITS);
    // digest: identical fold in the oracle (msg_hash)
    uint64_t hh = 0x9E3779B97F4A7C15ull ^ (((uint64_t)dst << 32) | L.me);
    hh = mix64(hh ^ (((uint64_t)s << 32) | (type << 16) | (ttl << 8) | nex));
    hh = mix64(hh ^ (((uint64_t)a0 << 32) | a1));
    hh = mix64(hh ^ a2);
    for (uint32_t i = 0; i < nex; i++) hh = mix64(hh ^ (((uint64_t)ex[i] << 32) | i));
    st_add(L, ST_DIGEST, hh);
    st_add(L, ST_EMIT + type, 1);
}

// maybe_connect + find (partisan_util.erl:75-134)
__device__ __forceinline__ bool connect_ok(const Lane& L, uint32_t dst) {
    if (dst >= L.a->n_nodes || dst == L.me) return false;
    return (L.a->flags[dst] & F_UP) && L.a->part[dst] == L.mypart;
}

// do_send_message/3 (hv:1274-1343); a successful send draws
// rand:uniform(1) in partisan_util:dispatch_pid/1 (util:190-195), which
// always consumes exactly one value.
__device__ void hv_send(Lane& L, uint32_t dst, uint32_t type, uint32_t ttl, uint32_t a0,
                        const uint32_t* ex, uint32_t nex) {
    if (!connect_ok(L, dst)) { st_add(L, ST_FAIL, 1); return; }
    L.h.rng++;
    emit(L, dst, type, ttl, a0, 0, 0, ex, nex);
}

// ------------------------------------------------------- disconnect ids --
__device__ __forceinline__ int map_find(const uint32_t* peer, uint32_t n, uint32_t p) {
    return find(peer, n, p);
}

__device__ void map_store(Lane& L, uint32_t* peer, uint32_t* id, uint8_t& n, uint8_t& head,
                          uint32_t p, uint32_t v) {
    int i = map_find(peer, n, p);
    if (i >= 0) { id[i] = v; return; }
    if (n < PSIM_IDMAP_CAP) { peer[n] = p; id[n] = v; n++; return; }
    st_add(L, ST_OVF, 1);
    peer[head] = p; id[head] = v;
    head = (uint8_t)((head + 1) % PSIM_IDMAP_CAP);
}

__device__ uint32_t current_id(Lane& L, uint32_t p) {   // hv:1622-1630
    int i = map_find(L.recvp, L.h.recv_n, p);
    return i >= 0 ? L.recvi[i] : ID_OF(1, 0);
}

__device__ uint32_t next_id(Lane& L, uint32_t p) {      // hv:1633-1639
    int i = map_find(L.sentp, L.h.sent_n, p);
    if (i >= 0 && ID_E(L.senti[i]) == L.h.epoch) return L.senti[i] + 1;
    return ID_OF(L.h.epoch, 1);
}

__device__ bool addable_epoch(Lane& L, uint32_t pe, uint32_t p) {   // hv:1670-1676
    int i = map_find(L.sentp, L.h.sent_n, p);
    return i < 0 || pe >= ID_E(L.senti[i]);
}

__device__ bool addable_id(Lane& L, uint32_t d, uint32_t p) {       // hv:1656-1669
    int i = map_find(L.sentp, L.h.sent_n, p);
    if (i < 0) return true;
    uint32_t s = L.senti[i];
    if (ID_E(d) != ID_E(s)) return ID_E(d) > ID_E(s);
    return ID_C(d) >= ID_C(s);
}

__device__ bool valid_disconnect(Lane& L, uint32_t p, uint32_t d) { // hv:1642-1653
    int i = map_find(L.recvp, L.h.recv_n, p);
    if (i < 0) return true;
    uint32_t s = L.recvi[i];
    if (ID_E(d) > ID_E(s)) return true;
    return ID_C(d) > ID_C(s);
}

// ---------------------------------------------------------- view updates --
__device__ void add_to_passive(Lane& L, uint32_t p) {   // hv:1423-1448
    if (p == L.me || find(L.act, L.h.act_n, p) >= 0 || find(L.pas, L.h.pas_n, p) >= 0) return;
    if (L.h.pas_n >= L.a->max_passive) {
        uint32_t r = select_random(L, L.pas, L.h.pas_n, L.me, L.me, L.me);
        if (r != PSIM_NONE) row_del(L.pas, L.h.pas_n, r);
    }
    view_add(L.pas, L.h.pas_n, p);
}

__device__ void drop_random_active(Lane& L) {           // hv:1467-1512
    uint32_t p = select_random(L, L.act, L.h.act_n, L.me, L.me, L.me);
    if (p == PSIM_NONE) return;
    row_del(L.act, L.h.act_n, p);
    add_to_passive(L, p);
    uint32_t nid = next_id(L, p);
    map_store(L, L.sentp, L.senti, L.h.sent_n, L.h.sent_head, p, nid);
    hv_send(L, p, PSIM_MSG_DISCONNECT, 0, nid, nullptr, 0);
}

__device__ void add_to_active(Lane& L, uint32_t p) {    // hv:1371-1420
    if (p == L.me || find(L.act, L.h.act_n, p) >= 0) return;
    row_del(L.pas, L.h.pas_n, p);
    if (L.h.act_n >= L.a->max_active) drop_random_active(L);
    view_add(L.act, L.h.act_n, p);
}

// usort([Myself] ++ sublist(Active, k_active) ++ sublist(Passive, k_passive))
__device__ uint32_t build_exchange(Lane& L, uint32_t* ex) {
    ex[0] = L.me;
    uint32_t n = 1;
    n = sublist(L, L.act, L.h.act_n, L.a->k_active, ex, n);
    n = sublist(L, L.pas, L.h.pas_n, L.a->k_passive, ex, n);
    return usort_small(ex, n);
}

// merge_exchange/2 (hv:1590-1595): usort(Exchange -- [Me | Active]) folded
// through add_to_passive_view in ascending id order.
__device__ void merge_exchange(Lane& L, const uint32_t* ex, uint32_t nex) {
    uint32_t prev = 0;
    bool first = true;
    for (;;) {
        uint32_t best = 0xFFFFFFFFu;
        bool found = false;
        for (uint32_t i = 0; i < nex; i++) {
            uint32_t e = ex[i];
            if (e == L.me || (!first && e <= prev)) continue;
            if (find(L.act, L.h.act_n, e) >= 0) continue;
            if (!found || e < best) { best = e; found = true; }
        }
        if (!found) break;
        add_to_passive(L, best);
        prev = best;
        first = false;
    }
}

__device__ void move_to_active(Lane& L, uint32_t p) {   // hv:1679-1709
    if (p == PSIM_NONE) return;
    uint32_t ex[1 + 2 * PSIM_EXCHANGE_CAP];
    uint32_t nex = build_exchange(L, ex);
    hv_send(L, p, PSIM_MSG_NEIGHBOR_REQUEST, 0, current_id(L, p), ex, nex);
}

// ------------------------------------------------------------ plumtree --
// notify/1 -> plumtree update/1: handle_cast({update, Members}) (pt:314-336)
__device__ void notify(Lane& L) {
    if (!L.a->plumtree) return;
    uint32_t cur[PSIM_ACTIVE_CAP];
    uint32_t nc = L.h.act_n;
    for (uint32_t i = 0; i < nc; i++) cur[i] = L.act[i];
    nc = usort_small(cur, nc);
    bool any_new = false;
    for (uint32_t i = 0; i < nc; i++)
        if (find(L.all, L.h.all_n, cur[i]) < 0) any_new = true;
    // Removed = all_members -- Current (computed before any reset)
    uint32_t rem[PSIM_PT_MEMBERS_CAP];
    uint32_t nr = 0;
    for (uint32_t i = 0; i < L.h.all_n; i++) {
        uint32_t e = L.all[i];
        bool in = false;
        for (uint32_t j = 0; j < nc; j++) in |= (cur[j] == e);
        if (!in) rem[nr++] = e;
    }
    if (any_new) {
        // common_eagers := (common_eagers U New); per-root sets wiped; all := Current
        for (uint32_t i = 0; i < nc; i++)
            if (find(L.all, L.h.all_n, cur[i]) < 0) {
                // insert into the sorted common row (room: |common| <= |all| <= 8 before removals)
                uint32_t e = cur[i];
                if (find(L.com, L.h.com_n, e) >= 0) continue;
                if (L.h.com_n >= PSIM_PT_MEMBERS_CAP) {
                    // drop a member that is about to be removed to make room
                    bool made = false;
                    for (uint32_t r = 0; r < nr && !made; r++) made = row_del(L.com, L.h.com_n, rem[r]);
                    if (!made) { st_add(L, ST_OVF, 1); continue; }
                }
                ord_add(L, L.com, L.h.com_n, PSIM_PT_MEMBERS_CAP, e);
            }
        L.h.pt_root = PSIM_NONE;
        for (uint32_t i = 0; i < L.h.eag_n; i++) L.eag[i] = 0;
        for (uint32_t i = 0; i < L.h.laz_n; i++) L.laz[i] = 0;
        L.h.eag_n = L.h.laz_n = 0;
        for (uint32_t i = 0; i < PSIM_PT_MEMBERS_CAP; i++) L.all[i] = i < nc ? cur[i] : 0u;
        L.h.all_n = (uint8_t)nc;
    }
    // neighbors_down(Removed, ..) (pt:404-423)
    for (uint32_t r = 0; r < nr; r++) {
        uint32_t e = rem[r];
        row_del(L.com, L.h.com_n, e);
        if (L.h.pt_root != PSIM_NONE) {
            row_del(L.eag, L.h.eag_n, e);
            row_del(L.laz, L.h.laz_n, e);
        }
        uint32_t j = 0;
        for (uint32_t k = 0; k < L.h.out_n; k++) {
            uint64_t o = L.out[k];
            if ((uint32_t)(o >> 32) != e) L.out[j++] = o;
        }
        for (uint32_t k = j; k < L.h.out_n; k++) L.out[k] = 0;
        L.h.out_n = (uint8_t)j;
    }
}

// the eager/lazy rows of Root: the per-root slot or the common default
__device__ __forceinline__ bool root_slot(const Lane& L, uint32_t root) {
    return L.h.pt_root != PSIM_NONE && L.h.pt_root == root;
}

// update_peers/5 (pt:599-609) for a single root slot
__device__ void pt_update(Lane& L, uint32_t from, uint32_t root, bool to_eager) {
    if (L.h.pt_root != PSIM_NONE && L.h.pt_root != root) { st_add(L, ST_OVF, 1); return; }
    if (L.h.pt_root == PSIM_NONE) {
        // first touch: the slot starts as (common_eagers, common_lazys = [])
        for (uint32_t i = 0; i < L.h.com_n; i++) L.eag[i] = L.com[i];
        L.h.eag_n = L.h.com_n;
        L.h.laz_n = 0;
        L.h.pt_root = root;
    }
    if (to_eager) {
        ord_add(L, L.eag, L.h.eag_n, PSIM_PT_SET_CAP, from);
        row_del(L.laz, L.h.laz_n, from);
    } else {
        row_del(L.eag, L.h.eag_n, from);
        ord_add(L, L.laz, L.h.laz_n, PSIM_PT_SET_CAP, from);
    }
}

// send/3 (pt:633-638): only over an existing connection of the manager
__device__ void pt_send(Lane& L, uint32_t ident, uint32_t type, uint32_t msg, uint32_t rnd,
                        uint32_t root) {
    uint32_t id = ident & ~PSIM_MAP_BIT;
    if (id == L.me || find(L.act, L.h.act_n, id) < 0 || !(L.a->flags[id] & F_UP) ||
        L.a->part[id] != L.mypart) {
        st_add(L, ST_FAIL, 1);
        return;
    }
    emit(L, id, type, 0, msg, rnd, root, nullptr, 0);
}

__device__ void pt_add_out(Lane& L, uint32_t peer, uint32_t msg, uint32_t rnd) {  // pt:574-579
    uint64_t key = ((uint64_t)peer << 32) | (msg << 16) | (rnd & 0xFFFFu);
    uint32_t i = L.h.out_n;
    while (i > 0 && L.out[i - 1] > key) i--;
    if (i > 0 && L.out[i - 1] == key) return;
    if (L.h.out_n >= PSIM_PT_OUT_CAP) { st_add(L, ST_OVF, 1); return; }
    for (uint32_t j = L.h.out_n; j > i; j--) L.out[j] = L.out[j - 1];
    L.out[i] = key;
    L.h.out_n++;
}

__device__ void pt_ack_out(Lane& L, uint32_t peer, uint32_t msg, uint32_t rnd) {  // pt:562-567
    uint64_t key = ((uint64_t)peer << 32) | (msg << 16) | (rnd & 0xFFFFu);
    for (uint32_t i = 0; i < L.h.out_n; i++)
        if (L.out[i] == key) {
            for (uint32_t j = i; j + 1 < L.h.out_n; j++) L.out[j] = L.out[j + 1];
            L.h.out_n--;
            L.out[L.h.out_n] = 0;
            return;
        }
}

// eager_push/7 + schedule_lazy_push/6 (pt:428-441)
__device__ void pt_push(Lane& L, uint32_t msg, uint32_t rnd, uint32_t root, uint32_t from) {
    if (root_slot(L, root)) {
        for (uint32_t i = 0; i < L.h.eag_n; i++)
            if (L.eag[i] != from) pt_send(L, L.eag[i], PSIM_MSG_PT_BROADCAST, msg, rnd, root);
        for (uint32_t i = 0; i < L.h.laz_n; i++)
            if (L.laz[i] != from) pt_add_out(L, L.laz[i], msg, rnd);
    } else {
        for (uint32_t i = 0; i < L.h.com_n; i++)
            if (L.com[i] != from) pt_send(L, L.com[i], PSIM_MSG_PT_BROADCAST, msg, rnd, root);
    }
}

__device__ __forceinline__ bool pt_have(const Lane& L, uint32_t msg) {
    return (L.h.have >> (msg & 31u)) & 1u;
}

__device__ void pt_handle(Lane& L, const Msg& m, uint32_t type) {
    uint32_t from = m.src | PSIM_MAP_BIT, msg = m.a0, rnd = m.a1, root = m.a2;
    switch (type) {
    case PSIM_MSG_PT_BROADCAST:                        // pt:288-293, :368-378
        if (!pt_have(L, msg)) {                        // backend merge/2
            L.h.have |= 1u << (msg & 31u);
            st_add(L, ST_FIRST, 1);
            if (msg == L.a->tracked_msg) { L.h.trk_round = L.a->round; L.h.trk_hop = rnd + 1; }
            pt_update(L, from, root, true);
            pt_push(L, msg, rnd + 1, root, from);
        } else {
            pt_update(L, from, root, false);
            pt_send(L, from, PSIM_MSG_PT_PRUNE, 0, 0, root);
        }
        break;
    case PSIM_MSG_PT_PRUNE:                            // pt:294-298
        pt_update(L, from, root, false);
        break;
    case PSIM_MSG_PT_IHAVE:                            // pt:299-303, :380-386
        if (pt_have(L, msg)) {
            pt_send(L, from, PSIM_MSG_PT_IGNORED_IHAVE, msg, rnd, root);
        } else {
            pt_send(L, from, PSIM_MSG_PT_GRAFT, msg, rnd, root);
            pt_update(L, from, root, true);
        }
        break;
    case PSIM_MSG_PT_IGNORED_IHAVE:                    // pt:304-307
        pt_ack_out(L, from, msg, rnd);
        break;
    case PSIM_MSG_PT_GRAFT:                            // pt:308-313, :388-402
        if (pt_have(L, msg)) {
            pt_update(L, from, root, true);
            pt_send(L, from, PSIM_MSG_PT_BROADCAST, msg, rnd, root);
        }
        break;
    default:
        break;
    }
}

// ----------------------------------------------------------- hyparview --
__device__ void hv_handle(Lane& L, const Msg& m, uint32_t type) {
    const RoundArgs& a = *L.a;
    uint32_t me = L.me, p = m.src;
    switch (type) {
    case PSIM_MSG_JOIN: {                              // hv:703-771
        uint32_t pe = m.a0;
        if (addable_epoch(L, pe, p) && find(L.act, L.h.act_n, p) < 0 && connect_ok(L, p)) {
            add_to_active(L, p);
            hv_send(L, p, PSIM_MSG_NEIGHBOR, 0, current_id(L, p), nullptr, 0);
            // (members(Active) -- [Myself]) -- [Peer], in to_list order; the
            // sends never change the active view, so iterate it in place
            for (uint32_t i = 0; i < L.h.act_n; i++) {
                uint32_t q = L.act[i];
                if (q != me && q != p) {
                    if (!connect_ok(L, q)) { st_add(L, ST_FAIL, 1); continue; }
                    L.h.rng++;
                    emit(L, q, PSIM_MSG_FORWARD_JOIN, a.arwl, p, pe, 0, nullptr, 0);
                }
            }
            notify(L);
        }
        break;
    }
    case PSIM_MSG_NEIGHBOR:                            // hv:774-805
        if (addable_id(L, m.a0, p) && connect_ok(L, p)) add_to_active(L, p);
        notify(L);
        break;
    case PSIM_MSG_FORWARD_JOIN: {                      // hv:808-923
        uint32_t q = m.a0, pe = m.a1, ttl = (m.tt >> 8) & 0xFF, sender = p;
        if (ttl == 0 || L.h.act_n == 1) {
            if (addable_epoch(L, pe, q) && find(L.act, L.h.act_n, q) < 0 && connect_ok(L, q)) {
                add_to_active(L, q);
                hv_send(L, q, PSIM_MSG_NEIGHBOR, 0, current_id(L, q), nullptr, 0);
            }
        } else {
            // the passive add at TTL == prwl never changes the active view,
            // so Active0 is the live row for the select and the membership test
            if (ttl == a.prwl) add_to_passive(L, q);
            uint32_t r = select_random(L, L.act, L.h.act_n, sender, me, q);
            if (r == PSIM_NONE) {
                if (addable_epoch(L, pe, q) && find(L.act, L.h.act_n, q) < 0 && connect_ok(L, q)) {
                    add_to_active(L, q);
                    hv_send(L, q, PSIM_MSG_NEIGHBOR, 0, current_id(L, q), nullptr, 0);
                }
            } else if (connect_ok(L, r)) {
                L.h.rng++;
                emit(L, r, PSIM_MSG_FORWARD_JOIN, ttl - 1, q, pe, 0, nullptr, 0);
            } else {
                st_add(L, ST_FAIL, 1);
            }
        }
        notify(L);
        break;
    }
    case PSIM_MSG_DISCONNECT: {                        // hv:926-972
        uint32_t d = m.a0;
        if (!valid_disconnect(L, p, d)) break;
        row_del(L.act, L.h.act_n, p);
        // select_random(Passive0, [Myself, Peer]) uses the passive view from
        // before the add below: draw over it first, in its own order, by
        // remembering whether the add evicts (the only change the add makes
        // besides inserting p, which is omitted from the draw anyway).
        uint32_t pas0[PSIM_PASSIVE_CAP];
        uint32_t np0 = L.h.pas_n;
        bool isolated;
        for (uint32_t i = 0; i < np0; i++) pas0[i] = L.pas[i];
        add_to_passive(L, p);
        map_store(L, L.recvp, L.recvi, L.h.recv_n, L.h.recv_head, p, d);
        isolated = (L.h.act_n == 1);
        if (isolated) move_to_active(L, select_random(L, pas0, np0, me, p, me));
        break;
    }
    case PSIM_MSG_NEIGHBOR_REQUEST: {                  // hv:975-1053
        uint32_t ack[1 + 2 * PSIM_EXCHANGE_CAP];
        uint32_t nack = build_exchange(L, ack);
        if (addable_id(L, m.a0, p)) {
            if (connect_ok(L, p)) {
                hv_send(L, p, PSIM_MSG_NEIGHBOR_ACCEPTED, 0, current_id(L, p), ack, nack);
                add_to_active(L, p);
            }
        } else {
            hv_send(L, p, PSIM_MSG_NEIGHBOR_REJECTED, 0, 0, ack, nack);
        }
        merge_exchange(L, m.ex, (m.tt >> 16) & 0xFF);
        notify(L);
        break;
    }
    case PSIM_MSG_NEIGHBOR_REJECTED:                   // hv:1056-1067
        merge_exchange(L, m.ex, (m.tt >> 16) & 0xFF);
        break;
    case PSIM_MSG_NEIGHBOR_ACCEPTED:                   // hv:1070-1089
        if (addable_id(L, m.a0, p)) add_to_active(L, p);
        merge_exchange(L, m.ex, (m.tt >> 16) & 0xFF);
        notify(L);
        break;
    case PSIM_MSG_SHUFFLE_REPLY:                       // hv:1091-1093
        merge_exchange(L, m.ex, (m.tt >> 16) & 0xFF);
        break;
    case PSIM_MSG_SHUFFLE: {                           // hv:1095-1136
        uint32_t ttl = (m.tt >> 8) & 0xFF, nex = (m.tt >> 16) & 0xFF;
        if (ttl > 0 && L.h.act_n > 1) {
            uint32_t r = select_random(L, L.act, L.h.act_n, p, me, me);
            if (r != PSIM_NONE) hv_send(L, r, PSIM_MSG_SHUFFLE, ttl - 1, 0, m.ex, nex);
        } else {
            uint32_t resp[PSIM_EXCHANGE_CAP];
            uint32_t nr = sublist(L, L.pas, L.h.pas_n, nex, resp, 0);
            hv_send(L, p, PSIM_MSG_SHUFFLE_REPLY, 0, 0, resp, nr);
            merge_exchange(L, m.ex, nex);
        }
        break;
    }
    default:
        break;
    }
}

__device__ __forceinline__ bool timer_due(uint32_t period, uint32_t r, uint32_t start) {
    return period > 0 && r > start && ((r - start) % period) == 0;
}

__device__ __forceinline__ void load_msg(const Msg* __restrict__ rec, uint32_t slot, Msg& m) {
    const uint4* q = reinterpret_cast<const uint4*>(&rec[slot]);
    uint4* d = reinterpret_cast<uint4*>(&m);
    d[0] = q[0]; d[1] = q[1]; d[2] = q[2]; d[3] = q[3];
}

__global__ void __launch_bounds__(256) k_consume(RoundArgs args) {
    __shared__ uint64_t sst[NST];
    for (int i = threadIdx.x; i < NST; i += blockDim.x) sst[i] = 0;
    __syncthreads();

    const RoundArgs& a = args;
    uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n < a.n_nodes) do {
        uint8_t fl = a.flags[n];
        uint32_t ib = a.in_beg[n], ik = a.in_cnt[n];
        if (!(fl & F_UP)) {
            if (ik) atomicAdd((unsigned long long*)&sst[ST_DROPPED], (unsigned long long)ik);
            break;
        }
        atomicAdd((unsigned long long*)&sst[ST_UP], 1ull);
        Lane L;
        L.a = &args;
        L.me = n;
        L.mypart = a.part[n];
        L.st = sst;
        {
            const uint4* q = reinterpret_cast<const uint4*>(&a.hdr[n]);
            uint4* d = reinterpret_cast<uint4*>(&L.h);
            d[0] = q[0]; d[1] = q[1]; d[2] = q[2]; d[3] = q[3];
        }
        const uint32_t r = a.round;
        if (L.h.start_round == r && ik) {       // fresh incarnation: no connections yet
            atomicAdd((unsigned long long*)&sst[ST_DROPPED], (unsigned long long)ik);
            ik = 0;
        }
        L.act = a.act + (size_t)n * PSIM_ACTIVE_CAP;
        bool promo = a.random_promotion && timer_due(a.promotion_period, r, L.h.start_round);
        bool shuf = timer_due(a.shuffle_period, r, L.h.start_round);
        bool origin = a.origin_now && a.origin_node == n && a.plumtree;
        bool lazy_due = a.plumtree && timer_due(a.lazy_tick_period, r, L.h.start_round);
        bool lazy = lazy_due && L.h.out_n > 0;
        bool joining = L.h.start_round == r && L.h.join_contact != PSIM_NONE;
        uint32_t exits[PSIM_ACTIVE_CAP];
        uint32_t nexit = 0;
        if (a.crash_round) {
            for (uint32_t i = 0; i < L.h.act_n; i++) {
                uint32_t d = L.act[i];
                if (d != n && (a.flags[d] & F_CRASHED)) exits[nexit++] = d;
            }
        }
        if (!(ik || joining || nexit || promo || shuf || origin || lazy)) break;
        atomicAdd((unsigned long long*)&sst[ST_PROC], 1ull);

        L.pas = a.pas + (size_t)n * PSIM_PASSIVE_CAP;
        L.sentp = a.sentp + (size_t)n * PSIM_IDMAP_CAP;
        L.senti = a.senti + (size_t)n * PSIM_IDMAP_CAP;
        L.recvp = a.recvp + (size_t)n * PSIM_IDMAP_CAP;
        L.recvi = a.recvi + (size_t)n * PSIM_IDMAP_CAP;
        L.all = a.pt_all + (size_t)n * PSIM_PT_MEMBERS_CAP;
        L.com = a.pt_com + (size_t)n * PSIM_PT_MEMBERS_CAP;
        L.eag = a.pt_eag + (size_t)n * PSIM_PT_SET_CAP;
        L.laz = a.pt_laz + (size_t)n * PSIM_PT_SET_CAP;
        L.out = a.pt_out + (size_t)n * PSIM_PT_OUT_CAP;
        L.ob = a.rec_out + a.obase[n];
        L.okey = a.okey + a.obase[n];
        L.seq = 0;

        if (joining)                                    // hv:500-515
            hv_send(L, L.h.join_contact, PSIM_MSG_JOIN, 0, L.h.epoch, nullptr, 0);

        for (uint32_t i = 0; i < nexit; i++) {          // hv:609-654
            uint32_t d = exits[i];
            atomicAdd((unsigned long long*)&sst[ST_EXITS], 1ull);
            row_del(L.pas, L.h.pas_n, d);
            if (row_del(L.act, L.h.act_n, d))
                move_to_active(L, select_random(L, L.pas, L.h.pas_n, n, n, n));
        }

        Msg m;
        for (uint32_t i = 0; i < ik; i++) {             // HyParView inbox, canonical order
            load_msg(a.rec_in, a.in_slot[ib + i], m);
            uint32_t type = m.tt & 0xFF;
            if (type < PSIM_MSG_PT_BROADCAST) {
                atomicAdd((unsigned long long*)&sst[ST_DELIV + type], 1ull);
                hv_handle(L, m, type);
            }
        }

        if (promo && L.h.act_n < a.min_active) {        // hv:542-561
            move_to_active(L, select_random(L, L.pas, L.h.pas_n, n, n, n));
        }
        if (shuf) {                                     // hv:572-607
            uint32_t ex[1 + 2 * PSIM_EXCHANGE_CAP];
            uint32_t nex = build_exchange(L, ex);
            uint32_t t = select_random(L, L.act, L.h.act_n, n, n, n);
            if (t != PSIM_NONE) hv_send(L, t, PSIM_MSG_SHUFFLE, a.arwl, 0, ex, nex);
        }

        if (a.plumtree) {
            for (uint32_t i = 0; i < ik; i++) {         // Plumtree inbox
                load_msg(a.rec_in, a.in_slot[ib + i], m);
                uint32_t type = m.tt & 0xFF;
                if (type >= PSIM_MSG_PT_BROADCAST && type <= PSIM_MSG_PT_GRAFT) {
                    atomicAdd((unsigned long long*)&sst[ST_DELIV + type], 1ull);
                    pt_handle(L, m, type);
                }
            }
            if (origin) {                               // pt:282-287, backend:179-200
                uint32_t my = n | PSIM_MAP_BIT;
                L.h.have |= 1u << (a.origin_msg & 31u);
                L.h.trk_round = r;
                L.h.trk_hop = 0;
                pt_push(L, a.origin_msg, 0, my, my);
            }
            if (lazy_due) {                             // pt:341-345, :443-453
                for (uint32_t i = 0; i < L.h.out_n; i++) {
                    uint64_t o = L.out[i];
                    pt_send(L, (uint32_t)(o >> 32), PSIM_MSG_PT_IHAVE, (uint32_t)(o >> 16) & 0xFFFFu,
                            (uint32_t)o & 0xFFFFu, a.bcast_root);
                }
            }
        }

        // write back the header and the outbox count
        {
            uint4* d = reinterpret_cast<uint4*>(&a.hdr[n]);
            const uint4* q = reinterpret_cast<const uint4*>(&L.h);
            d[0] = q[0]; d[1] = q[1]; d[2] = q[2]; d[3] = q[3];
        }
        a.ocnt[n] = L.seq;
        // only this lane writes its own flag byte; peers read just F_UP/F_CRASHED
        uint8_t nf = (fl & ~F_LAZY) | (L.h.out_n ? F_LAZY : 0);
        if (nf != fl) a.flags[n] = nf;
    } while (0);

    __syncthreads();
    for (int i = threadIdx.x; i < NST; i += blockDim.x)
        a.stat_part[(size_t)blockIdx.x * NST + i] = sst[i];
}

}  // namespace psim
