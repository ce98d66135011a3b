// psim_engine.hip -- device memory, event kernels, the message route
// (K-route) and the C ABI of include/partisan_gpu_sim.h.
//
// One round on one shard:
//   events   -> k_crash / k_join / k_bcast_reset        (pending API calls)
//   prepare  -> k_runs  : run lengths + outbox bounds of the sorted inbox
//               k_bounds: per-node outbox bound; scans -> in_beg, obase
//   consume  -> k_consume (psim_consume.hip)
//   route    -> scan(ocnt) -> k_compact -> radix sort by dst (stable, so
//               each inbox is in canonical (src, seq) order) -> next inbox
//   stats    -> k_stats_reduce
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "psim_device.h"
#include "psim_kernels.h"

using namespace psim;

namespace {

constexpr int BLK = 256;

#define HIP_TRY(x)                                                       \
    do {                                                                 \
        hipError_t e_ = (x);                                             \
        if (e_ != hipSuccess) {                                          \
            std::fprintf(stderr, "psim: %s failed: %s (%s:%d)\n", #x,    \
                         hipGetErrorString(e_), __FILE__, __LINE__);     \
            return PSIM_EDEVICE;                                         \
        }                                                                \
    } while (0)

// ------------------------------------------------------------ kernels --
__global__ void k_crash(uint8_t* flags, const uint32_t* ids, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t id = ids[i];
    uint8_t f = flags[id];
    if (f & F_UP) flags[id] = (uint8_t)((f & ~F_UP) | F_CRASHED);
}

__global__ void k_uncrash(uint8_t* flags, const uint32_t* ids, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    flags[ids[i]] &= (uint8_t)~F_CRASHED;
}

// node start: init/1 of the manager (hv:289-354) and of the broadcast
// server (pt:251-264, members = [own name]); one lane per joining node.
__global__ void k_join(RoundArgs a, const uint32_t* ids, const uint32_t* contacts, uint32_t n,
                       uint32_t persist_epoch) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t id = ids[i];
    Hdr h;
    uint32_t old_epoch = a.hdr[id].epoch;
    memset(&h, 0, sizeof h);
    h.epoch = persist_epoch ? old_epoch + 1 : 1;
    h.start_round = a.round;
    h.join_contact = contacts[i];
    h.pt_root = PSIM_NONE;
    h.trk_round = PSIM_NONE;
    h.act_n = 1; h.all_n = 1; h.com_n = 1;
    a.hdr[id] = h;
    uint32_t* act = a.act + (size_t)id * PSIM_ACTIVE_CAP;
    for (int k = 0; k < PSIM_ACTIVE_CAP; k++) act[k] = k == 0 ? id : 0u;
    uint32_t* pas = a.pas + (size_t)id * PSIM_PASSIVE_CAP;
    for (int k = 0; k < PSIM_PASSIVE_CAP; k++) pas[k] = 0;
    for (int k = 0; k < PSIM_IDMAP_CAP; k++) {
        a.sentp[(size_t)id * PSIM_IDMAP_CAP + k] = 0; a.senti[(size_t)id * PSIM_IDMAP_CAP + k] = 0;
        a.recvp[(size_t)id * PSIM_IDMAP_CAP + k] = 0; a.recvi[(size_t)id * PSIM_IDMAP_CAP + k] = 0;
    }
    for (int k = 0; k < PSIM_PT_MEMBERS_CAP; k++) {
        a.pt_all[(size_t)id * PSIM_PT_MEMBERS_CAP + k] = k == 0 ? id : 0u;
        a.pt_com[(size_t)id * PSIM_PT_MEMBERS_CAP + k] = k == 0 ? id : 0u;
    }
    for (int k = 0; k < PSIM_PT_SET_CAP; k++) {
        a.pt_eag[(size_t)id * PSIM_PT_SET_CAP + k] = 0;
        a.pt_laz[(size_t)id * PSIM_PT_SET_CAP + k] = 0;
    }
    for (int k = 0; k < PSIM_PT_OUT_CAP; k++) a.pt_out[(size_t)id * PSIM_PT_OUT_CAP + k] = 0;
    a.flags[id] = (uint8_t)((a.flags[id] & F_CRASHED) | F_UP | (1u < a.min_active ? F_LOWACT : 0));
    const_cast<uint32_t*>(a.start)[id] = a.round;
}

__global__ void k_bcast_reset(Hdr* hdr, uint32_t n, uint32_t bit) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    hdr[i].have &= ~bit;
    hdr[i].trk_round = PSIM_NONE;
    hdr[i].trk_hop = 0;
}

// Run lengths of the sorted inbox: the lane at the start of each dst run
// writes the run's length and the sum of its messages' emission bounds.
__global__ void k_runs(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ m_ptr,
                       uint32_t* cnt, uint32_t* bsum) {
    uint32_t m = *m_ptr;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        uint32_t k = keys[i], d = k & KEY_DST_MASK;
        if (i > 0 && (keys[i - 1] & KEY_DST_MASK) == d) continue;
        uint32_t j = i, s = 0;
        while (j < m && (keys[j] & KEY_DST_MASK) == d) { s += keys[j] >> KEY_DST_BITS; j++; }
        cnt[d] = j - i;
        bsum[d] = s;
    }
}

__device__ __forceinline__ bool due(uint32_t period, uint32_t r, uint32_t start) {
    return period > 0 && r > start && ((r - start) % period) == 0;
}

// Per node: the upper bound of its emissions this round (sizes its outbox
// region) and whether it has any work (inbox, join, timers, EXIT scan,
// origin, outstanding lazy pushes).  Also counts live nodes and messages
// addressed to dead ones.
__global__ void k_node_prep(RoundArgs a, const uint32_t* bsum, uint64_t* bound, uint32_t* work,
                            uint64_t* part) {
    __shared__ uint64_t s_up, s_drop;
    if (threadIdx.x == 0) { s_up = 0; s_drop = 0; }
    __syncthreads();
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.n_nodes) {
        uint8_t f = a.flags[i];
        uint64_t b = 0;
        uint32_t w = 0;
        uint32_t c = a.in_cnt[i];
        if (f & F_UP) {
            uint32_t st = a.start[i], r = a.round;
            b = bsum[i] + BOUND_BASE;
            if (f & F_LAZY) b += BOUND_LAZY;
            if (a.crash_round) b += BOUND_EXITS;
            if (a.origin_now && i == a.origin_node) b += BOUND_ORIGIN;
            w = c > 0 || st == r || a.crash_round || (f & F_LAZY) ||
                (a.origin_now && i == a.origin_node) ||
                (a.random_promotion && (f & F_LOWACT) && due(a.promotion_period, r, st)) ||
                due(a.shuffle_period, r, st);
            atomicAdd((unsigned long long*)&s_up, 1ull);
        } else if (c) {
            atomicAdd((unsigned long long*)&s_drop, (unsigned long long)c);
        }
        bound[i] = b;
        work[i] = w;
    }
    __syncthreads();
    if (threadIdx.x < NST) {
        uint64_t v = threadIdx.x == ST_UP ? s_up : threadIdx.x == ST_DROPPED ? s_drop : 0ull;
        part[(size_t)blockIdx.x * NST + threadIdx.x] = v;
    }
}

// Dense (key, slot) pairs of this round's emissions, in node (= src, seq) order.
__global__ void k_compact(const uint32_t* ocnt, const uint32_t* dpos, const uint64_t* obase,
                          const uint32_t* okey, uint32_t* keys, uint32_t* vals, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t c = ocnt[i];
    if (!c) return;
    uint32_t p = dpos[i];
    uint64_t b = obase[i];
    for (uint32_t j = 0; j < c; j++) {
        keys[p + j] = okey[b + j];
        vals[p + j] = (uint32_t)(b + j);
    }
}

// one block per stats slot; lanes stride over the per-block partials
__global__ void k_stats_reduce(const uint64_t* part, uint32_t nblocks, uint64_t* out) {
    __shared__ uint64_t red[BLK];
    uint32_t k = blockIdx.x;
    uint64_t s = 0;
    for (uint32_t b = threadIdx.x; b < nblocks; b += blockDim.x) s += part[(size_t)b * NST + k];
    red[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t w = blockDim.x / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[k] = red[0];
}

// ------------------------------------------------------------- buffers --
template <typename T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    int ensure(size_t want) {
        if (want <= n) return PSIM_OK;
        if (p) hipFree(p);
        p = nullptr; n = 0;
        size_t cap = std::max<size_t>(want + want / 4, 1024);
        if (hipMalloc(&p, cap * sizeof(T)) != hipSuccess) return PSIM_ENOMEM;
        n = cap;
        return PSIM_OK;
    }
    int alloc(size_t want) {   // exact, zeroed
        if (hipMalloc(&p, std::max<size_t>(want, 1) * sizeof(T)) != hipSuccess) return PSIM_ENOMEM;
        n = want;
        if (hipMemset(p, 0, std::max<size_t>(want, 1) * sizeof(T)) != hipSuccess) return PSIM_EDEVICE;
        return PSIM_OK;
    }
    void release() { if (p) hipFree(p); p = nullptr; n = 0; }
};

enum Kern { KT_EVENTS, KT_PREPARE, KT_CONSUME, KT_SCAN, KT_COMPACT, KT_SORT, KT_STATS, KT_N };
const char* kKernName[KT_N] = {"events", "prepare", "consume", "scan", "compact", "sort", "stats"};

}  // namespace

struct psim_handle {
    psim_config cfg;
    uint32_t N;
    int device;
    hipStream_t stream;
    uint64_t round = 0;
    // node state
    DBuf<uint8_t> flags, part;
    DBuf<Hdr> hdr;
    DBuf<uint32_t> act, pas, sentp, senti, recvp, recvi, pt_all, pt_com, pt_eag, pt_laz;
    DBuf<uint64_t> pt_out;
    // route
    DBuf<Msg> rec[2];
    DBuf<uint32_t> okey, ocnt, dpos, keys[2], vals[2], cnt, bsum, in_beg, start, work, alist, d_nact;
    DBuf<uint64_t> bound, obase;
    DBuf<uint32_t> d_m;          // [0] = messages in the current inbox
    DBuf<uint64_t> stat_part, stat_out;
    DBuf<uint8_t> cub_tmp;
    DBuf<uint32_t> ev_ids, ev_contacts;
    uint32_t cur = 0;            // rec[cur] holds the inbox records
    uint32_t m_in = 0;           // messages in the inbox
    // pending events
    std::vector<uint32_t> pend_crash, pend_join, pend_contact;
    std::vector<uint8_t> pend_part;
    bool pend_part_set = false, pend_part_clear = false;
    bool pend_bcast = false;
    uint32_t pend_root = 0, pend_msg = 0;
    uint32_t bcast_root = PSIM_NONE, tracked_msg = PSIM_NONE;
    // profiling
    hipEvent_t ev[KT_N][2];
    double kt_ms[KT_N] = {0};
    uint64_t kt_n[KT_N] = {0};
};

namespace {

RoundArgs make_args(psim_handle* h) {
    RoundArgs a;
    memset(&a, 0, sizeof a);
    const psim_config& c = h->cfg;
    a.n_nodes = h->N; a.round = (uint32_t)h->round; a.seed = c.seed;
    a.max_active = c.max_active_size; a.min_active = c.min_active_size;
    a.max_passive = c.max_passive_size; a.arwl = c.arwl; a.prwl = c.prwl;
    a.k_active = c.k_active; a.k_passive = c.k_passive;
    a.shuffle_period = c.shuffle_period; a.promotion_period = c.promotion_period;
    a.random_promotion = c.random_promotion; a.plumtree = c.plumtree;
    a.lazy_tick_period = c.lazy_tick_period;
    a.tracked_msg = h->tracked_msg; a.bcast_root = h->bcast_root;
    a.origin_node = PSIM_NONE;
    a.flags = h->flags.p; a.part = h->part.p; a.hdr = h->hdr.p;
    a.act = h->act.p; a.pas = h->pas.p; a.sentp = h->sentp.p; a.senti = h->senti.p;
    a.recvp = h->recvp.p; a.recvi = h->recvi.p;
    a.pt_all = h->pt_all.p; a.pt_com = h->pt_com.p; a.pt_eag = h->pt_eag.p; a.pt_laz = h->pt_laz.p;
    a.pt_out = h->pt_out.p;
    a.start = h->start.p;
    return a;
}

struct KTimer {
    psim_handle* h;
    int k;
    KTimer(psim_handle* h_, int k_) : h(h_), k(k_) { hipEventRecord(h->ev[k][0], h->stream); }
    ~KTimer() {
        hipEventRecord(h->ev[k][1], h->stream);
        hipEventSynchronize(h->ev[k][1]);
        float ms = 0;
        hipEventElapsedTime(&ms, h->ev[k][0], h->ev[k][1]);
        h->kt_ms[k] += ms;
        h->kt_n[k]++;
    }
};

inline uint32_t grid_for(uint64_t n) { return (uint32_t)std::max<uint64_t>(1, (n + BLK - 1) / BLK); }

int scan_u32(psim_handle* h, const uint32_t* in, uint32_t* out, uint32_t n) {
    size_t tb = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, n, h->stream));
    if (h->cub_tmp.ensure(tb)) return PSIM_ENOMEM;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(h->cub_tmp.p, tb, in, out, n, h->stream));
    return PSIM_OK;
}

int scan_u64(psim_handle* h, const uint64_t* in, uint64_t* out, uint32_t n) {
    size_t tb = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, n, h->stream));
    if (h->cub_tmp.ensure(tb)) return PSIM_ENOMEM;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(h->cub_tmp.p, tb, in, out, n, h->stream));
    return PSIM_OK;
}

template <typename T>
T read1(psim_handle* h, const T* p) {
    T v{};
    hipMemcpyAsync(&v, p, sizeof(T), hipMemcpyDeviceToHost, h->stream);
    hipStreamSynchronize(h->stream);
    return v;
}

int upload(psim_handle* h, DBuf<uint32_t>& b, const std::vector<uint32_t>& v) {
    if (b.ensure(v.size())) return PSIM_ENOMEM;
    HIP_TRY(hipMemcpyAsync(b.p, v.data(), v.size() * 4, hipMemcpyHostToDevice, h->stream));
    return PSIM_OK;
}

int dst_bits(uint32_t n) {
    int b = 1;
    while (b < (int)KEY_DST_BITS && (1ull << b) < n) b++;
    return b;
}

int run_round(psim_handle* h, uint64_t* stats_out) {
    const uint32_t N = h->N;
    RoundArgs a = make_args(h);
    int rc;
    bool crashes = !h->pend_crash.empty();
    // ---- events
    {
        KTimer t(h, KT_EVENTS);
        if (crashes) {
            if ((rc = upload(h, h->ev_ids, h->pend_crash))) return rc;
            k_crash<<<grid_for(h->pend_crash.size()), BLK, 0, h->stream>>>(
                h->flags.p, h->ev_ids.p, (uint32_t)h->pend_crash.size());
        }
        if (!h->pend_join.empty()) {
            if ((rc = upload(h, h->ev_ids, h->pend_join))) return rc;
            if ((rc = upload(h, h->ev_contacts, h->pend_contact))) return rc;
            k_join<<<grid_for(h->pend_join.size()), BLK, 0, h->stream>>>(
                a, h->ev_ids.p, h->ev_contacts.p, (uint32_t)h->pend_join.size(), h->cfg.persist_epoch);
        }
        if (h->pend_part_clear) HIP_TRY(hipMemsetAsync(h->part.p, 0, N, h->stream));
        if (h->pend_part_set)
            HIP_TRY(hipMemcpyAsync(h->part.p, h->pend_part.data(), N, hipMemcpyHostToDevice, h->stream));
        if (h->pend_bcast) {
            h->tracked_msg = h->pend_msg;
            k_bcast_reset<<<grid_for(N), BLK, 0, h->stream>>>(h->hdr.p, N, 1u << (h->pend_msg & 31u));
            // origin only if the root's manager is running after the events
            uint8_t f = 0;
            HIP_TRY(hipMemcpyAsync(&f, h->flags.p + h->pend_root, 1, hipMemcpyDeviceToHost, h->stream));
            HIP_TRY(hipStreamSynchronize(h->stream));
            if (f & F_UP) { a.origin_now = 1; a.origin_node = h->pend_root; a.origin_msg = h->pend_msg; }
        }
        a.tracked_msg = h->tracked_msg;
        a.crash_round = crashes;
    }
    std::vector<uint32_t> crashed = h->pend_crash;
    h->pend_crash.clear(); h->pend_join.clear(); h->pend_contact.clear();
    h->pend_part_set = h->pend_part_clear = false;
    h->pend_bcast = false;

    // ---- prepare: inbox run lengths, outbox bounds, offsets, active list
    uint64_t total_bound;
    const uint32_t pgrid = grid_for(N);
    const uint32_t cgrid = std::min<uint32_t>(grid_for(N), 2048);
    {
        KTimer t(h, KT_PREPARE);
        HIP_TRY(hipMemsetAsync(h->cnt.p, 0, (size_t)N * 4, h->stream));
        HIP_TRY(hipMemsetAsync(h->bsum.p, 0, (size_t)N * 4, h->stream));
        if (h->m_in) {
            uint32_t g = std::min<uint32_t>(grid_for(h->m_in), 4096);
            k_runs<<<g, BLK, 0, h->stream>>>(h->keys[0].p, h->d_m.p, h->cnt.p, h->bsum.p);
        }
        a.in_cnt = h->cnt.p;
        if (h->stat_part.ensure((size_t)(pgrid + cgrid) * NST)) return PSIM_ENOMEM;
        k_node_prep<<<pgrid, BLK, 0, h->stream>>>(a, h->bsum.p, h->bound.p, h->work.p, h->stat_part.p);
        {
            size_t tb = 0;
            hipcub::CountingInputIterator<uint32_t> ids(0);
            HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, ids, h->work.p, h->alist.p, h->d_nact.p,
                                                  N, h->stream));
            if (h->cub_tmp.ensure(tb)) return PSIM_ENOMEM;
            HIP_TRY(hipcub::DeviceSelect::Flagged(h->cub_tmp.p, tb, ids, h->work.p, h->alist.p,
                                                  h->d_nact.p, N, h->stream));
        }
        if ((rc = scan_u32(h, h->cnt.p, h->in_beg.p, N))) return rc;
        if ((rc = scan_u64(h, h->bound.p, h->obase.p, N))) return rc;
        uint64_t last_b = read1(h, h->bound.p + (N - 1));
        uint64_t last_o = read1(h, h->obase.p + (N - 1));
        total_bound = last_b + last_o;
    }
    if (total_bound >= 0xFFFFFFFFull) return PSIM_ENOMEM;
    uint32_t nxt = h->cur ^ 1;
    if (h->rec[nxt].ensure(total_bound + 1)) return PSIM_ENOMEM;
    if (h->okey.ensure(total_bound + 1)) return PSIM_ENOMEM;

    // ---- consume
    a.in_beg = h->in_beg.p; a.in_cnt = h->cnt.p; a.in_slot = h->vals[0].p;
    a.alist = h->alist.p; a.n_alist = h->d_nact.p;
    a.rec_in = h->rec[h->cur].p;
    a.obase = h->obase.p;
    a.rec_out = h->rec[nxt].p; a.okey = h->okey.p; a.ocnt = h->ocnt.p;
    a.stat_part = h->stat_part.p + (size_t)pgrid * NST;
    {
        KTimer t(h, KT_CONSUME);
        HIP_TRY(hipMemsetAsync(h->ocnt.p, 0, (size_t)N * 4, h->stream));
        k_consume<<<cgrid, BLK, 0, h->stream>>>(a);
        HIP_TRY(hipGetLastError());
    }
    // ---- route: dense (dst, slot) pairs, stable sort by dst
    uint32_t m_out;
    {
        KTimer t(h, KT_SCAN);
        if ((rc = scan_u32(h, h->ocnt.p, h->dpos.p, N))) return rc;
        uint32_t last_c = read1(h, h->ocnt.p + (N - 1));
        uint32_t last_p = read1(h, h->dpos.p + (N - 1));
        m_out = last_c + last_p;
    }
    for (int b = 0; b < 2; b++) {
        if (h->keys[b].ensure(m_out + 1) || h->vals[b].ensure(m_out + 1)) return PSIM_ENOMEM;
    }
    {
        KTimer t(h, KT_COMPACT);
        k_compact<<<grid_for(N), BLK, 0, h->stream>>>(h->ocnt.p, h->dpos.p, h->obase.p, h->okey.p,
                                                     h->keys[1].p, h->vals[1].p, N);
    }
    {
        KTimer t(h, KT_SORT);
        if (m_out) {
            size_t tb = 0;
            int bits = dst_bits(N);
            HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, h->keys[1].p, h->keys[0].p,
                                                       h->vals[1].p, h->vals[0].p, m_out, 0, bits,
                                                       h->stream));
            if (h->cub_tmp.ensure(tb)) return PSIM_ENOMEM;
            HIP_TRY(hipcub::DeviceRadixSort::SortPairs(h->cub_tmp.p, tb, h->keys[1].p, h->keys[0].p,
                                                       h->vals[1].p, h->vals[0].p, m_out, 0, bits,
                                                       h->stream));
        }
        HIP_TRY(hipMemcpyAsync(h->d_m.p, &m_out, 4, hipMemcpyHostToDevice, h->stream));
    }
    {
        KTimer t(h, KT_STATS);
        k_stats_reduce<<<NST, BLK, 0, h->stream>>>(h->stat_part.p, pgrid + cgrid, h->stat_out.p);
        if (!crashed.empty()) {
            if ((rc = upload(h, h->ev_ids, crashed))) return rc;
            k_uncrash<<<grid_for(crashed.size()), BLK, 0, h->stream>>>(h->flags.p, h->ev_ids.p,
                                                                      (uint32_t)crashed.size());
        }
        HIP_TRY(hipMemcpyAsync(stats_out, h->stat_out.p, NST * 8, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
    }
    h->m_in = m_out;
    h->cur = nxt;
    h->round++;
    return PSIM_OK;
}

void fill_stats(const uint64_t* s, uint64_t round, psim_round_stats* o) {
    memset(o, 0, sizeof *o);
    o->round = round;
    for (int i = 0; i < PSIM_MSG_NTYPES; i++) {
        o->emitted[i] = s[ST_EMIT + i];
        o->delivered[i] = s[ST_DELIV + i];
    }
    o->dropped = s[ST_DROPPED]; o->nodes_up = s[ST_UP]; o->nodes_processed = s[ST_PROC];
    o->exits = s[ST_EXITS]; o->send_fail = s[ST_FAIL]; o->first_deliveries = s[ST_FIRST];
    o->overflow = s[ST_OVF]; o->digest = s[ST_DIGEST]; o->state_bytes = s[ST_BYTES];
}

}  // namespace

// ================================================================ C ABI ==
extern "C" {

int psim_abi_version(void) { return PSIM_ABI_VERSION; }

const char* psim_strerror(int code) {
    switch (code) {
    case PSIM_OK: return "ok";
    case PSIM_EINVAL: return "invalid argument";
    case PSIM_ENOMEM: return "out of memory";
    case PSIM_EDEVICE: return "HIP runtime error";
    case PSIM_ESTATE: return "invalid state";
    case PSIM_ERANGE: return "node id out of range";
    case PSIM_ECOMM: return "communication error";
    case PSIM_EUNSUPPORTED: return "unsupported";
    default: return "unknown error";
    }
}

void psim_default_config(psim_config* cfg) {
    memset(cfg, 0, sizeof *cfg);
    cfg->abi_version = PSIM_ABI_VERSION;
    cfg->n_nodes = 32;
    cfg->seed = 1;
    cfg->max_active_size = 6; cfg->min_active_size = 3; cfg->max_passive_size = 30;
    cfg->arwl = 5; cfg->prwl = 30; cfg->k_active = 3; cfg->k_passive = 4;
    cfg->shuffle_period = 10; cfg->promotion_period = 5; cfg->random_promotion = 1;
    cfg->persist_epoch = 0; cfg->plumtree = 1; cfg->lazy_tick_period = 1;
    cfg->device = -1; cfg->n_shards = 1; cfg->shard_world = 1;
}

int psim_create(const psim_config* cfg, psim_handle** out) {
    if (!cfg || !out || cfg->abi_version != PSIM_ABI_VERSION || cfg->n_nodes == 0 ||
        cfg->n_nodes > KEY_DST_MASK || cfg->max_active_size < 2 ||
        cfg->max_active_size > PSIM_ACTIVE_CAP || cfg->max_passive_size < 1 ||
        cfg->max_passive_size > 30 || 1 + cfg->k_active + cfg->k_passive > PSIM_EXCHANGE_CAP ||
        cfg->arwl > 255 || cfg->prwl > 255)
        return PSIM_EINVAL;
    if (cfg->n_shards > 1 || cfg->shard_world > 1) return PSIM_EUNSUPPORTED;
    psim_handle* h = new (std::nothrow) psim_handle();
    if (!h) return PSIM_ENOMEM;
    h->cfg = *cfg;
    h->N = cfg->n_nodes;
    int dev = cfg->device;
    if (dev < 0) { if (hipGetDevice(&dev) != hipSuccess) { delete h; return PSIM_EDEVICE; } }
    if (hipSetDevice(dev) != hipSuccess) { delete h; return PSIM_EDEVICE; }
    h->device = dev;
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) { delete h; return PSIM_EDEVICE; }
    for (int k = 0; k < KT_N; k++) { hipEventCreate(&h->ev[k][0]); hipEventCreate(&h->ev[k][1]); }
    const size_t N = h->N;
    int rc = 0;
    rc |= h->flags.alloc(N); rc |= h->part.alloc(N); rc |= h->hdr.alloc(N);
    rc |= h->act.alloc(N * PSIM_ACTIVE_CAP); rc |= h->pas.alloc(N * PSIM_PASSIVE_CAP);
    rc |= h->sentp.alloc(N * PSIM_IDMAP_CAP); rc |= h->senti.alloc(N * PSIM_IDMAP_CAP);
    rc |= h->recvp.alloc(N * PSIM_IDMAP_CAP); rc |= h->recvi.alloc(N * PSIM_IDMAP_CAP);
    rc |= h->pt_all.alloc(N * PSIM_PT_MEMBERS_CAP); rc |= h->pt_com.alloc(N * PSIM_PT_MEMBERS_CAP);
    rc |= h->pt_eag.alloc(N * PSIM_PT_SET_CAP); rc |= h->pt_laz.alloc(N * PSIM_PT_SET_CAP);
    rc |= h->pt_out.alloc(N * PSIM_PT_OUT_CAP);
    rc |= h->ocnt.alloc(N); rc |= h->dpos.alloc(N); rc |= h->cnt.alloc(N); rc |= h->bsum.alloc(N);
    rc |= h->in_beg.alloc(N); rc |= h->bound.alloc(N); rc |= h->obase.alloc(N);
    rc |= h->start.alloc(N); rc |= h->work.alloc(N); rc |= h->alist.alloc(N); rc |= h->d_nact.alloc(1);
    rc |= h->d_m.alloc(1); rc |= h->stat_out.alloc(NST);
    rc |= h->keys[0].alloc(1024); rc |= h->vals[0].alloc(1024);
    rc |= h->rec[0].alloc(1024);
    if (rc) { psim_destroy(h); return PSIM_ENOMEM; }
    *out = h;
    return PSIM_OK;
}

void psim_destroy(psim_handle* h) {
    if (!h) return;
    hipSetDevice(h->device);
    hipStreamSynchronize(h->stream);
    h->flags.release(); h->part.release(); h->hdr.release();
    h->act.release(); h->pas.release(); h->sentp.release(); h->senti.release();
    h->recvp.release(); h->recvi.release(); h->pt_all.release(); h->pt_com.release();
    h->pt_eag.release(); h->pt_laz.release(); h->pt_out.release();
    for (int b = 0; b < 2; b++) { h->rec[b].release(); h->keys[b].release(); h->vals[b].release(); }
    h->okey.release(); h->ocnt.release(); h->dpos.release(); h->cnt.release(); h->bsum.release();
    h->in_beg.release(); h->bound.release(); h->obase.release(); h->d_m.release();
    h->start.release(); h->work.release(); h->alist.release(); h->d_nact.release();
    h->stat_part.release(); h->stat_out.release(); h->cub_tmp.release();
    h->ev_ids.release(); h->ev_contacts.release();
    for (int k = 0; k < KT_N; k++) { hipEventDestroy(h->ev[k][0]); hipEventDestroy(h->ev[k][1]); }
    hipStreamDestroy(h->stream);
    delete h;
}

int psim_join(psim_handle* h, const uint32_t* nodes, const uint32_t* contacts, size_t n) {
    if (!h || (n && (!nodes || !contacts))) return PSIM_EINVAL;
    for (size_t i = 0; i < n; i++)
        if (nodes[i] >= h->N || (contacts[i] != PSIM_NONE && contacts[i] >= h->N)) return PSIM_ERANGE;
    h->pend_join.insert(h->pend_join.end(), nodes, nodes + n);
    h->pend_contact.insert(h->pend_contact.end(), contacts, contacts + n);
    return PSIM_OK;
}

int psim_crash(psim_handle* h, const uint32_t* nodes, size_t n) {
    if (!h || (n && !nodes)) return PSIM_EINVAL;
    for (size_t i = 0; i < n; i++)
        if (nodes[i] >= h->N) return PSIM_ERANGE;
    h->pend_crash.insert(h->pend_crash.end(), nodes, nodes + n);
    return PSIM_OK;
}

int psim_set_partition(psim_handle* h, const uint8_t* group, size_t n) {
    if (!h || !group || n != h->N) return PSIM_EINVAL;
    h->pend_part.assign(group, group + n);
    h->pend_part_set = true; h->pend_part_clear = false;
    return PSIM_OK;
}

int psim_clear_partition(psim_handle* h) {
    if (!h) return PSIM_EINVAL;
    h->pend_part_clear = true; h->pend_part_set = false;
    return PSIM_OK;
}

int psim_broadcast(psim_handle* h, uint32_t root, uint32_t msg_id) {
    if (!h) return PSIM_EINVAL;
    if (root >= h->N || msg_id > 0xFFFF) return PSIM_ERANGE;
    uint32_t r = root | PSIM_MAP_BIT;
    if (h->bcast_root != PSIM_NONE && h->bcast_root != r) return PSIM_EUNSUPPORTED;
    h->bcast_root = r;
    h->pend_bcast = true; h->pend_root = root; h->pend_msg = msg_id;
    return PSIM_OK;
}

int psim_step(psim_handle* h, uint32_t n_rounds, psim_round_stats* stats) {
    if (!h) return PSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return PSIM_EDEVICE;
    for (int k = 0; k < KT_N; k++) { h->kt_ms[k] = 0; h->kt_n[k] = 0; }
    for (uint32_t i = 0; i < n_rounds; i++) {
        uint64_t st[NST];
        uint64_t r = h->round;
        int rc = run_round(h, st);
        if (rc) return rc;
        if (stats) fill_stats(st, r, &stats[i]);
    }
    return PSIM_OK;
}

int psim_get_round(psim_handle* h, uint64_t* round) {
    if (!h || !round) return PSIM_EINVAL;
    *round = h->round;
    return PSIM_OK;
}

int psim_get_nodes(psim_handle* h, uint32_t first, uint32_t count, psim_node_view* out) {
    if (!h || (count && !out)) return PSIM_EINVAL;
    if ((uint64_t)first + count > h->N) return PSIM_ERANGE;
    if (!count) return PSIM_OK;
    if (hipSetDevice(h->device) != hipSuccess) return PSIM_EDEVICE;
    std::vector<Hdr> hd(count);
    std::vector<uint8_t> fl(count);
    std::vector<uint32_t> act((size_t)count * PSIM_ACTIVE_CAP), pas((size_t)count * PSIM_PASSIVE_CAP);
    std::vector<uint32_t> sp((size_t)count * PSIM_IDMAP_CAP), si(sp.size()), rp(sp.size()), ri(sp.size());
    std::vector<uint32_t> all((size_t)count * PSIM_PT_MEMBERS_CAP), com(all.size());
    std::vector<uint32_t> eag((size_t)count * PSIM_PT_SET_CAP), laz(eag.size());
    std::vector<uint64_t> po((size_t)count * PSIM_PT_OUT_CAP);
    auto cp = [&](void* dst, const void* src, size_t bytes) {
        return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->stream);
    };
    HIP_TRY(cp(hd.data(), h->hdr.p + first, count * sizeof(Hdr)));
    HIP_TRY(cp(fl.data(), h->flags.p + first, count));
    HIP_TRY(cp(act.data(), h->act.p + (size_t)first * PSIM_ACTIVE_CAP, act.size() * 4));
    HIP_TRY(cp(pas.data(), h->pas.p + (size_t)first * PSIM_PASSIVE_CAP, pas.size() * 4));
    HIP_TRY(cp(sp.data(), h->sentp.p + (size_t)first * PSIM_IDMAP_CAP, sp.size() * 4));
    HIP_TRY(cp(si.data(), h->senti.p + (size_t)first * PSIM_IDMAP_CAP, si.size() * 4));
    HIP_TRY(cp(rp.data(), h->recvp.p + (size_t)first * PSIM_IDMAP_CAP, rp.size() * 4));
    HIP_TRY(cp(ri.data(), h->recvi.p + (size_t)first * PSIM_IDMAP_CAP, ri.size() * 4));
    HIP_TRY(cp(all.data(), h->pt_all.p + (size_t)first * PSIM_PT_MEMBERS_CAP, all.size() * 4));
    HIP_TRY(cp(com.data(), h->pt_com.p + (size_t)first * PSIM_PT_MEMBERS_CAP, com.size() * 4));
    HIP_TRY(cp(eag.data(), h->pt_eag.p + (size_t)first * PSIM_PT_SET_CAP, eag.size() * 4));
    HIP_TRY(cp(laz.data(), h->pt_laz.p + (size_t)first * PSIM_PT_SET_CAP, laz.size() * 4));
    HIP_TRY(cp(po.data(), h->pt_out.p + (size_t)first * PSIM_PT_OUT_CAP, po.size() * 8));
    HIP_TRY(hipStreamSynchronize(h->stream));
    for (uint32_t k = 0; k < count; k++) {
        psim_node_view* v = &out[k];
        const Hdr& x = hd[k];
        memset(v, 0, sizeof *v);
        v->up = fl[k] & F_UP; v->epoch = x.epoch; v->start_round = x.start_round; v->pt_root = x.pt_root;
        v->rng_ctr = x.rng;
        v->act_n = x.act_n; v->pas_n = x.pas_n;
        memcpy(v->act, &act[(size_t)k * PSIM_ACTIVE_CAP], sizeof v->act);
        memcpy(v->pas, &pas[(size_t)k * PSIM_PASSIVE_CAP], sizeof v->pas);
        v->sent_n = x.sent_n; v->sent_head = x.sent_head; v->recv_n = x.recv_n; v->recv_head = x.recv_head;
        memcpy(v->sent_peer, &sp[(size_t)k * PSIM_IDMAP_CAP], sizeof v->sent_peer);
        memcpy(v->sent_id, &si[(size_t)k * PSIM_IDMAP_CAP], sizeof v->sent_id);
        memcpy(v->recv_peer, &rp[(size_t)k * PSIM_IDMAP_CAP], sizeof v->recv_peer);
        memcpy(v->recv_id, &ri[(size_t)k * PSIM_IDMAP_CAP], sizeof v->recv_id);
        v->pt_all_n = x.all_n; v->pt_common_n = x.com_n; v->pt_eager_n = x.eag_n;
        v->pt_lazy_n = x.laz_n; v->pt_out_n = x.out_n;
        memcpy(v->pt_all, &all[(size_t)k * PSIM_PT_MEMBERS_CAP], sizeof v->pt_all);
        memcpy(v->pt_common, &com[(size_t)k * PSIM_PT_MEMBERS_CAP], sizeof v->pt_common);
        memcpy(v->pt_eager, &eag[(size_t)k * PSIM_PT_SET_CAP], sizeof v->pt_eager);
        memcpy(v->pt_lazy, &laz[(size_t)k * PSIM_PT_SET_CAP], sizeof v->pt_lazy);
        for (int j = 0; j < PSIM_PT_OUT_CAP; j++) {
            uint64_t o = po[(size_t)k * PSIM_PT_OUT_CAP + j];
            v->pt_out_peer[j] = (uint32_t)(o >> 32);
            v->pt_out_msg[j] = (uint32_t)(o >> 16) & 0xFFFFu;
            v->pt_out_round[j] = (uint32_t)o & 0xFFFFu;
        }
        v->have = x.have; v->trk_round = x.trk_round; v->trk_hop = x.trk_hop;
    }
    return PSIM_OK;
}

int psim_kernel_times(psim_handle* h, const char** names, double* ms, uint64_t* launches, int cap) {
    if (!h) return PSIM_EINVAL;
    int k = 0;
    for (; k < KT_N && k < cap; k++) {
        if (names) names[k] = kKernName[k];
        if (ms) ms[k] = h->kt_ms[k];
        if (launches) launches[k] = h->kt_n[k];
    }
    return k;
}

int psim_comm_id_size(void) { return 128; }

int psim_get_comm_id(void* buf, size_t cap) {
    (void)buf; (void)cap;
    return PSIM_EUNSUPPORTED;
}

}  // extern "C"
