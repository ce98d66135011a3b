// psim_engine.hip -- device memory, event kernels, the message route
// (K-route), the cross-shard exchange and the C ABI of
// include/partisan_gpu_sim.h.
//
// The global id space [0, N) is cut into G contiguous shards.  A process owns
// `n_shards` of them (virtual shards on its device, exchanged by device
// copies) or exactly one when run as an RCCL rank (shard_world > 1).  Per
// round and shard (DESIGN.md sections 3 and 7):
//   events   k_crash / k_join / k_bcast_reset    (same event list on every shard)
//   prepare  k_node_prep (packed bound | work flag per node), one scan of them,
//            k_desc (outbox bases + descriptors of the nodes with work)
//   consume  k_consume (psim_consume.hip)
//   route    G == 1: count (atomics) -> scan -> scatter -> per-run sort of
//                    source indices -> gather (stable radix sort when one run
//                    is too long)
//            G  > 1: stable partition by owner shard -> gather records ->
//                    all-to-all (counts, then records) -> the same grouping
//                    of the shard-ordered concatenation by dst
//   stats    k_stats_tiles + k_stats_final (+ sum over shards / the ranks' all-reduce)
// Ranks exchange through psim_comm.h: RCCL, or the loopback test vehicle.
// Grouping a (src, seq)-ordered stream -- or a concatenation ordered by
// source shard -- by dst, each group in stream order, yields each inbox in
// canonical (src, seq) order,
// so any shard count gives bit-identical results.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <set>
#include <vector>

#include "psim_comm.h"
#include "psim_device.h"
#include "psim_kernels.h"

using namespace psim;

namespace {

constexpr int BLK = 256;
constexpr uint32_t PREP_BLK = 1024;   // k_desc blocks (at most PREP_BLK of them)
#ifndef PSIM_PREP_NPT
#define PSIM_PREP_NPT 4       // (2: step 0.620 -> 0.615 ms at 2^20 against 1 node a thread, profiles/r05/ab_log.txt r6m, r6n)
#endif
constexpr uint32_t PREP_NPT = PSIM_PREP_NPT;   // k_node_prep: nodes a thread (loads a node ahead)
#ifndef PSIM_PREP_CHUNK
#define PSIM_PREP_CHUNK 4
#endif
constexpr uint32_t PREP_CHUNK = PSIM_PREP_CHUNK;   // k_node_prep: nodes a thread loads, works and stores together
constexpr uint32_t DESC_RANGES = 4;   // k_node_prep ranges a k_desc block takes (at most DESC_RANGES * PREP_BLK)
// pinned host words per shard (Shard::pin): NST stats, the consume span, the
// outbox total, the routed record count -- stored by kernels, read by the host
enum { PIN_TOTAL = NST + 2, PIN_M = NST + 3, PIN_OVF = NST + 4, PIN_BIGIN = NST + 5, PIN_OUTX = NST + 6 };
// the rank path's words of a round (RCCL ranks; all-reduced, so every rank
// reads the same): PIN_XAB ranks whose round aborted (a batch's capacity
// checks, exchange_fixed), PIN_XMH / PIN_XMT the ranks' largest per-owner head
// / tail counts, summed; then this rank's per-owner send counts (G words)
enum { PIN_XAB = NST + 8, PIN_XMH = NST + 9, PIN_XMT = NST + 10, PIN_XCNT = NST + 16 };
// ... then every rank's largest per-owner head count (word PIN_XRANK + r)
// and tail count (PIN_XRANK + 64 + r): each rank fills its own words and
// zeros the others', so the sum all-reduce leaves the exact maxima
constexpr uint32_t PIN_XRANK = PIN_XCNT + 64;
// slot 0 only: the largest outbox total (k_desc) and routed count (the
// route) since the host last cleared them (PSIM_TRACE_BOUND, psim_step)
enum { PIN_TMAX = NST + 7, PIN_MMAX = NST + 11 };
// stat_out: NST sums, the node-round span (2), the three x-words of the
// rank path (all-reduced with the sums)
constexpr uint32_t STAT_OUT_X = NST + 2, STAT_OUT_R = NST + 5, STAT_OUT_N = NST + 5 + 128;
// the pinned words: slot 0 holds the above (and a single round's stats);
// slot j + 1 the stats and node-round span of round j of a batch (run_batch)
constexpr uint32_t PIN_STRIDE = PIN_XRANK + 128;
constexpr uint32_t BATCH_MAX = 64;

#define HIP_TRY(x)                                                       \
    do {                                                                 \
        hipError_t e_ = (x);                                             \
        if (e_ != hipSuccess) {                                          \
            std::fprintf(stderr, "psim: %s failed: %s (%s:%d)\n", #x,    \
                         hipGetErrorString(e_), __FILE__, __LINE__);     \
            return PSIM_EDEVICE;                                         \
        }                                                                \
    } while (0)

#define TRY(x)                   \
    do {                         \
        int rc_ = (x);           \
        if (rc_) return rc_;     \
    } while (0)

// ------------------------------------------------------------ kernels --
__global__ void k_crash(uint8_t* flags, uint32_t* crash_bits, const uint32_t* ids, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t id = ids[i];
    uint8_t f = flags[id];
    if (f & F_UP) {
        flags[id] = (uint8_t)((f & ~F_UP) | F_CRASHED);
        const uint32_t g = id >> CRASH_GRAIN_SHIFT;
        atomicOr(crash_bits + (g >> 5), 1u << (g & 31));
    }
}

// leave/1 calls of this round (pluggable): Hdr pad1[0] = target + 1 at
// each actor this shard owns
__global__ void k_leave_set(Hdr* hdr, uint32_t lo, uint32_t n_local, const uint32_t* actors,
                            const uint32_t* targets, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t id = actors[i];
    if (id >= lo && id < lo + n_local) hdr[id - lo].pad1[0] = targets[i] + 1;
}

__global__ void k_uncrash(uint8_t* flags, uint32_t* crash_bits, const uint32_t* ids, uint32_t n, const uint32_t* ctl) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || *ctl) return;
    flags[ids[i]] &= (uint8_t)~F_CRASHED;
    crash_bits[ids[i] >> (CRASH_GRAIN_SHIFT + 5)] = 0;   // (every bit of the word is this round's)
}

// node start: init/1 of the manager (hv:289-354) and of the broadcast
// server (pt:251-264, members = [own name]).  Every shard marks every
// joining node up in its replicated flag array; only the owner initialises
// the node's rows.
__global__ void k_join(RoundArgs a, uint32_t* start, const uint32_t* ids, const uint32_t* contacts,
                       uint32_t n, uint32_t persist_epoch) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t id = ids[i];
    a.flags[id] = (uint8_t)((a.flags[id] & F_CRASHED) | F_UP | (1u < a.min_active ? F_LOWACT : 0));
    if (id < a.lo || id >= a.lo + a.n_local) return;
    uint32_t li = id - a.lo;
    Hdr h;
    const uint32_t old_epoch = a.hdr[li].epoch;
    const uint32_t sx = a.pl ? 0u : a.hdr[li].pad1[1], rx = a.pl ? 0u : a.hdr[li].pad1[2];
    const uint32_t ox = a.pl ? 0u : a.hdr[li].pad1[3];
    memset(&h, 0, sizeof h);
    h.pad1[1] = sx; h.pad1[2] = rx; h.pad1[3] = ox;   // a restart keeps its extension rows (zeroed)
    h.epoch = persist_epoch ? old_epoch + 1 : 1;
    h.start_round = a.round;
    h.join_contact = contacts[i];
    h.aux = 0;
    h.trk_round = PSIM_NONE;
    h.act_n = 1; h.all_n = 1; h.com_n = 1;
    a.hdr[li] = h;
    start[li] = a.round;
    uint32_t* act = a.act + (size_t)li * PSIM_ACTIVE_CAP;
    for (int k = 0; k < PSIM_ACTIVE_CAP; k++) act[k] = k == 0 ? id : 0u;
    uint32_t* pas = a.pas + (size_t)li * PSIM_PASSIVE_CAP;
    for (int k = 0; k < PSIM_PASSIVE_CAP; k++) pas[k] = 0;
    for (uint32_t k = 0; k < IDMAP_IN; k++) {
        a.sentm[(size_t)li * IDMAP_IN + k] = 0;
        a.recvm[(size_t)li * IDMAP_IN + k] = 0;
    }
    for (uint32_t k = 0; k < IDMAP_EXT; k++) {
        if (sx) a.mapx[(size_t)(sx - 1) * IDMAP_EXT + k] = 0;
        if (rx) a.mapx[(size_t)(rx - 1) * IDMAP_EXT + k] = 0;
    }
    for (int k = 0; k < PSIM_PT_MEMBERS_CAP; k++) {
        a.pt_all[(size_t)li * PSIM_PT_MEMBERS_CAP + k] = k == 0 ? id : 0u;
        a.pt_com[(size_t)li * PSIM_PT_MEMBERS_CAP + k] = k == 0 ? id : 0u;
    }
    for (uint32_t k = 0; k < RT_SET; k++) {
        a.pt_eag[(size_t)li * RT_SET + k] = 0;
        a.pt_laz[(size_t)li * RT_SET + k] = 0;
    }
    for (uint32_t k = 0; k < RT_WORDS; k++) a.pt_rt[(size_t)li * RT_WORDS + k] = k < PSIM_PT_ROOTS ? PSIM_NONE : 0u;
    for (uint32_t k = 0; k < OUT_IN; k++) a.pt_out[(size_t)li * OUT_IN + k] = 0;
    if (a.conn)                    // a fresh incarnation has no connections
        for (uint32_t k = 0; k < PSIM_CONN_CAP; k++) a.conn[(size_t)li * PSIM_CONN_CAP + k] = 0;
    if (ox)
        for (uint32_t k = 0; k < OUT_EXT; k++) a.outx[(size_t)(ox - 1) * OUT_EXT + k] = 0;
    if (a.pl) {                    // the pluggable manager's init/1 (pl:346-402) + Strategy:init/1
        Hdr& x = a.hdr[li];
        x.aux = PSIM_NONE;         // last ping: undefined
        x.have = 0;                // hello not sent
        x.act_n = a.strategy == PSIM_STRATEGY_FULL ? 0 : 1;
        x.pas_n = 0; x.all_n = 0; x.com_n = 0;
        if (a.strategy == PSIM_STRATEGY_FULL) {
            a.fbits[(size_t)li * 2 * a.fw + (id >> 5)] |= 1u << (id & 31u);   // new_state/1 full:171-175
        } else {
            for (int k = 0; k < PSIM_SVIEW_CAP; k++) {
                a.sview[(size_t)li * PSIM_SVIEW_CAP + k] = k == 0 ? id : 0u;   // [Myself]
                if (a.sinv) a.sinv[(size_t)li * PSIM_SVIEW_CAP + k] = 0u;
            }
        }
    }
}

// this round's broadcasts retire the previous ids of their message slots:
// the slots' delivery bits are cleared at every node (mask lo | hi << 32)
__global__ void k_bcast_reset(Hdr* hdr, uint32_t n, uint32_t lo, uint32_t hi) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    hdr[i].have &= ~lo;
    hdr[i].aux &= ~hi;
    hdr[i].trk_round = PSIM_NONE;
    hdr[i].trk_hop = 0;
}

// the roots of this round's broadcasts that run (after the round's crash and
// start events, which precede this on the stream) originate them:
// origin[root - lo] = msg + 1; clear = true resets the same entries
__global__ void k_origin(uint32_t* origin, uint32_t lo, uint32_t n_local, const uint32_t* roots,
                         const uint32_t* msgs, uint32_t k, const uint8_t* flags, bool clear, const uint32_t* ctl) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k || *ctl) return;
    const uint32_t r = roots[i];
    if (r < lo || r >= lo + n_local) return;
    if (clear) origin[r - lo] = 0;
    else if (flags[r] & F_UP) origin[r - lo] = msgs[i] + 1;
}

// ------------------------------------------------------------- route --
// The route groups a round's records by local destination; each group ends
// up in emission order -- ascending source index (an outbox slot, or a
// position in the source-shard-ordered receive buffer), i.e. (src, seq)
// order.  Destinations are cut into buckets of W = 2^wshift consecutive
// nodes, and everything per destination happens in one block's LDS:
//   k_bucket_hist<>    a block takes fixed steps of source records and
//                      histograms their buckets in LDS -> hist[b * nblk + blk]
//   k_bucket_offsets   a block per bucket: the scan of its row of hist --
//                      where block blk's records go within bucket b -- and
//                      the bucket's total
//   k_bucket_scatter<> the scan of the totals (each block; block 0 stores
//                      the bucket bases), then the same steps again: each
//                      record's (destination in bucket | bound class, source
//                      index) pair to its place
//   k_bucket_route     one block per bucket: per destination the count, the
//                      bound sum and the BROADCAST id mask (LDS atomics; the
//                      returned count is the record's rank in its run), the
//                      run starts (block scan), each source index into its
//                      run, and every run of <= RUN_SHORT sorted in registers
//                      -- then, in the same block, the runs of RUN_SHORT + 1
//                      .. 64 (a wave each, bitonic over the lanes) and the
//                      longer ones (the whole block: bitonic in LDS up to
//                      RUN_LDS, LDS-sorted chunks merged through `tmp`
//                      beyond), and the bucket's records copied into the
//                      inbox in run order (the gather, 128 B a record)
// Run order before the sort depends on atomic timing; sorting each run by
// source index makes the inbox deterministic.
constexpr uint32_t RUN_SHORT = 16;
constexpr uint32_t RUN_LDS = 2048;
#ifndef PSIM_RB_STEP
#define PSIM_RB_STEP 1024
#endif
// source nodes (or dense records) per block step = the block: 1024 threads
// keep 16 waves per CU on the two passes' load chains at 2^26 nodes, where the
// 64 KB LDS histograms (16 K buckets) allow two blocks per CU (k_bucket_hist
// 2.20 -> 0.85 ms a round, profiles/r03/p16; no change at 2^20)
constexpr uint32_t RB_STEP = PSIM_RB_STEP;
constexpr uint32_t RB_WAVES = RB_STEP / 64;
constexpr uint32_t RB_MAX_BLOCKS = 1024;   // blocks of the two passes over the sources
// ... by default: one resident generation (two 1024-thread blocks a CU) --
// 1024 blocks were two generations of latency-bound steps at 2^20 (step
// 0.619 -> 0.615 ms, profiles/r05/ab_log.txt r6n)
constexpr uint32_t RB_BLOCKS = 512;
#ifndef PSIM_RR_THREADS
#define PSIM_RR_THREADS 1024
#endif
// k_bucket_route block: 1024 threads keep 16 waves per CU on its one block
// per bucket (512: route 36 -> 31 us a round at 2^20, profiles/r03 p26)
constexpr uint32_t RR_THREADS = PSIM_RR_THREADS;
#ifndef PSIM_RR_REG
#define PSIM_RR_REG 6
#endif
constexpr uint32_t RR_REG = PSIM_RR_REG;   // k_bucket_route: pairs a thread holds in registers
// bucket widths 2^11 .. 2^13 (route_group): k_bucket_route's LDS holds 4 W
// words -- counts, bound sums, and W 64-bit BROADCAST masks whose 2 W words
// then carry the block sort's RUN_LDS-word buffer and the long-run list (at
// most W destinations), so W >= RUN_LDS; its run-start scan gives each
// thread W / RR_THREADS counts
constexpr uint32_t WSHIFT_MIN = 11, WSHIFT_MAX = 13;
constexpr uint32_t ROUTE_LIDX = 8192;   // k_bucket_route: a bucket's source indices LDS holds (at W = 2^11)
static_assert((1u << WSHIFT_MIN) * 16 + ROUTE_LIDX * 4 + (PSIM_RR_THREADS + 4) * 4 <= 80 * 1024,
              "k_bucket_route at W = 2^11 with its indices in LDS: two blocks a CU");
static_assert((1u << WSHIFT_MIN) >= RUN_LDS, "k_bucket_route: the sort buffer and the long-run list share 2 W words");
static_assert((1u << WSHIFT_MIN) % RR_THREADS == 0, "k_bucket_route: W / RR_THREADS counts a thread");
static_assert((1u << WSHIFT_MAX) * 16 <= 160 * 1024, "k_bucket_route: 16 W bytes of LDS");

// The exchange's wire format (G > 1): a record's first 32 B -- dst, src, type
// word, seq, a0-a2 and word 7 -- is its head; a record with exchange ids
// (nex > 0 in its type word: SHUFFLE, SHUFFLE_REPLY, X-BOT's) also sends its
// last 32 B, the tail.  Every other record's last 32 B are zeros, so 32 B
// of the 64 cross xGMI.  A sender writes, per owner shard, the heads of its
// records in (src, seq) order, then the tails in the same order, and puts a
// long record's tail index (among that owner's tails) in the head's word 7
// -- zero in every record that crosses shards: the full strategy's payload
// slot lives there, and that strategy runs on one shard (psim_create).  The
// receiver's heads and tails arrive in source-shard order; k_bucket_hist adds
// the source's tail base to each long head's word 7, and k_bucket_route
// gathers head + tail (or zeros) into the 64-B inbox record, word 7 zeroed.
struct __attribute__((aligned(16))) Wire {
    uint4 q[2];
};
static_assert(sizeof(Wire) == 32, "a wire unit is half a record");
__host__ __device__ __forceinline__ bool wire_long(uint32_t tt) { return ((tt >> 16) & 0xFFu) != 0u; }

// the sources of one route: the outbox runs of this shard's nodes (G == 1),
// or the received heads and tails (G > 1)
struct RouteIn {
    const Msg* rec;
    const uint32_t* okey;      // runs: route key of every outbox slot
    const uint64_t* obase;     // runs: each source node's first slot
    const uint32_t* ocnt;      // runs: and its record count
    uint32_t n_src;            // runs: source nodes; dense: records
    uint32_t lo;               // first local node id
    uint32_t pl;               // dense: pluggable manager (bound class 0)
    Wire* wire;                // dense: the heads (word 7 of a long one fixed up by k_bucket_hist)
    const Wire* tails;         // dense: the tails
    const uint32_t* seg;       // dense: per source shard its first head, then its first tail (2 (nseg + 1))
    uint32_t nseg;
    // dense, a batched rank round (exchange_fixed): source g's message is
    // XHDR header slots (xhdr_*: its counts, abort flag, largest counts and
    // stats) then its heads, at [g (XHDR + capH), ..); its tails at
    // [g capT, ..); capH = 0: the packed layout above
    uint32_t capH, capT;
    uint32_t round;            // (the abort word's round, k_bucket_hist's header pass)
};

// The header of a batched rank round's message to one owner (XHDR wire
// slots, read as 64-bit words): the record counts (heads | tails << 32), the
// sender's abort flag, its largest per-owner head and tail counts, then its
// NST stats sums -- the round's count all-to-all and stats all-reduce ride
// with the records (one grouped send / receive a round)
enum { XH_CNT = 0, XH_ABORT = 1, XH_MH = 2, XH_MT = 3, XH_STATS = 4 };
constexpr uint32_t XHDR = (XH_STATS + NST + 3) / 4;

// the source shard of received head i (seg: nseg + 1 increasing starts)
__device__ __forceinline__ uint32_t wire_source(const RouteIn& in, uint32_t i) {
    uint32_t a = 0, b = in.nseg;
    while (b - a > 1) {
        const uint32_t m = (a + b) >> 1;
        if (in.seg[m] <= i) a = m; else b = m;
    }
    return a;
}

// Calls f(g, d, cls) for every record of block step `step`: source index g,
// local destination d, bound class cls.  The runs form has a wave expand 64
// consecutive source nodes' runs into consecutive record numbers (lane l
// takes records l, l + 64, ..., so okey is read in slot order); every thread
// of the block must call it.
template <bool DENSE, bool FIX = false, typename F>
__device__ __forceinline__ void route_step(const RouteIn& in, uint32_t step, uint32_t (*spre)[65],
                                           uint64_t (*sbase)[64], F f) {
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const uint32_t i = step * RB_STEP + threadIdx.x;
    if (DENSE) {
        uint32_t g = 0;
        bool ok = i < in.n_src;
        if (in.capH && ok) {                          // (the fixed layout: a header slot, or one past its
            const uint32_t xs = XHDR + in.capH;       //  source's count, holds no record)
            g = i / xs;
            const uint32_t j = i - g * xs;
            const uint32_t c = (uint32_t)reinterpret_cast<const uint64_t*>(in.wire + (size_t)g * xs)[XH_CNT];
            ok = j >= XHDR && j - XHDR < min(c, in.capH);
        }
        if (ok) {
            const uint4 h0 = in.wire[i].q[0];        // dst, src, type word, seq
            // (FIX, k_bucket_hist: a long head's tail index becomes the
            // index among every received tail -- in the fixed layout kept
            // inside its source's region: a sender past its tail capacity
            // aborted the round, exchange_fixed)
            if (FIX && wire_long(h0.z)) {
                if (in.capH) in.wire[i].q[1].w = min(in.wire[i].q[1].w, in.capT - 1) + g * in.capT;
                else in.wire[i].q[1].w += in.seg[in.nseg + 1 + wire_source(in, i)];
            }
            f(i, h0.x - in.lo, in.pl ? 0u : max_emit(h0.z & 0xFF));
        }
        return;
    }
    const uint32_t c = i < in.n_src ? in.ocnt[i] : 0u;
    uint32_t inc = c;                                 // inclusive prefix over the wave
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o);
        if (l >= (uint32_t)o) inc += y;
    }
    __syncthreads();                                  // the previous step's readers are done
    spre[w][l + 1] = inc;
    if (l == 0) spre[w][0] = 0;
    sbase[w][l] = i < in.n_src ? in.obase[i] : 0ull;
    const uint32_t T = __shfl(inc, 63);
    __syncthreads();
    const uint32_t* pre = spre[w];
    for (uint32_t t = l; t < T; t += 64) {
        uint32_t a = 0, b = 64;                       // the node j with pre[j] <= t < pre[j + 1]
        while (b - a > 1) {
            const uint32_t mid = (a + b) >> 1;
            if (pre[mid] <= t) a = mid; else b = mid;
        }
        const uint64_t g = sbase[w][a] + (t - pre[a]);
        const uint32_t key = in.okey[g];
        f((uint32_t)g, (key & KEY_DST_MASK) - in.lo, key >> KEY_DST_BITS);
    }
}

// The round's stats: every kernel block left a row of NST partial sums,
// summed inside the route (no launches of their own: two small kernels cost
// ~12 us a round in launch and drain): block t < nt of k_bucket_hist sums a
// contiguous range of rows, one lane per column (coalesced rows), into tile
// row t; block 0 of k_bucket_scatter sums the tile rows.  The sums (and the
// node-round span, out[NST..NST+1]) are also stored straight into the
// shard's pinned host words, so the host reads them after its end-of-round
// wait without a copy.
constexpr uint32_t STAT_TILES = 256;
struct StatsIn {
    const uint64_t* part;      // nrows rows of NST partial sums
    uint32_t nrows, nt;        // nt tiles (<= STAT_TILES, <= the hist grid)
    uint64_t* tiles;
    uint64_t* out;             // the shard's stat_out (NST sums, then the span)
    uint64_t* hout;            // its pinned words
    const uint32_t* outx_top;  // the outstanding pool's rows taken (-> pinned slot 0, PIN_OUTX; may be null)
    uint64_t* hout0;           // pinned slot 0
};
// (red: the block's [waves][64] words of LDS; every thread calls these)
__device__ __forceinline__ void stats_tile(const StatsIn& st, uint32_t t, uint64_t (*red)[64]) {
    const uint32_t c = threadIdx.x & 63, g = threadIdx.x >> 6, ng = blockDim.x >> 6;
    const uint32_t per = (st.nrows + st.nt - 1) / st.nt;
    const uint32_t r0 = t * per, r1 = min(st.nrows, r0 + per);
    uint64_t v = 0;
    if (c < NST) {
#pragma unroll 4
        for (uint32_t r = r0 + g; r < r1; r += ng) v += st.part[(size_t)r * NST + c];
    }
    __syncthreads();                                  // (red's previous readers are done)
    red[g][c] = v;
    __syncthreads();
    if (g == 0 && c < NST) {
        uint64_t u = 0;
        for (uint32_t k = 0; k < ng; k++) u += red[k][c];
        st.tiles[(size_t)t * NST + c] = u;
    }
    __syncthreads();
}
__device__ __forceinline__ void stats_final(const StatsIn& st, uint64_t (*red)[64]) {
    const uint32_t c = threadIdx.x & 63, g = threadIdx.x >> 6, ng = blockDim.x >> 6;
    uint64_t v = 0;
    if (c < NST) {
#pragma unroll 4
        for (uint32_t b = g; b < st.nt; b += ng) v += st.tiles[(size_t)b * NST + c];
    }
    __syncthreads();
    red[g][c] = v;
    __syncthreads();
    if (g == 0 && c < NST) {
        uint64_t u = 0;
        for (uint32_t k = 0; k < ng; k++) u += red[k][c];
        st.out[c] = u;
        st.hout[c] = u;
    }
    if (threadIdx.x == 0) {
        st.hout[NST] = st.out[NST];
        st.hout[NST + 1] = st.out[NST + 1];
        if (st.outx_top) st.hout0[PIN_OUTX] = *st.outx_top;
    }
    __syncthreads();
}

// a batched rank round's received headers (block 0 of k_bucket_hist, the
// first kernel after the exchange, whatever the abort word says): the
// sources' stats summed into the round's pinned words, the ranks' abort flags
// (PIN_XAB) and largest counts (PIN_XRANK); a round any rank aborted stops
// this rank's later kernels too (code 4)
__device__ __forceinline__ void xhdr_reduce(const RouteIn& in, const StatsIn& st, uint32_t* ctl) {
    const uint32_t c = threadIdx.x, xs = XHDR + in.capH;
    auto hw = [&](uint32_t g, uint32_t k) { return reinterpret_cast<const uint64_t*>(in.wire + (size_t)g * xs)[k]; };
    if (c < NST) {
        uint64_t v = 0;
        for (uint32_t g = 0; g < in.nseg; g++) v += hw(g, XH_STATS + c);
        st.hout[c] = v;
    } else if (c >= 64 && c < 64 + in.nseg) {
        st.hout[PIN_XRANK + (c - 64)] = hw(c - 64, XH_MH);
        st.hout[PIN_XRANK + 64 + (c - 64)] = hw(c - 64, XH_MT);
    } else if (c == 256) {
        uint64_t ab = 0;
        for (uint32_t g = 0; g < in.nseg; g++) ab += hw(g, XH_ABORT);
        st.hout[PIN_XAB] = ab;
        if (ab && !ctl[0]) { ctl[1] = in.round; __threadfence(); ctl[0] = 4; }
    }
}

template <bool DENSE>
__global__ void __launch_bounds__(RB_STEP) k_bucket_hist(RouteIn in, uint32_t nsteps, uint32_t nb,
                                                         uint32_t wshift, uint32_t* hist, uint32_t* ctl,
                                                         unsigned long long* mark, StatsIn st) {
    __shared__ uint32_t s_dead;
    if (DENSE && in.capH && blockIdx.x == 0) xhdr_reduce(in, st, ctl);
    // (read once a block: block 0 above may be writing it)
    if (threadIdx.x == 0) s_dead = *ctl;
    __syncthreads();
    if (s_dead) return;                               // an aborted batch (run_batch)
    if (mark && blockIdx.x == 0 && threadIdx.x == 0) *mark = __builtin_amdgcn_s_memrealtime();   // (phase end)
    extern __shared__ uint32_t hcnt[];                // nb bucket counters
    __shared__ uint32_t spre[RB_WAVES][65];
    __shared__ uint64_t sbase[RB_WAVES][64];
    if (blockIdx.x < st.nt) stats_tile(st, blockIdx.x, sbase);   // (uniform; nt = 0: the headers')
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) hcnt[j] = 0;
    __syncthreads();
    for (uint32_t step = blockIdx.x; step < nsteps; step += gridDim.x)
        route_step<DENSE, DENSE>(in, step, spre, sbase,
                                 [&](uint32_t, uint32_t d, uint32_t) { atomicAdd(&hcnt[d >> wshift], 1u); });
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) hist[(size_t)j * gridDim.x + blockIdx.x] = hcnt[j];
}

template <typename T, uint32_t NT = BLK>
__device__ T block_excl(T v, T* total);   // (the exclusive-scan section below)

// Block b: row b of hist (nblk <= RB_MAX_BLOCKS counts, one a thread) scanned
// into hoff, the row's sum into tot[b].  One launch where a scan over the
// whole matrix took three (k_scan_tiles / _sums / _apply, ~15 us a round at
// 2^20 nodes, mostly launch and drain)
__global__ void __launch_bounds__(RB_MAX_BLOCKS) k_bucket_offsets(const uint32_t* __restrict__ hist, uint32_t nblk,
                                                                 uint32_t* __restrict__ hoff,
                                                                 uint32_t* __restrict__ tot, const uint32_t* ctl) {
    if (*ctl) return;                                 // an aborted batch (run_batch)
    const size_t r = (size_t)blockIdx.x * nblk;
    const uint32_t v = threadIdx.x < nblk ? hist[r + threadIdx.x] : 0u;
    uint32_t t;
    const uint32_t e = block_excl<uint32_t, RB_MAX_BLOCKS>(v, &t);
    if (threadIdx.x < nblk) hoff[r + threadIdx.x] = e;
    if (threadIdx.x == 0) tot[blockIdx.x] = t;
}

template <bool DENSE>
__global__ void __launch_bounds__(RB_STEP) k_bucket_scatter(RouteIn in, uint32_t nsteps, uint32_t nb,
                                                            uint32_t wshift, const uint32_t* __restrict__ off,
                                                            const uint32_t* __restrict__ tot, uint32_t* base,
                                                            uint2* pairs, uint64_t cap, uint64_t* hovf,
                                                            uint32_t* ctl, uint32_t round1, StatsIn st) {
    if (*ctl) return;                                 // an aborted batch (run_batch)
    extern __shared__ uint32_t hcnt[];                // nb rank counters
    __shared__ uint32_t spre[RB_WAVES][65];
    __shared__ uint64_t sbase[RB_WAVES][64];
    if (blockIdx.x == 0 && st.nt) stats_final(st, sbase);   // (the tiles are k_bucket_hist's; before any return)
    // the buckets' bases: the totals through LDS (coalesced), a run of them a
    // thread, one block scan of the run sums
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) hcnt[j] = tot[j];
    __syncthreads();
    const uint32_t per = (nb + RB_STEP - 1) / RB_STEP, j0 = min(nb, threadIdx.x * per), j1 = min(nb, j0 + per);
    uint32_t v = 0;
    for (uint32_t j = j0; j < j1; j++) v += hcnt[j];
    uint32_t m;                                       // the record count
    uint32_t run = block_excl<uint32_t, RB_STEP>(v, &m);
    if (blockIdx.x == 0 && threadIdx.x == 0) base[nb] = m;   // (k_bucket_route's overflow test too)
    if (m > cap) {                                    // the route buffers are too small:
        if (blockIdx.x == 0 && threadIdx.x == 0) {    // the host grows them and reruns
            *hovf = m;
            // (a batch: this round's route and every later kernel of the
            // batch stand still -- round round1 - 1, code 2)
            if (round1) { ctl[1] = round1 - 1; __threadfence(); ctl[0] = 2; }
        }
        return;
    }
    for (uint32_t j = j0; j < j1; j++) {
        const uint32_t x = hcnt[j];
        hcnt[j] = run;
        run += x;
    }
    __syncthreads();
    // each bucket's counter starts at this block's place in it: the returned
    // count is the pair's position (no per-record read of the offset matrix)
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) {
        const uint32_t b0 = hcnt[j];
        if (blockIdx.x == 0) base[j] = b0;
        hcnt[j] = b0 + off[(size_t)j * gridDim.x + blockIdx.x];
    }
    __syncthreads();
    const uint32_t wmask = (1u << wshift) - 1;
    for (uint32_t step = blockIdx.x; step < nsteps; step += gridDim.x)
        route_step<DENSE>(in, step, spre, sbase, [&](uint32_t g, uint32_t d, uint32_t cls) {
            pairs[atomicAdd(&hcnt[d >> wshift], 1u)] = make_uint2((d & wmask) | (cls << 16), g);
        });
}

// The fused route pass of one shard's own outbox (G == 1; route_group
// `fused`): k_bucket_hist, k_bucket_offsets and k_bucket_scatter in one
// launch.  Each block counts its records per bucket in LDS, reserves its
// share of every bucket it touches with one global atomic per bucket
// (gcnt, zeroed by k_node_prep), and scatters its pairs into the bucket's
// fixed region [b capb, (b + 1) capb) of `pairs`.  The order of a bucket's
// pairs then depends on the atomics' timing -- which k_bucket_route never
// relied on: it ranks each destination's records by LDS atomics and sorts
// every run by source index.  A bucket past capb (a join storm on a few
// destinations) stops the fused route: k_bucket_route returns, the round's
// records are routed again by the four-pass route (flag in ctl[2]).
#ifndef PSIM_FILL_REG
#define PSIM_FILL_REG 8
#endif
constexpr uint32_t FILL_REG = PSIM_FILL_REG;   // k_bucket_fill: records a thread keeps between its passes
template <bool DENSE>
__global__ void __launch_bounds__(RB_STEP) k_bucket_fill(RouteIn in, uint32_t nsteps, uint32_t nb, uint32_t wshift,
                                                         uint32_t* gcnt, uint32_t capb, uint2* pairs, uint32_t* ctl,
                                                         unsigned long long* mark, StatsIn st, uint32_t walk) {
    if (*ctl) return;                                 // an aborted batch (run_batch)
    if (mark && blockIdx.x == 0 && threadIdx.x == 0) *mark = __builtin_amdgcn_s_memrealtime();   // (phase end)
    extern __shared__ uint32_t hcnt[];                // nb bucket counters, then this block's bases
    __shared__ uint32_t spre[RB_WAVES][65];
    __shared__ uint64_t sbase[RB_WAVES][64];
    __shared__ uint32_t s_spill;
    if (blockIdx.x < st.nt) stats_tile(st, blockIdx.x, sbase);   // (uniform)
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) hcnt[j] = 0;
    if (threadIdx.x == 0) s_spill = walk;             // (walk: the second pass walks the runs, A/B)
    __syncthreads();
    // the first FILL_REG records a thread meets are kept in registers
    // (destination | class << 27, source index), so the scatter below need not
    // walk the outbox runs a second time; a block where some thread met more
    // walks them again
    uint32_t rk[FILL_REG], rg[FILL_REG], nr = 0;
    for (uint32_t step = blockIdx.x; step < nsteps; step += gridDim.x)
        route_step<DENSE>(in, step, spre, sbase, [&](uint32_t g, uint32_t d, uint32_t cls) {
            atomicAdd(&hcnt[d >> wshift], 1u);
#pragma unroll
            for (uint32_t k = 0; k < FILL_REG; k++)
                if (k == nr) { rk[k] = d | (cls << KEY_DST_BITS); rg[k] = g; }
            nr++;
        });
    if (nr > FILL_REG) s_spill = 1;
    __syncthreads();
    const bool spill = s_spill != 0;                  // (uniform)
    bool over = false;
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) {
        const uint32_t c = hcnt[j];
        const uint32_t b0 = c ? atomicAdd(&gcnt[j], c) : 0u;
        over |= b0 + c > capb;
        hcnt[j] = j * capb + b0;
    }
    if (over) ctl[2] = 1;                             // (read by k_bucket_route, a later launch)
    __syncthreads();
    const uint32_t wmask = (1u << wshift) - 1;
    auto put = [&](uint32_t g, uint32_t d, uint32_t cls) {
        const uint32_t j = d >> wshift, q = atomicAdd(&hcnt[j], 1u);
        if (q < (j + 1) * capb) pairs[q] = make_uint2((d & wmask) | (cls << 16), g);
    };
    if (!spill) {
#pragma unroll
        for (uint32_t k = 0; k < FILL_REG; k++)
            if (k < nr) put(rg[k], rk[k] & KEY_DST_MASK, rk[k] >> KEY_DST_BITS);
    } else {
        for (uint32_t step = blockIdx.x; step < nsteps; step += gridDim.x) route_step<DENSE>(in, step, spre, sbase, put);
    }
}

// G > 1, sender side: this shard's outbox runs stably partitioned by owner
// shard (owner = dst / per) straight into the send buffer in the wire format
// (Wire: the heads of every owner, then the tails of every owner), so each
// owner's records stay in (src, seq) order -- the receiver's route relies on
// it.  Two passes; block blk takes the consecutive block steps [blk * spb,
// (blk + 1) * spb), so block order is source order (a grid-stride step
// assignment would put a block's later steps before the next block's
// earlier ones and break the (src, seq) order once a block runs two steps):
//   WRITE = false  per block and owner the record count -> hist[q * nblk +
//                  blk] and the long records' count -> hist[(G + q) * nblk +
//                  blk] (hist[2 G nblk] = 0: the scan's extra entry, the total)
//   WRITE = true   after the scan, each record's head to off[q * nblk + blk]
//                  + its rank among the block's records of owner q, a long
//                  record's tail to off[(G + q) * nblk + blk] + its rank among
//                  the block's long records of owner q, and that tail's index
//                  among owner q's tails into the head's word 7
// A wave walks its 64 nodes' records in slot order, 64 at a time; the rank
// within a batch is a ballot over the lanes of the same owner, one ballot
// per distinct owner in the batch (<= G).
// A batched rank round (capH > 0, exchange_fixed) writes the fixed layout
// instead: owner q's message -- XHDR header slots (k_owner_offsets), then its
// heads -- at [q (XHDR + capH), (q + 1) (XHDR + capH)), its tails at
// G (XHDR + capH) + [q capT, (q + 1) capT); a record past its owner's
// capacity is not written (k_owner_offsets aborts the round, code 3).  The
// count pass's first blocks also sum the round's stats rows into tiles
// (st.nt > 0: the stats travel in the headers instead of an all-reduce).
template <bool WRITE>
__global__ void __launch_bounds__(RB_STEP) k_owner_part(RouteIn in, uint32_t nsteps, uint32_t spb, uint32_t G,
                                                        uint32_t per, uint32_t* hist,
                                                        const uint32_t* __restrict__ off, Wire* __restrict__ out,
                                                        unsigned long long* mark, uint32_t capH, uint32_t capT,
                                                        const uint32_t* ctl, StatsIn st) {
    if (*ctl) return;                                 // an aborted batch (run_batch_ranked)
    if (mark && blockIdx.x == 0 && threadIdx.x == 0) *mark = __builtin_amdgcn_s_memrealtime();   // (phase end)
    __shared__ uint32_t spre[RB_WAVES][65];
    __shared__ uint64_t sbase[RB_WAVES][64];
    if (!WRITE && blockIdx.x < st.nt) stats_tile(st, blockIdx.x, sbase);   // (uniform)
    __shared__ uint32_t wc[RB_WAVES][64], wl[RB_WAVES][64];   // per wave and owner: records / long ones this step
    __shared__ uint32_t run[64], runl[64];            // per owner: the block's next head / tail position
    __shared__ uint32_t tb[64];                       // per owner: its first tail (WRITE)
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63, nblk = gridDim.x;
    if (threadIdx.x < 64) {
        const uint32_t o = threadIdx.x;
        const bool q = WRITE && o < G;
        if (capH) {                                   // (each owner's region starts at its fixed base)
            const uint32_t xs = XHDR + capH;
            run[o] = q ? o * xs + XHDR + off[o * nblk + blockIdx.x] - off[o * nblk] : 0u;
            runl[o] = q ? G * xs + o * capT + off[(G + o) * nblk + blockIdx.x] - off[(G + o) * nblk] : 0u;
            tb[o] = q ? G * xs + o * capT : 0u;
        } else {
            run[o] = q ? off[o * nblk + blockIdx.x] : 0u;
            runl[o] = q ? off[(G + o) * nblk + blockIdx.x] : 0u;
            tb[o] = q ? off[(G + o) * nblk] : 0u;
        }
    }
    if (!WRITE && blockIdx.x == 0 && threadIdx.x == 0) hist[2 * G * nblk] = 0;
    const uint32_t s_end = min(nsteps, (blockIdx.x + 1) * spb);
    for (uint32_t step = blockIdx.x * spb; step < s_end; step++) {
        const uint32_t i = step * RB_STEP + threadIdx.x;
        const uint32_t c = i < in.n_src ? in.ocnt[i] : 0u;
        uint32_t inc = c;                             // inclusive prefix over the wave
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o);
            if (l >= (uint32_t)o) inc += y;
        }
        __syncthreads();                              // the previous step's readers are done
        spre[w][l + 1] = inc;
        if (l == 0) spre[w][0] = 0;
        sbase[w][l] = i < in.n_src ? in.obase[i] : 0ull;
        const uint32_t T = __shfl(inc, 63);
        __syncthreads();
        const uint32_t* pre = spre[w];
        // record t of the wave: its outbox slot and owner (none past T)
        auto rec_at = [&](uint32_t t, uint64_t& g) -> uint32_t {
            if (t >= T) return 0xFFFFFFFFu;
            uint32_t a = 0, b = 64;
            while (b - a > 1) {
                const uint32_t mid = (a + b) >> 1;
                if (pre[mid] <= t) a = mid; else b = mid;
            }
            g = sbase[w][a] + (t - pre[a]);
            return (in.okey[g] & KEY_DST_MASK) / per;
        };
        uint32_t cnt = 0, cntl = 0;                   // lane q: this wave's records / long records of owner q
        for (uint32_t t0 = 0; t0 < T; t0 += 64) {
            uint64_t g = 0;
            const uint32_t o = rec_at(t0 + l, g);
            const bool lg = o != 0xFFFFFFFFu && wire_long(in.rec[g].tt);
            for (uint64_t todo = __ballot(o != 0xFFFFFFFFu); todo;) {
                const uint32_t q = __builtin_amdgcn_readlane(o, __ffsll((long long)todo) - 1);
                const uint64_t m = __ballot(o == q), ml = __ballot(o == q && lg);
                cnt += l == q ? (uint32_t)__popcll(m) : 0u;
                cntl += l == q ? (uint32_t)__popcll(ml) : 0u;
                todo &= ~m;
            }
        }
        wc[w][l] = cnt;
        wl[w][l] = cntl;
        __syncthreads();
        if (WRITE) {
            uint32_t B = 0, BL = 0;                   // lane q: where this wave's next owner-q head / tail goes
            if (l < G) {
                B = run[l];
                BL = runl[l];
                for (uint32_t v = 0; v < w; v++) { B += wc[v][l]; BL += wl[v][l]; }
            }
            for (uint32_t t0 = 0; t0 < T; t0 += 64) {
                uint64_t g = 0;
                const uint32_t o = rec_at(t0 + l, g);
                uint4 x0 = make_uint4(0, 0, 0, 0), x1 = x0, x2 = x0, x3 = x0;
                if (o != 0xFFFFFFFFu) {
                    const uint4* sp = reinterpret_cast<const uint4*>(&in.rec[g]);
                    x0 = sp[0]; x1 = sp[1]; x2 = sp[2]; x3 = sp[3];
                }
                const bool lg = o != 0xFFFFFFFFu && wire_long(x0.z);
                uint32_t pos = 0, lpos = 0;
                for (uint64_t todo = __ballot(o != 0xFFFFFFFFu); todo;) {
                    const uint32_t q = __builtin_amdgcn_readlane(o, __ffsll((long long)todo) - 1);
                    const uint64_t m = __ballot(o == q), ml = __ballot(o == q && lg);
                    const uint64_t below = (1ull << l) - 1ull;
                    if (o == q) {
                        pos = __builtin_amdgcn_readlane(B, q) + (uint32_t)__popcll(m & below);
                        lpos = __builtin_amdgcn_readlane(BL, q) + (uint32_t)__popcll(ml & below);
                    }
                    B += l == q ? (uint32_t)__popcll(m) : 0u;
                    BL += l == q ? (uint32_t)__popcll(ml) : 0u;
                    todo &= ~m;
                }
                if (o != 0xFFFFFFFFu) {
                    if (lg) {
                        x1.w = lpos - tb[o];          // the tail's index among owner o's tails
                        if (!capH || x1.w < capT) {
                            out[lpos].q[0] = x2;
                            out[lpos].q[1] = x3;
                        }
                    }
                    if (!capH || pos < (o + 1) * (XHDR + capH)) {
                        out[pos].q[0] = x0;
                        out[pos].q[1] = x1;
                    }
                }
            }
        }
        __syncthreads();
        if (threadIdx.x < G)
            for (uint32_t v = 0; v < RB_WAVES; v++) { run[threadIdx.x] += wc[v][threadIdx.x]; runl[threadIdx.x] += wl[v][threadIdx.x]; }
    }
    if (!WRITE) {
        __syncthreads();
        if (threadIdx.x < G) {
            hist[threadIdx.x * nblk + blockIdx.x] = run[threadIdx.x];
            hist[(G + threadIdx.x) * nblk + blockIdx.x] = runl[threadIdx.x];
        }
    }
}

// each owner's first head and first tail in the send buffer (2 G + 1
// entries: heads of owners 0.., tails of owners 0.., the total) and, on RCCL
// ranks, each owner's record count | its long records' count << 32 straight
// into the send half of the count all-to-all (so the round reads both back
// at once)
// Also, for the rank path: the largest per-owner head and tail counts into
// the x-words (xw[1], xw[2]: all-reduced with the round's stats, they size
// the next batch's fixed exchange), and in a batched round (capH > 0) an
// owner past its capacity aborts the round (code 3, ctl[1] = round).  An
// aborted round sends counts of 0 (its send buffer was not written).
// (xw[3 + r] / xw[3 + 64 + r]: rank r's largest head / tail count, every
// other rank's word 0: the all-reduce sum keeps each rank's own)
constexpr uint32_t OO_THREADS = 1024;   // k_owner_offsets' block
// A batched round (capH > 0) writes each owner's message header instead:
// the counts, this rank's abort flag and largest counts, and the round's
// stats summed from the count pass's tiles; and the round's span, its own
// send counts (PIN_XCNT) and the outstanding pool's top into the pinned words
__global__ void k_owner_offsets(const uint32_t* hoff, uint32_t nblk, uint32_t G, uint64_t* d_off, uint64_t* cnt,
                                uint64_t* xw, uint32_t capH, uint32_t capT, uint32_t* ctl, uint32_t round,
                                uint32_t rank, Wire* sendbuf, StatsIn st) {
    __shared__ uint32_t smh, smt;
    __shared__ uint64_t ssum[64];
    __shared__ uint64_t sred[OO_THREADS / 64][64];
    const uint32_t q = threadIdx.x;
    const bool dead = *ctl != 0;
    if (capH) {
        const uint32_t xs = XHDR + capH;
        uint32_t mh = 0, mt = 0;
        for (uint32_t o = 0; o < G && !dead; o++) {
            mh = max(mh, hoff[(o + 1) * nblk] - hoff[o * nblk]);
            mt = max(mt, hoff[(G + o + 1) * nblk] - hoff[(G + o) * nblk]);
        }
        const bool over = !dead && (mh > capH || mt > capT);
        {                                             // the stats tiles' sums: 16 tiles a thread at most
            const uint32_t c = q & 63, g = q >> 6, ng = OO_THREADS / 64;
            uint64_t v = 0;
            if (c < NST) {
#pragma unroll 4
                for (uint32_t b = g; b < st.nt; b += ng) v += st.tiles[(size_t)b * NST + c];
            }
            sred[g][c] = v;
            __syncthreads();
            if (g == 0) {
                uint64_t u = 0;
                for (uint32_t k = 0; k < ng; k++) u += sred[k][c];
                ssum[c] = u;
            }
        }
        __syncthreads();
        for (uint32_t o = 0; o < G; o++) {
            uint64_t* hw = reinterpret_cast<uint64_t*>(sendbuf + (size_t)o * xs);
            const uint64_t c = dead ? 0ull
                                    : (uint64_t)(hoff[(o + 1) * nblk] - hoff[o * nblk]) |
                                          ((uint64_t)(hoff[(G + o + 1) * nblk] - hoff[(G + o) * nblk]) << 32);
            if (q == 0) { hw[XH_CNT] = c; hw[XH_ABORT] = dead || over ? 1u : 0u; hw[XH_MH] = mh; hw[XH_MT] = mt; }
            if (q < NST) hw[XH_STATS + q] = ssum[q];
            if (q == 1) st.hout[PIN_XCNT + o] = c;
        }
        if (q == 0) {
            st.hout[NST] = st.out[NST];               // (the node-round span)
            st.hout[NST + 1] = st.out[NST + 1];
            if (st.outx_top) st.hout0[PIN_OUTX] = *st.outx_top;
            if (over) { ctl[1] = round; __threadfence(); ctl[0] = 3; }
        }
        return;
    }
    if (q <= 2 * G) d_off[q] = hoff[q * nblk];
    if (cnt && q < G)
        cnt[q] = dead ? 0ull
                      : (uint64_t)(hoff[(q + 1) * nblk] - hoff[q * nblk]) |
                            ((uint64_t)(hoff[(G + q + 1) * nblk] - hoff[(G + q) * nblk]) << 32);
    if (!xw) return;                                  // (uniform)
    if (q == 0) {
        uint32_t mh = 0, mt = 0;
        for (uint32_t o = 0; o < G && !dead; o++) {
            mh = max(mh, hoff[(o + 1) * nblk] - hoff[o * nblk]);
            mt = max(mt, hoff[(G + o + 1) * nblk] - hoff[(G + o) * nblk]);
        }
        xw[1] = mh;
        xw[2] = mt;
        smh = mh; smt = mt;
        if (capH && !dead && (mh > capH || mt > capT)) { ctl[1] = round; __threadfence(); ctl[0] = 3; }
    }
    __syncthreads();
    if (q < 128) xw[3 + q] = q == rank ? smh : q == 64 + rank ? smt : 0u;
}




// bitonic sort of p[0..k) (k <= RUN_LDS) through LDS, whole block
__device__ __forceinline__ void block_sort_lds(uint32_t* sv, uint32_t* p, uint32_t k) {
    uint32_t P = 1;
    while (P < k) P <<= 1;
    for (uint32_t t = threadIdx.x; t < P; t += blockDim.x) sv[t] = t < k ? p[t] : 0xFFFFFFFFu;
    __syncthreads();
    for (uint32_t kk = 2; kk <= P; kk <<= 1) {
        for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
            for (uint32_t t = threadIdx.x; t < P; t += blockDim.x) {
                const uint32_t u = t ^ jj;
                if (u > t) {
                    const uint32_t a = sv[t], b = sv[u];
                    if ((a > b) == ((t & kk) == 0)) { sv[t] = b; sv[u] = a; }
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t t = threadIdx.x; t < k; t += blockDim.x) p[t] = sv[t];
    __syncthreads();
}

// a run longer than 64, whole block: RUN_LDS chunks sorted in LDS, then
// merged pairwise through y (the run's own range of the scratch)
__device__ __forceinline__ void sort_run_block(uint32_t* p, uint32_t k, uint32_t* y, uint32_t* sv) {
    for (uint32_t c0 = 0; c0 < k; c0 += RUN_LDS) block_sort_lds(sv, p + c0, min(RUN_LDS, k - c0));
    uint32_t* x = p;
    for (uint32_t wd = RUN_LDS; wd < k; wd *= 2) {
        for (uint32_t a0 = threadIdx.x * 2 * wd; a0 < k; a0 += blockDim.x * 2 * wd) {
            const uint32_t m0 = min(a0 + wd, k), e0 = min(a0 + 2 * wd, k);
            uint32_t u = a0, v = m0, o = a0;
            while (u < m0 && v < e0) y[o++] = x[u] <= x[v] ? x[u++] : x[v++];
            while (u < m0) y[o++] = x[u++];
            while (v < e0) y[o++] = x[v++];
        }
        __syncthreads();
        uint32_t* z = x; x = y; y = z;
    }
    if (x != p)
        for (uint32_t t = threadIdx.x; t < k; t += blockDim.x) p[t] = x[t];
    __syncthreads();
}

// p[0..k), RUN_SHORT < k <= 64, sorted by one wave: a bitonic network over
// the lanes (lane l holds element l; the missing ones sort last)
__device__ __forceinline__ void wave_sort64(uint32_t* p, uint32_t k) {
    const uint32_t l = threadIdx.x & 63;
    uint32_t v = l < k ? p[l] : 0xFFFFFFFFu;
#pragma unroll
    for (uint32_t kk = 2; kk <= 64; kk <<= 1) {
#pragma unroll
        for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
            const uint32_t u = (uint32_t)__shfl_xor((int)v, (int)j);
            const bool keep_min = ((l & j) == 0) == ((l & kk) == 0);
            v = keep_min ? min(v, u) : max(v, u);
        }
    }
    if (l < k) p[l] = v;
}

// 16-B piece p of received record k rebuilt from the wire: the head's two
// pieces (word 7, the tail index, back to 0 on a long record), then the
// tail's -- or zeros
__device__ __forceinline__ uint4 wire_piece(const Wire* __restrict__ heads, const Wire* __restrict__ tails,
                                            uint32_t k, uint32_t p) {
    if (p == 0) return heads[k].q[0];
    const uint32_t tt = heads[k].q[0].z;
    const uint4 h1 = heads[k].q[1];
    const bool lng = wire_long(tt);
    if (p == 1) return make_uint4(h1.x, h1.y, h1.z, lng ? 0u : h1.w);
    return lng ? tails[h1.w].q[p - 2] : make_uint4(0, 0, 0, 0);
}

// 16-B piece p of outbox record k for the inbox, p = the lane's index in its
// quad (the quad's lanes take one record's four pieces): a short record's
// tail (nex == 0: its emitter may leave it unwritten, PSIM_SHORT_TAIL) as
// zeros -- the type word from the quad's first lane (DPP quad_perm 0,0,0,0)
__device__ __forceinline__ uint4 rec_piece(const Msg* __restrict__ rec, uint32_t k, uint32_t p) {
    const uint4 v = reinterpret_cast<const uint4*>(&rec[k])[p];
    if (!PSIM_SHORT_TAIL) return v;
    const uint32_t tt = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.z, 0x00, 0xF, 0xF, false);
    return p < 2 || wire_long(tt) ? v : make_uint4(0, 0, 0, 0);
}

// One block per bucket of W destinations; LDS holds per destination the
// count, the bound sum (later the run start, in the same words) and the
// BROADCAST message-slot mask (64 bits): 4 x W words.
template <bool WIRE>
__global__ void __launch_bounds__(RR_THREADS) k_bucket_route(
    uint32_t n, uint32_t wshift, uint32_t regcap, const uint32_t* __restrict__ base,
    const uint2* __restrict__ pairs, const Msg* __restrict__ rec, const Wire* __restrict__ heads,
    const Wire* __restrict__ tails, uint32_t* rank, unsigned long long* cb,
    unsigned long long* bmask, uint32_t* in_beg, uint32_t* idx, uint32_t* tmp, Msg* __restrict__ inbox, uint64_t* hm,
    uint64_t cap, uint32_t* ctl, const uint32_t* gcnt, uint32_t capb, uint32_t round1, StatsIn st, uint32_t lcap) {
    if (*ctl) return;                                 // an aborted batch (run_batch)
    // (the dynamic words hold 64-bit masks: 8-byte aligned -- a 4-byte static
    // word in front of them misaligned ds_or_b64 and faulted; the long-run
    // count lives in spart's spare words instead)
    extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
    __shared__ __attribute__((aligned(16))) uint32_t spart[RR_THREADS + 4];
    uint32_t& s_nl = spart[RR_THREADS];
    const uint32_t W = 1u << wshift, wmask = W - 1, b = blockIdx.x;
    uint32_t* cnt = sm;
    uint32_t* bs = sm + W;
    unsigned long long* mk = reinterpret_cast<unsigned long long*>(sm + 2 * W);
    uint32_t* pre = bs;                               // (after the bound sums are written out)
    // the bucket's records: [s0, s1) of the inbox, from its pairs at q0 ..
    uint32_t s0, s1, q0;
    if (gcnt) {
        // the fused route (k_bucket_fill): the round's stats from its tiles,
        // then every block scans the bucket totals itself
        if (b == 0) stats_final(st, reinterpret_cast<uint64_t(*)[64]>(sm));
        const uint32_t nb = gridDim.x, per_t = (nb + blockDim.x - 1) / blockDim.x;
        const uint32_t t0 = min(nb, threadIdx.x * per_t), t1 = min(nb, t0 + per_t);
        uint32_t v = 0;
        for (uint32_t j = t0; j < t1; j++) v += gcnt[j];
        uint32_t m;
        const uint32_t run = block_excl<uint32_t, RR_THREADS>(v, &m);
        if (b >= t0 && b < t1) {
            uint32_t x = run;
            for (uint32_t j = t0; j < b; j++) x += gcnt[j];
            spart[RR_THREADS + 1] = x;
        }
        __syncthreads();
        s0 = spart[RR_THREADS + 1];
        s1 = s0 + gcnt[b];
        q0 = b * capb;
        if (ctl[2] || m > cap) {                      // a bucket past capb, or the records past the buffers
            if (b == 0 && threadIdx.x == 0) {         // (the host routes them again: four passes)
                *(hm + (PIN_OVF - PIN_M)) = max(m, 1u);
                if (round1) { ctl[1] = round1 - 1; __threadfence(); ctl[0] = 2; }
            }
            return;
        }
    } else {
        s0 = base[b]; s1 = base[b + 1]; q0 = s0;
        if (base[gridDim.x] > cap) return;            // overflow (k_bucket_scatter flagged it)
    }
    pairs += q0;                                      // (pair i of the bucket at pairs[i], its rank at rank[i])
    rank += q0;
    // the bucket's run-ordered source indices: in LDS after the 4 W words when
    // they fit (lcap > 0: the host sized the dynamic LDS for them; round 6 --
    // in memory, the runs' sorts and the gather each read back what the
    // placement had just stored, every such load behind the block's stores),
    // else in idx
    uint32_t* const ix = lcap && s1 - s0 <= lcap ? sm + 4 * W : idx + s0;
    for (uint32_t j = threadIdx.x; j < 4 * W; j += blockDim.x) sm[j] = 0;
    if (threadIdx.x == 0) s_nl = 0;
    __syncthreads();
    // each pair's rank in its run (LDS atomics), the bound sums and masks; a
    // bucket of at most RR_REG pairs a thread keeps its pairs and ranks in
    // registers for the run placement below (all its loads issued at once;
    // no rank array written and read back, no second read of the pairs)
    auto count = [&](const uint2& x) {
        const uint32_t dl = x.x & wmask, cls = x.x >> 16;
        const uint32_t r = atomicAdd(&cnt[dl], 1u);
        if (cls == KEY_BCAST) {                       // 1 (a duplicate's PRUNE) + the slot bit
            atomicAdd(&bs[dl], 1u);
            const uint32_t a0 = WIRE ? heads[x.y].q[1].x : rec[x.y].a0;
            atomicOr(&mk[dl], 1ull << (a0 % PSIM_MSG_SLOTS));
        } else if (cls) {
            atomicAdd(&bs[dl], cls);
        }
        return r;
    };
    const uint32_t np = s1 - s0;
    const bool inreg = np <= regcap * blockDim.x;     // (uniform; regcap <= RR_REG)
    uint2 px[RR_REG];
    uint32_t pr[RR_REG];
    if (inreg) {
#pragma unroll
        for (uint32_t k = 0; k < RR_REG; k++) {
            const uint32_t p = threadIdx.x + k * blockDim.x;
            px[k] = p < np ? pairs[p] : make_uint2(0, 0);
        }
#pragma unroll
        for (uint32_t k = 0; k < RR_REG; k++)
            if (threadIdx.x + k * blockDim.x < np) pr[k] = count(px[k]);
    } else {
        for (uint32_t p = threadIdx.x; p < np; p += blockDim.x) rank[p] = count(pairs[p]);
    }
    __syncthreads();
    // run starts: each thread scans W / RR_THREADS consecutive counts, then
    // the block scans the thread totals
    const uint32_t per = W / RR_THREADS, j0 = threadIdx.x * per;
    uint32_t sum = 0;
    for (uint32_t j = 0; j < per; j++) sum += cnt[j0 + j];
    {
        uint32_t tot;
        spart[threadIdx.x] = block_excl<uint32_t, RR_THREADS>(sum, &tot) + sum;   // (inclusive)
    }
    for (uint32_t dl = threadIdx.x; dl < W; dl += blockDim.x) {
        const uint32_t d = (b << wshift) + dl;
        if (d >= n) break;
        cb[d] = cnt[dl] | ((unsigned long long)bs[dl] << 32);
        bmask[d] = mk[dl];
    }
    __syncthreads();                                  // the bound sums are out: pre reuses them
    uint32_t run = spart[threadIdx.x] - sum;
    for (uint32_t j = 0; j < per; j++) {
        pre[j0 + j] = run;
        run += cnt[j0 + j];
    }
    __syncthreads();
    for (uint32_t dl = threadIdx.x; dl < W; dl += blockDim.x) {
        const uint32_t d = (b << wshift) + dl;
        if (d >= n) break;
        in_beg[d] = s0 + pre[dl];
    }
    if (b == gridDim.x - 1 && threadIdx.x == 0) {   // the record count
        in_beg[n] = s1;
        *hm = s1;
        if (s1 > hm[PIN_MMAX - PIN_M]) hm[PIN_MMAX - PIN_M] = s1;
    }
    if (inreg) {
#pragma unroll
        for (uint32_t k = 0; k < RR_REG; k++)
            if (threadIdx.x + k * blockDim.x < np) ix[pre[px[k].x & wmask] + pr[k]] = px[k].y;
    } else {
        for (uint32_t p = threadIdx.x; p < np; p += blockDim.x) {
            const uint2 x = pairs[p];
            ix[pre[x.x & wmask] + rank[p]] = x.y;
        }
    }
    __syncthreads();                                  // the runs are in place (same block)
    // the bucket's longer runs, listed in LDS (the BROADCAST masks are out:
    // their words hold the list and the block sort's buffer)
    uint32_t* sv = reinterpret_cast<uint32_t*>(mk);   // RUN_LDS words
    uint32_t* ll = sv + RUN_LDS;                      // <= W destinations (2 W words in all: W >= RUN_LDS)
    for (uint32_t dl = threadIdx.x; dl < W; dl += blockDim.x) {
        const uint32_t k = cnt[dl];
        if (k < 2) continue;
        if (k > RUN_SHORT) {
            ll[atomicAdd(&s_nl, 1u)] = dl;
            continue;
        }
        uint32_t* q = ix + pre[dl];
        uint32_t v[RUN_SHORT];
#pragma unroll
        for (uint32_t t = 0; t < RUN_SHORT; t++) v[t] = t < k ? q[t] : 0xFFFFFFFFu;
#pragma unroll
        for (uint32_t r = 0; r < RUN_SHORT; r++) {
#pragma unroll
            for (uint32_t t = r & 1; t + 1 < RUN_SHORT; t += 2) {
                const uint32_t lo_ = v[t], hi_ = v[t + 1];
                v[t] = min(lo_, hi_);
                v[t + 1] = max(lo_, hi_);
            }
        }
#pragma unroll
        for (uint32_t t = 0; t < RUN_SHORT; t++)
            if (t < k) q[t] = v[t];
    }
    __syncthreads();
    // runs of RUN_SHORT + 1 .. 64: one wave each (a bitonic network over the
    // lanes); longer ones -- a join storm on one contact -- the whole block
    const uint32_t nl = s_nl, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    for (uint32_t q = wv; q < nl; q += nwv) {
        const uint32_t dl = ll[q], k = cnt[dl];
        if (k <= 64) wave_sort64(ix + pre[dl], k);
    }
    __syncthreads();
    for (uint32_t q = 0; q < nl; q++) {               // (uniform)
        const uint32_t dl = ll[q], k = cnt[dl];
        if (k > 64) sort_run_block(ix + pre[dl], k, tmp + s0 + pre[dl], sv);
    }
    __syncthreads();
    // the bucket's records into the inbox in run order (16 B a lane; two
    // records' pieces in flight per thread)
    const uint32_t m4 = (s1 - s0) * 4, bd = blockDim.x;   // (bd: a multiple of 4 -- piece t & 3 = lane & 3)
    for (uint32_t t = threadIdx.x; t < m4; t += 2 * bd) {
        const uint32_t t2 = t + bd;
        uint4 a, c = make_uint4(0, 0, 0, 0);
        if (WIRE) {
            a = wire_piece(heads, tails, ix[t >> 2], t & 3);
            if (t2 < m4) c = wire_piece(heads, tails, ix[t2 >> 2], t2 & 3);
        } else {
            a = rec_piece(rec, ix[t >> 2], t & 3);
            if (t2 < m4) c = rec_piece(rec, ix[t2 >> 2], t2 & 3);
        }
        reinterpret_cast<uint4*>(&inbox[s0 + (t >> 2)])[t & 3] = a;
        if (t2 < m4) reinterpret_cast<uint4*>(&inbox[s0 + (t2 >> 2)])[t2 & 3] = c;
    }
}

constexpr uint64_t NODE_STATE_BYTES = 416;   // HyParView 304 + Plumtree 112 per node

__device__ __forceinline__ bool due(uint32_t period, uint32_t r, uint32_t start) {
    return period > 0 && r > start && ((r - start) % period) == 0;
}

#ifdef PSIM_BOUND_TERMS
// diagnostic build (make evariant V=bterms X=-DPSIM_BOUND_TERMS): the outbox
// bound's terms summed over the nodes of every round since psim_step last
// printed them (PSIM_TRACE_BOUND)
enum { BT_RESP, BT_TIMER, BT_PUSH, BT_PUSH_NE, BT_NPUSH, BT_LAZY, BT_ON, BT_NL, BT_LC, BT_CRASH, BT_XBOT,
       BT_BUMP, BT_TOTAL, BT_C, BT_QUIET, BT_ROUNDS, BT_N };
__device__ unsigned long long g_bterm[BT_N];
#define BTERM(k, v) (bt[k] += (v))
#else
#define BTERM(k, v) ((void)0)
#endif

// Per local node: the upper bound of its emissions this round (sizes its
// outbox region) and whether it has any work (inbox, join, timers, EXIT
// scan, origin, outstanding lazy pushes).  Also counts live nodes and
// messages addressed to dead ones.
__global__ void __launch_bounds__(BLK) k_node_prep(RoundArgs a, const unsigned long long* bmask, uint64_t* packed,
                                                   uint64_t* part, uint32_t* ocnt, unsigned long long* btot,
                                                   uint32_t per, uint64_t* tiles, uint32_t* gcnt, uint32_t ngcnt) {
    if (*a.ctl) return;                               // an aborted batch (run_batch)
    // the fused route's bucket counters and its overflow flag, for this
    // round's route (k_bucket_fill)
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < ngcnt; j += gridDim.x * blockDim.x) gcnt[j] = 0;
    if (gcnt && blockIdx.x == 0 && threadIdx.x == 0) const_cast<uint32_t*>(a.ctl)[2] = 0;
    __shared__ unsigned long long s_up, s_drop, s_b, s_w, s_qp, s_qf;
    if (threadIdx.x == 0) { s_up = 0; s_drop = 0; s_b = 0; s_w = 0; s_qp = 0; s_qf = 0; }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.ktime[0] = ~0ull; a.ktime[1] = 0; *a.n_slow = 0; *a.n_pt = 0;
        if (a.n_shuf) *a.n_shuf = 0;
        if (a.n_lite) { a.n_lite[0] = 0; a.n_lite[1] = 0; a.n_lite[2] = 0; a.n_lite[3] = 0; }
        if (a.n_ptl) { a.n_ptl[0] = 0; a.n_ptl[1] = 0; }
        if (a.n_stop) *a.n_stop = 0;
    }
    __syncthreads();
    // the peers' up-and-partition pairs for k_ptl's connection tests (every
    // global id: the flag and partition arrays are replicated)
    if (a.upart && a.upart_dirty)
        for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < a.n_nodes; g += gridDim.x * blockDim.x)
            a.upart[g] = (a.flags[g] & F_UP) ? (upart_t)a.part[g] : UPART_DOWN;
    unsigned long long up = 0, drop = 0, bs = 0, ws = 0;   // this thread's sums (wave-summed below)
    unsigned long long qp = 0, qf = 0;                     // quiet lazy ticks: nodes, failed sends
#ifdef PSIM_BOUND_TERMS
    unsigned long long bt[BT_N] = {};
#endif
    // block b takes the nodes [b * per, (b + 1) * per), blockDim at a time
    // (coalesced), so that its sums are a contiguous tile of the scan below
    const uint32_t i0 = blockIdx.x * per, i1 = min(a.n_local, i0 + per);
    // (the row words every live node reads, issued with the flag byte --
    // read under its test, they were a second dependent memory wait -- and
    // for the thread's next node before this one's work: PREP_NPT nodes a
    // thread, their loads overlapped)
    struct PrepIn {
        uint8_t f;
        unsigned long long cbi;                           // inbox count | bound sum << 32
        uint32_t st, org;
        unsigned long long bm;
    };
    auto prep_in = [&](uint32_t i) {
        PrepIn q{0, 0ull, 0u, 0u, 0ull};
        if (i < i1) {
            q.f = a.flags[a.lo + i];
            q.cbi = a.in_cb[i];
            q.st = a.start[i];
            q.org = a.pl ? 0u : a.origin[i];
            q.bm = a.pl ? 0ull : bmask[i];
        }
        return q;
    };
    // one node's packed (bound << 32 | work) word (no stores: gfx9 counts
    // loads and stores in one in-order counter, so a load issued after a
    // store waits for it -- the node's row loads behind the last node's
    // stores were a store latency per node, 64 nodes a thread at 2^26)
    auto node = [&](uint32_t i, const PrepIn& cur) -> uint64_t {
        uint8_t f = cur.f;
        uint64_t b = 0;
        uint32_t w = 0;
        const unsigned long long cbi = cur.cbi;
        uint32_t c = (uint32_t)cbi;
        const uint32_t st_ = cur.st;
        const uint32_t org_ = cur.org;
        const unsigned long long bm_ = cur.bm;
        if (f & F_UP) {
            uint32_t st = st_, r = a.round;
            if (a.pl) {            // emission bounds of the pluggable round (R0-P)
                const Hdr& x = a.hdr[i];
                bool pending = x.join_contact != PSIM_NONE;
                bool per = due(a.periodic, r, st);
                bool leave = x.pad1[0] != 0;
                if (a.strategy == PSIM_STRATEGY_FULL)
                    b = a.fanout ? (uint64_t)c + a.fanout + 1
                                 : ((uint64_t)c + 2 + (leave ? 1 : 0)) * (a.n_nodes + 1);
                else
                {
                    // the view at round start, grown by at most one id per
                    // inbox message (a kept subscription) and the contact:
                    // join = contact + members + picks, periodic = a
                    // resubscription + a ping per member, leave/1 (before
                    // the inbox) = one per member, any message = one send
                    const uint64_t vn = x.act_n, vg = vn + c + 1;
                    b = (uint64_t)c + (pending ? 1 + 2 * vg : 0) + (per ? 1 + vg : 0) + (leave ? vn : 0) + 1;
                }
                w = c > 0 || (pending && !x.have) || per || leave;
            } else {
                bool origin = org_ != 0;
                const Hdr& x = a.hdr[i];      // (read only where needed: a fresh start, a full nibble)
                // the due timers' sends: the JOIN of a fresh start, a
                // promotion's NEIGHBOR_REQUEST (the active view may shrink
                // during the round: any due promotion), a shuffle
                const bool promo = a.random_promotion && due(a.promotion_period, r, st);
                b = (cbi >> 32) + (st == r && x.join_contact != PSIM_NONE ? 1u : 0u) + (promo ? 1u : 0u) +
                    (due(a.shuffle_period, r, st) ? 1u : 0u);
                BTERM(BT_RESP, cbi >> 32);
                BTERM(BT_TIMER, b - (cbi >> 32));
                // per BROADCAST message slot a first delivery's eager push
                // and lazy adds (plus the origin's): at most the root's sets
                // at round start -- or the common eagers of a new root or of a
                // reset -- plus one per message handled before; the push's
                // sends need an active connection: at most two per active
                // member (its atom and its node_spec identity, App. A Q6)
                // (round 6: a slot's pushes and lazy adds together are at most
                // the root's eager and lazy sets at round start -- or the
                // common eagers of a new root or a reset -- plus one per
                // message handled before: update_peers/5 (pt:593-609) adds one
                // peer a message to their union, and the pushes go to the
                // eager set, the adds to the lazy one (pt:374-378))
                const unsigned long long bm = c ? bm_ : 0ull;
                const uint32_t pushes = (uint32_t)__popcll(bm) + (origin ? 1u : 0u);
                const bool lazy = a.plumtree && due(a.lazy_tick_period, r, st);
                uint32_t lazy_add = 0, push_sum = 0, union_sum = 0;
                if (pushes) {
                    const uint4 r0 = *reinterpret_cast<const uint4*>(a.pt_rt + (size_t)i * RT_WORDS);
                    const uint2 cn = *reinterpret_cast<const uint2*>(a.pt_rt + (size_t)i * RT_WORDS + RT_EN);
                    const uint32_t rts[4] = {r0.x, r0.y, r0.z, r0.w};
                    auto push = [&](uint32_t root) {
                        uint32_t ne = PSIM_PT_MEMBERS_CAP, nl = 0, ne0 = 0;
#pragma unroll
                        for (int k = 0; k < PSIM_PT_ROOTS; k++)
                            if (rts[k] == root) {
                                ne0 = (cn.x >> (8 * k)) & 0xFFu;
                                ne = max(ne, ne0);
                                nl = (cn.y >> (8 * k)) & 0xFFu;
                            }
                        const uint32_t pb = min(2u * PSIM_ACTIVE_CAP, ne + c);
                        push_sum += pb;
                        lazy_add += nl + c;
                        union_sum += min(pb + nl + c, max((uint32_t)PSIM_PT_MEMBERS_CAP, ne0 + nl) + c);
                        BTERM(BT_PUSH, min(2u * PSIM_ACTIVE_CAP, ne + c));
                        BTERM(BT_PUSH_NE, min(2u * PSIM_ACTIVE_CAP, ne));
                        BTERM(BT_NPUSH, 1);
                        BTERM(BT_NL, nl);
                        BTERM(BT_LC, c);
                    };
                    for (unsigned long long m = bm; m; m &= m - 1) push(a.slots[PSIM_MSG_SLOTS + __ffsll(m) - 1]);
                    if (origin) push((a.lo + i) | PSIM_MAP_BIT);
                }
                // a due lazy tick sends every outstanding entry: those left
                // from last round and those this round's pushes add, at most
                // PT_OUT_CAP
                // (the flag byte's nibble is min(out_n, 15) after the node's
                // last round: the header only when it saturates)
                // (with the tick: the pushes P and the tick's IHAVEs, at most
                // min(PT_OUT_CAP, on + L), where P + L is at most the slots'
                // union term)
                if (lazy) {
                    const uint32_t fo = (uint32_t)f >> F_OUTN_SHIFT;
                    const uint32_t on = fo < 15 ? fo : (uint32_t)x.out_n;
                    const uint32_t pl = min(push_sum + min((uint32_t)PSIM_PT_OUT_CAP, on + lazy_add), on + union_sum);
                    b += pl;
                    BTERM(BT_LAZY, pl - push_sum);
                    BTERM(BT_ON, on);
                } else {
                    b += push_sum;
                }
                if (pushes) BTERM(BT_C, c);
                // a crash round: a NEIGHBOR_REQUEST per crashed active member
                // (bounded over every crashed member); EXIT work for a
                // crashed member held over a connection -- an active member
                // not marked PSIM_CONN_DOWN, or a lingering peer (App. A Q11)
                bool exits = false;
                if (a.crash_round) {
                    const uint4* ar = reinterpret_cast<const uint4*>(a.act + (size_t)i * PSIM_ACTIVE_CAP);
                    const uint4 a0 = ar[0], a1 = ar[1];
                    const uint32_t av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
                    uint32_t cv[PSIM_CONN_CAP] = {};
                    const uint32_t cn = x.conn_n;
                    if (cn) {
                        const uint4* cr = reinterpret_cast<const uint4*>(a.conn + (size_t)i * PSIM_CONN_CAP);
                        const uint4 c0 = cr[0], c1 = cr[1];
                        cv[0] = c0.x; cv[1] = c0.y; cv[2] = c0.z; cv[3] = c0.w;
                        cv[4] = c1.x; cv[5] = c1.y; cv[6] = c1.z; cv[7] = c1.w;
                    }
#pragma unroll
                    for (int k = 0; k < PSIM_ACTIVE_CAP; k++)
                        if ((uint32_t)k < x.act_n && av[k] < a.n_nodes && av[k] != a.lo + i &&
                            crashed_now(a, av[k])) {
                            b++;
                            BTERM(BT_CRASH, 1);
                            bool down = false;
#pragma unroll
                            for (int j = 0; j < PSIM_CONN_CAP; j++) down |= (uint32_t)j < cn && cv[j] == (av[k] | PSIM_CONN_DOWN);
                            exits |= !down;
                        }
#pragma unroll
                    for (int j = 0; j < PSIM_CONN_CAP; j++)
                        exits |= (uint32_t)j < cn && !(cv[j] & PSIM_CONN_DOWN) && crashed_now(a, cv[j] & KEY_DST_MASK);
                }
                // a quiet node (entries outstanding, F_LAZY clear: its last
                // tick reached no peer) runs only for other work: its tick
                // fails every entry again (pt:443-453 over send/3), counted
                // here -- the node processed, a failed send per entry.  Only
                // with a tick every round (else a round without one could
                // connect a peer unseen) and no waking event
                const uint32_t fon = (uint32_t)f >> F_OUTN_SHIFT;
                const bool quiet_ok = a.lazy_tick_period == 1 && !a.lazy_wake && !(f & F_LAZY);
                w = c > 0 || st == r || exits || (fon && !quiet_ok) || origin ||
                    (a.random_promotion && (f & F_LOWACT) && due(a.promotion_period, r, st)) ||
                    due(a.shuffle_period, r, st);
                if (a.xbot) {
                    // X-BOT: a due xbot_execution sends to two candidates at
                    // most; the 'EXIT' of each connection pid stopped last
                    // round may promote (a NEIGHBOR_REQUEST each)
                    const bool xb = due(a.xbot_period, r, st);
                    const uint32_t cl = x.conn_cl;
                    b += (xb ? 2u : 0u) + cl;
                    BTERM(BT_XBOT, (xb ? 2u : 0u) + cl);
                    w = w || xb || cl;
                }
                // a working node's first slot is reserved: a wave that emits
                // nothing rewrites it (flush_recs' fixed store)
                if (w && b == 0) { b = 1; BTERM(BT_BUMP, 1); }
                if (!w && fon && lazy) {
                    qp++;
                    qf += fon < 15 ? fon : (uint32_t)x.out_n;
                    BTERM(BT_QUIET, 1);
                    b = 0;
                }
            }
            up++;
        } else {
            drop += c;
        }
        bs += b;
        ws += w;
        BTERM(BT_TOTAL, b);
        // one scan gives both the outbox base (high word: the bounds) and
        // the position in the active list (low word: the work flags)
        return (b << 32) | w;
    };
    // PREP_CHUNK nodes a thread at a time: their inputs loaded together (the
    // next chunk's issued before this chunk's stores), their words and the
    // consume counts stored together after the chunk's work
    PrepIn q[PREP_CHUNK], qn[PREP_CHUNK];
    const uint32_t cstep = PREP_CHUNK * blockDim.x;
#pragma unroll
    for (uint32_t k = 0; k < PREP_CHUNK; k++) q[k] = prep_in(i0 + threadIdx.x + k * blockDim.x);
    for (uint32_t c0 = i0 + threadIdx.x; c0 < i1; c0 += cstep) {
        uint64_t pk[PREP_CHUNK];
#pragma unroll
        for (uint32_t k = 0; k < PREP_CHUNK; k++) {
            const uint32_t i = c0 + k * blockDim.x;
            pk[k] = i < i1 ? node(i, q[k]) : 0ull;
        }
#pragma unroll
        for (uint32_t k = 0; k < PREP_CHUNK; k++) qn[k] = prep_in(c0 + cstep + k * blockDim.x);
#pragma unroll
        for (uint32_t k = 0; k < PREP_CHUNK; k++) {
            const uint32_t i = c0 + k * blockDim.x;
            if (i < i1) {
                packed[i] = pk[k];
                ocnt[i] = 0;       // consume writes the count of every node it runs
            }
        }
#pragma unroll
        for (uint32_t k = 0; k < PREP_CHUNK; k++) q[k] = qn[k];
    }
#ifdef PSIM_BOUND_TERMS
    if (blockIdx.x == 0 && threadIdx.x == 0) bt[BT_ROUNDS] = 1;
    for (int k = 0; k < BT_N; k++) {
        unsigned long long v = bt[k];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if ((threadIdx.x & 63) == 0 && v) atomicAdd(&g_bterm[k], v);
    }
#endif
    for (int o = 32; o > 0; o >>= 1) {
        up += __shfl_xor(up, o);
        drop += __shfl_xor(drop, o);
        bs += __shfl_xor(bs, o);
        ws += __shfl_xor(ws, o);
        qp += __shfl_xor(qp, o);
        qf += __shfl_xor(qf, o);
    }
    if ((threadIdx.x & 63) == 0) {
        if (up) atomicAdd(&s_up, up);
        if (drop) atomicAdd(&s_drop, drop);
        if (bs) atomicAdd(&s_b, bs);
        if (ws) atomicAdd(&s_w, ws);
        if (qp) atomicAdd(&s_qp, qp);
        if (qf) atomicAdd(&s_qf, qf);
    }
    __syncthreads();
    // the tile's sum of the packed words (wrapping like them past 2^32
    // slots) for the scan; the extra tile after the last is 0 (its prefix
    // becomes the total)
    if (threadIdx.x == 0) {
        tiles[blockIdx.x] = (s_b << 32) + s_w;
        if (blockIdx.x == gridDim.x - 1) tiles[gridDim.x] = 0;
    }
    // the exact total (the packed scan's high word wraps past 2^32 slots):
    // the block's sum in its own word, summed by k_desc's last block (one
    // same-address atomic per block serialised 4096 adds at L2 every round)
    if (threadIdx.x == 0) btot[blockIdx.x] = s_b;
    if (threadIdx.x < NST) {
        // (state_bytes, R0: the rows of the nodes the phase kernels run, read
        // and written once -- SURVEY 8(d)'s 416 B of HyParView + Plumtree state)
        uint64_t v = threadIdx.x == ST_UP ? s_up : threadIdx.x == ST_DROPPED ? s_drop : threadIdx.x == ST_PROC ? s_qp
                   : threadIdx.x == ST_FAIL ? s_qf : threadIdx.x == ST_BYTES && !a.pl ? s_w * (2 * NODE_STATE_BYTES)
                   : 0ull;
        part[(size_t)blockIdx.x * NST + threadIdx.x] = v;
    }
}

// the per-node inputs of a k_desc entry, loaded before the block scan (the
// scan's barriers then overlap their latency; loaded after it, they were a
// second dependent memory wait a pass)
struct DescIn {
    uint32_t in_beg, cnt, start, origin;
};
__device__ __forceinline__ DescIn desc_in(const RoundArgs& a, uint32_t li, uint64_t pk,
                                          const uint32_t* __restrict__ in_beg,
                                          const unsigned long long* __restrict__ cb,
                                          const uint32_t* __restrict__ start) {
    DescIn d{0, 0, 0, 0};
    if (pk & 1u) {
        d.in_beg = in_beg[li];
        d.cnt = (uint32_t)cb[li];
        d.start = start[li];
        d.origin = a.plumtree && !a.pl ? a.origin[li] : 0u;
    }
    return d;
}

// node li's entry of k_desc (li == n_local: the totals), from its prefix P
// of the packed words, its own packed word pk and its inputs
__device__ __forceinline__ void desc_entry(const RoundArgs& a, uint32_t li, uint64_t P, uint64_t pk, const DescIn& d,
                                           uint4* __restrict__ desc, uint64_t* __restrict__ obase, uint32_t* nact,
                                           unsigned long long tot, uint64_t* hout, uint64_t cap, uint32_t* ctl) {
    obase[li] = P >> 32;
    if (li == a.n_local) {
        *nact = (uint32_t)P;
        obase[li] = tot;
        hout[PIN_TOTAL] = tot;                        // the host's one mid-round read
        if (tot > hout[PIN_TMAX]) hout[PIN_TMAX] = tot;
        // a batch (cap > 0) checks the outbox here instead: a total past its
        // capacity stops the rest of the batch (code 1, this round)
        if (cap && tot + 1 > cap) { ctl[1] = a.round; __threadfence(); ctl[0] = 1; }
        return;
    }
    if (!(pk & 1u)) return;
    if (d.cnt > DESC_CNT_MASK) hout[PIN_BIGIN] = 1;   // (the descriptor packs it in 26 bits)
    const uint32_t st = d.start, r = a.round;
    const uint32_t tf = (a.random_promotion && due(a.promotion_period, r, st) ? DESC_PROMO : 0u) |
                        (due(a.shuffle_period, r, st) ? DESC_SHUFFLE : 0u) |
                        (a.plumtree && due(a.lazy_tick_period, r, st) ? DESC_LAZY : 0u) |
                        (d.origin ? DESC_ORIGIN : 0u);
    const uint32_t xb = a.xbot && due(a.xbot_period, r, st) ? DESC_XBOT_BIT : 0u;
    desc[(uint32_t)P] = make_uint4(a.lo + li, d.in_beg, d.cnt | xb | (tf << 28), (uint32_t)(P >> 32));
}

// the outbox total: the sum of k_node_prep's nbt block sums (every thread of
// the block calls it)
__device__ unsigned long long btot_sum(const unsigned long long* btot, uint32_t nbt) {
    __shared__ unsigned long long s_w[PREP_BLK / 64], s_tot;
    unsigned long long t = 0;
    for (uint32_t j = threadIdx.x; j < nbt; j += blockDim.x) t += btot[j];
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long u = 0;
        for (uint32_t k = 0; k < blockDim.x / 64; k++) u += s_w[k];
        s_tot = u;
    }
    __syncthreads();
    return s_tot;
}


// Per node, from the scan of the packed (bound, work) words: the outbox
// base, and for a node with work its descriptor at its active-list position
// -- every address k_consume needs first and which of the node's timers are
// due (hv:542-607, pt:341-345).  Entry n: the outbox total and the count.
// Block b walks k_node_prep's range of block b again, PREP_BLK nodes a pass:
// a block scan of their packed words on top of the range's prefix, which the
// block sums itself from k_node_prep's range sums (one per thread: the grid
// has at most PREP_BLK blocks) -- one launch in place of a tile-sum, a
// tile-scan and an apply pass (the one-block scan of the range sums alone
// took 8.5 us a round at 2^20 nodes over 4096 ranges)
__global__ void __launch_bounds__(PREP_BLK) k_desc(const uint64_t* __restrict__ packed,
                                                  const uint64_t* __restrict__ tiles, uint32_t per,
                                                  const uint32_t* __restrict__ in_beg,
                                                  const unsigned long long* __restrict__ cb,
                                                  const uint32_t* __restrict__ start, RoundArgs a,
                                                  uint4* __restrict__ desc, uint64_t* __restrict__ obase,
                                                  uint32_t* nact, const unsigned long long* btot,
                                                  uint32_t nranges, uint64_t* hout, uint64_t cap, uint32_t* ctl) {
    if (*ctl) return;                                 // (uniform)
    const bool last = blockIdx.x == gridDim.x - 1;
    const uint32_t r0 = blockIdx.x * DESC_RANGES;     // this block's first k_node_prep range
    const uint32_t i0 = r0 * per, i1 = min(a.n_local, i0 + DESC_RANGES * per);
    // (the sums of the ranges before this block's and the first pass's
    // inputs issued before either is used)
    uint64_t tp = 0;
#pragma unroll
    for (uint32_t k = 0; k < DESC_RANGES; k++) {
        const uint32_t j = threadIdx.x + k * PREP_BLK;
        tp += j < r0 ? tiles[j] : 0ull;
    }
    uint32_t li = i0 + threadIdx.x;
    uint64_t pk = li < i1 ? packed[li] : 0ull;
    DescIn d = desc_in(a, li, pk, in_beg, cb, start);
    const unsigned long long tot = last ? btot_sum(btot, nranges) : 0ull;   // (uniform)
    uint64_t carry;
    (void)block_excl<uint64_t, PREP_BLK>(tp, &carry);
    for (uint32_t k = i0; k < i1; k += PREP_BLK) {    // (uniform)
        if (k != i0) {
            li = k + threadIdx.x;
            pk = li < i1 ? packed[li] : 0ull;
            d = desc_in(a, li, pk, in_beg, cb, start);
        }
        uint64_t pass;
        const uint64_t e = block_excl<uint64_t, PREP_BLK>(pk, &pass);
        if (li < i1) desc_entry(a, li, carry + e, pk, d, desc, obase, nact, 0ull, hout, cap, ctl);
        carry += pass;
    }
    if (last && threadIdx.x == 0)                     // entry n: the totals (carry: every range's sum)
        desc_entry(a, a.n_local, carry, 0ull, DescIn{0, 0, 0, 0}, desc, obase, nact, tot, hout, cap, ctl);
}

// --------------------------------------------------------- overlay stats --
// psim_get_histograms: per live node its view sizes, the in-degree links it
// contributes (global id arrays, summed over shards / RCCL ranks) and the
// tracked broadcast's delivery.  hist layout: 5 histograms of
// PSIM_HIST_BINS, then n_up, delivered, last_round, active_links.
enum { H_AIN = 0, H_PIN = 1, H_AOUT = 2, H_PFILL = 3, H_HOP = 4, H_NUP = 5 * PSIM_HIST_BINS,
       H_DELIV, H_LAST, H_LINKS, H_N };

__device__ __forceinline__ uint32_t hbin(uint32_t v) { return v < PSIM_HIST_BINS ? v : PSIM_HIST_BINS - 1; }

__global__ void k_hist_out(const Hdr* __restrict__ hdr, const uint32_t* __restrict__ act,
                           const uint32_t* __restrict__ pas, const uint8_t* __restrict__ flags, uint32_t lo,
                           uint32_t n, uint64_t tbit, uint32_t* indeg_a, uint32_t* indeg_p,
                           unsigned long long* hist) {
    __shared__ unsigned long long sh[H_N];
    for (uint32_t j = threadIdx.x; j < H_N; j += blockDim.x) sh[j] = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && (flags[lo + i] & F_UP)) {
        const Hdr& x = hdr[i];
        const uint32_t me = lo + i;
        uint32_t out = 0;
        for (uint32_t k = 0; k < x.act_n; k++) {
            const uint32_t p = act[(size_t)i * PSIM_ACTIVE_CAP + k];
            if (p == me) continue;
            out++;
            if (flags[p] & F_UP) { atomicAdd(&indeg_a[p], 1u); atomicAdd(&sh[H_LINKS], 1ull); }
        }
        for (uint32_t k = 0; k < x.pas_n; k++) {
            const uint32_t p = pas[(size_t)i * PSIM_PASSIVE_CAP + k];
            if (p != me && (flags[p] & F_UP)) atomicAdd(&indeg_p[p], 1u);
        }
        atomicAdd(&sh[H_AOUT * PSIM_HIST_BINS + hbin(out)], 1ull);
        atomicAdd(&sh[H_PFILL * PSIM_HIST_BINS + hbin(x.pas_n)], 1ull);
        atomicAdd(&sh[H_NUP], 1ull);
        if (tbit && ((((uint64_t)x.aux << 32) | x.have) & tbit)) {
            atomicAdd(&sh[H_DELIV], 1ull);
            atomicAdd(&sh[H_HOP * PSIM_HIST_BINS + hbin(x.trk_hop)], 1ull);
            if (x.trk_round != PSIM_NONE) atomicMax(&sh[H_LAST], (unsigned long long)x.trk_round);
        }
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < H_N; j += blockDim.x) {
        if (!sh[j]) continue;
        if (j == H_LAST) atomicMax(&hist[j], sh[j]);
        else atomicAdd(&hist[j], sh[j]);
    }
}

__global__ void k_hist_in(const uint32_t* __restrict__ indeg_a, const uint32_t* __restrict__ indeg_p,
                          const uint8_t* __restrict__ flags, uint32_t lo, uint32_t n, unsigned long long* hist) {
    __shared__ unsigned long long sh[2 * PSIM_HIST_BINS];
    for (uint32_t j = threadIdx.x; j < 2 * PSIM_HIST_BINS; j += blockDim.x) sh[j] = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && (flags[lo + i] & F_UP)) {
        atomicAdd(&sh[hbin(indeg_a[lo + i])], 1ull);
        atomicAdd(&sh[PSIM_HIST_BINS + hbin(indeg_p[lo + i])], 1ull);
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < 2 * PSIM_HIST_BINS; j += blockDim.x)
        if (sh[j]) atomicAdd(&hist[H_AIN * PSIM_HIST_BINS + j], sh[j]);
}

// the whole overlay's active rows (gathered from every shard / RCCL rank into
// gact / gan by global id): reverse-link test and label propagation over live
// active links (min label, then pointer jumping)
__global__ void k_pack_act(const Hdr* __restrict__ hdr, const uint32_t* __restrict__ act, uint32_t n,
                           uint32_t* gact, uint8_t* gan) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = hdr[i].act_n;
    gan[i] = (uint8_t)k;
    for (uint32_t j = 0; j < PSIM_ACTIVE_CAP; j++) gact[(size_t)i * PSIM_ACTIVE_CAP + j] = act[(size_t)i * PSIM_ACTIVE_CAP + j];
}

__global__ void k_hist_sym(const uint8_t* __restrict__ gan, const uint32_t* __restrict__ act,
                           const uint8_t* __restrict__ flags, uint32_t n, unsigned long long* sym) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !(flags[i] & F_UP)) return;
    uint32_t c = 0;
    for (uint32_t k = 0; k < gan[i]; k++) {
        const uint32_t p = act[(size_t)i * PSIM_ACTIVE_CAP + k];
        if (p == i || p >= n || !(flags[p] & F_UP)) continue;
        for (uint32_t q = 0; q < gan[p]; q++)
            if (act[(size_t)p * PSIM_ACTIVE_CAP + q] == i) { c++; break; }
    }
    if (c) atomicAdd(sym, (unsigned long long)c);
}

__global__ void k_cc_init(const uint8_t* __restrict__ flags, uint32_t n, uint32_t* L) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) L[i] = (flags[i] & F_UP) ? i : PSIM_NONE;
}

__global__ void k_cc_hook(const uint8_t* __restrict__ gan, const uint32_t* __restrict__ act,
                          const uint8_t* __restrict__ flags, uint32_t n, uint32_t* L, uint32_t* changed) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !(flags[i] & F_UP)) return;
    for (uint32_t k = 0; k < gan[i]; k++) {
        const uint32_t p = act[(size_t)i * PSIM_ACTIVE_CAP + k];
        if (p == i || p >= n || !(flags[p] & F_UP)) continue;
        const uint32_t a = L[i], b = L[p];
        if (a < b) { if (atomicMin(&L[p], a) > a) *changed = 1; }
        else if (b < a) { if (atomicMin(&L[i], b) > b) *changed = 1; }
    }
}

__global__ void k_cc_jump(uint32_t n, uint32_t* L) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || L[i] == PSIM_NONE) return;
    uint32_t r = L[i];
    while (L[r] != r) r = L[r];
    L[i] = r;
}

__global__ void k_cc_count(const uint32_t* __restrict__ L, uint32_t n, uint32_t* size, unsigned long long* comps) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || L[i] == PSIM_NONE) return;
    atomicAdd(&size[L[i]], 1u);
    if (L[i] == i) atomicAdd(comps, 1ull);
}

__global__ void k_cc_max(const uint32_t* __restrict__ size, uint32_t n, unsigned long long* largest) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && size[i]) atomicMax(largest, (unsigned long long)size[i]);
}

// ------------------------------------------------------------- buffers --
template <typename T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    // grow to the next power of two (per-round sizes peak on broadcast
    // rounds; a 25 % step re-allocated -- 1 ms each -- for many rounds),
    // contents not kept
    // headroom: grow to the power of two at or above want * (1 + headroom / 4);
    // headroom < 0: exactly want, rounded up to 64 MiB past 1 GiB (an
    // up-front reservation sized against the free device memory)
    int ensure(size_t want, int headroom = 0) {
        if (want <= n) return PSIM_OK;
        static const bool trace = getenv("PSIM_TRACE_GROW") != nullptr;
        if (trace && want >= (1u << 20))
            std::fprintf(stderr, "psim: grow %zu -> %zu (want) x %zu B\n", n, want, sizeof(T));
        if (p) (void)hipFree(p);
        p = nullptr; n = 0;
        const size_t goal = want + want / 4 * (size_t)(headroom > 0 ? headroom : 0);
        size_t cap = 1024;
        while (cap < goal) cap <<= 1;
        // past 1 GiB a power of two (or the caller's headroom) may waste up
        // to half: 1/8 headroom in 64 MiB steps instead (at 2^26 nodes the
        // message buffers are tens of GB)
        if (headroom < 0) cap = want;
        if (cap * sizeof(T) > (1ull << 30)) {
            const size_t step = (64ull << 20) / sizeof(T);
            cap = (want + (headroom < 0 ? 0 : want / 8) + step - 1) / step * step;
        }
        if (hipMalloc(&p, cap * sizeof(T)) != hipSuccess) {
            size_t fr = 0, tot = 0;
            (void)hipGetLastError();
            if (hipMemGetInfo(&fr, &tot) == hipSuccess)
                std::fprintf(stderr, "psim: device allocation of %.2f GB failed (%.2f of %.2f GB free)\n",
                             cap * sizeof(T) / 1e9, fr / 1e9, tot / 1e9);
            p = nullptr;
            return PSIM_ENOMEM;
        }
        n = cap;
        return PSIM_OK;
    }
    // grow like ensure(), keeping the first `keep` elements (copied on `st`)
    int ensure_keep(size_t want, size_t keep, hipStream_t st) {
        if (want <= n) return PSIM_OK;
        if (!p || !keep) return ensure(want);
        DBuf<T> nb;
        TRY(nb.ensure(want));
        if (hipMemcpyAsync(nb.p, p, std::min(keep, n) * sizeof(T), hipMemcpyDeviceToDevice, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) {
            nb.release();
            return PSIM_EDEVICE;
        }
        release();
        p = nb.p; n = nb.n;
        return PSIM_OK;
    }
    int alloc(size_t want) {    // exact, zeroed
        static const bool trace = getenv("PSIM_TRACE_GROW") != nullptr;
        if (trace && want >= (1u << 20)) std::fprintf(stderr, "psim: alloc %zu x %zu B\n", want, sizeof(T));
        if (hipMalloc(&p, std::max<size_t>(want, 1) * sizeof(T)) != hipSuccess) return PSIM_ENOMEM;
        n = want;
        if (hipMemset(p, 0, std::max<size_t>(want, 1) * sizeof(T)) != hipSuccess) return PSIM_EDEVICE;
        return PSIM_OK;
    }
    // exact, zeroed on `st` (ordered before the stream's later kernels; the
    // null-stream fill of alloc() is not ordered with a non-blocking stream)
    int alloc_on(size_t want, hipStream_t st) {
        if (hipMalloc(&p, std::max<size_t>(want, 1) * sizeof(T)) != hipSuccess) return PSIM_ENOMEM;
        n = want;
        if (hipMemsetAsync(p, 0, std::max<size_t>(want, 1) * sizeof(T), st) != hipSuccess) return PSIM_EDEVICE;
        return PSIM_OK;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; n = 0; }
};

// a temporary device buffer, released on every return path
template <typename T>
struct TmpBuf : DBuf<T> {
    TmpBuf() = default;
    TmpBuf(const TmpBuf&) = delete;
    TmpBuf& operator=(const TmpBuf&) = delete;
    ~TmpBuf() { this->release(); }
};

enum Kern { KT_EVENTS, KT_PREPARE, KT_CONSUME, KT_SCAN, KT_COMPACT, KT_SORT, KT_EXCHANGE, KT_GATHER,
            KT_STATS, KT_N };
const char* kKernName[KT_N] = {"events", "prepare", "consume", "scan", "compact", "sort",
                               "exchange", "gather", "stats"};

inline uint32_t grid_for(uint64_t n) { return (uint32_t)std::max<uint64_t>(1, (n + BLK - 1) / BLK); }

int bits_for(uint64_t n) {
    int b = 1;
    while (b < 32 && (1ull << b) < n) b++;
    return b;
}

// Up-front reservations (the first round of a handle): a buffer that grows
// mid-run is a hipFree + hipMalloc, and the driver clears fresh device memory
// -- at 2^26 nodes one growth of the ~100 GB outbox took 2.3-3.1 s inside a
// timed window (profiles/r03/e26_attrib.txt) -- so the message buffers take
// their working size once, against the free device memory:
//   the route's records: RCAP_RESERVE per node where that takes at most
//   RCAP_FREE_FRAC of the free memory (else RCAP_PER_NODE, growing);
//   the outbox: RESERVE_PER_NODE slots per node, or what is left after the
//   route, less OUTBOX_SPARE (a growth past it still works, slowly)
constexpr uint64_t RESERVE_PER_NODE = 24;   // outbox slots per node reserved up front (round 6: 32 before the union bound)
constexpr uint64_t RCAP_PER_NODE = 4;       // initial route capacity (records) per node
constexpr uint64_t RCAP_RESERVE = 8;        // ... reserved up front where it fits
constexpr double RCAP_FREE_FRAC = 0.30;
constexpr double OUTBOX_SPARE = 0.12;

struct Shard {
    uint32_t idx = 0, lo = 0, n = 0;    // global shard index, owned [lo, lo + n)
    hipStream_t stream = nullptr;
    // replicated (global id)
    DBuf<uint8_t> flags, part;
    DBuf<upart_t> upart;                // k_node_prep's up-and-partition pairs (RoundArgs::upart)
    DBuf<uint8_t> lite_cm;              // k_relay's connection bits of lite-list nodes (RoundArgs::lite_cm)
    DBuf<uint32_t> crash_bits;   // RoundArgs::crash_bits
    DBuf<uint8_t> btab;          // RoundArgs::btab (psim_set_bucket_table), global id
    // local rows
    DBuf<Hdr> hdr;
    DBuf<uint32_t> act, pas, pt_all, pt_com, pt_eag, pt_laz, pt_rt, start;
    DBuf<uint64_t> sentm, recvm, mapx;  // id maps (id << 32 | peer): own rows, extension rows (pool)
    DBuf<uint32_t> mapx_top;
    DBuf<uint32_t> origin;              // per local node: msg id + 1 it originates this round
    DBuf<uint32_t> slots;               // the message slots (msg ids, then roots), a copy of the host's
    DBuf<uint32_t> bc_roots, bc_msgs;   // this round's broadcasts
    DBuf<uint64_t> pt_out, outx;        // outstanding: own rows, extension rows (pool)
    DBuf<uint32_t> conn;                // connection tables (PSIM_CONN_CAP per node; HyParView)
    DBuf<uint32_t> outx_top;
    // inbox of the next round: sorted (local dst | bound, record index) pairs
    DBuf<uint32_t> ikeys, ivals;
    uint32_t m_in = 0;
    DBuf<Msg> outbox;                   // this round's emissions (holes between node regions)
    // G > 1: the received records in the wire format, in source-shard order:
    // their heads, the long ones' tails, and per source its first head and
    // first tail (wseg, 2 (G + 1) words; its host copy until the next round)
    DBuf<Wire> recvh, recvt;
    DBuf<uint32_t> wseg;
    std::vector<uint32_t> wseg_host;
    // records by node run, in inbox order: read by this round's node-round
    // kernels, then (same stream) overwritten by the route with the next
    // round's -- one buffer, nothing reads a round's inbox after its consume
    DBuf<Msg> inbox;
    // per-round scratch
    DBuf<uint32_t> okey, ocnt, in_beg,
        d_nact, n_slow, n_pt, n_shuf, n_lite, n_ptl, rank, tmp, hist, hoff;
    DBuf<uint32_t> rtot, rbase;         // route: per bucket its record count, and its first pair
    DBuf<uint32_t> gcnt;                // fused route: per bucket its record count (k_bucket_fill's atomics)
    DBuf<unsigned long long> bmask;     // per local node: message slots of its BROADCAST records
    DBuf<uint2> pairs;                  // route: (destination in bucket | class, source index)
    DBuf<unsigned long long> cb;        // per local node: inbox count | bound sum << 32 (n + 1)
    DBuf<unsigned long long> btot;      // this round's outbox total (k_node_prep)
    DBuf<uint4> desc, desc_slow, desc_pt, desc_shuf, desc_lite, desc_ptl;   // work descriptors; those k_relay leaves to k_consume / k_pt / k_shuf
    DBuf<uint64_t> bound, pscan, obase, stat_part, stat_out, stat_tile, d_off;   // bound: packed (bound << 32 | work)
    DBuf<uint8_t> cub_tmp;              // the scan's tile totals
    DBuf<uint32_t> ev_ids, ev_contacts, stop_ids, n_stop;
    bool tomb_live = false;             // full: snapshots carry their remove rows
    DBuf<Wire> sendbuf;                 // G > 1: the outbox in the wire format, by owner (k_owner_part)
    // pluggable manager
    DBuf<uint32_t> sview, sinv, fbits, pay[2], pay_top;
    int pay_cur = 0;
    DBuf<uint8_t> faulted;              // omission faults: generally omitting nodes (global id)
    DBuf<uint64_t> omit;                // ... sorted send-omission pairs, then receive-omission pairs
    // per destination shard: the send buffer's offsets (2 G + 1: heads of
    // each owner, tails of each owner, the end), heads and tails sent
    std::vector<uint64_t> soff, scnt, lcnt;
    uint32_t pper = BLK;               // k_node_prep / k_desc: nodes per block (a multiple of BLK)
    uint32_t pgrid = 0, cgrid = 0, rgrid = 0, tgrid = 0, sgrid = 0, lgrid = 0, qgrid = 0;   // stats rows: prepare,
                                   // consume, relay, plumtree, shuffle-start, lite, Plumtree-lane blocks
    // pinned host words: NST stats and the consume span (stat_out), then the
    // outbox total and the routed record count: the round's two read-backs
    uint64_t* pin = nullptr;
    uint64_t* pin_dev = nullptr;        // the same words, as the kernels store them
    // phase timers: event pairs recorded on the stream and read back once per
    // round, after the round's final synchronisation (no sync per phase)
    static constexpr int MAXT = 32;
    hipEvent_t ev[MAXT][2];
    int tk[MAXT];
    int tn = 0;
    hipEvent_t wait_ev = nullptr;
    // the three HyParView kernels after k_relay take disjoint node lists and
    // run concurrently: k_shuf and k_consume on two side streams forked from
    // and joined back into `stream` (fork_ev, join_ev)
    hipStream_t side[2] = {nullptr, nullptr};
    hipEvent_t fork_ev = nullptr, join_ev[2] = {nullptr, nullptr};
    bool ev_live = false;
    bool reserved = false;              // first-round capacity reservation done
    bool upart_valid = false;           // upart holds this state's pairs (RoundArgs::upart_dirty)
    uint64_t rcap = 0;                  // records the route's buffers hold (G == 1: checked on the device)
    // batches of rounds without host waits (run_batch): the abort word
    // (code, round) in device memory; while a batch is enqueued, k_desc
    // checks the outbox against desc_cap and the route flags its overflow
    // for round batch_round1 - 1; round j's stats go to pinned slot j + 1
    DBuf<uint32_t> ctl;
    uint64_t desc_cap = 0;
    uint32_t batch_round1 = 0;
    uint32_t stat_slot = 0;
    bool outx_short = false;            // the outstanding pool failed to grow (reported once per shard)
    // the rank path's batches (run_batch_ranked): the fixed per-owner
    // capacities of the exchange (heads, tails; 0 = not known yet: no batch),
    // identical on every rank (set from all-reduced counts), and the next
    // batch's length (1 after an abort, doubling up to BATCH_MAX)
    uint32_t xcap_h = 0, xcap_t = 0;
    uint32_t xbatch = 1;
    uint64_t trace_tmax = 0, trace_mmax = 0;   // PSIM_TRACE_BOUND's high-water marks
};

}  // namespace

struct psim_handle {
    psim_config cfg;
    uint32_t N = 0, G = 1, per = 0;
    int device = 0;
    uint32_t consume_blocks = 1024;     // resident k_consume blocks on the device
    uint32_t pt_blocks = 1024;          // ... and k_pt blocks
    uint32_t lite_blocks = 1024;        // ... and k_consume_lite (k_lite_half) blocks
    // the lite list's kernel: k_lite_half, two nodes per wave (psim_lite.hip);
    // PSIM_LITE_WAVE=1 keeps the wave-per-node k_consume_lite (A/B)
    bool lite_half = true;
    uint32_t ptl_blocks = 1024;         // ... and k_ptl blocks
    uint64_t round = 0;
    // a round failed half-way (psim_step returned an error from inside a
    // round or batch): the state is not a round boundary any more, so every
    // later psim_step answers PSIM_ESTATE instead of running on it
    bool failed = false;
    std::vector<Shard*> shards;         // shards owned by this process
    int rank = 0, world = 1;
    // the rank path (one shard per rank, the owner partition, the exchange
    // and the collectives of psim_comm.h): world > 1, or a one-rank world
    // whose cfg.comm_id was given (the 1-GPU diagnostic of the RCCL path:
    // every collective, the self send/recv included, runs through the library)
    bool ranked = false;
    Comm* comm = nullptr;               // ranked: RCCL (or the loopback test vehicle), psim_comm.h
    DBuf<uint64_t> comm_cnt;            // RCCL: [send counts | recv counts]
    // the exchange since creation (psim_get_exchange_stats): records sent to
    // another shard, and their wire bytes (heads + tails)
    uint64_t x_records = 0, x_bytes = 0;
    // pending events
    std::vector<uint32_t> pend_crash, pend_join, pend_contact;
    std::vector<uint8_t> pend_join_mark;   // ids in pend_join (a node starts at most once per round)
    std::vector<uint32_t> pend_lv_a, pend_lv_t;     // leave/1 calls: actor, target
    std::vector<uint8_t> pend_part;
    bool pend_part_set = false, pend_part_clear = false;
    std::vector<uint32_t> pend_b_root, pend_b_msg;    // broadcasts of the next round, in call order
    uint32_t slot_tab[2 * PSIM_MSG_SLOTS];            // slot k: msg id [k], root [PSIM_MSG_SLOTS + k]
    uint32_t tracked_msg = PSIM_NONE;
    bool btab = false;                  // psim_set_bucket_table: the shards' btab rows are in use
    uint32_t btab_hash = 0;             // ... their FNV-1a | 1 (0 = the default table), in snapshots
    uint32_t fw = 0;                    // full strategy: words per member row (adds; removes beside)
    bool tomb = false;                  // full: an ORSet remove exists (leave/1): kernels read remove rows
    std::vector<uint8_t> started;       // full strategy: ids ever started (no restarts)
    // omission faults (pluggable): the next round's installed funs, edited by
    // psim_set_omission / psim_set_faulted and uploaded when changed; the
    // counts of the ones in force
    std::set<uint64_t> nx_omit_s, nx_omit_r;
    std::vector<uint8_t> nx_faulted;
    size_t nx_nfaulted = 0;
    bool faults_dirty = false;
    uint32_t faults = 0, n_omit_s = 0, n_omit_r = 0;
    double kt_ms[KT_N] = {0};
    uint64_t kt_n[KT_N] = {0};
    // per-phase event timers (PSIM_PHASE_TIMERS=1): each event pair puts a
    // ~10 us bubble between kernels, so by default only k_consume is timed,
    // from its in-kernel span (RoundArgs::ktime)
    bool phase_timers = false;
    // blocks of the route / owner-partition passes (RB_MAX_BLOCKS; a test
    // hook, PSIM_ROUTE_BLOCKS, lowers it so small runs take several steps per block)
    uint32_t rb_blocks = RB_BLOCKS;
    uint32_t rr_reg = RR_REG;           // k_bucket_route: pairs a thread may hold (PSIM_ROUTE_REG=0: the array path)
    // one shard's own outbox routed by the fused pass (k_bucket_fill) instead
    // of k_bucket_hist + k_bucket_offsets + k_bucket_scatter
    // (PSIM_ROUTE_FUSED=0: the four passes, for A/B; reroutes take them too)
    bool route_fused = true;
};

namespace {

// one shard in this process and no rank path: the round's emissions are
// grouped by destination in place (phase_route_local); otherwise they go
// through the owner partition and an exchange
inline bool local_route(const psim_handle* h) { return h->G == 1 && !h->ranked; }

RoundArgs make_args(psim_handle* h, Shard* s) {
    RoundArgs a;
    memset(&a, 0, sizeof a);
    const psim_config& c = h->cfg;
    a.n_nodes = h->N; a.round = (uint32_t)h->round; a.seed = c.seed;
    a.lo = s->lo; a.n_local = s->n;
    a.max_active = c.max_active_size; a.min_active = c.min_active_size;
    a.max_passive = c.max_passive_size; a.arwl = c.arwl; a.prwl = c.prwl;
    a.k_active = c.k_active; a.k_passive = c.k_passive;
    a.shuffle_period = c.shuffle_period; a.promotion_period = c.promotion_period;
    a.random_promotion = c.random_promotion; a.plumtree = c.plumtree;
    a.lazy_tick_period = c.lazy_tick_period;
    a.tracked_msg = h->tracked_msg;
    a.origin = s->origin.p;
    a.slots = s->slots.p;
    a.flags = s->flags.p; a.part = s->part.p; a.hdr = s->hdr.p; a.crash_bits = s->crash_bits.p;
    a.upart = s->upart.p;
    a.lite_cm = s->lite_cm.p;
    a.btab = h->btab ? s->btab.p : nullptr;
    a.act = s->act.p; a.pas = s->pas.p; a.sentm = s->sentm.p; a.recvm = s->recvm.p;
    a.mapx = s->mapx.p; a.mapx_top = s->mapx_top.p;
    a.mapx_rows = (uint32_t)(s->mapx.n / IDMAP_EXT);
    a.pt_all = s->pt_all.p; a.pt_com = s->pt_com.p; a.pt_eag = s->pt_eag.p; a.pt_laz = s->pt_laz.p;
    a.pt_rt = s->pt_rt.p;
    a.pt_out = s->pt_out.p; a.outx = s->outx.p; a.outx_top = s->outx_top.p;
    a.conn = s->conn.p;
    a.outx_rows = (uint32_t)(s->outx.n / OUT_EXT);
    a.start = s->start.p;
    a.pl = c.manager == PSIM_MANAGER_PLUGGABLE;
    a.xbot = c.manager == PSIM_MANAGER_XBOT; a.xbot_period = c.xbot_period;
    a.strategy = c.strategy; a.periodic = c.periodic_interval; a.scamp_c = c.scamp_c;
    a.fanout = c.fanout; a.fw = h->fw; a.tomb = h->tomb;
    a.fbits = s->fbits.p; a.sview = s->sview.p; a.sinv = s->sinv.p;
    a.ktime = reinterpret_cast<unsigned long long*>(s->stat_out.p + NST);
    a.ctl = s->ctl.p;
    a.desc_slow = s->desc_slow.p; a.n_slow = s->n_slow.p;
    a.desc_pt = s->desc_pt.p; a.n_pt = s->n_pt.p;
    a.desc_shuf = s->desc_shuf.p; a.n_shuf = s->n_shuf.p;
    a.desc_lite = s->desc_lite.p; a.n_lite = s->n_lite.p;
    a.desc_ptl = s->desc_ptl.p; a.n_ptl = s->n_ptl.p;
    a.stop_ids = s->stop_ids.p; a.n_stop = s->n_stop.p;
    a.faults = h->faults; a.n_omit_s = h->n_omit_s; a.n_omit_r = h->n_omit_r;
    a.faulted = s->faulted.p; a.omit = s->omit.p;
    return a;
}

// per-kernel-class device time, HIP events on the shard's stream; the
// elapsed times are collected by flush_timers once the round has synchronised
int route_buffers(Shard* s, bool both_inboxes);

struct KTimer {
    Shard* s;
    int slot;
    KTimer(psim_handle* h, Shard* s_, int k) : s(s_), slot(-1) {
        if (!h->phase_timers || s->tn >= Shard::MAXT) return;
        slot = s->tn++;
        s->tk[slot] = k;
        (void)hipEventRecord(s->ev[slot][0], s->stream);
    }
    ~KTimer() {
        if (slot >= 0) (void)hipEventRecord(s->ev[slot][1], s->stream);
    }
};

void flush_timers(psim_handle* h, Shard* s) {
    for (int i = 0; i < s->tn; i++) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, s->ev[i][0], s->ev[i][1]) != hipSuccess) continue;
        h->kt_ms[s->tk[i]] += ms;
        h->kt_n[s->tk[i]]++;
    }
    s->tn = 0;
}

// ------------------------------------------------ exclusive prefix sum --
// Reduce-then-scan over tiles of SCAN_TILE elements (256 threads x 8
// consecutive elements each): tile totals, one block scans the totals, each
// tile scans itself from its total's prefix.  Three launches, the input read
// twice (at 2^20 nodes: 8 MB per read, a few microseconds); a count that
// fits one tile is one launch.
constexpr uint32_t SCAN_ITEMS = 8, SCAN_TILE = BLK * SCAN_ITEMS;

// exclusive scan of one value per thread across the block; returns the
// block total in *total (every thread)
template <typename T, uint32_t NT>
__device__ T block_excl(T v, T* total) {
    __shared__ T wsum[NT / 64];
    const uint32_t l = threadIdx.x & 63, wv = threadIdx.x >> 6;
    T x = v;                                          // inclusive scan within the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const T y = __shfl_up(x, d);
        if (l >= (uint32_t)d) x += y;
    }
    if (l == 63) wsum[wv] = x;
    __syncthreads();
    T base = 0, tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < NT / 64; k++) {
        base += k < wv ? wsum[k] : T(0);
        tot += wsum[k];
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

template <typename T>
__global__ void __launch_bounds__(BLK) k_scan_tiles(const T* __restrict__ in, uint32_t n, T* __restrict__ sums) {
    const size_t b0 = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_ITEMS;
    T v = 0;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_ITEMS; k++) v += b0 + k < n ? in[b0 + k] : T(0);
    T tot;
    (void)block_excl(v, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// one block: exclusive scan of the nt tile totals in place -- each thread a
// contiguous run of ceil(nt / BLK) of them, one block scan of the run sums
// (a block scan per BLK chunk took 12.7 us for 4097 totals: 17 serial
// barrier pairs).  Up to SUMS_LDS totals go through LDS, loaded and stored
// coalesced (the runs read straight from memory were ceil(nt / BLK)
// dependent strided loads a thread: 8.6 us for 4097 totals)
constexpr uint32_t SUMS_LDS = 4096 + 2 * BLK;
template <typename T>
__global__ void __launch_bounds__(BLK) k_scan_sums(T* sums, uint32_t nt) {
    __shared__ T buf[SUMS_LDS];
    const bool lds = nt <= SUMS_LDS;                  // (uniform)
    T* p = lds ? buf : sums;
    if (lds) {
        for (uint32_t i = threadIdx.x; i < nt; i += BLK) buf[i] = sums[i];
        __syncthreads();
    }
    const uint32_t per = (nt + BLK - 1) / BLK, i0 = threadIdx.x * per, i1 = min(nt, i0 + per);
    T v = 0;
    for (uint32_t i = i0; i < i1; i++) v += p[i];
    T tot;
    T run = block_excl(v, &tot);
    for (uint32_t i = i0; i < i1; i++) {
        const T x = p[i];
        p[i] = run;
        run += x;
    }
    if (lds) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < nt; i += BLK) sums[i] = buf[i];
    }
}

template <typename T>
__global__ void __launch_bounds__(BLK) k_scan_apply(const T* __restrict__ in, T* __restrict__ out, uint32_t n,
                                                   const T* __restrict__ sums) {
    const size_t b0 = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_ITEMS;
    T x[SCAN_ITEMS], v = 0;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_ITEMS; k++) {
        x[k] = b0 + k < n ? in[b0 + k] : T(0);
        v += x[k];
    }
    T tot;
    T run = block_excl(v, &tot) + (sums ? sums[blockIdx.x] : T(0));
#pragma unroll
    for (uint32_t k = 0; k < SCAN_ITEMS; k++) {
        if (b0 + k < n) out[b0 + k] = run;
        run += x[k];
    }
}

template <typename T>
int scan_excl(Shard* s, const T* in, T* out, uint32_t n) {
    // (a single-pass decoupled look-back measured 1.5 % slower a step at
    // 2^20, profiles/r03/p25: its device-coherent status loads cost more than
    // the two launches it saves; removed in round 4)
    const uint32_t nt = (uint32_t)(((uint64_t)n + SCAN_TILE - 1) / SCAN_TILE);
    if (nt <= 1) {
        k_scan_apply<T><<<1, BLK, 0, s->stream>>>(in, out, n, nullptr);
    } else {
        TRY(s->cub_tmp.ensure((size_t)nt * sizeof(T)));
        T* sums = reinterpret_cast<T*>(s->cub_tmp.p);
        k_scan_tiles<T><<<nt, BLK, 0, s->stream>>>(in, n, sums);
        k_scan_sums<T><<<1, BLK, 0, s->stream>>>(sums, nt);
        k_scan_apply<T><<<nt, BLK, 0, s->stream>>>(in, out, n, sums);
    }
    HIP_TRY(hipGetLastError());
    return PSIM_OK;
}

// prepare's scan + descriptors: k_node_prep left its blocks' range sums in
// pscan[0..pgrid); k_desc sums the ones before its range and walks the range
// again
int scan_desc(Shard* s, const RoundArgs& a) {
    k_desc<<<(s->pgrid + DESC_RANGES - 1) / DESC_RANGES, PREP_BLK, 0, s->stream>>>(
        s->bound.p, s->pscan.p, s->pper, s->in_beg.p, s->cb.p, s->start.p, a, s->desc.p, s->obase.p, s->d_nact.p,
        s->btot.p, s->pgrid, s->pin_dev, s->desc_cap, s->ctl.p);
    HIP_TRY(hipGetLastError());
    return PSIM_OK;
}

// Wait for the shard's stream by polling an event: a blocking synchronise
// sleeps the host thread, and waking it cost ~100 us of idle GPU per round
int stream_wait(Shard* s) {
    HIP_TRY(hipEventRecord(s->wait_ev, s->stream));
    hipError_t e;
    while ((e = hipEventQuery(s->wait_ev)) == hipErrorNotReady) {
    }
    if (e != hipSuccess) {
        // an event query error is reported once and settled by a blocking
        // synchronise, which fails too if the stream itself has faulted
        static bool said = false;
        if (!said) std::fprintf(stderr, "psim: event query: %s; synchronising\n", hipGetErrorString(e));
        said = true;
        HIP_TRY(hipStreamSynchronize(s->stream));
    }
    return PSIM_OK;
}

template <typename T>
T read1(Shard* s, const T* p) {
    T v{};
    (void)hipMemcpyAsync(&v, p, sizeof(T), hipMemcpyDeviceToHost, s->stream);
    (void)stream_wait(s);
    return v;
}

int upload(Shard* s, DBuf<uint32_t>& b, const std::vector<uint32_t>& v) {
    TRY(b.ensure(v.size()));
    HIP_TRY(hipMemcpyAsync(b.p, v.data(), v.size() * 4, hipMemcpyHostToDevice, s->stream));
    return PSIM_OK;
}

struct RoundCtl {
    bool crashes = false;
    uint64_t bcast_clear = 0;           // message slots this round's broadcasts retire
};

// events + prepare for one shard; leaves `a` ready for k_consume.
// events = false: the round's events were applied already (the redo of a
// batch round, run_batch); batched: no host wait -- the outbox and route
// capacities stand and k_desc checks the outbox on the device (desc_cap)
int phase_events_prepare(psim_handle* h, Shard* s, const RoundCtl& ctl, RoundArgs& a, bool events = true,
                         bool batched = false) {
    const uint32_t n = s->n;
    if (events && h->faults_dirty) {    // interposition funs installed / removed
        std::vector<uint64_t> keys(h->nx_omit_s.begin(), h->nx_omit_s.end());
        keys.insert(keys.end(), h->nx_omit_r.begin(), h->nx_omit_r.end());
        TRY(s->faulted.ensure(h->N));
        TRY(s->omit.ensure(std::max<size_t>(keys.size(), 1)));
        HIP_TRY(hipMemcpyAsync(s->faulted.p, h->nx_faulted.data(), h->N, hipMemcpyHostToDevice, s->stream));
        if (!keys.empty())
            HIP_TRY(hipMemcpyAsync(s->omit.p, keys.data(), keys.size() * 8, hipMemcpyHostToDevice, s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));   // (the host vector goes out of scope)
    }
    a = make_args(h, s);
    a.crash_round = ctl.crashes;
    // the up-and-partition pairs change only with crash, start and partition
    // events (k_crash, k_join, the partition copy): rebuilt only then
    a.upart_dirty = !s->upart_valid ||
                    (events && (ctl.crashes || !h->pend_join.empty() || h->pend_part_set || h->pend_part_clear));
    // (a crash only disconnects, and a restarted peer's holders dropped it
    // in the EXIT of its crash round: neither wakes a quiet node)
    a.lazy_wake = !s->upart_valid || (events && (h->pend_part_set || h->pend_part_clear || h->faults_dirty ||
                                                 !h->pend_lv_a.empty()));
    s->upart_valid = true;
    if (events) {
        KTimer t(h, s, KT_EVENTS);
        if (ctl.crashes) {
            TRY(upload(s, s->ev_ids, h->pend_crash));
            k_crash<<<grid_for(h->pend_crash.size()), BLK, 0, s->stream>>>(
                s->flags.p, s->crash_bits.p, s->ev_ids.p, (uint32_t)h->pend_crash.size());
        }
        if (!h->pend_join.empty()) {
            TRY(upload(s, s->ev_ids, h->pend_join));
            TRY(upload(s, s->ev_contacts, h->pend_contact));
            k_join<<<grid_for(h->pend_join.size()), BLK, 0, s->stream>>>(
                a, s->start.p, s->ev_ids.p, s->ev_contacts.p, (uint32_t)h->pend_join.size(),
                h->cfg.persist_epoch);
        }
        if (!h->pend_lv_a.empty()) {
            TRY(upload(s, s->ev_ids, h->pend_lv_a));
            TRY(upload(s, s->ev_contacts, h->pend_lv_t));
            k_leave_set<<<grid_for(h->pend_lv_a.size()), BLK, 0, s->stream>>>(
                s->hdr.p, s->lo, s->n, s->ev_ids.p, s->ev_contacts.p, (uint32_t)h->pend_lv_a.size());
        }
        if (h->pend_part_clear) HIP_TRY(hipMemsetAsync(s->part.p, 0, h->N, s->stream));
        if (h->pend_part_set)
            HIP_TRY(hipMemcpyAsync(s->part.p, h->pend_part.data(), h->N, hipMemcpyHostToDevice, s->stream));
        if (!h->pend_b_root.empty()) {
            const uint32_t k = (uint32_t)h->pend_b_root.size();
            k_bcast_reset<<<grid_for(n), BLK, 0, s->stream>>>(s->hdr.p, n, (uint32_t)ctl.bcast_clear,
                                                               (uint32_t)(ctl.bcast_clear >> 32));
            TRY(upload(s, s->bc_roots, h->pend_b_root));
            TRY(upload(s, s->bc_msgs, h->pend_b_msg));
            HIP_TRY(hipMemcpyAsync(s->slots.p, h->slot_tab, sizeof h->slot_tab, hipMemcpyHostToDevice, s->stream));
            k_origin<<<grid_for(k), BLK, 0, s->stream>>>(s->origin.p, s->lo, n, s->bc_roots.p, s->bc_msgs.p, k,
                                                          s->flags.p, false, s->ctl.p);
        }
    }
    {
        KTimer t(h, s, KT_PREPARE);
        a.in_cb = s->cb.p;
        // grid-stride; 4096 blocks (16 waves per CU) keep the crash rounds'
        // dependent loads (active row -> members' flag bytes) in flight --
        // 512 blocks left 2 waves per SIMD and took 6.8 ms at 2^26 nodes
        // (contiguous ranges of pper nodes, a multiple of BLK: k_desc takes
        // DESC_RANGES consecutive ranges a block; 1024-thread blocks here
        // took 27.6 us against 21.5 at 2^20, profiles/r05/ab_log.txt r5r)
        {
            const uint32_t g = std::min<uint32_t>(std::max<uint32_t>(1, grid_for(n) / PREP_NPT), DESC_RANGES * PREP_BLK);
            s->pper = BLK * (uint32_t)(((uint64_t)n + (uint64_t)g * BLK - 1) / ((uint64_t)g * BLK));
            s->pgrid = std::max<uint32_t>(1, (uint32_t)(((uint64_t)n + s->pper - 1) / s->pper));
        }
        s->cgrid = std::min<uint32_t>(grid_for(n), h->consume_blocks);
        // one lane per possible working node (up to RELAY_MAX_BLOCKS, then grid-stride):
        // the relays are chains of dependent random loads, so latency wants lanes
        const bool hv = h->cfg.manager != PSIM_MANAGER_PLUGGABLE;
        s->rgrid = hv ? std::min<uint32_t>(grid_for(n), RELAY_MAX_BLOCKS) : 0;
        s->tgrid = hv && h->cfg.plumtree ? std::min<uint32_t>(grid_for(n), h->pt_blocks) : 0;
        s->sgrid = hv ? std::min<uint32_t>(grid_for(n), SHUF_MAX_BLOCKS) : 0;
        // (k_lite_half: two nodes per wave)
        const uint32_t lnodes = h->lite_half ? psim::lite_half_block() * 2 : psim::lite_block();
        s->lgrid = hv ? std::min<uint32_t>((uint32_t)((n + lnodes - 1) / lnodes), h->lite_blocks) : 0;
        const uint32_t qnodes = PTL_BLOCK;
        s->qgrid = hv && h->cfg.plumtree ? std::min<uint32_t>((uint32_t)((n + qnodes - 1) / qnodes), h->ptl_blocks) : 0;
        TRY(s->stat_part.ensure((size_t)(s->pgrid + s->cgrid + s->rgrid + s->tgrid + s->sgrid + s->lgrid + s->qgrid) *
                                NST));
        k_node_prep<<<s->pgrid, BLK, 0, s->stream>>>(a, s->bmask.p, s->bound.p, s->stat_part.p, s->ocnt.p,
                                                     s->btot.p, s->pper, s->pscan.p, s->gcnt.p, (uint32_t)s->gcnt.n);
        // (pscan: the ranges' sums of packed words; k_desc's last block sums them all)
        // obase[n] = the exact total (btot, summed by k_desc's last block)
        TRY(scan_desc(s, a));
        if (batched) goto args;
        TRY(stream_wait(s));                          // (k_desc stored the total in pin)
        if (s->pin[PIN_BIGIN]) { s->pin[PIN_BIGIN] = 0; return PSIM_ENOMEM; }   // an inbox count must fit 27 bits
        const uint64_t total = s->pin[PIN_TOTAL];
        if (total >= 0xFFFFFFFFull) return PSIM_ENOMEM;
        // the bound peaks on broadcast rounds and creeps up for many rounds:
        // each growth reserves 1.5x; the first round reserves the working
        // sizes instead (the constants above RESERVE_PER_NODE)
        uint64_t want = total + 1;
        int headroom = 2;
        const char* rcap_init = getenv("PSIM_RCAP_INIT");   // (test hook: a small route capacity
                                                            // exercises the regrow + reroute)
        if (local_route(h) && !s->rcap) {
            s->rcap = 4096;
            while (s->rcap < (uint64_t)n * RCAP_PER_NODE) s->rcap <<= 1;
            if (rcap_init) s->rcap = std::max<uint64_t>(16, strtoull(rcap_init, nullptr, 10));
        }
        if (!s->reserved) {
            s->reserved = true;
            size_t fr = 0, tot = 0;
            // (test hook: no reservation -- the outbox grows round by round,
            // inside batches through the abort word)
            if (!getenv("PSIM_NO_RESERVE") && hipMemGetInfo(&fr, &tot) == hipSuccess) {
                const uint64_t per_rec = sizeof(Msg) + 3 * sizeof(uint32_t) + sizeof(uint2);
                const uint64_t per_slot = sizeof(Msg) + sizeof(uint32_t);
                // (memory the current buffers hold comes back when they regrow)
                uint64_t avail = fr + (uint64_t)s->outbox.n * sizeof(Msg) + (uint64_t)s->okey.n * 4;
                // (PSIM_RESERVE_PER_NODE / PSIM_RCAP_RESERVE: other reservations,
                // for measurements of the memory a workload needs)
                static const uint64_t res_pn = getenv("PSIM_RESERVE_PER_NODE")
                                                   ? strtoull(getenv("PSIM_RESERVE_PER_NODE"), nullptr, 10) : RESERVE_PER_NODE;
                static const uint64_t rcap_pn = getenv("PSIM_RCAP_RESERVE")
                                                    ? strtoull(getenv("PSIM_RCAP_RESERVE"), nullptr, 10) : RCAP_RESERVE;
                if (local_route(h) && !rcap_init) {
                    const uint64_t rc = (uint64_t)n * rcap_pn;
                    if (rc > s->rcap && (double)(rc * per_rec) <= RCAP_FREE_FRAC * (double)avail) s->rcap = rc;
                    const uint64_t held = s->rcap * per_rec;
                    avail = avail > held ? avail - held : 0;
                }
                const uint64_t r = std::min<uint64_t>((uint64_t)n * res_pn,
                                                      (uint64_t)((1.0 - OUTBOX_SPARE) * (double)avail) / per_slot);
                if (r > want) {
                    want = r;
                    headroom = -1;
                    s->outbox.release();            // (its memory is part of avail)
                    s->okey.release();
                }
            }
        } else if (want > s->outbox.n && s->outbox.n * sizeof(Msg) > (1ull << 30)) {
            std::fprintf(stderr, "psim: round %llu: outbox grows past its reservation (%zu -> %llu slots)\n",
                         (unsigned long long)h->round, s->outbox.n, (unsigned long long)want);
        }
        TRY(s->outbox.ensure(want, headroom));
        TRY(s->okey.ensure(want, headroom));
        if (local_route(h)) TRY(route_buffers(s, s->m_in == 0));   // the route checks its capacity on the device
    }
args:
    a.in_beg = s->in_beg.p;
    a.desc = s->desc.p; a.n_alist = s->d_nact.p;
    a.rec_in = s->inbox.p;
    a.obase = s->obase.p;
    a.rec_out = s->outbox.p;
    a.okey = s->okey.p; a.ocnt = s->ocnt.p;
    a.stat_part = s->stat_part.p + (size_t)s->pgrid * NST;
    a.stat_relay = s->stat_part.p + (size_t)(s->pgrid + s->cgrid) * NST;
    a.stat_pt = s->stat_part.p + (size_t)(s->pgrid + s->cgrid + s->rgrid) * NST;
    a.stat_shuf = s->stat_part.p + (size_t)(s->pgrid + s->cgrid + s->rgrid + s->tgrid) * NST;
    a.stat_lite = s->stat_part.p + (size_t)(s->pgrid + s->cgrid + s->rgrid + s->tgrid + s->sgrid) * NST;
    a.stat_ptl = s->stat_part.p + (size_t)(s->pgrid + s->cgrid + s->rgrid + s->tgrid + s->sgrid + s->lgrid) * NST;
    return PSIM_OK;
}

void launch_lite(psim_handle* h, Shard* s, const RoundArgs& a, hipStream_t st) {
    if (h->lite_half) k_lite_half<<<s->lgrid, psim::lite_half_block(), 0, st>>>(a);
    else k_consume_lite<<<s->lgrid, psim::lite_block(), 0, st>>>(a);
}

int phase_consume(psim_handle* h, Shard* s, RoundArgs& a) {
    if (a.pl && a.strategy == PSIM_STRATEGY_FULL) {
        // snapshots: at most one per node plus one per inbox message
        uint64_t slots = (uint64_t)s->m_in + s->n + 1;
        if (slots > 0xFFFFFFFFull) return PSIM_ENOMEM;
        TRY(s->pay[s->pay_cur].ensure(slots * 2 * h->fw));
        if (h->tomb && !s->tomb_live) {
            // the first round with removes: last round's snapshots were
            // written without their remove rows
            DBuf<uint32_t>& in = s->pay[s->pay_cur ^ 1];
            const size_t rows = in.n / (2 * h->fw);
            if (rows)
                HIP_TRY(hipMemset2DAsync(in.p + h->fw, 2 * h->fw * 4, 0, h->fw * 4, rows, s->stream));
            s->tomb_live = true;
        }
        a.pay_out = s->pay[s->pay_cur].p;
        a.pay_in = s->pay[s->pay_cur ^ 1].p;
        a.pay_top = s->pay_top.p;
        a.pay_cap = (uint32_t)(s->pay[s->pay_cur].n / (2 * h->fw));
        HIP_TRY(hipMemsetAsync(s->pay_top.p, 0, 4, s->stream));
    }
    if (a.pl) {
        k_consume_pl<<<s->cgrid, BLK, 0, s->stream>>>(a);
    } else {
        // k_relay sorts the nodes with work: a lone SHUFFLE relay (and a
        // lazy tick) one lane each, more HyParView work one k_consume wave,
        // Plumtree work one k_pt wave after the node's HyParView phase
        k_relay<<<s->rgrid, BLK, 0, s->stream>>>(a);
        RoundArgs b = a;
        b.desc = s->desc_slow.p;
        b.n_alist = s->n_slow.p;
        // k_shuf, k_consume_lite and k_consume take k_relay's disjoint lists
        // and write only their own nodes' rows, records and stats rows: they
        // run side by side (k_shuf and k_consume, latency-bound at ~1 and
        // ~0.5 waves/SIMD, fill k_consume_lite's tail), then join before the
        // Plumtree phase.  PSIM_SERIAL_PHASE=1: one after another (A/B)
        // Serial in crash rounds: there k_consume carries the EXIT scans and
        // the crashed members' replacements of every holder (config E at
        // 2^26: 15 ms of wave work a round) and side by side with
        // k_consume_lite the two took longer than one after the other
        // (node-round phase 61.0 -> 68.3 ms, profiles/r03/p36)
        // Since round 4 (k_lite_half) the kernels run one after another by
        // default: side by side with k_lite_half's 128-VGPR waves the phase
        // took 0.61 ms against 0.58 serially, and the step 0.84 against 0.77
        // (profiles/r04/p8); PSIM_CONCURRENT_PHASE=1 restores the side streams
        // outside crash rounds (and, with the wave kernel, PSIM_LITE_WAVE=1)
        static const bool conc_env = getenv("PSIM_CONCURRENT_PHASE") != nullptr;
        static const bool serial_env = getenv("PSIM_SERIAL_PHASE") != nullptr;
        const bool serial = serial_env || a.crash_round || !(conc_env || !h->lite_half);
        if (serial) {
            k_shuf<<<s->sgrid, BLK, 0, s->stream>>>(a);
            launch_lite(h, s, a, s->stream);
            k_consume<<<s->cgrid, BLK, 0, s->stream>>>(b);
        } else {
            HIP_TRY(hipEventRecord(s->fork_ev, s->stream));
            HIP_TRY(hipStreamWaitEvent(s->side[0], s->fork_ev, 0));
            HIP_TRY(hipStreamWaitEvent(s->side[1], s->fork_ev, 0));
            k_consume<<<s->cgrid, BLK, 0, s->side[0]>>>(b);
            k_shuf<<<s->sgrid, BLK, 0, s->side[1]>>>(a);
            launch_lite(h, s, a, s->stream);
            for (int k = 0; k < 2; k++) {
                HIP_TRY(hipEventRecord(s->join_ev[k], s->side[k]));
                HIP_TRY(hipStreamWaitEvent(s->stream, s->join_ev[k], 0));
            }
        }
        if (s->qgrid) {
            k_ptl<<<s->qgrid, PTL_BLOCK, 0, s->stream>>>(a);
        }
        if (s->tgrid) {
            RoundArgs c = a;
            c.desc = s->desc_pt.p;
            c.n_alist = s->n_pt.p;
            c.stat_part = a.stat_pt;
            k_pt<<<s->tgrid, BLK, 0, s->stream>>>(c);
        }
    }
    HIP_TRY(hipGetLastError());
    s->pay_cur ^= 1;
    return PSIM_OK;
}

// The route (section comment above the kernels) over this shard's outbox
// runs (dense == nullptr) or the m records of `dense`; leaves cb, bmask,
// in_beg[0..n] (in_beg[n] = the record count), the sorted runs of source
// indices in ivals and the records themselves in the inbox in run order:
// k_consume reads each node's messages as one contiguous run.  No host
// synchronisation.
// where the first kernel after the HyParView node-round phase stamps the
// phase's end (RoundArgs::ktime[1]); the pluggable kernel keeps its own span
unsigned long long* phase_end_mark(psim_handle* h, Shard* s) {
    return h->cfg.manager == PSIM_MANAGER_PLUGGABLE ? nullptr
                                                    : reinterpret_cast<unsigned long long*>(s->stat_out.p + NST) + 1;
}

int route_group(psim_handle* h, Shard* s, bool dense, uint32_t m, bool fixed = false, bool exact = false) {
    const uint32_t n = s->n;
    // buckets of 2^wshift destinations, one k_bucket_route block each, at
    // most 16 K of them (the two passes' LDS histograms: 4 B per bucket).
    // Up to 2^22 nodes 2048-node buckets: twice the route's blocks (one per
    // CU at 2^20 with 4096) -- k_bucket_route 64 -> 56 us, the histogram
    // passes +4 us, the step 0.667 -> 0.663 ms (profiles/r05/ab_log.txt r5o);
    // in round 3, before the gather moved into the route, 1024-node buckets
    // measured 1 % slower a step (profiles/r03/ab_log.txt, p17)
    uint32_t wshift = n > (1u << 26) ? 13 : n > (1u << 22) ? 12 : 11;
    if (const char* e = getenv("PSIM_ROUTE_WSHIFT")) {  // (another bucket width, for measurements)
        const int v = atoi(e);
        if (v >= (int)WSHIFT_MIN && v <= (int)WSHIFT_MAX) wshift = (uint32_t)v;
    }
    const uint32_t W = 1u << wshift, nb = (n + W - 1) >> wshift;
    const RouteIn in{s->outbox.p, s->okey.p, s->obase.p, s->ocnt.p, dense ? m : n, s->lo,
                     h->cfg.manager == PSIM_MANAGER_PLUGGABLE, dense ? s->recvh.p : nullptr,
                     dense ? s->recvt.p : nullptr, dense && !fixed ? s->wseg.p : nullptr, dense ? h->G : 0u,
                     fixed ? s->xcap_h : 0u, fixed ? s->xcap_t : 0u, (uint32_t)h->round};
    const uint32_t nsteps = std::max<uint32_t>(1, (in.n_src + RB_STEP - 1) / RB_STEP);
    const uint32_t nblk = std::min<uint32_t>(nsteps, h->rb_blocks);
    const size_t nh = (size_t)nb * nblk;
    TRY(s->hist.ensure(nh));
    TRY(s->hoff.ensure(nh));
    TRY(s->rtot.ensure(nb));
    TRY(s->rbase.ensure(nb + 1));
    // (k_bucket_route: 16 W bytes, and at W = 2^11 the bucket's source
    // indices in LDS too when they fit -- 68 KiB a block, two blocks a CU;
    // PSIM_ROUTE_LIDX=0: in memory, for A/B)
    static const bool lidx_ok = !getenv("PSIM_ROUTE_LIDX") || atoi(getenv("PSIM_ROUTE_LIDX")) != 0;
    const uint32_t lcap = lidx_ok && W == (1u << WSHIFT_MIN) ? ROUTE_LIDX : 0u;
    const size_t lds_h = (size_t)nb * 4, lds_r = (size_t)W * 16 + (size_t)lcap * 4;
    // the round's stats rows (every node-phase kernel's blocks) are complete
    const uint32_t rows = s->pgrid + s->cgrid + s->rgrid + s->tgrid + s->sgrid + s->lgrid + s->qgrid;
    // (a batched rank round, fixed: the stats came summed in the message
    // headers -- k_bucket_hist's block 0 adds them up, no tiles here)
    const StatsIn st{s->stat_part.p, rows,
                     fixed ? 0u : std::min<uint32_t>(nblk, std::min<uint32_t>(STAT_TILES, std::max<uint32_t>(1, rows / 32))),
                     s->stat_tile.p, s->stat_out.p, s->pin_dev + (size_t)s->stat_slot * PIN_STRIDE,
                     s->outx.p ? s->outx_top.p : nullptr, s->pin_dev};
    KTimer t(h, s, KT_SORT);
    // (up to 2^26 nodes: the fused route's fixed bucket regions hold 1.5x the
    // route's pairs, ~3 GB more than the four passes at 2^26 nodes -- room
    // since round 6's tighter outbox bound, 296 -> 274 GB for E at 2^26;
    // beyond, the four passes)
    if (!dense && !exact && h->route_fused && n <= (1u << 26)) {
        // a bucket's fixed region holds 1.5x its share of the route's
        // capacity: only a hot spot (a join storm) overflows one, and that
        // round goes through the four passes again (run_round, run_batch)
        const uint64_t capb64 = (s->rcap + nb - 1) / nb * 3 / 2 + 64;
        const uint32_t capb = (uint32_t)std::min<uint64_t>(capb64, 0xFFFFFFFFull / nb);
        if (s->gcnt.n < nb) {
            TRY(s->gcnt.ensure(nb));
            HIP_TRY(hipMemsetAsync(s->gcnt.p, 0, s->gcnt.n * 4, s->stream));
        }
        TRY(s->pairs.ensure((size_t)nb * capb));
        TRY(s->rank.ensure((size_t)nb * capb));
        static const uint32_t walk = getenv("PSIM_FILL_WALK") && atoi(getenv("PSIM_FILL_WALK")) ? 1u : 0u;
        k_bucket_fill<false><<<nblk, RB_STEP, lds_h, s->stream>>>(in, nsteps, nb, wshift, s->gcnt.p, capb, s->pairs.p,
                                                                  s->ctl.p, phase_end_mark(h, s), st, walk);
        k_bucket_route<false><<<nb, RR_THREADS, lds_r, s->stream>>>(
            n, wshift, h->rr_reg, nullptr, s->pairs.p, in.rec, nullptr, nullptr, s->rank.p, s->cb.p, s->bmask.p,
            s->in_beg.p, s->ivals.p, s->tmp.p, s->inbox.p, s->pin_dev + PIN_M, s->rcap, s->ctl.p, s->gcnt.p, capb,
            s->batch_round1, st, lcap);
        HIP_TRY(hipGetLastError());
        return PSIM_OK;
    }
    if (dense)
        k_bucket_hist<true><<<nblk, RB_STEP, lds_h, s->stream>>>(in, nsteps, nb, wshift, s->hist.p, s->ctl.p,
                                                                 nullptr, st);
    else    // (G == 1: the first kernel after the node-round phase stamps its end)
        k_bucket_hist<false><<<nblk, RB_STEP, lds_h, s->stream>>>(in, nsteps, nb, wshift, s->hist.p, s->ctl.p,
                                                                  phase_end_mark(h, s), st);
    k_bucket_offsets<<<nb, RB_MAX_BLOCKS, 0, s->stream>>>(s->hist.p, nblk, s->hoff.p, s->rtot.p, s->ctl.p);
    if (dense)
        k_bucket_scatter<true><<<nblk, RB_STEP, lds_h, s->stream>>>(in, nsteps, nb, wshift, s->hoff.p, s->rtot.p,
                                                                    s->rbase.p, s->pairs.p, s->rcap,
                                                                    s->pin_dev + PIN_OVF, s->ctl.p,
                                                                    s->batch_round1, st);
    else
        k_bucket_scatter<false><<<nblk, RB_STEP, lds_h, s->stream>>>(in, nsteps, nb, wshift, s->hoff.p, s->rtot.p,
                                                                     s->rbase.p, s->pairs.p, s->rcap,
                                                                     s->pin_dev + PIN_OVF, s->ctl.p,
                                                                     s->batch_round1, st);
    if (dense)
        k_bucket_route<true><<<nb, RR_THREADS, lds_r, s->stream>>>(
            n, wshift, h->rr_reg, s->rbase.p, s->pairs.p, nullptr, in.wire, in.tails, s->rank.p, s->cb.p, s->bmask.p,
            s->in_beg.p, s->ivals.p, s->tmp.p, s->inbox.p, s->pin_dev + PIN_M, s->rcap, s->ctl.p, nullptr, 0u,
            s->batch_round1, st, lcap);
    else
        k_bucket_route<false><<<nb, RR_THREADS, lds_r, s->stream>>>(
            n, wshift, h->rr_reg, s->rbase.p, s->pairs.p, in.rec, nullptr, nullptr, s->rank.p, s->cb.p, s->bmask.p,
            s->in_beg.p, s->ivals.p, s->tmp.p, s->inbox.p, s->pin_dev + PIN_M, s->rcap, s->ctl.p, nullptr, 0u,
            s->batch_round1, st, lcap);
    HIP_TRY(hipGetLastError());
    return PSIM_OK;
}

// the route's buffers for rcap records (and the current inbox too when it
// holds nothing yet)
int route_buffers(Shard* s, bool both_inboxes) {
    const size_t c = s->rcap + 1;
    TRY(s->ivals.ensure(c)); TRY(s->tmp.ensure(c)); TRY(s->rank.ensure(c)); TRY(s->pairs.ensure(c));
    // the inbox may hold this round's records (the first round after a
    // restore): a growth keeps them
    (void)both_inboxes;
    TRY(s->inbox.ensure_keep(c, s->m_in, s->stream));
    return PSIM_OK;
}

// G == 1: the outbox runs grouped by destination are the whole route
// (m_in: read back with the round's stats; ivals, pairs, rank, tmp and the
// inbox were sized in prepare by the outbox total, which bounds it)
// exact: the four-pass route (a reroute after an overflow of the fused one)
int phase_route_local(psim_handle* h, Shard* s, bool exact = false) { return route_group(h, s, false, 0, false, exact); }

void send_counts(Shard* s, uint32_t G);

// G > 1, sender side: the outbox partitioned by owner shard into the send
// buffer in the wire format (k_owner_part); per-owner counts/offsets on the host
// fixed: a batched rank round (run_batch_ranked) -- the fixed layout of
// s->xcap_h / xcap_t per owner, nothing read back (the buffers were sized for
// the batch)
int phase_partition(psim_handle* h, Shard* s, bool fixed = false) {
    const uint32_t G = h->G;
    RouteIn in{};
    in.rec = s->outbox.p; in.okey = s->okey.p; in.obase = s->obase.p; in.ocnt = s->ocnt.p; in.n_src = s->n;
    const uint32_t nsteps = std::max<uint32_t>(1, (s->n + RB_STEP - 1) / RB_STEP);
    const uint32_t spb = (nsteps + h->rb_blocks - 1) / h->rb_blocks;    // consecutive steps per block
    const uint32_t nblk = (nsteps + spb - 1) / spb;
    const size_t nh = (size_t)2 * G * nblk + 1;
    TRY(s->hist.ensure(nh));
    TRY(s->hoff.ensure(nh));
    if (!fixed) TRY(s->sendbuf.ensure(2 * (s->pin[PIN_TOTAL] + 1), 2));   // (the outbox bound bounds the records)
    TRY(s->d_off.ensure(2 * G + 1));
    const bool rccl = h->ranked;
    if (rccl) TRY(h->comm_cnt.ensure(2 * G + 2));   // (send and receive counts, then 2 words of phase_stats)
    s->soff.assign(2 * G + 1, 0);
    const uint32_t capH = fixed ? s->xcap_h : 0u, capT = fixed ? s->xcap_t : 0u;
    // a batched round's stats: tiles from the count pass, summed into the
    // message headers by k_owner_offsets (the route sums the received ones)
    StatsIn st{};
    if (fixed) {
        const uint32_t rows = s->pgrid + s->cgrid + s->rgrid + s->tgrid + s->sgrid + s->lgrid + s->qgrid;
        st = StatsIn{s->stat_part.p, rows,
                     std::min<uint32_t>(nblk, std::min<uint32_t>(STAT_TILES, std::max<uint32_t>(1, rows / 32))),
                     s->stat_tile.p, s->stat_out.p, s->pin_dev + (size_t)s->stat_slot * PIN_STRIDE,
                     s->outx.p ? s->outx_top.p : nullptr, s->pin_dev};
    }
    {
        KTimer t(h, s, KT_SORT);
        k_owner_part<false><<<nblk, RB_STEP, 0, s->stream>>>(in, nsteps, spb, G, h->per, s->hist.p, nullptr,
                                                              nullptr, phase_end_mark(h, s), capH, capT, s->ctl.p, st);
        TRY(scan_excl(s, s->hist.p, s->hoff.p, (uint32_t)nh));
        k_owner_part<true><<<nblk, RB_STEP, 0, s->stream>>>(in, nsteps, spb, G, h->per, nullptr, s->hoff.p,
                                                             s->sendbuf.p, nullptr, capH, capT, s->ctl.p, StatsIn{});
        k_owner_offsets<<<1, OO_THREADS, 0, s->stream>>>(s->hoff.p, nblk, G, s->d_off.p, rccl ? h->comm_cnt.p : nullptr,
                                                  rccl ? s->stat_out.p + STAT_OUT_X : nullptr, capH, capT, s->ctl.p,
                                                  (uint32_t)h->round, s->idx, s->sendbuf.p, st);
        HIP_TRY(hipGetLastError());
        // an RCCL rank reads the offsets back with the received counts, after
        // the count all-to-all (exchange_rccl): one host wait a round, not two
        if (rccl) return PSIM_OK;
        HIP_TRY(hipMemcpyAsync(s->soff.data(), s->d_off.p, (2 * G + 1) * 8, hipMemcpyDeviceToHost, s->stream));
        TRY(stream_wait(s));
    }
    send_counts(s, G);
    return PSIM_OK;
}

// per owner the heads and the tails this shard sends (from soff)
void send_counts(Shard* s, uint32_t G) {
    s->scnt.resize(G);
    s->lcnt.resize(G);
    for (uint32_t g = 0; g < G; g++) {
        s->scnt[g] = s->soff[g + 1] - s->soff[g];
        s->lcnt[g] = s->soff[G + g + 1] - s->soff[G + g];
    }
}

// G > 1, receiver side: heads and tails from the G sources (hc[g] / lc[g]
// each), already in recvh / recvt in source order; the source table, then
// the route over the heads
int phase_receive(psim_handle* h, Shard* s, const std::vector<uint64_t>& hc, const std::vector<uint64_t>& lc) {
    const uint32_t G = h->G;
    s->wseg_host.assign(2 * (G + 1), 0);
    uint64_t m = 0, ml = 0;
    for (uint32_t g = 0; g < G; g++) {
        s->wseg_host[g] = (uint32_t)m;
        s->wseg_host[G + 1 + g] = (uint32_t)ml;
        m += hc[g];
        ml += lc[g];
    }
    s->wseg_host[G] = (uint32_t)m;
    s->wseg_host[2 * G + 1] = (uint32_t)ml;
    TRY(s->wseg.ensure(2 * (G + 1)));
    // (the host vector lives until the next round's receive: the copy is
    // ordered on the stream before the route reads it)
    HIP_TRY(hipMemcpyAsync(s->wseg.p, s->wseg_host.data(), s->wseg_host.size() * 4, hipMemcpyHostToDevice,
                           s->stream));
    s->rcap = std::max<uint64_t>(s->rcap, m);   // exact: the count is on the host here
    TRY(route_buffers(s, false));
    TRY(route_group(h, s, true, (uint32_t)m));
    s->m_in = (uint32_t)m;
    return PSIM_OK;
}

// virtual shards of this process: device copies between shard buffers
int exchange_local(psim_handle* h) {
    const uint32_t G = h->G;
    for (Shard* d : h->shards) {
        std::vector<uint64_t> hc(G), lc(G);
        uint64_t m = 0, ml = 0;
        for (Shard* s : h->shards) {
            hc[s->idx] = s->scnt[d->idx];
            lc[s->idx] = s->lcnt[d->idx];
            m += hc[s->idx];
            ml += lc[s->idx];
        }
        TRY(d->recvh.ensure(m + 1));
        TRY(d->recvt.ensure(ml + 1));
        {
            KTimer t(h, d, KT_EXCHANGE);
            uint64_t oh = 0, ot = 0;
            for (uint32_t g = 0; g < G; g++) {  // concatenation in source-shard order
                Shard* s = h->shards[g];
                if (hc[g])
                    HIP_TRY(hipMemcpyAsync(d->recvh.p + oh, s->sendbuf.p + s->soff[d->idx], hc[g] * sizeof(Wire),
                                           hipMemcpyDeviceToDevice, d->stream));
                if (lc[g])
                    HIP_TRY(hipMemcpyAsync(d->recvt.p + ot, s->sendbuf.p + s->soff[G + d->idx], lc[g] * sizeof(Wire),
                                           hipMemcpyDeviceToDevice, d->stream));
                if (g != d->idx) {
                    h->x_records += hc[g];
                    h->x_bytes += (hc[g] + lc[g]) * sizeof(Wire);
                }
                oh += hc[g];
                ot += lc[g];
            }
        }
        TRY(phase_receive(h, d, hc, lc));
    }
    return PSIM_OK;
}

// one shard per RCCL rank: counts by all-to-all, records by grouped send/recv
// (per peer its heads, then its tails)
int exchange_rccl(psim_handle* h) {
    Shard* s = h->shards[0];
    const uint32_t G = h->G;
    std::vector<uint64_t> hc(G), lc(G);
    {
        KTimer t(h, s, KT_EXCHANGE);
        // (k_owner_offsets wrote this rank's counts into comm_cnt[0, G))
        TRY(h->comm->all_to_all_u64(h->comm_cnt.p, h->comm_cnt.p + G, 1, s->stream));
        std::vector<uint64_t> rcnt(G);
        HIP_TRY(hipMemcpyAsync(rcnt.data(), h->comm_cnt.p + G, G * 8, hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(hipMemcpyAsync(s->soff.data(), s->d_off.p, (2 * G + 1) * 8, hipMemcpyDeviceToHost, s->stream));
        TRY(stream_wait(s));
        send_counts(s, G);
        uint64_t m = 0, ml = 0;
        std::vector<uint64_t> roh(G), rot(G);
        for (uint32_t g = 0; g < G; g++) {
            hc[g] = rcnt[g] & 0xFFFFFFFFull;
            lc[g] = rcnt[g] >> 32;
            roh[g] = m;
            rot[g] = ml;
            m += hc[g];
            ml += lc[g];
        }
        TRY(s->recvh.ensure(m + 1));
        TRY(s->recvt.ensure(ml + 1));
        std::vector<Xfer> sends, recvs;
        // a rank's own records: device copies, except in a one-rank world
        // (the diagnostic of the RCCL path), where the self send / receive
        // pairs go through the library like any other peer's
        const bool self_comm = h->world == 1;
        for (uint32_t g = 0; g < G; g++) {
            if (g == s->idx && !self_comm) continue;
            if (s->scnt[g]) sends.push_back({(int)g, s->sendbuf.p + s->soff[g], s->scnt[g] * sizeof(Wire)});
            if (s->lcnt[g]) sends.push_back({(int)g, s->sendbuf.p + s->soff[G + g], s->lcnt[g] * sizeof(Wire)});
            if (hc[g]) recvs.push_back({(int)g, s->recvh.p + roh[g], hc[g] * sizeof(Wire)});
            if (lc[g]) recvs.push_back({(int)g, s->recvt.p + rot[g], lc[g] * sizeof(Wire)});
            h->x_records += s->scnt[g];
            h->x_bytes += (s->scnt[g] + s->lcnt[g]) * sizeof(Wire);
        }
        TRY(h->comm->exchange(sends, recvs, s->stream));
        if (!self_comm) {
            const uint32_t g = s->idx;
            if (hc[g])
                HIP_TRY(hipMemcpyAsync(s->recvh.p + roh[g], s->sendbuf.p + s->soff[g], hc[g] * sizeof(Wire),
                                       hipMemcpyDeviceToDevice, s->stream));
            if (lc[g])
                HIP_TRY(hipMemcpyAsync(s->recvt.p + rot[g], s->sendbuf.p + s->soff[G + g], lc[g] * sizeof(Wire),
                                       hipMemcpyDeviceToDevice, s->stream));
        }
    }
    return phase_receive(h, s, hc, lc);
}

// A batched rank round (run_batch_ranked): no host wait.  The counts go
// through the all-to-all as always, but the records travel in fixed-size
// messages -- per peer xcap_h heads and xcap_t tails, identical on every rank
// -- so nothing is sized on the host; the receiver's route reads each
// source's region up to the count it received (the fixed layout of RouteIn).
// A sender whose owner count passed a capacity aborted the round
// (k_owner_offsets, code 3) and every rank redoes it exactly
// (run_batch_ranked).  The padding crosses the link too: a capacity is the
// largest per-owner count seen so far, 1.25x (xcaps_update).
int exchange_fixed(psim_handle* h) {
    Shard* s = h->shards[0];
    const uint32_t G = h->G, capT = s->xcap_t;
    const size_t xs = XHDR + s->xcap_h;               // (a message: its header, then the heads)
    KTimer t(h, s, KT_EXCHANGE);
    std::vector<Xfer> sends, recvs;
    const bool self_comm = h->world == 1;
    for (uint32_t g = 0; g < G; g++) {
        if (g == s->idx && !self_comm) continue;
        sends.push_back({(int)g, s->sendbuf.p + g * xs, xs * sizeof(Wire)});
        sends.push_back({(int)g, s->sendbuf.p + G * xs + (size_t)g * capT, (size_t)capT * sizeof(Wire)});
        recvs.push_back({(int)g, s->recvh.p + g * xs, xs * sizeof(Wire)});
        recvs.push_back({(int)g, s->recvt.p + (size_t)g * capT, (size_t)capT * sizeof(Wire)});
    }
    TRY(h->comm->exchange(sends, recvs, s->stream));
    if (!self_comm) {
        const uint32_t g = s->idx;
        HIP_TRY(hipMemcpyAsync(s->recvh.p + g * xs, s->sendbuf.p + g * xs, xs * sizeof(Wire), hipMemcpyDeviceToDevice,
                               s->stream));
        HIP_TRY(hipMemcpyAsync(s->recvt.p + (size_t)g * capT, s->sendbuf.p + G * xs + (size_t)g * capT,
                               (size_t)capT * sizeof(Wire), hipMemcpyDeviceToDevice, s->stream));
    }
    return route_group(h, s, true, (uint32_t)(G * xs), true);
}

// the fixed capacities of the next batch from the largest per-owner head /
// tail counts of any rank over a batch's rounds (every rank's own, in the
// headers or the all-reduced stats: the same on every rank): 1.5x and 1024
// more -- raised at once, lowered only once the batch's largest count falls
// below half the capacity (the padding crosses the links: a broadcast's peak
// should not fix it for good)
// (grow: a batch stopped on a count past its capacity -- the traffic is
// climbing, a broadcast's wave: 2x headroom, so the next batch is likelier to
// get through)
// (shrink = false: one exact round's counts only raise them)
void xcaps_set(Shard* s, uint64_t mh, uint64_t mt, bool grow = false, bool shrink = true) {
    const uint64_t ch = std::min<uint64_t>(grow ? 2 * mh + 1024 : mh + mh / 2 + 1024, 0x7FFFFFFFull);
    const uint64_t ct = std::min<uint64_t>(grow ? 2 * mt + 1024 : mt + mt / 2 + 1024, 0x7FFFFFFFull);
    if (ch > s->xcap_h || (shrink && 2 * mh < s->xcap_h)) s->xcap_h = (uint32_t)ch;
    if (ct > s->xcap_t || (shrink && 2 * mt < s->xcap_t)) s->xcap_t = (uint32_t)ct;
}
void xcaps_max(psim_handle* h, const uint64_t* p, uint64_t& mh, uint64_t& mt) {
    for (int r = 0; r < h->world && r < 64; r++) {
        mh = std::max<uint64_t>(mh, p[PIN_XRANK + r]);
        mt = std::max<uint64_t>(mt, p[PIN_XRANK + 64 + r]);
    }
}
void xcaps_update(psim_handle* h, Shard* s, const uint64_t* p) {
    uint64_t mh = 0, mt = 0;
    xcaps_max(h, p, mh, mt);
    xcaps_set(s, mh, mt, false, false);
}

// the round's end after its route (which summed the stats: StatsIn)
// batched: a batched rank round -- its stats came in the message headers
int phase_stats(psim_handle* h, Shard* s, const std::vector<uint32_t>& crashed, bool batched = false) {
    KTimer t(h, s, KT_STATS);
    if (h->ranked && !batched) {
        // the ranks' sums reduced on the device, on the shard's stream, and
        // stored over the pinned words: the end of the round waits once
        // (a host copy, an all-reduce and a second wait after it before).
        // The x-words go with them: whether a rank's round aborted (a batch),
        // the largest per-owner counts (the next batch's capacities)
        uint64_t* pw = s->pin_dev + (size_t)s->stat_slot * PIN_STRIDE;
        TRY(h->comm->all_reduce(s->stat_out.p, STAT_OUT_N, CType::U64, COp::SUM, s->stream));
        HIP_TRY(hipMemcpyAsync(pw, s->stat_out.p, NST * 8, hipMemcpyDeviceToDevice, s->stream));
        HIP_TRY(hipMemcpyAsync(pw + PIN_XRANK, s->stat_out.p + STAT_OUT_R, 128 * 8, hipMemcpyDeviceToDevice, s->stream));
    }
    if (!crashed.empty()) {
        TRY(upload(s, s->ev_ids, crashed));
        k_uncrash<<<grid_for(crashed.size()), BLK, 0, s->stream>>>(s->flags.p, s->crash_bits.p, s->ev_ids.p,
                                                                  (uint32_t)crashed.size(), s->ctl.p);
    }
    return PSIM_OK;
}

// the host side of a round's broadcast events: message slots, the tracked id
void bcast_slots(psim_handle* h, RoundCtl& ctl) {
    if (!h->pend_b_root.empty()) {
        // each broadcast takes its message slot (the previous id of the slot
        // retires); the roots' origin entries are set on the device after the
        // round's crash and start events (k_origin); the last is tracked
        for (size_t i = 0; i < h->pend_b_root.size(); i++) {
            const uint32_t k = h->pend_b_msg[i] % PSIM_MSG_SLOTS;
            ctl.bcast_clear |= 1ull << k;
            h->slot_tab[k] = h->pend_b_msg[i];
            h->slot_tab[PSIM_MSG_SLOTS + k] = h->pend_b_root[i] | PSIM_MAP_BIT;
        }
        h->tracked_msg = h->pend_b_msg.back();
    }
}

// One round, waited for.  events_applied: the pending events went to the
// device already (the redo of an aborted batch round): only their
// round-end halves run (crash-round EXIT checks, k_uncrash, origins spent).
// from_partition: the node-round phase ran already (a rank's redo of an
// aborted batch round, run_batch_ranked): the round goes on from its owner
// partition, over the outbox that phase left.
int run_round(psim_handle* h, uint64_t* st, bool events_applied = false, bool from_partition = false) {
    RoundCtl ctl;
    ctl.crashes = !h->pend_crash.empty();
    if (!events_applied) bcast_slots(h, ctl);
    if (h->faults_dirty) {              // the funs in force from this round
        if (h->nx_faulted.size() != h->N) h->nx_faulted.assign(h->N, 0);
        h->n_omit_s = (uint32_t)h->nx_omit_s.size();
        h->n_omit_r = (uint32_t)h->nx_omit_r.size();
        h->faults = h->n_omit_s || h->n_omit_r || h->nx_nfaulted;
    }
    for (Shard* s : h->shards) s->tn = 0;        // (timers of a round that failed)
    std::vector<RoundArgs> args(h->shards.size());   // (consume fills the payload arena fields)
    for (size_t i = 0; i < h->shards.size() && !from_partition; i++)
        TRY(phase_events_prepare(h, h->shards[i], ctl, args[i], !events_applied));
    // (test hook: this round fails half-way, after its events went to the
    // device, as an allocation failure inside a round would)
    static const long long fail_round = getenv("PSIM_TEST_FAIL_ROUND") ? atoll(getenv("PSIM_TEST_FAIL_ROUND")) : -1;
    if (fail_round >= 0 && h->round == (uint64_t)fail_round) {
        for (Shard* s : h->shards) (void)hipStreamSynchronize(s->stream);
        return PSIM_ENOMEM;
    }
    for (size_t i = 0; i < h->shards.size() && !from_partition; i++) TRY(phase_consume(h, h->shards[i], args[i]));
    if (local_route(h)) {
        TRY(phase_route_local(h, h->shards[0]));
    } else {
        for (Shard* s : h->shards) TRY(phase_partition(h, s));
        if (h->ranked) TRY(exchange_rccl(h));
        else TRY(exchange_local(h));
    }
    for (Shard* s : h->shards) {
        TRY(phase_stats(h, s, h->pend_crash));
        if (!h->pend_b_root.empty())        // this round's origins are spent
            k_origin<<<grid_for(h->pend_b_root.size()), BLK, 0, s->stream>>>(
                s->origin.p, s->lo, s->n, s->bc_roots.p, s->bc_msgs.p, (uint32_t)h->pend_b_root.size(), s->flags.p,
                true, s->ctl.p);
    }
    memset(st, 0, NST * 8);
    for (Shard* s : h->shards) {
        TRY(stream_wait(s));
        flush_timers(h, s);
        for (int k = 0; k < NST; k++) st[k] += s->pin[k];
        if (local_route(h) && s->pin[PIN_OVF]) {
            // the route found more records than its buffers hold: grow them
            // (1.5x, power of two) and route this round's outbox again
            const uint64_t m = s->pin[PIN_OVF];
            s->pin[PIN_OVF] = 0;
            if (s->rcap < m + m / 2) {
                // 1.5x, a power of two up to 2^26 records, then in 2^20 steps
                const uint64_t want = m + m / 2;
                if (want <= (1ull << 26)) while (s->rcap < want) s->rcap <<= 1;
                else s->rcap = (want + (1ull << 20) - 1) >> 20 << 20;
            }
            TRY(route_buffers(s, false));
            TRY(phase_route_local(h, s, true));
            TRY(stream_wait(s));
        }
        if (local_route(h)) s->m_in = (uint32_t)s->pin[PIN_M];   // routed this round
        if (h->ranked) xcaps_update(h, s, s->pin);   // (the next batch's exchange capacities)
        static const bool trace_relay = getenv("PSIM_TRACE_RELAY") != nullptr;
        if (trace_relay && s->rgrid)
        {
            uint64_t em = 0;
            for (int k = 0; k < ST_NTYPES; k++) em += s->pin[ST_EMIT + k];
            std::fprintf(stderr, "psim: round %llu shard %u: %u nodes with work, %u to k_consume, %u to k_pt, "
                         "%u to k_shuf, %u to k_consume_lite, %u to k_ptl, outbox bound %llu, emitted %llu\n",
                         (unsigned long long)h->round, s->idx, read1(s, s->d_nact.p), read1(s, s->n_slow.p),
                         read1(s, s->n_pt.p), read1(s, s->n_shuf.p), read1(s, s->n_lite.p) + read1(s, s->n_lite.p + 1) + read1(s, s->n_lite.p + 2) + read1(s, s->n_lite.p + 3),
                         read1(s, s->n_ptl.p) + read1(s, s->n_ptl.p + 1),
                         (unsigned long long)s->pin[PIN_TOTAL], (unsigned long long)em);
        }
        if (s->pin[NST] != ~0ull && s->pin[NST + 1] > s->pin[NST]) {   // 100 MHz ticks
            h->kt_ms[KT_CONSUME] += (double)(s->pin[NST + 1] - s->pin[NST]) * 1e-5;
            h->kt_n[KT_CONSUME]++;
        }
    }
    // (an RCCL rank's st[] is already the all-reduced sum: phase_stats)
    if (st[ST_BOUND]) {
        std::fprintf(stderr, "psim: round %llu: %llu nodes emitted past their outbox bound (engine bug)\n",
                     (unsigned long long)h->round, (unsigned long long)st[ST_BOUND]);
        return PSIM_EDEVICE;
    }
    for (uint32_t j : h->pend_join) h->pend_join_mark[j] = 0;
    h->pend_crash.clear(); h->pend_join.clear(); h->pend_contact.clear();
    h->pend_lv_a.clear(); h->pend_lv_t.clear();
    if (st[ST_STOP]) {
        // managers that stopped this round (psim_leave_node) are down from the
        // next round on: the next round's crash events, on every rank (the
        // count is the all-reduced one, so every rank of an RCCL handle is
        // here: its shard's list is all-gathered, padded to the longest)
        std::vector<uint32_t> ids;
        for (Shard* s : h->shards) {
            const size_t k = read1(s, s->n_stop.p);   // this shard's own (pin[] is the ranks' sum)
            if (!k) continue;
            const size_t at = ids.size();
            ids.resize(at + k);
            HIP_TRY(hipMemcpyAsync(ids.data() + at, s->stop_ids.p, k * 4, hipMemcpyDeviceToHost, s->stream));
            TRY(stream_wait(s));
        }
        if (h->ranked) {
            Shard* s = h->shards[0];
            const uint32_t W = h->world;
            std::vector<uint64_t> cnt(W), mine(ids.begin(), ids.end());
            const uint64_t k = mine.size();
            TRY(h->comm_cnt.ensure(W + 1));
            HIP_TRY(hipMemcpyAsync(h->comm_cnt.p + W, &k, 8, hipMemcpyHostToDevice, s->stream));
            TRY(h->comm->all_gather(h->comm_cnt.p + W, h->comm_cnt.p, 8, s->stream));
            HIP_TRY(hipMemcpyAsync(cnt.data(), h->comm_cnt.p, W * 8, hipMemcpyDeviceToHost, s->stream));
            TRY(stream_wait(s));
            const uint64_t mk = *std::max_element(cnt.begin(), cnt.end());
            mine.resize(mk, 0);
            std::vector<uint64_t> all((size_t)W * mk);
            TRY(h->comm_cnt.ensure((size_t)W * mk + mk));
            HIP_TRY(hipMemcpyAsync(h->comm_cnt.p + (size_t)W * mk, mine.data(), mk * 8, hipMemcpyHostToDevice,
                                   s->stream));
            TRY(h->comm->all_gather(h->comm_cnt.p + (size_t)W * mk, h->comm_cnt.p, mk * 8, s->stream));
            HIP_TRY(hipMemcpyAsync(all.data(), h->comm_cnt.p, all.size() * 8, hipMemcpyDeviceToHost, s->stream));
            TRY(stream_wait(s));
            ids.clear();
            for (uint32_t r = 0; r < W; r++)
                for (uint64_t j = 0; j < cnt[r]; j++) ids.push_back((uint32_t)all[(size_t)r * mk + j]);
        }
        std::sort(ids.begin(), ids.end());
        h->pend_crash.insert(h->pend_crash.end(), ids.begin(), ids.end());
    }
    h->pend_part_set = h->pend_part_clear = false;
    h->faults_dirty = false;
    h->pend_b_root.clear(); h->pend_b_msg.clear();
    h->round++;
    return PSIM_OK;
}

void fill_stats(const uint64_t* s, uint64_t round, psim_round_stats* o) {
    memset(o, 0, sizeof *o);
    o->round = round;
    for (int i = 0; i < ST_NTYPES; i++) {          // (types 22, 23: no slot, always 0)
        o->emitted[i] = s[ST_EMIT + i];
        o->delivered[i] = s[ST_DELIV + i];
    }
    o->dropped = s[ST_DROPPED]; o->nodes_up = s[ST_UP]; o->nodes_processed = s[ST_PROC];
    o->exits = s[ST_EXITS]; o->send_fail = s[ST_FAIL]; o->first_deliveries = s[ST_FIRST];
    o->overflow = s[ST_OVF]; o->digest = s[ST_DIGEST]; o->state_bytes = s[ST_BYTES];
    for (int k = 0; k < PSIM_OVF_NKINDS; k++) o->overflow_by[k] = s[ST_OVF_BY + k];
    o->omitted = s[ST_OMIT];
}

// Whether psim_step may run its rounds as batches (run_batch): one RCCL-free
// HyParView shard past its first round, no diagnostic mode that reads the
// device between kernels, no strict mode (it stops at the overflowing round)
bool batchable(psim_handle* h) {
    static const bool trace = getenv("PSIM_TRACE_RELAY") != nullptr;
    static const bool off = getenv("PSIM_NO_BATCH") != nullptr || getenv("PSIM_TEST_FAIL_ROUND") != nullptr;
    static const bool off_ranked = getenv("PSIM_NO_RANK_BATCH") != nullptr;
    if (off || trace || h->phase_timers || h->cfg.strict || h->cfg.manager == PSIM_MANAGER_PLUGGABLE ||
        !h->pend_lv_a.empty())
        return false;
    Shard* s = h->shards[0];
    // a rank batches once an exact round has set the exchange capacities.
    // Every rank must decide alike, so nothing local enters here (a rank that
    // has received no record yet has no route capacity: run_batch_ranked
    // sizes it) -- only the events, the config and the all-reduced caps
    if (h->ranked) return !off_ranked && s->reserved && s->outbox.n && s->xcap_h && s->xcap_t;
    return h->G == 1 && s->reserved && s->rcap && s->outbox.n;
}

// Up to BATCH_MAX rounds enqueued back to back with no host wait between
// them (the pending events go with the first), then one wait.  A round
// whose outbox bound passes the outbox capacity (k_desc, code 1) or whose
// records pass the route's (k_bucket_scatter, code 2) sets the abort word:
// every later kernel of the batch returns at once, the host grows the
// buffer and finishes that round waited for -- from prepare (code 1: nothing
// of it ran past k_desc) or from the route (code 2: its node phases ran).
// Returns the rounds done (>= 1) in *done; their stats in st_out.
int run_batch(psim_handle* h, uint32_t nb, psim_round_stats* st_out, uint32_t* done_out) {
    Shard* s = h->shards[0];
    const uint64_t r0 = h->round;
    RoundCtl ctl0;
    ctl0.crashes = !h->pend_crash.empty();
    bcast_slots(h, ctl0);
    const std::vector<uint32_t> crashed0 = h->pend_crash;
    const std::vector<uint32_t> none;
    const bool bc0 = !h->pend_b_root.empty();
    s->tn = 0;
    s->desc_cap = std::min<uint64_t>(s->outbox.n, s->okey.n);
    const auto t_enq = std::chrono::steady_clock::now();
    for (uint32_t j = 0; j < nb; j++) {
        s->stat_slot = j + 1;
        s->batch_round1 = (uint32_t)h->round + 1;
        RoundArgs a;
        const RoundCtl ctl = j == 0 ? ctl0 : RoundCtl{};
        TRY(phase_events_prepare(h, s, ctl, a, j == 0, true));
        TRY(phase_consume(h, s, a));
        TRY(phase_route_local(h, s));
        TRY(phase_stats(h, s, j == 0 ? crashed0 : none));
        if (j == 0 && bc0)                  // the first round's origins are spent
            k_origin<<<grid_for(h->pend_b_root.size()), BLK, 0, s->stream>>>(
                s->origin.p, s->lo, s->n, s->bc_roots.p, s->bc_msgs.p, (uint32_t)h->pend_b_root.size(), s->flags.p,
                true, s->ctl.p);
        HIP_TRY(hipGetLastError());
        h->round++;
    }
    s->stat_slot = 0; s->batch_round1 = 0; s->desc_cap = 0;
    uint32_t cw[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(cw, s->ctl.p, sizeof cw, hipMemcpyDeviceToHost, s->stream));
    const auto t_wait = std::chrono::steady_clock::now();
    TRY(stream_wait(s));
    static const bool trace_batch = getenv("PSIM_TRACE_BATCH") != nullptr;
    if (trace_batch)
        std::fprintf(stderr, "psim: batch of %u from round %llu: enqueue %.3f ms, wait %.3f ms\n", nb,
                     (unsigned long long)r0, std::chrono::duration<double, std::milli>(t_wait - t_enq).count(),
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_wait).count());
    if (s->pin[PIN_BIGIN]) {                          // a node's inbox count must fit 27 bits
        s->pin[PIN_BIGIN] = 0;
        HIP_TRY(hipMemsetAsync(s->ctl.p, 0, sizeof cw, s->stream));
        return PSIM_ENOMEM;                           // (psim_step marks the handle failed)
    }
    const uint32_t done = cw[0] ? (uint32_t)(cw[1] - r0) : nb;
    if (cw[0] && (cw[1] < r0 || done >= nb)) return PSIM_EDEVICE;
    for (uint32_t j = 0; j < done; j++) {
        const uint64_t* p = s->pin + (size_t)(j + 1) * PIN_STRIDE;
        if (p[ST_BOUND]) {
            std::fprintf(stderr, "psim: round %llu: %llu nodes emitted past their outbox bound (engine bug)\n",
                         (unsigned long long)(r0 + j), (unsigned long long)p[ST_BOUND]);
            return PSIM_EDEVICE;
        }
        if (st_out) fill_stats(p, r0 + j, &st_out[j]);
        if (p[NST] != ~0ull && p[NST + 1] > p[NST]) {     // 100 MHz ticks
            h->kt_ms[KT_CONSUME] += (double)(p[NST + 1] - p[NST]) * 1e-5;
            h->kt_n[KT_CONSUME]++;
        }
    }
    if (done > 0) {                           // the first round's events are spent
        for (uint32_t j : h->pend_join) h->pend_join_mark[j] = 0;
        h->pend_crash.clear(); h->pend_join.clear(); h->pend_contact.clear();
        h->pend_part_set = h->pend_part_clear = false;
        h->pend_b_root.clear(); h->pend_b_msg.clear();
        h->faults_dirty = false;
    }
    s->m_in = (uint32_t)s->pin[PIN_M];         // (the last route that ran)
    *done_out = done;
    if (!cw[0]) {
        h->round = r0 + nb;
        return PSIM_OK;
    }
    // round r0 + done stopped the batch: reset the word, grow, finish it
    HIP_TRY(hipMemsetAsync(s->ctl.p, 0, sizeof cw, s->stream));
    h->round = r0 + done;
    uint64_t st[NST];
    if (cw[0] == 1) {
        const uint64_t total = s->pin[PIN_TOTAL];
        if (total >= 0xFFFFFFFFull) return PSIM_ENOMEM;
        std::fprintf(stderr, "psim: round %llu: outbox grows past its capacity (%zu -> %llu slots)\n",
                     (unsigned long long)h->round, s->outbox.n, (unsigned long long)total + 1);
        TRY(s->outbox.ensure(total + 1, 2));
        TRY(s->okey.ensure(total + 1, 2));
        TRY(stream_wait(s));
        TRY(run_round(h, st, done == 0));     // (the first round's events are applied)
    } else {
        // its node phases ran: grow the route's buffers, route it again,
        // then its stats and round-end halves
        const uint64_t m = s->pin[PIN_OVF];
        s->pin[PIN_OVF] = 0;
        const uint64_t want = m + m / 2;
        if (want <= (1ull << 26)) while (s->rcap < want) s->rcap <<= 1;
        else s->rcap = (want + (1ull << 20) - 1) >> 20 << 20;
        TRY(route_buffers(s, false));
        TRY(phase_route_local(h, s, true));
        TRY(phase_stats(h, s, done == 0 ? crashed0 : none));
        if (done == 0 && bc0)
            k_origin<<<grid_for(h->pend_b_root.size()), BLK, 0, s->stream>>>(
                s->origin.p, s->lo, s->n, s->bc_roots.p, s->bc_msgs.p, (uint32_t)h->pend_b_root.size(), s->flags.p,
                true, s->ctl.p);
        TRY(stream_wait(s));
        for (int k = 0; k < NST; k++) st[k] = s->pin[k];
        if (st[ST_BOUND]) return PSIM_EDEVICE;
        s->m_in = (uint32_t)s->pin[PIN_M];
        if (s->pin[NST] != ~0ull && s->pin[NST + 1] > s->pin[NST]) {
            h->kt_ms[KT_CONSUME] += (double)(s->pin[NST + 1] - s->pin[NST]) * 1e-5;
            h->kt_n[KT_CONSUME]++;
        }
        if (done == 0) {
            for (uint32_t j : h->pend_join) h->pend_join_mark[j] = 0;
            h->pend_crash.clear(); h->pend_join.clear(); h->pend_contact.clear();
            h->pend_part_set = h->pend_part_clear = false;
            h->pend_b_root.clear(); h->pend_b_msg.clear();
            h->faults_dirty = false;
        }
        h->round++;
    }
    if (st_out) fill_stats(st, r0 + done, &st_out[done]);
    *done_out = done + 1;
    return PSIM_OK;
}

// The rank path's batch (RCCL ranks, or loopback): up to nb rounds enqueued
// back to back with no host wait -- the outbox checked against its capacity by
// k_desc (code 1), the exchange in fixed-size messages (exchange_fixed; an
// owner past its capacity, code 3), the route's capacity G * xcap_h records
// (never short) -- then one wait.  Every round all-reduces whether any rank
// aborted it (phase_stats: k_xabort, k_abort_sync), so all ranks stop at the
// same round r; its records are then exchanged again exactly by every rank
// (run_round from its owner partition; a rank whose outbox was short grows it
// and runs the round's node phase again first -- nothing of it ran past
// k_desc).  Rounds after r returned at once from every kernel; their
// collectives moved nothing anyone reads.
int run_batch_ranked(psim_handle* h, uint32_t nb, psim_round_stats* st_out, uint32_t* done_out) {
    Shard* s = h->shards[0];
    const uint32_t G = h->G, capH = s->xcap_h, capT = s->xcap_t;
    const uint64_t r0 = h->round;
    TRY(s->sendbuf.ensure((size_t)G * (XHDR + capH + capT) + 1));
    TRY(s->recvh.ensure((size_t)G * (XHDR + capH) + 1));
    TRY(s->recvt.ensure((size_t)G * capT + 1));
    TRY(h->comm_cnt.ensure(2 * G + 2));
    s->rcap = std::max<uint64_t>(s->rcap, (uint64_t)G * capH);    // (the route never overflows)
    TRY(route_buffers(s, false));
    RoundCtl ctl0;
    ctl0.crashes = !h->pend_crash.empty();
    bcast_slots(h, ctl0);
    const std::vector<uint32_t> crashed0 = h->pend_crash;
    const std::vector<uint32_t> none;
    const bool bc0 = !h->pend_b_root.empty();
    s->tn = 0;
    s->desc_cap = std::min<uint64_t>(s->outbox.n, s->okey.n);
    const auto t_enq = std::chrono::steady_clock::now();
    double tph[5] = {0, 0, 0, 0, 0};                  // (PSIM_TRACE_BATCH: host ms per phase)
    auto tick = [](std::chrono::steady_clock::time_point& t0, double& acc) {
        const auto t1 = std::chrono::steady_clock::now();
        acc += std::chrono::duration<double, std::milli>(t1 - t0).count();
        t0 = t1;
    };
    for (uint32_t j = 0; j < nb; j++) {
        s->stat_slot = j + 1;
        s->batch_round1 = (uint32_t)h->round + 1;
        RoundArgs a;
        const RoundCtl ctl = j == 0 ? ctl0 : RoundCtl{};
        auto t0 = std::chrono::steady_clock::now();
        TRY(phase_events_prepare(h, s, ctl, a, j == 0, true));
        tick(t0, tph[0]);
        TRY(phase_consume(h, s, a));
        tick(t0, tph[1]);
        TRY(phase_partition(h, s, true));
        tick(t0, tph[2]);
        TRY(exchange_fixed(h));
        tick(t0, tph[3]);
        TRY(phase_stats(h, s, j == 0 ? crashed0 : none, true));
        tick(t0, tph[4]);
        if (j == 0 && bc0)                  // the first round's origins are spent
            k_origin<<<grid_for(h->pend_b_root.size()), BLK, 0, s->stream>>>(
                s->origin.p, s->lo, s->n, s->bc_roots.p, s->bc_msgs.p, (uint32_t)h->pend_b_root.size(), s->flags.p,
                true, s->ctl.p);
        HIP_TRY(hipGetLastError());
        h->round++;
    }
    s->stat_slot = 0; s->batch_round1 = 0; s->desc_cap = 0;
    uint32_t cw[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(cw, s->ctl.p, sizeof cw, hipMemcpyDeviceToHost, s->stream));
    const auto t_wait = std::chrono::steady_clock::now();
    TRY(stream_wait(s));
    const auto t_end = std::chrono::steady_clock::now();
    if (s->pin[PIN_BIGIN]) {                          // a node's inbox count must fit 27 bits
        s->pin[PIN_BIGIN] = 0;
        HIP_TRY(hipMemsetAsync(s->ctl.p, 0, sizeof cw, s->stream));
        return PSIM_ENOMEM;
    }
    // the first round some rank aborted (the all-reduced x-word: every rank
    // finds the same one)
    uint32_t done = nb;
    for (uint32_t j = 0; j < nb; j++)
        if (s->pin[(size_t)(j + 1) * PIN_STRIDE + PIN_XAB]) { done = j; break; }
    if (done == nb && cw[0]) return PSIM_EDEVICE;     // (an abort no round reported)
    // the capacities grow with the largest counts the batch met -- the
    // stopped round's included, which is what the redo will need
    {
        uint64_t mh = 0, mt = 0;
        for (uint32_t j = 0; j <= done && j < nb; j++) xcaps_max(h, s->pin + (size_t)(j + 1) * PIN_STRIDE, mh, mt);
        xcaps_set(s, mh, mt, done < nb);
    }
    static const bool trace_batch = getenv("PSIM_TRACE_BATCH") != nullptr;
    if (trace_batch)
        std::fprintf(stderr, "psim: rank %d: batch of %u from round %llu: %u done%s; caps %u heads, %u tails; "
                     "enqueue %.3f ms (prepare %.3f, node phase %.3f, partition %.3f, exchange + route %.3f, end "
                     "%.3f), wait %.3f ms\n",
                     h->rank, nb, (unsigned long long)r0, done, done < nb ? " (one redone exactly)" : "", s->xcap_h,
                     s->xcap_t, std::chrono::duration<double, std::milli>(t_wait - t_enq).count(), tph[0], tph[1],
                     tph[2], tph[3], tph[4], std::chrono::duration<double, std::milli>(t_end - t_wait).count());
    const bool self_comm = h->world == 1;
    for (uint32_t j = 0; j < done; j++) {
        const uint64_t* p = s->pin + (size_t)(j + 1) * PIN_STRIDE;
        if (p[ST_BOUND]) {
            std::fprintf(stderr, "psim: round %llu: %llu nodes emitted past their outbox bound (engine bug)\n",
                         (unsigned long long)(r0 + j), (unsigned long long)p[ST_BOUND]);
            return PSIM_EDEVICE;
        }
        if (st_out) fill_stats(p, r0 + j, &st_out[j]);
        if (p[NST] != ~0ull && p[NST + 1] > p[NST]) {     // 100 MHz ticks
            h->kt_ms[KT_CONSUME] += (double)(p[NST + 1] - p[NST]) * 1e-5;
            h->kt_n[KT_CONSUME]++;
        }
        for (uint32_t g = 0; g < G; g++) {            // (the padded messages cross the links)
            if (g == s->idx && !self_comm) continue;
            h->x_records += p[PIN_XCNT + g] & 0xFFFFFFFFull;
            h->x_bytes += (uint64_t)(XHDR + capH + capT) * sizeof(Wire);
        }
    }
    if (done > 0) {                           // the first round's events are spent
        for (uint32_t j : h->pend_join) h->pend_join_mark[j] = 0;
        h->pend_crash.clear(); h->pend_join.clear(); h->pend_contact.clear();
        h->pend_part_set = h->pend_part_clear = false;
        h->pend_b_root.clear(); h->pend_b_msg.clear();
        h->faults_dirty = false;
    }
    s->m_in = (uint32_t)s->pin[PIN_M];         // (the last route that ran)
    *done_out = done;
    if (done == nb) {
        h->round = r0 + nb;
        s->xbatch = std::min<uint32_t>(2 * s->xbatch, BATCH_MAX);
        return PSIM_OK;
    }
    // round r0 + done stopped the batch on some rank: every rank redoes it
    // exactly (a rank whose own outbox was short from its node phase); the
    // next batch is a quarter as long (its dead tail, every round's padded
    // messages, is what a stop costs)
    s->xbatch = std::max<uint32_t>(2, s->xbatch / 4);
    HIP_TRY(hipMemsetAsync(s->ctl.p, 0, sizeof cw, s->stream));
    h->round = r0 + done;
    const bool short_outbox = cw[0] == 1 && cw[1] == (uint32_t)h->round;
    uint64_t st[NST];
    if (short_outbox) {
        std::fprintf(stderr, "psim: round %llu: outbox grows past its capacity (%zu -> %llu slots)\n",
                     (unsigned long long)h->round, s->outbox.n, (unsigned long long)s->pin[PIN_TOTAL] + 1);
        TRY(stream_wait(s));
    }
    TRY(run_round(h, st, done == 0, !short_outbox));
    if (st_out) fill_stats(st, r0 + done, &st_out[done]);
    *done_out = done + 1;
    return PSIM_OK;
}

int shard_alloc(psim_handle* h, Shard* s) {
    HIP_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&s->wait_ev, hipEventDisableTiming));
    for (int k = 0; k < 2; k++) {
        HIP_TRY(hipStreamCreateWithFlags(&s->side[k], hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&s->join_ev[k], hipEventDisableTiming));
    }
    HIP_TRY(hipEventCreateWithFlags(&s->fork_ev, hipEventDisableTiming));
    if (s->n > (1u << 26)) {    // route buckets of 8192 destinations: 128 KiB of LDS per block
        HIP_TRY(hipFuncSetAttribute((const void*)k_bucket_route<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    8192 * 16));
        HIP_TRY(hipFuncSetAttribute((const void*)k_bucket_route<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    8192 * 16));
    }
    HIP_TRY(hipHostMalloc((void**)&s->pin, (size_t)PIN_STRIDE * (1 + BATCH_MAX) * sizeof(uint64_t), hipHostMallocMapped));
    HIP_TRY(hipHostGetDevicePointer((void**)&s->pin_dev, s->pin, 0));
    memset(s->pin, 0, (size_t)PIN_STRIDE * (1 + BATCH_MAX) * sizeof(uint64_t));
    for (int k = 0; k < Shard::MAXT; k++) {
        HIP_TRY(hipEventCreate(&s->ev[k][0]));
        HIP_TRY(hipEventCreate(&s->ev[k][1]));
    }
    s->ev_live = true;
    const size_t N = h->N, n = std::max<uint32_t>(s->n, 1);
    int rc = 0;
    rc |= s->flags.alloc(N); rc |= s->part.alloc(N); rc |= s->hdr.alloc(n);
    if (h->cfg.manager != PSIM_MANAGER_PLUGGABLE) { rc |= s->upart.alloc(N); rc |= s->lite_cm.alloc(n); }
    rc |= s->crash_bits.alloc((N >> (CRASH_GRAIN_SHIFT + 5)) + 1);
    rc |= s->act.alloc(n * PSIM_ACTIVE_CAP); rc |= s->pas.alloc(n * PSIM_PASSIVE_CAP);
    rc |= s->sentm.alloc(n * IDMAP_IN); rc |= s->recvm.alloc(n * IDMAP_IN);
    if (h->cfg.manager != PSIM_MANAGER_PLUGGABLE) {
        // extension rows for 1/32 of the nodes (~1/1700 used at 2^23 under config E);
        // X-BOT's optimization rounds disconnect and rejoin peers all the time
        // (most nodes' maps pass 16 entries within 50 rounds at a 10-round
        // period): one row per map and node, the oracle's full 64 entries
        const size_t rows = h->cfg.manager == PSIM_MANAGER_XBOT ? 2 * n : std::max<size_t>(1024, n / 32);
        rc |= s->mapx.alloc(rows * IDMAP_EXT);
    }
    rc |= s->mapx_top.alloc(1);
    rc |= s->pt_all.alloc(n * PSIM_PT_MEMBERS_CAP); rc |= s->pt_com.alloc(n * PSIM_PT_MEMBERS_CAP);
    rc |= s->pt_eag.alloc(n * RT_SET); rc |= s->pt_laz.alloc(n * RT_SET); rc |= s->pt_rt.alloc(n * RT_WORDS);
    rc |= s->origin.alloc(n); rc |= s->slots.alloc(2 * PSIM_MSG_SLOTS);
    rc |= s->pt_out.alloc(n * OUT_IN); rc |= s->start.alloc(n);
    if (h->cfg.manager != PSIM_MANAGER_PLUGGABLE) rc |= s->conn.alloc(n * PSIM_CONN_CAP);
    // outstanding extension rows for 1/8 of the nodes: a lazy peer that is no
    // member (update_peers adds a PRUNE's or IHAVE's sender after its
    // neighbors_down) collects one entry per broadcast that no ack clears
    // (pt:443-453, :562-579), so tables grow for as long as broadcasts run --
    // under config E with the partition after the churn ~10 % of the nodes
    // pass 16 entries by phase round 230 (oracle, 2^16); at 1/32 the pool ran
    // out at 2^26
    if (h->cfg.manager != PSIM_MANAGER_PLUGGABLE) {
        // rows for 1/8 of the nodes to start with (grow_outx doubles it);
        // PSIM_OUTX_ROWS sets another start (tests of the growth)
        size_t rows = std::max<size_t>(1024, n / 8);
        if (const char* e = getenv("PSIM_OUTX_ROWS")) rows = std::max<size_t>(1, (size_t)atoll(e));
        rc |= s->outx.alloc(rows * OUT_EXT);
    }
    rc |= s->outx_top.alloc(1);
    rc |= s->ocnt.alloc(n); rc |= s->cb.alloc(n + 1);
    rc |= s->in_beg.alloc(n + 1); rc |= s->bound.alloc(n + 1); rc |= s->pscan.alloc(4097); rc |= s->obase.alloc(n + 1);
    rc |= s->bmask.alloc(n); rc |= s->btot.alloc(4096);
    rc |= s->desc.alloc(n); rc |= s->d_nact.alloc(1);
    rc |= s->desc_slow.alloc(n); rc |= s->n_slow.alloc(1);
    rc |= s->desc_pt.alloc(n); rc |= s->n_pt.alloc(1);
    rc |= s->desc_shuf.alloc(n); rc |= s->n_shuf.alloc(1);
    rc |= s->desc_lite.alloc(2 * n); rc |= s->n_lite.alloc(4);
    rc |= s->desc_ptl.alloc(n); rc |= s->n_ptl.alloc(2);
    if (h->cfg.manager == PSIM_MANAGER_PLUGGABLE) { rc |= s->stop_ids.alloc(n); rc |= s->n_stop.alloc(1); }
    rc |= s->stat_out.alloc(STAT_OUT_N);   // + the consume span, the rank path's x-words
    rc |= s->ctl.alloc(4);   // (the abort word: code, round; then the fused route's overflow flag)
    rc |= s->stat_tile.alloc((size_t)STAT_TILES * NST);
    rc |= s->ikeys.alloc(1024); rc |= s->ivals.alloc(1024);
    rc |= s->recvh.alloc(1024); rc |= s->recvt.alloc(1024); rc |= s->wseg.alloc(130); rc |= s->inbox.alloc(1024); rc |= s->outbox.alloc(1024);
    if (h->cfg.manager == PSIM_MANAGER_PLUGGABLE) {
        if (h->cfg.strategy == PSIM_STRATEGY_FULL) {
            rc |= s->fbits.alloc(n * 2 * h->fw);     // [adds | removes] per node
            rc |= s->pay_top.alloc(1);
            rc |= s->pay[0].alloc(2 * h->fw); rc |= s->pay[1].alloc(2 * h->fw);
        } else {
            rc |= s->sview.alloc(n * PSIM_SVIEW_CAP);
            if (h->cfg.strategy == PSIM_STRATEGY_SCAMP_V2) rc |= s->sinv.alloc(n * PSIM_SVIEW_CAP);
        }
    }
    if (rc) return PSIM_ENOMEM;
    // the zero fills above run on the null stream, which a non-blocking
    // stream does not wait for: finish them before any kernel of the shard
    HIP_TRY(hipDeviceSynchronize());
    return PSIM_OK;
}

void shard_free(Shard* s) {
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    s->flags.release(); s->part.release(); s->upart.release(); s->lite_cm.release(); s->hdr.release(); s->crash_bits.release(); s->btab.release();
    s->act.release(); s->pas.release(); s->sentm.release(); s->recvm.release();
    s->pt_all.release(); s->pt_com.release();
    s->mapx.release(); s->mapx_top.release();
    s->pt_eag.release(); s->pt_laz.release(); s->pt_out.release(); s->start.release(); s->conn.release();
    s->outx.release(); s->outx_top.release();
    s->pt_rt.release(); s->origin.release(); s->slots.release(); s->bc_roots.release(); s->bc_msgs.release();
    s->ikeys.release(); s->ivals.release(); s->recvh.release(); s->recvt.release(); s->wseg.release(); s->inbox.release();
    if (s->pin) (void)hipHostFree(s->pin);
    if (s->wait_ev) (void)hipEventDestroy(s->wait_ev);
    s->wait_ev = nullptr;
    for (int k = 0; k < 2; k++) {
        if (s->join_ev[k]) (void)hipEventDestroy(s->join_ev[k]);
        if (s->side[k]) (void)hipStreamDestroy(s->side[k]);
        s->join_ev[k] = nullptr;
        s->side[k] = nullptr;
    }
    if (s->fork_ev) (void)hipEventDestroy(s->fork_ev);
    s->fork_ev = nullptr;
    s->pin = nullptr;
    s->outbox.release(); s->okey.release(); s->ocnt.release();
    s->cb.release(); s->in_beg.release();
    s->rank.release(); s->bmask.release(); s->btot.release();
    s->hist.release(); s->hoff.release(); s->rtot.release(); s->rbase.release(); s->pairs.release(); s->tmp.release();
    s->stop_ids.release(); s->n_stop.release();
    s->desc.release(); s->d_nact.release(); s->desc_slow.release(); s->n_slow.release(); s->desc_pt.release(); s->n_pt.release(); s->desc_shuf.release(); s->n_shuf.release(); s->desc_lite.release(); s->n_lite.release(); s->desc_ptl.release(); s->n_ptl.release(); s->bound.release(); s->pscan.release();
    s->obase.release(); s->stat_part.release(); s->stat_out.release(); s->stat_tile.release(); s->d_off.release();
    s->cub_tmp.release(); s->ev_ids.release(); s->ev_contacts.release(); s->sendbuf.release(); s->ctl.release();
    s->sview.release(); s->sinv.release(); s->fbits.release(); s->pay[0].release(); s->pay[1].release();
    s->pay_top.release();
    if (s->ev_live)
        for (int k = 0; k < Shard::MAXT; k++) {
            (void)hipEventDestroy(s->ev[k][0]);
            (void)hipEventDestroy(s->ev[k][1]);
        }
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
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
    case PSIM_ECAPACITY: return "a fixed table overflowed (strict)";
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
    cfg->manager = PSIM_MANAGER_HYPARVIEW; cfg->strategy = PSIM_STRATEGY_FULL;
    cfg->periodic_interval = 10; cfg->scamp_c = 5; cfg->fanout = 0;
    cfg->xbot_period = 35;
}

uint32_t psim_xbot_latency(uint64_t seed, uint32_t a, uint32_t b) { return psim::xbot_latency(seed, a, b); }

void psim_destroy(psim_handle* h);

int psim_create(const psim_config* cfg, psim_handle** out) {
    if (!cfg || !out || cfg->abi_version != PSIM_ABI_VERSION || cfg->n_nodes == 0 ||
        cfg->n_nodes > KEY_DST_MASK || cfg->max_active_size < 2 ||
        cfg->max_active_size > PSIM_ACTIVE_CAP || cfg->max_passive_size < 1 ||
        cfg->max_passive_size > 30 || 1 + cfg->k_active + cfg->k_passive > PSIM_EXCHANGE_CAP ||
        cfg->arwl > 255 || cfg->prwl > 255 || cfg->manager > PSIM_MANAGER_XBOT ||
        cfg->strategy > PSIM_STRATEGY_SCAMP_V2 || cfg->scamp_c < 1 || cfg->scamp_c > 64 ||
        cfg->fanout > 64 || cfg->strict > 1)   /* (picks land in one 64-lane register) */
        return PSIM_EINVAL;
    {
        // every kernel TU compiled against the same layout (psim_kernels.h
        // layout_sig): a mixed A/B library is refused here, not in a kernel
        const uint32_t e = layout_sig(), c = layout_sig_consume(), l = layout_sig_lite(), st = layout_sig_strategy();
        if (c != e || l != e || st != e) {
            std::fprintf(stderr, "psim: library TUs built with different layouts (engine %08x, consume %08x, "
                         "lite %08x, strategy %08x): rebuild every TU with the same macros\n", e, c, l, st);
            return PSIM_ESTATE;
        }
    }
    const bool full = cfg->manager == PSIM_MANAGER_PLUGGABLE && cfg->strategy == PSIM_STRATEGY_FULL;
    uint32_t world = std::max<uint32_t>(cfg->shard_world, 1);
    uint32_t local = std::max<uint32_t>(cfg->n_shards, 1);
    // the rank path: world > 1, or one rank with a communicator id (the
    // 1-GPU diagnostic of the RCCL path)
    const bool ranked = world > 1 || cfg->comm_id != nullptr;
    if (ranked && (local != 1 || !cfg->comm_id || cfg->shard_rank >= world)) return PSIM_EINVAL;
    uint32_t G = ranked ? world : local;
    if (G > 64 || G > cfg->n_nodes) return PSIM_EINVAL;
    if (full && G > 1) return PSIM_EUNSUPPORTED;      // gossip payloads are shard-local
    psim_handle* h = new (std::nothrow) psim_handle();
    if (!h) return PSIM_ENOMEM;
    h->cfg = *cfg;
    if (full) {
        h->fw = ((cfg->n_nodes + 31) / 32 + 3) & ~3u;
        h->started.assign(cfg->n_nodes, 0);
    }
    h->N = cfg->n_nodes;
    h->G = G;
    for (uint32_t k = 0; k < 2 * PSIM_MSG_SLOTS; k++) h->slot_tab[k] = PSIM_NONE;
    h->per = (h->N + G - 1) / G;
    h->world = (int)world;
    h->ranked = ranked;
    h->rank = (int)cfg->shard_rank;
    int dev = cfg->device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) { delete h; return PSIM_EDEVICE; }
    if (hipSetDevice(dev) != hipSuccess) { delete h; return PSIM_EDEVICE; }
    // grids: PSIM_<KERNEL>_GRID=N (blocks) or =xK (K times the resident grid)
    // override them for measurements (profiles/grid_ab.sh)
    auto grid = [](const char* env, uint32_t resident, uint32_t dflt) -> uint32_t {
        const char* e = getenv(env);
        if (!e) return dflt;
        const bool mul = e[0] == 'x';
        const long v = strtol(e + (mul ? 1 : 0), nullptr, 10);
        if (v <= 0) return dflt;
        return mul ? (uint32_t)v * resident : (uint32_t)v;
    };
    h->consume_blocks = grid("PSIM_CONSUME_GRID", psim::consume_grid(), psim::consume_grid());
    h->pt_blocks = grid("PSIM_PT_GRID", psim::pt_grid(), psim::pt_grid());
    // k_consume_lite: four times the resident blocks -- the dispatcher hands
    // freed slots new blocks, which evens out the waves' uneven node mixes (the
    // resident grid left 4.1 of 6 waves/SIMD busy on average; 300 -> 272 us a
    // round on the survey line, profiles/r03/p10)
    h->lite_half = getenv("PSIM_LITE_WAVE") == nullptr;
    h->lite_blocks = h->lite_half ? grid("PSIM_LITE_GRID", psim::lite_half_grid(), 4 * psim::lite_half_grid())
                                  : grid("PSIM_LITE_GRID", psim::lite_grid(), 4 * psim::lite_grid());
    // k_ptl (a lane per node; round 4's four-nodes-per-wave k_ptq was
    // parity-exact but slower -- 0.602 against 0.584 ms a phase at 2^20, 79.3
    // against 68.1 ms at 2^26, profiles/r04/pq2: a row per node runs each
    // handler for 4 nodes where a lane per node runs it for 64 -- and was
    // removed in round 5)
    h->ptl_blocks = grid("PSIM_PTL_GRID", psim::ptl_grid(), psim::ptl_grid());
    {
        const char* e = getenv("PSIM_PHASE_TIMERS");
        h->phase_timers = e && *e && *e != '0';
        const char* b = getenv("PSIM_ROUTE_BLOCKS");
        if (b && *b) h->rb_blocks = std::max<uint32_t>(1, std::min<uint32_t>(RB_MAX_BLOCKS, (uint32_t)atoi(b)));
        const char* g = getenv("PSIM_ROUTE_REG");     // (test hook: the large-bucket path everywhere)
        if (g && *g) h->rr_reg = std::min<uint32_t>(RR_REG, (uint32_t)atoi(g));
        const char* f = getenv("PSIM_ROUTE_FUSED");   // (0: the four-pass route every round, A/B)
        if (f && *f) h->route_fused = atoi(f) != 0;
    }
    h->device = dev;
    for (uint32_t g = 0; g < G; g++) {
        if (ranked && g != cfg->shard_rank) continue;
        Shard* s = new (std::nothrow) Shard();
        if (!s) { psim_destroy(h); return PSIM_ENOMEM; }
        s->idx = g;
        s->lo = std::min<uint32_t>(g * h->per, h->N);
        s->n = std::min<uint32_t>(h->N, s->lo + h->per) - s->lo;
        h->shards.push_back(s);
        int rc = shard_alloc(h, s);
        if (!rc && hipMemcpy(s->slots.p, h->slot_tab, sizeof h->slot_tab, hipMemcpyHostToDevice) != hipSuccess)
            rc = PSIM_EDEVICE;
        if (rc) { psim_destroy(h); return rc; }
    }
    if (ranked) {
        // RCCL; an id from psim_loopback_comm_id selects the loopback test
        // vehicle instead (ranks as threads of this process, psim_comm.h)
        int rc;
        if (LoopbackComm::is_loopback_id(cfg->comm_id)) {
            LoopbackComm* c = new (std::nothrow) LoopbackComm();
            h->comm = c;
            rc = c ? c->init(cfg->comm_id, (int)cfg->shard_rank, (int)world) : PSIM_ENOMEM;
        } else {
            RcclComm* c = new (std::nothrow) RcclComm();
            h->comm = c;
            rc = c ? c->init(cfg->comm_id, (int)cfg->shard_rank, (int)world) : PSIM_ENOMEM;
            if (rc) std::fprintf(stderr, "psim: RCCL world %u, rank %u: no communicator\n", world, cfg->shard_rank);
        }
        if (rc) {
            psim_destroy(h);
            return rc;
        }
    }
    *out = h;
    return PSIM_OK;
}

void psim_destroy(psim_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    for (Shard* s : h->shards) shard_free(s);
    h->shards.clear();
    h->comm_cnt.release();
    delete h->comm;
    delete h;
}

int psim_join(psim_handle* h, const uint32_t* nodes, const uint32_t* contacts, size_t n) {
    if (!h || (n && (!nodes || !contacts))) return PSIM_EINVAL;
    for (size_t i = 0; i < n; i++)
        if (nodes[i] >= h->N || (contacts[i] != PSIM_NONE && contacts[i] >= h->N)) return PSIM_ERANGE;
    // a node starts at most once per round: k_join runs one thread per entry,
    // so two entries of one id would race on its rows
    if (h->pend_join_mark.size() != h->N) h->pend_join_mark.assign(h->N, 0);
    {
        size_t i = 0;
        for (; i < n; i++) {
            if (h->pend_join_mark[nodes[i]]) break;
            h->pend_join_mark[nodes[i]] = 1;
        }
        if (i < n) {                    // undo this call's marks
            for (size_t j = 0; j < i; j++) h->pend_join_mark[nodes[j]] = 0;
            return PSIM_EINVAL;
        }
    }
    if (!h->started.empty()) {          // an ORSet re-add would need per-incarnation tokens
        for (size_t i = 0; i < n; i++)
            if (h->started[nodes[i]]) {
                for (size_t j = 0; j < n; j++) h->pend_join_mark[nodes[j]] = 0;
                return PSIM_EUNSUPPORTED;
            }
        for (size_t i = 0; i < n; i++) h->started[nodes[i]] = 1;
    }
    h->pend_join.insert(h->pend_join.end(), nodes, nodes + n);
    h->pend_contact.insert(h->pend_contact.end(), contacts, contacts + n);
    return PSIM_OK;
}

int psim_revive(psim_handle* h, const uint32_t* nodes, size_t n) {
    if (!h || (n && !nodes)) return PSIM_EINVAL;
    std::vector<uint32_t> none(n, PSIM_NONE);
    return psim_join(h, nodes, none.data(), n);
}

int psim_crash(psim_handle* h, const uint32_t* nodes, size_t n) {
    if (!h || (n && !nodes)) return PSIM_EINVAL;
    for (size_t i = 0; i < n; i++)
        if (nodes[i] >= h->N) return PSIM_ERANGE;
    h->pend_crash.insert(h->pend_crash.end(), nodes, nodes + n);
    return PSIM_OK;
}

// leave/0 under the pluggable manager: handle_call({leave, Myself})
// (pl:502-515) runs internal_leave/2 (pl:1390-1420), whose Strategy:leave/2
// messages are casts to the manager itself (schedule_self_message_delivery/6
// pl:1585-1609), then returns {stop, normal}: the casts die in its mailbox and
// the node stops as if crashed.  HyParView's leave answers `error`
// (hv:363-364).
int psim_leave(psim_handle* h, const uint32_t* nodes, size_t n) {
    if (!h || (n && !nodes)) return PSIM_EINVAL;
    if (h->cfg.manager != PSIM_MANAGER_PLUGGABLE) return PSIM_EUNSUPPORTED;
    return psim_crash(h, nodes, n);
}

// leave/1: actors[i] removes targets[i] (pl:502-515 -> internal_leave/2
// :1390-1420); actor == target is leave/0.  A stop is learned from the
// owner shard's list after the round (RCCL ranks: all-gathered; every rank
// makes the same calls).
int psim_leave_node(psim_handle* h, const uint32_t* actors, const uint32_t* targets, size_t n) {
    if (!h || (n && (!actors || !targets))) return PSIM_EINVAL;
    if (h->cfg.manager != PSIM_MANAGER_PLUGGABLE) return PSIM_EUNSUPPORTED;
    for (size_t i = 0; i < n; i++) {
        if (actors[i] >= h->N || targets[i] >= h->N) return PSIM_ERANGE;
        for (uint32_t a : h->pend_lv_a) if (a == actors[i]) return PSIM_EINVAL;
        for (size_t j = 0; j < i; j++) if (actors[j] == actors[i]) return PSIM_EINVAL;
    }
    for (size_t i = 0; i < n; i++) {
        if (actors[i] == targets[i]) { TRY(psim_crash(h, &actors[i], 1)); continue; }
        if (h->cfg.strategy == PSIM_STRATEGY_FULL) h->tomb = true;
        h->pend_lv_a.push_back(actors[i]);
        h->pend_lv_t.push_back(targets[i]);
    }
    return PSIM_OK;
}

int psim_set_partition(psim_handle* h, const uint8_t* group, size_t n) {
    if (!h || !group || n != h->N) return PSIM_EINVAL;
    for (size_t i = 0; i < n; i++)
        if (group[i] == PSIM_PARTITION_MAX + 1) return PSIM_EINVAL;   // (255: the pair array's "down")
    h->pend_part.assign(group, group + n);
    h->pend_part_set = true; h->pend_part_clear = false;
    return PSIM_OK;
}

// The view-order table: the low 8 bits of every
// node_spec's erlang:phash(NodeSpec, 2^32) - 1, from which sets v1's slots
// follow (psim_device.h set_slot: 16 buckets for every HyParView view, the
// linear hash's wider tables for SCAMP v1 memberships past 80 ids): the order
// sets:to_list/1 yields views in, which every select_random index and every
// shuffle key pairing follows (hv:1230-1231, :1346-1361; sv1:45-279).  Before
// the first round only (the views already built would be in the old order);
// NULL restores the default table.
static int install_table(psim_handle* h, const std::vector<uint8_t>& tab) {
    if (hipSetDevice(h->device) != hipSuccess) return PSIM_EDEVICE;
    for (Shard* s : h->shards) {
        if (!s->btab.p && s->btab.alloc(h->N)) return PSIM_ENOMEM;
        if (hipMemcpy(s->btab.p, tab.data(), tab.size(), hipMemcpyHostToDevice) != hipSuccess) return PSIM_EDEVICE;
    }
    // (FNV-1a of the bytes, recorded in snapshots: psim_restore refuses a
    // snapshot made under another table)
    uint32_t x = 0x811C9DC5u;
    for (uint8_t b : tab) x = (x ^ b) * 0x01000193u;
    h->btab = true;
    h->btab_hash = x | 1u;
    return PSIM_OK;
}

int psim_set_bucket_table(psim_handle* h, const uint8_t* buckets, size_t n) {
    if (!h) return PSIM_EINVAL;
    if (h->round != 0) return PSIM_ESTATE;
    if (!buckets) { h->btab = false; h->btab_hash = 0; return PSIM_OK; }
    if (n != h->N) return PSIM_EINVAL;
    for (size_t i = 0; i < n; i++)
        if (buckets[i] > 15) return PSIM_EINVAL;
    return install_table(h, std::vector<uint8_t>(buckets, buckets + n));
}

int psim_set_phash_table(psim_handle* h, const uint32_t* phash, size_t n) {
    if (!h) return PSIM_EINVAL;
    if (h->round != 0) return PSIM_ESTATE;
    if (!phash) { h->btab = false; h->btab_hash = 0; return PSIM_OK; }
    if (n != h->N) return PSIM_EINVAL;
    std::vector<uint8_t> tab(n);
    for (size_t i = 0; i < n; i++) tab[i] = (uint8_t)phash[i];
    return install_table(h, tab);
}

int psim_clear_partition(psim_handle* h) {
    if (!h) return PSIM_EINVAL;
    h->pend_part_clear = true; h->pend_part_set = false;
    return PSIM_OK;
}

// omission faults: add_interposition_fun / remove_interposition_fun
// (pl:297-326) of the crash-fault model's {send_omission, Dst} and
// {receive_omission, Src} funs (prop_partisan_crash_fault_model:117-196)
int psim_set_omission(psim_handle* h, int kind, const uint32_t* src, const uint32_t* dst, size_t n, int on) {
    if (!h || (n && (!src || !dst))) return PSIM_EINVAL;
    if (h->cfg.manager != PSIM_MANAGER_PLUGGABLE) return PSIM_EUNSUPPORTED;
    if (kind != PSIM_OMIT_SEND && kind != PSIM_OMIT_RECEIVE) return PSIM_EINVAL;
    for (size_t i = 0; i < n; i++)
        if (src[i] >= h->N || dst[i] >= h->N) return PSIM_ERANGE;
    std::set<uint64_t>& l = kind == PSIM_OMIT_SEND ? h->nx_omit_s : h->nx_omit_r;
    for (size_t i = 0; i < n; i++) {
        const uint64_t k = (uint64_t)src[i] << 32 | dst[i];
        if (on) l.insert(k);
        else l.erase(k);
    }
    h->faults_dirty = true;
    return PSIM_OK;
}

// begin_omission / end_omission (crash_fault_model:93-114)
int psim_set_faulted(psim_handle* h, const uint32_t* nodes, size_t n, int on) {
    if (!h || (n && !nodes)) return PSIM_EINVAL;
    if (h->cfg.manager != PSIM_MANAGER_PLUGGABLE) return PSIM_EUNSUPPORTED;
    for (size_t i = 0; i < n; i++)
        if (nodes[i] >= h->N) return PSIM_ERANGE;
    if (h->nx_faulted.size() != h->N) h->nx_faulted.assign(h->N, 0);
    for (size_t i = 0; i < n; i++) {
        const uint8_t v = on ? 1 : 0;
        h->nx_nfaulted += (size_t)v - (size_t)h->nx_faulted[nodes[i]];
        h->nx_faulted[nodes[i]] = v;
    }
    h->faults_dirty = true;
    return PSIM_OK;
}

// resolve_all_faults_with_heal (crash_fault_model:198-229)
int psim_clear_faults(psim_handle* h) {
    if (!h) return PSIM_EINVAL;
    if (h->cfg.manager != PSIM_MANAGER_PLUGGABLE) return PSIM_EUNSUPPORTED;
    h->nx_omit_s.clear(); h->nx_omit_r.clear();
    h->nx_faulted.assign(h->N, 0);
    h->nx_nfaulted = 0;
    h->faults_dirty = true;
    return PSIM_OK;
}

int psim_broadcast(psim_handle* h, uint32_t root, uint32_t msg_id) {
    if (!h) return PSIM_EINVAL;
    if (h->cfg.manager == PSIM_MANAGER_PLUGGABLE) return PSIM_EUNSUPPORTED;   // Plumtree runs over HyParView
    if (root >= h->N || msg_id > 0xFFFF) return PSIM_ERANGE;
    for (size_t i = 0; i < h->pend_b_root.size(); i++)   // one per root and per slot per round
        if (h->pend_b_root[i] == root || h->pend_b_msg[i] % PSIM_MSG_SLOTS == msg_id % PSIM_MSG_SLOTS)
            return PSIM_EINVAL;
    h->pend_b_root.push_back(root);
    h->pend_b_msg.push_back(msg_id);
    return PSIM_OK;
}

// The outstanding tables' extension pool: a node takes a row for good the
// first time its table outgrows its own row, so the pool doubles at a round
// boundary once half of it is taken (read from the pinned word the route's
// stats pass leaves) -- up to a row per node, which never runs out.  A failed
// growth is reported once and leaves the pool as it is (a table that then
// finds no row counts a PSIM_OVF_PT_OUT overflow; cfg.strict fails the step).
int grow_outx(Shard* s) {
    if (!s->outx.p || s->outx_short) return PSIM_OK;   // (a growth that failed is not retried every round)
    const uint64_t rows = s->outx.n / OUT_EXT, used = std::min<uint64_t>(s->pin[PIN_OUTX], rows);
    if (rows >= s->n || used * 2 < rows) return PSIM_OK;
    const uint64_t want = std::min<uint64_t>(std::max<uint64_t>(2 * rows, used + 1024), s->n);
    if (s->outx.ensure_keep(want * OUT_EXT, used * OUT_EXT, s->stream) != PSIM_OK) {
        // (per shard: every handle in the process reports its own; the
        // tables that then find no row count PSIM_OVF_PT_OUT overflows in the
        // round's stats, and cfg.strict fails the step on the first)
        if (!s->outx_short) std::fprintf(stderr, "psim: shard %u: the outstanding pool could not grow past %llu rows\n",
                                         s->idx, (unsigned long long)rows);
        s->outx_short = true;
        return PSIM_OK;
    }
    HIP_TRY(hipMemsetAsync(s->outx.p + used * OUT_EXT, 0, (s->outx.n - used * OUT_EXT) * 8, s->stream));
    return PSIM_OK;
}

int psim_step(psim_handle* h, uint32_t n_rounds, psim_round_stats* stats) {
    if (!h) return PSIM_EINVAL;
    if (h->failed) return PSIM_ESTATE;
    if (hipSetDevice(h->device) != hipSuccess) return PSIM_EDEVICE;
    for (int k = 0; k < KT_N; k++) { h->kt_ms[k] = 0; h->kt_n[k] = 0; }
    for (uint32_t i = 0; i < n_rounds;) {
        if (batchable(h)) {                   // rounds back to back, one wait per batch
            uint32_t done = 0;
            int rc = h->ranked ? run_batch_ranked(h, std::min<uint32_t>(n_rounds - i, h->shards[0]->xbatch),
                                                  stats ? stats + i : nullptr, &done)
                               : run_batch(h, std::min<uint32_t>(n_rounds - i, BATCH_MAX), stats ? stats + i : nullptr, &done);
            if (rc) { h->failed = true; return rc; }
            for (Shard* s : h->shards)
                if ((rc = grow_outx(s))) { h->failed = true; return rc; }
            i += done;
            continue;
        }
        uint64_t st[NST];
        uint64_t r = h->round;
        int rc = run_round(h, st);
        if (rc) { h->failed = true; return rc; }
        for (Shard* s : h->shards)
            if ((rc = grow_outx(s))) { h->failed = true; return rc; }
        if (stats) fill_stats(st, r, &stats[i]);
        if (h->cfg.strict && st[ST_OVF]) return PSIM_ECAPACITY;   // cfg.strict: fail loudly
        i++;
    }
    // (diagnostic: the buffers' high-water marks, printed as they rise)
    static const bool trace = getenv("PSIM_TRACE_BOUND") != nullptr;
#ifdef PSIM_BOUND_TERMS
    if (trace) {
        unsigned long long v[BT_N];
        if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_bterm), sizeof v) == hipSuccess) {
            static const char* nm[BT_N] = {"resp", "timer", "push", "push_ne", "npush", "lazy", "on", "nl", "lc",
                                           "crash", "xbot", "bump", "total", "c", "quiet", "rounds"};
            std::fprintf(stderr, "psim: bound terms to round %llu:", (unsigned long long)h->round);
            for (int k = 0; k < BT_N; k++) std::fprintf(stderr, " %s=%llu", nm[k], v[k]);
            std::fprintf(stderr, "\n");
            std::memset(v, 0, sizeof v);
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bterm), v, sizeof v);
        }
    }
#endif
    if (trace)
        for (Shard* s : h->shards)
            if (s->pin[PIN_TMAX] > s->trace_tmax || s->pin[PIN_MMAX] > s->trace_mmax) {
                s->trace_tmax = std::max<uint64_t>(s->trace_tmax, s->pin[PIN_TMAX]);
                s->trace_mmax = std::max<uint64_t>(s->trace_mmax, s->pin[PIN_MMAX]);
                std::fprintf(stderr, "psim: round %llu shard %u: outbox total max %llu of %zu slots, routed max %llu "
                             "of %llu records\n", (unsigned long long)h->round, s->idx,
                             (unsigned long long)s->trace_tmax, s->outbox.n, (unsigned long long)s->trace_mmax,
                             (unsigned long long)s->rcap);
            }
    return PSIM_OK;
}

int psim_get_msg_slots(psim_handle* h, uint32_t* ids, uint32_t* roots, size_t cap) {
    if (!h || !ids || !roots || cap < PSIM_MSG_SLOTS) return PSIM_EINVAL;
    for (int k = 0; k < PSIM_MSG_SLOTS; k++) {
        ids[k] = h->slot_tab[k];
        roots[k] = h->slot_tab[PSIM_MSG_SLOTS + k];
    }
    return PSIM_OK;
}

int psim_get_round(psim_handle* h, uint64_t* round) {
    if (!h || !round) return PSIM_EINVAL;
    *round = h->round;
    return PSIM_OK;
}

static int get_shard_nodes(Shard* s, uint32_t first, uint32_t count, psim_node_view* out) {
    std::vector<Hdr> hd(count);
    std::vector<uint8_t> fl(count);
    std::vector<uint32_t> act((size_t)count * PSIM_ACTIVE_CAP), pas((size_t)count * PSIM_PASSIVE_CAP);
    std::vector<uint64_t> sm((size_t)count * IDMAP_IN), rm(sm.size());
    std::vector<uint32_t> all((size_t)count * PSIM_PT_MEMBERS_CAP), com(all.size());
    std::vector<uint32_t> eag((size_t)count * RT_SET), laz(eag.size()), rt((size_t)count * RT_WORDS);
    std::vector<uint64_t> po((size_t)count * OUT_IN);
    std::vector<uint32_t> cn((size_t)count * PSIM_CONN_CAP, 0u);
    const size_t li = first - s->lo;
    auto cp = [&](void* dst, const void* src, size_t bytes) {
        return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s->stream);
    };
    HIP_TRY(cp(hd.data(), s->hdr.p + li, count * sizeof(Hdr)));
    HIP_TRY(cp(fl.data(), s->flags.p + first, count));
    HIP_TRY(cp(act.data(), s->act.p + li * PSIM_ACTIVE_CAP, act.size() * 4));
    HIP_TRY(cp(pas.data(), s->pas.p + li * PSIM_PASSIVE_CAP, pas.size() * 4));
    HIP_TRY(cp(sm.data(), s->sentm.p + li * IDMAP_IN, sm.size() * 8));
    HIP_TRY(cp(rm.data(), s->recvm.p + li * IDMAP_IN, rm.size() * 8));
    // the extension rows taken so far (few)
    const uint32_t top = s->mapx.p ? std::min<uint32_t>(read1(s, s->mapx_top.p), (uint32_t)(s->mapx.n / IDMAP_EXT)) : 0u;
    std::vector<uint64_t> xm((size_t)top * IDMAP_EXT);
    if (top) HIP_TRY(cp(xm.data(), s->mapx.p, xm.size() * 8));
    HIP_TRY(cp(all.data(), s->pt_all.p + li * PSIM_PT_MEMBERS_CAP, all.size() * 4));
    HIP_TRY(cp(com.data(), s->pt_com.p + li * PSIM_PT_MEMBERS_CAP, com.size() * 4));
    HIP_TRY(cp(eag.data(), s->pt_eag.p + li * RT_SET, eag.size() * 4));
    HIP_TRY(cp(laz.data(), s->pt_laz.p + li * RT_SET, laz.size() * 4));
    HIP_TRY(cp(rt.data(), s->pt_rt.p + li * RT_WORDS, rt.size() * 4));
    HIP_TRY(cp(po.data(), s->pt_out.p + li * OUT_IN, po.size() * 8));
    if (s->conn.p) HIP_TRY(cp(cn.data(), s->conn.p + li * PSIM_CONN_CAP, cn.size() * 4));
    const uint32_t otop = s->outx.p ? std::min<uint32_t>(read1(s, s->outx_top.p), (uint32_t)(s->outx.n / OUT_EXT)) : 0u;
    std::vector<uint64_t> xo((size_t)otop * OUT_EXT);
    if (otop) HIP_TRY(cp(xo.data(), s->outx.p, xo.size() * 8));
    HIP_TRY(hipStreamSynchronize(s->stream));
    for (uint32_t k = 0; k < count; k++) {
        psim_node_view* v = &out[k];
        const Hdr& x = hd[k];
        memset(v, 0, sizeof *v);
        v->up = fl[k] & F_UP; v->epoch = x.epoch; v->start_round = x.start_round;
        v->rng_ctr = x.rng;
        v->act_n = x.act_n; v->pas_n = x.pas_n;
        memcpy(v->act, &act[(size_t)k * PSIM_ACTIVE_CAP], sizeof v->act);
        memcpy(v->pas, &pas[(size_t)k * PSIM_PASSIVE_CAP], sizeof v->pas);
        v->sent_n = x.sent_n; v->sent_head = x.sent_head; v->recv_n = x.recv_n; v->recv_head = x.recv_head;
        const uint32_t sx = x.pad1[1], rx = x.pad1[2];
        for (uint32_t j = 0; j < PSIM_IDMAP_CAP; j++) {
            const uint64_t e = j < IDMAP_IN ? sm[(size_t)k * IDMAP_IN + j]
                             : sx && sx <= top ? xm[(size_t)(sx - 1) * IDMAP_EXT + j - IDMAP_IN] : 0ull;
            const uint64_t f = j < IDMAP_IN ? rm[(size_t)k * IDMAP_IN + j]
                             : rx && rx <= top ? xm[(size_t)(rx - 1) * IDMAP_EXT + j - IDMAP_IN] : 0ull;
            v->sent_peer[j] = (uint32_t)e; v->sent_id[j] = (uint32_t)(e >> 32);
            v->recv_peer[j] = (uint32_t)f; v->recv_id[j] = (uint32_t)(f >> 32);
        }
        v->pt_all_n = x.all_n; v->pt_common_n = x.com_n; v->pt_out_n = x.out_n;
        const uint32_t* r8 = &rt[(size_t)k * RT_WORDS];
        for (int q = 0; q < PSIM_PT_ROOTS; q++) {
            v->pt_root[q] = r8[q];
            v->pt_eager_n[q] = (r8[RT_EN] >> (8 * q)) & 0xFFu;
            v->pt_lazy_n[q] = (r8[RT_LN] >> (8 * q)) & 0xFFu;
        }
        memcpy(v->pt_all, &all[(size_t)k * PSIM_PT_MEMBERS_CAP], sizeof v->pt_all);
        memcpy(v->pt_common, &com[(size_t)k * PSIM_PT_MEMBERS_CAP], sizeof v->pt_common);
        memcpy(v->pt_eager, &eag[(size_t)k * RT_SET], sizeof v->pt_eager);
        memcpy(v->pt_lazy, &laz[(size_t)k * RT_SET], sizeof v->pt_lazy);
        const uint32_t ox = x.pad1[3];
        for (uint32_t j = 0; j < PSIM_PT_OUT_CAP; j++) {
            const uint64_t o = j >= x.out_n ? 0ull
                             : j < OUT_IN ? po[(size_t)k * OUT_IN + j]
                             : ox && ox <= otop ? xo[(size_t)(ox - 1) * OUT_EXT + j - OUT_IN] : 0ull;
            v->pt_out_peer[j] = (uint32_t)(o >> 32);
            v->pt_out_msg[j] = (uint32_t)(o >> 16) & 0xFFFFu;
            v->pt_out_round[j] = (uint32_t)o & 0xFFFFu;
        }
        v->have = ((uint64_t)x.aux << 32) | x.have; v->trk_round = x.trk_round; v->trk_hop = x.trk_hop;
        v->conn_n = x.conn_n;
        for (uint32_t j = 0; j < x.conn_n && j < PSIM_CONN_CAP; j++) v->conn[j] = cn[(size_t)k * PSIM_CONN_CAP + j];
    }
    return PSIM_OK;
}

// nodes [first, first+count): every node must be owned by a shard of this process
int psim_get_nodes(psim_handle* h, uint32_t first, uint32_t count, psim_node_view* out) {
    if (!h || (count && !out)) return PSIM_EINVAL;
    if ((uint64_t)first + count > h->N) return PSIM_ERANGE;
    if (hipSetDevice(h->device) != hipSuccess) return PSIM_EDEVICE;
    uint32_t done = 0;
    while (done < count) {
        uint32_t id = first + done;
        Shard* s = nullptr;
        for (Shard* c : h->shards)
            if (id >= c->lo && id < c->lo + c->n) s = c;
        if (!s) return PSIM_ERANGE;
        uint32_t k = std::min<uint32_t>(count - done, s->lo + s->n - id);
        int rc = get_shard_nodes(s, id, k, out + done);
        if (rc) return rc;
        done += k;
    }
    return PSIM_OK;
}

static uint64_t mix64_host(uint64_t z) {
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27; z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z;
}

static uint64_t members_hash(const uint32_t* row, uint32_t words) {
    uint64_t x = 0;
    for (uint32_t w = 0; w < words; w++)
        for (uint32_t v = row[w]; v; v &= v - 1) x += mix64_host((uint64_t)(w * 32 + (uint32_t)__builtin_ctz(v)) + 1);
    return x;
}

static Shard* owner_of(psim_handle* h, uint32_t id) {
    for (Shard* c : h->shards)
        if (id >= c->lo && id < c->lo + c->n) return c;
    return nullptr;
}

int psim_get_strategy_nodes(psim_handle* h, uint32_t first, uint32_t count, psim_strategy_view* out) {
    if (!h || (count && !out)) return PSIM_EINVAL;
    if (h->cfg.manager != PSIM_MANAGER_PLUGGABLE) return PSIM_ESTATE;
    if ((uint64_t)first + count > h->N) return PSIM_ERANGE;
    if (hipSetDevice(h->device) != hipSuccess) return PSIM_EDEVICE;
    const bool full = h->cfg.strategy == PSIM_STRATEGY_FULL;
    uint32_t done = 0;
    while (done < count) {
        uint32_t id = first + done;
        Shard* s = owner_of(h, id);
        if (!s) return PSIM_ERANGE;
        uint32_t k = std::min<uint32_t>(count - done, s->lo + s->n - id);
        const size_t li = id - s->lo;
        std::vector<Hdr> hd(k);
        std::vector<uint8_t> fl(k);
        std::vector<uint32_t> view, inv, rows;
        HIP_TRY(hipMemcpyAsync(hd.data(), s->hdr.p + li, k * sizeof(Hdr), hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(hipMemcpyAsync(fl.data(), s->flags.p + id, k, hipMemcpyDeviceToHost, s->stream));
        if (full) {
            rows.resize((size_t)k * 2 * h->fw);
            HIP_TRY(hipMemcpyAsync(rows.data(), s->fbits.p + li * 2 * h->fw, rows.size() * 4,
                                   hipMemcpyDeviceToHost, s->stream));
        } else {
            view.resize((size_t)k * PSIM_SVIEW_CAP);
            HIP_TRY(hipMemcpyAsync(view.data(), s->sview.p + li * PSIM_SVIEW_CAP, view.size() * 4,
                                   hipMemcpyDeviceToHost, s->stream));
            if (s->sinv.p) {
                inv.resize(view.size());
                HIP_TRY(hipMemcpyAsync(inv.data(), s->sinv.p + li * PSIM_SVIEW_CAP, inv.size() * 4,
                                       hipMemcpyDeviceToHost, s->stream));
            }
        }
        HIP_TRY(hipStreamSynchronize(s->stream));
        for (uint32_t j = 0; j < k; j++) {
            psim_strategy_view* v = &out[done + j];
            const Hdr& x = hd[j];
            memset(v, 0, sizeof *v);
            bool started = x.epoch != 0;       // k_join sets epoch >= 1
            v->up = fl[j] & F_UP; v->start_round = x.start_round; v->rng_ctr = x.rng;
            v->pending = started ? x.join_contact : PSIM_NONE;
            v->last_ping = started ? x.aux : PSIM_NONE;
            v->view_n = x.act_n; v->in_n = x.pas_n;
            if (full) {
                const uint32_t* row = &rows[(size_t)j * 2 * h->fw];
                std::vector<uint32_t> mem(h->fw);
                uint32_t c = 0;
                for (uint32_t w = 0; w < h->fw; w++) {
                    mem[w] = row[w] & ~row[h->fw + w];       // add & ~remove
                    c += (uint32_t)__builtin_popcount(mem[w]);
                }
                v->members = c;
                v->members_hash = members_hash(mem.data(), h->fw);
            } else {
                memcpy(v->view, &view[(size_t)j * PSIM_SVIEW_CAP], sizeof v->view);
                if (h->cfg.strategy == PSIM_STRATEGY_SCAMP_V1 && x.act_n) v->view_slots = 16 + x.pad1[1];
                if (!inv.empty()) memcpy(v->in_view, &inv[(size_t)j * PSIM_SVIEW_CAP], sizeof v->in_view);
            }
        }
        done += k;
    }
    return PSIM_OK;
}

int psim_get_member_bits(psim_handle* h, uint32_t node, uint32_t* words, size_t n_words) {
    if (!h || !words) return PSIM_EINVAL;
    if (h->cfg.manager != PSIM_MANAGER_PLUGGABLE || h->cfg.strategy != PSIM_STRATEGY_FULL) return PSIM_ESTATE;
    if (node >= h->N) return PSIM_ERANGE;
    const uint32_t W = (h->N + 31) / 32;
    if (n_words < W) return PSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return PSIM_EDEVICE;
    Shard* s = owner_of(h, node);
    if (!s) return PSIM_ERANGE;
    std::vector<uint32_t> row(2 * h->fw);
    HIP_TRY(hipMemcpyAsync(row.data(), s->fbits.p + (size_t)(node - s->lo) * 2 * h->fw, row.size() * 4,
                           hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    for (uint32_t w = 0; w < W; w++) words[w] = row[w] & ~row[h->fw + w];
    return PSIM_OK;
}


int psim_get_delivery(psim_handle* h, uint32_t first, uint32_t count, uint8_t* have, uint32_t* round,
                      uint32_t* hop) {
    if (!h || (count && (!have || !round || !hop))) return PSIM_EINVAL;
    if ((uint64_t)first + count > h->N) return PSIM_ERANGE;
    if (hipSetDevice(h->device) != hipSuccess) return PSIM_EDEVICE;
    const uint64_t bit = h->tracked_msg == PSIM_NONE ? 0ull : 1ull << (h->tracked_msg % PSIM_MSG_SLOTS);
    uint32_t done = 0;
    while (done < count) {
        const uint32_t id = first + done;
        Shard* s = owner_of(h, id);
        if (!s) return PSIM_ERANGE;
        const uint32_t k = std::min<uint32_t>(count - done, s->lo + s->n - id);
        std::vector<Hdr> hd(k);
        HIP_TRY(hipMemcpyAsync(hd.data(), s->hdr.p + (id - s->lo), k * sizeof(Hdr), hipMemcpyDeviceToHost,
                               s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));
        for (uint32_t j = 0; j < k; j++) {
            have[done + j] = ((((uint64_t)hd[j].aux << 32) | hd[j].have) & bit) ? 1 : 0;
            round[done + j] = hd[j].trk_round;
            hop[done + j] = hd[j].trk_hop;
        }
        done += k;
    }
    return PSIM_OK;
}

int psim_get_histograms(psim_handle* h, psim_histograms* out) {
    if (!h || !out) return PSIM_EINVAL;
    if (h->cfg.manager == PSIM_MANAGER_PLUGGABLE) return PSIM_EUNSUPPORTED;
    if (hipSetDevice(h->device) != hipSuccess) return PSIM_EDEVICE;
    memset(out, 0, sizeof *out);
    Shard* s0 = h->shards[0];
    hipStream_t st = s0->stream;
    for (Shard* s : h->shards) HIP_TRY(hipStreamSynchronize(s->stream));
    const size_t N = h->N;
    TmpBuf<uint32_t> ind;                        // in-degrees, active then passive, by global id
    TmpBuf<unsigned long long> hist;
    TRY(ind.alloc_on(2 * N, st));
    TRY(hist.alloc_on(H_N + 4, st));
    const uint64_t tbit = h->tracked_msg == PSIM_NONE ? 0ull : 1ull << (h->tracked_msg % PSIM_MSG_SLOTS);
    for (Shard* s : h->shards)
        k_hist_out<<<grid_for(s->n), BLK, 0, st>>>(s->hdr.p, s->act.p, s->pas.p, s->flags.p, s->lo, s->n, tbit,
                                                   ind.p, ind.p + N, hist.p);
    if (h->ranked) {
        TRY(h->comm->all_reduce(ind.p, 2 * N, CType::U32, COp::SUM, st));
    }
    for (Shard* s : h->shards)
        k_hist_in<<<grid_for(s->n), BLK, 0, st>>>(ind.p, ind.p + N, s->flags.p, s->lo, s->n, hist.p);
    std::vector<unsigned long long> hv(H_N + 4, 0);
    HIP_TRY(hipMemcpyAsync(hv.data(), hist.p, (H_N + 4) * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (h->ranked) {                             // sums over ranks; the latest round: max
        hv[H_N] = hv[H_LAST];
        TRY(h->comm_cnt.ensure(H_N + 4));
        HIP_TRY(hipMemcpyAsync(h->comm_cnt.p, hv.data(), (H_N + 4) * 8, hipMemcpyHostToDevice, st));
        TRY(h->comm->all_reduce(h->comm_cnt.p, H_N, CType::U64, COp::SUM, st));
        TRY(h->comm->all_reduce(h->comm_cnt.p + H_N, 1, CType::U64, COp::MAX, st));
        HIP_TRY(hipMemcpyAsync(hv.data(), h->comm_cnt.p, (H_N + 4) * 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        hv[H_LAST] = hv[H_N];
    }
    for (int k = 0; k < PSIM_HIST_BINS; k++) {
        out->active_in[k] = hv[H_AIN * PSIM_HIST_BINS + k];
        out->passive_in[k] = hv[H_PIN * PSIM_HIST_BINS + k];
        out->active_out[k] = hv[H_AOUT * PSIM_HIST_BINS + k];
        out->passive_fill[k] = hv[H_PFILL * PSIM_HIST_BINS + k];
        out->hop[k] = hv[H_HOP * PSIM_HIST_BINS + k];
    }
    out->n_up = hv[H_NUP]; out->delivered = hv[H_DELIV]; out->last_round = hv[H_LAST];
    out->active_links = hv[H_LINKS];
    {
        // symmetry and components need every node's active row: the shards'
        // rows are gathered by global id (device copies for virtual shards,
        // an in-place ncclAllGather of equal per-rank slots for RCCL ranks;
        // 33 B per node), and every process then runs the same kernels over
        // the whole overlay
        const uint32_t per = h->per, n = h->N;
        const size_t npad = (size_t)per * h->G;
        TmpBuf<uint32_t> gact, L, sz, flag;
        TmpBuf<uint8_t> gan;
        TmpBuf<unsigned long long> r;
        TRY(gact.alloc_on(npad * PSIM_ACTIVE_CAP, st)); TRY(gan.alloc_on(npad, st));
        for (Shard* s : h->shards)
            if (s->n)
                k_pack_act<<<grid_for(s->n), BLK, 0, st>>>(s->hdr.p, s->act.p, s->n,
                                                           gact.p + (size_t)s->lo * PSIM_ACTIVE_CAP, gan.p + s->lo);
        if (h->ranked) {
            const size_t off = (size_t)h->rank * per;
            TRY(h->comm->all_gather(gact.p + off * PSIM_ACTIVE_CAP, gact.p, (size_t)per * PSIM_ACTIVE_CAP * 4, st));
            TRY(h->comm->all_gather(gan.p + off, gan.p, per, st));
        }
        const uint8_t* fl = s0->flags.p;         // replicated: every shard holds all N
        TRY(L.alloc_on(n, st)); TRY(sz.alloc_on(n, st)); TRY(flag.alloc_on(1, st)); TRY(r.alloc_on(3, st));
        k_hist_sym<<<grid_for(n), BLK, 0, st>>>(gan.p, gact.p, fl, n, r.p);
        k_cc_init<<<grid_for(n), BLK, 0, st>>>(fl, n, L.p);
        for (int it = 0; it < 4096; it++) {
            uint32_t changed = 0;
            HIP_TRY(hipMemsetAsync(flag.p, 0, 4, st));
            k_cc_hook<<<grid_for(n), BLK, 0, st>>>(gan.p, gact.p, fl, n, L.p, flag.p);
            k_cc_jump<<<grid_for(n), BLK, 0, st>>>(n, L.p);
            HIP_TRY(hipMemcpyAsync(&changed, flag.p, 4, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            if (!changed) break;
        }
        k_cc_count<<<grid_for(n), BLK, 0, st>>>(L.p, n, sz.p, r.p + 1);
        k_cc_max<<<grid_for(n), BLK, 0, st>>>(sz.p, n, r.p + 2);
        unsigned long long rv[3];
        HIP_TRY(hipMemcpyAsync(rv, r.p, sizeof rv, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        out->symmetric_links = rv[0]; out->components = rv[1]; out->largest_component = rv[2];
    }
    return PSIM_OK;
}


// ----------------------------------------------------------- snapshot --
// Layout: SnapHead, then per local shard a ShardHead and its arrays in
// snap_sections() order.  Pending (not yet applied) events are not state:
// a snapshot with events pending is refused.
struct SnapHead {
    uint32_t magic, abi, n_nodes, n_local_shards, manager, strategy, fw, started_n;
    uint64_t round;
    uint32_t tracked_msg, btab_hash, G, world;
    uint32_t slot_tab[2 * PSIM_MSG_SLOTS];
};
struct ShardHead {
    uint32_t lo, n, m_in, in_cur, pay_cur, pay_rows, pad[2];
    uint32_t out_rows, pad2[3];     // outstanding extension rows taken
};
constexpr uint32_t SNAP_MAGIC = 0x4D495350u;   // "PSIM"

struct Section { void* p; size_t bytes; };

// the arrays that make up a shard's state between rounds
static std::vector<Section> snap_sections(psim_handle* h, Shard* s, const ShardHead& sh) {
    const size_t N = h->N, n = s->n;
    std::vector<Section> v = {
        {s->flags.p, N}, {s->part.p, N}, {s->hdr.p, n * sizeof(Hdr)},
        {s->act.p, n * PSIM_ACTIVE_CAP * 4}, {s->pas.p, n * PSIM_PASSIVE_CAP * 4},
        {s->sentm.p, n * IDMAP_IN * 8}, {s->recvm.p, n * IDMAP_IN * 8},
        {s->mapx.p, (size_t)sh.pad[1] * IDMAP_EXT * 8},
        {s->pt_all.p, n * PSIM_PT_MEMBERS_CAP * 4}, {s->pt_com.p, n * PSIM_PT_MEMBERS_CAP * 4},
        {s->pt_eag.p, n * RT_SET * 4}, {s->pt_laz.p, n * RT_SET * 4}, {s->pt_rt.p, n * RT_WORDS * 4},
        {s->pt_out.p, n * OUT_IN * 8}, {s->outx.p, (size_t)sh.out_rows * OUT_EXT * 8}, {s->start.p, n * 4},
        {s->conn.p, s->conn.p ? n * PSIM_CONN_CAP * 4 : 0},
        {s->cb.p, (n + 1) * 8}, {s->bmask.p, n * 8}, {s->in_beg.p, (n + 1) * 4},
        {s->inbox.p, (size_t)sh.m_in * sizeof(Msg)},
    };
    if (h->cfg.manager == PSIM_MANAGER_PLUGGABLE) {
        if (s->sview.p) v.push_back({s->sview.p, n * PSIM_SVIEW_CAP * 4});
        if (s->sinv.p) v.push_back({s->sinv.p, n * PSIM_SVIEW_CAP * 4});
        if (s->fbits.p) v.push_back({s->fbits.p, n * 2 * h->fw * 4});
        if (sh.pay_rows) v.push_back({s->pay[sh.pay_cur ^ 1].p, (size_t)sh.pay_rows * 2 * h->fw * 4});
    }
    return v;
}

int psim_snapshot(psim_handle* h, void* buf, size_t cap, size_t* need) {
    if (!h || !need) return PSIM_EINVAL;
    if (!h->pend_crash.empty() || !h->pend_join.empty() || !h->pend_lv_a.empty() || h->pend_part_set || h->pend_part_clear ||
        !h->pend_b_root.empty() || h->faults || h->faults_dirty)   // (faults: host state, not snapshotted)
        return PSIM_ESTATE;
    if (hipSetDevice(h->device) != hipSuccess) return PSIM_EDEVICE;
    std::vector<ShardHead> heads;
    size_t total = sizeof(SnapHead) + h->started.size();
    for (Shard* s : h->shards) {
        HIP_TRY(hipStreamSynchronize(s->stream));
        ShardHead sh{s->lo, s->n, s->m_in, 0u, (uint32_t)s->pay_cur, 0, {0, 0}, 0, {0, 0, 0}};
        if (h->cfg.manager == PSIM_MANAGER_PLUGGABLE && s->pay_top.p)
            sh.pay_rows = read1(s, s->pay_top.p);
        sh.pad[0] = s->tomb_live ? 1u : 0u;            // full: snapshots carry remove rows
        sh.pad[1] = s->mapx.p ? std::min<uint32_t>(read1(s, s->mapx_top.p), (uint32_t)(s->mapx.n / IDMAP_EXT)) : 0u;
        sh.out_rows = s->outx.p ? std::min<uint32_t>(read1(s, s->outx_top.p), (uint32_t)(s->outx.n / OUT_EXT)) : 0u;
        heads.push_back(sh);
        total += sizeof(ShardHead);
        for (const Section& x : snap_sections(h, s, sh)) total += x.bytes;
    }
    *need = total;
    if (!buf || cap < total) return PSIM_OK;
    char* o = static_cast<char*>(buf);
    SnapHead hd{SNAP_MAGIC, PSIM_ABI_VERSION, h->N, (uint32_t)h->shards.size(), h->cfg.manager, h->cfg.strategy,
                h->fw, (uint32_t)h->started.size(), h->round, h->tracked_msg, h->btab_hash, h->G, (uint32_t)h->world, {}};
    memcpy(hd.slot_tab, h->slot_tab, sizeof h->slot_tab);
    memcpy(o, &hd, sizeof hd); o += sizeof hd;
    if (!h->started.empty()) { memcpy(o, h->started.data(), h->started.size()); o += h->started.size(); }
    for (size_t k = 0; k < h->shards.size(); k++) {
        Shard* s = h->shards[k];
        memcpy(o, &heads[k], sizeof(ShardHead)); o += sizeof(ShardHead);
        for (const Section& x : snap_sections(h, s, heads[k])) {
            if (x.bytes) HIP_TRY(hipMemcpy(o, x.p, x.bytes, hipMemcpyDeviceToHost));
            o += x.bytes;
        }
    }
    return PSIM_OK;
}

int psim_restore(psim_handle* h, const void* buf, size_t size) {
    if (!h || !buf || size < sizeof(SnapHead)) return PSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return PSIM_EDEVICE;
    const char* o = static_cast<const char*>(buf);
    const char* end = o + size;
    SnapHead hd;
    memcpy(&hd, o, sizeof hd); o += sizeof hd;
    if (hd.magic != SNAP_MAGIC || hd.abi != PSIM_ABI_VERSION || hd.n_nodes != h->N ||
        hd.n_local_shards != h->shards.size() || hd.manager != h->cfg.manager || hd.strategy != h->cfg.strategy ||
        hd.fw != h->fw || hd.G != h->G || hd.world != (uint32_t)h->world)
        return PSIM_EINVAL;
    if (hd.btab_hash != h->btab_hash) return PSIM_EINVAL;   // another view-order table
    // the whole layout is checked before any state changes: every shard head
    // and every section must lie inside the buffer, so a short or mismatched
    // snapshot leaves the handle as it was
    {
        const char* q = o;
        if ((size_t)(end - q) < hd.started_n) return PSIM_EINVAL;
        q += hd.started_n;
        for (Shard* s : h->shards) {
            if ((size_t)(end - q) < sizeof(ShardHead)) return PSIM_EINVAL;
            ShardHead sh;
            memcpy(&sh, q, sizeof sh); q += sizeof sh;
            if (sh.lo != s->lo || sh.n != s->n || sh.pay_cur > 1) return PSIM_EINVAL;
            if ((size_t)sh.pad[1] * IDMAP_EXT > s->mapx.n) return PSIM_EINVAL;
            if (sh.out_rows && !s->outx.p) return PSIM_EINVAL;
            for (const Section& x : snap_sections(h, s, sh)) {
                if ((size_t)(end - q) < x.bytes) return PSIM_EINVAL;
                q += x.bytes;
            }
        }
    }
    // from here on a failure (an allocation, a copy) leaves a half-restored
    // state: the handle stays failed (psim_step answers PSIM_ESTATE) until a
    // restore succeeds
    h->failed = true;
    if (hd.started_n) {
        h->started.assign(o, o + hd.started_n); o += hd.started_n;
    }
    for (Shard* s : h->shards) {
        HIP_TRY(hipStreamSynchronize(s->stream));
        ShardHead sh;
        memcpy(&sh, o, sizeof sh); o += sizeof sh;
        s->m_in = sh.m_in; s->pay_cur = (int)sh.pay_cur;
        s->tomb_live = sh.pad[0] != 0;
        if (s->tomb_live) h->tomb = true;
        TRY(s->inbox.ensure((size_t)sh.m_in + 1));
        if (sh.pay_rows) TRY(s->pay[s->pay_cur ^ 1].ensure((size_t)sh.pay_rows * 2 * h->fw));
        if (h->cfg.manager == PSIM_MANAGER_PLUGGABLE && s->pay_top.p)
            HIP_TRY(hipMemcpy(s->pay_top.p, &sh.pay_rows, 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(s->mapx_top.p, &sh.pad[1], 4, hipMemcpyHostToDevice));
        if (s->outx.p) {
            // (a grown pool: this handle's grows to hold the snapshot's rows;
            // the rows past them zeroed, as a fresh pool's are)
            TRY(s->outx.ensure((size_t)sh.out_rows * OUT_EXT));
            HIP_TRY(hipMemset(s->outx.p + (size_t)sh.out_rows * OUT_EXT, 0,
                              (s->outx.n - (size_t)sh.out_rows * OUT_EXT) * 8));
            s->pin[PIN_OUTX] = sh.out_rows;
        }
        HIP_TRY(hipMemcpy(s->outx_top.p, &sh.out_rows, 4, hipMemcpyHostToDevice));
        for (const Section& x : snap_sections(h, s, sh)) {
            if (x.bytes) HIP_TRY(hipMemcpy(x.p, o, x.bytes, hipMemcpyHostToDevice));
            o += x.bytes;
        }
        // the per-round words a round that failed half-way may have left set
        // (a broadcast's origin entries, crashed-this-round bits, the batch
        // abort word, the stop list): a round boundary has them clear
        if (s->origin.p) HIP_TRY(hipMemset(s->origin.p, 0, s->origin.n * sizeof(uint32_t)));
        if (s->crash_bits.p) HIP_TRY(hipMemset(s->crash_bits.p, 0, s->crash_bits.n * sizeof(uint32_t)));
        if (s->ctl.p) HIP_TRY(hipMemset(s->ctl.p, 0, s->ctl.n * sizeof(uint32_t)));
        if (s->n_stop.p) HIP_TRY(hipMemset(s->n_stop.p, 0, s->n_stop.n * sizeof(uint32_t)));
        s->reserved = false;
        s->upart_valid = false;
    }
    h->round = hd.round; h->tracked_msg = hd.tracked_msg;
    memcpy(h->slot_tab, hd.slot_tab, sizeof h->slot_tab);
    for (Shard* s : h->shards)
        HIP_TRY(hipMemcpy(s->slots.p, h->slot_tab, sizeof h->slot_tab, hipMemcpyHostToDevice));
    HIP_TRY(hipDeviceSynchronize());
    // back on a round boundary: a handle a failed step poisoned runs again
    h->failed = false;
    h->pend_crash.clear(); h->pend_join.clear(); h->pend_contact.clear();
    h->pend_lv_a.clear(); h->pend_lv_t.clear();
    h->pend_join_mark.assign(h->pend_join_mark.size(), 0);
    h->pend_part_set = h->pend_part_clear = false;
    h->pend_b_root.clear(); h->pend_b_msg.clear();
    return PSIM_OK;
}

int psim_get_exchange_stats(psim_handle* h, uint64_t* records, uint64_t* bytes) {
    if (!h || !records || !bytes) return PSIM_EINVAL;
    *records = h->x_records;
    *bytes = h->x_bytes;
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

// diagnostic: per node-round kernel of the last round (shard 0's blocks; the
// stats rows every block leaves, before the route sums them), in the order
// k_relay, k_shuf, k_lite_half / k_consume_lite, k_consume, k_ptl,
// k_pt: out[4 k] nodes processed (stats nodes_processed), out[4 k + 1]
// records delivered, out[4 k + 2] records emitted, out[4 k + 3] 0; with cap
// >= 28 then k_node_prep's quiet lazy ticks (nodes processed without a
// kernel).  Returns the number of entries (6 or 7); 0 for the pluggable
// manager's one kernel.
int psim_debug_kernel_counts(psim_handle* h, uint64_t* out, int cap) {
    if (!h || !out || cap < 24) return PSIM_EINVAL;
    if (h->cfg.manager == PSIM_MANAGER_PLUGGABLE) return 0;
    Shard* s = h->shards[0];
    const uint32_t rows = s->pgrid + s->cgrid + s->rgrid + s->tgrid + s->sgrid + s->lgrid + s->qgrid;
    std::vector<uint64_t> st((size_t)rows * NST);
    HIP_TRY(hipStreamSynchronize(s->stream));
    HIP_TRY(hipMemcpy(st.data(), s->stat_part.p, st.size() * 8, hipMemcpyDeviceToHost));
    // row ranges (make_args: prepare, consume, relay, pt, shuf, lite, ptl)
    const uint32_t b_cons = s->pgrid, b_rel = b_cons + s->cgrid, b_pt = b_rel + s->rgrid, b_sh = b_pt + s->tgrid,
                   b_li = b_sh + s->sgrid, b_pl = b_li + s->lgrid, b_end = b_pl + s->qgrid;
    const uint32_t rng[7][2] = {{b_rel, b_pt}, {b_sh, b_li}, {b_li, b_pl}, {b_cons, b_rel}, {b_pl, b_end}, {b_pt, b_sh},
                                {0, b_cons}};
    const int nk = cap >= 28 ? 7 : 6;
    for (int k = 0; k < nk; k++) {
        uint64_t v[3] = {0, 0, 0};
        for (uint32_t r = rng[k][0]; r < rng[k][1]; r++) {
            const uint64_t* row = st.data() + (size_t)r * NST;
            v[0] += row[ST_PROC];
            for (int t = 0; t < ST_NTYPES; t++) { v[1] += row[ST_DELIV + t]; v[2] += row[ST_EMIT + t]; }
        }
        out[4 * k] = v[0]; out[4 * k + 1] = v[1]; out[4 * k + 2] = v[2]; out[4 * k + 3] = 0;
    }
    return nk;
}

// diagnostic: per-phase s_memtime sums of k_consume / k_pt, k_consume_lite and
// k_lite_half (96 entries; 0 returned unless built with -DPSIM_STAMPS)
int psim_debug_stamps(unsigned long long* out, int cap) {
    if (!out || cap < 96) return PSIM_EINVAL;
    return psim::debug_stamps(out);
}

int psim_comm_id_size(void) { return (int)sizeof(ncclUniqueId); }

// a loopback world's id (test vehicle of the rank code path, psim_comm.h)
int psim_loopback_comm_id(void* buf, size_t cap) { return psim::loopback_new_id(buf, cap); }

int psim_get_comm_id(void* buf, size_t cap) {
    if (!buf || cap < sizeof(ncclUniqueId)) return PSIM_EINVAL;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return PSIM_ECOMM;
    memcpy(buf, &id, sizeof id);
    return PSIM_OK;
}

}  // extern "C"
