// psim_kernels.h -- kernel argument blocks shared by the kernel TUs and the host.
#pragma once
#include <stddef.h>

#include "psim_device.h"

namespace psim {

// the up-and-partition pair of a node (RoundArgs::upart): its partition
// group while it is up, UPART_DOWN if not -- one byte (groups 0..254:
// psim_set_partition), so the array is the size of the flag bytes (64 MB at
// 2^26 nodes) and caches as well; PSIM_UPART8=0 keeps round 4's 2-byte pairs
// (A/B builds)
#ifndef PSIM_UPART8
#define PSIM_UPART8 1
#endif
#if PSIM_UPART8
typedef uint8_t upart_t;
#else
typedef uint16_t upart_t;
#endif

struct RoundArgs {
    // config
    uint32_t n_nodes, round;
    uint32_t lo, n_local;       // this shard owns global ids [lo, lo + n_local)
    uint64_t seed;
    uint32_t max_active, min_active, max_passive, arwl, prwl, k_active, k_passive;
    uint32_t shuffle_period, promotion_period, random_promotion, plumtree, lazy_tick_period;
    uint32_t xbot, xbot_period;   // X-BOT manager (PSIM_MANAGER_XBOT) and its xbot_execution period
    // per-round scalars
    uint32_t crash_round, tracked_msg;
    uint32_t upart_dirty;       // this round's events changed F_UP or a partition: k_node_prep rebuilds upart
    uint32_t lazy_wake;         // this round's events may connect a quiet node's outstanding peers (a
                                // partition change, faults, a leave, a fresh or restored state): every
                                // quiet node runs its lazy tick (k_node_prep, F_LAZY)
    // node state: flags/part are replicated and indexed by global id;
    // every other row is local (index = id - lo)
    uint8_t* flags;
    const uint8_t* part;
    // per global id: its partition group while it is up, UPART_DOWN if not --
    // built by k_node_prep after the round's events (F_UP and the groups
    // change only there), so a connection test of a peer reads one byte pair
    // instead of a flag byte and a partition byte on two random lines (k_ptl:
    // eight members a node, 63 GB a round at 2^26 before; k_relay, k_shuf,
    // k_lite_half likewise; HyParView / X-BOT handles only)
    upart_t* upart;
    // per local node of k_relay's lite list: bit j = active member j is up in
    // this node's partition group (k_relay reads the pairs for it before its
    // list appends; k_lite_half reads the byte with the node's rows, a node
    // ahead, instead of eight dependent pair loads as the node starts)
    uint8_t* lite_cm;
    // this round's crashed ids, one bit per CRASH_GRAIN ids (replicated,
    // zero outside crash rounds): a filter in L2 in front of the flag bytes
    const uint32_t* crash_bits;
    // the sets v1 bucket of every global id (psim_set_bucket_table), or
    // nullptr for the default (bucket16_default): the view order of App. A Q1
    const uint8_t* btab;
    Hdr* hdr;
    uint32_t *act, *pas;
    uint64_t *sentm, *recvm;    // id maps: the IDMAP_IN own entries, id << 32 | peer
    uint64_t* mapx;             // id-map extension rows (IDMAP_EXT entries), a shared pool
    uint32_t* mapx_top;         // pool rows taken
    uint32_t mapx_rows;         // pool rows
    uint32_t *pt_all, *pt_com, *pt_eag, *pt_laz, *pt_rt;
    uint32_t* conn;             // connections beyond the active view: PSIM_CONN_CAP per node
                                // (Hdr conn_n / conn_dn)
    uint64_t* pt_out;           // outstanding: the OUT_IN own entries
    uint64_t* outx;             // outstanding extension rows (OUT_EXT entries), a shared pool
    uint32_t* outx_top;
    uint32_t outx_rows;
    // broadcasts: per local node the message id + 1 it originates this
    // round (0 = none); the message slots (id of slot k in word k, its root
    // in word PSIM_MSG_SLOTS + k, PSIM_NONE = free)
    const uint32_t* origin;
    const uint32_t* slots;
    // inbox (this round) and outbox (next round)
    const uint32_t* in_beg;
    const unsigned long long* in_cb;   // inbox count | emission-bound sum << 32
    const uint32_t* start;      // start round per node (timer phases)
    const uint4* desc;          // per node with work: (id, inbox begin, inbox count, outbox base)
    const uint32_t* n_alist;
    // k_relay: the nodes it leaves to k_consume (desc_slow[0..*n_slow)), its
    // per-block stats rows
    uint4* desc_slow;
    uint32_t* n_slow;
    uint4* desc_pt;             // ... and the nodes with Plumtree work, for k_pt
    uint32_t* n_pt;
    uint4* desc_shuf;           // ... and the nodes whose HyParView phase ends in a shuffle start, for k_shuf
    uint32_t* n_shuf;
    uint64_t* stat_shuf;        // k_shuf's per-block stats rows
    uint4* desc_lite;           // ... and the nodes with SHUFFLE terminals / replies, for k_lite_half:
    uint32_t* n_lite;           // 2 n_local slots, four bins (lite_at): [0] and [1] from the first
                                // half's front and back, [2] and [3] from the second's
    uint64_t* stat_lite;        // k_consume_lite's per-block stats rows
    uint4* desc_ptl;            // ... and the nodes with Plumtree work and no origin, for k_ptl:
    uint32_t* n_ptl;            // [0] from the front, those with a BROADCAST in their inbox, [1] from
                                // the back (desc_ptl[n_local - 1 - i]), the others (ptl_desc)
    uint64_t* stat_ptl;         // k_ptl's per-block stats rows
    uint64_t* stat_relay;
    uint64_t* stat_pt;          // k_pt's per-block stats rows
    const Msg* rec_in;          // dense, in inbox order (node runs at in_beg)
    const uint64_t* obase;
    Msg* rec_out;
    uint32_t* okey;
    uint32_t* ocnt;
    uint64_t* stat_part;   // [gridDim.x][NST]
    // the node-round phase's span (s_memrealtime, 100 MHz): [0] stamped by
    // k_relay's first block as it starts, [1] by the first kernel after the
    // phase (the route's first pass) as it starts -- two stores a round on
    // the shard's stream, no marker launches and no same-address atomics
    // (the pluggable kernel takes its own min start / max end); reset by
    // k_node_prep
    unsigned long long* ktime;
    // the batch's abort word (psim_engine.hip run_batch): nonzero once a round
    // of the batch has overflowed a buffer; every kernel that reads or writes
    // round state returns at once (uniformly, before any barrier)
    const uint32_t* ctl;
    // pluggable manager (k_consume_pl); Hdr fields are reused as
    // join_contact = pending contact, aux = last ping round,
    // have = hello sent, act_n = view length, pas_n = in_view length
    uint32_t pl, strategy, periodic, scamp_c, fanout;
    uint32_t fw;                 // full: words per member bitset (multiple of 4); a node's row
                                 // is 2 fw words: adds, then removes (ORSet tombstones)
    uint32_t tomb;               // full: removes exist -- read and carry the remove rows
    uint32_t* fbits;             // full: n_local rows of fw words
    const uint32_t* pay_in;      // full: snapshots read this round (slot * fw)
    uint32_t* pay_out;           // full: snapshots written this round
    uint32_t* pay_top;           // full: next free slot of pay_out
    uint32_t pay_cap;
    uint32_t* sview;             // scamp: n_local rows of PSIM_SVIEW_CAP ids
    uint32_t* sinv;              // scamp v2: in_view rows
    uint32_t* stop_ids;          // pluggable: managers that stopped this round
    uint32_t* n_stop;            //   (their count, reset by k_node_prep)
    // pluggable: omission faults (interposition funs, pl:297-326): the
    // generally omitting nodes (global id) and the sorted pair keys
    // src << 32 | dst of the send omissions, then those of the receive
    // omissions; `faults` = any installed (else nothing is read)
    uint32_t faults, n_omit_s, n_omit_r;
    const uint8_t* faulted;
    const uint64_t* omit;
};

__global__ void k_consume(RoundArgs args);
// lane-per-node SHUFFLE relays ahead of k_consume (psim_consume.hip)
constexpr uint32_t RELAY_MAX_BLOCKS = 8192;
constexpr uint32_t SHUF_MAX_BLOCKS = 1024;     // k_shuf: grid-stride over its list
#ifndef PSIM_PTL_BLOCK
#define PSIM_PTL_BLOCK 64
#endif
// k_ptl's block (psim_consume.hip PTL_BLK): one wave, so that its 224 B of
// LDS per lane leave no block-sized hole (9 resident blocks per CU against 4
// of 128 lanes, measured 2 % faster); the grid strides over its list with
// the resident blocks (ptl_grid())
constexpr uint32_t PTL_BLOCK = PSIM_PTL_BLOCK;
__global__ void k_relay(RoundArgs args);
__global__ void k_consume_pl(RoundArgs args);
// lane-per-node shuffle starts of the nodes k_relay listed (psim_consume.hip)
__global__ void k_shuf(RoundArgs args);
// wave-per-node SHUFFLE terminals, replies and their merges (psim_consume.hip)
__global__ void k_consume_lite(RoundArgs args);
// the same with two nodes per wave, one per 32-lane half (psim_lite.hip)
__global__ void k_lite_half(RoundArgs args);
uint32_t lite_half_grid();
uint32_t lite_half_block();
// lane-per-node Plumtree phases (psim_consume.hip); hands k_pt what does not fit
__global__ void k_ptl(RoundArgs args);
// the Plumtree phase of the nodes k_relay listed (psim_consume.hip)
__global__ void k_pt(RoundArgs args);
// diagnostic builds (-DPSIM_STAMPS): per-phase cycle sums of k_consume, reset on read
int debug_stamps(unsigned long long* out);
int debug_stamps_half(unsigned long long* out);   // k_lite_half's 32 (psim_lite.hip)
// resident-block count of k_consume on the current device
uint32_t consume_grid();
uint32_t lite_grid();
uint32_t lite_block();
uint32_t pt_grid();
uint32_t ptl_grid();

// The launch's RoundArgs, read through an opaque constant-address pointer
// (in a kernel whose only argument is a RoundArgs): each helper re-reads the
// fields it needs with scalar loads, instead of the kernel holding all 188
// dwords of arguments in SGPRs (which spilled to VGPR lanes: a v_readlane
// per reuse on the hot path).
// a crash round's EXIT scan: is peer `id` one of this round's crashed nodes?
// (every node tests its active members and connections: 14 random flag-byte
// loads per node from HBM, 5 ms a crash round at 2^26 nodes; the 512 KB
// filter answers ~97 % of them from L2 -- 134k crashes in 4M grains)
constexpr uint32_t CRASH_GRAIN_SHIFT = 4;
constexpr upart_t UPART_DOWN = (upart_t)(PSIM_UPART8 ? 0xFFu : 0x100u);
__device__ __forceinline__ bool crash_filter(const uint32_t* bits, uint32_t id) {
    const uint32_t g = id >> CRASH_GRAIN_SHIFT;
    return (bits[g >> 5] >> (g & 31)) & 1u;
}
template <class Args>   // (RoundArgs or the kernarg view KArgs)
__device__ __forceinline__ bool crashed_now(Args& a, uint32_t id) {
    return crash_filter(a.crash_bits, id) && (a.flags[id] & F_CRASHED);
}

typedef const __attribute__((address_space(4))) RoundArgs KArgs;

// entry i of k_ptl's list: the BROADCAST nodes k_relay put at the front, then
// the others it put at the back -- so a wave's lanes mostly run the same
// handlers (a first delivery's eager push and lazy adds, or the light IHAVE
// answers, acks and lazy ticks), not the union of both
template <class Args>
__device__ __forceinline__ uint4 ptl_desc(Args& a, uint32_t n0, uint32_t i) {
    return a.desc_ptl[i < n0 ? i : a.n_local - 1 - (i - n0)];
}
// entry i of the lite list, in four bins k_relay fills: nodes with a SHUFFLE
// terminal (a sublist of the passive view, a reply and a merge) and nothing
// else, nodes with only replies' merges, then the same two with more work
// beside (SHUFFLE relays in the inbox, a due shuffle start) -- k_lite_half
// pairs adjacent entries in a wave's two halves, so most pairs run the same
// handlers and neither half waits on the other's extra work
template <class Args>
__device__ __forceinline__ uint32_t lite_at(Args& a, const uint32_t (&c)[4], uint32_t i) {
    const uint32_t n = a.n_local;
    return i < c[0] ? i
         : i < c[0] + c[1] ? n - 1 - (i - c[0])
         : i < c[0] + c[1] + c[2] ? n + (i - c[0] - c[1])
         : 2 * n - 1 - (i - c[0] - c[1] - c[2]);
}
template <class Args>
__device__ __forceinline__ void lite_counts(Args& a, uint32_t (&c)[4], uint32_t& na) {
    c[0] = a.n_lite[0]; c[1] = a.n_lite[1]; c[2] = a.n_lite[2]; c[3] = a.n_lite[3];
    na = c[0] + c[1] + c[2] + c[3];
}
// A record without exchange ids (nex == 0 in its type word: Plumtree,
// DISCONNECT, NEIGHBOR_*) leaves its last 32 B unwritten in the outbox; the
// route's gather writes zeros there (as the exchange's wire format does)
// (PSIM_SHORT_TAIL=0: every tail written and copied, for A/B)
#ifndef PSIM_SHORT_TAIL
#define PSIM_SHORT_TAIL 1
#endif

// The layout every kernel TU was compiled against: the shared structs' sizes
// and field offsets, the record-format and table macros a -D can change, the
// ABI.  Each TU returns its own value (layout_sig_consume/lite/strategy, and
// the engine's) and psim_create refuses a library whose TUs disagree: an A/B
// build that recompiles one TU with a layout macro (make variant / lvariant /
// evariant X=...) and links it against the other TUs' objects would otherwise
// hand the route records and keys in another format (round 5's r4lite fault
// in k_bucket_route, profiles/r05/ab_log.txt).
constexpr uint32_t layout_mix(uint32_t h, uint64_t v) {
    return ((h ^ (uint32_t)v) * 0x01000193u ^ (uint32_t)(v >> 32)) * 0x01000193u;
}
constexpr uint32_t layout_sig() {
    uint32_t h = 0x811C9DC5u;
    const uint64_t v[] = {
        PSIM_ABI_VERSION, sizeof(RoundArgs), offsetof(RoundArgs, flags), offsetof(RoundArgs, upart),
        offsetof(RoundArgs, hdr), offsetof(RoundArgs, conn), offsetof(RoundArgs, outx_rows),
        offsetof(RoundArgs, desc), offsetof(RoundArgs, desc_lite), offsetof(RoundArgs, stat_pt),
        offsetof(RoundArgs, rec_out), offsetof(RoundArgs, okey), offsetof(RoundArgs, ktime),
        offsetof(RoundArgs, ctl), offsetof(RoundArgs, fbits), offsetof(RoundArgs, omit),
        sizeof(Hdr), sizeof(Msg), sizeof(upart_t), PSIM_SHORT_TAIL, PTL_BLOCK, KEY_DST_BITS, KEY_BCAST,
        PSIM_ACTIVE_CAP, PSIM_PASSIVE_CAP, PSIM_EXCHANGE_CAP, PSIM_PT_ROOTS, PSIM_PT_OUT_CAP, PSIM_IDMAP_CAP,
        PSIM_CONN_CAP, PSIM_SVIEW_CAP, OUT_IN, IDMAP_IN, RT_SET, RT_WORDS, NST, CRASH_GRAIN_SHIFT};
    for (uint64_t x : v) h = layout_mix(h, x);
    return h;
}
uint32_t layout_sig_consume();
uint32_t layout_sig_lite();
uint32_t layout_sig_strategy();

__device__ __forceinline__ KArgs& kargs() {
    KArgs* p = (KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *p;
}

}  // namespace psim
