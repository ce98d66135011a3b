// psim_device.h -- device-side data layout and primitives of the MI355X
// overlay simulator (gfx950).  See DESIGN.md section 3 for the HBM layout.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/partisan_gpu_sim.h"

namespace psim {

// ---------------------------------------------------------------- layout --
// Per-node header: one 64-B line holding every scalar of a node.
struct __attribute__((aligned(16))) Hdr {
    uint64_t rng;          // Philox draw counter of the node's manager process
    uint32_t start_round;  // round the node (re)started
    uint32_t join_contact; // contact to JOIN at start_round, PSIM_NONE for seeds
    uint32_t epoch;
    uint32_t aux;          // HyParView: delivery mask bits 32-63; pluggable: round of the last ping
    uint32_t have;         // HyParView: delivery mask bits 0-31 (plumtree_backend ETS, bit =
                           // msg id mod PSIM_MSG_SLOTS); pluggable: hello sent
    uint32_t trk_round;    // round of first delivery of the tracked broadcast
    uint32_t trk_hop;      // plumtree Round + 1 at that delivery (0 at the root)
    uint8_t act_n, pas_n, sent_n, sent_head;
    uint8_t recv_n, recv_head, all_n, com_n;
    uint8_t conn_n, conn_dn, out_n, conn_cl; // connection table (RoundArgs::conn): entries, of
                                             // which | PSIM_CONN_DOWN (active members without one);
                                             // X-BOT: of which | PSIM_CONN_CLOSING (stopped pids)
    uint32_t pad1[4];      // pluggable: pad1[0] = leave/1 target of this round + 1, 0 = none;
                           // pad1[1] = the SCAMP v1 membership set's active slots - 16;
                           // HyParView: pad1[1] / pad1[2] = the sent / recv id map's
                           // extension row + 1 (0 = none), words HW_SENT_EXT / HW_RECV_EXT;
                           // pad1[3] = the outstanding table's, word HW_OUT_EXT
};
static_assert(sizeof(Hdr) == 64, "Hdr must be one 64-B line");

// Message record (64 B): written once by the sender, read once by the
// receiver.  tt = type | ttl << 8 | nex << 16.
struct __attribute__((aligned(16))) Msg {
    uint32_t dst, src, tt, seq;
    uint32_t a0, a1, a2, pad;
    uint32_t ex[PSIM_EXCHANGE_CAP];
};
static_assert(sizeof(Msg) == 64, "Msg must be 64 B");

// node flag byte
// F_LAZY: outstanding lazy pushes that a lazy tick may send -- clear with
// entries outstanding ("quiet") when the node's last lazy tick found none of
// their peers connected (k_node_prep then counts the next ticks without
// running the node, until a handler or a partition change can connect one);
// F_LOWACT: |active| < min_active_size (a due promotion timer can act)
// high nibble: the node's outstanding lazy pushes after its last round,
// saturating at 15 (the next round's lazy-tick bound, k_node_prep; 0 = none)
enum : uint8_t { F_UP = 1, F_CRASHED = 2, F_LAZY = 4, F_LOWACT = 8 };
constexpr uint32_t F_OUTN_SHIFT = 4;

// per-root Plumtree sets: the eager entries of all PSIM_PT_ROOTS slots pooled
// in one 64-entry row (slot 0's first, then slot 1's, ...), the lazy ones in
// another; the root row (RT_WORDS per node): root of slot k in word k
// (PSIM_NONE = free), then the eager counts and the lazy counts, one byte per
// slot (slot k's entries start at the sum of the counts below it)
constexpr uint32_t RT_SET = PSIM_PT_SET_POOL;
constexpr uint32_t RT_WORDS = 8;
constexpr uint32_t RT_EN = PSIM_PT_ROOTS, RT_LN = PSIM_PT_ROOTS + 1;
static_assert(RT_SET == 64, "the eager / lazy rows are one 64-lane register");

// Disconnect-id maps (sent_message_map / recv_message_map, PSIM_IDMAP_CAP
// entries each): the first IDMAP_IN entries in the node's own rows, the rest
// in an extension row of a shared pool, taken once per node and map the first
// time the map outgrows its own rows (few nodes ever do: at 2^23 nodes under
// config E the largest map holds ~30 entries, most hold 0-4)
constexpr uint32_t IDMAP_IN = 16;
constexpr uint32_t IDMAP_EXT = PSIM_IDMAP_CAP - IDMAP_IN;
constexpr uint32_t HW_SENT_EXT = 13, HW_RECV_EXT = 14;   // header words (Hdr pad1[1], pad1[2])
// Plumtree outstanding table (PSIM_PT_OUT_CAP entries): likewise OUT_IN in
// the node's row, the rest in an extension row of another pool.  A wave holds
// the first OUT_HEAD entries in one 64-lane register; the tail (entries
// OUT_HEAD.., a node with more than 64 lazy pushes outstanding -- rare, the
// ramp of a 2^26-node broadcast) is read and written in place in the
// extension row, from offset OUT_TAIL_AT
constexpr uint32_t OUT_IN = 16;
constexpr uint32_t OUT_EXT = PSIM_PT_OUT_CAP - OUT_IN;
constexpr uint32_t OUT_HEAD = 64;
constexpr uint32_t OUT_TAIL_AT = OUT_HEAD - OUT_IN;
static_assert(PSIM_PT_OUT_CAP <= 2 * OUT_HEAD, "the tail is one 64-lane register");
constexpr uint32_t HW_OUT_EXT = 15;
// the connection table's counts: header word 11, bytes 0 (entries), 1
// (PSIM_CONN_DOWN entries) and 3 (PSIM_CONN_CLOSING entries); byte 2 is the
// outstanding count
constexpr uint32_t HW_CONN = 11;

// route key: dst in the low 27 bits, the sender-side emission bound of the
// message type in the top 5 (used to size the receiver's next outbox).
constexpr uint32_t KEY_DST_BITS = 27;
constexpr uint32_t KEY_DST_MASK = (1u << KEY_DST_BITS) - 1;

// outbox bound: per inbox message (by type) and per node
constexpr uint32_t KEY_BCAST = 31;
__host__ __device__ constexpr uint32_t max_emit(uint32_t type) {
    // JOIN: DISCONNECT + NEIGHBOR + FORWARD_JOIN to up to ACTIVE_CAP-2 peers
    return type == PSIM_MSG_JOIN ? 2 + (PSIM_ACTIVE_CAP - 2)
         : type == PSIM_MSG_FORWARD_JOIN ? 2
         : type == PSIM_MSG_NEIGHBOR ? 1
         : type == PSIM_MSG_DISCONNECT ? 1
         : type == PSIM_MSG_NEIGHBOR_REQUEST ? 2
         : type == PSIM_MSG_NEIGHBOR_ACCEPTED ? 1
         : type == PSIM_MSG_SHUFFLE ? 1
         // a marker, not a count: the route counts a BROADCAST as 1 (the
         // PRUNE of a duplicate) and k_node_prep adds an eager push
         // and lazy adds once per distinct message slot the destination
         // receives
         : type == PSIM_MSG_PT_BROADCAST ? KEY_BCAST
         : type == PSIM_MSG_PT_IHAVE ? 1
         : type == PSIM_MSG_PT_GRAFT ? 1
         // X-BOT: a send_join and a reply at most (xbot:1171-1314)
         : type == PSIM_MSG_XBOT_OPTIMIZATION ? 2
         : type == PSIM_MSG_XBOT_OPTIMIZATION_REPLY ? 1
         : type == PSIM_MSG_XBOT_REPLACE ? 1
         : type == PSIM_MSG_XBOT_REPLACE_REPLY ? 2
         : type == PSIM_MSG_XBOT_SWITCH ? 2
         : type == PSIM_MSG_XBOT_SWITCH_REPLY ? 2
         : 0;
}
static_assert(PSIM_ACTIVE_CAP < KEY_BCAST, "max_emit must fit the 5-bit key field below the marker");
// (the per-node terms of the outbox bound -- due timers, pushes, the lazy
// tick, crash-round exits -- are k_node_prep's, psim_engine.hip)

// work descriptor (id, inbox begin, inbox count | due timers << 28, outbox
// base): the timers k_desc found due this round for the node
constexpr uint32_t DESC_CNT_MASK = (1u << 26) - 1;
enum : uint32_t { DESC_PROMO = 1, DESC_SHUFFLE = 2, DESC_LAZY = 4, DESC_ORIGIN = 8 };
// bit 26: X-BOT's xbot_execution timer is due (xbot:587-606, k_desc)
constexpr uint32_t DESC_XBOT_BIT = 1u << 26;
// bit 27 of k_consume's descriptors (k_relay): the node's HyParView phase may
// read or write its disconnect-id maps (a JOIN .. NEIGHBOR_ACCEPTED message,
// an EXIT, a promotion)
constexpr uint32_t DESC_MAPS_BIT = 1u << 27;

// stats slots in the per-block partial arrays (a wave counts slot k in lane
// k of one register, so there are at most 64): the message types with a
// slot are 0 .. PSIM_MSG_XBOT_SWITCH_REPLY (PSIM_MSG_NTYPES rounds up)
constexpr int ST_NTYPES = PSIM_MSG_XBOT_SWITCH_REPLY + 1;
enum {
    ST_EMIT = 0, ST_DELIV = ST_NTYPES, ST_DROPPED = 2 * ST_NTYPES, ST_UP, ST_PROC, ST_EXITS,
    ST_FAIL, ST_FIRST,
    ST_OVF, ST_DIGEST, ST_BYTES, ST_STOP,
    ST_BOUND,       // nodes that emitted more records than their outbox bound (an engine bug: fails the round)
    ST_OMIT,        // pluggable: strategy messages an omission fault dropped
    ST_OVF_BY, NST = ST_OVF_BY + PSIM_OVF_NKINDS
};
static_assert(NST <= 64, "a wave's stats counter holds one slot per lane");

// ------------------------------------------------------------------ RNG --
// Philox4x32-10; key = seed, counter = (draw#, node id, stream).
__device__ __forceinline__ void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                       uint32_t k0, uint32_t k1, uint32_t& o0, uint32_t& o1) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        // one 32x32->64 multiply-add per product (v_mad_u64_u32): 1.3x the
        // rate of separate low/high multiplies on gfx950 (measured)
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    o0 = c0; o1 = c1;
}

__device__ __forceinline__ uint64_t draw58_at(uint64_t ctr, uint32_t node, uint64_t seed) {
    uint32_t o0, o1;
    philox((uint32_t)ctr, (uint32_t)(ctr >> 32), node, 0u, (uint32_t)seed, (uint32_t)(seed >> 32),
           o0, o1);
    return ((((uint64_t)o1) << 32) | o0) >> 6;
}

// sets v1 slots of an element (OTP sets.erl get_slot/2: erlang:phash(E,
// MaxN), MaxN = 16, 32, ..) come from the low bits of its 32-bit hash
// erlang:phash(NodeSpec, 2^32) - 1.  The handle's table
// (psim_set_phash_table / psim_set_bucket_table: one byte per global id, the
// hash's low 8 bits, replicated on every shard) or, without one, the default
// stand-in -- murmur3's fmix32 of the id
__host__ __device__ __forceinline__ uint32_t phash_default(uint32_t id) {
    uint32_t h = id;
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
    return h;
}
__host__ __device__ __forceinline__ uint32_t bucket16_default(uint32_t id) { return phash_default(id) & 15u; }
// (the table's byte load waited for on its own branch: merged with the
// default branch, the load left its register "pending" at the join and the
// compiler's path-insensitive wait there became an s_waitcnt vmcnt(0) on the
// default branch too -- draining every load and store in flight, a node's
// prefetched rows among them, twice per k_lite_half merge.  The immediate is
// gfx9's field layout -- vmcnt in bits 3:0 and 15:14 -- so other targets take
// the plain load)
__device__ __forceinline__ uint32_t phash8(const uint8_t* tab, uint32_t id) {
    uint32_t b;
    if (tab) {
        b = tab[id];
#if defined(__gfx950__) || defined(__gfx942__) || defined(__gfx940__) || defined(__gfx90a__)
        __builtin_amdgcn_s_waitcnt(0x0F70);      // vmcnt(0), expcnt / lgkmcnt untouched
#endif
    } else {
        b = phash_default(id) & 255u;
    }
    return b;
}
// the 16-slot bucket, erlang:phash(NodeSpec, 16) - 1: every set of <= 80
// elements (every HyParView view)
__device__ __forceinline__ uint32_t bucket16(const uint8_t* tab, uint32_t id) { return phash8(tab, id) & 15u; }
// the slot of an element in a sets v1 set with ns active slots (16 <= ns <=
// 256): H = phash(E, MaxN) - 1 for MaxN the power of two >= ns; H >= ns ->
// H - MaxN / 2 (the buddy slot, sets.erl get_slot/2)
__host__ __device__ __forceinline__ uint32_t set_maxn(uint32_t ns) {
    uint32_t m = 16;
    while (m < ns) m <<= 1;
    return m;
}
__device__ __forceinline__ uint32_t set_slot(const uint8_t* tab, uint32_t id, uint32_t ns) {
    const uint32_t m = set_maxn(ns), x = phash8(tab, id) & (m - 1);
    return x < ns ? x : x - m / 2;
}

// digest multiplier of record word j (oracle msg_hash): odd, position-distinct
__device__ __forceinline__ uint64_t digest_mul(uint32_t j) {
    return (uint64_t)(uint32_t)(0x9E3779B1u + 2u * j * 0x632BE5ABu);
}

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27; z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z;
}

// X-BOT's ping time from a to b (psim_xbot_latency): nodes hash-placed on a
// 1024 x 1024 torus, toroidal L1 distance
__host__ __device__ __forceinline__ uint32_t xbot_axis(uint32_t a, uint32_t b) {
    const uint32_t d = a > b ? a - b : b - a;
    return d < 1024u - d ? d : 1024u - d;
}
__host__ __device__ __forceinline__ uint32_t xbot_latency(uint64_t seed, uint32_t a, uint32_t b) {
    if (a == b) return 0;
    const uint32_t p = (uint32_t)mix64(seed ^ ((uint64_t)a * 0x9E3779B97F4A7C15ull)) & 0xFFFFFu;
    const uint32_t q = (uint32_t)mix64(seed ^ ((uint64_t)b * 0x9E3779B97F4A7C15ull)) & 0xFFFFFu;
    return xbot_axis(p & 1023u, q & 1023u) + xbot_axis(p >> 10, q >> 10);
}

}  // namespace psim
