/*
 * partisan_gpu_sim.h -- C ABI of the MI355X overlay simulator.
 *
 * This is the drop-in boundary for the hot path named in BASELINE.json
 * `north_star`: partisan's HyParView membership manager and Plumtree
 * broadcast, simulated one BSP round at a time with all node state resident
 * in HBM.  The Erlang host keeps partisan's callback surfaces and drives this
 * library through a NIF shim (erlang/c_src/partisan_gpu_sim_nif.c); Python
 * drives it through ctypes (partisan_amd/_lib.py).
 *
 * Each entry point replaces one reference interface (cited as file:line under
 * /root/reference, read-only):
 *
 *   psim_create / psim_destroy
 *       partisan_hyparview_peer_service_manager:init/1          (:289-354)
 *       partisan_plumtree_broadcast:init/1                      (:251-264)
 *       config keys of partisan_config:init/0                   (partisan_config.erl:102-145)
 *   psim_join
 *       partisan_peer_service:join/1 -> hyparview join/1,
 *       handle_cast({join, Peer})                               (hyparview:225-226, :500-515)
 *   psim_crash
 *       connection death -> handle_info({'EXIT', ...})          (hyparview:609-654)
 *   psim_revive
 *       a restarted manager: init/1 without a join              (hyparview:289-354)
 *   psim_leave
 *       leave/0 under the pluggable manager                     (pluggable:283-284, :502-515)
 *   psim_set_partition / psim_clear_partition
 *       inject_partition/2, resolve_partition/1                 (hyparview:244-250, :1731-1797)
 *       (modelled as a network partition)
 *   psim_broadcast
 *       partisan_plumtree_broadcast:broadcast/2 with the default
 *       partisan_plumtree_backend handler, any number of roots  (plumtree:176-178, backend:179-200)
 *   psim_step
 *       one BSP round of every node's timers and inbox:
 *       hyparview handle_message/2 (:693-1166), handle_info timers (:542-607),
 *       plumtree handle_cast/2 (:282-336), lazy_tick (:341-345)
 *   psim_set_bucket_table
 *       the sets v1 order of every view: sets:to_list/1 yields bucket
 *       erlang:phash(NodeSpec, 16) 1..16, oldest first   (hyparview:1230-1231, :1346-1361)
 *   psim_get_nodes
 *       debug getters active/0, passive/0 (hyparview:261-281),
 *       plumtree debug_get_peers/2,3 (:222-231), broadcast_members/0 (:188-195)
 *
 * With cfg.manager = PSIM_MANAGER_PLUGGABLE a handle simulates
 * partisan_pluggable_peer_service_manager driving one membership strategy
 * (partisan_membership_strategy.erl:32-36) instead:
 *   psim_join    internal_join/3 + the hello/state handshake + Strategy:join/3
 *                (pluggable:1423-1458, :986-1044; server:125-148)
 *   psim_step    Strategy:handle_message/2 per inbox message (pluggable:1153-1195)
 *                and Strategy:periodic/1 (pluggable:881-903)
 *   psim_get_strategy_nodes / psim_get_member_bits
 *                get_local_state/0 (pluggable:625-626), members/0 (:618-620)
 *
 * Conventions: every function returns 0 on success or a negative PSIM_E*
 * code; psim_strerror() names it.  No exceptions or aborts cross the ABI.
 * A handle is thread-compatible (not thread-safe): the NIF shim serialises
 * calls per handle and runs psim_step on a dirty CPU scheduler.
 * The library owns all device memory; the caller owns every host buffer.
 */
#ifndef PARTISAN_GPU_SIM_H
#define PARTISAN_GPU_SIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSIM_ABI_VERSION 12

/* error codes */
#define PSIM_OK 0
#define PSIM_EINVAL -1      /* bad argument / config                 */
#define PSIM_ENOMEM -2      /* device or host allocation failed       */
#define PSIM_EDEVICE -3     /* HIP runtime error                      */
#define PSIM_ESTATE -4      /* call not valid in the current state    */
#define PSIM_ERANGE -5      /* node id out of range                   */
#define PSIM_ECOMM -6       /* RCCL / transport error                 */
#define PSIM_EUNSUPPORTED -7
#define PSIM_ECAPACITY -8   /* cfg.strict: a fixed table overflowed this round */

/* message types (the record `type` field; also stats indices) */
enum psim_msg_type {
    PSIM_MSG_JOIN = 0,              /* {join, Peer, Tag, Epoch}                  hyparview:703  */
    PSIM_MSG_FORWARD_JOIN = 1,      /* {forward_join, Peer, Tag, Epoch, TTL, S}  hyparview:808  */
    PSIM_MSG_NEIGHBOR = 2,          /* {neighbor, Peer, Tag, DisconnectId, _}    hyparview:774  */
    PSIM_MSG_DISCONNECT = 3,        /* {disconnect, Peer, DisconnectId}          hyparview:926  */
    PSIM_MSG_NEIGHBOR_REQUEST = 4,  /* {neighbor_request, Peer, high, ...}       hyparview:975  */
    PSIM_MSG_NEIGHBOR_ACCEPTED = 5, /* {neighbor_accepted, Peer, Tag, Id, Ex}    hyparview:1070 */
    PSIM_MSG_NEIGHBOR_REJECTED = 6, /* {neighbor_rejected, Peer, Ex}             hyparview:1056 */
    PSIM_MSG_SHUFFLE = 7,           /* {shuffle, Exchange, TTL, Sender}          hyparview:1095 */
    PSIM_MSG_SHUFFLE_REPLY = 8,     /* {shuffle_reply, Exchange, Sender}         hyparview:1091 */
    PSIM_MSG_PT_BROADCAST = 9,      /* {broadcast, Id, M, Mod, Round, Root, From} plumtree:288 */
    PSIM_MSG_PT_PRUNE = 10,         /* {prune, Root, From}                       plumtree:294  */
    PSIM_MSG_PT_IHAVE = 11,         /* {i_have, Id, Mod, Round, Root, From}      plumtree:299  */
    PSIM_MSG_PT_IGNORED_IHAVE = 12, /* {ignored_i_have, ...}                     plumtree:304  */
    PSIM_MSG_PT_GRAFT = 13,         /* {graft, Id, Mod, Round, Root, From}       plumtree:308  */
    /* X-BOT (cfg.manager = PSIM_MANAGER_XBOT): the record carries
     * a0 = OldNode, a1 = InitiatorNode, a2 = CandidateNode, word 7 (a3) =
     * DisconnectNode (PSIM_NONE = undefined), ttl = the reply's answer (1 true,
     * 0 false); xbot = src/partisan_hyparview_xbot_peer_service_manager.erl */
    PSIM_MSG_XBOT_OPTIMIZATION = 16,       /* {optimization, _, Old, I, C, undefined}       xbot:1205 */
    PSIM_MSG_XBOT_OPTIMIZATION_REPLY = 17, /* {optimization_reply, Ans, Old, I, C, D}       xbot:1171 */
    PSIM_MSG_XBOT_REPLACE = 18,            /* {replace, _, Old, I, C, D}                    xbot:1252 */
    PSIM_MSG_XBOT_REPLACE_REPLY = 19,      /* {replace_reply, Ans, Old, I, C, D}            xbot:1227 */
    PSIM_MSG_XBOT_SWITCH = 20,             /* {switch, _, Old, I, C, D}                     xbot:1295 */
    PSIM_MSG_XBOT_SWITCH_REPLY = 21,       /* {switch_reply, Ans, Old, I, C, D}             xbot:1270 */
    PSIM_MSG_NTYPES = 24
};

/* message types of a PLUGGABLE handle (same record and stats slots) */
enum psim_pl_msg_type {
    PSIM_PL_HELLO = 0,     /* client hello on connect             peer_service_client:246-260 */
    PSIM_PL_STATE = 1,     /* server reply {state, Tag, LocalState}  peer_service_server:125-148 */
    PSIM_PL_GOSSIP = 2,    /* full: {membership_strategy, {Myself, State}}   full:127-144 */
    PSIM_PL_FWD_SUB = 3,   /* scamp: {forward_subscription, Node}  scamp_v1:212-252, v2:284-327 */
    PSIM_PL_PING = 4,      /* scamp: {ping, SourceNode}           scamp_v1:177-188, v2:181-191 */
    PSIM_PL_KEEP_SUB = 5,  /* scamp v2: {keep_subscription, Node}  scamp_v2:328-338 */
    PSIM_PL_REMOVE_SUB = 6,  /* scamp v1: {remove_subscription, Node}  scamp_v1:102-122, :190-211 */
    PSIM_PL_BOOT_REMOVE = 7  /* scamp v2: {bootstrap_remove_subscription, Node}  scamp_v2:116-127, :192-238 */
};

/* cfg.manager */
#define PSIM_MANAGER_HYPARVIEW 0   /* partisan_hyparview_peer_service_manager (+ Plumtree) */
#define PSIM_MANAGER_PLUGGABLE 1   /* partisan_pluggable_peer_service_manager + cfg.strategy */
#define PSIM_MANAGER_XBOT 2        /* partisan_hyparview_xbot_peer_service_manager (+ Plumtree) */
/* cfg.strategy (PLUGGABLE) */
#define PSIM_STRATEGY_FULL 0       /* partisan_full_membership_strategy */
#define PSIM_STRATEGY_SCAMP_V1 1   /* partisan_scamp_v1_membership_strategy */
#define PSIM_STRATEGY_SCAMP_V2 2   /* partisan_scamp_v2_membership_strategy */
#define PSIM_SVIEW_CAP 128         /* SCAMP membership / partial_view / in_view slots */

/* Plumtree peer identities: an atom name is the bare node id; a node_spec
 * map (myself(), From, Root) has this bit set.  Erlang term order puts every
 * atom before every map, which is exactly unsigned order of the encoding.
 * See SURVEY.md App. A Q6 and plumtree:662-663. */
#define PSIM_MAP_BIT 0x80000000u
#define PSIM_NONE 0xFFFFFFFFu

/* capacities of the fixed-size per-node tables */
#define PSIM_ACTIVE_CAP 8
#define PSIM_PASSIVE_CAP 32
#define PSIM_IDMAP_CAP 64   /* sent_message_map / recv_message_map slots */
#define PSIM_PT_MEMBERS_CAP 8
/* Connections of a node's HyParView manager beyond its active view
 * (SURVEY App. A Q11): partisan_util:maybe_connect/2 opens one before every
 * send and only disconnect/2 (hyparview:1237-1258) or the peer's death
 * (EXIT, :609-654) closes it, so a shuffle terminal keeps the connection to
 * its Sender (:1127-1131), a neighbor_request receiver to a rejected
 * requester (:987), a promoting node to the passive peer it asked (:1701),
 * a joiner to its contact (:506).  The table holds those lingering peers and,
 * with PSIM_CONN_DOWN set, the rare active members whose connection a
 * neighbor_rejected closed (:1063) -- an add to a full table counts an
 * overflow (PSIM_OVF_CONN) and is dropped. */
#define PSIM_CONN_CAP 8
#define PSIM_CONN_DOWN 0x80000000u
/* X-BOT handles: an active member whose connection do_disconnect/2 stopped
 * while the state that pruned it was thrown away (xbot:1367-1379 -- every
 * optimization handler discards it), so the dead pid stays in the dict until
 * its 'EXIT' (xbot:608-653) is handled at the start of the next round; sends
 * to it draw the dispatch value and fail.  At most one per member. */
#define PSIM_CONN_CLOSING 0x40000000u
#define PSIM_PT_OUT_CAP 128
#define PSIM_EXCHANGE_CAP 8
/* Plumtree roots a node keeps per-root eager/lazy sets for at once
 * (eager_sets / lazy_sets orddicts, plumtree:76-84, :599-631): a root
 * touched with every slot taken counts an overflow and is served from the
 * common sets.  The sets of all slots share one pool of PSIM_PT_SET_POOL
 * eager and one of PSIM_PT_SET_POOL lazy entries (slot k's entries follow
 * those of slots 0..k-1); an add to a full pool counts an overflow. */
#define PSIM_PT_ROOTS 4
#define PSIM_PT_SET_POOL 64
/* Live broadcast messages: message id m owns slot m mod PSIM_MSG_SLOTS of
 * every node's delivery mask (plumtree_backend's ETS set, :140-167); a new
 * broadcast retires the previous id of its slot, and a message of a retired
 * id still in flight counts an overflow and is treated as stale. */
#define PSIM_MSG_SLOTS 64
/* psim_round_stats.overflow_by: which fixed table overflowed */
#define PSIM_OVF_IDMAP 0     /* sent / recv disconnect-id maps (oldest entry replaced) */
#define PSIM_OVF_PT_OUT 1    /* Plumtree outstanding IHAVE entries (the new entry dropped) */
#define PSIM_OVF_PT 2        /* Plumtree members, per-root sets, root slots, retired message ids */
#define PSIM_OVF_STRATEGY 3  /* pluggable: SCAMP views, full-membership snapshot payload */
#define PSIM_OVF_CONN 4      /* HyParView connections beyond the active view (the new one dropped) */
#define PSIM_OVF_NKINDS 5

typedef struct psim_config {
    uint32_t abi_version;        /* must be PSIM_ABI_VERSION */
    uint32_t n_nodes;            /* global node-id space [0, n_nodes) */
    uint64_t seed;               /* Philox key (partisan_config random_seed) */
    /* HyParView keys, partisan_config.erl:102-145 (init/0 defaults) */
    uint32_t max_active_size;    /* 6, includes self */
    uint32_t min_active_size;    /* 3 */
    uint32_t max_passive_size;   /* 30 */
    uint32_t arwl;               /* 5 */
    uint32_t prwl;               /* 30 */
    uint32_t k_active;           /* 3  (hyparview:1560) */
    uint32_t k_passive;          /* 4  (hyparview:1564) */
    uint32_t shuffle_period;     /* rounds; passive_view_shuffle_period 10000 ms */
    uint32_t promotion_period;   /* rounds; RANDOM_PROMOTION_INTERVAL 5000 ms */
    uint32_t random_promotion;   /* 1 */
    uint32_t persist_epoch;      /* 0: epoch restarts at 1 (no partisan_data_dir) */
    /* Plumtree */
    uint32_t plumtree;           /* 1: run the broadcast layer */
    uint32_t lazy_tick_period;   /* rounds; DEFAULT_LAZY_TICK_PERIOD 1000 ms */
    /* execution */
    int32_t device;              /* HIP device ordinal, -1 = current */
    uint32_t n_shards;           /* node-range shards of this process (virtual shards), 1 */
    uint32_t shard_rank;         /* RCCL rank (multi-process), 0 */
    uint32_t shard_world;        /* RCCL world size, 1 */
    const void *comm_id;         /* ncclUniqueId bytes when shard_world > 1; with shard_world = 1
                                    a non-NULL id selects the rank path on a one-rank communicator
                                    (the 1-GPU diagnostic of the RCCL path: owner partition,
                                    ncclAllToAll, self ncclSend/ncclRecv, ncclAllReduce,
                                    ncclAllGather); NULL = the in-place route */
    uint64_t max_msgs_per_round; /* 0 = auto */
    /* pluggable manager */
    uint32_t manager;            /* PSIM_MANAGER_*, 0 = HyParView */
    uint32_t strategy;           /* PSIM_STRATEGY_* when manager = PLUGGABLE */
    uint32_t periodic_interval;  /* rounds; periodic_interval 10000 ms (partisan_config.erl:130) */
    uint32_t scamp_c;            /* scamp_c, ?SCAMP_C_VALUE = 5 (partisan.hrl:31); <= 64 */
    uint32_t fanout;             /* full: 0 = gossip to every member (reference);
                                    k > 0 = k uniformly drawn members (config B extension); <= 64 */
    uint32_t strict;             /* 0: a fixed-table overflow is counted (stats.overflow_by) and the
                                    round goes on; 1: psim_step fails with PSIM_ECAPACITY after the
                                    round in which any overflow happened (e.g. a fifth live Plumtree
                                    root at a node, or a 65th live message id) */
    uint32_t xbot_period;        /* rounds; xbot_interval (partisan_config.erl:100, :145: 5000 +
                                    uniform(60000) ms, drawn per VM from an unseeded generator --
                                    a fixed period here, default 35); X-BOT handles */
    uint32_t reserved1;
} psim_config;

typedef struct psim_round_stats {
    uint64_t round;                          /* round number just executed */
    uint64_t emitted[PSIM_MSG_NTYPES];       /* messages sent (successful sends) by type */
    uint64_t delivered[PSIM_MSG_NTYPES];     /* messages processed by a live recipient */
    uint64_t dropped;                        /* messages whose recipient was down */
    uint64_t nodes_up;
    uint64_t nodes_processed;                /* nodes with inbox, timer or event work */
    uint64_t exits;                          /* EXIT events handled */
    uint64_t send_fail;                      /* sends refused: no connection */
    uint64_t first_deliveries;               /* plumtree merge() == true this round */
    uint64_t overflow;                       /* fixed-table overflows (must be 0 in parity runs) */
    uint64_t digest;                         /* sum of per-message hashes of emitted messages */
    uint64_t state_bytes;                    /* algorithmic state bytes read+written */
    uint64_t overflow_by[PSIM_OVF_NKINDS];   /* overflow by table (PSIM_OVF_*), summing to overflow */
    uint64_t omitted;                        /* pluggable: strategy messages an omission fault dropped
                                                (at the sender: never sent, no draw; at the
                                                receiver: never handled) -- psim_set_omission */
} psim_round_stats;

/* Canonical per-node view (inspection; unused slots zero). */
typedef struct psim_node_view {
    uint32_t up, epoch, start_round;
    uint32_t conn_n;                         /* entries of conn[] */
    uint64_t rng_ctr;
    uint32_t act_n, pas_n;
    uint32_t act[PSIM_ACTIVE_CAP];           /* sets:to_list order, self included */
    uint32_t pas[PSIM_PASSIVE_CAP];          /* sets:to_list order */
    uint32_t sent_n, sent_head, recv_n, recv_head;
    uint32_t sent_peer[PSIM_IDMAP_CAP], sent_id[PSIM_IDMAP_CAP];
    uint32_t recv_peer[PSIM_IDMAP_CAP], recv_id[PSIM_IDMAP_CAP];
    uint32_t pt_all_n, pt_common_n, pt_out_n, pt_pad;
    uint32_t pt_all[PSIM_PT_MEMBERS_CAP], pt_common[PSIM_PT_MEMBERS_CAP];
    /* per-root sets, slot k: root pt_root[k] (PSIM_NONE = free); its eager
     * entries are pt_eager[o .. o + pt_eager_n[k]) with o the sum of
     * pt_eager_n[0..k) (ordsets order), the lazy ones likewise */
    uint32_t pt_root[PSIM_PT_ROOTS], pt_eager_n[PSIM_PT_ROOTS], pt_lazy_n[PSIM_PT_ROOTS];
    uint32_t pt_eager[PSIM_PT_SET_POOL], pt_lazy[PSIM_PT_SET_POOL];
    uint32_t pt_out_peer[PSIM_PT_OUT_CAP], pt_out_msg[PSIM_PT_OUT_CAP], pt_out_round[PSIM_PT_OUT_CAP];
    uint64_t have;                           /* delivered: bit (msg id mod PSIM_MSG_SLOTS) */
    uint32_t trk_round, trk_hop;
    /* connections beyond the active view (lingering peers), and active
     * members without one (| PSIM_CONN_DOWN), in insertion order */
    uint32_t conn[PSIM_CONN_CAP];
} psim_node_view;

/* Per-node state of a PLUGGABLE handle (inspection; unused slots zero). */
typedef struct psim_strategy_view {
    uint32_t up, start_round;
    uint32_t pending;                        /* contact of an unfinished join, PSIM_NONE */
    uint32_t last_ping;                      /* scamp: round of the last ping, PSIM_NONE = undefined */
    uint64_t rng_ctr;
    uint32_t view_n, in_n;
    uint32_t view[PSIM_SVIEW_CAP];           /* scamp v1 membership (sets:to_list order) /
                                                scamp v2 partial_view (list order) */
    uint32_t in_view[PSIM_SVIEW_CAP];        /* scamp v2 in_view (list order) */
    uint32_t members;                        /* full: size of query(ORSet) */
    uint32_t view_slots;                     /* scamp v1: active slots of the membership set
                                                (OTP sets v1: 16, one more past each 5 per slot;
                                                0 for an empty view and other strategies) */
    uint64_t members_hash;                   /* full: sum of mix64(id + 1) over members */
} psim_strategy_view;

/* Overlay statistics of a HyParView handle (SURVEY 8(b) psim_get_histograms,
 * 8(d) configs C/D): histograms over live nodes, bin k = value k, the last
 * bin = PSIM_HIST_BINS - 1 or more.  Links count live -> live only.
 * Replaces the reference's overlay checks: orchestration graph BFS
 * (partisan_orchestration_backend.erl:333-413, 467-489) and the SUITE's
 * connected + symmetric active views (test/partisan_SUITE.erl:2044-2108). */
#define PSIM_HIST_BINS 64
typedef struct psim_histograms {
    uint64_t n_up;                           /* live nodes */
    uint64_t active_in[PSIM_HIST_BINS];      /* by active in-degree */
    uint64_t passive_in[PSIM_HIST_BINS];     /* by passive in-degree */
    uint64_t active_out[PSIM_HIST_BINS];     /* by active view size (self excluded) */
    uint64_t passive_fill[PSIM_HIST_BINS];   /* by passive view size */
    uint64_t hop[PSIM_HIST_BINS];            /* tracked broadcast: delivered nodes by hop count */
    uint64_t delivered;                      /* live nodes holding the tracked broadcast */
    uint64_t last_round;                     /* latest first-delivery round of it (0: none) */
    uint64_t active_links;                   /* directed active links between live nodes */
    uint64_t symmetric_links;                /* ... whose reverse link exists */
    uint64_t components;                     /* weakly connected components of live nodes over
                                                active links */
    uint64_t largest_component;
    uint64_t reserved[6];
} psim_histograms;

typedef struct psim_handle psim_handle;

void psim_default_config(psim_config *cfg);
int psim_create(const psim_config *cfg, psim_handle **out);
void psim_destroy(psim_handle *h);
const char *psim_strerror(int code);
int psim_abi_version(void);

/* Events take effect at the start of the next round. */
int psim_join(psim_handle *h, const uint32_t *nodes, const uint32_t *contacts, size_t n);
int psim_crash(psim_handle *h, const uint32_t *nodes, size_t n);
/* Restart nodes (crashed, or never started) without a join: each comes back
 * with init/1 state -- empty views, a fresh incarnation (epoch + 1 when
 * persist_epoch), its draw counter back at 0 -- and waits to be reached
 * (hyparview:289-354; a node restarted by its supervisor, not told to
 * join).  Same as psim_join with every contact PSIM_NONE. */
int psim_revive(psim_handle *h, const uint32_t *nodes, size_t n);
/* leave/0 at each node (pluggable manager only; the HyParView manager's
 * leave answers `error`, hv:363-364, so PSIM_EUNSUPPORTED there).  The
 * manager stops inside handle_call({leave, Myself}) (pluggable:502-515)
 * before the Strategy:leave/2 messages it cast to itself are sent
 * (pluggable:1390-1420, :1585-1609), so the node goes down without a word,
 * exactly as psim_crash.  Revive with psim_revive. */
int psim_leave(psim_handle *h, const uint32_t *nodes, size_t n);
/* leave/1: actors[i] removes targets[i] from the cluster
 * (handle_call({leave, Node}) pluggable:502-515 -> internal_leave/2
 * :1390-1420); actor == target is leave/0 above.  SCAMP v1 / v2 handles:
 *   v1: the actor drops the target and sends {remove_subscription, T} to its
 *       old membership (scamp_v1:102-122); a receiver holding T crashes on
 *       the swapped sets:del_element/2 arguments (scamp_v1:197, SURVEY App. A
 *       Q12) -- T itself included;
 *   v2: the actor sends {bootstrap_remove_subscription, T} to its partial
 *       view (scamp_v2:116-127); T, on receipt, stops before its replacement
 *       casts go out (lists:nth(0, ..) or the self-less reset, :192-238);
 *   full: the actor tombstones T's add in its ORSet and gossips the new state
 *       to its old members (full:58-89); merges carry the removal on, and a
 *       node that merges a removal of itself stops (pluggable:1182-1188).
 * A stopping manager sends nothing in that round (its sends are casts to
 * itself) and is down from the next round on.  One call per actor per
 * round.  Multi-rank handles: every rank makes the same calls; a stop
 * reported by the target's rank is all-gathered after the round.
 * PSIM_EUNSUPPORTED for HyParView handles. */
int psim_leave_node(psim_handle *h, const uint32_t *actors, const uint32_t *targets, size_t n);
/* group[i]: node i's partition group, 0..PSIM_PARTITION_MAX (PSIM_EINVAL for
 * any other value); nodes in different groups cannot exchange messages from
 * the next round on (partisan_SUITE's partition injection). */
#define PSIM_PARTITION_MAX 254
int psim_set_partition(psim_handle *h, const uint8_t *group, size_t n);
/* View order.  Views are kept in sets:to_list/1 order of
 * OTP's sets v1, a linear hash table (stdlib sets.erl: 16 slots up to 80
 * elements, yielded slot 1..n, oldest first within a slot; one more slot
 * each time the size passes 5 n, one fewer when it drops below 3 n), so every
 * select_random index and every shuffle key pairing (hyparview:1230-1231,
 * :1346-1361; scamp_v1's membership, scamp_v1:45-279) depends on the slot of
 * each element, erlang:phash(NodeSpec, MaxN) with MaxN = 16, 32, ...
 * psim_set_phash_table takes the whole hash: phash[i] =
 * erlang:phash(NodeSpec_i, 4294967296) - 1 for node i (phash(T, R) - 1 is
 * that value mod R for every power of two R), n = n_nodes -- e.g. the table
 * the in-BEAM harness exports (erlang/harness, `B id hash` lines).  The
 * engine keeps its low 8 bits: every set it holds (views of <= 128 ids) has
 * MaxN <= 32.  psim_set_bucket_table takes the 16-slot bucket alone
 * (phash(NodeSpec, 16) - 1, 0..15): enough for every HyParView view; a SCAMP
 * v1 view past 80 ids then reads the missing bits as 0.  Without a table the
 * handle uses a stand-in hash (murmur3 fmix32(id)).  Valid only before the
 * first round (PSIM_ESTATE after); NULL restores the stand-in.  Multi-rank
 * handles: every rank passes the same table.  The table is not part of
 * psim_snapshot, but a snapshot records its hash: set the same table on the
 * new handle before psim_restore (PSIM_EINVAL otherwise). */
int psim_set_bucket_table(psim_handle *h, const uint8_t *buckets, size_t n);
int psim_set_phash_table(psim_handle *h, const uint32_t *phash, size_t n);
int psim_clear_partition(psim_handle *h);
/* Omission faults of the pluggable manager's interposition layer
 * (add_interposition_fun/2, remove_interposition_fun/1 pluggable:297-326;
 * the folds in handle_cast({forward_message, ..}) :669-836 and
 * handle_cast({receive_message, ..}) :634-667), as the crash-fault model
 * installs them (test/prop_partisan_crash_fault_model.erl:93-196):
 *   PSIM_OMIT_SEND     {send_omission, Dst} at Src (:158-196): a strategy
 *                      message Src forwards to Dst becomes `undefined` -- not
 *                      sent, no connection lookup, no dispatch draw;
 *   PSIM_OMIT_RECEIVE  {receive_omission, Src} at Dst (:117-155): a strategy
 *                      message Dst receives from Src is dropped unhandled.
 * on = 1 installs (src[i], dst[i]) pairs, on = 0 removes them (installing a
 * pair twice keeps one: the funs are a dict keyed by name).
 * psim_set_faulted is the general omission begin_omission/end_omission
 * (:93-114, `faulted` read by the interposition funs of
 * partisan_trace_orchestrator:621-656): every strategy message the node
 * sends or receives is dropped.  The hello/state handshake is the
 * client/server processes' and passes.  psim_clear_faults removes all
 * (resolve_all_faults_with_heal :198-229 removes every interposition fun,
 * the `faulted` reader included).  Changes take effect at the start of
 * the next round; dropped messages count in psim_round_stats.omitted.
 * PSIM_EUNSUPPORTED for HyParView handles (that manager has no interposition
 * layer). */
#define PSIM_OMIT_SEND 0
#define PSIM_OMIT_RECEIVE 1
int psim_set_omission(psim_handle *h, int kind, const uint32_t *src, const uint32_t *dst, size_t n, int on);
int psim_set_faulted(psim_handle *h, const uint32_t *nodes, size_t n, int on);
int psim_clear_faults(psim_handle *h);
/* broadcast/2 at `root` (plumtree:176-178) with the partisan_plumtree_backend
 * heartbeat semantics (backend:179-200), originated in the next round.  Any
 * node can be a root; per round at most one broadcast per root and per
 * message slot (msg_id mod PSIM_MSG_SLOTS), else PSIM_EINVAL.  The last call
 * names the tracked broadcast of psim_get_delivery / psim_get_histograms. */
int psim_broadcast(psim_handle *h, uint32_t root, uint32_t msg_id);

/* Run n_rounds BSP rounds; stats (may be NULL) receives one entry per round.
 * An error from inside a round (PSIM_ENOMEM, PSIM_EDEVICE, PSIM_ECOMM) leaves
 * the state off a round boundary: the handle is unusable -- every later
 * psim_step answers PSIM_ESTATE -- until psim_restore loads a snapshot into
 * it.  PSIM_ECAPACITY (cfg.strict) is returned after a whole round and does
 * not poison the handle. */
int psim_step(psim_handle *h, uint32_t n_rounds, psim_round_stats *stats);

/* Inspection: views of nodes [first, first+count) into caller buffers. */
int psim_get_nodes(psim_handle *h, uint32_t first, uint32_t count, psim_node_view *out);
int psim_get_round(psim_handle *h, uint64_t *round);
/* PLUGGABLE handles: strategy state of nodes [first, first+count) */
int psim_get_strategy_nodes(psim_handle *h, uint32_t first, uint32_t count, psim_strategy_view *out);
/* full strategy: the member bitset of one node (bit j of word j/32 = node j) */
int psim_get_member_bits(psim_handle *h, uint32_t node, uint32_t *words, size_t n_words);
/* Delivery state of the tracked broadcast (the last psim_broadcast) at nodes
 * [first, first+count): have (0/1), first-delivery round and hop count
 * (plumtree_backend merge/2 + the broadcast's Round field, pt:288-293). */
int psim_get_delivery(psim_handle *h, uint32_t first, uint32_t count, uint8_t *have, uint32_t *round,
                      uint32_t *hop);
/* Overlay statistics (psim_histograms above); HyParView handles only.
 * Symmetry and connectivity cover the whole overlay for any shard count:
 * sharded handles gather every node's active row first (device copies, or an
 * ncclAllGather across RCCL ranks -- a collective: every rank must call). */
int psim_get_histograms(psim_handle *h, psim_histograms *out);
/* Snapshot of the whole simulation state of this process (node rows,
 * in-flight messages, round, events not yet applied are not included):
 * with buf == NULL (or cap too small) only *need is set.  psim_restore
 * loads it into a handle created with the same config (and the same
 * view-order table, whose hash the snapshot records: PSIM_EINVAL otherwise);
 * the rounds that follow are identical to the original's (HyParView
 * handles).  A restore replaces the whole state -- events queued and not yet
 * applied are dropped -- and puts a handle a failed psim_step left unusable
 * back into service. */
int psim_snapshot(psim_handle *h, void *buf, size_t cap, size_t *need);
int psim_restore(psim_handle *h, const void *buf, size_t size);

/* The live Plumtree message slots (plumtree_backend's ETS set keyed by
 * message id, :140-167): ids[k] = the message id owning slot k (PSIM_NONE =
 * free) and roots[k] its root (node_spec identity, | PSIM_MAP_BIT), for
 * k < PSIM_MSG_SLOTS; cap must be >= PSIM_MSG_SLOTS.  A node's delivery bit
 * k (psim_node_view.have) answers is_stale/1 for ids[k] only. */
int psim_get_msg_slots(psim_handle *h, uint32_t *ids, uint32_t *roots, size_t cap);

/* X-BOT's latency oracle (is_better/3 + is_better_node_by_latency/2,
 * xbot:1318-1333: timer:tc of net_adm:ping from the deciding node).  The
 * simulator places every node on a 1024 x 1024 torus from a hash of (seed,
 * id) and takes the ping time from a to b as their toroidal L1 distance
 * (0 for a == b); a crashed or never-started node answers pang.  Exported so
 * hosts and tests can read the same metric. */
uint32_t psim_xbot_latency(uint64_t seed, uint32_t a, uint32_t b);

/* Wire format of a partisan peer connection, for mixed
 * clusters of real and simulated nodes: a frame is {packet, 4} -- a 4-byte
 * big-endian length (peer_service_client.erl:214) -- around
 * partisan_util:term_to_iolist/1 of the message -- what the connection's
 * send path writes (client:95, :130, :275; util:235-297; the receiver,
 * peer_service_server.erl:172-182, takes any term encoding).  A
 * record is the engine's 64-B message record (words: dst, src,
 * type | ttl << 8 | nex << 16, seq, a0, a1, a2, a3, ex[0..8)); its term is
 * the one the reference's handler sends (HyParView hv:506-1131, Plumtree as
 * {forward_message, partisan_plumtree_broadcast, {'$gen_cast', Msg}}
 * (cast_message/3 hv:147-154, forward_message hv:441-460) with the
 * backend's heartbeat ids {RootName, Counter}, X-BOT xbot:1171-1314; the
 * table is in partisan_amd/csrc/psim_wire.cpp).  Node id i is the node_spec
 * #{name => '<prefix><i>@<host>', listen_addrs => [#{ip => ip_base + i,
 * port => port}], channels => [undefined], parallelism => 1}
 * (partisan_peer_service_manager.erl:71-76). */
typedef struct psim_wire_names {
    const char *prefix;          /* node name prefix, e.g. "n" */
    const char *host;            /* node name host part, e.g. "127.0.0.1" */
    uint32_t ip_base;            /* IPv4 of node 0 (host order); node i has ip_base + i */
    uint32_t port;               /* listen port (PEER_PORT 9090, partisan.hrl:3) */
} psim_wire_names;
/* One record to one frame (*len bytes).  With buf == NULL or cap < *len only
 * *len is set.  PSIM_EINVAL for a record no handler sends (an IHAVE of a
 * retired id: no root). */
int psim_wire_encode(const uint32_t rec[16], const psim_wire_names *names, uint8_t *buf, size_t cap, size_t *len);
/* The first frame of buf back to a record (dst = the connection's peer,
 * passed in; seq = 0: the order of a connection is its sequence); *used =
 * the frame's bytes.  PSIM_ERANGE: buf holds no complete frame yet;
 * PSIM_EINVAL: not one of the messages above. */
int psim_wire_decode(const uint8_t *buf, size_t len, const psim_wire_names *names, uint32_t dst, uint32_t rec[16],
                     size_t *used);

/* Diagnostic: per node-round kernel of the last round (k_relay, k_shuf,
 * k_lite_half, k_consume, k_ptl, k_pt; this process's first shard), 4 words
 * each: nodes processed, records delivered, records emitted, 0 -- the
 * kernel's share of the algorithmic bytes (bench.py --kernel-counts,
 * profiles/pmc_record.py).  With cap >= 28 a seventh entry, k_node_prep:
 * the quiet lazy ticks it counted without running their nodes (processed,
 * 0, 0, 0).  Returns 6 or 7 (0 under the pluggable
 * manager). */
int psim_debug_kernel_counts(psim_handle *h, uint64_t *out, int cap);

/* Per-kernel device time (ms) accumulated over the last psim_step call:
 * names[i] is a static string; returns the number of entries. */
int psim_kernel_times(psim_handle *h, const char **names, double *ms, uint64_t *launches, int cap);

/* The cross-shard exchange since psim_create (G > 1: virtual shards or RCCL
 * ranks; this process's shards): *records = records sent to another shard,
 * *bytes = their bytes on the wire -- 32 B a record (dst, src, type word, seq,
 * a0-a2, word 7) plus 32 B for one with exchange ids (nex > 0), against 64 B
 * a record in memory.  Both 0 on one shard. */
int psim_get_exchange_stats(psim_handle *h, uint64_t *records, uint64_t *bytes);

/* RCCL bootstrap for multi-process sharding (rank 0 creates, all pass it in cfg). */
int psim_comm_id_size(void);
int psim_get_comm_id(void *buf, size_t cap);
/* TEST VEHICLE, not a product backend: the id of a new loopback world
 * (psim_comm_id_size() bytes).  Handles created with it as cfg.comm_id
 * (shard_world = W, shard_rank = r, all on one device, in this process) run
 * the multi-rank code path -- owner partition, count all-to-all, record
 * exchange, stats reduce, leave/1 stop-list gather, overlay gathers -- with
 * device copies and a host barrier in place of RCCL, so it can run where
 * RCCL cannot (one GPU).  The W ranks are W host threads, each making the
 * same calls as RCCL ranks would (collective calls must be concurrent). */
int psim_loopback_comm_id(void *buf, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* PARTISAN_GPU_SIM_H */
