/*
 * partisan_gpu_sim_nif.c -- Erlang NIF shim over include/partisan_gpu_sim.h.
 *
 * Built only where erl_nif.h exists (not in this image):
 *   cc -O2 -fPIC -shared -I$(ERTS_INCLUDE_DIR) -I../../include \
 *      -o ../priv/partisan_gpu_sim_nif.so partisan_gpu_sim_nif.c \
 *      -L../../partisan_amd/csrc -lpartisan_gpu_sim
 *
 * One resource per simulator handle; calls on a handle are serialised by a
 * mutex (the ABI is thread-compatible, not thread-safe).  psim_step and the
 * other long calls run on dirty schedulers and wait for the mutex; the short
 * NIFs run on normal schedulers and never block one: when the handle is busy
 * (a step in progress) they return {error, busy}; the wrappers in
 * partisan_gpu_sim.erl retry those with a bounded back-off (call/1 there),
 * so a caller sees {error, busy} only after ~10 s of steps.
 */
#include <erl_nif.h>
#include <string.h>

#include "partisan_gpu_sim.h"

typedef struct { psim_handle *h; ErlNifMutex *mu; uint32_t n_nodes; } sim_res;
static ErlNifResourceType *SIM_RT;

static void sim_dtor(ErlNifEnv *env, void *obj) {
    sim_res *r = (sim_res *)obj;
    if (r->h) psim_destroy(r->h);
    if (r->mu) enif_mutex_destroy(r->mu);
}

static int load(ErlNifEnv *env, void **priv, ERL_NIF_TERM info) {
    SIM_RT = enif_open_resource_type(env, NULL, "psim", sim_dtor, ERL_NIF_RT_CREATE, NULL);
    return SIM_RT ? 0 : -1;
}

static ERL_NIF_TERM err(ErlNifEnv *env, int rc) {
    return enif_make_tuple2(env, enif_make_atom(env, "error"),
                            enif_make_atom(env, psim_strerror(rc)));
}

static ERL_NIF_TERM busy(ErlNifEnv *env) {
    return enif_make_tuple2(env, enif_make_atom(env, "error"), enif_make_atom(env, "busy"));
}

/* normal-scheduler NIFs: take the handle's mutex only if it is free */
#define LOCK_OR_BUSY(r) do { if (enif_mutex_trylock((r)->mu) != 0) return busy(env); } while (0)
/* the same, releasing an enif_alloc'ed buffer on the busy path */
#define LOCK_OR_BUSY_FREE(r, p) do { if (enif_mutex_trylock((r)->mu) != 0) { enif_free(p); return busy(env); } } while (0)

static int get_u32(ErlNifEnv *env, ERL_NIF_TERM map, const char *k, uint32_t *out) {
    ERL_NIF_TERM v;
    unsigned int x;
    if (!enif_get_map_value(env, map, enif_make_atom(env, k), &v)) return 1; /* keep default */
    if (!enif_get_uint(env, v, &x)) return 0;
    *out = x;
    return 1;
}

/* create(#{n_nodes => N, seed => S, max_active_size => .., ...,
 *         manager => 0 | 1 | 2, strategy => 0 | 1 | 2, fanout => K, scamp_c => C,
 *         periodic_interval => Rounds, xbot_period => Rounds}) -> {ok, Ref}
 * manager 1 = the pluggable manager with strategy 0 full, 1 scamp v1, 2 scamp v2;
 * manager 2 = partisan_hyparview_xbot_peer_service_manager (X-BOT) */
static ERL_NIF_TERM nif_create(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    psim_config c;
    ErlNifUInt64 seed;
    ERL_NIF_TERM v;
    psim_default_config(&c);
    if (!get_u32(env, argv[0], "n_nodes", &c.n_nodes) ||
        !get_u32(env, argv[0], "max_active_size", &c.max_active_size) ||
        !get_u32(env, argv[0], "min_active_size", &c.min_active_size) ||
        !get_u32(env, argv[0], "max_passive_size", &c.max_passive_size) ||
        !get_u32(env, argv[0], "arwl", &c.arwl) || !get_u32(env, argv[0], "prwl", &c.prwl) ||
        !get_u32(env, argv[0], "shuffle_period", &c.shuffle_period) ||
        !get_u32(env, argv[0], "plumtree", &c.plumtree) ||
        !get_u32(env, argv[0], "manager", &c.manager) ||
        !get_u32(env, argv[0], "strategy", &c.strategy) ||
        !get_u32(env, argv[0], "fanout", &c.fanout) || !get_u32(env, argv[0], "strict", &c.strict) ||
        !get_u32(env, argv[0], "scamp_c", &c.scamp_c) ||
        !get_u32(env, argv[0], "periodic_interval", &c.periodic_interval) ||
        !get_u32(env, argv[0], "xbot_period", &c.xbot_period))
        return enif_make_badarg(env);
    if (enif_get_map_value(env, argv[0], enif_make_atom(env, "seed"), &v) &&
        enif_get_uint64(env, v, &seed))
        c.seed = seed;
    sim_res *r = enif_alloc_resource(SIM_RT, sizeof *r);
    r->mu = enif_mutex_create("psim");
    r->n_nodes = c.n_nodes;
    int rc = psim_create(&c, &r->h);
    if (rc) { r->h = NULL; enif_release_resource(r); return err(env, rc); }
    ERL_NIF_TERM t = enif_make_resource(env, r);
    enif_release_resource(r);
    return enif_make_tuple2(env, enif_make_atom(env, "ok"), t);
}

/* join(Ref, NodesBin, ContactsBin): little-endian u32 arrays */
static ERL_NIF_TERM nif_join(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r; ErlNifBinary a, b;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r) ||
        !enif_inspect_binary(env, argv[1], &a) || !enif_inspect_binary(env, argv[2], &b) ||
        a.size != b.size || a.size % 4)
        return enif_make_badarg(env);
    LOCK_OR_BUSY(r);
    int rc = psim_join(r->h, (const uint32_t *)a.data, (const uint32_t *)b.data, a.size / 4);
    enif_mutex_unlock(r->mu);
    return rc ? err(env, rc) : enif_make_atom(env, "ok");
}

static ERL_NIF_TERM nif_crash(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r; ErlNifBinary a;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r) ||
        !enif_inspect_binary(env, argv[1], &a) || a.size % 4)
        return enif_make_badarg(env);
    LOCK_OR_BUSY(r);
    int rc = psim_crash(r->h, (const uint32_t *)a.data, a.size / 4);
    enif_mutex_unlock(r->mu);
    return rc ? err(env, rc) : enif_make_atom(env, "ok");
}

/* psim_revive: restart without a join (hyparview init/1 again) */
static ERL_NIF_TERM nif_revive(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r; ErlNifBinary a;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r) ||
        !enif_inspect_binary(env, argv[1], &a) || a.size % 4)
        return enif_make_badarg(env);
    LOCK_OR_BUSY(r);
    int rc = psim_revive(r->h, (const uint32_t *)a.data, a.size / 4);
    enif_mutex_unlock(r->mu);
    return rc ? err(env, rc) : enif_make_atom(env, "ok");
}

/* psim_leave: leave/0 at each node under the pluggable manager */
static ERL_NIF_TERM nif_leave(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r; ErlNifBinary a;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r) ||
        !enif_inspect_binary(env, argv[1], &a) || a.size % 4)
        return enif_make_badarg(env);
    LOCK_OR_BUSY(r);
    int rc = psim_leave(r->h, (const uint32_t *)a.data, a.size / 4);
    enif_mutex_unlock(r->mu);
    return rc ? err(env, rc) : enif_make_atom(env, "ok");
}

/* psim_leave_node: leave/1, Actors[i] removes Targets[i] */
static ERL_NIF_TERM nif_leave_node(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r; ErlNifBinary a, t;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r) ||
        !enif_inspect_binary(env, argv[1], &a) || !enif_inspect_binary(env, argv[2], &t) ||
        a.size % 4 || a.size != t.size)
        return enif_make_badarg(env);
    LOCK_OR_BUSY(r);
    int rc = psim_leave_node(r->h, (const uint32_t *)a.data, (const uint32_t *)t.data, a.size / 4);
    enif_mutex_unlock(r->mu);
    return rc ? err(env, rc) : enif_make_atom(env, "ok");
}

static ERL_NIF_TERM nif_broadcast(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r; unsigned root, id;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r) ||
        !enif_get_uint(env, argv[1], &root) || !enif_get_uint(env, argv[2], &id))
        return enif_make_badarg(env);
    LOCK_OR_BUSY(r);
    int rc = psim_broadcast(r->h, root, id);
    enif_mutex_unlock(r->mu);
    return rc ? err(env, rc) : enif_make_atom(env, "ok");
}

/* msg_slots_nif(Ref) -> {ok, [{Slot, Id, Root}]}: the live message slots
 * (psim_get_msg_slots; plumtree_backend's ETS set, :140-167) */
static ERL_NIF_TERM nif_msg_slots(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r;
    uint32_t ids[PSIM_MSG_SLOTS], roots[PSIM_MSG_SLOTS];
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r)) return enif_make_badarg(env);
    LOCK_OR_BUSY(r);
    int rc = psim_get_msg_slots(r->h, ids, roots, PSIM_MSG_SLOTS);
    enif_mutex_unlock(r->mu);
    if (rc) return err(env, rc);
    ERL_NIF_TERM l = enif_make_list(env, 0);
    for (int k = PSIM_MSG_SLOTS - 1; k >= 0; k--)
        if (ids[k] != PSIM_NONE)
            l = enif_make_list_cell(env, enif_make_tuple3(env, enif_make_uint(env, (unsigned)k),
                                                          enif_make_uint(env, ids[k]),
                                                          enif_make_uint(env, roots[k] & ~PSIM_MAP_BIT)), l);
    return enif_make_tuple2(env, enif_make_atom(env, "ok"), l);
}

/* omission_nif(Ref, Kind, SrcBin, DstBin, On): install / remove
 * {send_omission, Dst} funs at Src (Kind 0) or {receive_omission, Src} funs
 * at Dst (Kind 1) -- add/remove_interposition_fun (pluggable:297-326) */
static ERL_NIF_TERM nif_omission(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r; ErlNifBinary a, b; int kind, on;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r) || !enif_get_int(env, argv[1], &kind) ||
        !enif_inspect_binary(env, argv[2], &a) || !enif_inspect_binary(env, argv[3], &b) ||
        !enif_get_int(env, argv[4], &on) || a.size % 4 || a.size != b.size)
        return enif_make_badarg(env);
    LOCK_OR_BUSY(r);
    int rc = psim_set_omission(r->h, kind, (const uint32_t *)a.data, (const uint32_t *)b.data, a.size / 4, on);
    enif_mutex_unlock(r->mu);
    return rc ? err(env, rc) : enif_make_atom(env, "ok");
}

/* faulted_nif(Ref, NodesBin, On): begin_omission / end_omission */
static ERL_NIF_TERM nif_faulted(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r; ErlNifBinary a; int on;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r) || !enif_inspect_binary(env, argv[1], &a) ||
        !enif_get_int(env, argv[2], &on) || a.size % 4)
        return enif_make_badarg(env);
    LOCK_OR_BUSY(r);
    int rc = psim_set_faulted(r->h, (const uint32_t *)a.data, a.size / 4, on);
    enif_mutex_unlock(r->mu);
    return rc ? err(env, rc) : enif_make_atom(env, "ok");
}

/* clear_faults(Ref): resolve_all_faults_with_heal */
static ERL_NIF_TERM nif_clear_faults(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r)) return enif_make_badarg(env);
    LOCK_OR_BUSY(r);
    int rc = psim_clear_faults(r->h);
    enif_mutex_unlock(r->mu);
    return rc ? err(env, rc) : enif_make_atom(env, "ok");
}

/* step(Ref, Rounds) -> {ok, [{Round, Emitted, Delivered, FirstDeliveries}]} (dirty CPU) */
static ERL_NIF_TERM nif_step(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r; unsigned n;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r) || !enif_get_uint(env, argv[1], &n) ||
        n == 0 || n > 100000)
        return enif_make_badarg(env);
    psim_round_stats *st = enif_alloc(n * sizeof *st);
    enif_mutex_lock(r->mu);
    int rc = psim_step(r->h, n, st);
    enif_mutex_unlock(r->mu);
    if (rc) { enif_free(st); return err(env, rc); }
    ERL_NIF_TERM list = enif_make_list(env, 0);
    for (unsigned i = n; i-- > 0;) {
        uint64_t em = 0, de = 0;
        for (int t = 0; t < PSIM_MSG_NTYPES; t++) { em += st[i].emitted[t]; de += st[i].delivered[t]; }
        ERL_NIF_TERM e = enif_make_tuple4(env, enif_make_uint64(env, st[i].round),
                                          enif_make_uint64(env, em), enif_make_uint64(env, de),
                                          enif_make_uint64(env, st[i].first_deliveries));
        list = enif_make_list_cell(env, e, list);
    }
    enif_free(st);
    return enif_make_tuple2(env, enif_make_atom(env, "ok"), list);
}

/* active(Ref, Node) -> {ok, [Id]} : sets:to_list(Active) of one node */
static ERL_NIF_TERM nif_active(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r; unsigned node;
    psim_node_view v;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r) || !enif_get_uint(env, argv[1], &node))
        return enif_make_badarg(env);
    LOCK_OR_BUSY(r);
    int rc = psim_get_nodes(r->h, node, 1, &v);
    enif_mutex_unlock(r->mu);
    if (rc) return err(env, rc);
    ERL_NIF_TERM ids[PSIM_ACTIVE_CAP];
    for (uint32_t i = 0; i < v.act_n; i++) ids[i] = enif_make_uint(env, v.act[i]);
    return enif_make_tuple2(env, enif_make_atom(env, "ok"), enif_make_list_from_array(env, ids, v.act_n));
}

/* members(Ref, Node) -> {ok, [Id]} : the pluggable manager's membership of one
 * node -- full: query(ORSet) in id order; scamp: the view in list order */
static ERL_NIF_TERM nif_members(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r; unsigned node, n_nodes;
    psim_strategy_view v;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r) || !enif_get_uint(env, argv[1], &node) ||
        !enif_get_uint(env, argv[2], &n_nodes))
        return enif_make_badarg(env);
    if (n_nodes != r->n_nodes) return enif_make_badarg(env);
    LOCK_OR_BUSY(r);
    int rc = psim_get_strategy_nodes(r->h, node, 1, &v);
    uint32_t *bits = NULL;
    size_t words = (r->n_nodes + 31) / 32;     /* psim_get_member_bits fills exactly these */
    if (!rc && v.members) {           /* full strategy */
        bits = enif_alloc(words * 4);
        if (!bits) rc = PSIM_ENOMEM;
        else {
            memset(bits, 0, words * 4);
            rc = psim_get_member_bits(r->h, node, bits, words);
        }
    }
    enif_mutex_unlock(r->mu);
    if (rc) { if (bits) enif_free(bits); return err(env, rc); }
    ERL_NIF_TERM list = enif_make_list(env, 0);
    if (bits) {
        for (size_t i = words; i-- > 0;)
            for (int b = 31; b >= 0; b--)
                if ((bits[i] >> b) & 1u)
                    list = enif_make_list_cell(env, enif_make_uint(env, (unsigned)(i * 32 + b)), list);
        enif_free(bits);
    } else {
        for (uint32_t i = v.view_n; i-- > 0;)
            list = enif_make_list_cell(env, enif_make_uint(env, v.view[i]), list);
    }
    return enif_make_tuple2(env, enif_make_atom(env, "ok"), list);
}

/* delivery(Ref, Node) -> {ok, {Have, Round, Hop}} : the tracked broadcast at
 * one node (plumtree_backend merge/2 and the Round field, pt:288-293) */
static ERL_NIF_TERM nif_delivery(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r; unsigned node;
    uint8_t have; uint32_t rnd, hop;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r) || !enif_get_uint(env, argv[1], &node))
        return enif_make_badarg(env);
    LOCK_OR_BUSY(r);
    int rc = psim_get_delivery(r->h, node, 1, &have, &rnd, &hop);
    enif_mutex_unlock(r->mu);
    if (rc) return err(env, rc);
    return enif_make_tuple2(env, enif_make_atom(env, "ok"),
                            enif_make_tuple3(env, enif_make_atom(env, have ? "true" : "false"),
                                             enif_make_uint(env, rnd), enif_make_uint(env, hop)));
}

/* histograms(Ref) -> {ok, #{...}} : overlay statistics (psim_histograms) */
static ERL_NIF_TERM nif_histograms(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r;
    psim_histograms hs;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r)) return enif_make_badarg(env);
    enif_mutex_lock(r->mu);
    int rc = psim_get_histograms(r->h, &hs);
    enif_mutex_unlock(r->mu);
    if (rc) return err(env, rc);
    const uint64_t *bins[5] = {hs.active_in, hs.passive_in, hs.active_out, hs.passive_fill, hs.hop};
    const char *bnames[5] = {"active_in", "passive_in", "active_out", "passive_fill", "hop"};
    ERL_NIF_TERM m = enif_make_new_map(env);
    for (int k = 0; k < 5; k++) {
        ERL_NIF_TERM v[PSIM_HIST_BINS];
        for (int b = 0; b < PSIM_HIST_BINS; b++) v[b] = enif_make_uint64(env, bins[k][b]);
        enif_make_map_put(env, m, enif_make_atom(env, bnames[k]),
                          enif_make_list_from_array(env, v, PSIM_HIST_BINS), &m);
    }
    const char *snames[7] = {"n_up", "delivered", "last_round", "active_links", "symmetric_links",
                             "components", "largest_component"};
    const uint64_t svals[7] = {hs.n_up, hs.delivered, hs.last_round, hs.active_links, hs.symmetric_links,
                               hs.components, hs.largest_component};
    for (int k = 0; k < 7; k++)
        enif_make_map_put(env, m, enif_make_atom(env, snames[k]), enif_make_uint64(env, svals[k]), &m);
    return enif_make_tuple2(env, enif_make_atom(env, "ok"), m);
}

/* snapshot(Ref) -> {ok, Binary} ; restore(Ref, Binary) -> ok */
static ERL_NIF_TERM nif_snapshot(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r;
    size_t need = 0;
    ErlNifBinary bin;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r)) return enif_make_badarg(env);
    int have_bin = 0;
    enif_mutex_lock(r->mu);
    int rc = psim_snapshot(r->h, NULL, 0, &need);
    if (!rc) {
        if (enif_alloc_binary(need, &bin)) have_bin = 1;
        else rc = PSIM_ENOMEM;
    }
    if (!rc) rc = psim_snapshot(r->h, bin.data, bin.size, &need);
    enif_mutex_unlock(r->mu);
    if (rc) {
        if (have_bin) enif_release_binary(&bin);
        return err(env, rc);
    }
    return enif_make_tuple2(env, enif_make_atom(env, "ok"), enif_make_binary(env, &bin));
}

static ERL_NIF_TERM nif_restore(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r;
    ErlNifBinary bin;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r) || !enif_inspect_binary(env, argv[1], &bin))
        return enif_make_badarg(env);
    enif_mutex_lock(r->mu);
    int rc = psim_restore(r->h, bin.data, bin.size);
    enif_mutex_unlock(r->mu);
    return rc ? err(env, rc) : enif_make_atom(env, "ok");
}

/* set_partition(Ref, GroupsBin): one byte per node, the partition group of
 * each (inject_partition/2 as a network partition);
 * clear_partition(Ref): resolve_partition/1 */
static ERL_NIF_TERM nif_set_partition(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r; ErlNifBinary g;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r) || !enif_inspect_binary(env, argv[1], &g) ||
        g.size != r->n_nodes)
        return enif_make_badarg(env);
    LOCK_OR_BUSY(r);
    int rc = psim_set_partition(r->h, (const uint8_t *)g.data, g.size);
    enif_mutex_unlock(r->mu);
    return rc ? err(env, rc) : enif_make_atom(env, "ok");
}

/* set_phash_table(Ref, HashesBin): one native-endian uint32 per node,
 * erlang:phash(NodeSpec, 2^32) - 1 -- the sets v1 slots of every set the
 * engine keeps (16 buckets, or the linear hash's wider tables for SCAMP v1
 * memberships past 80 ids); before the first step only */
static ERL_NIF_TERM nif_set_phash_table(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r; ErlNifBinary b;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r) || !enif_inspect_binary(env, argv[1], &b) ||
        b.size != (size_t)r->n_nodes * 4)
        return enif_make_badarg(env);
    /* (binary data -- a sub-binary's above all -- need not be 4-byte
     * aligned: the hashes are copied into an aligned buffer first) */
    uint32_t *ph = enif_alloc(b.size ? b.size : 4);
    if (!ph) return enif_make_badarg(env);
    memcpy(ph, b.data, b.size);
    LOCK_OR_BUSY_FREE(r, ph);
    int rc = psim_set_phash_table(r->h, ph, r->n_nodes);
    enif_mutex_unlock(r->mu);
    enif_free(ph);
    return rc ? err(env, rc) : enif_make_atom(env, "ok");
}

/* set_bucket_table(Ref, BucketsBin): one byte per node, erlang:phash(NodeSpec,
 * 16) - 1 -- the sets v1 order of every view; before the
 * first step only */
static ERL_NIF_TERM nif_set_bucket_table(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r; ErlNifBinary b;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r) || !enif_inspect_binary(env, argv[1], &b) ||
        b.size != r->n_nodes)
        return enif_make_badarg(env);
    LOCK_OR_BUSY(r);
    int rc = psim_set_bucket_table(r->h, (const uint8_t *)b.data, b.size);
    enif_mutex_unlock(r->mu);
    return rc ? err(env, rc) : enif_make_atom(env, "ok");
}

static ERL_NIF_TERM nif_clear_partition(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r)) return enif_make_badarg(env);
    LOCK_OR_BUSY(r);
    int rc = psim_clear_partition(r->h);
    enif_mutex_unlock(r->mu);
    return rc ? err(env, rc) : enif_make_atom(env, "ok");
}

static ERL_NIF_TERM id_list(ErlNifEnv *env, const uint32_t *v, uint32_t n) {
    ERL_NIF_TERM l = enif_make_list(env, 0);
    for (uint32_t i = n; i-- > 0;) l = enif_make_list_cell(env, enif_make_uint(env, v[i]), l);
    return l;
}

/* node(Ref, Node) -> {ok, #{up, epoch, active, passive, have, round}} :
 * one node's HyParView views (sets:to_list order) and its Plumtree
 * delivery mask (bit m: message id m mod 64 merged, plumtree_backend ETS) */
static ERL_NIF_TERM nif_node(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    sim_res *r; unsigned node;
    psim_node_view v;
    uint64_t round = 0;
    if (!enif_get_resource(env, argv[0], SIM_RT, (void **)&r) || !enif_get_uint(env, argv[1], &node))
        return enif_make_badarg(env);
    LOCK_OR_BUSY(r);
    int rc = psim_get_nodes(r->h, node, 1, &v);
    if (!rc) rc = psim_get_round(r->h, &round);
    enif_mutex_unlock(r->mu);
    if (rc) return err(env, rc);
    ERL_NIF_TERM m = enif_make_new_map(env);
    enif_make_map_put(env, m, enif_make_atom(env, "up"), enif_make_atom(env, v.up ? "true" : "false"), &m);
    enif_make_map_put(env, m, enif_make_atom(env, "epoch"), enif_make_uint(env, v.epoch), &m);
    enif_make_map_put(env, m, enif_make_atom(env, "active"), id_list(env, v.act, v.act_n), &m);
    enif_make_map_put(env, m, enif_make_atom(env, "passive"), id_list(env, v.pas, v.pas_n), &m);
    enif_make_map_put(env, m, enif_make_atom(env, "have"), enif_make_uint64(env, v.have), &m);
    enif_make_map_put(env, m, enif_make_atom(env, "round"), enif_make_uint64(env, round), &m);
    return enif_make_tuple2(env, enif_make_atom(env, "ok"), m);
}

static ErlNifFunc funcs[] = {
    {"create", 1, nif_create, 0},
    {"join_nif", 3, nif_join, 0},
    {"crash_nif", 2, nif_crash, 0},
    {"revive_nif", 2, nif_revive, 0},
    {"leave_nif", 2, nif_leave, 0},
    {"leave_node_nif", 3, nif_leave_node, 0},
    {"broadcast_nif", 3, nif_broadcast, 0},
    {"step", 2, nif_step, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"active_nif", 2, nif_active, 0},
    {"members_nif", 3, nif_members, 0},
    {"delivery_nif", 2, nif_delivery, 0},
    {"histograms", 1, nif_histograms, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"set_partition_nif", 2, nif_set_partition, 0},
    {"clear_partition_nif", 1, nif_clear_partition, 0},
    {"set_bucket_table_nif", 2, nif_set_bucket_table, 0},
    {"set_phash_table_nif", 2, nif_set_phash_table, 0},
    {"omission_nif", 5, nif_omission, 0},
    {"faulted_nif", 3, nif_faulted, 0},
    {"clear_faults_nif", 1, nif_clear_faults, 0},
    {"node_nif", 2, nif_node, 0},
    {"msg_slots_nif", 1, nif_msg_slots, 0},
    {"snapshot", 1, nif_snapshot, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"restore", 2, nif_restore, ERL_NIF_DIRTY_JOB_IO_BOUND},
};

ERL_NIF_INIT(partisan_gpu_sim, funcs, load, NULL, NULL, NULL)
