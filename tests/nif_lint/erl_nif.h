/*
 * tests/nif_lint/erl_nif.h -- TEST INFRASTRUCTURE ONLY: a minimal restatement
 * of the erl_nif API that erlang/c_src/partisan_gpu_sim_nif.c uses, written
 * from the published erl_nif documentation (OTP 19-22; LP64 widths) so the
 * NIF shim can be syntax- and type-checked in an image without Erlang
 * (tests/test_nif_lint.py).  Not the real header: a real build uses
 * $(ERTS_INCLUDE_DIR)/erl_nif.h.
 */
#ifndef PSIM_NIF_LINT_ERL_NIF_H
#define PSIM_NIF_LINT_ERL_NIF_H
#include <stddef.h>

typedef unsigned long ERL_NIF_TERM;
typedef unsigned long ErlNifUInt64;
typedef long ErlNifSInt64;
typedef struct enif_environment_t ErlNifEnv;
typedef struct enif_mutex_t ErlNifMutex;
typedef struct enif_resource_type_t ErlNifResourceType;
typedef void ErlNifResourceDtor(ErlNifEnv *, void *);
typedef enum { ERL_NIF_RT_CREATE = 1, ERL_NIF_RT_TAKEOVER = 2 } ErlNifResourceFlags;
enum { ERL_NIF_DIRTY_JOB_CPU_BOUND = 1, ERL_NIF_DIRTY_JOB_IO_BOUND = 2 };

typedef struct {
    size_t size;
    unsigned char *data;
    void *ref_bin;
    void *__spare__[2];
} ErlNifBinary;

typedef struct {
    const char *name;
    unsigned arity;
    ERL_NIF_TERM (*fptr)(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]);
    unsigned flags;
} ErlNifFunc;

typedef struct {
    int major, minor;
    const char *name;
    int num_of_funcs;
    ErlNifFunc *funcs;
    int (*load)(ErlNifEnv *, void **priv_data, ERL_NIF_TERM load_info);
    int (*reload)(ErlNifEnv *, void **priv_data, ERL_NIF_TERM load_info);
    int (*upgrade)(ErlNifEnv *, void **priv_data, void **old_priv_data, ERL_NIF_TERM load_info);
    void (*unload)(ErlNifEnv *, void *priv_data);
} ErlNifEntry;

void *enif_alloc(size_t size);
void enif_free(void *ptr);
int enif_alloc_binary(size_t size, ErlNifBinary *bin);
void enif_release_binary(ErlNifBinary *bin);
int enif_inspect_binary(ErlNifEnv *env, ERL_NIF_TERM bin_term, ErlNifBinary *bin);
int enif_get_int(ErlNifEnv *env, ERL_NIF_TERM term, int *ip);
int enif_get_uint(ErlNifEnv *env, ERL_NIF_TERM term, unsigned *ip);
int enif_get_uint64(ErlNifEnv *env, ERL_NIF_TERM term, ErlNifUInt64 *ip);
int enif_get_map_value(ErlNifEnv *env, ERL_NIF_TERM map, ERL_NIF_TERM key, ERL_NIF_TERM *value);
int enif_make_map_put(ErlNifEnv *env, ERL_NIF_TERM map_in, ERL_NIF_TERM key, ERL_NIF_TERM value,
                      ERL_NIF_TERM *map_out);
ERL_NIF_TERM enif_make_new_map(ErlNifEnv *env);
ERL_NIF_TERM enif_make_badarg(ErlNifEnv *env);
ERL_NIF_TERM enif_make_atom(ErlNifEnv *env, const char *name);
ERL_NIF_TERM enif_make_uint(ErlNifEnv *env, unsigned i);
ERL_NIF_TERM enif_make_uint64(ErlNifEnv *env, ErlNifUInt64 i);
ERL_NIF_TERM enif_make_binary(ErlNifEnv *env, ErlNifBinary *bin);
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv *env, ERL_NIF_TERM e1, ERL_NIF_TERM e2);
ERL_NIF_TERM enif_make_tuple3(ErlNifEnv *env, ERL_NIF_TERM e1, ERL_NIF_TERM e2, ERL_NIF_TERM e3);
ERL_NIF_TERM enif_make_tuple4(ErlNifEnv *env, ERL_NIF_TERM e1, ERL_NIF_TERM e2, ERL_NIF_TERM e3, ERL_NIF_TERM e4);
ERL_NIF_TERM enif_make_list(ErlNifEnv *env, unsigned cnt, ...);
ERL_NIF_TERM enif_make_list_cell(ErlNifEnv *env, ERL_NIF_TERM car, ERL_NIF_TERM cdr);
ERL_NIF_TERM enif_make_list_from_array(ErlNifEnv *env, const ERL_NIF_TERM arr[], unsigned cnt);
ErlNifMutex *enif_mutex_create(char *name);
void enif_mutex_destroy(ErlNifMutex *mtx);
int enif_mutex_trylock(ErlNifMutex *mtx);
void enif_mutex_lock(ErlNifMutex *mtx);
void enif_mutex_unlock(ErlNifMutex *mtx);
ErlNifResourceType *enif_open_resource_type(ErlNifEnv *env, const char *module_str, const char *name_str,
                                            ErlNifResourceDtor *dtor, ErlNifResourceFlags flags,
                                            ErlNifResourceFlags *tried);
void *enif_alloc_resource(ErlNifResourceType *type, size_t size);
void enif_release_resource(void *obj);
ERL_NIF_TERM enif_make_resource(ErlNifEnv *env, void *obj);
int enif_get_resource(ErlNifEnv *env, ERL_NIF_TERM term, ErlNifResourceType *type, void **objp);

/* the module's entry point (the real macro also carries the VM's version
 * and option fields) */
#define ERL_NIF_INIT(NAME, FUNCS, LOAD, RELOAD, UPGRADE, UNLOAD)                              \
    ErlNifEntry *nif_init(void);                                                             \
    ErlNifEntry *nif_init(void) {                                                            \
        static ErlNifEntry entry = {2, 11, #NAME, sizeof(FUNCS) / sizeof(*(FUNCS)), (FUNCS), \
                                    (LOAD), (RELOAD), (UPGRADE), (UNLOAD)};                   \
        return &entry;                                                                       \
    }
#endif
