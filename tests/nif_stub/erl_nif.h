/* Declarations of the public erl_nif API used by c_src/synctree_hip_nif.c,
 * restated from the erl_nif documentation so that the NIF shim can be
 * compile-checked (gcc -fsyntax-only) in an image without Erlang/OTP.  Test
 * infrastructure only: the real build uses the OTP installation's header
 * (INTEGRATION.md §1).  Nothing here is linked or executed. */
#ifndef NIF_STUB_ERL_NIF_H
#define NIF_STUB_ERL_NIF_H
#include <stddef.h>
#include <stdint.h>

typedef uintptr_t ERL_NIF_TERM;
typedef struct enif_environment_t ErlNifEnv;
typedef struct enif_resource_type_t ErlNifResourceType;
typedef uint64_t ErlNifUInt64;
typedef int64_t ErlNifSInt64;

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

typedef enum { ERL_NIF_LATIN1 = 1, ERL_NIF_UTF8 = 2 } ErlNifCharEncoding;
typedef enum { ERL_NIF_RT_CREATE = 1, ERL_NIF_RT_TAKEOVER = 2 } ErlNifResourceFlags;
typedef enum { ERL_NIF_DIRTY_JOB_CPU_BOUND = 1, ERL_NIF_DIRTY_JOB_IO_BOUND = 2 } ErlNifDirtyTaskFlags;
typedef void ErlNifResourceDtor(ErlNifEnv *, void *);

ErlNifResourceType *enif_open_resource_type(ErlNifEnv *env, const char *module_str, const char *name,
                                            ErlNifResourceDtor *dtor, ErlNifResourceFlags flags,
                                            ErlNifResourceFlags *tried);
void *enif_alloc_resource(ErlNifResourceType *type, size_t size);
void enif_release_resource(void *obj);
ERL_NIF_TERM enif_make_resource(ErlNifEnv *env, void *obj);
int enif_get_resource(ErlNifEnv *env, ERL_NIF_TERM term, ErlNifResourceType *type, void **objp);

void *enif_alloc(size_t size);
void enif_free(void *ptr);

ERL_NIF_TERM enif_make_atom(ErlNifEnv *env, const char *name);
ERL_NIF_TERM enif_make_string(ErlNifEnv *env, const char *string, ErlNifCharEncoding encoding);
ERL_NIF_TERM enif_make_badarg(ErlNifEnv *env);
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv *env, ERL_NIF_TERM e1, ERL_NIF_TERM e2);
ERL_NIF_TERM enif_make_tuple3(ErlNifEnv *env, ERL_NIF_TERM e1, ERL_NIF_TERM e2, ERL_NIF_TERM e3);
ERL_NIF_TERM enif_make_list(ErlNifEnv *env, unsigned cnt, ...);
ERL_NIF_TERM enif_make_list_from_array(ErlNifEnv *env, const ERL_NIF_TERM arr[], unsigned cnt);
ERL_NIF_TERM enif_make_list_cell(ErlNifEnv *env, ERL_NIF_TERM head, ERL_NIF_TERM tail);
ERL_NIF_TERM enif_make_uint(ErlNifEnv *env, unsigned i);
ERL_NIF_TERM enif_make_uint64(ErlNifEnv *env, ErlNifUInt64 i);
unsigned char *enif_make_new_binary(ErlNifEnv *env, size_t size, ERL_NIF_TERM *termp);

int enif_get_uint(ErlNifEnv *env, ERL_NIF_TERM term, unsigned *ip);
int enif_get_int(ErlNifEnv *env, ERL_NIF_TERM term, int *ip);
int enif_get_uint64(ErlNifEnv *env, ERL_NIF_TERM term, ErlNifUInt64 *ip);
int enif_get_tuple(ErlNifEnv *env, ERL_NIF_TERM term, int *arity, const ERL_NIF_TERM **array);
int enif_get_list_length(ErlNifEnv *env, ERL_NIF_TERM term, unsigned *len);
int enif_get_list_cell(ErlNifEnv *env, ERL_NIF_TERM list, ERL_NIF_TERM *head, ERL_NIF_TERM *tail);
int enif_inspect_binary(ErlNifEnv *env, ERL_NIF_TERM bin_term, ErlNifBinary *bin);
int enif_is_identical(ERL_NIF_TERM lhs, ERL_NIF_TERM rhs);
int enif_is_list(ErlNifEnv *env, ERL_NIF_TERM term);

#define ERL_NIF_INIT(NAME, FUNCS, LOAD, RELOAD, UPGRADE, UNLOAD)                        \
    const void *nif_init_##NAME(void);                                                  \
    const void *nif_init_##NAME(void) {                                                 \
        int (*l)(ErlNifEnv *, void **, ERL_NIF_TERM) = LOAD;                            \
        (void)l;                                                                        \
        return (const void *)FUNCS;                                                     \
    }
#endif
