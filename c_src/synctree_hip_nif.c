/* synctree_hip_nif.c — the Erlang NIF over libsynctree_hip.so (C-ABI in
 * include/synctree_hip.h).  It is the binding riak_ensemble would load as
 * priv/synctree_hip_nif.so behind the backend module src/synctree_hip.erl
 * (INTEGRATION.md §2-3), so that synctree:new(Id, W, S, synctree_hip) runs on
 * the GPU with the reference's call sites unchanged:
 *
 *   backend behaviour (synctree_ets.erl:22-66)   new/3, fetch/3, store/2
 *   synctree bulk hooks      insert_batch/2, insert/3, get/2,
 *                                                rehash/2, verify/2, top_hash/1,
 *                                                set_record_top/2, exchange_get/3,
 *                                                compare/3, corrupt/2
 *   exchange (riak_ensemble_exchange.erl:71-97)  exchange_apply/2, exchange_plan/2
 *   ensembles of one GPU (peer.erl:1845-1846)    rehash_group/1
 *   checkpoint (synctree_leveldb.erl:104-152)    snapshot/2, restore/3, set_etf_atoms/2
 *
 * Keys cross as {Type, Bin} built by synctree_hip:enc/1 (ensure_binary/1,
 * synctree.erl:261-268): 0 integer (<<K:64/big>>), 1 atom (utf8), 2 binary,
 * 3 any other term (term_to_binary(K)).  Values are binaries.  Corruption is
 * a value, {corrupted, Level, Bucket}, as in synctree.erl:306-320.  Calls
 * that can take more than ~1 ms are registered on dirty CPU schedulers.
 *
 * Erlang/OTP is not installed in the build image of this repository: this
 * file is compile-checked against the erl_nif API declarations in
 * tests/nif_stub/erl_nif.h (tests/test_nif_shim.py) and is built for real by
 * the rebar port spec of INTEGRATION.md §1.
 */
#include <erl_nif.h>
#include <string.h>

#include "synctree_hip.h"

static ErlNifResourceType *TREE_RT;
typedef struct {
    st_tree *t;
} tree_res;

static ERL_NIF_TERM A_OK, A_ERROR, A_NOTFOUND, A_CORRUPTED, A_UNDEFINED, A_NONE, A_TRUE, A_FALSE, A_PUT, A_DELETE,
    A_EXCHANGE_FAILED;

static void tree_dtor(ErlNifEnv *env, void *obj) {
    (void)env;
    tree_res *r = (tree_res *)obj;
    if (r->t) st_destroy(r->t);
    r->t = NULL;
}

static int load(ErlNifEnv *env, void **priv, ERL_NIF_TERM info) {
    (void)priv;
    (void)info;
    TREE_RT = enif_open_resource_type(env, NULL, "synctree_hip", tree_dtor, ERL_NIF_RT_CREATE, NULL);
    A_OK = enif_make_atom(env, "ok");
    A_ERROR = enif_make_atom(env, "error");
    A_NOTFOUND = enif_make_atom(env, "notfound");
    A_CORRUPTED = enif_make_atom(env, "corrupted");
    A_UNDEFINED = enif_make_atom(env, "undefined");
    A_NONE = enif_make_atom(env, "$none");
    A_TRUE = enif_make_atom(env, "true");
    A_FALSE = enif_make_atom(env, "false");
    A_PUT = enif_make_atom(env, "put");
    A_DELETE = enif_make_atom(env, "delete");
    A_EXCHANGE_FAILED = enif_make_atom(env, "exchange_failed");
    return TREE_RT ? 0 : 1;
}

/* {error, Reason} with the library's last message (library errors are
 * programmer errors or device failures: the reference would crash) */
static ERL_NIF_TERM err(ErlNifEnv *env) {
    return enif_make_tuple2(env, A_ERROR, enif_make_string(env, st_last_error(), ERL_NIF_LATIN1));
}

static ERL_NIF_TERM corrupted(ErlNifEnv *env, uint32_t level, uint64_t bucket) {
    return enif_make_tuple3(env, A_CORRUPTED, enif_make_uint(env, level), enif_make_uint64(env, (ErlNifUInt64)bucket));
}

static int get_tree(ErlNifEnv *env, ERL_NIF_TERM t, st_tree **out) {
    tree_res *r;
    if (!enif_get_resource(env, t, TREE_RT, (void **)&r) || !r->t) return 0;
    *out = r->t;
    return 1;
}

static ERL_NIF_TERM bin_term(ErlNifEnv *env, const uint8_t *p, uint64_t n) {
    ERL_NIF_TERM b;
    unsigned char *d = enif_make_new_binary(env, (size_t)n, &b);
    if (n) memcpy(d, p, (size_t)n);
    return b;
}

/* ------------------------------------------------------------ packed inputs */

/* A packed key (and optional value) list: the heaps point into the callers'
 * binaries, copied once into contiguous arrays. */
typedef struct {
    unsigned n;
    uint8_t *kt, *kh, *vh;
    uint64_t *ko, *vo;
} packed;

static void packed_free(packed *p) {
    enif_free(p->kt);
    enif_free(p->kh);
    enif_free(p->vh);
    enif_free(p->ko);
    enif_free(p->vo);
    memset(p, 0, sizeof(*p));
}

/* key term {Type, Bin} */
static int get_key(ErlNifEnv *env, ERL_NIF_TERM k, unsigned *ty, ErlNifBinary *b) {
    const ERL_NIF_TERM *kv;
    int a;
    return enif_get_tuple(env, k, &a, &kv) && a == 2 && enif_get_uint(env, kv[0], ty) && *ty <= ST_KEY_TERM &&
           enif_inspect_binary(env, kv[1], b);
}

/* list of Key (with_values = 0), of {Key, Value} (1), or of {Type, Bin,
 * Value} (2: the insert_batch form) */
static int pack(ErlNifEnv *env, ERL_NIF_TERM list, int with_values, packed *p) {
    unsigned n;
    memset(p, 0, sizeof(*p));
    if (!enif_get_list_length(env, list, &n)) return 0;
    p->n = n;
    p->kt = enif_alloc(n + 1);
    p->ko = enif_alloc(8 * ((size_t)n + 1));
    p->vo = enif_alloc(8 * ((size_t)n + 1));
    ErlNifBinary *kb = enif_alloc(sizeof(ErlNifBinary) * ((size_t)n + 1));
    ErlNifBinary *vb = enif_alloc(sizeof(ErlNifBinary) * ((size_t)n + 1));
    int ok = p->kt && p->ko && p->vo && kb && vb;
    uint64_t kk = 0, vv = 0;
    ERL_NIF_TERM h, t = list;
    for (unsigned i = 0; ok && i < n; i++) {
        unsigned ty;
        ok = enif_get_list_cell(env, t, &h, &t);
        if (!ok) break;
        if (with_values == 0) {
            ok = get_key(env, h, &ty, &kb[i]);
            vb[i].size = 0;
        } else {
            const ERL_NIF_TERM *e;
            int a;
            ok = enif_get_tuple(env, h, &a, &e);
            if (ok && with_values == 1) ok = a == 2 && get_key(env, e[0], &ty, &kb[i]) && enif_inspect_binary(env, e[1], &vb[i]);
            else if (ok) ok = a == 3 && enif_get_uint(env, e[0], &ty) && ty <= ST_KEY_TERM &&
                             enif_inspect_binary(env, e[1], &kb[i]) && enif_inspect_binary(env, e[2], &vb[i]);
        }
        if (!ok) break;
        p->kt[i] = (uint8_t)ty;
        p->ko[i] = kk;
        p->vo[i] = vv;
        kk += kb[i].size;
        vv += vb[i].size;
    }
    if (ok) {
        p->ko[n] = kk;
        p->vo[n] = vv;
        p->kh = enif_alloc((size_t)kk + 1);
        p->vh = enif_alloc((size_t)vv + 1);
        ok = p->kh && p->vh;
        for (unsigned i = 0; ok && i < n; i++) {
            if (kb[i].size) memcpy(p->kh + p->ko[i], kb[i].data, kb[i].size);
            if (with_values && vb[i].size) memcpy(p->vh + p->vo[i], vb[i].data, vb[i].size);
        }
    }
    enif_free(kb);
    enif_free(vb);
    if (!ok) packed_free(p);
    return ok;
}

/* ------------------------------------------------------------ lifecycle */

/* new(Width, Segments, Device) -> {ok, Ref}   (synctree:new/5, synctree.erl:151-170) */
static ERL_NIF_TERM nif_new(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    ErlNifUInt64 w, s;
    int dev;
    (void)argc;
    if (!enif_get_uint64(env, argv[0], &w) || !enif_get_uint64(env, argv[1], &s) || !enif_get_int(env, argv[2], &dev))
        return enif_make_badarg(env);
    st_tree *t;
    if (st_create((uint64_t)w, (uint64_t)s, dev, &t) != ST_OK) return err(env);   /* bad geometry: the reference crashes */
    tree_res *r = enif_alloc_resource(TREE_RT, sizeof(tree_res));
    r->t = t;
    ERL_NIF_TERM ref = enif_make_resource(env, r);
    enif_release_resource(r);
    return enif_make_tuple2(env, A_OK, ref);
}

/* height(Ref) -> H   (synctree.erl:179-181) */
static ERL_NIF_TERM nif_height(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree *t;
    (void)argc;
    if (!get_tree(env, argv[0], &t)) return enif_make_badarg(env);
    return enif_make_uint(env, st_height(t));
}

/* ------------------------------------------------------------ writes */

static ERL_NIF_TERM status_list(ErlNifEnv *env, unsigned n, const int32_t *st, const uint32_t *cl, const uint64_t *cb) {
    ERL_NIF_TERM res = enif_make_list(env, 0);
    for (unsigned i = n; i-- > 0;)
        res = enif_make_list_cell(env, st[i] == ST_CORRUPTED ? corrupted(env, cl[i], cb[i]) : A_OK, res);
    return res;
}

/* insert_batch(Ref, [{Type, KeyBin, Value}]) -> [ok | {corrupted, L, B}]
 * = N x synctree:insert/3 (synctree.erl:189-209), last writer wins.  DIRTY. */
static ERL_NIF_TERM nif_insert_batch(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree *t;
    packed p;
    (void)argc;
    if (!get_tree(env, argv[0], &t) || !pack(env, argv[1], 2, &p)) return enif_make_badarg(env);
    int32_t *st = enif_alloc(4 * ((size_t)p.n + 1));
    uint32_t *cl = enif_alloc(4 * ((size_t)p.n + 1));
    uint64_t *cb = enif_alloc(8 * ((size_t)p.n + 1));
    ERL_NIF_TERM res;
    if (st_insert_batch(t, p.n, p.kt, p.kh, p.ko, p.vh, p.vo, st, cl, cb) < 0) res = err(env);
    else res = status_list(env, p.n, st, cl, cb);
    enif_free(st);
    enif_free(cl);
    enif_free(cb);
    packed_free(&p);
    return res;
}

/* insert(Ref, {Type, KeyBin}, Value) -> ok | {corrupted, L, B}
 * (synctree:insert/3, synctree.erl:189-209; peer_tree do_insert, :224-234).
 * One key: the small-batch device path (one fused kernel). */
static ERL_NIF_TERM nif_insert(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree *t;
    unsigned ty;
    ErlNifBinary kb, vb;
    (void)argc;
    if (!get_tree(env, argv[0], &t) || !get_key(env, argv[1], &ty, &kb) || !enif_inspect_binary(env, argv[2], &vb))
        return enif_make_badarg(env);   /* a non-binary value: function_clause (synctree.erl:190) */
    uint32_t cl;
    uint64_t cb;
    const int st = st_insert1(t, (uint8_t)ty, kb.data, (uint32_t)kb.size, vb.data, (uint32_t)vb.size, &cl, &cb);
    if (st < 0) return err(env);
    return st == ST_CORRUPTED ? corrupted(env, cl, cb) : A_OK;
}

/* corrupt(Ref, {Type, KeyBin}) -> ok   (synctree:corrupt/2, synctree.erl:241-247) */
static ERL_NIF_TERM nif_corrupt(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree *t;
    unsigned ty;
    ErlNifBinary kb;
    (void)argc;
    if (!get_tree(env, argv[0], &t) || !get_key(env, argv[1], &ty, &kb)) return enif_make_badarg(env);
    return st_corrupt(t, (uint8_t)ty, kb.data, (uint32_t)kb.size) == ST_OK ? A_OK : err(env);
}

/* one {Level, Bucket} */
static int get_id(ErlNifEnv *env, ERL_NIF_TERM id, unsigned *level, ErlNifUInt64 *bucket) {
    const ERL_NIF_TERM *e;
    int a;
    return enif_get_tuple(env, id, &a, &e) && a == 2 && enif_get_uint(env, e[0], level) &&
           enif_get_uint64(env, e[1], bucket);
}

/* put of an inner node [{ChildId, Hash17}] */
static int store_inner(ErlNifEnv *env, st_tree *t, unsigned level, uint64_t bucket, ERL_NIF_TERM node) {
    unsigned n;
    if (!enif_get_list_length(env, node, &n)) return ST_EINVAL;
    uint64_t *ch = enif_alloc(8 * ((size_t)n + 1));
    uint8_t *hs = enif_alloc(17 * ((size_t)n + 1));
    ERL_NIF_TERM h, l = node;
    int rc = ST_OK;
    for (unsigned i = 0; i < n && rc == ST_OK; i++) {
        const ERL_NIF_TERM *e;
        int a;
        ErlNifUInt64 c;
        ErlNifBinary hb;
        if (!enif_get_list_cell(env, l, &h, &l) || !enif_get_tuple(env, h, &a, &e) || a != 2 ||
            !enif_get_uint64(env, e[0], &c) || !enif_inspect_binary(env, e[1], &hb) || hb.size != 17)
            rc = ST_EINVAL;   /* outside the device node domain */
        else {
            ch[i] = (uint64_t)c;
            memcpy(hs + 17 * (size_t)i, hb.data, 17);
        }
    }
    if (rc == ST_OK) rc = st_store_inner(t, level, bucket, n, ch, hs);
    enif_free(ch);
    enif_free(hs);
    return rc;
}

/* store(Ref, [{put, {L, B}, Node} | {delete, {L, B}}]) -> ok
 * Mod:store/2 (synctree_ets.erl:51-66): the m_flush batch of m_store updates
 * (synctree.erl:453-485).  Node: a 17-byte hash for {0,0}; [{ChildId, Hash}]
 * for inner levels; [{{Type, KeyBin}, Value}] for segments (keys encoded by
 * synctree_hip:enc/1).  Applied in list order.  DIRTY. */
static ERL_NIF_TERM nif_store(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree *t;
    (void)argc;
    if (!get_tree(env, argv[0], &t)) return enif_make_badarg(env);
    const unsigned H = st_height(t);
    ERL_NIF_TERM h, l = argv[1];
    if (!enif_is_list(env, l)) return enif_make_badarg(env);
    while (enif_get_list_cell(env, l, &h, &l)) {
        const ERL_NIF_TERM *u;
        int a;
        unsigned level;
        ErlNifUInt64 bucket;
        if (!enif_get_tuple(env, h, &a, &u) || a < 2 || !get_id(env, u[1], &level, &bucket)) return enif_make_badarg(env);
        int rc;
        if (a == 2 && enif_is_identical(u[0], A_DELETE)) {
            rc = level == 0 ? st_store_top(t, NULL, 0) : st_delete_node(t, level, (uint64_t)bucket);
        } else if (a == 3 && enif_is_identical(u[0], A_PUT)) {
            if (level == 0) {
                ErlNifBinary hb;
                if (!enif_inspect_binary(env, u[2], &hb) || hb.size != 17) return enif_make_badarg(env);
                rc = st_store_top(t, hb.data, 0);
            } else if (level <= H) {
                rc = store_inner(env, t, level, (uint64_t)bucket, u[2]);
            } else {
                packed p;
                if (!pack(env, u[2], 1, &p)) return enif_make_badarg(env);
                rc = st_store_segment(t, (uint64_t)bucket, p.n, p.kt, p.kh, p.ko, p.vh, p.vo);
                packed_free(&p);
            }
        } else {
            return enif_make_badarg(env);
        }
        if (rc != ST_OK) return err(env);
    }
    return A_OK;
}

/* set_record_top(Ref, Hash | undefined) -> ok: the #tree.top_hash field of the
 * record in hand, before a verified operation (synctree.erl:302-304) */
static ERL_NIF_TERM nif_set_record_top(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree *t;
    ErlNifBinary hb;
    (void)argc;
    if (!get_tree(env, argv[0], &t)) return enif_make_badarg(env);
    if (enif_is_identical(argv[1], A_UNDEFINED)) return st_set_record_top(t, NULL) == ST_OK ? A_OK : err(env);
    if (!enif_inspect_binary(env, argv[1], &hb) || hb.size != 17) return enif_make_badarg(env);
    return st_set_record_top(t, hb.data) == ST_OK ? A_OK : err(env);
}

/* ------------------------------------------------------------ rehash / verify */

/* rehash(Ref, Upper) -> ok   (rehash/1, rehash_upper/1, synctree.erl:489-543).  DIRTY. */
static ERL_NIF_TERM nif_rehash(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree *t;
    int upper;
    (void)argc;
    if (!get_tree(env, argv[0], &t) || !enif_get_int(env, argv[1], &upper)) return enif_make_badarg(env);
    return st_rehash(t, upper) == ST_OK ? A_OK : err(env);
}

/* verify(Ref, Upper) -> boolean()   (verify/1, verify_upper/1, synctree.erl:549-571).  DIRTY. */
static ERL_NIF_TERM nif_verify(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree *t;
    int upper, ok = 0;
    (void)argc;
    if (!get_tree(env, argv[0], &t) || !enif_get_int(env, argv[1], &upper)) return enif_make_badarg(env);
    if (st_verify(t, upper, &ok) != ST_OK) return err(env);
    return ok ? A_TRUE : A_FALSE;
}

/* top_hash(Ref) -> binary() | undefined   (synctree.erl:183-185) */
static ERL_NIF_TERM nif_top_hash(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree *t;
    int present;
    uint8_t h[17];
    (void)argc;
    if (!get_tree(env, argv[0], &t)) return enif_make_badarg(env);
    if (st_top_hash(t, h, &present) != ST_OK) return err(env);
    return present ? bin_term(env, h, 17) : A_UNDEFINED;
}

/* rehash_group([Ref]) -> ok: the trees of the ensembles one GPU hosts (one
 * tree per peer, riak_ensemble_peer.erl:1845-1846) rehashed as one batch.  DIRTY. */
static ERL_NIF_TERM nif_rehash_group(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    unsigned n;
    ERL_NIF_TERM l = argv[0], h;
    (void)argc;
    if (!enif_get_list_length(env, l, &n)) return enif_make_badarg(env);
    st_tree **ts = enif_alloc(sizeof(st_tree *) * ((size_t)n + 1));
    for (unsigned i = 0; i < n; i++) {
        if (!enif_get_list_cell(env, l, &h, &l) || !get_tree(env, h, &ts[i])) {
            enif_free(ts);
            return enif_make_badarg(env);
        }
    }
    const int rc = st_rehash_group(ts, n);
    enif_free(ts);
    return rc == ST_OK ? A_OK : err(env);
}

/* The requests of many trees: a list of {Ref, {Type, KeyBin}} (with_values
 * 0) or {Ref, {Type, KeyBin}, Value} (1) -> the trees and the packed keys. */
static int pack_multi(ErlNifEnv *env, ERL_NIF_TERM list, int with_values, st_tree ***trees, packed *p) {
    unsigned n;
    if (!enif_get_list_length(env, list, &n)) return 0;
    st_tree **ts = enif_alloc(sizeof(st_tree *) * ((size_t)n + 1));
    ERL_NIF_TERM *keys = enif_alloc(sizeof(ERL_NIF_TERM) * ((size_t)n + 1));
    int ok = ts && keys;
    ERL_NIF_TERM h, t = list;
    for (unsigned i = 0; ok && i < n; i++) {
        const ERL_NIF_TERM *e;
        int a;
        ok = enif_get_list_cell(env, t, &h, &t) && enif_get_tuple(env, h, &a, &e) && a == 2 + with_values &&
             get_tree(env, e[0], &ts[i]);
        if (ok) keys[i] = with_values ? enif_make_tuple2(env, e[1], e[2]) : e[1];
    }
    if (ok) ok = pack(env, enif_make_list_from_array(env, keys, n), with_values, p);
    enif_free(keys);
    if (!ok) {
        enif_free(ts);
        return 0;
    }
    *trees = ts;
    return 1;
}

/* insert_multi([{Ref, {Type, KeyBin}, Value}]) -> [ok | {corrupted, L, B}]:
 * insert/3 of each request into its tree (synctree.erl:189-209; the puts of
 * many peer trees, riak_ensemble_peer_tree.erl:224-234), a tree's requests in
 * list order, every tree's batch in one device launch.  DIRTY. */
static ERL_NIF_TERM nif_insert_multi(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree **ts;
    packed p;
    (void)argc;
    if (!pack_multi(env, argv[0], 1, &ts, &p)) return enif_make_badarg(env);
    int32_t *st = enif_alloc(4 * ((size_t)p.n + 1));
    uint32_t *cl = enif_alloc(4 * ((size_t)p.n + 1));
    uint64_t *cb = enif_alloc(8 * ((size_t)p.n + 1));
    ERL_NIF_TERM res;
    if (st_insert1_multi(ts, p.n, p.kt, p.kh, p.ko, p.vh, p.vo, st, cl, cb) < 0) res = err(env);
    else res = status_list(env, p.n, st, cl, cb);
    enif_free(st);
    enif_free(cl);
    enif_free(cb);
    enif_free(ts);
    packed_free(&p);
    return res;
}

/* get_multi([{Ref, {Type, KeyBin}}]) -> [Value | notfound | {corrupted, L, B}]
 * (synctree:get/2, synctree.erl:213-227, of many trees in one launch).  A
 * value buffer that turns out too small (ST_ERANGE) is resized to the bytes
 * the call reports in vo[n] and the (read-only) call run once more.  DIRTY. */
static ERL_NIF_TERM nif_get_multi(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree **ts;
    packed p;
    (void)argc;
    if (!pack_multi(env, argv[0], 0, &ts, &p)) return enif_make_badarg(env);
    int32_t *st = enif_alloc(4 * ((size_t)p.n + 1));
    uint32_t *cl = enif_alloc(4 * ((size_t)p.n + 1));
    uint64_t *cb = enif_alloc(8 * ((size_t)p.n + 1));
    uint64_t *vo = enif_alloc(8 * ((size_t)p.n + 2));
    uint64_t cap = 64 * ((uint64_t)p.n + 16);
    uint8_t *vout = enif_alloc((size_t)cap);
    int rc = vout ? st_get1_multi(ts, p.n, p.kt, p.kh, p.ko, vout, cap, vo, st, cl, cb) : ST_ENOMEM;
    if (rc == ST_ERANGE) {   /* a concurrent put may grow a value again: at most one more try */
        cap = vo[p.n] + vo[p.n] / 4 + 64;
        enif_free(vout);
        vout = enif_alloc((size_t)cap);
        rc = vout ? st_get1_multi(ts, p.n, p.kt, p.kh, p.ko, vout, cap, vo, st, cl, cb) : ST_ENOMEM;
    }
    ERL_NIF_TERM res;
    if (rc < 0) {
        res = err(env);
    } else {
        res = enif_make_list(env, 0);
        for (unsigned i = p.n; i-- > 0;) {
            ERL_NIF_TERM v;
            if (st[i] == ST_CORRUPTED) v = corrupted(env, cl[i], cb[i]);
            else if (st[i] == ST_NOTFOUND) v = A_NOTFOUND;
            else v = bin_term(env, vout + vo[i], vo[i + 1] - vo[i]);
            res = enif_make_list_cell(env, v, res);
        }
    }
    enif_free(vout);
    enif_free(vo);
    enif_free(st);
    enif_free(cl);
    enif_free(cb);
    enif_free(ts);
    packed_free(&p);
    return res;
}

/* ------------------------------------------------------------ reads */

/* One node of a result block as the orddict the ETS backend holds:
 * [{ChildId, Hash17}] for inner levels, [{{Type, KeyBin}, Value}] for
 * segments (synctree_hip:dec/1 turns the keys back into terms). */
static ERL_NIF_TERM node_term(ErlNifEnv *env, const st_result *res, uint64_t i, int segment_level) {
    ERL_NIF_TERM l = enif_make_list(env, 0);
    for (uint64_t e = res->eoff[i + 1]; e-- > res->eoff[i];) {
        ERL_NIF_TERM k, v;
        if (!segment_level) {
            k = enif_make_uint64(env, (ErlNifUInt64)res->child[e]);
            v = bin_term(env, res->hash17 + 17 * e, 17);
        } else {
            k = enif_make_tuple2(env, enif_make_uint(env, res->ktype[e]),
                                 bin_term(env, res->kheap + res->koff[e], res->koff[e + 1] - res->koff[e]));
            v = bin_term(env, res->aheap + res->aoff[e], res->aoff[e + 1] - res->aoff[e]);
        }
        l = enif_make_list_cell(env, enif_make_tuple2(env, k, v), l);
    }
    return l;
}

static int get_buckets(ErlNifEnv *env, ERL_NIF_TERM list, unsigned *n, uint64_t **out) {
    if (!enif_get_list_length(env, list, n)) return 0;
    uint64_t *bs = enif_alloc(8 * ((size_t)*n + 1));
    ERL_NIF_TERM h, t = list;
    for (unsigned i = 0; i < *n; i++) {
        ErlNifUInt64 b;
        if (!enif_get_list_cell(env, t, &h, &t) || !enif_get_uint64(env, h, &b)) {
            enif_free(bs);
            return 0;
        }
        bs[i] = (uint64_t)b;
    }
    *out = bs;
    return 1;
}

/* fetch(Ref, Level, Bucket) -> Node | []   (Mod:fetch/3, synctree_ets.erl:38-44;
 * the raw image, no verification).  Level 0: [{0, TopHash}] or []. */
static ERL_NIF_TERM nif_fetch(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree *t;
    unsigned level;
    ErlNifUInt64 b;
    st_result *res;
    (void)argc;
    if (!get_tree(env, argv[0], &t) || !enif_get_uint(env, argv[1], &level) || !enif_get_uint64(env, argv[2], &b))
        return enif_make_badarg(env);
    uint64_t bb = (uint64_t)b;
    if (st_fetch_batch(t, level, 1, &bb, &res) < 0) return err(env);
    ERL_NIF_TERM out = node_term(env, res, 0, level == st_height(t) + 1);
    st_free_result(res);
    return out;
}

/* exchange_get(Ref, Level, [Bucket]) -> [Node | {corrupted, L, B}]
 * (exchange_get/3 + verified_hashes, synctree.erl:231-237,288-298), one call
 * per level: the batched start_exchange_level protocol
 * (test/synctree_remote.erl:25-35).  DIRTY. */
static ERL_NIF_TERM nif_exchange_get(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree *t;
    unsigned level, n;
    uint64_t *bs;
    (void)argc;
    if (!get_tree(env, argv[0], &t) || !enif_get_uint(env, argv[1], &level) || !get_buckets(env, argv[2], &n, &bs))
        return enif_make_badarg(env);
    st_result *res;
    const int rc = st_exchange_get_batch(t, level, n, bs, &res);
    enif_free(bs);
    if (rc < 0) return err(env);
    const int seg = level == st_height(t) + 1;
    ERL_NIF_TERM out = enif_make_list(env, 0);
    for (uint64_t i = n; i-- > 0;)
        out = enif_make_list_cell(env, res->status[i] == ST_CORRUPTED ? corrupted(env, res->clevel[i], res->cbucket[i])
                                                                      : node_term(env, res, i, seg), out);
    st_free_result(res);
    return out;
}

/* get(Ref, [{Type, KeyBin}]) -> [Value | notfound | {corrupted, L, B}]
 * (synctree:get/2, synctree.erl:213-227, for a list of keys).  DIRTY. */
static ERL_NIF_TERM nif_get(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree *t;
    packed p;
    (void)argc;
    if (!get_tree(env, argv[0], &t) || !pack(env, argv[1], 0, &p)) return enif_make_badarg(env);
    st_result *res;
    const int rc = st_get_batch(t, p.n, p.kt, p.kh, p.ko, &res);
    packed_free(&p);
    if (rc < 0) return err(env);
    ERL_NIF_TERM out = enif_make_list(env, 0);
    for (uint64_t i = res->n; i-- > 0;) {
        ERL_NIF_TERM v;
        if (res->status[i] == ST_CORRUPTED) v = corrupted(env, res->clevel[i], res->cbucket[i]);
        else if (res->status[i] == ST_NOTFOUND) v = A_NOTFOUND;
        else {
            const uint64_t e = res->eoff[i];
            v = bin_term(env, res->aheap + res->aoff[e], res->aoff[e + 1] - res->aoff[e]);
        }
        out = enif_make_list_cell(env, v, out);
    }
    st_free_result(res);
    return out;
}

/* compare(RefA, RefB, Filter) -> [{{Type, KeyBin}, {A | '$none', B | '$none'}}]
 * in reference order (Keys ++ Acc: descending segment, ascending key; filter
 * 0 all, 1 local_only, 2 remote_only, synctree.erl:421-449), or {corrupted,
 * L, B} where the reference's exchange process crashes.  DIRTY. */
static ERL_NIF_TERM nif_compare(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree *a, *b;
    int filt, side;
    uint32_t cl;
    uint64_t cb;
    st_result *res;
    (void)argc;
    if (!get_tree(env, argv[0], &a) || !get_tree(env, argv[1], &b) || !enif_get_int(env, argv[2], &filt))
        return enif_make_badarg(env);
    const int rc = st_compare(a, b, filt, &res, &cl, &cb, &side);
    if (rc == ST_CORRUPTED) return corrupted(env, cl, cb);
    if (rc < 0) return err(env);
    ERL_NIF_TERM out = enif_make_list(env, 0);
    for (uint64_t e = res->n_entries; e-- > 0;) {
        ERL_NIF_TERM va = A_NONE, vb = A_NONE;
        if (res->kind[e] != ST_DIFF_REMOTE_ONLY) va = bin_term(env, res->aheap + res->aoff[e], res->aoff[e + 1] - res->aoff[e]);
        if (res->kind[e] != ST_DIFF_LOCAL_ONLY) vb = bin_term(env, res->bheap + res->boff[e], res->boff[e + 1] - res->boff[e]);
        ERL_NIF_TERM k = enif_make_tuple2(env, enif_make_uint(env, res->ktype[e]),
                                          bin_term(env, res->kheap + res->koff[e], res->koff[e + 1] - res->koff[e]));
        out = enif_make_list_cell(env, enif_make_tuple2(env, k, enif_make_tuple2(env, va, vb)), out);
    }
    st_free_result(res);
    return out;
}

/* ------------------------------------------------------------ exchange */

/* exchange_apply(RefLocal, RefRemote) -> {ok, Applied} | {exchange_failed,
 * Applied} | {corrupted, L, B}: riak_ensemble_exchange:exchange/5
 * (exchange.erl:71-97) against a remote peer whose tree is on the same
 * device: compare + valid_obj_hash + one batched insert/3, replacing the
 * per-diff riak_ensemble_peer_tree:insert calls.  DIRTY. */
static ERL_NIF_TERM nif_exchange_apply(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree *a, *b;
    uint64_t nd, na, nr, cb;
    uint32_t cl;
    int crashed, side;
    (void)argc;
    if (!get_tree(env, argv[0], &a) || !get_tree(env, argv[1], &b)) return enif_make_badarg(env);
    const int rc = st_exchange_apply(a, b, &nd, &na, &nr, &crashed, &cl, &cb, &side);
    if (rc == ST_CORRUPTED) return corrupted(env, cl, cb);   /* exchange_get threw: nothing applied */
    if (rc < 0) return err(env);
    return enif_make_tuple2(env, crashed ? A_EXCHANGE_FAILED : A_OK, enif_make_uint64(env, (ErlNifUInt64)na));
}

/* exchange_plan(RefLocal, RefRemote) -> {ok | exchange_failed, Diffs, Take} |
 * {corrupted, L, B}: the same with nothing applied (st_exchange_plan), for
 * a partitioned exchange that applies partitions in diff order.  DIRTY. */
static ERL_NIF_TERM nif_exchange_plan(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree *a, *b;
    uint64_t nd, nt, cb;
    uint32_t cl;
    int crashed, side;
    (void)argc;
    if (!get_tree(env, argv[0], &a) || !get_tree(env, argv[1], &b)) return enif_make_badarg(env);
    const int rc = st_exchange_plan(a, b, &nd, &nt, &crashed, &cl, &cb, &side);
    if (rc == ST_CORRUPTED) return corrupted(env, cl, cb);
    if (rc < 0) return err(env);
    return enif_make_tuple3(env, crashed ? A_EXCHANGE_FAILED : A_OK, enif_make_uint64(env, (ErlNifUInt64)nd),
                            enif_make_uint64(env, (ErlNifUInt64)nt));
}

/* ------------------------------------------------------------ checkpoint */

/* snapshot(Ref, TreeId) -> [{DbKey, TermBin}] in (Level, Bucket) order: the
 * records synctree_leveldb holds for the tree (synctree_leveldb.erl:104-152).  DIRTY. */
static ERL_NIF_TERM nif_snapshot(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree *t;
    ErlNifBinary id;
    st_kv *kv;
    (void)argc;
    if (!get_tree(env, argv[0], &t) || !enif_inspect_binary(env, argv[1], &id)) return enif_make_badarg(env);
    if (st_snapshot_leveldb(t, id.data, (uint32_t)id.size, &kv) != ST_OK) return err(env);
    ERL_NIF_TERM list = enif_make_list(env, 0);
    for (uint64_t i = kv->n; i-- > 0;) {
        ERL_NIF_TERM k = bin_term(env, kv->kheap + kv->koff[i], kv->koff[i + 1] - kv->koff[i]);
        ERL_NIF_TERM v = bin_term(env, kv->vheap + kv->voff[i], kv->voff[i + 1] - kv->voff[i]);
        list = enif_make_list_cell(env, enif_make_tuple2(env, k, v), list);
    }
    st_free_kv(kv);
    return list;
}

/* restore(Ref, TreeId, [{DbKey, TermBin}]) -> {ok, Loaded, Skipped}: replace
 * the tree with the nodes of the records (new/5 over synctree_leveldb +
 * reload_top_hash, synctree.erl:151-175).  DIRTY. */
static ERL_NIF_TERM nif_restore(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree *t;
    ErlNifBinary id;
    unsigned n;
    (void)argc;
    if (!get_tree(env, argv[0], &t) || !enif_inspect_binary(env, argv[1], &id) || !enif_get_list_length(env, argv[2], &n))
        return enif_make_badarg(env);
    ErlNifBinary *kb = enif_alloc(sizeof(ErlNifBinary) * ((size_t)n + 1));
    ErlNifBinary *vb = enif_alloc(sizeof(ErlNifBinary) * ((size_t)n + 1));
    uint64_t *ko = enif_alloc(8 * ((size_t)n + 1)), *vo = enif_alloc(8 * ((size_t)n + 1));
    ERL_NIF_TERM h, l = argv[2], res = enif_make_badarg(env);
    uint64_t kk = 0, vv = 0;
    int ok = 1;
    for (unsigned i = 0; ok && i < n; i++) {
        const ERL_NIF_TERM *e;
        int a;
        ok = enif_get_list_cell(env, l, &h, &l) && enif_get_tuple(env, h, &a, &e) && a == 2 &&
             enif_inspect_binary(env, e[0], &kb[i]) && enif_inspect_binary(env, e[1], &vb[i]);
        if (ok) {
            ko[i] = kk;
            vo[i] = vv;
            kk += kb[i].size;
            vv += vb[i].size;
        }
    }
    if (ok) {
        ko[n] = kk;
        vo[n] = vv;
        uint8_t *kh = enif_alloc((size_t)kk + 1), *vh = enif_alloc((size_t)vv + 1);
        for (unsigned i = 0; i < n; i++) {
            if (kb[i].size) memcpy(kh + ko[i], kb[i].data, kb[i].size);
            if (vb[i].size) memcpy(vh + vo[i], vb[i].data, vb[i].size);
        }
        uint64_t loaded = 0, skipped = 0;
        if (st_restore_leveldb(t, id.data, (uint32_t)id.size, n, kh, ko, vh, vo, &loaded, &skipped) != ST_OK) res = err(env);
        else res = enif_make_tuple3(env, A_OK, enif_make_uint64(env, (ErlNifUInt64)loaded),
                                    enif_make_uint64(env, (ErlNifUInt64)skipped));
        enif_free(kh);
        enif_free(vh);
    }
    enif_free(kb);
    enif_free(vb);
    enif_free(ko);
    enif_free(vo);
    return res;
}

/* set_etf_atoms(Ref, Utf8) -> ok: 0 = atom keys in snapshots as term_to_binary
 * writes them before OTP 26 (ATOM_EXT, the default), 1 = OTP 26+.  A node
 * sets it from erlang:system_info(otp_release) once. */
static ERL_NIF_TERM nif_set_etf_atoms(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    st_tree *t;
    int utf8;
    (void)argc;
    if (!get_tree(env, argv[0], &t) || !enif_get_int(env, argv[1], &utf8)) return enif_make_badarg(env);
    return st_set_etf_atoms(t, utf8) == ST_OK ? A_OK : err(env);
}

static ErlNifFunc funcs[] = {
    {"new", 3, nif_new, 0},
    {"height", 1, nif_height, 0},
    {"insert_batch", 2, nif_insert_batch, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"insert", 3, nif_insert, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"insert_multi", 1, nif_insert_multi, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"get_multi", 1, nif_get_multi, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"corrupt", 2, nif_corrupt, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"store", 2, nif_store, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"set_record_top", 2, nif_set_record_top, 0},
    {"rehash", 2, nif_rehash, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"verify", 2, nif_verify, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"top_hash", 1, nif_top_hash, 0},
    {"rehash_group", 1, nif_rehash_group, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"fetch", 3, nif_fetch, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"exchange_get", 3, nif_exchange_get, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"get", 2, nif_get, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"compare", 3, nif_compare, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"exchange_apply", 2, nif_exchange_apply, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"exchange_plan", 2, nif_exchange_plan, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"snapshot", 2, nif_snapshot, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"restore", 3, nif_restore, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"set_etf_atoms", 2, nif_set_etf_atoms, 0},
};

ERL_NIF_INIT(synctree_hip_nif, funcs, load, NULL, NULL, NULL)
