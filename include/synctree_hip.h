/* synctree_hip.h — C-ABI of libsynctree_hip.so, the MI355X (gfx950) synctree
 * hashing & exchange path of riak_ensemble.
 *
 * Plain C types only (no torch / HIP types cross this boundary).  Every entry
 * point names the reference interface it replaces (jrwest/riak_ensemble,
 * paths relative to the repository root).  The Erlang-side binding a
 * maintainer would add (a NIF + a synctree backend module) is shown in
 * INTEGRATION.md; the Python mirror used by this repo's tests lives in
 * riak_ensemble_amd/synctree.py.
 *
 * Conventions:
 *  - Trees are device-resident and each handle is owned by one lock, like
 *    the gen_server that owns a tree (src/riak_ensemble_peer_tree.erl:58-59):
 *    every entry point holds the handle's lock for the whole call, so calls
 *    on one handle from different threads run one after the other, and
 *    different handles run concurrently (each has its own stream).  A call
 *    that reads a SECOND tree (st_compare*, st_exchange_apply/plan) holds
 *    both locks, taken in address order, and drains its device work before
 *    releasing them: the remote tree is read only through its owner's lock,
 *    as the reference reads it only through the remote peer_tree process
 *    (src/riak_ensemble_exchange.erl:72-81, peer_tree.erl:155-157).
 *    st_rehash_group / st_tops_to_device lock every tree of the group.
 *  - Device work is enqueued asynchronously where the call returns nothing
 *    that depends on it (st_rehash); a device error of such work is
 *    reported (ST_EDEVICE) by the first call that waits for it (st_sync,
 *    st_top_hash, any read), and the tree then refuses every read with
 *    ST_EDEVICE until a full st_rehash completes without error.
 *  - Corruption is a VALUE, not an error: ST_CORRUPTED plus the (Level,
 *    Bucket) of the first node on the root->leaf path whose hash does not
 *    match its parent's entry, exactly like {corrupted, Level, Bucket}
 *    (src/synctree.erl:306-320).
 *  - Keys are passed as (type, ensure_binary bytes) (src/synctree.erl:261-268):
 *      ST_KEY_INT    bytes = <<Key:64/big>>  (integer keys in int64 range;
 *                    ordered numerically)
 *      ST_KEY_ATOM   bytes = atom_to_binary(Key, utf8)
 *      ST_KEY_BINARY bytes = the binary
 *      ST_KEY_TERM   bytes = term_to_binary(Key) (any other key: tuples,
 *                    lists, maps, floats, integers outside int64; the
 *                    reference hashes term_to_binary(Key), or <<Key:64>> for
 *                    an integer; riak_ensemble_amd/csrc/term_key.h)
 *    Keys are kept in Erlang term order (number < atom < tuple < map < nil <
 *    list < binary; numbers by value, atoms and binaries bytewise with a
 *    proper prefix first, maps by size, then keys, then values).  Pids,
 *    ports, refs, funs and bitstrings that are not binaries are rejected
 *    with ST_EINVAL; an int64 / atom / binary passed as ST_KEY_TERM is the
 *    same key as its plain form.
 *  - Packed variable-length arrays: element i of a heap is
 *    heap[off[i] .. off[i+1]) with off[] of n+1 entries.
 *  - Hashes are 17 bytes: <<?H_MD5 = 0, md5/binary>> (src/synctree.erl:255-259).
 */
#ifndef SYNCTREE_HIP_H
#define SYNCTREE_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ST_OK 0
#define ST_NOTFOUND 1
#define ST_CORRUPTED 2
#define ST_EINVAL (-1)   /* bad argument / geometry (reference: crash) */
#define ST_EDEVICE (-2)  /* HIP runtime error */
#define ST_ENOMEM (-3)
#define ST_ERANGE (-4)   /* output buffer too small: the size needed is in the call's size out-param */

#define ST_KEY_INT 0
#define ST_KEY_ATOM 1
#define ST_KEY_BINARY 2
#define ST_KEY_TERM 3

#define ST_FILTER_ALL 0
#define ST_FILTER_LOCAL_ONLY 1   /* drops {K,{_, '$none'}}  (synctree.erl:438-442) */
#define ST_FILTER_REMOTE_ONLY 2  /* drops {K,{'$none', _}}  (synctree.erl:445-449) */

#define ST_DIFF_BOTH 0        /* {K, {A, B}}       */
#define ST_DIFF_LOCAL_ONLY 1  /* {K, {A, '$none'}} */
#define ST_DIFF_REMOTE_ONLY 2 /* {K, {'$none', B}} */

typedef struct st_tree st_tree;

/* ---- lifecycle ------------------------------------------------------ */

/* synctree:new/3..5 (src/synctree.erl:143-170): Height = log_W(Segments),
 * Shift = log2(W).  Returns ST_EINVAL where the reference crashes
 * (compute_height/compute_shift case_clause, synctree.erl:270-284).
 * device: HIP device ordinal. */
int st_create(uint64_t width, uint64_t segments, int device, st_tree **out);
void st_destroy(st_tree *t);

/* Enqueue this tree's work on an external hipStream_t (e.g. torch's
 * current stream); NULL restores the tree's own stream.  The library tracks
 * only the work it enqueues itself: work the CALLER puts on that stream
 * (or any other) must be complete, or ordered by the caller, before a
 * multi-tree call (st_rehash_group, st_tops_to_device*) reads the tree --
 * those calls skip the synchronisation of a tree with nothing of the
 * library's pending. */
int st_set_stream(st_tree *t, void *hip_stream);
int st_sync(st_tree *t);

/* synctree:height/1 (synctree.erl:179-181) */
uint32_t st_height(const st_tree *t);
uint64_t st_width(const st_tree *t);
uint64_t st_segments(const st_tree *t);
/* number of {Key,Value} entries over all segments */
uint64_t st_num_entries(st_tree *t);
/* Device bytes this tree holds, by part: out[0] node slot arrays, out[1]
 * the segment CSR, out[2] the hash-ready tiles (+ their per-segment
 * metadata), out[3] the spare CSR kept for the next merge, out[4] the
 * per-key overlay, out[5] bytes in the process-wide cache of freed blocks
 * (all trees of the process).  No reference counterpart (memory report). */
int st_mem_stats(st_tree *t, uint64_t out[6]);
/* the last error message of this thread */
const char *st_last_error(void);

/* ---- writes --------------------------------------------------------- */

/* insert/3 (synctree.erl:189-209) for n keys, with the semantics of n
 * sequential inserts: last writer wins; a key whose root->segment path fails
 * verification is not inserted and reports ST_CORRUPTED + (level, bucket);
 * other keys are inserted and their paths rehashed (dirty-path update).
 * status/clevel/cbucket: per-key outputs (may be NULL).  Host pointers. */
int st_insert_batch(st_tree *t, uint64_t n, const uint8_t *ktype, const uint8_t *kheap, const uint64_t *koff,
                    const uint8_t *vheap, const uint64_t *voff, int32_t *status, uint32_t *clevel,
                    uint64_t *cbucket);

/* Same for integer keys (ST_KEY_INT) and fixed-width values.
 * keys[n] (int64), vals[n*vlen].  inputs_on_device != 0: both pointers are
 * device memory on this tree's device (no host staging), written by work on
 * the device's NULL stream (torch's default stream): the library orders its
 * reads after that stream's work enqueued before the call (an event, no host
 * wait) -- st_insert_int64_dev names another producer stream.  The call
 * returns after its last read of the inputs.  *n_corrupted (may be NULL)
 * receives the number of rejected keys. */
int st_insert_int64(st_tree *t, uint64_t n, const int64_t *keys, const uint8_t *vals, uint32_t vlen,
                    int inputs_on_device, uint64_t *n_corrupted);
/* st_insert_int64 with device inputs produced on `producer_stream` (a
 * hipStream_t; NULL = the null stream): the tree's reads wait for the work
 * enqueued on it before the call.  No caller-side synchronisation needed. */
int st_insert_int64_dev(st_tree *t, uint64_t n, const int64_t *keys, const uint8_t *vals, uint32_t vlen,
                        void *producer_stream, uint64_t *n_corrupted);

/* corrupt/2 (synctree.erl:241-247): erase Key from its segment without
 * updating the path (test aid). */
int st_corrupt(st_tree *t, uint8_t ktype, const uint8_t *kbytes, uint32_t klen);

/* Raw backend writes (Mod:store/2,3 of synctree_ets.erl:51-66, used through
 * m_batch/m_flush by riak_ensemble_peer_tree repair, peer_tree.erl:264-277,
 * and by the corruption intercepts, test/synctree_intercepts.erl).
 * Inner node content = [{ChildId, Hash17}] with ChildId in
 * [bucket*W, bucket*W+W) (n may be 0 = store []).  Segment content is
 * [{Key,Value}] and must be strictly ascending in key order. */
int st_store_inner(st_tree *t, uint32_t level, uint64_t bucket, uint32_t n, const uint64_t *children,
                   const uint8_t *hashes17);
int st_store_segment(st_tree *t, uint64_t segment, uint64_t n, const uint8_t *ktype, const uint8_t *kheap,
                     const uint64_t *koff, const uint8_t *vheap, const uint64_t *voff);
int st_delete_node(st_tree *t, uint32_t level, uint64_t bucket);
/* store {0,0}: hash17 or NULL (delete); also_record != 0 also sets the
 * #tree.top_hash field (as insert/rehash do) */
int st_store_top(st_tree *t, const uint8_t *hash17, int also_record);
/* Set only the #tree.top_hash record field (hash17 NULL = undefined).  An
 * Erlang tree record is a value: a caller holding an older record of the same
 * backend (e.g. the ETS table) verifies against ITS top hash
 * (synctree.erl:302-304); this lets a host mirror reproduce that exactly. */
int st_set_record_top(st_tree *t, const uint8_t *hash17);

/* ---- rehash / verify ------------------------------------------------ */

/* rehash/1 (upper = 0) and rehash_upper/1 (upper = 1), synctree.erl:489-543:
 * recompute every inner node and the top hash from the segments (or from the
 * stored level-Height nodes).  Kernels K1 segment_hash + K2 level_rehash. */
int st_rehash(st_tree *t, int upper);

/* rehash/1 of n independent trees (e.g. the ensembles one GPU hosts) as ONE
 * batch: same effect as st_rehash(trees[i], 0) for every i.  Width 16,
 * height 3..6, one geometry, one device, no partitions. */
int st_rehash_group(st_tree **trees, uint32_t n);

/* verify/1 (upper = 0) and verify_upper/1 (upper = 1), synctree.erl:549-571 */
int st_verify(st_tree *t, int upper, int *ok);

/* top_hash/1 (synctree.erl:183-185): *present = 0 <=> undefined */
int st_top_hash(st_tree *t, uint8_t out17[17], int *present);

/* Entries recorded for every bucket of `level` (1..Height+1) in its parent
 * node (level 1: the #tree top hash): present[W^(level-1)],
 * hashes17[W^(level-1) * 17].  Used for per-level parity checks. */
int st_level_entries(st_tree *t, uint32_t level, uint8_t *present, uint8_t *hashes17);

/* ---- exchange diff application -------------------
 * riak_ensemble_exchange.erl:71-97 for one remote peer: compare(local,
 * remote) with default options, then for each diff in reference order
 * {K,{'$none',B}} -> insert B; {K,{_, '$none'}} -> nothing; {K,{A,B}} ->
 * insert B iff valid_obj_hash(B, A) (B >= A, riak_ensemble_peer.erl:1726-1729),
 * all as ONE batched insert/3 into the local tree.  valid_obj_hash has no
 * clause unless both hashes start with ?H_OBJ_NONE (0): such a pair is the
 * exchange's function_clause crash, reported as *crashed = 1 with the diffs
 * before it (only) applied.  A corrupted node met during the compare returns
 * ST_CORRUPTED (+ level/bucket/side) and applies nothing (the reference
 * throws out of compare/3).  n_rejected: inserts refused by path
 * verification (insert/3 -> corrupted, ignored by the exchange). */
int st_exchange_apply(st_tree *local, st_tree *remote, uint64_t *n_diffs, uint64_t *n_applied,
                      uint64_t *n_rejected, int *crashed, uint32_t *clevel, uint64_t *cbucket, int *cside);

/* Dry run of st_exchange_apply: compare + valid_obj_hash selection, nothing
 * inserted.  *n_take = remote values an apply would insert (those before the
 * first crash), *crashed = the apply would end in the function_clause crash.
 * Used by the partitioned exchange (parallel.py) to apply only the
 * partitions that precede the first crash in the reference's diff order
 * (riak_ensemble_exchange.erl:71-97).  Returns ST_CORRUPTED like st_compare. */
int st_exchange_plan(st_tree *local, st_tree *remote, uint64_t *n_diffs, uint64_t *n_take, int *crashed,
                     uint32_t *clevel, uint64_t *cbucket, int *cside);

/* ETF atom forms written by st_snapshot_leveldb (synctree_leveldb.erl:134-
 * 152 term_to_binary): utf8 = 0 (default) as OTP < 26 writes them (ATOM_EXT
 * for Latin-1 atoms, the reference's era), 1 = OTP >= 26 (UTF-8 forms). */
int st_set_etf_atoms(st_tree *t, int utf8);

/* The device key record of one key (host-only helper, no device needed):
 * memcmp-then-length order of records is Erlang term order. */
int st_key_record(uint8_t ktype, const uint8_t *bytes, uint64_t len, uint8_t *out, uint64_t cap, uint64_t *out_len);

/* ---- multi-GPU: segment-range partition of one tree ------
 * No reference counterpart: riak_ensemble keeps a tree on one node.  This is
 * the sharding of a single huge tree across the GPUs of one node.
 *
 * st_set_partition: this handle owns segments [seg_lo, seg_hi) only (width
 * 16, height >= 4, whole level-2 subtrees: S/16-aligned; call before the
 * first insert; [0, S) clears it).  Inserts keep the owned keys and drop the
 * rest; st_rehash (upper = 0) hashes the owned subtrees up to level 2 and
 * leaves level 1 + top to st_combine_upper.
 *
 * st_combine_upper: store the 16 level-2 entries (present16[16],
 * hashes17[16*17], all-gathered from every partition) and recompute level 1
 * and the top hash, so every partition holds the global tree's top hash. */
int st_set_partition(st_tree *t, uint64_t seg_lo, uint64_t seg_hi);
int st_combine_upper(st_tree *t, const uint8_t *present16, const uint8_t *hashes17);

/* Ensemble sharding (riak_ensemble_peer.erl:1845-1846: one tree per peer):
 * the top-hash records of n trees on one device written to DEVICE memory
 * `out` (18 bytes per tree: present byte, then the 17-byte hash), the payload
 * of the cross-GPU all-gather of top hashes.  The write into `out` waits for
 * the work enqueued on the null stream before the call (a previous collective
 * may still read `out`); the call returns after it.  st_tops_to_device_on
 * names the caller's stream instead (NULL = the null stream). */
int st_tops_to_device(st_tree **trees, uint32_t n, void *out);
int st_tops_to_device_on(st_tree **trees, uint32_t n, void *out, void *stream);

/* ---- reads ---------------------------------------------------------- */

/* Library-allocated result blocks; free with st_free_result(). */
typedef struct st_result {
    uint64_t n;          /* records */
    int32_t *status;     /* ST_OK / ST_NOTFOUND / ST_CORRUPTED */
    uint32_t *clevel;    /* corruption level (status == ST_CORRUPTED) */
    uint64_t *cbucket;   /* corruption bucket */
    uint64_t *eoff;      /* n+1: entries of record i are [eoff[i], eoff[i+1]) */
    uint64_t n_entries;
    /* inner-level entries */
    uint64_t *child;     /* n_entries */
    uint8_t *hash17;     /* n_entries * 17 */
    /* key/value entries (segments, get, compare) */
    uint8_t *ktype;      /* n_entries */
    uint64_t *koff;      /* n_entries + 1 */
    uint8_t *kheap;
    uint64_t *aoff;      /* n_entries + 1 (value, or local value for diffs) */
    uint8_t *aheap;
    uint64_t *boff;      /* n_entries + 1 (remote value for diffs) */
    uint8_t *bheap;
    uint8_t *kind;       /* n_entries: ST_DIFF_* for compare results */
    uint64_t *seg;       /* n_entries: segment of each diff record */
} st_result;
void st_free_result(st_result *r);

/* get/2 (synctree.erl:213-227) for n keys: per key ST_OK (value = entry
 * eoff[i] of aoff/aheap), ST_NOTFOUND, or ST_CORRUPTED. */
int st_get_batch(st_tree *t, uint64_t n, const uint8_t *ktype, const uint8_t *kheap, const uint64_t *koff,
                 st_result **out);

/* get/2 and insert/3 of ONE key (synctree.erl:189-227) with caller buffers
 * (no result block): the per-key path of the NIF and of
 * riak_ensemble_peer_tree (peer_tree.erl:224-246).  st_get1 returns ST_OK
 * (value in vout[0..*vlen)), ST_NOTFOUND or ST_CORRUPTED (clevel, cbucket);
 * a value longer than vcap sets *vlen and returns ST_EINVAL.  st_insert1
 * returns ST_OK or ST_CORRUPTED. */
int st_get1(st_tree *t, uint8_t ktype, const uint8_t *kbytes, uint32_t klen, uint8_t *vout, uint32_t vcap,
            uint32_t *vlen, uint32_t *clevel, uint64_t *cbucket);
int st_insert1(st_tree *t, uint8_t ktype, const uint8_t *kbytes, uint32_t klen, const uint8_t *value, uint32_t vlen,
               uint32_t *clevel, uint64_t *cbucket);

/* The per-key path of many trees at once (many peer trees of one node
 * taking puts / gets together, riak_ensemble_peer_tree.erl:224-246): request
 * i is insert/3 (or get/2) of key i into trees[i]; trees may repeat.  The
 * requests of each tree are served in request order (the semantics of the
 * per-tree calls one after the other), and the batches of all trees run in
 * ONE device launch (a workgroup per tree, <= 16 keys per tree a launch;
 * more keys: further launches).  Per-request outputs as st_insert1 /
 * st_get1; get values packed in request order into vout with
 * voff_out[n+1].  If vcap is too small: ST_ERANGE with nothing copied and
 * voff_out[n] = the bytes needed (the reads happened: retry with that
 * capacity).  Trees on one device. */
int st_insert1_multi(st_tree **trees, uint32_t n, const uint8_t *ktype, const uint8_t *kheap, const uint64_t *koff,
                     const uint8_t *vheap, const uint64_t *voff, int32_t *status, uint32_t *clevel, uint64_t *cbucket);
int st_get1_multi(st_tree **trees, uint32_t n, const uint8_t *ktype, const uint8_t *kheap, const uint64_t *koff,
                  uint8_t *vout, uint64_t vcap, uint64_t *voff_out, int32_t *status, uint32_t *clevel,
                  uint64_t *cbucket);

/* exchange_get/3 (synctree.erl:231-237) at one level for n buckets, each
 * verified root->node (verified_hashes, synctree.erl:288-298).  Level 0
 * (bucket 0) is answered as [{0, TopHash}] by the caller from st_top_hash.
 * Inner levels fill child/hash17; the segment level fills ktype/koff/kheap
 * and aoff/aheap.  This is also the batched form of the streaming
 * start_exchange_level protocol (test/synctree_remote.erl:25-35). */
int st_exchange_get_batch(st_tree *t, uint32_t level, uint64_t n, const uint64_t *buckets, st_result **out);

/* Mod:fetch({Level,Bucket}, [], State) (synctree_ets.erl:38-44) for n
 * buckets of one level, WITHOUT verification (the raw backend image).
 * Level 0 returns the stored {0,0} top hash as one inner entry (child 0). */
int st_fetch_batch(st_tree *t, uint32_t level, uint64_t n, const uint64_t *buckets, st_result **out);

/* compare/3,5 between two trees on the same device (local_compare/2,
 * synctree.erl:361-382, with filters :421-449): level-synchronous tree
 * diff (kernel K3).  On success returns ST_OK and the diff records in
 * reference order (AccFun = Keys ++ Acc: descending segment, ascending key)
 * in out->ktype/koff/kheap, out->kind, out->aoff/aheap (local value),
 * out->boff/bheap (remote value), out->seg.  If a visited node fails
 * verification the reference crashes (orddict_delta has no clause for the
 * {corrupted,L,B} tuple): returns ST_CORRUPTED with the first such node in
 * reference visiting order in *clevel, *cbucket and *cside (0 local,
 * 1 remote) and no records. */
int st_compare(st_tree *local, st_tree *remote, int filter, st_result **out, uint32_t *clevel,
               uint64_t *cbucket, int *cside);

/* The same compare with the ordered diff records kept in device memory (the
 * local tree's compare workspace, valid until its next compare): each record
 * names the key's entry in the local and/or remote tree, in reference order.
 * *n_diffs receives the number of records.  st_compare = this + the record
 * bytes gathered and copied to the host.  One host round trip per call. */
int st_compare_device(st_tree *local, st_tree *remote, int filter, uint64_t *n_diffs, uint32_t *clevel,
                      uint64_t *cbucket, int *cside);

/* Diagnostics of the last compare on `local`: visited[l] = nodes visited at
 * level l (l = 1..Height+1; visited[0] unused), and the algorithmic bytes of
 * the final-level segment pairs (offsets, key records, values, entries). */
int st_compare_stats(st_tree *local, uint64_t *visited, uint32_t max_levels, uint64_t *seg_bytes);

/* ---- synctree_leveldb on-disk format ---------------
 * The records src/synctree_leveldb.erl writes for this tree: one per stored
 * node {Level, Bucket}, key <<0, TreeId/binary, Level:8,
 * (binary:encode_unsigned(Bucket))/binary>> (synctree_leveldb.erl:104-109),
 * value term_to_binary(Node) (:134-152): the 17-byte top hash at {0,0},
 * [{ChildId, Hash17}] for inner nodes, [{Key, Value}] for segments.  Empty
 * nodes are not written (rehash/1 deletes them, synctree.erl:529-531) unless
 * their own entry is still present -- the [] record a raw store or corrupt/2
 * leaves (synctree.erl:246-247) until the next rehash.  Records are in
 * (Level, Bucket) order.  Atom keys: ATOM_EXT for Latin-1 atoms as
 * term_to_binary writes them before OTP 26 (default), or the UTF-8 forms
 * (st_set_etf_atoms); term keys: the caller's term_to_binary bytes.  A
 * checkpoint into an existing DB must also delete the tree's records that
 * the new snapshot no longer holds. */
typedef struct st_kv {
    uint64_t n;          /* records */
    uint64_t *koff;      /* n+1 */
    uint8_t *kheap;
    uint64_t *voff;      /* n+1 */
    uint8_t *vheap;
} st_kv;
void st_free_kv(st_kv *kv);

/* Encode the whole tree on the device and copy the records to the host. */
int st_snapshot_leveldb(st_tree *t, const uint8_t *tree_id, uint32_t id_len, st_kv **out);
/* The same encode with the records left in (then freed from) device memory:
 * the bench path; reports the record count and key/value byte totals. */
int st_snapshot_leveldb_device(st_tree *t, const uint8_t *tree_id, uint32_t id_len, uint64_t *n_records,
                               uint64_t *key_bytes, uint64_t *value_bytes);
/* Replace the tree's content with the nodes stored in n LevelDB records (any
 * order; for a repeated key the later record wins, as in one write batch) and
 * set #tree.top_hash from {0,0} (new/5 + reload_top_hash, synctree.erl:
 * 151-175).  Records of other tree ids, or keys db_key/3 never produces for
 * this geometry, are ignored (a shared DB, synctree_leveldb.erl:66-83).  A
 * value binary_to_term cannot decode (malformed, truncated, trailing bytes)
 * leaves that node absent, as fetch/3 answers Default for it
 * (synctree_leveldb.erl:111-123), and counts in *n_skipped.  A decodable node
 * the device cannot hold (non-17-byte hashes, child ids outside the node,
 * keys outside the int64/atom/binary domain -- term keys are restored with
 * st_store_segment --, non-binary values, unsorted orddicts, compressed
 * terms) returns ST_EINVAL and changes nothing. */
int st_restore_leveldb(st_tree *t, const uint8_t *tree_id, uint32_t id_len, uint64_t n, const uint8_t *kheap,
                       const uint64_t *koff, const uint8_t *vheap, const uint64_t *voff, uint64_t *n_loaded,
                       uint64_t *n_skipped);

/* ---- diagnostics ---------------------------------------------------- */

/* Key -> segment (get_segment/2, synctree.erl:251-253) on the device. */
int st_segment_of_batch(st_tree *t, uint64_t n, const uint8_t *ktype, const uint8_t *kheap,
                        const uint64_t *koff, uint64_t *segments_out);

/* Enable per-kernel HIP-event timing on this tree's stream; st_kernel_stats
 * returns the accumulated launch count and milliseconds of the named
 * kernel ("segment_hash", "level_rehash", "key_segment", "tree_compare"...). */
int st_set_timing(st_tree *t, int enabled);
int st_kernel_stats(st_tree *t, const char *kernel, uint64_t *launches, double *total_ms);

/* Fault injection for tests (no reference counterpart; the reference's
 * equivalent is rt_intercept, test/synctree_intercepts.erl).
 * ST_DBG_SKIP_MAIL: the next fused rehash launches of this tree do not store
 * the mailbox entry of window `value` (a level-(Height-2) subtree; -1 = off),
 * so the launch's climb never sees it: the bounded wait then reports
 * ST_EDEVICE instead of hashing a stale entry into the top hash. */
#define ST_DBG_SKIP_MAIL 1
/* ST_DBG_PAGES: streaming insert batches in the paged segment layout with
 * `value` percent of slack per page (0 = the default, 25 %), from the next
 * streaming batch on (by default the first batch after any other call merges
 * into the CSR and the second builds the pages); -1 = off (every batch merges
 * into the canonical CSR; the pages are folded first). */
#define ST_DBG_PAGES 2
/* ST_DBG_PAGE_CHECK: value != 0 validates every page before and after each
 * paged batch, bounds-checks the pages the batch's positions and verify
 * kernels read, and runs the merge checked (a store outside its page is not
 * performed): any violation is ST_EDEVICE (the tree then refuses reads until
 * a clean full rehash) instead of an access outside the page arrays. */
#define ST_DBG_PAGE_CHECK 3
/* ST_DBG_PAGE_POISON: fault injection for the checked mode: segment `value`'s
 * page (pages on) claims entries past its capacity. */
#define ST_DBG_PAGE_POISON 4
/* ST_DBG_PAGE_DOWN: which in-place page merges shift the entries before the
 * batch's insert positions down into the page's head slack instead of those
 * after them up into its tail slack: 0 (default) never -- pages then keep
 * all their slack after their content --, 1 when that moves fewer bytes, 2
 * whenever the growth fits the head (tests, A/B; pages built from then on
 * split their slack).  Measured slower: a page shifted down
 * starts its values off 16-byte alignment, and the verify and the hash of
 * its segment then read every MD5 block unaligned. */
#define ST_DBG_PAGE_DOWN 5
int st_debug_knob(st_tree *t, int knob, int64_t value);

/* The paged segment layout of streaming insert batches (no reference
 * counterpart: the reference's backend stores each touched segment's
 * orddict, synctree.erl:201-209, :468-485).  An insert batch
 * small next to the tree rewrites only the tails of the segments it touches
 * inside per-segment pages with slack; every other call folds the pages back
 * into the canonical CSR first.  out[0] = pages in use, out[1] = batches
 * through the pages, out[2] = page builds (the first batch's, and rebuilds
 * when moved segments fill the append region), out[3] = folds, out[4] =
 * entry slots of the segments moved to new pages, out[5] = value bytes of
 * the segments the batches touched (before each merge). */
int st_page_stats(st_tree *t, uint64_t out[6]);

#ifdef __cplusplus
}
#endif
#endif
