// synctree_hip.hip — libsynctree_hip.so: C-ABI (include/synctree_hip.h) over
// the gfx950 kernels in st_kernels.h.  Host code only orchestrates: every
// hash, comparison, sort and merge of tree data runs on the device.
//
// Reference: src/synctree.erl (jrwest/riak_ensemble); see the header for the
// per-function mapping and DESIGN.md for layouts and rooflines.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>

#include <hip/hip_runtime.h>
#include <chrono>
#include <atomic>
#include <map>
#include <mutex>
#include <unordered_map>
#include <string>
#include <vector>
#include <algorithm>

#include "../../include/synctree_hip.h"
#include "st_kernels.h"
#include "rehash_win.h"
#include "leveldb_fmt.h"
#include "small_path.h"
#include "pages.h"

static thread_local std::string g_err;
static const uint64_t HEAP_SLACK = 256;   // md5_global over-reads <= 64 B past a range

#define HIPCHK(x)                                                                         \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            g_err = std::string(#x) + ": " + hipGetErrorString(e_);                       \
            return ST_EDEVICE;                                                            \
        }                                                                                 \
    } while (0)

#define CHK(x)                                     \
    do {                                           \
        int r_ = (x);                              \
        if (r_ != ST_OK) return r_;                \
    } while (0)

struct CmpWork {
    uint32_t nw = 0;                 // waves of the compare walk (fixed grid)
    uint64_t R = 0;                  // scratch records per wave
    uint64_t *wcnt = nullptr, *wbytes = nullptr, *werr = nullptr;
    uint32_t *wst = nullptr;         // [nw][ST_STATW] visited nodes per level
    uint64_t *res = nullptr, *res_dev = nullptr;   // host-mapped: total, max per-wave count, first error
    DiffRec *rec = nullptr, *scratch = nullptr;
    uint64_t cap = 0;
    // wcnt: the waves' epoch-stamped record counts; werr[0..1]: the epoch-
    // stamped first error (atomic min) and largest overflowing count (max)
    uint32_t epoch = 0;
};

struct Pending {
    std::string name;
    hipEvent_t a, b;
};

// One segment CSR's buffers (st_tree's current arrays or its spare set).
struct CsrSet {
    uint64_t *seg_off = nullptr, *seg_voff = nullptr, *koff = nullptr, *voff = nullptr;
    uint8_t *kheap = nullptr, *vheap = nullptr;
    uint64_t cap_n = 0, cap_k = 0, cap_v = 0;
};

// The paged segment layout of streaming insert batches (pages.h): page
// metadata, entry slots and heaps with an append region after the pages.
struct Pages {
    bool on = false;
    PageMeta m{};
    uint64_t *koff = nullptr, *voff = nullptr;
    uint8_t *kheap = nullptr, *vheap = nullptr;
    uint64_t cap_e = 0, cap_k = 0, cap_v = 0;   // allocated entry slots / heap bytes
    uint64_t use_e = 0, use_k = 0, use_v = 0;   // the append region starts here
    uint64_t batches = 0, builds = 0, folds = 0, reloc_e = 0, touched_v = 0;
};

struct st_tree {
    int device = 0;
    int ncu = 256;   // compute units of the device (fixed-grid kernels)
    uint32_t flags = 0;   // DevTree.flags (ST_FLAG_ATOM_UTF8)
    hipStream_t own_stream = nullptr, stream = nullptr;
    hipEvent_t ev_order = nullptr;   // cross-stream ordering of caller device buffers (order_after)
    uint64_t W = 16, S = 1 << 20;
    uint32_t shift = 4, H = 5;
    uint64_t base[ST_MAXLEV + 2] = {0};
    uint64_t nslots = 0;
    uint4 *md5 = nullptr;
    uint16_t *tag = nullptr;
    uint8_t *mark = nullptr, *ok = nullptr;
    // erec[slot] = 1: the backend holds the [] record for this node (a raw
    // store of [] or a corrupt/2 that emptied the segment, synctree.erl:
    // 246-247); snapshots write it while the node is empty.  Allocated on
    // first use.
    uint8_t *erec = nullptr;
    uint32_t *flag = nullptr;
    unsigned long long *cnt64 = nullptr;
    // segment CSR
    uint64_t n = 0, kbytes = 0, vbytes = 0;
    uint64_t *seg_off = nullptr, *seg_voff = nullptr, *koff = nullptr, *voff = nullptr;
    uint8_t *kheap = nullptr, *vheap = nullptr;
    // capacities of the current koff/voff (entries) and heaps (bytes), and the
    // retired previous CSR kept as the next merge's output buffers (csr_take)
    uint64_t cap_n = 0, cap_k = 0, cap_v = 0;
    CsrSet spare;
    // streaming insert batches go to the paged layout (pages.h) while
    // pg_slack >= 0 (percent of slack per page; st_debug_knob ST_DBG_PAGES);
    // any other call folds it back into the CSR first
    Pages pg;
    int pg_slack = 25;
    uint32_t pg_streak = 0;   // streaming batches since the last other call (pages are built at the second)
    bool pg_check = false;   // st_debug_knob ST_DBG_PAGE_CHECK: the checked page merge + a layout check per batch
    int pg_down = 0;         // st_debug_knob ST_DBG_PAGE_DOWN: in-place merges shift down 0 never, 1 by the bytes, 2 when they
                             // fit (pages built while it is 0 keep all their slack after their content)
    bool fresh = true;
    uint32_t *seg_perm = nullptr;   // segments by MD5 block count (K1 order)
    bool perm_valid = false;
    bool perm_any = false;   // seg_perm holds a permutation (perhaps no longer by size)
    // hash-ready tiled messages in seg_perm order (K1; st_kernels.h)
    uint4 *tiles = nullptr;
    uint64_t tiles_cap = 0;         // uint4 units
    uint32_t *tseg = nullptr, *tln = nullptr;
    TileInfo *tinfo = nullptr;
    uint64_t *tpres = nullptr;      // per-window segment presence bitmaps (fused rehash)
    uint16_t *tnoff = nullptr;      // per-window level-H message offsets (fused rehash LDS layout)
    uint32_t *tmhmax = nullptr;     // the largest window's level-H message bytes (device word)
    uint32_t mh_bytes = 0;          // ... as read back at the last tile build
    bool tiles_valid = false;
    bool tiles_wanted = false;      // a full rehash since the tiles went stale: the next one builds them
    uint32_t *lvl_cnt = nullptr;    // finished-children counters (k_rehash_fused climb)
    MailEntry *mail = nullptr;      // climb mailboxes (levels 1..H-2)
    uint32_t mail_epoch = 0;        // epoch of the last fused launch over this tree (MailEntry)
    // segment-range partition (st_set_partition): owned segments [part_lo, part_hi)
    bool partitioned = false;
    uint64_t part_lo = 0, part_hi = 0;
    // compare (K3) workspace, grown on demand
    CmpWork cw;
    // small pinned host buffer for scalar results (one D2H per call)
    uint64_t *pin = nullptr;
    // pinned host staging for result records (st_compare), grown on demand
    uint8_t *rpin = nullptr;
    uint64_t rpin_cap = 0;
    // per-key latency path (small_path.h): overlay of segments changed by
    // small inserts, and the mapped pinned result block of k_small
    Overlay ov{nullptr, nullptr, nullptr, 0};
    bool ov_pending = false;
    SmallOut *sout = nullptr, *sout_dev = nullptr;
    SmallReq *sreq = nullptr, *sreq_dev = nullptr;   // SMALL_SLOTS request slots (host memory)
    SmallRes sres;                                    // the last call's validated results
    uint32_t small_seq = 0;   // sequence number of the last k_small call
    std::atomic<uint64_t> sync_epoch{0};   // host synchronisations of `stream` (tsync; block reuse)
    // the handle's owner lock (one caller at a time, like the tree's
    // gen_server, riak_ensemble_peer_tree.erl:58-59); recursive: entry points
    // call one another
    std::recursive_mutex mu;
    // device-error word in host-mapped memory (ST_DERR_*, set by kernels,
    // checked after every synchronisation) and the poisoned state it leaves:
    // reads refuse with ST_EDEVICE until a full rehash completes cleanly
    uint32_t *derr = nullptr, *derr_dev = nullptr;
    bool poisoned = false;
    uint32_t dbg_skip_mail = ~0u;   // st_debug_knob(ST_DBG_SKIP_MAIL)
    // device work that reads ANOTHER tree's buffers (compare / exchange) may
    // still be in flight on this tree's stream (cleared by a completed wait)
    bool reads_remote = false;
    // work enqueued on `stream` that the call did not wait for (st_rehash):
    // another stream's launch over this tree synchronises it first
    bool async_pending = false;
    // timing
    bool timing = false;
    std::vector<Pending> pending;
    std::map<std::string, std::pair<uint64_t, double>> stats;
};

// ------------------------------------------------------------------ device memory
// Every device buffer of the library comes from one process-wide cache of
// hipMalloc'd blocks, never from the stream-ordered pool (hipMallocAsync /
// hipFreeAsync).  With the pool, the round-2 small-batch ingest lost CSR
// entries and faulted on some MI355X boxes (deterministically on those, at
// the same step of tools/stress_small.py) and never on others; on a failing
// box, plain hipMalloc/hipFree and a never-unmapped block cache both ran the
// same sequence clean (gpurun_out A/B logs in profiles/).
//
// A freed block becomes reusable only after the stream of the tree that freed
// it has been synchronised by the host (tsync): every GPU use enqueued before
// the free has then completed, on any stream.  Blocks are cached by size class
// (1/8-power-of-two steps, <= 12.5 % slack) per device and released to the
// driver only when an allocation runs out of memory.
struct MemBlock {
    void *p;
    uint64_t cls;
    int device;
    const st_tree *owner;   // tree that freed it (nullptr: no pending use)
    uint64_t epoch;         // owner's sync epoch at the free
};
static std::mutex g_mem_mu;
static std::multimap<uint64_t, MemBlock> g_mem_free;          // size class -> free blocks
static std::unordered_map<void *, std::pair<uint64_t, int>> g_mem_live;   // live block -> (class, device)

static uint64_t size_class(uint64_t b) {
    if (b <= 4096) return (b + 255) & ~255ull;
    const int k = 63 - __builtin_clzll(b);
    const uint64_t step = 1ull << (k - 3);
    return (b + step - 1) & ~(step - 1);
}
static bool block_ready(const MemBlock &m) {
    return !m.owner || m.owner->sync_epoch.load(std::memory_order_acquire) > m.epoch;
}
// Release cached blocks of `device` to the driver (all of them after a device
// synchronisation when `all`, else the ready ones).  g_mem_mu held.
static void mem_release_locked(int device, bool all) {
    for (auto it = g_mem_free.begin(); it != g_mem_free.end();) {
        if (it->second.device == device && (all || block_ready(it->second))) {
            (void)hipFree(it->second.p);
            it = g_mem_free.erase(it);
        } else {
            ++it;
        }
    }
}

static int dalloc(st_tree *t, void **p, uint64_t bytes) {
    *p = nullptr;
    const uint64_t c = size_class(bytes ? bytes : 16);
    std::lock_guard<std::mutex> g(g_mem_mu);
    auto rng = g_mem_free.equal_range(c);
    for (auto it = rng.first; it != rng.second; ++it)
        if (it->second.device == t->device && block_ready(it->second)) {
            *p = it->second.p;
            g_mem_free.erase(it);
            g_mem_live[*p] = {c, t->device};
            return ST_OK;
        }
    hipError_t e = hipMalloc(p, c);
    if (e == hipErrorOutOfMemory) {   // give cached blocks back: the ready ones, then all after a device sync
        (void)hipGetLastError();
        mem_release_locked(t->device, false);
        e = hipMalloc(p, c);
        if (e == hipErrorOutOfMemory) {
            (void)hipGetLastError();
            (void)hipDeviceSynchronize();
            mem_release_locked(t->device, true);
            e = hipMalloc(p, c);
        }
    }
    if (e != hipSuccess) {
        *p = nullptr;
        (void)hipGetLastError();
        g_err = std::string("hipMalloc: ") + hipGetErrorString(e);
        return e == hipErrorOutOfMemory ? ST_ENOMEM : ST_EDEVICE;
    }
    g_mem_live[*p] = {c, t->device};
    return ST_OK;
}
template <typename T>
static int dalloc_t(st_tree *t, T **p, uint64_t count) {
    return dalloc(t, (void **)p, count * sizeof(T));
}
static void dfree(st_tree *t, void *p) {
    if (!p) return;
    std::lock_guard<std::mutex> g(g_mem_mu);
    auto it = g_mem_live.find(p);
    if (it == g_mem_live.end()) return;   // not ours (never happens)
    g_mem_free.emplace(it->second.first, MemBlock{p, it->second.first, it->second.second, t,
                                                 t->sync_epoch.load(std::memory_order_relaxed)});
    g_mem_live.erase(it);
}
// A tree's pending frees are safe once its stream is idle (st_destroy).
static void mem_forget_owner(const st_tree *t) {
    std::lock_guard<std::mutex> g(g_mem_mu);
    for (auto &kv : g_mem_free)
        if (kv.second.owner == t) kv.second.owner = nullptr;
}

// Host synchronisation of a tree's stream; it also makes the blocks the tree
// freed before it reusable.
static int synced(st_tree *t);
static int tsync(st_tree *t) {
    const hipError_t e = hipStreamSynchronize(t->stream);
    if (e != hipSuccess) {
        g_err = std::string("hipStreamSynchronize: ") + hipGetErrorString(e);
        return ST_EDEVICE;
    }
    return synced(t);
}
// The tree's stream has drained (synchronised here, or idle while its work
// ran and completed on a stream that was): bookkeeping and its device-error word.
static int synced(st_tree *t) {
    t->sync_epoch.fetch_add(1, std::memory_order_release);
    t->reads_remote = false;
    t->async_pending = false;
    // every kernel enqueued before has completed: its device-error word is final
    if (t->derr && __atomic_load_n(t->derr, __ATOMIC_ACQUIRE)) {
        const uint32_t w = __atomic_exchange_n(t->derr, 0u, __ATOMIC_ACQ_REL);
        t->poisoned = true;
        g_err = std::string("device error 0x") + std::to_string(w) +
                ((w & ST_DERR_MAIL) ? ": fused rehash: a window root's mailbox entry never arrived (bounded wait "
                                      "timed out); the tree's upper levels are invalid until a clean full rehash"
                : (w & ST_DERR_CMP) ? ": compare walk: a wave's record count never arrived (bounded wait timed out)"
                                    : "");
        return ST_EDEVICE;
    }
    return ST_OK;
}

// Reads of a tree whose last device work failed are refused (ST_EDEVICE)
// until a full rehash completes cleanly.
static int alive(const st_tree *t) {
    if (!t->poisoned) return ST_OK;
    g_err = "tree is in error after a failed device launch (rehash it)";
    return ST_EDEVICE;
}

// Entry-point guards.  ENTER: the handle's owner lock for the whole call (+
// its device, + refuse a poisoned tree); ENTER_ANY: the same without the
// poison check (rehash, sync, destroy, stats).
#define ENTER_ANY(t)                                                \
    if (!(t)) { g_err = "NULL tree"; return ST_EINVAL; }            \
    std::lock_guard<std::recursive_mutex> enter_lk_((t)->mu);       \
    CHK(use_device(t))
#define ENTER(t)   \
    ENTER_ANY(t);  \
    CHK(alive(t))

// Two trees read by one call (compare / exchange): both owner locks, taken in
// address order (no lock-order deadlock between two exchanges A->B and B->A),
// and the local stream drained before they are released, so no device work
// that reads the remote tree's buffers outlives the remote's lock (the
// remote's owner may free or replace them as soon as it runs again).
struct PairLock {
    st_tree *a, *b;
    std::unique_lock<std::recursive_mutex> l1, l2;
    PairLock(st_tree *x, st_tree *y) : a(x), b(y) {
        st_tree *lo = x < y ? x : y, *hi = x < y ? y : x;
        l1 = std::unique_lock<std::recursive_mutex>(lo->mu);
        if (hi != lo) l2 = std::unique_lock<std::recursive_mutex>(hi->mu);
    }
    PairLock(const PairLock &) = delete;
    ~PairLock() {
        if (a != b && a->reads_remote) (void)tsync(a);
    }
};
#define ENTER_PAIR(x, y)                                                             \
    if (!(x) || !(y)) { g_err = "NULL tree"; return ST_EINVAL; }                     \
    PairLock enter_pl_(x, y);                                                        \
    CHK(use_device(x));                                                              \
    CHK(alive(x));                                                                   \
    CHK(alive(y))

// Every tree of a group call, locked in address order (duplicates once).
struct GroupLock {
    std::vector<std::unique_lock<std::recursive_mutex>> ls;
    GroupLock(st_tree **trees, uint32_t n) {
        std::vector<st_tree *> v(trees, trees + n);
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
        for (st_tree *u : v)
            if (u) ls.emplace_back(u->mu);
    }
};

// Stream-ordered scratch buffers freed when the scope ends, on every return
// path (error returns from LAUNCH / HIPCHK / CHK included).  release() hands a
// buffer over to the caller (e.g. a new CSR swapped into the tree).
struct Scratch {
    st_tree *t;
    std::vector<void *> ps;
    explicit Scratch(st_tree *t_) : t(t_) {}
    Scratch(const Scratch &) = delete;
    ~Scratch() {
        for (void *p : ps) dfree(t, p);
    }
    template <typename T>
    int alloc(T **p, uint64_t count) {
        int r = dalloc(t, (void **)p, count * sizeof(T));
        if (r == ST_OK) ps.push_back((void *)*p);
        return r;
    }
    int bytes(uint8_t **p, uint64_t n) { return alloc(p, n); }
    void release(void *p) {
        for (auto &q : ps)
            if (q == p) q = nullptr;
    }
};

// ------------------------------------------------------------------ CSR buffers
// A merge writes a whole new CSR.  Allocating (and first touching) GBs of
// fresh pool memory per batch costs milliseconds at 100M keys, so the CSR a
// merge retires is kept as the spare set and becomes the next merge's output
// (grown with 1/4 headroom when too small).  Small trees (< 16 MB of CSR)
// keep no spare.
static const uint64_t CSR_KEEP_SPARE = 16ull << 20;

static void csr_free(st_tree *t, CsrSet &c) {
    for (void *p : {(void *)c.seg_off, (void *)c.seg_voff, (void *)c.koff, (void *)c.voff, (void *)c.kheap, (void *)c.vheap})
        dfree(t, p);
    c = CsrSet();
}

// Output buffers for a CSR of n1 offsets (n entries + 1) and kb / vb heap
// bytes: the spare set, grown where too small.  On failure the spare keeps
// what it has.
static int csr_take(st_tree *t, uint64_t n1, uint64_t kb, uint64_t vb, CsrSet &o) {
    CsrSet &sp = t->spare;
    if (!sp.seg_off) CHK(dalloc_t(t, &sp.seg_off, t->S + 1));
    if (!sp.seg_voff) CHK(dalloc_t(t, &sp.seg_voff, t->S + 1));
    if (sp.cap_n < n1 || !sp.koff || !sp.voff) {
        dfree(t, sp.koff); dfree(t, sp.voff);
        sp.koff = sp.voff = nullptr;
        sp.cap_n = 0;
        const uint64_t want = n1 + n1 / 4;
        CHK(dalloc_t(t, &sp.koff, want));
        CHK(dalloc_t(t, &sp.voff, want));
        sp.cap_n = want;
    }
    if (sp.cap_k < kb || !sp.kheap) {
        dfree(t, sp.kheap);
        sp.kheap = nullptr;
        sp.cap_k = 0;
        CHK(dalloc(t, (void **)&sp.kheap, kb + kb / 4));
        sp.cap_k = kb + kb / 4;
    }
    if (sp.cap_v < vb || !sp.vheap) {
        dfree(t, sp.vheap);
        sp.vheap = nullptr;
        sp.cap_v = 0;
        CHK(dalloc(t, (void **)&sp.vheap, vb + vb / 4));
        sp.cap_v = vb + vb / 4;
    }
    o = sp;
    sp = CsrSet();
    return ST_OK;
}

// Make o the tree's CSR; the retired one becomes the spare set.
static void csr_install(st_tree *t, const CsrSet &o) {
    CsrSet old;
    old.seg_off = t->seg_off; old.seg_voff = t->seg_voff; old.koff = t->koff; old.voff = t->voff;
    old.kheap = t->kheap; old.vheap = t->vheap;
    old.cap_n = t->cap_n; old.cap_k = t->cap_k; old.cap_v = t->cap_v;
    csr_free(t, t->spare);
    if (old.cap_n * 16 + old.cap_k + old.cap_v >= CSR_KEEP_SPARE) t->spare = old; else csr_free(t, old);
    t->seg_off = o.seg_off; t->seg_voff = o.seg_voff; t->koff = o.koff; t->voff = o.voff;
    t->kheap = o.kheap; t->vheap = o.vheap;
    t->cap_n = o.cap_n; t->cap_k = o.cap_k; t->cap_v = o.cap_v;
}

// A taken set goes back to the spare slot unless installed.
struct CsrTaken {
    st_tree *t;
    CsrSet o;
    bool installed = false;
    explicit CsrTaken(st_tree *t_) : t(t_) {}
    CsrTaken(const CsrTaken &) = delete;
    ~CsrTaken() {
        if (installed) return;
        csr_free(t, t->spare);
        t->spare = o;
    }
    void install() { csr_install(t, o); installed = true; }
};

// The tree as kernels see it: the canonical CSR, or the paged layout while
// streaming batches are in it (pages.h).
static DevTree view(const st_tree *t) {
    DevTree d;
    memset(&d, 0, sizeof(d));
    d.W = (uint32_t)t->W;
    d.shift = t->shift;
    d.H = t->H;
    d.flags = t->flags;
    d.S = t->S;
    for (int i = 0; i < ST_MAXLEV + 2; i++) d.base[i] = t->base[i];
    d.md5 = gp(t->md5);
    d.tag = gp(t->tag);
    if (t->pg.on) {
        d.seg_off = gp(t->pg.m.beg);
        d.seg_end = gp(t->pg.m.end);
        d.seg_voff = gp(t->pg.m.vbeg);
        d.seg_vend = gp(t->pg.m.vend);
        d.koff = gp(t->pg.koff);
        d.kheap = gp(t->pg.kheap);
        d.voff = gp(t->pg.voff);
        d.vheap = gp(t->pg.vheap);
        return d;
    }
    d.seg_off = gp(t->seg_off);
    d.seg_end = gp(t->seg_off + 1);
    d.seg_voff = gp(t->seg_voff);
    d.seg_vend = gp(t->seg_voff + 1);
    d.koff = gp(t->koff);
    d.kheap = gp(t->kheap);
    d.voff = gp(t->voff);
    d.vheap = gp(t->vheap);
    return d;
}

static uint32_t grid_for(uint64_t n, uint32_t block = 256, uint32_t cap = 16384) {
    uint64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (uint32_t)g;
}

struct TimedLaunch {
    st_tree *t;
    const char *name;
    hipEvent_t a = nullptr, b = nullptr;
    TimedLaunch(st_tree *t_, const char *n) : t(t_), name(n) {
        if (t->timing) {
            (void)hipEventCreate(&a);
            (void)hipEventCreate(&b);
            (void)hipEventRecord(a, t->stream);
        }
    }
    ~TimedLaunch() {
        if (t->timing) {
            (void)hipEventRecord(b, t->stream);
            t->pending.push_back({name, a, b});
        }
    }
};

// Every launch leaves work on the tree's stream that the call may not wait
// for: async_pending tells a launch on ANOTHER stream over this tree
// (k_small_multi) to synchronise it first; tsync clears it.
#define LAUNCH(t, name, kern, grid, block, shmem, ...)                            \
    do {                                                                          \
        TimedLaunch tl_(t, name);                                                 \
        (t)->async_pending = true;                                                \
        hipLaunchKernelGGL(kern, dim3(grid), dim3(block), shmem, (t)->stream, __VA_ARGS__); \
        hipError_t e_ = hipGetLastError();                                        \
        if (e_ != hipSuccess) {                                                   \
            g_err = std::string("launch ") + name + ": " + hipGetErrorString(e_); \
            return ST_EDEVICE;                                                    \
        }                                                                         \
    } while (0)

// Wait for a device-written flag in host-mapped memory (the kernel writes it
// after a system-scope fence, last): a spin of a few microseconds instead of
// a stream synchronisation call; after 5 ms fall back to the blocking sync
// (which also reports a faulted kernel).
static int wait_mapped(st_tree *t, volatile uint32_t *flag, uint32_t want = 0) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0;; i++) {
        // acquire: the reads of the results the kernel wrote before the flag
        // may not move above this load (a volatile read alone does not order
        // the plain reads that follow it).  want != 0: wait for that value
        // (a call's sequence number), else for any non-zero value.
        const uint32_t v = __atomic_load_n(const_cast<uint32_t *>(flag), __ATOMIC_ACQUIRE);
        if (want ? v == want : v != 0) return ST_OK;
        if ((i & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(5)) break;
        __builtin_ia32_pause();
    }
    CHK(tsync(t));
    return ST_OK;
}

static int use_device(st_tree *t) {
    HIPCHK(hipSetDevice(t->device));
    return ST_OK;
}

// Exclusive scan (reduce, scan the tile sums, scan the tiles): three plain
// launches with no inter-workgroup communication inside a kernel (it replaced
// a look-back scan while chasing the round-2 ingest defect, DESIGN.md §3.3;
// the issue is upstream of the scan: its INPUT is seen differently).
constexpr uint32_t SCAN_T = 256, SCAN_I = 16, SCAN_TILE = SCAN_T * SCAN_I;

template <typename T>
__device__ T block_exclusive(T v, T *sh, T *total) {   // sh: SCAN_T elements of LDS
    const uint32_t x = threadIdx.x;
    sh[x] = v;
    __syncthreads();
    for (uint32_t d = 1; d < SCAN_T; d <<= 1) {   // inclusive (Hillis-Steele)
        const T a = x >= d ? sh[x - d] : T(0);
        __syncthreads();
        if (x >= d) sh[x] = sh[x] + a;
        __syncthreads();
    }
    *total = sh[SCAN_T - 1];
    const T r = x ? sh[x - 1] : T(0);
    __syncthreads();
    return r;
}

#define SCAN_SHARED(T) \
    __shared__ __attribute__((aligned(16))) uint8_t sh_raw_[SCAN_T * sizeof(T)]; \
    T *sh = reinterpret_cast<T *>(sh_raw_)

template <typename T>
__global__ void __launch_bounds__(SCAN_T) k_scan_reduce(const T *in, uint64_t n, T *part) {
    SCAN_SHARED(T);
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
    T acc(0);
    for (uint32_t k = 0; k < SCAN_I; k++) {
        const uint64_t i = base + (uint64_t)k * SCAN_T + threadIdx.x;
        if (i < n) acc = acc + in[i];
    }
    T tot;
    (void)block_exclusive(acc, sh, &tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

template <typename T>
__global__ void __launch_bounds__(SCAN_T) k_scan_parts(T *part, uint64_t nb) {
    SCAN_SHARED(T);
    const uint64_t per = (nb + SCAN_T - 1) / SCAN_T, b0 = threadIdx.x * per;
    T acc(0);
    for (uint64_t b = b0; b < b0 + per && b < nb; b++) acc = acc + part[b];
    T tot;
    T off = block_exclusive(acc, sh, &tot);
    for (uint64_t b = b0; b < b0 + per && b < nb; b++) {
        const T v = part[b];
        part[b] = off;
        off = off + v;
    }
}

template <typename T>
__global__ void __launch_bounds__(SCAN_T) k_scan_tiles(const T *in, uint64_t n, const T *part, T *out) {
    SCAN_SHARED(T);
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_I;   // thread-contiguous items
    T acc(0);
    for (uint32_t k = 0; k < SCAN_I; k++)
        if (base + k < n) acc = acc + in[base + k];
    T tot;
    T off = block_exclusive(acc, sh, &tot);
    off = part[blockIdx.x] + off;
    for (uint32_t k = 0; k < SCAN_I; k++)
        if (base + k < n) {
            const T v = in[base + k];
            out[base + k] = off;
            off = off + v;
        }
}

template <typename T>
static int exclusive_scan(st_tree *t, const T *in, T *out, uint64_t n) {
    if (n == 0) return ST_OK;
    const uint64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    T *part = nullptr;
    CHK(dalloc_t(t, &part, nb));
    int r = ST_OK;
    hipLaunchKernelGGL(k_scan_reduce<T>, dim3((uint32_t)nb), dim3(SCAN_T), 0, t->stream, in, n, part);
    hipLaunchKernelGGL(k_scan_parts<T>, dim3(1), dim3(SCAN_T), 0, t->stream, part, nb);
    hipLaunchKernelGGL(k_scan_tiles<T>, dim3((uint32_t)nb), dim3(SCAN_T), 0, t->stream, in, n, (const T *)part, out);
    hipError_t e = hipGetLastError();
    dfree(t, part);
    if (e != hipSuccess) { g_err = std::string("scan launch: ") + hipGetErrorString(e); r = ST_EDEVICE; }
    if (r) return r;
    return ST_OK;
}

static int d2h(st_tree *t, void *dst, const void *src, uint64_t bytes) {
    if (!bytes) return ST_OK;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, t->stream));
    CHK(tsync(t));
    return ST_OK;
}
// the tree's pinned staging buffer, at least `bytes` (contents not kept)
static int rpin_reserve(st_tree *t, uint64_t bytes) {
    if (bytes <= t->rpin_cap) return ST_OK;
    uint64_t cap = t->rpin_cap ? t->rpin_cap : 65536;
    while (cap < bytes) cap *= 2;
    if (t->rpin) { CHK(tsync(t)); (void)hipHostFree(t->rpin); t->rpin = nullptr; t->rpin_cap = 0; }
    if (hipHostMalloc((void **)&t->rpin, cap, hipHostMallocDefault) != hipSuccess) {
        t->rpin = nullptr;
        g_err = "hipHostMalloc (staging) failed";
        return ST_ENOMEM;
    }
    t->rpin_cap = cap;
    return ST_OK;
}
static int h2d(st_tree *t, void *dst, const void *src, uint64_t bytes) {
    if (!bytes) return ST_OK;
    t->async_pending = true;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, t->stream));
    return ST_OK;
}

// Device buffers a caller hands in (or wants written) are produced / consumed
// by work on the caller's own stream: the tree's next work is ordered after
// everything enqueued on `producer` so far (an event, no host wait).  NULL is
// the device's null stream -- torch's default stream -- which the library's
// non-blocking streams are otherwise NOT ordered against.
static int order_after(st_tree *t, hipStream_t producer) {
    if (producer == t->stream) return ST_OK;
    if (!t->ev_order) HIPCHK(hipEventCreateWithFlags(&t->ev_order, hipEventDisableTiming));
    HIPCHK(hipEventRecord(t->ev_order, producer));
    HIPCHK(hipStreamWaitEvent(t->stream, t->ev_order, 0));
    t->async_pending = true;
    return ST_OK;
}
// (The consumer side needs no event: every call that writes caller memory
// returns after a host synchronisation of its stream.)

static uint32_t inner_block(const st_tree *t) { return 64; }
static size_t inner_shmem(const st_tree *t) { return (size_t)inner_block(t) * lane_region_bytes((uint32_t)t->W); }

// ------------------------------------------------------------------ lifecycle
extern "C" const char *st_last_error(void) { return g_err.c_str(); }

extern "C" int st_create(uint64_t width, uint64_t segments, int device, st_tree **out) {
    *out = nullptr;
    if (width < 2 || segments < 1) { g_err = "bad geometry"; return ST_EINVAL; }
    // compute_height / compute_shift (synctree.erl:270-284), same libm math
    const double hd = std::log((double)segments) / std::log((double)width);
    const uint64_t height = (uint64_t)std::trunc(hd);
    if ((uint64_t)std::trunc(std::pow((double)width, (double)height)) != segments) {
        g_err = "segments is not a power of width (case_clause)";
        return ST_EINVAL;
    }
    const double sd = std::log((double)width) / std::log(2.0);
    const uint64_t shift = (uint64_t)std::trunc(sd);
    if ((uint64_t)std::trunc(std::pow(2.0, (double)shift)) != width) {
        g_err = "width is not a power of 2 (case_clause)";
        return ST_EINVAL;
    }
    if (width > 64 || segments > (1ull << 31) || height + 1 > ST_MAXLEV) {
        g_err = "geometry outside the device domain (W <= 64, Segments <= 2^31)";
        return ST_EINVAL;
    }
    st_tree *t = new st_tree();
    t->device = device;
    t->W = width;
    t->S = segments;
    t->shift = (uint32_t)shift;
    t->H = (uint32_t)height;
    // slot 0: #tree.top_hash; levels 1..H+1
    t->base[0] = 0;
    t->base[1] = 1;
    uint64_t sz = 1;
    for (uint32_t l = 1; l <= t->H + 1; l++) {
        t->base[l + 1] = t->base[l] + sz;
        sz *= width;
    }
    for (uint32_t l = t->H + 3; l < ST_MAXLEV + 2; l++) t->base[l] = t->base[t->H + 2];
    t->nslots = t->base[t->H + 2];
    int r = ST_OK;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&t->own_stream, hipStreamNonBlocking) != hipSuccess) {
        g_err = "hipSetDevice/hipStreamCreate failed";
        delete t;
        return ST_EDEVICE;
    }
    t->stream = t->own_stream;
    if (hipDeviceGetAttribute(&t->ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || t->ncu <= 0)
        t->ncu = 256;
    if (hipHostMalloc((void **)&t->pin, 64 * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess) {
        g_err = "hipHostMalloc failed";
        t->pin = nullptr;
        st_destroy(t);
        return ST_EDEVICE;
    }
    // the device-error word: fine-grained host memory the kernels store into
    if (hipHostMalloc((void **)&t->derr, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void **)&t->derr_dev, t->derr, 0) != hipSuccess) {
        g_err = "hipHostMalloc (mapped) failed";
        st_destroy(t);
        return ST_EDEVICE;
    }
    memset(t->derr, 0, 64);
    if ((r = dalloc_t(t, &t->md5, t->nslots)) || (r = dalloc_t(t, &t->tag, t->nslots)) ||
        (r = dalloc_t(t, &t->mark, t->nslots)) || (r = dalloc_t(t, &t->ok, t->nslots)) ||
        (r = dalloc_t(t, &t->flag, 4)) || (r = dalloc_t(t, &t->cnt64, 2)) ||
        (r = dalloc_t(t, &t->seg_off, t->S + 1)) || (r = dalloc_t(t, &t->seg_voff, t->S + 1)) ||
        (r = dalloc_t(t, &t->koff, 1)) || (r = dalloc_t(t, &t->voff, 1)) || (r = dalloc(t, (void **)&t->kheap, HEAP_SLACK)) ||
        (r = dalloc(t, (void **)&t->vheap, HEAP_SLACK)) || (r = dalloc_t(t, &t->seg_perm, t->S))) {
        st_destroy(t);
        return r;
    }
    (void)hipMemsetAsync(t->md5, 0, t->nslots * sizeof(uint4), t->stream);
    (void)hipMemsetAsync(t->tag, 0, t->nslots * sizeof(uint16_t), t->stream);
    (void)hipMemsetAsync(t->seg_off, 0, (t->S + 1) * 8, t->stream);
    (void)hipMemsetAsync(t->seg_voff, 0, (t->S + 1) * 8, t->stream);
    (void)hipMemsetAsync(t->koff, 0, 8, t->stream);
    (void)hipMemsetAsync(t->voff, 0, 8, t->stream);
    (void)hipMemsetAsync(t->kheap, 0, HEAP_SLACK, t->stream);
    (void)hipMemsetAsync(t->vheap, 0, HEAP_SLACK, t->stream);
    if (hipStreamSynchronize(t->stream) != hipSuccess) {
        g_err = "init failed";
        st_destroy(t);
        return ST_EDEVICE;
    }
    *out = t;
    return ST_OK;
}

static void pages_free(st_tree *t, Pages &g);
extern "C" void st_destroy(st_tree *t) {
    if (!t) return;
    // wait for a call still running on the handle (a caller must not use it
    // after destroy; this only orders destroy after calls already inside)
    { std::lock_guard<std::recursive_mutex> g(t->mu); }
    (void)hipSetDevice(t->device);
    if (t->stream) (void)hipStreamSynchronize(t->stream);   // nothing of this tree is pending after this
    void *ps[] = {t->erec, t->md5, t->tag, t->mark, t->ok, t->flag, t->cnt64, t->seg_off, t->seg_voff, t->koff, t->voff, t->kheap, t->vheap,
                  t->seg_perm, t->tiles, t->tseg, t->tln, t->tinfo, t->tpres, t->tnoff, t->tmhmax, t->lvl_cnt, t->cw.wcnt, t->cw.wbytes, t->cw.werr,
                  t->cw.wst, t->cw.rec, t->cw.scratch, t->mail};
    for (void *p : ps) dfree(t, p);
    for (void *p : {(void *)t->spare.seg_off, (void *)t->spare.seg_voff, (void *)t->spare.koff, (void *)t->spare.voff,
                    (void *)t->spare.kheap, (void *)t->spare.vheap})
        dfree(t, p);
    pages_free(t, t->pg);
    dfree(t, t->ov.idx);
    dfree(t, t->ov.heap);
    dfree(t, t->ov.used);
    if (t->pin) (void)hipHostFree(t->pin);
    if (t->rpin) (void)hipHostFree(t->rpin);
    if (t->derr) (void)hipHostFree(t->derr);
    if (t->sout) (void)hipHostFree(t->sout);
    if (t->sreq) (void)hipHostFree(t->sreq);
    if (t->cw.res) (void)hipHostFree(t->cw.res);
    if (t->ev_order) (void)hipEventDestroy(t->ev_order);
    for (auto &p : t->pending) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
    mem_forget_owner(t);   // the stream was idle: the blocks freed above have no pending use
    if (t->own_stream) (void)hipStreamDestroy(t->own_stream);
    delete t;
}

extern "C" int st_set_stream(st_tree *t, void *s) {
    ENTER_ANY(t);
    CHK(tsync(t));
    t->stream = s ? (hipStream_t)s : t->own_stream;
    return ST_OK;
}

extern "C" int st_sync(st_tree *t) {
    ENTER_ANY(t);
    CHK(tsync(t));
    return ST_OK;
}

extern "C" uint32_t st_height(const st_tree *t) { return t->H; }   // geometry: immutable after st_create
extern "C" uint64_t st_width(const st_tree *t) { return t->W; }
extern "C" uint64_t st_segments(const st_tree *t) { return t->S; }
extern "C" uint64_t st_num_entries(st_tree *t) {
    std::lock_guard<std::recursive_mutex> g(t->mu);
    return t->n;
}

static int pages_fold(st_tree *t);
extern "C" int st_debug_knob(st_tree *t, int knob, int64_t value) {
    ENTER_ANY(t);
    if (knob == ST_DBG_SKIP_MAIL) {
        t->dbg_skip_mail = value < 0 ? ~0u : (uint32_t)value;
        return ST_OK;
    }
    if (knob == ST_DBG_PAGES) {
        if (value < 0) CHK(pages_fold(t));   // pages off: streaming batches merge into the CSR
        t->pg_slack = value < 0 ? -1 : value == 0 ? 25 : (int)std::min<int64_t>(value, 400);
        if (value >= 0) t->pg_streak = std::max<uint32_t>(t->pg_streak, 1);   // pages from the next streaming batch
        return ST_OK;
    }
    if (knob == ST_DBG_PAGE_CHECK) {
        t->pg_check = value != 0;
        return ST_OK;
    }
    if (knob == ST_DBG_PAGE_DOWN) {
        if (value < 0 || value > 2) { g_err = "ST_DBG_PAGE_DOWN takes 0, 1 or 2"; return ST_EINVAL; }
        t->pg_down = (int)value;
        return ST_OK;
    }
    if (knob == ST_DBG_PAGE_POISON) {   // a page whose entries leave its capacity (the checked mode must refuse it)
        if (!t->pg.on || value < 0 || (uint64_t)value >= t->S) { g_err = "no pages / segment out of range"; return ST_EINVAL; }
        LAUNCH(t, "page_poison", k_page_poison, 1, 64, 0, t->pg.m, (uint64_t)value);
        CHK(tsync(t));
        return ST_OK;
    }
    g_err = "unknown debug knob";
    return ST_EINVAL;
}

extern "C" int st_page_stats(st_tree *t, uint64_t out[6]) {
    ENTER_ANY(t);
    out[0] = t->pg.on ? 1 : 0;
    out[1] = t->pg.batches;
    out[2] = t->pg.builds;
    out[3] = t->pg.folds;
    out[4] = t->pg.reloc_e;
    out[5] = t->pg.touched_v;
    return ST_OK;
}

static uint64_t num_tiles(const st_tree *t);
extern "C" int st_mem_stats(st_tree *t, uint64_t out[6]) {
    ENTER_ANY(t);
    out[0] = t->nslots * (sizeof(uint4) + sizeof(uint16_t) + 2);   // md5, tag, mark, ok
    out[1] = (t->S + 1) * 16 + t->cap_n * 16 + t->cap_k + t->cap_v;
    out[2] = t->tiles_cap * sizeof(uint4) + (t->tseg ? num_tiles(t) * (64 * 8 + sizeof(TileInfo)) : 0);
    out[3] = (t->spare.koff ? (t->S + 1) * 16 + t->spare.cap_n * 16 + t->spare.cap_k + t->spare.cap_v : 0) +
             (t->pg.koff ? t->S * 56 + t->pg.cap_e * 16 + t->pg.cap_k + t->pg.cap_v : 0);
    out[4] = t->ov.idx ? t->S * 8 + t->ov.cap : 0;
    std::lock_guard<std::mutex> g(g_mem_mu);
    uint64_t c = 0;
    for (auto &kv : g_mem_free) c += kv.first;
    out[5] = c;
    return ST_OK;
}

extern "C" int st_set_timing(st_tree *t, int enabled) {
    ENTER_ANY(t);
    t->timing = enabled != 0;
    return ST_OK;
}

extern "C" int st_kernel_stats(st_tree *t, const char *kernel, uint64_t *launches, double *total_ms) {
    ENTER_ANY(t);
    CHK(tsync(t));
    for (auto &p : t->pending) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, p.a, p.b);
        auto &s = t->stats[p.name];
        s.first += 1;
        s.second += ms;
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    t->pending.clear();
    auto it = t->stats.find(kernel ? kernel : "");
    if (kernel && std::string(kernel) == "*reset*") {
        t->stats.clear();
        return ST_OK;
    }
    *launches = it == t->stats.end() ? 0 : it->second.first;
    *total_ms = it == t->stats.end() ? 0.0 : it->second.second;
    return ST_OK;
}

// ------------------------------------------------------------------ key records
// Host packing of (type, ensure_binary bytes) into device key records.
struct HostRecords {
    std::vector<uint8_t> heap;
    std::vector<uint64_t> off;
};

static int pack_records(uint64_t n, const uint8_t *ktype, const uint8_t *kheap, const uint64_t *koff, HostRecords &r) {
    r.off.resize(n + 1);
    r.heap.clear();
    r.heap.reserve((koff ? koff[n] : 0) + n + HEAP_SLACK);
    for (uint64_t i = 0; i < n; i++) {
        r.off[i] = r.heap.size();
        const uint8_t ty = ktype[i];
        const uint64_t len = koff[i + 1] - koff[i];
        const uint8_t *p = kheap + koff[i];
        if (ty == ST_KEY_INT) {
            if (len != 8) { g_err = "integer key must be 8 bytes (<<K:64>>)"; return ST_EINVAL; }
            r.heap.push_back(KEYTAG_INT);
            r.heap.push_back(p[0] ^ 0x80);
            r.heap.insert(r.heap.end(), p + 1, p + 8);
        } else if (ty == ST_KEY_ATOM || ty == ST_KEY_BINARY) {
            r.heap.push_back(ty == ST_KEY_ATOM ? KEYTAG_ATOM : KEYTAG_BINARY);
            r.heap.insert(r.heap.end(), p, p + len);
        } else if (ty == ST_KEY_TERM) {
            const std::string e = termkey::record_from_etf(p, len, r.heap);
            if (!e.empty()) { g_err = "key " + std::to_string(i) + ": " + e; return ST_EINVAL; }
        } else {
            g_err = "unknown key type";
            return ST_EINVAL;
        }
    }
    r.off[n] = r.heap.size();
    r.heap.resize(r.heap.size() + HEAP_SLACK, 0);
    return ST_OK;
}

static int host_rec_cmp(const uint8_t *a, uint64_t la, const uint8_t *b, uint64_t lb) {
    la = krec_order_len(a, la);
    lb = krec_order_len(b, lb);
    uint64_t m = la < lb ? la : lb;
    int c = m ? memcmp(a, b, m) : 0;
    if (c) return c < 0 ? -1 : 1;
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

// ------------------------------------------------------------------ rehash pieces
static int rehash_levels(st_tree *t, uint32_t top_level, const uint8_t *mask) {
    DevTree d = view(t);
    for (uint32_t l = top_level; l >= 1; l--) {
        const uint64_t nodes = t->base[l + 1] - t->base[l];
        LAUNCH(t, "level_rehash", (k_level_hash<MODE_STORE>), grid_for(nodes, inner_block(t)), inner_block(t),
               inner_shmem(t), d, l, l, mask, (const uint32_t *)nullptr, (const uint32_t *)nullptr, (uint8_t *)nullptr,
               (uint32_t *)nullptr);
    }
    return ST_OK;
}

// seg_perm: segments by MD5 block count (descending), the K1 order.
static int ensure_perm(st_tree *t) {
    if (t->perm_valid) return ST_OK;
    DevTree d = view(t);
    Scratch sc(t);
    uint32_t *cnt = nullptr;
    CHK(sc.alloc(&cnt, PERM_BINS));
    HIPCHK(hipMemsetAsync(cnt, 0, PERM_BINS * 4, t->stream));
    LAUNCH(t, "seg_perm", k_seg_perm_count, grid_for(t->S, 256, 1024), 256, 0, d, cnt);
    LAUNCH(t, "seg_perm", k_seg_perm_scan, 1, 256, 0, cnt);
    LAUNCH(t, "seg_perm", k_seg_perm_scatter, grid_for(t->S, 256, 1024), 256, 0, d, cnt, t->seg_perm);
    t->perm_valid = true;
    t->perm_any = true;
    return ST_OK;
}
// Any permutation of the segments will do (the order only balances a wave's
// lanes): the streaming batches reuse the last one instead of re-sorting.
static int ensure_perm_any(st_tree *t) {
    if (t->perm_any) return ST_OK;
    return ensure_perm(t);
}

// Build the hash-ready tiled messages from the CSR (k_tile_order, scan,
// k_tile_fill).  Called at the end of every ingest and lazily by rehash.
static uint64_t num_tiles(const st_tree *t) { return (t->S + 63) / 64; }

// Build the hash-ready tiled messages from the CSR in seg_perm order
// (k_tile_order_global, scan, k_tile_fill).  Called at the end of every bulk
// ingest and lazily by rehash.
// the fused kernel's last window hashes the upper levels a thread per node:
// at most 256 nodes at level H-3 (H <= 6)
static bool fused_geometry(const st_tree *t) { return t->W == 16 && t->H >= 3 && t->H <= 6; }

// Level-H message bytes of the fused rehash's LDS: the largest window's
// packed messages, and room for the climb's nodes (nwin / 16 of them, one
// RW_MSG each) in the tree's last window.
static uint32_t fused_mh_bytes(uint32_t mh, uint64_t nwin) {
    const uint64_t climb = (nwin / 16) * RW_MSG;
    return (uint32_t)std::max<uint64_t>(std::max<uint64_t>(mh, climb), 64);
}

static int ensure_tiles(st_tree *t) {
    if (t->tiles_valid) return ST_OK;
    if (!fused_geometry(t)) CHK(ensure_perm(t));
    const uint64_t ntiles = num_tiles(t);
    if (!t->tseg) {
        CHK(dalloc_t(t, &t->tseg, ntiles * 64));
        CHK(dalloc_t(t, &t->tln, ntiles * 64));
        CHK(dalloc_t(t, &t->tinfo, ntiles));
    }
    if (fused_geometry(t) && !t->tpres) {
        CHK(dalloc_t(t, &t->tpres, t->S / 64));
        CHK(dalloc_t(t, &t->tnoff, t->S / 16));
        CHK(dalloc_t(t, &t->tmhmax, 4));
    }
    if (fused_geometry(t)) HIPCHK(hipMemsetAsync(t->tmhmax, 0, 4, t->stream));
    Scratch sc(t);
    uint64_t *tsize = nullptr, *tbase = nullptr;
    CHK(sc.alloc(&tsize, ntiles + 1));
    CHK(sc.alloc(&tbase, ntiles + 1));
    HIPCHK(hipMemsetAsync(tsize + ntiles, 0, 8, t->stream));
    if (fused_geometry(t))   // window-local order (k_rehash_fused)
        LAUNCH(t, "tile_build", k_tile_order_window, (uint32_t)(t->S / 4096), 256, 0, view(t), t->tseg, t->tln, t->tinfo,
               tsize, t->tpres, t->tnoff, t->tmhmax);
    else
        LAUNCH(t, "tile_build", k_tile_order_global, grid_for(ntiles * 64, 256, 1u << 30), 256, 0, view(t),
               (const uint32_t *)t->seg_perm, t->tseg, t->tln, t->tinfo, tsize, ntiles);
    CHK(exclusive_scan<uint64_t>(t, tsize, tbase, ntiles + 1));
    uint64_t total = 0;
    HIPCHK(hipMemcpyAsync(&total, tbase + ntiles, 8, hipMemcpyDeviceToHost, t->stream));
    uint32_t mh = 0;
    if (fused_geometry(t)) HIPCHK(hipMemcpyAsync(&mh, t->tmhmax, 4, hipMemcpyDeviceToHost, t->stream));
    CHK(tsync(t));
    t->mh_bytes = mh;
    if (total + 1 > t->tiles_cap) {
        dfree(t, t->tiles);
        t->tiles = nullptr;
        t->tiles_cap = 0;
        const uint64_t cap = total + total / 8 + 256;   // slack: a tile of zero stored rows still issues row-0 loads
        CHK(dalloc_t(t, &t->tiles, cap));
        t->tiles_cap = cap;
    }
    LAUNCH(t, "tile_build", k_tile_info, grid_for(ntiles), 256, 0, (const uint64_t *)tbase, ntiles, t->tinfo);
    LAUNCH(t, "tile_build", k_tile_fill, (uint32_t)ntiles, 256, 0, (const uint64_t *)t->seg_voff, (const uint8_t *)t->vheap,
           (const uint32_t *)t->tseg, (const uint32_t *)t->tln, (const TileInfo *)t->tinfo, t->tiles);
    t->tiles_valid = true;
    return ST_OK;
}

static TreeTiles tree_tiles(const st_tree *t) {
    TreeTiles x;
    x.md5 = t->md5;
    x.tag = t->tag;
    x.cnt = t->lvl_cnt;
    x.mail = t->mail;
    x.tinfo = t->tinfo;
    x.tseg = t->tseg;
    x.tln = t->tln;
    x.tiles = t->tiles;
    x.pres = t->tpres;
    x.noff = t->tnoff;
    x.err = t->derr_dev;
    x.epoch = t->mail_epoch;
    x.skip_root = t->dbg_skip_mail;
    return x;
}
// A fused launch's mailbox epoch for tree t: 1..65535, never the epoch of
// the tree's previous launch (whose words its mailboxes still hold).
static TreeTiles launch_tiles(st_tree *t) {
    t->mail_epoch = t->mail_epoch % 65535u + 1u;
    return tree_tiles(t);
}

static int ensure_lvl_cnt(st_tree *t) {
    if (t->lvl_cnt || t->H < 3) return ST_OK;
    CHK(dalloc_t(t, &t->mail, t->base[t->H - 1]));
    HIPCHK(hipMemsetAsync(t->mail, 0, t->base[t->H - 1] * sizeof(MailEntry), t->stream));   // epoch 0: never a launch's
    CHK(dalloc_t(t, &t->lvl_cnt, t->base[t->H - 2]));
    HIPCHK(hipMemsetAsync(t->lvl_cnt, 0, t->base[t->H - 2] * 4, t->stream));
    return ST_OK;
}

static int ensure_erec(st_tree *t) {
    if (t->erec) return ST_OK;
    CHK(dalloc_t(t, &t->erec, t->nslots));
    HIPCHK(hipMemsetAsync(t->erec, 0, t->nslots, t->stream));
    return ST_OK;
}

static int set_erec(st_tree *t, uint64_t slot, uint8_t v) {
    if (!t->erec && !v) return ST_OK;
    CHK(ensure_erec(t));
    HIPCHK(hipMemsetAsync(t->erec + slot, v, 1, t->stream));
    return ST_OK;
}

// rehash/1 deletes every empty inner node (delete_existing_batch,
// synctree.erl:529-531) but keeps a stored [] segment (its final level only
// fetches, :510-513)
static int erec_after_rehash(st_tree *t) {
    if (t->erec && t->H >= 1) HIPCHK(hipMemsetAsync(t->erec + 1, 0, t->base[t->H + 1] - 1, t->stream));
    return ST_OK;
}

// Inner levels of a W == 16 tree from level `top` down to 1 (dirty path:
// only marked nodes) with the per-level kernels: k_level16 while a level is
// wider than 256 nodes, then k_upper16 for the rest in one workgroup.
static int levels16(st_tree *t, uint32_t top, const uint8_t *mask) {
    DevTree d = view(t);
    uint32_t l = top;
    for (; l >= 1 && t->base[l + 1] - t->base[l] > 256; l--)
        LAUNCH(t, "level_rehash", k_level16, grid_for(t->base[l + 1] - t->base[l], 64), 64,
               (size_t)64 * lane_region_bytes(16), d, l, mask);
    if (l >= 1)
        LAUNCH(t, "level_rehash", k_upper16, 1, 256, (size_t)256 * lane_region_bytes(16), d, 1u, l, mask);
    return ST_OK;
}

// ST_LEVEL_STAMPS=1: the fused rehash's per-window phase stamps (100 MHz
// wall clock + shader cycles, 32 words a window) summarised to stderr.
static void fused_stamps_report(const std::vector<uint64_t> &h, uint32_t nwg) {
    uint64_t t0 = ~0ull;
    for (uint32_t w = 0; w < nwg; w++) t0 = std::min(t0, h[w * 32]);
    if (const char *dump = getenv("ST_STAMP_DUMP")) {   // raw per-window stamps (ticks from t0)
        if (FILE *f = fopen(dump, "a")) {
            for (uint32_t w = 0; w < nwg; w++) {
                for (int k = 0; k < 16; k++) fprintf(f, "%lld ", h[w * 32 + k] ? (long long)(h[w * 32 + k] - t0) : -1ll);
                fprintf(f, "\n");
            }
            fclose(f);
        }
    }
    static const char *names[16] = {"start", "K1 done", "H hashed", "H barrier", "H-1 hashed", "H-1 barrier",
                                    "H-2 hashed", "mail stored", "cnt won", "mail read", "climb 1st hashed",
                                    "-", "-", "-", "climb last hashed", "exit"};
    for (int k = 0; k < 16; k++) {
        std::vector<double> v;
        for (uint32_t w = 0; w < nwg; w++) if (h[w * 32 + k]) v.push_back((h[w * 32 + k] - t0) / 100.0);
        if (v.empty()) continue;
        std::sort(v.begin(), v.end());
        fprintf(stderr, "fused stamp %d %-15s n=%4zu min %7.2f med %7.2f max %7.2f us\n", k, names[k], v.size(), v[0],
                v[v.size() / 2], v.back());
    }
    // shader cycles and clock (s_memtime / s_memrealtime) over the hash intervals
    const int iv[5][2] = {{1, 2}, {3, 4}, {5, 6}, {9, 10}, {10, 14}};
    for (auto &q : iv) {
        double cyc = 0, us = 0;
        int m = 0;
        for (uint32_t w = 0; w < nwg; w++) {
            const uint64_t *r = &h[w * 32];
            if (!r[q[0]] || !r[q[1]]) continue;
            cyc += (double)(r[16 + q[1]] - r[16 + q[0]]);
            us += (r[q[1]] - r[q[0]]) / 100.0;
            m++;
        }
        if (m) fprintf(stderr, "fused cycles %s -> %s: %.0f cycles, %.2f us, %.2f GHz (n=%d)\n", names[q[0]], names[q[1]],
                       cyc / m, us / m, cyc / us / 1e3, m);
    }
    for (int k = 1; k < 16; k++) {   // each phase from its window's own start (a group's windows start over the launch)
        std::vector<double> dur;
        for (uint32_t w = 0; w < nwg; w++)
            if (h[w * 32] && h[w * 32 + k]) dur.push_back((h[w * 32 + k] - h[w * 32]) / 100.0);
        if (dur.empty()) continue;
        std::sort(dur.begin(), dur.end());
        fprintf(stderr, "fused from start %-17s n=%zu min %7.2f med %7.2f p90 %7.2f max %7.2f us\n", names[k], dur.size(),
                dur[0], dur[dur.size() / 2], dur[dur.size() * 9 / 10], dur.back());
    }
}

// Full rehash.  W == 16, H >= 3: ONE launch of k_rehash_fused, a workgroup
// per level-(H-2) window: K1 over the window's tiles, its levels H..H-2 from
// LDS, the levels above by last-arriving workgroups.  Other geometries: K1
// (k_segment_hash_tiled_p over globally ordered tiles), then the per-level
// kernels.
static int rehash_tiled(st_tree *t) {
    CHK(ensure_tiles(t));
    DevTree d = view(t);
    if (fused_geometry(t)) {
        CHK(ensure_lvl_cnt(t));
        // a partition hashes only its own windows (4096 segments each) and
        // stops at level 2; st_combine_upper finishes level 1 + top
        const uint64_t nroots = t->S / 4096;
        const uint64_t root0 = t->partitioned ? t->part_lo / 4096 : 0;
        const uint32_t nwg = t->partitioned ? (uint32_t)((t->part_hi - t->part_lo) / 4096) : (uint32_t)nroots;
        if (root0 + nwg > nroots || nwg == 0) { g_err = "rehash window range out of bounds"; return ST_EINVAL; }
        const uint32_t lmin = t->partitioned ? 2u : 1u;
        const uint32_t mhb = fused_mh_bytes(t->mh_bytes, nroots);
        static const int stamp = getenv("ST_LEVEL_STAMPS") ? atoi(getenv("ST_LEVEL_STAMPS")) : 0;
        if (!stamp) {
            LAUNCH(t, "rehash_fused", (k_rehash_fused<false, false, 16>), nwg, 1024, fused_lds_bytes(mhb), d, launch_tiles(t),
                   (const TreeTiles *)nullptr, 0u, root0, lmin, (uint64_t *)nullptr, mhb);
            return ST_OK;
        }
        // diagnostic: per-phase wall-clock stamps (100 MHz) to stderr
        Scratch sc(t);
        uint64_t *st = nullptr;
        CHK(sc.alloc(&st, (uint64_t)nwg * 32));
        HIPCHK(hipMemsetAsync(st, 0, (uint64_t)nwg * 32 * 8, t->stream));
        LAUNCH(t, "rehash_fused", (k_rehash_fused<true, false, 16>), nwg, 1024, fused_lds_bytes(mhb), d, launch_tiles(t),
               (const TreeTiles *)nullptr, 0u, root0, lmin, st, mhb);
        std::vector<uint64_t> h((uint64_t)nwg * 32);
        HIPCHK(hipMemcpyAsync(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost, t->stream));
        CHK(tsync(t));
        fused_stamps_report(h, nwg);
        return ST_OK;
    }
    const uint64_t ntl = num_tiles(t);
    LAUNCH(t, "segment_hash", k_segment_hash_tiled_p, (uint32_t)std::min<uint64_t>((ntl + 3) / 4, 1024u), 256, 0, d,
           tree_tiles(t), ntl);
    if (t->H == 0) return ST_OK;
    if (t->W == 16) return levels16(t, t->H, nullptr);
    return rehash_levels(t, t->H, nullptr);
}

// Full (mask == NULL) or dirty-path (mask: marked segments + ancestors) rehash.
// The dirty path hashes the marked segments straight from the CSR (or the
// pages) in block-count order (k_segment_hash_perm), then the marked inner
// nodes: W == 16, H >= 3: k_levels3_16 per level-(H-2) subtree + the
// per-level kernels above; other geometries: one k_level_hash launch per level.
// ps: the prefix states of a streaming batch's verify (k_verify_cap) or NULL.
// hb (a streaming batch's list, k_page_place): the changed segments in bins by blocks left.
// few (mask): so few segments are marked that ordering them by length costs
// more than it saves (the length permutation is stale after every merge):
// they are hashed in segment order.
static int rehash_all(st_tree *t, const uint8_t *mask, const PrefixState *ps = nullptr,
                      HashBins hb = HashBins{nullptr, nullptr, 0, 0, 0}, bool few = false) {
    if (!mask) {
        // The first full rehash after a mutation hashes straight from the
        // CSR (a lane per segment, no tile build: the repair path's
        // rehash/1, riak_ensemble_peer_tree.erl:264-277); the next one, the
        // tree unchanged since, builds the tiles for the fused kernel.
        if (t->tiles_valid || t->tiles_wanted || t->partitioned) return rehash_tiled(t);
        t->tiles_wanted = true;
        CHK(ensure_perm_any(t));
        LAUNCH(t, "segment_hash", k_segment_hash_perm, grid_for(t->S), 256, 0, view(t), (const uint32_t *)t->seg_perm,
               (const uint8_t *)nullptr, (const PrefixState *)nullptr, (const uint32_t *)nullptr);
    } else if (hb.list) {
        LAUNCH(t, "segment_hash", k_segment_hash_perm, grid_for(t->S), 256, 0, view(t), (const uint32_t *)nullptr, mask, ps,
               (const uint32_t *)nullptr, hb);
    } else if (few && !t->perm_valid) {
        LAUNCH(t, "segment_hash", k_segment_hash_perm, grid_for(t->S), 256, 0, view(t), (const uint32_t *)nullptr, mask, ps,
               (const uint32_t *)nullptr);
    } else {
        CHK(ensure_perm(t));
        LAUNCH(t, "segment_hash", k_segment_hash_perm, grid_for(t->S), 256, 0, view(t), (const uint32_t *)t->seg_perm, mask,
               ps, (const uint32_t *)nullptr);
    }
    if (t->H == 0) return ST_OK;
    // the inner levels (mask NULL: every node).  W == 16, H >= 3: levels
    // H..H-2 of each level-(H-2) subtree in one workgroup from LDS, then the
    // per-level kernels above
    const DevTree d = view(t);
    if (t->W == 16 && t->H >= 3) {
        LAUNCH(t, "level_rehash", k_levels3_16, (uint32_t)(t->base[t->H - 1] - t->base[t->H - 2]), 256, levels3_16_lds_bytes(),
               d, mask);
        if (t->H - 3 >= 1) CHK(levels16(t, t->H - 3, mask));
        return ST_OK;
    }
    if (t->W == 16) return levels16(t, t->H, mask);
    return rehash_levels(t, t->H, mask);
}

// Verify the inner nodes marked in t->mark (levels 1..min(L, H)); results in t->ok.
static int verify_levels(st_tree *t, uint32_t L) {
    DevTree d = view(t);
    const uint32_t lmax = L < t->H ? L : t->H;
    if (lmax >= 1) {
        const uint64_t nodes = t->base[lmax + 1] - t->base[1];
        LAUNCH(t, "level_verify", (k_level_hash<MODE_VERIFY>), grid_for(nodes, inner_block(t)), inner_block(t),
               inner_shmem(t), d, 1u, lmax, (const uint8_t *)t->mark, (const uint32_t *)nullptr,
               (const uint32_t *)nullptr, t->ok, (uint32_t *)nullptr);
    }
    return ST_OK;
}

// Verify every node marked in t->mark (levels 1..L); results in t->ok.
static int verify_marked(st_tree *t, uint32_t L) {
    DevTree d = view(t);
    if (L == t->H + 1) {   // segments in the length order of seg_perm: lanes of a wave hash alike-sized messages
        CHK(ensure_perm(t));
        LAUNCH(t, "segment_verify", (k_segment_hash<MODE_VERIFY>), grid_for(t->S), 256, 0, d, (const uint8_t *)t->mark,
               (const uint32_t *)t->seg_perm, (const uint32_t *)nullptr, t->ok, (uint32_t *)nullptr);
    }
    return verify_levels(t, L);
}

// ------------------------------------------------------------------ ingest
// Merge n device key records (+ values) into the tree.
//  seg_given: precomputed segment per record (raw segment store) or NULL
//  bop: per-record ERASE flags (device) or NULL
//  seg_replace: per-segment replace flags (device) or NULL
//  verify_rehash: insert semantics (path verification + dirty-path rehash)
//  clevel_out: per-record corruption level (device, n) or NULL
//  seg_out: per-record segment (device, n) or NULL
struct IngestIn {
    uint64_t n;
    const uint8_t *krec;
    const uint64_t *koff;
    const uint8_t *vheap;
    const uint64_t *voff;
    const uint32_t *seg_given;
    const uint8_t *bop;
    const uint8_t *seg_replace;
    bool verify_rehash;
    uint32_t *clevel_out;
    uint32_t *seg_out;
    uint64_t n_rejected;
    bool int9;               // every record an int64 key (insert_int64's packing: record i at krec + 9 i)
    bool count_rejected;     // the caller wants clevel_out's nonzero count ...
    bool rejected_counted;   // ... and the paged path counted it with its totals (n_rejected)
};

// The batch in merge order: segment per record (seg), sorted segments
// (sseg), sorted record order (perm), run bounds per segment (bseg_off), and
// the last writer of every key (keep).
struct BatchPrep {
    uint32_t *seg = nullptr, *sseg = nullptr, *perm = nullptr;
    uint64_t *bseg_off = nullptr;
    uint8_t *keep = nullptr;
};

// zero (optional): more buffers the caller needs zeroed, cleared by the same
// launch as the histogram's counters
static int batch_prepare(st_tree *t, IngestIn &in, Scratch &sc, BatchPrep &bp, const ZeroSpans *zero = nullptr) {
    const uint64_t n = in.n, S = t->S;
    CHK(sc.alloc(&bp.keep, n));
    CHK(sc.alloc(&bp.seg, n));
    CHK(sc.alloc(&bp.sseg, n));
    CHK(sc.alloc(&bp.perm, n));
    CHK(sc.alloc(&bp.bseg_off, S + 1));
    // bucket by segment: histogram + ranks (with the key's segment), scan (=
    // the runs' bounds), scatter
    unsigned long long *cnt = nullptr;
    uint32_t *rank = nullptr;
    CHK(sc.alloc(&cnt, S + 1));
    CHK(sc.alloc(&rank, n));
    {
        ZeroSpans z{};
        if (zero) z = *zero;
        z.p[z.k] = reinterpret_cast<uint8_t *>(cnt);
        z.n[z.k++] = (S + 1) * 8;
        LAUNCH(t, "bucket", k_zero_spans, grid_for((S + 1) / 2), 256, 0, z);
    }
    if (in.seg_given) {
        HIPCHK(hipMemcpyAsync(bp.seg, in.seg_given, n * 4, hipMemcpyDeviceToDevice, t->stream));
        LAUNCH(t, "bucket", k_seg_hist, grid_for(n), 256, 0, (const uint32_t *)bp.seg, n, cnt, rank);
    } else {
        LAUNCH(t, "key_segment", k_key_segment, grid_for(n), 256, 0, in.krec, in.koff, n, S - 1, bp.seg, cnt, rank);
    }
    if (in.seg_out) HIPCHK(hipMemcpyAsync(in.seg_out, bp.seg, n * 4, hipMemcpyDeviceToDevice, t->stream));
    CHK(exclusive_scan<uint64_t>(t, reinterpret_cast<const uint64_t *>(cnt), bp.bseg_off, S + 1));
    LAUNCH(t, "bucket", k_seg_scatter, grid_for(n), 256, 0, (const uint32_t *)bp.seg, (const uint32_t *)rank, n,
           (const uint64_t *)bp.bseg_off, bp.sseg, bp.perm);
    if (t->partitioned)
        LAUNCH(t, "clamp_runs", k_clamp_runs, grid_for(S + 1), 256, 0, bp.bseg_off, S, t->part_lo, t->part_hi);
    BatchView bv{in.krec, in.koff, in.int9};
    LAUNCH(t, "run_sort", k_run_sort, grid_for(S), 256, 0, bv, bp.perm, (const uint64_t *)bp.bseg_off, S, bp.keep);
    return ST_OK;
}

// Path verification of the touched segments (insert semantics): rejects[S]
// = first failing level of each touched segment's root->segment path.
static int verify_batch_paths(st_tree *t, const BatchPrep &bp, Scratch &sc, uint8_t **reject) {
    const uint64_t S = t->S;
    CHK(sc.alloc(reject, S));
    if (t->fresh) {
        HIPCHK(hipMemsetAsync(*reject, 0, S, t->stream));
        return ST_OK;
    }
    DevTree d = view(t);
    HIPCHK(hipMemsetAsync(t->mark, 0, t->nslots, t->stream));
    LAUNCH(t, "mark_paths", k_mark_paths, grid_for(S), 256, 0, d, t->H + 1, (const uint64_t *)bp.bseg_off,
           (const uint64_t *)nullptr, S, t->mark);
    CHK(verify_marked(t, t->H + 1));
    LAUNCH(t, "path_status", k_path_status, grid_for(S), 256, 0, d, t->H + 1, (const uint64_t *)bp.bseg_off,
           (const uint64_t *)nullptr, S, (const uint8_t *)t->ok, *reject, (uint32_t *)nullptr);
    return ST_OK;
}

static MergeArgs merge_args(const st_tree *t, const DevTree &d, const IngestIn &in, const BatchPrep &bp, const uint8_t *reject,
                            uint64_t S) {
    MergeArgs ma;
    ma.seg_off = d.seg_off;
    ma.seg_end = d.seg_end;
    ma.koff = d.koff;
    ma.kheap = d.kheap;
    ma.voff = d.voff;
    ma.vheap = d.vheap;
    ma.perm = bp.perm;
    ma.bseg_off = bp.bseg_off;
    ma.keep = bp.keep;
    ma.bop = in.bop;
    ma.seg_reject = reject;
    ma.seg_replace = in.seg_replace;
    ma.bv = BatchView{in.krec, in.koff, in.int9};
    ma.bvoff = in.voff;
    ma.bvheap = in.vheap;
    ma.kbeg = nullptr;
    ma.klen = nullptr;
    ma.vlen = nullptr;
    ma.S = S;
    ma.plo = t->partitioned ? t->part_lo : 0;   // the runs batch_prepare kept (k_clamp_runs)
    ma.phi = t->partitioned ? t->part_hi : S;
    return ma;
}

// The batch merged into the base CSR (a whole new CSR).
static int ingest_direct(st_tree *t, IngestIn &in) {
    const uint64_t n = in.n, S = t->S;
    Scratch sc(t);
    BatchPrep bp;
    CHK(batch_prepare(t, in, sc, bp));
    uint8_t *reject = nullptr, *dirty = nullptr;
    uint32_t *mpos = nullptr;
    if (in.verify_rehash) {
        CHK(verify_batch_paths(t, bp, sc, &reject));
        if (in.clevel_out) LAUNCH(t, "key_status", k_key_status, grid_for(n), 256, 0, (const uint32_t *)bp.seg, n,
                                  (const uint8_t *)reject, in.clevel_out);
    }

    // merge (k_merge_pos / k_merge_old / k_merge_new): count, scan, write
    MergeArgs ma = merge_args(t, view(t), in, bp, reject, S);
    BatchSums *bs = nullptr, *bx = nullptr;
    SegSums *ss = nullptr, *sx = nullptr;
    CHK(sc.alloc(&ss, S + 1));
    CHK(sc.alloc(&sx, S + 1));
    CHK(sc.alloc(&dirty, S));
    CHK(sc.alloc(&mpos, n));
    CHK(sc.alloc(&bs, n + 1));
    CHK(sc.alloc(&bx, n + 1));
    HIPCHK(hipMemsetAsync(ss + S, 0, sizeof(SegSums), t->stream));
    // records outside every run (a partition's clamped runs) keep sums 0
    HIPCHK(hipMemsetAsync(bs, 0, (n + 1) * sizeof(BatchSums), t->stream));
    LAUNCH(t, "merge_count", k_merge_keys, grid_for(n), 256, 0, ma, (const uint32_t *)bp.sseg, n, mpos, bs, (RecAt *)nullptr);
    LAUNCH(t, "merge_count", k_merge_sums, grid_for(S), 256, 0, ma, (const BatchSums *)bs, (const uint32_t *)mpos, ss, dirty);
    CHK(exclusive_scan<BatchSums>(t, bs, bx, n + 1));
    CHK(exclusive_scan<SegSums>(t, ss, sx, S + 1));
    SegSums tot(0);
    CHK(d2h(t, &tot, sx + S, sizeof(SegSums)));
    const uint64_t n_new = tot.v[0];
    CsrTaken out(t);
    CHK(csr_take(t, n_new + 1, tot.v[1] + HEAP_SLACK, tot.v[2] + HEAP_SLACK, out.o));
    HIPCHK(hipMemsetAsync(out.o.kheap + tot.v[1], 0, HEAP_SLACK, t->stream));
    HIPCHK(hipMemsetAsync(out.o.vheap + tot.v[2], 0, HEAP_SLACK, t->stream));
    MergeOut mo;
    mo.seg_off = out.o.seg_off; mo.seg_voff = out.o.seg_voff; mo.koff = out.o.koff; mo.voff = out.o.voff;
    mo.kheap = out.o.kheap; mo.vheap = out.o.vheap;
    LAUNCH(t, "merge_write", k_merge_old, (uint32_t)((S + 255) / 256), 256, 0, ma, (const uint32_t *)mpos,
           (const BatchSums *)bx, (const SegSums *)sx, mo);
    LAUNCH(t, "merge_write", k_merge_new, grid_for(n), 256, 0, ma, (const uint32_t *)bp.sseg, n, (const uint32_t *)mpos,
           (const BatchSums *)bx, (const SegSums *)sx, mo);
    const uint64_t tot_k = tot.v[1], tot_v = tot.v[2];
    // swap in the new CSR (the old one becomes the spare set, in stream order)
    out.install();
    t->n = n_new; t->kbytes = tot_k; t->vbytes = tot_v;
    t->perm_valid = false;
    // the hash-ready tiles are stale now; the next full rehash rebuilds them
    // (streaming batches never pay for a tile rebuild they do not use)
    t->tiles_valid = false;
    t->tiles_wanted = false;

    if (in.verify_rehash) {
        // dirty-path rehash: segments whose content changed and their ancestors
        HIPCHK(hipMemsetAsync(t->mark, 0, t->nslots, t->stream));
        LAUNCH(t, "mark_dirty", k_mark_from_segments, grid_for(S), 256, 0, view(t), (const uint8_t *)dirty, t->mark);
        CHK(rehash_all(t, t->mark, nullptr, HashBins{nullptr, nullptr, 0, 0, 0}, n * 64 <= S));   // <= n segments dirty
    }
    t->fresh = false;
    return ST_OK;
}

// ------------------------------------------------------------------ the paged layout (pages.h)
// Streaming insert batches (insert semantics, a batch small next to the
// tree) go to the paged layout: the first one copies the CSR into pages with
// slack; each batch then rewrites only the tails of the segments it touches
// (or moves a segment that outgrew its page to the append region); a batch
// whose moves do not fit the append region first rebuilds the pages (fresh
// slack, an empty append region).  Every other call folds the pages back into
// the canonical CSR first (flush_all).

static void pages_free(st_tree *t, Pages &g) {
    for (void *p : {(void *)g.m.beg, (void *)g.m.end, (void *)g.m.vbeg, (void *)g.m.vend, (void *)g.m.kbeg, (void *)g.m.ecap, (void *)g.m.kcap,
                    (void *)g.m.vcap, (void *)g.m.ebot, (void *)g.m.kbot, (void *)g.m.vbot, (void *)g.m.klen, (void *)g.m.vlen, (void *)g.koff, (void *)g.voff, (void *)g.kheap, (void *)g.vheap})
        dfree(t, p);
    const uint64_t b = g.batches, bu = g.builds, f = g.folds, r = g.reloc_e, tv = g.touched_v;
    g = Pages();
    g.batches = b; g.builds = bu; g.folds = f; g.reloc_e = r; g.touched_v = tv;
}

// Copy the tree's segments (CSR or pages) into a new layout: pages with
// slack_pct percent of slack and an append region of at least `reserve`
// (entries, key bytes, value bytes), or (slack_pct < 0) the canonical CSR.
static int pages_build(st_tree *t, int slack_pct, const PageSums &reserve) {
    const uint64_t S = t->S;
    const DevTree src = view(t);
    // a paged source: its uniform pages keep no per-entry offsets (pages.h)
    const uint16_t *sklen = t->pg.on ? t->pg.m.klen : nullptr, *svlen = t->pg.on ? t->pg.m.vlen : nullptr;
    Scratch sc(t);
    PageSums *sz = nullptr, *base = nullptr;
    CHK(sc.alloc(&sz, S + 1));
    CHK(sc.alloc(&base, S + 1));
    HIPCHK(hipMemsetAsync(sz + S, 0, sizeof(PageSums), t->stream));
    LAUNCH(t, "page_build", k_page_sizes, grid_for(S), 256, 0, src, slack_pct, sz);
    CHK(exclusive_scan<PageSums>(t, sz, base, S + 1));
    PageSums tot(0);
    CHK(d2h(t, &tot, base + S, sizeof(PageSums)));
    const uint32_t grid = (uint32_t)std::min<uint64_t>((S + 3) / 4, 65536);
    if (slack_pct < 0) {   // back to the canonical CSR
        CsrTaken out(t);
        CHK(csr_take(t, tot.v[0] + 1, tot.v[1] + HEAP_SLACK, tot.v[2] + HEAP_SLACK, out.o));
        HIPCHK(hipMemsetAsync(out.o.kheap + tot.v[1], 0, HEAP_SLACK, t->stream));
        HIPCHK(hipMemsetAsync(out.o.vheap + tot.v[2], 0, HEAP_SLACK, t->stream));
        PageDst d{};
        d.koff = out.o.koff; d.voff = out.o.voff; d.kheap = out.o.kheap; d.vheap = out.o.vheap;
        d.cseg_off = out.o.seg_off; d.cseg_voff = out.o.seg_voff;
        LAUNCH(t, "page_fold", k_page_copy, grid, 256, 0, src, (const PageSums *)base, (const PageSums *)sz, d, sklen, svlen);
        out.install();
        t->n = tot.v[0]; t->kbytes = tot.v[1]; t->vbytes = tot.v[2];
        CHK(tsync(t));   // the pages' buffers are free once the copy has read them
        pages_free(t, t->pg);
        t->pg.folds++;
        t->perm_valid = false;
        return ST_OK;
    }
    // the append region: slack_pct percent of the pages, or the room asked for
    Pages g;
    g.cap_e = tot.v[0] + std::max<uint64_t>(reserve.v[0], tot.v[0] * slack_pct / 100) + 1;
    g.cap_k = tot.v[1] + std::max<uint64_t>(reserve.v[1], tot.v[1] * slack_pct / 100);
    g.cap_v = tot.v[2] + std::max<uint64_t>(reserve.v[2], tot.v[2] * slack_pct / 100);
    struct Undo {   // a failed build frees what it allocated
        st_tree *t; Pages &g; bool done = false;
        ~Undo() { if (!done) pages_free(t, g); }
    } undo{t, g};
    for (uint64_t **a : {&g.m.beg, &g.m.end, &g.m.vbeg, &g.m.vend, &g.m.kbeg, &g.m.ecap, &g.m.kcap, &g.m.vcap, &g.m.ebot,
                         &g.m.kbot, &g.m.vbot})
        CHK(dalloc_t(t, a, S));
    CHK(dalloc_t(t, &g.m.klen, S));
    CHK(dalloc_t(t, &g.m.vlen, S));
    CHK(dalloc_t(t, &g.koff, g.cap_e));
    CHK(dalloc_t(t, &g.voff, g.cap_e));
    CHK(dalloc(t, (void **)&g.kheap, g.cap_k + HEAP_SLACK));
    CHK(dalloc(t, (void **)&g.vheap, g.cap_v + HEAP_SLACK));
    HIPCHK(hipMemsetAsync(g.kheap + g.cap_k, 0, HEAP_SLACK, t->stream));
    HIPCHK(hipMemsetAsync(g.vheap + g.cap_v, 0, HEAP_SLACK, t->stream));
    PageDst d{};
    d.koff = g.koff; d.voff = g.voff; d.kheap = g.kheap; d.vheap = g.vheap; d.m = g.m;
    d.slack_pct = t->pg_down ? slack_pct : -1;   // head slack only for merges that may shift down (page_head)
    LAUNCH(t, "page_build", k_page_copy, grid, 256, 0, src, (const PageSums *)base, (const PageSums *)sz, d, sklen, svlen);
    g.use_e = tot.v[0]; g.use_k = tot.v[1]; g.use_v = tot.v[2];
    g.on = true;
    g.batches = t->pg.batches; g.builds = t->pg.builds + 1; g.folds = t->pg.folds; g.reloc_e = t->pg.reloc_e;
    g.touched_v = t->pg.touched_v;
    CHK(tsync(t));   // the old pages (if any) were read
    pages_free(t, t->pg);
    t->pg = g;
    undo.done = true;
    // while the pages hold the segments no merge writes a CSR: the spare set
    // (a whole retired CSR) is released, the fold back allocates its own
    csr_free(t, t->spare);
    t->perm_valid = false;
    return ST_OK;
}

// trees from this many entries delete segments in the pages (st_store_segment)
#define PAGED_DELETE_MIN (1ull << 20)

static int pages_fold(st_tree *t) {
    if (!t->pg.on) return ST_OK;
    return pages_build(t, -1, PageSums(0));
}

// A streaming batch: insert semantics, small next to the (owned part of the) tree.
static bool pages_eligible(const st_tree *t, const IngestIn &in) {
    if (t->pg_slack < 0 || !in.verify_rehash || in.seg_given || in.bop || in.seg_replace || t->fresh || t->n == 0) return false;
    const double own = t->partitioned ? (double)(t->part_hi - t->part_lo) / (double)t->S : 1.0;
    return (double)in.n * own * 32.0 <= (double)t->n;
}

// The checked mode's verdict (ST_DBG_PAGE_CHECK): any violation the kernels
// counted in chk is ST_EDEVICE, with the first one in the message, and the
// tree refuses reads until a clean full rehash (its pages are not trusted).
static int page_check_report(st_tree *t, const unsigned long long *chk, const char *when) {
    unsigned long long h[32];
    CHK(d2h(t, h, chk, 256));
    if (!h[0]) return ST_OK;
    g_err = std::string("page check ") + when + ": " + std::to_string(h[0]) + " violations; first code " +
            std::to_string(h[1]) + " segment " + std::to_string(h[2]) + " at " + std::to_string(h[3]) + " bound " +
            std::to_string(h[4]) + "; batch " + std::to_string(t->pg.batches) + "; koff";
    for (int q = 0; q < 12; q++) g_err += " " + std::to_string(h[5 + q]);
    g_err += "; voff";
    for (int q = 0; q < 12; q++) g_err += " " + std::to_string(h[17 + q]);
    t->poisoned = true;
    return ST_EDEVICE;
}

static int ingest_paged(st_tree *t, IngestIn &in) {
    const uint64_t n = in.n, S = t->S;
    if (!t->pg.on) CHK(pages_build(t, t->pg_slack, PageSums(0)));
    Scratch sc(t);
    // acc: the batch's totals (k_page_place, a line apart), then the rejected
    // records (insert_int64's count, read with them); hcnt: the hash list's
    // bin counts; both and the path marks zeroed with the bucketing's counters
    unsigned long long *acc = nullptr, *hcnt = nullptr;
    CHK(sc.alloc(&acc, 6 * PP_LINE));
    CHK(sc.alloc(&hcnt, (uint64_t)HB * PP_LINE));
    ZeroSpans z{};
    z.p[0] = reinterpret_cast<uint8_t *>(acc); z.n[0] = 6 * PP_LINE * 8;
    z.p[1] = reinterpret_cast<uint8_t *>(hcnt); z.n[1] = HB * PP_LINE * 8;
    z.p[2] = t->mark; z.n[2] = t->nslots;
    z.k = 3;
    BatchPrep bp;
    CHK(batch_prepare(t, in, sc, bp, &z));
    uint8_t *reject = nullptr, *dirty = nullptr, *mode = nullptr;
    BatchSums *bs = nullptr, *bx = nullptr;
    SegSums *sm = nullptr;
    unsigned long long *fpos = nullptr;
    PlanSums *rsz = nullptr, *rbase = nullptr;
    uint32_t *mpos = nullptr;
    RecAt *rat = nullptr;
    PrefixState *ps = nullptr;
    uint32_t *hlist = nullptr;
    const uint64_t hcap = std::min<uint64_t>(S, n);   // a changed segment has a run
    CHK(sc.alloc(&hlist, (uint64_t)HB * hcap));
    CHK(sc.alloc(&reject, S));
    CHK(sc.alloc(&ps, S));
    CHK(sc.alloc(&rat, n));
    CHK(sc.alloc(&sm, S));
    CHK(sc.alloc(&fpos, S));
    CHK(sc.alloc(&dirty, S));
    CHK(sc.alloc(&mode, S));
    CHK(sc.alloc(&rsz, S));
    CHK(sc.alloc(&rbase, S));
    CHK(sc.alloc(&mpos, n));
    CHK(sc.alloc(&bs, n + 1));
    CHK(sc.alloc(&bx, n));
    // No memsets of the per-segment plan: k_run_plan writes every segment
    // with a run, k_page_place every other one; the per-record sums are read
    // only inside runs.
    // merge positions (a lane per record, the segments' size deltas by
    // atomics), then the touched segments' verify (saving each one's
    // unchanged-prefix MD5 state) and the inner nodes of their paths
    // checked mode: every page is validated BEFORE the batch too (a page a
    // defect left outside its capacity is refused here, ST_EDEVICE, instead of
    // being indexed by the kernels below), and the positions and verify
    // kernels bounds-check the pages they read
    unsigned long long *chk = nullptr;
    if (t->pg_check) {
        CHK(sc.alloc(&chk, 32));
        HIPCHK(hipMemsetAsync(chk, 0, 256, t->stream));
        LAUNCH(t, "page_check", k_page_validate, grid_for(S), 256, 0, t->pg.m, (const uint64_t *)t->pg.koff,
               (const uint64_t *)t->pg.voff, S, t->pg.cap_e, t->pg.cap_k, t->pg.cap_v, chk);
        CHK(page_check_report(t, chk, "before the batch"));
    }
    MergeArgs ma = merge_args(t, view(t), in, bp, nullptr, S);
    ma.kbeg = t->pg.m.kbeg;
    ma.klen = t->pg.m.klen;
    ma.vlen = t->pg.m.vlen;
    const PageBounds pb{t->pg.cap_e, t->pg.cap_k, t->pg.cap_v, chk};
    {
        const DevTree d = view(t);
        LAUNCH(t, "mark_paths", k_mark_paths, grid_for(S), 256, 0, d, t->H + 1, (const uint64_t *)bp.bseg_off,
               (const uint64_t *)nullptr, S, t->mark);   // (the marks were zeroed with the bucketing's counters)
        CHK(ensure_perm_any(t));
        // then the per-segment sums and the runs' prefix sums by each run's first lane (no atomics, no scan)
        LAUNCH(t, "merge_count", k_merge_keys, grid_for(n), 256, 0, ma, (const uint32_t *)bp.sseg, n, mpos, bs, rat,
               (SegSums *)nullptr, (uint8_t *)nullptr, (unsigned long long *)nullptr, pb);
        // each run summed and its page planned by the run's first lane (in place
        // or moved; a rejected segment's plan is dropped by k_page_place below)
        LAUNCH(t, "page_plan", k_run_plan, grid_for(n), 256, 0, (const uint32_t *)bp.sseg, (const uint64_t *)bp.bseg_off, n,
               (const BatchSums *)bs, (const RecAt *)rat, t->pg.m, (const uint64_t *)t->pg.koff,
               (const uint64_t *)t->pg.voff, t->pg_slack, dirty, fpos, bx, sm, mode, rsz, t->pg_down);
        LAUNCH(t, "segment_verify", k_verify_cap, grid_for(S), 256, 0, d, (const uint32_t *)t->seg_perm,
               (const uint8_t *)t->mark, t->ok, (const unsigned long long *)fpos, ps, pb, (const uint32_t *)nullptr);
        CHK(verify_levels(t, t->H + 1));
    }
    // the plan settled (rejections, places in the append region, totals),
    // the merge, the dirty-path rehash, then ONE read of the totals: a batch
    // whose moves did not fit the append region was not merged (k_page_merge
    // checks the totals itself) -- the pages are rebuilt with room for them
    // and the batch planned and merged again
    for (int pass = 0;; pass++) {
        if (pass) {
            HIPCHK(hipMemsetAsync(hcnt, 0, HB * PP_LINE * 8, t->stream));
            HIPCHK(hipMemsetAsync(acc, 0, 5 * PP_LINE * 8, t->stream));
            LAUNCH(t, "page_plan", k_run_plan, grid_for(n), 256, 0, (const uint32_t *)bp.sseg, (const uint64_t *)bp.bseg_off,
                   n, (const BatchSums *)bs, (const RecAt *)rat, t->pg.m, (const uint64_t *)t->pg.koff,
                   (const uint64_t *)t->pg.voff, t->pg_slack, dirty, fpos, bx, sm, mode, rsz, t->pg_down);
        }
        LAUNCH(t, "page_place", k_page_place, (uint32_t)((S + 256 * PP_ITER - 1) / (256 * PP_ITER)), 256, 0, view(t), (const uint64_t *)bp.bseg_off,
               (const uint8_t *)t->ok, reject, mode, dirty, (const PlanSums *)rsz, rbase, acc, (const PrefixState *)ps,
               (const SegSums *)sm, hlist, hcap, hcnt);
        if (!pass && in.clevel_out)
            LAUNCH(t, "key_status", k_key_status, grid_for(n), 256, 0, (const uint32_t *)bp.seg, n, (const uint8_t *)reject,
                   in.clevel_out);
        ma.seg_reject = reject;
        const Pages &g = t->pg;
        PageMergeArgs pa;
        pa.a = ma;
        pa.m = g.m;
        pa.koff = g.koff; pa.voff = g.voff; pa.kheap = g.kheap; pa.vheap = g.vheap;
        pa.pos = mpos; pa.rat = rat; pa.bx = bx; pa.ss = sm; pa.mode = mode; pa.rbase = rbase; pa.rsz = rsz;
        pa.e0 = g.use_e; pa.k0 = g.use_k; pa.v0 = g.use_v;
        pa.ce = g.cap_e; pa.ck = g.cap_k; pa.cv = g.cap_v;
        pa.acc = acc;
        pa.slack_pct = t->pg_down ? t->pg_slack : -1;
        pa.chk = nullptr;
        // uniform pages a record of another length turns mixed: their offsets first
        LAUNCH(t, "page_merge", k_page_materialize, grid_for(S, 256, 4096), 256, 0, g.m, g.koff, g.voff,
               (const uint8_t *)mode, (const uint8_t *)reject, S);
        if (!t->pg_check) {
            LAUNCH(t, "page_merge", k_page_merge<false>, grid_for(S), 256, 0, pa);
        } else {   // checked build (debug knob): merges that would leave their pages reported, not performed
            pa.chk = chk;   // (the pre-batch check found nothing: zero)
            LAUNCH(t, "page_merge", k_page_merge<true>, grid_for(S), 256, 0, pa);
            LAUNCH(t, "page_check", k_page_validate, grid_for(S), 256, 0, g.m, (const uint64_t *)g.koff,
                   (const uint64_t *)g.voff, S, g.cap_e, g.cap_k, g.cap_v, pa.chk);
            CHK(page_check_report(t, chk, "after the merge"));
        }
        // dirty-path rehash over the pages, each segment from its unchanged
        // prefix's MD5 state (a batch not merged hashes its old content again:
        // the same hashes)
        HIPCHK(hipMemsetAsync(t->mark, 0, t->nslots, t->stream));
        LAUNCH(t, "mark_dirty", k_mark_from_segments, grid_for(S), 256, 0, view(t), (const uint8_t *)dirty, t->mark);
        CHK(rehash_all(t, t->mark, ps, HashBins{hlist, hcnt, hcap, HB, PP_LINE}));
        if (!pass && in.clevel_out && in.count_rejected)
            LAUNCH(t, "key_status", k_count_nonzero, grid_for(n), 256, 0, (const uint32_t *)in.clevel_out, n,
                   acc + 5 * PP_LINE);
        unsigned long long accv[6 * PP_LINE], tot[6];
        CHK(d2h(t, accv, acc, sizeof(accv)));
        for (int q = 0; q < 6; q++) tot[q] = accv[q * PP_LINE];
        if (!pass && in.clevel_out && in.count_rejected) { in.n_rejected = tot[5]; in.rejected_counted = true; }
        if (g.use_e + tot[0] + 1 <= g.cap_e && g.use_k + tot[1] <= g.cap_k && g.use_v + tot[2] <= g.cap_v) {
            t->pg.use_e += tot[0]; t->pg.use_k += tot[1]; t->pg.use_v += tot[2];
            t->pg.reloc_e += tot[0];
            t->pg.touched_v += tot[4];
            t->pg.batches++;
            t->n += tot[3];
            break;
        }
        if (pass) { g_err = "page build left no room for the batch's moves"; return ST_EDEVICE; }
        // rebuild: every page gets fresh slack, the append region room for these moves
        PageSums want(0);
        for (int q = 0; q < 3; q++) want.v[q] = 2 * tot[q];
        CHK(pages_build(t, t->pg_slack, want));
        ma = merge_args(t, view(t), in, bp, reject, S);
        ma.kbeg = t->pg.m.kbeg;
        ma.klen = t->pg.m.klen;
        ma.vlen = t->pg.m.vlen;
    }
    t->perm_valid = false;
    t->tiles_valid = false;
    t->tiles_wanted = false;
    t->fresh = false;
    return ST_OK;
}

// A streaming batch goes to the pages -- except a lone one: the first after
// any other call merges into the CSR (building the pages copies the whole
// tree, which only a run of batches pays back).
static int ingest(st_tree *t, IngestIn &in) {
    in.n_rejected = 0;
    if (in.n == 0) return ST_OK;
    if (pages_eligible(t, in) && (t->pg.on || t->pg_streak++ > 0)) return ingest_paged(t, in);
    if (!pages_eligible(t, in)) t->pg_streak = 0;
    CHK(pages_fold(t));
    return ingest_direct(t, in);
}

// ------------------------------------------------------------------ overlay (small_path.h)
// Merge the segments small inserts left in the overlay into the CSR: their
// records become one ingest batch with replace flags (their hashes are already
// in the slot arrays, so nothing is rehashed).  Every entry point that reads
// segments other than the small kernels calls this first.
static int flush_overlay(st_tree *t) {
    if (!t->ov_pending) return ST_OK;
    const uint64_t S = t->S;
    Scratch sc(t);
    uint64_t *cnt = nullptr, *kbs = nullptr, *vbs = nullptr, *eoff = nullptr, *ko0 = nullptr, *vo0 = nullptr;
    uint8_t *rep = nullptr;
    CHK(sc.alloc(&cnt, S + 1));
    CHK(sc.alloc(&kbs, S + 1));
    CHK(sc.alloc(&vbs, S + 1));
    CHK(sc.alloc(&eoff, S + 1));
    CHK(sc.alloc(&ko0, S + 1));
    CHK(sc.alloc(&vo0, S + 1));
    CHK(sc.alloc(&rep, S));
    LAUNCH(t, "ov_flush", k_ov_sizes, grid_for(S + 1), 256, 0, t->ov, S, cnt, kbs, vbs, rep);
    CHK(exclusive_scan<uint64_t>(t, cnt, eoff, S + 1));
    CHK(exclusive_scan<uint64_t>(t, kbs, ko0, S + 1));
    CHK(exclusive_scan<uint64_t>(t, vbs, vo0, S + 1));
    HIPCHK(hipMemcpyAsync(t->pin, eoff + S, 8, hipMemcpyDeviceToHost, t->stream));
    HIPCHK(hipMemcpyAsync(t->pin + 1, ko0 + S, 8, hipMemcpyDeviceToHost, t->stream));
    HIPCHK(hipMemcpyAsync(t->pin + 2, vo0 + S, 8, hipMemcpyDeviceToHost, t->stream));
    CHK(tsync(t));
    const uint64_t n = t->pin[0], kt = t->pin[1], vt = t->pin[2];
    if (n) {
        uint8_t *krec = nullptr, *vh = nullptr;
        uint64_t *ko = nullptr, *vo = nullptr;
        uint32_t *segs = nullptr;
        CHK(sc.bytes(&krec, kt + HEAP_SLACK));
        CHK(sc.bytes(&vh, vt + HEAP_SLACK));
        CHK(sc.alloc(&ko, n + 1));
        CHK(sc.alloc(&vo, n + 1));
        CHK(sc.alloc(&segs, n));
        HIPCHK(hipMemsetAsync(krec + kt, 0, HEAP_SLACK, t->stream));
        HIPCHK(hipMemsetAsync(vh + vt, 0, HEAP_SLACK, t->stream));
        LAUNCH(t, "ov_flush", k_ov_gather, grid_for(S), 256, 0, t->ov, S, (const uint64_t *)eoff, (const uint64_t *)ko0,
               (const uint64_t *)vo0, krec, ko, vh, vo, segs);
        LAUNCH(t, "ov_flush", k_ov_terminate, 1, 64, 0, n, (const uint64_t *)(ko0 + S), (const uint64_t *)(vo0 + S), ko, vo);
        IngestIn in{};
        in.n = n; in.krec = krec; in.koff = ko; in.vheap = vh; in.voff = vo;
        in.seg_given = segs; in.seg_replace = rep; in.verify_rehash = false;
        CHK(ingest(t, in));
    }
    HIPCHK(hipMemsetAsync(t->ov.idx, 0xff, S * 8, t->stream));
    HIPCHK(hipMemsetAsync(t->ov.used, 0, 8, t->stream));
    t->ov_pending = false;
    return ST_OK;
}

// Every entry point that reads segments: the small inserts' overlay and the
// streaming batches' pages folded into the canonical CSR first.
static int flush_all(st_tree *t) {
    CHK(flush_overlay(t));
    CHK(pages_fold(t));
    t->pg_streak = 0;
    return ST_OK;
}
#define FLUSH(t) CHK(flush_all(t))

static int ensure_small(st_tree *t) {
    if (!t->ov.idx) {
        const uint64_t cap = 64ull << 20;
        CHK(dalloc_t(t, &t->ov.idx, t->S));
        CHK(dalloc(t, (void **)&t->ov.heap, cap + HEAP_SLACK));
        CHK(dalloc_t(t, &t->ov.used, 1));
        HIPCHK(hipMemsetAsync(t->ov.idx, 0xff, t->S * 8, t->stream));
        HIPCHK(hipMemsetAsync(t->ov.heap + cap, 0, HEAP_SLACK, t->stream));
        HIPCHK(hipMemsetAsync(t->ov.used, 0, 8, t->stream));
        t->ov.cap = cap;
        t->async_pending = true;   // another stream's k_small_multi waits for these
    }
    if (!t->sout) {
        // fine-grained (coherent) host memory for the result block and the
        // request slots: the GPU reads the request and writes the results
        // across PCIe, nothing of either is cached in its L2
        if (hipHostMalloc((void **)&t->sout, sizeof(SmallOut), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostMalloc((void **)&t->sreq, SMALL_SLOTS * sizeof(SmallReq), hipHostMallocMapped | hipHostMallocCoherent) !=
                hipSuccess) {
            g_err = "hipHostMalloc (mapped) failed";
            return ST_EDEVICE;
        }
        memset(t->sout, 0, sizeof(SmallOut));   // no valid record before the first call
        memset(t->sreq, 0, SMALL_SLOTS * sizeof(SmallReq));
        HIPCHK(hipHostGetDevicePointer((void **)&t->sout_dev, t->sout, 0));
        HIPCHK(hipHostGetDevicePointer((void **)&t->sreq_dev, t->sreq, 0));
    }
    return ST_OK;
}

// One validated 16-byte record of the result block (small_path.h): copied
// out with volatile reads, valid iff it carries `seq` and its check word.
static bool small_rec(const SmallOut *o, int i, uint32_t seq, uint32_t *w, uint32_t *x) {
    const volatile uint32_t *r = reinterpret_cast<const volatile uint32_t *>(i < 0 ? &o->hdr : &o->rec[i]);
    const uint32_t s0 = r[0], w0 = r[1], x0 = r[2], c0 = r[3];
    if (s0 != seq || c0 != small_check(s0, w0, x0)) return false;
    *w = w0;
    *x = x0;
    return true;
}

// All of a call's results present and consistent?  Fills t->sres.
static bool small_collect(st_tree *t, uint32_t seq, uint32_t n, int op) {
    SmallRes &r = t->sres;
    uint32_t w, x;
    if (!small_rec(t->sout, -1, seq, &w, &x)) return false;
    r.retry = (w & 1u) != 0;
    r.new_entries = w >> 1;
    if (r.retry) return true;
    r.voff[0] = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (!small_rec(t->sout, (int)i, seq, &w, &x)) return false;
        r.status[i] = (int32_t)(w & 0xffu);
        r.clevel[i] = (w >> 8) & 0xffu;
        const uint32_t vlen = w >> 16;
        r.cbucket[i] = r.status[i] == ST_CORRUPTED ? x : 0;
        r.voff[i + 1] = r.voff[i] + (op == 0 && r.status[i] == ST_OK ? vlen : 0);
        if (op == 0 && r.status[i] == ST_OK) {   // the value bytes arrived too?
            const volatile uint8_t *v = t->sout->vbytes + r.voff[i];
            uint32_t h = FNV1A_INIT;
            for (uint32_t b = 0; b < vlen; b++) h = fnv1a_step(h, v[b]);
            if (h != x) return false;
        }
    }
    return true;
}

// Fill t's next request slot for one get/2 (op 0) or insert/3 (op 1) batch of
// k_small; *ok = 0 when the batch does not fit the kernel (the caller takes
// the bulk path).  Host pointers, records packed by the caller.
static int small_prepare(st_tree *t, int op, uint64_t n, const HostRecords &hr, const uint8_t *vheap, const uint64_t *voff,
                         int *ok, SmallItem *item) {
    *ok = 0;
    const uint64_t kbytes = hr.off[n];
    const uint64_t vbytes = op == 1 ? voff[n] - voff[0] : 0;
    if (n == 0 || n > SB_MAX || kbytes > SB_KB || vbytes > SB_VB || t->W > 32 || t->partitioned ||
        small_lds_bytes((uint32_t)t->W) > 160 * 1024)
        return ST_OK;
    // a launch the tree did not wait for (st_rehash returns before its
    // kernel ends): its device error must be seen before k_small reads the
    // upper levels it wrote (st_rehash's error is reported by the next call
    // that waits, and that is this one)
    if (t->async_pending) CHK(tsync(t));
    CHK(pages_fold(t));   // k_small and its overlay flush work on the canonical CSR
    CHK(ensure_small(t));
    if (++t->small_seq == 0) t->small_seq = 1;
    const uint32_t seq = t->small_seq;
    // the request slot (alternating, so a slot is never rewritten while the
    // previous call's kernel could still be reading it)
    SmallReq *rq = &t->sreq[seq % SMALL_SLOTS];
    rq->t = view(t);
    rq->ov = t->ov;
    SmallIn &in = rq->in;
    in.n = (uint32_t)n;
    in.op = (uint32_t)op;
    static const int sdbg = getenv("ST_SMALL_STAMPS") ? atoi(getenv("ST_SMALL_STAMPS")) : 0;
    in.dbg = sdbg ? 1u : 0u;
    in.seq = seq;
    for (uint64_t i = 0; i <= n; i++) in.koff[i] = (uint32_t)hr.off[i];
    memcpy(in.kb, hr.heap.data(), kbytes);
    if (op == 1) {
        for (uint64_t i = 0; i <= n; i++) in.voff[i] = (uint32_t)(voff[i] - voff[0]);
        memcpy(in.vb, vheap + voff[0], vbytes);
    }
    item->req = t->sreq_dev + seq % SMALL_SLOTS;
    item->out = t->sout_dev;
    *ok = 1;
    return ST_OK;
}

// After the host validated a served batch's results (t->sres).
static void small_served(st_tree *t, int op) {
    if (op == 1) {
        t->n += t->sres.new_entries;
        t->ov_pending = true;
        t->fresh = false;
        t->tiles_valid = false;
        t->tiles_wanted = false;
        t->perm_valid = false;
    }
}

// One get/2 (op 0) or insert/3 (op 1) batch through k_small when it fits:
// returns ST_OK with *served = 1 and t->sres filled (get values in
// t->sout->vbytes), or *served = 0 (the caller takes the bulk path).  Host
// pointers, records packed by the caller.
static int small_call(st_tree *t, int op, uint64_t n, const HostRecords &hr, const uint8_t *vheap, const uint64_t *voff,
                      int *served) {
    *served = 0;
    int ok = 0;
    SmallItem item;
    CHK(small_prepare(t, op, n, hr, vheap, voff, &ok, &item));
    if (!ok) return ST_OK;
    const uint32_t seq = t->small_seq;
    std::atomic_thread_fence(std::memory_order_release);   // the request is in memory before the launch
    LAUNCH(t, "small", k_small, 1, 256, small_lds_bytes((uint32_t)t->W), item.req, item.out);
    // spin on the result records; after 5 ms (a faulted or very slow kernel)
    // a stream synchronisation, after which every write of the kernel is visible
    bool done = false;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0; !(done = small_collect(t, seq, (uint32_t)n, op)); i++) {
        if ((i & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(5)) break;
        __builtin_ia32_pause();
    }
    if (!done) {
        CHK(tsync(t));
        if (!small_collect(t, seq, (uint32_t)n, op)) { g_err = "small-batch kernel results incomplete"; return ST_EDEVICE; }
    }
    static const int sdbg = getenv("ST_SMALL_STAMPS") ? atoi(getenv("ST_SMALL_STAMPS")) : 0;
    if (sdbg) {   // diagnostic: phase times (µs from kernel start) to stderr
        CHK(tsync(t));
        const uint64_t *st = t->sout->stamp;
        fprintf(stderr, "small op=%d n=%llu:", op, (unsigned long long)n);
        for (int k = 1; k < 8; k++)
            if (st[k]) fprintf(stderr, " %d:%.2f", k, (st[k] - st[0]) / 100.0);
        // the shader clock over the kernel: cycles / wall between stamp 0 and the last
        int kl = 0;
        for (int k = 1; k < 8; k++)
            if (st[k] && st[8 + k]) kl = k;
        if (kl && st[kl] > st[0]) fprintf(stderr, " | %.2f GHz", (double)(st[8 + kl] - st[8]) / ((st[kl] - st[0]) * 10.0));
        fprintf(stderr, "\n");
        memset((void *)t->sout->stamp, 0, sizeof(t->sout->stamp));
    }
    // the results came after every earlier launch on the stream (stream order)
    t->async_pending = false;
    if (t->sres.retry) return ST_OK;
    *served = 1;
    small_served(t, op);
    return ST_OK;
}

// ------------------------------------------------------------------ per-key requests of many trees
// The per-key path of many ensembles at once (every
// peer tree of a node takes puts at the same time, riak_ensemble_peer_tree.erl:
// 224-234): the requests of each tree (in order, <= SB_MAX keys a round)
// become one k_small batch, and the batches of all trees run in ONE launch of
// k_small_multi, a workgroup per tree.  Same results as the per-tree calls in
// request order.  Each calling thread keeps its own host-mapped item array.
static thread_local SmallItem *t_items = nullptr, *t_items_dev = nullptr;
static thread_local uint32_t t_items_cap = 0;

static int items_reserve(uint32_t n) {
    if (n <= t_items_cap) return ST_OK;
    if (t_items) (void)hipHostFree(t_items);
    t_items = t_items_dev = nullptr;
    t_items_cap = 0;
    const uint32_t cap = std::max<uint32_t>(n, 256);
    if (hipHostMalloc((void **)&t_items, cap * sizeof(SmallItem), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void **)&t_items_dev, t_items, 0) != hipSuccess) {
        t_items = nullptr;
        g_err = "hipHostMalloc (mapped) failed";
        return ST_EDEVICE;
    }
    t_items_cap = cap;
    return ST_OK;
}

// op 0: get/2 (values into vout at voff_out), op 1: insert/3.
static int small_multi(int op, st_tree **trees, uint32_t n, const uint8_t *ktype, const uint8_t *kheap, const uint64_t *koff,
                       const uint8_t *vheap, const uint64_t *voff, int32_t *status, uint32_t *clevel, uint64_t *cbucket,
                       uint8_t *vout, uint64_t vcap, uint64_t *voff_out) {
    if (n == 0) {
        if (voff_out) voff_out[0] = 0;
        return ST_OK;
    }
    for (uint32_t i = 0; i < n; i++)
        if (!trees[i]) { g_err = "NULL tree"; return ST_EINVAL; }
    GroupLock glk(trees, n);
    // requests per tree, in request order
    std::vector<st_tree *> order;
    std::unordered_map<st_tree *, std::vector<uint32_t>> reqs;
    for (uint32_t i = 0; i < n; i++) {
        auto &v = reqs[trees[i]];
        if (v.empty()) order.push_back(trees[i]);
        v.push_back(i);
    }
    for (st_tree *u : order) {
        CHK(use_device(u));
        CHK(alive(u));
        if (u->device != trees[0]->device) { g_err = "trees on different devices"; return ST_EINVAL; }
    }
    std::vector<uint64_t> vlen(n, 0);             // get: value length of request i (status ST_OK)
    std::vector<std::vector<uint8_t>> vals(op == 0 ? n : 0);
    std::unordered_map<st_tree *, size_t> next;   // the tree's next request (index into reqs[u])
    st_tree *t0 = trees[0];
    hipStream_t s0 = t0->stream;
    for (;;) {
        // this round: the next <= SB_MAX requests of every tree with requests left
        struct Part { st_tree *t; std::vector<uint32_t> idx; uint32_t seq; bool small; };
        std::vector<Part> parts;
        for (st_tree *u : order) {
            auto &v = reqs[u];
            size_t &k = next[u];
            if (k == v.size()) continue;
            Part pt{u, {}, 0, false};
            uint64_t kb = 0, vb = 0;
            while (k < v.size() && pt.idx.size() < SB_MAX) {
                const uint32_t i = v[k];
                const uint64_t kl = koff[i + 1] - koff[i] + 16, vl = op == 1 ? voff[i + 1] - voff[i] : 0;
                if (!pt.idx.empty() && (kb + kl > SB_KB || vb + vl > SB_VB)) break;
                kb += kl;
                vb += vl;
                pt.idx.push_back(i);
                k++;
            }
            parts.push_back(std::move(pt));
        }
        if (parts.empty()) break;
        CHK(items_reserve((uint32_t)parts.size()));
        uint32_t m = 0;
        size_t lds = 0;
        for (Part &pt : parts) {
            st_tree *u = pt.t;
            const uint64_t c = pt.idx.size();
            std::vector<uint8_t> kt(c);
            std::vector<uint64_t> ko(c + 1, 0), vo(c + 1, 0);
            std::vector<uint8_t> kh, vh;
            for (uint64_t j = 0; j < c; j++) {
                const uint32_t i = pt.idx[j];
                kt[j] = ktype[i];
                kh.insert(kh.end(), kheap + koff[i], kheap + koff[i + 1]);
                ko[j + 1] = kh.size();
                if (op == 1) vh.insert(vh.end(), vheap + voff[i], vheap + voff[i + 1]);
                vo[j + 1] = vh.size();
            }
            HostRecords hr;
            CHK(pack_records(c, kt.data(), kh.data(), ko.data(), hr));
            int ok = 0;
            SmallItem it;
            CHK(small_prepare(u, op, c, hr, vh.data(), vo.data(), &ok, &it));
            if (!ok) continue;   // served below through the per-tree bulk path
            if (u->stream != s0 && u->async_pending) CHK(tsync(u));   // its own work first (e.g. an st_rehash)
            pt.small = true;
            pt.seq = u->small_seq;
            lds = std::max<size_t>(lds, small_lds_bytes((uint32_t)u->W));
            t_items[m++] = it;
        }
        if (m) {
            std::atomic_thread_fence(std::memory_order_release);   // requests and items are in memory before the launch
            hipLaunchKernelGGL(k_small_multi, dim3(m), dim3(256), lds, s0, (const SmallItem *)t_items_dev);
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) { g_err = std::string("launch small_multi: ") + hipGetErrorString(e); return ST_EDEVICE; }
        }
        // collect every served batch (spin; after 5 ms a synchronisation of the launch stream)
        const auto tw = std::chrono::steady_clock::now();
        std::vector<char> got(parts.size(), 0);
        size_t left = m;
        bool synced = false;
        while (left) {
            for (size_t p = 0; p < parts.size(); p++) {
                if (!parts[p].small || got[p]) continue;
                if (small_collect(parts[p].t, parts[p].seq, (uint32_t)parts[p].idx.size(), op)) { got[p] = 1; left--; }
            }
            if (!left) break;
            if (synced) { g_err = "small-batch kernel results incomplete"; return ST_EDEVICE; }
            if (std::chrono::steady_clock::now() - tw > std::chrono::milliseconds(5)) {
                if (hipStreamSynchronize(s0) != hipSuccess) { g_err = "hipStreamSynchronize (small_multi)"; return ST_EDEVICE; }
                synced = true;
            }
            __builtin_ia32_pause();
        }
        // outputs; batches the kernel did not serve (retry) or could not take go through the bulk path
        for (Part &pt : parts) {
            st_tree *u = pt.t;
            const uint64_t c = pt.idx.size();
            if (pt.small && !u->sres.retry) {
                small_served(u, op);
                for (uint64_t j = 0; j < c; j++) {
                    const uint32_t i = pt.idx[j];
                    status[i] = u->sres.status[j];
                    if (clevel) clevel[i] = u->sres.clevel[j];
                    if (cbucket) cbucket[i] = u->sres.cbucket[j];
                    if (op == 0 && status[i] == ST_OK) {
                        const uint32_t a = u->sres.voff[j], b = u->sres.voff[j + 1];
                        vals[i].assign((const uint8_t *)u->sout->vbytes + a, (const uint8_t *)u->sout->vbytes + b);
                    }
                }
                continue;
            }
            std::vector<uint8_t> kt(c);
            std::vector<uint64_t> ko(c + 1, 0), vo(c + 1, 0);
            std::vector<uint8_t> kh, vh;
            for (uint64_t j = 0; j < c; j++) {
                const uint32_t i = pt.idx[j];
                kt[j] = ktype[i];
                kh.insert(kh.end(), kheap + koff[i], kheap + koff[i + 1]);
                ko[j + 1] = kh.size();
                if (op == 1) vh.insert(vh.end(), vheap + voff[i], vheap + voff[i + 1]);
                vo[j + 1] = vh.size();
            }
            kh.push_back(0);
            vh.push_back(0);
            if (op == 1) {
                std::vector<int32_t> st(c);
                std::vector<uint32_t> cl(c);
                std::vector<uint64_t> cb(c);
                CHK(st_insert_batch(u, c, kt.data(), kh.data(), ko.data(), vh.data(), vo.data(), st.data(), cl.data(), cb.data()));
                for (uint64_t j = 0; j < c; j++) {
                    status[pt.idx[j]] = st[j];
                    if (clevel) clevel[pt.idx[j]] = cl[j];
                    if (cbucket) cbucket[pt.idx[j]] = cb[j];
                }
            } else {
                st_result *res = nullptr;
                CHK(st_get_batch(u, c, kt.data(), kh.data(), ko.data(), &res));
                for (uint64_t j = 0; j < c; j++) {
                    const uint32_t i = pt.idx[j];
                    status[i] = res->status[j];
                    if (clevel) clevel[i] = res->clevel[j];
                    if (cbucket) cbucket[i] = res->cbucket[j];
                    if (status[i] == ST_OK) {
                        const uint64_t e = res->eoff[j];
                        vals[i].assign(res->aheap + res->aoff[e], res->aheap + res->aoff[e + 1]);
                    }
                }
                st_free_result(res);
            }
        }
    }
    if (op == 0) {   // the values, packed in request order
        uint64_t need = 0;
        for (uint32_t i = 0; i < n; i++) need += status[i] == ST_OK ? vals[i].size() : 0;
        if (need > vcap) {
            voff_out[n] = need;
            g_err = "value buffer too small (" + std::to_string(need) + " bytes needed)";
            return ST_ERANGE;
        }
        uint64_t o = 0;
        voff_out[0] = 0;
        for (uint32_t i = 0; i < n; i++) {
            const uint64_t l = status[i] == ST_OK ? vals[i].size() : 0;
            if (l) memcpy(vout + o, vals[i].data(), l);
            o += l;
            voff_out[i + 1] = o;
        }
    }
    return ST_OK;
}

extern "C" int st_insert1_multi(st_tree **trees, uint32_t n, const uint8_t *ktype, const uint8_t *kheap, const uint64_t *koff,
                                const uint8_t *vheap, const uint64_t *voff, int32_t *status, uint32_t *clevel,
                                uint64_t *cbucket) {
    return small_multi(1, trees, n, ktype, kheap, koff, vheap, voff, status, clevel, cbucket, nullptr, 0, nullptr);
}

extern "C" int st_get1_multi(st_tree **trees, uint32_t n, const uint8_t *ktype, const uint8_t *kheap, const uint64_t *koff,
                             uint8_t *vout, uint64_t vcap, uint64_t *voff_out, int32_t *status, uint32_t *clevel,
                             uint64_t *cbucket) {
    return small_multi(0, trees, n, ktype, kheap, koff, nullptr, nullptr, status, clevel, cbucket, vout, vcap, voff_out);
}

// ------------------------------------------------------------------ writes
static int upload_records(st_tree *t, uint64_t n, const uint8_t *ktype, const uint8_t *kheap, const uint64_t *koff,
                          uint8_t **d_krec, uint64_t **d_koff) {
    HostRecords hr;
    CHK(pack_records(n, ktype, kheap, koff, hr));
    CHK(dalloc(t, (void **)d_krec, hr.heap.size()));
    CHK(dalloc_t(t, d_koff, n + 1));
    CHK(h2d(t, *d_krec, hr.heap.data(), hr.heap.size()));
    CHK(h2d(t, *d_koff, hr.off.data(), (n + 1) * 8));
    CHK(tsync(t));   // host vectors die here
    return ST_OK;
}

static int upload_values(st_tree *t, uint64_t n, const uint8_t *vheap, const uint64_t *voff, uint8_t **d_vheap,
                         uint64_t **d_voff) {
    const uint64_t vb = voff[n] - voff[0];
    CHK(dalloc(t, (void **)d_vheap, vb + HEAP_SLACK));
    CHK(dalloc_t(t, d_voff, n + 1));
    std::vector<uint64_t> vo(n + 1);
    for (uint64_t i = 0; i <= n; i++) vo[i] = voff[i] - voff[0];
    CHK(h2d(t, *d_vheap, vheap + voff[0], vb));
    HIPCHK(hipMemsetAsync(*d_vheap + vb, 0, HEAP_SLACK, t->stream));
    CHK(h2d(t, *d_voff, vo.data(), (n + 1) * 8));
    CHK(tsync(t));
    return ST_OK;
}

extern "C" int st_insert_batch(st_tree *t, uint64_t n, const uint8_t *ktype, const uint8_t *kheap, const uint64_t *koff,
                               const uint8_t *vheap, const uint64_t *voff, int32_t *status, uint32_t *clevel,
                               uint64_t *cbucket) {
    ENTER(t);
    if (n == 0) return ST_OK;
    if (n <= SB_MAX) {   // per-key latency path: one launch, one sync
        HostRecords hr;
        CHK(pack_records(n, ktype, kheap, koff, hr));
        int served = 0;
        CHK(small_call(t, 1, n, hr, vheap, voff, &served));
        if (served) {
            for (uint64_t i = 0; i < n; i++) {
                if (status) status[i] = t->sres.status[i];
                if (clevel) clevel[i] = t->sres.clevel[i];
                if (cbucket) cbucket[i] = t->sres.cbucket[i];
            }
            return ST_OK;
        }
    }
    CHK(flush_overlay(t));   // the pages stay: a streaming batch may go to them (ingest)
    uint8_t *krec = nullptr, *dv = nullptr;
    uint64_t *dko = nullptr, *dvo = nullptr;
    uint32_t *dcl = nullptr, *dseg = nullptr;
    int r = upload_records(t, n, ktype, kheap, koff, &krec, &dko);
    if (!r) r = upload_values(t, n, vheap, voff, &dv, &dvo);
    if (!r && (status || clevel || cbucket)) {
        r = dalloc_t(t, &dcl, n);
        if (!r) r = dalloc_t(t, &dseg, n);
    }
    if (!r) {
        IngestIn in{};
        in.n = n; in.krec = krec; in.koff = dko; in.vheap = dv; in.voff = dvo;
        in.verify_rehash = true; in.clevel_out = dcl; in.seg_out = dseg;
        r = ingest(t, in);
    }
    if (!r && dcl) {
        std::vector<uint32_t> cl(n), sg(n);
        r = d2h(t, cl.data(), dcl, n * 4);
        if (!r) r = d2h(t, sg.data(), dseg, n * 4);
        if (!r)
            for (uint64_t i = 0; i < n; i++) {
                if (status) status[i] = cl[i] ? ST_CORRUPTED : ST_OK;
                if (clevel) clevel[i] = cl[i];
                if (cbucket) cbucket[i] = cl[i] ? ((uint64_t)sg[i] >> (t->shift * (t->H + 1 - cl[i]))) : 0;
            }
    }
    dfree(t, krec); dfree(t, dko); dfree(t, dv); dfree(t, dvo); dfree(t, dcl); dfree(t, dseg);
    if (!r) CHK(tsync(t));
    return r;
}

static int insert_int64(st_tree *t, uint64_t n, const int64_t *keys, const uint8_t *vals, uint32_t vlen,
                        int on_device, hipStream_t producer, uint64_t *n_corrupted);
extern "C" int st_insert_int64(st_tree *t, uint64_t n, const int64_t *keys, const uint8_t *vals, uint32_t vlen,
                               int on_device, uint64_t *n_corrupted) {
    ENTER(t);
    return insert_int64(t, n, keys, vals, vlen, on_device, nullptr, n_corrupted);
}
extern "C" int st_insert_int64_dev(st_tree *t, uint64_t n, const int64_t *keys, const uint8_t *vals, uint32_t vlen,
                                   void *producer_stream, uint64_t *n_corrupted) {
    ENTER(t);
    return insert_int64(t, n, keys, vals, vlen, 1, (hipStream_t)producer_stream, n_corrupted);
}
static int insert_int64(st_tree *t, uint64_t n, const int64_t *keys, const uint8_t *vals, uint32_t vlen,
                        int on_device, hipStream_t producer, uint64_t *n_corrupted) {
    CHK(flush_overlay(t));   // the pages stay: a streaming batch may go to them (ingest)
    if (n_corrupted) *n_corrupted = 0;
    if (n == 0) return ST_OK;
    // device inputs: read only after the producer's writes (the call returns
    // after its last read of them, so the caller may reuse them at once)
    if (on_device) CHK(order_after(t, producer));
    const int64_t *dkeys = keys;
    const uint8_t *dvals = vals;
    int64_t *tk = nullptr;
    uint8_t *tv = nullptr, *krec = nullptr;
    uint64_t *dko = nullptr, *dvo = nullptr;
    uint32_t *dcl = nullptr;
    bool dcl_counted = false;
    int r = ST_OK;
    if (!on_device) {
        r = dalloc_t(t, &tk, n);
        if (!r) r = dalloc(t, (void **)&tv, (uint64_t)n * vlen + HEAP_SLACK);
        if (!r) r = h2d(t, tk, keys, n * 8);
        if (!r) r = h2d(t, tv, vals, (uint64_t)n * vlen);
        dkeys = tk;
        dvals = tv;
    }
    if (!r) r = dalloc(t, (void **)&krec, 9 * n + HEAP_SLACK);
    if (!r) r = dalloc_t(t, &dko, n + 1);
    if (!r) r = dalloc_t(t, &dvo, n + 1);
    if (!r && n_corrupted) r = dalloc_t(t, &dcl, n);
    if (!r) {
        TimedLaunch tl(t, "pack_int64");   // (it zeroes the key heap's slack too)
        hipLaunchKernelGGL(k_pack_int64, dim3(grid_for(n + 1)), dim3(256), 0, t->stream, dkeys, n, krec, dko, dvo, vlen,
                           (uint32_t)HEAP_SLACK);
        if (hipGetLastError() != hipSuccess) { r = ST_EDEVICE; g_err = "pack_int64 launch"; }
    }
    if (!r) {
        IngestIn in{};
        in.n = n; in.krec = krec; in.koff = dko; in.vheap = dvals; in.voff = dvo;
        in.verify_rehash = true; in.clevel_out = dcl; in.count_rejected = dcl != nullptr; in.int9 = true;
        r = ingest(t, in);
        if (!r && in.rejected_counted) { *n_corrupted = in.n_rejected; dcl_counted = true; }
    }
    if (!r && n_corrupted && dcl && !dcl_counted) {
        // count per-key rejections on the device (8 bytes back, not n statuses)
        if (hipMemsetAsync(t->cnt64, 0, 8, t->stream) != hipSuccess) { r = ST_EDEVICE; g_err = "memset"; }
        if (!r) {
            hipLaunchKernelGGL(k_count_nonzero, dim3(grid_for(n)), dim3(256), 0, t->stream, (const uint32_t *)dcl, n, t->cnt64);
            if (hipGetLastError() != hipSuccess) { r = ST_EDEVICE; g_err = "count_nonzero launch"; }
        }
        if (!r) r = d2h(t, t->pin, t->cnt64, 8);
        if (!r) *n_corrupted = t->pin[0];
    }
    dfree(t, tk); dfree(t, tv); dfree(t, krec); dfree(t, dko); dfree(t, dvo); dfree(t, dcl);
    if (!r) CHK(tsync(t));
    return r;
}

extern "C" int st_corrupt(st_tree *t, uint8_t ktype, const uint8_t *kbytes, uint32_t klen) {
    ENTER(t);
    FLUSH(t);
    uint64_t koff[2] = {0, klen};
    uint8_t *krec = nullptr, *dv = nullptr, *bop = nullptr;
    uint64_t *dko = nullptr, *dvo = nullptr;
    int r = upload_records(t, 1, &ktype, kbytes, koff, &krec, &dko);
    uint64_t voff[2] = {0, 0};
    uint8_t dummy = 0;
    if (!r) r = upload_values(t, 1, &dummy, voff, &dv, &dvo);
    if (!r) r = dalloc_t(t, &bop, 1);
    if (!r) {
        (void)hipMemsetAsync(bop, 1, 1, t->stream);
        IngestIn in{};
        in.n = 1; in.krec = krec; in.koff = dko; in.vheap = dv; in.voff = dvo; in.bop = bop;
        in.verify_rehash = false;
        r = ingest(t, in);
    }
    if (!r) r = ensure_erec(t);
    if (!r) {   // the segment it emptied now holds the [] record
        hipLaunchKernelGGL(k_erec_emptied, dim3(1), dim3(64), 0, t->stream, view(t), (const uint8_t *)krec,
                           (const uint64_t *)dko, t->erec);
        if (hipGetLastError() != hipSuccess) { g_err = "launch erec_emptied"; r = ST_EDEVICE; }
    }
    dfree(t, krec); dfree(t, dko); dfree(t, dv); dfree(t, dvo); dfree(t, bop);
    if (!r) CHK(tsync(t));
    return r;
}

extern "C" int st_store_segment(st_tree *t, uint64_t segment, uint64_t n, const uint8_t *ktype, const uint8_t *kheap,
                                const uint64_t *koff, const uint8_t *vheap, const uint64_t *voff) {
    ENTER(t);
    if (segment >= t->S) { g_err = "segment out of range"; return ST_EINVAL; }
    if (n == 0 && !t->partitioned && t->pg_slack >= 0 && (t->pg.on || t->n >= PAGED_DELETE_MIN)) {
        // an emptied segment (delete_node, the repair path) in the pages: no
        // CSR rewrite, the page just ends where it begins
        CHK(flush_overlay(t));
        if (!t->pg.on) CHK(pages_build(t, t->pg_slack, PageSums(0)));
        Scratch sc(t);
        uint64_t *dc = nullptr, c = 0;
        CHK(sc.alloc(&dc, 1));
        LAUNCH(t, "page_clear", k_page_clear, 1, 64, 0, t->pg.m, segment, dc);
        CHK(d2h(t, &c, dc, 8));
        t->n -= c;
        t->perm_valid = false;
        t->tiles_valid = false;
        t->tiles_wanted = false;
        t->fresh = false;
        CHK(set_erec(t, t->base[t->H + 1] + segment, 1));
        CHK(tsync(t));
        return ST_OK;
    }
    FLUSH(t);
    HostRecords hr;
    CHK(pack_records(n, ktype, kheap, koff, hr));
    for (uint64_t i = 1; i < n; i++)
        if (host_rec_cmp(hr.heap.data() + hr.off[i - 1], hr.off[i] - hr.off[i - 1], hr.heap.data() + hr.off[i],
                         hr.off[i + 1] - hr.off[i]) >= 0) {
            g_err = "segment content must be strictly ascending in key order";
            return ST_EINVAL;
        }
    uint8_t *krec = nullptr, *dv = nullptr, *rep = nullptr;
    uint64_t *dko = nullptr, *dvo = nullptr;
    uint32_t *dseg = nullptr;
    int r = ST_OK;
    uint64_t nn = n;
    // an empty store still needs one (erased) record to drive the replace
    std::vector<uint64_t> vz;
    if (n == 0) {
        uint8_t kt = ST_KEY_BINARY;
        uint64_t ko[2] = {0, 0};
        CHK(pack_records(1, &kt, nullptr, ko, hr));
        nn = 1;
    }
    r = dalloc(t, (void **)&krec, hr.heap.size());
    if (!r) r = dalloc_t(t, &dko, nn + 1);
    if (!r) r = h2d(t, krec, hr.heap.data(), hr.heap.size());
    if (!r) r = h2d(t, dko, hr.off.data(), (nn + 1) * 8);
    if (!r) {
        if (n) {
            r = upload_values(t, n, vheap, voff, &dv, &dvo);
        } else {
            uint64_t vo[2] = {0, 0};
            uint8_t z = 0;
            r = upload_values(t, 1, &z, vo, &dv, &dvo);
        }
    }
    uint8_t *bop = nullptr;
    if (!r) r = dalloc_t(t, &dseg, nn);
    if (!r) r = dalloc_t(t, &rep, t->S);
    if (!r && n == 0) {
        r = dalloc_t(t, &bop, 1);
        if (!r) (void)hipMemsetAsync(bop, 1, 1, t->stream);
    }
    if (!r) {
        std::vector<uint32_t> sg(nn, (uint32_t)segment);
        r = h2d(t, dseg, sg.data(), nn * 4);
        (void)hipMemsetAsync(rep, 0, t->S, t->stream);
        (void)hipMemsetAsync(rep + segment, 1, 1, t->stream);
        if (!r) {
            CHK(tsync(t));
            IngestIn in{};
            in.n = nn; in.krec = krec; in.koff = dko; in.vheap = dv; in.voff = dvo;
            in.seg_given = dseg; in.seg_replace = rep; in.bop = bop;
            in.verify_rehash = false;
            r = ingest(t, in);
        }
    }
    dfree(t, krec); dfree(t, dko); dfree(t, dv); dfree(t, dvo); dfree(t, dseg); dfree(t, rep); dfree(t, bop);
    if (!r) r = set_erec(t, t->base[t->H + 1] + segment, n == 0 ? 1 : 0);
    if (!r) CHK(tsync(t));
    return r;
}

static void set_entry_host(uint16_t &tag, uint4 &m, const uint8_t *h17) {
    tag = (uint16_t)(TAG_PRESENT | h17[0]);
    uint32_t w[4];
    for (int k = 0; k < 4; k++)
        w[k] = (uint32_t)h17[1 + 4 * k] | ((uint32_t)h17[2 + 4 * k] << 8) | ((uint32_t)h17[3 + 4 * k] << 16) |
               ((uint32_t)h17[4 + 4 * k] << 24);
    m = make_uint4(w[0], w[1], w[2], w[3]);
}

extern "C" int st_store_inner(st_tree *t, uint32_t level, uint64_t bucket, uint32_t n, const uint64_t *children,
                              const uint8_t *hashes17) {
    ENTER(t);
    if (level < 1 || level > t->H) { g_err = "inner level out of range"; return ST_EINVAL; }
    if (bucket >= t->base[level + 1] - t->base[level]) { g_err = "bucket out of range"; return ST_EINVAL; }
    std::vector<uint16_t> tags(t->W, 0);
    std::vector<uint4> md(t->W, make_uint4(0, 0, 0, 0));
    for (uint32_t i = 0; i < n; i++) {
        if (children[i] < bucket * t->W || children[i] >= (bucket + 1) * t->W || (i && children[i] <= children[i - 1])) {
            g_err = "child ids must be ascending and within the node's range";
            return ST_EINVAL;
        }
        const uint64_t j = children[i] - bucket * t->W;
        set_entry_host(tags[j], md[j], hashes17 + 17 * i);
    }
    const uint64_t c0 = t->base[level + 1] + bucket * t->W;
    CHK(h2d(t, t->tag + c0, tags.data(), t->W * 2));
    CHK(h2d(t, t->md5 + c0, md.data(), t->W * 16));
    CHK(set_erec(t, t->base[level] + bucket, n == 0 ? 1 : 0));
    CHK(tsync(t));
    t->fresh = false;
    return ST_OK;
}

extern "C" int st_delete_node(st_tree *t, uint32_t level, uint64_t bucket) {
    ENTER(t);
    if (level == 0) return st_store_top(t, nullptr, 0);
    if (level == t->H + 1) CHK(st_store_segment(t, bucket, 0, nullptr, nullptr, nullptr, nullptr, nullptr));
    else CHK(st_store_inner(t, level, bucket, 0, nullptr, nullptr));
    CHK(set_erec(t, t->base[level] + bucket, 0));   // no record at all
    CHK(tsync(t));
    return ST_OK;
}

extern "C" int st_store_top(st_tree *t, const uint8_t *hash17, int also_record) {
    ENTER(t);
    uint16_t tg = 0;
    uint4 m = make_uint4(0, 0, 0, 0);
    if (hash17) set_entry_host(tg, m, hash17);
    CHK(h2d(t, t->tag + 1, &tg, 2));
    CHK(h2d(t, t->md5 + 1, &m, 16));
    if (also_record) {
        CHK(h2d(t, t->tag, &tg, 2));
        CHK(h2d(t, t->md5, &m, 16));
    }
    CHK(tsync(t));
    t->fresh = false;
    return ST_OK;
}

extern "C" int st_set_record_top(st_tree *t, const uint8_t *hash17) {
    ENTER(t);
    uint16_t tg = 0;
    uint4 m = make_uint4(0, 0, 0, 0);
    if (hash17) set_entry_host(tg, m, hash17);
    CHK(h2d(t, t->tag, &tg, 2));
    CHK(h2d(t, t->md5, &m, 16));
    CHK(tsync(t));
    if (hash17) t->fresh = false;
    return ST_OK;
}

// ------------------------------------------------------------------ rehash / verify
extern "C" int st_rehash(st_tree *t, int upper) {
    ENTER_ANY(t);
    if (upper) CHK(alive(t));   // only a full rehash recomputes every level of a tree in error
    CHK(flush_overlay(t));
    // the pages stay (no fold) unless this rehash builds the tiles (from the
    // CSR): the upper levels, the rehash straight from the segments
    // (rehash_all) and the fused kernel over valid tiles do not read the CSR
    if (!upper && !t->tiles_valid && (t->tiles_wanted || t->partitioned)) CHK(pages_fold(t));
    if (upper && t->H == 0) { g_err = "rehash_upper at Height 0 does not terminate in the reference"; return ST_EINVAL; }
    if (t->partitioned && upper) {
        g_err = "a segment-range partition supports the full rehash (st_rehash upper = 0) only";
        return ST_EINVAL;
    }
    if (upper) CHK(rehash_levels(t, t->H, nullptr));
    else CHK(rehash_all(t, nullptr));
    CHK(erec_after_rehash(t));
    t->fresh = false;
    t->async_pending = true;
    if (t->poisoned) {   // a tree in error becomes readable again once this rehash completed cleanly
        CHK(tsync(t));
        t->poisoned = false;
    }
    return ST_OK;
}

// rehash/1 of n trees of one geometry (W == 16, H >= 3) as one batch: one
// launch of the fused rehash over the windows of every tree (workgroup =
// (tree, window)), each tree climbing to its own top hash.  The
// latency-bound level chains of the trees overlap one another's K1 (SURVEY
// §8d config 4: many ensembles per GPU).
extern "C" int st_rehash_group(st_tree **trees, uint32_t n) {
    if (n == 0) return ST_OK;
    for (uint32_t i = 0; i < n; i++)
        if (!trees[i]) { g_err = "NULL tree"; return ST_EINVAL; }
    GroupLock glk(trees, n);
    st_tree *t = trees[0];
    CHK(use_device(t));
    for (uint32_t i = 0; i < n; i++) {
        st_tree *u = trees[i];
        if (!fused_geometry(u) || u->S != t->S || u->device != t->device || u->partitioned) {
            g_err = "group rehash needs unpartitioned width-16 trees of one geometry (height 3..6) on one device";
            return ST_EINVAL;
        }
        for (uint32_t j = 0; j < i; j++)
            if (trees[j] == u) { g_err = "a tree appears twice in the group"; return ST_EINVAL; }
    }
    // each tree ready (tiles, counters) and its stream drained -- a tree with
    // nothing enqueued since its last synchronisation is not waited for
    // (hundreds of trees per group: the launch is not held up by idle syncs)
    for (uint32_t i = 0; i < n; i++) {
        st_tree *u = trees[i];
        const bool idle = !u->async_pending && u->tiles_valid && u->lvl_cnt && !u->pg.on && !u->ov_pending;
        CHK(flush_all(u));
        CHK(ensure_tiles(u));
        CHK(ensure_lvl_cnt(u));
        if (!idle || u->stream == t->stream) CHK(tsync(u));
    }
    // every window of every tree in ONE launch of the fused kernel (K1 +
    // levels + top per tree): the trees' tails overlap each other's K1
    std::vector<TreeTiles> h(n);
    for (uint32_t i = 0; i < n; i++) h[i] = launch_tiles(trees[i]);
    Scratch sc(t);
    TreeTiles *dtt = nullptr;
    CHK(sc.alloc(&dtt, n));
    HIPCHK(hipMemcpyAsync(dtt, h.data(), n * sizeof(TreeTiles), hipMemcpyHostToDevice, t->stream));
    const uint32_t nwin = (uint32_t)(t->S / 4096);
    const uint64_t nwg = (uint64_t)nwin * n;
    if (nwg > 0x7fffffffull) { g_err = "group too large for one launch"; return ST_EINVAL; }
    // 8 waves per window and LDS sized for the group's largest window: two
    // (dense trees) or three (sparse trees, <= 53 KB) windows per CU, so one
    // window's level chain overlaps other windows' K1
    uint32_t mh = 0;
    for (uint32_t i = 0; i < n; i++) mh = std::max(mh, trees[i]->mh_bytes);
    const uint32_t mhb = fused_mh_bytes(mh, nwin);
    static const int stamp = getenv("ST_LEVEL_STAMPS") ? atoi(getenv("ST_LEVEL_STAMPS")) : 0;
    if (!stamp) {
        LAUNCH(t, "rehash_group", (k_rehash_fused<false, true, 8>), (uint32_t)nwg, 512, fused_lds_bytes(mhb), view(t), h[0],
               (const TreeTiles *)dtt, nwin, (uint64_t)0, 1u, (uint64_t *)nullptr, mhb);
    } else {   // diagnostic: the per-window phase stamps (fused_stamps_report)
        uint64_t *st = nullptr;
        CHK(sc.alloc(&st, nwg * 32));
        HIPCHK(hipMemsetAsync(st, 0, nwg * 32 * 8, t->stream));
        LAUNCH(t, "rehash_group", (k_rehash_fused<true, true, 8>), (uint32_t)nwg, 512, fused_lds_bytes(mhb), view(t), h[0],
               (const TreeTiles *)dtt, nwin, (uint64_t)0, 1u, st, mhb);
        std::vector<uint64_t> hs(nwg * 32);
        HIPCHK(hipMemcpyAsync(hs.data(), st, hs.size() * 8, hipMemcpyDeviceToHost, t->stream));
        CHK(tsync(t));
        fused_stamps_report(hs, (uint32_t)nwg);
    }
    // the levels above level H: every tree's nodes of a level in one launch
    const DevTree d0 = view(t);
    for (uint32_t l = t->H - 1; l >= 1; l--)
        LAUNCH(t, "rehash_group", k_level16_group, grid_for((d0.base[l + 1] - d0.base[l]) * n, 64, 65536), 64,
               (size_t)level16_group_lds_bytes(), d0, (const TreeTiles *)dtt, n, l);
    // every tree's device-error word is checked (tsync): a tree whose climb
    // timed out is left in error (ST_EDEVICE returned), the others are clean
    int first = ST_OK;
    if (hipStreamSynchronize(t->stream) != hipSuccess) CHK(tsync(t));   // a launch fault: report it
    for (uint32_t i = 0; i < n; i++) {
        // every tree's stream was drained before the launch, which completed:
        // only the device-error words remain to be read
        const int r = synced(trees[i]);
        if (trees[i]->erec) {
            CHK(erec_after_rehash(trees[i]));
            trees[i]->async_pending = true;
        }
        if (r == ST_OK) {
            trees[i]->fresh = false;
            trees[i]->poisoned = false;
        } else if (first == ST_OK) {
            first = r;
        }
    }
    return first;
}

extern "C" int st_verify(st_tree *t, int upper, int *ok) {
    ENTER(t);
    FLUSH(t);
    const uint32_t maxd = upper ? t->H : t->H + 1;
    if (maxd == 0) { g_err = "verify_upper at Height 0 crashes in the reference"; return ST_EINVAL; }
    // one launch (k_verify_tree); the answer comes back through a word of the
    // tree's host-mapped block (zeroed here, ORed by a failing wave)
    const uint32_t lmax = maxd < t->H ? maxd : t->H;
    volatile uint32_t *fl = t->derr + 8;
    *fl = 0;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    if (lmax >= 1)   // the inner nodes: a 64-lane block, each lane's message staged in LDS
        LAUNCH(t, "verify_upper", k_verify_tree, grid_for(t->base[lmax + 1] - t->base[1], inner_block(t)), inner_block(t),
               inner_shmem(t), view(t), lmax, 0, t->derr_dev + 8);
    if (maxd == t->H + 1)   // the segments (verify/1): no LDS, full occupancy
        LAUNCH(t, "segment_verify", k_verify_tree, grid_for(t->S), 256, 0, view(t), 0u, 1, t->derr_dev + 8);
    CHK(tsync(t));
    *ok = __atomic_load_n(const_cast<uint32_t *>(fl), __ATOMIC_ACQUIRE) == 0;
    return ST_OK;
}

static void entry_to_h17(uint16_t tg, const uint4 &m, uint8_t *out) {
    out[0] = (uint8_t)(tg & 0xff);
    const uint32_t w[4] = {m.x, m.y, m.z, m.w};
    for (int k = 0; k < 16; k++) out[1 + k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
}

extern "C" int st_top_hash(st_tree *t, uint8_t out17[17], int *present) {
    ENTER(t);
    uint16_t tg = 0;
    uint4 m;
    HIPCHK(hipMemcpyAsync(&tg, t->tag, 2, hipMemcpyDeviceToHost, t->stream));
    HIPCHK(hipMemcpyAsync(&m, t->md5, 16, hipMemcpyDeviceToHost, t->stream));
    CHK(tsync(t));
    *present = (tg & TAG_PRESENT) ? 1 : 0;
    if (*present) entry_to_h17(tg, m, out17);
    return ST_OK;
}

extern "C" int st_set_partition(st_tree *t, uint64_t seg_lo, uint64_t seg_hi) {
    ENTER(t);
    FLUSH(t);
    if (seg_lo == 0 && seg_hi == t->S) { t->partitioned = false; return ST_OK; }
    const uint64_t l2 = t->W == 16 && t->H >= 4 ? t->S / 16 : 0;
    if (!l2 || seg_lo >= seg_hi || seg_hi > t->S || seg_lo % l2 || seg_hi % l2) {
        g_err = "partition needs width 16, height >= 4 and a range of whole level-2 subtrees";
        return ST_EINVAL;
    }
    if (t->n) { g_err = "set the partition before the first insert"; return ST_EINVAL; }
    t->partitioned = true;
    t->part_lo = seg_lo;
    t->part_hi = seg_hi;
    return ST_OK;
}

extern "C" int st_combine_upper(st_tree *t, const uint8_t *present16, const uint8_t *hashes17) {
    ENTER(t);
    if (t->W != 16 || t->H < 2) { g_err = "combine needs width 16 and height >= 2"; return ST_EINVAL; }
    uint16_t tg[16];
    uint4 m[16];
    for (int b = 0; b < 16; b++) {
        tg[b] = 0;
        m[b] = make_uint4(0, 0, 0, 0);
        if (present16[b]) set_entry_host(tg[b], m[b], hashes17 + 17 * b);
    }
    CHK(h2d(t, t->tag + t->base[2], tg, sizeof(tg)));
    CHK(h2d(t, t->md5 + t->base[2], m, sizeof(m)));
    DevTree d = view(t);
    LAUNCH(t, "level_rehash", k_upper16, 1, 256, (size_t)256 * lane_region_bytes(16), d, 1u, 1u, (const uint8_t *)nullptr);
    CHK(tsync(t));
    t->fresh = false;
    return ST_OK;
}

extern "C" int st_level_entries(st_tree *t, uint32_t level, uint8_t *present, uint8_t *hashes17) {
    ENTER(t);
    if (level < 1 || level > t->H + 1) { g_err = "level out of range"; return ST_EINVAL; }
    const uint64_t n = t->base[level + 1] - t->base[level];
    std::vector<uint16_t> tg(n);
    std::vector<uint4> m(n);
    HIPCHK(hipMemcpyAsync(tg.data(), t->tag + t->base[level], n * 2, hipMemcpyDeviceToHost, t->stream));
    HIPCHK(hipMemcpyAsync(m.data(), t->md5 + t->base[level], n * 16, hipMemcpyDeviceToHost, t->stream));
    CHK(tsync(t));
    for (uint64_t i = 0; i < n; i++) {
        present[i] = (tg[i] & TAG_PRESENT) ? 1 : 0;
        if (present[i]) entry_to_h17(tg[i], m[i], hashes17 + 17 * i);
        else memset(hashes17 + 17 * i, 0, 17);
    }
    return ST_OK;
}

// ------------------------------------------------------------------ result blocks
static st_result *new_result(uint64_t n) {
    st_result *r = (st_result *)calloc(1, sizeof(st_result));
    r->n = n;
    r->status = (int32_t *)calloc(n + 1, 4);
    r->clevel = (uint32_t *)calloc(n + 1, 4);
    r->cbucket = (uint64_t *)calloc(n + 1, 8);
    r->eoff = (uint64_t *)calloc(n + 1, 8);
    return r;
}

extern "C" void st_free_result(st_result *r) {
    if (!r) return;
    void *ps[] = {r->status, r->clevel, r->cbucket, r->eoff, r->child, r->hash17, r->ktype, r->koff, r->kheap,
                  r->aoff, r->aheap, r->boff, r->bheap, r->kind, r->seg};
    for (void *p : ps) free(p);
    free(r);
}

// Device entries (by index, ~0 = none) -> host key/value heaps of a result.
static int fetch_entries(st_tree *t, const uint64_t *d_idx, uint64_t n, st_result *res, bool keys) {
    DevTree d = view(t);
    Scratch sc(t);   // every device temporary is freed on every return path
    uint64_t *kl = nullptr, *vl = nullptr, *ko = nullptr, *vo = nullptr;
    uint8_t *kh = nullptr, *vh = nullptr;
    CHK(sc.alloc(&kl, n + 1));
    CHK(sc.alloc(&vl, n + 1));
    CHK(sc.alloc(&ko, n + 1));
    CHK(sc.alloc(&vo, n + 1));
    LAUNCH(t, "entry_lengths", k_entry_lengths, grid_for(n + 1), 256, 0, d, d_idx, n, kl, vl);
    CHK(exclusive_scan<uint64_t>(t, kl, ko, n + 1));
    CHK(exclusive_scan<uint64_t>(t, vl, vo, n + 1));
    res->koff = (uint64_t *)calloc(n + 1, 8);
    res->aoff = (uint64_t *)calloc(n + 1, 8);
    HIPCHK(hipMemcpyAsync(res->koff, ko, (n + 1) * 8, hipMemcpyDeviceToHost, t->stream));
    CHK(d2h(t, res->aoff, vo, (n + 1) * 8));
    const uint64_t kb = res->koff[n], vb = res->aoff[n];
    CHK(sc.bytes(&kh, kb + 16));
    CHK(sc.bytes(&vh, vb + 16));
    LAUNCH(t, "entry_gather", k_entry_gather, grid_for(n), 256, 0, d, d_idx, n, (const uint64_t *)ko, kh,
           (const uint64_t *)vo, vh);
    res->kheap = (uint8_t *)malloc(kb + 1);
    res->aheap = (uint8_t *)malloc(vb + 1);
    if (kb) HIPCHK(hipMemcpyAsync(res->kheap, kh, kb, hipMemcpyDeviceToHost, t->stream));
    CHK(d2h(t, res->aheap, vh, vb));
    CHK(tsync(t));
    (void)keys;
    return ST_OK;
}

// Convert device key records (tag + payload') of a result into (ktype, ensure_binary bytes).
static void records_to_keys(st_result *res, uint64_t n) {
    res->ktype = (uint8_t *)calloc(n + 1, 1);
    uint64_t *nk = (uint64_t *)calloc(n + 1, 8);
    uint8_t *nh = (uint8_t *)malloc(res->koff[n] + 1);
    uint64_t o = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t *p = res->kheap + res->koff[i];
        const uint64_t len = res->koff[i + 1] - res->koff[i];
        nk[i] = o;
        if (len == 0) continue;
        if (krec_is_term(p, len)) {   // the caller's term_to_binary bytes
            uint64_t ea, sa;
            uint32_t el, sl;
            krec_term_parts(p, len, &ea, &el, &sa, &sl);
            res->ktype[i] = ST_KEY_TERM;
            memcpy(nh + o, p + ea, el);
            o += el;
            continue;
        }
        res->ktype[i] = p[0] == KEYTAG_INT ? ST_KEY_INT : (p[0] == KEYTAG_ATOM ? ST_KEY_ATOM : ST_KEY_BINARY);
        memcpy(nh + o, p + 1, len - 1);
        if (p[0] == KEYTAG_INT) nh[o] ^= 0x80;
        o += len - 1;
    }
    nk[n] = o;
    free(res->koff);
    free(res->kheap);
    res->koff = nk;
    res->kheap = nh;
}

// Verify the root->target paths (targets at level L, device list) and
// return the first failing level per target (device, n).
static int verify_paths(st_tree *t, uint32_t L, const uint64_t *d_targets, uint64_t n, uint32_t *d_status) {
    DevTree d = view(t);
    HIPCHK(hipMemsetAsync(t->mark, 0, t->nslots, t->stream));
    LAUNCH(t, "mark_paths", k_mark_paths, grid_for(n), 256, 0, d, L, (const uint64_t *)nullptr, d_targets, n, t->mark);
    CHK(verify_marked(t, L));
    LAUNCH(t, "path_status", k_path_status, grid_for(n), 256, 0, d, L, (const uint64_t *)nullptr, d_targets, n,
           (const uint8_t *)t->ok, (uint8_t *)nullptr, d_status);
    return ST_OK;
}

__global__ void k_u32_to_u64(const uint32_t *a, uint64_t n, uint64_t *b) {
    for (uint64_t i = gtid(); i < n; i += gstride()) b[i] = a[i];
}

// get/2 of ONE key (synctree.erl:213-227) into caller buffers: ST_OK (value
// bytes in vout, *vlen; a value longer than vcap sets *vlen and returns
// ST_EINVAL), ST_NOTFOUND, or ST_CORRUPTED with (clevel, cbucket).  The NIF's
// get/2 path: no result block.
extern "C" int st_get1(st_tree *t, uint8_t ktype, const uint8_t *kbytes, uint32_t klen, uint8_t *vout, uint32_t vcap,
                       uint32_t *vlen, uint32_t *clevel, uint64_t *cbucket) {
    ENTER(t);
    const uint64_t koff[2] = {0, klen};
    HostRecords hr;
    CHK(pack_records(1, &ktype, kbytes, koff, hr));
    int served = 0;
    CHK(small_call(t, 0, 1, hr, nullptr, nullptr, &served));
    int32_t st;
    if (served) {
        const SmallRes &so = t->sres;
        st = so.status[0];
        *clevel = so.clevel[0];
        *cbucket = so.cbucket[0];
        *vlen = so.voff[1];
        if (st == ST_OK) {
            if (*vlen > vcap) { g_err = "value longer than the buffer"; return ST_EINVAL; }
            memcpy(vout, t->sout->vbytes, *vlen);
        }
        return st;
    }
    st_result *res = nullptr;
    CHK(st_get_batch(t, 1, &ktype, kbytes, koff, &res));
    st = res->status[0];
    *clevel = res->clevel ? res->clevel[0] : 0;
    *cbucket = res->cbucket ? res->cbucket[0] : 0;
    *vlen = 0;
    if (st == ST_OK) {
        const uint64_t e = res->eoff[0];
        *vlen = (uint32_t)(res->aoff[e + 1] - res->aoff[e]);
        if (*vlen > vcap) { st_free_result(res); g_err = "value longer than the buffer"; return ST_EINVAL; }
        memcpy(vout, res->aheap + res->aoff[e], *vlen);
    }
    st_free_result(res);
    return st;
}

// insert/3 of ONE key (synctree.erl:189-209): ST_OK or ST_CORRUPTED with
// (clevel, cbucket).  The NIF's insert/3 and riak_ensemble_peer_tree's
// do_insert (peer_tree.erl:224-234).
extern "C" int st_insert1(st_tree *t, uint8_t ktype, const uint8_t *kbytes, uint32_t klen, const uint8_t *value,
                          uint32_t vlen, uint32_t *clevel, uint64_t *cbucket) {
    ENTER(t);
    const uint64_t koff[2] = {0, klen}, voff[2] = {0, vlen};
    int32_t st = ST_OK;
    CHK(st_insert_batch(t, 1, &ktype, kbytes, koff, value, voff, &st, clevel, cbucket));
    return st;
}

extern "C" int st_get_batch(st_tree *t, uint64_t n, const uint8_t *ktype, const uint8_t *kheap, const uint64_t *koff,
                            st_result **out) {
    ENTER(t);
    *out = nullptr;
    if (n >= 1 && n <= SB_MAX) {   // per-key latency path: one launch, one sync
        HostRecords hr;
        CHK(pack_records(n, ktype, kheap, koff, hr));
        int served = 0;
        CHK(small_call(t, 0, n, hr, nullptr, nullptr, &served));
        if (served) {
            const SmallRes &so = t->sres;
            st_result *res = new_result(n);
            res->n_entries = n;
            res->koff = (uint64_t *)calloc(n + 1, 8);
            res->aoff = (uint64_t *)calloc(n + 1, 8);
            res->ktype = (uint8_t *)calloc(n + 1, 1);
            res->kheap = (uint8_t *)malloc(1);
            res->aheap = (uint8_t *)malloc(so.voff[n] + 1);
            for (uint64_t i = 0; i < n; i++) {
                res->status[i] = so.status[i];
                res->clevel[i] = so.clevel[i];
                res->cbucket[i] = so.cbucket[i];
                res->eoff[i + 1] = i + 1;
                res->aoff[i + 1] = so.voff[i + 1];
            }
            memcpy(res->aheap, t->sout->vbytes, so.voff[n]);
            *out = res;
            return ST_OK;
        }
    }
    FLUSH(t);
    st_result *res = new_result(n);
    int present = 0;
    uint8_t top[17];
    CHK(st_top_hash(t, top, &present));
    if (!present || n == 0) {   // get/2: undefined top => notfound (synctree.erl:216-218)
        for (uint64_t i = 0; i < n; i++) res->status[i] = ST_NOTFOUND;
        res->koff = (uint64_t *)calloc(n + 1, 8);
        res->aoff = (uint64_t *)calloc(n + 1, 8);
        res->kheap = (uint8_t *)malloc(1);
        res->aheap = (uint8_t *)malloc(1);
        res->ktype = (uint8_t *)calloc(n + 1, 1);
        *out = res;
        return ST_OK;
    }
    uint8_t *krec = nullptr;
    uint64_t *dko = nullptr, *tg64 = nullptr, *found = nullptr;
    uint32_t *seg = nullptr, *pst = nullptr;
    int r = upload_records(t, n, ktype, kheap, koff, &krec, &dko);
    if (!r) r = dalloc_t(t, &seg, n);
    if (!r) r = dalloc_t(t, &tg64, n);
    if (!r) r = dalloc_t(t, &pst, n);
    if (!r) r = dalloc_t(t, &found, n);
    DevTree d = view(t);
    auto launched = [&](const char *what) {
        const hipError_t e = hipGetLastError();
        if (e == hipSuccess) return ST_OK;
        g_err = std::string("launch ") + what + ": " + hipGetErrorString(e);
        return ST_EDEVICE;
    };
    if (!r) {
        hipLaunchKernelGGL(k_key_segment, dim3(grid_for(n)), dim3(256), 0, t->stream, krec, dko, n, t->S - 1, seg);
        r = launched("key_segment");
    }
    if (!r) {
        hipLaunchKernelGGL(k_u32_to_u64, dim3(grid_for(n)), dim3(256), 0, t->stream, seg, n, tg64);
        r = launched("u32_to_u64");
    }
    if (!r) r = verify_paths(t, t->H + 1, tg64, n, pst);
    if (!r) {
        BatchView bv{krec, dko};
        hipLaunchKernelGGL(k_lookup, dim3(grid_for(n)), dim3(256), 0, t->stream, d, bv, seg, n, found);
        r = launched("lookup");
    }
    if (!r) {
        std::vector<uint32_t> ps(n), sg(n);
        std::vector<uint64_t> fd(n);
        // one sync for the three per-key outputs
        hipError_t e = hipMemcpyAsync(ps.data(), pst, n * 4, hipMemcpyDeviceToHost, t->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(sg.data(), seg, n * 4, hipMemcpyDeviceToHost, t->stream);
        if (e != hipSuccess) {
            g_err = std::string("hipMemcpyAsync: ") + hipGetErrorString(e);
            r = ST_EDEVICE;
        }
        if (!r) r = d2h(t, fd.data(), found, n * 8);
        if (!r) {
            for (uint64_t i = 0; i < n; i++) {
                if (ps[i]) {
                    res->status[i] = ST_CORRUPTED;
                    res->clevel[i] = ps[i];
                    res->cbucket[i] = (uint64_t)sg[i] >> (t->shift * (t->H + 1 - ps[i]));
                    fd[i] = ~0ull;
                } else {
                    res->status[i] = fd[i] == ~0ull ? ST_NOTFOUND : ST_OK;
                }
                res->eoff[i + 1] = i + 1;   // entry i <-> key i (value valid iff ST_OK)
            }
            res->n_entries = n;
            r = h2d(t, found, fd.data(), n * 8);
            if (!r) r = fetch_entries(t, found, n, res, false);
            if (!r) records_to_keys(res, n);
        }
    }
    dfree(t, krec); dfree(t, dko); dfree(t, seg); dfree(t, tg64); dfree(t, pst); dfree(t, found);
    if (r) { st_free_result(res); return r; }
    CHK(tsync(t));
    *out = res;
    return ST_OK;
}

__global__ void k_gather_children(DevTree t, uint32_t level, const uint64_t *targets, uint64_t n, uint16_t *tags,
                                  uint4 *md) {
    const uint64_t total = n * t.W;
    for (uint64_t i = gtid(); i < total; i += gstride()) {
        const uint64_t k = i / t.W, j = i % t.W;
        const uint64_t slot = t.base[level + 1] + targets[k] * t.W + j;
        tags[i] = t.tag[slot];
        md[i] = t.md5[slot];
    }
}

__global__ void k_target_counts(DevTree t, const uint64_t *targets, uint64_t n, const uint32_t *status, uint64_t *cnt) {
    for (uint64_t i = gtid(); i <= n; i += gstride()) {
        if (i == n) { cnt[i] = 0; break; }
        const uint64_t s = targets[i];
        cnt[i] = status[i] ? 0 : t.seg_end[s] - t.seg_off[s];
    }
}

__global__ void k_expand_ranges(DevTree t, const uint64_t *targets, uint64_t n, const uint32_t *status,
                                const uint64_t *eoff, uint64_t *idx) {
    for (uint64_t i = gtid(); i < n; i += gstride()) {
        if (status[i]) continue;
        const uint64_t s = targets[i], e0 = t.seg_off[s];
        const uint64_t m = eoff[i + 1] - eoff[i];
        for (uint64_t k = 0; k < m; k++) idx[eoff[i] + k] = e0 + k;
    }
}

static int node_images(st_tree *t, uint32_t level, uint64_t n, const uint64_t *buckets, st_result **out, bool verify) {
    *out = nullptr;
    if (level < 1 || level > t->H + 1) { g_err = "level out of range (level 0 is answered from the top hash)"; return ST_EINVAL; }
    const uint64_t lsize = t->base[level + 1] - t->base[level];
    for (uint64_t i = 0; i < n; i++)
        if (buckets[i] >= lsize) { g_err = "bucket out of range"; return ST_EINVAL; }
    st_result *res = new_result(n);
    uint64_t *dt = nullptr, *cnt = nullptr, *eo = nullptr, *idx = nullptr;
    uint32_t *pst = nullptr;
    uint16_t *tg = nullptr;
    uint4 *md = nullptr;
    DevTree d = view(t);
    int r = dalloc_t(t, &dt, n ? n : 1);
    if (!r) r = dalloc_t(t, &pst, n ? n : 1);
    if (!r) r = h2d(t, dt, buckets, n * 8);
    if (!r && n) {
        if (verify) r = verify_paths(t, level, dt, n, pst);
        else HIPCHK(hipMemsetAsync(pst, 0, n * 4, t->stream));
    }
    std::vector<uint32_t> ps(n);
    if (!r) r = d2h(t, ps.data(), pst, n * 4);
    for (uint64_t i = 0; i < n && !r; i++)
        if (ps[i]) {
            res->status[i] = ST_CORRUPTED;
            res->clevel[i] = ps[i];
            res->cbucket[i] = buckets[i] >> (t->shift * (level - ps[i]));
        }
    if (!r && level <= t->H) {
        const uint64_t m = n * t->W;
        r = dalloc_t(t, &tg, m ? m : 1);
        if (!r) r = dalloc_t(t, &md, m ? m : 1);
        if (!r && m) hipLaunchKernelGGL(k_gather_children, dim3(grid_for(m)), dim3(256), 0, t->stream, d, level, dt, n, tg, md);
        std::vector<uint16_t> htg(m);
        std::vector<uint4> hmd(m);
        if (!r) r = d2h(t, htg.data(), tg, m * 2);
        if (!r) r = d2h(t, hmd.data(), md, m * 16);
        if (!r) {
            uint64_t tot = 0;
            for (uint64_t i = 0; i < n; i++) {
                res->eoff[i] = tot;
                if (!ps[i])
                    for (uint64_t j = 0; j < t->W; j++) tot += (htg[i * t->W + j] & TAG_PRESENT) != 0;
            }
            res->eoff[n] = tot;
            res->n_entries = tot;
            res->child = (uint64_t *)calloc(tot + 1, 8);
            res->hash17 = (uint8_t *)calloc(tot + 1, 17);
            uint64_t e = 0;
            for (uint64_t i = 0; i < n; i++) {
                if (ps[i]) continue;
                for (uint64_t j = 0; j < t->W; j++) {
                    const uint64_t q = i * t->W + j;
                    if (!(htg[q] & TAG_PRESENT)) continue;
                    res->child[e] = buckets[i] * t->W + j;
                    entry_to_h17(htg[q], hmd[q], res->hash17 + 17 * e);
                    e++;
                }
            }
        }
    } else if (!r) {
        r = dalloc_t(t, &cnt, n + 1);
        if (!r) r = dalloc_t(t, &eo, n + 1);
        if (!r) hipLaunchKernelGGL(k_target_counts, dim3(grid_for(n + 1)), dim3(256), 0, t->stream, d, dt, n, pst, cnt);
        if (!r) r = exclusive_scan<uint64_t>(t, cnt, eo, n + 1);
        if (!r) r = d2h(t, res->eoff, eo, (n + 1) * 8);
        const uint64_t tot = r ? 0 : res->eoff[n];
        res->n_entries = tot;
        if (!r) r = dalloc_t(t, &idx, tot + 1);
        if (!r && n) hipLaunchKernelGGL(k_expand_ranges, dim3(grid_for(n)), dim3(256), 0, t->stream, d, dt, n, pst, eo, idx);
        if (!r) r = fetch_entries(t, idx, tot, res, true);
        if (!r) records_to_keys(res, tot);
    }
    dfree(t, dt); dfree(t, pst); dfree(t, tg); dfree(t, md); dfree(t, cnt); dfree(t, eo); dfree(t, idx);
    if (r) { st_free_result(res); return r; }
    CHK(tsync(t));
    *out = res;
    return ST_OK;
}

extern "C" int st_exchange_get_batch(st_tree *t, uint32_t level, uint64_t n, const uint64_t *buckets, st_result **out) {
    ENTER(t);
    FLUSH(t);
    return node_images(t, level, n, buckets, out, true);
}

extern "C" int st_fetch_batch(st_tree *t, uint32_t level, uint64_t n, const uint64_t *buckets, st_result **out) {
    ENTER(t);
    FLUSH(t);
    if (level == 0) {
        st_result *res = new_result(n);
        uint16_t tg = 0;
        uint4 m;
        HIPCHK(hipMemcpyAsync(&tg, t->tag + 1, 2, hipMemcpyDeviceToHost, t->stream));
        HIPCHK(hipMemcpyAsync(&m, t->md5 + 1, 16, hipMemcpyDeviceToHost, t->stream));
        CHK(tsync(t));
        const uint64_t e = (tg & TAG_PRESENT) ? 1 : 0;
        res->child = (uint64_t *)calloc(n + 1, 8);
        res->hash17 = (uint8_t *)calloc(n + 1, 17);
        for (uint64_t i = 0; i < n; i++) {
            res->eoff[i + 1] = res->eoff[i] + e;
            if (e) entry_to_h17(tg, m, res->hash17 + 17 * i);
        }
        res->n_entries = res->eoff[n];
        *out = res;
        return ST_OK;
    }
    return node_images(t, level, n, buckets, out, false);
}

extern "C" int st_segment_of_batch(st_tree *t, uint64_t n, const uint8_t *ktype, const uint8_t *kheap,
                                   const uint64_t *koff, uint64_t *segments_out) {
    ENTER(t);
    if (n == 0) return ST_OK;
    uint8_t *krec = nullptr;
    uint64_t *dko = nullptr;
    uint32_t *seg = nullptr;
    int r = upload_records(t, n, ktype, kheap, koff, &krec, &dko);
    if (!r) r = dalloc_t(t, &seg, n);
    std::vector<uint32_t> sg(n);
    if (!r) {
        hipLaunchKernelGGL(k_key_segment, dim3(grid_for(n)), dim3(256), 0, t->stream, krec, dko, n, t->S - 1, seg);
        r = d2h(t, sg.data(), seg, n * 4);
    }
    for (uint64_t i = 0; i < n && !r; i++) segments_out[i] = sg[i];
    dfree(t, krec); dfree(t, dko); dfree(t, seg);
    return r;
}

// ------------------------------------------------------------------ compare (K3)
static uint32_t cmp_slice(const st_tree *t) { return cmp_slice_bytes((uint32_t)t->W); }
static const uint32_t CMP_WPG = 4;   // waves per compare-walk workgroup

static int ensure_cmp_work(st_tree *t) {
    CmpWork &w = t->cw;
    if (w.wcnt) return ST_OK;
    const uint32_t per_cu = std::max<uint32_t>(1, (160 * 1024) / (CMP_WPG * cmp_slice(t)));
    w.nw = std::min<uint32_t>((uint32_t)std::max(1, t->ncu) * per_cu * CMP_WPG, 4096);   // <= 64 count words per lane
    CHK(dalloc_t(t, &w.wcnt, w.nw));
    CHK(dalloc_t(t, &w.wbytes, w.nw));
    CHK(dalloc_t(t, &w.wst, (uint64_t)w.nw * ST_STATW));
    CHK(dalloc_t(t, &w.werr, 2));
    w.epoch = 0;   // the first compare resets the words (epoch wrap)
    if (hipHostMalloc((void **)&w.res, 4 * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
        w.res = nullptr;
        g_err = "hipHostMalloc failed";
        return ST_EDEVICE;
    }
    HIPCHK(hipHostGetDevicePointer((void **)&w.res_dev, w.res, 0));
    return ST_OK;
}

// record buffer >= cap records, scratch >= nw * R records
static int grow_records(st_tree *t, uint64_t cap, uint64_t R) {
    CmpWork &w = t->cw;
    if (cap > w.cap) {
        dfree(t, w.rec);
        w.rec = nullptr;
        w.cap = 0;
        cap += cap / 4 + 1024;
        CHK(dalloc_t(t, &w.rec, cap));
        w.cap = cap;
    }
    if (R > w.R) {
        dfree(t, w.scratch);
        w.scratch = nullptr;
        w.R = 0;
        R += R / 4 + 64;
        CHK(dalloc_t(t, &w.scratch, (uint64_t)w.nw * R));
        w.R = R;
    }
    return ST_OK;
}

struct CompareOut {
    uint64_t n = 0;
    const DiffRec *rec = nullptr;   // device, in the local tree's compare workspace
};

// K3: the compare walk (frontier, verification, merge-join: one launch) and
// the gather of its per-wave records; ONE host round trip (a second compare
// when the record buffers have to grow).  A partitioned pair compares its own
// segment range only (same partition on both sides).
static int compare_core(st_tree *A, st_tree *B, int filter, CompareOut &co, uint32_t *clevel, uint64_t *cbucket,
                        int *cside, int *status) {
    *status = ST_OK;
    co = CompareOut();
    if (A->W != B->W || A->S != B->S) { g_err = "trees of different shape"; return ST_EINVAL; }
    if (filter < 0 || filter > 2) { g_err = "both local_only and remote_only (case_clause)"; return ST_EINVAL; }
    if (A->device != B->device) { g_err = "trees on different devices"; return ST_EINVAL; }
    if (A->partitioned != B->partitioned || (A->partitioned && (A->part_lo != B->part_lo || A->part_hi != B->part_hi))) {
        g_err = "compare needs both trees partitioned alike";
        return ST_EINVAL;
    }
    st_tree *t = A;   // work is enqueued on the local tree's stream
    // the remote's own pending work (an st_rehash it did not wait for) first;
    // an idle remote stream is not synchronised (a host round trip per compare)
    if (B->stream != A->stream && B->async_pending) CHK(tsync(B));
    CHK(ensure_cmp_work(t));
    CmpWork &w = t->cw;
    CHK(grow_records(t, 4096, 64));
    DevTree da = view(A), db = view(B);
    uint64_t lo2 = 0, hi2 = ~0ull;
    if (A->partitioned) {
        const uint64_t per2 = A->S / A->W;   // segments under one level-2 bucket
        lo2 = A->part_lo / per2;
        hi2 = A->part_hi / per2;
    }
    const uint32_t slice = cmp_slice(t);
    for (int attempt = 0; attempt < 2; attempt++) {
        static const int stamp = getenv("ST_CMP_STAMPS") ? atoi(getenv("ST_CMP_STAMPS")) : 0;
        Scratch sc(t);
        uint64_t *stamps = nullptr;
        if (stamp) {   // diagnostic: per-wave phase stamps (100 MHz) to stderr
            CHK(sc.alloc(&stamps, (uint64_t)w.nw * 16));
            HIPCHK(hipMemsetAsync(stamps, 0, (uint64_t)w.nw * 128, t->stream));
        }
        if (++w.epoch > 0xFFFFu || w.epoch == 1) {   // the words' epochs wrap: start them afresh
            w.epoch = 1;
            HIPCHK(hipMemsetAsync(w.wcnt, 0, (uint64_t)w.nw * 8, t->stream));
            HIPCHK(hipMemsetAsync(w.werr, 0xFF, 8, t->stream));
            HIPCHK(hipMemsetAsync(w.werr + 1, 0, 8, t->stream));
        }
        w.res[0] = w.res[1] = w.res[2] = w.res[3] = 0;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        A->reads_remote = true;   // until the walk's completion word is seen
        LAUNCH(t, "cmp_walk", k_cmp_walk, (w.nw + CMP_WPG - 1) / CMP_WPG, 64 * CMP_WPG, (size_t)CMP_WPG * slice, da, db,
               filter, lo2, hi2, w.nw, slice, w.scratch, w.R, w.wcnt, w.wst, w.wbytes, w.werr, w.epoch, w.rec, w.cap,
               w.res_dev, t->derr_dev, stamps);
        if (stamp) {
            std::vector<uint64_t> h((uint64_t)w.nw * 16);
            HIPCHK(hipMemcpyAsync(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost, t->stream));
            CHK(tsync(t));
            uint64_t t0 = ~0ull;
            for (uint32_t x = 0; x < w.nw; x++) t0 = std::min(t0, h[x * 16]);
            static const char *nm[16] = {"start", "levels", "children", "verify", "merge", "end", "", "staged",
                                         "flush", "inner", "values", "placed", "m.offs", "m.bytes", "m.merged", "m.pfx"};
            for (int k = 0; k < 16; k++) {
                if (k == 6) continue;
                std::vector<double> v;
                for (uint32_t x = 0; x < w.nw; x++)
                    if (h[x * 16 + k]) v.push_back((h[x * 16 + k] - t0) / 100.0);
                if (v.empty()) continue;
                std::sort(v.begin(), v.end());
                fprintf(stderr, "cmp stamp %-9s n=%4zu min %7.2f med %7.2f p90 %7.2f max %7.2f us\n", nm[k], v.size(), v[0],
                        v[v.size() / 2], v[v.size() * 9 / 10], v.back());
            }
            std::vector<uint32_t> ord(w.nw);   // the slowest waves: visited segments and phase ends
            for (uint32_t x = 0; x < w.nw; x++) ord[x] = x;
            std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return h[a * 16 + 4] > h[b * 16 + 4]; });
            for (uint32_t r = 0; r < 6 && r < w.nw; r++) {
                const uint32_t x = ord[r];
                fprintf(stderr, "cmp slow wave %4u segs %3llu verify %7.2f merge %7.2f end %7.2f us\n", x,
                        (unsigned long long)h[x * 16 + 6], (h[x * 16 + 3] - t0) / 100.0, (h[x * 16 + 4] - t0) / 100.0,
                        (h[x * 16 + 5] - t0) / 100.0);
            }
        }
        CHK(wait_mapped(t, reinterpret_cast<volatile uint32_t *>(&w.res[3])));
        A->reads_remote = false;   // wave 0 writes it after every wave's count: every read of B has completed
        const uint64_t ntot = w.res[0], need = w.res[1], e = w.res[2];
        if (e != ~0ull) {
            *status = ST_CORRUPTED;
            *clevel = (uint32_t)(e >> 56);
            *cbucket = (e & ((1ull << 56) - 1)) >> 1;
            *cside = (int)(e & 1);
            return ST_OK;
        }
        if (ntot <= w.cap && need <= w.R) {
            co.n = ntot;
            co.rec = w.rec;
            return ST_OK;
        }
        CHK(grow_records(t, ntot, need));   // first compare with this many records
    }
    g_err = "compare record buffer did not converge";
    return ST_EDEVICE;
}

extern "C" int st_compare_device(st_tree *local, st_tree *remote, int filter, uint64_t *n_diffs, uint32_t *clevel,
                                 uint64_t *cbucket, int *cside) {
    ENTER_PAIR(local, remote);
    CHK(flush_all(local));
    CHK(flush_all(remote));
    CompareOut co;
    int status = ST_OK;
    CHK(compare_core(local, remote, filter, co, clevel, cbucket, cside, &status));
    *n_diffs = co.n;
    return status;
}

// Exchange diff application (riak_ensemble_exchange.erl:71-97): compare the
// local tree against the remote one (K3, default options), then insert into
// the local tree, with insert/3 semantics, every remote value the exchange
// would take (k_diff_apply_*), as ONE device batch instead of one
// peer_tree:insert gen_server call per diff.
static int exchange_core(st_tree *local, st_tree *remote, bool apply, uint64_t *n_diffs, uint64_t *n_applied,
                         uint64_t *n_rejected, int *crashed, uint32_t *clevel, uint64_t *cbucket, int *cside) {
    ENTER_PAIR(local, remote);
    CHK(flush_all(local));
    CHK(flush_all(remote));
    *n_diffs = 0;
    *n_applied = 0;
    *n_rejected = 0;
    *crashed = 0;
    CompareOut co;
    int status = ST_OK;
    CHK(compare_core(local, remote, ST_FILTER_ALL, co, clevel, cbucket, cside, &status));
    *n_diffs = co.n;
    if (status != ST_OK || co.n == 0) return status;
    st_tree *t = local;
    const uint64_t n = co.n;
    DevTree da = view(local), db = view(remote);
    Scratch sc(t);
    uint8_t *take = nullptr, *kh = nullptr, *vh = nullptr;
    unsigned long long *fb = nullptr;
    uint64_t *one = nullptr, *kl = nullptr, *vl = nullptr, *pos = nullptr, *ko = nullptr, *vo = nullptr, *bko = nullptr,
             *bvo = nullptr;
    uint32_t *dcl = nullptr;
    CHK(sc.alloc(&take, n));
    CHK(sc.alloc(&fb, 1));
    CHK(sc.alloc(&one, n + 1));
    CHK(sc.alloc(&kl, n + 1));
    CHK(sc.alloc(&vl, n + 1));
    CHK(sc.alloc(&pos, n + 1));
    CHK(sc.alloc(&ko, n + 1));
    CHK(sc.alloc(&vo, n + 1));
    HIPCHK(hipMemsetAsync(fb, 0xff, 8, t->stream));
    t->reads_remote = true;
    LAUNCH(t, "diff_apply", k_diff_apply_select, grid_for(n), 256, 0, da, db, co.rec, n, take, fb);
    LAUNCH(t, "diff_apply", k_diff_apply_lengths, grid_for(n + 1), 256, 0, db, co.rec, n, (const uint8_t *)take,
           (const unsigned long long *)fb, one, kl, vl);
    CHK(exclusive_scan<uint64_t>(t, one, pos, n + 1));
    CHK(exclusive_scan<uint64_t>(t, kl, ko, n + 1));
    CHK(exclusive_scan<uint64_t>(t, vl, vo, n + 1));
    HIPCHK(hipMemcpyAsync(t->pin, pos + n, 8, hipMemcpyDeviceToHost, t->stream));
    HIPCHK(hipMemcpyAsync(t->pin + 1, ko + n, 8, hipMemcpyDeviceToHost, t->stream));
    HIPCHK(hipMemcpyAsync(t->pin + 2, vo + n, 8, hipMemcpyDeviceToHost, t->stream));
    HIPCHK(hipMemcpyAsync(t->pin + 3, fb, 8, hipMemcpyDeviceToHost, t->stream));
    CHK(tsync(t));
    const uint64_t m = t->pin[0], kb = t->pin[1], vb = t->pin[2];
    *crashed = t->pin[3] != ~0ull ? 1 : 0;
    if (!apply) {
        *n_applied = m;   // what an apply would take
        return ST_OK;
    }
    if (m) {
        CHK(sc.bytes(&kh, kb + HEAP_SLACK));
        CHK(sc.bytes(&vh, vb + HEAP_SLACK));
        CHK(sc.alloc(&bko, m + 1));
        CHK(sc.alloc(&bvo, m + 1));
        CHK(sc.alloc(&dcl, m));
        t->reads_remote = true;
        LAUNCH(t, "diff_apply", k_diff_apply_gather, grid_for(n + 1), 256, 0, db, co.rec, n, (const uint64_t *)pos,
               (const uint64_t *)ko, (const uint64_t *)vo, kh, bko, vh, bvo);
        IngestIn in{};
        in.n = m; in.krec = kh; in.koff = bko; in.vheap = vh; in.voff = bvo;
        in.verify_rehash = true; in.clevel_out = dcl;
        CHK(ingest(t, in));
        std::vector<uint32_t> cl(m);
        CHK(d2h(t, cl.data(), dcl, m * 4));
        uint64_t rej = 0;
        for (uint64_t i = 0; i < m; i++) rej += cl[i] != 0;
        *n_rejected = rej;
        *n_applied = m - rej;
    }
    CHK(tsync(t));
    return ST_OK;
}

extern "C" int st_exchange_apply(st_tree *local, st_tree *remote, uint64_t *n_diffs, uint64_t *n_applied,
                                 uint64_t *n_rejected, int *crashed, uint32_t *clevel, uint64_t *cbucket, int *cside) {
    return exchange_core(local, remote, true, n_diffs, n_applied, n_rejected, crashed, clevel, cbucket, cside);
}

// The same compare + valid_obj_hash selection with nothing applied: the
// number of diffs, how many remote values an apply would take (before the
// first crash), whether it would crash, or the corruption.  A partitioned
// exchange plans on every rank first so that only the partitions before the
// first crash (in the reference's order: highest segments first) apply.
extern "C" int st_exchange_plan(st_tree *local, st_tree *remote, uint64_t *n_diffs, uint64_t *n_take, int *crashed,
                                uint32_t *clevel, uint64_t *cbucket, int *cside) {
    uint64_t rej = 0;
    return exchange_core(local, remote, false, n_diffs, n_take, &rej, crashed, clevel, cbucket, cside);
}

extern "C" int st_compare(st_tree *local, st_tree *remote, int filter, st_result **out, uint32_t *clevel,
                          uint64_t *cbucket, int *cside) {
    ENTER_PAIR(local, remote);
    CHK(flush_all(local));
    CHK(flush_all(remote));
    *out = nullptr;
    CompareOut co;
    int status = ST_OK;
    CHK(compare_core(local, remote, filter, co, clevel, cbucket, cside, &status));
    if (status != ST_OK) return status;
    st_tree *t = local;
    const uint64_t n = co.n;
    st_result *res = new_result(0);
    res->n = 1;
    res->eoff[0] = 0;
    res->eoff[1] = n;
    res->n_entries = n;
    res->koff = (uint64_t *)calloc(n + 1, 8);
    res->aoff = (uint64_t *)calloc(n + 1, 8);
    res->boff = (uint64_t *)calloc(n + 1, 8);
    res->kind = (uint8_t *)calloc(n + 1, 1);
    res->seg = (uint64_t *)calloc(n + 1, 8);
    if (n == 0) {
        res->ktype = (uint8_t *)calloc(1, 1);
        res->kheap = (uint8_t *)malloc(1);
        res->aheap = (uint8_t *)malloc(1);
        res->bheap = (uint8_t *)malloc(1);
        *out = res;
        return ST_OK;
    }
    // The records to host memory with two synchronisations: the lengths of
    // every key and value as ONE array [keys | local values | remote values]
    // (n + 1 each, the last 0) and ONE scan, so the three offset arrays are
    // windows of the scan and the three heaps are ranges of one buffer; the
    // scan comes back in one copy (the heap sizes), then the heaps, segments
    // and kinds in one more.
    DevTree da = view(local), db = view(remote);
    Scratch sc(t);
    const uint64_t m = n + 1, m3 = 3 * m;
    uint64_t *len = nullptr, *off = nullptr;
    uint8_t *D = nullptr;
    int r = ST_OK;
    auto fail = [&](int rc) { st_free_result(res); return rc; };
    if ((r = sc.alloc(&len, m3)) || (r = sc.alloc(&off, m3))) return fail(r);
    t->reads_remote = true;
    hipLaunchKernelGGL(k_diff_lengths, dim3(grid_for(m)), dim3(256), 0, t->stream, da, db, co.rec, n, len, len + m, len + 2 * m);
    if ((r = exclusive_scan<uint64_t>(t, len, off, m3)) || (r = rpin_reserve(t, m3 * 8))) return fail(r);
    HIPCHK(hipMemcpyAsync(t->rpin, off, m3 * 8, hipMemcpyDeviceToHost, t->stream));
    if ((r = tsync(t))) return fail(r);
    const uint64_t *S = reinterpret_cast<const uint64_t *>(t->rpin);
    const uint64_t kb = S[n], ab = S[2 * m - 1] - S[m], bb = S[m3 - 1] - S[2 * m];
    for (uint64_t i = 0; i <= n; i++) {
        res->koff[i] = S[i];
        res->aoff[i] = S[m + i] - S[m];
        res->boff[i] = S[2 * m + i] - S[2 * m];
    }
    const uint64_t hb = (S[m3 - 1] + 7) & ~7ull;   // the three heaps, back to back
    if ((r = sc.bytes(&D, hb + 9 * n + 16))) return fail(r);
    uint64_t *dseg = reinterpret_cast<uint64_t *>(D + hb);
    uint8_t *dkind = D + hb + 8 * n;
    hipLaunchKernelGGL(k_diff_gather, dim3(grid_for(n)), dim3(256), 0, t->stream, da, db, co.rec, n, (const uint64_t *)off, D,
                       (const uint64_t *)(off + m), D, (const uint64_t *)(off + 2 * m), D, dkind, dseg);
    if (hipGetLastError() != hipSuccess) { g_err = "launch diff_gather"; return fail(ST_EDEVICE); }
    if ((r = rpin_reserve(t, hb + 9 * n))) return fail(r);
    HIPCHK(hipMemcpyAsync(t->rpin, D, hb + 9 * n, hipMemcpyDeviceToHost, t->stream));
    if ((r = tsync(t))) return fail(r);
    res->kheap = (uint8_t *)malloc(kb + 1);
    res->aheap = (uint8_t *)malloc(ab + 1);
    res->bheap = (uint8_t *)malloc(bb + 1);
    if (!res->kheap || !res->aheap || !res->bheap) { g_err = "malloc"; return fail(ST_ENOMEM); }
    memcpy(res->kheap, t->rpin, kb);
    memcpy(res->aheap, t->rpin + kb, ab);
    memcpy(res->bheap, t->rpin + kb + ab, bb);
    memcpy(res->seg, t->rpin + hb, 8 * n);
    memcpy(res->kind, t->rpin + hb + 8 * n, n);
    records_to_keys(res, n);
    *out = res;
    return ST_OK;
}

// The last compare's frontier: visited nodes per level (levels 1..H+1) and
// the algorithmic bytes of its final-level segment pairs (bench roofline).
extern "C" int st_compare_stats(st_tree *local, uint64_t *visited, uint32_t max_levels, uint64_t *seg_bytes) {
    ENTER(local);
    CmpWork &w = local->cw;
    if (!w.wcnt) { g_err = "no compare has run on this tree"; return ST_EINVAL; }
    std::vector<uint32_t> st((uint64_t)w.nw * ST_STATW);
    std::vector<uint64_t> wb(w.nw);
    HIPCHK(hipMemcpyAsync(st.data(), w.wst, st.size() * 4, hipMemcpyDeviceToHost, local->stream));
    HIPCHK(hipMemcpyAsync(wb.data(), w.wbytes, wb.size() * 8, hipMemcpyDeviceToHost, local->stream));
    CHK(tsync(local));
    const uint32_t L1 = local->H + 1;
    for (uint32_t l = 0; l < max_levels; l++) {
        uint64_t v = 0;
        if (l >= 1 && l <= L1)
            for (uint32_t x = 0; x < w.nw; x++) v += st[(uint64_t)x * ST_STATW + l];
        visited[l] = v;
    }
    uint64_t b = 0;
    for (uint32_t x = 0; x < w.nw; x++) b += wb[x];
    *seg_bytes = b;
    return ST_OK;
}

// ETF atom forms of snapshots: 0 = as term_to_binary writes them before OTP
// 26 (ATOM_EXT for Latin-1 atoms: the reference's era), 1 = OTP >= 26
// (SMALL_ATOM_UTF8_EXT / ATOM_UTF8_EXT only).
extern "C" int st_set_etf_atoms(st_tree *t, int utf8) {
    if (!t) { g_err = "NULL tree"; return ST_EINVAL; }
    std::lock_guard<std::recursive_mutex> g(t->mu);
    t->flags = utf8 ? (t->flags | ST_FLAG_ATOM_UTF8) : (t->flags & ~ST_FLAG_ATOM_UTF8);
    return ST_OK;
}

// The device key record of one key (host only, no device): memcmp order of
// records = Erlang term order (term_key.h).  *out_len = record length (the
// record is written when it fits in cap).
extern "C" int st_key_record(uint8_t ktype, const uint8_t *bytes, uint64_t len, uint8_t *out, uint64_t cap,
                             uint64_t *out_len) {
    const uint64_t off[2] = {0, len};
    HostRecords r;
    CHK(pack_records(1, &ktype, bytes, off, r));
    const uint64_t n = r.off[1];
    *out_len = n;
    if (out && n <= cap) memcpy(out, r.heap.data(), n);
    return ST_OK;
}

// Top-hash records of n trees (one device) into device memory `out`
// (18 bytes per tree: present, hash17), for an RCCL all-gather.
extern "C" int st_tops_to_device(st_tree **trees, uint32_t n, void *out) {
    return st_tops_to_device_on(trees, n, out, nullptr);
}
extern "C" int st_tops_to_device_on(st_tree **trees, uint32_t n, void *out, void *stream) {
    if (n == 0) return ST_OK;
    for (uint32_t i = 0; i < n; i++)
        if (!trees[i]) { g_err = "NULL tree"; return ST_EINVAL; }
    GroupLock glk(trees, n);
    st_tree *t = trees[0];
    CHK(use_device(t));
    for (uint32_t i = 0; i < n; i++) CHK(alive(trees[i]));
    std::vector<TreeTiles> h(n);
    for (uint32_t i = 0; i < n; i++) {
        if (trees[i]->device != t->device) { g_err = "trees on different devices"; return ST_EINVAL; }
        // a tree with nothing enqueued since its last synchronisation is not waited for
        if (trees[i]->stream != t->stream && trees[i]->async_pending) CHK(tsync(trees[i]));
        h[i] = tree_tiles(trees[i]);
    }
    Scratch sc(t);
    TreeTiles *dtt = nullptr;
    CHK(sc.alloc(&dtt, n));
    HIPCHK(hipMemcpyAsync(dtt, h.data(), n * sizeof(TreeTiles), hipMemcpyHostToDevice, t->stream));
    // `out` may still be read by the caller's stream (e.g. the previous
    // all-gather): written only after that stream's work so far
    CHK(order_after(t, (hipStream_t)stream));
    LAUNCH(t, "tops_out", k_tops_out, grid_for((uint64_t)n * 18), 256, 0, (const TreeTiles *)dtt, n, (uint8_t *)out);
    CHK(tsync(t));
    return ST_OK;
}

// ------------------------------------------------------------------ synctree_leveldb format
// device tree <-> the LevelDB records synctree_leveldb
// writes (src/synctree_leveldb.erl:104-109, 134-152).  Encoding and decoding
// both run on the device (leveldb_fmt.h): restore copies the caller's host
// records to HBM once and commits the decoded slot arrays and CSR only when
// every record decoded.

extern "C" void st_free_kv(st_kv *kv) {
    if (!kv) return;
    free(kv->koff); free(kv->kheap); free(kv->voff); free(kv->vheap);
    free(kv);
}

static int snapshot_device(st_tree *t, const uint8_t *tree_id, uint32_t id_len, uint64_t *n_out, uint64_t **okoff,
                           uint8_t **kout, uint64_t **ovoff, uint8_t **vout, uint64_t tot[3]) {
    const uint64_t R = t->nslots;
    DevTree d = view(t);
    const uint64_t ne = t->n;
    uint64_t *pres = nullptr, *kl = nullptr, *vl = nullptr, *rank = nullptr, *ko = nullptr, *vo = nullptr;
    uint64_t *es = nullptr, *eo = nullptr;
    uint8_t *did = nullptr;
    int r = ST_OK;
    auto done = [&]() {
        dfree(t, pres); dfree(t, kl); dfree(t, vl); dfree(t, rank); dfree(t, ko); dfree(t, vo); dfree(t, did);
        dfree(t, es); dfree(t, eo);
    };
    if ((r = dalloc_t(t, &es, ne + 1)) || (r = dalloc_t(t, &eo, ne + 1)) || (r = dalloc_t(t, &pres, R + 1)) || (r = dalloc_t(t, &kl, R + 1)) || (r = dalloc_t(t, &vl, R + 1)) ||
        (r = dalloc_t(t, &rank, R + 1)) || (r = dalloc_t(t, &ko, R + 1)) || (r = dalloc_t(t, &vo, R + 1)) ||
        (r = dalloc(t, (void **)&did, id_len + 1)) || (r = h2d(t, did, tree_id, id_len))) { done(); return r; }
    LAUNCH(t, "snap_entry_sizes", k_snap_entry_sizes, grid_for(ne + 1), 256, 0, d, ne, es);
    if ((r = exclusive_scan<uint64_t>(t, es, eo, ne + 1))) { done(); return r; }
    LAUNCH(t, "snap_sizes", k_snap_sizes, grid_for(R + 1), 256, 0, d, id_len, R, (const uint64_t *)eo,
           (const uint8_t *)t->erec, pres, kl, vl);
    if ((r = exclusive_scan<uint64_t>(t, pres, rank, R + 1)) || (r = exclusive_scan<uint64_t>(t, kl, ko, R + 1)) ||
        (r = exclusive_scan<uint64_t>(t, vl, vo, R + 1))) { done(); return r; }
    HIPCHK(hipMemcpyAsync(&tot[0], rank + R, 8, hipMemcpyDeviceToHost, t->stream));
    HIPCHK(hipMemcpyAsync(&tot[1], ko + R, 8, hipMemcpyDeviceToHost, t->stream));
    HIPCHK(hipMemcpyAsync(&tot[2], vo + R, 8, hipMemcpyDeviceToHost, t->stream));
    CHK(tsync(t));
    const uint64_t n = tot[0];
    if ((r = dalloc_t(t, okoff, n + 1)) || (r = dalloc_t(t, ovoff, n + 1)) || (r = dalloc(t, (void **)kout, tot[1] + 16)) ||
        (r = dalloc(t, (void **)vout, tot[2] + 16))) { done(); return r; }
    LAUNCH(t, "snap_write", k_snap_write, grid_for(R), 256, 0, d, (const uint8_t *)did, id_len, R, (const uint64_t *)rank,
           (const uint64_t *)ko, (const uint64_t *)vo, (const uint64_t *)eo, *kout, *vout, *okoff, *ovoff);
    if (ne) LAUNCH(t, "snap_entries", k_snap_entries, grid_for(ne), 256, 0, d, ne, t->base[t->H + 1], (const uint64_t *)vo,
                   (const uint64_t *)eo, *vout);
    HIPCHK(hipMemcpyAsync(*okoff + n, &tot[1], 8, hipMemcpyHostToDevice, t->stream));
    HIPCHK(hipMemcpyAsync(*ovoff + n, &tot[2], 8, hipMemcpyHostToDevice, t->stream));
    CHK(tsync(t));
    done();
    *n_out = n;
    return ST_OK;
}

extern "C" int st_snapshot_leveldb(st_tree *t, const uint8_t *tree_id, uint32_t id_len, st_kv **out) {
    *out = nullptr;
    ENTER(t);
    FLUSH(t);
    if (t->partitioned) { g_err = "snapshot of a partitioned tree (one partition is not a synctree)"; return ST_EINVAL; }
    if (id_len && !tree_id) { g_err = "tree_id is NULL"; return ST_EINVAL; }
    uint64_t n = 0, tot[3] = {0, 0, 0}, *okoff = nullptr, *ovoff = nullptr;
    uint8_t *kout = nullptr, *vout = nullptr;
    int r = snapshot_device(t, tree_id, id_len, &n, &okoff, &kout, &ovoff, &vout, tot);
    st_kv *kv = nullptr;
    if (!r) {
        kv = (st_kv *)calloc(1, sizeof(st_kv));
        kv->n = n;
        kv->koff = (uint64_t *)malloc((n + 1) * 8);
        kv->voff = (uint64_t *)malloc((n + 1) * 8);
        kv->kheap = (uint8_t *)malloc(tot[1] + 1);
        kv->vheap = (uint8_t *)malloc(tot[2] + 1);
        if (!kv->koff || !kv->voff || !kv->kheap || !kv->vheap) { g_err = "host allocation"; r = ST_ENOMEM; }
        if (!r) r = d2h(t, kv->koff, okoff, (n + 1) * 8);
        if (!r) r = d2h(t, kv->voff, ovoff, (n + 1) * 8);
        if (!r) r = d2h(t, kv->kheap, kout, tot[1]);
        if (!r) r = d2h(t, kv->vheap, vout, tot[2]);
    }
    dfree(t, okoff); dfree(t, ovoff); dfree(t, kout); dfree(t, vout);
    if (r) { st_free_kv(kv); return r; }
    *out = kv;
    return ST_OK;
}

extern "C" int st_snapshot_leveldb_device(st_tree *t, const uint8_t *tree_id, uint32_t id_len, uint64_t *n_records,
                                          uint64_t *key_bytes, uint64_t *value_bytes) {
    ENTER(t);
    FLUSH(t);
    if (t->partitioned) { g_err = "snapshot of a partitioned tree"; return ST_EINVAL; }
    if (id_len && !tree_id) { g_err = "tree_id is NULL"; return ST_EINVAL; }
    uint64_t n = 0, tot[3] = {0, 0, 0}, *okoff = nullptr, *ovoff = nullptr;
    uint8_t *kout = nullptr, *vout = nullptr;
    int r = snapshot_device(t, tree_id, id_len, &n, &okoff, &kout, &ovoff, &vout, tot);
    dfree(t, okoff); dfree(t, ovoff); dfree(t, kout); dfree(t, vout);
    if (!r) CHK(tsync(t));
    if (n_records) *n_records = n;
    if (key_bytes) *key_bytes = tot[1];
    if (value_bytes) *value_bytes = tot[2];
    return r;
}

extern "C" int st_restore_leveldb(st_tree *t, const uint8_t *tree_id, uint32_t id_len, uint64_t n,
                                  const uint8_t *kheap, const uint64_t *koff, const uint8_t *vheap,
                                  const uint64_t *voff, uint64_t *n_loaded, uint64_t *n_skipped) {
    ENTER(t);
    FLUSH(t);
    if (t->partitioned) { g_err = "restore into a partitioned tree"; return ST_EINVAL; }
    if (id_len && !tree_id) { g_err = "tree_id is NULL"; return ST_EINVAL; }
    const uint64_t R = t->nslots, S = t->S;
    const uint64_t kin = n ? koff[n] - koff[0] : 0, vin = n ? voff[n] - voff[0] : 0;
    DevTree d = view(t);
    // staging: nothing of the tree changes until every record has decoded
    uint8_t *dkh = nullptr, *dvh = nullptr, *did = nullptr, *segok = nullptr, *serec = nullptr;
    uint64_t *dko = nullptr, *dvo = nullptr, *ec = nullptr, *kc = nullptr, *vc = nullptr;
    uint64_t *nso = nullptr, *kbase = nullptr, *vbase = nullptr, *nsvo = nullptr, *nko = nullptr, *nvo = nullptr;
    uint8_t *nkh = nullptr, *nvh = nullptr;
    unsigned long long *recof = nullptr, *ctr = nullptr;
    uint16_t *stag = nullptr;
    uint4 *smd = nullptr;
    uint64_t *dhs = nullptr, *dhe = nullptr, *dhko = nullptr, *dhvo = nullptr;
    uint8_t *dhk = nullptr, *dhv = nullptr;
    auto done = [&](bool keep_new) {
        void *ps[] = {dkh, dvh, did, segok, serec, dko, dvo, ec, kc, vc, kbase, vbase, recof, ctr, stag, smd,
                      dhs, dhe, dhko, dhvo, dhk, dhv};
        for (void *p : ps) dfree(t, p);
        if (!keep_new) { dfree(t, nso); dfree(t, nsvo); dfree(t, nko); dfree(t, nvo); dfree(t, nkh); dfree(t, nvh); }
    };
#define RCHK(x)                               \
    do {                                      \
        int r_ = (x);                         \
        if (r_ != ST_OK) { done(false); return r_; } \
    } while (0)
    // records as they lie in the caller's buffers (offsets rebased to 0)
    std::vector<uint64_t> ko0(n + 1), vo0(n + 1);
    for (uint64_t i = 0; i <= n; i++) { ko0[i] = koff[i] - koff[0]; vo0[i] = voff[i] - voff[0]; }
    RCHK(dalloc(t, (void **)&dkh, kin + 16)); RCHK(dalloc(t, (void **)&dvh, vin + 16));
    RCHK(dalloc_t(t, &dko, n + 1)); RCHK(dalloc_t(t, &dvo, n + 1)); RCHK(dalloc(t, (void **)&did, id_len + 1));
    RCHK(h2d(t, dkh, kheap + (n ? koff[0] : 0), kin)); RCHK(h2d(t, dvh, vheap + (n ? voff[0] : 0), vin));
    RCHK(h2d(t, dko, ko0.data(), (n + 1) * 8)); RCHK(h2d(t, dvo, vo0.data(), (n + 1) * 8));
    RCHK(h2d(t, did, tree_id, id_len));
    RCHK(dalloc_t(t, &recof, R)); RCHK(dalloc_t(t, &ctr, 5)); RCHK(dalloc_t(t, &stag, R)); RCHK(dalloc_t(t, &smd, R));
    RCHK(dalloc_t(t, &ec, S + 1)); RCHK(dalloc_t(t, &kc, S + 1)); RCHK(dalloc_t(t, &vc, S + 1)); RCHK(dalloc_t(t, &segok, S));
    RCHK(dalloc_t(t, &serec, R));
    HIPCHK(hipMemsetAsync(serec, 0, R, t->stream));
    HIPCHK(hipMemsetAsync(recof, 0, R * 8, t->stream));
    HIPCHK(hipMemsetAsync(ctr, 0, 3 * 8, t->stream));
    HIPCHK(hipMemsetAsync(ctr + RST_DOMSLOT, 0xFF, 8, t->stream));
    HIPCHK(hipMemsetAsync(ctr + RST_HOST, 0, 8, t->stream));
    HIPCHK(hipMemsetAsync(stag, 0, R * 2, t->stream));
    HIPCHK(hipMemsetAsync(smd, 0, R * 16, t->stream));
    HIPCHK(hipMemsetAsync(ec + S, 0, 8, t->stream));
    HIPCHK(hipMemsetAsync(kc + S, 0, 8, t->stream));
    HIPCHK(hipMemsetAsync(vc + S, 0, 8, t->stream));
    if (n) LAUNCH(t, "rest_keys", k_rest_keys, grid_for(n), 256, 0, d, (const uint8_t *)did, id_len, n,
                  (const uint8_t *)dkh, (const uint64_t *)dko, recof);
    LAUNCH(t, "rest_nodes", k_rest_nodes, grid_for(R), 256, 0, d, R, (const unsigned long long *)recof,
           (const uint8_t *)dvh, (const uint64_t *)dvo, stag, smd, ec, kc, vc, segok, serec, ctr);
    unsigned long long hc[5] = {0, 0, 0, 0, 0};
    auto domain_error = [&]() {
        const uint64_t r = hc[RST_DOMSLOT];
        uint32_t L = 0;
        while (L <= t->H && r >= t->base[L + 1]) L++;
        const uint64_t b = r == 0 ? 0 : r - t->base[L];
        g_err = "node {" + std::to_string(L) + "," + std::to_string(b) +
                "} decodes to a term outside the device node domain (hash size, child id, key/value type or order)";
        done(false);
        return ST_EINVAL;
    };
    RCHK(d2h(t, hc, ctr, sizeof(hc)));
    if (hc[RST_DOM]) return domain_error();
    // segments whose keys the device decoder leaves to the host (maps,
    // FLOAT_EXT, deep nesting): decoded here (term_key.h), sized into the
    // scans, written after them
    std::vector<uint64_t> hs, he{0}, hko{0}, hvo{0};
    std::vector<uint8_t> hk, hv;
    if (hc[RST_HOST]) {
        const uint64_t sb = t->base[t->H + 1];
        std::vector<uint8_t> ok(S);
        std::vector<unsigned long long> rof(S);
        RCHK(d2h(t, ok.data(), segok, S));
        RCHK(d2h(t, rof.data(), recof + sb, S * 8));
        auto rcmp = [&](uint64_t j) {   // record j-1 vs record j, Erlang term order (rec_cmp)
            const uint8_t *a = hk.data() + hko[j - 1], *b = hk.data() + hko[j];
            const uint64_t la = krec_order_len(a, hko[j] - hko[j - 1]), lb = krec_order_len(b, hko[j + 1] - hko[j]);
            const int c = memcmp(a, b, std::min(la, lb));
            return c ? c : (la < lb ? -1 : la > lb ? 1 : 0);
        };
        for (uint64_t sg = 0; sg < S; sg++) {
            if (ok[sg] != 2) continue;
            const uint64_t i = rof[sg] - 1;
            const size_t kz = hk.size(), vz = hv.size(), ez = hko.size();
            int st = termkey::segment_from_etf(vheap + voff[i], voff[i + 1] - voff[i], hk, hko, hv, hvo);
            for (uint64_t j = ez; st == termkey::SEG_OK && j + 1 < hko.size(); j++)
                if (rcmp(j) >= 0) st = termkey::SEG_DOM;   // an orddict: strictly ascending
            if (st == termkey::SEG_DOM) { hc[RST_DOMSLOT] = sb + sg; return domain_error(); }
            if (st == termkey::SEG_BAD) {   // binary_to_term raises: the node is absent
                hk.resize(kz); hv.resize(vz); hko.resize(ez); hvo.resize(ez);
                hc[RST_SKIPPED]++;
                continue;
            }
            hs.push_back(sg);
            he.push_back(hko.size() - 1);
            hc[RST_LOADED]++;
        }
    }
    const uint64_t nh = hs.size();
    if (nh) {
        RCHK(dalloc_t(t, &dhs, nh)); RCHK(dalloc_t(t, &dhe, nh + 1));
        RCHK(dalloc_t(t, &dhko, hko.size())); RCHK(dalloc_t(t, &dhvo, hvo.size()));
        RCHK(dalloc(t, (void **)&dhk, hk.size() + 1)); RCHK(dalloc(t, (void **)&dhv, hv.size() + 1));
        RCHK(h2d(t, dhs, hs.data(), nh * 8)); RCHK(h2d(t, dhe, he.data(), (nh + 1) * 8));
        RCHK(h2d(t, dhko, hko.data(), hko.size() * 8)); RCHK(h2d(t, dhvo, hvo.data(), hvo.size() * 8));
        RCHK(h2d(t, dhk, hk.data(), hk.size())); RCHK(h2d(t, dhv, hv.data(), hv.size()));
        LAUNCH(t, "rest_host_sizes", k_rest_host_sizes, grid_for(nh), 256, 0, nh, (const uint64_t *)dhs,
               (const uint64_t *)dhe, (const uint64_t *)dhko, (const uint64_t *)dhvo, ec, kc, vc);
    }
    RCHK(dalloc_t(t, &nso, S + 1)); RCHK(dalloc_t(t, &kbase, S + 1)); RCHK(dalloc_t(t, &vbase, S + 1));
    RCHK(exclusive_scan<uint64_t>(t, ec, nso, S + 1));
    RCHK(exclusive_scan<uint64_t>(t, kc, kbase, S + 1));
    RCHK(exclusive_scan<uint64_t>(t, vc, vbase, S + 1));
    uint64_t tot[3] = {0, 0, 0};
    HIPCHK(hipMemcpyAsync(&tot[0], nso + S, 8, hipMemcpyDeviceToHost, t->stream));
    HIPCHK(hipMemcpyAsync(&tot[1], kbase + S, 8, hipMemcpyDeviceToHost, t->stream));
    HIPCHK(hipMemcpyAsync(&tot[2], vbase + S, 8, hipMemcpyDeviceToHost, t->stream));
    CHK(tsync(t));
    const uint64_t ne = tot[0], kb = tot[1], vb = tot[2];
    RCHK(dalloc_t(t, &nko, ne + 1)); RCHK(dalloc_t(t, &nvo, ne + 1)); RCHK(dalloc_t(t, &nsvo, S + 1));
    RCHK(dalloc(t, (void **)&nkh, kb + HEAP_SLACK)); RCHK(dalloc(t, (void **)&nvh, vb + HEAP_SLACK));
    HIPCHK(hipMemsetAsync(nkh + kb, 0, HEAP_SLACK, t->stream));
    HIPCHK(hipMemsetAsync(nvh + vb, 0, HEAP_SLACK, t->stream));
    RCHK(h2d(t, nko + ne, &tot[1], 8));
    RCHK(h2d(t, nvo + ne, &tot[2], 8));
    LAUNCH(t, "rest_segments", k_rest_segments, grid_for(S), 256, 0, d, (const unsigned long long *)recof,
           (const uint8_t *)dvh, (const uint64_t *)dvo, (const uint8_t *)segok, (const uint64_t *)nso,
           (const uint64_t *)kbase, (const uint64_t *)vbase, nko, nkh, nvo, nvh, ctr);
    if (nh)
        LAUNCH(t, "rest_host_write", k_rest_host_write, grid_for(nh), 256, 0, nh, (const uint64_t *)dhs,
               (const uint64_t *)dhe, (const uint64_t *)dhko, (const uint64_t *)dhvo, (const uint8_t *)dhk,
               (const uint8_t *)dhv, (const uint64_t *)nso, (const uint64_t *)kbase, (const uint64_t *)vbase, nko,
               nkh, nvo, nvh);
    LAUNCH(t, "seg_voff", k_seg_voff, grid_for(S + 1), 256, 0, (const uint64_t *)nso, (const uint64_t *)nvo, S, nsvo);
    {
        unsigned long long hd[5];
        RCHK(d2h(t, hd, ctr, sizeof(hd)));
        if (hd[RST_DOM]) { hc[RST_DOMSLOT] = hd[RST_DOMSLOT]; return domain_error(); }
    }
    // commit: node arrays and the new CSR
    HIPCHK(hipMemcpyAsync(t->tag, stag, R * 2, hipMemcpyDeviceToDevice, t->stream));
    HIPCHK(hipMemcpyAsync(t->md5, smd, R * 16, hipMemcpyDeviceToDevice, t->stream));
    RCHK(ensure_erec(t));   // the [] records among them
    HIPCHK(hipMemcpyAsync(t->erec, serec, R, hipMemcpyDeviceToDevice, t->stream));
    {
        CsrSet o;
        o.seg_off = nso; o.seg_voff = nsvo; o.koff = nko; o.voff = nvo; o.kheap = nkh; o.vheap = nvh;
        o.cap_n = ne + 1; o.cap_k = kb + HEAP_SLACK; o.cap_v = vb + HEAP_SLACK;
        csr_install(t, o);
    }
    t->n = ne; t->kbytes = kb; t->vbytes = vb;
    t->perm_valid = false;
    t->tiles_valid = false;
    t->tiles_wanted = false;
    t->fresh = false;
    done(true);
    CHK(tsync(t));   // the caller's buffers may go after return
#undef RCHK
    if (n_loaded) *n_loaded = hc[RST_LOADED];
    if (n_skipped) *n_skipped = hc[RST_SKIPPED];
    return ST_OK;
}
