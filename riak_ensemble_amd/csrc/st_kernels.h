// st_kernels.h — gfx950 kernels of the synctree path (included once, by
// synctree_hip.hip).  Reference: src/synctree.erl (jrwest/riak_ensemble).
//
// Device layout of one tree:
//  * node entries: one slot per (Level, Bucket) for Level 1..H+1 plus slot 0
//    for the #tree.top_hash record field.  slot(l, b) = base[l] + b.  A slot
//    holds the 17-byte entry the PARENT node records for that child:
//    md5[slot] (16 B) + tag[slot] (bit 8 = present, bits 0..7 = prefix byte).
//    slot(1,0) is the stored {0,0}; slot 0 the cached record (they only
//    differ after raw backend writes).  The content of inner node (l, b) is
//    the present slots among children (l+1, b*W .. b*W+W-1) — exactly the
//    [{ChildId, Hash}] orddict of synctree.erl:516-533.
//  * segments: CSR.  seg_off[S+1] entry offsets; key records (tag byte +
//    ensure_binary payload, integer payload with its sign bit flipped so that
//    memcmp-then-length IS Erlang term order) in kheap/koff; values in
//    vheap/voff; seg_voff[S+1] = voff[seg_off[s]] so that a segment's hash
//    input (the concatenation of its values, synctree.erl:255-259) is ONE
//    contiguous byte range.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "md5_dev.h"
#include "term_key.h"

#define ST_MAXLEV 33
#define TAG_PRESENT 0x100u

#define MODE_STORE 0
#define MODE_VERIFY 1

#define ST_FLAG_ATOM_UTF8 1u   // DevTree.flags: ETF atoms as OTP >= 26 writes them (utf8 forms only)

// Device code sees the tree's pointers as global memory (address space 1):
// a DevTree read from LDS or from memory -- the per-key kernel's request, a
// group's descriptors -- would otherwise hand every access to FLAT, whose
// waits cover LDS and memory alike.  The host pass sees plain pointers (the
// layout is the same).
#if defined(__HIP_DEVICE_COMPILE__)
#define ST_GAS __attribute__((address_space(1)))
#else
#define ST_GAS
#endif
// a host pointer stored into a DevTree (the device pass of host code sees the
// address-space-qualified fields)
template <class T>
__host__ __device__ __forceinline__ T ST_GAS *gp(T *p) {
    return (T ST_GAS *)p;
}
struct DevTree {
    uint32_t W, shift, H, flags;
    uint64_t S;
    uint64_t base[ST_MAXLEV + 2];
    uint4 ST_GAS *md5;
    uint16_t ST_GAS *tag;
    // segment s: entries [seg_off[s], seg_end[s]) of koff/voff (each entry's
    // key and value end at the next entry's offsets; entry seg_end[s] holds
    // the ends of the last one), values [seg_voff[s], seg_vend[s]).  The
    // canonical CSR is gap-free (seg_end = seg_off + 1, seg_vend = seg_voff +
    // 1); the paged layout of streaming batches (pages.h) leaves slack after
    // every segment's page.
    const uint64_t ST_GAS *seg_off;
    const uint64_t ST_GAS *seg_end;
    const uint64_t ST_GAS *seg_voff;
    const uint64_t ST_GAS *seg_vend;
    const uint64_t ST_GAS *koff;
    const uint8_t ST_GAS *kheap;
    const uint64_t ST_GAS *voff;
    const uint8_t ST_GAS *vheap;
};

// Key records (term_key.h): the plain int64 / atom / binary form, or a term
// record [SK][ETF][Seg][etf_len u16][seg_len u16].
__host__ __device__ __forceinline__ bool krec_is_term(const uint8_t *p, uint64_t len) {
    const uint8_t t = p[0];
    return !(t == KEYTAG_ATOM || t == KEYTAG_BINARY || (t == KEYTAG_INT && len == 9));
}
// term record -> offsets of its ETF and Seg bytes
__host__ __device__ __forceinline__ void krec_term_parts(const uint8_t *p, uint64_t len, uint64_t *etf_at, uint32_t *etf_len,
                                                         uint64_t *seg_at, uint32_t *seg_len) {
    const uint32_t el = (uint32_t)p[len - 4] | ((uint32_t)p[len - 3] << 8);
    const uint32_t sl = (uint32_t)p[len - 2] | ((uint32_t)p[len - 1] << 8);
    const uint64_t tail = len - 4 - (sl == 0xFFFF ? 0 : sl);
    *etf_at = tail - el;
    *etf_len = el;
    *seg_at = sl == 0xFFFF ? tail - el : tail;
    *seg_len = sl == 0xFFFF ? el : sl;
}
// ensure_binary(Key) bytes of a non-int64 record (synctree.erl:261-268)
__host__ __device__ __forceinline__ void krec_seg_bytes(const uint8_t *p, uint64_t len, const uint8_t **sp, uint64_t *sl) {
    if (krec_is_term(p, len)) {
        uint64_t ea, sa;
        uint32_t el, sln;
        krec_term_parts(p, len, &ea, &el, &sa, &sln);
        *sp = p + sa;
        *sl = sln;
    } else {
        *sp = p + 1;
        *sl = len - 1;
    }
}

__device__ __forceinline__ uint64_t gtid() { return (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ uint64_t gstride() { return (uint64_t)gridDim.x * blockDim.x; }

// Bytes of a key record that decide its place in Erlang term order: the
// whole plain record, or the SK part of a term record (term_key.h).  Two keys
// whose SKs are equal are EQUAL keys (==): 1 and 1.0, {1} and {1.0} --
// orddict:store/erase, lists:keyfind and orddict_delta compare with ==
// (synctree.erl:206, :342-348; riak_ensemble_util.erl:120-125), so such keys
// share one entry; the trailing ETF/Seg bytes only say which form is stored.
__host__ __device__ __forceinline__ uint64_t krec_order_len(const uint8_t *p, uint64_t len) {
    if (!krec_is_term(p, len)) return len;
    const uint32_t el = (uint32_t)p[len - 4] | ((uint32_t)p[len - 3] << 8);
    const uint32_t sl = (uint32_t)p[len - 2] | ((uint32_t)p[len - 1] << 8);
    return len - 4 - el - (sl == 0xFFFF ? 0 : sl);
}

// The 8 big-endian bytes at p (any alignment) as an integer.
__device__ __forceinline__ uint64_t krec_be64(const uint8_t *p) {
    uint64_t v = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) v = (v << 8) | p[i];
    return v;
}

// Plain byte order: memcmp over the common prefix, then length.
__device__ __forceinline__ int bytes_cmp(const uint8_t *a, uint64_t la, const uint8_t *b, uint64_t lb) {
    uint64_t m = la < lb ? la : lb;
    uint64_t i = 0;
    for (; i + 8 <= m; i += 8) {
        uint64_t x, y;
        __builtin_memcpy(&x, a + i, 8);
        __builtin_memcpy(&y, b + i, 8);
        if (x != y) {
            x = __builtin_bswap64(x);
            y = __builtin_bswap64(y);
            return x < y ? -1 : 1;
        }
    }
    for (; i < m; i++)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

// Erlang term order (== for equality) on key records.
__device__ __forceinline__ int rec_cmp(const uint8_t *a, uint64_t la, const uint8_t *b, uint64_t lb) {
    return bytes_cmp(a, krec_order_len(a, la), b, krec_order_len(b, lb));
}

__device__ __forceinline__ bool bytes_eq(const uint8_t *a, uint64_t la, const uint8_t *b, uint64_t lb) {
    if (la != lb) return false;
    uint64_t i = 0;
    for (; i + 8 <= la; i += 8) {
        uint64_t x, y;
        __builtin_memcpy(&x, a + i, 8);
        __builtin_memcpy(&y, b + i, 8);
        if (x != y) return false;
    }
    for (; i < la; i++)
        if (a[i] != b[i]) return false;
    return true;
}

__device__ __forceinline__ void copy_bytes(uint8_t *d, const uint8_t *s, uint64_t n) {
    uint64_t i = 0;
    for (; i + 16 <= n; i += 16) {
        uint4 v;
        __builtin_memcpy(&v, s + i, 16);
        __builtin_memcpy(d + i, &v, 16);
    }
    if (i + 8 <= n) {
        uint64_t v;
        __builtin_memcpy(&v, s + i, 8);
        __builtin_memcpy(d + i, &v, 8);
        i += 8;
    }
    if (i + 4 <= n) {
        uint32_t v;
        __builtin_memcpy(&v, s + i, 4);
        __builtin_memcpy(d + i, &v, 4);
        i += 4;
    }
    for (; i < n; i++) d[i] = s[i];
}

// ---------------------------------------------------------------------------
// Ingest helpers

// int64 keys -> key records (9 bytes: tag 0, <<K:64/big>> with sign bit flipped)
// slack: zero bytes the heap keeps after the records (over-reads), written here
__global__ void k_pack_int64(const int64_t *keys, uint64_t n, uint8_t *kheap, uint64_t *koff, uint64_t *voff,
                             uint32_t vlen, uint32_t slack = 0) {
    for (uint64_t i = gtid(); i <= n; i += gstride()) {
        koff[i] = 9 * i;
        voff[i] = (uint64_t)vlen * i;
        if (i == n) {
            for (uint32_t b = 0; b < slack; b++) kheap[9 * n + b] = 0;
            break;
        }
        uint64_t k = (uint64_t)keys[i] ^ 0x8000000000000000ull;
        uint8_t *p = kheap + 9 * i;
        p[0] = KEYTAG_INT;
        uint64_t be = __builtin_bswap64(k);
        __builtin_memcpy(p + 1, &be, 8);
    }
}

// Several buffers zeroed by one launch (each a memset kernel of its own
// otherwise, ~5 us apiece on a batch's critical path).  Spans start 16-byte
// aligned (device allocations); a span's last n % 16 bytes go byte by byte.
#define ZS_MAX 6
struct ZeroSpans {
    uint8_t *p[ZS_MAX];
    uint64_t n[ZS_MAX];
    uint32_t k;
};
__global__ void __launch_bounds__(256) k_zero_spans(ZeroSpans z) {
    for (uint32_t q = 0; q < z.k; q++) {
        uint4 *w = reinterpret_cast<uint4 *>(z.p[q]);
        const uint64_t nw = z.n[q] / 16;
        for (uint64_t i = gtid(); i < nw; i += gstride()) w[i] = make_uint4(0u, 0u, 0u, 0u);
        for (uint64_t i = nw * 16 + gtid(); i < z.n[q]; i += gstride()) z.p[q][i] = 0;
    }
}

// K1a key_segment: get_segment/2 (synctree.erl:251-253) — md5 of the key's
// ensure_binary bytes read as a big-endian 128-bit integer, rem Segments
// (a power of two: the low bits of digest bytes 8..15).
// cnt / rank (optional): the bucketing's histogram, each record's rank in its
// segment's bucket from the same atomic (k_seg_hist).
__global__ void k_key_segment(const uint8_t *kheap, const uint64_t *koff, uint64_t n, uint64_t segmask,
                              uint32_t *seg_out, unsigned long long *cnt = nullptr, uint32_t *rank = nullptr) {
    for (uint64_t i = gtid(); i < n; i += gstride()) {
        const uint64_t o = koff[i];
        const uint64_t len = koff[i + 1] - o;
        const uint8_t *p = kheap + o;
        uint32_t d[4];
        if (p[0] == KEYTAG_INT && len == 9) {
            uint2 x;
            __builtin_memcpy(&x, p + 1, 8);
            uint32_t m[16];
            m[0] = x.x ^ 0x80u;  // unflip the sign bit: message = <<Key:64/big>>
            m[1] = x.y;
            m[2] = 0x80u;
#pragma unroll
            for (int w = 3; w < 16; w++) m[w] = 0u;
            m[14] = 64u;
            stmd5::init(d);
            stmd5::compress<true>(d, m);
        } else {
            const uint8_t *sp;
            uint64_t sl;
            krec_seg_bytes(p, len, &sp, &sl);
            stmd5::md5_global_pf<true>(sp, sl, d);
        }
        const uint64_t lo = ((uint64_t)__builtin_bswap32(d[2]) << 32) | (uint64_t)__builtin_bswap32(d[3]);
        const uint32_t s = (uint32_t)(lo & segmask);
        seg_out[i] = s;
        if (cnt) rank[i] = (uint32_t)atomicAdd(&cnt[s], 1ull);
    }
}

// Bucketing of a batch by segment (a counting sort: histogram with each
// record's rank in its bucket from the same atomic, scan = the run bounds,
// scatter to bound + rank: no second atomic pass).  The order inside a run is
// whatever the atomics give; k_run_sort then orders every run by (key, batch index).
__global__ void k_seg_hist(const uint32_t *seg, uint64_t n, unsigned long long *cnt, uint32_t *rank) {
    for (uint64_t i = gtid(); i < n; i += gstride()) rank[i] = (uint32_t)atomicAdd(&cnt[seg[i]], 1ull);
}
__global__ void k_seg_scatter(const uint32_t *seg, const uint32_t *rank, uint64_t n, const uint64_t *bseg_off,
                              uint32_t *sseg, uint32_t *perm) {
    for (uint64_t i = gtid(); i < n; i += gstride()) {
        const uint32_t s = seg[i];
        const uint64_t p = bseg_off[s] + rank[i];
        sseg[p] = s;
        perm[p] = (uint32_t)i;
    }
}

struct BatchView {
    const uint8_t *kheap;
    const uint64_t *koff;
    bool int9;   // every record an int64 key (insert_int64): record i at kheap + 9 i, koff not read
};

// A 9-byte key record's tag and big-endian payload in ONE round trip: three
// dword loads of its aligned window (its bytes and up to 3 of the next
// record's; heaps keep slack).
__device__ __forceinline__ void krec9_load(const uint8_t *p, uint32_t &tag, uint64_t &pv) {
    const uintptr_t ad = reinterpret_cast<uintptr_t>(p);
    const uint32_t o = (uint32_t)(ad & 3);
    const uint32_t ST_GAS *w = reinterpret_cast<const uint32_t ST_GAS *>(ad - o);
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    const uint32_t x = __builtin_amdgcn_alignbyte(w1, w0, o), y = __builtin_amdgcn_alignbyte(w2, w1, o);
    const uint32_t z = (uint32_t)(((uint64_t)w2 >> (8 * o)) & 0xffu);
    tag = x & 0xffu;
    // payload bytes 1..8 little-endian in (lo32, hi32), then big-endian order
    const uint32_t p0 = (x >> 8) | (y << 24), p1 = (y >> 8) | (z << 24);
    pv = ((uint64_t)__builtin_bswap32(p0) << 32) | __builtin_bswap32(p1);
}
#ifndef MI_W
#define MI_W 8    // k_merge_keys' interpolation window (keys): 72 bytes, one round trip (16: 0.19, 8: 0.175 ms
                  // a config-5 batch's positions; 4: 0.186, 24: 0.24 -- profiles/r06ba_interp_window_ab/)
#endif
__device__ __forceinline__ void cas_kx(uint64_t &ka, uint32_t &ia, uint64_t &kb, uint32_t &ib) {
    const bool sw = kb < ka || (kb == ka && ib < ia);
    const uint64_t k = sw ? kb : ka, k2 = sw ? ka : kb;
    const uint32_t i = sw ? ib : ia, i2 = sw ? ia : ib;
    ka = k; kb = k2; ia = i; ib = i2;
}

__device__ __forceinline__ int batch_cmp(const BatchView &b, uint32_t x, uint32_t y) {
    int c = rec_cmp(b.kheap + b.koff[x], b.koff[x + 1] - b.koff[x], b.kheap + b.koff[y], b.koff[y + 1] - b.koff[y]);
    if (c) return c;
    return x < y ? -1 : (x > y ? 1 : 0);
}

__device__ void heap_sift(const BatchView &bv, uint32_t *a, uint64_t start, uint64_t end) {
    uint64_t root = start;
    while (2 * root + 1 < end) {
        uint64_t child = 2 * root + 1, sw = root;
        if (batch_cmp(bv, a[sw], a[child]) < 0) sw = child;
        if (child + 1 < end && batch_cmp(bv, a[sw], a[child + 1]) < 0) sw = child + 1;
        if (sw == root) return;
        uint32_t t = a[root]; a[root] = a[sw]; a[sw] = t;
        root = sw;
    }
}

// Sort each segment's run of the batch by (key record, batch index) and mark
// the last writer of every key (sequential insert semantics: last wins).
__global__ void k_run_sort(BatchView bv, uint32_t *perm, const uint64_t *bseg_off, uint64_t S, uint8_t *keep) {
    for (uint64_t s = gtid(); s < S; s += gstride()) {
        const uint64_t a = bseg_off[s], b = bseg_off[s + 1];
        if (a == b) continue;
        uint32_t *r = perm + a;
        const uint64_t n = b - a;
        if (bv.int9 && n <= 4) {
            // int64 keys, a run of <= 4 (nearly all of them): the keys in
            // registers (one round trip), a sorting network on (key, index)
            uint64_t k[4];
            uint32_t x[4];
#pragma unroll
            for (int q = 0; q < 4; q++) { x[q] = q < (int)n ? r[q] : ~0u; k[q] = ~0ull; }
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (q < (int)n) { uint32_t tg; krec9_load(bv.kheap + 9ull * x[q], tg, k[q]); }
            cas_kx(k[0], x[0], k[1], x[1]);
            cas_kx(k[2], x[2], k[3], x[3]);
            cas_kx(k[0], x[0], k[2], x[2]);
            cas_kx(k[1], x[1], k[3], x[3]);
            cas_kx(k[1], x[1], k[2], x[2]);
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (q < (int)n) {
                    r[q] = x[q];
                    keep[a + q] = (q + 1 == (int)n || k[q] != k[q + 1 < 4 ? q + 1 : 3]) ? 1 : 0;
                }
            continue;
        }
        if (n <= 32) {
            for (uint64_t i = 1; i < n; i++) {
                uint32_t x = r[i];
                uint64_t j = i;
                while (j > 0 && batch_cmp(bv, r[j - 1], x) > 0) { r[j] = r[j - 1]; j--; }
                r[j] = x;
            }
        } else {
            for (uint64_t st = n / 2; st-- > 0;) heap_sift(bv, r, st, n);
            for (uint64_t e = n - 1; e > 0; e--) {
                uint32_t t = r[0]; r[0] = r[e]; r[e] = t;
                heap_sift(bv, r, 0, e);
            }
        }
        for (uint64_t i = 0; i < n; i++) {
            bool last = (i + 1 == n);
            if (!last) {
                const uint32_t x = r[i], y = r[i + 1];
                last = rec_cmp(bv.kheap + bv.koff[x], bv.koff[x + 1] - bv.koff[x], bv.kheap + bv.koff[y],
                               bv.koff[y + 1] - bv.koff[y]) != 0;
            }
            keep[a + i] = last ? 1 : 0;
        }
    }
}

// ---------------------------------------------------------------------------
// Paths: marks, verification status

// Mark every node on the root->target path (levels 1..L) of each target.
// Targets are either the segments with a batch run (bseg_off != NULL) or an
// explicit list of buckets at level L.
__global__ void k_mark_paths(DevTree t, uint32_t L, const uint64_t *bseg_off, const uint64_t *targets,
                             uint64_t ntargets, uint8_t *mark) {
    for (uint64_t i = gtid(); i < ntargets; i += gstride()) {
        uint64_t tb;
        if (bseg_off) {
            if (bseg_off[i] == bseg_off[i + 1]) continue;
            tb = i;
        } else {
            tb = targets[i];
        }
        for (uint32_t l = 1; l <= L; l++) {
            const uint64_t b = tb >> (t.shift * (L - l));
            mark[t.base[l] + b] = 1;
        }
    }
}

// Mark the ancestors (levels 1..H+1) of segments flagged in segflag[].
__global__ void k_mark_from_segments(DevTree t, const uint8_t *segflag, uint8_t *mark) {
    const uint32_t L = t.H + 1;
    for (uint64_t s = gtid(); s < t.S; s += gstride()) {
        if (!segflag[s]) continue;
        for (uint32_t l = 1; l <= L; l++) mark[t.base[l] + (s >> (t.shift * (L - l)))] = 1;
    }
}

// First failing level on each target's root->target path (0 = verified).
// (A streaming batch's segments: k_page_place, pages.h.)
__global__ void k_path_status(DevTree t, uint32_t L, const uint64_t *bseg_off, const uint64_t *targets,
                              uint64_t ntargets, const uint8_t *ok, uint8_t *seg_reject, uint32_t *tstatus) {
    for (uint64_t i = gtid(); i < ntargets; i += gstride()) {
        uint64_t tb;
        if (bseg_off) {
            if (bseg_off[i] == bseg_off[i + 1]) { seg_reject[i] = 0; continue; }
            tb = i;
        } else {
            tb = targets[i];
        }
        uint32_t bad = 0;
        for (uint32_t l = 1; l <= L; l++) {
            const uint64_t b = tb >> (t.shift * (L - l));
            if (!ok[t.base[l] + b]) { bad = l; break; }
        }
        if (seg_reject) seg_reject[i] = (uint8_t)bad;
        if (tstatus) tstatus[i] = bad;
    }
}

// ---------------------------------------------------------------------------
// K1 segment_hash: hash(Segment) = <<0, md5(V1 ‖ … ‖ Vn)>> (synctree.erl:255-259)
// one lane per segment; the values of a segment are one contiguous range.
// MODE_STORE writes the parent's entry (rehash, synctree.erl:515-527);
// MODE_VERIFY checks it like verify_hash/2 (synctree.erl:322-340).
template <int MODE>
__global__ void k_segment_hash(DevTree t, const uint8_t *mask, const uint32_t *list, const uint32_t *list_cnt,
                               uint8_t *ok, uint32_t *fail) {
    const uint32_t L = t.H + 1;
    const uint64_t n = (list && list_cnt) ? (uint64_t)*list_cnt : t.S;   // list without a count: a permutation of the segments
    for (uint64_t i = gtid(); i < n; i += gstride()) {
        const uint64_t s = list ? list[i] : i;
        const uint64_t slot = t.base[L] + s;
        if (mask && !mask[slot]) continue;
        const uint64_t e0 = t.seg_off[s], e1 = t.seg_end[s];
        const uint64_t eslot = (L == 1) ? 0 : slot;
        if (MODE == MODE_VERIFY) {
            const uint16_t et = t.tag[eslot];
            bool good;
            if (!(et & TAG_PRESENT)) {
                good = (e0 == e1);
            } else {
                uint32_t d[4];
                const uint64_t v0 = t.seg_voff[s];
                stmd5::md5_global_pf<true>(t.vheap + v0, t.seg_vend[s] - v0, d);
                const uint4 e = t.md5[eslot];
                good = (et == TAG_PRESENT) && e.x == d[0] && e.y == d[1] && e.z == d[2] && e.w == d[3];
            }
            if (ok) ok[slot] = good ? 1 : 0;
            if (!good && fail) atomicOr(fail, 1u);
        } else {
            if (e0 == e1) {
                t.tag[slot] = 0;
                if (L == 1) t.tag[0] = 0;
            } else {
                uint32_t d[4];
                const uint64_t v0 = t.seg_voff[s];
                stmd5::md5_global_pf<true>(t.vheap + v0, t.seg_vend[s] - v0, d);
                const uint4 e = make_uint4(d[0], d[1], d[2], d[3]);
                t.md5[slot] = e;
                t.tag[slot] = TAG_PRESENT;
                if (L == 1) { t.md5[0] = e; t.tag[0] = TAG_PRESENT; }
            }
        }
    }
}

// Appends bytes to a lane's LDS message with a 64-bit shift accumulator,
// emitting aligned dwords (instead of one ds_write_b8 per byte).
struct MsgWriter {
    uint32_t *w;
    uint64_t acc;
    uint32_t nb, nw;
    __device__ __forceinline__ void init(uint8_t *reg) { w = reinterpret_cast<uint32_t *>(reg); acc = 0; nb = 0; nw = 0; }
    __device__ __forceinline__ void push(uint32_t x, uint32_t bits) {
        acc |= (uint64_t)x << nb;
        nb += bits;
        if (nb >= 32) { w[nw++] = (uint32_t)acc; acc >>= 32; nb -= 32; }
    }
    __device__ __forceinline__ void entry(uint32_t tag, const uint4 &h) {
        push(tag & 0xffu, 8); push(h.x, 32); push(h.y, 32); push(h.z, 32); push(h.w, 32);
    }
    __device__ __forceinline__ uint32_t finish() {
        if (nb) w[nw] = (uint32_t)acc;
        return nw * 4 + nb / 8;
    }
};

// Stage the content of inner node (l, b) — the present child entries, 17
// bytes each in child order — into this lane's LDS region; returns its length.
// All W child entries are loaded before any is inspected (one memory round
// trip per 16 children, not one per child).
__device__ __forceinline__ uint32_t stage_inner(const DevTree &t, uint32_t l, uint64_t b, uint8_t *reg) {
    const uint64_t c0 = t.base[l + 1] + b * t.W;
    uint32_t len = 0;
    for (uint32_t j0 = 0; j0 < t.W; j0 += 16) {
        uint32_t tg[16];
        uint4 h[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            if (j0 + j < t.W) { tg[j] = t.tag[c0 + j0 + j]; h[j] = t.md5[c0 + j0 + j]; }
            else tg[j] = 0;
        }
        bool all = t.W == 16;
#pragma unroll
        for (int j = 0; j < 16; j++) all = all && (tg[j] & TAG_PRESENT);
        if (all) {   // W = 16, every child present: the byte positions are compile-time constants
            MsgWriter m16;
            m16.init(reg);
#pragma unroll
            for (int j = 0; j < 16; j++) m16.entry(tg[j], h[j]);
            return m16.finish();
        }
        // some child absent: each present entry at 17 x its rank, byte stores
        // (compact code: these kernels run it once per launch, cold)
        uint32_t pres = 0;
#pragma unroll
        for (int j = 0; j < 16; j++) pres |= (tg[j] & TAG_PRESENT) ? (1u << j) : 0u;
#pragma unroll
        for (int j = 0; j < 16; j++)
            if ((pres >> j) & 1u) {
                uint8_t *q = reg + len + 17u * (uint32_t)__builtin_popcount(pres & ((1u << j) - 1u));
                const uint32_t w4[4] = {h[j].x, h[j].y, h[j].z, h[j].w};
                q[0] = (uint8_t)tg[j];
#pragma unroll
                for (int x = 0; x < 16; x++) q[1 + x] = (uint8_t)(w4[x >> 2] >> (8 * (x & 3)));
            }
        len += 17u * (uint32_t)__builtin_popcount(pres);
    }
    return len;
}

// Bytes of LDS per lane for inner-node staging (odd dword stride).
__host__ __device__ __forceinline__ uint32_t lane_region_bytes(uint32_t W) {
    uint32_t dw = (W * 17 + 72 + 3) / 4;
    if ((dw & 1) == 0) dw++;
    return dw * 4;
}

// K2 level_rehash: one lane per inner node of a level (rehash/4 inner part,
// synctree.erl:515-535), children staged in LDS.  Nodes of level l are
// processed after level l+1.  With levels == 0 the kernel covers every level
// in [lmin, lmax] in one launch (only valid for MODE_VERIFY, whose nodes are
// independent).
template <int MODE>
__global__ void k_level_hash(DevTree t, uint32_t lmin, uint32_t lmax, const uint8_t *mask, const uint32_t *list,
                             const uint32_t *list_cnt, uint8_t *ok, uint32_t *fail) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t *reg = lds + threadIdx.x * lane_region_bytes(t.W);
    const uint64_t lo = t.base[lmin], hi = t.base[lmax + 1];
    const uint64_t n = list ? (uint64_t)*list_cnt : (hi - lo);
    for (uint64_t i = gtid(); i < n; i += gstride()) {
        uint64_t slot;
        uint32_t l = lmin;
        if (list) {
            slot = t.base[lmin] + list[i];
        } else {
            slot = lo + i;
            while (t.base[l + 1] <= slot) l++;
        }
        if (mask && !mask[slot]) continue;
        const uint64_t b = slot - t.base[l];
        const uint32_t len = stage_inner(t, l, b, reg);
        const uint64_t eslot = (l == 1) ? 0 : slot;
        if (MODE == MODE_VERIFY) {
            const uint16_t et = t.tag[eslot];
            bool good;
            if (!(et & TAG_PRESENT)) {
                good = (len == 0);
            } else {
                uint32_t d[4];
                stmd5::md5_lds(reg, len, d);
                const uint4 e = t.md5[eslot];
                good = (et == TAG_PRESENT) && e.x == d[0] && e.y == d[1] && e.z == d[2] && e.w == d[3];
            }
            if (ok) ok[slot] = good ? 1 : 0;
            if (!good && fail) atomicOr(fail, 1u);
        } else {
            if (len == 0) {
                t.tag[slot] = 0;
                if (l == 1) t.tag[0] = 0;
            } else {
                uint32_t d[4];
                stmd5::md5_lds(reg, len, d);
                const uint4 e = make_uint4(d[0], d[1], d[2], d[3]);
                t.md5[slot] = e;
                t.tag[slot] = TAG_PRESENT;
                if (l == 1) { t.md5[0] = e; t.tag[0] = TAG_PRESENT; }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Merge a sorted batch into the segment CSR (insert/3's orddict:store,
// synctree.erl:206, applied per segment with last-writer-wins).

struct MergeArgs {
    // old tree (canonical CSR or pages: segment s = entries [seg_off[s], seg_end[s]))
    const uint64_t *seg_off;
    const uint64_t *seg_end;
    const uint64_t *koff;
    const uint8_t *kheap;
    const uint64_t *voff;
    const uint8_t *vheap;
    // batch (sorted order = perm, runs = bseg_off, keep = last writer)
    const uint32_t *perm;
    const uint64_t *bseg_off;
    const uint8_t *keep;
    const uint8_t *bop;         // NULL: all PUT; else 1 = ERASE
    const uint8_t *seg_reject;  // NULL or per segment: nonzero => batch run ignored
    const uint8_t *seg_replace; // NULL or per segment: nonzero => old run dropped
    BatchView bv;
    const uint64_t *bvoff;
    const uint8_t *bvheap;
    const uint64_t *kbeg;       // NULL or per segment (PageMeta::kbeg): koff[seg_off[s]]
    const uint16_t *klen;       // NULL or per segment (pages.h PageMeta::klen): every key record this long
    const uint16_t *vlen;       // NULL or per segment (PageMeta::vlen): every value this long (with klen: a uniform
                                // page, whose per-entry offsets are by stride, pages.h)
    uint64_t S;
    uint64_t plo, phi;          // the segments the batch keeps: [0, S), or a partition's (k_clamp_runs)
};

// Running sums of the merge: per sorted batch record (BatchSums: eq = kept and
// overwrites/erases an old entry, ne = kept and not an ERASE, i.e. produces an
// entry; ke/ve = key/value bytes of the old entry it drops, kn/vn = its own
// key/value bytes when it produces an entry) and per segment (SegSums: entry
// count, key bytes, value bytes of the merged segment).  Exclusive scans of
// both give every merged entry its index and heap offsets in closed form.
template <int N>
struct USum {
    uint64_t v[N];
    __host__ __device__ USum() {}
    __host__ __device__ USum(int z) {
        for (int i = 0; i < N; i++) v[i] = (uint64_t)z;
    }
    __host__ __device__ USum operator+(const USum &o) const {
        USum r;
        for (int i = 0; i < N; i++) r.v[i] = v[i] + o.v[i];
        return r;
    }
};
typedef USum<6> BatchSums;   // eq, ne, ke, kn, ve, vn
typedef USum<4> SegSums;     // count, key bytes, value bytes, new keys of the tree
enum { BS_EQ = 0, BS_NE, BS_KE, BS_KN, BS_VE, BS_VN };

// ---------------------------------------------------------------------------
// Parallel merge.  Only the batch runs are walked: every kept batch record r
// of segment s gets pos_r = lower_bound(old keys of s, key_r), eq_r (key
// present) and ne_r (not an ERASE).  With exclusive scans of the BatchSums
// over the sorted batch (E = eq count, N = ne count, KE/KN/VE/VN = bytes) and
// of the SegSums over the segments (C, K, V), the merged layout is closed-form:
//   old entry li of s (dropped iff some eq_r has pos_r == li), with
//   k = #{r in run: pos_r <= li}, k2 = #{r in run: pos_r < li}:
//     index = C[s] + li - E(k2) + N(k)
//     key   = K[s] + (okoff[li] - okoff[0]) - KE(k2) + KN(k)   (values alike)
//   batch record r with ne_r:
//     index = C[s] + pos_r - E(r) + N(r)
//     key   = K[s] + (okoff[pos_r] - okoff[0]) - KE(r) + KN(r)
// (run-relative sums), so k_merge_old moves every old entry -- offsets and
// bytes -- in one coalesced pass and k_merge_new places the batch records:
// the whole CSR is rewritten once, with no per-entry source list, length
// arrays or entry-sized scans.
// Per sorted batch record, for the paged merge (pages.h): the old key and
// value offsets of the entry at its position, relative to its segment's
// first ones (a page rebuild moves segments, not their content), and its own
// batch offsets.
// The checked mode of streaming batches (st_debug_knob ST_DBG_PAGE_CHECK):
// the page arrays' capacities, and the violation record (pages.h pg_ok) the
// kernels that read pages fill instead of indexing out of them.
struct PageBounds {
    uint64_t cap_e, cap_k, cap_v;
    unsigned long long *chk;   // nullptr: unchecked
};
__device__ __forceinline__ bool page_bounds_ok(unsigned long long *chk, bool ok, uint32_t code, uint64_t s, uint64_t x,
                                               uint64_t bound) {
    if (ok || !chk) return true;
    if (atomicAdd(&chk[0], 1ull) == 0) { chk[1] = code; chk[2] = s; chk[3] = x; chk[4] = bound; }
    return false;
}
#define KLEN_MIXED_ 0        // = pages.h KLEN_MIXED (no uniform key length)
#define KLEN_NONE_ 0xFFFFu   // = pages.h KLEN_NONE (an empty segment)
struct RecAt {
    uint64_t ku, vu, bk, bv;
};

// Merge positions, a lane per sorted batch record: binary search of its key
// among its segment's old keys.  (A lane per segment searched its run's keys
// one after another: the longest run of a wave set its time, and the lanes of
// untouched segments idled.)  Records outside every run (a partition's
// clamped runs) are skipped and keep sums 0; a rejected segment's records get
// position 0 and sums 0.
// sd (optional, zeroed; the streaming batch): every segment's merged-size
// DELTAS (entries, key bytes, value bytes -- mod 2^64 -- and new keys) by
// atomics, dirty (zeroed) set by a kept record, fpos (all ones) = the
// smallest value offset a kept record changes (atomicMin): the per-segment
// sums without a pass over every segment.
// pb.chk (checked mode): a segment whose entries or key / value bytes lie
// outside the page arrays is reported (codes 30, 31) and not searched.
__global__ void k_merge_keys(MergeArgs a, const uint32_t *sseg, uint64_t n, uint32_t *pos, BatchSums *bs, RecAt *rat,
                             SegSums *sd = nullptr, uint8_t *dirty = nullptr, unsigned long long *fpos = nullptr,
                             PageBounds pb = PageBounds{0, 0, 0, nullptr}) {
    // a record is kept iff it lies in the kept segments' records [A, B) (the
    // runs are sorted by segment, and k_clamp_runs empties the runs outside
    // [plo, phi)): a wave-uniform check, not a load of its own run's bounds
    const uint64_t A = a.bseg_off[a.plo], B = a.bseg_off[a.phi];
    for (uint64_t j = gtid(); j < n; j += gstride()) {
        if (j < A || j >= B) continue;
        const uint64_t s = sseg[j];
        BatchSums f(0);
        if (a.seg_reject && a.seg_reject[s]) { pos[j] = 0; bs[j] = f; continue; }
        const uint64_t i0 = a.seg_off ? a.seg_off[s] : 0;
        if (pb.chk && a.seg_off) {
            const uint64_t e1 = a.seg_end[s];
            if (!page_bounds_ok(pb.chk, i0 <= e1 && e1 < pb.cap_e, 30, s, e1, pb.cap_e) ||
                !page_bounds_ok(pb.chk, a.koff[i0] <= a.koff[e1] && a.koff[e1] <= pb.cap_k && a.voff[i0] <= a.voff[e1] &&
                                            a.voff[e1] <= pb.cap_v, 31, s, a.koff[e1], pb.cap_k)) {
                pos[j] = 0;
                bs[j] = f;
                if (rat) rat[j] = RecAt{0, 0, 0, 0};
                continue;
            }
        }
        const uint64_t nold = (!a.seg_off || (a.seg_replace && a.seg_replace[s])) ? 0 : a.seg_end[s] - i0;
        const uint32_t bi = a.perm[j];
        const uint8_t *kb = a.bv.kheap + a.bv.koff[bi];
        const uint64_t kl = a.bv.koff[bi + 1] - a.bv.koff[bi];
        uint32_t L = (a.klen && nold) ? a.klen[s] : KLEN_MIXED_;
        if (L == KLEN_NONE_) L = KLEN_MIXED_;
        uint32_t V = (a.vlen && nold) ? a.vlen[s] : KLEN_MIXED_;   // uniform values: offsets by stride
        if (V == KLEN_NONE_ || L == KLEN_MIXED_) V = KLEN_MIXED_;
        uint64_t lo = 0, hi = nold, ke = 0;
        bool eq;
        if (L == 9 && kl == 9 && kb[0] == KEYTAG_INT) {
            // int64 keys among 9-byte records (a 9-byte record with the int
            // tag is an int64, krec_is_term): each probe is (tag, 8-byte
            // big-endian payload), all of it in ONE round trip (three dword
            // loads of the aligned window -- a record's bytes and up to 3 of
            // its neighbour's, heaps keep slack); a different tag decides
            // by itself (its first order byte).
            const uint8_t *k0 = a.kheap + (a.kbeg ? a.kbeg[s] : a.koff[i0]);
            const uint64_t kv = krec_be64(kb + 1);
            bool hit = false;
#ifndef ST_NO_INTERP
            // INTERPOLATION first (a segment's keys are a uniform sample of the
            // key space: the segment is the key's MD5): the page's first and
            // last keys (one round trip), then a window of MI_W keys around the
            // interpolated position (one more); the bisection below only
            // finishes a miss, inside the side the window leaves.  Every bound
            // is a probed key, so the position and `hit` are the bisection's.
            if (nold >= MI_W + 2) {
                uint32_t tf, tl;
                uint64_t pf, pl;
                krec9_load(k0, tf, pf);
                krec9_load(k0 + 9 * (nold - 1), tl, pl);
                if (tf == KEYTAG_INT && tl == KEYTAG_INT) {   // every key int-tagged (sorted: first and last are)
                    if (kv <= pf) {
                        hit = kv == pf; hi = 0;                 // position 0
                    } else if (kv >= pl) {
                        hit = kv == pl; lo = hi = kv == pl ? nold - 1 : nold;
                    } else {                                    // position in [1, nold - 1]
                        const double fr = (double)(kv - pf) / (double)(pl - pf);
                        const int64_t g = (int64_t)(fr * (double)(nold - 1)) - MI_W / 2;
                        const uint64_t w0 = g < 1 ? 1 : ((uint64_t)g + MI_W + 1 > nold ? nold - 1 - MI_W : (uint64_t)g);
                        uint32_t c = 0;
#pragma unroll
                        for (int q = 0; q < MI_W; q++) {
                            uint32_t tg;
                            uint64_t pv;
                            krec9_load(k0 + 9 * (w0 + q), tg, pv);
                            c += pv < kv ? 1u : 0u;
                            hit |= pv == kv;
                        }
                        if (c == 0) { lo = 1; hi = w0; }                       // key[w0] >= kv was probed
                        else if (c == MI_W) { lo = w0 + MI_W; hi = nold - 1; } // key[nold - 1] > kv
                        else { lo = hi = w0 + c; }
                    }
                }
            }
#endif
            while (lo < hi) {
                const uint64_t mid = (lo + hi) >> 1;
                uint32_t tag;
                uint64_t pv;
                krec9_load(k0 + 9 * mid, tag, pv);
                const int c = tag != KEYTAG_INT ? (tag < KEYTAG_INT ? -1 : 1) : (pv < kv ? -1 : (pv > kv ? 1 : 0));
                hit |= c == 0;
                if (c < 0) lo = mid + 1; else hi = mid;
            }
            eq = hit;   // the keys of a segment are unique: an equal probe is where the search ends
            ke = L;
        } else if (L != KLEN_MIXED_) {   // every old key L bytes: entry i's key at k0 + L i, no offset loads
            const uint8_t *k0 = a.kheap + (a.kbeg ? a.kbeg[s] : a.koff[i0]);
            while (lo < hi) {
                const uint64_t mid = (lo + hi) >> 1;
                if (rec_cmp(k0 + L * mid, L, kb, kl) < 0) lo = mid + 1; else hi = mid;
            }
            eq = lo < nold && rec_cmp(k0 + L * lo, L, kb, kl) == 0;
            ke = L;
        } else {
            while (lo < hi) {
                const uint64_t mid = (lo + hi) >> 1, e = i0 + mid;
                if (rec_cmp(a.kheap + a.koff[e], a.koff[e + 1] - a.koff[e], kb, kl) < 0) lo = mid + 1; else hi = mid;
            }
            const uint64_t e = i0 + lo;
            eq = lo < nold && rec_cmp(a.kheap + a.koff[e], a.koff[e + 1] - a.koff[e], kb, kl) == 0;
            if (eq) ke = a.koff[e + 1] - a.koff[e];
        }
        const uint64_t e = i0 + lo;
        pos[j] = (uint32_t)lo;
        if (rat)
            rat[j] = RecAt{L != KLEN_MIXED_ ? L * lo : a.koff[e] - a.koff[i0],
                           V != KLEN_MIXED_ ? V * lo : a.voff[e] - a.voff[i0], a.bv.koff[bi], a.bvoff[bi]};
        const bool kept = a.keep[j] != 0;
        const bool ne = kept && !(a.bop && a.bop[bi]);
        if (kept && eq) {
            f.v[BS_EQ] = 1;
            f.v[BS_KE] = ke;
            f.v[BS_VE] = V != KLEN_MIXED_ ? V : a.voff[e + 1] - a.voff[e];
        }
        if (ne) {
            f.v[BS_NE] = 1;
            f.v[BS_KN] = kl;
            f.v[BS_VN] = a.bvoff[bi + 1] - a.bvoff[bi];
        }
        bs[j] = f;
        if (sd && kept) {
            unsigned long long *d = reinterpret_cast<unsigned long long *>(&sd[s]);
            if (f.v[BS_NE] != f.v[BS_EQ]) atomicAdd(&d[0], (unsigned long long)(f.v[BS_NE] - f.v[BS_EQ]));
            if (f.v[BS_KN] != f.v[BS_KE]) atomicAdd(&d[1], (unsigned long long)(f.v[BS_KN] - f.v[BS_KE]));
            if (f.v[BS_VN] != f.v[BS_VE]) atomicAdd(&d[2], (unsigned long long)(f.v[BS_VN] - f.v[BS_VE]));
            if (ne && !eq) atomicAdd(&d[3], 1ull);   // a new key of the tree
            dirty[s] = 1;
            atomicMin(&fpos[s], (unsigned long long)(V != KLEN_MIXED_ ? V * lo : a.voff[e] - a.voff[i0]));
        }
    }
}

// A segment's merged sizes (SegSums: entries, key bytes, value bytes, new
// keys) from its old sizes and its run's BatchSums; dirty = a kept record.
// Returns the value offset (relative to the segment's first value) of the
// first entry the merge changes -- the first kept record's position -- or ~0.
__device__ __forceinline__ uint64_t merge_sums_seg(const MergeArgs &a, uint64_t s, const BatchSums *bs, const RecAt *rat,
                                                   const uint32_t *pos, SegSums *ss, uint8_t *dirty) {
    const uint64_t i0 = a.seg_off ? a.seg_off[s] : 0;
    const uint64_t nold = (!a.seg_off || (a.seg_replace && a.seg_replace[s])) ? 0 : a.seg_end[s] - i0;
    const uint64_t j0 = a.bseg_off[s], je = a.bseg_off[s + 1];
    SegSums tot;
    tot.v[0] = nold;
    tot.v[1] = nold ? a.koff[i0 + nold] - a.koff[i0] : 0;
    tot.v[2] = nold ? a.voff[i0 + nold] - a.voff[i0] : 0;
    tot.v[3] = 0;
    uint64_t first = ~0ull;
    if (!(a.seg_reject && a.seg_reject[s]))
        for (uint64_t j = j0; j < je; j++) {
            const BatchSums f = bs[j];
            if (first == ~0ull && a.keep[j]) first = rat ? rat[j].vu : (pos[j] ? a.voff[i0 + pos[j]] - a.voff[i0] : 0);
            if (f.v[BS_NE] && !f.v[BS_EQ]) tot.v[3] += 1;   // a new key of the tree
            tot.v[0] += f.v[BS_NE] - f.v[BS_EQ];
            tot.v[1] += f.v[BS_KN] - f.v[BS_KE];
            tot.v[2] += f.v[BS_VN] - f.v[BS_VE];
        }
    ss[s] = tot;
    if (dirty) dirty[s] = first != ~0ull ? 1 : 0;
    return first;
}

__global__ void k_merge_sums(MergeArgs a, const BatchSums *bs, const uint32_t *pos, SegSums *ss, uint8_t *dirty) {
    for (uint64_t s = gtid(); s < a.S; s += gstride()) merge_sums_seg(a, s, bs, nullptr, pos, ss, dirty);
}

// The MD5 state of a segment's values before the first block its merge
// changes (k = that block; k == 0: none kept), saved by the verify of a
// streaming batch for the hash after the merge.
// The MD5 form of the lane-per-segment span hashes (verify, dirty hash): the
// latency form (add3), measured faster here than the throughput form that
// K1 uses -- these lanes wait on their own chains (config-5 batch: hash 0.301
// -> 0.287 ms, verify 0.381 -> 0.377 ms; profiles/r06ak_span_md5_form_ab/).
#ifndef ST_SPAN_TPUT
#define ST_SPAN_TPUT false
#endif
struct PrefixState {
    uint4 st;
    uint64_t k;
};

// A streaming batch's verify (insert/3's get_path check of each touched
// segment, synctree.erl:189-209, 302-340): a lane per segment in seg_perm
// order hashes a touched segment's old values, saving the state before the
// first block its merge changes (fpos, k_merge_keys) in ps for the hash after
// the merge.
// pb.chk (checked mode): a segment whose value span lies outside the value
// array is reported (code 32) and not hashed.
// ntot (optional): perm is a list of *ntot segments, not all S.
__global__ void __launch_bounds__(256) k_verify_cap(DevTree t, const uint32_t *perm, const uint8_t *mask, uint8_t *ok,
                                                    const unsigned long long *fpos, PrefixState *ps,
                                                    PageBounds pb = PageBounds{0, 0, 0, nullptr},
                                                    const uint32_t *ntot = nullptr) {
    const uint32_t L = t.H + 1;
    const uint64_t n = ntot ? (uint64_t)*ntot : t.S;
    for (uint64_t i = gtid(); i < n; i += gstride()) {
        const uint64_t s = perm[i];
        const uint64_t slot = t.base[L] + s;
        if (!mask[slot]) continue;
        const uint64_t eslot = (L == 1) ? 0 : slot;
        const uint16_t et = t.tag[eslot];
        PrefixState p;
        p.k = 0;
        p.st = make_uint4(0u, 0u, 0u, 0u);
        bool good;
        if (!page_bounds_ok(pb.chk, t.seg_voff[s] <= t.seg_vend[s] && t.seg_vend[s] <= pb.cap_v, 32, s, t.seg_vend[s],
                            pb.cap_v)) {
            good = false;
        } else if (!(et & TAG_PRESENT)) {
            good = t.seg_off[s] == t.seg_end[s];
        } else {
            uint32_t st[4], cap[4] = {0u, 0u, 0u, 0u};
            stmd5::init(st);
            const uint64_t first = fpos[s];
            const uint64_t ck = first == ~0ull ? ~0ull : first / 64;
            const uint64_t v0 = t.seg_voff[s];
            stmd5::md5_global_span<ST_SPAN_TPUT>(t.vheap + v0, t.seg_vend[s] - v0, 0, st, ck, cap);
            const uint4 e = t.md5[eslot];
            good = (et == TAG_PRESENT) && e.x == st[0] && e.y == st[1] && e.z == st[2] && e.w == st[3];
            if (ck != ~0ull && ck > 0) {
                p.k = ck;
                p.st = make_uint4(cap[0], cap[1], cap[2], cap[3]);
            }
        }
        ok[slot] = good ? 1 : 0;
        ps[s] = p;
    }
}


__device__ __forceinline__ uint64_t bound_pos(const uint32_t *pos, uint64_t lo, uint64_t hi, uint64_t li, bool upper) {
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        const bool go = upper ? pos[mid] <= li : pos[mid] < li;
        if (go) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// Output of the merge: the new CSR.
struct MergeOut {
    uint64_t *seg_off, *seg_voff;   // S + 1
    uint64_t *koff, *voff;          // n_new + 1
    uint8_t *kheap, *vheap;
};

// Old entries: a workgroup per 256 consecutive segments walks their old
// entries with consecutive threads on consecutive entries, writing each
// surviving entry's new offsets and bytes; it also writes the new segment
// offsets of its segments (and the terminal offsets, from the last segment).
// Everything an entry needs besides its own offsets and bytes -- its
// segment's bounds, merged sums, replace / reject flags, first key and value
// offsets, and the segment's batch run (positions and run-relative sums) --
// is staged in LDS once per workgroup, so an entry costs one round trip for
// its offsets and one for its bytes instead of a chain of per-entry loads.
#define MO_RUNCAP 512   // batch records of a workgroup's segments staged in LDS (more: read from global memory)
__global__ void __launch_bounds__(256) k_merge_old(MergeArgs a, const uint32_t *pos, const BatchSums *bx,
                                                   const SegSums *sx, MergeOut o) {
    __shared__ uint64_t so[257], sb[257], kb0[257], vb0[257];
    __shared__ SegSums sxs[256];
    __shared__ uint8_t flg[256];                  // 1 = old run replaced, 2 = batch run rejected
    __shared__ uint32_t rpos[MO_RUNCAP];
    __shared__ uint32_t rbx[MO_RUNCAP + 1][6];    // batch sums relative to the workgroup's first record
    const uint32_t tid = threadIdx.x;
    const uint64_t s0 = (uint64_t)blockIdx.x * 256;
    const uint64_t ns = a.S - s0 < 256 ? a.S - s0 : 256;
    for (uint32_t i = tid; i <= ns; i += 256) {
        so[i] = a.seg_off ? a.seg_off[s0 + i] : 0;
        sb[i] = a.bseg_off[s0 + i];
        if (i < ns || s0 + i == a.S) {
            const SegSums x = sx[s0 + i];
            if (i < ns) sxs[i] = x;
            o.seg_off[s0 + i] = x.v[0];
            o.seg_voff[s0 + i] = x.v[2];
            if (s0 + i == a.S) { o.koff[x.v[0]] = x.v[1]; o.voff[x.v[0]] = x.v[2]; }
        }
        if (i < ns)
            flg[i] = (uint8_t)((a.seg_replace && a.seg_replace[s0 + i] ? 1u : 0u) | (a.seg_reject && a.seg_reject[s0 + i] ? 2u : 0u));
    }
    __syncthreads();
    for (uint32_t i = tid; i <= ns; i += 256) {   // first key / value offsets of each segment
        kb0[i] = a.seg_off ? a.koff[so[i]] : 0;
        vb0[i] = a.seg_off ? a.voff[so[i]] : 0;
    }
    const uint64_t j0w = sb[0], nbw = sb[ns] - sb[0];
    const bool staged = nbw + 1 <= MO_RUNCAP;
    if (staged) {
        for (uint64_t j = tid; j <= nbw; j += 256) {
            if (j < nbw) rpos[j] = pos[j0w + j];
            const BatchSums &x = bx[j0w + j], &x0 = bx[j0w];
#pragma unroll
            for (int q = 0; q < 6; q++) rbx[j][q] = (uint32_t)(x.v[q] - x0.v[q]);
        }
    }
    __syncthreads();
    const uint64_t e0 = so[0], e1 = so[ns];
    for (uint64_t e = e0 + tid; e < e1; e += 256) {
        uint32_t lo = 0, hi = (uint32_t)ns;   // local segment: so[k] <= e < so[k+1]
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (so[mid] <= e) lo = mid; else hi = mid;
        }
        const uint8_t f = flg[lo];
        if (f & 1) continue;
        const uint64_t i0 = so[lo], li = e - i0;
        const uint64_t okb = a.koff[e], ovb = a.voff[e];
        const uint64_t kl = a.koff[e + 1] - okb, vl = a.voff[e + 1] - ovb;
        const SegSums &base = sxs[lo];
        uint64_t nw = base.v[0] + li, nk = base.v[1] + (okb - kb0[lo]), nv = base.v[2] + (ovb - vb0[lo]);
        const uint64_t j0 = sb[lo], je = sb[lo + 1];
        if (j0 != je && !(f & 2)) {
            if (staged) {
                const uint32_t r0 = (uint32_t)(j0 - j0w), re = (uint32_t)(je - j0w);
                uint32_t k = r0, hk = re;   // upper bound: first pos > li
                while (k < hk) { const uint32_t mid = (k + hk) >> 1; if (rpos[mid] <= li) k = mid + 1; else hk = mid; }
                uint32_t k2 = r0, h2 = re;  // lower bound: first pos >= li
                while (k2 < h2) { const uint32_t mid = (k2 + h2) >> 1; if (rpos[mid] < li) k2 = mid + 1; else h2 = mid; }
                if (rbx[k][BS_EQ] != rbx[k2][BS_EQ]) continue;   // overwritten or erased by the batch
                // (each run-relative difference is >= 0; the sum may not be: 64-bit wrap as above)
                nw += (uint64_t)(rbx[k][BS_NE] - rbx[r0][BS_NE]) - (uint64_t)(rbx[k2][BS_EQ] - rbx[r0][BS_EQ]);
                nk += (uint64_t)(rbx[k][BS_KN] - rbx[r0][BS_KN]) - (uint64_t)(rbx[k2][BS_KE] - rbx[r0][BS_KE]);
                nv += (uint64_t)(rbx[k][BS_VN] - rbx[r0][BS_VN]) - (uint64_t)(rbx[k2][BS_VE] - rbx[r0][BS_VE]);
            } else {
                const uint64_t k = bound_pos(pos, j0, je, li, true), k2 = bound_pos(pos, j0, je, li, false);
                const BatchSums &B0 = bx[j0], &Bk = bx[k], &Bk2 = bx[k2];
                if (Bk.v[BS_EQ] != Bk2.v[BS_EQ]) continue;
                nw += (Bk.v[BS_NE] - B0.v[BS_NE]) - (Bk2.v[BS_EQ] - B0.v[BS_EQ]);
                nk += (Bk.v[BS_KN] - B0.v[BS_KN]) - (Bk2.v[BS_KE] - B0.v[BS_KE]);
                nv += (Bk.v[BS_VN] - B0.v[BS_VN]) - (Bk2.v[BS_VE] - B0.v[BS_VE]);
            }
        }
        o.koff[nw] = nk;
        o.voff[nw] = nv;
        copy_bytes(o.kheap + nk, a.kheap + okb, kl);
        copy_bytes(o.vheap + nv, a.vheap + ovb, vl);
    }
}

// Batch records that produce an entry (kept, not ERASE, run not rejected).
__global__ void k_merge_new(MergeArgs a, const uint32_t *sseg, uint64_t n, const uint32_t *pos, const BatchSums *bx,
                            const SegSums *sx, MergeOut o) {
    for (uint64_t j = gtid(); j < n; j += gstride()) {
        const BatchSums &Bj = bx[j];
        if (bx[j + 1].v[BS_NE] == Bj.v[BS_NE]) continue;
        const uint64_t s = sseg[j], j0 = a.bseg_off[s], p = pos[j];
        const BatchSums &B0 = bx[j0];
        const SegSums base = sx[s];
        uint64_t dk = 0, dv = 0;   // old bytes before pos (none when the old run is replaced)
        if (p) {
            const uint64_t i0 = a.seg_off[s];
            dk = a.koff[i0 + p] - a.koff[i0];
            dv = a.voff[i0 + p] - a.voff[i0];
        }
        const uint64_t nw = base.v[0] + p + (Bj.v[BS_NE] - B0.v[BS_NE]) - (Bj.v[BS_EQ] - B0.v[BS_EQ]);
        const uint64_t nk = base.v[1] + dk + (Bj.v[BS_KN] - B0.v[BS_KN]) - (Bj.v[BS_KE] - B0.v[BS_KE]);
        const uint64_t nv = base.v[2] + dv + (Bj.v[BS_VN] - B0.v[BS_VN]) - (Bj.v[BS_VE] - B0.v[BS_VE]);
        const uint32_t bi = a.perm[j];
        const uint64_t bk = a.bv.koff[bi], bv = a.bvoff[bi];
        o.koff[nw] = nk;
        o.voff[nw] = nv;
        copy_bytes(o.kheap + nk, a.bv.kheap + bk, a.bv.koff[bi + 1] - bk);
        copy_bytes(o.vheap + nv, a.bvheap + bv, a.bvoff[bi + 1] - bv);
    }
}

__global__ void k_seg_voff(const uint64_t *seg_off, const uint64_t *voff, uint64_t S, uint64_t *seg_voff) {
    for (uint64_t s = gtid(); s <= S; s += gstride()) seg_voff[s] = voff[seg_off[s]];
}

// Per batch key: insert status from its segment's path status.
__global__ void k_key_status(const uint32_t *seg, uint64_t n, const uint8_t *seg_reject, uint32_t *clevel) {
    for (uint64_t i = gtid(); i < n; i += gstride()) clevel[i] = seg_reject[seg[i]];
}

// Number of nonzero statuses (rejected keys of an insert batch): a wave
// reduction per wave, one global add per wave into *out (zeroed by the host).
__global__ void k_count_nonzero(const uint32_t *v, uint64_t n, unsigned long long *out) {
    unsigned long long c = 0;
    for (uint64_t i = gtid(); i < n; i += gstride()) c += v[i] != 0;
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

// ---------------------------------------------------------------------------
// Reads: get/2 lookups and exchange_get node images

// For each key (segment seg[i], record i of the batch): index of the entry in
// the tree with an equal key, or UINT64_MAX.  (orddict_find, synctree.erl:342-348)
__global__ void k_lookup(DevTree t, BatchView bv, const uint32_t *seg, uint64_t n, uint64_t *found) {
    for (uint64_t i = gtid(); i < n; i += gstride()) {
        const uint64_t s = seg[i];
        uint64_t lo = t.seg_off[s], hi = t.seg_end[s];
        const uint8_t *k = bv.kheap + bv.koff[i];
        const uint64_t kl = bv.koff[i + 1] - bv.koff[i];
        while (lo < hi) {
            const uint64_t m = (lo + hi) / 2;
            if (rec_cmp(t.kheap + t.koff[m], t.koff[m + 1] - t.koff[m], k, kl) < 0) lo = m + 1; else hi = m;
        }
        uint64_t r = ~0ull;
        if (lo < t.seg_end[s] && rec_cmp(t.kheap + t.koff[lo], t.koff[lo + 1] - t.koff[lo], k, kl) == 0) r = lo;
        found[i] = r;
    }
}

// ---------------------------------------------------------------------------
// K3 tree_compare: the level-synchronous diff of compare/3 (exchange,
// exchange_level, exchange_final: synctree.erl:372-417) of two trees of the
// same geometry, in passes with no host round trip in between.
//
// The frontier is evaluated without a level-by-level loop.  Node (L, b) is
// visited at level L iff the two top hashes differ (level 0,
// exchange_get(0,0) is not verified) and, for every level 2 <= k <= L, the
// two trees' entries of its level-k ancestor differ under the filter
// (orddict_delta, riak_ensemble_util.erl:115-141, plus filter/2,
// synctree.erl:434-449) -- exactly the set the reference's level loop reaches,
// since a child is added to the next frontier iff its parent was visited and
// its entries differ.  k_cmp_walk evaluates it per node, verifies every
// visited node on both sides against its parent's entry (exchange_get's
// verified_hashes, synctree.erl:288-298) and merge-joins every visited
// segment pair (exchange_final); each wave then writes its records after those
// of the waves above it.  Only the entries under visited nodes beyond level H are
// read.  err: min over (level, bucket, side) of a failed verification -- the
// reference's first crash in visiting order (local before remote).

__device__ __forceinline__ bool verify_inner_node(const DevTree &t, uint32_t l, uint64_t b, uint8_t *reg) {
    const uint64_t slot = t.base[l] + b;
    const uint64_t eslot = (l == 1) ? 0 : slot;
    // the parent's entry is loaded with the children (one round trip), not
    // after the hash: the compare at the end waits for nothing
    const uint16_t et = t.tag[eslot];
    const uint4 e = t.md5[eslot];
    const uint32_t len = stage_inner(t, l, b, reg);
    if (!(et & TAG_PRESENT)) return len == 0;
    uint32_t d[4];
    stmd5::md5_lds(reg, len, d);
    return (et == TAG_PRESENT) && e.x == d[0] && e.y == d[1] && e.z == d[2] && e.w == d[3];
}

__device__ __forceinline__ bool verify_segment(const DevTree &t, uint64_t s) {
    const uint32_t L = t.H + 1;
    const uint64_t slot = t.base[L] + s;
    const uint64_t eslot = (L == 1) ? 0 : slot;
    const uint16_t et = t.tag[eslot];
    if (!(et & TAG_PRESENT)) return t.seg_off[s] == t.seg_end[s];
    uint32_t d[4];
    const uint64_t v0 = t.seg_voff[s];
    stmd5::md5_global_pf(t.vheap + v0, t.seg_vend[s] - v0, d);
    const uint4 e = t.md5[eslot];
    return (et == TAG_PRESENT) && e.x == d[0] && e.y == d[1] && e.z == d[2] && e.w == d[3];
}

// verify/1 and verify_upper/1 (synctree.erl:549-571) in one launch: the
// top-down walk checks node (l, b) iff every entry on its path below the top
// (levels 2..l, its own included) is present -- a node whose parent entry
// is absent is never fetched -- and the answer is false iff a checked
// node's hash differs from its parent's entry.  A lane per slot of levels
// 1..lmax, then (segs) a lane per segment; reachability from the ancestors'
// tags inline (no mark pass, no memsets); a failure sets *fail, a word of
// host-mapped memory the host zeroed (system-scope OR, no copy back).
__device__ __forceinline__ bool path_present(const DevTree &t, uint32_t l, uint64_t b) {
    uint32_t all = TAG_PRESENT;   // the ancestors' tags eight at a time (one round trip, not one per level)
    for (uint32_t q0 = 2; q0 <= l; q0 += 8) {
#pragma unroll
        for (uint32_t k = 0; k < 8; k++)
            if (q0 + k <= l) all &= t.tag[t.base[q0 + k] + (b >> (t.shift * (l - q0 - k)))];
    }
    return (all & TAG_PRESENT) != 0;
}
__global__ void k_verify_tree(DevTree t, uint32_t lmax, int segs, uint32_t *fail) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t *reg = lds + threadIdx.x * lane_region_bytes(t.W);
    const uint64_t lo = t.base[1], nin = t.base[lmax + 1] - lo;
    const uint64_t n = nin + (segs ? t.S : 0);
    bool bad = false;
    for (uint64_t i = gtid(); i < n; i += gstride()) {
        if (i < nin) {
            const uint64_t slot = lo + i;
            uint32_t l = 1;
            while (t.base[l + 1] <= slot) l++;
            const uint64_t b = slot - t.base[l];
            if (path_present(t, l, b)) bad |= !verify_inner_node(t, l, b, reg);
        } else {
            const uint64_t s = i - nin;
            if (path_present(t, t.H + 1, s)) bad |= !verify_segment(t, s);
        }
    }
    if (__ballot(bad) && (threadIdx.x & 63) == __ffsll((long long)__ballot(bad)) - 1)
        __hip_atomic_fetch_or(fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint64_t err_code(uint32_t level, uint64_t bucket, uint32_t side) {
    return ((uint64_t)level << 56) | (bucket << 1) | side;
}

// One diff record: entry indices into the two trees' CSR (~0 = '$none').
struct DiffRec {
    uint64_t a, b, seg;
    uint32_t kind, pad;
};

// Does child entry `slot` differ between the trees under the filter?
// (1 = local_only drops {C,{H,'$none'}}, 2 = remote_only drops {C,{'$none',H}})
__device__ __forceinline__ bool entry_differs(uint16_t ta, uint16_t tb, const uint4 &x, const uint4 &y, int filter) {
    const bool pa = ta & TAG_PRESENT, pb = tb & TAG_PRESENT;
    if (pa && pb) return ta != tb || x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w;
    if (pa) return filter != 1;
    if (pb) return filter != 2;
    return false;
}

// Per-wave LDS of the segment merge-join: key offsets and key bytes of both
// segments, and one packed record per slot of the merged key sequence.
#define CMP_CAP 256     // entries per side handled from LDS (larger: lane 0 walks them)
#define CMP_KB 4096     // key bytes per side
#define CMP_VB 6144     // value bytes per side (larger: values compared in global memory)
__host__ __device__ __forceinline__ uint32_t cmp_merge_lds_bytes() {
    return (CMP_CAP + 1) * 4 * 4 + 2 * CMP_CAP * 4 + CMP_KB * 2 + CMP_VB * 2 + 2 * CMP_CAP * 16;
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Byte order of two strings staged in LDS at arbitrary byte offsets (byte
// reads: no unaligned wide LDS access).
__device__ __forceinline__ int lds_bytes_cmp(const uint8_t *a, uint32_t la, const uint8_t *b, uint32_t lb) {
    const uint32_t m = la < lb ? la : lb;
    for (uint32_t i = 0; i < m; i++) {
        const uint32_t x = a[i], y = b[i];
        if (x != y) return x < y ? -1 : 1;
    }
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

// Erlang term order of two key records staged in LDS
__device__ __forceinline__ int lds_rec_cmp(const uint8_t *a, uint32_t la, const uint8_t *b, uint32_t lb) {
    return lds_bytes_cmp(a, (uint32_t)krec_order_len(a, la), b, (uint32_t)krec_order_len(b, lb));
}

// Order prefix of a key record staged in LDS: its first 12 order bytes
// (krec_order_len) big-endian in x..z, zero-padded, and the order length in
// w.  Two prefixes decide the order unless both order lengths exceed 12 and
// the 12 bytes tie (pfx_cmp returns 2: compare the staged bytes).
__device__ __forceinline__ uint4 lds_key_prefix(const uint8_t *p, uint32_t len) {
    const uint32_t ol = (uint32_t)krec_order_len(p, len);
    uint32_t w[3] = {0, 0, 0};
#pragma unroll
    for (int k = 0; k < 12; k++)
        if ((uint32_t)k < ol) w[k >> 2] |= (uint32_t)p[k] << (24 - 8 * (k & 3));
    return make_uint4(w[0], w[1], w[2], ol);
}
__device__ __forceinline__ int pfx_cmp(const uint4 &x, const uint4 &y) {
    if (x.x != y.x) return x.x < y.x ? -1 : 1;
    if (x.y != y.y) return x.y < y.y ? -1 : 1;
    if (x.z != y.z) return x.z < y.z ? -1 : 1;
    if (x.w > 12 && y.w > 12) return 2;
    return x.w == y.w ? 0 : (x.w < y.w ? -1 : 1);
}

// lower_bound of key k (prefix kp, staged bytes k / kl) in the n staged keys
// of a segment (prefixes pk, offsets off, bytes kb); *eq: equal key found (a
// step that meets an equal key lands on it: keys of a segment are unique).
__device__ __forceinline__ uint32_t lds_lower_bound(const uint4 *pk, const uint32_t *off, const uint8_t *kb, uint32_t n,
                                                    const uint4 &kp, const uint8_t *k, uint32_t kl, bool *eq) {
    uint32_t lo = 0, hi = n;
    bool found = false;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        int c = pfx_cmp(pk[m], kp);
        if (c == 2) c = lds_rec_cmp(kb + off[m], off[m + 1] - off[m], k, kl);
        found |= c == 0;
        if (c < 0) lo = m + 1; else hi = m;
    }
    *eq = found;
    return lo;
}

// Equality of two byte strings staged in LDS: eight independent byte reads
// per step (one LDS round trip), no early exit inside a step.
__device__ __forceinline__ bool lds_bytes_eq(const uint8_t *a, uint32_t la, const uint8_t *b, uint32_t lb) {
    if (la != lb) return false;
    for (uint32_t i = 0; i < la; i += 8) {
        uint32_t d = 0;
#pragma unroll
        for (uint32_t k = 0; k < 8; k++)
            if (i + k < la) d |= (uint32_t)(a[i + k] ^ b[i + k]);
        if (d) return false;
    }
    return true;
}

__device__ __forceinline__ uint32_t wave_prefix_count(bool f, uint32_t lane) {
    const uint64_t bal = __ballot(f);
    return (uint32_t)__popcll(bal & ((1ull << lane) - 1));
}

// Wave-cooperative copy of up to 4 byte runs from global memory into LDS
// (destinations 4-byte aligned): a lane per destination dword, the two source
// dwords it straddles loaded (the run's first word aligned down; nothing read
// past the run's last dword) and joined with one v_alignbyte, one ds_write_b32
// per dword (byte stores only for a run's last partial dword).  Every load of
// an iteration is in flight together, so runs up to 1 KB cost one memory
// round trip.  One out-of-line copy per kernel (instruction-cache footprint).
// The sources are read as global memory and the destinations written as LDS
// (address-space casts): as generic pointers every access was a FLAT one,
// whose waits cover both memory and LDS traffic.
typedef __attribute__((address_space(1))) const uint32_t wc_gu32;
typedef __attribute__((address_space(3))) uint32_t wc_lu32;
typedef __attribute__((address_space(3))) uint8_t wc_lu8;
__device__ __noinline__ void wave_copy4(const uint8_t *s0, uint32_t n0, uint8_t *d0, const uint8_t *s1, uint32_t n1,
                                           uint8_t *d1, const uint8_t *s2, uint32_t n2, uint8_t *d2, const uint8_t *s3,
                                           uint32_t n3, uint8_t *d3) {
    const uint32_t lane = threadIdx.x & 63;
    const uint8_t *src[4] = {s0, s1, s2, s3};
    uint8_t *dst[4] = {d0, d1, d2, d3};
    const uint32_t len[4] = {n0, n1, n2, n3};
    uint32_t mx = n0 > n1 ? n0 : n1;
    mx = mx > n2 ? mx : n2;
    mx = mx > n3 ? mx : n3;
    for (uint32_t q0 = 0; q0 < mx; q0 += 1024) {
        uint32_t lo[4][4], hi[4][4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const uintptr_t a = reinterpret_cast<uintptr_t>(src[r]);
            const uint32_t mis = (uint32_t)(a & 3);
            wc_gu32 *w = (wc_gu32 *)(a - mis);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t q = q0 / 4 + u * 64 + lane;
                lo[r][u] = 4 * q < len[r] ? w[q] : 0u;
                hi[r][u] = mis && 4 * (q + 1) < len[r] + mis ? w[q + 1] : 0u;
            }
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(src[r]) & 3);
            wc_lu32 *dw = (wc_lu32 *)dst[r];
            wc_lu8 *db = (wc_lu8 *)dst[r];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t q = q0 / 4 + u * 64 + lane;
                const uint32_t v = __builtin_amdgcn_alignbyte(hi[r][u], lo[r][u], mis);
                if (4 * q + 4 <= len[r]) {
                    dw[q] = v;
                } else if (4 * q < len[r]) {
                    const uint32_t nb = len[r] - 4 * q;   // 1..3
                    db[4 * q] = (uint8_t)v;
                    if (nb > 1) db[4 * q + 1] = (uint8_t)(v >> 8);
                    if (nb > 2) db[4 * q + 2] = (uint8_t)(v >> 16);
                }
            }
        }
    }
}

// Exclusive prefix sum over the wave's lanes.
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x - v;
}

// exchange_final of one segment pair staged in LDS (orddict_delta +
// filter, riak_ensemble_util.erl:115-141, synctree.erl:434-449): ao / bo the
// key offsets (relative, n + 1), avo / bvo the value offsets (relative),
// ak / bk the key bytes, av / bv the values (vl: staged, else compared in
// global memory), ur nA + nB union slots.  Writes the pair's records in
// ascending key order to out[base..lim); returns their count.
__device__ uint64_t lds_merge_pair(const DevTree &A, const DevTree &B, uint64_t s, int filter, uint64_t a0, uint64_t b0,
                                   uint32_t nA, uint32_t nB, const uint32_t *ao, const uint32_t *bo, const uint32_t *avo,
                                   const uint32_t *bvo, const uint8_t *ak, const uint8_t *bk, const uint8_t *av,
                                   const uint8_t *bv, bool vl, uint32_t *ur, uint4 *pa, uint4 *pb, DiffRec *out,
                                   uint64_t base, uint64_t lim, uint64_t *stamp = nullptr) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nu_max = (uint32_t)(nA + nB);
    for (uint32_t u = lane; u < nu_max; u += 64) ur[u] = 0xffffffffu;
    for (uint32_t i = lane; i < nA; i += 64) pa[i] = lds_key_prefix(ak + ao[i], ao[i + 1] - ao[i]);
    for (uint32_t j = lane; j < nB; j += 64) pb[j] = lds_key_prefix(bk + bo[j], bo[j + 1] - bo[j]);
    wave_sync_lds();
    if (stamp && (threadIdx.x & 63) == 0) stamp[15] = __builtin_amdgcn_s_memrealtime();
    uint64_t cnt = 0;
    uint32_t mcarry = 0;
    for (uint32_t c = 0; c < nA; c += 64) {   // A side: matched-and-different or local-only
        const uint32_t i = c + lane;
        bool eq = false, emit = false;
        uint32_t rb = 0;
        if (i < nA) {
            rb = lds_lower_bound(pb, bo, bk, (uint32_t)nB, pa[i], ak + ao[i], ao[i + 1] - ao[i], &eq);
            if (eq) {
                if (vl) {
                    emit = !lds_bytes_eq(av + avo[i], avo[i + 1] - avo[i], bv + bvo[rb], bvo[rb + 1] - bvo[rb]);
                } else {
                    const uint64_t x = a0 + i, y = b0 + rb;
                    emit = !bytes_eq(A.vheap + A.voff[x], A.voff[x + 1] - A.voff[x], B.vheap + B.voff[y],
                                     B.voff[y + 1] - B.voff[y]);
                }
            } else {
                emit = filter != 1;
            }
        }
        const uint32_t m = mcarry + wave_prefix_count(eq, lane);
        mcarry += (uint32_t)__popcll(__ballot(eq));
        cnt += (uint32_t)__popcll(__ballot(emit));
        if (emit) ur[i + rb - m] = (eq ? 0u : (1u << 30)) | (i << 15) | rb;
    }
    mcarry = 0;
    for (uint32_t c = 0; c < nB; c += 64) {   // B side: remote-only
        const uint32_t j = c + lane;
        bool eq = false, emit = false;
        uint32_t ra = 0;
        if (j < nB) {
            ra = lds_lower_bound(pa, ao, ak, (uint32_t)nA, pb[j], bk + bo[j], bo[j + 1] - bo[j], &eq);
            emit = !eq && filter != 2;
        }
        const uint32_t m = mcarry + wave_prefix_count(eq, lane);
        mcarry += (uint32_t)__popcll(__ballot(eq));
        cnt += (uint32_t)__popcll(__ballot(emit));
        if (emit) ur[j + ra - m] = (2u << 30) | (ra << 15) | j;
    }
    wave_sync_lds();
    uint64_t pos = base;
    for (uint32_t c = 0; c < nu_max && cnt; c += 64) {   // union slots in key order -> records
        const uint32_t u = c + lane;
        const uint32_t r = u < nu_max ? ur[u] : 0xffffffffu;
        const bool e = r != 0xffffffffu;
        const uint64_t p = pos + wave_prefix_count(e, lane);
        if (e && p < lim) {
            DiffRec d;
            const uint32_t kind = r >> 30, x = (r >> 15) & 0x7fffu, y = r & 0x7fffu;
            d.kind = kind;
            d.pad = 0;
            d.seg = s;
            d.a = kind == 2 ? ~0ull : a0 + x;
            d.b = kind == 1 ? ~0ull : b0 + y;
            out[p] = d;
        }
        pos += (uint32_t)__popcll(__ballot(e));
    }
    wave_sync_lds();
    return cnt;
}

// exchange_final for one segment pair (orddict_delta + filter), one wave:
// writes the pair's records in ascending key order to out[base..] (records
// at or past lim are counted, not written: the host grows the buffer and
// runs the compare again) and returns their count.  Record kinds: 0 = {K,{A,B}}, 1 = {K,{A,'$none'}},
// 2 = {K,{'$none',B}}.
// The CSR bounds of one segment pair (entry and value-byte ranges, both sides).
struct SegPair {
    uint64_t a0, a1, b0, b1, va0, va1, vb0, vb1;
};
__device__ __forceinline__ SegPair seg_pair(const DevTree &A, const DevTree &B, uint64_t s) {
    SegPair p;
    p.a0 = A.seg_off[s]; p.a1 = A.seg_end[s]; p.b0 = B.seg_off[s]; p.b1 = B.seg_end[s];
    p.va0 = A.seg_voff[s]; p.va1 = A.seg_vend[s]; p.vb0 = B.seg_voff[s]; p.vb1 = B.seg_vend[s];
    return p;
}
__device__ __forceinline__ SegPair shfl_pair(const SegPair &p, int j) {
    SegPair q;
    q.a0 = __shfl(p.a0, j, 64); q.a1 = __shfl(p.a1, j, 64); q.b0 = __shfl(p.b0, j, 64); q.b1 = __shfl(p.b1, j, 64);
    q.va0 = __shfl(p.va0, j, 64); q.va1 = __shfl(p.va1, j, 64); q.vb0 = __shfl(p.vb0, j, 64); q.vb1 = __shfl(p.vb1, j, 64);
    return q;
}

#define MS_STAMP(st, k) do { if ((st) && (threadIdx.x & 63) == 0) (st)[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
__device__ uint64_t seg_merge_wave(const DevTree &A, const DevTree &B, uint64_t s, const SegPair &P, int filter,
                                   uint8_t *lds, DiffRec *out, uint64_t base, uint64_t lim, uint64_t *algo_bytes,
                                   uint64_t *stamp = nullptr) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t a0 = P.a0, a1 = P.a1, b0 = P.b0, b1 = P.b1;
    const uint64_t va0 = P.va0, va1 = P.va1, vb0 = P.vb0, vb1 = P.vb1;
    const uint64_t nA = a1 - a0, nB = b1 - b0;
    // algorithmic bytes of this segment pair (bench roofline): per side the
    // offsets, key records, values and the parent's entry (key bytes added below)
    *algo_bytes = 2 * (16 + 16 + 18) + 16 * (nA + nB + 2) + (va1 - va0) + (vb1 - vb0);
    if (nA <= CMP_CAP && nB <= CMP_CAP) {
        uint32_t *ao = reinterpret_cast<uint32_t *>(lds);    // key offsets (low 32 bits, relative after the copy)
        uint32_t *bo = ao + CMP_CAP + 1;
        uint32_t *avo = bo + CMP_CAP + 1;                     // value offsets
        uint32_t *bvo = avo + CMP_CAP + 1;
        uint32_t *ur = bvo + CMP_CAP + 1;
        uint8_t *ak = reinterpret_cast<uint8_t *>(ur + 2 * CMP_CAP);
        uint8_t *bk = ak + CMP_KB;
        uint8_t *av = bk + CMP_KB;
        uint8_t *bv = av + CMP_VB;
        uint4 *pa = reinterpret_cast<uint4 *>(bv + CMP_VB);  // key order prefixes (16-B aligned)
        uint4 *pb = pa + CMP_CAP;
        // one round trip: the four offset runs (+ both key bases, broadcast)
        const uint64_t ka0 = A.koff[a0], kb0 = B.koff[b0];
        for (uint64_t i = lane; i <= nA; i += 64) { ao[i] = (uint32_t)A.koff[a0 + i]; avo[i] = (uint32_t)(A.voff[a0 + i] - va0); }
        for (uint64_t i = lane; i <= nB; i += 64) { bo[i] = (uint32_t)B.koff[b0 + i]; bvo[i] = (uint32_t)(B.voff[b0 + i] - vb0); }
        wave_sync_lds();
        MS_STAMP(stamp, 12);
        const uint32_t bytesA = ao[nA] - (uint32_t)ka0, bytesB = bo[nB] - (uint32_t)kb0;
        *algo_bytes += (uint64_t)bytesA + bytesB;
        const uint64_t vA = va1 - va0, vB = vb1 - vb0;
        const bool vl = vA <= CMP_VB && vB <= CMP_VB;   // values staged too
        if (bytesA <= CMP_KB && bytesB <= CMP_KB) {
            for (uint64_t i = lane; i <= nA; i += 64) ao[i] -= (uint32_t)ka0;
            for (uint64_t i = lane; i <= nB; i += 64) bo[i] -= (uint32_t)kb0;
            // one round trip: key bytes and value bytes of both sides
            wave_copy4(A.kheap + ka0, bytesA, ak, B.kheap + kb0, bytesB, bk, A.vheap + va0, vl ? (uint32_t)vA : 0u, av,
                       B.vheap + vb0, vl ? (uint32_t)vB : 0u, bv);
            MS_STAMP(stamp, 13);
            const uint64_t cnt = lds_merge_pair(A, B, s, filter, a0, b0, (uint32_t)nA, (uint32_t)nB, ao, bo, avo, bvo, ak, bk,
                                                av, bv, vl, ur, pa, pb, out, base, lim, stamp);
            MS_STAMP(stamp, 14);
            return cnt;
        }
        *algo_bytes -= (uint64_t)bytesA + bytesB;   // counted again below
        wave_sync_lds();
    }
    *algo_bytes += (A.koff[a1] - A.koff[a0]) + (B.koff[b1] - B.koff[b0]);
    // oversized segments: lane 0 walks the two key lists
    uint64_t c = 0;
    if (lane == 0) {
        uint64_t x = a0, y = b0;
        while (x < a1 || y < b1) {
            int cmp;
            if (x < a1 && y < b1)
                cmp = rec_cmp(A.kheap + A.koff[x], A.koff[x + 1] - A.koff[x], B.kheap + B.koff[y], B.koff[y + 1] - B.koff[y]);
            else
                cmp = x < a1 ? -1 : 1;
            DiffRec r;
            r.seg = s;
            r.pad = 0;
            bool emit;
            if (cmp < 0) {
                r.a = x; r.b = ~0ull; r.kind = 1;
                emit = filter != 1;
                x++;
            } else if (cmp > 0) {
                r.a = ~0ull; r.b = y; r.kind = 2;
                emit = filter != 2;
                y++;
            } else {
                emit = !bytes_eq(A.vheap + A.voff[x], A.voff[x + 1] - A.voff[x], B.vheap + B.voff[y],
                                 B.voff[y + 1] - B.voff[y]);
                r.a = x; r.b = y; r.kind = 0;
                x++; y++;
            }
            if (emit) {
                if (base + c < lim) out[base + c] = r;
                c++;
            }
        }
    }
    return __shfl(c, 0, 64);
}

// LDS of a compare-walk wave: the shared area (lane regions for inner-node
// staging / the merge-join), then the work list, then per-level counters
#define CMP_LIST 256
__host__ __device__ __forceinline__ uint32_t cmp_shared_bytes(uint32_t W) {
    const uint32_t a = 64 * lane_region_bytes(W), m = cmp_merge_lds_bytes();
    return ((a > m ? a : m) + 15) & ~15u;
}
__host__ __device__ __forceinline__ uint32_t cmp_slice_bytes(uint32_t W) {
    return (cmp_shared_bytes(W) + CMP_LIST * 8 + ST_MAXLEV * 8 + 15) & ~15u;   // 16-B aligned wave slices
}

// Does the level-k entry `anc` differ between the trees under the filter (and,
// at level 2, lie in the partition's bucket range [lo2, hi2))?
__device__ __forceinline__ bool cmp_entry_in(const DevTree &A, const DevTree &B, int filter, uint32_t k, uint64_t anc,
                                             uint64_t lo2, uint64_t hi2) {
    const uint64_t slot = A.base[k] + anc;
    if (k == 2 && (anc < lo2 || anc >= hi2)) return false;
    return entry_differs(A.tag[slot], B.tag[slot], A.md5[slot], B.md5[slot], filter);
}

// Is inner node (L, b) visited, given that the top hashes differ?  Every
// ancestor entry at levels L..2 differs (deepest first: the most selective).
__device__ __forceinline__ bool cmp_visited(const DevTree &A, const DevTree &B, int filter, uint32_t L, uint64_t b,
                                            uint64_t lo2, uint64_t hi2) {
    for (uint32_t k = L; k >= 2; k--)
        if (!cmp_entry_in(A, B, filter, k, b >> (A.shift * (L - k)), lo2, hi2)) return false;
    return true;
}

// The whole compare walk in one launch, a fixed grid of nw waves.  Wave w
// owns the level-H nodes [w*P, (w+1)*P) (P = ceil(nodes(H) / nw)), the
// segments under them and every inner node whose first level-H descendant
// it owns.  Per 64 of its level-H nodes (highest first) it
//  * evaluates the frontier top-down over the levels 2..H covering them (a
//    lane per node, the parent's flag by a shuffle: one memory round trip per
//    level) and lists its visited inner nodes;
//  * checks the children of the visited level-H nodes (a lane per child,
//    64 / W nodes per round trip) and lists the visited segments, highest
//    first;
//  * flushes the list: every listed node / segment is verified on both sides
//    at once (a lane per item and side: the MD5 chains run side by side), then
//    the segment pairs are merge-joined in list order into the wave's own
//    scratch region [w*R, (w+1)*R).  AccFun = Keys ++ Acc over ascending
//    segments (synctree.erl:373-375) => the wave's records are already in
//    reference order, and the regions concatenate from the highest wave down.
// Per-wave outputs: wcnt[w] records, wst[w*ST_STATW + l] visited nodes per
// level, wbytes[w] algorithmic bytes of its segment pairs; *need = max
// records of a wave that overflowed R.  No same-address atomics on the
// success path.
#define ST_STATW (ST_MAXLEV + 2)
#define CMP_SPEC 5   // frontier levels loaded up front (2..6: H <= 6)

struct CmpWalk {
    uint8_t *shared;       // lane regions / merge area
    uint64_t *list;        // (level << 56) | index
    uint32_t *cnt;         // visited per level
    DiffRec *scratch;
    uint64_t rb, lim, pos, bytes;
    int filter;
    uint64_t errmin;       // this lane's first failed verification (err_code), ~0 if none
    uint64_t *stamp;       // diagnostic: this wave's 8 phase stamps, or null
};
#define CW_STAMP(c, k) do { if ((c).stamp && (threadIdx.x & 63) == 0) (c).stamp[k] = __builtin_amdgcn_s_memrealtime(); } while (0)


// Verify the listed items on both sides, then merge-join the listed segments.
// Verification: a lane per (item, side); each message -- an inner node's
// child entries (stage_inner) or a segment's value run (copied by the whole
// wave, coalesced) -- is staged in the shared LDS area first, so every lane
// runs the same md5_lds chain; runs that do not fit are hashed from global
// memory.

__device__ __forceinline__ void cmp_flush(const DevTree &A, const DevTree &B, CmpWalk &c, uint32_t n) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t L1 = A.H + 1;
    const uint32_t SH0 = cmp_shared_bytes(A.W);
    CW_STAMP(c, 8);
    // the first 32 items' segment bounds (lane 2i: item i's local side, 2i + 1
    // its remote side), kept for the merge-joins (no second round trip)
    uint64_t kv0 = 0, kvl = 0, ks0 = 0, ks1 = 0;
    for (uint32_t k0 = 0; k0 < 2 * n; k0 += 64) {
        const uint32_t k = k0 + lane;
        const bool act = k < 2 * n;
        const uint64_t it = act ? c.list[k >> 1] : 0;
        const uint32_t l = (uint32_t)(it >> 56), side = k & 1;
        const uint64_t b = it & ((1ull << 56) - 1);
        const bool inner = act && l < L1, seg = act && l == L1;
        const uint32_t isz = inner ? lane_region_bytes(A.W) : 0;
        const uint32_t ioff = wave_excl_scan(isz);
        const uint32_t itot = __shfl(ioff + isz, 63, 64);
        uint16_t et = 0;
        uint4 e = make_uint4(0, 0, 0, 0);
        uint64_t v0 = 0, len = 0;
        bool empty = false;
        if (act) {
            const uint64_t eslot = (l == 1) ? 0 : A.base[l] + b;
            if (side) { et = B.tag[eslot]; e = B.md5[eslot]; } else { et = A.tag[eslot]; e = A.md5[eslot]; }
        }
        if (seg) {
            uint64_t s0, s1;
            if (side) { v0 = B.seg_voff[b]; len = B.seg_vend[b] - v0; s0 = B.seg_off[b]; s1 = B.seg_end[b]; }
            else      { v0 = A.seg_voff[b]; len = A.seg_vend[b] - v0; s0 = A.seg_off[b]; s1 = A.seg_end[b]; }
            empty = s0 == s1;
            if (k0 == 0) { kv0 = v0; kvl = len; ks0 = s0; ks1 = s1; }
        }
        // inner nodes: the child entries, loaded while the loads above are in flight
        uint32_t mlen = 0;
        if (inner) mlen = side ? stage_inner(B, l, b, c.shared + ioff) : stage_inner(A, l, b, c.shared + ioff);
        CW_STAMP(c, 9);
        const uint32_t SH = SH0;
        const uint32_t ssz = seg ? (uint32_t)(len + 64 + 15 < SH ? ((len + 64 + 15) & ~15ull) : SH + 16) : 0;
        const uint32_t soff = itot + wave_excl_scan(ssz);
        const bool sfit = seg && (et & TAG_PRESENT) && soff + ssz <= SH;
        // the fitting value runs, four per round trip
        for (uint64_t m = __ballot(sfit); m;) {
            const uint8_t *sp[4] = {nullptr, nullptr, nullptr, nullptr};
            uint8_t *dp[4] = {c.shared, c.shared, c.shared, c.shared};
            uint32_t ln[4] = {0, 0, 0, 0};
#pragma unroll
            for (int r = 0; r < 4; r++) {
                if (!m) break;
                const int j = __ffsll((long long)m) - 1;
                m &= m - 1;
                sp[r] = (__shfl((int)side, j, 64) ? B.vheap : A.vheap) + __shfl(v0, j, 64);
                ln[r] = (uint32_t)__shfl(len, j, 64);
                dp[r] = c.shared + __shfl(soff, j, 64);
            }
            wave_copy4(sp[0], ln[0], dp[0], sp[1], ln[1], dp[1], sp[2], ln[2], dp[2], sp[3], ln[3], dp[3]);
        }
        CW_STAMP(c, 10);
        wave_sync_lds();
        CW_STAMP(c, 7);
        if (act) {
            bool ok;
            if (!(et & TAG_PRESENT)) {
                ok = inner ? (mlen == 0) : empty;
            } else {
                uint32_t d[4];
                if (inner || sfit)   // one inlined chain for every staged message (branches would run one after another)
                    stmd5::md5_lds(c.shared + (inner ? ioff : soff), inner ? mlen : (uint32_t)len, d);
                else
                    stmd5::md5_global_pf((side ? B.vheap : A.vheap) + v0, len, d);
                ok = et == TAG_PRESENT && e.x == d[0] && e.y == d[1] && e.z == d[2] && e.w == d[3];
            }
            if (!ok) {
                const uint64_t ec = err_code(l, b, side);
                if (ec < c.errmin) c.errmin = ec;
            }
        }
        wave_sync_lds();
    }
    CW_STAMP(c, 3);
    // the listed segments' CSR bounds, 64 per round trip (lane i: the i-th
    // item), handed to each merge-join by shuffles in list order
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
        const uint32_t i = i0 + lane;
        const uint64_t it = i < n ? c.list[i] : 0;
        const bool sg = i < n && (uint32_t)(it >> 56) == L1;
        const uint64_t sj = it & ((1ull << 56) - 1);
        SegPair p = {0, 0, 0, 0, 0, 0, 0, 0};
        if (i0 == 0 && n <= 32) {   // every item's bounds are in the phase-1 registers
            const int la = (int)(2 * (lane & 31)), lb = la + 1;
            p.a0 = __shfl(ks0, la, 64); p.a1 = __shfl(ks1, la, 64);
            p.va0 = __shfl(kv0, la, 64); p.va1 = p.va0 + __shfl(kvl, la, 64);
            p.b0 = __shfl(ks0, lb, 64); p.b1 = __shfl(ks1, lb, 64);
            p.vb0 = __shfl(kv0, lb, 64); p.vb1 = p.vb0 + __shfl(kvl, lb, 64);
        } else if (sg) {
            p = seg_pair(A, B, sj);
        }
        for (uint64_t m = __ballot(sg); m; m &= m - 1) {
            const int j = __ffsll((long long)m) - 1;
            uint64_t by;
            c.pos += seg_merge_wave(A, B, __shfl(sj, j, 64), shfl_pair(p, j), c.filter, c.shared, c.scratch, c.rb + c.pos,
                                    c.lim, &by, c.stamp);
            c.bytes += by;
            wave_sync_lds();
        }
    }
    CW_STAMP(c, 4);
}

// append the ballot's lanes (item value per lane) to the list
__device__ __forceinline__ void cmp_append(uint64_t *list, uint32_t &n, bool f, uint64_t item) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t m = __ballot(f);
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    if (f) list[n + __popcll(m & below)] = item;
    n += (uint32_t)__popcll(m);
}

#define ST_DERR_CMP 2u   // TreeTiles::err / tree error bit: a compare wave's count never arrived
__global__ void __launch_bounds__(256) k_cmp_walk(DevTree A, DevTree B, int filter, uint64_t lo2, uint64_t hi2, uint32_t nw,
                                                 uint32_t slice, DiffRec *scratch, uint64_t R, uint64_t *look,
                                                 uint32_t *wst, uint64_t *wbytes, uint64_t *rare, uint32_t ep, DiffRec *out,
                                                 uint64_t cap, uint64_t *res, uint32_t *derr, uint64_t *stamps) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t gw = blockIdx.x * (blockDim.x >> 6) + wave;
    if (gw >= nw) return;
    const uint32_t w = nw - 1 - gw;   // the top of the grid first: a wave waits only for waves dispatched before it
    uint8_t *wl = lds + (uint64_t)wave * slice;
    const uint32_t H = A.H, L1 = H + 1, sh = A.shift, W = A.W;
    CmpWalk c;
    c.stamp = stamps ? stamps + (uint64_t)w * 16 : nullptr;
    CW_STAMP(c, 0);
    c.shared = wl;
    c.list = reinterpret_cast<uint64_t *>(wl + cmp_shared_bytes(W));
    c.cnt = reinterpret_cast<uint32_t *>(c.list + CMP_LIST);
    c.scratch = scratch;
    c.rb = (uint64_t)w * R;
    c.lim = c.rb + R;
    c.pos = 0;
    c.bytes = 0;
    c.filter = filter;
    c.errmin = ~0ull;
    for (uint32_t l = lane; l < ST_STATW; l += 64) c.cnt[l] = 0;
    const uint64_t nH = A.base[L1] - A.base[H];   // level-H nodes
    const uint64_t P = (nH + nw - 1) / nw;
    const uint64_t h0 = (uint64_t)w * P < nH ? (uint64_t)w * P : nH;
    const uint64_t h1 = h0 + P < nH ? h0 + P : nH;
    // H <= CMP_SPEC + 1: the entries of every level 2..H under a chunk of 64
    // level-H nodes are loaded up front (a lane per node, index clamped), so
    // the frontier costs one memory round trip instead of one per level; only
    // the flags chain through the levels.  The first chunk's loads go out with
    // the top entries' (one round trip for both).
    const bool spec = H <= CMP_SPEC + 1;
    uint16_t sta[CMP_SPEC], stb[CMP_SPEC];
    uint4 sxa[CMP_SPEC], sxb[CMP_SPEC];
    auto spec_load = [&](uint64_t c0, uint64_t c1) {
#pragma unroll
        for (uint32_t i = 0; i < CMP_SPEC; i++) {
            if (2 + i > H) break;
            const uint32_t up = sh * (H - 2 - i);
            const uint64_t lo = c0 >> up, hi = (c1 - 1) >> up;
            const uint64_t slot = A.base[2 + i] + (lo + lane <= hi ? lo + lane : hi);
            sta[i] = A.tag[slot]; stb[i] = B.tag[slot]; sxa[i] = A.md5[slot]; sxb[i] = B.md5[slot];
        }
    };
    auto spec_mask = [&](uint64_t c0) {
        uint32_t dm = 0;
#pragma unroll
        for (uint32_t i = 0; i < CMP_SPEC; i++) {
            if (2 + i > H) break;
            const uint64_t b = (c0 >> (sh * (H - 2 - i))) + lane;
            const bool d = entry_differs(sta[i], stb[i], sxa[i], sxb[i], filter) && (i != 0 || (b >= lo2 && b < hi2));
            dm |= (uint32_t)d << (2 + i);
        }
        return dm;
    };
    const uint64_t cfirst = h1 > h0 ? h0 + ((h1 - h0 - 1) & ~63ull) : 0;
    if (spec && h1 > h0) spec_load(cfirst, cfirst + 64 < h1 ? cfirst + 64 : h1);
    bool topdiff;
    {
        const uint16_t ta = A.tag[0], tb = B.tag[0];
        const uint4 x = A.md5[0], y = B.md5[0];
        topdiff = ta != tb || ((ta & TAG_PRESENT) && (x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w));
    }
    uint32_t n = 0;
    wave_sync_lds();
    if (topdiff && H == 0) {   // one segment under the top hash (segments = 1): wave 0
        if (w == 0) {
            cmp_append(c.list, n, lane == 0, (1ull << 56));
            if (lane == 0) c.cnt[1] += 1;
            cmp_flush(A, B, c, n);
            n = 0;
        }
    } else if (topdiff && h1 > h0) {
        if (h0 == 0) {   // the root (level 1) belongs to wave 0
            cmp_append(c.list, n, lane == 0, (1ull << 56));
            if (lane == 0) c.cnt[1] += 1;
        }
        for (uint64_t c0 = cfirst;; c0 -= 64) {
            const uint64_t c1 = c0 + 64 < h1 ? c0 + 64 : h1;   // level-H nodes [c0, c1)
            uint32_t dmask = 0;
            if (spec) {
                if (c0 != cfirst) spec_load(c0, c1);
                dmask = spec_mask(c0);
            }
            bool f = true;       // this lane's node flag at the previous level (level 1: the root)
            for (uint32_t l = 2; l <= H; l++) {
                const uint32_t up = sh * (H - l);
                const uint64_t lo = c0 >> up, hi = (c1 - 1) >> up;
                const uint64_t b = lo + lane;
                const uint64_t plo = lo >> sh;
                const uint32_t plane = (uint32_t)((b >> sh) - plo);
                const bool fp = __shfl((int)f, (int)(plane < 64 ? plane : 0), 64) != 0;
                f = b <= hi && fp && (spec ? ((dmask >> l) & 1u) != 0 : cmp_entry_in(A, B, filter, l, b, lo2, hi2));
                const bool owned = f && (b << up) >= c0 && (b << up) < c1;
                if (n + 64 > CMP_LIST) { cmp_flush(A, B, c, n); n = 0; }
                const uint32_t n0 = n;
                cmp_append(c.list, n, owned, ((uint64_t)l << 56) | b);
                if (lane == 0) c.cnt[l] += n - n0;
            }
            CW_STAMP(c, 1);
            // f: flags of the level-H nodes c0 + lane
            uint64_t vm = __ballot(f && c0 + lane < c1);
            const uint32_t G = 64 / W;   // level-H nodes per children round trip
            while (vm) {
                // the next G visited nodes, highest first: lane -> (node, child)
                const uint32_t g = lane / W, ch = lane % W;
                uint64_t x = vm;
                uint32_t j = 64;
                for (uint32_t q = 0; q <= g && x; q++) {
                    j = 63 - __clzll(x);
                    x &= ~(1ull << j);
                    if (q != g) j = 64;
                }
                uint32_t taken = 0;
                for (uint32_t q = 0; q < G && vm; q++) { vm &= ~(1ull << (63 - __clzll(vm))); taken++; }
                const bool have = g < taken && j < 64;
                const uint64_t s = ((c0 + j) << sh) + (W - 1 - ch);   // children highest first
                const bool in = have && cmp_entry_in(A, B, filter, L1, s, lo2, hi2);
                if (n + 64 > CMP_LIST) { cmp_flush(A, B, c, n); n = 0; }
                const uint32_t n0 = n;
                cmp_append(c.list, n, in, ((uint64_t)L1 << 56) | s);
                if (lane == 0) c.cnt[L1] += n - n0;
            }
            if (c0 == h0) break;
        }
        CW_STAMP(c, 2);
        if (n) cmp_flush(A, B, c, n);
    }
    wave_sync_lds();
    CW_STAMP(c, 5);
    if (c.stamp && lane == 0) c.stamp[6] = c.cnt[L1];
    uint64_t em = c.errmin;
    for (int o = 32; o; o >>= 1) {
        const uint64_t y = __shfl_xor(em, o, 64);
        em = y < em ? y : em;
    }
    if (lane == 0) wbytes[w] = c.bytes;
    for (uint32_t l = lane; l < ST_STATW; l += 64) wst[(uint64_t)w * ST_STATW + l] = (l >= 1 && l <= L1) ? c.cnt[l] : 0;

    // The wave's records go after those of every higher wave (AccFun = Keys
    // ++ Acc, highest segments first): each wave publishes its record count
    // in an epoch-stamped word (one atomic store: no ordering argument between
    // words) and sums the counts of the waves above it.  Waves are numbered
    // from the top of the grid down (w = nw-1 is dispatched first), so a wave
    // only waits for waves dispatched before it.  The rare cases -- records
    // past a wave's scratch region, a failed verification -- go to two words
    // by atomic max / min before the count is published (epoch in the high
    // bits, so a stale word never wins).  Wave 0 holds the total and reports
    // it to the host-mapped result block.
    const uint64_t cnt = c.pos;
    const uint64_t EP = (uint64_t)ep << 48;
    if (lane == 0) {
        if (cnt > R) (void)__hip_atomic_fetch_max(&rare[1], EP | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (em != ~0ull) {   // (level << 40) | (bucket << 1) | side: the same order as err_code
            const uint64_t pk = ((em >> 56) << 40) | (em & ((1ull << 40) - 1));
            (void)__hip_atomic_fetch_min(&rare[0], ((uint64_t)(0xFFFFu - ep) << 48) | pk, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
        }
        __hip_atomic_store(&look[w], EP | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    uint64_t above = 0;
    bool lost = false;
    {
        const uint32_t K = (nw - 1 - w + 63) / 64;   // <= 64 words per lane (nw <= 4096)
        for (uint32_t k0 = 0; k0 < K; k0 += 16) {
            uint32_t pend = 0;
            for (uint32_t k = 0; k < 16 && k0 + k < K; k++)
                if (w + 1 + (k0 + k) * 64 + lane < nw) pend |= 1u << k;
            for (uint32_t it = 0; __ballot(pend != 0) && it < (1u << 18); it++) {
                for (uint32_t m = pend; m; m &= m - 1) {
                    const uint32_t k = (uint32_t)__builtin_ctz(m);
                    const uint64_t x = __hip_atomic_load(&look[w + 1 + (k0 + k) * 64 + lane], __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
                    if ((x >> 48) == ep) { above += x & ((1ull << 48) - 1); pend &= ~(1u << k); }
                }
                if (__ballot(pend != 0)) __builtin_amdgcn_s_sleep(1);
            }
            lost |= pend != 0;
        }
        for (int o = 32; o; o >>= 1) above += __shfl_xor(above, o, 64);
        lost = __ballot(lost) != 0;
    }
    if (lost) {   // a count never arrived (bounded wait): an error, not a result
        if (derr) __hip_atomic_store(derr, ST_DERR_CMP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    // this wave's records (those its scratch region holds) to their place
    const uint64_t own = cnt < R ? cnt : R;
    for (uint64_t i = lane; i < own; i += 64)
        if (above + i < cap) out[above + i] = scratch[c.rb + i];
    CW_STAMP(c, 11);
    if (w == 0 && lane == 0) {
        const uint64_t nd = __hip_atomic_load(&rare[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t er = __hip_atomic_load(&rare[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        res[0] = above + cnt;
        res[1] = (nd >> 48) == ep ? nd & ((1ull << 48) - 1) : 0;
        res[2] = (er >> 48) == 0xFFFFu - ep ? (((er >> 40) & 0xFFu) << 56) | (er & ((1ull << 40) - 1)) : ~0ull;
        __threadfence_system();
        __hip_atomic_store(reinterpret_cast<uint32_t *>(&res[3]), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}


// Diff records -> byte lengths of key / local value / remote value
__global__ void k_diff_lengths(DevTree A, DevTree B, const DiffRec *r, uint64_t n, uint64_t *kl, uint64_t *al,
                               uint64_t *bl) {
    for (uint64_t i = gtid(); i <= n; i += gstride()) {
        if (i == n) { kl[i] = al[i] = bl[i] = 0; break; }
        const DiffRec d = r[i];
        if (d.a != ~0ull) {
            kl[i] = A.koff[d.a + 1] - A.koff[d.a];
            al[i] = A.voff[d.a + 1] - A.voff[d.a];
        } else {
            kl[i] = B.koff[d.b + 1] - B.koff[d.b];
            al[i] = 0;
        }
        bl[i] = d.b != ~0ull ? B.voff[d.b + 1] - B.voff[d.b] : 0;
    }
}

__global__ void k_diff_gather(DevTree A, DevTree B, const DiffRec *r, uint64_t n, const uint64_t *koff,
                              uint8_t *kheap, const uint64_t *aoff, uint8_t *aheap, const uint64_t *boff,
                              uint8_t *bheap, uint8_t *kind, uint64_t *seg) {
    for (uint64_t i = gtid(); i < n; i += gstride()) {
        const DiffRec d = r[i];
        if (d.a != ~0ull) {
            copy_bytes(kheap + koff[i], A.kheap + A.koff[d.a], A.koff[d.a + 1] - A.koff[d.a]);
            copy_bytes(aheap + aoff[i], A.vheap + A.voff[d.a], A.voff[d.a + 1] - A.voff[d.a]);
        } else {
            copy_bytes(kheap + koff[i], B.kheap + B.koff[d.b], B.koff[d.b + 1] - B.koff[d.b]);
        }
        if (d.b != ~0ull) copy_bytes(bheap + boff[i], B.vheap + B.voff[d.b], B.voff[d.b + 1] - B.voff[d.b]);
        kind[i] = (uint8_t)d.kind;
        seg[i] = d.seg;
    }
}

// ---------------------------------------------------------------------------
// Diff application (riak_ensemble_exchange.erl:85-97): for every diff record
// in reference order decide whether the local tree takes the remote value:
//   {K, {'$none', B}} -> insert B;  {K, {_, '$none'}} -> nothing;
//   {K, {A, B}}       -> insert B iff valid_obj_hash(B, A), i.e. B >= A as
//                        Erlang binaries (riak_ensemble_peer.erl:1726-1729).
// valid_obj_hash has a clause only for two <<?H_OBJ_NONE, _>> hashes: any
// other pair is a function_clause crash of the exchange, which has applied
// the diffs before it (list comprehension order) and none after: first_bad
// records the smallest such index.
__device__ __forceinline__ bool erl_bin_ge(const uint8_t *x, uint64_t lx, const uint8_t *y, uint64_t ly) {
    const uint64_t m = lx < ly ? lx : ly;
    for (uint64_t i = 0; i < m; i++)
        if (x[i] != y[i]) return x[i] > y[i];
    return lx >= ly;
}

__global__ void k_diff_apply_select(DevTree A, DevTree B, const DiffRec *r, uint64_t n, uint8_t *take,
                                    unsigned long long *first_bad) {
    for (uint64_t i = gtid(); i < n; i += gstride()) {
        const DiffRec d = r[i];
        bool tk = false;
        if (d.b != ~0ull) {
            if (d.a == ~0ull) {
                tk = true;
            } else {
                const uint8_t *va = A.vheap + A.voff[d.a], *vb = B.vheap + B.voff[d.b];
                const uint64_t la = A.voff[d.a + 1] - A.voff[d.a], lb = B.voff[d.b + 1] - B.voff[d.b];
                if (la == 0 || lb == 0 || va[0] != 0 || vb[0] != 0)
                    atomicMin(first_bad, (unsigned long long)i);
                else
                    tk = erl_bin_ge(vb, lb, va, la);
            }
        }
        take[i] = tk ? 1 : 0;
    }
}

// Lengths of the records to insert (0 for skipped diffs and for every diff at
// or after the first crash), n + 1 entries with a zero terminator.
__global__ void k_diff_apply_lengths(DevTree B, const DiffRec *r, uint64_t n, const uint8_t *take,
                                     const unsigned long long *first_bad, uint64_t *one, uint64_t *kl, uint64_t *vl) {
    const unsigned long long fb = *first_bad;
    for (uint64_t i = gtid(); i <= n; i += gstride()) {
        const bool tk = i < n && i < fb && take[i];
        one[i] = tk ? 1 : 0;
        if (tk) {
            const DiffRec d = r[i];
            kl[i] = B.koff[d.b + 1] - B.koff[d.b];
            vl[i] = B.voff[d.b + 1] - B.voff[d.b];
        } else {
            kl[i] = vl[i] = 0;
        }
    }
}

// Pack the taken remote entries as an ingest batch (key records + values).
__global__ void k_diff_apply_gather(DevTree B, const DiffRec *r, uint64_t n, const uint64_t *pos, const uint64_t *ko,
                                    const uint64_t *vo, uint8_t *kheap, uint64_t *koff, uint8_t *vheap, uint64_t *voff) {
    for (uint64_t i = gtid(); i <= n; i += gstride()) {
        const uint64_t p = pos[i];
        if (i == n) { koff[p] = ko[n]; voff[p] = vo[n]; break; }
        if (pos[i + 1] == p) continue;   // not taken
        const DiffRec d = r[i];
        koff[p] = ko[i];
        voff[p] = vo[i];
        copy_bytes(kheap + ko[i], B.kheap + B.koff[d.b], B.koff[d.b + 1] - B.koff[d.b]);
        copy_bytes(vheap + vo[i], B.vheap + B.voff[d.b], B.voff[d.b + 1] - B.voff[d.b]);
    }
}

// Gather entries by index list (get results / segment images) into packed heaps.
__global__ void k_entry_lengths(DevTree t, const uint64_t *idx, uint64_t n, uint64_t *kl, uint64_t *vl) {
    for (uint64_t i = gtid(); i <= n; i += gstride()) {
        if (i == n) { kl[i] = vl[i] = 0; break; }
        const uint64_t e = idx[i];
        if (e == ~0ull) { kl[i] = vl[i] = 0; continue; }
        kl[i] = t.koff[e + 1] - t.koff[e];
        vl[i] = t.voff[e + 1] - t.voff[e];
    }
}

__global__ void k_entry_gather(DevTree t, const uint64_t *idx, uint64_t n, const uint64_t *koff, uint8_t *kheap,
                               const uint64_t *voff, uint8_t *vheap) {
    for (uint64_t i = gtid(); i < n; i += gstride()) {
        const uint64_t e = idx[i];
        if (e == ~0ull) continue;
        if (kheap) copy_bytes(kheap + koff[i], t.kheap + t.koff[e], t.koff[e + 1] - t.koff[e]);
        copy_bytes(vheap + voff[i], t.vheap + t.voff[e], t.voff[e + 1] - t.voff[e]);
    }
}

// ---------------------------------------------------------------------------
// Rehash v3 kernels.
//
// k_seg_perm_*: order segments by MD5 block count (descending; empty last),
// computed once per ingest and kept in the tree, so that the 64 lanes of every
// K1 wave run loops of equal length (K1 is VALU-bound: divergence is waste).

#define PERM_BINS 256
__device__ __forceinline__ uint32_t perm_bin(const DevTree &t, uint64_t s) {
    if (t.seg_off[s] == t.seg_end[s]) return PERM_BINS - 1;
    const uint64_t blocks = (t.seg_vend[s] - t.seg_voff[s] + 8) / 64 + 1;
    return blocks >= PERM_BINS - 1 ? 0u : (uint32_t)(PERM_BINS - 1 - blocks);
}

// Segment-range partition: empty the batch runs of segments outside
// [lo, hi) (clamp the run bounds), so ingest keeps only the owned keys.
__global__ void k_clamp_runs(uint64_t *bseg_off, uint64_t S, uint64_t lo, uint64_t hi) {
    const uint64_t a = bseg_off[lo], b = bseg_off[hi];
    for (uint64_t s = gtid(); s <= S; s += gstride()) {
        if (s == lo || s == hi) continue;
        const uint64_t x = bseg_off[s];
        bseg_off[s] = x < a ? a : (x > b ? b : x);
    }
}

// Pass 1: per-workgroup histograms reserved from global bin counters.
__global__ void __launch_bounds__(256) k_seg_perm_count(DevTree t, uint32_t *gcount) {
    __shared__ uint32_t h[PERM_BINS];
    h[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t s = gtid(); s < t.S; s += gstride()) atomicAdd(&h[perm_bin(t, s)], 1u);
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&gcount[threadIdx.x], h[threadIdx.x]);
}

// Pass 2: exclusive scan of the 256 bin counts into cursors (one workgroup).
__global__ void __launch_bounds__(256) k_seg_perm_scan(uint32_t *gcount) {
    __shared__ uint32_t h[PERM_BINS];
    h[threadIdx.x] = gcount[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int b = 0; b < PERM_BINS; b++) { const uint32_t c = h[b]; h[b] = acc; acc += c; }
    }
    __syncthreads();
    gcount[threadIdx.x] = h[threadIdx.x];
}

// Pass 3: scatter (one global atomic per workgroup and bin).
__global__ void __launch_bounds__(256) k_seg_perm_scatter(DevTree t, uint32_t *gcur, uint32_t *perm) {
    __shared__ uint32_t h[PERM_BINS], base[PERM_BINS];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t chunk = (t.S + gridDim.x - 1) / gridDim.x;
    const uint64_t a = blockIdx.x * chunk, b = (a + chunk < t.S) ? a + chunk : t.S;
    for (uint64_t s = a + threadIdx.x; s < b; s += blockDim.x) atomicAdd(&h[perm_bin(t, s)], 1u);
    __syncthreads();
    base[threadIdx.x] = h[threadIdx.x] ? atomicAdd(&gcur[threadIdx.x], h[threadIdx.x]) : 0;
    h[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t s = a + threadIdx.x; s < b; s += blockDim.x) {
        const uint32_t bin = perm_bin(t, s);
        perm[base[bin] + atomicAdd(&h[bin], 1u)] = (uint32_t)s;
    }
}

// A list in bins (k_page_place, pages.h): bin b's cnt[b * line] entries at list[b * cap ...].
struct HashBins {
    const uint32_t *list;
    const unsigned long long *cnt;
    uint64_t cap;
    uint32_t nbins, line;
};

// K1 segment_hash over the block-count order.
// ps (optional): per segment, the MD5 state of its unchanged prefix (PrefixState, k_verify_cap).
// ntot (optional): perm is a list of *ntot segments, not all S.
// hb.list (optional): the list in bins instead (perm unused; a streaming batch's changed segments).
__global__ void __launch_bounds__(256) k_segment_hash_perm(DevTree t, const uint32_t *perm, const uint8_t *mask,
                                                           const PrefixState *ps, const uint32_t *ntot = nullptr,
                                                           HashBins hb = HashBins{nullptr, nullptr, 0, 0, 0}) {
    const uint32_t L1 = t.H + 1;
    __shared__ uint32_t pre[257];
    uint64_t n = ntot ? (uint64_t)*ntot : t.S;
    if (hb.list) {   // the bins' starts in the list order
        if (threadIdx.x == 0) {
            uint32_t a = 0;
            for (uint32_t b = 0; b < hb.nbins; b++) { pre[b] = a; a += (uint32_t)hb.cnt[b * hb.line]; }
            pre[hb.nbins] = a;
        }
        __syncthreads();
        n = pre[hb.nbins];
    }
    for (uint64_t i = gtid(); i < n; i += gstride()) {
        uint64_t s;
        if (hb.list) {
            uint32_t lo = 0, hi = hb.nbins;   // the last bin with pre[b] <= i
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (pre[mid] <= i) lo = mid; else hi = mid;
            }
            s = hb.list[lo * hb.cap + (i - pre[lo])];
        } else {
            s = perm ? perm[i] : i;   // no perm: segment order (a few marked segments)
        }
        const uint64_t slot = t.base[L1] + s;
        if (mask && !mask[slot]) continue;
        if (t.seg_off[s] == t.seg_end[s]) {
            t.tag[slot] = 0;
            if (L1 == 1) t.tag[0] = 0;
            continue;
        }
        uint32_t dg[4], cap[4];
        const uint64_t v0 = t.seg_voff[s];
        uint64_t k0 = 0;
        if (ps && ps[s].k) {
            const uint4 q = ps[s].st;
            k0 = ps[s].k;
            dg[0] = q.x; dg[1] = q.y; dg[2] = q.z; dg[3] = q.w;
        } else {
            stmd5::init(dg);
        }
        stmd5::md5_global_span<ST_SPAN_TPUT>(t.vheap + v0, t.seg_vend[s] - v0, k0, dg, ~0ull, cap);
        const uint4 e = make_uint4(dg[0], dg[1], dg[2], dg[3]);
        t.md5[slot] = e;
        t.tag[slot] = TAG_PRESENT;
        if (L1 == 1) { t.md5[0] = e; t.tag[0] = TAG_PRESENT; }
    }
}

// Hash inner node (l, b) of a W == 16 tree into its parent's entry.  Nodes
// with all 16 children present hash from registers (md5_node16); others stage
// the present entries in the lane's LDS region.
__device__ __forceinline__ void hash_node16(const DevTree &t, uint32_t l, uint64_t b, uint8_t *reg) {
    const uint64_t slot = t.base[l] + b;
    const uint64_t c0 = t.base[l + 1] + b * 16;
    uint32_t tg[16];
    uint4 h[16];
#pragma unroll
    for (int j = 0; j < 16; j++) { tg[j] = t.tag[c0 + j]; h[j] = t.md5[c0 + j]; }
    uint32_t full = 1;
#pragma unroll
    for (int j = 0; j < 16; j++) full &= (tg[j] >> 8) & 1u;
    uint32_t dg[4];
    uint32_t len = 1;
    if (full) {
        uint32_t pf[16];
#pragma unroll
        for (int j = 0; j < 16; j++) pf[j] = tg[j] & 0xffu;
        stmd5::md5_node16(pf, h, dg);
    } else {
        MsgWriter mw;
        mw.init(reg);
#pragma unroll
        for (int j = 0; j < 16; j++)
            if (tg[j] & TAG_PRESENT) mw.entry(tg[j], h[j]);
        len = mw.finish();
        if (len) stmd5::md5_lds(reg, len, dg);
    }
    uint32_t ot = 0;
    uint4 e = make_uint4(0, 0, 0, 0);
    if (len) {
        e = make_uint4(dg[0], dg[1], dg[2], dg[3]);
        ot = TAG_PRESENT;
        t.md5[slot] = e;
    }
    t.tag[slot] = (uint16_t)ot;
    if (l == 1) { t.md5[0] = e; t.tag[0] = (uint16_t)ot; }
}

// One inner level (W == 16), one lane per node.
__global__ void __launch_bounds__(64) k_level16(DevTree t, uint32_t l, const uint8_t *mask) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t *reg = lds + threadIdx.x * lane_region_bytes(16);
    const uint64_t nodes = t.base[l + 1] - t.base[l];
    for (uint64_t b = gtid(); b < nodes; b += gstride()) {
        if (mask && !mask[t.base[l] + b]) continue;
        hash_node16(t, l, b, reg);
    }
}

// Levels lmax..lmin (W == 16, <= 256 nodes each) in one workgroup.
__global__ void __launch_bounds__(256) k_upper16(DevTree t, uint32_t lmin, uint32_t lmax, const uint8_t *mask) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t *reg = lds + threadIdx.x * lane_region_bytes(16);
    for (uint32_t l = lmax; l >= lmin; l--) {
        const uint64_t nodes = t.base[l + 1] - t.base[l];
        for (uint64_t b = threadIdx.x; b < nodes; b += blockDim.x) {
            if (mask && !mask[t.base[l] + b]) continue;
            hash_node16(t, l, b, reg);
        }
        __syncthreads();
        if (l == lmin) break;
    }
}

// ---------------------------------------------------------------------------
// K2 level_rehash for W == 16: levels H, H-1, H-2 of one level-(H-2) subtree
// per workgroup (256 threads), all in LDS.
//
// The subtree's 4096 child entries (level H+1) are contiguous in the slot
// arrays: they are staged with coalesced 16-byte loads into per-node blocks
// of 16 x 16 B (+16 B pad: conflict-free ds_read_b128 by node).  Each level
// is then one lane per node: full nodes hash from registers (md5_node16),
// others write their message over their own (already consumed) child block
// and hash it from LDS.  Results go to global memory and to the next level's
// LDS blocks.  With a mask (dirty-path rehash) unmarked nodes keep their
// stored entry.
#define NB16 272           // bytes per staged node block (16 x 16 B + pad)
#define TB16 48            // bytes per staged tag block (16 x u16 + pad)

__device__ __forceinline__ void node_lds16(uint8_t *blk, const uint16_t *tags, uint32_t dg[4], uint32_t &present) {
    const uint4 *hb = reinterpret_cast<const uint4 *>(blk);
    uint4 h[16];
    uint32_t tg[16];
#pragma unroll
    for (int j = 0; j < 16; j++) { h[j] = hb[j]; tg[j] = tags[j]; }
    uint32_t full = 1, any = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) { full &= (tg[j] >> 8) & 1u; any |= (tg[j] >> 8) & 1u; }
    present = any;
    if (!any) return;
    if (full) {
        uint32_t pf[16];
#pragma unroll
        for (int j = 0; j < 16; j++) pf[j] = tg[j] & 0xffu;
        stmd5::md5_node16(pf, h, dg);
    } else {
        MsgWriter mw;
        mw.init(blk);             // own block: its entries are in registers now
#pragma unroll
        for (int j = 0; j < 16; j++)
            if (tg[j] & TAG_PRESENT) mw.entry(tg[j], h[j]);
        stmd5::md5_lds(blk, mw.finish(), dg);
    }
}

__global__ void __launch_bounds__(256) k_levels3_16(DevTree t, const uint8_t *mask) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t *A = lds;                                        // 256 node blocks (level H children)
    uint16_t *At = reinterpret_cast<uint16_t *>(A + 256 * NB16);
    uint8_t *Bb = A + 256 * NB16 + 256 * TB16;               // 16 node blocks (level H-1 children)
    uint16_t *Bt = reinterpret_cast<uint16_t *>(Bb + 16 * NB16);
    uint8_t *Cb = Bb + 16 * NB16 + 16 * TB16;                // 1 node block (level H-2 children)
    uint16_t *Ct = reinterpret_cast<uint16_t *>(Cb + NB16);
    const uint32_t tid = threadIdx.x;
    const uint32_t H = t.H;
    const uint64_t root = blockIdx.x;                        // bucket at level H-2
    if (mask && !mask[t.base[H - 2] + root]) return;
    // ---- stage the 4096 level-(H+1) entries
    const uint64_t c0 = t.base[H + 1] + root * 4096;
#pragma unroll 4
    for (uint32_t it = 0; it < 16; it++) {
        const uint32_t e = it * 256 + tid;
        *reinterpret_cast<uint4 *>(A + (e >> 4) * NB16 + (e & 15) * 16) = t.md5[c0 + e];
    }
    {
        const uint4 *tg = reinterpret_cast<const uint4 *>(t.tag + c0);   // 8 tags per 16 B
        for (uint32_t it = 0; it < 2; it++) {
            const uint32_t q = it * 256 + tid;                             // 512 chunks
            *reinterpret_cast<uint4 *>(reinterpret_cast<uint8_t *>(At) + (q >> 1) * TB16 + (q & 1) * 16) = tg[q];
        }
    }
    __syncthreads();
    // ---- level H: lane = node
    {
        const uint64_t b = root * 256 + tid;
        const uint64_t slot = t.base[H] + b;
        uint4 e;
        uint32_t tg;
        if (mask && !mask[slot]) {
            e = t.md5[slot];
            tg = t.tag[slot];
        } else {
            uint32_t dg[4], pr;
            node_lds16(A + tid * NB16, reinterpret_cast<const uint16_t *>(reinterpret_cast<uint8_t *>(At) + tid * TB16), dg, pr);
            e = make_uint4(dg[0], dg[1], dg[2], dg[3]);
            tg = pr ? TAG_PRESENT : 0u;
            if (pr) t.md5[slot] = e;
            t.tag[slot] = (uint16_t)tg;
        }
        *reinterpret_cast<uint4 *>(Bb + (tid >> 4) * NB16 + (tid & 15) * 16) = e;
        *reinterpret_cast<uint16_t *>(reinterpret_cast<uint8_t *>(Bt) + (tid >> 4) * TB16 + (tid & 15) * 2) = (uint16_t)tg;
    }
    __syncthreads();
    // ---- level H-1: 16 nodes
    if (tid < 16) {
        const uint64_t b = root * 16 + tid;
        const uint64_t slot = t.base[H - 1] + b;
        uint4 e;
        uint32_t tg;
        if (mask && !mask[slot]) {
            e = t.md5[slot];
            tg = t.tag[slot];
        } else {
            uint32_t dg[4], pr;
            node_lds16(Bb + tid * NB16, reinterpret_cast<const uint16_t *>(reinterpret_cast<uint8_t *>(Bt) + tid * TB16), dg, pr);
            e = make_uint4(dg[0], dg[1], dg[2], dg[3]);
            tg = pr ? TAG_PRESENT : 0u;
            if (pr) t.md5[slot] = e;
            t.tag[slot] = (uint16_t)tg;
        }
        *reinterpret_cast<uint4 *>(Cb + tid * 16) = e;
        Ct[tid] = (uint16_t)tg;
    }
    __syncthreads();
    // ---- level H-2: the root
    if (tid == 0) {
        const uint64_t slot = t.base[H - 2] + root;
        uint32_t dg[4], pr;
        node_lds16(Cb, Ct, dg, pr);
        const uint4 e = make_uint4(dg[0], dg[1], dg[2], dg[3]);
        if (pr) t.md5[slot] = e;
        t.tag[slot] = pr ? (uint16_t)TAG_PRESENT : (uint16_t)0;
        if (H - 2 == 1) { t.md5[0] = e; t.tag[0] = pr ? (uint16_t)TAG_PRESENT : (uint16_t)0; }
    }
}

__host__ __device__ __forceinline__ uint32_t levels3_16_lds_bytes() {
    return 256 * NB16 + 256 * TB16 + 16 * NB16 + 16 * TB16 + NB16 + TB16 + 128;
}

// ---------------------------------------------------------------------------
// Hash-ready tiled layout (full rehash, K1).
//
// The tree keeps, next to the CSR, every segment's hash input as its padded
// MD5 message (values in key order, 0x80, zeros, 64-bit bit length; RFC 1321
// §3.1-3.2) in a TILED layout built at ingest: segments in seg_perm order
// (descending MD5 block count) are cut into tiles of 64; tile t stores 16-byte
// chunk q of block k of its lane j at tiles[tbase[t] + (k*4 + q)*64 + j].  A
// wave hashing one tile then reads 1 KiB contiguous per load instruction, its
// 64 lanes run (nearly) equal-length MD5 loops, and no padding logic runs in
// the hot loop.  The layout is rebuilt whenever the CSR changes (every
// mutation goes through ingest), so a rehash always hashes the current
// segments.
struct TileInfo {
    uint64_t base;   // in uint4 units
    uint32_t B;      // blocks of the longest message in the tile
    uint32_t R;      // 16-byte rows stored per lane: the longest message's data rows
};

// Per-lane message descriptor of a tile (tln): 0 = no message (an empty
// segment or a padding lane), else the message length + 1.  A tile stores
// only the rows that hold message bytes of some lane (R); the rows past them
// (padding zeros, the 0x80 terminator, the bit length) are synthesized in
// registers by the hashing wave, so they cost no HBM traffic.
__host__ __device__ __forceinline__ uint32_t ln_blocks(uint32_t ln) {
    return ln ? (uint32_t)(((uint64_t)ln - 1 + 8) / 64 + 1) : 0u;
}
__host__ __device__ __forceinline__ uint32_t ln_rows(uint32_t ln) { return ln ? (uint32_t)(((uint64_t)ln - 1 + 15) / 16) : 0u; }

// Row `row` (bytes 16 row .. 16 row + 15) of a lane's padded message: loaded
// when the tile stores it, else zeros plus the terminator / bit length where
// they fall (RFC 1321 §3.1-3.2).  R is wave-uniform: the branch is scalar.
__device__ __forceinline__ uint4 tile_synth(uint32_t row, uint32_t ln) {
    const uint32_t len = ln - 1;   // ln == 0: the lane hashes nothing
    uint4 c = make_uint4(0, 0, 0, 0);
    if ((len >> 4) == row) {       // only when len == 16 R: the terminator opens this row
        const uint32_t v = 0x80u << (8 * (len & 3)), w = (len >> 2) & 3;
        c.x = w == 0 ? v : 0u; c.y = w == 1 ? v : 0u; c.z = w == 2 ? v : 0u; c.w = w == 3 ? v : 0u;
    }
    if (row == 4 * ln_blocks(ln) - 1) { c.z |= len << 3; c.w |= len >> 29; }
    return c;
}
__device__ __forceinline__ uint4 tile_row(const uint4 *tiles, uint64_t base, uint32_t lane, uint32_t row, uint32_t R,
                                          uint32_t ln) {
    if (row < R) return tiles[base + (uint64_t)row * 64 + lane];
    return tile_synth(row, ln);
}

// Per-tree pointers of a batched (multi-tree) rehash: trees of one geometry,
// e.g. the ensembles one GPU hosts.
// Mailbox of one inner-node entry that a climbing lane of another workgroup
// (possibly on another XCD, behind another L2) reads: written and read with
// agent-scope atomics, which are coherent across XCDs without a write-back of
// the writer's L2 or an invalidate of the reader's.
// A window root's entry for the tree's last window: the 16-byte MD5 and the
// tag in three 64-bit words of 48 payload bits, each stamped with the launch's
// epoch in its top 16 bits (TreeTiles::epoch, never 0; the mailboxes start
// zeroed).  Every word is one atomic store, so a reader that sees the epoch in
// all three has the whole entry, whatever order the stores become visible in.
struct MailEntry {
    unsigned long long w[3];
    uint64_t pad;
};

struct TreeTiles {
    uint4 *md5;
    uint16_t *tag;
    uint32_t *cnt;
    MailEntry *mail;
    const TileInfo *tinfo;
    const uint32_t *tseg, *tln;
    const uint4 *tiles;
    const uint64_t *pres;   // per-window segment presence bitmaps (tile build)
    const uint16_t *noff;   // per window: the 256 level-H message offsets in LDS, 4-byte units (tile build)
    uint32_t *err;          // the tree's device-error word (host-mapped): set when a mailbox wait times out
    uint32_t epoch;         // this launch's mailbox epoch for the tree (1..65535, differs from its last launch)
    uint32_t skip_root;     // fault injection (st_debug_knob ST_DBG_SKIP_MAIL): this window stores no mailbox; ~0u = none
};
#define ST_DERR_MAIL 1u     // TreeTiles::err bit: a window root's mailbox entry did not arrive


// One workgroup per tile: write the tile's stored rows (row r of lane j at
// tiles[base + r * 64 + j]) of the padded messages.
__global__ void __launch_bounds__(256) k_tile_fill(const uint64_t *__restrict__ seg_voff, const uint8_t *__restrict__ vheap,
                                                   const uint32_t *__restrict__ tseg, const uint32_t *__restrict__ tln,
                                                   const TileInfo *__restrict__ tinfo, uint4 *__restrict__ tiles) {
    const uint32_t tid = threadIdx.x, q = tid >> 6, j = tid & 63;
    const uint64_t tl = blockIdx.x;
    const TileInfo ti = tinfo[tl];
    if (ti.R == 0) return;
    const uint32_t ln = tln[tl * 64 + j];
    const uint64_t v0 = ln ? seg_voff[tseg[tl * 64 + j]] : 0;
    const uint64_t len = ln ? ln - 1 : 0;
    const uint32_t nb = ln_blocks(ln);
    for (uint32_t row = q; row < ti.R; row += 4) {
        uint4 c = make_uint4(0, 0, 0, 0);
        if ((row >> 2) < nb) {
            const uint64_t off = 16ull * row;
            if (off < len) __builtin_memcpy(&c, vheap + v0 + off, 16);
            const int64_t rem = (int64_t)len - (int64_t)off;
            c.x = stmd5::tail_word(c.x, rem >= 4 ? 4 : (int)rem);
            c.y = stmd5::tail_word(c.y, rem - 4 >= 4 ? 4 : (int)(rem - 4));
            c.z = stmd5::tail_word(c.z, rem - 8 >= 4 ? 4 : (int)(rem - 8));
            c.w = stmd5::tail_word(c.w, rem - 12 >= 4 ? 4 : (int)(rem - 12));
            if (row == 4 * nb - 1) { c.z = (uint32_t)(len << 3); c.w = (uint32_t)(len >> 29); }
        }
        tiles[ti.base + (uint64_t)row * 64 + j] = c;
    }
}

__global__ void k_tile_info(const uint64_t *tbase, uint64_t ntiles, TileInfo *info) {
    for (uint64_t i = gtid(); i < ntiles; i += gstride()) info[i].base = tbase[i];
}

// Tile shape from its 64 lanes' descriptors (one wave per tile): B = the
// most blocks, R = the most data rows; tsize = the stored uint4s (scanned
// into the tile bases).
__device__ __forceinline__ void tile_shape(uint32_t ln, uint64_t tl, bool lead, TileInfo *tinfo, uint64_t *tsize) {
    uint32_t b = ln_blocks(ln), r = ln_rows(ln);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t yb = __shfl_xor(b, o, 64), yr = __shfl_xor(r, o, 64);
        b = yb > b ? yb : b;
        r = yr > r ? yr : r;
    }
    if (lead) {
        tinfo[tl].B = b;
        tinfo[tl].R = r;
        tsize[tl] = (uint64_t)r * 64;
    }
}

// ---------------------------------------------------------------------------
// K1 over tiles in the GLOBAL block-count order (seg_perm): tile tl holds the
// segments at positions [64 tl, 64 tl + 64) of seg_perm, so a wave's 64 lanes
// run (nearly) equal-length MD5 loops across the whole tree, and every load
// instruction reads 1 KiB contiguous.  Positions past S are padding
// (tseg = 0xffffffff, nb = 0).
__global__ void __launch_bounds__(256) k_tile_order_global(DevTree t, const uint32_t *__restrict__ perm,
                                                           uint32_t *__restrict__ tseg, uint32_t *__restrict__ tln,
                                                           TileInfo *__restrict__ tinfo, uint64_t *__restrict__ tsize,
                                                           uint64_t ntiles) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t tl = i >> 6;
    uint32_t s = 0xffffffffu, ln = 0;
    if (i < t.S) {
        s = perm[i];
        if (t.seg_off[s] != t.seg_end[s]) ln = (uint32_t)(t.seg_vend[s] - t.seg_voff[s] + 1);
    }
    if (tl < ntiles) {
        tseg[i] = s;
        tln[i] = ln;
    }
    tile_shape(ln, tl, (threadIdx.x & 63) == 0 && tl < ntiles, tinfo, tsize);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS
// operations, not for its global loads and stores.
__device__ __forceinline__ void lds_barrier() {
    __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Mailbox of one inner-node entry read by another workgroup (possibly on
// another XCD, behind another L2): agent-scope atomics, coherent across XCDs
// without a write-back of the writer's L2 or an invalidate of the reader's.
__device__ __forceinline__ void mail_put(MailEntry *m, const uint4 &e, uint32_t tg, uint32_t ep) {
    const unsigned long long E = (unsigned long long)ep << 48;
    const unsigned long long w0 = (unsigned long long)e.x | ((unsigned long long)(e.y & 0xffffu) << 32);
    const unsigned long long w1 = (unsigned long long)(e.y >> 16) | ((unsigned long long)e.z << 16);
    const unsigned long long w2 = (unsigned long long)e.w | ((unsigned long long)(tg & 0xffffu) << 32);
    __hip_atomic_store(&m->w[0], w0 | E, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&m->w[1], w1 | E, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&m->w[2], w2 | E, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Reads a mailbox written in this launch: each word is re-read until it
// carries the epoch.  The wait is bounded (2^18 polls, a fraction of a
// second; a hand-off that works takes microseconds) so a defect cannot hang
// the GPU, and a word that never carries the epoch is an ERROR, not a value:
// mail_get returns false and the caller sets the tree's error word, which
// the host reports as ST_EDEVICE (the climb's hashes are then discarded).
__device__ __forceinline__ bool mail_word(unsigned long long *w, uint32_t ep, unsigned long long &v) {
    v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t it = 0; (uint32_t)(v >> 48) != ep && it < (1u << 18); it++) {
        __builtin_amdgcn_s_sleep(1);
        v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return (uint32_t)(v >> 48) == ep;
}
__device__ __forceinline__ bool mail_get(MailEntry *m, uint4 &e, uint16_t &tg, uint32_t ep) {
    unsigned long long w0 = 0, w1 = 0, w2 = 0;
    bool ok = mail_word(&m->w[0], ep, w0);
    if (ok) ok = mail_word(&m->w[1], ep, w1);   // after a timeout no further waiting
    if (ok) ok = mail_word(&m->w[2], ep, w2);
    e = make_uint4((uint32_t)w0, (uint32_t)((w0 >> 32) & 0xffffu) | ((uint32_t)w1 << 16), (uint32_t)(w1 >> 16),
                   (uint32_t)w2);
    tg = (uint16_t)(w2 >> 32);
    return ok;
}
// Raise a bit of a tree's device-error word (host-mapped, read by the host
// after its next stream synchronisation).  A vector store at system scope.
__device__ __forceinline__ void raise_derr(uint32_t *err, uint32_t bit) {
    if (err) __hip_atomic_store(err, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Window-local tile order (fused rehash): one workgroup per window of 4096
// segments sorts them by stored rows (message length in 16-byte rows,
// descending; LDS counting sort) into the window's 64 tiles:
// tseg/tln[window*4096 + position]; tinfo[tile].B / .R and tsize[tile] from
// tile_shape; pres[window*64 + w]: the window's segment presence bitmap (the
// fused rehash packs each entry at its rank among the present siblings).
__global__ void __launch_bounds__(256) k_tile_order_window(DevTree t, uint32_t *__restrict__ tseg, uint32_t *__restrict__ tln,
                                                           TileInfo *__restrict__ tinfo, uint64_t *__restrict__ tsize,
                                                           uint64_t *__restrict__ pres, uint16_t *__restrict__ noff,
                                                           uint32_t *__restrict__ mhmax) {
    __shared__ uint32_t hist[256];
    __shared__ uint32_t pln[4096];
    __shared__ uint32_t ncnt[256];
    const uint32_t tid = threadIdx.x;
    const uint64_t seg0 = (uint64_t)blockIdx.x * 4096;
    hist[tid] = 0;
    ncnt[tid] = 0;
    __syncthreads();
    uint32_t ln[16], bin[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint64_t s = seg0 + k * 256 + tid;
        ln[k] = t.seg_off[s] != t.seg_end[s] ? (uint32_t)(t.seg_vend[s] - t.seg_voff[s] + 1) : 0u;
        const uint32_t r = ln_rows(ln[k]) + (ln[k] != 0);   // present-but-empty values sort above absent
        bin[k] = 255u - (r > 255u ? 255u : r);
        atomicAdd(&hist[bin[k]], 1u);
        // presence bitmap: bit j of word w = segment 64 w + j has entries
        const unsigned long long bits = __ballot(ln[k] != 0);
        if ((tid & 63) == 0) pres[blockIdx.x * 64 + k * 4 + (tid >> 6)] = bits;
        if (ln[k]) atomicAdd(&ncnt[k * 16 + (tid >> 4)], 1u);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t acc = 0;
        for (int x = 0; x < 256; x++) { const uint32_t c = hist[x]; hist[x] = acc; acc += c; }
    }
    // level-H node tid's message (17 B per present segment) at a 4-byte
    // aligned offset in the fused rehash's LDS: exclusive scan of the sizes
    const uint32_t nsz = (17u * ncnt[tid] + 3u) / 4u;
    __syncthreads();
    ncnt[tid] = nsz;
    __syncthreads();
    for (uint32_t o = 1; o < 256; o <<= 1) {
        const uint32_t x = tid >= o ? ncnt[tid - o] : 0u;
        __syncthreads();
        ncnt[tid] += x;
        __syncthreads();
    }
    noff[blockIdx.x * 256 + tid] = (uint16_t)(ncnt[tid] - nsz);
    if (tid == 255) atomicMax(mhmax, 4u * ncnt[255]);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t pos = atomicAdd(&hist[bin[k]], 1u);
        tseg[seg0 + pos] = (uint32_t)(seg0 + k * 256 + tid);
        tln[seg0 + pos] = ln[k];
        pln[pos] = ln[k];
    }
    __syncthreads();
    const uint32_t lane = tid & 63, wave = tid >> 6;
    for (uint32_t j = wave; j < 64; j += 4) tile_shape(pln[j * 64 + lane], blockIdx.x * 64 + j, lane == 0, tinfo, tsize);
}

// K1 over the tiles: persistent waves, grid-stride over tiles; the next
// tile's info and first block are fetched while the current tile's last
// block is hashed.
__device__ __forceinline__ void tile_store(const DevTree &t, uint4 *md5, uint16_t *tag, uint32_t seg, uint32_t nb,
                                           const uint32_t st[4]) {
    if (seg == 0xffffffffu) return;
    const uint32_t L1 = t.H + 1;
    const uint64_t slot = t.base[L1] + seg;
    if (!nb) {
        tag[slot] = 0;
        if (L1 == 1) tag[0] = 0;
        return;
    }
    const uint4 e = make_uint4(st[0], st[1], st[2], st[3]);
    md5[slot] = e;
    tag[slot] = TAG_PRESENT;
    if (L1 == 1) { md5[0] = e; tag[0] = TAG_PRESENT; }
}

// Persistent K1 (geometries the fused kernel does not cover): wave w hashes
// tiles w, w + nw, ... of `one`.
__global__ void __launch_bounds__(256) k_segment_hash_tiled_p(DevTree t, TreeTiles one, uint64_t ntiles) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    uint64_t g = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (g >= ntiles) return;
    TreeTiles cur = one;
    uint64_t tl = g;
    TileInfo ti = cur.tinfo[tl];
    uint32_t seg = cur.tseg[tl * 64 + lane], ln = cur.tln[tl * 64 + lane];
    uint4 n0 = make_uint4(0, 0, 0, 0), n1 = n0, n2 = n0, n3 = n0;
    if (ti.B) {
        n0 = tile_row(cur.tiles, ti.base, lane, 0, ti.R, ln); n1 = tile_row(cur.tiles, ti.base, lane, 1, ti.R, ln);
        n2 = tile_row(cur.tiles, ti.base, lane, 2, ti.R, ln); n3 = tile_row(cur.tiles, ti.base, lane, 3, ti.R, ln);
    }
    for (;;) {
        const uint64_t gx = g + nw;
        TreeTiles nxt = cur;
        uint64_t tn_l = 0;
        TileInfo tn;
        tn.base = 0; tn.B = 0; tn.R = 0;
        uint32_t segn = 0xffffffffu, lnn = 0;
        if (gx < ntiles) {
            tn_l = gx;
            tn = nxt.tinfo[tn_l];
            segn = nxt.tseg[tn_l * 64 + lane];
            lnn = nxt.tln[tn_l * 64 + lane];
        }
        uint32_t st[4];
        stmd5::init(st);
        const uint32_t nb = ln_blocks(ln);
        for (uint32_t k = 0; k < ti.B; k++) {
            uint32_t m[16] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, n3.x, n3.y, n3.z, n3.w};
            if (k + 1 < ti.B) {
                const uint32_t r = 4 * (k + 1);
                n0 = tile_row(cur.tiles, ti.base, lane, r, ti.R, ln); n1 = tile_row(cur.tiles, ti.base, lane, r + 1, ti.R, ln);
                n2 = tile_row(cur.tiles, ti.base, lane, r + 2, ti.R, ln); n3 = tile_row(cur.tiles, ti.base, lane, r + 3, ti.R, ln);
            } else if (tn.B) {
                n0 = tile_row(nxt.tiles, tn.base, lane, 0, tn.R, lnn); n1 = tile_row(nxt.tiles, tn.base, lane, 1, tn.R, lnn);
                n2 = tile_row(nxt.tiles, tn.base, lane, 2, tn.R, lnn); n3 = tile_row(nxt.tiles, tn.base, lane, 3, tn.R, lnn);
            }
            if (k < nb) stmd5::compress<true>(st, m);
        }
        tile_store(t, cur.md5, cur.tag, seg, nb, st);
        if (gx >= ntiles) break;
        if (ti.B == 0 && tn.B) {
            n0 = tile_row(nxt.tiles, tn.base, lane, 0, tn.R, lnn); n1 = tile_row(nxt.tiles, tn.base, lane, 1, tn.R, lnn);
            n2 = tile_row(nxt.tiles, tn.base, lane, 2, tn.R, lnn); n3 = tile_row(nxt.tiles, tn.base, lane, 3, tn.R, lnn);
        }
        g = gx;
        cur = nxt;
        ti = tn;
        seg = segn;
        ln = lnn;
    }
}


// Top-hash records of many trees into one device array, 18 bytes per tree
// (present byte + the 17-byte hash): the payload of the cross-GPU all-gather
// of ensemble top hashes, built without a host round trip.
__global__ void k_tops_out(const TreeTiles *__restrict__ trees, uint32_t n, uint8_t *out) {
    for (uint64_t i = gtid(); i < (uint64_t)n * 18; i += gstride()) {
        const uint64_t t = i / 18, k = i % 18;
        const uint16_t tg = trees[t].tag[0];
        uint8_t b = 0;
        if (tg & TAG_PRESENT) {
            if (k == 0) b = 1;
            else if (k == 1) b = (uint8_t)(tg & 0xffu);
            else {
                const uint4 m = trees[t].md5[0];
                const uint32_t w[4] = {m.x, m.y, m.z, m.w};
                const uint32_t j = (uint32_t)k - 2;
                b = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
            }
        }
        out[i] = b;
    }
}
