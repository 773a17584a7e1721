// small_path.h — the per-key latency path of insert/3 and get/2 (SURVEY §8f
// rank 4; src/synctree.erl:189-227): a batch of at most SB_MAX keys is served
// by ONE workgroup in ONE launch, with the keys passed as kernel arguments and
// the results written straight into mapped pinned host memory, so a call costs
// one launch and one stream synchronisation.
//
// Segments changed by small inserts are not merged into the CSR at once: the
// new content of a segment goes to an OVERLAY record (ov.idx[s] -> offset in
// ov.heap, a bump-allocated device heap), and the segment's path is rehashed in
// the slot arrays immediately.  Only the small kernels read through the
// overlay; every other entry point first merges the overlay into the CSR
// (flush_overlay in synctree_hip.hip: one ingest with replace flags), so the
// bulk kernels never see it.
//
// Overlay record at ov.heap + off (16-byte aligned):
//   u32 n, kbytes, vbytes, pad; u32 koff[n+1]; u32 voff[n+1];
//   key records [kbytes]; values [vbytes]
// (key records: the CSR's tag + ensure_binary encoding; values contiguous, so
// a segment's hash input is one byte range, as in the CSR).
#pragma once
#include "st_kernels.h"

#define SB_MAX 16        // keys per small batch
#define SB_KB 512        // key-record bytes per small batch
#define SB_VB 512        // value bytes per small batch (insert)
#define SB_OUT_VB 4096   // value bytes a small get returns
#define SB_SEG_CAP 1024  // entries of one segment a small insert rewrites (larger: bulk path)
#define SB_VERIFY 96     // threads that verify path nodes (SB_MAX keys x 6 levels)

struct SmallIn {
    uint32_t n, op;       // op: 0 = get/2, 1 = insert/3
    uint32_t koff[SB_MAX + 1];
    uint32_t voff[SB_MAX + 1];
    uint8_t kb[SB_KB];
    uint8_t vb[SB_VB];
};

struct SmallOut {
    int32_t status[SB_MAX];    // ST_OK / ST_NOTFOUND / ST_CORRUPTED
    uint32_t clevel[SB_MAX];
    uint64_t cbucket[SB_MAX];
    uint32_t voff[SB_MAX + 1]; // get: value i = vbytes[voff[i] .. voff[i+1])
    uint32_t retry;            // 1: not served (overlay full, segment too large): use the bulk path
    uint32_t new_entries;      // insert: keys that were not in their segment before
    uint32_t done;             // set last (host sanity check)
    uint32_t pad;
    uint8_t vbytes[SB_OUT_VB];
};

struct Overlay {
    uint64_t *idx;              // [S], ~0 = segment not in the overlay
    uint8_t *heap;
    unsigned long long *used;   // bump pointer (device)
    uint64_t cap;
};

// get_segment/2 (synctree.erl:251-253) of one key record (tag + payload)
__device__ __forceinline__ uint64_t record_segment(const uint8_t *p, uint64_t len, uint64_t segmask) {
    uint32_t d[4];
    if (p[0] == KEYTAG_INT && len == 9) {
        uint32_t m[16];
        uint32_t x0 = 0, x1 = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) { x0 |= (uint32_t)p[1 + i] << (8 * i); x1 |= (uint32_t)p[5 + i] << (8 * i); }
        m[0] = x0 ^ 0x80u;   // unflip the sign bit: message = <<Key:64/big>>
        m[1] = x1;
        m[2] = 0x80u;
#pragma unroll
        for (int w = 3; w < 16; w++) m[w] = 0u;
        m[14] = 64u;
        stmd5::init(d);
        stmd5::compress(d, m);
    } else {
        const uint8_t *sp;
        uint64_t sl;
        krec_seg_bytes(p, len, &sp, &sl);
        stmd5::md5_global_pf(sp, sl, d);
    }
    const uint64_t lo = ((uint64_t)__builtin_bswap32(d[2]) << 32) | (uint64_t)__builtin_bswap32(d[3]);
    return lo & segmask;
}

// Read-only view of one segment's content: its overlay record if it has one,
// else its CSR range.
struct SegView {
    uint64_t n, e0;
    const uint8_t *kh, *vh;          // key / value byte bases
    const uint64_t *ko64, *vo64;     // CSR: absolute offsets (index e0 + i)
    const uint32_t *ko32, *vo32;     // overlay: relative offsets
    __device__ __forceinline__ uint64_t koff(uint64_t i) const { return ko32 ? ko32[i] : ko64[e0 + i]; }
    __device__ __forceinline__ uint64_t voff(uint64_t i) const { return vo32 ? vo32[i] : vo64[e0 + i]; }
    __device__ __forceinline__ const uint8_t *key(uint64_t i) const { return kh + koff(i); }
    __device__ __forceinline__ uint64_t klen(uint64_t i) const { return koff(i + 1) - koff(i); }
    __device__ __forceinline__ const uint8_t *val(uint64_t i) const { return vh + voff(i); }
    __device__ __forceinline__ uint64_t vlen(uint64_t i) const { return voff(i + 1) - voff(i); }
};

__device__ __forceinline__ SegView seg_view(const DevTree &t, const Overlay &ov, uint64_t s) {
    SegView v;
    const uint64_t o = ov.idx[s];
    if (o != ~0ull) {
        const uint32_t *h = reinterpret_cast<const uint32_t *>(ov.heap + o);
        const uint32_t n = h[0], kb = h[1];
        v.n = n;
        v.e0 = 0;
        v.ko32 = h + 4;
        v.vo32 = h + 4 + (n + 1);
        v.kh = reinterpret_cast<const uint8_t *>(h + 4 + 2 * (n + 1));
        v.vh = v.kh + kb;
        v.ko64 = v.vo64 = nullptr;
    } else {
        v.e0 = t.seg_off[s];
        v.n = t.seg_off[s + 1] - v.e0;
        v.kh = t.kheap;
        v.vh = t.vheap;
        v.ko64 = t.koff;
        v.vo64 = t.voff;
        v.ko32 = v.vo32 = nullptr;
    }
    return v;
}

__device__ __forceinline__ uint64_t ov_record_bytes(uint64_t n, uint64_t kb, uint64_t vb) {
    return (16 + 8 * (n + 1) + kb + vb + 15) & ~15ull;
}

// verify_hash of segment s (synctree.erl:322-340) through the overlay
__device__ __forceinline__ bool verify_segment_ov(const DevTree &t, const Overlay &ov, uint64_t s) {
    const uint32_t L = t.H + 1;
    const uint64_t slot = t.base[L] + s;
    const uint64_t eslot = (L == 1) ? 0 : slot;
    const uint16_t et = t.tag[eslot];
    const SegView v = seg_view(t, ov, s);
    if (!(et & TAG_PRESENT)) return v.n == 0;
    uint32_t d[4];
    const uint64_t a = v.voff(0);
    stmd5::md5_global_pf(v.vh + a, v.voff(v.n) - a, d);
    const uint4 e = t.md5[eslot];
    return (et == TAG_PRESENT) && e.x == d[0] && e.y == d[1] && e.z == d[2] && e.w == d[3];
}

// lower_bound of key record k among the segment's keys
__device__ __forceinline__ uint64_t seg_lower_bound(const SegView &v, const uint8_t *k, uint64_t kl, bool *eq) {
    uint64_t lo = 0, hi = v.n;
    while (lo < hi) {
        const uint64_t m = (lo + hi) >> 1;
        if (rec_cmp(v.key(m), v.klen(m), k, kl) < 0) lo = m + 1; else hi = m;
    }
    *eq = lo < v.n && rec_cmp(v.key(lo), v.klen(lo), k, kl) == 0;
    return lo;
}

// Dynamic LDS of k_small: SB_VERIFY node-staging regions, then per wave a
// merge plan of SB_SEG_CAP + SB_MAX output entries (source, key length, value
// length).
__host__ __device__ __forceinline__ uint32_t small_lds_bytes(uint32_t W) {
    return SB_VERIFY * lane_region_bytes(W) + 4 * (SB_SEG_CAP + SB_MAX) * 12;
}

// The small-batch kernel (one workgroup of 256 threads, 4 waves).
//  1. key -> segment (lane per key; key records copied from the kernel
//     arguments into LDS first)
//  2. path verification: thread per (key, level) verifies node (level,
//     bucket) of the key's path against its parent's entry (get_path,
//     synctree.erl:302-320); a key's first failing level is its {corrupted,
//     Level, Bucket}
//  3. get: lane per key: orddict_find in the segment, value bytes to `out`.
//     insert: wave per distinct touched segment: orddict:store of the batch's
//     keys of that segment in batch order (last writer wins) into a new
//     overlay record (sizes and space reserved for every segment first, so a
//     batch that does not fit changes nothing); then the dirty path bottom-up,
//     one thread per distinct node, a barrier per level (update_path,
//     synctree.erl:201-209).
// `out` is mapped pinned host memory: the host reads it after the stream sync.
__global__ void __launch_bounds__(256) k_small(DevTree t, Overlay ov, SmallIn in, SmallOut *out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    __shared__ uint8_t kb[SB_KB + 64];
    __shared__ uint8_t vb[SB_VB + 64];
    __shared__ uint64_t seg[SB_MAX];
    __shared__ uint32_t bad[SB_MAX];            // first failing level (~0 = none)
    __shared__ uint32_t grp[SB_MAX];            // key -> group (distinct segment) index
    __shared__ uint32_t keep[SB_MAX];           // insert: last writer of its key (and path verified)
    __shared__ uint64_t gseg[SB_MAX];
    __shared__ uint64_t goff[SB_MAX];           // overlay offset of the group's new record
    __shared__ uint32_t gn[SB_MAX], gkb[SB_MAX], gvb[SB_MAX], gnew[SB_MAX];
    __shared__ uint64_t dnode[SB_MAX];
    __shared__ uint32_t ngrp, nd, retry;
    __shared__ uint32_t vlen_out[SB_MAX + 1];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t n = in.n, L1 = t.H + 1;
    for (uint32_t i = tid; i < in.koff[n]; i += blockDim.x) kb[i] = in.kb[i];
    for (uint32_t i = tid; in.op == 1 && i < in.voff[n]; i += blockDim.x) vb[i] = in.vb[i];
    if (tid < SB_MAX) { bad[tid] = ~0u; keep[tid] = 0; }
    if (tid == 0) { ngrp = 0; nd = 0; retry = 0; }
    __syncthreads();
    if (tid < n) seg[tid] = record_segment(kb + in.koff[tid], in.koff[tid + 1] - in.koff[tid], t.S - 1);
    __syncthreads();
    const bool undefined_top = (t.tag[0] & TAG_PRESENT) == 0;
    if (in.op == 0 && undefined_top) {   // get/2: undefined top => notfound (synctree.erl:216-218)
        if (tid < n) { out->status[tid] = ST_NOTFOUND; out->clevel[tid] = 0; out->cbucket[tid] = 0; }
        if (tid <= n) out->voff[tid] = 0;
        __threadfence_system();
        __syncthreads();
        if (tid == 0) { out->retry = 0; out->new_entries = 0; __threadfence_system(); out->done = 1; }
        return;
    }
    // ---- 2. path verification: thread x = key * L1 + (level - 1)
    for (uint32_t x = tid; x < n * L1; x += SB_VERIFY) {
        if (tid >= SB_VERIFY) break;
        const uint32_t i = x / L1, l = x % L1 + 1;
        const uint64_t s = seg[i];
        bool good;
        if (l == L1) good = verify_segment_ov(t, ov, s);
        else good = verify_inner_node(t, l, s >> (t.shift * (L1 - l)), dyn + tid * lane_region_bytes(t.W));
        if (!good) atomicMin(&bad[i], l);
    }
    __syncthreads();
    if (in.op == 0) {
        // ---- 3 (get): orddict_find (synctree.erl:342-348)
        uint32_t len = 0;
        uint64_t at = 0;
        const uint8_t *src = nullptr;
        if (tid < n) {
            if (bad[tid] != ~0u) {
                out->status[tid] = ST_CORRUPTED;
                out->clevel[tid] = bad[tid];
                out->cbucket[tid] = seg[tid] >> (t.shift * (L1 - bad[tid]));
            } else {
                const SegView v = seg_view(t, ov, seg[tid]);
                bool eq;
                at = seg_lower_bound(v, kb + in.koff[tid], in.koff[tid + 1] - in.koff[tid], &eq);
                out->status[tid] = eq ? ST_OK : ST_NOTFOUND;
                out->clevel[tid] = 0;
                out->cbucket[tid] = 0;
                if (eq) { len = (uint32_t)v.vlen(at); src = v.val(at); }
            }
            vlen_out[tid + 1] = len;
        }
        __syncthreads();
        if (tid == 0) {
            vlen_out[0] = 0;
            for (uint32_t i = 1; i <= n; i++) vlen_out[i] += vlen_out[i - 1];
            retry = vlen_out[n] > SB_OUT_VB;
        }
        __syncthreads();
        if (tid <= n) out->voff[tid] = vlen_out[tid];
        if (tid < n && !retry && src)
            for (uint32_t b = 0; b < len; b++) out->vbytes[vlen_out[tid] + b] = src[b];
        __threadfence_system();
        __syncthreads();
        if (tid == 0) { out->retry = retry; out->new_entries = 0; __threadfence_system(); out->done = 1; }
        return;
    }
    // ---- 3 (insert): groups = distinct verified segments, last writer per key
    if (tid == 0) {
        for (uint32_t i = 0; i < n; i++) {
            if (bad[i] != ~0u) continue;
            uint32_t g = 0;
            while (g < ngrp && gseg[g] != seg[i]) g++;
            if (g == ngrp) { gseg[g] = seg[i]; ngrp++; }
            grp[i] = g;
            keep[i] = 1;
            for (uint32_t j = i + 1; j < n; j++)   // a later write of the same key wins
                if (seg[j] == seg[i] && rec_cmp(kb + in.koff[i], in.koff[i + 1] - in.koff[i], kb + in.koff[j],
                                                in.koff[j + 1] - in.koff[j]) == 0) { keep[i] = 0; break; }
        }
    }
    __syncthreads();
    // sizes of every group's new record, space reserved before anything is
    // written (pass 0); then every record written (pass 1).  The merge plan of
    // a group (its output entries' sources and lengths) is rebuilt in each
    // pass by the group's wave (lane 0): a wave's plan area holds one group.
    uint32_t *plan = reinterpret_cast<uint32_t *>(dyn + SB_VERIFY * lane_region_bytes(t.W)) + wave * 3 * (SB_SEG_CAP + SB_MAX);
    uint32_t *pk = plan + (SB_SEG_CAP + SB_MAX), *pv = pk + (SB_SEG_CAP + SB_MAX);
    for (int pass = 0; pass < 2; pass++) {
        for (uint32_t g = wave; g < ngrp; g += 4) {
            const SegView v = seg_view(t, ov, gseg[g]);
            if (lane == 0) {
                // batch keys of the group in key order (<= SB_MAX, insertion sort)
                uint32_t m = 0, idx[SB_MAX];
                for (uint32_t i = 0; i < n; i++)
                    if (keep[i] && grp[i] == g) {
                        uint32_t q = m++;
                        while (q > 0 && rec_cmp(kb + in.koff[idx[q - 1]], in.koff[idx[q - 1] + 1] - in.koff[idx[q - 1]],
                                                kb + in.koff[i], in.koff[i + 1] - in.koff[i]) > 0) {
                            idx[q] = idx[q - 1];
                            q--;
                        }
                        idx[q] = i;
                    }
                // merged order: old entries and batch keys (bit 31), equal keys replaced
                uint64_t x = 0, out_n = 0, kbytes = 0, vbytes = 0, news = 0;
                bool fits = true;
                auto emit = [&](uint32_t src, uint32_t kl, uint32_t vl) {
                    if (out_n >= SB_SEG_CAP) { fits = false; return; }
                    plan[out_n] = src;
                    pk[out_n] = kl;
                    pv[out_n] = vl;
                    kbytes += kl;
                    vbytes += vl;
                    out_n++;
                };
                for (uint32_t r = 0; r < m && fits; r++) {
                    const uint32_t i = idx[r];
                    const uint8_t *k = kb + in.koff[i];
                    const uint64_t kl = in.koff[i + 1] - in.koff[i];
                    bool eq;
                    const uint64_t pos = seg_lower_bound(v, k, kl, &eq);
                    for (; x < pos && fits; x++) emit((uint32_t)x, (uint32_t)v.klen(x), (uint32_t)v.vlen(x));
                    emit(0x80000000u | i, (uint32_t)kl, in.voff[i + 1] - in.voff[i]);
                    if (eq) x++;
                    else news++;
                }
                for (; x < v.n && fits; x++) emit((uint32_t)x, (uint32_t)v.klen(x), (uint32_t)v.vlen(x));
                if (pass == 0) {
                    if (!fits) {
                        atomicOr(&retry, 1u);
                    } else {
                        const uint64_t bytes = ov_record_bytes(out_n, kbytes, vbytes);
                        const uint64_t off = atomicAdd(ov.used, (unsigned long long)bytes);
                        if (off + bytes > ov.cap) atomicOr(&retry, 1u);
                        goff[g] = off;
                        gn[g] = (uint32_t)out_n;
                        gkb[g] = (uint32_t)kbytes;
                        gvb[g] = (uint32_t)vbytes;
                        gnew[g] = (uint32_t)news;
                    }
                } else {   // header and offset tables
                    uint32_t *h = reinterpret_cast<uint32_t *>(ov.heap + goff[g]);
                    const uint32_t mm = gn[g];
                    uint32_t *ko = h + 4, *vo = h + 4 + (mm + 1);
                    h[0] = mm; h[1] = gkb[g]; h[2] = gvb[g]; h[3] = 0;
                    uint32_t a = 0, c = 0;
                    for (uint32_t q = 0; q < mm; q++) { ko[q] = a; vo[q] = c; a += pk[q]; c += pv[q]; }
                    ko[mm] = a;
                    vo[mm] = c;
                }
            }
            if (pass == 1) {   // entry bytes, lane per entry
                wave_sync_lds();
                __threadfence_block();
                uint32_t *h = reinterpret_cast<uint32_t *>(ov.heap + goff[g]);
                const uint32_t mm = gn[g];
                const uint32_t *ko = h + 4, *vo = h + 4 + (mm + 1);
                uint8_t *kd = reinterpret_cast<uint8_t *>(h + 4 + 2 * (mm + 1));
                uint8_t *vd = kd + gkb[g];
                for (uint32_t q = lane; q < mm; q += 64) {
                    const uint32_t src = plan[q];
                    const uint8_t *ks, *vs;
                    if (src & 0x80000000u) {
                        const uint32_t i = src & 0x7fffffffu;
                        ks = kb + in.koff[i];
                        vs = vb + in.voff[i];
                    } else {
                        ks = v.key(src);
                        vs = v.val(src);
                    }
                    for (uint32_t b = 0; b < pk[q]; b++) kd[ko[q] + b] = ks[b];
                    for (uint32_t b = 0; b < pv[q]; b++) vd[vo[q] + b] = vs[b];
                }
                wave_sync_lds();
            }
        }
        __syncthreads();
        if (pass == 0 && retry) {   // nothing was written: the host takes the bulk path
            if (tid == 0) { out->retry = 1; __threadfence_system(); out->done = 1; }
            return;
        }
    }
    __threadfence_block();
    __syncthreads();
    // the new records replace the segments' content; rehash the dirty paths
    if (tid < ngrp) ov.idx[gseg[tid]] = goff[tid];
    __threadfence_block();
    __syncthreads();
    if (tid < ngrp) {   // level H+1: the segment entries
        const uint64_t s = gseg[tid], slot = t.base[L1] + s;
        const SegView v = seg_view(t, ov, s);
        uint32_t d[4];
        const uint64_t a = v.voff(0);
        stmd5::md5_global_pf(v.vh + a, v.voff(v.n) - a, d);
        const uint4 e = make_uint4(d[0], d[1], d[2], d[3]);
        t.md5[slot] = e;
        t.tag[slot] = TAG_PRESENT;
        if (L1 == 1) { t.md5[0] = e; t.tag[0] = TAG_PRESENT; }
    }
    for (uint32_t l = L1 - 1; l >= 1; l--) {
        __threadfence_block();
        __syncthreads();
        if (tid == 0) {
            uint32_t c = 0;
            for (uint32_t g = 0; g < ngrp; g++) {
                const uint64_t b = gseg[g] >> (t.shift * (L1 - l));
                uint32_t q = 0;
                while (q < c && dnode[q] != b) q++;
                if (q == c) dnode[c++] = b;
            }
            nd = c;
        }
        __syncthreads();
        if (tid < nd) {
            const uint64_t b = dnode[tid], slot = t.base[l] + b;
            uint8_t *reg = dyn + tid * lane_region_bytes(t.W);
            const uint32_t len = stage_inner(t, l, b, reg);
            uint32_t d[4];
            stmd5::md5_lds(reg, len, d);   // an insert never empties a node: len > 0
            const uint4 e = make_uint4(d[0], d[1], d[2], d[3]);
            t.md5[slot] = e;
            t.tag[slot] = TAG_PRESENT;
            if (l == 1) { t.md5[0] = e; t.tag[0] = TAG_PRESENT; }
        }
    }
    __syncthreads();
    if (tid < n) {
        if (bad[tid] != ~0u) {
            out->status[tid] = ST_CORRUPTED;
            out->clevel[tid] = bad[tid];
            out->cbucket[tid] = seg[tid] >> (t.shift * (L1 - bad[tid]));
        } else {
            out->status[tid] = ST_OK;
            out->clevel[tid] = 0;
            out->cbucket[tid] = 0;
        }
    }
    if (tid == 0) {
        uint32_t c = 0;
        for (uint32_t g = 0; g < ngrp; g++) c += gnew[g];
        out->new_entries = c;
        out->retry = 0;
    }
    __threadfence_system();
    __syncthreads();
    if (tid == 0) out->done = 1;
}

// Overlay flush, step 1: per segment, the number of overlay entries and
// their key / value bytes (0 for segments without an overlay record).
__global__ void k_ov_sizes(Overlay ov, uint64_t S, uint64_t *cnt, uint64_t *kbytes, uint64_t *vbytes, uint8_t *rep) {
    for (uint64_t s = gtid(); s <= S; s += gstride()) {
        if (s == S) { cnt[s] = kbytes[s] = vbytes[s] = 0; break; }
        const uint64_t o = ov.idx[s];
        if (o == ~0ull) { cnt[s] = kbytes[s] = vbytes[s] = 0; rep[s] = 0; continue; }
        const uint32_t *h = reinterpret_cast<const uint32_t *>(ov.heap + o);
        cnt[s] = h[0];
        kbytes[s] = h[1];
        vbytes[s] = h[2];
        rep[s] = 1;
    }
}

// Overlay flush, step 2: the overlay entries as one ingest batch (segment
// order), with their segment ids (seg_given).
__global__ void k_ov_gather(Overlay ov, uint64_t S, const uint64_t *eoff, const uint64_t *koff0, const uint64_t *voff0,
                            uint8_t *krec, uint64_t *koff, uint8_t *vheap, uint64_t *voff, uint32_t *segs) {
    for (uint64_t s = gtid(); s < S; s += gstride()) {
        const uint64_t o = ov.idx[s];
        if (o == ~0ull) continue;
        const uint32_t *h = reinterpret_cast<const uint32_t *>(ov.heap + o);
        const uint32_t n = h[0], kbn = h[1];
        const uint32_t *ko = h + 4, *vo = h + 4 + (n + 1);
        const uint8_t *kd = reinterpret_cast<const uint8_t *>(h + 4 + 2 * (n + 1)), *vd = kd + kbn;
        const uint64_t e = eoff[s];
        for (uint32_t i = 0; i < n; i++) {
            koff[e + i] = koff0[s] + ko[i];
            voff[e + i] = voff0[s] + vo[i];
            segs[e + i] = (uint32_t)s;
        }
        copy_bytes(krec + koff0[s], kd, kbn);
        copy_bytes(vheap + voff0[s], vd, h[2]);
    }
}

__global__ void k_ov_terminate(uint64_t n, const uint64_t *ktot, const uint64_t *vtot, uint64_t *koff, uint64_t *voff) {
    if (gtid() == 0) { koff[n] = *ktot; voff[n] = *vtot; }
}

// After corrupt/2 (synctree.erl:241-247): if the key's segment is now empty
// the backend holds [] for it (erec).  One thread.
__global__ void k_erec_emptied(DevTree t, const uint8_t *krec, const uint64_t *koff, uint8_t *erec) {
    if (threadIdx.x != 0) return;
    const uint64_t s = record_segment(krec + koff[0], koff[1] - koff[0], t.S - 1);
    if (t.seg_off[s] == t.seg_off[s + 1]) erec[t.base[t.H + 1] + s] = 1;
}
