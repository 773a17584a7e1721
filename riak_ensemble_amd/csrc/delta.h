// delta.h — the streaming-insert delta of a large tree (SURVEY §8d config 5:
// 1M-key write batches into a 100M-key tree).
//
// insert/3 (synctree.erl:189-209) rewrites one segment orddict per key
// (orddict:store, :206).  A batch of 1M keys touches ~63 % of the 2^20
// segments of a 100M-key tree; merging it into the segment CSR moves every
// entry of the tree (the whole 100M-entry heap) on every batch.  Instead a
// batch merges into a DELTA CSR of the entries inserted since the last
// compaction (same layout as the base CSR, a few % of its size), and every
// segment's content is the MERGED VIEW of its base run and its delta run:
// the union of their keys in key order, a delta entry replacing the base
// entry of an equal key (last writer wins, exactly orddict:store).  The base
// never changes between compactions, so each delta entry records, when it
// enters, WHERE its value goes in the base run:
//   aux.x = the byte position (segment-relative, in the base run's value
//           bytes) of the first base entry whose key is >= its key, with bit
//           31 set iff that base key is equal (the entry replaces it);
//   aux.y = the value bytes of the replaced base entry (0 if none).
// A segment's hash input (its values in key order, synctree.erl:255-259) is
// then a sequence of byte ranges -- base run pieces between the delta
// entries' positions and the delta values -- which the merged-view MD5 below
// streams with no key comparison and no copy.  The delta is folded into the
// base (one full merge) when it exceeds its limit, and before any call other
// than a streaming insert (compare, get, snapshot, rehash, ...).
#pragma once

#define DELTA_EQ 0x80000000u

// The delta CSR as the kernels read it.
struct DeltaView {
    const uint64_t *seg_off;   // S + 1 (entries of segment s: [seg_off[s], seg_off[s+1]))
    const uint64_t *voff;      // entries + 1
    const uint8_t *vheap;
    const uint2 *aux;          // entries: (base byte position | DELTA_EQ, replaced base bytes)
};

// Segment of every delta entry (the compaction merges the delta as a batch
// already in segment order).
__global__ void k_delta_entry_seg(const uint64_t *seg_off, uint64_t S, uint32_t *seg) {
    for (uint64_t s = gtid(); s < S; s += gstride())
        for (uint64_t e = seg_off[s]; e < seg_off[s + 1]; e++) seg[e] = (uint32_t)s;
}

// ---------------------------------------------------------------------------
// The merged value stream of one segment as a cursor over its pieces: base
// piece [bpos, next delta position), delta value, base piece, ... , base
// piece up to the end of the run.  Stream offsets are byte positions in the
// merged message.  The descriptors (value bounds, aux) of the next two delta
// entries are held in registers and the one after is loaded when an entry is
// emitted, so a piece boundary does not wait on a dependent load chain.
struct MStream {
    const uint8_t *bsrc;    // the segment's base values
    uint32_t blen;          // their bytes
    const uint8_t *bheap;   // heap starts (guard: a load before a piece's start must stay inside its heap)
    const uint8_t *dheap;
    const uint64_t *dvo;
    const uint2 *aux;
    uint64_t d0;
    uint32_t nd, j;         // delta entries of the segment; the next one to emit
    uint32_t bpos;          // base byte position of the current base piece's start
    bool delta;             // the current piece is a delta value
    bool done;              // past the last piece: L is the stream length
    const uint8_t *src;     // current piece: its bytes, stream range [plo, phi)
    uint64_t plo, phi;
    uint64_t va0, va1, vb1; // value bounds of delta entries j ([va0, va1)) and j + 1 ([va1, vb1))
    uint2 xa, xb;           // their aux
};

__device__ __forceinline__ void ms_init(MStream &m) {
    m.done = false;
    m.delta = false;
    m.j = 0;
    m.bpos = 0;
    m.src = m.bsrc;
    m.plo = 0;
    m.va0 = m.va1 = m.vb1 = 0;
    m.xa = m.xb = make_uint2(0, 0);
    if (m.nd) { m.va0 = m.dvo[m.d0]; m.va1 = m.dvo[m.d0 + 1]; m.xa = m.aux[m.d0]; }
    if (m.nd > 1) { m.vb1 = m.dvo[m.d0 + 2]; m.xb = m.aux[m.d0 + 1]; }
    m.phi = m.nd ? (m.xa.x & ~DELTA_EQ) : m.blen;
}

// Move to the next non-empty piece (or past the end).  The current piece
// ends at stream offset phi.
__device__ __forceinline__ void ms_advance(MStream &m) {
    for (;;) {
        const uint64_t o = m.phi;
        if (!m.delta) {   // a base piece ended: the next delta value, or the end
            if (m.j == m.nd) { m.done = true; m.plo = m.phi = o; return; }
            m.bpos = (m.xa.x & ~DELTA_EQ) + m.xa.y;   // the base piece after it resumes past the replaced entry
            m.delta = true;
            m.src = m.dheap + m.va0;
            m.plo = o;
            m.phi = o + (m.va1 - m.va0);
            // shift the descriptor window; load entry j + 2's
            m.j++;
            m.va0 = m.va1;
            m.va1 = m.vb1;
            m.xa = m.xb;
            if (m.j + 1 < m.nd) { m.vb1 = m.dvo[m.d0 + m.j + 2]; m.xb = m.aux[m.d0 + m.j + 1]; }
        } else {          // a delta value ended: the base piece up to the next delta position
            const uint32_t e = m.j < m.nd ? (m.xa.x & ~DELTA_EQ) : m.blen;
            m.delta = false;
            m.src = m.bsrc + m.bpos;
            m.plo = o;
            m.phi = o + (e - m.bpos);
        }
        if (m.phi > m.plo) return;
    }
}

__device__ __forceinline__ uint4 ld16(const uint8_t *p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);   // unaligned global load (gfx950: unaligned access enabled)
    return v;
}

// 16 bytes whose byte i is p[i - k] for i >= k (0 below): for a piece that
// starts k bytes into a chunk.  One unaligned load from p - k when that stays
// inside the piece's heap, else byte loads (a piece within 16 bytes of its
// heap's start).
__device__ __forceinline__ uint4 ld16_from(const uint8_t *p, uint32_t k, const uint8_t *heap) {
    if ((uint64_t)(p - heap) >= k) return ld16(p - k);
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint32_t i = k; i < 16; i++) w[i >> 2] |= (uint32_t)p[i - k] << (8 * (i & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// Bytes >= k (0..15) of the chunk from y, the rest from x.
__device__ __forceinline__ uint4 bytesel(const uint4 &x, const uint4 &y, uint32_t k) {
    const uint32_t xs[4] = {x.x, x.y, x.z, x.w}, ys[4] = {y.x, y.y, y.z, y.w};
    uint32_t r[4];
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const int d = (int)k - 4 * w;   // bytes of this word that stay x
        const uint32_t m = d <= 0 ? 0xffffffffu : (d >= 4 ? 0u : (0xffffffffu << (8 * d)));
        r[w] = (ys[w] & m) | (xs[w] & ~m);
    }
    return make_uint4(r[0], r[1], r[2], r[3]);
}

// The 16 stream bytes at stream offset P (a multiple of 16).  Bytes past the
// stream's end are garbage (the caller pads).
__device__ __forceinline__ uint4 ms_chunk(MStream &m, uint64_t P) {
    while (!m.done && m.phi <= P) ms_advance(m);
    if (m.done) return make_uint4(0, 0, 0, 0);
    uint4 x = ld16(m.src + (P - m.plo));
    while (!m.done && m.phi < P + 16) {
        ms_advance(m);
        if (m.done) break;
        const uint32_t k = (uint32_t)(m.plo - P);
        x = bytesel(x, ld16_from(m.src, k, m.delta ? m.dheap : m.bheap), k);
    }
    return x;
}

// The merged view's MD5 (synctree.erl:255-259 over the merged orddict) of a
// segment with at least one entry (its values may all be empty: L = 0).
__device__ void md5_merged(MStream &m, uint32_t out[4]) {
    ms_init(m);
    if (m.phi == 0) ms_advance(m);
    uint32_t st[4];
    stmd5::init(st);
    for (uint64_t k = 0;; k++) {
        const uint64_t P = 64 * k;
        const uint4 c0 = ms_chunk(m, P), c1 = ms_chunk(m, P + 16), c2 = ms_chunk(m, P + 32), c3 = ms_chunk(m, P + 48);
        uint32_t w[16] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w, c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, c3.w};
        bool last = false;
        if (m.done) {   // the stream ended at L = plo: pad this block
            const uint64_t L = m.plo;
            const uint64_t nblk = (L + 8) / 64 + 1;
            last = k + 1 == nblk;
            const int64_t rem = (int64_t)L - (int64_t)P;
            if (rem < 64) stmd5::pad_block(w, rem, last, L);
        }
        stmd5::compress<true>(st, w);
        if (last) break;
    }
    out[0] = st[0]; out[1] = st[1]; out[2] = st[2]; out[3] = st[3];
}

// K1 over the merged views of the segments marked in `mask` (a lane per
// segment, in the block-count order `perm` of the base runs): MODE_STORE
// writes the parent's entry (the dirty-path rehash), MODE_VERIFY checks it
// (the insert path's verification, verify_hash/2, synctree.erl:322-340).
template <int MODE>
__global__ void __launch_bounds__(256) k_segment_hash_merged(DevTree t, DeltaView dv, const uint32_t *perm, const uint8_t *mask,
                                                             uint8_t *ok) {
    const uint32_t L1 = t.H + 1;
    for (uint64_t i = gtid(); i < t.S; i += gstride()) {
        const uint64_t s = perm[i];
        const uint64_t slot = t.base[L1] + s;
        if (!mask[slot]) continue;
        MStream m;
        const uint64_t v0 = t.seg_voff[s];
        m.bsrc = t.vheap + v0;
        m.blen = (uint32_t)(t.seg_voff[s + 1] - v0);
        m.bheap = t.vheap;
        m.dheap = dv.vheap;
        m.dvo = dv.voff;
        m.aux = dv.aux;
        m.d0 = dv.seg_off[s];
        m.nd = (uint32_t)(dv.seg_off[s + 1] - m.d0);
        uint32_t d[4] = {0, 0, 0, 0};
        const bool present = t.seg_off[s] != t.seg_off[s + 1] || m.nd;   // delta entries are puts: never fewer entries
        if (present) md5_merged(m, d);
        const uint64_t eslot = (L1 == 1) ? 0 : slot;
        if (MODE == MODE_VERIFY) {
            const uint16_t et = t.tag[eslot];
            bool good;
            if (!(et & TAG_PRESENT)) {
                good = !present;
            } else {
                const uint4 e = t.md5[eslot];
                good = present && et == TAG_PRESENT && e.x == d[0] && e.y == d[1] && e.z == d[2] && e.w == d[3];
            }
            ok[slot] = good ? 1 : 0;
        } else {
            if (!present) {
                t.tag[slot] = 0;
                if (L1 == 1) t.tag[0] = 0;
            } else {
                const uint4 e = make_uint4(d[0], d[1], d[2], d[3]);
                t.md5[slot] = e;
                t.tag[slot] = TAG_PRESENT;
                if (L1 == 1) { t.md5[0] = e; t.tag[0] = TAG_PRESENT; }
            }
        }
    }
}
