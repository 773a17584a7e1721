// pages.h — the paged segment layout of streaming insert batches (SURVEY
// §8(d) config 5: 1M-key insert/3 batches into a 100M-key tree).
//
// The canonical CSR (st_kernels.h) is gap-free: a batch that adds entries
// to 61 % of the segments shifts every entry after the first change, so a
// merge rewrites the whole CSR (~42 B per entry read and written).  The
// reference rewrites only the segments a batch touches (orddict:store into
// the fetched segment and a backend store of it, synctree.erl:201-209,
// :468-485).  In the paged layout every segment owns a PAGE: a run of entry
// slots (koff/voff) and byte ranges of the key and value heaps, each with
// slack after the segment's content.  A batch rewrites only the TAIL of each
// touched segment -- the entries from the first changed position on -- in
// place (staged through LDS, so sources are read before they are
// overwritten); a segment that outgrows its page moves to a new page in the
// append region at the end of the arrays.  Views of the paged layout are
// ordinary DevTrees (seg_off / seg_end / seg_voff / seg_vend), so path
// verification and the dirty-path hash run unchanged on it.
//
// Layout per segment s: entries [beg[s], end[s]) (slot end[s] holds the
// ends of the last entry's key and value), entry capacity up to ecap[s]
// (end[s] < ecap[s]), key bytes [koff[beg], koff[end]) below kcap[s], value
// bytes [vbeg[s] = voff[beg], vend[s] = voff[end]) below vcap[s].
#pragma once

struct PageMeta {
    uint64_t *beg, *end, *vbeg, *vend;   // S each: the DevTree view's seg_off / seg_end / seg_voff / seg_vend
    uint64_t *ecap, *kcap, *vcap;        // S each: page capacities (entry slot end, key / value byte ends)
};

typedef USum<4> PageSums;   // entries, key bytes, value bytes, new keys (k_page_plan) / unused

// Page capacity for a segment of c entries, kb key bytes and vb value bytes
// (slack_pct: percent of slack; < 0: none, a gap-free CSR).  Byte caps are
// 16-byte multiples so every page starts 16-byte aligned.
__host__ __device__ __forceinline__ PageSums page_caps(uint64_t c, uint64_t kb, uint64_t vb, int slack_pct) {
    PageSums r(0);
    if (slack_pct < 0) {
        r.v[0] = c; r.v[1] = kb; r.v[2] = vb;   // canonical: the next segment's first entry is this one's end
        return r;
    }
    const uint64_t se = c ? (c * (uint64_t)slack_pct / 100 > 4 ? c * (uint64_t)slack_pct / 100 : 4) : 0;
    const uint64_t sk = c ? (kb * (uint64_t)slack_pct / 100 > 32 ? kb * (uint64_t)slack_pct / 100 : 32) : 0;
    const uint64_t sv = c ? (vb * (uint64_t)slack_pct / 100 > 48 ? vb * (uint64_t)slack_pct / 100 : 48) : 0;
    r.v[0] = c + 1 + se;
    r.v[1] = (kb + sk + 15) & ~15ull;
    r.v[2] = (vb + sv + 15) & ~15ull;
    return r;
}

// Sizes of every segment's new page (k_page_copy's destinations, scanned).
__global__ void k_page_sizes(DevTree t, int slack_pct, PageSums *sz) {
    for (uint64_t s = gtid(); s < t.S; s += gstride()) {
        const uint64_t b = t.seg_off[s], e = t.seg_end[s];
        sz[s] = page_caps(e - b, t.koff[e] - t.koff[b], t.seg_vend[s] - t.seg_voff[s], slack_pct);
    }
}

// Copy n bytes from global src to global dst (any alignments) with the whole
// wave: a lane per destination dword, the source bytes joined from two
// aligned dword loads (heaps keep slack past their ends); the first and last
// destination dwords, which other segments' bytes may share, by byte stores.
__device__ __forceinline__ void wave_copy_gg(uint8_t *dst, const uint8_t *src, uint64_t n) {
    if (!n) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t d0 = reinterpret_cast<uintptr_t>(dst), d1 = d0 + n;
    const uint64_t q0 = d0 >> 2, q1 = (d1 + 3) >> 2;   // destination dwords [q0, q1)
    for (uint64_t q = q0 + lane; q < q1; q += 64) {
        const uint64_t g = q << 2;   // the dword's first byte
        if (g >= d0 && g + 4 <= d1) {
            const uint64_t a = reinterpret_cast<uintptr_t>(src) + (g - d0);
            const uint32_t *w = reinterpret_cast<const uint32_t *>(a & ~3ull);
            const uint32_t v = __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(a & 3));
            *reinterpret_cast<uint32_t *>(g) = v;
        } else {
            for (uint32_t i = 0; i < 4; i++)
                if (g + i >= d0 && g + i < d1) reinterpret_cast<uint8_t *>(g + i)[0] = src[g + i - d0];
        }
    }
}

// Copy every segment's entries into a new layout: entry offsets rebased,
// key and value byte ranges copied by the whole wave.  dst: the new arrays;
// base: exclusive scan of the pages' sizes (k_page_sizes).  Writes the new
// page metadata (paged destination) or seg_off / seg_voff (canonical
// destination, meta.beg == nullptr: cseg_off / cseg_voff, S + 1 each).
struct PageDst {
    uint64_t *koff, *voff;
    uint8_t *kheap, *vheap;
    PageMeta m;                      // paged destination (m.beg != nullptr)
    uint64_t *cseg_off, *cseg_voff;  // canonical destination
    uint64_t e0, k0, v0;             // bases added to the scanned offsets
};
__global__ void __launch_bounds__(256) k_page_copy(DevTree t, const PageSums *base, const PageSums *sz, PageDst d) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t s = w0; s < t.S; s += nw) {
        const uint64_t b = t.seg_off[s], e = t.seg_end[s], c = e - b;
        const PageSums B = base[s];
        const uint64_t De = d.e0 + B.v[0], Dk = d.k0 + B.v[1], Dv = d.v0 + B.v[2];
        const uint64_t kb0 = t.koff[b], vb0 = t.voff[b];
        for (uint64_t i = lane; i <= c; i += 64) {   // offsets incl. the end slot
            d.koff[De + i] = Dk + (t.koff[b + i] - kb0);
            d.voff[De + i] = Dv + (t.voff[b + i] - vb0);
        }
        wave_copy_gg(d.kheap + Dk, t.kheap + kb0, t.koff[e] - kb0);
        wave_copy_gg(d.vheap + Dv, t.vheap + vb0, t.voff[e] - vb0);
        if (lane == 0) {
            if (d.m.beg) {
                const PageSums Z = sz[s];
                d.m.beg[s] = De;
                d.m.end[s] = De + c;
                d.m.vbeg[s] = Dv;
                d.m.vend[s] = Dv + (t.voff[e] - vb0);
                d.m.ecap[s] = De + Z.v[0];
                d.m.kcap[s] = Dk + Z.v[1];
                d.m.vcap[s] = Dv + Z.v[2];
            } else {
                d.cseg_off[s] = De;
                d.cseg_voff[s] = Dv;
                if (s + 1 == t.S) {
                    d.cseg_off[s + 1] = De + c;
                    d.cseg_voff[s + 1] = Dv + (t.voff[e] - vb0);
                }
            }
        }
    }
}

// A page merge stages at most this much of a segment's tail in LDS (a wave's
// share of the workgroup's LDS); longer tails move the segment to a new page
// (no staging: sources and destinations are disjoint).
#define PG_TAIL_E 128                       // entries of the tail, end slot included
#define PG_TAIL_B 4096                      // key + value bytes of the tail
#define PG_WAVE_LDS (PG_TAIL_E * 16 + PG_TAIL_B + 64)

// Per touched segment: merge in place (1) or move to a new page (2), or
// nothing (0: no run, a rejected run, no kept record).  reloc = the new
// page's sizes (mode 2), scanned for its place in the append region;
// v[3] = the segment's new keys (for the tree's entry count).
__global__ void k_page_plan(DevTree t, PageMeta m, const uint64_t *bseg_off, const uint8_t *reject, const uint32_t *pos,
                            const SegSums *ss, const uint8_t *dirty, int slack_pct, uint8_t *mode, PageSums *reloc) {
    for (uint64_t s = gtid(); s < t.S; s += gstride()) {
        const uint64_t j0 = bseg_off[s], je = bseg_off[s + 1];
        PageSums r(0);
        uint8_t md = 0;
        if (j0 != je && !(reject && reject[s]) && dirty[s]) {
            const uint64_t b = m.beg[s], e = m.end[s], c = e - b;
            const SegSums x = ss[s];
            const uint64_t kb = t.koff[b], vb = t.voff[b];
            const bool fits = b + x.v[0] < m.ecap[s] && kb + x.v[1] <= m.kcap[s] && vb + x.v[2] <= m.vcap[s];
            const uint64_t p0 = pos[j0];
            const uint64_t tb = (t.koff[e] - t.koff[b + p0]) + (t.voff[e] - t.voff[b + p0]);
            md = fits && c - p0 + 1 <= PG_TAIL_E && tb + 8 <= PG_TAIL_B ? 1 : 2;
            if (md == 2) r = page_caps(x.v[0], x.v[1], x.v[2], slack_pct < 0 ? 0 : slack_pct);
            r.v[3] = x.v[3];
        }
        mode[s] = md;
        reloc[s] = r;
    }
}

// The merge of one batch run into its segment's page (mode 1, in place) or
// into a new page (mode 2): the closed form of k_merge_old / k_merge_new
// (st_kernels.h) per segment, with the run's scanned BatchSums.  A wave per
// segment.  Mode 1 first stages the tail (entries from the run's first
// position on: offsets and bytes) in LDS, so every source is read before any
// write lands on it; entries before the first position stay where they are.
struct PageMergeArgs {
    MergeArgs a;
    PageMeta m;
    uint64_t *koff, *voff;        // the page arrays (a.koff / a.voff, writable)
    uint8_t *kheap, *vheap;
    const uint32_t *pos;
    const BatchSums *bx;          // exclusive scan over the sorted batch
    const SegSums *ss;            // per segment: merged count, key bytes, value bytes
    const uint8_t *mode;
    const PageSums *rbase;        // exclusive scan of the relocation sizes
    const PageSums *rsz;          // the relocation sizes
    uint64_t e0, k0, v0;          // the append region's bases
};

__device__ __forceinline__ uint64_t pg_bound(const uint32_t *pos, uint64_t lo, uint64_t hi, uint64_t li, bool upper) {
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (upper ? pos[mid] <= li : pos[mid] < li) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(256) k_page_merge(PageMergeArgs p) {
    __shared__ __attribute__((aligned(16))) uint8_t lds_raw[4 * PG_WAVE_LDS];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // this wave's staging area: the tail's key offsets, value offsets, then
    // its key bytes and (4-byte aligned) value bytes
    uint64_t *sko = reinterpret_cast<uint64_t *>(lds_raw + wv * PG_WAVE_LDS);
    uint64_t *svo = sko + PG_TAIL_E;
    uint8_t *sby = reinterpret_cast<uint8_t *>(svo + PG_TAIL_E);
    const MergeArgs &a = p.a;
    const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t s = w0; s < a.S; s += nw) {
        const uint8_t md = p.mode[s];
        if (!md) continue;
        const uint64_t j0 = a.bseg_off[s], je = a.bseg_off[s + 1];
        const uint64_t b = p.m.beg[s], c = p.m.end[s] - b;
        const uint64_t Kb = p.koff[b], Vb = p.voff[b];
        const SegSums X = p.ss[s];
        uint64_t De = b, Dk = Kb, Dv = Vb, p0 = p.pos[j0];
        if (md == 2) {
            const PageSums R = p.rbase[s];
            De = p.e0 + R.v[0]; Dk = p.k0 + R.v[1]; Dv = p.v0 + R.v[2];
            p0 = 0;
        }
        const BatchSums &B0 = p.bx[j0];
        // mode 1: stage the tail [p0, c] (offsets incl. the end slot, bytes)
        const uint64_t tk0 = p.koff[b + p0], tv0 = p.voff[b + p0];
        const uint64_t tkn = p.koff[b + c] - tk0, tvn = p.voff[b + c] - tv0;
        const uint32_t tvo = (uint32_t)((tkn + 3) & ~3ull);   // value bytes' start in the staging area
        if (md == 1) {
            for (uint64_t i = lane; i <= c - p0; i += 64) {
                sko[i] = p.koff[b + p0 + i];
                svo[i] = p.voff[b + p0 + i];
            }
            wave_copy4(p.kheap + tk0, (uint32_t)tkn, sby, p.vheap + tv0, (uint32_t)tvn, sby + tvo, p.kheap, 0, sby, p.kheap, 0,
                       sby);
            wave_sync_lds();
        }
        // old entries li in [p0, c): kept ones move to their merged place
        for (uint64_t l0 = p0; l0 < c; l0 += 64) {
            const uint64_t li = l0 + lane;
            if (li >= c) break;
            const uint64_t k = pg_bound(p.pos, j0, je, li, true), k2 = pg_bound(p.pos, j0, je, li, false);
            const BatchSums &Bk = p.bx[k], &Bk2 = p.bx[k2];
            if (Bk.v[BS_EQ] != Bk2.v[BS_EQ]) continue;   // overwritten by the batch
            uint64_t okb, ovb, kl, vl;
            const uint8_t *ks, *vs;
            if (md == 1) {
                const uint32_t r = (uint32_t)(li - p0);
                okb = sko[r]; ovb = svo[r];
                kl = sko[r + 1] - okb; vl = svo[r + 1] - ovb;
                ks = sby + (okb - tk0);
                vs = sby + tvo + (ovb - tv0);
            } else {
                okb = p.koff[b + li]; ovb = p.voff[b + li];
                kl = p.koff[b + li + 1] - okb; vl = p.voff[b + li + 1] - ovb;
                ks = p.kheap + okb;
                vs = p.vheap + ovb;
            }
            const uint64_t nwi = De + li + (Bk.v[BS_NE] - B0.v[BS_NE]) - (Bk2.v[BS_EQ] - B0.v[BS_EQ]);
            const uint64_t nk = Dk + (okb - Kb) + (Bk.v[BS_KN] - B0.v[BS_KN]) - (Bk2.v[BS_KE] - B0.v[BS_KE]);
            const uint64_t nv = Dv + (ovb - Vb) + (Bk.v[BS_VN] - B0.v[BS_VN]) - (Bk2.v[BS_VE] - B0.v[BS_VE]);
            if (md == 2 || nwi != b + li || nk != okb) {
                p.koff[nwi] = nk;
                copy_bytes(p.kheap + nk, ks, kl);
            }
            if (md == 2 || nwi != b + li || nv != ovb) {
                p.voff[nwi] = nv;
                copy_bytes(p.vheap + nv, vs, vl);
            }
        }
        // the batch records that produce an entry
        for (uint64_t j = j0 + lane; j < je; j += 64) {
            const BatchSums &Bj = p.bx[j];
            if (p.bx[j + 1].v[BS_NE] == Bj.v[BS_NE]) continue;
            const uint64_t ps = p.pos[j];
            uint64_t ok;
            uint64_t ov;
            if (md == 1) { ok = sko[ps - p0]; ov = svo[ps - p0]; }
            else { ok = p.koff[b + ps]; ov = p.voff[b + ps]; }
            const uint64_t nwi = De + ps + (Bj.v[BS_NE] - B0.v[BS_NE]) - (Bj.v[BS_EQ] - B0.v[BS_EQ]);
            const uint64_t nk = Dk + (ok - Kb) + (Bj.v[BS_KN] - B0.v[BS_KN]) - (Bj.v[BS_KE] - B0.v[BS_KE]);
            const uint64_t nv = Dv + (ov - Vb) + (Bj.v[BS_VN] - B0.v[BS_VN]) - (Bj.v[BS_VE] - B0.v[BS_VE]);
            const uint32_t bi = a.perm[j];
            const uint64_t bk = a.bv.koff[bi], bvv = a.bvoff[bi];
            p.koff[nwi] = nk;
            p.voff[nwi] = nv;
            copy_bytes(p.kheap + nk, a.bv.kheap + bk, a.bv.koff[bi + 1] - bk);
            copy_bytes(p.vheap + nv, a.bvheap + bvv, a.bvoff[bi + 1] - bvv);
        }
        if (lane == 0) {
            p.koff[De + X.v[0]] = Dk + X.v[1];   // the end slot
            p.voff[De + X.v[0]] = Dv + X.v[2];
            p.m.end[s] = De + X.v[0];
            p.m.vend[s] = Dv + X.v[2];
            if (md == 2) {
                const PageSums Z = p.rsz[s];
                p.m.beg[s] = De;
                p.m.vbeg[s] = Dv;
                p.m.ecap[s] = De + Z.v[0];
                p.m.kcap[s] = Dk + Z.v[1];
                p.m.vcap[s] = Dv + Z.v[2];
            }
        }
        wave_sync_lds();   // the staging area is reused by the wave's next segment
    }
}
