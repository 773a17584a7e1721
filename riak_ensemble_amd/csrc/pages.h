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

typedef USum<5> PageSums;   // entries, key bytes, value bytes; k_page_plan: + new keys, octet jobs

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

#define PG_GR 4   // runs of at most this many records: an octet per segment (k_page_tails); longer: k_page_wide

// Per touched segment: merge in place (1) or move to a new page (2), or
// nothing (0: no run, a rejected run, no kept record).  In place needs room
// in the page and every prefix of the run adding >= 0 key and value bytes
// (no replacement that shrinks the bytes before a piece: the moves run from
// the highest address down); otherwise the segment moves.  reloc = the new
// page's sizes (mode 2), scanned for its place in the append region; v[3] =
// the segment's new keys (for the tree's entry count); kv0 = the page's key
// and value bases before the merge (the record placement reads them after).
__global__ void k_page_plan(PageMeta m, const uint64_t *koff, const uint64_t *voff, const uint64_t *bseg_off,
                            const uint8_t *reject, const BatchSums *bs, const SegSums *ss, const uint8_t *dirty, uint64_t S,
                            int slack_pct, uint8_t *mode, PageSums *reloc, uint2 *kv0) {
    for (uint64_t s = gtid(); s < S; s += gstride()) {
        const uint64_t j0 = bseg_off[s], je = bseg_off[s + 1];
        PageSums r(0);
        uint8_t md = 0;
        if (j0 != je && !(reject && reject[s]) && dirty[s]) {
            const uint64_t b = m.beg[s];
            const SegSums x = ss[s];
            const uint64_t kb = koff[b], vb = voff[b];
            const bool fits = b + x.v[0] < m.ecap[s] && kb + x.v[1] <= m.kcap[s] && vb + x.v[2] <= m.vcap[s];
            bool grow = true;
            int64_t dk = 0, dv = 0;
            for (uint64_t j = j0; j < je && grow; j++) {
                const BatchSums &f = bs[j];
                dk += (int64_t)f.v[BS_KN] - (int64_t)f.v[BS_KE];
                dv += (int64_t)f.v[BS_VN] - (int64_t)f.v[BS_VE];
                grow = dk >= 0 && dv >= 0;
            }
            md = fits && grow ? 1 : 2;
            if (md == 2) r = page_caps(x.v[0], x.v[1], x.v[2], slack_pct < 0 ? 0 : slack_pct);
            r.v[3] = x.v[3];
            r.v[4] = je - j0 <= PG_GR ? 1 : 0;   // an octet job (k_page_jobs / k_page_tails)
            kv0[2 * s] = make_uint2((uint32_t)kb, (uint32_t)(kb >> 32));
            kv0[2 * s + 1] = make_uint2((uint32_t)vb, (uint32_t)(vb >> 32));
        }
        mode[s] = md;
        reloc[s] = r;
    }
}

// The merge of one batch run into its segment's page (mode 1, in place) or
// into a new page (mode 2): the closed form of k_merge_old / k_merge_new
// (st_kernels.h) per segment.  The run's records with one position u form a
// GROUP; after group g the old entries [u_g (+1 if its last record replaces
// entry u_g), u_{g+1}) -- a PIECE -- keep their order and shift by the
// running sums through the group (entries +NE-EQ, key bytes +KN-KE, value
// bytes +VN-VE).  k_page_tails moves the pieces (in place: only the tail from
// the first record's position on), k_page_records then writes the records
// into the gaps.
struct PageMergeArgs {
    MergeArgs a;
    PageMeta m;
    uint64_t *koff, *voff;        // the page arrays (a.koff / a.voff, writable)
    uint8_t *kheap, *vheap;
    const uint32_t *pos;
    const uint32_t *sseg;         // segment of each sorted batch record
    const RecAt *rat;             // per record: old offsets at its position (page-relative), its batch offsets
    const BatchSums *bx;          // exclusive scan over the sorted batch
    const SegSums *ss;            // per segment: merged count, key bytes, value bytes
    const uint8_t *mode;
    const PageSums *rbase;        // exclusive scan of the relocation sizes
    const PageSums *rsz;          // the relocation sizes
    const uint2 *kv0;             // per segment: the page's key / value bases before the merge
    uint64_t e0, k0, v0;          // the append region's bases
    unsigned long long *chk;      // checked build (st_debug_knob ST_DBG_PAGE_CHECK): [0] violations, [1..4] the first
};

// Checked build: a store outside its page is counted and skipped, and the
// first one recorded (code, segment, address, bound), instead of faulting.
__device__ __forceinline__ bool pg_ok(unsigned long long *chk, bool ok, uint32_t code, uint64_t s, uint64_t x, uint64_t bound) {
    if (ok || !chk) return true;
    if (atomicAdd(&chk[0], 1ull) == 0) { chk[1] = code; chk[2] = s; chk[3] = x; chk[4] = bound; }
    return false;
}

__device__ __forceinline__ uint64_t pg_kv0(const uint2 *kv0, uint64_t s, int which) {
    const uint2 x = kv0[2 * s + which];
    return ((uint64_t)x.y << 32) | x.x;
}

// n bytes from src to dst, highest 16 bytes first (dst >= src, or the two
// disjoint): every chunk is loaded before a lower chunk's store can reach it.
// Unaligned 16-byte global loads / stores (the heaps keep slack).
__device__ __forceinline__ void lane_move_down(uint8_t *dst, const uint8_t *src, uint64_t n) {
    uint64_t i = n;
    while (i >= 16) {
        uint4 v;
        __builtin_memcpy(&v, src + i - 16, 16);
        __builtin_memcpy(dst + i - 16, &v, 16);
        i -= 16;
    }
    while (i) {
        i--;
        dst[i] = src[i];
    }
}

// A run of more than PG_GR records: the whole segment by one lane, the
// groups from the last to the first (each piece moved highest first, then
// the group's records).
__device__ void page_merge_lane(const PageMergeArgs &p, uint64_t s, uint8_t md, uint64_t b, uint64_t c, uint64_t De,
                                uint64_t Dk, uint64_t Dv) {
    const MergeArgs &a = p.a;
    const uint64_t j0 = a.bseg_off[s], je = a.bseg_off[s + 1];
    const uint64_t Kb = p.koff[b], Vb = p.voff[b];
    const BatchSums B0 = p.bx[j0];
    uint64_t hi = c, khi = p.koff[b + c], vhi = p.voff[b + c];
    uint64_t j = je;
    while (j > j0) {
        const uint64_t u = p.pos[j - 1];
        uint64_t g0 = j - 1;
        while (g0 > j0 && p.pos[g0 - 1] == u) g0--;
        const BatchSums Bj = p.bx[j];
        const bool eq = Bj.v[BS_EQ] != p.bx[j - 1].v[BS_EQ];   // the group's last record replaces entry u
        const uint64_t lo = u + (eq ? 1 : 0);
        const uint64_t de = (Bj.v[BS_NE] - B0.v[BS_NE]) - (Bj.v[BS_EQ] - B0.v[BS_EQ]);
        const uint64_t dk = (Bj.v[BS_KN] - B0.v[BS_KN]) - (Bj.v[BS_KE] - B0.v[BS_KE]);
        const uint64_t dv = (Bj.v[BS_VN] - B0.v[BS_VN]) - (Bj.v[BS_VE] - B0.v[BS_VE]);
        RecAt R = p.rat[j - 1];   // entry u's old offsets
        R.ku += Kb;
        R.vu += Vb;
        if (lo < hi) {
            const uint64_t k0 = p.koff[b + lo], v0 = p.voff[b + lo];
            lane_move_down(p.kheap + Dk + (k0 - Kb) + dk, p.kheap + k0, khi - k0);
            lane_move_down(p.vheap + Dv + (v0 - Vb) + dv, p.vheap + v0, vhi - v0);
            for (uint64_t i = hi; i > lo; i--) {
                p.koff[De + i - 1 + de] = Dk + (p.koff[b + i - 1] - Kb) + dk;
                p.voff[De + i - 1 + de] = Dv + (p.voff[b + i - 1] - Vb) + dv;
            }
        }
        for (uint64_t r = j; r > g0; r--) {
            const BatchSums &Br = p.bx[r - 1];
            if (p.bx[r].v[BS_NE] == Br.v[BS_NE]) continue;
            const uint64_t nwi = De + u + (Br.v[BS_NE] - B0.v[BS_NE]) - (Br.v[BS_EQ] - B0.v[BS_EQ]);
            const uint64_t nk = Dk + (R.ku - Kb) + (Br.v[BS_KN] - B0.v[BS_KN]) - (Br.v[BS_KE] - B0.v[BS_KE]);
            const uint64_t nv = Dv + (R.vu - Vb) + (Br.v[BS_VN] - B0.v[BS_VN]) - (Br.v[BS_VE] - B0.v[BS_VE]);
            const RecAt Q = p.rat[r - 1];
            p.koff[nwi] = nk;
            p.voff[nwi] = nv;
            copy_bytes(p.kheap + nk, a.bv.kheap + Q.bk, p.bx[r].v[BS_KN] - Br.v[BS_KN]);
            copy_bytes(p.vheap + nv, a.bvheap + Q.bv, p.bx[r].v[BS_VN] - Br.v[BS_VN]);
        }
        hi = u; khi = R.ku; vhi = R.vu;
        j = g0;
    }
    if (md == 2 && hi) {   // the entries before the first record, unshifted, into the new page
        lane_move_down(p.kheap + Dk, p.kheap + Kb, khi - Kb);
        lane_move_down(p.vheap + Dv, p.vheap + Vb, vhi - Vb);
        for (uint64_t i = 0; i < hi; i++) {
            p.koff[De + i] = Dk + (p.koff[b + i] - Kb);
            p.voff[De + i] = Dv + (p.voff[b + i] - Vb);
        }
    }
}

__device__ __forceinline__ uint8_t u4_byte(const uint4 &v, uint32_t k) {
    const uint32_t w = (k & 8) ? ((k & 4) ? v.w : v.z) : ((k & 4) ? v.y : v.x);
    return (uint8_t)(w >> (8 * (k & 3)));
}

// The octet jobs, packed (k_page_plan counted them, the relocation scan
// placed them): everything a segment's octet needs before its records, in
// one 128-byte record it loads with one round trip.  Byte positions are
// relative to the page's key / value base (pages are 16-byte aligned).
struct PageJob {
    uint64_t w[16];
};
__global__ void k_page_jobs(PageMergeArgs p, PageJob *jobs) {
    const MergeArgs &a = p.a;
    for (uint64_t s = gtid(); s < a.S; s += gstride()) {
        const uint8_t md = p.mode[s];
        if (!md) continue;
        const uint64_t j0 = a.bseg_off[s], nr = a.bseg_off[s + 1] - j0;
        if (nr > PG_GR) continue;
        const uint64_t b = p.m.beg[s], C = p.m.end[s] - b;
        const uint64_t KB = p.koff[b], VB = p.voff[b], KEND = p.koff[b + C], VEND = p.voff[b + C];
        const PageSums R = p.rbase[s];
        const RecAt r0 = p.rat[j0];
        const uint64_t U0 = p.pos[j0];
        const SegSums X = p.ss[s];
        uint64_t DE = b, DK = KB, DV = VB, EC = 0, KC = 0, VC = 0;
        if (md == 2) {
            DE = p.e0 + R.v[0]; DK = p.k0 + R.v[1]; DV = p.v0 + R.v[2];
            const PageSums Z = p.rsz[s];
            EC = DE + Z.v[0]; KC = DK + Z.v[1]; VC = DV + Z.v[2];
        } else {
            EC = p.m.ecap[s]; KC = p.m.kcap[s]; VC = p.m.vcap[s];
        }
        PageJob J;
        J.w[0] = s | ((uint64_t)md << 32) | (nr << 40);
        J.w[1] = j0;
        J.w[2] = b;
        J.w[3] = C | (U0 << 32);
        J.w[4] = KB; J.w[5] = VB;
        J.w[6] = DE; J.w[7] = DK; J.w[8] = DV;
        J.w[9] = (KEND - KB) | ((VEND - VB) << 32);
        J.w[10] = r0.ku | (r0.vu << 32);   // the first record's position: in place, the moves start here
        J.w[11] = X.v[0] | (X.v[1] << 32);  // merged entries, key bytes
        J.w[12] = X.v[2];                   // merged value bytes
        J.w[13] = EC; J.w[14] = KC; J.w[15] = VC;
        jobs[R.v[4]] = J;
    }
}

typedef unsigned __int128 u128;
// chunk bytes [o, o + n) taken from v (v's byte 0 = chunk byte o); n >= 1, o + n <= 16
__device__ __forceinline__ u128 pg_merge16(u128 acc, u128 v, uint32_t o, uint32_t n) {
    const u128 m = (n >= 16 ? ~(u128)0 : (((u128)1 << (8 * n)) - 1)) << (8 * o);
    return (acc & ~m) | ((v << (8 * o)) & m);
}

// The pieces and records of every octet job, eight lanes (an OCTET) per
// segment.  The octet's lanes hold the run's records (<= PG_GR).  The new
// content of each heap's moving range is written as 16-byte DESTINATION
// chunks (the pages are 16-byte aligned): every chunk's bytes are gathered
// from at most PG_HITS source intervals -- the unchanged prefix, a record's
// bytes from the batch, a piece's old bytes (shifted) -- and stored with one
// aligned 16-byte store (the last chunk's tail lands in the page's slack).
// Chunks go from the highest down in ROUNDS, each round's loads before its
// stores: in place every source byte a chunk uses lies at or below the
// chunk (all shifts >= 0), i.e. in a chunk not yet written.  Entry offsets
// move the same way, 8 bytes each; k_page_records writes the records'
// offsets.  Positions are page-relative 32-bit values.
#define PG_KC 1     // key chunks per lane a round
#define PG_VC 2     // value chunks per lane a round
#define PG_EC 2     // entries per lane a round (each of koff / voff)
#define PG_HITS 3   // source intervals gathered per chunk in one round trip (more: one interval at a time)
template <bool CHECK>
__global__ void __launch_bounds__(256, 3) k_page_tails(PageMergeArgs p, const PageJob *jobs, uint64_t njobs) {
    const uint32_t ol = threadIdx.x & 7;   // lane in the octet
    unsigned long long *chk = CHECK ? p.chk : nullptr;
    const uint64_t o0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3, no = ((uint64_t)gridDim.x * blockDim.x) >> 3;
    const int ob = (int)(threadIdx.x & 63 & ~7u);   // the octet's first lane in the wave
    const uint64_t iters = (njobs + no - 1) / no;   // every octet of a wave the same count (shuffles)
    for (uint64_t it = 0; it < iters; it++) {
        const uint64_t ji = o0 + it * no;
        const bool on = ji < njobs;
        uint64_t w0 = 0, w1 = 0;   // lane k of the octet: job words 2k, 2k + 1
        if (on) { w0 = jobs[ji].w[2 * ol]; w1 = jobs[ji].w[2 * ol + 1]; }
        auto jw = [&](int k) { return __shfl((k & 1) ? w1 : w0, ob + (k >> 1), 64); };
        const uint64_t h0 = jw(0);
        const uint64_t s = (uint32_t)h0;
        const uint32_t md = on ? (uint32_t)(h0 >> 32) & 0xff : 0u, nr = on ? (uint32_t)(h0 >> 40) : 0u;
        const uint64_t j0 = jw(1), b = jw(2), h3 = jw(3);
        const uint32_t C = (uint32_t)h3, U0 = (uint32_t)(h3 >> 32);
        const uint64_t KB = jw(4), VB = jw(5), DE = jw(6), DK = jw(7), DV = jw(8), h9 = jw(9), h10 = jw(10), h11 = jw(11);
        const uint32_t kend = (uint32_t)h9, vend = (uint32_t)(h9 >> 32), k0r = (uint32_t)h10, v0r = (uint32_t)(h10 >> 32);
        const uint32_t NC = (uint32_t)h11, NK = (uint32_t)(h11 >> 32), NV = (uint32_t)jw(12);
        const uint64_t ECAP = jw(13), KCAP = jw(14), VCAP = jw(15);
        // the records: lane k = record j0 + k (k < nr); lane nr holds the run's end sums
        const bool rl = on && ol < nr;
        BatchSums E(0);
        uint32_t u = 0, ku = 0, vu = 0;
        uint64_t bk = 0, bv = 0;
        if (on && ol <= nr) E = p.bx[j0 + ol];
        if (rl) {
            u = p.pos[j0 + ol];
            const RecAt R = p.rat[j0 + ol];
            ku = (uint32_t)R.ku; vu = (uint32_t)R.vu;
            bk = R.bk; bv = R.bv;
        }
        auto osh = [&](uint32_t x, uint32_t k) { return (uint32_t)__shfl((int)x, ob + (int)(k & 7), 64); };
        uint32_t nx[6], ni[6];   // this record's exclusive and inclusive running sums (32-bit differences)
#pragma unroll
        for (int f = 0; f < 6; f++) {
            const uint64_t e0 = __shfl(E.v[f], ob, 64), e1 = __shfl(E.v[f], ob + (int)((ol + 1) & 7), 64);
            nx[f] = (uint32_t)(E.v[f] - e0);
            ni[f] = (uint32_t)(e1 - e0);
        }
        const bool eqr = rl && ni[BS_EQ] != nx[BS_EQ];   // this record replaces entry u
        const bool isne = rl && ni[BS_NE] != nx[BS_NE];   // it produces an entry
        const uint32_t nu = osh(u, ol + 1), nku = osh(ku, ol + 1), nvu = osh(vu, ol + 1);
        const bool last = rl && ol + 1 == nr;
        const uint32_t glf = rl && (last || nu != u) ? 1u : 0u;   // the last record of its group: a piece follows
        // the record's new bytes [rk, rk + rkn) and the piece after it: old [pkl, pkh) at shift sdk (values alike)
        const uint32_t rk = ku + nx[BS_KN] - nx[BS_KE], rkn = isne ? ni[BS_KN] - nx[BS_KN] : 0u;
        const uint32_t rv = vu + nx[BS_VN] - nx[BS_VE], rvn = isne ? ni[BS_VN] - nx[BS_VN] : 0u;
        const uint32_t plo = u + (eqr ? 1 : 0), phi = last ? C : nu;
        const uint32_t pkl = ku + (eqr ? ni[BS_KE] - nx[BS_KE] : 0), pkh = last ? kend : nku;
        const uint32_t pvl = vu + (eqr ? ni[BS_VE] - nx[BS_VE] : 0), pvh = last ? vend : nvu;
        const uint32_t sde = ni[BS_NE] - ni[BS_EQ], sdk = ni[BS_KN] - ni[BS_KE], sdv = ni[BS_VN] - ni[BS_VE];
        // in place the moving ranges start at the first record's position (16-byte aligned down for the bytes);
        // a moved page is written whole
        const uint32_t ka0 = md == 2 ? 0u : k0r & ~15u, va0 = md == 2 ? 0u : v0r & ~15u, ex0 = md == 2 ? 0u : U0;
        const bool ok_rng = !on || pg_ok(chk, NK >= ka0 && NV >= va0 && C >= ex0 && (uint64_t)NK + 16 <= KCAP - DK + 16 &&
                                             DK + ((NK + 15) & ~15u) <= KCAP && DV + ((NV + 15) & ~15u) <= VCAP, 10, s, NK, ka0);
        const uint32_t nkq = on && ok_rng ? (NK - ka0 + 15) >> 4 : 0, nvq = on && ok_rng ? (NV - va0 + 15) >> 4 : 0;
        const uint32_t neq = on && ok_rng ? C - ex0 : 0;
        uint32_t nround = (nkq + 8 * PG_KC - 1) / (8 * PG_KC);
        nround = max(nround, (nvq + 8 * PG_VC - 1) / (8 * PG_VC));
        nround = max(nround, (neq + 8 * PG_EC - 1) / (8 * PG_EC));
        uint32_t gmax = nr;
        for (int o = 32; o >= 1; o >>= 1) {
            nround = max(nround, (uint32_t)__shfl_xor((int)nround, o, 64));
            gmax = max(gmax, (uint32_t)__shfl_xor((int)gmax, o, 64));
        }
        const uint8_t *bkh = p.a.bv.kheap, *bvh = p.a.bvheap;
        const uint8_t *okp = p.kheap + KB, *ovp = p.vheap + VB;   // old pages
        uint8_t *dkp = p.kheap + DK, *dvp = p.vheap + DV;         // destination pages
        for (uint32_t Rn = 0; Rn < nround; Rn++) {
            // ---- the chunks of this round (the highest not yet written) and their source intervals
            uint32_t kq[PG_KC], vq[PG_VC];
            const uint8_t *ksrc[PG_KC][PG_HITS], *vsrc[PG_VC][PG_HITS];
            uint32_t kon[PG_KC][PG_HITS], von[PG_VC][PG_HITS];   // (o << 8) | n; 0 = no hit
            uint32_t kovf = 0, vovf = 0;
#pragma unroll
            for (int i = 0; i < PG_KC; i++) {
                const uint32_t q = Rn * 8 * PG_KC + i * 8 + ol;
                kq[i] = q < nkq ? ka0 + 16 * (nkq - 1 - q) : ~0u;   // chunk start (relative)
#pragma unroll
                for (int h = 0; h < PG_HITS; h++) { kon[i][h] = 0; ksrc[i][h] = okp; }
            }
#pragma unroll
            for (int i = 0; i < PG_VC; i++) {
                const uint32_t q = Rn * 8 * PG_VC + i * 8 + ol;
                vq[i] = q < nvq ? va0 + 16 * (nvq - 1 - q) : ~0u;
#pragma unroll
                for (int h = 0; h < PG_HITS; h++) { von[i][h] = 0; vsrc[i][h] = ovp; }
            }
            // an interval [lo, hi) of new positions whose byte x comes from src[x - lo]
            auto hitk = [&](uint32_t lo, uint32_t hi, const uint8_t *src) {
#pragma unroll
                for (int i = 0; i < PG_KC; i++) {
                    if (kq[i] == ~0u) continue;
                    const uint32_t aa = max(kq[i], lo), ee = min(kq[i] + 16, hi);
                    if (aa >= ee) continue;
                    bool put = false;
#pragma unroll
                    for (int h = 0; h < PG_HITS; h++)
                        if (!put && kon[i][h] == 0) { kon[i][h] = ((aa - kq[i]) << 8) | (ee - aa); ksrc[i][h] = src + (aa - lo); put = true; }
                    if (!put) kovf |= 1u << i;
                }
            };
            auto hitv = [&](uint32_t lo, uint32_t hi, const uint8_t *src) {
#pragma unroll
                for (int i = 0; i < PG_VC; i++) {
                    if (vq[i] == ~0u) continue;
                    const uint32_t aa = max(vq[i], lo), ee = min(vq[i] + 16, hi);
                    if (aa >= ee) continue;
                    bool put = false;
#pragma unroll
                    for (int h = 0; h < PG_HITS; h++)
                        if (!put && von[i][h] == 0) { von[i][h] = ((aa - vq[i]) << 8) | (ee - aa); vsrc[i][h] = src + (aa - lo); put = true; }
                    if (!put) vovf |= 1u << i;
                }
            };
            if (on) { hitk(0, k0r, okp); hitv(0, v0r, ovp); }   // the unchanged prefix (moved as is in a moved page)
            for (uint32_t g = 0; g < gmax; g++) {
                const uint32_t g_rk = osh(rk, g), g_rkn = osh(rkn, g), g_rv = osh(rv, g), g_rvn = osh(rvn, g);
                const uint32_t g_gl = osh(glf, g), g_pkl = osh(pkl, g), g_pkh = osh(pkh, g), g_pvl = osh(pvl, g), g_pvh = osh(pvh, g);
                const uint32_t g_dk = osh(sdk, g), g_dv = osh(sdv, g);
                const uint64_t g_bk = __shfl(bk, ob + (int)g, 64), g_bv = __shfl(bv, ob + (int)g, 64);
                if (!on || g >= nr) continue;
                if (g_rkn) hitk(g_rk, g_rk + g_rkn, bkh + g_bk);
                if (g_rvn) hitv(g_rv, g_rv + g_rvn, bvh + g_bv);
                if (g_gl) {
                    hitk(g_pkl + g_dk, g_pkh + g_dk, okp + g_pkl);
                    hitv(g_pvl + g_dv, g_pvh + g_dv, ovp + g_pvl);
                }
            }
            // ---- loads: every hit of every chunk, then the old entry offsets
            u128 kd[PG_KC][PG_HITS], vd[PG_VC][PG_HITS];
#pragma unroll
            for (int i = 0; i < PG_KC; i++)
#pragma unroll
                for (int h = 0; h < PG_HITS; h++)
                    if (kon[i][h]) __builtin_memcpy(&kd[i][h], ksrc[i][h], 16);
#pragma unroll
            for (int i = 0; i < PG_VC; i++)
#pragma unroll
                for (int h = 0; h < PG_HITS; h++)
                    if (von[i][h]) __builtin_memcpy(&vd[i][h], vsrc[i][h], 16);
            uint32_t ei[PG_EC];
            uint64_t eo[PG_EC], ev[PG_EC];
#pragma unroll
            for (int i = 0; i < PG_EC; i++) {
                const uint32_t q = Rn * 8 * PG_EC + i * 8 + ol;
                ei[i] = q < neq ? C - 1 - q : ~0u;   // old entry index (page-relative)
                if (ei[i] != ~0u) { eo[i] = p.koff[b + ei[i]]; ev[i] = p.voff[b + ei[i]]; }
            }
            // chunks with more intervals than PG_HITS: byte by byte, every interval in turn (rare: tiny keys)
            // (gathered before any store of the round: a lower chunk's store may cover their sources)
            u128 ka[PG_KC], va[PG_VC];
#pragma unroll
            for (int i = 0; i < PG_KC; i++) ka[i] = 0;
#pragma unroll
            for (int i = 0; i < PG_VC; i++) va[i] = 0;
            if (__ballot(kovf != 0 || vovf != 0)) {
                auto slowk = [&](uint32_t lo, uint32_t hi, const uint8_t *src) {
#pragma unroll
                    for (int i = 0; i < PG_KC; i++) {
                        if (!((kovf >> i) & 1u)) continue;
                        const uint32_t aa = max(kq[i], lo), ee = min(kq[i] + 16, hi);
                        for (uint32_t x = aa; x < ee; x++) ka[i] = pg_merge16(ka[i], (u128)src[x - lo], x - kq[i], 1);
                    }
                };
                auto slowv = [&](uint32_t lo, uint32_t hi, const uint8_t *src) {
#pragma unroll
                    for (int i = 0; i < PG_VC; i++) {
                        if (!((vovf >> i) & 1u)) continue;
                        const uint32_t aa = max(vq[i], lo), ee = min(vq[i] + 16, hi);
                        for (uint32_t x = aa; x < ee; x++) va[i] = pg_merge16(va[i], (u128)src[x - lo], x - vq[i], 1);
                    }
                };
                if (on) { slowk(0, k0r, okp); slowv(0, v0r, ovp); }
                for (uint32_t g = 0; g < gmax; g++) {
                    const uint32_t g_rk = osh(rk, g), g_rkn = osh(rkn, g), g_rv = osh(rv, g), g_rvn = osh(rvn, g);
                    const uint32_t g_gl = osh(glf, g), g_pkl = osh(pkl, g), g_pkh = osh(pkh, g), g_pvl = osh(pvl, g), g_pvh = osh(pvh, g);
                    const uint32_t g_dk = osh(sdk, g), g_dv = osh(sdv, g);
                    const uint64_t g_bk = __shfl(bk, ob + (int)g, 64), g_bv = __shfl(bv, ob + (int)g, 64);
                    if (!on || g >= nr) continue;
                    if (g_rkn) slowk(g_rk, g_rk + g_rkn, bkh + g_bk);
                    if (g_rvn) slowv(g_rv, g_rv + g_rvn, bvh + g_bv);
                    if (g_gl) {
                        slowk(g_pkl + g_dk, g_pkh + g_dk, okp + g_pkl);
                        slowv(g_pvl + g_dv, g_pvh + g_dv, ovp + g_pvl);
                    }
                }
            }
            // ---- the chunks: merged and stored whole
#pragma unroll
            for (int i = 0; i < PG_KC; i++) {
                if (kq[i] == ~0u) continue;
                u128 acc = ka[i];
                if (!((kovf >> i) & 1u))
#pragma unroll
                    for (int h = 0; h < PG_HITS; h++)
                        if (kon[i][h]) acc = pg_merge16(acc, kd[i][h], kon[i][h] >> 8, kon[i][h] & 0xff);
                if (pg_ok(chk, DK + kq[i] + 16 <= KCAP, 11, s, DK + kq[i], KCAP)) __builtin_memcpy(dkp + kq[i], &acc, 16);
            }
#pragma unroll
            for (int i = 0; i < PG_VC; i++) {
                if (vq[i] == ~0u) continue;
                u128 acc = va[i];
                if (!((vovf >> i) & 1u))
#pragma unroll
                    for (int h = 0; h < PG_HITS; h++)
                        if (von[i][h]) acc = pg_merge16(acc, vd[i][h], von[i][h] >> 8, von[i][h] & 0xff);
                if (pg_ok(chk, DV + vq[i] + 16 <= VCAP, 12, s, DV + vq[i], VCAP)) __builtin_memcpy(dvp + vq[i], &acc, 16);
            }
            // ---- entry offsets: each to its piece's shift (an entry in no piece is a replaced one, dropped, or
            // in a moved page one before the first record, unshifted)
            uint32_t ed[PG_EC], ek[PG_EC], evv[PG_EC], ein = 0;
#pragma unroll
            for (int i = 0; i < PG_EC; i++) ed[i] = ek[i] = evv[i] = 0;
            for (uint32_t g = 0; g < gmax; g++) {
                const uint32_t g_gl = osh(glf, g), g_lo = osh(plo, g), g_hi = osh(phi, g), g_de = osh(sde, g), g_dk = osh(sdk, g),
                               g_dv = osh(sdv, g);
                if (!on || g >= nr || !g_gl) continue;
#pragma unroll
                for (int i = 0; i < PG_EC; i++)
                    if (ei[i] != ~0u && ei[i] >= g_lo && ei[i] < g_hi) { ed[i] = g_de; ek[i] = g_dk; evv[i] = g_dv; ein |= 1u << i; }
            }
#pragma unroll
            for (int i = 0; i < PG_EC; i++) {
                if (ei[i] == ~0u || (!((ein >> i) & 1u) && ei[i] >= U0)) continue;
                const uint64_t nidx = DE + ei[i] + ed[i];
                if (!pg_ok(chk, nidx < ECAP, 13, s, nidx, ECAP)) continue;
                if (md == 2 || ed[i] || ek[i]) p.koff[nidx] = DK + (eo[i] - KB) + (int64_t)(int32_t)ek[i];
                if (md == 2 || ed[i] || evv[i]) p.voff[nidx] = DV + (ev[i] - VB) + (int64_t)(int32_t)evv[i];
            }
        }
        if (on && ol == 0 && pg_ok(chk, DE + NC < ECAP && DK + NK <= KCAP && DV + NV <= VCAP, 15, s, DE + NC, ECAP)) {
            p.koff[DE + NC] = DK + NK;   // the end slot
            p.voff[DE + NC] = DV + NV;
            p.m.end[s] = DE + NC;
            p.m.vend[s] = DV + NV;
            if (md == 2) {
                p.m.beg[s] = DE;
                p.m.vbeg[s] = DV;
                p.m.ecap[s] = ECAP;
                p.m.kcap[s] = KCAP;
                p.m.vcap[s] = VCAP;
            }
        }
    }
}

// Segments whose runs have more than PG_GR records: one lane each
// (page_merge_lane: pieces and records), then the end slot and page metadata.
template <bool CHECK>
__global__ void k_page_wide(PageMergeArgs p) {
    const MergeArgs &a = p.a;
    for (uint64_t s = gtid(); s < a.S; s += gstride()) {
        const uint8_t md = p.mode[s];
        if (!md || a.bseg_off[s + 1] - a.bseg_off[s] <= PG_GR) continue;
        const uint64_t b = p.m.beg[s], C = p.m.end[s] - b;
        const SegSums X = p.ss[s];
        uint64_t DE = b, DK = p.koff[b], DV = p.voff[b];
        if (md == 2) {
            const PageSums R = p.rbase[s];
            DE = p.e0 + R.v[0]; DK = p.k0 + R.v[1]; DV = p.v0 + R.v[2];
        }
        page_merge_lane(p, s, md, b, C, DE, DK, DV);
        p.koff[DE + X.v[0]] = DK + X.v[1];   // the end slot
        p.voff[DE + X.v[0]] = DV + X.v[2];
        p.m.end[s] = DE + X.v[0];
        p.m.vend[s] = DV + X.v[2];
        if (md == 2) {
            const PageSums Z = p.rsz[s];
            p.m.beg[s] = DE;
            p.m.vbeg[s] = DV;
            p.m.ecap[s] = DE + Z.v[0];
            p.m.kcap[s] = DK + Z.v[1];
            p.m.vcap[s] = DV + Z.v[2];
        }
    }
}

// The records' entry offsets of every octet job (a thread per sorted batch
// record), after k_page_tails wrote their bytes and moved the pieces.  Runs
// of more than PG_GR records were written whole by page_merge_lane.
template <bool CHECK>
__global__ void k_page_records(PageMergeArgs p, uint64_t n) {
    const MergeArgs &a = p.a;
    unsigned long long *chk = CHECK ? p.chk : nullptr;
    for (uint64_t j = gtid(); j < n; j += gstride()) {
        const BatchSums &Bj = p.bx[j], &Bn = p.bx[j + 1];
        if (Bn.v[BS_NE] == Bj.v[BS_NE]) continue;        // no entry (not kept / erase)
        const uint64_t s = p.sseg[j];
        const uint8_t md = p.mode[s];
        if (!md) continue;
        const uint64_t j0 = a.bseg_off[s], je = a.bseg_off[s + 1];
        if (je - j0 > PG_GR) continue;
        const BatchSums &B0 = p.bx[j0];
        // the page after the merge: its first entry slot and byte bases
        const uint64_t DE = p.m.beg[s], DV = p.m.vbeg[s];
        const uint64_t DK = md == 2 ? p.k0 + p.rbase[s].v[1] : pg_kv0(p.kv0, s, 0);
        const RecAt R = p.rat[j];
        const uint64_t nwi = DE + p.pos[j] + (Bj.v[BS_NE] - B0.v[BS_NE]) - (Bj.v[BS_EQ] - B0.v[BS_EQ]);
        const uint64_t nk = DK + R.ku + (Bj.v[BS_KN] - B0.v[BS_KN]) - (Bj.v[BS_KE] - B0.v[BS_KE]);
        const uint64_t nv = DV + R.vu + (Bj.v[BS_VN] - B0.v[BS_VN]) - (Bj.v[BS_VE] - B0.v[BS_VE]);
        if (CHECK && !pg_ok(chk, nwi < p.m.end[s], 16, s, nwi, p.m.end[s])) continue;
        p.koff[nwi] = nk;
        p.voff[nwi] = nv;
    }
}

// k_merge_pos for streaming batches (no replace / erase flags), eight lanes
// (an OCTET) per segment: the records of the run in order, each placed by an
// 8-ary search over the segment's old keys (8 probes a round trip, from the
// previous record's position on) instead of one lane's binary search, so a
// record costs ~3 rounds of probes instead of ~7 dependent probes.  Same
// outputs as k_merge_pos.
__device__ __forceinline__ int pg_key_cmp(const MergeArgs &a, uint64_t e, const uint8_t *kb, uint64_t kl) {
    const uint64_t o = a.koff[e];
    return rec_cmp(a.kheap + o, a.koff[e + 1] - o, kb, kl);
}
__global__ void __launch_bounds__(256) k_merge_pos8(MergeArgs a, uint32_t *pos, BatchSums *bs, SegSums *ss, uint8_t *dirty,
                                                   RecAt *rat) {
    const uint32_t ol = threadIdx.x & 7;
    const uint32_t lane = threadIdx.x & 63, ob = lane & ~7u;
    const uint64_t o0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3, no = ((uint64_t)gridDim.x * blockDim.x) >> 3;
    const uint64_t iters = (a.S + no - 1) / no;
    for (uint64_t it = 0; it < iters; it++) {
        const uint64_t s = o0 + it * no;
        const bool on = s < a.S;
        uint64_t i0 = 0, nold = 0, j0 = 0, je = 0;
        bool rej = false;
        if (on) {
            i0 = a.seg_off[s]; nold = a.seg_end[s] - i0;
            j0 = a.bseg_off[s]; je = a.bseg_off[s + 1];
            rej = a.seg_reject && a.seg_reject[s];
        }
        const uint64_t k0 = on ? a.koff[i0] : 0, v0 = on ? a.voff[i0] : 0;   // an empty page has its end slot
        SegSums tot;
        tot.v[0] = nold;
        tot.v[1] = nold ? a.koff[i0 + nold] - k0 : 0;
        tot.v[2] = nold ? a.voff[i0 + nold] - v0 : 0;
        tot.v[3] = 0;
        uint32_t nrec = on ? (uint32_t)(je - j0) : 0u, rmax = nrec;
        for (int o = 32; o >= 1; o >>= 1) rmax = max(rmax, (uint32_t)__shfl_xor((int)rmax, o, 64));
        uint64_t lo = 0;
        bool changed = false;
        for (uint32_t q = 0; q < rmax; q++) {
            const bool act = q < nrec;
            const uint64_t j = j0 + q;
            uint32_t bi = 0;
            const uint8_t *kb = a.bv.kheap;
            uint64_t kl = 0;
            if (act) {
                bi = a.perm[j];
                kb = a.bv.kheap + a.bv.koff[bi];
                kl = a.bv.koff[bi + 1] - a.bv.koff[bi];
            }
            // 8-ary search for the first old key >= the record's, in [lo, nold)
            uint64_t L = lo, H = act && !rej ? nold : lo;
            for (;;) {
                const bool wide = H - L > 8;
                if (!__ballot(wide)) break;
                uint64_t pr = 0;
                bool less = false;
                if (wide) {
                    pr = L + (ol + 1) * (H - L) / 9;
                    less = pg_key_cmp(a, i0 + pr, kb, kl) < 0;
                }
                const uint32_t m = (uint32_t)(__ballot(less) >> ob) & 0xffu;   // probes below the key: a prefix of the 8
                const uint32_t cnt = __popc(m);
                const uint64_t plo = __shfl(pr, (int)(ob + (cnt ? cnt - 1 : 0)), 64), phi = __shfl(pr, (int)(ob + (cnt < 8 ? cnt : 7)), 64);
                if (wide) {
                    if (cnt) L = plo + 1;
                    if (cnt < 8) H = phi;
                }
            }
            // the last <= 8 candidates at once
            const bool cand = ol < H - L;
            const bool lt = cand && pg_key_cmp(a, i0 + L + ol, kb, kl) < 0;
            const uint64_t p = L + __popc((uint32_t)(__ballot(lt) >> ob) & 0xffu);
            if (act && !rej) {
                // lane 0 of the octet finishes the record: equality, its sums, its offsets
                if (ol == 0) {
                    const uint64_t e = i0 + p;
                    const bool eq = p < nold && pg_key_cmp(a, e, kb, kl) == 0;
                    pos[j] = (uint32_t)p;
                    rat[j] = RecAt{a.koff[e] - k0, a.voff[e] - v0, a.bv.koff[bi], a.bvoff[bi]};
                    BatchSums f(0);
                    const bool kept = a.keep[j] != 0;
                    if (kept && eq) {
                        f.v[BS_EQ] = 1;
                        f.v[BS_KE] = a.koff[e + 1] - a.koff[e];
                        f.v[BS_VE] = a.voff[e + 1] - a.voff[e];
                    }
                    if (kept) {
                        f.v[BS_NE] = 1;
                        f.v[BS_KN] = kl;
                        f.v[BS_VN] = a.bvoff[bi + 1] - a.bvoff[bi];
                    }
                    bs[j] = f;
                    changed |= kept;
                    if (kept && !eq) tot.v[3] += 1;
                    tot.v[0] += f.v[BS_NE] - f.v[BS_EQ];
                    tot.v[1] += f.v[BS_KN] - f.v[BS_KE];
                    tot.v[2] += f.v[BS_VN] - f.v[BS_VE];
                }
                lo = p;
            } else if (act && ol == 0) {
                pos[j] = 0;
                bs[j] = BatchSums(0);
            }
        }
        if (on && ol == 0) {
            ss[s] = tot;
            if (dirty) dirty[s] = changed ? 1 : 0;
        }
    }
}

// Checked build: every segment's page is consistent (entries and bytes
// inside its capacities, offsets nondecreasing, the view's value bounds).
__global__ void k_page_validate(PageMeta m, const uint64_t *koff, const uint64_t *voff, uint64_t S, uint64_t cap_e,
                                uint64_t cap_k, uint64_t cap_v, unsigned long long *chk) {
    for (uint64_t s = gtid(); s < S; s += gstride()) {
        const uint64_t b = m.beg[s], e = m.end[s];
        if (!pg_ok(chk, b <= e && e < m.ecap[s] && m.ecap[s] <= cap_e, 20, s, e, m.ecap[s])) continue;
        if (!pg_ok(chk, koff[b] <= koff[e] && koff[e] <= m.kcap[s] && m.kcap[s] <= cap_k, 21, s, koff[e], m.kcap[s])) continue;
        if (!pg_ok(chk, voff[b] <= voff[e] && voff[e] <= m.vcap[s] && m.vcap[s] <= cap_v, 22, s, voff[e], m.vcap[s])) continue;
        if (!pg_ok(chk, m.vbeg[s] == voff[b] && m.vend[s] == voff[e], 23, s, m.vbeg[s], voff[b])) continue;
        for (uint64_t i = b; i < e; i++)
            if (!pg_ok(chk, koff[i] <= koff[i + 1] && voff[i] <= voff[i + 1], 24, s, i, b)) {
                if (chk[2] == s && chk[3] == i)   // the first violation: the page's offsets for the report
                    for (uint64_t q = 0; q < 12 && b + q <= e; q++) { chk[5 + q] = koff[b + q]; chk[17 + q] = voff[b + q]; }
                break;
            }
    }
}
