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
// bytes [vbeg[s] = voff[beg], vend[s] = voff[end]) below vcap[s]; kbeg[s] =
// koff[beg] (the page's first key byte: the per-segment kernels read the
// page bounds from these S-wide arrays, consecutive segments side by side,
// not from the entry slots a page apart).  With st_debug_knob
// ST_DBG_PAGE_DOWN a page's slack is split: half after its content, half
// before it (ebot <= beg, kbot <= kbeg, vbot <= vbeg), and a batch that
// inserts into a page may shift the entries before its last insert position
// down into the head slack (mode 3) instead of those after its first one up
// into the tail slack (mode 1) -- half the moved bytes for an insert at a
// uniform position.  Off by default: measured slower, because a page shifted
// down no longer starts its values 16-byte aligned and every MD5 block of
// its verify and hash is then an unaligned read.  Without
// it ebot = beg etc. and every merge shifts up.
//
// UNIFORM pages: when every key record of a segment has one length L (klen)
// and every value one length V (vlen) -- int64 keys and 17-byte ObjHash
// values always do (riak_ensemble_peer.erl:1717-1724) -- entry i's offsets
// are koff[beg] + L i and voff[beg] + V i, and a page keeps only its first
// and end slots (page_uniform): a batch then moves key and value bytes, not
// the two 8-byte offset arrays (16 of the 42 bytes an entry moves).  A batch
// that puts a record of another length into a uniform page first writes
// every offset of that page (k_page_materialize), and the page keeps them
// from then on.
#pragma once

struct PageMeta {
    uint64_t *beg, *end, *vbeg, *vend;   // S each: the DevTree view's seg_off / seg_end / seg_voff / seg_vend
    uint64_t *kbeg;                      // S: koff[beg]
    uint64_t *ecap, *kcap, *vcap;        // S each: page capacities (entry slot end, key / value byte ends)
    uint64_t *ebot, *kbot, *vbot;        // S each: the page's first entry slot and key / value bytes (its content
                                         // starts at or above them: the head slack a merge may shift down into)
    uint16_t *klen;                      // S: the length every key record of the segment has (KLEN_MIXED: not
                                         // one length, KLEN_NONE: no entries) -- fixed-stride merge positions
    uint16_t *vlen;                      // S: the same for its values
};
#define KLEN_MIXED KLEN_MIXED_   // st_kernels.h
#define KLEN_NONE KLEN_NONE_
// the uniform key length of a segment after adding records of length l
__device__ __forceinline__ uint32_t klen_add(uint32_t cur, uint64_t l) {
    if (l == 0 || l >= KLEN_NONE) return KLEN_MIXED;
    return cur == KLEN_NONE ? (uint32_t)l : (cur == l ? cur : KLEN_MIXED);
}

// A page whose entry offsets are implicit (only its first and end slots kept)
__device__ __forceinline__ bool page_uniform(uint32_t kl, uint32_t vl) { return kl != KLEN_MIXED && vl != KLEN_MIXED; }

typedef USum<4> PageSums;   // entries, key bytes, value bytes (+ a spare)
typedef USum<5> PlanSums;   // k_run_plan: a moved segment's new page (entries, key bytes, value bytes), new keys,
                            // the touched segment's value bytes before the merge

// Page capacity for a segment of c entries, kb key bytes and vb value bytes
// (slack_pct: percent of slack; < 0: none, a gap-free CSR).  Byte caps are
// 16-byte multiples so every page starts 16-byte aligned.
__host__ __device__ __forceinline__ PageSums page_slack(uint64_t c, uint64_t kb, uint64_t vb, int slack_pct) {
    PageSums r(0);
    r.v[0] = c ? (c * (uint64_t)slack_pct / 100 > 4 ? c * (uint64_t)slack_pct / 100 : 4) : 0;
    r.v[1] = c ? (kb * (uint64_t)slack_pct / 100 > 32 ? kb * (uint64_t)slack_pct / 100 : 32) : 0;
    r.v[2] = c ? (vb * (uint64_t)slack_pct / 100 > 48 ? vb * (uint64_t)slack_pct / 100 : 48) : 0;
    return r;
}
__host__ __device__ __forceinline__ PageSums page_caps(uint64_t c, uint64_t kb, uint64_t vb, int slack_pct) {
    PageSums r(0);
    if (slack_pct < 0) {
        r.v[0] = c; r.v[1] = kb; r.v[2] = vb;   // canonical: the next segment's first entry is this one's end
        return r;
    }
    const PageSums x = page_slack(c, kb, vb, slack_pct);
    r.v[0] = c + 1 + x.v[0];
    r.v[1] = (kb + x.v[1] + 15) & ~15ull;
    r.v[2] = (vb + x.v[2] + 15) & ~15ull;
    return r;
}
// The head of such a page (before its content): half its slack (bytes in
// 16-byte units, so the content starts 16-byte aligned where the page does).
__host__ __device__ __forceinline__ PageSums page_head(uint64_t c, uint64_t kb, uint64_t vb, int slack_pct) {
    PageSums r(0);
    if (slack_pct < 0) return r;
    const PageSums x = page_slack(c, kb, vb, slack_pct);
    r.v[0] = x.v[0] / 2;
    r.v[1] = (x.v[1] / 2) & ~15ull;
    r.v[2] = (x.v[2] / 2) & ~15ull;
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
    int slack_pct;                   // paged destination: the pages' slack (page_head)
};
// sm: the source's page metadata when the source is paged (its uniform pages
// keep no per-entry offsets: generated here), else nullptr (a CSR).
__global__ void __launch_bounds__(256) k_page_copy(DevTree t, const PageSums *base, const PageSums *sz, PageDst d,
                                                   const uint16_t *sklen, const uint16_t *svlen) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t s = w0; s < t.S; s += nw) {
        const uint64_t b = t.seg_off[s], e = t.seg_end[s], c = e - b;
        const PageSums B = base[s];
        const uint64_t kb0 = t.koff[b], vb0 = t.voff[b];
        const PageSums Hd = d.m.beg ? page_head(c, t.koff[e] - kb0, t.voff[e] - vb0, d.slack_pct) : PageSums(0);
        const uint64_t De = d.e0 + B.v[0] + Hd.v[0], Dk = d.k0 + B.v[1] + Hd.v[1], Dv = d.v0 + B.v[2] + Hd.v[2];
        const uint32_t SL = sklen ? sklen[s] : KLEN_MIXED, SV = svlen ? svlen[s] : KLEN_MIXED;
        const bool gen = sklen && page_uniform(SL, SV) && c;   // a uniform source page: offsets by stride
        const uint64_t l0 = c ? (gen ? SL : t.koff[b + 1] - kb0) : 0;
        const uint64_t w0v = c ? (gen ? SV : t.voff[b + 1] - vb0) : 0;
        bool mixed = false, mixedv = false;
        for (uint64_t i = lane; i <= c; i += 64) {   // offsets incl. the end slot
            const uint64_t ko = gen ? kb0 + SL * i : t.koff[b + i];
            const uint64_t vo = gen ? vb0 + SV * i : t.voff[b + i];
            d.koff[De + i] = Dk + (ko - kb0);
            d.voff[De + i] = Dv + (vo - vb0);
            if (i < c && !gen) {
                mixed |= t.koff[b + i + 1] - ko != l0;
                mixedv |= t.voff[b + i + 1] - vo != w0v;
            }
        }
        const bool any_mixed = __ballot(mixed) != 0, any_mixedv = __ballot(mixedv) != 0;
        wave_copy_gg(d.kheap + Dk, t.kheap + kb0, t.koff[e] - kb0);
        wave_copy_gg(d.vheap + Dv, t.vheap + vb0, t.voff[e] - vb0);
        if (lane == 0) {
            if (d.m.beg) {
                const PageSums Z = sz[s];
                d.m.klen[s] = (uint16_t)(c == 0 ? KLEN_NONE : any_mixed ? KLEN_MIXED : klen_add(KLEN_NONE, l0));
                d.m.vlen[s] = (uint16_t)(c == 0 ? KLEN_NONE : any_mixedv ? KLEN_MIXED : klen_add(KLEN_NONE, w0v));
                d.m.beg[s] = De;
                d.m.end[s] = De + c;
                d.m.vbeg[s] = Dv;
                d.m.kbeg[s] = Dk;
                d.m.vend[s] = Dv + (t.voff[e] - vb0);
                d.m.ebot[s] = De - Hd.v[0];
                d.m.kbot[s] = Dk - Hd.v[1];
                d.m.vbot[s] = Dv - Hd.v[2];
                d.m.ecap[s] = d.m.ebot[s] + Z.v[0];
                d.m.kcap[s] = d.m.kbot[s] + Z.v[1];
                d.m.vcap[s] = d.m.vbot[s] + Z.v[2];
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

// A uniform page a batch turns mixed (k_run_plan mode bit 8): every entry's
// offsets written from the stride before the merge moves them.  A wave per
// such segment (rare: only a record of another length meets a uniform page).
__global__ void __launch_bounds__(256) k_page_materialize(PageMeta m, uint64_t *koff, uint64_t *voff, const uint8_t *mode,
                                                          const uint8_t *reject, uint64_t S) {
    const uint32_t lane = threadIdx.x & 63;
    // (a batch without room in the append region is merged only after a page
    // build; materialising first is harmless: a uniform page's offsets written out)
    const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t s0 = w0 * 64; s0 < S; s0 += nw * 64) {
        const uint64_t mine = s0 + lane;
        uint64_t todo = __ballot(mine < S && (mode[mine] & 8) && !(reject && reject[mine]));
        while (todo) {
            const uint32_t j = (uint32_t)__builtin_ctzll(todo);
            todo &= todo - 1;
            const uint64_t s = s0 + j;
            const uint64_t b = m.beg[s], c = m.end[s] - b;
            const uint64_t L = m.klen[s], V = m.vlen[s], K0 = koff[b], V0 = voff[b];
            for (uint64_t i = lane; i <= c; i += 64) {
                koff[b + i] = K0 + L * i;
                voff[b + i] = V0 + V * i;
            }
        }
    }
}

// The runs' sums and the pages' plan in one pass: the lane of each run's
// first record sums the run (its BatchSums' inclusive prefix sums into bxl
// -- k_page_merge's growth before and through each group --, the segment's
// size deltas, dirty, fpos = the smallest value offset a kept record
// changes) and plans its page: merge in place shifting up (1) or down (3),
// or move to a new page (2) -- in place up needs room after the content and
// every prefix of the run adding >= 0 key and value bytes (the moves run
// from the highest address down), in place down room before the content and
// every suffix adding >= 0 (the moves run from the lowest address up); with
// both possible the side with fewer bytes to move wins (down: 0 never, 1 by
// the bytes, 2 whenever it fits) --,
// reloc = the new page's sizes (mode 2, scanned for its place in the append
// region, k_page_place), v[3] its new keys, v[4] its value bytes before the
// merge; mode bit 4: the merged page keeps per-entry offsets (not uniform),
// bit 8: a uniform page turning mixed (k_page_materialize first).  No pass
// over all S segments.  Runs before the verify: k_page_place drops a rejected
// segment's plan and writes mode / dirty 0 for the segments without a run.
__global__ void k_run_plan(const uint32_t *sseg, const uint64_t *bseg_off, uint64_t n, const BatchSums *bs,
                           const RecAt *rat, PageMeta m, const uint64_t *koff, const uint64_t *voff, int slack_pct,
                           uint8_t *dirty, unsigned long long *fpos, BatchSums *bxl, SegSums *sm, uint8_t *mode,
                           PlanSums *reloc, int down) {
    for (uint64_t j = gtid(); j < n; j += gstride()) {
        const uint64_t s = sseg[j];
        if (j != bseg_off[s]) continue;
        const uint64_t je = bseg_off[s + 1];
        SegSums d(0);
        BatchSums acc(0);
        uint64_t fp = ~0ull;
        bool grow = true;
        int64_t dk = 0, dv = 0, mk = 0, mv = 0;   // the growth so far and its largest prefix
        uint64_t up_cost = ~0ull, down_cost = 0;   // bytes after the first / before the last shifting record's position
        const uint32_t kl0 = m.klen[s], vl0 = m.vlen[s];
        uint32_t kl = kl0, vl = vl0;
        for (uint64_t r = j; r < je; r++) {
            const BatchSums f = bs[r];
            acc = acc + f;
            bxl[r] = acc;
            dk += (int64_t)f.v[BS_KN] - (int64_t)f.v[BS_KE];
            dv += (int64_t)f.v[BS_VN] - (int64_t)f.v[BS_VE];
            grow = grow && dk >= 0 && dv >= 0;
            mk = dk > mk ? dk : mk;
            mv = dv > mv ? dv : mv;
            if (f.v[BS_NE] != f.v[BS_EQ] || f.v[BS_KN] != f.v[BS_KE] || f.v[BS_VN] != f.v[BS_VE]) {
                const RecAt q = rat[r];   // the run is in key order: positions ascend
                if (up_cost == ~0ull) up_cost = q.ku + q.vu;   // (made relative to the page's end below)
                down_cost = q.ku + q.vu;
            }
            if (f.v[BS_NE]) { kl = klen_add(kl, f.v[BS_KN]); vl = klen_add(vl, f.v[BS_VN]); }
            if (!f.v[BS_NE] && !f.v[BS_EQ]) continue;
            d.v[0] += f.v[BS_NE] - f.v[BS_EQ];
            d.v[1] += f.v[BS_KN] - f.v[BS_KE];
            d.v[2] += f.v[BS_VN] - f.v[BS_VE];
            d.v[3] += (f.v[BS_NE] && !f.v[BS_EQ]) ? 1 : 0;
            fp = std::min<uint64_t>(fp, rat[r].vu);
        }
        if (fp == ~0ull) {   // no kept record: nothing to merge (no memsets before: every run's segment is written)
            dirty[s] = 0;
            fpos[s] = ~0ull;
            mode[s] = 0;
            continue;
        }
        dirty[s] = 1;
        fpos[s] = fp;
        // the page's bounds from the S-wide arrays (a uniform page's key bytes by stride)
        const uint64_t b = m.beg[s], e = m.end[s], kb = m.kbeg[s], vb = m.vbeg[s], ve = m.vend[s];
        const uint64_t kbytes = e == b ? 0 : (page_uniform(kl0, vl0) ? (uint64_t)kl0 * (e - b) : koff[e] - kb);
        SegSums x;
        x.v[0] = (e - b) + d.v[0];
        x.v[1] = kbytes + d.v[1];
        x.v[2] = (ve - vb) + d.v[2];
        x.v[3] = d.v[3];
        sm[s] = x;
        const bool fits = b + x.v[0] < m.ecap[s] && kb + x.v[1] <= m.kcap[s] && vb + x.v[2] <= m.vcap[s];
        // down: the growth fits before the content and no suffix of the run shrinks
        const bool dfits = down && dk >= 0 && dv >= 0 && mk <= dk && mv <= dv && b - m.ebot[s] >= d.v[0] &&
                           kb - m.kbot[s] >= (uint64_t)dk && vb - m.vbot[s] >= (uint64_t)dv;
        up_cost = up_cost == ~0ull ? 0 : kbytes + (ve - vb) - up_cost;
        uint8_t md = fits && grow ? 1 : 2;
        if (dfits && (md == 2 || down == 2 || down_cost < up_cost)) md = 3;
        const bool expl = !page_uniform(kl, vl);
        md |= (expl ? 4 : 0) | (expl && page_uniform(kl0, vl0) && e > b ? 8 : 0);
        PlanSums r(0);
        if ((md & 3) == 2) {
            const PageSums c = page_caps(x.v[0], x.v[1], x.v[2], slack_pct < 0 ? 0 : slack_pct);
            r.v[0] = c.v[0]; r.v[1] = c.v[1]; r.v[2] = c.v[2];
        }
        r.v[3] = x.v[3];
        r.v[4] = ve - vb;
        mode[s] = md;
        reloc[s] = r;
    }
}

// The plan settled after the verify, a lane per segment (S-wide): the path
// status of every segment with a run (k_path_status: the first level whose
// node failed; a rejected segment's plan is dropped -- no merge, no rehash,
// no new keys counted), mode / dirty 0 for the segments without one, and
// every moved page's place in the append region: a workgroup scan of the
// moved pages' sizes and one atomic per workgroup and quantity (the order of
// the places across workgroups is the atomics' order: the layout may differ
// from run to run, the content does not).  acc (zeroed by the caller), at
// q * PP_LINE for q = 0..4: the moves' entries / key bytes / value bytes, the
// batch's new keys, the touched segments' value bytes before the merge.  No scan over S, and
// the host reads the totals once, at the end of the batch: a batch whose moves
// do not fit the append region is not merged (page_room below) and the host
// rebuilds the pages and merges it again.
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x, uint32_t lane) {
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    return x;
}
//
// It also lists the segments the batch changes for the dirty-path hash, by
// the MD5 blocks each has left after its verified prefix (PrefixState.k, the
// merged value bytes sm[s].v[2]): HB bins, longest first, bin b's entries at
// hlist[b * hcap ...], counted in hcnt[b * PP_LINE] -- a list in block-count
// order without a pass of its own (k_segment_hash_perm, HashBins).
#define PP_ITER 4    // segments per thread: a workgroup owns 1024 consecutive segments, one atomic per quantity
#define PP_LINE 16   // acc quantities a 128-byte line apart (no two atomics' addresses share a line)
#define HB 64        // hash-list bins: blocks left 63+, 62, ..., 0
__device__ __forceinline__ uint32_t hb_bin(uint64_t vbytes, uint64_t k) {
    const uint64_t rem = (vbytes + 8) / 64 + 1 - k;
    return rem >= HB - 1 ? 0u : (uint32_t)(HB - 1 - rem);
}
__global__ void __launch_bounds__(256) k_page_place(DevTree t, const uint64_t *bseg_off, const uint8_t *ok,
                                                    uint8_t *reject, uint8_t *mode, uint8_t *dirty, const PlanSums *rsz,
                                                    PlanSums *rbase, unsigned long long *acc, const PrefixState *ps,
                                                    const SegSums *sm, uint32_t *hlist, uint64_t hcap,
                                                    unsigned long long *hcnt) {
    __shared__ uint64_t wt[PP_ITER][4][3], wr[4][2], base[3];
    __shared__ uint32_t hh[HB], hbase[HB];
    if (threadIdx.x < HB) hh[threadIdx.x] = 0;
    __syncthreads();
    uint32_t hbin[PP_ITER], hrank[PP_ITER];
    const uint32_t L = t.H + 1, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint64_t s0 = (uint64_t)blockIdx.x * 256 * PP_ITER;
    uint64_t c[PP_ITER][3], x[PP_ITER][3], r3 = 0, r4 = 0;
#pragma unroll
    for (int it = 0; it < PP_ITER; it++) {
        const uint64_t s = s0 + (uint64_t)it * 256 + tid;
        c[it][0] = c[it][1] = c[it][2] = 0;
        hbin[it] = HB;
        if (s < t.S) {
            if (bseg_off[s] == bseg_off[s + 1]) {
                reject[s] = 0; mode[s] = 0; dirty[s] = 0;
            } else {
                uint32_t bad = 0;
                for (uint32_t l = 1; l <= L; l++)
                    if (!ok[t.base[l] + (s >> (t.shift * (L - l)))]) { bad = l; break; }
                reject[s] = (uint8_t)bad;
                const uint8_t md = mode[s];
                if (bad) {
                    mode[s] = 0; dirty[s] = 0;
                } else if (md) {
                    const PlanSums z = rsz[s];
                    if ((md & 3) == 2) { c[it][0] = z.v[0]; c[it][1] = z.v[1]; c[it][2] = z.v[2]; }
                    r3 += z.v[3]; r4 += z.v[4];
                    hbin[it] = hb_bin(sm[s].v[2], ps[s].k);
                    hrank[it] = atomicAdd(&hh[hbin[it]], 1u);
                }
            }
        }
#pragma unroll
        for (int q = 0; q < 3; q++) {
            x[it][q] = wave_incl_scan(c[it][q], lane);
            if (lane == 63) wt[it][w][q] = x[it][q];
        }
    }
    for (int o = 32; o > 0; o >>= 1) { r3 += __shfl_xor(r3, o); r4 += __shfl_xor(r4, o); }
    if (lane == 0) { wr[w][0] = r3; wr[w][1] = r4; }
    __syncthreads();
    if (tid < 5) {   // one atomic per quantity and workgroup, each on its own line
        uint64_t tot = 0;
        for (int v = 0; v < 4; v++) {
            if (tid < 3)
                for (int it = 0; it < PP_ITER; it++) tot += wt[it][v][tid];
            else
                tot += wr[v][tid - 3];
        }
        const uint64_t b0 = tot ? atomicAdd(&acc[tid * PP_LINE], (unsigned long long)tot) : 0;
        if (tid < 3) base[tid] = b0;
    }
    if (tid < HB) hbase[tid] = hh[tid] ? (uint32_t)atomicAdd(&hcnt[tid * PP_LINE], (unsigned long long)hh[tid]) : 0u;
    __syncthreads();
    uint64_t run[3] = {base[0], base[1], base[2]};
#pragma unroll
    for (int it = 0; it < PP_ITER; it++) {
        const uint64_t s = s0 + (uint64_t)it * 256 + tid;
        uint64_t before[3];
#pragma unroll
        for (int q = 0; q < 3; q++) {
            before[q] = run[q] + x[it][q] - c[it][q];
            for (uint32_t v = 0; v < 4; v++) {
                if (v < w) before[q] += wt[it][v][q];
                run[q] += wt[it][v][q];
            }
        }
        if (hbin[it] < HB) hlist[hbin[it] * hcap + hbase[hbin[it]] + hrank[it]] = (uint32_t)s;
        if (s < t.S && (c[it][0] | c[it][1] | c[it][2])) {   // a moved page (its caps are never all zero)
            PlanSums R(0);
            R.v[0] = before[0]; R.v[1] = before[1]; R.v[2] = before[2];
            rbase[s] = R;
        }
    }
}
// the batch's moves fit the append region (the host's check after the batch is the same)
__device__ __forceinline__ bool page_room(const unsigned long long *acc, uint64_t e0, uint64_t k0, uint64_t v0,
                                          uint64_t ce, uint64_t ck, uint64_t cv) {
    return e0 + acc[0] + 1 <= ce && k0 + acc[PP_LINE] <= ck && v0 + acc[2 * PP_LINE] <= cv;
}

// The merge of one batch run into its segment's page (mode 1, in place) or
// into a new page (mode 2): the closed form of k_merge_old / k_merge_new
// (st_kernels.h) per segment, a lane per segment.  The run's records with
// one position u form a GROUP; after group g the old entries [u_g (+1 if its
// last record replaces entry u_g), u_{g+1}) -- a PIECE -- keep their order
// and shift by the running sums through the group (entries +NE-EQ, key bytes
// +KN-KE, value bytes +VN-VE).  The groups are visited from the last to the
// first; each piece moves highest address first (in place every shift is >=
// 0, k_run_plan, so no source is overwritten before it is read), then the
// group's records are written into the gap.
struct PageMergeArgs {
    MergeArgs a;
    PageMeta m;
    uint64_t *koff, *voff;        // the page arrays (a.koff / a.voff, writable)
    uint8_t *kheap, *vheap;
    const uint32_t *pos;
    const RecAt *rat;             // per record: old offsets at its position (page-relative), its batch offsets
    const BatchSums *bx;          // per run: inclusive prefix sums of its records' BatchSums (k_run_plan)
    const SegSums *ss;            // per segment: merged count, key bytes, value bytes
    const uint8_t *mode;
    const PlanSums *rbase;        // the moved pages' places (k_page_place)
    const PlanSums *rsz;          // the relocation sizes
    uint64_t e0, k0, v0;          // the append region's bases
    uint64_t ce, ck, cv;          // ... and its ends
    const unsigned long long *acc;   // the batch's totals (k_page_place): no room, no merge
    int slack_pct;                // the pages' slack (a moved page's head, page_head)
    unsigned long long *chk;      // checked build (st_debug_knob ST_DBG_PAGE_CHECK): [0] violations, [1..4] the first
};

// Checked build: a store outside its page is counted and skipped, and the
// first one recorded (code, segment, address, bound), instead of faulting.
__device__ __forceinline__ bool pg_ok(unsigned long long *chk, bool ok, uint32_t code, uint64_t s, uint64_t x, uint64_t bound) {
    if (ok || !chk) return true;
    if (atomicAdd(&chk[0], 1ull) == 0) { chk[1] = code; chk[2] = s; chk[3] = x; chk[4] = bound; }
    return false;
}

// A piece job: key bytes, value bytes, key offsets, value offsets
struct PieceJob {
    uint64_t kd, ks, nk, vd, vs, nv, ko, vo, a, e, de, dk, dv, fl;   // fl: bit 0 keys, 1 values, 2 key offs, 3 value offs
};
#define PM_ASC 16u   // PieceJob::fl: the piece moves down (dst <= src): its units run bottom up
// The jobs' memory accesses.  A job's addresses are rebuilt from readlanes,
// so the compiler cannot tell their address space: as generic pointers every
// access was a FLAT one, and the waits FLAT needs serialised a unit's loads
// one behind the other and each behind the previous stores.  Buffer
// accesses through a job's (wave-uniform) bases, every lane issuing every
// access: a lane with nothing to move gets an offset past the buffer's range
// (loads return 0, stores are dropped), so a unit is four loads, one wait and
// four stores, with no branch (and no wait) between them.
typedef uint32_t pm_u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t pm_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) uint8_t g_u8;
#define PM_OOB 0x80000000u   // past every job buffer's range (0x7fffffff bytes)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pm_rsrc(uint64_t base) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, 0x7fffffff, 0x00020000);
}

// Wave-cooperative piece moves (every lane of the wave, a wave-uniform job):
// every lane's job (has = this lane has one), one after another by the whole
// wave.  A job's four arrays (key bytes, value bytes, key offsets, value
// offsets) advance together, unit by unit -- 64 lanes x 16 bytes of each heap
// and 64 entries of each offset array -- top down (dst >= src, or disjoint).
// The lowest chunk of a piece clamps to its first 16 bytes (the bytes it
// shares with the chunk above get the same values twice, both loaded in that
// unit); fewer than 16 bytes left below the last full unit form a byte unit
// of their own (a lane a byte: a clamped chunk would read bytes the unit
// above already rewrote).  The units run as one sequence across the wave's
// jobs (a unit's four loads and two byte loads, then its stores; PM_PIPE
// issues the next unit's loads before them -- no unit reads what the unit
// before it writes: moves go up, a piece's units top down, and different
// jobs are different segments).  A wave's loads touch 8-9 lines, where a
// lane per segment moving its own bytes touched 64: 1.43 against 1.75 ms a
// config-5 batch.
__device__ __forceinline__ uint64_t rl64(uint64_t x, uint32_t l) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)x, l), hi = __builtin_amdgcn_readlane((uint32_t)(x >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t bunits(uint64_t n) { return n >= 16 ? (n - 16) / 1024 + 1 : 0; }
struct PmJob {   // a job's wave-uniform registers
    __amdgpu_buffer_rsrc_t KS, KD, VS, VD, KO, VO, KOD, VOD;
    uint64_t nk, nv, a, e, dk, dv, units, fl;
};
struct PmUnit {   // one unit's offsets (PM_OOB: nothing) and loaded data
    uint32_t kc, vc, kt, vt, ok, ov;
    pm_u32x4 kx, vx;
    pm_u32x2 ox, px;
    uint32_t kb, vb;
};
__device__ __forceinline__ bool pm_next_job(uint64_t &jm, const PieceJob &J, PmJob &q) {
    if (!jm) return false;
    const uint32_t L = (uint32_t)__builtin_ctzll(jm);
    jm &= jm - 1;
    q.fl = rl64(J.fl, L);
    q.nk = (q.fl & 1) ? rl64(J.nk, L) : 0;
    q.nv = (q.fl & 2) ? rl64(J.nv, L) : 0;
    q.a = rl64(J.a, L);
    q.e = (q.fl & 12) ? rl64(J.e, L) : q.a;
    q.dk = rl64(J.dk, L);
    q.dv = rl64(J.dv, L);
    const uint64_t de = rl64(J.de, L), ko = rl64(J.ko, L), vo = rl64(J.vo, L);
    q.KS = pm_rsrc(rl64(J.ks, L)); q.KD = pm_rsrc(rl64(J.kd, L));
    q.VS = pm_rsrc(rl64(J.vs, L)); q.VD = pm_rsrc(rl64(J.vd, L));
    q.KO = pm_rsrc(ko); q.VO = pm_rsrc(vo); q.KOD = pm_rsrc(ko + 8 * de); q.VOD = pm_rsrc(vo + 8 * de);
    const uint64_t uk = bunits(q.nk) + (q.nk > 1024 * bunits(q.nk) ? 1 : 0);   // + the byte unit
    const uint64_t uv = bunits(q.nv) + (q.nv > 1024 * bunits(q.nv) ? 1 : 0);
    q.units = std::max(std::max(uk, uv), (q.e - q.a + 63) / 64);
    return true;
}
// unit u's offsets for one heap of n bytes: a 16-byte chunk (c) or a byte (t)
__device__ __forceinline__ void pm_heap_offs(uint64_t n, uint64_t u, uint32_t lane, uint32_t &c, uint32_t &t) {
    const uint64_t U = bunits(n);
    c = t = PM_OOB;
    if (u < U) {
        const int64_t h = (int64_t)n - 1024 * (int64_t)u - 16 * (int64_t)lane;
        if (h > 0) c = h >= 16 ? (uint32_t)(h - 16) : 0u;
    } else if (u == U && n > 1024 * U && lane < n - 1024 * U) {   // the byte unit (fewer than 16 bytes left)
        t = lane;
    }
}
// A piece moving down (PM_ASC) takes the mirror image of the same units:
// byte x of the top-down order is byte n - 1 - x, entry i is entry a + e - 1 - i,
// so unit u covers the lowest bytes and entries not yet moved, the clamped
// chunk is the top one and the byte unit holds the top bytes.
__device__ __forceinline__ void pm_load(const PmJob &q, uint64_t u, uint32_t lane, PmUnit &d) {
    pm_heap_offs(q.nk, u, lane, d.kc, d.kt);
    pm_heap_offs(q.nv, u, lane, d.vc, d.vt);
    const uint64_t top = q.e - std::min(q.e - q.a, 64 * u);
    uint32_t oo = top > q.a + lane ? (uint32_t)(8 * (top - 1 - lane)) : PM_OOB;
    if (q.fl & PM_ASC) {
        if (d.kc != PM_OOB) d.kc = (uint32_t)q.nk - 16 - d.kc;
        if (d.vc != PM_OOB) d.vc = (uint32_t)q.nv - 16 - d.vc;
        if (d.kt != PM_OOB) d.kt = (uint32_t)q.nk - 1 - d.kt;
        if (d.vt != PM_OOB) d.vt = (uint32_t)q.nv - 1 - d.vt;
        if (oo != PM_OOB) oo = (uint32_t)(8 * (q.a + q.e - 1)) - oo;
    }
    d.ok = (q.fl & 4) ? oo : PM_OOB;
    d.ov = (q.fl & 8) ? oo : PM_OOB;
    d.kx = __builtin_amdgcn_raw_buffer_load_b128(q.KS, d.kc, 0, 0);
    d.vx = __builtin_amdgcn_raw_buffer_load_b128(q.VS, d.vc, 0, 0);
    d.ox = __builtin_amdgcn_raw_buffer_load_b64(q.KO, d.ok, 0, 0);
    d.px = __builtin_amdgcn_raw_buffer_load_b64(q.VO, d.ov, 0, 0);
    d.kb = __builtin_amdgcn_raw_buffer_load_b8(q.KS, d.kt, 0, 0);
    d.vb = __builtin_amdgcn_raw_buffer_load_b8(q.VS, d.vt, 0, 0);
}
__device__ __forceinline__ void pm_store(const PmJob &q, const PmUnit &d) {
    const uint64_t o1 = (((uint64_t)d.ox.y << 32) | d.ox.x) + q.dk, p1 = (((uint64_t)d.px.y << 32) | d.px.x) + q.dv;
    __builtin_amdgcn_raw_buffer_store_b128(d.kx, q.KD, d.kc, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(d.vx, q.VD, d.vc, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b64(pm_u32x2{(uint32_t)o1, (uint32_t)(o1 >> 32)}, q.KOD, d.ok, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b64(pm_u32x2{(uint32_t)p1, (uint32_t)(p1 >> 32)}, q.VOD, d.ov, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)d.kb, q.KD, d.kt, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)d.vb, q.VD, d.vt, 0, 0);
}
// PM_PIPE 1: the next unit's loads before the current unit's stores (two
// units in flight).  Slower: 1.11 against 1.02 ms a config-5 batch (the
// second unit's registers spill more at 5 waves per SIMD).
#ifndef PM_PIPE
#define PM_PIPE 0
#endif
__device__ __forceinline__ void wave_run_jobs(const PieceJob &J, bool has, uint32_t lane) {
    uint64_t jm = __ballot(has);
    PmJob A, B;
    PmUnit DA, DB;
    uint64_t uA = 0, uB = 0;
    bool hA = pm_next_job(jm, J, A);
    if (hA) pm_load(A, 0, lane, DA);
    while (hA) {
        bool hB = true;
        if (uA + 1 < A.units) {
            B = A;
            uB = uA + 1;
        } else {
            hB = pm_next_job(jm, J, B);
            uB = 0;
            if (!hB) { B = A; uB = A.units; }   // past every array: loads of nothing (no branch, no join wait)
        }
        if (PM_PIPE) {
            pm_load(B, uB, lane, DB);
            pm_store(A, DA);
        } else {
            pm_store(A, DA);
            pm_load(B, uB, lane, DB);
        }
        A = B; DA = DB; uA = uB; hA = hB;
    }
}

// A record's key and value bytes into the page (sources in the batch, never
// overlapping their destinations): up to 32 bytes each in at most two
// (overlapping) loads, all four loads before any store -- one round trip
// where copy_bytes' load/store pairs took one each.  Longer: copy_bytes.
__device__ __forceinline__ void small_load(const uint8_t *s, uint64_t n, uint4 &a, uint4 &b) {
    if (n >= 16) {
        __builtin_memcpy(&a, s, 16);
        __builtin_memcpy(&b, s + n - 16, 16);
    } else if (n >= 8) {
        __builtin_memcpy(&a, s, 8);
        __builtin_memcpy(&b, s + n - 8, 8);
    } else if (n >= 4) {
        __builtin_memcpy(&a, s, 4);
        __builtin_memcpy(&b, s + n - 4, 4);
    } else if (n) {
        a.x = s[0]; a.y = s[n >> 1]; b.x = s[n - 1];
    }
}
__device__ __forceinline__ void small_store(uint8_t *d, uint64_t n, const uint4 &a, const uint4 &b) {
    if (n >= 16) {
        __builtin_memcpy(d, &a, 16);
        __builtin_memcpy(d + n - 16, &b, 16);
    } else if (n >= 8) {
        __builtin_memcpy(d, &a, 8);
        __builtin_memcpy(d + n - 8, &b, 8);
    } else if (n >= 4) {
        __builtin_memcpy(d, &a, 4);
        __builtin_memcpy(d + n - 4, &b, 4);
    } else if (n) {
        d[0] = (uint8_t)a.x; d[n >> 1] = (uint8_t)a.y; d[n - 1] = (uint8_t)b.x;
    }
}
__device__ __forceinline__ void copy2_disjoint(uint8_t *d1, const uint8_t *s1, uint64_t n1, uint8_t *d2,
                                               const uint8_t *s2, uint64_t n2) {
    if (n1 > 32 || n2 > 32) {
        copy_bytes(d1, s1, n1);
        copy_bytes(d2, s2, n2);
        return;
    }
    uint4 a1 = make_uint4(0u, 0u, 0u, 0u), b1 = a1, a2 = a1, b2 = a1;
    small_load(s1, n1, a1, b1);
    small_load(s2, n2, a2, b2);
    __asm__ volatile("" ::: "memory");   // every load before any store
    small_store(d1, n1, a1, b1);
    small_store(d2, n2, a2, b2);
}

// The growth of a run's records [j0, x): their BatchSums summed (0 at j0).
__device__ __forceinline__ BatchSums pm_bx(const PageMergeArgs &p, uint64_t j0, uint64_t x) {
    return x == j0 ? BatchSums(0) : p.bx[x - 1];
}

// The merge, a lane per segment for its control (groups, records) and the
// whole wave for every piece move: the wave's lanes step through their groups
// together, top down; each round moves every lane's piece (wave_run_jobs),
// then each lane writes its group's records into the gap above it.
template <bool CHECK>
// 4 waves per SIMD (<= 128 VGPRs: 127, no spill).  Round 5 took 5 (1.39 ->
// 1.22 ms against 3); with the uniform pages' state the 5-wave build spills 46
// VGPRs and the 4-wave one is faster: 0.624 against 0.689 ms a config-5 batch
// (6 waves 0.762, two units in flight 0.79; profiles/r06i_merge_waves_ab.txt)
#ifndef PM_WAVES
#define PM_WAVES 4
#endif
__global__ void __launch_bounds__(256, PM_WAVES) k_page_merge(PageMergeArgs p) {
    const MergeArgs &a = p.a;
    unsigned long long *chk = CHECK ? p.chk : nullptr;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    if (!page_room(p.acc, p.e0, p.k0, p.v0, p.ce, p.ck, p.cv)) return;   // the host rebuilds the pages and merges again
    for (uint64_t sb = w0 * 64; sb < a.S; sb += nw * 64) {
        const uint64_t s = sb + lane;
        const uint8_t mb = s < a.S ? p.mode[s] : 0, md = mb & 3;
        const bool expl = (mb & 4) != 0;   // the merged page keeps per-entry offsets (pages.h: uniform pages do not)
        uint64_t j0 = 0, je = 0, b = 0, Kb = 0, Vb = 0, De = 0, Dk = 0, Dv = 0;
        bool nz = false;   // the merged segment has entries
        const BatchSums B0(0);   // the growth before the run's first record (pm_bx: run-local sums)
        bool live = md != 0;
        // the page as it is: uniform = entry i's offsets by stride (its slots between the first and the end are stale)
        const uint32_t L0 = live ? p.m.klen[s] : KLEN_MIXED, V0 = live ? p.m.vlen[s] : KLEN_MIXED;
        const bool stride = page_uniform(L0, V0);
        uint64_t hi = 0, khi = 0, vhi = 0;   // the current piece's end (modes 1, 2) or start (mode 3)
        if (live) {
            j0 = a.bseg_off[s]; je = a.bseg_off[s + 1];
            b = p.m.beg[s];
            const uint64_t c = p.m.end[s] - b;
            Kb = p.m.kbeg[s]; Vb = p.m.vbeg[s];
            hi = c; khi = stride ? Kb + (uint64_t)L0 * c : p.koff[b + c]; vhi = p.m.vend[s];
            const SegSums X = p.ss[s];   // (read again at the end: not kept in registers through the merge)
            nz = X.v[0] != 0;
            uint64_t EC = p.m.ecap[s], KC = p.m.kcap[s], VC = p.m.vcap[s];
            De = b; Dk = Kb; Dv = Vb;
            uint64_t EB = b, KB = Kb, VB = Vb;   // the lowest entry slot / key byte / value byte a store may touch
            if (md == 2) {
                const PlanSums R = p.rbase[s], Z = p.rsz[s];
                const PageSums Hd = page_head(X.v[0], X.v[1], X.v[2], p.slack_pct);
                EB = p.e0 + R.v[0]; KB = p.k0 + R.v[1]; VB = p.v0 + R.v[2];
                De = EB + Hd.v[0]; Dk = KB + Hd.v[1]; Dv = VB + Hd.v[2];
                EC = EB + Z.v[0]; KC = KB + Z.v[1]; VC = VB + Z.v[2];
            } else if (md == 3) {   // the content's end stays, its start moves down by the growth
                De = b - (X.v[0] - c); Dk = Kb - (X.v[1] - (khi - Kb)); Dv = Vb - (X.v[2] - (vhi - Vb));
                EB = p.m.ebot[s]; KB = p.m.kbot[s]; VB = p.m.vbot[s];
                hi = 0; khi = Kb; vhi = Vb;
            }
            // the merged segment fits its (new) page: every move below stays inside it
            live = pg_ok(chk, De + X.v[0] < EC && Dk + X.v[1] <= KC && Dv + X.v[2] <= VC, 14, s, De + X.v[0], EC) &&
                   pg_ok(chk, De >= EB && Dk >= KB && Dv >= VB, 15, s, De, EB);
        }
        uint32_t kl = (live && nz) ? p.m.klen[s] : KLEN_NONE;   // the merged segment's uniform key length
        uint32_t vl = (live && nz) ? p.m.vlen[s] : KLEN_NONE;   // ... and value length
        // modes 1, 2: the groups from the last down, each piece above its group
        // moved up first; mode 3: from the first up, each piece below its group
        // moved down first
        const bool upw = md != 3;
        uint64_t j = upw ? je : j0;
        while (__ballot(live && (upw ? j > j0 : j < je))) {
            const bool mine = live && (upw ? j > j0 : j < je);
            PieceJob J{};
            bool has = false;
            uint64_t u = 0, g0 = 0, g1 = 0, ku = 0, vu = 0;
            if (mine) {
                if (upw) {
                    g1 = j;
                    u = p.pos[g1 - 1];
                    g0 = g1 - 1;
                    while (g0 > j0 && p.pos[g0 - 1] == u) g0--;
                } else {
                    g0 = j;
                    u = p.pos[g0];
                    g1 = g0 + 1;
                    while (g1 < je && p.pos[g1] == u) g1++;
                }
                // the group's last record replaces entry u
                const bool eq = pm_bx(p, j0, g1).v[BS_EQ] != pm_bx(p, j0, g1 - 1).v[BS_EQ];
                const RecAt R = p.rat[g1 - 1];   // entry u's old offsets, page-relative (read before any rewrite)
                ku = Kb + R.ku;
                vu = Vb + R.vu;
                // the piece: above the group up to hi, shifted by the growth through
                // it (modes 1, 2), or from hi up to the group, shifted by the growth
                // before it (mode 3)
                const uint64_t pa = upw ? u + (eq ? 1 : 0) : hi, pe = upw ? hi : u;
                if (pa < pe) {
                    const BatchSums Bg = pm_bx(p, j0, upw ? g1 : g0);
                    const uint64_t de = (Bg.v[BS_NE] - B0.v[BS_NE]) - (Bg.v[BS_EQ] - B0.v[BS_EQ]);
                    const uint64_t dk = (Bg.v[BS_KN] - B0.v[BS_KN]) - (Bg.v[BS_KE] - B0.v[BS_KE]);
                    const uint64_t dv = (Bg.v[BS_VN] - B0.v[BS_VN]) - (Bg.v[BS_VE] - B0.v[BS_VE]);
                    const uint64_t k0 = !upw ? khi : stride ? Kb + (uint64_t)L0 * pa : p.koff[b + pa];
                    const uint64_t v0 = !upw ? vhi : stride ? Vb + (uint64_t)V0 * pa : p.voff[b + pa];
                    const uint64_t k1 = upw ? khi : ku, v1 = upw ? vhi : vu;
                    J.kd = (uint64_t)(p.kheap + Dk + (k0 - Kb) + dk); J.ks = (uint64_t)(p.kheap + k0); J.nk = k1 - k0;
                    J.vd = (uint64_t)(p.vheap + Dv + (v0 - Vb) + dv); J.vs = (uint64_t)(p.vheap + v0); J.nv = v1 - v0;
                    J.ko = (uint64_t)(p.koff + b); J.vo = (uint64_t)(p.voff + b);
                    J.a = pa; J.e = pe; J.de = (De - b) + de; J.dk = (Dk - Kb) + dk; J.dv = (Dv - Vb) + dv;
                    J.fl = ((md == 2 || J.dk) ? 1u : 0u) | ((md == 2 || J.dv) ? 2u : 0u) |
                           (expl && (md == 2 || J.de || J.dk) ? 4u : 0u) | (expl && (md == 2 || J.de || J.dv) ? 8u : 0u);
                    has = J.fl != 0;
                    J.fl |= upw ? 0u : PM_ASC;
                }
            }
            wave_run_jobs(J, has, lane);
            if (mine) {
                for (uint64_t r = g1; r > g0; r--) {   // the group's records that produce an entry, highest first
                    const BatchSums Br = pm_bx(p, j0, r - 1), Bn = pm_bx(p, j0, r);
                    if (Bn.v[BS_NE] == Br.v[BS_NE]) continue;
                    const uint64_t nwi = De + u + (Br.v[BS_NE] - B0.v[BS_NE]) - (Br.v[BS_EQ] - B0.v[BS_EQ]);
                    const uint64_t nk = Dk + (ku - Kb) + (Br.v[BS_KN] - B0.v[BS_KN]) - (Br.v[BS_KE] - B0.v[BS_KE]);
                    const uint64_t nv = Dv + (vu - Vb) + (Br.v[BS_VN] - B0.v[BS_VN]) - (Br.v[BS_VE] - B0.v[BS_VE]);
                    const RecAt Q = p.rat[r - 1];
                    if (nz) {
                        kl = klen_add(kl, Bn.v[BS_KN] - Br.v[BS_KN]);
                        vl = klen_add(vl, Bn.v[BS_VN] - Br.v[BS_VN]);
                    }
                    if (expl) {
                        p.koff[nwi] = nk;
                        p.voff[nwi] = nv;
                    }
                    copy2_disjoint(p.kheap + nk, a.bv.kheap + Q.bk, Bn.v[BS_KN] - Br.v[BS_KN], p.vheap + nv,
                                   a.bvheap + Q.bv, Bn.v[BS_VN] - Br.v[BS_VN]);
                }
                if (upw) {
                    hi = u; khi = ku; vhi = vu;
                    j = g0;
                } else {   // the next piece starts after entry u if the group replaced it (its old offsets: not
                           // yet overwritten, every store so far went below it)
                    const bool eq = pm_bx(p, j0, g1).v[BS_EQ] != pm_bx(p, j0, g1 - 1).v[BS_EQ];
                    hi = u + (eq ? 1 : 0);
                    khi = !eq ? ku : stride ? Kb + (uint64_t)L0 * hi : p.koff[b + hi];
                    vhi = !eq ? vu : stride ? Vb + (uint64_t)V0 * hi : p.voff[b + hi];
                    j = g1;
                }
            }
        }
        {   // mode 2: the entries before the first record, unshifted, into the new page
            PieceJob J{};
            const bool has = live && md == 2 && hi;
            if (has) {
                J.kd = (uint64_t)(p.kheap + Dk); J.ks = (uint64_t)(p.kheap + Kb); J.nk = khi - Kb;
                J.vd = (uint64_t)(p.vheap + Dv); J.vs = (uint64_t)(p.vheap + Vb); J.nv = vhi - Vb;
                J.ko = (uint64_t)(p.koff + b); J.vo = (uint64_t)(p.voff + b);
                J.a = 0; J.e = hi; J.de = De - b; J.dk = Dk - Kb; J.dv = Dv - Vb; J.fl = expl ? 15 : 3;
            }
            wave_run_jobs(J, has, lane);
        }
        if (live) {
            const SegSums X = p.ss[s];
            if (kl != p.m.klen[s]) p.m.klen[s] = (uint16_t)kl;
            if (vl != p.m.vlen[s]) p.m.vlen[s] = (uint16_t)vl;
            p.koff[De + X.v[0]] = Dk + X.v[1];   // the end slot
            p.voff[De + X.v[0]] = Dv + X.v[2];
            if (md >= 2) {   // the first slot (a uniform page keeps no other)
                p.koff[De] = Dk;
                p.voff[De] = Dv;
            }
            p.m.end[s] = De + X.v[0];
            p.m.vend[s] = Dv + X.v[2];
            if (md >= 2) {
                p.m.beg[s] = De;
                p.m.vbeg[s] = Dv;
                p.m.kbeg[s] = Dk;
            }
            if (md == 2) {   // the new page's bounds
                const PlanSums R = p.rbase[s], Z = p.rsz[s];
                p.m.ebot[s] = p.e0 + R.v[0];
                p.m.kbot[s] = p.k0 + R.v[1];
                p.m.vbot[s] = p.v0 + R.v[2];
                p.m.ecap[s] = p.e0 + R.v[0] + Z.v[0];
                p.m.kcap[s] = p.k0 + R.v[1] + Z.v[1];
                p.m.vcap[s] = p.v0 + R.v[2] + Z.v[2];
            }
        }
    }
}

// Checked build: every segment's page is consistent (entries and bytes
// inside its capacities, above its bottoms, offsets nondecreasing, the view's
// value bounds).
__global__ void k_page_validate(PageMeta m, const uint64_t *koff, const uint64_t *voff, uint64_t S, uint64_t cap_e,
                                uint64_t cap_k, uint64_t cap_v, unsigned long long *chk) {
    for (uint64_t s = gtid(); s < S; s += gstride()) {
        const uint64_t b = m.beg[s], e = m.end[s];
        if (!pg_ok(chk, b <= e && e < m.ecap[s] && m.ecap[s] <= cap_e, 20, s, e, m.ecap[s])) continue;
        if (!pg_ok(chk, koff[b] <= koff[e] && koff[e] <= m.kcap[s] && m.kcap[s] <= cap_k, 21, s, koff[e], m.kcap[s])) continue;
        if (!pg_ok(chk, voff[b] <= voff[e] && voff[e] <= m.vcap[s] && m.vcap[s] <= cap_v, 22, s, voff[e], m.vcap[s])) continue;
        if (!pg_ok(chk, m.vbeg[s] == voff[b] && m.vend[s] == voff[e] && m.kbeg[s] == koff[b], 23, s, m.vbeg[s], voff[b]))
            continue;
        if (!pg_ok(chk, m.ebot[s] <= b && m.kbot[s] <= koff[b] && m.vbot[s] <= voff[b], 27, s, b, m.ebot[s])) continue;
        const uint32_t L = m.klen[s], V = m.vlen[s];   // the uniform lengths, if any, hold
        if (!pg_ok(chk, (L != KLEN_NONE && V != KLEN_NONE) || b == e, 25, s, e - b, L)) continue;
        if (page_uniform(L, V)) {   // offsets by stride: only the first and end slots are kept
            const uint64_t n = e - b;
            pg_ok(chk, b == e || (koff[e] - koff[b] == (uint64_t)L * n && voff[e] - voff[b] == (uint64_t)V * n), 26, s, L, b);
            continue;
        }
        bool kl_ok = true;
        for (uint64_t i = b; i < e && L != KLEN_MIXED && L != KLEN_NONE; i++) kl_ok &= koff[i + 1] - koff[i] == L;
        for (uint64_t i = b; i < e && V != KLEN_MIXED && V != KLEN_NONE; i++) kl_ok &= voff[i + 1] - voff[i] == V;
        if (!pg_ok(chk, kl_ok, 26, s, L, b)) continue;
        for (uint64_t i = b; i < e; i++)
            if (!pg_ok(chk, koff[i] <= koff[i + 1] && voff[i] <= voff[i + 1], 24, s, i, b)) {
                if (chk[2] == s && chk[3] == i)   // the first violation: the page's offsets for the report
                    for (uint64_t q = 0; q < 12 && b + q <= e; q++) { chk[5 + q] = koff[b + q]; chk[17 + q] = voff[b + q]; }
                break;
            }
    }
}

// Fault injection (st_debug_knob ST_DBG_PAGE_POISON): segment s's page now
// claims entries past its capacity -- what a merge that stored outside its
// page would leave -- so the checked mode can be shown to refuse it.
__global__ void k_page_poison(PageMeta m, uint64_t s) {
    if (threadIdx.x | blockIdx.x) return;
    m.end[s] = m.ecap[s] + 7;
}

// Empty segment s in place (a segment node deleted or stored as []): its
// page keeps its capacity; *cnt = the entries it held.
__global__ void k_page_clear(PageMeta m, uint64_t s, uint64_t *cnt) {
    if (threadIdx.x | blockIdx.x) return;
    *cnt = m.end[s] - m.beg[s];
    m.end[s] = m.beg[s];
    m.vend[s] = m.vbeg[s];
    m.klen[s] = KLEN_NONE;
    m.vlen[s] = KLEN_NONE;
}
