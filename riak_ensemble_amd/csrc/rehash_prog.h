// rehash_prog.h — the progressive fused rehash (W == 16, H >= 3).
//
// One workgroup of 1024 threads per WINDOW = level-(H-2) subtree (4096
// segments), like k_rehash_fused, but the window's inner levels are hashed
// WHILE its segments are, so only the last two MD5 blocks of each of levels
// H, H-1, H-2 remain after the window's last segment (rehash/1 + rehash_upper/1,
// synctree.erl:489-543; a node's hash is md5 of its present children's 17-byte
// entries in child order, :255-259, :516-533).
//
// Why that works: an inner node's message is 16 x 17 = 272 bytes, 5 blocks;
// blocks 0-2 (bytes 0..191) hold only children 0..11 when all are present.
// So the window's segments are hashed in CLASSES (digits d2 d1 d0 of the
// segment index inside the window; "late" = digit >= 12):
//
//   class 0: d2 < 12, d1 < 12            36 tiles  -> level-H nodes of d2<12, d1<12 complete
//   class 3: d2 >= 12, d1 < 12           12 tiles  -> level-H nodes of d2>=12, d1<12 complete
//   class 1: d2 < 12, d1 >= 12, d0 < 12   9 tiles  -> prefix (blocks 0-2) of level-H d2<12, d1>=12
//   class 4: d2 >= 12, d1 >= 12, d0 < 12  3 tiles  -> prefix of level-H d2>=12, d1>=12
//   class 2: d2 < 12, d1 >= 12, d0 >= 12  3 tiles  -> those level-H nodes finish; H-1 nodes 0..11 finish
//   class 5: d2 >= 12, d1 >= 12, d0 >= 12 1 tile   -> the rest: 2 + 2 + 2 blocks
//
// (tiles in this order, each class sorted by message length: k_tile_order_cls).
// Waves 0..11 hash tiles taken from an LDS counter (dynamic balance) and
// write each segment's entry straight into its parent's packed message in LDS
// (byte offset 17 x rank among the present siblings; presence is known from
// the window's segment bitmap before any hashing).  Waves 12..15 are CHAIN
// waves at raised issue priority: lane n of chain wave c owns level-H node
// 64c + n; lanes with d1 == 0 also own H-1 node 4c + n/16, and lane 1 of wave
// 15 owns the window root.  Each chain lane advances its node's MD5 by as many
// complete 64-byte blocks as the ready prefix of the message allows (present
// children whose class is done), and finishes it (padding, RFC 1321 §3.1-3.2)
// once every child is in.  With absent children the ready prefix is shorter
// and more blocks are left for the finish: correct for any presence pattern.
//
// The window's root entry then climbs exactly as in k_rehash_fused (mailbox +
// one per-tree counter; the last window hashes the upper levels).
#pragma once

#define PG_K1W 12        // K1 waves (0..11); waves 12..15 are the chain waves
#define PG_MSG 272       // one node's message region: 16 x 17 bytes
#define PG_MH 0                              // 256 level-H messages
#define PG_M1 (PG_MH + 256 * PG_MSG)         // 16 H-1 messages
#define PG_M0 (PG_M1 + 16 * PG_MSG)          // the window root's message (+ read slack to 320)
#define PG_TI (PG_M0 + 320)                  // 64 TileInfo
#define PG_TLN (PG_TI + 64 * 16)             // 4096 x u32 message descriptors (window tile order)
#define PG_TLI (PG_TLN + 4096 * 4)           // 4096 x u16 segment index in the window
#define PG_PRES (PG_TLI + 4096 * 2)          // 64 x u64 segment presence bitmap
#define PG_K_END (PG_PRES + 512)
// the climb (last window only, after the K1 phase): node blocks of the
// mailbox level (entries, tags), sparse-node message regions, and two
// ping-pong sets of 16 node blocks for the levels above
#define PG_CE 0
#define PG_CT (PG_CE + 256 * NB16)
#define PG_CR (PG_CT + 256 * TB16)
#define PG_CB (PG_CR + 256 * PG_MSG)
#define PG_CBSZ (16 * NB16 + 16 * TB16)
#define PG_C_END (PG_CB + 2 * PG_CBSZ)
#define PG_CNT (PG_C_END > PG_K_END ? PG_C_END : PG_K_END)   // counters (u32), never overlaid
#define PG_LDS (PG_CNT + 64)
// counters: [0] tile grab, [1 + c] tiles of class c done, [7] chain waves 0..2
// with every H-1 node finished, [8] tiles done (all classes), [9] s_last
#define PG_C_GRAB 0
#define PG_C_DONE 1
#define PG_C_H1 7
#define PG_C_ALL 8
#define PG_C_LAST 9

__host__ __device__ __forceinline__ uint32_t prog_lds_bytes() { return PG_LDS; }

// class of a segment by its index li (0..4095) in the window
__host__ __device__ __forceinline__ uint32_t pg_seg_class(uint32_t li) {
    const uint32_t d2 = li >> 8, d1 = (li >> 4) & 15, d0 = li & 15;
    return (d2 >= 12 ? 3u : 0u) + (d1 >= 12 ? (d0 >= 12 ? 2u : 1u) : 0u);
}
// position of a class in the tile order, and its tile range
__host__ __device__ __forceinline__ uint32_t pg_class_seq(uint32_t c) {
    // order 0, 3, 1, 4, 2, 5
    return c == 0 ? 0u : c == 3 ? 1u : c == 1 ? 2u : c == 4 ? 3u : c == 2 ? 4u : 5u;
}
__host__ __device__ __forceinline__ uint32_t pg_tile_class(uint32_t tl) {
    return tl < 36 ? 0u : tl < 48 ? 3u : tl < 57 ? 1u : tl < 60 ? 4u : tl < 63 ? 2u : 5u;
}
__host__ __device__ __forceinline__ uint32_t pg_class_tiles(uint32_t c) {
    return c == 0 ? 36u : c == 1 ? 9u : c == 2 ? 3u : c == 3 ? 12u : c == 4 ? 3u : 1u;
}

// Window-local tile order for k_rehash_prog: one workgroup per window sorts
// its 4096 segments by (class position, stored rows descending) into the 64
// tiles (LDS counting sort over 6 x 256 bins), and writes the window's
// segment presence bitmap (pres[window * 64 + w], bit j = segment 64w + j
// non-empty).
__global__ void __launch_bounds__(256) k_tile_order_cls(DevTree t, uint32_t *__restrict__ tseg, uint32_t *__restrict__ tln,
                                                        TileInfo *__restrict__ tinfo, uint64_t *__restrict__ tsize,
                                                        uint64_t *__restrict__ pres) {
    __shared__ uint32_t hist[6 * 256];
    __shared__ uint32_t pln[4096];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t seg0 = (uint64_t)blockIdx.x * 4096;
    for (uint32_t i = tid; i < 6 * 256; i += 256) hist[i] = 0;
    __syncthreads();
    uint32_t ln[16], bin[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t li = k * 256 + tid;
        const uint64_t s = seg0 + li;
        ln[k] = t.seg_off[s] != t.seg_off[s + 1] ? (uint32_t)(t.seg_voff[s + 1] - t.seg_voff[s] + 1) : 0u;
        const uint32_t r = ln_rows(ln[k]) + (ln[k] != 0);   // present-but-empty values sort above absent
        bin[k] = pg_class_seq(pg_seg_class(li)) * 256 + 255u - (r > 255u ? 255u : r);
        atomicAdd(&hist[bin[k]], 1u);
        const unsigned long long bits = __ballot(ln[k] != 0);   // segments 64 (4k + wave) .. + 63
        if (lane == 0) pres[blockIdx.x * 64 + (k * 256 + wave * 64) / 64] = bits;
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t acc = 0;
        for (int x = 0; x < 6 * 256; x++) { const uint32_t c = hist[x]; hist[x] = acc; acc += c; }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t pos = atomicAdd(&hist[bin[k]], 1u);
        tseg[seg0 + pos] = (uint32_t)(seg0 + k * 256 + tid);
        tln[seg0 + pos] = ln[k];
        pln[pos] = ln[k];
    }
    __syncthreads();
    for (uint32_t j = wave; j < 64; j += 4) tile_shape(pln[j * 64 + lane], blockIdx.x * 64 + j, lane == 0, tinfo, tsize);
}

// 17-byte entry <<Prefix, MD5:16/binary>> at any byte offset of LDS.
__device__ __forceinline__ void pg_put17(uint8_t *p, uint32_t pfx, const uint32_t s[4]) {
    p[0] = (uint8_t)pfx;
#pragma unroll
    for (int w = 0; w < 4; w++) {
#pragma unroll
        for (int b = 0; b < 4; b++) p[1 + 4 * w + b] = (uint8_t)(s[w] >> (8 * b));
    }
}

// 16 bytes at any byte offset of LDS (aligned dword reads + funnel shifts).
__device__ __forceinline__ uint4 pg_get16(const uint8_t *lds, uint32_t o) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(lds + (o & ~3u));
    const uint32_t sh = (o & 3u) * 8u;
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
    return make_uint4(__builtin_amdgcn_alignbit(w1, w0, sh), __builtin_amdgcn_alignbit(w2, w1, sh),
                      __builtin_amdgcn_alignbit(w3, w2, sh), __builtin_amdgcn_alignbit(w4, w3, sh));
}

// Advance the MD5 of a `len`-byte message in LDS at p from block k to block
// kend (per lane; kend = the message's block count finishes it with the
// padding).  Latency form: a few lanes per wave run these chains.
__device__ __forceinline__ void pg_advance(const uint8_t *p, uint32_t len, uint32_t &k, uint32_t kend, uint32_t st[4]) {
    const uint32_t nblk = (len + 8) / 64 + 1;
    const uint32_t *pw = reinterpret_cast<const uint32_t *>(p);
    while (k < kend) {
        uint32_t m[16];
#pragma unroll
        for (int w = 0; w < 16; w++) m[w] = pw[16 * k + w];
        const int32_t rem = (int32_t)len - (int32_t)(64 * k);
        if (rem < 64) stmd5::pad_block(m, rem, k + 1 == nblk, len);
        stmd5::compress(st, m);
        k++;
    }
}

__device__ __forceinline__ void pg_wait_lds() { __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ uint32_t pg_ld(const uint32_t *p) {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}

// STAMP (diagnostic, ST_LEVEL_STAMPS=1 with ST_REHASH=prog): wall-clock (100
// MHz) at [blockIdx * 32 + k] and shader clock at [.. + 16 + k]: 0 start, 1
// staged, 2 wave 0 out of tiles, 3 every tile done (wave 0), 4 copy-out done
// (wave 0), 5 chain waves 0..2 done (root lane), 6 root prefix hashed, 7 wave
// 15's H-1 nodes done, 8 root finished, 9 climb counter won, 10 mailboxes
// read, 11 first climb level hashed, 12 second, 15 exit.
template <bool STAMP, bool GROUP>
__global__ void __launch_bounds__(1024) k_rehash_prog(DevTree t, TreeTiles tt0, const TreeTiles *__restrict__ group,
                                                      uint32_t nwin, uint64_t root0, uint32_t lmin, uint64_t *stamps) {
#define PG_STAMP(cond, k) do { if (STAMP && (cond)) { stamps[blockIdx.x * 32 + (k)] = __builtin_amdgcn_s_memrealtime(); \
                                                      stamps[blockIdx.x * 32 + 16 + (k)] = __builtin_amdgcn_s_memtime(); } } while (0)
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    PG_STAMP(tid == 0, 0);
    const uint32_t gi = GROUP ? blockIdx.x / nwin : 0;
    const uint64_t root = GROUP ? (uint64_t)(blockIdx.x - gi * nwin) : root0 + blockIdx.x;
#define RFT(f) (GROUP ? group[gi].f : tt0.f)
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    TileInfo *TI = reinterpret_cast<TileInfo *>(lds + PG_TI);
    uint32_t *TLN = reinterpret_cast<uint32_t *>(lds + PG_TLN);
    uint16_t *TLI = reinterpret_cast<uint16_t *>(lds + PG_TLI);
    uint64_t *PRES = reinterpret_cast<uint64_t *>(lds + PG_PRES);
    uint32_t *CNT = reinterpret_cast<uint32_t *>(lds + PG_CNT);
    const uint32_t H = t.H;
    const uint64_t seg0 = root * 4096;

    // ---- stage the window's tile descriptors, message descriptors, segment
    // indices and presence bitmap
    {
        const uint64_t w0 = root * 4096;
        const uint4 a = reinterpret_cast<const uint4 *>(RFT(tln) + w0)[tid];
        const uint4 s = reinterpret_cast<const uint4 *>(RFT(tseg) + w0)[tid];
        reinterpret_cast<uint4 *>(TLN)[tid] = a;
        const uint32_t l0 = (uint32_t)(s.x - seg0), l1 = (uint32_t)(s.y - seg0), l2 = (uint32_t)(s.z - seg0),
                       l3 = (uint32_t)(s.w - seg0);
        reinterpret_cast<uint2 *>(TLI)[tid] = make_uint2(l0 | (l1 << 16), l2 | (l3 << 16));
        if (tid < 64) {
            const TileInfo ti = RFT(tinfo)[root * 64 + tid];
            TI[tid] = ti;
            PRES[tid] = RFT(pres)[root * 64 + tid];
        }
        if (tid < 16) CNT[tid] = tid == PG_C_GRAB ? (uint32_t)PG_K1W : 0u;
    }
    __syncthreads();
    PG_STAMP(tid == 0, 1);
    auto pres16 = [&](uint32_t n) { return (uint32_t)(PRES[n >> 2] >> (16 * (n & 3))) & 0xffffu; };

    if (wave < PG_K1W) {
        // ================= K1 waves: dynamic tiles, one flat block stream
        auto grab = [&]() -> uint32_t {
            for (;;) {
                uint32_t v = 0;
                if (lane == 0) v = __hip_atomic_fetch_add(&CNT[PG_C_GRAB], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const uint32_t tl = __builtin_amdgcn_readfirstlane(v);
                if (tl >= 64) return 64u;
                if (__builtin_amdgcn_readfirstlane(TI[tl].B)) return tl;
                if (lane == 0) {   // a tile of absent segments: nothing to hash or write
                    __hip_atomic_fetch_add(&CNT[PG_C_DONE + pg_tile_class(tl)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_fetch_add(&CNT[PG_C_ALL], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
        };
        uint32_t ft = wave;   // the first tile is static
        if (!__builtin_amdgcn_readfirstlane(TI[ft].B)) {
            if (lane == 0) {
                __hip_atomic_fetch_add(&CNT[PG_C_DONE + pg_tile_class(ft)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&CNT[PG_C_ALL], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            ft = grab();
        }
        if (ft < 64) {
            // fetch cursor (ft, fk) two blocks ahead of the hash cursor (ht, hk);
            // q1, q2: tiles the fetch cursor entered beyond the hash cursor's
            const uint4 *tiles = RFT(tiles);
            uint32_t fk = 0, fB = 0, fL = 0;
            uint64_t fbase = 0;
            auto fload = [&](uint32_t tl) {
                const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)TI[tl].base),
                               hi = __builtin_amdgcn_readfirstlane((uint32_t)(TI[tl].base >> 32));
                fbase = ((uint64_t)hi << 32) | lo;
                const uint32_t R = __builtin_amdgcn_readfirstlane(TI[tl].R);
                fL = R ? R - 1 : 0;
                fB = __builtin_amdgcn_readfirstlane(TI[tl].B);
            };
            fload(ft);
            uint32_t q1 = 64, q2 = 64;
            auto fetch = [&](uint4 &a, uint4 &b, uint4 &c, uint4 &d) {
                const uint32_t r = 4 * fk, last = fL;
                const uint4 *p = tiles + fbase;
                a = (p + (uint64_t)(r < last ? r : last) * 64)[lane];
                b = (p + (uint64_t)(r + 1 < last ? r + 1 : last) * 64)[lane];
                c = (p + (uint64_t)(r + 2 < last ? r + 2 : last) * 64)[lane];
                d = (p + (uint64_t)(r + 3 < last ? r + 3 : last) * 64)[lane];
                if (ft >= 64) return;   // past the stream: a dummy fetch of the last tile
                if (++fk == fB) {
                    fk = 0;
                    const uint32_t nt = grab();
                    if (nt < 64) {
                        ft = nt;
                        fload(nt);
                        if (q1 >= 64) q1 = nt; else q2 = nt;
                    } else {
                        ft = 64;
                    }
                }
            };
            uint32_t ht = ft, hk = 0, hB = 0, hR = 0, hln = 0, hli = 0, hnb = 0;
            auto hload = [&](uint32_t tl) {
                hB = __builtin_amdgcn_readfirstlane(TI[tl].B);
                hR = __builtin_amdgcn_readfirstlane(TI[tl].R);
                hln = TLN[tl * 64 + lane];
                hli = TLI[tl * 64 + lane];
                hnb = ln_blocks(hln);
            };
            hload(ht);
            uint4 a0, a1, a2, a3, b0, b1, b2, b3;
            fetch(a0, a1, a2, a3);
            fetch(b0, b1, b2, b3);
            uint32_t st[4];
            stmd5::init(st);
            auto hash_block = [&](const uint4 &x0, const uint4 &x1, const uint4 &x2, const uint4 &x3) {
                const uint32_t r = 4 * hk;
                if (r + 3 >= hR) {
                    const uint4 y0 = r >= hR ? tile_synth(r, hln) : x0, y1 = r + 1 >= hR ? tile_synth(r + 1, hln) : x1,
                                y2 = r + 2 >= hR ? tile_synth(r + 2, hln) : x2, y3 = tile_synth(r + 3, hln);
                    const uint32_t m[16] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w,
                                            y2.x, y2.y, y2.z, y2.w, y3.x, y3.y, y3.z, y3.w};
                    if (hk < hnb) stmd5::compress<true>(st, m);
                } else {
                    const uint32_t m[16] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w,
                                            x2.x, x2.y, x2.z, x2.w, x3.x, x3.y, x3.z, x3.w};
                    if (hk < hnb) stmd5::compress<true>(st, m);
                }
                if (++hk == hB) {
                    // the tile's segment entries into their parents' messages
                    if (hnb) {
                        const uint32_t n = hli >> 4, j = hli & 15;
                        const uint32_t o = n * PG_MSG + 17u * __builtin_popcount(pres16(n) & ((1u << j) - 1u));
                        pg_put17(lds + PG_MH + o, 0u, st);
                    }
                    pg_wait_lds();
                    if (lane == 0) {
                        __hip_atomic_fetch_add(&CNT[PG_C_DONE + pg_tile_class(ht)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_fetch_add(&CNT[PG_C_ALL], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                    stmd5::init(st);
                    hk = 0;
                    ht = q1;
                    q1 = q2;
                    q2 = 64;
                    if (ht < 64) hload(ht);
                }
            };
            for (;;) {
                hash_block(a0, a1, a2, a3);
                fetch(a0, a1, a2, a3);
                if (ht >= 64) break;
                hash_block(b0, b1, b2, b3);
                fetch(b0, b1, b2, b3);
                if (ht >= 64) break;
            }
        }
        PG_STAMP(tid == 0, 2);
        // ---- every tile done: the window's segment entries to the slot arrays
        // (write-through md5 stores, coalesced; absent segments: tag 0, md5 0)
        while (pg_ld(&CNT[PG_C_ALL]) < 64) __builtin_amdgcn_s_sleep(1);
        PG_STAMP(tid == 0, 3);
        const uint64_t c0 = t.base[H + 1] + seg0;
        const uint64_t nbytes = (t.base[H + 1] + t.S) * 16;
        const __amdgpu_buffer_rsrc_t md5r = __builtin_amdgcn_make_buffer_rsrc(
            GROUP ? group[gi].md5 : t.md5, (short)0, (int)(nbytes < 0xffffffffull ? nbytes : 0xffffffffull), 0x00020000);
        uint16_t *tagp = GROUP ? group[gi].tag : t.tag;
        for (uint32_t i = tid; i < 4096; i += PG_K1W * 64) {
            const uint32_t n = i >> 4, j = i & 15, p16 = pres16(n);
            uint4 e = make_uint4(0, 0, 0, 0);
            uint16_t tg = 0;
            if ((p16 >> j) & 1u) {
                e = pg_get16(lds + PG_MH, n * PG_MSG + 17u * __builtin_popcount(p16 & ((1u << j) - 1u)) + 1u);
                tg = (uint16_t)TAG_PRESENT;
            }
            const u32x4 v = {e.x, e.y, e.z, e.w};
            __builtin_amdgcn_raw_buffer_store_b128(v, md5r, (int)((c0 + i) * 16), 0, 16 /* sc1 */);
            tagp[c0 + i] = tg;
        }
        PG_STAMP(tid == 0, 4);
    } else {
        // ================= chain waves
        __builtin_amdgcn_s_setprio(3);
        const uint32_t c = wave - PG_K1W;            // 0..3
        const bool hi = c == 3;                      // d2 >= 12
        const uint32_t n = 64 * c + lane;            // level-H node in the window
        const uint32_t d1 = lane & 15, g = lane >> 4, m1 = 4 * c + g;
        const uint32_t p16 = pres16(n);
        const unsigned long long pmw = __ballot(p16 != 0);
        const uint32_t pm16 = (uint32_t)(pmw >> (16 * g)) & 0xffffu;   // H-1 node m1's level-H presence
        uint32_t rb = 0;
        if (lane < 16) rb = (PRES[4 * lane] | PRES[4 * lane + 1] | PRES[4 * lane + 2] | PRES[4 * lane + 3]) != 0;
        const uint32_t rootmask = (uint32_t)__ballot(rb) & 0xffffu;     // the window root's H-1 presence
        const uint32_t cA = hi ? 3u : 0u, cB = hi ? 4u : 1u, cC = hi ? 5u : 2u;
        const bool aux_h1 = d1 == 0, aux_root = hi && lane == 1;
        // own job: level-H node n
        const uint32_t len_o = 17u * __builtin_popcount(p16);
        const uint32_t pfx_o = d1 >= 12 ? (17u * __builtin_popcount(p16 & 0xfffu)) / 64u : 0u;
        uint32_t k_o = 0, ph_o = 0;                  // 0 waiting, 1 prefix hashed, 2 finished
        uint32_t so[4];
        stmd5::init(so);
        // aux job: H-1 node m1 (d1 == 0) or the window root (wave 15 lane 1)
        const uint32_t len_a = aux_h1 ? 17u * __builtin_popcount(pm16) : aux_root ? 17u * __builtin_popcount(rootmask) : 0u;
        const uint32_t pfx_a = aux_h1 ? (17u * __builtin_popcount(pm16 & 0xfffu)) / 64u
                                      : aux_root ? (17u * __builtin_popcount(rootmask & 0xfffu)) / 64u : 0u;
        uint32_t k_a = 0, ph_a = (aux_h1 || aux_root) ? 0u : 2u;
        uint32_t sa[4];
        stmd5::init(sa);
        const uint8_t *msg_o = lds + PG_MH + n * PG_MSG;
        const uint8_t *msg_a = aux_h1 ? lds + PG_M1 + m1 * PG_MSG : lds + PG_M0;
        bool h1_signalled = hi;                      // waves 0..2 count themselves into CNT[PG_C_H1] once
        uint32_t stampd = 0;
        for (;;) {
            const bool evA = pg_ld(&CNT[PG_C_DONE + cA]) >= pg_class_tiles(cA);
            const bool evB = pg_ld(&CNT[PG_C_DONE + cB]) >= pg_class_tiles(cB);
            const bool evC = pg_ld(&CNT[PG_C_DONE + cC]) >= pg_class_tiles(cC);
            const uint32_t h1 = hi ? pg_ld(&CNT[PG_C_H1]) : 0u;
            // group readiness (this wave's lanes): own nodes finished
            const unsigned long long fin_o = __ballot(ph_o == 2);
            const uint32_t grp = (uint32_t)(fin_o >> (16 * g)) & 0xffffu;
            const bool grp_lo = (grp & 0x0fffu) == 0x0fffu, grp_all = grp == 0xffffu;
            const unsigned long long fin_a = __ballot(aux_h1 && ph_a == 2);
            const bool my_h1_done = ((uint32_t)fin_a & 1u) && ((uint32_t)(fin_a >> 16) & 1u) && ((uint32_t)(fin_a >> 32) & 1u) &&
                                    ((uint32_t)(fin_a >> 48) & 1u);
            if (!h1_signalled && my_h1_done) {
                // waves 0..2: every H-1 node of this wave is in the root's message
                pg_wait_lds();
                if (lane == 0) __hip_atomic_fetch_add(&CNT[PG_C_H1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                h1_signalled = true;
            }
            // this lane's job this round: 0 none, 1 own, 2 aux; and its target block
            uint32_t job = 0, kend = 0;
            if (ph_o != 2) {
                if (d1 < 12) {
                    if (evA) { job = 1; kend = (len_o + 8) / 64 + 1; }
                } else if (evC && evB) {
                    job = 1; kend = (len_o + 8) / 64 + 1;
                } else if (ph_o == 0 && evB) {
                    job = 1; kend = pfx_o;
                }
                if (len_o == 0 && job == 1) kend = 0;
            } else if (ph_a != 2) {
                if (aux_h1) {
                    if (grp_all) { job = 2; kend = (len_a + 8) / 64 + 1; }
                    else if (ph_a == 0 && grp_lo) { job = 2; kend = pfx_a; }
                } else {   // the window root
                    if (h1 >= 3 && my_h1_done) { job = 2; kend = (len_a + 8) / 64 + 1; }
                    else if (ph_a == 0 && h1 >= 3) { job = 2; kend = pfx_a; }
                }
                if (len_a == 0 && job == 2) kend = 0;
            }
            if (__ballot(job != 0) == 0) {
                if (__ballot(ph_o != 2 || ph_a != 2) == 0 && h1_signalled) break;   // every job of this wave finished
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            // one advance for every lane with a job (the own or the aux state)
            {
                const bool aux = job == 2;
                uint32_t s4[4] = {aux ? sa[0] : so[0], aux ? sa[1] : so[1], aux ? sa[2] : so[2], aux ? sa[3] : so[3]};
                uint32_t kk = aux ? k_a : k_o;
                if (job) pg_advance(aux ? msg_a : msg_o, aux ? len_a : len_o, kk, kend, s4);
                if (job == 1) { so[0] = s4[0]; so[1] = s4[1]; so[2] = s4[2]; so[3] = s4[3]; k_o = kk; }
                if (job == 2) { sa[0] = s4[0]; sa[1] = s4[1]; sa[2] = s4[2]; sa[3] = s4[3]; k_a = kk; }
            }
            const uint32_t nbo = (len_o + 8) / 64 + 1, nba = (len_a + 8) / 64 + 1;
            // finished nodes: entries into the parent's message and the slot arrays
            if (job == 1) {
                if (len_o == 0 || k_o == nbo) {
                    ph_o = 2;
                    const uint64_t slot = t.base[H] + root * 256 + n;
                    if (len_o) {
                        pg_put17(lds + PG_M1 + m1 * PG_MSG + 17u * __builtin_popcount(pm16 & ((1u << d1) - 1u)), 0u, so);
                        (GROUP ? group[gi].md5 : t.md5)[slot] = make_uint4(so[0], so[1], so[2], so[3]);
                    }
                    (GROUP ? group[gi].tag : t.tag)[slot] = len_o ? (uint16_t)TAG_PRESENT : (uint16_t)0;
                } else {
                    ph_o = 1;
                }
            }
            if (job == 2) {
                if (len_a == 0 || k_a == nba) {
                    ph_a = 2;
                    if (aux_h1) {
                        const uint64_t slot = t.base[H - 1] + root * 16 + m1;
                        if (len_a) {
                            pg_put17(lds + PG_M0 + 17u * __builtin_popcount(rootmask & ((1u << m1) - 1u)), 0u, sa);
                            (GROUP ? group[gi].md5 : t.md5)[slot] = make_uint4(sa[0], sa[1], sa[2], sa[3]);
                        }
                        (GROUP ? group[gi].tag : t.tag)[slot] = len_a ? (uint16_t)TAG_PRESENT : (uint16_t)0;
                    }
                } else {
                    ph_a = 1;
                }
            }
            if (STAMP && hi) {
                if (!(stampd & 1) && h1 >= 3) { PG_STAMP(lane == 1, 5); stampd |= 1; }
                if (!(stampd & 2) && __ballot(aux_root && ph_a >= 1)) { PG_STAMP(lane == 1, 6); stampd |= 2; }
                if (!(stampd & 4) && my_h1_done) { PG_STAMP(lane == 1, 7); stampd |= 4; }
            }
            pg_wait_lds();
        }
        // ---- the window root: slot arrays, and the climb hand-off
        if (aux_root) {
            const uint32_t l = H - 2;
            const uint64_t slot = t.base[l] + root;
            const uint4 e = make_uint4(sa[0], sa[1], sa[2], sa[3]);
            const uint32_t tg = len_a ? TAG_PRESENT : 0u;
            if (tg) (GROUP ? group[gi].md5 : t.md5)[slot] = e;
            (GROUP ? group[gi].tag : t.tag)[slot] = (uint16_t)tg;
            if (l == 1) { (GROUP ? group[gi].md5 : t.md5)[0] = e; (GROUP ? group[gi].tag : t.tag)[0] = (uint16_t)tg; }
            PG_STAMP(true, 8);
            uint32_t last = 0;
            if (l > lmin) {
                mail_put(RFT(mail) + slot, e, tg);   // read by the tree's last window
                __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const uint32_t nw = GROUP ? nwin : gridDim.x;
                uint32_t *cp = RFT(cnt);
                const uint32_t old = __hip_atomic_fetch_add(cp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last = old + 1 == nw;
                if (last) {
                    __hip_atomic_store(cp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    PG_STAMP(true, 9);
                }
            }
            CNT[PG_C_LAST] = last;
        }
    }
    __syncthreads();
    // ---- the levels above the windows, by the tree's last window (as in
    // k_rehash_fused): level H-3 from the window roots' mailboxes, then each
    // level from the previous one's outputs in LDS; a lane per node
    if (CNT[PG_C_LAST]) {
        const uint32_t nw = GROUP ? nwin : gridDim.x;
        uint32_t l = H - 3;
        uint64_t nlo = (GROUP ? 0 : root0) >> 4, nn = nw >> 4;
        const uint8_t *ent = lds + PG_CE + (tid & 255) * NB16, *tgs = lds + PG_CT + (tid & 255) * TB16;
        uint8_t *reg = lds + PG_CR + (tid & 255) * PG_MSG;
        auto blk = [&](uint32_t k) { return lds + PG_CB + k * PG_CBSZ; };
        for (uint32_t lev = 0;; lev++) {
            if (tid < nn) {
                const uint64_t b = nlo + tid;
                if (lev == 0) {
                    const uint64_t cc = t.base[l + 1] + b * 16;
                    uint4 h[16];
                    uint16_t g[16];
#pragma unroll
                    for (int j = 0; j < 16; j++) mail_get(RFT(mail) + cc + j, h[j], g[j]);
#pragma unroll
                    for (int j = 0; j < 16; j++) {
                        *reinterpret_cast<uint4 *>(const_cast<uint8_t *>(ent) + j * 16) = h[j];
                        *reinterpret_cast<uint16_t *>(const_cast<uint8_t *>(tgs) + j * 2) = g[j];
                    }
                    PG_STAMP(tid == 0, 10);
                }
                uint4 e;
                uint32_t tg;
                node16_any(reinterpret_cast<const uint4 *>(ent), reinterpret_cast<const uint16_t *>(tgs), reg, e, tg);
                PG_STAMP(tid == 0, lev == 0 ? 11 : 12);
                const uint64_t slot = t.base[l] + b;
                if (tg) (GROUP ? group[gi].md5 : t.md5)[slot] = e;
                (GROUP ? group[gi].tag : t.tag)[slot] = (uint16_t)tg;
                if (l == 1) { (GROUP ? group[gi].md5 : t.md5)[0] = e; (GROUP ? group[gi].tag : t.tag)[0] = (uint16_t)tg; }
                if (l > lmin) {   // the parent's child entry, in the next level's node block
                    uint8_t *nb = blk(lev & 1);
                    *reinterpret_cast<uint4 *>(nb + (tid >> 4) * NB16 + (tid & 15) * 16) = e;
                    *reinterpret_cast<uint16_t *>(nb + 16 * NB16 + (tid >> 4) * TB16 + (tid & 15) * 2) = (uint16_t)tg;
                }
            }
            if (l <= lmin) break;
            __syncthreads();
            l--;
            nlo >>= 4;
            nn = (nn + 15) >> 4;
            ent = blk(lev & 1) + (tid & 15) * NB16;
            tgs = blk(lev & 1) + 16 * NB16 + (tid & 15) * TB16;
        }
    }
    if (STAMP && tid == 0) {
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        PG_STAMP(true, 15);
    }
#undef RFT
#undef PG_STAMP
}
