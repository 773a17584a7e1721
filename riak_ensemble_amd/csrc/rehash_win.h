// rehash_win.h — the fused full rehash (W == 16, 3 <= H <= 6): K1 and every
// inner level in ONE launch (rehash/1 + rehash_upper/1, synctree.erl:489-543).
//
// One workgroup of NW waves per WINDOW = level-(H-2) subtree (4096 segments,
// 64 tiles in window-local block-count order, k_tile_order_window).
//
//  * K1: wave w hashes tiles w, 2NW-1-w, 2NW+w, ... (snake order over the
//    length-sorted tiles) as one flat stream of MD5 blocks, two blocks in
//    flight (ping-pong register buffers).  Each finished segment's entry
//    <<0, MD5:16/binary>> goes straight into its level-H parent's MESSAGE in
//    LDS: 17 bytes at 17 x (rank among the present siblings) -- presence is
//    known before any hashing from the window's segment bitmap (tpres), so
//    the message of every inner node is packed as its children finish, with
//    no separate entry array, tag array or packing pass.
//  * Level H: a lane per node hashes its packed message (md5 of the present
//    children's entries in child order, synctree.erl:255-259, 516-533) and
//    writes its own entry into its parent's message; then level H-1 (16
//    lanes) and the window root (1 lane).  Meanwhile the other waves copy the
//    4096 segment entries to the slot arrays (coalesced, write-through).
//  * Above the windows: the root's entry goes to a mailbox (agent-scope
//    atomics), every window counts itself into one per-tree counter, and the
//    last arriver hashes the upper levels a lane per node, children from the
//    mailboxes, each level packed into LDS messages like the window's.
//
// LDS is 75 KB (the messages of one window's 256 + 16 + 1 inner nodes, the
// presence bitmap), so two 8-wave workgroups fit on a CU: the group rehash of
// many small trees (config 4) runs NW = 8 and overlaps one window's
// latency-bound level chain with another window's K1; a single tree runs
// NW = 16 (one window per CU, every wave in K1).
#pragma once

#define RW_MSG 272                          // one node's message at most: 16 x 17 bytes
// LDS layout for `mhb` bytes of level-H messages (the window's 256 messages
// packed at 4-byte aligned offsets, NOFF; the climb's up to 256 messages at
// RW_MSG stride; the host passes the largest need of the launch's windows):
//   MH [0, mhb + 80)   M1 16 x RW_MSG (the 64 tile descriptors while K1 runs)
//   M0 320   PRES 64 x u64   NOFF 256 x u16 (4-byte units)   MISC 20 x u32
// PRES + NOFF hold the climb's node masks (after the window's levels).
struct RwLayout {
    uint32_t m1, m0, pres, noff, misc, total;
    __host__ __device__ explicit RwLayout(uint32_t mhb) {
        m1 = (mhb + 80 + 15) & ~15u;   // a message's last block may read 72 bytes past its end
        m0 = m1 + 16 * RW_MSG;
        pres = m0 + 320;
        noff = pres + 512;
        misc = noff + 512;
        total = misc + 80;
    }
};
__host__ __device__ __forceinline__ uint32_t fused_lds_bytes(uint32_t mhb) { return RwLayout(mhb).total; }

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// The entry <<Prefix, MD5:16/binary>> at any byte offset of LDS.
__device__ __forceinline__ void rw_put17(uint8_t *p, uint32_t pfx, const uint4 &e) {
    const uint32_t w[4] = {e.x, e.y, e.z, e.w};
    p[0] = (uint8_t)pfx;
#pragma unroll
    for (int i = 0; i < 4; i++) {
#pragma unroll
        for (int b = 0; b < 4; b++) p[1 + 4 * i + b] = (uint8_t)(w[i] >> (8 * b));
    }
}

// 16 bytes at any byte offset of LDS (aligned dword reads + funnel shifts).
__device__ __forceinline__ uint4 rw_get16(const uint8_t *base, uint32_t o) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(base + (o & ~3u));
    const uint32_t sh = (o & 3u) * 8u;
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
    return make_uint4(__builtin_amdgcn_alignbit(w1, w0, sh), __builtin_amdgcn_alignbit(w2, w1, sh),
                      __builtin_amdgcn_alignbit(w3, w2, sh), __builtin_amdgcn_alignbit(w4, w3, sh));
}

// Node (16 children) presence from the window bitmap: segments 16n..16n+15.
__device__ __forceinline__ uint32_t rw_pres16(const uint64_t *pres, uint32_t n) {
    return (uint32_t)(pres[n >> 2] >> (16 * (n & 3))) & 0xffffu;
}
// Children presence of level-(H-1) node m: bit j = level-H node 16m + j has a segment.
__device__ __forceinline__ uint32_t rw_hmask(const uint64_t *pres, uint32_t m) {
    uint32_t r = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint64_t w = pres[4 * m + q];
#pragma unroll
        for (int k = 0; k < 4; k++) r |= (((w >> (16 * k)) & 0xffffu) != 0 ? 1u : 0u) << (4 * q + k);
    }
    return r;
}
// MD5 of a packed node message of `len` bytes in LDS (0 bytes: absent node).
__device__ __forceinline__ void rw_node(const uint8_t *msg, uint32_t len, uint4 &e, uint32_t &tg) {
    e = make_uint4(0, 0, 0, 0);
    tg = 0;
    if (!len) return;
    uint32_t dg[4];
    stmd5::md5_lds_node(msg, len, dg);
    e = make_uint4(dg[0], dg[1], dg[2], dg[3]);
    tg = TAG_PRESENT;
}

// STAMP (diagnostic, ST_LEVEL_STAMPS=1): wall-clock stamps (100 MHz) per
// workgroup at phase boundaries into stamps[blockIdx.x * 32 + k], the shader
// clock (s_memtime) at the same points into [.. + 16 + k] (thread 0's view:
// 0 start, 1 K1 done, 2/4/6 level H/H-1/H-2 hashed, 3/5 level H/H-1 barrier
// passed, 7 mailbox stored, 8 climb counter won, 9 mailboxes read, 10 / 14
// the first / last climb level hashed, 15 exit).
//
// GROUP: the windows of many trees of one geometry in one launch (the
// ensembles one GPU hosts, riak_ensemble_peer.erl:1845-1846): workgroup g
// takes window g % nwin of tree group[g / nwin], each tree with its own slot
// arrays, tiles, counters and mailboxes.
#if defined(__HIP_DEVICE_COMPILE__)
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T *rw_global(T *p) {
    return (__attribute__((address_space(1))) T *)p;
}
#else   // the host pass of device code (address-space-qualified class objects do not copy there)
template <class T>
__device__ __forceinline__ T *rw_global(T *p) {
    return p;
}
#endif
#ifndef RW_K1_TPUT
#define RW_K1_TPUT true   // K1's MD5 in the throughput form (§3.1 cost model)
#endif
template <bool STAMP, bool GROUP, int NW>
__global__ void __launch_bounds__(NW * 64, GROUP ? 6 : 1) k_rehash_fused(DevTree t, TreeTiles tt0, const TreeTiles *__restrict__ group,
                                                          uint32_t nwin, uint64_t root0, uint32_t lmin, uint64_t *stamps,
                                                          uint32_t mhb) {
#define RF_STAMP(k) do { if (STAMP && threadIdx.x == 0) { stamps[blockIdx.x * 32 + (k)] = __builtin_amdgcn_s_memrealtime(); \
                                                          stamps[blockIdx.x * 32 + 16 + (k)] = __builtin_amdgcn_s_memtime(); } } while (0)
    constexpr int NT = 64 / NW;   // tiles per wave
    RF_STAMP(0);
    const uint32_t gi = GROUP ? blockIdx.x / nwin : 0;
    const uint64_t root = GROUP ? (uint64_t)(blockIdx.x - gi * nwin) : root0 + blockIdx.x;
#define RFT(f) (GROUP ? group[gi].f : tt0.f)
    // the group's pointers come from memory, so the compiler cannot tell their
    // address space: as global ones the fetches are global loads, not FLAT
    // (whose waits cover the LDS traffic too)
#define RFG(f) (rw_global(RFT(f)))
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const RwLayout LY(mhb);
    uint8_t *MH = lds;
    uint8_t *M1 = lds + LY.m1;
    uint8_t *M0 = lds + LY.m0;
    uint64_t *PRES = reinterpret_cast<uint64_t *>(lds + LY.pres);
    uint32_t *MISC = reinterpret_cast<uint32_t *>(lds + LY.misc);
    uint16_t *NOFF = reinterpret_cast<uint16_t *>(lds + LY.noff);   // level-H message offsets, 4-byte units
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t H = t.H;
    const uint64_t seg0 = root * 4096;

    // ---- the window's tile descriptors and presence bitmap into LDS
    TileInfo *TI = reinterpret_cast<TileInfo *>(lds + LY.m1);   // M1 is free until level H
    if (tid < 64) {
        TI[tid] = RFG(tinfo)[root * 64 + tid];
        PRES[tid] = RFG(pres)[root * 64 + tid];
        reinterpret_cast<uint64_t *>(NOFF)[tid] = ((const __attribute__((address_space(1))) uint64_t *)(RFG(noff) + root * 256))[tid];
    }
    if (tid < 4) MISC[tid] = 0;
    lds_barrier();
    if (wave == NW - 1) {   // the window's inner-node presence masks, once
        const uint32_t hm = lane < 16 ? rw_hmask(PRES, lane) : 0u;
        const uint32_t rm = (uint32_t)__ballot(lane < 16 && hm != 0) & 0xffffu;
        if (lane < 16) MISC[4 + lane] = hm;
        if (lane == 0) MISC[2] = rm;
    }

    // ---- phase 1: K1.  Wave w hashes its NT tiles (snake order over the
    // length-sorted tiles: w, 2NW-1-w, 2NW+w, ...) as one flat stream of MD5
    // blocks.  A fetch cursor runs two blocks ahead of the hashing; every
    // fetch fills a ping-pong buffer with the block's four 16-B rows AND
    // everything hashing it needs: the lane's message descriptor and segment
    // (per lane), the block index, the tile's block count and stored rows
    // (wave-uniform).  So the hashing keeps no per-tile state, and every fetch
    // issues the same six loads (past the stream: dummies), which lets the
    // compiler count the other buffer's loads as in flight at every wait.
    struct Buf {
        uint4 x0, x1, x2, x3;
        uint32_t ln, li;   // per lane: message length + 1 (0: none), segment index in the window
        uint32_t k, B, R;  // wave-uniform: block in the tile, the tile's blocks and stored rows (B = 0: no block)
    };
    const uint64_t w0 = root * 4096;
    auto tile_of = [&](uint32_t q) { return (uint32_t)(NW * q + ((q & 1) ? NW - 1 - wave : wave)); };
    auto next_q = [&](uint32_t q) {
        while (q < NT && __builtin_amdgcn_readfirstlane(TI[tile_of(q)].B) == 0) q++;
        return q;
    };
    uint32_t T = 0;   // blocks in the wave's stream
    for (uint32_t q = 0; q < NT; q++) T += __builtin_amdgcn_readfirstlane(TI[tile_of(q)].B);
    uint32_t fq = next_q(0), fk = 0, fB = 0, fR = 0, fL = 0, ft = tile_of(0);
    uint64_t fbase = 0;
    auto fload = [&](uint32_t q) {
        ft = tile_of(q);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)TI[ft].base),
                       hi = __builtin_amdgcn_readfirstlane((uint32_t)(TI[ft].base >> 32));
        fbase = ((uint64_t)hi << 32) | lo;
        fB = __builtin_amdgcn_readfirstlane(TI[ft].B);
        fR = __builtin_amdgcn_readfirstlane(TI[ft].R);
        fL = fR ? fR - 1 : 0;   // the last stored row (fetch clamp)
    };
    if (fq < NT) fload(fq);
    auto fetch = [&](Buf &b) {
        const uint32_t r = 4 * fk, last = fL;
        const auto p = RFG(tiles) + fbase;
        b.x0 = (p + (uint64_t)(r < last ? r : last) * 64)[lane];
        b.x1 = (p + (uint64_t)(r + 1 < last ? r + 1 : last) * 64)[lane];
        b.x2 = (p + (uint64_t)(r + 2 < last ? r + 2 : last) * 64)[lane];
        b.x3 = (p + (uint64_t)(r + 3 < last ? r + 3 : last) * 64)[lane];
        b.ln = RFG(tln)[w0 + ft * 64 + lane];
        b.li = (uint32_t)(RFG(tseg)[w0 + ft * 64 + lane] - seg0);
        b.k = fk;
        b.B = fq < NT ? fB : 0u;
        b.R = fR;
        if (fq >= NT) return;   // past the stream: a dummy fetch (the fixed load pattern)
        if (++fk == fB) {
            fk = 0;
            fq = next_q(fq + 1);
            if (fq < NT) fload(fq);
        }
    };
    // a segment's entry into its parent's message (absent segments: nothing)
    auto put_entry = [&](uint32_t li, const uint32_t st[4]) {
        const uint32_t n = li >> 4, j = li & 15;
        const uint32_t o = 4u * NOFF[n] + 17u * __builtin_popcount(rw_pres16(PRES, n) & ((1u << j) - 1u));
        rw_put17(MH + o, 0u, make_uint4(st[0], st[1], st[2], st[3]));
    };
    {
        Buf A, Bf;
        fetch(A);
        fetch(Bf);
        uint32_t st[4];
        stmd5::init(st);
        auto hash_block = [&](const Buf &b) {
            if (b.B == 0) return;
            const uint32_t r = 4 * b.k, nb = ln_blocks(b.ln);
            if (r + 3 >= b.R) {   // rows past the stored ones (a tile's last block or two)
                const uint4 y0 = r >= b.R ? tile_synth(r, b.ln) : b.x0, y1 = r + 1 >= b.R ? tile_synth(r + 1, b.ln) : b.x1,
                            y2 = r + 2 >= b.R ? tile_synth(r + 2, b.ln) : b.x2, y3 = tile_synth(r + 3, b.ln);
                const uint32_t m[16] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w,
                                        y2.x, y2.y, y2.z, y2.w, y3.x, y3.y, y3.z, y3.w};
                if (b.k < nb) stmd5::compress<RW_K1_TPUT>(st, m);
            } else {             // the common case: the loaded registers feed the compression as they are
                const uint32_t m[16] = {b.x0.x, b.x0.y, b.x0.z, b.x0.w, b.x1.x, b.x1.y, b.x1.z, b.x1.w,
                                        b.x2.x, b.x2.y, b.x2.z, b.x2.w, b.x3.x, b.x3.y, b.x3.z, b.x3.w};
                if (b.k < nb) stmd5::compress<RW_K1_TPUT>(st, m);
            }
            if (b.k + 1 == b.B) {
                if (nb) put_entry(b.li, st);
                stmd5::init(st);
            }
        };
        for (uint32_t f = 0; f < T; f += 2) {
            hash_block(A);
            fetch(A);
            if (f + 1 < T) hash_block(Bf);
            fetch(Bf);
        }
    }
    lds_barrier();
    RF_STAMP(1);

    // ---- phase 2: the window's segment entries to the slot arrays, coalesced,
    // by waves 4.. while waves 0..3 hash level H from the same LDS.  The md5
    // words go out WRITE-THROUGH (sc1 buffer stores): the lines leave the
    // XCD's L2 during the launch instead of being written back, dirty, at its
    // end.  Absent segments: tag 0, md5 0.
    if (tid >= 256) {
        const uint64_t c0 = t.base[H + 1] + seg0;
        const uint64_t nbytes = (t.base[H + 1] + t.S) * 16;
        const __amdgpu_buffer_rsrc_t md5r = __builtin_amdgcn_make_buffer_rsrc(
            GROUP ? group[gi].md5 : t.md5, (short)0, (int)(nbytes < 0xffffffffull ? nbytes : 0xffffffffull), 0x00020000);
        const auto tagp = rw_global(GROUP ? group[gi].tag : t.tag);
        for (uint32_t i = tid - 256; i < 4096; i += NW * 64 - 256) {
            const uint32_t n = i >> 4, j = i & 15, p16 = rw_pres16(PRES, n);
            uint4 e = make_uint4(0, 0, 0, 0);
            uint16_t tg = 0;
            if ((p16 >> j) & 1u) {
                e = rw_get16(MH, 4u * NOFF[n] + 17u * __builtin_popcount(p16 & ((1u << j) - 1u)) + 1u);
                tg = (uint16_t)TAG_PRESENT;
            }
            const u32x4 v = {e.x, e.y, e.z, e.w};
            __builtin_amdgcn_raw_buffer_store_b128(v, md5r, (int)((c0 + i) * 16), 0, 16 /* sc1 */);
            tagp[c0 + i] = tg;
        }
    }

    // ---- phase 3: the inner levels, ONE loop with one node-hash call site
    // (the unrolled MD5 stays hot in the instruction cache): levels H, H-1,
    // H-2 of the window from its packed messages (256, 16, 1 lanes); then, in
    // the tree's last window only, the levels above (H-3 .. lmin), level H-3
    // from the window roots' mailboxes, each level above from the previous
    // one's packed messages, a lane per node.
    const uint32_t nwt = GROUP ? nwin : gridDim.x;   // this launch's windows of the tree
    uint32_t l = H, ph = 0;                          // level; phase 0..2 window levels, 3.. climb levels
    uint64_t nlo = 0, nn = 0;                        // climb: this level's nodes [nlo, nlo + nn)
    bool act = tid < 256;
    for (;;) {
        uint4 e = make_uint4(0, 0, 0, 0);
        uint32_t tg = 0;
        if (act) {
            const uint8_t *msg;
            uint32_t len;
            uint64_t b;
            if (ph == 0) { msg = MH + 4u * NOFF[tid]; len = 17u * __builtin_popcount(rw_pres16(PRES, tid)); b = root * 256 + tid; }
            else if (ph == 1) { msg = M1 + tid * RW_MSG; len = 17u * __builtin_popcount(MISC[4 + tid]); b = root * 16 + tid; }
            else if (ph == 2) { msg = M0; len = 17u * __builtin_popcount(MISC[2]); b = root; }
            else {
                msg = (ph == 3 ? MH : ph == 4 ? M1 : M0) + tid * RW_MSG;
                len = 17u * __builtin_popcount(reinterpret_cast<const uint32_t *>(lds + LY.pres)[tid]);
                b = nlo + tid;
            }
            rw_node(msg, len, e, tg);
            RF_STAMP(ph == 0 ? 2 : ph == 1 ? 4 : ph == 2 ? 6 : ph == 3 ? 10 : 14);
            const uint64_t slot = t.base[l] + b;
            if (tg) rw_global(GROUP ? group[gi].md5 : t.md5)[slot] = e;
            rw_global(GROUP ? group[gi].tag : t.tag)[slot] = (uint16_t)tg;
            if (l == 1) { rw_global(GROUP ? group[gi].md5 : t.md5)[0] = e; rw_global(GROUP ? group[gi].tag : t.tag)[0] = (uint16_t)tg; }
        }
        // a group stops after level H: the levels above, every tree's nodes of
        // a level at once, are k_level16_group's (the window's 16- and 1-lane
        // chains held its LDS and its place on the CU for ~13 us)
        if (GROUP) break;
        if (l <= lmin) break;
        if (ph == 0) {          // level-H entries into the H-1 messages
            if (act && tg) {
                const uint32_t m = tid >> 4, j = tid & 15;
                rw_put17(M1 + m * RW_MSG + 17u * __builtin_popcount(MISC[4 + m] & ((1u << j) - 1u)), 0u, e);
            }
            // waves 0..3 meet through an LDS counter, not a workgroup barrier:
            // the copy-out waves go on (they meet the others at the root)
            if (tid < 256) {
                __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (lane == 0) __hip_atomic_fetch_add(&MISC[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (wave == 0)
                while (__hip_atomic_load(&MISC[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 4u) __builtin_amdgcn_s_sleep(1);
            RF_STAMP(3);
            act = tid < 16;
        } else if (ph == 1) {   // H-1 entries into the root's message (one wave: no barrier)
            if (act && tg) rw_put17(M0 + 17u * __builtin_popcount(MISC[2] & ((1u << tid) - 1u)), 0u, e);
            __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            RF_STAMP(5);
            act = tid == 0;
        } else if (ph == 2) {   // the window root: mailbox, counter; the last window climbs
            if (tid == 0) {
                const uint64_t slot = t.base[l] + root;
                if (root != RFT(skip_root)) mail_put(RFT(mail) + slot, e, tg, RFT(epoch));   // read by the tree's last window
                // this window's mailbox stores have completed (agent-coherent)
                // before the counter moves; no L2 write-back / invalidate
                __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
                RF_STAMP(7);
                uint32_t *c = RFT(cnt);
                const uint32_t old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                MISC[0] = old + 1 == nwt;
                if (old + 1 == nwt) {
                    __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    RF_STAMP(8);
                }
            }
            __syncthreads();
            if (!MISC[0]) break;
            nlo = (GROUP ? 0 : root0) >> 4;
            nn = nwt >> 4;
            // level H-3: the children are the window roots, from their
            // mailboxes: 16 lanes per node read one mailbox each (one round
            // trip, 5 registers a lane) and place the entry at its rank in the
            // node's message; the node's presence mask goes to CLM
            uint32_t *CLM = reinterpret_cast<uint32_t *>(lds + LY.pres);   // climb masks (PRES and NOFF are dead)
            for (uint64_t c0 = 0; c0 < nn * 16; c0 += NW * 64) {
                const uint64_t ci = c0 + tid;   // child ci % 16 of this level's node ci / 16
                uint4 h = make_uint4(0, 0, 0, 0);
                uint16_t g = 0;
                if (ci < nn * 16 && !mail_get(RFT(mail) + t.base[l] + nlo * 16 + ci, h, g, RFT(epoch)))
                    raise_derr(RFT(err), ST_DERR_MAIL);
                const unsigned long long pb = __ballot(ci < nn * 16 && (g & TAG_PRESENT));
                const uint32_t sib = (uint32_t)(pb >> (16 * ((tid & 63) >> 4))) & 0xffffu, j = tid & 15;
                if (g & TAG_PRESENT) rw_put17(MH + (ci >> 4) * RW_MSG + 17u * __builtin_popcount(sib & ((1u << j) - 1u)), g & 0xffu, h);
                if (ci < nn * 16 && j == 0) CLM[ci >> 4] = sib;
            }
            lds_barrier();
            act = tid < nn;
            RF_STAMP(9);
        } else {                // climb: entries into the next level's messages (siblings are lanes of one wave)
            const unsigned long long pb = __ballot(act && tg != 0);
            const uint32_t sib = (uint32_t)(pb >> (16 * ((tid & 63) >> 4))) & 0xffffu;
            __syncthreads();   // every lane has read this level's masks and messages
            if (act) {
                const uint32_t j = tid & 15;
                if (tg) rw_put17((ph == 3 ? M1 : M0) + (tid >> 4) * RW_MSG + 17u * __builtin_popcount(sib & ((1u << j) - 1u)), 0u, e);
                if (j == 0) reinterpret_cast<uint32_t *>(lds + LY.pres)[tid >> 4] = sib;
            }
            __syncthreads();
            nlo >>= 4;
            nn = (nn + 15) >> 4;
            act = tid < nn;
        }
        ph++;
        l--;
    }
    if (STAMP && tid == 0) {
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        RF_STAMP(15);
    }
#undef RFT
#undef RF_STAMP
}

// The levels above level H of a group rehash (st_rehash_group: its fused
// launch stops after level H): level l of every tree of the group in one
// launch, a lane per node, node i of the launch = tree i / nper, node i % nper
// of the level.  A node with all 16 children present (nearly every node of
// these levels) hashes from registers (md5_node16); the others stage their
// packed message in one of 16 LDS regions the wave's partial nodes take in
// turns, so a 64-lane workgroup holds 5.6 KB of LDS, not 22 KB (which had
// capped the launch at 7 waves a CU).
#define LG_REGIONS 16
__host__ __device__ __forceinline__ uint32_t level16_group_lds_bytes() { return LG_REGIONS * lane_region_bytes(16); }
__global__ void __launch_bounds__(64) k_level16_group(DevTree t0, const TreeTiles *__restrict__ group, uint32_t ntrees,
                                                      uint32_t l) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nper = t0.base[l + 1] - t0.base[l];
    const uint64_t total = nper * ntrees;
    for (uint64_t i0 = (uint64_t)blockIdx.x * 64; i0 < total; i0 += (uint64_t)gridDim.x * 64) {   // wave-uniform
        const uint64_t i = i0 + lane;
        const bool valid = i < total;
        const uint32_t gi = valid ? (uint32_t)(i / nper) : 0u;
        const uint64_t b = valid ? i - (uint64_t)gi * nper : 0;
        uint4 ST_GAS *md5 = rw_global(group[gi].md5);
        uint16_t ST_GAS *tag = rw_global(group[gi].tag);
        const uint64_t slot = t0.base[l] + b, c0 = t0.base[l + 1] + b * 16;
        uint32_t tg[16];
        uint4 h[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            tg[j] = valid ? tag[c0 + j] : 0u;
            h[j] = valid ? md5[c0 + j] : make_uint4(0u, 0u, 0u, 0u);
        }
        uint32_t full = valid ? 1u : 0u;
#pragma unroll
        for (int j = 0; j < 16; j++) full &= (tg[j] >> 8) & 1u;
        uint32_t dg[4] = {0u, 0u, 0u, 0u};
        uint32_t len = 0;
        if (full) {
            uint32_t pf[16];
#pragma unroll
            for (int j = 0; j < 16; j++) pf[j] = tg[j] & 0xffu;
            stmd5::md5_node16<true, true>(pf, h, dg);
            len = 1;
        }
        // the partial nodes, 16 at a time through the shared regions (their
        // children loaded again: the registers above are free by then)
        const uint64_t pm = __ballot(valid && !full);
        const uint32_t rank = __builtin_popcountll(pm & ((1ull << lane) - 1ull));
        const uint32_t np = __builtin_popcountll(pm);
        for (uint32_t r0 = 0; r0 < np; r0 += LG_REGIONS) {
            if (valid && !full && rank >= r0 && rank < r0 + LG_REGIONS) {
                uint8_t *reg = lds + (rank - r0) * lane_region_bytes(16);
                MsgWriter mw;
                mw.init(reg);
                for (int j = 0; j < 16; j++) {
                    const uint32_t g = tag[c0 + j];
                    if (g & TAG_PRESENT) mw.entry(g, md5[c0 + j]);
                }
                len = mw.finish();
                if (len) stmd5::md5_lds(reg, len, dg);
            }
            __builtin_amdgcn_wave_barrier();   // the regions are reused by the next 16
        }
        if (valid) {
            uint32_t ot = 0;
            uint4 e = make_uint4(0u, 0u, 0u, 0u);
            if (len) {
                e = make_uint4(dg[0], dg[1], dg[2], dg[3]);
                ot = TAG_PRESENT;
                md5[slot] = e;
            }
            tag[slot] = (uint16_t)ot;
            if (l == 1) { md5[0] = e; tag[0] = (uint16_t)ot; }
        }
    }
}
