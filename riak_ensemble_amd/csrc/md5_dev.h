// md5_dev.h — RFC 1321 MD5 for gfx950 (one message per lane).
//
// The reference hashes with OTP `crypto:hash(md5, IoList)` (src/synctree.erl:
// 252, 258): segment ids from md5(ensure_binary(Key)) and node hashes from the
// md5 of the concatenated child values.  MD5 is serial within a message, so
// the device parallelism is across messages: every lane owns one message.
//
// Codegen notes (check the .s with -save-temps):
//  * rotl(x, s) is __builtin_amdgcn_alignbit(x, x, 32 - s)   -> v_alignbit_b32
//  * F, G, H, I are one v_bitop3_b32 each (__builtin_amdgcn_bitop3_b32)
//  * (a + M + K) + F                                        -> v_add3_u32 + v_add_u32
//  so a step is 5 VALU ops, 14 SIMD cycles per wave64 (add / bitop3 2,
//  add3 / alignbit 4, measured: profiles/r01_valu_peak.txt); a 64-byte block
//  ~916 SIMD cycles (k_segment_hash_tiled's loop, ISA count).
//  * message blocks from global memory are fetched with four unaligned
//    global_load_dwordx4 (gfx950 runs with unaligned access enabled; hipcc
//    emits the wide loads for byte pointers) — no shuffling in registers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace stmd5 {

__device__ __forceinline__ uint32_t rotl(uint32_t x, int s) { return __builtin_amdgcn_alignbit(x, x, 32 - s); }

// The four round functions as single v_bitop3_b32 (gfx950): truth tables
// over (b, c, d) = (0xF0, 0xCC, 0xAA).  Written as plain and/or/xor the
// compiler splits F and G into and + andn + two adds (18 SIMD cycles a
// step instead of 14).
#define STMD5_F(b, c, d) __builtin_amdgcn_bitop3_b32((b), (c), (d), 0xCA)   // (b & c) | (~b & d)
#define STMD5_G(b, c, d) __builtin_amdgcn_bitop3_b32((b), (c), (d), 0xE4)   // (b & d) | (c & ~d)
#define STMD5_H(b, c, d) __builtin_amdgcn_bitop3_b32((b), (c), (d), 0x96)   // b ^ c ^ d
#define STMD5_I(b, c, d) __builtin_amdgcn_bitop3_b32((b), (c), (d), 0x39)   // c ^ (b | ~d)
#define STMD5_STEP_L(f, a, b, c, d, m, k, s) a = (b) + rotl(((a) + (m) + (k)) + f((b), (c), (d)), (s))

// Throughput form of a step: ((a + K) + M) + F as three v_add_u32 (K as the
// 32-bit literal of a VOP2 add) instead of v_add_u32 + v_add3_u32 (the
// compiler fuses a three-term sum into add3).  On gfx950 a SIMD running >= 2
// waves of MD5 issues this mix ~40 % faster (tools/microbench/md5_variants.cpp
// V9: 149 vs 106 G lane-blocks/s at 16 waves/CU), while a lone wave's
// dependent chain is ~35 % slower (0.77 vs 0.58 us per block).  Hence two forms:
// compress<true> for the bulk segment hashing (K1, 16 waves per CU), the
// default for the latency-bound inner-node chains.
__device__ __forceinline__ uint32_t vadd(uint32_t x, uint32_t y) {
    uint32_t r;
    asm("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}
__device__ __forceinline__ uint32_t vaddk(uint32_t x, uint32_t k) {
    uint32_t r;
    asm("v_add_u32 %0, %2, %1" : "=v"(r) : "v"(x), "i"(k));
    return r;
}
#define STMD5_STEP_T(f, a, b, c, d, m, k, s) a = (b) + rotl(vadd(vadd(vaddk((a), (k)), (m)), f((b), (c), (d))), (s))
#define STMD5_STEP(f, a, b, c, d, m, k, s)                     \
    do {                                                       \
        if (TPUT) STMD5_STEP_T(f, a, b, c, d, m, k, s);        \
        else STMD5_STEP_L(f, a, b, c, d, m, k, s);             \
    } while (0)

__device__ __forceinline__ void init(uint32_t s[4]) {
    s[0] = 0x67452301u; s[1] = 0xefcdab89u; s[2] = 0x98badcfeu; s[3] = 0x10325476u;
}

template <bool TPUT = false>
__device__ __forceinline__ void compress(uint32_t st[4], const uint32_t m[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    STMD5_STEP(STMD5_F, a, b, c, d, m[0], 0xd76aa478u, 7);
    STMD5_STEP(STMD5_F, d, a, b, c, m[1], 0xe8c7b756u, 12);
    STMD5_STEP(STMD5_F, c, d, a, b, m[2], 0x242070dbu, 17);
    STMD5_STEP(STMD5_F, b, c, d, a, m[3], 0xc1bdceeeu, 22);
    STMD5_STEP(STMD5_F, a, b, c, d, m[4], 0xf57c0fafu, 7);
    STMD5_STEP(STMD5_F, d, a, b, c, m[5], 0x4787c62au, 12);
    STMD5_STEP(STMD5_F, c, d, a, b, m[6], 0xa8304613u, 17);
    STMD5_STEP(STMD5_F, b, c, d, a, m[7], 0xfd469501u, 22);
    STMD5_STEP(STMD5_F, a, b, c, d, m[8], 0x698098d8u, 7);
    STMD5_STEP(STMD5_F, d, a, b, c, m[9], 0x8b44f7afu, 12);
    STMD5_STEP(STMD5_F, c, d, a, b, m[10], 0xffff5bb1u, 17);
    STMD5_STEP(STMD5_F, b, c, d, a, m[11], 0x895cd7beu, 22);
    STMD5_STEP(STMD5_F, a, b, c, d, m[12], 0x6b901122u, 7);
    STMD5_STEP(STMD5_F, d, a, b, c, m[13], 0xfd987193u, 12);
    STMD5_STEP(STMD5_F, c, d, a, b, m[14], 0xa679438eu, 17);
    STMD5_STEP(STMD5_F, b, c, d, a, m[15], 0x49b40821u, 22);
    STMD5_STEP(STMD5_G, a, b, c, d, m[1], 0xf61e2562u, 5);
    STMD5_STEP(STMD5_G, d, a, b, c, m[6], 0xc040b340u, 9);
    STMD5_STEP(STMD5_G, c, d, a, b, m[11], 0x265e5a51u, 14);
    STMD5_STEP(STMD5_G, b, c, d, a, m[0], 0xe9b6c7aau, 20);
    STMD5_STEP(STMD5_G, a, b, c, d, m[5], 0xd62f105du, 5);
    STMD5_STEP(STMD5_G, d, a, b, c, m[10], 0x02441453u, 9);
    STMD5_STEP(STMD5_G, c, d, a, b, m[15], 0xd8a1e681u, 14);
    STMD5_STEP(STMD5_G, b, c, d, a, m[4], 0xe7d3fbc8u, 20);
    STMD5_STEP(STMD5_G, a, b, c, d, m[9], 0x21e1cde6u, 5);
    STMD5_STEP(STMD5_G, d, a, b, c, m[14], 0xc33707d6u, 9);
    STMD5_STEP(STMD5_G, c, d, a, b, m[3], 0xf4d50d87u, 14);
    STMD5_STEP(STMD5_G, b, c, d, a, m[8], 0x455a14edu, 20);
    STMD5_STEP(STMD5_G, a, b, c, d, m[13], 0xa9e3e905u, 5);
    STMD5_STEP(STMD5_G, d, a, b, c, m[2], 0xfcefa3f8u, 9);
    STMD5_STEP(STMD5_G, c, d, a, b, m[7], 0x676f02d9u, 14);
    STMD5_STEP(STMD5_G, b, c, d, a, m[12], 0x8d2a4c8au, 20);
    STMD5_STEP(STMD5_H, a, b, c, d, m[5], 0xfffa3942u, 4);
    STMD5_STEP(STMD5_H, d, a, b, c, m[8], 0x8771f681u, 11);
    STMD5_STEP(STMD5_H, c, d, a, b, m[11], 0x6d9d6122u, 16);
    STMD5_STEP(STMD5_H, b, c, d, a, m[14], 0xfde5380cu, 23);
    STMD5_STEP(STMD5_H, a, b, c, d, m[1], 0xa4beea44u, 4);
    STMD5_STEP(STMD5_H, d, a, b, c, m[4], 0x4bdecfa9u, 11);
    STMD5_STEP(STMD5_H, c, d, a, b, m[7], 0xf6bb4b60u, 16);
    STMD5_STEP(STMD5_H, b, c, d, a, m[10], 0xbebfbc70u, 23);
    STMD5_STEP(STMD5_H, a, b, c, d, m[13], 0x289b7ec6u, 4);
    STMD5_STEP(STMD5_H, d, a, b, c, m[0], 0xeaa127fau, 11);
    STMD5_STEP(STMD5_H, c, d, a, b, m[3], 0xd4ef3085u, 16);
    STMD5_STEP(STMD5_H, b, c, d, a, m[6], 0x04881d05u, 23);
    STMD5_STEP(STMD5_H, a, b, c, d, m[9], 0xd9d4d039u, 4);
    STMD5_STEP(STMD5_H, d, a, b, c, m[12], 0xe6db99e5u, 11);
    STMD5_STEP(STMD5_H, c, d, a, b, m[15], 0x1fa27cf8u, 16);
    STMD5_STEP(STMD5_H, b, c, d, a, m[2], 0xc4ac5665u, 23);
    STMD5_STEP(STMD5_I, a, b, c, d, m[0], 0xf4292244u, 6);
    STMD5_STEP(STMD5_I, d, a, b, c, m[7], 0x432aff97u, 10);
    STMD5_STEP(STMD5_I, c, d, a, b, m[14], 0xab9423a7u, 15);
    STMD5_STEP(STMD5_I, b, c, d, a, m[5], 0xfc93a039u, 21);
    STMD5_STEP(STMD5_I, a, b, c, d, m[12], 0x655b59c3u, 6);
    STMD5_STEP(STMD5_I, d, a, b, c, m[3], 0x8f0ccc92u, 10);
    STMD5_STEP(STMD5_I, c, d, a, b, m[10], 0xffeff47du, 15);
    STMD5_STEP(STMD5_I, b, c, d, a, m[1], 0x85845dd1u, 21);
    STMD5_STEP(STMD5_I, a, b, c, d, m[8], 0x6fa87e4fu, 6);
    STMD5_STEP(STMD5_I, d, a, b, c, m[15], 0xfe2ce6e0u, 10);
    STMD5_STEP(STMD5_I, c, d, a, b, m[6], 0xa3014314u, 15);
    STMD5_STEP(STMD5_I, b, c, d, a, m[13], 0x4e0811a1u, 21);
    STMD5_STEP(STMD5_I, a, b, c, d, m[4], 0xf7537e82u, 6);
    STMD5_STEP(STMD5_I, d, a, b, c, m[11], 0xbd3af235u, 10);
    STMD5_STEP(STMD5_I, c, d, a, b, m[2], 0x2ad7d2bbu, 15);
    STMD5_STEP(STMD5_I, b, c, d, a, m[9], 0xeb86d391u, 21);
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
}

// The latency form as ONE out-of-line copy per kernel (STMD5_NOINLINE=1): the
// per-key and compare kernels run their MD5 chains once per launch on a cold
// instruction cache, and every inlined compression is ~2.5 KB of code
// (k_small carried 11 copies, k_cmp_walk 8).  Twenty scalar arguments and a
// four-word result stay in registers (the AMDGPU calling convention passes up
// to 32 VGPR arguments); the call costs ~30 instructions a block.  Measured
// again in round 5 the smaller code did not pay: the inline form is the
// default.
struct St4 { uint32_t a, b, c, d; };
__device__ __noinline__ St4 compress_ool(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t m0, uint32_t m1,
                                         uint32_t m2, uint32_t m3, uint32_t m4, uint32_t m5, uint32_t m6, uint32_t m7,
                                         uint32_t m8, uint32_t m9, uint32_t m10, uint32_t m11, uint32_t m12,
                                         uint32_t m13, uint32_t m14, uint32_t m15) {
    uint32_t st[4] = {a, b, c, d};
    const uint32_t m[16] = {m0, m1, m2, m3, m4, m5, m6, m7, m8, m9, m10, m11, m12, m13, m14, m15};
    compress(st, m);
    return St4{st[0], st[1], st[2], st[3]};
}
#ifndef STMD5_NOINLINE
#define STMD5_NOINLINE 0   // round 5 A/B (tools/ab_latency.sh): inline is no slower -- insert1 kernel 34.3 vs 34.8 us, k_cmp_walk 43.6 vs 45.3 us
#endif
__device__ __forceinline__ void compress_lat(uint32_t st[4], const uint32_t m[16]) {
#if STMD5_NOINLINE
    const St4 r = compress_ool(st[0], st[1], st[2], st[3], m[0], m[1], m[2], m[3], m[4], m[5], m[6], m[7], m[8], m[9], m[10],
                               m[11], m[12], m[13], m[14], m[15]);
    st[0] = r.a; st[1] = r.b; st[2] = r.c; st[3] = r.d;
#else
    compress(st, m);
#endif
}

// Keep the `valid` leading bytes of little-endian word w (0..4 valid), put
// the 0x80 terminator right after them when they end inside this word.
// Branch-free (selects only): lanes of a wave hold messages of different
// lengths, and a per-lane branch per word would run every path.
__device__ __forceinline__ uint32_t tail_word(uint32_t w, int valid) {
    const int v = valid < 0 ? -1 : (valid > 4 ? 4 : valid);
    const uint32_t n = v < 0 ? 0u : (uint32_t)v;                    // bytes kept, 0..4
    const uint32_t keep = (uint32_t)(0xffffffffull >> (32 - 8 * n));
    const uint32_t term = (v >= 0 && v < 4) ? (0x80u << (8 * n)) : 0u;
    return (w & keep) | term;
}

// Apply MD5 padding to block k of a `len`-byte message whose raw words
// (possibly garbage beyond len) are in m[].  rem = len - 64k.
__device__ __forceinline__ void pad_block(uint32_t m[16], int64_t rem, bool last, uint64_t len) {
#pragma unroll
    for (int w = 0; w < 16; w++) {
        int64_t v = rem - 4 * w;
        m[w] = tail_word(m[w], v > 4 ? 4 : (int)v);
    }
    if (last) {
        m[14] = (uint32_t)(len << 3);
        m[15] = (uint32_t)(len >> 29);
    }
}

// compress_lat with the MD5 padding of block k of a `len`-byte message applied
// first (rem = len - 64k; a no-op for rem >= 64): the padding's selects live
// in the one out-of-line copy too.
__device__ __noinline__ St4 compress_pad_ool(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t m0, uint32_t m1,
                                             uint32_t m2, uint32_t m3, uint32_t m4, uint32_t m5, uint32_t m6, uint32_t m7,
                                             uint32_t m8, uint32_t m9, uint32_t m10, uint32_t m11, uint32_t m12,
                                             uint32_t m13, uint32_t m14, uint32_t m15, int32_t rem, uint32_t last,
                                             uint32_t len_lo, uint32_t len_hi) {
    uint32_t st[4] = {a, b, c, d};
    uint32_t m[16] = {m0, m1, m2, m3, m4, m5, m6, m7, m8, m9, m10, m11, m12, m13, m14, m15};
    if (rem < 64) pad_block(m, rem, last != 0, ((uint64_t)len_hi << 32) | len_lo);
    compress(st, m);
    return St4{st[0], st[1], st[2], st[3]};
}
__device__ __forceinline__ void compress_pad_lat(uint32_t st[4], uint32_t m[16], int64_t rem, bool last, uint64_t len) {
#if STMD5_NOINLINE
    const int32_t r = rem > 64 ? 64 : (int32_t)rem;
    const St4 x = compress_pad_ool(st[0], st[1], st[2], st[3], m[0], m[1], m[2], m[3], m[4], m[5], m[6], m[7], m[8], m[9],
                                   m[10], m[11], m[12], m[13], m[14], m[15], r, last ? 1u : 0u, (uint32_t)len,
                                   (uint32_t)(len >> 32));
    st[0] = x.a; st[1] = x.b; st[2] = x.c; st[3] = x.d;
#else
    if (rem < 64) pad_block(m, rem, last, len);
    compress(st, m);
#endif
}

__device__ __forceinline__ void load_block_global(const uint8_t *p, uint32_t m[16]) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
        uint4 v;
        __builtin_memcpy(&v, p + 16 * q, 16);
        m[4 * q + 0] = v.x; m[4 * q + 1] = v.y; m[4 * q + 2] = v.z; m[4 * q + 3] = v.w;
    }
}

// MD5 of p[0..len) in global memory, any alignment.  The buffer must stay
// readable for 64 bytes past p+len (heaps are allocated with slack).
__device__ __forceinline__ void md5_global(const uint8_t *p, uint64_t len, uint32_t out[4]) {
    uint32_t st[4];
    init(st);
    const uint64_t nblk = (len + 8) / 64 + 1;
    for (uint64_t k = 0; k < nblk; k++) {
        uint32_t m[16];
        const int64_t rem = (int64_t)len - (int64_t)(64 * k);
        if (rem >= 64) {
            load_block_global(p + 64 * k, m);
        } else {
            if (rem > 0) {
                load_block_global(p + 64 * k, m);
            } else {
#pragma unroll
                for (int w = 0; w < 16; w++) m[w] = 0u;
            }
            pad_block(m, rem, k + 1 == nblk, len);
        }
        compress_lat(st, m);
    }
    out[0] = st[0]; out[1] = st[1]; out[2] = st[2]; out[3] = st[3];
}

// Same, with the next block's loads issued before the current block is
// compressed (software pipelining: the loads' latency hides under ~330 VALU
// ops of the compression).
template <bool TPUT = false>
__device__ __forceinline__ void md5_global_pf(const uint8_t *p, uint64_t len, uint32_t out[4]) {
    uint32_t st[4];
    init(st);
    const uint64_t nblk = (len + 8) / 64 + 1;
    uint32_t nx[16];
#pragma unroll
    for (int w = 0; w < 16; w++) nx[w] = 0u;
    if (len > 0) load_block_global(p, nx);
    for (uint64_t k = 0; k < nblk; k++) {
        uint32_t m[16];
#pragma unroll
        for (int w = 0; w < 16; w++) m[w] = nx[w];
        const int64_t rem = (int64_t)len - (int64_t)(64 * k);
        if (rem - 64 > 0) load_block_global(p + 64 * (k + 1), nx);
        if (TPUT) {
            if (rem < 64) pad_block(m, rem, k + 1 == nblk, len);
            compress<true>(st, m);
        } else {
            compress_pad_lat(st, m, rem, k + 1 == nblk, len);
        }
    }
    out[0] = st[0]; out[1] = st[1]; out[2] = st[2]; out[3] = st[3];
}

// md5_global_pf from block k0 on (st = the state after blocks [0, k0), the
// message still `len` bytes from p); when cap_k is one of the blocks
// visited, the state before it is copied to cap.  The streaming insert
// saves the state before the first block a merge changes while it verifies
// the old segment, and resumes from there to hash the merged one.
template <bool TPUT>
__device__ __forceinline__ void md5_global_span(const uint8_t *p, uint64_t len, uint64_t k0, uint32_t st[4],
                                                uint64_t cap_k, uint32_t cap[4]) {
    const uint64_t nblk = (len + 8) / 64 + 1;
    uint32_t nx[16];
#pragma unroll
    for (int w = 0; w < 16; w++) nx[w] = 0u;
    if (len > 64 * k0) load_block_global(p + 64 * k0, nx);
    for (uint64_t k = k0; k < nblk; k++) {
        if (k == cap_k) { cap[0] = st[0]; cap[1] = st[1]; cap[2] = st[2]; cap[3] = st[3]; }
        uint32_t m[16];
#pragma unroll
        for (int w = 0; w < 16; w++) m[w] = nx[w];
        const int64_t rem = (int64_t)len - (int64_t)(64 * k);
        if (rem - 64 > 0) load_block_global(p + 64 * (k + 1), nx);
        if (TPUT) {
            if (rem < 64) pad_block(m, rem, k + 1 == nblk, len);
            compress<true>(st, m);
        } else {
            compress_pad_lat(st, m, rem, k + 1 == nblk, len);
        }
    }
}

// MD5 of a message of `len` bytes staged in LDS at a 4-byte aligned address
// (bytes beyond len are ignored; the region must be readable up to the next
// 64-byte boundary past len).  Next block's words are read before the
// current block is compressed.
__device__ __forceinline__ void md5_lds(const uint8_t *p, uint32_t len, uint32_t out[4]) {
    uint32_t st[4];
    init(st);
    const uint32_t nblk = (len + 8) / 64 + 1;
    const uint32_t *pw = reinterpret_cast<const uint32_t *>(p);
    uint32_t nx[16];
#pragma unroll
    for (int w = 0; w < 16; w++) nx[w] = pw[w];
    for (uint32_t k = 0; k < nblk; k++) {
        uint32_t m[16];
#pragma unroll
        for (int w = 0; w < 16; w++) m[w] = nx[w];
        const int32_t rem = (int32_t)len - (int32_t)(64 * k);
        if (k + 1 < nblk && rem > 64) {
#pragma unroll
            for (int w = 0; w < 16; w++) nx[w] = pw[16 * (k + 1) + w];
        }
        compress_pad_lat(st, m, rem, k + 1 == nblk, len);
    }
    out[0] = st[0]; out[1] = st[1]; out[2] = st[2]; out[3] = st[3];
}

// MD5 of an inner node's message (the present children's 17-byte entries,
// at most 16 x 17 = 272 bytes) staged at a 4-byte aligned LDS address and
// readable up to byte 320: at most 5 blocks, unrolled; block k + 1's words
// are read before block k is compressed (the garbage past len is replaced by
// the padding).
__device__ __forceinline__ void md5_lds_node(const uint8_t *p, uint32_t len, uint32_t out[4]) {
    const uint32_t *q = reinterpret_cast<const uint32_t *>(p);
    const uint32_t nblk = (len + 8) / 64 + 1;
    uint32_t st[4];
    init(st);
    uint32_t nx[16];
#pragma unroll
    for (int w = 0; w < 16; w++) nx[w] = q[w];
#pragma unroll
    for (int k = 0; k < 5; k++) {
        if ((uint32_t)k < nblk) {
            uint32_t m[16];
#pragma unroll
            for (int w = 0; w < 16; w++) m[w] = nx[w];
            if (k < 4 && (uint32_t)k + 1 < nblk) {
                __asm__ volatile("" ::: "memory");   // only one block ahead (not all 80 words hoisted)
#pragma unroll
                for (int w = 0; w < 16; w++) nx[w] = q[16 * (k + 1) + w];
            }
            const int32_t rem = (int32_t)len - 64 * k;
            if (k == 4 && __ballot(len != 272) == 0) {
                // every lane of the wave holds a node with 16 children: the
                // last block is 16 data bytes, the terminator, the bit length
                m[4] = 0x80u;
#pragma unroll
                for (int w = 5; w < 16; w++) m[w] = 0u;
                m[14] = 272u * 8u;
            } else if (rem < 64) {
                pad_block(m, rem, (uint32_t)k + 1 == nblk, len);
            }
            compress(st, m);
        }
    }
    out[0] = st[0]; out[1] = st[1]; out[2] = st[2]; out[3] = st[3];
}


// The state after the first nfull (complete) blocks of an LDS message: the
// prefix a later md5_lds_resume continues from.
__device__ __forceinline__ void md5_lds_prefix(const uint8_t *p, uint32_t nfull, uint32_t st[4]) {
    init(st);
    const uint32_t *pw = reinterpret_cast<const uint32_t *>(p);
    for (uint32_t k = 0; k < nfull; k++) {
        uint32_t m[16];
#pragma unroll
        for (int w = 0; w < 16; w++) m[w] = pw[16 * k + w];
        compress_lat(st, m);
    }
}

// md5_lds of the whole `len`-byte message, given the state after its first
// k0 blocks (md5_lds_prefix): only blocks k0.. are compressed.
__device__ __forceinline__ void md5_lds_resume(const uint8_t *p, uint32_t len, uint32_t k0, const uint32_t st0[4],
                                               uint32_t out[4]) {
    uint32_t st[4] = {st0[0], st0[1], st0[2], st0[3]};
    const uint32_t nblk = (len + 8) / 64 + 1;
    const uint32_t *pw = reinterpret_cast<const uint32_t *>(p);
    for (uint32_t k = k0; k < nblk; k++) {
        uint32_t m[16];
#pragma unroll
        for (int w = 0; w < 16; w++) m[w] = pw[16 * k + w];
        const int32_t rem = (int32_t)len - (int32_t)(64 * k);
        compress_pad_lat(st, m, rem, k + 1 == nblk, len);
    }
    out[0] = st[0]; out[1] = st[1]; out[2] = st[2]; out[3] = st[3];
}

// MD5 of a FULL W=16 inner node: 16 present children, message = 16 x
// (prefix byte ‖ 16 md5 bytes) = 272 bytes = 5 blocks, assembled in
// registers.  Chunk j starts at byte 17j, so the byte alignment cycles every
// 4 chunks (68 bytes = 17 dwords): pack4 builds those 17 dwords with
// alignbit / lshl_or only (~15 ops per 4 children).
__device__ __forceinline__ void pack4(const uint32_t *pf, const uint4 *h, uint32_t *w) {
    w[0] = (h[0].x << 8) | pf[0];
    w[1] = __builtin_amdgcn_alignbit(h[0].y, h[0].x, 24);
    w[2] = __builtin_amdgcn_alignbit(h[0].z, h[0].y, 24);
    w[3] = __builtin_amdgcn_alignbit(h[0].w, h[0].z, 24);
    const uint32_t x = (h[1].x << 8) | pf[1];
    w[4] = __builtin_amdgcn_alignbit(x, h[0].w, 24);
    w[5] = __builtin_amdgcn_alignbit(h[1].y, h[1].x, 16);
    w[6] = __builtin_amdgcn_alignbit(h[1].z, h[1].y, 16);
    w[7] = __builtin_amdgcn_alignbit(h[1].w, h[1].z, 16);
    const uint32_t y = (h[2].x << 8) | pf[2];
    w[8] = __builtin_amdgcn_alignbit(y, h[1].w, 16);
    w[9] = __builtin_amdgcn_alignbit(h[2].y, h[2].x, 8);
    w[10] = __builtin_amdgcn_alignbit(h[2].z, h[2].y, 8);
    w[11] = __builtin_amdgcn_alignbit(h[2].w, h[2].z, 8);
    w[12] = __builtin_amdgcn_alignbit(pf[3], h[2].w, 8);
    w[13] = h[3].x;
    w[14] = h[3].y;
    w[15] = h[3].z;
    w[16] = h[3].w;
}

// Message words 16k..16k+15 of the 80-word padded message of a node with n
// (15 or 16) present children compacted into h[0..n-1], pf[0..n-1].  For n ==
// 15 the caller sets pf[15] = 0x80 (the terminator lands on byte 255, where
// the 16th tag byte would be) and h[15] = 0; the last block then differs only
// in word 68 (0x80 for n == 16, zero for n == 15) and the bit length.
__device__ __forceinline__ void node16_block(int k, const uint32_t pf[16], const uint4 h[16], uint32_t m[16],
                                             uint32_t n = 16) {
    uint32_t a[17], b[17];
    switch (k) {
    case 0:
        pack4(pf, h, a);
#pragma unroll
        for (int w = 0; w < 16; w++) m[w] = a[w];
        break;
    case 1:
        pack4(pf, h, a);
        pack4(pf + 4, h + 4, b);
        m[0] = a[16];
#pragma unroll
        for (int w = 1; w < 16; w++) m[w] = b[w - 1];
        break;
    case 2:
        pack4(pf + 4, h + 4, a);
        pack4(pf + 8, h + 8, b);
        m[0] = a[15];
        m[1] = a[16];
#pragma unroll
        for (int w = 2; w < 16; w++) m[w] = b[w - 2];
        break;
    case 3:
        pack4(pf + 8, h + 8, a);
        pack4(pf + 12, h + 12, b);
        m[0] = a[14];
        m[1] = a[15];
        m[2] = a[16];
#pragma unroll
        for (int w = 3; w < 16; w++) m[w] = b[w - 3];
        break;
    default:
        pack4(pf + 12, h + 12, a);
        m[0] = a[13];
        m[1] = a[14];
        m[2] = a[15];
        m[3] = a[16];
        m[4] = n == 16 ? 0x80u : 0u;
#pragma unroll
        for (int w = 5; w < 16; w++) m[w] = 0u;
        m[14] = 17u * 8u * n;
        break;
    }
}

// One compress in a rolled loop: these kernels run a few waves per CU once
// through the code, so straight-line unrolled MD5 (~14 KB) would be bound by
// instruction-cache misses.
// TPUT: the throughput form of the compression (a level of many nodes hashed
// at once, k_level16_group) instead of the latency form (a chain)
template <bool UNROLL = false, bool TPUT = false>
__device__ __forceinline__ void md5_node16(const uint32_t pf[16], const uint4 h[16], uint32_t out[4], uint32_t n = 16) {
    uint32_t st[4];
    init(st);
#pragma unroll (UNROLL ? 5 : 1)
    for (int k = 0; k < 5; k++) {
        uint32_t m[16];
        node16_block(k, pf, h, m, n);
        if (TPUT) compress<true>(st, m);
        else compress_lat(st, m);
    }
    out[0] = st[0]; out[1] = st[1]; out[2] = st[2]; out[3] = st[3];
}

}  // namespace stmd5
