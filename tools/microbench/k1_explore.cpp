// Diagnostic microbenchmark (not product code): where does K1's time go?
// Synthetic 10M-key CSR (Poisson(9.54) keys per segment, 17-byte values),
// the same DevTree layout as the library.  Variants:
//   base      k_segment_hash_perm (block-count order, per-lane unaligned 16-B loads)
//   loadonly  same loads, XOR instead of MD5
//   compute   same block counts, no value loads
//   al16      block-count order, 16-B ALIGNED loads + funnel shift in registers
//   natlds    natural order: a workgroup stages its 256 consecutive segments'
//             values into LDS with coalesced aligned 16-B loads, lanes hash from LDS
//   natlds_s  natlds + lanes re-assigned by block count inside the workgroup
// Every variant's digests are checked against base.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>
#include "../../riak_ensemble_amd/csrc/st_kernels.h"

using namespace stmd5;

__global__ void __launch_bounds__(256) k_loadonly(DevTree t, const uint32_t *perm) {
    for (uint64_t i = gtid(); i < t.S; i += gstride()) {
        const uint64_t s = perm[i];
        const uint64_t v0 = t.seg_voff[s], len = t.seg_voff[s + 1] - v0;
        uint32_t acc = 0;
        const uint64_t nblk = (len + 8) / 64 + 1;
        if (t.seg_off[s] != t.seg_off[s + 1])
            for (uint64_t k = 0; k < nblk; k++) {
                uint32_t m[16];
                load_block_global(t.vheap + v0 + 64 * k, m);
#pragma unroll
                for (int w = 0; w < 16; w++) acc ^= m[w];
            }
        t.md5[t.base[t.H + 1] + s] = make_uint4(acc, 0, 0, 0);
    }
}

__global__ void __launch_bounds__(256) k_compute(DevTree t, const uint32_t *perm) {
    for (uint64_t i = gtid(); i < t.S; i += gstride()) {
        const uint64_t s = perm[i];
        const uint64_t v0 = t.seg_voff[s], len = t.seg_voff[s + 1] - v0;
        uint32_t st[4];
        init(st);
        const uint64_t nblk = (len + 8) / 64 + 1;
        if (t.seg_off[s] != t.seg_off[s + 1])
            for (uint64_t k = 0; k < nblk; k++) {
                uint32_t m[16];
#pragma unroll
                for (int w = 0; w < 16; w++) m[w] = (uint32_t)(v0 + w + k);
                compress(st, m);
            }
        t.md5[t.base[t.H + 1] + s] = make_uint4(st[0], st[1], st[2], st[3]);
    }
}

// ---- aligned loads: 5 aligned chunks cover any 64 B window; shift by (p & 15)
__device__ __forceinline__ uint32_t fsh(uint32_t lo, uint32_t hi, uint32_t r) {
    // bytes r..r+3 of (hi:lo), r in 0..3
    return __builtin_amdgcn_alignbyte(hi, lo, r);
}
__device__ __forceinline__ void load_aligned(const uint8_t *p, uint32_t m[16]) {
    const uintptr_t a = (uintptr_t)p;
    const uint4 *b = reinterpret_cast<const uint4 *>(a & ~(uintptr_t)15);
    const uint32_t sh = (uint32_t)(a & 15), q = sh >> 2, r = sh & 3;
    uint32_t w[20];
#pragma unroll
    for (int c = 0; c < 5; c++) {
        const uint4 v = b[c];
        w[4 * c] = v.x; w[4 * c + 1] = v.y; w[4 * c + 2] = v.z; w[4 * c + 3] = v.w;
    }
    uint32_t x[17];
#pragma unroll
    for (int i = 0; i < 17; i++) {
        const uint32_t a0 = w[i], a1 = w[i + 1], a2 = w[i + 2], a3 = w[i + 3 < 20 ? i + 3 : 19];
        x[i] = q == 0 ? a0 : (q == 1 ? a1 : (q == 2 ? a2 : a3));
    }
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = fsh(x[i], x[i + 1], r);
}
__device__ __forceinline__ void md5_al16(const uint8_t *p, uint64_t len, uint32_t out[4]) {
    uint32_t st[4];
    init(st);
    const uint64_t nblk = (len + 8) / 64 + 1;
    uint32_t nx[16];
    load_aligned(p, nx);
    for (uint64_t k = 0; k < nblk; k++) {
        uint32_t m[16];
#pragma unroll
        for (int w = 0; w < 16; w++) m[w] = nx[w];
        const int64_t rem = (int64_t)len - (int64_t)(64 * k);
        if (rem - 64 > 0) load_aligned(p + 64 * (k + 1), nx);
        if (rem < 64) pad_block(m, rem, k + 1 == nblk, len);
        compress(st, m);
    }
    out[0] = st[0]; out[1] = st[1]; out[2] = st[2]; out[3] = st[3];
}
__global__ void __launch_bounds__(256) k_al16(DevTree t, const uint32_t *perm) {
    for (uint64_t i = gtid(); i < t.S; i += gstride()) {
        const uint64_t s = perm[i];
        const uint64_t slot = t.base[t.H + 1] + s;
        if (t.seg_off[s] == t.seg_off[s + 1]) { t.tag[slot] = 0; continue; }
        uint32_t dg[4];
        const uint64_t v0 = t.seg_voff[s];
        md5_al16(t.vheap + v0, t.seg_voff[s + 1] - v0, dg);
        t.md5[slot] = make_uint4(dg[0], dg[1], dg[2], dg[3]);
        t.tag[slot] = TAG_PRESENT;
    }
}

// ---- natural order, LDS staging
#define NAT_SEGS 256
#define NAT_CAP (56 * 1024)
// MD5 of len bytes at an arbitrary LDS byte address (aligned dword reads + alignbyte)
__device__ __forceinline__ void lds_words(const uint8_t *p, uint32_t m[16]) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t *b = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
    const uint32_t r = (uint32_t)(a & 3);
    uint32_t w[17];
#pragma unroll
    for (int i = 0; i < 17; i++) w[i] = b[i];
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = fsh(w[i], w[i + 1], r);
}
__device__ __forceinline__ void md5_lds_any(const uint8_t *p, uint32_t len, uint32_t out[4]) {
    uint32_t st[4];
    init(st);
    const uint32_t nblk = (len + 8) / 64 + 1;
    for (uint32_t k = 0; k < nblk; k++) {
        uint32_t m[16];
        const int32_t rem = (int32_t)len - (int32_t)(64 * k);
        if (rem > 0) lds_words(p + 64 * k, m);
        else {
#pragma unroll
            for (int w = 0; w < 16; w++) m[w] = 0;
        }
        if (rem < 64) pad_block(m, rem, k + 1 == nblk, len);
        compress(st, m);
    }
    out[0] = st[0]; out[1] = st[1]; out[2] = st[2]; out[3] = st[3];
}
template <bool SORT>
__global__ void __launch_bounds__(256) k_natlds(DevTree t) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ uint32_t hist[8], ord[NAT_SEGS];
    const uint32_t tid = threadIdx.x;
    const uint64_t s0 = (uint64_t)blockIdx.x * NAT_SEGS;
    const uint64_t vb = t.seg_voff[s0], ve = t.seg_voff[s0 + NAT_SEGS];
    const uint64_t ab = vb & ~15ull;
    const uint64_t nchunk = (ve - ab + 15) / 16 + 4;     // + slack for the last block's reads
    const bool staged = nchunk * 16 <= NAT_CAP;
    if (staged) {
        const uint4 *src = reinterpret_cast<const uint4 *>(t.vheap + ab);
        uint4 *dst = reinterpret_cast<uint4 *>(lds);
        for (uint64_t c = tid; c < nchunk; c += 256) dst[c] = src[c];
    }
    uint32_t me = tid;
    if (SORT) {
        if (tid < 8) hist[tid] = 0;
        __syncthreads();
        const uint64_t s = s0 + tid;
        const uint64_t len = t.seg_voff[s + 1] - t.seg_voff[s];
        uint32_t nb = t.seg_off[s] == t.seg_off[s + 1] ? 0u : (uint32_t)((len + 8) / 64 + 1);
        nb = nb > 7 ? 7 : nb;
        const uint32_t pos = atomicAdd(&hist[nb], 1u);
        __syncthreads();
        if (tid == 0) {
            uint32_t acc = 0;
            for (int b = 7; b >= 0; b--) { const uint32_t c = hist[b]; hist[b] = acc; acc += c; }
        }
        __syncthreads();
        ord[hist[nb] + pos] = tid;
        __syncthreads();
        me = ord[tid];
    } else {
        __syncthreads();
    }
    const uint64_t s = s0 + me;
    const uint64_t slot = t.base[t.H + 1] + s;
    if (t.seg_off[s] == t.seg_off[s + 1]) { t.tag[slot] = 0; return; }
    const uint64_t v0 = t.seg_voff[s], len = t.seg_voff[s + 1] - v0;
    uint32_t dg[4];
    if (staged) md5_lds_any(lds + (v0 - ab), (uint32_t)len, dg);
    else md5_global_pf(t.vheap + v0, len, dg);
    t.md5[slot] = make_uint4(dg[0], dg[1], dg[2], dg[3]);
    t.tag[slot] = TAG_PRESENT;
}


// ---- meta only: perm + offsets + entry write, no values
__global__ void __launch_bounds__(256) k_meta(DevTree t, const uint32_t *perm) {
    for (uint64_t i = gtid(); i < t.S; i += gstride()) {
        const uint64_t s = perm[i];
        const uint64_t v0 = t.seg_voff[s], v1 = t.seg_voff[s + 1];
        const bool ne = t.seg_off[s] != t.seg_off[s + 1];
        t.md5[t.base[t.H + 1] + s] = make_uint4((uint32_t)v0, (uint32_t)v1, ne, 0);
    }
}

// ---- block-count order, whole segment (<= 4 blocks) loaded before hashing
template <int B>
__device__ __forceinline__ void md5_pre(const uint8_t *p, uint32_t len, uint32_t out[4]) {
    uint32_t m[B][16];
#pragma unroll
    for (int k = 0; k < B; k++) load_block_global(p + 64 * k, m[k]);
    uint32_t st[4];
    init(st);
#pragma unroll
    for (int k = 0; k < B; k++) {
        const int32_t rem = (int32_t)len - 64 * k;
        if (rem < 64) pad_block(m[k], rem, k + 1 == B, len);
        compress(st, m[k]);
    }
    out[0] = st[0]; out[1] = st[1]; out[2] = st[2]; out[3] = st[3];
}
__global__ void __launch_bounds__(256) k_pfall(DevTree t, const uint32_t *perm) {
    for (uint64_t i = gtid(); i < t.S; i += gstride()) {
        const uint64_t s = perm[i];
        const uint64_t slot = t.base[t.H + 1] + s;
        if (t.seg_off[s] == t.seg_off[s + 1]) { t.tag[slot] = 0; continue; }
        uint32_t dg[4];
        const uint64_t v0 = t.seg_voff[s];
        const uint32_t len = (uint32_t)(t.seg_voff[s + 1] - v0);
        const uint32_t nb = (len + 8) / 64 + 1;
        const uint8_t *p = t.vheap + v0;
        if (nb == 3) md5_pre<3>(p, len, dg);
        else if (nb == 2) md5_pre<2>(p, len, dg);
        else if (nb == 4) md5_pre<4>(p, len, dg);
        else if (nb == 1) md5_pre<1>(p, len, dg);
        else md5_global_pf(p, len, dg);
        t.md5[slot] = make_uint4(dg[0], dg[1], dg[2], dg[3]);
        t.tag[slot] = TAG_PRESENT;
    }
}

// ---- natural order, LDS staging with all loads in flight at once
#define N2_SEGS 256
#define N2_PER 12                       // 16-B chunks per thread: 48 KiB per workgroup
template <bool SORT>
__global__ void __launch_bounds__(256) k_natlds2(DevTree t) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ uint32_t hist[8], ord[N2_SEGS];
    const uint32_t tid = threadIdx.x;
    const uint64_t s0 = (uint64_t)blockIdx.x * N2_SEGS;
    const uint64_t vb = t.seg_voff[s0], ve = t.seg_voff[s0 + N2_SEGS];
    const uint64_t ab = vb & ~15ull;
    const uint64_t nchunk = (ve - ab + 15) / 16 + 4;
    const bool staged = nchunk <= (uint64_t)N2_PER * 256;
    const uint64_t s = s0 + tid;
    const uint64_t mv0 = t.seg_voff[s], mv1 = t.seg_voff[s + 1];
    const bool mne = t.seg_off[s] != t.seg_off[s + 1];
    if (staged) {
        const uint4 *src = reinterpret_cast<const uint4 *>(t.vheap + ab);
        uint4 *dst = reinterpret_cast<uint4 *>(lds);
        uint4 v[N2_PER];
#pragma unroll
        for (int j = 0; j < N2_PER; j++) {
            const uint64_t c = (uint64_t)j * 256 + tid;
            if (c < nchunk) v[j] = src[c];
        }
#pragma unroll
        for (int j = 0; j < N2_PER; j++) {
            const uint64_t c = (uint64_t)j * 256 + tid;
            if (c < nchunk) dst[c] = v[j];
        }
    }
    uint32_t me = tid;
    if (SORT) {
        if (tid < 8) hist[tid] = 0;
        __syncthreads();
        uint32_t nb = mne ? (uint32_t)((mv1 - mv0 + 8) / 64 + 1) : 0u;
        nb = nb > 7 ? 7 : nb;
        const uint32_t pos = atomicAdd(&hist[nb], 1u);
        __syncthreads();
        if (tid == 0) {
            uint32_t acc = 0;
            for (int b = 7; b >= 0; b--) { const uint32_t c = hist[b]; hist[b] = acc; acc += c; }
        }
        __syncthreads();
        ord[hist[nb] + pos] = tid;
        __syncthreads();
        me = ord[tid];
    } else {
        __syncthreads();
    }
    const uint64_t sm = s0 + me;
    const uint64_t slot = t.base[t.H + 1] + sm;
    const uint64_t v0 = SORT ? t.seg_voff[sm] : mv0;
    const uint64_t len = (SORT ? t.seg_voff[sm + 1] : mv1) - v0;
    const bool ne = SORT ? t.seg_off[sm] != t.seg_off[sm + 1] : mne;
    if (!ne) { t.tag[slot] = 0; return; }
    uint32_t dg[4];
    if (staged) md5_lds_any(lds + (v0 - ab), (uint32_t)len, dg);
    else md5_global_pf(t.vheap + v0, len, dg);
    t.md5[slot] = make_uint4(dg[0], dg[1], dg[2], dg[3]);
    t.tag[slot] = TAG_PRESENT;
}


// ---- v6: descriptors in block-count order + wave-cooperative gather into
// padded LDS slots (segment j's message words at j*(16B+1) + w: conflict-free
// per-lane reads), then per-lane MD5 from LDS.  1-wave workgroups.
struct KDesc { uint64_t v0; uint32_t len; uint32_t seg; };   // len bit31 = non-empty
template <int MAXB>
__global__ void __launch_bounds__(64) k_v6(DevTree t, const KDesc *desc) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lw[];
    const uint32_t lane = threadIdx.x;
    const uint64_t p = (uint64_t)blockIdx.x * 64 + lane;
    const KDesc d = desc[p];
    const bool ne = d.len >> 31;
    const uint32_t len = d.len & 0x7fffffffu;
    const uint32_t nb = ne ? (len + 8) / 64 + 1 : 0u;
    const uint32_t B = __builtin_amdgcn_readfirstlane(nb);
    const bool uni = __ballot(nb != B) == 0ull;
    const uint64_t slot = t.base[t.H + 1] + d.seg;
    uint32_t dg[4];
    if (uni && B >= 1 && B <= MAXB) {
        const uint32_t per = 4 * B;                  // 16-B chunks per segment
        const uint32_t stride = 16 * B + 1;          // words per LDS slot
        uint4 v[4 * MAXB];
#pragma unroll
        for (int it = 0; it < 4 * MAXB; it++) {
            if ((uint32_t)it < per) {
                const uint32_t q = it * 64 + lane;
                const uint32_t j = q / per, k = q - j * per;
                const uint64_t vj = __shfl(d.v0, (int)j, 64);
                __builtin_memcpy(&v[it], t.vheap + vj + 16ull * k, 16);
            }
        }
#pragma unroll
        for (int it = 0; it < 4 * MAXB; it++) {
            if ((uint32_t)it < per) {
                const uint32_t q = it * 64 + lane;
                const uint32_t j = q / per, k = q - j * per;
                uint32_t *dst = lw + j * stride + 4 * k;
                dst[0] = v[it].x; dst[1] = v[it].y; dst[2] = v[it].z; dst[3] = v[it].w;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const uint32_t *mw = lw + lane * stride;
        uint32_t st[4];
        init(st);
        for (uint32_t k = 0; k < B; k++) {
            uint32_t m[16];
#pragma unroll
            for (int w = 0; w < 16; w++) m[w] = mw[16 * k + w];
            const int32_t rem = (int32_t)len - (int32_t)(64 * k);
            if (rem < 64) pad_block(m, rem, k + 1 == B, len);
            compress(st, m);
        }
        dg[0] = st[0]; dg[1] = st[1]; dg[2] = st[2]; dg[3] = st[3];
    } else if (ne) {
        md5_global_pf(t.vheap + d.v0, len, dg);
    }
    if (!ne) { t.tag[slot] = 0; return; }
    t.md5[slot] = make_uint4(dg[0], dg[1], dg[2], dg[3]);
    t.tag[slot] = TAG_PRESENT;
}
// descriptors only + per-lane global MD5 (isolates the meta-load saving)
__global__ void __launch_bounds__(256) k_descpf(DevTree t, const KDesc *desc) {
    const uint64_t p = gtid();
    const KDesc d = desc[p];
    const uint64_t slot = t.base[t.H + 1] + d.seg;
    if (!(d.len >> 31)) { t.tag[slot] = 0; return; }
    uint32_t dg[4];
    md5_global_pf(t.vheap + d.v0, d.len & 0x7fffffffu, dg);
    t.md5[slot] = make_uint4(dg[0], dg[1], dg[2], dg[3]);
    t.tag[slot] = TAG_PRESENT;
}


// ---- memory-pattern references
__global__ void __launch_bounds__(256) k_stream(const uint4 *p, uint64_t n16, uint32_t *out) {
    uint32_t acc = 0;
    for (uint64_t i = gtid(); i < n16; i += gstride()) { const uint4 v = p[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    if (acc == 0x12345678u) out[0] = acc;
}


// ---- v7: descriptors in block-count order; per 64-B block, the wave gathers
// block k of all 64 segments (4 x 16-B chunks per lane, consecutive lanes on
// consecutive chunks of one segment) into a padded LDS tile (lane j's words at
// j*17 + w), double-buffered so the gather of block k+1 is in flight while
// block k is compressed.  1-wave workgroups, 8.7 KB LDS per wave.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__global__ void __launch_bounds__(64) k_v7(DevTree t, const KDesc *desc) {
    __shared__ uint32_t tile[2][64 * 17];
    const uint32_t lane = threadIdx.x;
    const uint64_t p = (uint64_t)blockIdx.x * 64 + lane;
    const KDesc d = desc[p];
    const bool ne = d.len >> 31;
    const uint32_t len = d.len & 0x7fffffffu;
    const uint32_t nb = ne ? (len + 8) / 64 + 1 : 0u;
    uint32_t B = nb;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) { const uint32_t y = __shfl_xor(B, o, 64); B = B > y ? B : y; }
    B = __builtin_amdgcn_readfirstlane(B);
    const uint64_t slot = t.base[t.H + 1] + d.seg;
    // chunk c (0..255) of block k: segment j = c >> 2, quarter c & 3 -> lane = c & 63 handles
    // chunks lane, lane+64, lane+128, lane+192
    uint4 v[4];
    auto gather = [&](uint32_t k) {
#pragma unroll
        for (int it = 0; it < 4; it++) {
            const uint32_t c = it * 64 + lane, j = c >> 2, q = c & 3;
            const uint64_t vj = __shfl(d.v0, (int)j, 64);
            const uint32_t lj = __shfl(len, (int)j, 64);
            const uint32_t off = 64 * k + 16 * q;
            if (off < lj) __builtin_memcpy(&v[it], t.vheap + vj + off, 16);
            else v[it] = make_uint4(0, 0, 0, 0);
        }
    };
    auto put = [&](uint32_t *tl) {
#pragma unroll
        for (int it = 0; it < 4; it++) {
            const uint32_t c = it * 64 + lane, j = c >> 2, q = c & 3;
            uint32_t *dst = tl + j * 17 + 4 * q;
            dst[0] = v[it].x; dst[1] = v[it].y; dst[2] = v[it].z; dst[3] = v[it].w;
        }
    };
    uint32_t st[4];
    init(st);
    if (B > 0) {
        gather(0);
        put(tile[0]);
        wave_sync();
        for (uint32_t k = 0; k < B; k++) {
            if (k + 1 < B) gather(k + 1);
            uint32_t m[16];
            const uint32_t *mw = tile[k & 1] + lane * 17;
#pragma unroll
            for (int w = 0; w < 16; w++) m[w] = mw[w];
            if (k < nb) {
                const int32_t rem = (int32_t)len - (int32_t)(64 * k);
                if (rem < 64) pad_block(m, rem, k + 1 == nb, len);
                compress(st, m);
            }
            if (k + 1 < B) {
                put(tile[(k + 1) & 1]);
                wave_sync();
            }
        }
    }
    if (!ne) { t.tag[slot] = 0; return; }
    t.md5[slot] = make_uint4(st[0], st[1], st[2], st[3]);
    t.tag[slot] = TAG_PRESENT;
}


// ---- msg: segments stored as MD5-ready padded messages (64-B aligned, 0x80,
// zeros, bit length); desc = {moff, nb, seg}; aligned per-lane block loads.
struct MDesc { uint64_t moff; uint32_t nb; uint32_t seg; };
__global__ void __launch_bounds__(256) k_msg(DevTree t, const MDesc *desc, const uint4 *msg) {
    for (uint64_t p = gtid(); p < t.S; p += gstride()) {
        const MDesc d = desc[p];
        const uint64_t slot = t.base[t.H + 1] + d.seg;
        if (d.nb == 0) { t.tag[slot] = 0; continue; }
        const uint4 *b = msg + (d.moff >> 4);
        uint32_t st[4];
        init(st);
        uint4 n0 = b[0], n1 = b[1], n2 = b[2], n3 = b[3];
        for (uint32_t k = 0; k < d.nb; k++) {
            uint32_t m[16] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, n3.x, n3.y, n3.z, n3.w};
            if (k + 1 < d.nb) { const uint4 *q = b + 4 * (k + 1); n0 = q[0]; n1 = q[1]; n2 = q[2]; n3 = q[3]; }
            compress(st, m);
        }
        t.md5[slot] = make_uint4(st[0], st[1], st[2], st[3]);
        t.tag[slot] = TAG_PRESENT;
    }
}


// ---- msgwin: natural-order windows of WIN segments per workgroup, lanes
// assigned by block count inside the window (LDS counting sort); msg layout.
template <int WIN>
__global__ void __launch_bounds__(256) k_msgwin(DevTree t, const uint64_t *moff, const uint4 *msg) {
    __shared__ uint32_t hist[8], ord[WIN];
    const uint32_t tid = threadIdx.x;
    const uint64_t s0 = (uint64_t)blockIdx.x * WIN;
    if (tid < 8) hist[tid] = 0;
    __syncthreads();
    uint32_t pos[WIN / 256], nbv[WIN / 256];
#pragma unroll
    for (int r = 0; r < WIN / 256; r++) {
        const uint64_t s = s0 + r * 256 + tid;
        uint32_t nb = (uint32_t)((moff[s + 1] - moff[s]) >> 6);
        nb = nb > 7 ? 7 : nb;
        nbv[r] = nb;
        pos[r] = atomicAdd(&hist[nb], 1u);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t acc = 0;
        for (int b = 7; b >= 0; b--) { const uint32_t c = hist[b]; hist[b] = acc; acc += c; }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < WIN / 256; r++) ord[hist[nbv[r]] + pos[r]] = r * 256 + tid;
    __syncthreads();
#pragma unroll 1
    for (int r = 0; r < WIN / 256; r++) {
        const uint64_t sg = s0 + ord[r * 256 + tid];
        const uint64_t slot = t.base[t.H + 1] + sg;
        const uint64_t m0 = moff[sg];
        const uint32_t nb = (uint32_t)((moff[sg + 1] - m0) >> 6);
        if (nb == 0) { t.tag[slot] = 0; continue; }
        const uint4 *b = msg + (m0 >> 4);
        uint32_t st[4];
        init(st);
        uint4 n0 = b[0], n1 = b[1], n2 = b[2], n3 = b[3];
        for (uint32_t k = 0; k < nb; k++) {
            uint32_t m[16] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, n3.x, n3.y, n3.z, n3.w};
            if (k + 1 < nb) { const uint4 *q = b + 4 * (k + 1); n0 = q[0]; n1 = q[1]; n2 = q[2]; n3 = q[3]; }
            compress(st, m);
        }
        t.md5[slot] = make_uint4(st[0], st[1], st[2], st[3]);
        t.tag[slot] = TAG_PRESENT;
    }
}


// ---- v7m: msg layout + per-block cooperative gather (4 lanes per 64-B line)
// into a padded LDS tile, double-buffered.  1-wave workgroups.
template <int WAVES>
__global__ void __launch_bounds__(64 * WAVES) k_v7m(DevTree t, const MDesc *desc, const uint4 *msg) {
    __shared__ uint32_t tiles[WAVES][2][64 * 17];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t p = ((uint64_t)blockIdx.x * WAVES + wv) * 64 + lane;
    const MDesc d = desc[p];
    uint32_t B = d.nb;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) { const uint32_t y = __shfl_xor(B, o, 64); B = B > y ? B : y; }
    B = __builtin_amdgcn_readfirstlane(B);
    const uint64_t slot = t.base[t.H + 1] + d.seg;
    uint4 v[4];
    uint64_t mj[4];
    uint32_t nj[4];
#pragma unroll
    for (int it = 0; it < 4; it++) {
        const uint32_t j = (it * 64 + lane) >> 2;
        mj[it] = __shfl(d.moff, (int)j, 64) >> 4;
        nj[it] = __shfl(d.nb, (int)j, 64);
    }
    auto gather = [&](uint32_t k) {
#pragma unroll
        for (int it = 0; it < 4; it++) {
            const uint32_t q = lane & 3;
            if (k < nj[it]) v[it] = msg[mj[it] + 4 * k + q];
        }
    };
    auto put = [&](uint32_t *tl) {
#pragma unroll
        for (int it = 0; it < 4; it++) {
            const uint32_t c = it * 64 + lane, j = c >> 2, q = c & 3;
            uint32_t *dst = tl + j * 17 + 4 * q;
            dst[0] = v[it].x; dst[1] = v[it].y; dst[2] = v[it].z; dst[3] = v[it].w;
        }
    };
    uint32_t st[4];
    init(st);
    if (B > 0) {
        gather(0);
        put(tiles[wv][0]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t k = 0; k < B; k++) {
            if (k + 1 < B) gather(k + 1);
            uint32_t m[16];
            const uint32_t *mw = tiles[wv][k & 1] + lane * 17;
#pragma unroll
            for (int w = 0; w < 16; w++) m[w] = mw[w];
            if (k < d.nb) compress(st, m);
            if (k + 1 < B) {
                put(tiles[wv][(k + 1) & 1]);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
    }
    if (d.nb == 0) { t.tag[slot] = 0; return; }
    t.md5[slot] = make_uint4(st[0], st[1], st[2], st[3]);
    t.tag[slot] = TAG_PRESENT;
}


template <int MODE>   // 0: compute only (no value loads), 1: loads only
__global__ void __launch_bounds__(256) k_msgx(DevTree t, const MDesc *desc, const uint4 *msg) {
    for (uint64_t p = gtid(); p < t.S; p += gstride()) {
        const MDesc d = desc[p];
        const uint64_t slot = t.base[t.H + 1] + d.seg;
        if (d.nb == 0) { t.tag[slot] = 0; continue; }
        const uint4 *b = msg + (d.moff >> 4);
        uint32_t st[4];
        init(st);
        if (MODE == 0) {
            uint32_t m[16];
#pragma unroll
            for (int w = 0; w < 16; w++) m[w] = (uint32_t)d.moff + w;
            for (uint32_t k = 0; k < d.nb; k++) { compress(st, m); m[k & 15] ^= st[0]; }
        } else {
            for (uint32_t k = 0; k < d.nb; k++) {
                const uint4 *q = b + 4 * k;
                const uint4 a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3];
                st[0] ^= a0.x ^ a1.y ^ a2.z ^ a3.w; st[1] ^= a0.y ^ a1.z ^ a2.w ^ a3.x;
                st[2] ^= a0.z ^ a1.w ^ a2.x ^ a3.y; st[3] ^= a0.w ^ a1.x ^ a2.y ^ a3.z;
            }
        }
        t.md5[slot] = make_uint4(st[0], st[1], st[2], st[3]);
        t.tag[slot] = TAG_PRESENT;
    }
}


// ---- subtree: one 1024-thread workgroup per level-(H-2) node (4096
// segments): segments hashed from msg in block-count order (LDS counting
// sort), entries kept in LDS, then levels H, H-1, H-2 hashed from LDS.
#define SB_NB 272
#define SB_TB 48
__device__ __forceinline__ void node_from_lds(uint8_t *blk, const uint16_t *tags, uint32_t dg[4], uint32_t &present) {
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
        md5_node16(pf, h, dg);
    } else {
        MsgWriter mw;
        mw.init(blk);
#pragma unroll
        for (int j = 0; j < 16; j++)
            if (tg[j] & TAG_PRESENT) mw.entry(tg[j], h[j]);
        md5_lds(blk, mw.finish(), dg);
    }
}
__global__ void __launch_bounds__(1024) k_subtree(DevTree t, const uint64_t *moff, const uint4 *msg) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t *E6 = lds;                                   // 256 blocks
    uint8_t *T6 = E6 + 256 * SB_NB;                      // 256 tag blocks
    uint8_t *E5 = T6 + 256 * SB_TB;                      // 16 blocks
    uint8_t *T5 = E5 + 16 * SB_NB;
    uint8_t *E4 = T5 + 16 * SB_TB;                       // 1 block
    uint8_t *T4 = E4 + SB_NB;
    uint16_t *ord = reinterpret_cast<uint16_t *>(T4 + SB_TB);   // 4096
    uint32_t *hist = reinterpret_cast<uint32_t *>(ord + 4096);  // 8
    const uint32_t tid = threadIdx.x;
    const uint32_t H = t.H;
    const uint64_t root = blockIdx.x;
    const uint64_t s0 = root * 4096;
    if (tid < 8) hist[tid] = 0;
    __syncthreads();
    uint32_t nbv[4], pos[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const uint64_t s = s0 + r * 1024 + tid;
        uint32_t nb = (uint32_t)((moff[s + 1] - moff[s]) >> 6);
        nbv[r] = nb > 7 ? 7 : nb;
        pos[r] = atomicAdd(&hist[nbv[r]], 1u);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t acc = 0;
        for (int b = 7; b >= 0; b--) { const uint32_t c = hist[b]; hist[b] = acc; acc += c; }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; r++) ord[hist[nbv[r]] + pos[r]] = (uint16_t)(r * 1024 + tid);
    __syncthreads();
    // ---- segments
#pragma unroll 1
    for (int r = 0; r < 4; r++) {
        const uint32_t i = ord[r * 1024 + tid];
        const uint64_t sg = s0 + i;
        const uint64_t m0 = moff[sg];
        const uint32_t nb = (uint32_t)((moff[sg + 1] - m0) >> 6);
        uint4 e = make_uint4(0, 0, 0, 0);
        uint16_t tg = 0;
        if (nb) {
            const uint4 *b = msg + (m0 >> 4);
            uint32_t st[4];
            init(st);
            uint4 n0 = b[0], n1 = b[1], n2 = b[2], n3 = b[3];
            for (uint32_t k = 0; k < nb; k++) {
                uint32_t m[16] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, n3.x, n3.y, n3.z, n3.w};
                if (k + 1 < nb) { const uint4 *q = b + 4 * (k + 1); n0 = q[0]; n1 = q[1]; n2 = q[2]; n3 = q[3]; }
                compress(st, m);
            }
            e = make_uint4(st[0], st[1], st[2], st[3]);
            tg = TAG_PRESENT;
            t.md5[t.base[H + 1] + sg] = e;
        }
        t.tag[t.base[H + 1] + sg] = tg;
        *reinterpret_cast<uint4 *>(E6 + (i >> 4) * SB_NB + (i & 15) * 16) = e;
        *reinterpret_cast<uint16_t *>(T6 + (i >> 4) * SB_TB + (i & 15) * 2) = tg;
    }
    __syncthreads();
    // ---- level H: 256 nodes
    if (tid < 256) {
        uint32_t dg[4], pr;
        node_from_lds(E6 + tid * SB_NB, reinterpret_cast<const uint16_t *>(T6 + tid * SB_TB), dg, pr);
        const uint64_t slot = t.base[H] + root * 256 + tid;
        const uint4 e = pr ? make_uint4(dg[0], dg[1], dg[2], dg[3]) : make_uint4(0, 0, 0, 0);
        if (pr) t.md5[slot] = e;
        t.tag[slot] = pr ? (uint16_t)TAG_PRESENT : (uint16_t)0;
        *reinterpret_cast<uint4 *>(E5 + (tid >> 4) * SB_NB + (tid & 15) * 16) = e;
        *reinterpret_cast<uint16_t *>(T5 + (tid >> 4) * SB_TB + (tid & 15) * 2) = pr ? (uint16_t)TAG_PRESENT : (uint16_t)0;
    }
    __syncthreads();
    if (tid < 16) {
        uint32_t dg[4], pr;
        node_from_lds(E5 + tid * SB_NB, reinterpret_cast<const uint16_t *>(T5 + tid * SB_TB), dg, pr);
        const uint64_t slot = t.base[H - 1] + root * 16 + tid;
        const uint4 e = pr ? make_uint4(dg[0], dg[1], dg[2], dg[3]) : make_uint4(0, 0, 0, 0);
        if (pr) t.md5[slot] = e;
        t.tag[slot] = pr ? (uint16_t)TAG_PRESENT : (uint16_t)0;
        *reinterpret_cast<uint4 *>(E4 + tid * 16) = e;
        *reinterpret_cast<uint16_t *>(T4 + tid * 2) = pr ? (uint16_t)TAG_PRESENT : (uint16_t)0;
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t dg[4], pr;
        node_from_lds(E4, reinterpret_cast<const uint16_t *>(T4), dg, pr);
        const uint64_t slot = t.base[H - 2] + root;
        if (pr) t.md5[slot] = make_uint4(dg[0], dg[1], dg[2], dg[3]);
        t.tag[slot] = pr ? (uint16_t)TAG_PRESENT : (uint16_t)0;
    }
}


// ---- lean-argument variants (no DevTree by value: fewer SGPRs, more waves/CU)
__global__ void __launch_bounds__(256) k_perm_lean(const uint32_t *__restrict__ perm, const uint64_t *__restrict__ seg_off,
                                                   const uint64_t *__restrict__ seg_voff, const uint8_t *__restrict__ vheap,
                                                   uint4 *__restrict__ md5s, uint16_t *__restrict__ tags, uint32_t S) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < S; i += gridDim.x * blockDim.x) {
        const uint32_t s = perm[i];
        if (seg_off[s] == seg_off[s + 1]) { tags[s] = 0; continue; }
        uint32_t dg[4];
        const uint64_t v0 = seg_voff[s];
        md5_global_pf(vheap + v0, seg_voff[s + 1] - v0, dg);
        md5s[s] = make_uint4(dg[0], dg[1], dg[2], dg[3]);
        tags[s] = TAG_PRESENT;
    }
}
__global__ void __launch_bounds__(256) k_msg_lean(const MDesc *__restrict__ desc, const uint4 *__restrict__ msg,
                                                  uint4 *__restrict__ md5s, uint16_t *__restrict__ tags, uint32_t S) {
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < S; p += gridDim.x * blockDim.x) {
        const MDesc d = desc[p];
        if (d.nb == 0) { tags[d.seg] = 0; continue; }
        const uint4 *b = msg + (d.moff >> 4);
        uint32_t st[4];
        init(st);
        uint4 n0 = b[0], n1 = b[1], n2 = b[2], n3 = b[3];
        for (uint32_t k = 0; k < d.nb; k++) {
            uint32_t m[16] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, n3.x, n3.y, n3.z, n3.w};
            if (k + 1 < d.nb) { const uint4 *q = b + 4 * (k + 1); n0 = q[0]; n1 = q[1]; n2 = q[2]; n3 = q[3]; }
            compress(st, m);
        }
        md5s[d.seg] = make_uint4(st[0], st[1], st[2], st[3]);
        tags[d.seg] = TAG_PRESENT;
    }
}
template <int WIN>
__global__ void __launch_bounds__(256) k_msgwin_lean(const uint64_t *__restrict__ moff, const uint4 *__restrict__ msg,
                                                     uint4 *__restrict__ md5s, uint16_t *__restrict__ tags) {
    __shared__ uint32_t hist[8];
    __shared__ uint16_t ord[WIN];
    const uint32_t tid = threadIdx.x;
    const uint32_t s0 = blockIdx.x * WIN;
    if (tid < 8) hist[tid] = 0;
    __syncthreads();
    uint32_t pos[WIN / 256], nbv[WIN / 256];
#pragma unroll
    for (int r = 0; r < WIN / 256; r++) {
        const uint32_t s = s0 + r * 256 + tid;
        uint32_t nb = (uint32_t)((moff[s + 1] - moff[s]) >> 6);
        nbv[r] = nb > 7 ? 7 : nb;
        pos[r] = atomicAdd(&hist[nbv[r]], 1u);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t acc = 0;
        for (int b = 7; b >= 0; b--) { const uint32_t c = hist[b]; hist[b] = acc; acc += c; }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < WIN / 256; r++) ord[hist[nbv[r]] + pos[r]] = (uint16_t)(r * 256 + tid);
    __syncthreads();
#pragma unroll 1
    for (int r = 0; r < WIN / 256; r++) {
        const uint32_t sg = s0 + ord[r * 256 + tid];
        const uint64_t m0 = moff[sg];
        const uint32_t nb = (uint32_t)((moff[sg + 1] - m0) >> 6);
        if (nb == 0) { tags[sg] = 0; continue; }
        const uint4 *b = msg + (m0 >> 4);
        uint32_t st[4];
        init(st);
        uint4 n0 = b[0], n1 = b[1], n2 = b[2], n3 = b[3];
        for (uint32_t k = 0; k < nb; k++) {
            uint32_t m[16] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, n3.x, n3.y, n3.z, n3.w};
            if (k + 1 < nb) { const uint4 *q = b + 4 * (k + 1); n0 = q[0]; n1 = q[1]; n2 = q[2]; n3 = q[3]; }
            compress(st, m);
        }
        md5s[sg] = make_uint4(st[0], st[1], st[2], st[3]);
        tags[sg] = TAG_PRESENT;
    }
}


// ---- tiled: 64 segments per tile (K1 order), block k / quarter q of lane j's
// message at tile_base + ((k*4 + q)*64 + j)*16: every load instruction reads
// 1 KiB contiguous.  tinfo[t] = {uint64 base16 (in uint4 units), B}.
struct TInfo { uint64_t base; uint32_t B; uint32_t pad; };
template <int WAVES>
__global__ void __launch_bounds__(64 * WAVES) k_tiled(const TInfo *__restrict__ tinfo, const uint32_t *__restrict__ tseg,
                                                     const uint8_t *__restrict__ tnb, const uint4 *__restrict__ tiles,
                                                     uint4 *__restrict__ md5s, uint16_t *__restrict__ tags, uint32_t ntiles) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t tl = blockIdx.x * WAVES + (threadIdx.x >> 6);
    if (tl >= ntiles) return;
    const TInfo ti = tinfo[tl];
    const uint32_t seg = tseg[tl * 64 + lane];
    const uint32_t nb = tnb[tl * 64 + lane];
    const uint32_t B = ti.B;
    const uint4 *b = tiles + ti.base + lane;
    uint32_t st[4];
    init(st);
    if (B) {
        uint4 n0 = b[0], n1 = b[64], n2 = b[128], n3 = b[192];
        for (uint32_t k = 0; k < B; k++) {
            uint32_t m[16] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, n3.x, n3.y, n3.z, n3.w};
            if (k + 1 < B) { const uint4 *q = b + 256 * (k + 1); n0 = q[0]; n1 = q[64]; n2 = q[128]; n3 = q[192]; }
            if (k < nb) compress(st, m);
        }
    }
    if (seg == 0xffffffffu) return;
    if (nb == 0) { tags[seg] = 0; return; }
    md5s[seg] = make_uint4(st[0], st[1], st[2], st[3]);
    tags[seg] = TAG_PRESENT;
}

int main() {
    const uint64_t S = 1 << 20;
    std::mt19937_64 rng(1);
    std::poisson_distribution<int> pd(9.54);
    std::vector<uint64_t> so(S + 1), sv(S + 1);
    so[0] = sv[0] = 0;
    for (uint64_t s = 0; s < S; s++) { int n = pd(rng); so[s + 1] = so[s] + n; sv[s + 1] = sv[s] + 17ull * n; }
    printf("entries %lu bytes %lu\n", (unsigned long)so[S], (unsigned long)sv[S]);
    DevTree t;
    memset(&t, 0, sizeof(t));
    t.W = 16; t.shift = 4; t.H = 5; t.S = S; t.base[0] = 0; t.base[1] = 1;
    uint64_t sz = 1;
    for (uint32_t l = 1; l <= 6; l++) { t.base[l + 1] = t.base[l] + sz; sz *= 16; }
    for (uint32_t l = 8; l < ST_MAXLEV + 2; l++) t.base[l] = t.base[7];
    uint64_t *dso, *dsv;
    uint8_t *vh;
    uint32_t *perm;
    (void)hipMalloc(&dso, (S + 1) * 8); (void)hipMalloc(&dsv, (S + 1) * 8); (void)hipMalloc(&vh, sv[S] + 1024);
    (void)hipMemcpy(dso, so.data(), (S + 1) * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(dsv, sv.data(), (S + 1) * 8, hipMemcpyHostToDevice);
    std::vector<uint8_t> hv(sv[S] + 1024);
    for (size_t i = 0; i < hv.size(); i++) hv[i] = (uint8_t)(rng() >> 13);
    (void)hipMemcpy(vh, hv.data(), hv.size(), hipMemcpyHostToDevice);
    (void)hipMalloc(&t.md5, t.base[7] * 16); (void)hipMalloc(&t.tag, t.base[7] * 2);
    t.seg_off = dso; t.seg_voff = dsv; t.vheap = vh;
    std::vector<uint32_t> p(S);
    for (uint64_t s = 0; s < S; s++) p[s] = (uint32_t)s;
    auto blk = [&](uint32_t s) { return so[s] == so[s + 1] ? 0ull : (sv[s + 1] - sv[s] + 8) / 64 + 1; };
    std::stable_sort(p.begin(), p.end(), [&](uint32_t a, uint32_t b) { return blk(a) > blk(b); });
    (void)hipMalloc(&perm, S * 4);
    (void)hipMemcpy(perm, p.data(), S * 4, hipMemcpyHostToDevice);
    const uint64_t L6 = t.base[6];
    std::vector<uint4> ref(S), got(S);
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    auto run = [&](const char *name, bool check, auto launch) {
        (void)hipMemset(t.md5 + L6, 0, S * 16);
        float best = 1e9;
        for (int r = 0; r < 6; r++) {
            (void)hipEventRecord(a); launch(); (void)hipEventRecord(b); (void)hipEventSynchronize(b);
            float ms; (void)hipEventElapsedTime(&ms, a, b); best = std::min(best, ms);
        }
        (void)hipMemcpy(got.data(), t.md5 + L6, S * 16, hipMemcpyDeviceToHost);
        bool ok = true;
        if (check) for (uint64_t s = 0; s < S && ok; s++) if (blk(s) && memcmp(&got[s], &ref[s], 16)) ok = false;
        printf("%-12s %8.2f us  %s\n", name, best * 1000, check ? (ok ? "digests OK" : "DIGESTS DIFFER") : "");
    };
    run("base", false, [&] { hipLaunchKernelGGL(k_segment_hash_perm, dim3(4096), dim3(256), 0, 0, t, perm, (const uint8_t *)nullptr, (const PrefixState *)nullptr); });
    (void)hipMemcpy(ref.data(), t.md5 + L6, S * 16, hipMemcpyDeviceToHost);
    run("loadonly", false, [&] { hipLaunchKernelGGL(k_loadonly, dim3(4096), dim3(256), 0, 0, t, perm); });
    run("compute", false, [&] { hipLaunchKernelGGL(k_compute, dim3(4096), dim3(256), 0, 0, t, perm); });
    std::vector<KDesc> hd(S);
    for (uint64_t i = 0; i < S; i++) { uint32_t sg = p[i]; hd[i].v0 = sv[sg]; hd[i].len = (uint32_t)(sv[sg + 1] - sv[sg]) | (so[sg] != so[sg + 1] ? 0x80000000u : 0u); hd[i].seg = sg; }
    KDesc *dd; (void)hipMalloc(&dd, S * sizeof(KDesc)); (void)hipMemcpy(dd, hd.data(), S * sizeof(KDesc), hipMemcpyHostToDevice);
    {
        uint32_t *o; (void)hipMalloc(&o, 64);
        run("stream170MB", false, [&] { hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, (const uint4 *)vh, sv[S] / 16, o); });
        uint32_t *idp; (void)hipMalloc(&idp, S * 4);
        std::vector<uint32_t> id(S); for (uint64_t i = 0; i < S; i++) id[i] = (uint32_t)i;
        (void)hipMemcpy(idp, id.data(), S * 4, hipMemcpyHostToDevice);
        run("loadonly_nat", false, [&] { hipLaunchKernelGGL(k_loadonly, dim3(4096), dim3(256), 0, 0, t, idp); });
        run("base_nat", false, [&] { hipLaunchKernelGGL(k_segment_hash_perm, dim3(4096), dim3(256), 0, 0, t, idp, (const uint8_t *)nullptr, (const PrefixState *)nullptr); });
    }
    run("descpf", true, [&] { hipLaunchKernelGGL(k_descpf, dim3(S / 256), dim3(256), 0, 0, t, dd); });
    {
        std::vector<uint64_t> mo(S + 1); mo[0] = 0;
        for (uint64_t s2 = 0; s2 < S; s2++) mo[s2 + 1] = mo[s2] + 64 * blk(s2);
        std::vector<uint8_t> hm(mo[S] + 64, 0);
        for (uint64_t s2 = 0; s2 < S; s2++) {
            if (!blk(s2)) continue;
            const uint64_t L = sv[s2 + 1] - sv[s2];
            memcpy(&hm[mo[s2]], &hv[sv[s2]], L);
            hm[mo[s2] + L] = 0x80;
            const uint64_t bits = L * 8;
            memcpy(&hm[mo[s2 + 1] - 8], &bits, 8);
        }
        uint8_t *dm; (void)hipMalloc(&dm, hm.size()); (void)hipMemcpy(dm, hm.data(), hm.size(), hipMemcpyHostToDevice);
        std::vector<MDesc> md(S);
        for (uint64_t i = 0; i < S; i++) { uint32_t sg = p[i]; md[i].moff = mo[sg]; md[i].nb = (uint32_t)blk(sg); md[i].seg = sg; }
        MDesc *dmd; (void)hipMalloc(&dmd, S * sizeof(MDesc)); (void)hipMemcpy(dmd, md.data(), S * sizeof(MDesc), hipMemcpyHostToDevice);
        printf("msg bytes %lu\n", (unsigned long)mo[S]);
        run("msg_g4096", true, [&] { hipLaunchKernelGGL(k_msg, dim3(4096), dim3(256), 0, 0, t, dmd, (const uint4 *)dm); });
        uint64_t *dmo; (void)hipMalloc(&dmo, (S + 1) * 8); (void)hipMemcpy(dmo, mo.data(), (S + 1) * 8, hipMemcpyHostToDevice);
        run("msgwin256", true, [&] { hipLaunchKernelGGL(k_msgwin<256>, dim3(S / 256), dim3(256), 0, 0, t, dmo, (const uint4 *)dm); });
        run("msgwin512", true, [&] { hipLaunchKernelGGL(k_msgwin<512>, dim3(S / 512), dim3(256), 0, 0, t, dmo, (const uint4 *)dm); });
        run("msgwin1024", true, [&] { hipLaunchKernelGGL(k_msgwin<1024>, dim3(S / 1024), dim3(256), 0, 0, t, dmo, (const uint4 *)dm); });
        run("v7m_w1", true, [&] { hipLaunchKernelGGL(k_v7m<1>, dim3(S / 64), dim3(64), 0, 0, t, dmd, (const uint4 *)dm); });
        run("v7m_w4", true, [&] { hipLaunchKernelGGL(k_v7m<4>, dim3(S / 256), dim3(256), 0, 0, t, dmd, (const uint4 *)dm); });
        run("msg_compute", false, [&] { hipLaunchKernelGGL(k_msgx<0>, dim3(4096), dim3(256), 0, 0, t, dmd, (const uint4 *)dm); });
        run("msg_load", false, [&] { hipLaunchKernelGGL(k_msgx<1>, dim3(4096), dim3(256), 0, 0, t, dmd, (const uint4 *)dm); });
        const size_t sb_lds = 256 * SB_NB + 256 * SB_TB + 16 * SB_NB + 16 * SB_TB + SB_NB + SB_TB + 4096 * 2 + 64;
        run("subtree", true, [&] { hipLaunchKernelGGL(k_subtree, dim3(S / 4096), dim3(1024), sb_lds, 0, t, dmo, (const uint4 *)dm); });
        run("base+lv3", false, [&] { hipLaunchKernelGGL(k_segment_hash_perm, dim3(4096), dim3(256), 0, 0, t, perm, (const uint8_t *)nullptr, (const PrefixState *)nullptr);
                                     hipLaunchKernelGGL(k_levels3_16, dim3(256), dim3(256), levels3_16_lds_bytes(), 0, t, (const uint8_t *)nullptr, (const PrefixState *)nullptr); });
        uint4 *m6 = t.md5 + L6; uint16_t *t6 = t.tag + L6;
        run("perm_lean", true, [&] { hipLaunchKernelGGL(k_perm_lean, dim3(4096), dim3(256), 0, 0, perm, dso, dsv, vh, m6, t6, (uint32_t)S); });
        run("msg_lean", true, [&] { hipLaunchKernelGGL(k_msg_lean, dim3(4096), dim3(256), 0, 0, dmd, (const uint4 *)dm, m6, t6, (uint32_t)S); });
        run("msgwin_lean1024", true, [&] { hipLaunchKernelGGL(k_msgwin_lean<1024>, dim3(S / 1024), dim3(256), 0, 0, dmo, (const uint4 *)dm, m6, t6); });
        run("msgwin_lean256", true, [&] { hipLaunchKernelGGL(k_msgwin_lean<256>, dim3(S / 256), dim3(256), 0, 0, dmo, (const uint4 *)dm, m6, t6); });
        {
            const uint32_t ntl = (uint32_t)(S / 64);
            std::vector<TInfo> ti(ntl);
            std::vector<uint32_t> ts(S);
            std::vector<uint8_t> tn(S);
            uint64_t cur = 0;
            for (uint32_t tt = 0; tt < ntl; tt++) {
                uint32_t B = 0;
                for (int j = 0; j < 64; j++) { uint32_t sg = p[tt * 64 + j]; ts[tt * 64 + j] = sg; tn[tt * 64 + j] = (uint8_t)blk(sg); B = std::max<uint32_t>(B, (uint32_t)blk(sg)); }
                ti[tt].base = cur; ti[tt].B = B; cur += (uint64_t)B * 256;
            }
            std::vector<uint32_t> hw(cur * 4 + 4, 0);
            for (uint32_t tt = 0; tt < ntl; tt++)
                for (int j = 0; j < 64; j++) {
                    uint32_t sg = ts[tt * 64 + j];
                    for (uint32_t k = 0; k < tn[tt * 64 + j]; k++)
                        for (int q = 0; q < 4; q++)
                            memcpy(&hw[(ti[tt].base + (k * 4 + q) * 64 + j) * 4], &hm[mo[sg] + 64 * k + 16 * q], 16);
                }
            printf("tiled bytes %lu\n", (unsigned long)(cur * 16));
            TInfo *dti; uint32_t *dts; uint8_t *dtn; uint4 *dtw;
            (void)hipMalloc(&dti, ntl * sizeof(TInfo)); (void)hipMalloc(&dts, S * 4); (void)hipMalloc(&dtn, S); (void)hipMalloc(&dtw, hw.size() * 4);
            (void)hipMemcpy(dti, ti.data(), ntl * sizeof(TInfo), hipMemcpyHostToDevice);
            (void)hipMemcpy(dts, ts.data(), S * 4, hipMemcpyHostToDevice);
            (void)hipMemcpy(dtn, tn.data(), S, hipMemcpyHostToDevice);
            (void)hipMemcpy(dtw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
            run("tiled_w1", true, [&] { hipLaunchKernelGGL(k_tiled<1>, dim3(ntl), dim3(64), 0, 0, dti, dts, dtn, dtw, m6, t6, ntl); });
            run("tiled_w4", true, [&] { hipLaunchKernelGGL(k_tiled<4>, dim3(ntl / 4), dim3(256), 0, 0, dti, dts, dtn, dtw, m6, t6, ntl); });
            run("stream_tiles", false, [&] { uint32_t *o; hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, (const uint4 *)dtw, cur, (uint32_t *)m6); });
        }
        run("msg_g2048", true, [&] { hipLaunchKernelGGL(k_msg, dim3(2048), dim3(256), 0, 0, t, dmd, (const uint4 *)dm); });
        run("msg_g1024", true, [&] { hipLaunchKernelGGL(k_msg, dim3(1024), dim3(256), 0, 0, t, dmd, (const uint4 *)dm); });
    }
    run("v7", true, [&] { hipLaunchKernelGGL(k_v7, dim3(S / 64), dim3(64), 0, 0, t, dd); });
    run("v6_b3", true, [&] { hipLaunchKernelGGL(k_v6<3>, dim3(S / 64), dim3(64), 64 * (16 * 3 + 1) * 4, 0, t, dd); });
    run("v6_b4", true, [&] { hipLaunchKernelGGL(k_v6<4>, dim3(S / 64), dim3(64), 64 * (16 * 4 + 1) * 4, 0, t, dd); });
    run("v6_b6", true, [&] { hipLaunchKernelGGL(k_v6<6>, dim3(S / 64), dim3(64), 64 * (16 * 6 + 1) * 4, 0, t, dd); });
    run("meta", false, [&] { hipLaunchKernelGGL(k_meta, dim3(4096), dim3(256), 0, 0, t, perm); });
    run("pfall", true, [&] { hipLaunchKernelGGL(k_pfall, dim3(4096), dim3(256), 0, 0, t, perm); });
    run("natlds2", true, [&] { hipLaunchKernelGGL(k_natlds2<false>, dim3(S / N2_SEGS), dim3(256), N2_PER * 256 * 16, 0, t); });
    run("natlds2_s", true, [&] { hipLaunchKernelGGL(k_natlds2<true>, dim3(S / N2_SEGS), dim3(256), N2_PER * 256 * 16, 0, t); });
    run("al16", true, [&] { hipLaunchKernelGGL(k_al16, dim3(4096), dim3(256), 0, 0, t, perm); });
    run("natlds", true, [&] { hipLaunchKernelGGL(k_natlds<false>, dim3(S / NAT_SEGS), dim3(256), NAT_CAP, 0, t); });
    run("natlds_s", true, [&] { hipLaunchKernelGGL(k_natlds<true>, dim3(S / NAT_SEGS), dim3(256), NAT_CAP, 0, t); });
    return 0;
}
