// Diagnostic microbenchmark: the lane-per-segment span MD5 (md5_global_span,
// the streaming verify / dirty hash) over 2 KB spans that start 16-byte
// aligned, 4-byte aligned, or at an odd byte -- and the odd start read as
// dword-aligned loads joined by v_alignbyte.  Why: a page whose values move
// down by 17 k bytes starts unaligned (the head-slack A/B).
// 64 spans a wave, one span a lane, spans 2 KB apart plus the misalignment.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../riak_ensemble_amd/csrc/md5_dev.h"

// one 64-byte block from a dword-aligned base: 17 dword loads, joined
__device__ __forceinline__ void load_block_join(const uint8_t *p, uint32_t m[16]) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t mis = (uint32_t)(a & 3);
    const uint32_t *w = reinterpret_cast<const uint32_t *>(a - mis);
    uint32_t x[17];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        uint4 v;
        __builtin_memcpy(&v, w + 4 * q, 16);
        x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
    }
    x[16] = w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = __builtin_amdgcn_alignbyte(x[i + 1], x[i], mis);
}

// one 64-byte block from 16-byte aligned loads: 5 x 16 B, a dword shift by
// (p & 12) / 4 in two conditional rounds, then v_alignbyte by p & 3
__device__ __forceinline__ void load_block_shift(const uint8_t *p, uint32_t m[16]) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t sh = (uint32_t)(a & 15);
    const uint4 *w = reinterpret_cast<const uint4 *>(a - sh);
    uint32_t x[20];
#pragma unroll
    for (int q = 0; q < 5; q++) {
        const uint4 v = w[q];
        x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
    }
    // the selects as bit-field inserts with all-ones / zero masks (a select of
    // array elements became a dynamically indexed array in scratch)
    const uint32_t M2 = (sh & 8) ? ~0u : 0u, M1 = (sh & 4) ? ~0u : 0u;
    uint32_t y[18], z[17];
#pragma unroll
    for (int i = 0; i < 18; i++) y[i] = (x[i + 2] & M2) | (x[i] & ~M2);
#pragma unroll
    for (int i = 0; i < 17; i++) z[i] = (y[i + 1] & M1) | (y[i] & ~M1);
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = __builtin_amdgcn_alignbyte(z[i + 1], z[i], sh & 3);
}

template <int MODE>   // 0: md5_global_span's loads; 1: joined dword loads; 2: 16-byte loads, shifted
__global__ void __launch_bounds__(256) k(const uint8_t *base, uint32_t mis, uint32_t len, uint32_t *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint8_t *p = base + (uint64_t)i * 2048 + mis;
    uint32_t st[4];
    stmd5::init(st);
    const uint32_t nblk = len / 64;
    uint32_t nx[16];
    if (MODE == 0) stmd5::load_block_global(p, nx); else if (MODE == 1) load_block_join(p, nx); else load_block_shift(p, nx);
    for (uint32_t b = 0; b < nblk; b++) {
        uint32_t m[16];
#pragma unroll
        for (int w = 0; w < 16; w++) m[w] = nx[w];
        if (b + 1 < nblk) {
            if (MODE == 0) stmd5::load_block_global(p + 64 * (b + 1), nx);
            else if (MODE == 1) load_block_join(p + 64 * (b + 1), nx);
            else load_block_shift(p + 64 * (b + 1), nx);
        }
        stmd5::compress_lat(st, m);
    }
    out[i] = st[0] ^ st[1] ^ st[2] ^ st[3];
}


// Prefetch depth 2 (blocks k+1 and k+2 in flight while k is compressed), and
// the same loop at 8 waves per SIMD (<= 64 VGPRs): is the aligned span hash
// short of loads in flight?
template <int DEPTH, int WAVES>
__global__ void __launch_bounds__(256, WAVES) kd(const uint8_t *base, uint32_t len, uint32_t *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint8_t *p = base + (uint64_t)i * 2048;
    uint32_t st[4];
    stmd5::init(st);
    const uint32_t nblk = len / 64;
    uint32_t b0[16], b1[16];
    stmd5::load_block_global(p, b0);
    if (DEPTH > 1) stmd5::load_block_global(p + 64, b1);
    for (uint32_t b = 0; b < nblk; b++) {
        uint32_t m[16];
#pragma unroll
        for (int w = 0; w < 16; w++) m[w] = b0[w];
        if (DEPTH > 1) {
#pragma unroll
            for (int w = 0; w < 16; w++) b0[w] = b1[w];
            if (b + 2 < nblk) stmd5::load_block_global(p + 64 * (b + 2), b1);
        } else if (b + 1 < nblk) {
            stmd5::load_block_global(p + 64 * (b + 1), b0);
        }
        stmd5::compress_lat(st, m);
    }
    out[i] = st[0] ^ st[1] ^ st[2] ^ st[3];
}

int main() {
    const uint32_t n = 2540 * 256, len = 1984;   // spans of the config-5 verify: ~650 k touched segments, ~31 blocks
    uint8_t *buf;
    uint32_t *out;
    hipMalloc(&buf, (uint64_t)n * 2048 + 4096);
    hipMalloc(&out, n * 4);
    hipMemset(buf, 7, (uint64_t)n * 2048 + 4096);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char *names[] = {"aligned 16", "aligned 4", "odd byte", "odd byte, joined dword loads", "aligned 16, joined",
                           "odd byte, 16 B loads shifted", "byte 7, 16 B loads shifted", "aligned 16, shifted"};
    const uint32_t miss[] = {0, 4, 1, 1, 0, 1, 7, 0};
    const int modes[] = {0, 0, 0, 1, 1, 2, 2, 2};
    for (int rep = 0; rep < 2; rep++)
        for (int v = 0; v < 8; v++) {
            float best = 1e9f;
            for (int it = 0; it < 5; it++) {
                hipEventRecord(a);
                if (modes[v] == 0) hipLaunchKernelGGL(k<0>, dim3(n / 256), dim3(256), 0, 0, buf, miss[v], len, out);
                else if (modes[v] == 1) hipLaunchKernelGGL(k<1>, dim3(n / 256), dim3(256), 0, 0, buf, miss[v], len, out);
                else hipLaunchKernelGGL(k<2>, dim3(n / 256), dim3(256), 0, 0, buf, miss[v], len, out);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                best = ms < best ? ms : best;
            }
            printf("%-30s %.3f ms  (%.2f GB/s)\n", names[v], best, (double)n * len / best / 1e6);
        }
    for (int rep = 0; rep < 2; rep++) {
        const char *dn[] = {"aligned 16, depth 1, 6 waves", "aligned 16, depth 2, 6 waves", "aligned 16, depth 1, 8 waves",
                            "aligned 16, depth 2, 8 waves"};
        for (int v = 0; v < 4; v++) {
            float best = 1e9f;
            for (int it = 0; it < 5; it++) {
                hipEventRecord(a);
                if (v == 0) hipLaunchKernelGGL((kd<1, 6>), dim3(n / 256), dim3(256), 0, 0, buf, len, out);
                if (v == 1) hipLaunchKernelGGL((kd<2, 6>), dim3(n / 256), dim3(256), 0, 0, buf, len, out);
                if (v == 2) hipLaunchKernelGGL((kd<1, 8>), dim3(n / 256), dim3(256), 0, 0, buf, len, out);
                if (v == 3) hipLaunchKernelGGL((kd<2, 8>), dim3(n / 256), dim3(256), 0, 0, buf, len, out);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                best = ms < best ? ms : best;
            }
            printf("%-30s %.3f ms  (%.2f GB/s)\n", dn[v], best, (double)n * len / best / 1e6);
        }
    }
    return 0;
}
