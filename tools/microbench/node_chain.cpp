// Diagnostic microbenchmark: latency of one inner-node hash (16 children =
// 272-byte message, 5 MD5 blocks) as the fused rehash's level chain runs it,
// one wave, lanes 0..A-1 active.  Variants:
//   A  stmd5::md5_lds_node from LDS (the kernel's call)
//   B  the 68 message words loaded from LDS into registers first, then the
//      5 compressions (md5_node16-like, no LDS traffic inside the chain)
//   C  compress<false> x 5 on register words only (the floor)
//   D  A with the message length a run-time value (as in the kernel)
//   E  D for ONE node per launch (instruction cache cold, as at level H)
//   F  stmd5::md5_lds_node_rolled (block loop rolled), run-time length
//   G  F for ONE node per launch
// Build: hipcc -O3 --offload-arch=gfx950 -I riak_ensemble_amd/csrc tools/microbench/node_chain.cpp
#include <hip/hip_runtime.h>
#include <cstdio>
#include "md5_dev.h"

// (variant F/G, measured and not used by the library) md5_lds_node with the block loop rolled (one compression body in the
// code, ~1/5 of the unrolled form's instruction bytes): for chains that run
// once per launch, where the unrolled form's first pass is instruction-fetch
// bound.  Lanes with fewer blocks keep their state (select, not a branch).
namespace stmd5 {
__device__ __forceinline__ void md5_lds_node_rolled(const uint8_t *p, uint32_t len, uint32_t out[4]) {
    const uint32_t *q = reinterpret_cast<const uint32_t *>(p);
    const uint32_t nblk = (len + 8) / 64 + 1;
    const uint32_t kmax = __builtin_amdgcn_readfirstlane(nblk) | 0u;
    uint32_t nmax = nblk;
    for (int o = 32; o; o >>= 1) { const uint32_t x = __shfl_xor(nmax, o); nmax = x > nmax ? x : nmax; }
    nmax = __builtin_amdgcn_readfirstlane(nmax);
    (void)kmax;
    uint32_t st[4];
    init(st);
    uint32_t nx[16];
#pragma unroll
    for (int w = 0; w < 16; w++) nx[w] = q[w];
#pragma unroll 1
    for (uint32_t k = 0; k < nmax; k++) {
        uint32_t m[16];
#pragma unroll
        for (int w = 0; w < 16; w++) m[w] = nx[w];
        if (k + 1 < nmax) {
#pragma unroll
            for (int w = 0; w < 16; w++) nx[w] = q[16 * (k + 1) + w];
        }
        const int32_t rem = (int32_t)len - 64 * (int32_t)k;
        if (rem < 64) pad_block(m, rem, k + 1 == nblk, len);
        uint32_t t4[4] = {st[0], st[1], st[2], st[3]};
        compress(t4, m);
        if (k < nblk) { st[0] = t4[0]; st[1] = t4[1]; st[2] = t4[2]; st[3] = t4[3]; }
    }
    out[0] = st[0]; out[1] = st[1]; out[2] = st[2]; out[3] = st[3];
}
}  // namespace stmd5

template <int V>
__global__ void __launch_bounds__(64) k(int n, int active, uint32_t len, uint32_t *sink, unsigned long long *cyc) {
    __shared__ __attribute__((aligned(16))) uint8_t msg[64 * 320];
    const int lane = threadIdx.x;
    uint8_t *my = msg + lane * 320;
    for (int i = 0; i < 320; i++) my[i] = (uint8_t)(i * 7 + lane);
    __syncthreads();
    uint32_t d[4] = {1, 2, 3, 4};
    const unsigned long long t0 = clock64();
    if (lane < active) {
        for (int r = 0; r < n; r++) {
            if (V == 0) {
                stmd5::md5_lds_node(my, 272, d);
            } else if (V == 3 || V == 4) {
                stmd5::md5_lds_node(my, len, d);
            } else if (V >= 5) {
                stmd5::md5_lds_node_rolled(my, len, d);
            } else if (V == 1) {
                const uint32_t *q = reinterpret_cast<const uint32_t *>(my);
                uint32_t w[80];
#pragma unroll
                for (int i = 0; i < 68; i++) w[i] = q[i];
                w[68] = 0x80u;
#pragma unroll
                for (int i = 69; i < 80; i++) w[i] = 0u;
                w[78] = 272u * 8u;
                uint32_t st[4];
                stmd5::init(st);
#pragma unroll
                for (int b = 0; b < 5; b++) stmd5::compress(st, w + 16 * b);
                d[0] = st[0]; d[1] = st[1]; d[2] = st[2]; d[3] = st[3];
            } else {
                uint32_t w[16];
#pragma unroll
                for (int i = 0; i < 16; i++) w[i] = d[i & 3] + i;
                uint32_t st[4];
                stmd5::init(st);
#pragma unroll
                for (int b = 0; b < 5; b++) { stmd5::compress(st, w); w[b] ^= st[0]; }
                d[0] = st[0]; d[1] = st[1]; d[2] = st[2]; d[3] = st[3];
            }
            reinterpret_cast<uint32_t *>(my)[r & 63] = d[0];   // next message depends on this digest
        }
    }
    const unsigned long long t1 = clock64();
    sink[lane] = d[0] ^ d[1] ^ d[2] ^ d[3];
    if (lane == 0) cyc[0] = t1 - t0;
}

template <int V>
void run(uint32_t *s, unsigned long long *c, int active) {
    const int n = (V == 4 || V == 6) ? 1 : 200;
    hipLaunchKernelGGL(k<V>, dim3(1), dim3(64), 0, 0, n, active, 272u, s, c);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(k<V>, dim3(1), dim3(64), 0, 0, n, active, 272u, s, c);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    unsigned long long cyc;
    hipMemcpy(&cyc, c, 8, hipMemcpyDeviceToHost);
    printf("variant %c active %2d: %7.3f us per node (event), %7.0f shader cycles per node, %6.0f per block\n",
           "ABCDEFG"[V], active, ms * 1e3 / n, (double)cyc / n, (double)cyc / n / 5);
}

int main() {
    uint32_t *s;
    unsigned long long *c;
    hipMalloc(&s, 4096);
    hipMalloc(&c, 64);
    run<0>(s, c, 64);   // warm-up (clocks)
    for (int active : {1, 16, 64}) {
        run<0>(s, c, active); run<1>(s, c, active); run<2>(s, c, active); run<3>(s, c, active); run<4>(s, c, active);
        run<5>(s, c, active); run<6>(s, c, active);
    }
    return 0;
}
