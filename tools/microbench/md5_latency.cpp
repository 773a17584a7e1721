// Diagnostic microbenchmark (not part of the product): single-wave latency
// of the MD5 building blocks used by the level kernels, in shader cycles
// (s_memtime).  Build: hipcc --offload-arch=gfx950 -O3 -o md5_latency md5_latency.cpp
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../riak_ensemble_amd/csrc/md5_dev.h"

__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// 0: n chained compress() on register data; 1: md5_lds of len bytes;
// 2: md5_global of len bytes; 3: md5_global_pf
__global__ void k(int mode, int n, int len, const uint8_t *g, uint64_t *out, uint32_t *sink) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[64 * 400];
    uint8_t *reg = lds + threadIdx.x * 400;
    for (int i = 0; i < 400; i++) reg[i] = (uint8_t)(i * 7 + threadIdx.x);
    __syncthreads();
    uint32_t st[4] = {threadIdx.x, 2, 3, 4}, m[16];
    for (int i = 0; i < 16; i++) m[i] = i * threadIdx.x;
    uint64_t t0 = stamp();
    if (mode == 0) {
        for (int i = 0; i < n; i++) { stmd5::compress(st, m); m[0] ^= st[1]; }
    } else if (mode == 1) {
        for (int i = 0; i < n; i++) { stmd5::md5_lds(reg, len, st); reg[0] ^= (uint8_t)st[0]; }
    } else if (mode == 2) {
        for (int i = 0; i < n; i++) { stmd5::md5_global(g + threadIdx.x * 512 + (st[0] & 1), len, st); }
    } else {
        for (int i = 0; i < n; i++) { stmd5::md5_global_pf(g + threadIdx.x * 512 + (st[0] & 1), len, st); }
    }
    uint64_t t1 = stamp();
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + threadIdx.x] = st[0] ^ st[1] ^ st[2] ^ st[3];
}

int main() {
    uint8_t *g; uint64_t *o; uint32_t *s;
    hipMalloc(&g, 1 << 20); hipMemset(g, 1, 1 << 20);
    hipMalloc(&o, 8 * 1024); hipMalloc(&s, 4 * 64 * 1024);
    const char *names[] = {"compress x n (regs)", "md5_lds(len) x n", "md5_global(len) x n", "md5_global_pf(len) x n"};
    struct { int mode, n, len, blocks; } cases[] = {
        {0, 100, 0, 1}, {0, 100, 0, 256}, {0, 100, 0, 2048},
        {1, 20, 272, 1}, {1, 20, 55, 1}, {2, 20, 272, 1}, {3, 20, 272, 1}, {2, 20, 162, 1}, {2, 20, 162, 2048}};
    for (auto &c : cases) {
        for (int rep = 0; rep < 2; rep++) {
            hipLaunchKernelGGL(k, dim3(c.blocks), dim3(64), 0, 0, c.mode, c.n, c.len, g, o, s);
            hipDeviceSynchronize();
        }
        uint64_t h[1];
        hipMemcpy(h, o, 8, hipMemcpyDeviceToHost);
        int nblk = c.mode == 0 ? 1 : (c.len + 8) / 64 + 1;
        printf("%-26s n=%3d len=%3d wgs=%4d : %8.0f cycles/call  %6.0f cycles/block  %6.1f cycles/step\n", names[c.mode], c.n,
               c.len, c.blocks, (double)h[0] / c.n, (double)h[0] / c.n / nblk, (double)h[0] / c.n / nblk / 64);
    }
    return 0;
}
