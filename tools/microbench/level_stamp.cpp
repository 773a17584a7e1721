// Diagnostic: where does a level-5-shaped kernel spend its cycles?
// 65536 nodes, one lane per node, 16 children (u16 tag + uint4 md5 each).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include "../../riak_ensemble_amd/csrc/md5_dev.h"

__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

__global__ void __launch_bounds__(64) k(const uint16_t *tag, const uint4 *md5, uint4 *out, uint64_t *st, int mode) {
    const uint64_t b = blockIdx.x * 64ull + threadIdx.x;
    const uint64_t t0 = stamp();
    uint32_t tg[16];
    uint4 h[16];
#pragma unroll
    for (int j = 0; j < 16; j++) { tg[j] = tag[b * 16 + j]; h[j] = md5[b * 16 + j]; }
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) acc += tg[j] + h[j].x;
    asm volatile("" ::"v"(acc));
    const uint64_t t1 = stamp();
    uint32_t pf[16], dg[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 16; j++) pf[j] = tg[j] & 0xff;
    if (mode == 0) stmd5::md5_node16(pf, h, dg);
    const uint64_t t2 = stamp();
    out[b] = make_uint4(dg[0], dg[1], dg[2], dg[3] ^ acc);
    if (threadIdx.x == 0) { st[blockIdx.x * 3] = t0; st[blockIdx.x * 3 + 1] = t1; st[blockIdx.x * 3 + 2] = t2; }
}

int main() {
    const int N = 65536;
    uint16_t *tag; uint4 *md5, *out; uint64_t *st;
    hipMalloc(&tag, N * 16 * 2); hipMalloc(&md5, N * 16 * 16); hipMalloc(&out, N * 16); hipMalloc(&st, 8 * 3 * 1024);
    hipMemset(tag, 1, N * 32); hipMemset(md5, 3, N * 256);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int mode = 0; mode < 2; mode++) {
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(a);
            hipLaunchKernelGGL(k, dim3(N / 64), dim3(64), 0, 0, tag, md5, out, st, mode);
            hipEventRecord(b);
            hipEventSynchronize(b);
        }
        float ms; hipEventElapsedTime(&ms, a, b);
        std::vector<uint64_t> h(3 * 1024);
        hipMemcpy(h.data(), st, 8 * 3 * 1024, hipMemcpyDeviceToHost);
        std::vector<double> ld, md, start;
        uint64_t t0min = ~0ull;
        for (int i = 0; i < 1024; i++) t0min = std::min(t0min, h[3 * i]);
        for (int i = 0; i < 1024; i++) { ld.push_back(h[3*i+1]-h[3*i]); md.push_back(h[3*i+2]-h[3*i+1]); start.push_back(h[3*i]-t0min); }
        std::sort(ld.begin(), ld.end()); std::sort(md.begin(), md.end()); std::sort(start.begin(), start.end());
        printf("mode %d (%s): kernel %.2f us | loads median %.0f max %.0f cyc | md5 median %.0f max %.0f cyc | wave start spread median %.0f max %.0f cyc\n",
               mode, mode ? "loads only" : "loads+node16", ms * 1000, ld[512], ld[1023], md[512], md[1023], start[512], start[1023]);
    }
    return 0;
}
