// Diagnostic: phase stamps (s_memtime = shader clock, s_memrealtime = 100 MHz)
// inside a copy of k_levels3_16 on a synthetic all-present W=16 tree.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include <algorithm>
#include "../../riak_ensemble_amd/csrc/st_kernels.h"

__device__ __forceinline__ uint64_t clk() { uint64_t t; asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory"); return t; }
__device__ __forceinline__ uint64_t rt() { uint64_t t; asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory"); return t; }

__global__ void __launch_bounds__(256) kst(DevTree t, uint64_t *st) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t *A = lds;
    uint16_t *At = reinterpret_cast<uint16_t *>(A + 256 * NB16);
    uint8_t *Bb = A + 256 * NB16 + 256 * TB16;
    uint16_t *Bt = reinterpret_cast<uint16_t *>(Bb + 16 * NB16);
    uint8_t *Cb = Bb + 16 * NB16 + 16 * TB16;
    uint16_t *Ct = reinterpret_cast<uint16_t *>(Cb + NB16);
    const uint32_t tid = threadIdx.x, H = t.H;
    const uint64_t root = blockIdx.x;
    uint64_t c[5], r[5];
    c[0] = clk(); r[0] = rt();
    const uint64_t c0 = t.base[H + 1] + root * 4096;
    for (uint32_t it = 0; it < 16; it++) { const uint32_t e = it * 256 + tid; *reinterpret_cast<uint4 *>(A + (e >> 4) * NB16 + (e & 15) * 16) = t.md5[c0 + e]; }
    { const uint4 *tg = reinterpret_cast<const uint4 *>(t.tag + c0);
      for (uint32_t it = 0; it < 2; it++) { const uint32_t q = it * 256 + tid; *reinterpret_cast<uint4 *>(reinterpret_cast<uint8_t *>(At) + (q >> 1) * TB16 + (q & 1) * 16) = tg[q]; } }
    __syncthreads();
    c[1] = clk(); r[1] = rt();
    { uint32_t dg[4], pr; node_lds16(A + tid * NB16, reinterpret_cast<const uint16_t *>(reinterpret_cast<uint8_t *>(At) + tid * TB16), dg, pr);
      *reinterpret_cast<uint4 *>(Bb + (tid >> 4) * NB16 + (tid & 15) * 16) = make_uint4(dg[0], dg[1], dg[2], dg[3]);
      *reinterpret_cast<uint16_t *>(reinterpret_cast<uint8_t *>(Bt) + (tid >> 4) * TB16 + (tid & 15) * 2) = pr ? 0x100 : 0; }
    __syncthreads();
    c[2] = clk(); r[2] = rt();
    if (tid < 16) { uint32_t dg[4], pr; node_lds16(Bb + tid * NB16, reinterpret_cast<const uint16_t *>(reinterpret_cast<uint8_t *>(Bt) + tid * TB16), dg, pr);
      *reinterpret_cast<uint4 *>(Cb + tid * 16) = make_uint4(dg[0], dg[1], dg[2], dg[3]); Ct[tid] = pr ? 0x100 : 0; }
    __syncthreads();
    c[3] = clk(); r[3] = rt();
    uint32_t dg[4] = {0,0,0,0}, pr = 0;
    if (tid == 0) node_lds16(Cb, Ct, dg, pr);
    __syncthreads();
    c[4] = clk(); r[4] = rt();
    if (tid == 0) { t.md5[root] = make_uint4(dg[0], dg[1], dg[2], pr); for (int i = 0; i < 5; i++) { st[root * 10 + i] = c[i]; st[root * 10 + 5 + i] = r[i]; } }
}

int main() {
    const uint32_t W = 16, H = 5;
    DevTree t; memset(&t, 0, sizeof(t));
    t.W = W; t.shift = 4; t.H = H; t.S = 1u << 20; t.base[0] = 0; t.base[1] = 1;
    uint64_t sz = 1;
    for (uint32_t l = 1; l <= H + 1; l++) { t.base[l + 1] = t.base[l] + sz; sz *= W; }
    for (uint32_t l = H + 3; l < ST_MAXLEV + 2; l++) t.base[l] = t.base[H + 2];
    const uint64_t ns = t.base[H + 2];
    hipMalloc(&t.md5, ns * 16); hipMalloc(&t.tag, ns * 2); hipMemset(t.md5, 7, ns * 16);
    std::vector<uint16_t> tg(ns, 0x100); hipMemcpy(t.tag, tg.data(), ns * 2, hipMemcpyHostToDevice);
    uint64_t *st; hipMalloc(&st, 256 * 10 * 8);
    for (int rep = 0; rep < 3; rep++) { hipLaunchKernelGGL(kst, dim3(256), dim3(256), levels3_16_lds_bytes(), 0, t, st); hipDeviceSynchronize(); }
    std::vector<uint64_t> h(2560); hipMemcpy(h.data(), st, 2560 * 8, hipMemcpyDeviceToHost);
    const char *ph[] = {"stage", "L5", "L4", "L3"};
    for (int p = 0; p < 4; p++) {
        std::vector<double> cy, us;
        for (int w = 0; w < 256; w++) { cy.push_back(h[w * 10 + p + 1] - h[w * 10 + p]); us.push_back((h[w * 10 + 6 + p] - h[w * 10 + 5 + p]) / 100.0); }
        std::sort(cy.begin(), cy.end()); std::sort(us.begin(), us.end());
        printf("%-6s median %7.0f cycles %6.2f us (max %7.0f cycles %6.2f us) -> %.2f GHz\n", ph[p], cy[128], us[128], cy[255], us[255], cy[128] / us[128] / 1000);
    }
    return 0;
}
