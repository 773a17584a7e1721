// Diagnostic: K1 variants on a synthetic 10M-key CSR (Poisson(9.54) keys per
// segment, 17-byte values), kernel time + per-wave phase stamps.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include <random>
#include <algorithm>
#include "../../riak_ensemble_amd/csrc/st_kernels.h"

__device__ __forceinline__ uint64_t clk() { uint64_t t; asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory"); return t; }

// stamped copy of k_segment_hash_perm's body (one segment per lane)
__global__ void __launch_bounds__(256) k_perm_st(DevTree t, const uint32_t *perm, uint64_t *st) {
    const uint64_t i = gtid();
    const uint64_t c0 = clk();
    const uint64_t s = perm[i];
    const uint64_t v0 = t.seg_voff[s], v1 = t.seg_voff[s + 1];
    const bool ne = t.seg_off[s] != t.seg_off[s + 1];
    asm volatile("" ::"v"((uint32_t)v0), "v"((uint32_t)v1), "v"((uint32_t)ne));
    const uint64_t c1 = clk();
    uint32_t dg[4] = {0, 0, 0, 0};
    if (ne) stmd5::md5_global_pf(t.vheap + v0, v1 - v0, dg);
    const uint64_t c2 = clk();
    t.md5[t.base[t.H + 1] + s] = make_uint4(dg[0], dg[1], dg[2], dg[3]);
    if ((threadIdx.x & 63) == 0) { const uint64_t w = i >> 6; st[w * 3] = c0; st[w * 3 + 1] = c1; st[w * 3 + 2] = c2; }
}

// descriptor-driven K1: desc[i] = {voff, len | nonempty<<31, seg} in K1 order
struct Desc { uint64_t v0; uint32_t len; uint32_t seg; };
__global__ void __launch_bounds__(256) k_desc(DevTree t, const Desc *desc) {
    const uint64_t i = gtid();
    const Desc d = desc[i];
    uint32_t dg[4] = {0, 0, 0, 0};
    if (d.len >> 31) stmd5::md5_global_pf(t.vheap + d.v0, d.len & 0x7fffffffu, dg);
    t.md5[t.base[t.H + 1] + d.seg] = make_uint4(dg[0], dg[1], dg[2], dg[3]);
}

int main(int argc, char **argv) {
    const uint64_t S = 1 << 20;
    const bool uniform = argc > 1;
    std::mt19937_64 rng(1);
    std::poisson_distribution<int> pd(9.54);
    std::vector<uint64_t> so(S + 1), sv(S + 1);
    so[0] = sv[0] = 0;
    for (uint64_t s = 0; s < S; s++) { int n = uniform ? 9 + (s & 1) : pd(rng); so[s + 1] = so[s] + n; sv[s + 1] = sv[s] + 17ull * n; }
    printf("entries %lu bytes %lu\n", so[S], sv[S]);
    DevTree t; memset(&t, 0, sizeof(t));
    t.W = 16; t.shift = 4; t.H = 5; t.S = S; t.base[0] = 0; t.base[1] = 1;
    uint64_t sz = 1;
    for (uint32_t l = 1; l <= 6; l++) { t.base[l + 1] = t.base[l] + sz; sz *= 16; }
    for (uint32_t l = 8; l < ST_MAXLEV + 2; l++) t.base[l] = t.base[7];
    uint64_t *dso, *dsv; uint8_t *vh; uint32_t *perm;
    hipMalloc(&dso, (S + 1) * 8); hipMalloc(&dsv, (S + 1) * 8); hipMalloc(&vh, sv[S] + 256);
    hipMemcpy(dso, so.data(), (S + 1) * 8, hipMemcpyHostToDevice); hipMemcpy(dsv, sv.data(), (S + 1) * 8, hipMemcpyHostToDevice);
    hipMemset(vh, 0x5a, sv[S] + 256);
    hipMalloc(&t.md5, t.base[7] * 16); hipMalloc(&t.tag, t.base[7] * 2);
    t.seg_off = dso; t.seg_voff = dsv; t.vheap = vh;
    // block-count order (host)
    std::vector<uint32_t> p(S);
    for (uint64_t s = 0; s < S; s++) p[s] = s;
    auto blk = [&](uint32_t s) { return so[s] == so[s + 1] ? 0ull : (sv[s + 1] - sv[s] + 8) / 64 + 1; };
    std::stable_sort(p.begin(), p.end(), [&](uint32_t a, uint32_t b) { return blk(a) > blk(b); });
    hipMalloc(&perm, S * 4); hipMemcpy(perm, p.data(), S * 4, hipMemcpyHostToDevice);
    std::vector<uint32_t> ident(S); for (uint64_t s = 0; s < S; s++) ident[s] = s;
    uint32_t *idp; hipMalloc(&idp, S * 4); hipMemcpy(idp, ident.data(), S * 4, hipMemcpyHostToDevice);
    uint64_t *st; hipMalloc(&st, 16384 * 3 * 8);
    // windowed order: block-count sort inside windows of 4096 segments; descriptors
    std::vector<uint32_t> wp(S);
    for (uint64_t s = 0; s < S; s++) wp[s] = s;
    for (uint64_t w = 0; w < S; w += 4096)
        std::stable_sort(wp.begin() + w, wp.begin() + w + 4096, [&](uint32_t a, uint32_t b) { return blk(a) > blk(b); });
    auto mkdesc = [&](const std::vector<uint32_t> &ord) {
        std::vector<Desc> d(S);
        for (uint64_t i = 0; i < S; i++) { uint32_t s = ord[i]; d[i].v0 = sv[s]; d[i].len = (uint32_t)(sv[s + 1] - sv[s]) | ((so[s] != so[s + 1]) ? 0x80000000u : 0u); d[i].seg = s; }
        Desc *dd; hipMalloc(&dd, S * sizeof(Desc)); hipMemcpy(dd, d.data(), S * sizeof(Desc), hipMemcpyHostToDevice); return dd;
    };
    Desc *d_ident = mkdesc(ident), *d_perm = mkdesc(p), *d_win = mkdesc(wp);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    auto run = [&](const char *name, auto launch) {
        float best = 1e9;
        for (int r = 0; r < 5; r++) { hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b); best = std::min(best, ms); }
        printf("%-40s %8.2f us\n", name, best * 1000);
    };
    run("k_segment_hash_perm (perm)", [&] { hipLaunchKernelGGL(k_segment_hash_perm, dim3(4096), dim3(256), 0, 0, t, perm, (const uint8_t *)nullptr); });
    run("k_segment_hash_perm (identity)", [&] { hipLaunchKernelGGL(k_segment_hash_perm, dim3(4096), dim3(256), 0, 0, t, idp, (const uint8_t *)nullptr); });
    run("k_segment_hash_v5 (perm)", [&] { hipLaunchKernelGGL(k_segment_hash_v5, dim3(S / 64), dim3(64), 64 * 64 * K1U_MAXB, 0, t, perm, (const uint8_t *)nullptr); });
    run("k_segment_hash_perm 1024 blocks (perm)", [&] { hipLaunchKernelGGL(k_segment_hash_perm, dim3(1024), dim3(256), 0, 0, t, perm, (const uint8_t *)nullptr); });
    run("k_desc identity", [&] { hipLaunchKernelGGL(k_desc, dim3(4096), dim3(256), 0, 0, t, d_ident); });
    run("k_desc global perm", [&] { hipLaunchKernelGGL(k_desc, dim3(4096), dim3(256), 0, 0, t, d_perm); });
    run("k_desc windowed(4096) perm", [&] { hipLaunchKernelGGL(k_desc, dim3(4096), dim3(256), 0, 0, t, d_win); });
    run("k_perm_st (stamped)", [&] { hipLaunchKernelGGL(k_perm_st, dim3(4096), dim3(256), 0, 0, t, perm, st); });
    std::vector<uint64_t> h(16384 * 3); hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> m1, m2;
    for (int w = 0; w < 16384; w++) { m1.push_back(h[w * 3 + 1] - h[w * 3]); m2.push_back(h[w * 3 + 2] - h[w * 3 + 1]); }
    std::sort(m1.begin(), m1.end()); std::sort(m2.begin(), m2.end());
    printf("per wave: meta loads median %.0f p90 %.0f cyc | md5 median %.0f p90 %.0f cyc\n", m1[8192], m1[14745], m2[8192], m2[14745]);
    // blocks per wave in perm order
    double tot = 0; for (uint64_t s = 0; s < S; s++) tot += blk(s);
    printf("total md5 blocks %.0f\n", tot);
    return 0;
}
