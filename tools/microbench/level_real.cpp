// Diagnostic: the product's k_level16 / k_upper16 in isolation on a synthetic
// all-present W=16 tree, timed with events (vs tools/microbench/level_stamp).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include "../../riak_ensemble_amd/csrc/st_kernels.h"

int main() {
    const uint32_t W = 16, H = 5;
    DevTree t;
    memset(&t, 0, sizeof(t));
    t.W = W; t.shift = 4; t.H = H; t.S = 1u << 20;
    t.base[0] = 0; t.base[1] = 1;
    uint64_t sz = 1;
    for (uint32_t l = 1; l <= H + 1; l++) { t.base[l + 1] = t.base[l] + sz; sz *= W; }
    for (uint32_t l = H + 3; l < ST_MAXLEV + 2; l++) t.base[l] = t.base[H + 2];
    const uint64_t ns = t.base[H + 2];
    hipMalloc(&t.md5, ns * 16); hipMalloc(&t.tag, ns * 2);
    hipMemset(t.md5, 7, ns * 16);
    std::vector<uint16_t> tg(ns, 0x100);
    hipMemcpy(t.tag, tg.data(), ns * 2, hipMemcpyHostToDevice);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int l = 5; l >= 4; l--) {
        const uint64_t nodes = t.base[l + 1] - t.base[l];
        float ms = 0;
        for (int rep = 0; rep < 5; rep++) {
            hipEventRecord(a);
            hipLaunchKernelGGL(k_level16, dim3((nodes + 63) / 64), dim3(64), 64 * lane_region_bytes(16), 0, t, (uint32_t)l, (const uint8_t *)nullptr);
            hipEventRecord(b);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms, a, b);
        }
        printf("k_level16 level %d nodes %lu: %.2f us\n", l, nodes, ms * 1000);
    }
    float ms = 0;
    for (int rep = 0; rep < 5; rep++) {
        hipEventRecord(a);
        hipLaunchKernelGGL(k_upper16, dim3(1), dim3(256), 256 * lane_region_bytes(16), 0, t, 1u, 3u, (const uint8_t *)nullptr);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
    }
    printf("k_upper16 levels 3..1: %.2f us\n", ms * 1000);
    return 0;
}
