// Diagnostic microbenchmark: MD5 compress throughput vs resident waves.
// Each wave runs n chained compress() on register data; we report the
// kernel wall time and the implied chip-wide block rate.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../riak_ensemble_amd/csrc/md5_dev.h"

__global__ void __launch_bounds__(256) k(int n, uint32_t *sink) {
    uint32_t st[4] = {threadIdx.x, blockIdx.x, 3, 4}, m[16];
    for (int i = 0; i < 16; i++) m[i] = i * threadIdx.x + blockIdx.x;
    for (int i = 0; i < n; i++) { stmd5::compress(st, m); m[i & 15] ^= st[1]; }
    sink[blockIdx.x * blockDim.x + threadIdx.x] = st[0] ^ st[1] ^ st[2] ^ st[3];
}

int main() {
    uint32_t *s;
    hipMalloc(&s, 4 << 24);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    int tpb[] = {64, 256};
    for (int bs : tpb)
        for (int wpc : {1, 2, 4, 8, 12, 16, 24, 32}) {       // waves per CU
            int blocks = 256 * wpc * 64 / bs;
            if (blocks < 1) continue;
            int n = 200;
            hipLaunchKernelGGL(k, dim3(blocks), dim3(bs), 0, 0, n, s);
            hipEventRecord(a);
            hipLaunchKernelGGL(k, dim3(blocks), dim3(bs), 0, 0, n, s);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            double lane_blocks = (double)blocks * bs * n;
            printf("block=%3d waves/CU=%2d : %8.3f ms  %8.2f G lane-blocks/s  (%.1f T lane-ops/s at 330 ops/block)\n", bs, wpc,
                   ms, lane_blocks / ms / 1e6, lane_blocks * 330 / ms / 1e9);
        }
    return 0;
}
