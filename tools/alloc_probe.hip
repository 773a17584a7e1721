// Probe: host cost of stream-ordered allocation of multi-GB buffers that grow
// a little each round (the ingest CSR swap pattern), release threshold = max.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdint>
static double now() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
__global__ void touch(uint8_t *p, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 16; i += (uint64_t)gridDim.x * blockDim.x)
        reinterpret_cast<uint4 *>(p)[i] = make_uint4(1, 2, 3, 4);
}
int main() {
    hipStream_t s; hipStreamCreate(&s);
    hipMemPool_t pool; hipDeviceGetDefaultMemPool(&pool, 0);
    uint64_t thr = UINT64_MAX; hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
    uint64_t sz = 3ull << 30;
    void *cur = nullptr;
    hipMallocAsync(&cur, sz, s); touch<<<4096, 256, 0, s>>>((uint8_t *)cur, sz); hipStreamSynchronize(s);
    for (int mode = 0; mode < 2; mode++) {
        for (int r = 0; r < 6; r++) {
            uint64_t nsz = sz + (uint64_t)(r + 1) * (mode ? 0 : 20ull << 20);
            double t0 = now();
            void *nw = nullptr;
            hipError_t e = hipMallocAsync(&nw, nsz, s);
            double t1 = now();
            touch<<<4096, 256, 0, s>>>((uint8_t *)nw, nsz);
            hipFreeAsync(cur, s);
            double t2 = now();
            hipStreamSynchronize(s);
            double t3 = now();
            cur = nw;
            printf("mode %s r%d alloc %.3f ms free %.3f ms sync %.3f ms (%s)\n", mode ? "same" : "grow", r, t1 - t0, t2 - t1,
                   t3 - t2, hipGetErrorString(e));
        }
    }
    // plain touch baseline
    double t0 = now(); touch<<<4096, 256, 0, s>>>((uint8_t *)cur, sz); hipStreamSynchronize(s);
    printf("touch only %.3f ms\n", now() - t0);
    return 0;
}
