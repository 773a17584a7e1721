// Diagnostic microbenchmark: chip-wide int32 VALU issue rate on gfx950 for the
// instruction mix of MD5 (v_add_u32, v_add3_u32, v_alignbit_b32, v_bitop3_b32).
// 8 independent chains per lane, 32 waves/CU; reports lane-ops/s.  Pins the
// integer VALU peak used by bench.py's roofline.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ void __launch_bounds__(256) k(int n, uint32_t *sink) {
    uint32_t x[8];
#pragma unroll
    for (int j = 0; j < 8; j++) x[j] = threadIdx.x * (j + 1) + blockIdx.x;
    const uint32_t c = sink[0], d = sink[1];
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[j]) : "v"(c));
                if (OP == 1) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[j]) : "v"(c), "v"(d));
                if (OP == 2) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(x[j]));
                if (OP == 3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(x[j]) : "v"(c), "v"(d));
                if (OP == 4) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[j]) : "v"(c));
            }
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) s ^= x[j];
    sink[2 + blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
void run(const char *name, uint32_t *s) {
    const int blocks = 256 * 8;   // 8 WGs of 256 = 32 waves per CU
    const int n = 400;
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, n, s);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, n, s);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double lane_ops = (double)blocks * 256 * n * 16 * 8;
    printf("%-16s %8.3f ms  %7.2f T lane-ops/s\n", name, ms, lane_ops / ms / 1e9);
}

int main() {
    uint32_t *s;
    hipMalloc(&s, (2 + 256 * 8 * 256) * 4);
    hipMemset(s, 0, 8);
    run<0>("v_add_u32", s);
    run<1>("v_add3_u32", s);
    run<2>("v_alignbit_b32", s);
    run<3>("v_bitop3_b32", s);
    run<4>("v_xor_b32", s);
    return 0;
}
