// Diagnostic microbenchmark: MD5 step instruction-selection variants and
// per-lane ILP, chip-wide lane-blocks/s vs waves per CU (gfx950).
//   V0  compiler default: bitop3, add, add3, alignbit, add (md5_dev.h)
//   V1  add3 split into two v_add_u32
//   V2  rotate as v_lshlrev + v_lshrrev + v_or (no alignbit)
//   V3  rotate as v_lshrrev + v_lshl_or_b32
//   V4  V0 with two independent messages per lane (ILP 2)
//   V5  V1 + V2 (only 2-operand adds/shifts + bitop3)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#pragma clang diagnostic ignored "-Wunused-value"
#pragma clang diagnostic ignored "-Wunused-result"

#define F_(b, c, d) __builtin_amdgcn_bitop3_b32((b), (c), (d), 0xCA)
#define G_(b, c, d) __builtin_amdgcn_bitop3_b32((b), (c), (d), 0xE4)
#define H_(b, c, d) __builtin_amdgcn_bitop3_b32((b), (c), (d), 0x96)
#define I_(b, c, d) __builtin_amdgcn_bitop3_b32((b), (c), (d), 0x39)

__device__ __forceinline__ uint32_t add2(uint32_t x, uint32_t y) {
    uint32_t r;
    asm("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}
__device__ __forceinline__ uint32_t addk(uint32_t x, uint32_t k) {
    uint32_t r;
    asm("v_add_u32 %0, %2, %1" : "=v"(r) : "v"(x), "i"(k));
    return r;
}
template <int V>
__device__ __forceinline__ uint32_t rot(uint32_t x, int s) {
    if (V == 6) {
        uint32_t r, o;
        asm("v_lshrrev_b32 %0, %1, %2" : "=v"(r) : "i"(32 - s), "v"(x));
        asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(o) : "v"(x), "i"(s), "v"(r));
        return o;
    }
    if (V == 2 || V == 5) {
        uint32_t l, r, o;
        asm("v_lshlrev_b32 %0, %1, %2" : "=v"(l) : "i"(s), "v"(x));
        asm("v_lshrrev_b32 %0, %1, %2" : "=v"(r) : "i"(32 - s), "v"(x));
        asm("v_or_b32 %0, %1, %2" : "=v"(o) : "v"(l), "v"(r));
        return o;
    } else if (V == 3) {
        uint32_t r, o;
        asm("v_lshrrev_b32 %0, %1, %2" : "=v"(r) : "i"(32 - s), "v"(x));
        asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(o) : "v"(x), "i"(s), "v"(r));
        return o;
    }
    return __builtin_amdgcn_alignbit(x, x, 32 - s);
}
template <int V>
__device__ __forceinline__ uint32_t sum4(uint32_t a, uint32_t m, uint32_t k, uint32_t f) {
    if (V == 1 || V == 5 || V == 6 || V == 8) return add2(addk(add2(a, m), k), f);
    if (V == 7) {
        uint32_t mk = addk(m, k), r;
        asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(mk), "v"(f));
        return r;
    }
    if (V == 9) {   // K folded with a first: (a + K) + m + F as VOP2 adds, F last
        return add2(add2(addk(a, k), m), f);
    }
    return a + m + k + f;
}
#define ST(V, f, a, b, c, d, m, k, s) a = (b) + rot<V>(sum4<V>((a), (m), (k), f((b), (c), (d))), (s))

template <int V>
__device__ __forceinline__ void compress(uint32_t st[4], const uint32_t m[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    ST(V, F_, a, b, c, d, m[0], 0xd76aa478u, 7); ST(V, F_, d, a, b, c, m[1], 0xe8c7b756u, 12);
    ST(V, F_, c, d, a, b, m[2], 0x242070dbu, 17); ST(V, F_, b, c, d, a, m[3], 0xc1bdceeeu, 22);
    ST(V, F_, a, b, c, d, m[4], 0xf57c0fafu, 7); ST(V, F_, d, a, b, c, m[5], 0x4787c62au, 12);
    ST(V, F_, c, d, a, b, m[6], 0xa8304613u, 17); ST(V, F_, b, c, d, a, m[7], 0xfd469501u, 22);
    ST(V, F_, a, b, c, d, m[8], 0x698098d8u, 7); ST(V, F_, d, a, b, c, m[9], 0x8b44f7afu, 12);
    ST(V, F_, c, d, a, b, m[10], 0xffff5bb1u, 17); ST(V, F_, b, c, d, a, m[11], 0x895cd7beu, 22);
    ST(V, F_, a, b, c, d, m[12], 0x6b901122u, 7); ST(V, F_, d, a, b, c, m[13], 0xfd987193u, 12);
    ST(V, F_, c, d, a, b, m[14], 0xa679438eu, 17); ST(V, F_, b, c, d, a, m[15], 0x49b40821u, 22);
    ST(V, G_, a, b, c, d, m[1], 0xf61e2562u, 5); ST(V, G_, d, a, b, c, m[6], 0xc040b340u, 9);
    ST(V, G_, c, d, a, b, m[11], 0x265e5a51u, 14); ST(V, G_, b, c, d, a, m[0], 0xe9b6c7aau, 20);
    ST(V, G_, a, b, c, d, m[5], 0xd62f105du, 5); ST(V, G_, d, a, b, c, m[10], 0x02441453u, 9);
    ST(V, G_, c, d, a, b, m[15], 0xd8a1e681u, 14); ST(V, G_, b, c, d, a, m[4], 0xe7d3fbc8u, 20);
    ST(V, G_, a, b, c, d, m[9], 0x21e1cde6u, 5); ST(V, G_, d, a, b, c, m[14], 0xc33707d6u, 9);
    ST(V, G_, c, d, a, b, m[3], 0xf4d50d87u, 14); ST(V, G_, b, c, d, a, m[8], 0x455a14edu, 20);
    ST(V, G_, a, b, c, d, m[13], 0xa9e3e905u, 5); ST(V, G_, d, a, b, c, m[2], 0xfcefa3f8u, 9);
    ST(V, G_, c, d, a, b, m[7], 0x676f02d9u, 14); ST(V, G_, b, c, d, a, m[12], 0x8d2a4c8au, 20);
    ST(V, H_, a, b, c, d, m[5], 0xfffa3942u, 4); ST(V, H_, d, a, b, c, m[8], 0x8771f681u, 11);
    ST(V, H_, c, d, a, b, m[11], 0x6d9d6122u, 16); ST(V, H_, b, c, d, a, m[14], 0xfde5380cu, 23);
    ST(V, H_, a, b, c, d, m[1], 0xa4beea44u, 4); ST(V, H_, d, a, b, c, m[4], 0x4bdecfa9u, 11);
    ST(V, H_, c, d, a, b, m[7], 0xf6bb4b60u, 16); ST(V, H_, b, c, d, a, m[10], 0xbebfbc70u, 23);
    ST(V, H_, a, b, c, d, m[13], 0x289b7ec6u, 4); ST(V, H_, d, a, b, c, m[0], 0xeaa127fau, 11);
    ST(V, H_, c, d, a, b, m[3], 0xd4ef3085u, 16); ST(V, H_, b, c, d, a, m[6], 0x04881d05u, 23);
    ST(V, H_, a, b, c, d, m[9], 0xd9d4d039u, 4); ST(V, H_, d, a, b, c, m[12], 0xe6db99e5u, 11);
    ST(V, H_, c, d, a, b, m[15], 0x1fa27cf8u, 16); ST(V, H_, b, c, d, a, m[2], 0xc4ac5665u, 23);
    ST(V, I_, a, b, c, d, m[0], 0xf4292244u, 6); ST(V, I_, d, a, b, c, m[7], 0x432aff97u, 10);
    ST(V, I_, c, d, a, b, m[14], 0xab9423a7u, 15); ST(V, I_, b, c, d, a, m[5], 0xfc93a039u, 21);
    ST(V, I_, a, b, c, d, m[12], 0x655b59c3u, 6); ST(V, I_, d, a, b, c, m[3], 0x8f0ccc92u, 10);
    ST(V, I_, c, d, a, b, m[10], 0xffeff47du, 15); ST(V, I_, b, c, d, a, m[1], 0x85845dd1u, 21);
    ST(V, I_, a, b, c, d, m[8], 0x6fa87e4fu, 6); ST(V, I_, d, a, b, c, m[15], 0xfe2ce6e0u, 10);
    ST(V, I_, c, d, a, b, m[6], 0xa3014314u, 15); ST(V, I_, b, c, d, a, m[13], 0x4e0811a1u, 21);
    ST(V, I_, a, b, c, d, m[4], 0xf7537e82u, 6); ST(V, I_, d, a, b, c, m[11], 0xbd3af235u, 10);
    ST(V, I_, c, d, a, b, m[2], 0x2ad7d2bbu, 15); ST(V, I_, b, c, d, a, m[9], 0xeb86d391u, 21);
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
}

template <int V>
__global__ void __launch_bounds__(256) k(int n, uint32_t *sink) {
    uint32_t st[4] = {threadIdx.x, blockIdx.x, 3, 4}, m[16];
    for (int i = 0; i < 16; i++) m[i] = i * threadIdx.x + blockIdx.x;
    if (V == 4 || V == 8) {
        uint32_t s2[4] = {threadIdx.x + 7, blockIdx.x * 3, 5, 6}, m2[16];
        for (int i = 0; i < 16; i++) m2[i] = i * threadIdx.x + blockIdx.x * 5;
        for (int i = 0; i < n / 2; i++) {
            compress<V == 8 ? 1 : 0>(st, m);
            compress<V == 8 ? 1 : 0>(s2, m2);
            m[i & 15] ^= st[1];
            m2[i & 15] ^= s2[1];
        }
        st[0] ^= s2[0]; st[1] ^= s2[1];
    } else {
        for (int i = 0; i < n; i++) { compress<V>(st, m); m[i & 15] ^= st[1]; }
    }
    sink[blockIdx.x * blockDim.x + threadIdx.x] = st[0] ^ st[1] ^ st[2] ^ st[3];
}

template <int V>
void run(uint32_t *s, hipEvent_t a, hipEvent_t b) {
    for (int wpc : {0, 4, 8, 16, 32}) {
        const int bs = wpc ? 256 : 64, blocks = wpc ? 256 * wpc * 64 / bs : 1, n = 200;
        hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(bs), 0, 0, n, s);
        hipEventRecord(a);
        for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(bs), 0, 0, n, s);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double lb = 5.0 * blocks * bs * n;
        if (wpc)
            printf("V%d waves/CU=%2d : %8.3f ms  %8.2f G lane-blocks/s\n", V, wpc, ms / 5, lb / ms / 1e6);
        else
            printf("V%d lone wave   : %8.3f us per block (dependent chain)\n", V, ms / 5 * 1e3 / n);
    }
}

int main() {
    uint32_t *s;
    hipMalloc(&s, 4 << 24);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    run<0>(s, a, b); run<1>(s, a, b); run<2>(s, a, b); run<3>(s, a, b); run<4>(s, a, b); run<5>(s, a, b);
    run<6>(s, a, b); run<7>(s, a, b); run<8>(s, a, b); run<9>(s, a, b);
    return 0;
}
