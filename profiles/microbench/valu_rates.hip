// VALU throughput of the integer operations the Bloom / hash code uses
// (gfx950): each kernel runs N independent chains per lane, timed with HIP
// events; prints G lane-ops/s per operation.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096
#define CH 8

template <int OP>
__global__ __launch_bounds__(256) void k_op(uint64_t *out, uint32_t seed) {
    uint32_t a[CH];
    uint64_t b[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) {
        a[c] = seed * (threadIdx.x + 1) + c * 0x9E3779B9u + blockIdx.x;
        b[c] = ((uint64_t)a[c] << 32) | (a[c] ^ 0xdeadbeefu);
    }
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
            if (OP == 0) a[c] = a[c] * 0x9E3779B1u + c;                            // v_mul_lo_u32 (+add)
            if (OP == 1) a[c] = __umul24(a[c], 0x9E3779u) + c;       // v_mul_u32_u24 / mad_u32_u24
            if (OP == 2) b[c] = b[c] * 0xff51afd7ed558ccdull + c;                  // 64 x 64 -> 64 multiply
            if (OP == 3) b[c] = (b[c] << (a[c] & 63)) ^ b[c] ^ c;                 // 64-bit variable shift + xor
            if (OP == 4) a[c] = (a[c] ^ (a[c] >> 7)) + c;                          // 32-bit shift/xor/add
            if (OP == 5) a[c] = __builtin_amdgcn_alignbit(a[c], a[c] ^ c, 13);    // v_alignbit_b32 (rotate)
            if (OP == 6) a[c] = __umulhi(a[c], 0x9E3779B1u) ^ c;                  // v_mul_hi_u32
        }
    }
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s ^= a[c] ^ b[c];
    if (s == 0x123456789ull) out[0] = s;
}

template <int OP>
double run(uint64_t *d) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * 8;
    hipLaunchKernelGGL(k_op<OP>, dim3(blocks), dim3(256), 0, 0, d, 7u);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_op<OP>, dim3(blocks), dim3(256), 0, 0, d, 11u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return (double)blocks * 256 * ITERS * CH / (ms * 1e-3) / 1e9;
}

int main() {
    uint64_t *d;
    hipMalloc(&d, 8);
    const char *names[] = {"mul_lo_u32+add", "mul_u32_u24+add", "mul64x64+add", "shl64_var+xor64", "shr32+xor+add",
                           "alignbit_b32", "mul_hi_u32+xor"};
    double r[7] = {run<0>(d), run<1>(d), run<2>(d), run<3>(d), run<4>(d), run<5>(d), run<6>(d)};
    printf("{");
    for (int i = 0; i < 7; i++) printf("%s\"%s\": %.1f", i ? ", " : "", names[i], r[i]);
    printf("}  (G lane-ops/s of each expression)\n");
    return 0;
}
