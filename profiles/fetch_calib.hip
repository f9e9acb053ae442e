// FETCH_SIZE calibration and random-line throughput of the align kernels'
// access shapes on gfx950 (MI355X).
//
// MI355X_MICROARCH.md: FETCH_SIZE (TCC_EA0_RDREQ x 64 B as rocprofv3 derives
// it) reports 1/2 of the bytes of a wide coalesced streaming read on gfx950,
// and "other access widths are uncalibrated: calibrate on a known byte count
// in your own access pattern".  The lane kernel (csrc/pa_lane.h) mostly reads
// narrow items at random 64-B lines (table slots, flag planes, genome words,
// neighbour words, Bloom words) plus its reads' bytes as a stream.  This
// program reads known numbers of distinct lines of a 16 GiB buffer (64x the
// Infinity Cache) and of small regions, and prints for every kernel the
// lines and bytes it touched and its time (HIP events):
//   rand16/rand8     one 16-B / 8-B load per lane at a random line
//   rand16_nt        the same with nontemporal loads
//   rand64           four 16-B loads per lane of one random line
//   rand128          eight 16-B loads per lane over two adjacent lines
//   rand16_mall<MB>  random lines of a MB-sized region (Infinity Cache sized)
//   mix_<a>_<b>      per lane one random line of the big buffer (plain or
//                    nontemporal) + one of a 64 MB region: does the region stay
//                    in the Infinity Cache behind the big random reads?
//   stream16         coalesced 16 B per lane, sequential (the guide's 1/2 case)
// Run under `rocprofv3 --kernel-trace --pmc FETCH_SIZE -- ./fetch_calib` and
// divide: bytes touched / FETCH_SIZE bytes = the correction of that shape;
// lines / time = the random-line rate (profiles/fetch_calib.json).
//
// Measurement tool only (not part of libpa.so); built by build_native.build_tools.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <algorithm>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e = (x);                                                                     \
        if (e != hipSuccess) {                                                                  \
            std::fprintf(stderr, "HIP error %s at line %d\n", hipGetErrorString(e), __LINE__);  \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

template <bool NT>
__device__ __forceinline__ uint4 ld16(const uint4 *p) {
    if (NT) {
        uint4 v;
        v.x = __builtin_nontemporal_load(&((const uint32_t *)p)[0]);
        v.y = __builtin_nontemporal_load(&((const uint32_t *)p)[1]);
        v.z = __builtin_nontemporal_load(&((const uint32_t *)p)[2]);
        v.w = __builtin_nontemporal_load(&((const uint32_t *)p)[3]);
        return v;
    }
    return *p;
}

// SHAPE 16 / 8 / 64 / 128 bytes per random access (see above); R independent
// accesses per lane, all issued before any is used.
template <int SHAPE, bool NT, int R>
__global__ __launch_bounds__(256) void k_rand(const uint4 *__restrict__ buf, uint64_t n_lines, uint64_t seed,
                                              uint32_t *out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < R; i++) {
        const uint64_t h = mix(seed ^ (t * 0x9E3779B97F4A7C15ull + (uint64_t)i));
        if (SHAPE == 128) {
            const uint64_t line = __umul64hi(h, n_lines - 1) & ~1ull;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint4 v = ld16<NT>(buf + line * 4 + j);
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            }
        } else {
            const uint64_t line = __umul64hi(h, n_lines);
            if (SHAPE == 16) {
                const uint4 v = ld16<NT>(buf + line * 4 + (h & 3));
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            } else if (SHAPE == 8) {
                const uint2 v = ((const uint2 *)buf)[line * 8 + (h & 7)];
                acc ^= v.x ^ v.y;
            } else {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint4 v = ld16<NT>(buf + line * 4 + j);
                    acc ^= v.x ^ v.y ^ v.z ^ v.w;
                }
            }
        }
    }
    if (acc == 0x12345679u) out[t & 0xFFFFF] = acc;  // practically never: no write traffic
}

// Per lane R pairs: a random line of the big buffer (plain or nontemporal) and
// a random line of a small region.
template <bool NT_BIG, int R>
__global__ __launch_bounds__(256) void k_mix(const uint4 *__restrict__ big, uint64_t big_lines,
                                             const uint4 *__restrict__ small, uint64_t small_lines, uint64_t seed,
                                             uint32_t *out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < R; i++) {
        const uint64_t h = mix(seed ^ (t * 0x9E3779B97F4A7C15ull + (uint64_t)i));
        const uint4 a = ld16<NT_BIG>(big + __umul64hi(h, big_lines) * 4 + (h & 3));
        const uint64_t h2 = mix(h);
        const uint4 b = small[__umul64hi(h2, small_lines) * 4 + (h2 & 3)];
        acc ^= a.x ^ a.w ^ b.y ^ b.z;
    }
    if (acc == 0x12345679u) out[t & 0xFFFFF] = acc;
}

__global__ __launch_bounds__(256) void k_stream16(const uint4 *__restrict__ buf, uint64_t n16, uint32_t *out) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = buf[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345679u) out[0] = acc;
}

static hipEvent_t e0, e1;
static bool first_row = true;

template <typename F>
static void timed(const char *name, uint64_t lines, uint64_t bytes, F launch) {
    launch();  // warm (also the clock)
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("%s {\"kernel\": \"%s\", \"lines\": %llu, \"line_bytes\": %llu, \"ms\": %.4f, \"glines_per_s\": %.2f, "
                "\"line_gb_per_s\": %.1f}\n",
                first_row ? " " : ",", name, (unsigned long long)lines, (unsigned long long)bytes, ms,
                lines / (ms * 1e6), bytes / (ms * 1e6));
    first_row = false;
}

// --footprint: random 16-B loads over buffers of 16 GiB up to ~250 GB (the
// C4 / C5 indexes' footprints: ~100 / ~250 GB touched by the lane kernel), to
// see whether the random-line ceiling falls as a buffer outgrows the TLB reach.
static int footprint_sweep() {
    size_t fr = 0, tot = 0;
    CK(hipMemGetInfo(&fr, &tot));
    uint64_t bytes = std::min<uint64_t>(250ull * 1000 * 1000 * 1000, (uint64_t)fr - (12ull << 30));
    bytes &= ~((1ull << 30) - 1);
    uint4 *buf = nullptr;
    uint32_t *out = nullptr;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 4u << 20));
    CK(hipMemset(buf, 0x5A, bytes));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipDeviceSynchronize());
    const unsigned blocks = 16384;
    const uint64_t lanes = (uint64_t)blocks * 256;
    constexpr int R = 8;
    const uint64_t L = lanes * R;
    std::printf("{\"buffer_bytes\": %llu, \"footprint_sweep\": [\n", (unsigned long long)bytes);
    for (uint64_t gb : {16ull, 32ull, 64ull, 100ull, 128ull, 192ull, 250ull}) {
        const uint64_t nb = std::min<uint64_t>(gb * 1000 * 1000 * 1000, bytes);
        if (gb > 16 && nb < gb * 1000 * 1000 * 1000) break;
        char name[64];
        std::snprintf(name, sizeof name, "k_rand<16>@%lluGB", (unsigned long long)gb);
        timed(name, L, L * 64, [&] { hipLaunchKernelGGL((k_rand<16, false, R>), dim3(blocks), dim3(256), 0, 0, buf, nb / 64, 11ull + gb, out); });
        std::snprintf(name, sizeof name, "k_rand<16,nt>@%lluGB", (unsigned long long)gb);
        timed(name, L, L * 64, [&] { hipLaunchKernelGGL((k_rand<16, true, R>), dim3(blocks), dim3(256), 0, 0, buf, nb / 64, 12ull + gb, out); });
    }
    std::printf("]}\n");
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}

int main(int argc, char **argv) {
    if (argc > 1 && std::string(argv[1]) == "--footprint") return footprint_sweep();
    const uint64_t bytes = 16ull << 30, n_lines = bytes / 64;
    uint4 *buf = nullptr;
    uint32_t *out = nullptr;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 4u << 20));
    CK(hipMemset(buf, 0x5A, bytes));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipDeviceSynchronize());
    const unsigned blocks = 16384;  // 4 M lanes (16 waves per CU of 256 CUs, 16 rounds)
    const uint64_t lanes = (uint64_t)blocks * 256;
    constexpr int R = 8;            // 32 M random lines per kernel: 12 % of the buffer's lines
    const uint64_t L = lanes * R;
    std::printf("{\"buffer_bytes\": %llu, \"kernels\": [\n", (unsigned long long)bytes);
    // each kernel is launched twice (warm + timed): the counters see two dispatches of it
    timed("k_rand<16>", L, L * 64, [&] { hipLaunchKernelGGL((k_rand<16, false, R>), dim3(blocks), dim3(256), 0, 0, buf, n_lines, 1ull, out); });
    timed("k_rand<16,nt>", L, L * 64, [&] { hipLaunchKernelGGL((k_rand<16, true, R>), dim3(blocks), dim3(256), 0, 0, buf, n_lines, 2ull, out); });
    timed("k_rand<8>", L, L * 64, [&] { hipLaunchKernelGGL((k_rand<8, false, R>), dim3(blocks), dim3(256), 0, 0, buf, n_lines, 3ull, out); });
    timed("k_rand<64>", L, L * 64, [&] { hipLaunchKernelGGL((k_rand<64, false, R>), dim3(blocks), dim3(256), 0, 0, buf, n_lines, 4ull, out); });
    timed("k_rand<128>", 2 * L, 2 * L * 64, [&] { hipLaunchKernelGGL((k_rand<128, false, R>), dim3(blocks), dim3(256), 0, 0, buf, n_lines, 5ull, out); });
    for (uint64_t mb : {32ull, 64ull, 128ull, 200ull}) {
        char name[64];
        std::snprintf(name, sizeof name, "k_rand<16>@%lluMB", (unsigned long long)mb);
        const uint64_t nl = (mb << 20) / 64;
        timed(name, L, L * 64, [&] { hipLaunchKernelGGL((k_rand<16, false, R>), dim3(blocks), dim3(256), 0, 0, buf, nl, 6ull + mb, out); });
    }
    const uint64_t small_lines = (64ull << 20) / 64;
    const uint4 *small = buf + (8ull << 30) / 16;  // a 64 MB region in the middle of the buffer
    timed("k_mix<plain,64MB>", 2 * L, 2 * L * 64, [&] { hipLaunchKernelGGL((k_mix<false, R>), dim3(blocks), dim3(256), 0, 0, buf, n_lines / 2, small, small_lines, 9ull, out); });
    timed("k_mix<nt,64MB>", 2 * L, 2 * L * 64, [&] { hipLaunchKernelGGL((k_mix<true, R>), dim3(blocks), dim3(256), 0, 0, buf, n_lines / 2, small, small_lines, 10ull, out); });
    const uint64_t n16 = (4ull << 30) / 16;
    timed("k_stream16", n16 / 4, n16 * 16, [&] { hipLaunchKernelGGL(k_stream16, dim3(8192), dim3(256), 0, 0, buf, n16, out); });
    std::printf("]}\n");
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
