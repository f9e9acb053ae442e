// Probe: HIP virtual memory (hipMemCreate / hipMemMap) on MI355X against
// hipMalloc -- creation/mapping time, re-mapping kept chunks, and the rate of
// random 16-B reads (the table probes' access pattern) over a 64 GiB range.
//   hipcc --offload-arch=gfx950 -O3 scripts/vmm_probe.hip -o /tmp/vmm_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void k_random(const uint4 *p, uint64_t n16, uint32_t iters, unsigned long long *out) {
    uint64_t h = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * 0x9E3779B97F4A7C15ull + 1;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < iters; i++) {
        h ^= h >> 31, h *= 0xBF58476D1CE4E5B9ull, h ^= h >> 29;
        const uint4 v = p[h % n16];
        acc += v.x ^ v.w;
    }
    if (acc == 0x12345678u) atomicAdd(out, 1ull);
}

static double rate(const void *p, size_t bytes, unsigned long long *out) {
    const uint32_t blocks = 256 * 64, iters = 64;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_random, dim3(blocks), dim3(256), 0, 0, (const uint4 *)p, bytes / 16, iters, out);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 3; r++) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_random, dim3(blocks), dim3(256), 0, 0, (const uint4 *)p, bytes / 16, iters, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
    }
    return (double)blocks * 256 * iters / (best * 1e-3) / 1e9;  // G random reads / s
}

struct Vmm {
    void *va = nullptr;
    size_t size = 0;
    std::vector<hipMemGenericAllocationHandle_t> h;
};

static hipMemAllocationProp prop0() {
    hipMemAllocationProp p = {};
    p.type = hipMemAllocationTypePinned;
    p.location.type = hipMemLocationTypeDevice;
    p.location.id = 0;
    return p;
}

static void map_all(Vmm &v, size_t chunk) {
    CK(hipMemAddressReserve(&v.va, v.size, 0, nullptr, 0));
    for (size_t i = 0; i < v.h.size(); i++) CK(hipMemMap((char *)v.va + i * chunk, chunk, 0, v.h[i], 0));
    hipMemAccessDesc d = {};
    d.location.type = hipMemLocationTypeDevice;
    d.location.id = 0;
    d.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess(v.va, v.size, &d, 1));
}

static void unmap_all(Vmm &v) {
    CK(hipMemUnmap(v.va, v.size));
    CK(hipMemAddressFree(v.va, v.size));
    v.va = nullptr;
}

static Vmm make(size_t size, size_t chunk) {
    Vmm v;
    v.size = size;
    hipMemAllocationProp p = prop0();
    for (size_t o = 0; o < size; o += chunk) {
        hipMemGenericAllocationHandle_t h;
        CK(hipMemCreate(&h, chunk, &p, 0));
        v.h.push_back(h);
    }
    map_all(v, chunk);
    return v;
}

int main() {
    CK(hipSetDevice(0));
    int vmm = 0;
    CK(hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, 0));
    hipMemAllocationProp p = prop0();
    size_t gmin = 0, grec = 0;
    CK(hipMemGetAllocationGranularity(&gmin, &p, hipMemAllocationGranularityMinimum));
    CK(hipMemGetAllocationGranularity(&grec, &p, hipMemAllocationGranularityRecommended));
    std::printf("vmm supported %d granularity min %zu recommended %zu\n", vmm, gmin, grec);
    unsigned long long *out;
    CK(hipMalloc(&out, 8));
    const size_t G = 1ull << 30, S = 64 * G;

    double t = now();
    void *m = nullptr;
    CK(hipMalloc(&m, S));
    CK(hipMemset(m, 1, S));
    CK(hipDeviceSynchronize());
    std::printf("hipMalloc+memset 64 GiB %.3f s\n", now() - t);
    std::printf("random reads hipMalloc      %.2f G/s\n", rate(m, S, out));
    t = now();
    CK(hipFree(m));
    std::printf("hipFree %.3f s\n", now() - t);

    t = now();
    Vmm a = make(S, G);
    std::printf("create+map 64 x 1 GiB (after the free) %.3f s\n", now() - t);
    t = now();
    CK(hipMemset(a.va, 1, S));
    CK(hipDeviceSynchronize());
    std::printf("memset %.3f s\n", now() - t);
    std::printf("random reads vmm 1 GiB      %.2f G/s\n", rate(a.va, S, out));
    t = now();
    unmap_all(a);
    map_all(a, G);
    std::printf("unmap + re-reserve + re-map kept chunks %.3f s\n", now() - t);
    std::printf("random reads vmm remapped   %.2f G/s\n", rate(a.va, S, out));
    // the same chunks in another order (a reused pool: any free chunk anywhere)
    unmap_all(a);
    for (size_t i = 0; i < a.h.size() / 2; i++) std::swap(a.h[i], a.h[a.h.size() - 1 - i]);
    map_all(a, G);
    std::printf("random reads vmm reversed   %.2f G/s\n", rate(a.va, S, out));
    unmap_all(a);
    for (auto h : a.h) CK(hipMemRelease(h));

    t = now();
    Vmm b = make(S, 256ull << 20);
    std::printf("create+map 256 x 256 MiB %.3f s\n", now() - t);
    CK(hipMemset(b.va, 1, S));
    CK(hipDeviceSynchronize());
    std::printf("random reads vmm 256 MiB    %.2f G/s\n", rate(b.va, S, out));
    unmap_all(b);
    for (auto h : b.h) CK(hipMemRelease(h));

    t = now();
    Vmm c = make(4 * G, 2ull << 20);
    std::printf("create+map 2048 x 2 MiB %.3f s\n", now() - t);
    CK(hipMemset(c.va, 1, 4 * G));
    CK(hipDeviceSynchronize());
    void *m2 = nullptr;
    CK(hipMalloc(&m2, 4 * G));
    CK(hipMemset(m2, 1, 4 * G));
    std::printf("random reads 4 GiB: vmm 2 MiB %.2f G/s, hipMalloc %.2f G/s\n", rate(c.va, 4 * G, out),
                rate(m2, 4 * G, out));
    unmap_all(c);
    for (auto h : c.h) CK(hipMemRelease(h));
    CK(hipFree(m2));
    std::printf("done\n");
    return 0;
}
