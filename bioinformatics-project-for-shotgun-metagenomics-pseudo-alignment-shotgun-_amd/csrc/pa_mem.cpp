// pa_mem.cpp -- device memory of libpa.so: large buffers from a per-device
// pool of slabs that the library keeps.
//
// Why: giving a large buffer back to the driver is cheap, but the driver
// reclaims freed device memory before it hands it out again, at ~60 GB/s
// (scripts/malloc_probe.py on MI355X: hipMalloc of 8 GB took 3.6-4.7 s once
// ~160 GB had been freed earlier in the process; the same frees made eager by
// GPU_RESOURCE_CACHE_SIZE=0 took 2.5 s themselves).  The EXTSIM flow (C5)
// frees its first index (~200 GB) and builds the index of the kept genomes
// right after, which paid 3.3 s of such stalls.  So buffers of at least
// kPoolMin bytes are carved from slabs (each slab one hipMalloc, never freed
// until pa_mem_trim or an allocation that cannot be met otherwise); a freed
// buffer's range goes back to its slab and is reused, best fit, split and
// coalesced.  Smaller buffers go to hipMalloc / hipFree directly.
//
// PA_POOL=0 turns the pool off (A/B); PA_POOL_MIN_MB overrides kPoolMin.
#include <algorithm>
#include <cstdlib>
#include <iterator>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "pa_internal.h"

namespace pa {

namespace {

constexpr size_t kGranule = 2ull << 20;  // ranges in 2 MiB units

struct Slab {
    int dev;
    char *base;
    size_t size;
    std::map<size_t, size_t> free;  // offset -> length, coalesced
    size_t free_bytes;
};

struct Live {
    size_t slab, off, len;
};

struct Pool {
    std::mutex mu;
    std::vector<Slab> slabs;  // (a trimmed slab keeps its entry with base == nullptr)
    std::unordered_map<void *, Live> live;
    bool on = true;
    size_t min_bytes = 256ull << 20;
    Pool() {
        if (const char *e = std::getenv("PA_POOL")) on = e[0] != '0';
        if (const char *e = std::getenv("PA_POOL_MIN_MB")) min_bytes = std::max<size_t>(1, std::strtoull(e, nullptr, 10)) << 20;
    }
};

Pool &pool() {
    static Pool *p = new Pool();  // (never destroyed: frees may come from static destructors)
    return *p;
}

// Best fit among the free ranges of dev's slabs: (slab, offset) or false.
bool best_fit(Pool &P, int dev, size_t len, size_t &si, size_t &off) {
    size_t best = ~(size_t)0;
    bool found = false;
    for (size_t i = 0; i < P.slabs.size(); i++) {
        const Slab &s = P.slabs[i];
        if (s.dev != dev || !s.base || s.free_bytes < len) continue;
        for (const auto &r : s.free)
            if (r.second >= len && r.second < best) {
                best = r.second, si = i, off = r.first, found = true;
            }
    }
    return found;
}

void take(Slab &s, size_t off, size_t len) {
    auto it = s.free.find(off);
    const size_t rl = it->second;
    s.free.erase(it);
    if (rl > len) s.free[off + len] = rl - len;
    s.free_bytes -= len;
}

void give(Slab &s, size_t off, size_t len) {
    auto next = s.free.lower_bound(off);
    if (next != s.free.end() && off + len == next->first) {
        len += next->second;
        next = s.free.erase(next);
    }
    if (next != s.free.begin()) {
        auto prev = std::prev(next);
        if (prev->first + prev->second == off) {
            prev->second += len;
            return;
        }
    }
    s.free[off] = len;
}

// Slabs of dev with nothing allocated from them go back to the driver.
size_t trim_locked(Pool &P, int dev) {
    size_t n = 0;
    for (Slab &s : P.slabs)
        if (s.base && (dev < 0 || s.dev == dev) && s.free_bytes == s.size) {
            int cur = 0;
            hipGetDevice(&cur);
            if (cur != s.dev) hipSetDevice(s.dev);
            hipFree(s.base);
            if (cur != s.dev) hipSetDevice(cur);
            n += s.size;
            s.base = nullptr;
            s.free.clear();
            s.free_bytes = 0;
        }
    return n;
}

}  // namespace

hipError_t dev_malloc_raw(void **p, size_t n) {
    Pool &P = pool();
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (!P.on || n < P.min_bytes) {
        e = hipMalloc(p, n);
        if (e == hipSuccess || !P.on) return e;
        // small buffers too: idle slabs can hold most of the device's memory
        (void)hipGetLastError();
        {
            std::lock_guard<std::mutex> g(P.mu);
            trim_locked(P, dev);
        }
        return hipMalloc(p, n);
    }
    const size_t len = (n + kGranule - 1) / kGranule * kGranule;
    std::lock_guard<std::mutex> g(P.mu);
    size_t si = 0, off = 0;
    if (!best_fit(P, dev, len, si, off)) {
        void *b = nullptr;
        e = hipMalloc(&b, len);
        if (e != hipSuccess) {  // the pool's idle slabs back to the driver, then once more
            (void)hipGetLastError();
            trim_locked(P, dev);
            e = hipMalloc(&b, len);
            if (e != hipSuccess) return e;
        }
        Slab s;
        s.dev = dev, s.base = (char *)b, s.size = len, s.free_bytes = len;
        s.free[0] = len;
        P.slabs.push_back(std::move(s));
        si = P.slabs.size() - 1, off = 0;
    }
    Slab &s = P.slabs[si];
    take(s, off, len);
    *p = s.base + off;
    P.live[*p] = Live{si, off, len};
    return hipSuccess;
}

hipError_t dev_malloc_try(void **p, size_t n) {
    Pool &P = pool();
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (!P.on || n < P.min_bytes) return dev_malloc_raw(p, n);
    const size_t len = (n + kGranule - 1) / kGranule * kGranule;
    std::lock_guard<std::mutex> g(P.mu);
    size_t si = 0, off = 0;
    if (!best_fit(P, dev, len, si, off)) {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr < len + (1ull << 30)) return hipErrorOutOfMemory;
        void *b = nullptr;
        e = hipMalloc(&b, len);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return hipErrorOutOfMemory;
        }
        Slab s;
        s.dev = dev, s.base = (char *)b, s.size = len, s.free_bytes = len;
        s.free[0] = len;
        P.slabs.push_back(std::move(s));
        si = P.slabs.size() - 1, off = 0;
    }
    Slab &s = P.slabs[si];
    take(s, off, len);
    *p = s.base + off;
    P.live[*p] = Live{si, off, len};
    return hipSuccess;
}

// A pooled range is reusable only once no queued work can still touch it:
// hipFree waits for the device, so the pool does too before the range goes
// back (kernels of the public async API on a caller's stream may still read a
// buffer whose handle was freed; the next dev_malloc could hand the range to a
// memset or copy on another stream).  The range stays in `live` while
// waiting, so no other thread can take it meanwhile.
hipError_t dev_free(void *p) {
    if (!p) return hipSuccess;
    Pool &P = pool();
    int sdev = -1;
    {
        std::lock_guard<std::mutex> g(P.mu);
        auto it = P.live.find(p);
        if (it != P.live.end()) sdev = P.slabs[it->second.slab].dev;
    }
    if (sdev < 0) return hipFree(p);
    int cur = 0;
    hipGetDevice(&cur);
    if (cur != sdev) hipSetDevice(sdev);
    const hipError_t e = hipDeviceSynchronize();
    if (cur != sdev) hipSetDevice(cur);
    std::lock_guard<std::mutex> g(P.mu);
    auto it = P.live.find(p);
    if (it != P.live.end()) {
        Slab &s = P.slabs[it->second.slab];
        s.free_bytes += it->second.len;
        give(s, it->second.off, it->second.len);
        P.live.erase(it);
    }
    return e;
}

// Free memory as one allocation could use it: the driver's free bytes, plus
// every idle slab (a request that fits none is met by trimming them), plus
// the largest free range of a slab in use -- not the sum of scattered ranges,
// which no single buffer can span.  Callers size tables and tiles on this.
size_t dev_pool_largest_free() {
    Pool &P = pool();
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    std::lock_guard<std::mutex> g(P.mu);
    size_t largest = 0;
    for (const Slab &s : P.slabs) {
        if (!s.base || s.dev != dev) continue;
        for (const auto &r : s.free) largest = std::max(largest, r.second);
    }
    return largest;
}

hipError_t dev_mem_info(size_t *free_b, size_t *total_b) {
    hipError_t e = hipMemGetInfo(free_b, total_b);
    if (e != hipSuccess) return e;
    Pool &P = pool();
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return hipSuccess;
    std::lock_guard<std::mutex> g(P.mu);
    size_t largest = 0;
    for (const Slab &s : P.slabs) {
        if (!s.base || s.dev != dev) continue;
        if (s.free_bytes == s.size) {
            *free_b += s.size;
            continue;
        }
        for (const auto &r : s.free) largest = std::max(largest, r.second);
    }
    *free_b += largest;
    return hipSuccess;
}

void dev_pool_stats(int dev, size_t *slab_bytes, size_t *free_bytes) {
    Pool &P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    *slab_bytes = *free_bytes = 0;
    for (const Slab &s : P.slabs)
        if (s.base && s.dev == dev) *slab_bytes += s.size, *free_bytes += s.free_bytes;
}

size_t dev_trim(int dev) {
    Pool &P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    return trim_locked(P, dev);
}

}  // namespace pa

extern "C" pa_status pa_mem_trim(int device, uint64_t *released) {
    const size_t n = pa::dev_trim(device);
    if (released) *released = n;
    return PA_OK;
}
