// pa_dump.hip -- dumpref at scale: the "Kmers" object of
// KmerReference.get_summary() (src/kmer.py:300-329) and its per-genome
// "Summary" counts, made from the device index and streamed to a file
// descriptor as json.dumps(..., indent=4) text.
//
// The reference builds `kmers: Dict[str, Dict[Record, Set[int]]]` (609 B per
// k-mer; C2 would need ~28 GB and hours) and prints, per k-mer in insertion
// order, every genome holding it (FASTA order) with the sorted positions.  The
// same order falls out of one device sort:
//
//   k_dump_first   every indexed window t of the genomes: the first position
//                  fp of its k-mer (atomicMin per table slot) -- the reference's
//                  insertion order is the order of first occurrences;
//   k_dump_keys    K[t] = fp of the window's k-mer (windows of genomes dropped
//                  by EXTSIM, N windows and genome tails: past the end);
//   radix sort     (K, t) pairs by K, stable: the windows of one k-mer become
//                  one run, runs in insertion order, t ascending inside a run
//                  (= genome order, then position: the sorted position lists);
//   k_group_flags  a bit per element: a new k-mer starts here.
//
// The host then formats the runs on `threads` threads (round by round, in
// order) and writes them; the Summary counts (unique / multi-mapping k-mers,
// first appearance, total_bases of the last genome seen) are gathered in the
// same pass.  With EXTSIM the index holds ALL genomes and `keep` masks the
// dropped ones: the reference deletes dropped genomes' entries from the full
// dict (src/kmer.py:232-245), so the surviving k-mers keep the full build's
// order -- which a build from the kept genomes alone would not reproduce.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <cstdlib>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <string>
#include <thread>
#include <vector>

#include "pa_device.h"
#include "pa_internal.h"

using namespace pad;

namespace {

constexpr int kBlock = 256;
constexpr int kRun = 16;  // windows per thread in the genome scans

inline unsigned grid_for(uint64_t n, unsigned block = kBlock) {
    uint64_t g = (n + block - 1) / block;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(g, 1u << 30));
}

template <typename T>
__global__ void k_fill(T *p, uint64_t n, T v) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

template <typename T>
__global__ void k_iota(T *p, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = (T)i;
}

// First position of every k-mer: the smallest window position holding it.
template <int NW>
__global__ void k_dump_first(const uint8_t *__restrict__ codes, uint64_t gstart, uint64_t nwin, int k, uint64_t mask0,
                             const Slot<NW> *__restrict__ table, HomeCfg hc, unsigned long long *fp) {
    const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * kRun;
    if (w0 >= nwin) return;
    const uint64_t w1 = min(w0 + (uint64_t)kRun, nwin);
    const uint8_t *s = codes + gstart + w0;
    Key<NW> key;
#pragma unroll
    for (int j = 0; j < NW; j++) key.w[j] = 0;
    int run = 0;
    for (int i = 0; i < k - 1; i++) {
        const uint32_t c = s[i];
        run = c > 3 ? 0 : run + 1;
        key_push(key, c & 3, mask0);
    }
    for (uint64_t w = w0; w < w1; w++) {
        const uint32_t c = s[w - w0 + k - 1];
        run = c > 3 ? 0 : run + 1;
        key_push(key, c & 3, mask0);
        if (run < k) continue;  // (N windows are not indexed, src/kmer.py:145)
        uint64_t slot;
        uint32_t cls, tpos;
        if (!table_find<NW, true>(table, hc.cap, key, home_of(key, key_hash(key), hc), slot, cls, tpos)) continue;
        const unsigned long long t = gstart + w;
        if (fp[slot] > t) atomicMin(&fp[slot], t);  // (a stale plain load only costs an atomic)
    }
}

// K[t] = first position of the k-mer at window t (windows of a kept genome).
template <int NW, typename T>
__global__ void k_dump_keys(const uint8_t *__restrict__ codes, uint64_t gstart, uint64_t nwin, int k, uint64_t mask0,
                            const Slot<NW> *__restrict__ table, HomeCfg hc, const unsigned long long *__restrict__ fp,
                            T *K, unsigned long long *n_valid) {
    const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * kRun;
    uint32_t cnt = 0;
    if (w0 < nwin) {
        const uint64_t w1 = min(w0 + (uint64_t)kRun, nwin);
        const uint8_t *s = codes + gstart + w0;
        Key<NW> key;
#pragma unroll
        for (int j = 0; j < NW; j++) key.w[j] = 0;
        int run = 0;
        for (int i = 0; i < k - 1; i++) {
            const uint32_t c = s[i];
            run = c > 3 ? 0 : run + 1;
            key_push(key, c & 3, mask0);
        }
        for (uint64_t w = w0; w < w1; w++) {
            const uint32_t c = s[w - w0 + k - 1];
            run = c > 3 ? 0 : run + 1;
            key_push(key, c & 3, mask0);
            if (run < k) continue;
            uint64_t slot;
            uint32_t cls, tpos;
            if (!table_find<NW, true>(table, hc.cap, key, home_of(key, key_hash(key), hc), slot, cls, tpos)) continue;
            K[gstart + w] = (T)fp[slot];
            cnt++;
        }
    }
    // one atomic per wave
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_down(cnt, o);
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(n_valid, (unsigned long long)cnt);
}

// Bit i of flags: element i starts a new k-mer (its key differs from i - 1).
template <typename T>
__global__ void k_group_flags(const T *__restrict__ K, uint64_t n, unsigned long long *flags) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool start = i < n && (i == 0 || K[i] != K[i - 1]);
    const unsigned long long m = __ballot(start);
    if ((threadIdx.x & 63) == 0 && i < n) flags[i >> 6] = m;
}

template <int NW>
void launch_first(const pa_index *idx, unsigned long long *fp, hipStream_t st) {
    const int k = (int)idx->k;
    const int bits = 2 * k - 64 * (NW - 1);
    const uint64_t mask0 = bits >= 64 ? ~0ull : ((1ull << bits) - 1);
    for (uint32_t g = 0; g < idx->n_genomes; g++) {
        const uint64_t len = idx->h_goff[g + 1] - idx->h_goff[g];
        if ((uint64_t)k > len) continue;
        const uint64_t nwin = len - k + 1;
        hipLaunchKernelGGL(k_dump_first<NW>, dim3(grid_for((nwin + kRun - 1) / kRun)), dim3(kBlock), 0, st,
                           idx->codes, idx->h_goff[g], nwin, k, mask0, (const Slot<NW> *)idx->table, idx->home, fp);
    }
}

template <int NW, typename T>
void launch_keys(const pa_index *idx, const uint8_t *keep, const unsigned long long *fp, T *K,
                 unsigned long long *n_valid, hipStream_t st) {
    const int k = (int)idx->k;
    const int bits = 2 * k - 64 * (NW - 1);
    const uint64_t mask0 = bits >= 64 ? ~0ull : ((1ull << bits) - 1);
    for (uint32_t g = 0; g < idx->n_genomes; g++) {
        const uint64_t len = idx->h_goff[g + 1] - idx->h_goff[g];
        if ((uint64_t)k > len || (keep && !keep[g])) continue;
        const uint64_t nwin = len - k + 1;
        hipLaunchKernelGGL((k_dump_keys<NW, T>), dim3(grid_for((nwin + kRun - 1) / kRun)), dim3(kBlock), 0, st,
                           idx->codes, idx->h_goff[g], nwin, k, mask0, (const Slot<NW> *)idx->table, idx->home, fp, K,
                           n_valid);
    }
}

// ---- host side: the runs -> json.dumps(indent=4) text ------------------------------

struct DescAcc {  // the Summary entry of one description, gathered per thread
    uint64_t uniq = 0, multi = 0;
    uint64_t first_e = ~0ull, first_j = 0;  // first appearance: (run start, place in the run's genome list)
    uint64_t last_e = 0, last_j = 0;        // last appearance (its genome gives total_bases)
    uint32_t last_g = 0xFFFFFFFFu;
};

struct Runs {
    const uint64_t *t;          // sorted window positions (as uint64)
    const uint64_t *flags;      // run starts
    uint64_t n;
    int64_t k;
    const uint8_t *codes;       // host copy of the genome codes (k-mer text)
    const std::vector<uint64_t> *goff;
    const uint32_t *desc_of;
    const char *const *desc_json;
    bool dup_desc;              // two genomes share a description (dict-key merge, quirk 9)

    bool is_start(uint64_t i) const { return (flags[i >> 6] >> (i & 63)) & 1ull; }
    uint64_t next_start(uint64_t i) const {  // first run start >= i (n if none)
        while (i < n) {
            const uint64_t w = flags[i >> 6] >> (i & 63);
            if (w) return std::min(n, i + (uint64_t)__builtin_ctzll(w));
            i = (i | 63) + 1;
        }
        return n;
    }
    uint32_t genome_of(uint64_t t) const {
        return (uint32_t)(std::upper_bound(goff->begin(), goff->end(), t) - goff->begin() - 1);
    }
};

inline void put_u64(std::string &s, uint64_t v) {
    char b[24];
    const auto r = std::to_chars(b, b + sizeof b, v);
    s.append(b, r.ptr);
}

// Runs starting in [a, e) (a is a run start, e a run start or n) into `out`.
void format_runs(const Runs &R, uint64_t a, uint64_t e, std::string &out, std::vector<DescAcc> &acc) {
    static const char kBase[4] = {'A', 'C', 'G', 'T'};
    struct Ent {
        uint32_t g;
        uint64_t b, e;  // element range
    };
    std::vector<Ent> ents;
    std::vector<int> show;  // indices into ents, one per description in first-appearance order
    for (uint64_t s = a; s < e;) {
        const uint64_t end = R.next_start(s + 1);
        ents.clear();
        for (uint64_t i = s; i < end;) {
            const uint32_t g = R.genome_of(R.t[i]);
            const uint64_t ge = (*R.goff)[g + 1];
            uint64_t j = i + 1;
            while (j < end && R.t[j] < ge) j++;
            ents.push_back({g, i, j});
            i = j;
        }
        const bool uniq = ents.size() == 1;
        show.clear();
        if (!R.dup_desc) {
            for (int j = 0; j < (int)ents.size(); j++) show.push_back(j);
        } else {  // a dict keyed by description: first key position, last genome's positions
            for (int j = 0; j < (int)ents.size(); j++) {
                bool seen = false;
                for (int &x : show)
                    if (R.desc_of[ents[x].g] == R.desc_of[ents[j].g]) {
                        x = j;
                        seen = true;
                        break;
                    }
                if (!seen) show.push_back(j);
            }
        }
        // Summary counts: each description once per k-mer; appearances in the
        // reference's walk order (k-mers, then each k-mer's genomes)
        for (int j = 0; j < (int)ents.size(); j++) {
            DescAcc &d = acc[R.desc_of[ents[j].g]];
            if (d.first_e == ~0ull || s < d.first_e || (s == d.first_e && (uint64_t)j < d.first_j)) {
                d.first_e = s;
                d.first_j = (uint64_t)j;
            }
            if (s > d.last_e || (s == d.last_e && (uint64_t)j >= d.last_j) || d.last_g == 0xFFFFFFFFu) {
                d.last_e = s;
                d.last_j = (uint64_t)j;
                d.last_g = ents[j].g;
            }
        }
        for (int x : show) {
            DescAcc &d = acc[R.desc_of[ents[x].g]];
            (uniq ? d.uniq : d.multi)++;
        }
        // text
        if (s != 0) out.append(",\n");
        out.append(8, ' ');
        out.push_back('"');
        const uint64_t t0 = R.t[s];
        for (int64_t q = 0; q < R.k; q++) out.push_back(kBase[R.codes[t0 + q] & 3]);
        out.append("\": {\n");
        for (size_t xi = 0; xi < show.size(); xi++) {
            const Ent &en = ents[show[xi]];
            out.append(12, ' ');
            out.append(R.desc_json[R.desc_of[en.g]]);
            out.append(": [\n");
            const uint64_t base = (*R.goff)[en.g];
            for (uint64_t i = en.b; i < en.e; i++) {
                out.append(16, ' ');
                put_u64(out, R.t[i] - base);
                out.append(i + 1 < en.e ? ",\n" : "\n");
            }
            out.append(12, ' ');
            out.append(xi + 1 < show.size() ? "],\n" : "]\n");
        }
        out.append(8, ' ');
        out.push_back('}');
        s = end;
    }
}

bool write_all(int fd, const std::string &s) {
    const char *p = s.data();
    size_t left = s.size();
    while (left) {
        const ssize_t w = ::write(fd, p, left);
        if (w < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        p += w;
        left -= (size_t)w;
    }
    return true;
}

template <typename T, int NW>
pa_status dump_t(const pa_index *idx, const uint8_t *keep, unsigned long long *fp, uint64_t total, hipStream_t st,
                 std::vector<uint64_t> &h_t, std::vector<uint64_t> &h_flags, uint64_t &n_valid) {
    T *K = nullptr, *K2 = nullptr, *V = nullptr, *V2 = nullptr;
    unsigned long long *d_n = nullptr, *d_flags = nullptr;
    void *tmp = nullptr;
    auto cleanup = [&] {
        pa::dev_free(K); pa::dev_free(K2); pa::dev_free(V); pa::dev_free(V2); pa::dev_free(d_n); pa::dev_free(d_flags); pa::dev_free(tmp);
    };
#define D_HIP(call)                                                                                       \
    do {                                                                                                  \
        hipError_t e_ = (call);                                                                           \
        if (e_ != hipSuccess) {                                                                           \
            pa::set_error(std::string("pa_index_dumpref: ") + hipGetErrorString(e_) + " (" #call ")");  \
            cleanup();                                                                                    \
            return e_ == hipErrorOutOfMemory ? PA_ENOMEM : PA_EDEVICE;                                    \
        }                                                                                                 \
    } while (0)
    const unsigned fg = grid_for(total) > 65536 ? 65536 : grid_for(total);
    D_HIP(pa::dev_malloc(&K, total * sizeof(T)));
    D_HIP(pa::dev_malloc(&K2, total * sizeof(T)));
    D_HIP(pa::dev_malloc(&V, total * sizeof(T)));
    D_HIP(pa::dev_malloc(&V2, total * sizeof(T)));
    D_HIP(pa::dev_malloc(&d_n, 8));
    D_HIP(hipMemsetAsync(d_n, 0, 8, st));
    hipLaunchKernelGGL(k_fill<T>, dim3(fg), dim3(kBlock), 0, st, K, total, (T)total);
    hipLaunchKernelGGL(k_iota<T>, dim3(fg), dim3(kBlock), 0, st, V, total);
    launch_keys<NW, T>(idx, keep, fp, K, d_n, st);
    D_HIP(hipGetLastError());
    unsigned end_bit = 1;
    while (end_bit < 8 * sizeof(T) && (total >> end_bit)) end_bit++;
    rocprim::double_buffer<T> kb(K, K2), vb(V, V2);
    size_t tmp_bytes = 0;
    D_HIP(rocprim::radix_sort_pairs(nullptr, tmp_bytes, kb, vb, total, 0, end_bit, st));
    D_HIP(pa::dev_malloc(&tmp, std::max<size_t>(tmp_bytes, 16)));
    D_HIP(rocprim::radix_sort_pairs(tmp, tmp_bytes, kb, vb, total, 0, end_bit, st));
    unsigned long long nv = 0;
    D_HIP(hipMemcpyAsync(&nv, d_n, 8, hipMemcpyDeviceToHost, st));
    D_HIP(hipStreamSynchronize(st));
    n_valid = nv;
    const uint64_t nwords = (nv + 63) / 64;
    D_HIP(pa::dev_malloc(&d_flags, std::max<uint64_t>(nwords, 1) * 8));
    if (nv) {
        hipLaunchKernelGGL(k_group_flags<T>, dim3((unsigned)((nv + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                           kb.current(), nv, d_flags);
        D_HIP(hipGetLastError());
    }
    h_flags.assign(std::max<uint64_t>(nwords, 1), 0);
    h_t.resize(std::max<uint64_t>(nv, 1));
    std::vector<T> tv(std::max<uint64_t>(nv, 1));
    if (nv) {
        D_HIP(hipMemcpyAsync(h_flags.data(), d_flags, nwords * 8, hipMemcpyDeviceToHost, st));
        D_HIP(hipMemcpyAsync(tv.data(), vb.current(), nv * sizeof(T), hipMemcpyDeviceToHost, st));
    }
    D_HIP(hipStreamSynchronize(st));
#undef D_HIP
    cleanup();
    for (uint64_t i = 0; i < nv; i++) h_t[i] = tv[i];
    return PA_OK;
}

template <int NW>
pa_status dump_nw(const pa_index *idx, const uint8_t *keep, hipStream_t st, std::vector<uint64_t> &h_t,
                  std::vector<uint64_t> &h_flags, uint64_t &n_valid) {
    const uint64_t total = idx->h_goff[idx->n_genomes];
    unsigned long long *fp = nullptr;
    PA_HIP(pa::dev_malloc(&fp, idx->cap * 8));
    const unsigned fg = grid_for(idx->cap) > 65536 ? 65536 : grid_for(idx->cap);
    hipLaunchKernelGGL(k_fill<unsigned long long>, dim3(fg), dim3(kBlock), 0, st, fp, idx->cap, ~0ull);
    launch_first<NW>(idx, fp, st);
    hipError_t e = hipGetLastError();
    pa_status rc = PA_OK;
    if (e != hipSuccess) {
        pa::set_error(std::string("pa_index_dumpref: ") + hipGetErrorString(e));
        rc = PA_EDEVICE;
    } else if (total < 0xFFFFFFFFull) {
        rc = dump_t<uint32_t, NW>(idx, keep, fp, total, st, h_t, h_flags, n_valid);
    } else {
        rc = dump_t<uint64_t, NW>(idx, keep, fp, total, st, h_t, h_flags, n_valid);
    }
    hipStreamSynchronize(st);
    pa::dev_free(fp);
    return rc;
}

}  // namespace

namespace pa {

pa_status index_dumpref(const pa_index *idx, const uint8_t *keep, const uint32_t *desc_of, uint32_t n_desc,
                        const char *const *desc_json, int fd, int threads, uint64_t *desc_unique, uint64_t *desc_multi,
                        uint64_t *desc_order, uint32_t *desc_last_genome, uint64_t *n_kmers_out, hipStream_t st) {
    const uint32_t G = idx->n_genomes;
    for (uint32_t d = 0; d < n_desc; d++) {
        desc_unique[d] = desc_multi[d] = 0;
        desc_order[d] = ~0ull;
        desc_last_genome[d] = 0xFFFFFFFFu;
    }
    for (uint32_t g = 0; g < G; g++)
        if (desc_of[g] >= n_desc) {
            set_error("pa_index_dumpref: desc_of[g] >= n_desc");
            return PA_EINVAL;
        }
    std::vector<uint64_t> h_t, h_flags;
    uint64_t nv = 0;
    if (idx->k > 0 && idx->n_kmers > 0) {
        pa_status rc = PA_EUNSUPPORTED;
        switch (idx->nw) {
            case 1: rc = dump_nw<1>(idx, keep, st, h_t, h_flags, nv); break;
            case 2: rc = dump_nw<2>(idx, keep, st, h_t, h_flags, nv); break;
            case 3: rc = dump_nw<3>(idx, keep, st, h_t, h_flags, nv); break;
            case 4: rc = dump_nw<4>(idx, keep, st, h_t, h_flags, nv); break;
            case 5: rc = dump_nw<5>(idx, keep, st, h_t, h_flags, nv); break;
            case 6: rc = dump_nw<6>(idx, keep, st, h_t, h_flags, nv); break;
            case 7: rc = dump_nw<7>(idx, keep, st, h_t, h_flags, nv); break;
            case 8: rc = dump_nw<8>(idx, keep, st, h_t, h_flags, nv); break;
            default: set_error("unsupported k");
        }
        if (rc != PA_OK) return rc;
    }
    if (nv == 0) {
        if (n_kmers_out) *n_kmers_out = 0;
        return write_all(fd, "{}") ? PA_OK : (set_error("pa_index_dumpref: write failed"), PA_EIO);
    }
    // the genome codes (k-mer text) on the host
    const uint64_t total = idx->h_goff[G];
    std::vector<uint8_t> codes(total);
    PA_HIP(hipMemcpy(codes.data(), idx->codes, total, hipMemcpyDeviceToHost));
    std::vector<uint32_t> seen_desc(n_desc, 0);
    bool dup = false;
    for (uint32_t g = 0; g < G; g++) dup |= seen_desc[desc_of[g]]++ > 0;
    Runs R{h_t.data(), h_flags.data(), nv, idx->k, codes.data(), &idx->h_goff, desc_of, desc_json, dup};
    const int T = std::max(1, std::min(threads, 64));
    std::vector<std::vector<DescAcc>> acc(T, std::vector<DescAcc>(n_desc));
    std::vector<std::string> bufs(T);
    uint64_t runs = 0;
    for (uint64_t i = 0; i < (nv + 63) / 64; i++) runs += (uint64_t)__builtin_popcountll(h_flags[i]);
    if (!write_all(fd, "{\n")) {
        set_error("pa_index_dumpref: write failed");
        return PA_EIO;
    }
    uint64_t kRound = 8ull << 20;  // elements per round (bounded text in memory); PA_DUMP_ROUND: tests
    if (const char *r = std::getenv("PA_DUMP_ROUND")) kRound = std::max<uint64_t>(1, std::strtoull(r, nullptr, 10));
    for (uint64_t a = 0; a < nv;) {
        const uint64_t e = R.next_start(std::min(nv, a + kRound));
        std::vector<uint64_t> cut(T + 1);
        cut[0] = a;
        cut[T] = e;
        for (int t = 1; t < T; t++) cut[t] = std::max(cut[t - 1], R.next_start(a + (e - a) * t / T));
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                bufs[t].clear();
                if (cut[t] < cut[t + 1]) format_runs(R, cut[t], cut[t + 1], bufs[t], acc[t]);
            });
        for (auto &x : th) x.join();
        for (int t = 0; t < T; t++)
            if (!write_all(fd, bufs[t])) {
                set_error("pa_index_dumpref: write failed");
                return PA_EIO;
            }
        a = e;
    }
    if (!write_all(fd, "\n    }")) {
        set_error("pa_index_dumpref: write failed");
        return PA_EIO;
    }
    // merge the threads' Summary counts; order = first appearance
    std::vector<DescAcc> m(n_desc);
    for (int t = 0; t < T; t++)
        for (uint32_t d = 0; d < n_desc; d++) {
            const DescAcc &x = acc[t][d];
            DescAcc &y = m[d];
            y.uniq += x.uniq;
            y.multi += x.multi;
            if (x.first_e != ~0ull && (y.first_e == ~0ull || x.first_e < y.first_e ||
                                       (x.first_e == y.first_e && x.first_j < y.first_j))) {
                y.first_e = x.first_e;
                y.first_j = x.first_j;
            }
            if (x.last_g != 0xFFFFFFFFu && (y.last_g == 0xFFFFFFFFu || x.last_e > y.last_e ||
                                            (x.last_e == y.last_e && x.last_j >= y.last_j))) {
                y.last_e = x.last_e;
                y.last_j = x.last_j;
                y.last_g = x.last_g;
            }
        }
    std::vector<uint32_t> order;
    for (uint32_t d = 0; d < n_desc; d++)
        if (m[d].first_e != ~0ull) order.push_back(d);
    std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
        return m[x].first_e != m[y].first_e ? m[x].first_e < m[y].first_e : m[x].first_j < m[y].first_j;
    });
    for (size_t r = 0; r < order.size(); r++) desc_order[order[r]] = r;
    for (uint32_t d = 0; d < n_desc; d++) {
        desc_unique[d] = m[d].uniq;
        desc_multi[d] = m[d].multi;
        desc_last_genome[d] = m[d].last_g;
    }
    if (n_kmers_out) *n_kmers_out = runs;
    return PA_OK;
}

}  // namespace pa

namespace {
__global__ void k_warm_dump() {}
}  // namespace

namespace pa {
// Loads this file's code object (a first launch from a module loads it): the
// CLI's runtime-start thread calls it so that the load overlaps host work.
void warm_dump(hipStream_t st) { hipLaunchKernelGGL(k_warm_dump, dim3(1), dim3(64), 0, st); }
}  // namespace pa
