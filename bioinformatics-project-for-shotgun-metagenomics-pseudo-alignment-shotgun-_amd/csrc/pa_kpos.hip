// Positions of k-mers in the genomes: KmerReference.get_kmer_references
// (src/kmer.py:292-298: kmers[kmer] = {genome record: set of positions}) and
// get_kmer_and_reverse_references (src/kmer.py:331-351: the k-mer's and its
// reverse complement's positions, merged per genome) as one batched device pass.
//
// The index keeps, per k-mer, its genome set and its first occurrence only (the
// align path needs nothing else), so positions come from a scan of the genome
// codes the index holds (idx->codes, 1 B per base): the query keys -- forward
// and, on request, reverse-complement, deduplicated -- go into a small
// open-addressing table (L2-resident), and one thread per run of kScanRun
// windows rolls the 2-bit key over its bases and probes that table for every
// window that lies inside one genome and holds only A/C/G/T (the reference
// skips 'N' k-mers, src/kmer.py:145).  HBM-bound: 1 B of codes per window
// (C2: 100 MB, ~20 us at 5 TB/s), against the reference's dict of every
// position of every k-mer in host memory.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "pa_device.h"
#include "pa_internal.h"

using namespace pad;

namespace {

constexpr int kBlock = 256;
constexpr int kScanRun = 64;  // windows per thread

// Query-table entry: a packed key (NW words, the index's layout) and the id of
// the distinct key it stands for.  key[0] == EMPTY marks a free entry.
template <int NW>
struct QEnt {
    uint64_t key[NW];
    uint32_t id;
    uint32_t pad;
};

// Device hit: distinct key id, genome, genome-local window position.
struct DevHit {
    uint32_t id;
    uint32_t genome;
    uint64_t pos;
};

inline uint64_t mask0_host(int k, int nw) {
    const int bits = 2 * k - 64 * (nw - 1);
    return bits >= 64 ? ~0ull : ((1ull << bits) - 1);
}

inline uint64_t host_fmix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

template <int NW>
__global__ void k_kmer_scan(const uint8_t *__restrict__ codes, const uint64_t *__restrict__ goff, uint32_t G,
                            int k, uint64_t mask0, const QEnt<NW> *__restrict__ qt, uint64_t qmask,
                            unsigned long long *__restrict__ n_hits, DevHit *__restrict__ hits, uint64_t cap) {
    const uint64_t total = goff[G];
    const uint64_t t0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * kScanRun;
    if (t0 >= total) return;
    const uint64_t t1 = min(t0 + (uint64_t)kScanRun, total);
    // genome holding t0: the last g with goff[g] <= t0 (empty genomes skipped)
    uint32_t lo = 0, hi = G;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (goff[mid] <= t0)
            lo = mid;
        else
            hi = mid;
    }
    uint32_t g = lo;
    uint64_t gend = goff[g + 1];
    while (gend <= t0 && g + 1 < G) gend = goff[++g + 1];
    Key<NW> key;
#pragma unroll
    for (int j = 0; j < NW; j++) key.w[j] = 0;
    // the last non-ACGT position seen (the window [t, t + k) is clean iff bad < t)
    int64_t bad = (int64_t)t0 - 1;
    for (int i = 0; i < k - 1; i++) {
        const uint64_t p = t0 + i;
        const uint32_t c = p < total ? codes[p] : 4u;
        if (c > 3) bad = (int64_t)p;
        key_push(key, c & 3, mask0);
    }
    for (uint64_t t = t0; t < t1; t++) {
        const uint64_t p = t + k - 1;
        const uint32_t c = p < total ? codes[p] : 4u;
        if (c > 3) bad = (int64_t)p;
        key_push(key, c & 3, mask0);
        while (t >= gend && g + 1 < G) gend = goff[++g + 1];
        if (bad >= (int64_t)t || t + k > gend) continue;  // N inside, or across a genome end
        uint64_t e = key_hash(key) & qmask;
        for (;;) {
            const QEnt<NW> q = qt[e];
            if (q.key[0] == EMPTY) break;
            bool eq = true;
#pragma unroll
            for (int j = 0; j < NW; j++) eq &= q.key[j] == key.w[j];
            if (eq) {
                const unsigned long long slot = atomicAdd(n_hits, 1ull);
                if (slot < cap) hits[slot] = DevHit{q.id, g, t - goff[g]};
                break;
            }
            e = (e + 1) & qmask;
        }
    }
}

// 2-bit packing of one k-mer text (MSB-first, the index's key layout); false
// when it holds anything but A/C/G/T.
bool pack_host(const char *s, int k, int nw, uint64_t *w) {
    for (int j = 0; j < nw; j++) w[j] = 0;
    const int bits0 = 2 * k - 64 * (nw - 1);
    const uint64_t mask0 = bits0 >= 64 ? ~0ull : ((1ull << bits0) - 1);
    for (int i = 0; i < k; i++) {
        uint32_t c;
        switch (s[i]) {
            case 'A': c = 0; break;
            case 'C': c = 1; break;
            case 'G': c = 2; break;
            case 'T': c = 3; break;
            default: return false;
        }
        for (int j = 0; j < nw - 1; j++) w[j] = (w[j] << 2) | (w[j + 1] >> 62);
        w[nw - 1] = (w[nw - 1] << 2) | c;
        w[0] &= mask0;
    }
    return true;
}

template <int NW>
pa_status scan_nw(const pa_index *idx, const std::vector<uint64_t> &keys, size_t n_keys,
                  std::vector<DevHit> &out, hipStream_t st) {
    const int k = (int)idx->k;
    uint64_t qsize = 64;
    while (qsize < 2 * n_keys) qsize <<= 1;
    std::vector<QEnt<NW>> qt(qsize);
    for (auto &q : qt) {
        for (int j = 0; j < NW; j++) q.key[j] = EMPTY;
        q.id = 0;
        q.pad = 0;
    }
    for (size_t u = 0; u < n_keys; u++) {
        const uint64_t *w = &keys[u * NW];
        uint64_t h = 0x9E3779B97F4A7C15ull;  // key_hash (pa_device.h)
        for (int j = 0; j < NW; j++) h = host_fmix64(h ^ w[j]);
        uint64_t e = h & (qsize - 1);
        while (qt[e].key[0] != EMPTY) e = (e + 1) & (qsize - 1);
        for (int j = 0; j < NW; j++) qt[e].key[j] = w[j];
        qt[e].id = (uint32_t)u;
    }
    const uint64_t total = idx->h_goff[idx->n_genomes];
    const uint64_t threads = (total + kScanRun - 1) / kScanRun;
    const unsigned grid = (unsigned)std::max<uint64_t>((threads + kBlock - 1) / kBlock, 1);
    QEnt<NW> *d_qt = nullptr;
    unsigned long long *d_n = nullptr;
    DevHit *d_hits = nullptr;
    uint64_t cap = 1u << 16;
    pa_status rc = PA_OK;
    // (every exit below goes through the one cleanup at the end)
    if (pa::dev_malloc(&d_qt, qsize * sizeof(QEnt<NW>)) != hipSuccess || pa::dev_malloc(&d_n, 8) != hipSuccess) {
        pa::set_error("pa_index_positions: out of device memory for the query table");
        rc = PA_ENOMEM;
    } else if (hipMemcpyAsync(d_qt, qt.data(), qsize * sizeof(QEnt<NW>), hipMemcpyHostToDevice, st) != hipSuccess) {
        pa::set_error("pa_index_positions: HIP error copying the query table");
        rc = PA_EDEVICE;
    }
    for (int attempt = 0; rc == PA_OK && attempt < 2; attempt++) {
        if (pa::dev_malloc(&d_hits, cap * sizeof(DevHit)) != hipSuccess) {
            d_hits = nullptr;
            pa::set_error("pa_index_positions: out of device memory for the hits");
            rc = PA_ENOMEM;
            break;
        }
        unsigned long long n = 0;
        if (hipMemsetAsync(d_n, 0, 8, st) != hipSuccess) rc = PA_EDEVICE;
        if (rc == PA_OK && total >= (uint64_t)k && k > 0)
            hipLaunchKernelGGL(k_kmer_scan<NW>, dim3(grid), dim3(kBlock), 0, st, idx->codes, idx->goff,
                               idx->n_genomes, k, mask0_host(k, NW), d_qt, qsize - 1, d_n, d_hits, cap);
        if (rc == PA_OK && (hipGetLastError() != hipSuccess ||
                            hipMemcpyAsync(&n, d_n, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
                            hipStreamSynchronize(st) != hipSuccess)) {
            pa::set_error("pa_index_positions: HIP error in the scan");
            rc = PA_EDEVICE;
        }
        if (rc != PA_OK) break;
        if (n <= cap) {
            out.resize(n);
            if (n && hipMemcpy(out.data(), d_hits, n * sizeof(DevHit), hipMemcpyDeviceToHost) != hipSuccess) {
                pa::set_error("pa_index_positions: HIP error copying the hits");
                rc = PA_EDEVICE;
            }
            break;
        }
        pa::dev_free(d_hits);  // more hits than room: once more with room for all of them
        d_hits = nullptr;
        cap = n;
    }
    if (d_hits) pa::dev_free(d_hits);
    if (d_qt) pa::dev_free(d_qt);
    if (d_n) pa::dev_free(d_n);
    return rc;
}

}  // namespace

namespace pa {

// (pa_index_positions, include/pa.h)
pa_status index_positions(const pa_index *idx, const char *kmers, uint64_t n, uint32_t kmer_len, uint32_t flags,
                          pa_kmer_hit *hits, uint64_t cap, uint64_t *n_hits, hipStream_t st) {
    *n_hits = 0;
    // k-mers of another length, or with anything but A/C/G/T, are not keys of
    // the reference's dict (src/kmer.py:140-150): no positions
    if (n == 0 || (int64_t)kmer_len != idx->k || idx->k <= 0 || idx->n_kmers == 0) return PA_OK;
    const int k = (int)idx->k, nw = idx->nw;
    // distinct keys: a query's forward key, and with PA_POS_REVERSE its
    // reverse complement unless that is the same k-mer (src/kmer.py:342-343);
    // refs[u] lists the (query << 1 | strand) entries key u answers
    std::vector<uint64_t> keys;
    std::vector<std::vector<uint32_t>> refs;
    std::vector<uint64_t> w(nw), wr(nw);
    std::vector<char> rc(kmer_len);
    // exact dedup by sort of (key words, entry)
    std::vector<std::pair<std::vector<uint64_t>, uint32_t>> ent;
    ent.reserve((flags & PA_POS_REVERSE) ? 2 * n : n);
    for (uint64_t q = 0; q < n; q++) {
        const char *s = kmers + q * kmer_len;
        if (!pack_host(s, k, nw, w.data())) continue;
        ent.emplace_back(w, (uint32_t)(q << 1));
        if (flags & PA_POS_REVERSE) {
            for (int i = 0; i < k; i++) {
                const char c = s[k - 1 - i];
                rc[i] = c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : 'A';
            }
            pack_host(rc.data(), k, nw, wr.data());
            if (wr != w) ent.emplace_back(wr, (uint32_t)(q << 1 | 1));
        }
    }
    if (ent.empty()) return PA_OK;
    std::sort(ent.begin(), ent.end());
    for (size_t i = 0; i < ent.size(); i++) {
        if (i == 0 || ent[i].first != ent[i - 1].first) {
            keys.insert(keys.end(), ent[i].first.begin(), ent[i].first.end());
            refs.emplace_back();
        }
        refs.back().push_back(ent[i].second);
    }
    std::vector<DevHit> dh;
    pa_status s;
    switch (nw) {
        case 1: s = scan_nw<1>(idx, keys, refs.size(), dh, st); break;
        case 2: s = scan_nw<2>(idx, keys, refs.size(), dh, st); break;
        case 3: s = scan_nw<3>(idx, keys, refs.size(), dh, st); break;
        case 4: s = scan_nw<4>(idx, keys, refs.size(), dh, st); break;
        case 5: s = scan_nw<5>(idx, keys, refs.size(), dh, st); break;
        case 6: s = scan_nw<6>(idx, keys, refs.size(), dh, st); break;
        case 7: s = scan_nw<7>(idx, keys, refs.size(), dh, st); break;
        default: s = scan_nw<8>(idx, keys, refs.size(), dh, st); break;
    }
    if (s != PA_OK) return s;
    std::vector<pa_kmer_hit> outv;
    for (const DevHit &h : dh)
        for (uint32_t e : refs[h.id]) outv.push_back(pa_kmer_hit{(e >> 1) | ((e & 1u) << 31), h.genome, h.pos});
    // (query, strand, genome, position) ascending
    std::sort(outv.begin(), outv.end(), [](const pa_kmer_hit &a, const pa_kmer_hit &b) {
        const uint64_t ka = ((uint64_t)(a.query & 0x7FFFFFFFu) << 1) | (a.query >> 31);
        const uint64_t kb = ((uint64_t)(b.query & 0x7FFFFFFFu) << 1) | (b.query >> 31);
        if (ka != kb) return ka < kb;
        if (a.genome != b.genome) return a.genome < b.genome;
        return a.position < b.position;
    });
    *n_hits = outv.size();
    if (hits && cap) std::memcpy(hits, outv.data(), std::min<uint64_t>(cap, outv.size()) * sizeof(pa_kmer_hit));
    return PA_OK;
}

}  // namespace pa
