// pa_fastq.hip -- FASTQ files parsed ON THE DEVICE, streamed into the align
// pass (pa_align_fastq_file).
//
// The reference reads a whole FASTQ file into a str (src/data_file.py:117-158),
// parses it with a regular expression (src/records.py:245-302) and aligns the
// records one by one (src/kmer.py:600-620).  Here the host only moves bytes:
// the file is read in windows (multi-threaded pread, or zlib for .gz) into
// pinned buffers and copied to HBM on a copy stream, and the device does the
// rest on the align stream, window after window while the host reads the next:
//
//   k_nl_count / scan / k_nl_write   line breaks of the window (4 KiB tiles,
//                                    16 B per lane, coalesced)
//   k_window_meta                    complete records in the window; the
//                                    incomplete tail is carried into the next
//   k_records                        per record: header / "+" / lengths, the
//                                    id's hash into a device set (duplicates)
//   scan, k_compact                  every byte checked against its line's
//                                    class; sequence and quality bytes packed
//                                    into the align path's columns (CSR)
//   pa::align                        the window's reads (global read index =
//                                    record index in the file)
//
// Accepted is a strict subset of the reference grammar: LF line ends only,
// exactly four lines per record from the first byte on, "@" + id of bytes
// 0x21-0x7E / space / tab that neither starts nor ends with space or tab,
// a non-empty A C G T sequence, a "+" line, qualities 0x21-0x7E of the
// sequence's length, one optional final line break, ids unique.  Inside it the
// records are exactly the reference's; anything else -- a CRLF file, a "+id"
// line, a blank line, a duplicate id -- returns PA_ENOTCANON and the caller
// parses the file with the exact grammar (records.py), which reproduces the
// reference's records or its exception.

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <chrono>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <string>
#include <deque>
#include <thread>
#include <vector>

#include "pa_device.h"
#include "pa_gz.h"
#include "pa_internal.h"

using namespace pad;

namespace {

constexpr int kTile = 4096;         // bytes per newline tile (256 lanes x 16 B)
constexpr int kScanBlock = 1024;    // items per block of the three-phase scan
constexpr uint64_t kCarryMax = 1ull << 20;  // longest record carried between windows
constexpr uint32_t kErrGrammar = 1u, kErrDup = 2u, kErrSet = 4u;

struct Meta {                 // window bookkeeping, device -> host once per window
    unsigned long long n_nl;  // line breaks in the window
    unsigned long long n_rec; // complete records
    unsigned long long end;   // first byte after the last complete record (absolute)
    unsigned long long max_len;
    unsigned long long err;
    unsigned long long q_low;  // 255 - the smallest quality byte so far (0: none yet)
};

// Per-byte "is a line feed" bits of a dword, in [lo, hi) of absolute positions.
__device__ __forceinline__ uint32_t lf_bits(uint32_t x, uint64_t p, uint64_t lo, uint64_t hi) {
    const uint32_t v = x ^ 0x0A0A0A0Au;
    const uint32_t z = ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v | 0x7F7F7F7Fu);  // 0x80 in every zero byte
    uint32_t m = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) m |= ((z >> (8 * b + 7)) & 1u) << b;
#pragma unroll
    for (int b = 0; b < 4; b++)
        if (p + b < lo || p + b >= hi) m &= ~(1u << b);
    return m;
}

// 16 line-feed bits of the lane's chunk (bit j <-> byte 16 t + j of the tile).
__device__ __forceinline__ uint32_t chunk_lf(const uint8_t *D, uint64_t c0, uint64_t lo, uint64_t hi) {
    if (c0 + 16 <= lo || c0 >= hi) return 0u;
    const uint4 v = *(const uint4 *)(D + c0);
    return lf_bits(v.x, c0, lo, hi) | (lf_bits(v.y, c0 + 4, lo, hi) << 4) | (lf_bits(v.z, c0 + 8, lo, hi) << 8) |
           (lf_bits(v.w, c0 + 12, lo, hi) << 12);
}

// Block-wide exclusive scan of one uint32 per thread (256 threads); *total = sum.
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t *s_wave, uint32_t &total) {
    const int lane = lane_id(), wv = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_scan(v);
    if (lane == 63) s_wave[wv] = incl;
    __syncthreads();
    uint32_t before = 0;
    total = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        before += i < wv ? s_wave[i] : 0u;
        total += s_wave[i];
    }
    __syncthreads();
    return before + incl - v;
}

__global__ __launch_bounds__(256) void k_nl_count(const uint8_t *D, uint64_t t0, uint64_t lo, uint64_t hi,
                                                  uint32_t *tile_cnt) {
    __shared__ uint32_t s_wave[4];
    const uint64_t c0 = t0 + (uint64_t)blockIdx.x * kTile + 16 * threadIdx.x;
    const uint32_t c = __popc(chunk_lf(D, c0, lo, hi));
    uint32_t total;
    block_excl_scan256(c, s_wave, total);
    if (threadIdx.x == 0) tile_cnt[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void k_nl_write(const uint8_t *D, uint64_t t0, uint64_t lo, uint64_t hi,
                                                  const unsigned long long *tile_off, uint32_t *nl) {
    __shared__ uint32_t s_wave[4];
    const uint64_t c0 = t0 + (uint64_t)blockIdx.x * kTile + 16 * threadIdx.x;
    uint32_t m = chunk_lf(D, c0, lo, hi);
    uint32_t total;
    uint64_t o = tile_off[blockIdx.x] + block_excl_scan256(__popc(m), s_wave, total);
    while (m) {
        const int j = __builtin_ctz(m);
        m &= m - 1;
        nl[o++] = (uint32_t)(c0 + j - t0);  // relative to the window's first tile: < 2^32 for any file size
    }
}

// Three-phase exclusive scan of n uint32 (in) into n + 1 uint64 (out[n] = sum).
__global__ __launch_bounds__(256) void k_scan_sums(const uint32_t *in, uint64_t n, unsigned long long *bsum) {
    __shared__ unsigned long long s[4];
    const uint64_t b0 = (uint64_t)blockIdx.x * kScanBlock;
    unsigned long long v = 0;
    for (uint32_t i = threadIdx.x; i < kScanBlock; i += 256)
        if (b0 + i < n) v += in[b0 + i];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o);
    if (lane_id() == 0) s[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) bsum[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

__global__ __launch_bounds__(1024) void k_scan_blocks(unsigned long long *bsum, uint64_t nb,
                                                      unsigned long long *total) {
    __shared__ unsigned long long s[1024];
    const uint64_t per = (nb + 1023) / 1024;
    const uint64_t a = threadIdx.x * per, e = min(nb, a + per);
    unsigned long long v = 0;
    for (uint64_t i = a; i < e; i++) v += bsum[i];
    s[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const unsigned long long x = threadIdx.x >= (unsigned)o ? s[threadIdx.x - o] : 0ull;
        __syncthreads();
        s[threadIdx.x] += x;
        __syncthreads();
    }
    unsigned long long run = s[threadIdx.x] - v;
    for (uint64_t i = a; i < e; i++) {
        const unsigned long long x = bsum[i];
        bsum[i] = run;
        run += x;
    }
    if (threadIdx.x == 1023) *total = s[1023];
}

__global__ __launch_bounds__(256) void k_scan_apply(const uint32_t *in, uint64_t n, const unsigned long long *bsum,
                                                    unsigned long long *out) {
    __shared__ uint32_t s_wave[4];
    const uint64_t b0 = (uint64_t)blockIdx.x * kScanBlock;
    unsigned long long run = bsum[blockIdx.x];
    for (uint32_t c = 0; c < kScanBlock; c += 256) {
        const uint64_t i = b0 + c + threadIdx.x;
        const uint32_t v = i < n ? in[i] : 0u;
        uint32_t total;
        const uint32_t ex = block_excl_scan256(v, s_wave, total);
        if (i < n) out[i] = run + ex;
        run += total;
    }
    if (b0 + kScanBlock >= n && threadIdx.x == 0) out[n] = run;
}

// Complete records of the window: the last window may end without a line
// feed (one optional final line break); any other window ends at the line
// feed of its last complete record, the rest is carried.
__global__ void k_window_meta(const uint8_t *D, uint64_t t0, uint64_t lo, uint64_t hi, int last, uint32_t *nl,
                              const unsigned long long *n_nl, Meta *meta) {
    if (threadIdx.x || blockIdx.x) return;
    uint64_t lines = *n_nl;
    meta->n_nl = lines;
    uint64_t end = lo;
    if (last) {
        if (hi > lo && D[hi - 1] != '\n') nl[lines++] = (uint32_t)(hi - t0);  // the final line, no line feed
        if (lines % 4) meta->err |= kErrGrammar;
        end = hi;
    } else if (lines >= 4) {
        end = t0 + (uint64_t)nl[(lines / 4) * 4 - 1] + 1;
    }
    meta->n_rec = lines / 4;
    meta->end = end;
}

__device__ __forceinline__ bool id_byte(uint8_t c) { return c >= 0x21 && c <= 0x7E; }

// One record per thread: header, "+" line, lengths, the id's hash.
__global__ void k_records(const uint8_t *D, uint64_t t0, uint64_t lo, const uint32_t *nl, const Meta *meta, uint32_t *len,
                          unsigned long long *ids, uint64_t ids_cap, Meta *meta_out) {
    const uint64_t R = meta->n_rec;
    uint32_t bad = 0, mx = 0;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < R; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t hs = r ? t0 + nl[4 * r - 1] + 1 : lo, he = t0 + nl[4 * r];
        const uint64_t ss = he + 1, se = t0 + nl[4 * r + 1], ps = se + 1, pe = t0 + nl[4 * r + 2], qs = pe + 1,
                       qe = t0 + nl[4 * r + 3];
        const uint64_t n = se - ss;
        bool ok = he >= hs + 2 && D[hs] == '@' && id_byte(D[hs + 1]) && id_byte(D[he - 1]);
        ok = ok && n >= 1 && pe == ps + 1 && D[ps] == '+' && qe - qs == n && n < (1ull << 31);
        // the id (the header without "@": no leading / trailing blank, so the
        // reference's stripped identifier is these bytes): FNV-1a, mixed
        uint64_t h = 0xCBF29CE484222325ull;
        if (ok)
            for (uint64_t p = hs + 1; p < he; p++) {
                const uint8_t c = D[p];
                ok = ok && (id_byte(c) || c == ' ' || c == '\t');
                h = (h ^ c) * 0x100000001B3ull;
            }
        len[r] = ok ? (uint32_t)n : 0u;
        if (!ok) {
            bad |= kErrGrammar;
            continue;
        }
        mx = max(mx, (uint32_t)n);
        h = fmix64(h ^ (he - hs));
        if (h == 0) h = 1;
        uint64_t pos = h & (ids_cap - 1);
        for (uint32_t it = 0;; it++) {
            if (it >= 4096) {
                bad |= kErrSet;
                break;
            }
            const unsigned long long old = atomicCAS(&ids[pos], 0ull, (unsigned long long)h);
            if (old == 0ull) break;
            if (old == h) {  // the same id hash: a duplicate id (or a 2^-64 collision) -> the exact parser
                bad |= kErrDup;
                break;
            }
            pos = (pos + 1) & (ids_cap - 1);
        }
    }
    if (bad) atomicOr(&meta_out->err, (unsigned long long)bad);
    if (mx) atomicMax(&meta_out->max_len, (unsigned long long)mx);
}

// Every byte of the window's complete records against its line's class;
// sequence and quality bytes to their columns.  Line index of a byte = line
// feeds before it (tile offset + block scan + bits below it in the chunk).
__global__ __launch_bounds__(256) void k_compact(const uint8_t *D, uint64_t t0, uint64_t lo, const Meta *meta,
                                                 const unsigned long long *tile_off, const uint32_t *nl,
                                                 const unsigned long long *rec_off, uint8_t *seq, uint8_t *qual,
                                                 Meta *meta_out) {
    __shared__ uint32_t s_wave[4];
    const uint64_t hi = meta->end;
    const uint64_t c0 = t0 + (uint64_t)blockIdx.x * kTile + 16 * threadIdx.x;
    const uint32_t m = chunk_lf(D, c0, lo, hi);
    uint32_t total;
    const uint64_t li0 = tile_off[blockIdx.x] + block_excl_scan256(__popc(m), s_wave, total);
    uint32_t bad = 0, q_low = 0;
    if (!(c0 + 16 <= lo || c0 >= hi)) {  // (no early return: the wave reduces q_low below)
    const uint4 v = *(const uint4 *)(D + c0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint64_t li = li0;
    uint64_t ls = li ? t0 + nl[li - 1] + 1 : lo;  // start of the line holding byte c0 (or lo)
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const uint64_t p = c0 + j;
        const uint8_t c = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
        if (p < lo || p >= hi) continue;
        if ((m >> j) & 1u) {  // a line feed ends line li
            li++;
            ls = p + 1;
            continue;
        }
        const uint32_t type = (uint32_t)(li & 3);
        const uint64_t r = li >> 2, col = p - ls;
        if (type == 1) {
            if (!(c == 'A' || c == 'C' || c == 'G' || c == 'T')) bad = 1;
            else if (rec_off[r] + col < rec_off[r + 1]) seq[rec_off[r] + col] = c;
        } else if (type == 3) {
            if (!id_byte(c)) bad = 1;
            else if (rec_off[r] + col < rec_off[r + 1]) qual[rec_off[r] + col] = c;
            q_low = max(q_low, 255u - c);
        }
    }
    }
    if (bad) atomicOr(&meta_out->err, (unsigned long long)kErrGrammar);
    for (int o = 32; o > 0; o >>= 1) q_low = max(q_low, (uint32_t)__shfl_down(q_low, o));
    if (lane_id() == 0 && q_low) atomicMax(&meta_out->q_low, (unsigned long long)q_low);
}

struct Source {  // plain file (positional reads on host threads) or gzip (pa_gz.cpp: BGZF on all threads)
    int fd = -1;
    pa::Gz *gz = nullptr;
    uint64_t size = 0, pos = 0;
    bool eof = false;
    int threads = 8;

    // Read up to n bytes into dst; returns the count, sets eof at the end.
    bool read(uint8_t *dst, uint64_t n, uint64_t &got) {
        got = 0;
        if (gz) return pa::gz_read(gz, dst, n, &got, &eof) == PA_OK;
        const uint64_t want = std::min<uint64_t>(n, size - pos);
        const int nt = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)threads, want >> 22));
        std::vector<std::thread> th;
        std::vector<int> ok(nt, 1);
        for (int t = 0; t < nt; t++)
            th.emplace_back([&, t] {
                uint64_t a = want * t / nt, e = want * (t + 1) / nt;
                while (a < e) {
                    const ssize_t r = pread(fd, dst + a, (size_t)std::min<uint64_t>(e - a, 1u << 30), (off_t)(pos + a));
                    if (r <= 0) {
                        ok[t] = 0;
                        return;
                    }
                    a += (uint64_t)r;
                }
            });
        for (auto &x : th) x.join();
        for (int x : ok)
            if (!x) return false;
        pos += want;
        got = want;
        eof = pos >= size;
        return true;
    }
};

}  // namespace

namespace pa {

// The occupied entries of an id set, compacted (order unspecified).
__global__ void k_ids_compact(const unsigned long long *ids, uint64_t cap, unsigned long long *out, uint64_t out_cap,
                              unsigned long long *n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long h = ids[i];
        if (!h) continue;
        const unsigned long long at = atomicAdd(n, 1ull);
        if (at < out_cap) out[at] = h;
    }
}

// Insert the id hashes of several ranges into one set; *dup = 1 when a hash
// arrives twice (within a range the parse already refused duplicates, so a
// repeat is a duplicate id across ranges -- or a 2^-64 collision: the exact
// parser decides).
__global__ void k_ids_union(const unsigned long long *h_in, uint64_t n, unsigned long long *set, uint64_t cap,
                            unsigned int *dup) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long h = h_in[i];
        uint64_t pos = h & (cap - 1);
        for (uint64_t it = 0; it < cap; it++) {
            const unsigned long long old = atomicCAS(&set[pos], 0ull, h);
            if (old == 0ull) break;
            if (old == h) {
                atomicOr(dup, 1u);
                break;
            }
            pos = (pos + 1) & (cap - 1);
        }
    }
}

// Device buffers of the per-window parse (sized for windows of up to `span`
// bytes of text) and the id set of the whole file.
struct ParseBufs {
    uint8_t *seq = nullptr, *qual = nullptr;
    uint32_t *tile_cnt = nullptr, *nl = nullptr, *len = nullptr;
    unsigned long long *tile_off = nullptr, *bsum = nullptr, *rec_off = nullptr, *ids = nullptr, *tot = nullptr;
    Meta *meta = nullptr, *h_meta = nullptr;
    uint64_t ids_cap = 0, max_rec = 0;

    hipError_t alloc(uint64_t span, uint64_t est_rec, hipStream_t st) {
        const uint64_t max_tiles = span / kTile + 2;
        const uint64_t max_nl = span + 8;  // (a text of line feeds only: every byte)
        max_rec = span / 8 + 2;
        ids_cap = 1024;
        while (ids_cap < 2 * est_rec) ids_cap <<= 1;
        hipError_t e = hipSuccess;
        auto m = [&](void **p, uint64_t b) {
            if (e == hipSuccess) e = pa::dev_malloc(p, b);
        };
        m((void **)&seq, span + kReadPad);
        m((void **)&qual, span + kReadPad);
        m((void **)&tile_cnt, max_tiles * 4);
        m((void **)&tile_off, (max_tiles + 1) * 8);
        m((void **)&nl, max_nl * 4);
        m((void **)&len, max_rec * 4);
        m((void **)&rec_off, (max_rec + 1) * 8);
        m((void **)&bsum, (std::max(max_tiles, max_rec) / kScanBlock + 2) * 8);
        m((void **)&ids, ids_cap * 8);
        m((void **)&tot, 8);
        m((void **)&meta, sizeof(Meta));
        if (e == hipSuccess) e = hipHostMalloc((void **)&h_meta, sizeof(Meta), hipHostMallocDefault);
        if (e == hipSuccess) e = hipMemsetAsync(ids, 0, ids_cap * 8, st);
        if (e == hipSuccess) e = hipMemsetAsync(meta, 0, sizeof(Meta), st);
        return e;
    }
    void release() {
        pa::dev_free(seq); pa::dev_free(qual); pa::dev_free(tile_cnt); pa::dev_free(nl); pa::dev_free(len); pa::dev_free(tile_off);
        pa::dev_free(bsum); pa::dev_free(rec_off); pa::dev_free(ids); pa::dev_free(tot); pa::dev_free(meta);
        hipHostFree(h_meta);
        *this = ParseBufs{};
    }
};

// Window outcome: records aligned, the end of the last complete record, or a
// reason to leave the file to the exact host parser.
struct WindowOut {
    uint64_t records = 0, end = 0;
    bool fail = false;
};

// Parse the text [lo, hi) of D (t0 = lo & ~15; `last`: the file ends at hi)
// and align its complete records as global reads base, base + 1, ...
// Host waits: the window's record count (one sync), then the grammar flags of
// its bytes (a second one).
pa_status parse_align_window(ParseBufs &B, const uint8_t *D, uint64_t lo, uint64_t hi, bool last, pa_index *idx,
                             const DevParams &prm, uint64_t base, pa_result *acc, hipStream_t st, WindowOut &out,
                             double *t_meta, double *t_rec) {
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    out = WindowOut{};
    out.end = lo;
    const uint64_t t0 = lo & ~15ull;
    const uint64_t ntiles = (hi - t0 + kTile - 1) / kTile;
    const unsigned sgrid = (unsigned)((ntiles + kScanBlock - 1) / kScanBlock);
    PA_HIP(hipMemsetAsync(B.meta, 0, offsetof(Meta, max_len), st));
    hipLaunchKernelGGL(k_nl_count, dim3((unsigned)ntiles), dim3(256), 0, st, D, t0, lo, hi, B.tile_cnt);
    hipLaunchKernelGGL(k_scan_sums, dim3(sgrid), dim3(256), 0, st, B.tile_cnt, ntiles, B.bsum);
    hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, st, B.bsum, (uint64_t)sgrid, B.tot);
    hipLaunchKernelGGL(k_scan_apply, dim3(sgrid), dim3(256), 0, st, B.tile_cnt, ntiles, B.bsum, B.tile_off);
    hipLaunchKernelGGL(k_nl_write, dim3((unsigned)ntiles), dim3(256), 0, st, D, t0, lo, hi, B.tile_off, B.nl);
    hipLaunchKernelGGL(k_window_meta, dim3(1), dim3(1), 0, st, D, t0, lo, hi, last ? 1 : 0, B.nl, B.tot, B.meta);
    PA_HIP(hipGetLastError());
    PA_HIP(hipMemcpyAsync(B.h_meta, B.meta, sizeof(Meta), hipMemcpyDeviceToHost, st));
    auto tw = now();
    PA_HIP(hipStreamSynchronize(st));
    *t_meta += ms(tw, now());
    const uint64_t R = B.h_meta->n_rec, end = B.h_meta->end;
    if (B.h_meta->err || (R == 0 && !last) || R > B.max_rec) {
        out.fail = true;
        return PA_OK;
    }
    out.end = end;
    if (R == 0) return PA_OK;
    const unsigned rgrid = (unsigned)std::min<uint64_t>((R + 255) / 256, 65536);
    const unsigned lgrid = (unsigned)((R + kScanBlock - 1) / kScanBlock);
    hipLaunchKernelGGL(k_records, dim3(rgrid), dim3(256), 0, st, D, t0, lo, B.nl, B.meta, B.len, B.ids, B.ids_cap, B.meta);
    hipLaunchKernelGGL(k_scan_sums, dim3(lgrid), dim3(256), 0, st, B.len, R, B.bsum);
    hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, st, B.bsum, (uint64_t)lgrid, B.tot);
    hipLaunchKernelGGL(k_scan_apply, dim3(lgrid), dim3(256), 0, st, B.len, R, B.bsum, B.rec_off);
    hipLaunchKernelGGL(k_compact, dim3((unsigned)((end - t0 + kTile - 1) / kTile)), dim3(256), 0, st, D, t0, lo,
                       B.meta, B.tile_off, B.nl, B.rec_off, B.seq, B.qual, B.meta);
    PA_HIP(hipGetLastError());
    PA_HIP(hipMemcpyAsync(B.h_meta, B.meta, sizeof(Meta), hipMemcpyDeviceToHost, st));
    tw = now();
    PA_HIP(hipStreamSynchronize(st));
    *t_rec += ms(tw, now());
    if (B.h_meta->err) {
        out.fail = true;
        return PA_OK;
    }
    pa_reads r{};
    r.device = idx->device;
    r.n = R;
    r.n_bases = 0;  // (not read by the align path)
    r.max_len = (uint32_t)B.h_meta->max_len;
    r.seq = B.seq;
    r.qual = B.qual;
    r.off = (uint64_t *)B.rec_off;
    r.q_min = 255 - (int32_t)B.h_meta->q_low;  // (over the file so far: <= this window's smallest byte)
    r.len_min = 1;                              // (the grammar: a non-empty sequence)
    PA_TRY(align(idx, &r, prm, base, acc, st));
    out.records = R;
    return PA_OK;
}

bool env_on(const char *name) {
    const char *e = std::getenv(name);
    return e && e[0] == '1';
}

}  // namespace pa

// ---- prefetch: the whole file into device memory, in the background ---------------

struct pa_fastq_prefetch {
    int device = 0;
    std::string path;
    uint64_t size = 0;
    uint64_t window = 0;
    uint8_t *text = nullptr;    // device: the file, plus kTile * 2 bytes of slack for the 16-B tile loads
    pa::ParseBufs bufs;         // the per-window parse buffers (made by the prefetch thread too)
    hipStream_t st = nullptr;   // the prefetch thread's copy stream
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    uint64_t ready = 0;         // bytes of the file on the device (copies complete)
    bool done = false;
    pa_status rc = PA_OK;
    std::string err;
    int threads = 8;
    double t_total_ms = 0;
    uint64_t est_records = ~0ull;  // records in the file, from the line feeds of its first chunk (set before ready > 0)
};

namespace {

// The prefetch thread: parallel positional reads into a ring of pinned chunks,
// each copied to its place in `text` in file order.
void prefetch_run(pa_fastq_prefetch *pf) {
    const auto t_start = std::chrono::steady_clock::now();
    auto fail = [&](pa_status rc, const std::string &msg) {
        std::lock_guard<std::mutex> g(pf->mu);
        pf->rc = rc;
        pf->err = msg;
        pf->done = true;
        pf->cv.notify_all();
    };
    hipError_t e = hipSetDevice(pf->device);
    size_t free_b = 0, total_b = 0;
    if (e == hipSuccess) e = pa::dev_mem_info(&free_b, &total_b);
    // a file that would take more than a quarter of the free device memory
    // (text + parse buffers ~ 21 B per window byte) is left to the windowed stream
    uint64_t cap = free_b / 4;  // PA_PREFETCH_MAX_BYTES: a lower limit (tests: the windowed fallback)
    if (const char *m = std::getenv("PA_PREFETCH_MAX_BYTES")) cap = std::min<uint64_t>(cap, std::strtoull(m, nullptr, 10));
    if (e == hipSuccess && pf->size + 24 * pf->window > cap) {
        fail(PA_EUNSUPPORTED, "FASTQ file too large to prefetch whole");
        return;
    }
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&pf->st, hipStreamNonBlocking);
    if (e == hipSuccess) e = pa::dev_malloc(&pf->text, pf->size + 2 * kTile + 16);
    if (e == hipSuccess) e = pf->bufs.alloc(pf->window + 16, pf->size / 16 + 1024, pf->st);
    if (e != hipSuccess) {
        fail(e == hipErrorOutOfMemory ? PA_ENOMEM : PA_EDEVICE,
             std::string("HIP error in the FASTQ prefetch: ") + hipGetErrorString(e));
        return;
    }
    const int fd = open(pf->path.c_str(), O_RDONLY);
    if (fd < 0) {
        fail(PA_EIO, "cannot open " + pf->path);
        return;
    }
    uint64_t kChunk = 8ull << 20;  // PA_PREFETCH_CHUNK: another chunk size (tests: many chunks, ring wrap)
    if (const char *c = std::getenv("PA_PREFETCH_CHUNK")) kChunk = std::max<uint64_t>(4096, std::strtoull(c, nullptr, 10));
    const int nslot = 16;  // 128 MiB of pinned ring
    const uint64_t nchunk = (pf->size + kChunk - 1) / kChunk;
    const int nread = std::max(1, std::min(pf->threads, nslot - 4));
    uint8_t *ring = nullptr;
    e = hipHostMalloc((void **)&ring, kChunk * nslot, hipHostMallocDefault);
    if (e != hipSuccess) {
        close(fd);
        fail(PA_ENOMEM, std::string("pinned ring of the FASTQ prefetch: ") + hipGetErrorString(e));
        return;
    }
    // chunk c goes to slot c % nslot; state[slot] = the chunk it holds once read (-1 free)
    std::mutex rm;
    std::condition_variable rcv;
    std::vector<int64_t> slot_chunk(nslot, -1), slot_free_for(nslot);
    for (int s = 0; s < nslot; s++) slot_free_for[s] = s;  // the next chunk allowed into the slot
    bool read_error = false, abort = false;
    std::vector<std::thread> readers;
    for (int t = 0; t < nread; t++)
        readers.emplace_back([&, t] {
            for (uint64_t c = t; c < nchunk; c += nread) {
                const int s = (int)(c % nslot);
                {
                    std::unique_lock<std::mutex> g(rm);
                    rcv.wait(g, [&] { return abort || slot_free_for[s] == (int64_t)c; });
                    if (abort) return;
                }
                const uint64_t a = c * kChunk, n = std::min(kChunk, pf->size - a);
                uint64_t got = 0;
                while (got < n) {
                    const ssize_t r = pread(fd, ring + (uint64_t)s * kChunk + got, n - got, (off_t)(a + got));
                    if (r <= 0) break;
                    got += (uint64_t)r;
                }
                std::lock_guard<std::mutex> g(rm);
                if (got < n) read_error = true;
                slot_chunk[s] = (int64_t)c;
                rcv.notify_all();
            }
        });
    pa_status rc = PA_OK;
    std::string msg;
    // Copies stay queued on the stream, up to `inflight` of them: each chunk's
    // event is waited for only when its slot is needed again or the next
    // chunk must be announced (a synchronize after every 8 MiB copy left the
    // DMA engine idle for a host round trip per chunk).  PA_PREFETCH_INFLIGHT=1
    // is the one-at-a-time loop.
    int inflight = 4;
    if (const char *v = std::getenv("PA_PREFETCH_INFLIGHT")) inflight = std::max(1, std::min(nslot - 1, atoi(v)));
    std::vector<hipEvent_t> ev(nslot, nullptr);
    for (int s = 0; s < nslot && e == hipSuccess; s++) e = hipEventCreateWithFlags(&ev[s], hipEventDisableTiming);
    std::deque<uint64_t> q;  // chunks whose copies are queued, in file order
    auto retire = [&]() -> hipError_t {  // the oldest queued copy done: its slot free, its bytes announced
        const uint64_t c0 = q.front();
        const int s0 = (int)(c0 % nslot);
        const hipError_t r = hipEventSynchronize(ev[s0]);
        if (r != hipSuccess) return r;
        q.pop_front();
        {
            std::lock_guard<std::mutex> g(rm);
            slot_chunk[s0] = -1;
            slot_free_for[s0] = (int64_t)(c0 + nslot);
            rcv.notify_all();
        }
        std::lock_guard<std::mutex> g(pf->mu);
        pf->ready = std::min(pf->size, (c0 + 1) * kChunk);
        pf->cv.notify_all();
        return hipSuccess;
    };
    if (e != hipSuccess) {
        rc = PA_EDEVICE;
        msg = std::string("HIP error in the FASTQ prefetch: ") + hipGetErrorString(e);
    }
    // copies already finished are announced without blocking (hipEventQuery),
    // also while this loop waits for the readers: a consumer must not stall on
    // bytes that are in HBM because the next chunk is still being read
    auto retire_done = [&]() -> hipError_t {
        while (!q.empty()) {
            const hipError_t r = hipEventQuery(ev[(int)(q.front() % nslot)]);
            if (r == hipErrorNotReady) return hipSuccess;
            if (r != hipSuccess) return r;
            const hipError_t x = retire();
            if (x != hipSuccess) return x;
        }
        return hipSuccess;
    };
    for (uint64_t c = 0; c < nchunk && rc == PA_OK; c++) {
        const int s = (int)(c % nslot);
        bool failed_read = false;
        for (;;) {
            e = retire_done();
            if (e != hipSuccess) break;
            std::unique_lock<std::mutex> g(rm);
            auto ready = [&] { return read_error || slot_chunk[s] == (int64_t)c; };
            if (q.empty())
                rcv.wait(g, ready);
            else
                rcv.wait_for(g, std::chrono::microseconds(200), ready);
            if (ready()) {
                failed_read = read_error;
                break;
            }
        }
        if (e != hipSuccess) {
            rc = PA_EDEVICE;
            msg = std::string("HIP error in the FASTQ prefetch copy: ") + hipGetErrorString(e);
            break;
        }
        if (failed_read) {
            rc = PA_EIO;
            msg = "read error in " + pf->path;
            break;
        }
        const uint64_t a = c * kChunk, n = std::min(kChunk, pf->size - a);
        if (c == 0) {  // records ~ line feeds / 4 of the first chunk, scaled to the file
            const uint8_t *h = ring;
            const uint64_t m = std::min<uint64_t>(n, 4ull << 20);
            uint64_t nl = 0;
            for (uint64_t i = 0; i < m; i++) nl += h[i] == '\n';
            pf->est_records = m ? (uint64_t)((double)pf->size * (double)(nl / 4 + 1) / (double)m) : 0;
        }
        e = hipMemcpyAsync(pf->text + a, ring + (uint64_t)s * kChunk, n, hipMemcpyHostToDevice, pf->st);
        if (e == hipSuccess) e = hipEventRecord(ev[s], pf->st);
        if (e == hipSuccess) q.push_back(c);
        while (e == hipSuccess && !q.empty() && (q.size() >= (size_t)inflight || c + 1 == nchunk)) e = retire();
        if (e != hipSuccess) {
            rc = PA_EDEVICE;
            msg = std::string("HIP error in the FASTQ prefetch copy: ") + hipGetErrorString(e);
            break;
        }
    }
    if (rc != PA_OK) hipStreamSynchronize(pf->st);  // (no copy may still read the ring)
    for (hipEvent_t x : ev)
        if (x) hipEventDestroy(x);
    {
        std::lock_guard<std::mutex> g(rm);
        abort = true;
        rcv.notify_all();
    }
    for (auto &x : readers) x.join();
    close(fd);
    hipHostFree(ring);
    pf->t_total_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    if (rc != PA_OK) {
        fail(rc, msg);
        return;
    }
    std::lock_guard<std::mutex> g(pf->mu);
    pf->done = true;
    pf->cv.notify_all();
}

}  // namespace

namespace pa {

pa_status fastq_prefetch_start(const char *path, int device, int threads, uint64_t window, pa_fastq_prefetch **out) {
    *out = nullptr;
    const size_t pl = strlen(path);
    if (pl >= 3 && strcmp(path + pl - 3, ".gz") == 0) {
        set_error("pa_fastq_prefetch_start: gzip files are read by the windowed stream (pa_align_fastq_file)");
        return PA_EUNSUPPORTED;
    }
    struct stat sb;
    if (stat(path, &sb) != 0 || !S_ISREG(sb.st_mode)) {
        set_error(std::string("cannot open ") + path);
        return PA_EIO;
    }
    auto *pf = new pa_fastq_prefetch();
    pf->device = device;
    pf->path = path;
    pf->size = (uint64_t)sb.st_size;
    // (<= 2 GiB: line-feed offsets are kept relative to a window's first tile as uint32)
    pf->window = std::min<uint64_t>(std::max<uint64_t>(window, 1 << 16), 1ull << 31) & ~(uint64_t)(kTile - 1);
    pf->threads = std::max(1, threads);
    pf->th = std::thread(prefetch_run, pf);
    *out = pf;
    return PA_OK;
}

void fastq_prefetch_free(pa_fastq_prefetch *pf) {
    if (!pf) return;
    if (pf->th.joinable()) pf->th.join();
    hipSetDevice(pf->device);
    if (pf->st) hipStreamSynchronize(pf->st);
    pa::dev_free(pf->text);
    pf->bufs.release();
    if (pf->st) hipStreamDestroy(pf->st);
    delete pf;
}

// The prefetched file, parsed and aligned window by window as soon as each
// window's bytes are on the device: no carries (the text is contiguous), the
// index's align-side view made while the copies run.
pa_status align_fastq_prefetched(pa_index *idx, pa_fastq_prefetch *pf, const DevParams &prm, uint64_t base,
                                 pa_result *acc, hipStream_t st, uint64_t *n_reads) {
    const bool timing = env_on("PA_STREAM_TIMING");
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    const auto t_start = now();
    double t_meta = 0, t_rec = 0, t_wait = 0;
    if (pf->device != idx->device) {
        set_error("pa_align_fastq_prefetched: the prefetch and the index live on different devices");
        return PA_EINVAL;
    }
    double t_prepare = 0;
    auto wait_for = [&](uint64_t need) -> pa_status {
        const auto tw = now();
        std::unique_lock<std::mutex> g(pf->mu);
        pf->cv.wait(g, [&] { return pf->done || pf->ready >= need; });
        t_wait += ms(tw, now());
        if (pf->rc != PA_OK) {
            set_error(pf->err);
            return pf->rc;
        }
        return PA_OK;
    };
    {  // (the parse buffers exist once a byte is on the device, or the thread is done)
        const pa_status rc = wait_for(1);
        if (rc == PA_EUNSUPPORTED)  // not prefetched (too large): the windowed stream
            return align_fastq_file(idx, pf->path.c_str(), prm, base, acc, pf->threads, pf->window, st, n_reads);
        PA_TRY(rc);
    }
    {  // the align-side view, for the reads this file holds (a file of few reads skips the neighbour bits)
        const auto tp = now();
        PA_TRY(index_prepare(idx, st, pf->est_records));
        t_prepare = ms(tp, now());
    }
    PA_TRY(reserve_queues(idx, pf->bufs.max_rec));
    // the parse stream must see the prefetch thread's allocations and memsets
    PA_HIP(hipStreamSynchronize(pf->st));
    uint64_t lo = 0, records = 0;
    bool fail = pf->size == 0;
    while (!fail) {
        const uint64_t hi = std::min(pf->size, lo + pf->window);
        PA_TRY(wait_for(hi));
        const bool last = hi == pf->size;
        WindowOut w;
        PA_TRY(parse_align_window(pf->bufs, pf->text, lo, hi, last, idx, prm, base + records, acc, st, w, &t_meta,
                                  &t_rec));
        if (w.fail) {
            fail = true;
            break;
        }
        records += w.records;
        if (last) break;
        lo = w.end;
    }
    if (records == 0) fail = true;  // no records: the exact parser raises
    PA_HIP(hipStreamSynchronize(st));
    if (timing)
        fprintf(stderr, "[pa_stream] prefetched %llu records: prefetch thread %.1f ms, prepare %.1f ms, waits: "
                        "copies %.1f, window meta %.1f, records %.1f ms; total %.1f ms\n",
                (unsigned long long)records, pf->t_total_ms, t_prepare, t_wait, t_meta, t_rec, ms(t_start, now()));
    if (fail) {
        set_error("FASTQ file outside the device-parsed subset of the grammar (or a duplicate id)");
        return PA_ENOTCANON;
    }
    if (n_reads) *n_reads = records;
    return PA_OK;
}
pa_status align_fastq_file(pa_index *idx, const char *path, const DevParams &prm, uint64_t base, pa_result *acc,
                           int threads, uint64_t window, hipStream_t st, uint64_t *n_reads, uint64_t offset,
                           uint64_t length, std::vector<uint64_t> *ids_out) {
    // PA_STREAM_TIMING=1: where the time goes (stderr)
    const bool timing = env_on("PA_STREAM_TIMING");
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    const auto t_start = now();
    double t_alloc = 0, t_prepare = 0, t_wait_read = 0, t_wait_meta = 0, t_wait_rec = 0;
    Source src;
    src.threads = std::max(1, threads);
    {
        const size_t pl = strlen(path);
        const bool gz = pl >= 3 && strcmp(path + pl - 3, ".gz") == 0;
        if (gz) {
            if (offset != 0 || length != ~0ull) {
                set_error("pa_align_fastq_range: byte ranges of plain files only");
                return PA_EUNSUPPORTED;
            }
            PA_TRY(pa::gz_open(path, src.threads, &src.gz));  // (not gzip data: PA_ENOTCANON, the exact path)
        } else {
            src.fd = open(path, O_RDONLY);
            struct stat sb;
            if (src.fd < 0 || fstat(src.fd, &sb) != 0) {
                if (src.fd >= 0) close(src.fd);
                set_error(std::string("cannot open ") + path);
                return PA_EIO;
            }
            // a byte range [offset, offset + length) read as if it were the file
            // (pa_align_fastq_range: the caller cuts on record boundaries)
            src.size = std::min<uint64_t>((uint64_t)sb.st_size, offset + std::min<uint64_t>(length, ~0ull - offset));
            src.pos = std::min<uint64_t>(offset, src.size);
        }
    }
    const uint64_t W = std::min<uint64_t>(std::max<uint64_t>(window, 1 << 16), 1ull << 31) & ~(uint64_t)(kTile - 1);
    const uint64_t dbytes = kCarryMax + W + 2 * kTile;       // one device text buffer
    const uint64_t est_rec = src.gz ? std::max<uint64_t>(1ull << 24, pa::gz_text_size(src.gz) / 16 + 1024)
                                    : (src.size - src.pos) / 16 + 1024;

    uint8_t *H[2] = {nullptr, nullptr}, *D[2] = {nullptr, nullptr};
    ParseBufs B;
    hipStream_t cs = nullptr;
    hipEvent_t ev_h2d[2] = {nullptr, nullptr}, ev_carry[2] = {nullptr, nullptr};
    std::thread reader;
    pa_status rc = PA_OK;
    auto cleanup = [&]() {
        if (reader.joinable()) reader.join();
        if (cs) hipStreamSynchronize(cs);
        hipStreamSynchronize(st);
        for (int i = 0; i < 2; i++) {
            hipHostFree(H[i]);
            pa::dev_free(D[i]);
            if (ev_h2d[i]) hipEventDestroy(ev_h2d[i]);
            if (ev_carry[i]) hipEventDestroy(ev_carry[i]);
        }
        B.release();
        if (cs) hipStreamDestroy(cs);
        if (src.gz) pa::gz_close(src.gz);
        if (src.fd >= 0) close(src.fd);
    };
#define F_HIP(call)                                                                                      \
    do {                                                                                                 \
        hipError_t e_ = (call);                                                                          \
        if (e_ != hipSuccess) {                                                                          \
            set_error(std::string("HIP error in pa_align_fastq_file: ") + hipGetErrorString(e_) + " (" #call ")"); \
            cleanup();                                                                                   \
            return e_ == hipErrorOutOfMemory ? PA_ENOMEM : PA_EDEVICE;                                   \
        }                                                                                                \
    } while (0)
    for (int i = 0; i < 2; i++) {
        F_HIP(hipHostMalloc((void **)&H[i], W, hipHostMallocDefault));
        F_HIP(pa::dev_malloc(&D[i], dbytes));
        F_HIP(hipEventCreateWithFlags(&ev_h2d[i], hipEventDisableTiming));
        F_HIP(hipEventCreateWithFlags(&ev_carry[i], hipEventDisableTiming));
    }
    F_HIP(B.alloc(kCarryMax + W, est_rec, st));
    F_HIP(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    t_alloc = ms(t_start, now());
    // the index's align-side view and the align queues, while window 0 is read
    uint64_t got_next = 0;
    bool read_ok = true;
    reader = std::thread([&] { read_ok = src.read(H[0], W, got_next); });
    auto tw = now();
    rc = index_prepare(idx, st);
    if (rc == PA_OK) rc = reserve_queues(idx, B.max_rec);
    if (rc != PA_OK) {
        cleanup();
        return rc;
    }
    t_prepare = ms(tw, now());
    tw = now();
    reader.join();
    t_wait_read += ms(tw, now());
    if (!read_ok) {  // (a corrupt .gz: the exact path raises the reference's error)
        set_error(std::string("read error in ") + path);
        const bool gz = src.gz != nullptr;
        cleanup();
        return gz ? PA_ENOTCANON : PA_EIO;
    }
    uint64_t carry = 0, records = 0, prev_end = 0;
    int cur = 0;
    bool last = src.eof, fail_grammar = false;
    uint64_t got = got_next;
    F_HIP(hipMemcpyAsync(D[0] + kCarryMax, H[0], got, hipMemcpyHostToDevice, cs));
    F_HIP(hipEventRecord(ev_h2d[0], cs));
    for (uint64_t win = 0;; win++) {
        // the host reads window win + 1 into the other pinned buffer meanwhile
        const int nxt = cur ^ 1;
        bool next_started = false;
        if (!last) {
            if (win > 0) F_HIP(hipEventSynchronize(ev_h2d[nxt]));  // its previous copy is done
            reader = std::thread([&, nxt] { read_ok = src.read(H[nxt], W, got_next); });
            next_started = true;
        }
        // this window's text: [lo, hi) of D[cur], the carried tail in front of it
        const uint64_t lo = kCarryMax - carry, hi = kCarryMax + got;
        F_HIP(hipStreamWaitEvent(st, ev_h2d[cur], 0));
        if (carry) F_HIP(hipMemcpyAsync(D[cur] + lo, D[nxt] + prev_end, carry, hipMemcpyDeviceToDevice, st));
        F_HIP(hipEventRecord(ev_carry[cur], st));
        if (hi == lo) break;  // (an empty last window: nothing after the previous records)
        WindowOut w;
        rc = parse_align_window(B, D[cur], lo, hi, last, idx, prm, base + records, acc, st, w, &t_wait_meta,
                                &t_wait_rec);
        if (rc != PA_OK) break;
        // (a record longer than the carry limit is left to the host parser too)
        if (w.fail || (!last && hi - w.end > kCarryMax)) {
            fail_grammar = true;
            break;
        }
        records += w.records;
        if (last) break;
        carry = hi - w.end;
        prev_end = w.end;
        // the next window's copy waits for this window's carry copy (which reads D[cur]'s tail later
        // only from the next window's perspective: D[nxt] is rewritten next)
        if (next_started) {
            tw = now();
            reader.join();
            t_wait_read += ms(tw, now());
            if (!read_ok) {  // a corrupt .gz: the exact path (Python gzip) raises the reference's error
                set_error(std::string("read error in ") + path);
                rc = src.gz ? PA_ENOTCANON : PA_EIO;
                break;
            }
            got = got_next;
            last = src.eof;
            F_HIP(hipStreamWaitEvent(cs, ev_carry[cur], 0));
            F_HIP(hipMemcpyAsync(D[nxt] + kCarryMax, H[nxt], got, hipMemcpyHostToDevice, cs));
            F_HIP(hipEventRecord(ev_h2d[nxt], cs));
        }
        cur = nxt;
    }
#undef F_HIP
    if (reader.joinable()) reader.join();
    if (rc == PA_OK && records == 0) fail_grammar = true;  // no records: the exact parser raises
    if (rc == PA_OK && fail_grammar) {
        set_error("FASTQ file outside the device-parsed subset of the grammar (or a duplicate id)");
        rc = PA_ENOTCANON;
    }
    if (rc == PA_OK && n_reads) *n_reads = records;
    if (rc == PA_OK && ids_out) {  // the range's id hashes (pa_idsets_disjoint: duplicates across ranges)
        unsigned long long *d_out = nullptr, *d_n = nullptr;
        unsigned long long h_n = 0;
        hipError_t e = pa::dev_malloc(&d_out, std::max<uint64_t>(records, 1) * 8);
        if (e == hipSuccess) e = pa::dev_malloc(&d_n, 8);
        if (e == hipSuccess) e = hipMemsetAsync(d_n, 0, 8, st);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_ids_compact, dim3((unsigned)std::min<uint64_t>((B.ids_cap + 255) / 256, 65536)),
                               dim3(256), 0, st, B.ids, B.ids_cap, d_out, std::max<uint64_t>(records, 1), d_n);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpyAsync(&h_n, d_n, 8, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e == hipSuccess && h_n != records) e = hipErrorUnknown;  // (one hash per record: the set holds them all)
        if (e == hipSuccess) {
            ids_out->resize(h_n);
            e = hipMemcpyAsync(ids_out->data(), d_out, h_n * 8, hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
        }
        pa::dev_free(d_out);
        pa::dev_free(d_n);
        if (e != hipSuccess) {
            set_error(std::string("pa_align_fastq_range: id set export: ") + hipGetErrorString(e));
            rc = PA_EDEVICE;
        }
    }
    const auto t_c = now();
    cleanup();
    if (timing)
        fprintf(stderr, "[pa_stream] %llu records: alloc %.1f ms, index prepare %.1f ms, waits: reader %.1f, window "
                        "meta %.1f, records %.1f ms; cleanup %.1f ms; total %.1f ms\n",
                (unsigned long long)records, t_alloc, t_prepare, t_wait_read, t_wait_meta, t_wait_rec, ms(t_c, now()),
                ms(t_start, now()));
    return rc;
}

}  // namespace pa

namespace pa {

// Whether id hash sets (one per byte range of a file) are pairwise disjoint:
// all inserted into one device set on `device`.
pa_status idsets_disjoint(const std::vector<const std::vector<uint64_t> *> &sets, int device, bool *disjoint) {
    *disjoint = true;
    uint64_t total = 0;
    for (auto *v : sets) total += v->size();
    if (total == 0) return PA_OK;
    PA_HIP(hipSetDevice(device));
    uint64_t cap = 1024;
    while (cap < 2 * total) cap <<= 1;
    unsigned long long *set = nullptr, *in = nullptr;
    unsigned int *dup = nullptr, h_dup = 0;
    hipStream_t st = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (e == hipSuccess) e = pa::dev_malloc(&set, cap * 8);
    if (e == hipSuccess) e = pa::dev_malloc(&in, total * 8);
    if (e == hipSuccess) e = pa::dev_malloc(&dup, 4);
    if (e == hipSuccess) e = hipMemsetAsync(set, 0, cap * 8, st);
    if (e == hipSuccess) e = hipMemsetAsync(dup, 0, 4, st);
    uint64_t at = 0;
    for (auto *v : sets) {
        if (e == hipSuccess && !v->empty())
            e = hipMemcpyAsync(in + at, v->data(), v->size() * 8, hipMemcpyHostToDevice, st);
        at += v->size();
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_ids_union, dim3((unsigned)std::min<uint64_t>((total + 255) / 256, 65536)), dim3(256), 0, st,
                           in, total, set, cap, dup);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(&h_dup, dup, 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (st) hipStreamSynchronize(st);
    pa::dev_free(set);
    pa::dev_free(in);
    pa::dev_free(dup);
    if (st) hipStreamDestroy(st);
    PA_HIP(e);
    *disjoint = h_dup == 0;
    return PA_OK;
}

}  // namespace pa

namespace {
__global__ void k_warm_fastq() {}
}  // namespace

namespace pa {
// Loads this file's code object (a first launch from a module loads it): the
// CLI's runtime-start thread calls it so that the load overlaps host work.
void warm_fastq(hipStream_t st) { hipLaunchKernelGGL(k_warm_fastq, dim3(1), dim3(64), 0, st); }
}  // namespace pa
