// extern "C" entry points of libpa.so (declared in include/pa.h).
//
// Argument checks mirror the reference's (src/kmer.py:125-126, 501-510);
// EXTQUALITY thresholds are clamped to ranges where the strict comparisons of
// src/kmer.py:420, 425, 587 keep their meaning, so the kernels can use 32-bit
// arithmetic:
//   mean quality < T  with byte qualities in [0, 255]:  T <= 0 never, T >= 256 always
//   set size > mg     with set sizes in [1, G]:          mg < 0 always, mg >= G never
//   top >= second + m with counts <= windows < 2^31:     m clamped to 2^30
//   max - mapped > p  likewise p clamped to 2^30 (p < 0 keeps "skip")
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <string>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "pa_internal.h"

namespace pa {
static thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }
}  // namespace pa

using pa::set_error;

#define PA_CHECK(cond, code, msg) \
    do {                          \
        if (!(cond)) {            \
            set_error(msg);       \
            return code;          \
        }                         \
    } while (0)

namespace {

hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

int64_t clampi(int64_t v, int64_t lo, int64_t hi) { return v < lo ? lo : (v > hi ? hi : v); }

pa_status to_dev_params(const pa_params *p, uint32_t n_genomes, pa::DevParams *out) {
    PA_CHECK(p != nullptr, PA_EINVAL, "params must not be NULL");
    PA_CHECK(p->m >= 0, PA_EINVAL, "m must be bigger than or equal to 0");
    PA_CHECK((p->flags & ~7u) == 0, PA_EINVAL, "unknown flag bits in pa_params.flags");
    out->m = (int32_t)clampi(p->m, 0, 1 << 30);
    out->p = (int32_t)clampi(p->p, -1, 1 << 30);
    out->mrq = (int32_t)clampi(p->min_read_quality, 0, 256);
    out->mkq = (int32_t)clampi(p->min_kmer_quality, 0, 256);
    out->mg = (int32_t)clampi(p->max_genomes, -1, (int64_t)n_genomes);
    out->flags = p->flags;
    return PA_OK;
}

}  // namespace

extern "C" {

const char *pa_last_error(void) { return pa::g_err.c_str(); }

// PA_SOURCE_HASH: SHA-256 of csrc/*, include/pa.h and the compile flags, put on
// this file's command line by build_native.py, so a test or a bench line can
// tie the loaded binary to the checkout it came from.
#ifndef PA_SOURCE_HASH
#define PA_SOURCE_HASH "unknown"
#endif
const char *pa_version(void) { return "libpa 0.2 (gfx950) src=" PA_SOURCE_HASH; }

namespace {
struct RuntimeStarter {  // joined at exit, before the HIP runtime's own teardown (it was loaded first)
    std::thread th;
    ~RuntimeStarter() {
        if (th.joinable()) th.join();
    }
};
RuntimeStarter g_runtime_starter;
}  // namespace

pa_status pa_runtime_start(int32_t device) {
    if (g_runtime_starter.th.joinable()) return PA_OK;
    g_runtime_starter.th = std::thread([device] {
        const auto t0 = std::chrono::steady_clock::now();
        const char *w = std::getenv("PA_RUNTIME_WARM");  // 0: the context only (A/B)
        if (hipSetDevice(device) == hipSuccess && hipFree(nullptr) == hipSuccess && !(w && w[0] == '0')) {
            pa::warm_index(nullptr);  // the code objects too, not at the first real launch
            pa::warm_align(nullptr);
            pa::warm_fastq(nullptr);
            pa::warm_dump(nullptr);
            hipDeviceSynchronize();
        }
        if (const char *e = std::getenv("PA_CLI_TIMING"); e && e[0] == '1')
            fprintf(stderr, "[pa_runtime] HIP runtime started in %.1f ms\n",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    });
    return PA_OK;
}

pa_status pa_device_count(int32_t *n) {
    PA_CHECK(n != nullptr, PA_EINVAL, "n must not be NULL");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) {
        *n = 0;
        set_error(std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
        return PA_EDEVICE;
    }
    *n = c;
    return PA_OK;
}

pa_status pa_index_build(int32_t device, const char *genomes, const uint64_t *genome_off, uint32_t n_genomes,
                         int64_t k, void *stream, pa_index **out) {
    return pa_index_build_ex(device, genomes, genome_off, n_genomes, k, 0u, stream, out);
}

pa_status pa_index_build_ex(int32_t device, const char *genomes, const uint64_t *genome_off, uint32_t n_genomes,
                            int64_t k, uint32_t flags, void *stream, pa_index **out) {
    PA_CHECK(out != nullptr, PA_EINVAL, "out must not be NULL");
    *out = nullptr;
    PA_CHECK((flags & ~(PA_BUILD_DEFER_TILES | PA_BUILD_COMPACT)) == 0, PA_EINVAL, "unknown build flag bits");
    PA_CHECK(genome_off != nullptr, PA_EINVAL, "genome_off must not be NULL");
    PA_CHECK(k <= PA_MAX_K, PA_EUNSUPPORTED, "k-mer length above PA_MAX_K (255) is not supported");
    PA_CHECK(n_genomes <= PA_MAX_GENOMES, PA_EUNSUPPORTED,
             "more than PA_MAX_GENOMES (2^20 - 1) genomes: the Summary order keys hold a list position in 20 bits");
    for (uint32_t g = 0; g < n_genomes; g++)
        PA_CHECK(genome_off[g + 1] >= genome_off[g], PA_EINVAL, "genome_off must be non-decreasing");
    const uint64_t total = genome_off[n_genomes] - genome_off[0];
    PA_CHECK(total == 0 || genomes != nullptr, PA_EINVAL, "genomes must not be NULL");
    // (FASTA grammar: genome text is uppercase ACGTN, src/constants.py:1-6, src/records.py:225-233 --
    // checked on the device by the build's encode pass, PA_EINVAL with the first bad byte)
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        set_error("no HIP device available (libpa.so has no CPU fallback)");
        return PA_EDEVICE;
    }
    PA_CHECK(device >= 0 && device < ndev, PA_EINVAL, "device ordinal out of range");
    PA_HIP(hipSetDevice(device));
    pa_index *idx = new (std::nothrow) pa_index();
    PA_CHECK(idx != nullptr, PA_ENOMEM, "out of host memory");
    idx->device = device;
    idx->compact_table = (flags & PA_BUILD_COMPACT) != 0;
    pa_status rc = pa::index_build(idx, genomes, genome_off, n_genomes, k, as_stream(stream),
                                   (flags & PA_BUILD_DEFER_TILES) != 0);
    if (rc != PA_OK) {
        pa::index_release(idx);
        delete idx;
        return rc;
    }
    *out = idx;
    return PA_OK;
}

pa_status pa_index_reduce(pa_index *idx, const uint32_t *keep, uint32_t n_keep, uint32_t flags, void *stream) {
    PA_CHECK(idx != nullptr && (n_keep == 0 || keep != nullptr), PA_EINVAL, "NULL argument");
    PA_CHECK(!idx->released, PA_EINVAL, "the index was released by a failed pa_index_reduce: it may only be freed");
    for (uint32_t i = 0; i < n_keep; i++) {
        PA_CHECK(keep[i] < idx->n_genomes, PA_EINVAL, "genome number out of range");
        PA_CHECK(i == 0 || keep[i] > keep[i - 1], PA_EINVAL, "genome numbers must be ascending");
    }
    PA_CHECK((flags & ~(PA_BUILD_DEFER_TILES | PA_BUILD_COMPACT)) == 0, PA_EINVAL, "unknown build flag bits");
    PA_HIP(hipSetDevice(idx->device));
    idx->compact_table = (flags & PA_BUILD_COMPACT) != 0;
    PA_TRY(pa::index_reduce(idx, keep, n_keep, as_stream(stream), (flags & PA_BUILD_DEFER_TILES) != 0));
    return PA_OK;
}

pa_status pa_index_prepare(pa_index *idx, void *stream) {
    PA_CHECK(idx != nullptr, PA_EINVAL, "NULL argument");
    PA_CHECK(!idx->released, PA_EINVAL, "the index was released by a failed pa_index_reduce: it may only be freed");
    PA_HIP(hipSetDevice(idx->device));
    PA_TRY(pa::index_prepare(idx, as_stream(stream), ~0ull, true));
    PA_HIP(hipStreamSynchronize(as_stream(stream)));
    return PA_OK;
}

pa_status pa_index_prepare_ex(pa_index *idx, uint64_t expected_reads, void *stream) {
    PA_CHECK(idx != nullptr, PA_EINVAL, "NULL argument");
    PA_CHECK(!idx->released, PA_EINVAL, "the index was released by a failed pa_index_reduce: it may only be freed");
    PA_HIP(hipSetDevice(idx->device));
    PA_TRY(pa::index_prepare(idx, as_stream(stream), expected_reads, true));
    PA_HIP(hipStreamSynchronize(as_stream(stream)));
    return PA_OK;
}

void pa_index_free(pa_index *idx) {
    if (!idx) return;
    hipSetDevice(idx->device);
    pa::index_release(idx);
    delete idx;
}

pa_status pa_index_get_info(const pa_index *idx, pa_index_info *out) {
    PA_CHECK(idx && out, PA_EINVAL, "NULL argument");
    std::memset(out, 0, sizeof(*out));
    out->k = (uint32_t)std::max<int64_t>(idx->k, 0);
    out->n_genomes = idx->n_genomes;
    out->key_words = (uint32_t)idx->nw;
    out->slot_bytes = (uint32_t)pa::slot_bytes(idx->nw);
    out->n_kmers = idx->n_kmers;
    out->n_multi_classes = idx->n_multi;
    out->class_genome_entries = idx->class_entries;
    out->table_slots = idx->cap;
    out->table_bytes = idx->cap * (uint64_t)pa::slot_bytes(idx->nw);
    out->total_windows = idx->total_windows;
    out->device_bytes = idx->device_bytes;
    return PA_OK;
}

pa_status pa_index_lookup(const pa_index *idx, const char *kmers, uint64_t n, uint32_t kmer_len, int64_t *cls_out,
                          uint32_t *size_out, void *stream) {
    PA_CHECK(idx && cls_out && (n == 0 || kmers), PA_EINVAL, "NULL argument");
    PA_CHECK(!idx->released, PA_EINVAL, "the index was released by a failed pa_index_reduce: it may only be freed");
    PA_HIP(hipSetDevice(idx->device));
    return pa::index_lookup(idx, kmers, n, kmer_len, cls_out, size_out, as_stream(stream));
}

pa_status pa_index_positions(const pa_index *idx, const char *kmers, uint64_t n, uint32_t kmer_len, uint32_t flags,
                             pa_kmer_hit *hits, uint64_t cap, uint64_t *n_hits, void *stream) {
    PA_CHECK(idx && n_hits && (n == 0 || kmers), PA_EINVAL, "NULL argument");
    PA_CHECK(!idx->released, PA_EINVAL, "the index was released by a failed pa_index_reduce: it may only be freed");
    PA_CHECK((flags & ~PA_POS_REVERSE) == 0, PA_EINVAL, "unknown flag bits");
    PA_CHECK(n < PA_POS_RC_BIT, PA_EINVAL, "too many queries");
    PA_HIP(hipSetDevice(idx->device));
    return pa::index_positions(idx, kmers, n, kmer_len, flags, hits, cap, n_hits, as_stream(stream));
}

pa_status pa_index_class_genomes(const pa_index *idx, int64_t cls, uint32_t *genomes, uint32_t cap, uint32_t *n,
                                 void *stream) {
    PA_CHECK(idx && n, PA_EINVAL, "NULL argument");
    PA_CHECK(!idx->released, PA_EINVAL, "the index was released by a failed pa_index_reduce: it may only be freed");
    PA_CHECK(cls >= 0 && (uint64_t)cls < (uint64_t)idx->n_genomes + idx->class_entries, PA_EINVAL,
             "class id out of range");
    if ((uint64_t)cls < idx->n_genomes) {
        *n = 1;
        if (genomes && cap >= 1) genomes[0] = (uint32_t)cls;
        return PA_OK;
    }
    // multi-genome class: id = G + word offset of its [size, genomes...] record
    PA_HIP(hipSetDevice(idx->device));
    const uint64_t rec = (uint64_t)cls - idx->n_genomes;
    uint32_t size = 0;
    hipStream_t st = as_stream(stream);
    PA_HIP(hipMemcpyAsync(&size, idx->class_genomes + rec, 4, hipMemcpyDeviceToHost, st));
    PA_HIP(hipStreamSynchronize(st));
    PA_CHECK(rec + 1 + size <= idx->class_entries, PA_EINVAL, "not a class id");
    *n = size;
    if (genomes && cap > 0) {
        PA_HIP(hipMemcpyAsync(genomes, idx->class_genomes + rec + 1, (uint64_t)std::min(cap, size) * 4,
                              hipMemcpyDeviceToHost, st));
        PA_HIP(hipStreamSynchronize(st));
    }
    return PA_OK;
}

pa_status pa_index_extsim_stats(const pa_index *idx, const uint32_t *group_of, uint32_t n_groups, uint64_t *total,
                                uint64_t *uniq, uint64_t *inter, void *stream) {
    PA_CHECK(idx && total && uniq && inter && (idx->n_genomes == 0 || group_of), PA_EINVAL, "NULL argument");
    PA_CHECK(!idx->released, PA_EINVAL, "the index was released by a failed pa_index_reduce: it may only be freed");
    for (uint32_t g = 0; g < idx->n_genomes; g++)
        PA_CHECK(group_of[g] < n_groups, PA_EINVAL, "group_of entry out of range");
    PA_HIP(hipSetDevice(idx->device));
    return pa::index_extsim_stats(idx, group_of, n_groups, total, uniq, inter, as_stream(stream));
}

pa_status pa_reads_upload(int32_t device, const uint8_t *seq, const uint8_t *qual, const uint64_t *read_off,
                          uint64_t n_reads, void *stream, pa_reads **out) {
    PA_CHECK(out && read_off, PA_EINVAL, "NULL argument");
    *out = nullptr;
    const uint64_t nb = read_off[n_reads] - read_off[0];
    PA_CHECK(nb == 0 || (seq && qual), PA_EINVAL, "seq/qual must not be NULL");
    uint32_t max_len = 0;
    for (uint64_t i = 0; i < n_reads; i++) {
        PA_CHECK(read_off[i + 1] >= read_off[i], PA_EINVAL, "read_off must be non-decreasing");
        uint64_t l = read_off[i + 1] - read_off[i];
        PA_CHECK(l < (1ull << 31), PA_EUNSUPPORTED, "reads longer than 2^31 bases are not supported");
        max_len = std::max<uint32_t>(max_len, (uint32_t)l);
    }
    PA_HIP(hipSetDevice(device));
    pa_reads *r = new (std::nothrow) pa_reads();
    PA_CHECK(r != nullptr, PA_ENOMEM, "out of host memory");
    r->device = device;
    r->n = n_reads;
    r->n_bases = nb;
    r->max_len = max_len;
    hipStream_t st = as_stream(stream);
    auto fail = [&](hipError_t e) {
        set_error(std::string("pa_reads_upload: ") + hipGetErrorString(e));
        pa::dev_free(r->seq); pa::dev_free(r->qual); pa::dev_free(r->off);
        delete r;
        return e == hipErrorOutOfMemory ? PA_ENOMEM : PA_EDEVICE;
    };
    hipError_t e;
    if ((e = pa::dev_malloc(&r->seq, nb + pa::kReadPad)) != hipSuccess) return fail(e);
    if ((e = pa::dev_malloc(&r->qual, nb + pa::kReadPad)) != hipSuccess) return fail(e);
    if ((e = pa::dev_malloc(&r->off, (n_reads + 1) * 8)) != hipSuccess) return fail(e);
    if (nb) {
        if ((e = hipMemcpyAsync(r->seq, seq + read_off[0], nb, hipMemcpyHostToDevice, st)) != hipSuccess) return fail(e);
        if ((e = hipMemcpyAsync(r->qual, qual + read_off[0], nb, hipMemcpyHostToDevice, st)) != hipSuccess) return fail(e);
    }
    if (read_off[0] == 0) {
        if ((e = hipMemcpyAsync(r->off, read_off, (n_reads + 1) * 8, hipMemcpyHostToDevice, st)) != hipSuccess)
            return fail(e);
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return fail(e);
    } else {
        uint64_t *tmp = new (std::nothrow) uint64_t[n_reads + 1];
        if (!tmp) return fail(hipErrorOutOfMemory);
        for (uint64_t i = 0; i <= n_reads; i++) tmp[i] = read_off[i] - read_off[0];
        e = hipMemcpyAsync(r->off, tmp, (n_reads + 1) * 8, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        delete[] tmp;
        if (e != hipSuccess) return fail(e);
    }
    if (pa::reads_measure(r, st) != PA_OK) return fail(hipErrorUnknown);
    *out = r;
    return PA_OK;
}

pa_status pa_reads_synthesize_mix(const pa_index *idx, uint64_t n_reads, uint32_t read_len, uint64_t first_read,
                                  uint64_t seed, double sub_rate, double rc_rate, double foreign_rate, void *stream,
                                  pa_reads **out) {
    PA_CHECK(idx && out, PA_EINVAL, "NULL argument");
    PA_CHECK(!idx->released, PA_EINVAL, "the index was released by a failed pa_index_reduce: it may only be freed");
    *out = nullptr;
    PA_CHECK(read_len > 0, PA_EINVAL, "read_len must be positive");
    PA_CHECK(rc_rate >= 0 && foreign_rate >= 0 && rc_rate + foreign_rate <= 1, PA_EINVAL,
             "rc_rate and foreign_rate must be >= 0 with a sum <= 1");
    PA_HIP(hipSetDevice(idx->device));
    pa_reads *r = new (std::nothrow) pa_reads();
    PA_CHECK(r != nullptr, PA_ENOMEM, "out of host memory");
    pa_status rc = pa::reads_synthesize(idx, r, n_reads, read_len, first_read, seed, sub_rate, rc_rate, foreign_rate,
                                        as_stream(stream));
    if (rc == PA_OK) rc = pa::reads_measure(r, as_stream(stream));
    if (rc != PA_OK) {
        pa::dev_free(r->seq); pa::dev_free(r->qual); pa::dev_free(r->off);
        delete r;
        return rc;
    }
    *out = r;
    return PA_OK;
}

pa_status pa_reads_synthesize(const pa_index *idx, uint64_t n_reads, uint32_t read_len, uint64_t first_read,
                              uint64_t seed, double sub_rate, void *stream, pa_reads **out) {
    return pa_reads_synthesize_mix(idx, n_reads, read_len, first_read, seed, sub_rate, 0.0, 0.0, stream, out);
}

pa_status pa_reads_info(const pa_reads *reads, uint64_t *n_reads, uint64_t *n_bases, uint32_t *max_len) {
    PA_CHECK(reads != nullptr, PA_EINVAL, "NULL argument");
    if (n_reads) *n_reads = reads->n;
    if (n_bases) *n_bases = reads->n_bases;
    if (max_len) *max_len = reads->max_len;
    return PA_OK;
}

pa_status pa_params_effective(const pa_reads *reads, const pa_params *in, pa_params *out, int32_t *q_min,
                              void *stream) {
    PA_CHECK(reads && in && out, PA_EINVAL, "NULL argument");
    pa::DevParams dp, eff;
    PA_TRY(to_dev_params(in, 1u << 20, &dp));
    PA_HIP(hipSetDevice(reads->device));
    PA_TRY(pa::effective_params(reads, dp, eff, as_stream(stream)));
    const pa_params copy = *in;
    *out = copy;
    out->flags = eff.flags;
    if (q_min) *q_min = reads->q_min < 0 ? 255 : reads->q_min;
    return PA_OK;
}

pa_status pa_reads_download(const pa_reads *reads, uint64_t first, uint64_t count, uint8_t *seq, uint8_t *qual,
                            uint64_t *read_off, void *stream) {
    PA_CHECK(reads && read_off, PA_EINVAL, "NULL argument");
    PA_CHECK(first + count <= reads->n, PA_EINVAL, "read range out of bounds");
    PA_HIP(hipSetDevice(reads->device));
    hipStream_t st = as_stream(stream);
    PA_HIP(hipMemcpyAsync(read_off, reads->off + first, (count + 1) * 8, hipMemcpyDeviceToHost, st));
    PA_HIP(hipStreamSynchronize(st));
    const uint64_t b0 = read_off[0], nb = read_off[count] - b0;
    if (nb) {
        if (seq) PA_HIP(hipMemcpyAsync(seq, reads->seq + b0, nb, hipMemcpyDeviceToHost, st));
        if (qual) PA_HIP(hipMemcpyAsync(qual, reads->qual + b0, nb, hipMemcpyDeviceToHost, st));
        PA_HIP(hipStreamSynchronize(st));
    }
    for (uint64_t i = 0; i <= count; i++) read_off[i] -= b0;
    return PA_OK;
}

void pa_reads_free(pa_reads *reads) {
    if (!reads) return;
    hipSetDevice(reads->device);
    pa::dev_free(reads->seq);
    pa::dev_free(reads->qual);
    pa::dev_free(reads->off);
    delete reads;
}

pa_status pa_result_create(const pa_index *idx, pa_result **out) {
    PA_CHECK(idx && out, PA_EINVAL, "NULL argument");
    PA_CHECK(!idx->released, PA_EINVAL, "the index was released by a failed pa_index_reduce: it may only be freed");
    *out = nullptr;
    PA_HIP(hipSetDevice(idx->device));
    pa_result *r = new (std::nothrow) pa_result();
    PA_CHECK(r != nullptr, PA_ENOMEM, "out of host memory");
    r->device = idx->device;
    r->n_genomes = idx->n_genomes;
    const uint64_t G = idx->n_genomes;
    if (pa::dev_malloc(&r->sum_block, (6 + 2 * G) * 8) != hipSuccess ||
        pa::dev_malloc(&r->min_block, std::max<uint64_t>(G, 1) * 8) != hipSuccess) {
        pa::dev_free(r->sum_block);
        delete r;
        set_error("pa_result_create: device allocation failed");
        return PA_ENOMEM;
    }
    pa_status rc = pa_result_reset(r, nullptr);
    if (rc == PA_OK && hipStreamSynchronize(nullptr) != hipSuccess) rc = PA_EDEVICE;
    if (rc != PA_OK) {
        pa_result_free(r);
        return rc;
    }
    *out = r;
    return PA_OK;
}

pa_status pa_result_reset(pa_result *res, void *stream) {
    PA_CHECK(res != nullptr, PA_EINVAL, "NULL argument");
    PA_HIP(hipSetDevice(res->device));
    return pa::result_reset(res, as_stream(stream));  // async: memset + fill kernel
}

pa_status pa_result_copy_out(const pa_result *res, void *sum_dst, void *min_dst, void *stream) {
    PA_CHECK(res != nullptr, PA_EINVAL, "NULL argument");
    PA_HIP(hipSetDevice(res->device));
    hipStream_t st = as_stream(stream);
    const uint64_t G = res->n_genomes;
    if (sum_dst) PA_HIP(hipMemcpyAsync(sum_dst, res->sum_block, (6 + 2 * G) * 8, hipMemcpyDeviceToDevice, st));
    if (min_dst && G) PA_HIP(hipMemcpyAsync(min_dst, res->min_block, G * 8, hipMemcpyDeviceToDevice, st));
    return PA_OK;
}

pa_status pa_result_copy_in(pa_result *res, const void *sum_src, const void *min_src, void *stream) {
    PA_CHECK(res != nullptr, PA_EINVAL, "NULL argument");
    PA_HIP(hipSetDevice(res->device));
    hipStream_t st = as_stream(stream);
    const uint64_t G = res->n_genomes;
    if (sum_src) PA_HIP(hipMemcpyAsync(res->sum_block, sum_src, (6 + 2 * G) * 8, hipMemcpyDeviceToDevice, st));
    if (min_src && G) PA_HIP(hipMemcpyAsync(res->min_block, min_src, G * 8, hipMemcpyDeviceToDevice, st));
    return PA_OK;
}

pa_status pa_result_load(pa_result *res, const uint64_t *sum_block, const uint64_t *min_block) {
    PA_CHECK(res && sum_block && (res->n_genomes == 0 || min_block), PA_EINVAL, "NULL argument");
    PA_HIP(hipSetDevice(res->device));
    const uint64_t G = res->n_genomes;
    PA_HIP(hipMemcpy(res->sum_block, sum_block, (6 + 2 * G) * 8, hipMemcpyHostToDevice));
    if (G) PA_HIP(hipMemcpy(res->min_block, min_block, G * 8, hipMemcpyHostToDevice));
    return PA_OK;
}

pa_status pa_result_fetch(const pa_result *res, pa_stats *stats, uint64_t *unique_reads, uint64_t *ambiguous_reads,
                          uint64_t *first_key, void *stream) {
    PA_CHECK(res != nullptr, PA_EINVAL, "NULL argument");
    PA_HIP(hipSetDevice(res->device));
    hipStream_t st = as_stream(stream);
    const uint64_t G = res->n_genomes;
    if (stats) PA_HIP(hipMemcpyAsync(stats, res->sum_block, 6 * 8, hipMemcpyDeviceToHost, st));
    if (unique_reads && G) PA_HIP(hipMemcpyAsync(unique_reads, res->sum_block + 6, G * 8, hipMemcpyDeviceToHost, st));
    if (ambiguous_reads && G)
        PA_HIP(hipMemcpyAsync(ambiguous_reads, res->sum_block + 6 + G, G * 8, hipMemcpyDeviceToHost, st));
    if (first_key && G) PA_HIP(hipMemcpyAsync(first_key, res->min_block, G * 8, hipMemcpyDeviceToHost, st));
    PA_HIP(hipStreamSynchronize(st));
    return PA_OK;
}

pa_status pa_result_device_view(pa_result *res, uint64_t **sum_block, uint64_t *n_sum, uint64_t **min_block,
                                uint64_t *n_min) {
    PA_CHECK(res != nullptr, PA_EINVAL, "NULL argument");
    if (sum_block) *sum_block = res->sum_block;
    if (n_sum) *n_sum = 6 + 2ull * res->n_genomes;
    if (min_block) *min_block = res->min_block;
    if (n_min) *n_min = res->n_genomes;
    return PA_OK;
}

void pa_result_free(pa_result *res) {
    if (!res) return;
    hipSetDevice(res->device);
    pa::dev_free(res->sum_block);
    pa::dev_free(res->min_block);
    delete res;
}

pa_status pa_align(const pa_index *idx, const pa_reads *reads, const pa_params *params, uint64_t read_index_base,
                   pa_result *acc, void *stream) {
    PA_CHECK(idx && reads && acc, PA_EINVAL, "NULL argument");
    PA_CHECK(!idx->released, PA_EINVAL, "the index was released by a failed pa_index_reduce: it may only be freed");
    PA_CHECK(acc->n_genomes == idx->n_genomes, PA_EINVAL, "result was created for a different index");
    PA_CHECK(reads->device == idx->device && acc->device == idx->device, PA_EINVAL,
             "index, reads and result must live on the same device");
    PA_CHECK(read_index_base + reads->n < (1ull << 44), PA_EUNSUPPORTED, "read index beyond 2^44");
    pa::DevParams dp;
    PA_TRY(to_dev_params(params, idx->n_genomes, &dp));
    PA_HIP(hipSetDevice(idx->device));
    PA_TRY(pa::index_prepare(const_cast<pa_index *>(idx), as_stream(stream)));
    return pa::align(const_cast<pa_index *>(idx), reads, dp, read_index_base, acc, as_stream(stream));
}

pa_status pa_align_fastq_file(const pa_index *idx, const char *path, const pa_params *params,
                              uint64_t read_index_base, pa_result *acc, int32_t threads, uint64_t window_bytes,
                              void *stream, uint64_t *n_reads) {
    PA_CHECK(idx && path && acc, PA_EINVAL, "NULL argument");
    PA_CHECK(!idx->released, PA_EINVAL, "the index was released by a failed pa_index_reduce: it may only be freed");
    PA_CHECK(acc->n_genomes == idx->n_genomes, PA_EINVAL, "result was created for a different index");
    PA_CHECK(acc->device == idx->device, PA_EINVAL, "index and result must live on the same device");
    pa::DevParams dp;
    PA_TRY(to_dev_params(params, idx->n_genomes, &dp));
    PA_HIP(hipSetDevice(idx->device));
    if (n_reads) *n_reads = 0;
    return pa::align_fastq_file(const_cast<pa_index *>(idx), path, dp, read_index_base, acc, threads > 0 ? threads : 8,
                                window_bytes ? window_bytes : (128ull << 20), as_stream(stream), n_reads);
}

pa_status pa_align_fastq_range(const pa_index *idx, const char *path, uint64_t offset, uint64_t length,
                               const pa_params *params, uint64_t read_index_base, pa_result *acc, int32_t threads,
                               uint64_t window_bytes, void *stream, uint64_t *n_reads, pa_idset **ids) {
    PA_CHECK(idx && path && acc, PA_EINVAL, "NULL argument");
    PA_CHECK(!idx->released, PA_EINVAL, "the index was released by a failed pa_index_reduce: it may only be freed");
    PA_CHECK(acc->n_genomes == idx->n_genomes, PA_EINVAL, "result was created for a different index");
    PA_CHECK(acc->device == idx->device, PA_EINVAL, "index and result must live on the same device");
    PA_CHECK(length > 0, PA_EINVAL, "empty byte range");
    if (ids) *ids = nullptr;
    pa::DevParams dp;
    PA_TRY(to_dev_params(params, idx->n_genomes, &dp));
    PA_HIP(hipSetDevice(idx->device));
    if (n_reads) *n_reads = 0;
    pa_idset *set = nullptr;
    if (ids) {
        set = new (std::nothrow) pa_idset();
        PA_CHECK(set != nullptr, PA_ENOMEM, "out of host memory");
    }
    const pa_status rc = pa::align_fastq_file(const_cast<pa_index *>(idx), path, dp, read_index_base, acc,
                                              threads > 0 ? threads : 8, window_bytes ? window_bytes : (128ull << 20),
                                              as_stream(stream), n_reads, offset, length, set ? &set->h : nullptr);
    if (rc != PA_OK) {
        delete set;
        return rc;
    }
    if (ids) *ids = set;
    return PA_OK;
}

pa_status pa_idsets_disjoint(const pa_idset *const *sets, uint32_t n_sets, int32_t device, int32_t *disjoint) {
    PA_CHECK(disjoint && (n_sets == 0 || sets), PA_EINVAL, "NULL argument");
    std::vector<const std::vector<uint64_t> *> v;
    for (uint32_t i = 0; i < n_sets; i++) {
        PA_CHECK(sets[i] != nullptr, PA_EINVAL, "NULL id set");
        v.push_back(&sets[i]->h);
    }
    bool d = true;
    PA_TRY(pa::idsets_disjoint(v, device, &d));
    *disjoint = d ? 1 : 0;
    return PA_OK;
}

void pa_idset_free(pa_idset *ids) { delete ids; }

pa_status pa_index_dumpref(const pa_index *idx, const uint8_t *keep, const uint32_t *desc_of, uint32_t n_desc,
                           const char *const *desc_json, int32_t fd, int32_t threads, uint64_t *desc_unique,
                           uint64_t *desc_multi, uint64_t *desc_order, uint32_t *desc_last_genome, uint64_t *n_kmers) {
    PA_CHECK(idx && desc_of && desc_json && desc_unique && desc_multi && desc_order && desc_last_genome, PA_EINVAL,
             "NULL argument");
    PA_CHECK(!idx->released, PA_EINVAL, "the index was released by a failed pa_index_reduce: it may only be freed");
    PA_CHECK(fd >= 0, PA_EINVAL, "bad file descriptor");
    for (uint32_t d = 0; d < n_desc; d++) PA_CHECK(desc_json[d], PA_EINVAL, "NULL description");
    PA_HIP(hipSetDevice(idx->device));
    return pa::index_dumpref(idx, keep, desc_of, n_desc, desc_json, fd, threads > 0 ? threads : 8, desc_unique,
                             desc_multi, desc_order, desc_last_genome, n_kmers, nullptr);
}

pa_status pa_fastq_prefetch_start(const char *path, int32_t device, int32_t threads, uint64_t window_bytes,
                                  pa_fastq_prefetch **out) {
    PA_CHECK(path && out, PA_EINVAL, "NULL argument");
    *out = nullptr;
    PA_CHECK(device >= 0, PA_EINVAL, "no such device");
    // (no HIP call here: the runtime starts on the prefetch thread, beside the caller's FASTA parse;
    // a bad device is reported by pa_align_fastq_prefetched)
    return pa::fastq_prefetch_start(path, device, threads > 0 ? threads : 8,
                                    window_bytes ? window_bytes : (128ull << 20), out);
}

void pa_fastq_prefetch_free(pa_fastq_prefetch *pf) { pa::fastq_prefetch_free(pf); }

pa_status pa_align_fastq_prefetched(const pa_index *idx, pa_fastq_prefetch *pf, const pa_params *params,
                                    uint64_t read_index_base, pa_result *acc, void *stream, uint64_t *n_reads) {
    PA_CHECK(idx && pf && acc, PA_EINVAL, "NULL argument");
    PA_CHECK(!idx->released, PA_EINVAL, "the index was released by a failed pa_index_reduce: it may only be freed");
    PA_CHECK(acc->n_genomes == idx->n_genomes, PA_EINVAL, "result was created for a different index");
    PA_CHECK(acc->device == idx->device, PA_EINVAL, "index and result must live on the same device");
    pa::DevParams dp;
    PA_TRY(to_dev_params(params, idx->n_genomes, &dp));
    PA_HIP(hipSetDevice(idx->device));
    if (n_reads) *n_reads = 0;
    return pa::align_fastq_prefetched(const_cast<pa_index *>(idx), pf, dp, read_index_base, acc, as_stream(stream),
                                      n_reads);
}

pa_status pa_align_detail(const pa_index *idx, const pa_reads *reads, const pa_params *params, uint8_t *read_type,
                          uint32_t *filtered_kmers, uint32_t *redundant_kmers, uint64_t *list_off, uint32_t *lists,
                          uint64_t list_cap, uint64_t *list_total, void *stream) {
    PA_CHECK(idx && reads && read_type && filtered_kmers && redundant_kmers && list_off, PA_EINVAL, "NULL argument");
    PA_CHECK(!idx->released, PA_EINVAL, "the index was released by a failed pa_index_reduce: it may only be freed");
    PA_CHECK(reads->device == idx->device, PA_EINVAL, "index and reads must live on the same device");
    pa::DevParams dp;
    PA_TRY(to_dev_params(params, idx->n_genomes, &dp));
    PA_HIP(hipSetDevice(idx->device));
    PA_TRY(pa::index_prepare(const_cast<pa_index *>(idx), as_stream(stream)));
    return pa::align_detail(const_cast<pa_index *>(idx), reads, dp, read_type, filtered_kmers, redundant_kmers,
                            list_off, lists, list_cap, list_total, as_stream(stream));
}

pa_status pa_align_batch(const pa_index *idx, const uint8_t *seq, const uint8_t *qual, const uint64_t *read_off,
                         uint64_t n_reads, uint64_t read_index_base, const pa_params *params, pa_stats *stats,
                         uint64_t *unique_reads, uint64_t *ambiguous_reads, uint64_t *first_key, void *stream) {
    PA_CHECK(idx != nullptr, PA_EINVAL, "NULL argument");
    PA_CHECK(!idx->released, PA_EINVAL, "the index was released by a failed pa_index_reduce: it may only be freed");
    pa_reads *r = nullptr;
    pa_result *res = nullptr;
    PA_TRY(pa_reads_upload(idx->device, seq, qual, read_off, n_reads, stream, &r));
    pa_status rc = pa_result_create(idx, &res);
    if (rc == PA_OK) rc = pa_align(idx, r, params, read_index_base, res, stream);
    const uint64_t G = idx->n_genomes;
    if (rc == PA_OK) {
        pa_stats s{};
        uint64_t *u = new (std::nothrow) uint64_t[3 * G + 1];
        if (!u) {
            rc = PA_ENOMEM;
        } else {
            rc = pa_result_fetch(res, &s, u, u + G, u + 2 * G, stream);
            if (rc == PA_OK) {
                if (stats) {
                    stats->unique_mapped_reads += s.unique_mapped_reads;
                    stats->ambiguous_mapped_reads += s.ambiguous_mapped_reads;
                    stats->unmapped_reads += s.unmapped_reads;
                    stats->filtered_quality_reads += s.filtered_quality_reads;
                    stats->filtered_quality_kmers += s.filtered_quality_kmers;
                    stats->filtered_hr_kmers += s.filtered_hr_kmers;
                }
                for (uint64_t g = 0; g < G; g++) {
                    if (unique_reads) unique_reads[g] += u[g];
                    if (ambiguous_reads) ambiguous_reads[g] += u[G + g];
                    if (first_key) first_key[g] = std::min(first_key[g], u[2 * G + g]);
                }
            }
            delete[] u;
        }
    }
    pa_result_free(res);
    pa_reads_free(r);
    return rc;
}

pa_status pa_profile_enable(pa_index *idx, int32_t enable) {
    PA_CHECK(idx != nullptr, PA_EINVAL, "NULL argument");
    idx->profile = enable != 0;
    return PA_OK;
}

pa_status pa_profile_read(pa_index *idx, double *main_ms, uint64_t *launches, uint64_t *deferred_reads) {
    PA_CHECK(idx != nullptr, PA_EINVAL, "NULL argument");
    PA_HIP(hipSetDevice(idx->device));
    double ms = 0;
    for (size_t i = 0; i < idx->ev_start.size(); i++) {
        PA_HIP(hipEventSynchronize(idx->ev_stop[i]));
        float t = 0;
        PA_HIP(hipEventElapsedTime(&t, idx->ev_start[i], idx->ev_stop[i]));
        ms += t;
        hipEventDestroy(idx->ev_start[i]);
        hipEventDestroy(idx->ev_stop[i]);
    }
    const uint64_t nl = idx->ev_start.size();
    idx->ev_start.clear();
    idx->ev_stop.clear();
    uint64_t dt = 0;
    PA_HIP(hipDeviceSynchronize());
    PA_HIP(hipMemcpy(&dt, idx->counters + 1, 8, hipMemcpyDeviceToHost));
    PA_HIP(hipMemset(idx->counters + 1, 0, 8));
    if (main_ms) *main_ms = ms;
    if (launches) *launches = nl;
    if (deferred_reads) *deferred_reads = dt;
    return PA_OK;
}

pa_status pa_profile_read_kernels(pa_index *idx, double *ms, uint64_t *launches) {
    PA_CHECK(idx != nullptr && ms != nullptr && launches != nullptr, PA_EINVAL, "NULL argument");
    PA_HIP(hipSetDevice(idx->device));
    for (int i = 0; i < PA_PROF_KERNELS; i++) {
        ms[i] = 0;
        launches[i] = 0;
    }
    pa_status rc = PA_OK;
    for (const auto &e : idx->kev) {
        float t = 0;
        hipError_t he = hipEventSynchronize(e.stop);
        if (he == hipSuccess) he = hipEventElapsedTime(&t, e.start, e.stop);
        if (he != hipSuccess && rc == PA_OK) {
            pa::set_error(std::string("pa_profile_read_kernels: ") + hipGetErrorString(he));
            rc = PA_EDEVICE;
        }
        ms[e.slot] += t;
        launches[e.slot]++;
        hipEventDestroy(e.start);
        hipEventDestroy(e.stop);
    }
    idx->kev.clear();
    return rc;
}

}  // extern "C"
