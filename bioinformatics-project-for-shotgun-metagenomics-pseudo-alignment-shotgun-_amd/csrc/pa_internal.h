// Internal host-side structures of libpa.so (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/pa.h"
#include "pa_home.h"

namespace pa {

// Last error, thread-local; set by the PA_* macros below.
void set_error(const std::string &msg);

#define PA_HIP(call)                                                                              \
    do {                                                                                          \
        hipError_t e_ = (call);                                                                   \
        if (e_ != hipSuccess) {                                                                   \
            ::pa::set_error(std::string("HIP error: ") + hipGetErrorString(e_) + " at " __FILE__ ":" + \
                            std::to_string(__LINE__) + " (" #call ")");                          \
            return PA_EDEVICE;                                                                    \
        }                                                                                         \
    } while (0)

#define PA_TRY(call)                         \
    do {                                     \
        pa_status s_ = (call);               \
        if (s_ != PA_OK) return s_;          \
    } while (0)

// Number of 64-bit words of a packed k-mer key: 2k bits, top word < 64 bits
// so that an all-ones top word can never be a key (empty-slot sentinel).
inline int key_words(int64_t k) { return (int)(k / 32) + 1; }
// Bytes per hash-table slot: key words + {uint32 class, uint32 tile position}.
inline int slot_bytes(int nw) { return 8 * nw + 8; }
// Read buffers are over-allocated so a wave may fetch a whole staging window
// (up to 512 B) past any read start without a bounds check.
constexpr uint64_t kReadPad = 1024;

// Device arguments of the per-read kernels (clamped, see pa_api.cpp).
struct DevParams {
    int32_t m, p;          // m >= 0; p < 0 -> no validation
    int32_t mrq, mkq, mg;  // already clamped to ranges where semantics are unchanged
    uint32_t flags;
};

// Device memory (pa_mem.cpp): large buffers from the library's slab pool,
// small ones straight from hipMalloc.  Every device buffer of libpa.so is
// taken and given back through these; dev_mem_info counts the pool's free
// ranges as free.
hipError_t dev_malloc_raw(void **p, size_t n);
template <typename T>
inline hipError_t dev_malloc(T **p, size_t n) {
    return dev_malloc_raw((void **)p, n);
}
hipError_t dev_free(void *p);
// Like dev_malloc but never gives the pool's idle slabs back to the driver to
// make room (whose reclaim stalls): hipErrorOutOfMemory when no free range of
// the pool and no free device memory can hold n bytes.
hipError_t dev_malloc_try(void **p, size_t n);
size_t dev_pool_largest_free();  // the largest free range of the current device's slabs
hipError_t dev_mem_info(size_t *free_b, size_t *total_b);
size_t dev_trim(int dev);
void dev_pool_stats(int dev, size_t *slab_bytes, size_t *free_bytes);

struct Workspace {  // grow-only device scratch owned by an index
    void *ptr = nullptr;
    size_t bytes = 0;
};

}  // namespace pa

struct pa_index {
    int device = 0;
    int64_t k = 0;
    int nw = 1;
    uint32_t n_genomes = 0;
    // open-addressing table: slots of {uint64 key[nw]; uint32 cls; uint32 tpos}
    void *table = nullptr;
    uint64_t cap = 0;
    pad::HomeCfg home{};               // home-slot function
    uint64_t n_kmers = 0;
    // classes: cls < n_genomes means {cls}; cls >= n_genomes is multi class (cls - n_genomes)
    uint64_t n_multi = 0;
    uint64_t *class_off = nullptr;    // [n_multi]
    uint32_t *class_size = nullptr;   // [n_multi]
    uint32_t *class_genomes = nullptr;
    uint64_t class_entries = 0;
    uint64_t *class_mask = nullptr;     // G <= 64: membership mask per set, indexed like class_genomes
    // genome codes (0-3 ACGT, 4 other) kept for read synthesis
    uint8_t *codes = nullptr;
    uint64_t *goff = nullptr;          // device [n_genomes+1]
    std::vector<uint64_t> h_goff;
    uint64_t total_windows = 0;
    int tpos_local = 0;                // slot.tpos genome-local (references of >= 2^32 bases), else concatenated
    uint64_t distinct_estimate = 0;    // HyperLogLog estimate (+3 %) when the table was sized on it, else 0
    int released = 0;                  // a failed pa_index_reduce emptied it: it may only be freed
    int force_large = 0;               // PA_LAYOUT=large: the layout of a reference too large for the default one
    int compact_table = 0;             // PA_BUILD_COMPACT: 2 slots per genome window (a job of few reads)
    // genome tiling (single-word keys, < 2^32 genome bases): the genomes as one
    // concatenated 2-bit string plus the class of the k-mer starting at every
    // position (NONE where no indexed window starts); slots point into it (tpos)
    uint64_t tile_n = 0;               // concatenated bases (0: no tiling)
    int tiles_pending = 0;             // 1: the tiles below are still to be made (index_prepare)
    uint32_t *tile_cls = nullptr;      // [tile_n]
    uint64_t *tile_pk = nullptr;       // [tile_n / 32 + 32] MSB-first 2-bit words (padded)
    uint64_t *tile_lw = nullptr;       // [4 (tile_n / 64 + 5)] lane-walk blocks: 2-bit words + flag planes (k_tile_walk)
    uint64_t *tile_big = nullptr;      // [tile_n / 64 + 4] plane "set size > tile_big_mg" (pa_align, cached)
    int64_t tile_big_mg = -1;          // the --max-genomes value tile_big was made for (-1: none)
    void *tile_nb = nullptr;           // [3 tile_n] one-substitution neighbour bits (k_nb_build), optional:
    int nb_spec = 0;                   //   1: 64-bit words, present | specific << 32; 0: 32-bit words, present
    void *tile_nb1 = nullptr;          //   its second piece, words nb_split.. (null: one piece; pa_device.h NbW)
    uint64_t nb_split = ~0ull;
    uint32_t *tile_rcnb = nullptr;     // [3 tile_n] the same for the neighbours' reverse complements (present), optional
    int rcnb_pending = 0;              //   1: left for the first pass that queues enough seedless reads (pa_align.hip)
    int rcnb_checks = 0;               //   passes that looked and found too few
    uint32_t *tile_nbbig = nullptr;    // [3 tile_n] neighbour present with a set > tile_nbbig_mg (pa_align, cached)
    int64_t tile_nbbig_mg = -1;
    uint4 *tile_nbm = nullptr;         // [3 tile_n] {present, specific, set > tile_nbm_mg, 0}: tile_nb and tile_nbbig
    int64_t tile_nbm_mg = -1;          //   interleaved, one 16-B load per mismatch (pa_align, cached; when it fits)
    int nb_skip = 0;                   // (index_prepare) make the tiles without the neighbour bits
    int nb_pending = 0;                // 1: tiles made, neighbour bits not yet (too few reads expected)
    uint64_t reads_seen = 0;           // reads aligned so far (the neighbour bits follow at kNbReadsPerKBase / 1000 per base)
    uint32_t *tile_gblk = nullptr;     // [(tile_n >> 16) + 2] the genome holding position j << 16
    uint64_t *bloom = nullptr;         // [2^bloom_lg] Bloom filter of the table's keys (k_bloom_build), optional
    uint32_t *mm_bits = nullptr;       // [2^mm_lg / 32] minimizer presence bitmap (k_mm_build), optional
    uint32_t mm_lg = 0;
    uint64_t *tile_rcp = nullptr;      // [tile_n / 64 + 5] bit t: the reverse complement of the k-mer at t may be
                                       //   a key (present, or no indexed window at t) -- k_tile_rcp, optional
    uint32_t bloom_lg = 0;
    uint64_t device_bytes = 0;
    // align scratch
    pa::Workspace ws;
    uint32_t *queue = nullptr;         // read indices deferred to the exact kernel
    uint32_t *queue_hard = nullptr;    // read indices the lane kernel leaves to the wave kernel
    uint32_t *queue_na = nullptr;      // read indices the lane kernel found no seed for (k_align_lane_rc / _na)
    uint32_t *queue_na2 = nullptr;     // those tested window by window (k_align_lane_na)
    uint64_t *queue_na_keys = nullptr; // [2 per queue_na entry] their outer seeds' reverse complements (k_rc_seeds)
    uint32_t *queue_rc = nullptr;      // reads with a reverse-complement seed (k_align_lane_rc)
    uint64_t *queue_rc_anc = nullptr;  //   its first occurrence | seed << 63
    uint4 *qmask = nullptr;            // per read: windows failing --min-kmer-quality (k_quality_masks)
    uint8_t *qdrop = nullptr;          // per read: fails --min-read-quality
    uint64_t qmask_cap = 0;
    unsigned long long *na_count = nullptr;
    uint32_t *seg_cnt = nullptr;       // [kSegMaxWaves] the lane kernel's per-wave queue segments (pa_align.hip)
    uint64_t queue_cap = 0;            // entries of every queue (the reads of a batch + kSegSlack)
    uint64_t *counters = nullptr;      // [0] queue length, [1] deferred total, [2] error flags, [3] hard reads,
                                       // [4..31] PA_STATS counters
    // profiling
    bool profile = false;
    std::vector<hipEvent_t> ev_start, ev_stop;
    struct KernelEvents {
        int slot;  // PA_PROF_* (include/pa.h)
        hipEvent_t start, stop;
    };
    std::vector<KernelEvents> kev;     // one pair per kernel launch of the align pass
    double prof_ms = 0;
    uint64_t prof_launches = 0;
};

struct pa_reads {
    int device = 0;
    uint64_t n = 0;
    uint64_t n_bases = 0;
    uint32_t max_len = 0;
    uint8_t *seq = nullptr;
    uint8_t *qual = nullptr;
    uint64_t *off = nullptr;  // [n+1]
    // (pa_align) the smallest quality byte and read length, once measured
    // (-1: not yet): quality thresholds no read can fail are then not applied
    int32_t q_min = -1;
    int64_t len_min = -1;
};

struct pa_idset {  // id hashes of a FASTQ byte range (pa_align_fastq_range)
    std::vector<uint64_t> h;
};

struct pa_result {
    int device = 0;
    uint32_t n_genomes = 0;
    uint64_t *sum_block = nullptr;  // [6 + 2G]
    uint64_t *min_block = nullptr;  // [G]
};

namespace pa {
pa_status index_build(pa_index *idx, const char *genomes, const uint64_t *goff, uint32_t n, int64_t k,
                      hipStream_t st, bool defer_tiles, uint8_t *dev_codes = nullptr);
pa_status index_reduce(pa_index *idx, const uint32_t *sel, uint32_t n, hipStream_t st, bool defer_tiles);
// The tiles of a deferred build (no-op otherwise).  reads_hint: the reads the
// caller expects to align with this index; below kNbReadsPerKBase / 1000 per genome
// base the neighbour bits are left for later (index_note_reads makes them once
// the reads aligned pass that point): they cost ~0.5 ns per base and save
// ~0.25 ns per read on C2 (3.43 vs 1.87 G reads/s; build 0.36 vs 0.24 s).
constexpr uint64_t kNbReadsPerKBase = PA_NB_READS_PER_KBASE;
// reads past the neighbour bits' break-even for an index of `bases` genome
// bases and keys of nw words (two- and three-word keys' bits cost more to make)
inline bool nb_repaid(uint64_t reads, uint64_t bases, int nw = 1) {
    const uint64_t per_k = nw >= 3 ? PA_NB_READS_PER_KBASE_3W : nw == 2 ? PA_NB_READS_PER_KBASE_2W : kNbReadsPerKBase;
    return reads >= (bases * per_k + 999) / 1000;
}
// complete: also make neighbour bits left pending, when reads_hint (the reads
// still to come; ~0: unknown) passes the break-even (pa_index_prepare[_ex]).
pa_status index_prepare(pa_index *idx, hipStream_t st, uint64_t reads_hint = ~0ull, bool complete = false);
pa_status index_note_reads(pa_index *idx, uint64_t n, hipStream_t st);
pa_status index_build_rcnb(pa_index *idx, hipStream_t st);  // the pending reverse-complement neighbour bits, now
pa_status index_lookup(const pa_index *idx, const char *kmers, uint64_t n, uint32_t kmer_len, int64_t *cls_out,
                       uint32_t *size_out, hipStream_t st);
pa_status index_positions(const pa_index *idx, const char *kmers, uint64_t n, uint32_t kmer_len, uint32_t flags,
                          pa_kmer_hit *hits, uint64_t cap, uint64_t *n_hits, hipStream_t st);
pa_status index_extsim_stats(const pa_index *idx, const uint32_t *group_of, uint32_t n_groups, uint64_t *total,
                             uint64_t *uniq, uint64_t *inter, hipStream_t st);
pa_status reads_synthesize(const pa_index *idx, pa_reads *r, uint64_t n, uint32_t len, uint64_t first,
                           uint64_t seed, double sub_rate, double rc_rate, double foreign_rate, hipStream_t st);
pa_status align(pa_index *idx, const pa_reads *r, const DevParams &p, uint64_t base, pa_result *acc,
                hipStream_t st);
pa_status align_detail(pa_index *idx, const pa_reads *r, const DevParams &p, uint8_t *type, uint32_t *qf,
                       uint32_t *hr, uint64_t *list_off, uint32_t *lists, uint64_t list_cap, uint64_t *list_total,
                       hipStream_t st);
pa_status reads_measure(pa_reads *r, hipStream_t st);  // q_min / len_min of a batch (at its creation)
// the filters an align of batch r applies: quality thresholds no read can fail dropped
pa_status effective_params(const pa_reads *r, const DevParams &p, DevParams &out, hipStream_t st);
pa_status ensure_workspace(pa_index *idx, size_t bytes);
pa_status reserve_queues(pa_index *idx, uint64_t n);  // align queues for batches of up to n reads
pa_status ensure_qmask(pa_index *idx, uint64_t n);    // quality-filter masks for batches of up to n reads
// offset / length: a byte range of a plain file, cut on record boundaries
// (pa_align_fastq_range); ids_out: the range's id hashes
pa_status align_fastq_file(pa_index *idx, const char *path, const DevParams &prm, uint64_t base, pa_result *acc,
                           int threads, uint64_t window, hipStream_t st, uint64_t *n_reads, uint64_t offset = 0,
                           uint64_t length = ~0ull, std::vector<uint64_t> *ids_out = nullptr);
pa_status idsets_disjoint(const std::vector<const std::vector<uint64_t> *> &sets, int device, bool *disjoint);
pa_status fastq_prefetch_start(const char *path, int device, int threads, uint64_t window, pa_fastq_prefetch **out);
void fastq_prefetch_free(pa_fastq_prefetch *pf);
pa_status align_fastq_prefetched(pa_index *idx, pa_fastq_prefetch *pf, const DevParams &prm, uint64_t base,
                                 pa_result *acc, hipStream_t st, uint64_t *n_reads);
pa_status index_dumpref(const pa_index *idx, const uint8_t *keep, const uint32_t *desc_of, uint32_t n_desc,
                        const char *const *desc_json, int fd, int threads, uint64_t *desc_unique, uint64_t *desc_multi,
                        uint64_t *desc_order, uint32_t *desc_last_genome, uint64_t *n_kmers_out, hipStream_t st);
pa_status result_reset(pa_result *res, hipStream_t st);
void index_release(pa_index *idx);
void warm_index(hipStream_t st);  // one empty launch per source file: loads its code object
void warm_align(hipStream_t st);
void warm_fastq(hipStream_t st);
void warm_dump(hipStream_t st);
}  // namespace pa
