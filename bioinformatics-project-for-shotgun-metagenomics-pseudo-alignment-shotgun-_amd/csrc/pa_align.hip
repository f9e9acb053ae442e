// Per-read pseudo-alignment kernels: Read.pseudo_align + PseudoAlignment
// counters of the reference (src/kmer.py:394-657), bit-exact.
//
// Two kernels implement the same per-read semantics:
//
//  * k_align_fast<NW, WPL> -- the hot path.  One wavefront per read (reads
//    grid-strided over a persistent grid, 4 waves per workgroup), WPL windows
//    per lane (W <= 64*WPL).  Per read:
//      1. raw-ASCII quality prefix sums by a wave scan (quirk 5);
//      2. the read is 2-bit packed in LDS by 32-lane OR reductions, non-ACGT
//         bases recorded in a ballot bitmap; every window key is then an O(1)
//         funnel shift out of the packed words;
//      3. all WPL hash probes of a lane are issued together (independent 16-B
//         HBM loads) -- this is the dominant cost;
//      4. distinct k-mers (quirk 3) by an LDS hash keyed on the table slot, the
//         first window of every slot kept with ds_min;
//      5. the distinct k-mers are grouped by genome set ("class") in a second
//         LDS hash (count + first window); singleton classes are the specific
//         k-mers, so the m-decision (quirk 7) is a wave max/second-max;
//      6. p-validation (quirk 8) expands the multi-genome classes of the read
//         into an LDS genome hash (total counts + first window) -- reads whose
//         genome union does not fit are deferred to the exact kernel;
//      7. per-genome unique/ambiguous counts and first-appearance keys go to
//         per-workgroup LDS counters, flushed with one atomic per genome at
//         the end (no global atomics per read).
//  * k_align_exact<NW> -- one workgroup per read with dense per-genome scratch
//    in global memory; handles any read length / genome-set size.  It runs the
//    deferred reads of the fast kernel and every read of the per-read detail
//    API (PseudoAlignment.reads, Read.pseudo_align).
//
// Summary key order (quirk 9): get_summary inserts genomes in the order they
// first appear in genomes_mapped_to lists walked read by read.  Each genome's
// first appearance is kept as key = (global read index << 20) | position in
// that read's list, min-reduced; the host sorts by it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "pa_device.h"
#include "pa_internal.h"

using namespace pad;

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
// k_align_lane's queue segments (AlignArgs::na_seg): one per wave of its
// grid, 64 entries per chunk of reads the wave takes; the queues hold the
// reads of a batch plus one chunk per wave of slack.
constexpr uint32_t kSegMaxWaves = 16384;
constexpr uint64_t kSegSlack = 64ull * kSegMaxWaves;
constexpr uint32_t kLdsGenomeCap = 2048;  // per-workgroup LDS counters up to this many genomes

enum : uint32_t { F_MRQ = 1, F_MKQ = 2, F_MG = 4 };

struct AlignArgs {
    const void *table;
    uint64_t cap;
    HomeCfg home;
    uint32_t G;
    int k;
    const uint32_t *class_genomes;  // multi-genome set records [size, genomes...], id = G + offset
    const uint64_t *class_mask;     // G <= 64: membership mask of each record (same offsets)
    const uint32_t *tile_cls;       // genome tiling (pa_index.hip); tile_n == 0: none
    const uint64_t *tile_pk;
    uint64_t tile_n;
    const uint64_t *goff;           // genome start positions [G + 1] (concatenated coordinates)
    const uint64_t *tile_lw;        // lane kernel walk blocks (2-bit words + flag planes per 64 positions)
    const uint64_t *tile_big;       // lane kernel, --max-genomes >= 2: plane "set size > mg" (else null)
    const void *tile_nb;            // one-substitution neighbour bits (null: none)
    uint64_t nb_base1, nb_split;    //   words nb_split.. at nb_base1 + i * word bytes (pa_device.h NbW; ~0: one piece)
    const uint32_t *nbbig_ld;       //   the --max-genomes >= 2 half's loads: tile_nbbig, or a dummy word 0
    uint64_t nbbig_mask;            //   ~0 with tile_nbbig, 0 without (the loads read word 0 of a valid buffer)
    int nb_spec;                    //   1: 64-bit present | specific << 32, 0: 32-bit present
    const uint32_t *tile_nbbig;     // --max-genomes >= 2: neighbour present with a set > mg (k_nb_big; null: none)
    const uint4 *tile_nbm;          //   the same interleaved with tile_nb's words (k_nb_merge; null: none)
    int mg_nb;                      // --max-genomes: the neighbour bits tell every present neighbour's set vs mg
    const uint32_t *gblk;           // the genome holding position j << 16 (tiled indexes)
    const uint64_t *bloom;          // Bloom filter of the keys (null: none), 2^bloom_lg words
    const uint64_t *tile_rcp;       // reverse-complement plane (k_tile_rcp; null: none)
    const uint32_t *mm_bits;        // minimizer presence bitmap (k_mm_build; null: none), 2^mm_lg bits
    uint32_t mm_lg;
    const uint32_t *tile_rcnb;      // reverse-complement one-substitution neighbour bits (null: none)
    uint32_t bloom_lg;
    int walk_rounds;
    int tpos_local;                 // slot.tpos genome-local (first_pos), else concatenated
    uint32_t lane_maxpend;  // lane kernel: more unwalked windows than this -> wave kernel
    int lane_noanchor;      // lane kernel: a read without any seed in the index probes all its windows
                            // (Bloom filter first) instead of going to the wave kernel
    int dbg_mode;  // PA_STATS / PA_DISSECT builds: stop each read after phase N (timing dissection; results invalid)
    const uint8_t *seq;
    const uint8_t *qual;
    const uint64_t *off;
    uint64_t n;
    uint64_t base;  // global index of read 0
    pa::DevParams prm;
    // accumulators
    unsigned long long *stats;   // [6]
    unsigned long long *uniq;    // [G]
    unsigned long long *amb;     // [G]
    unsigned long long *first;   // [G]
    // deferral to the exact kernel
    uint32_t *queue;
    unsigned long long *qcount;
    unsigned long long *deferred_total;
    // lane kernel: reads it leaves to the wave kernel
    uint32_t *queue_hard;
    unsigned long long *queue_hard_count;
    uint32_t *queue_na;                    // lane kernel: reads with no seed in the index (null: to the wave kernel)
    unsigned long long *queue_na_count;
    uint64_t *queue_na_keys;               // lane kernel: their outer seeds' reverse complements (k_rc_seeds; null: none)
    uint32_t *queue_rc;                    // k_rc_seeds: reads with a reverse-complement seed in the index,
    uint64_t *queue_rc_anc;                //   its first occurrence | seed << 63 (k_align_lane_rc)
    unsigned long long *queue_rc_count;
    uint32_t *queue_na2;                   // k_rc_seeds / k_align_lane_rc: the reads to test window by window
    unsigned long long *queue_na2_count;   //   (k_align_lane_na)
    uint64_t na_min;                       // fewer than this: k_align_lane_na hands them to the wave kernel
    uint32_t na_seg;                       // k_align_lane queues its seedless reads (queue_na, queue_na_keys) in
    uint32_t *seg_cnt;                     //   per-wave segments, without atomics: wave s of its grid writes
    uint32_t nseg;                         //   entries s * seg_cap ... and their number to seg_cnt[s]; k_rc_seeds
    uint64_t seg_cap;                      //   takes them (nseg: the grid's waves)
    uint64_t queue_cap;                    // entries of every queue
    const uint4 *qmask;                    // (quality filters) per read: windows failing --min-kmer-quality
    const uint8_t *qdrop;                  //   and 1 if the read fails --min-read-quality (k_quality_masks)
    // wave kernel input: a list of read indices (null: reads 0 .. n-1)
    const uint32_t *rlist;
    const unsigned long long *rlist_count;
    unsigned long long *dbg;  // PA_STATS builds: [0] windows [1] probed [2] walk-resolved [3] anchors (wave
                              // kernel), [4..11] lane kernel: reads left to the wave kernel, by reason
};

__device__ __forceinline__ uint64_t first_key(uint64_t read, uint32_t rank) { return (read << 20) | rank; }

// ---------------------------------------------------------------------------
// fast kernel
// ---------------------------------------------------------------------------

struct WgCounters {
    uint32_t *uniq;
    uint32_t *amb;
    unsigned long long *first;
    bool lds;
};

__device__ __forceinline__ void count_genome(const AlignArgs &a, const WgCounters &c, uint32_t g, bool unique,
                                             uint32_t times, uint64_t key) {
    if (c.lds) {
        atomicAdd(unique ? &c.uniq[g] : &c.amb[g], times);
        if (key < c.first[g]) atomicMin(&c.first[g], (unsigned long long)key);
    } else {
        atomicAdd(unique ? &a.uniq[g] : &a.amb[g], (unsigned long long)times);
        atomicMin(&a.first[g], (unsigned long long)key);
    }
}

#include "pa_fast.h"

// The quality filters of the lane kernels, made for all reads up front (a
// kernel of its own, instead of the lane kernels' tight registers): per read,
// whether its raw-ASCII quality sum is below mrq * len (mean_quality <
// min_read_quality, src/kmer.py:394-399, 587) and the windows whose sum is
// below mkq * k (Read.kmer_quality < min_kmer_quality, src/kmer.py:404-408,
// 420-423) as a 128-bit mask.  One read per thread, all in registers: its
// 16-B chunks loaded at once, realigned to the read's first byte (v_alignbit),
// the bytes k earlier made by a second realignment (k >> 2 is a template
// parameter, dispatched once per launch: every index below is a constant), a
// running window sum per byte and the window test as a bit of a 176-bit mask
// in end-position coordinates, shifted down by k - 1 at the end.  Reads longer
// than the lane kernels take (176) get nothing (they go to the wave kernel).
constexpr int kQmDwords = 44;  // 176 bytes
template <int KQ>
__device__ __forceinline__ void quality_read(const uint8_t *__restrict__ qual, uint64_t o, uint32_t len, int k,
                                             uint32_t T, int64_t mrq, uint32_t flags, uint4 &mask, uint8_t &drop) {
    // 16-B loads from the read's first dword (global loads need 4-B alignment
    // only), all twelve: the read buffers carry kReadPad bytes past the last read
    // (a vector type that states its 4-B alignment: the address is a dword's,
    // not a 16-B one, and the compiler may not assume more)
    typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
    const u32x4_a4 *sp = (const u32x4_a4 *)(qual + (o & ~3ull));
    const uint32_t sb = 8 * (uint32_t)(o & 3);
    uint32_t dw[kQmDwords + 4];
#pragma unroll
    for (int c = 0; c < (kQmDwords + 4) / 4; c++) {
        const u32x4_a4 v = sp[c];
        dw[4 * c] = v.x, dw[4 * c + 1] = v.y, dw[4 * c + 2] = v.z, dw[4 * c + 3] = v.w;
    }
    // rd[j] = bytes 4j .. 4j + 3 of the read
    uint32_t rd[kQmDwords];
#pragma unroll
    for (int j = 0; j < kQmDwords; j++) rd[j] = __builtin_amdgcn_alignbit(dw[j + 1], dw[j], sb);
    // total of the read's bytes: the sum of the whole dwords below len >> 2
    // (selected, no branch), then the rest
    const uint32_t nfull = len >> 2, pmask = (len & 3) ? (1u << (8 * (len & 3))) - 1 : 0u;
    uint32_t run_tot = 0, total = 0, part = 0;
#pragma unroll
    for (int j = 0; j < kQmDwords; j++) {
        const bool at = (uint32_t)j == nfull;
        total = at ? run_tot : total;
        part = at ? rd[j] : part;
        run_tot = __builtin_amdgcn_sad_u8(rd[j], 0u, run_tot);
    }
    total = nfull >= (uint32_t)kQmDwords ? run_tot : total;
    total = __builtin_amdgcn_sad_u8(part & pmask, 0u, total);
    drop = ((flags & 1u) && (int64_t)total < mrq * (int64_t)len) ? 1 : 0;
    mask = make_uint4(0, 0, 0, 0);
    if (!(flags & 2u) || len < (uint32_t)k) return;
    // E bit i: the window ending at byte i fails (its sum < T); bytes i - k
    // from rk (0 before the read).  run carries the window sum minus T, whose
    // sign is the test (sums and T < 2^31); each sign bit is shifted in at the
    // bottom of e (v_alignbit: e << 1 | run >> 31), so a word is built
    // bit-reversed and turned round once.
    const uint32_t kb = 8 * ((uint32_t)k & 3);
    uint32_t E[kQmDwords / 8 + 3] = {};  // (+2 zero words: the shift by up to k - 1 = 94 bits below)
    uint32_t run = 0u - T, e = 0;
#pragma unroll
    for (int j = 0; j < kQmDwords; j++) {
        const uint32_t a1 = j - KQ >= 0 ? rd[j - KQ] : 0u, a0 = j - KQ - 1 >= 0 ? rd[j - KQ - 1] : 0u;
        const uint32_t rk = kb ? __builtin_amdgcn_alignbit(a1, a0, 32 - kb) : a1;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            run += ((rd[j] >> (8 * b)) & 255u) - ((rk >> (8 * b)) & 255u);
            e = __builtin_amdgcn_alignbit(e, run, 31);
        }
        if (j % 8 == 7) E[j / 8] = __builtin_bitreverse32(e), e = 0;
    }
    static_assert(kQmDwords % 8 == 4, "the last mask word holds 16 window ends");
    E[kQmDwords / 8] = __builtin_bitreverse32(e << 16);
    // only windows inside the read (ends k - 1 .. len - 1), bit w = the window starting at w
#pragma unroll
    for (int d = 0; d <= kQmDwords / 8; d++) {
        const int32_t hi = (int32_t)len - 32 * d;
        E[d] &= hi >= 32 ? ~0u : hi <= 0 ? 0u : (1u << hi) - 1;
    }
    const uint32_t sh = (uint32_t)k - 1, shb = sh & 31, q = sh >> 5;  // (k <= 95: up to two words and 30 bits)
    uint32_t F[4];
#pragma unroll
    for (int d = 0; d < 4; d++)
        F[d] = __builtin_amdgcn_alignbit(q >= 2 ? E[d + 3] : q == 1 ? E[d + 2] : E[d + 1],
                                         q >= 2 ? E[d + 2] : q == 1 ? E[d + 1] : E[d], shb);
    mask = make_uint4(F[0], F[1], F[2], F[3]);
}

template <int KQ>
__device__ __forceinline__ void quality_reads(const uint8_t *__restrict__ qual, const uint64_t *__restrict__ off,
                                              uint64_t n, int k, uint32_t T, int64_t mrq, uint32_t flags,
                                              uint4 *__restrict__ qmask, uint8_t *__restrict__ qdrop) {
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t o = off[r], L64 = off[r + 1] - o;
        uint4 m = make_uint4(0, 0, 0, 0);
        uint8_t d = 0;
        if (L64 <= 4u * kQmDwords) {
            quality_read<KQ>(qual, o, (uint32_t)L64, k, T, mrq, flags, m, d);
        } else if (flags & 1u) {  // a longer read (the 250-bp lane shape): its mean test only
            uint64_t tot = 0;
            for (uint64_t i = 0; i < L64; i++) tot += qual[o + i];
            d = (int64_t)tot < mrq * (int64_t)L64 ? 1 : 0;
        }
        qmask[r] = m;
        qdrop[r] = d;
    }
}

// LONG: k > 63 (three-word keys), a kernel of its own so that the longer
// realignments do not raise the registers of the k <= 63 one
template <bool LONG = false>
__global__ __launch_bounds__(256) void k_quality_masks(const uint8_t *__restrict__ qual, const uint64_t *__restrict__ off,
                                                       uint64_t n, int k, int64_t mrq, int64_t mkq, uint32_t flags,
                                                       uint4 *__restrict__ qmask, uint8_t *__restrict__ qdrop) {
    const int64_t T64 = mkq * (int64_t)k;
    const uint32_t T = T64 <= 0 ? 0u : (T64 > (1 << 24) ? (1u << 24) : (uint32_t)T64);
    if (LONG) {
        switch (k >> 2) {
            case 16: quality_reads<16>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
            case 17: quality_reads<17>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
            case 18: quality_reads<18>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
            case 19: quality_reads<19>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
            case 20: quality_reads<20>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
            case 21: quality_reads<21>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
            case 22: quality_reads<22>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
            case 23: quality_reads<23>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
            default: break;  // (unreachable: 63 < k <= 95)
        }
        return;
    }
    switch (k >> 2) {  // (k <= 63 here; uniform)
        case 0: quality_reads<0>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
        case 1: quality_reads<1>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
        case 2: quality_reads<2>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
        case 3: quality_reads<3>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
        case 4: quality_reads<4>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
        case 5: quality_reads<5>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
        case 6: quality_reads<6>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
        case 7: quality_reads<7>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
        case 8: quality_reads<8>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
        case 9: quality_reads<9>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
        case 10: quality_reads<10>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
        case 11: quality_reads<11>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
        case 12: quality_reads<12>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
        case 13: quality_reads<13>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
        case 14: quality_reads<14>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
        case 15: quality_reads<15>(qual, off, n, k, T, mrq, flags, qmask, qdrop); break;
        default: break;  // (unreachable: k > 63 takes the LONG kernel)
    }
}

#include "pa_lane.h"

// Plane of the windows whose genome set is larger than mg (--max-genomes,
// src/kmer.py:425-427), bit i of word j <-> position 64 j + i, from tile_cls
// and the set records: the lane walk then tests a walked window with one bit.
// Made once per (index, mg) and cached in the index.
__global__ __launch_bounds__(256) void k_tile_big(const uint32_t *__restrict__ tile_cls, uint64_t n, uint32_t G,
                                                  const uint32_t *__restrict__ class_genomes, int32_t mg,
                                                  uint64_t *__restrict__ big, uint64_t n_words) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t j = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); j < n_words; j += nw) {
        const uint64_t t = 64 * j + lane;
        const uint32_t v = t < n ? tile_cls[t] : NONE;
        const bool ok = v != NONE && (int64_t)class_size_of(v & ~PA_TILE_REP, G, class_genomes) > (int64_t)mg;
        const uint64_t b = __ballot(ok);
        if (lane == 0) big[j] = b;
    }
}


// tile_nb's 64-bit words and tile_nbbig's 32-bit ones interleaved as one 16-B
// record per (position, substitution), for the walks under --max-genomes: a
// mismatch then costs the walk one line instead of one in each array.
__global__ __launch_bounds__(256) void k_nb_merge(const uint64_t *__restrict__ nb, const uint32_t *__restrict__ nbbig,
                                                  uint64_t n_words, uint4 *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_words; i += stride) {
        const uint64_t v = nb[i];
        out[i] = make_uint4((uint32_t)v, (uint32_t)(v >> 32), nbbig[i], 0u);
    }
}

// The neighbour bits' "set size > mg" half for one --max-genomes value mg >= 2
// (cached in the index like tile_big): bit i of nbbig[3 p + b] is set when the
// one-substitution neighbour of tile_nb's word 3 p + b, bit i, is present with
// more than mg genomes.  Only present, multi-genome neighbours are probed --
// one thread per word, most words are zero.
__global__ __launch_bounds__(256) void k_nb_big(const uint64_t *__restrict__ pk, const uint64_t *__restrict__ nb,
                                                uint64_t n_words, int k, const Slot<1> *__restrict__ table, HomeCfg hc,
                                                uint32_t G, const uint32_t *__restrict__ class_genomes, int32_t mg,
                                                uint32_t *__restrict__ nbbig) {
    const int sh = 64 - 2 * k;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_words; i += stride) {
        const uint64_t v = nb[i];
        uint32_t cand = (uint32_t)v & ~(uint32_t)(v >> 32);  // present, not specific (size 1 <= mg)
        uint32_t big = 0;
        const uint64_t p = i / 3;
        const uint32_t b = (uint32_t)(i - 3 * p);
        while (cand) {
            const uint32_t q = __builtin_ctz(cand);
            cand &= cand - 1;
            const uint64_t w = p - (uint64_t)(k - 1) + q;  // the window (bit q of the word)
            const uint64_t K = get64_at(pk, 2 * w) >> sh;
            const int bs = 2 * (k - 1 - (int)(p - w));
            const uint64_t cj = (K >> bs) & 3;
            uint64_t key[1] = {K ^ ((cj ^ ((cj + 1 + b) & 3)) << bs)};
            uint32_t cls[1];
            if (probe_lines<1>(table, hc, key, cls) && (int64_t)class_size_of(cls[0], G, class_genomes) > (int64_t)mg)
                big |= 1u << q;
        }
        nbbig[i] = big;
    }
}

// ---------------------------------------------------------------------------
// exact kernel (one workgroup per read, dense per-genome scratch)
// ---------------------------------------------------------------------------

struct ExactArgs {
    AlignArgs a;
    int detail;           // 0: counters; 1: per-read type/qf/hr/list length; 2: also write lists
    uint8_t *type_out;
    uint32_t *qf_out, *hr_out, *len_out;
    const uint64_t *list_off;
    uint32_t *lists;
    unsigned char *ws;    // per-workgroup scratch
    uint64_t ws_stride;
    uint32_t wcap;        // windows capacity
    uint32_t dh;          // dedup hash size (power of two >= 2*wcap)
    int use_queue;
};

struct ExactWs {
    uint64_t *wslot;
    uint32_t *wcls;
    uint64_t *dh_key;
    uint32_t *dh_min;
    uint32_t *ch_key, *ch_cnt, *ch_min;  // distinct multi-genome sets of the read: id, k-mers, first window
    uint32_t *cls_list;                  // their hash positions, in insertion order
    uint32_t *g_spec, *g_specmin, *g_tot, *g_totmin, *touched;
};

__host__ __device__ inline uint64_t exact_ws_stride(uint32_t wcap, uint32_t dh, uint32_t G) {
    uint64_t b = (uint64_t)wcap * 8 + (uint64_t)dh * 8 + (uint64_t)wcap * 4 + (uint64_t)dh * 4 + (uint64_t)dh * 12 +
                 (uint64_t)wcap * 4 + (uint64_t)G * 20;
    return (b + 255) / 256 * 256;
}

__device__ inline ExactWs exact_ws(unsigned char *base, uint32_t wcap, uint32_t dh, uint32_t G) {
    ExactWs w;
    w.wslot = (uint64_t *)base;
    w.dh_key = w.wslot + wcap;
    w.wcls = (uint32_t *)(w.dh_key + dh);
    w.dh_min = w.wcls + wcap;
    w.ch_key = w.dh_min + dh;
    w.ch_cnt = w.ch_key + dh;
    w.ch_min = w.ch_cnt + dh;
    w.cls_list = w.ch_min + dh;
    w.g_spec = w.cls_list + wcap;
    w.g_specmin = w.g_spec + G;
    w.g_tot = w.g_specmin + G;
    w.g_totmin = w.g_tot + G;
    w.touched = w.g_totmin + G;
    return w;
}

__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t *red) {
    v = wave_sum(v);
    __syncthreads();
    if (lane_id() == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    uint32_t s = 0;
    for (int i = 0; i < kWaves; i++) s += red[i];
    __syncthreads();
    return s;
}

__device__ __forceinline__ uint64_t block_sum64(uint64_t v, unsigned long long *red) {
    v = wave_sum64(v);
    __syncthreads();
    if (lane_id() == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    uint64_t s = 0;
    for (int i = 0; i < kWaves; i++) s += red[i];
    __syncthreads();
    return s;
}

__device__ __forceinline__ uint32_t block_max(uint32_t v, uint32_t *red) {
    v = wave_max(v);
    __syncthreads();
    if (lane_id() == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    uint32_t s = 0;
    for (int i = 0; i < kWaves; i++) s = max(s, red[i]);
    __syncthreads();
    return s;
}

constexpr uint32_t kRankLds = 2048;  // genomes of a read's list ranked in LDS (16 KB); more: over the scratch
template <int NW>
__global__ __launch_bounds__(kBlock) void k_align_exact(ExactArgs x) {
    const AlignArgs &a = x.a;
    __shared__ uint32_t red[kWaves];
    __shared__ unsigned long long red64[kWaves];
    __shared__ uint32_t n_touched, n_cls, n_rank;
    __shared__ uint64_t rank_key[kRankLds];  // the listed genomes' order keys (ranks of genomes_mapped_to)
    const uint32_t G = a.G;
    const int k = a.k;
    const uint64_t mask0 = k > 0 ? mask0_of(k, NW) : 0;
    const Slot<NW> *table = (const Slot<NW> *)a.table;
    const bool has_mrq = a.prm.flags & F_MRQ, has_mkq = a.prm.flags & F_MKQ, has_mg = a.prm.flags & F_MG;
    ExactWs ws = exact_ws(x.ws + (uint64_t)blockIdx.x * x.ws_stride, x.wcap, x.dh, G);
    // scratch invariant: g_* clean (0 / NONE) between reads
    for (uint32_t g = threadIdx.x; g < G; g += kBlock) {
        st_agent(&ws.g_spec[g], 0u);
        st_agent(&ws.g_specmin[g], NONE);
        st_agent(&ws.g_tot[g], 0u);
        st_agent(&ws.g_totmin[g], NONE);
    }
    if (threadIdx.x == 0) n_touched = n_cls = 0;
    __syncthreads();
    const uint64_t nq = x.use_queue ? *a.qcount : a.n;
    if (blockIdx.x == 0 && threadIdx.x == 0 && x.use_queue && a.deferred_total) atomicAdd(a.deferred_total, nq);
    for (uint64_t q = blockIdx.x; q < nq; q += gridDim.x) {
        const uint64_t r = x.use_queue ? a.queue[q] : q;
        const uint64_t off = a.off[r];
        const uint32_t len = (uint32_t)(a.off[r + 1] - off);
        const uint32_t W = (k > 0 && len >= (uint32_t)k) ? len - k + 1 : 0;
        const uint64_t read_idx = a.base + r;
        // ---- mean read quality
        if (has_mrq) {
            uint64_t s = 0;
            for (uint32_t i = threadIdx.x; i < len; i += kBlock) s += a.qual[off + i];
            s = block_sum64(s, red64);
            if ((int64_t)s < (int64_t)a.prm.mrq * (int64_t)len) {
                if (threadIdx.x == 0) {
                    if (x.detail) {
                        x.type_out[r] = PA_DROPPED;
                        x.qf_out[r] = 0;
                        x.hr_out[r] = 0;
                        x.len_out[r] = 0;
                    } else {
                        atomicAdd(&a.stats[3], 1ull);
                    }
                }
                continue;
            }
        }
        for (uint32_t i = threadIdx.x; i < x.dh; i += kBlock) {
            st_agent(&ws.dh_key[i], EMPTY);
            st_agent(&ws.dh_min[i], NONE);
            st_agent(&ws.ch_key[i], NONE);
            st_agent(&ws.ch_cnt[i], 0u);
            st_agent(&ws.ch_min[i], NONE);
        }
        __syncthreads();
        // ---- windows
        uint32_t qf = 0, hr = 0, any = 0;
        for (uint32_t w = threadIdx.x; w < W; w += kBlock) {
            ws.wslot[w] = EMPTY;
            if (has_mkq) {
                uint32_t s = 0;
                for (int i = 0; i < k; i++) s += a.qual[off + w + i];
                if ((int64_t)s < (int64_t)a.prm.mkq * k) {
                    qf++;
                    continue;
                }
            }
            Key<NW> key;
#pragma unroll
            for (int j = 0; j < NW; j++) key.w[j] = 0;
            bool clean = true;
            for (int i = 0; i < k; i++) {
                uint32_t c = base_code(a.seq[off + w + i]);
                clean &= c < 4;
                key_push(key, c & 3, mask0);
            }
            if (!clean) continue;
            uint64_t slot;
            uint32_t cls, tpos;
            if (!table_find<NW, true>(table, a.cap, key, home_of(key, key_hash(key), a.home), slot, cls, tpos)) continue;
            if (has_mg && (int64_t)class_size_of(cls, G, a.class_genomes) > (int64_t)a.prm.mg) {
                hr++;
                continue;
            }
            ws.wslot[w] = slot;
            ws.wcls[w] = cls_of(cls);
            any = 1;
            uint32_t p = (uint32_t)(fmix64(slot) & (x.dh - 1));
            for (;;) {
                uint64_t old = atomicCAS((unsigned long long *)&ws.dh_key[p], (unsigned long long)EMPTY,
                                         (unsigned long long)slot);
                if (old == EMPTY || old == slot) break;
                p = (p + 1) & (x.dh - 1);
            }
            atomicMin(&ws.dh_min[p], w);
        }
        qf = block_sum(qf, red);
        hr = block_sum(hr, red);
        any = block_sum(any, red);
        uint8_t type = PA_UNMAPPED;
        uint32_t list_len = 0;
        if (any) {
            // ---- distinct k-mers -> specific and total counts per genome.  A
            // specific k-mer counts for its genome directly; the others are first
            // grouped by genome set (a read's k-mers fall in a handful of sets, e.g.
            // one set of every genome for a conserved stretch), and every set then
            // adds its k-mer count and first window to its genomes once, the
            // block striding over the set's genome list.
            for (uint32_t w = threadIdx.x; w < W; w += kBlock) {
                const uint64_t slot = ws.wslot[w];
                if (slot == EMPTY) continue;
                uint32_t p = (uint32_t)(fmix64(slot) & (x.dh - 1));
                while (ld_agent(&ws.dh_key[p]) != slot) p = (p + 1) & (x.dh - 1);
                if (ld_agent(&ws.dh_min[p]) != w) continue;
                const uint32_t c = ws.wcls[w];
                if (c < G) {
                    atomicAdd(&ws.g_spec[c], 1u);
                    atomicMin(&ws.g_specmin[c], w);
                    if (atomicAdd(&ws.g_tot[c], 1u) == 0) ws.touched[atomicAdd(&n_touched, 1u)] = c;
                    atomicMin(&ws.g_totmin[c], w);
                } else {
                    uint32_t q = (uint32_t)(fmix64(c) & (x.dh - 1));
                    for (;;) {
                        const uint32_t old = atomicCAS(&ws.ch_key[q], NONE, c);
                        if (old == NONE) {
                            ws.cls_list[atomicAdd(&n_cls, 1u)] = q;
                            break;
                        }
                        if (old == c) break;
                        q = (q + 1) & (x.dh - 1);
                    }
                    atomicAdd(&ws.ch_cnt[q], 1u);
                    atomicMin(&ws.ch_min[q], w);
                }
            }
            __syncthreads();
            const uint32_t ncl = n_cls;
            for (uint32_t i = 0; i < ncl; i++) {
                const uint32_t q = ld_agent(&ws.cls_list[i]);
                const uint32_t c = ld_agent(&ws.ch_key[q]), cnt = ld_agent(&ws.ch_cnt[q]), mw = ld_agent(&ws.ch_min[q]);
                const uint32_t *rec = a.class_genomes + (c - G);  // [size, genomes...]
                const uint32_t sz = rec[0];
                for (uint32_t j = threadIdx.x; j < sz; j += kBlock) {
                    const uint32_t g = rec[1 + j];
                    if (atomicAdd(&ws.g_tot[g], cnt) == 0) ws.touched[atomicAdd(&n_touched, 1u)] = g;
                    atomicMin(&ws.g_totmin[g], mw);
                }
            }
            __syncthreads();
            const uint32_t nt = n_touched;
            // ---- decision (src/kmer.py:444-480)
            uint32_t nspec = 0, maxcnt = 0;
            for (uint32_t t = threadIdx.x; t < nt; t += kBlock) {
                uint32_t c = ld_agent(&ws.g_spec[ws.touched[t]]);
                nspec += c > 0;
                maxcnt = max(maxcnt, c);
            }
            nspec = block_sum(nspec, red);
            maxcnt = block_max(maxcnt, red);
            type = PA_AMBIGUOUSLY_MAPPED;
            uint32_t gstar = NONE;
            bool unique = false, demote = false;
            uint32_t tstar = 0;
            if (nspec > 0) {
                // top = first-inserted genome among those with the max count
                uint32_t best = 0;  // encodes (NONE - first window) to take a max
                for (uint32_t t = threadIdx.x; t < nt; t += kBlock) {
                    uint32_t g = ws.touched[t];
                    if (ld_agent(&ws.g_spec[g]) == maxcnt) best = max(best, NONE - ld_agent(&ws.g_specmin[g]));
                }
                best = block_max(best, red);
                uint32_t sec = 0, gs = 0;
                for (uint32_t t = threadIdx.x; t < nt; t += kBlock) {
                    uint32_t g = ws.touched[t];
                    uint32_t c = ld_agent(&ws.g_spec[g]);
                    if (c == maxcnt && NONE - ld_agent(&ws.g_specmin[g]) == best)
                        gs = g + 1;
                    else
                        sec = max(sec, c);
                }
                gstar = block_max(gs, red) - 1;
                sec = block_max(sec, red);
                unique = nspec == 1 || (int64_t)maxcnt >= (int64_t)sec + a.prm.m;
                if (unique && a.prm.p >= 0) {
                    tstar = ld_agent(&ws.g_tot[gstar]);
                    uint32_t mx = 0;
                    for (uint32_t t = threadIdx.x; t < nt; t += kBlock)
                        mx = max(mx, ld_agent(&ws.g_tot[ws.touched[t]]));
                    mx = block_max(mx, red);
                    demote = (int64_t)mx - (int64_t)tstar > a.prm.p;
                }
            }
            // ---- emit genomes_mapped_to with list positions
            if (unique && !demote) {
                type = PA_UNIQUELY_MAPPED;
                list_len = 1;
                if (threadIdx.x == 0) {
                    if (x.detail == 2) x.lists[x.list_off[r]] = gstar;
                    if (!x.detail) {
                        atomicAdd(&a.uniq[gstar], 1ull);
                        atomicMin(&a.first[gstar], (unsigned long long)first_key(read_idx, 0));
                    }
                }
            } else if (unique && demote) {
                // the listed genomes' order keys (first window << 32 | genome)
                // staged in LDS once, so that each one's rank is counted over
                // LDS rather than over the scratch in global memory (2 nt loads
                // per genome: ~1 ms for the reads of C5's families)
                if (threadIdx.x == 0) n_rank = 0;
                __syncthreads();
                uint32_t nq = 0;
                for (uint32_t t = threadIdx.x; t < nt; t += kBlock) {
                    const uint32_t g = ws.touched[t];
                    if (ld_agent(&ws.g_tot[g]) < tstar) continue;
                    nq++;
                    const uint32_t i = atomicAdd(&n_rank, 1u);
                    if (i < kRankLds) rank_key[i] = ((uint64_t)ld_agent(&ws.g_totmin[g]) << 32) | g;
                }
                nq = block_sum(nq, red);  // (its barriers also publish rank_key)
                list_len = 1 + nq;
                for (uint32_t t = threadIdx.x; t < nt; t += kBlock) {
                    const uint32_t g = ws.touched[t];
                    const uint32_t tg = ld_agent(&ws.g_tot[g]);
                    if (tg < tstar) continue;
                    const uint64_t me = ((uint64_t)ld_agent(&ws.g_totmin[g]) << 32) | g;
                    uint32_t rank = 1;
                    if (nq <= kRankLds) {
                        for (uint32_t u = 0; u < nq; u++) rank += rank_key[u] < me;
                    } else {
                        for (uint32_t u = 0; u < nt; u++) {
                            const uint32_t h = ws.touched[u];
                            if (ld_agent(&ws.g_tot[h]) >= tstar &&
                                (((uint64_t)ld_agent(&ws.g_totmin[h]) << 32) | h) < me)
                                rank++;
                        }
                    }
                    if (x.detail == 2) x.lists[x.list_off[r] + rank] = g;
                    if (!x.detail) {
                        atomicAdd(&a.amb[g], g == gstar ? 2ull : 1ull);
                        atomicMin(&a.first[g], (unsigned long long)first_key(read_idx, g == gstar ? 0 : rank));
                    }
                }
                if (threadIdx.x == 0 && x.detail == 2) x.lists[x.list_off[r]] = gstar;
            } else if (nspec > 0) {
                list_len = nspec;
                // (the genomes with specific k-mers: their first windows staged in LDS, as above)
                if (threadIdx.x == 0) n_rank = 0;
                __syncthreads();
                for (uint32_t t = threadIdx.x; t < nt; t += kBlock) {
                    const uint32_t g = ws.touched[t];
                    if (ld_agent(&ws.g_spec[g]) == 0) continue;
                    const uint32_t i = atomicAdd(&n_rank, 1u);
                    if (i < kRankLds) rank_key[i] = ld_agent(&ws.g_specmin[g]);
                }
                __syncthreads();
                for (uint32_t t = threadIdx.x; t < nt; t += kBlock) {
                    const uint32_t g = ws.touched[t];
                    if (ld_agent(&ws.g_spec[g]) == 0) continue;
                    const uint32_t mw = ld_agent(&ws.g_specmin[g]);
                    uint32_t rank = 0;
                    if (nspec <= kRankLds) {
                        for (uint32_t u = 0; u < nspec; u++) rank += rank_key[u] < mw;
                    } else {
                        for (uint32_t u = 0; u < nt; u++) {
                            const uint32_t h = ws.touched[u];
                            if (ld_agent(&ws.g_spec[h]) > 0 && ld_agent(&ws.g_specmin[h]) < mw) rank++;
                        }
                    }
                    if (x.detail == 2) x.lists[x.list_off[r] + rank] = g;
                    if (!x.detail) {
                        atomicAdd(&a.amb[g], 1ull);
                        atomicMin(&a.first[g], (unsigned long long)first_key(read_idx, rank));
                    }
                }
            }
            __syncthreads();
            // ---- restore the scratch invariant
            for (uint32_t t = threadIdx.x; t < nt; t += kBlock) {
                const uint32_t g = ws.touched[t];
                st_agent(&ws.g_spec[g], 0u);
                st_agent(&ws.g_specmin[g], NONE);
                st_agent(&ws.g_tot[g], 0u);
                st_agent(&ws.g_totmin[g], NONE);
            }
            __syncthreads();
            if (threadIdx.x == 0) n_touched = n_cls = 0;
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            if (x.detail) {
                x.type_out[r] = type;
                x.qf_out[r] = qf;
                x.hr_out[r] = hr;
                x.len_out[r] = list_len;
            } else {
                atomicAdd(&a.stats[type == PA_UNMAPPED ? 2 : (type == PA_UNIQUELY_MAPPED ? 0 : 1)], 1ull);
                if (has_mkq && qf) atomicAdd(&a.stats[4], (unsigned long long)qf);
                if (has_mg && hr) atomicAdd(&a.stats[5], (unsigned long long)hr);
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------

size_t fast_lds_bytes(uint32_t G, int wpl, bool need_q) {
    size_t cnt = G <= kLdsGenomeCap ? (((size_t)((G + 1) & ~1u) * 16 + 15) / 16 * 16) : 0;
    size_t wl = wpl == 1 ? fast_wave_bytes<1>(need_q) : wpl == 2 ? fast_wave_bytes<2>(need_q) : fast_wave_bytes<4>(need_q);
    return cnt + kWaves * wl;
}

template <int NW, int WPL, bool DENSE>
pa_status launch_fast(const AlignArgs &a, size_t shm, hipStream_t st) {
    auto kern = k_align_fast<NW, WPL, DENSE>;
    if (shm > 64 * 1024) PA_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    int per_cu = 0;
    PA_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kBlock, shm));
    int dev = 0, cus = 256;
    PA_HIP(hipGetDevice(&dev));
    PA_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    uint64_t want = (a.n + kWaves - 1) / kWaves;
    uint64_t resident = (uint64_t)std::max(1, per_cu) * (uint64_t)cus;
    unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(want, resident));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), shm, st, a);
    PA_HIP(hipGetLastError());
    return PA_OK;
}

// Per-kernel profile events (pa_profile_read_kernels): a pair around one
// launch on its stream while the index's profiling is on.
struct KernelTimer {
    pa_index *idx;
    hipStream_t st;
    int slot;
    hipEvent_t e0 = nullptr;
    KernelTimer(pa_index *i, hipStream_t s, int sl) : idx(i), st(s), slot(sl) {
        if (idx && idx->profile && hipEventCreate(&e0) == hipSuccess) hipEventRecord(e0, st);
    }
    ~KernelTimer() {
        hipEvent_t e1 = nullptr;
        if (e0 && hipEventCreate(&e1) == hipSuccess && hipEventRecord(e1, st) == hipSuccess)
            idx->kev.push_back({slot, e0, e1});
        else if (e0)
            hipEventDestroy(e0);
    }
};

// long_reads: the batch holds reads longer than the 150-bp shape takes (176
// bases): the 250-bp shape (NM = 4, <= 272 bases, <= 256 windows) walks them,
// unless --min-kmer-quality is set (its window masks cover 128 windows: such
// reads then go to the wave kernel).
// nw: key words (2: 31 < k <= 63, 3: 63 < k <= 95 -- the 150-bp shape, no
// reverse-strand path: reads without a seed go to the wave kernel).
constexpr uint64_t kRcnbMinReads = 32768;  // seedless reads in a pass that make the reverse-complement bits worth it
pa_status launch_lane(const AlignArgs &a0, hipStream_t st, pa_index *prof = nullptr, bool long_reads = false,
                      int nw = 1) {
    const bool need_q = (a0.prm.flags & (F_MRQ | F_MKQ)) != 0;
    const bool win_q = (a0.prm.flags & F_MKQ) != 0;
    const bool mg = (a0.prm.flags & F_MG) != 0;
    const bool nm4 = long_reads && !win_q && nw == 1;
    AlignArgs a = a0;
    const size_t shm = lane_lds_bytes(a.G, nm4 ? 4 : 2);
    auto kern = nw == 3
                    ? (win_q ? (mg ? k_align_lane<true, true, true, 2, 3> : k_align_lane<true, true, false, 2, 3>)
                       : need_q ? (mg ? k_align_lane<true, false, true, 2, 3> : k_align_lane<true, false, false, 2, 3>)
                                : (mg ? k_align_lane<false, false, true, 2, 3> : k_align_lane<false, false, false, 2, 3>))
              : nw == 2
                    ? (win_q ? (mg ? k_align_lane<true, true, true, 2, 2> : k_align_lane<true, true, false, 2, 2>)
                       : need_q ? (mg ? k_align_lane<true, false, true, 2, 2> : k_align_lane<true, false, false, 2, 2>)
                                : (mg ? k_align_lane<false, false, true, 2, 2> : k_align_lane<false, false, false, 2, 2>))
              : nm4 ? (need_q ? (mg ? k_align_lane<true, false, true, 4> : k_align_lane<true, false, false, 4>)
                              : (mg ? k_align_lane<false, false, true, 4> : k_align_lane<false, false, false, 4>))
              : win_q ? (mg ? k_align_lane<true, true, true> : k_align_lane<true, true, false>)
              : need_q ? (mg ? k_align_lane<true, false, true> : k_align_lane<true, false, false>)
                       : (mg ? k_align_lane<false, false, true> : k_align_lane<false, false, false>);
    if (shm > 64 * 1024) PA_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    int per_cu = 0, dev = 0, cus = 256;
    PA_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kBlock, shm));
    PA_HIP(hipGetDevice(&dev));
    PA_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const uint64_t want = (a.n + kBlock - 1) / kBlock;
    const uint64_t resident = (uint64_t)std::max(1, per_cu) * (uint64_t)cus;
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(want, resident));
    // the seedless reads for k_rc_seeds in per-wave queue segments: one
    // atomic per wave and chunk on the queue's counter serialised, and cost
    // c2rc (half its reads seedless) 0.27 ms per 10 M reads (PA_NA_SEG=0: the
    // flat queue, A/B)
    {
        const char *e = std::getenv("PA_NA_SEG");
        const uint64_t waves = (uint64_t)grid * kWaves, chunks = (a.n + 63) / 64;
        a.nseg = (uint32_t)waves;
        a.seg_cap = 64 * ((chunks + waves - 1) / waves);
        a.na_seg = a.queue_na && a.queue_na_keys && a.seg_cnt && !nm4 && nw == 1 && waves <= kSegMaxWaves &&
                   waves * a.seg_cap <= a.queue_cap && !(e && e[0] == '0');
    }
    {
        KernelTimer kt(prof, st, PA_PROF_LANE);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), shm, st, a);
        PA_HIP(hipGetLastError());
    }
    if (a.queue_na) {  // the reads without a seed in the index (count on the device)
        AlignArgs b = a;
        // the reverse-complement neighbour bits, left out by the build
        // (build_nb), are made by the first pass that queues enough seedless
        // reads; passes that queue too few look twice, then stop looking (the
        // reverse-strand walk runs without them, exactly, only slower)
        if (prof && prof->rcnb_pending && a.queue_na_keys) {
            unsigned long long c = 0;
            PA_HIP(hipMemcpyAsync(&c, a.queue_na_count, 8, hipMemcpyDeviceToHost, st));
            PA_HIP(hipStreamSynchronize(st));
            if (c >= std::max<uint64_t>(kRcnbMinReads, a.n / 64)) {
                PA_TRY(pa::index_build_rcnb(prof, st));
                const char *e = std::getenv("PA_NA_RCNB");
                if (!(e && e[0] == '0')) b.tile_rcnb = prof->tile_rcnb;
            } else if (++prof->rcnb_checks >= 2) {
                prof->rcnb_pending = 0;
            }
        }
        if (a.queue_na_keys) {  // reverse-complement seeds, the reverse-strand walk; the rest on to k_align_lane_na
            {
                KernelTimer kt(prof, st, PA_PROF_RC_SEEDS);
                const unsigned sgrid = a.na_seg ? (a.nseg + kSegGroup - 1) / kSegGroup  // (a group of segments per block)
                                                : (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(
                                                      (a.n + kBlock * 4 - 1) / (kBlock * 4), 8192));
                hipLaunchKernelGGL(k_rc_seeds, dim3(sgrid), dim3(kBlock), 0, st, b);
                PA_HIP(hipGetLastError());
            }
            auto rc = win_q ? (mg ? k_align_lane_rc<true, true, true> : k_align_lane_rc<true, true, false>)
                    : need_q ? (mg ? k_align_lane_rc<true, false, true> : k_align_lane_rc<true, false, false>)
                             : (mg ? k_align_lane_rc<false, false, true> : k_align_lane_rc<false, false, false>);
            int rc_cu = 0;
            PA_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&rc_cu, rc, kBlock, 0));
            const unsigned rgrid = (unsigned)std::max<uint64_t>(
                1, std::min<uint64_t>(want, (uint64_t)std::max(1, rc_cu) * (uint64_t)cus));
            KernelTimer kt(prof, st, PA_PROF_LANE_RC);
            hipLaunchKernelGGL(rc, dim3(rgrid), dim3(kBlock), 0, st, b);
            PA_HIP(hipGetLastError());
            b.queue_na = a.queue_na2;
            b.queue_na_count = a.queue_na2_count;
        }
        auto na = nw == 3 ? (win_q ? (mg ? k_align_lane_naw<true, true, true, 3> : k_align_lane_naw<true, true, false, 3>)
                             : need_q ? (mg ? k_align_lane_naw<true, false, true, 3> : k_align_lane_naw<true, false, false, 3>)
                                      : (mg ? k_align_lane_naw<false, false, true, 3> : k_align_lane_naw<false, false, false, 3>))
                : nw == 2 ? (win_q ? (mg ? k_align_lane_naw<true, true, true, 2> : k_align_lane_naw<true, true, false, 2>)
                             : need_q ? (mg ? k_align_lane_naw<true, false, true, 2> : k_align_lane_naw<true, false, false, 2>)
                                      : (mg ? k_align_lane_naw<false, false, true, 2> : k_align_lane_naw<false, false, false, 2>))
                : win_q ? (mg ? k_align_lane_na<true, true, true> : k_align_lane_na<true, true, false>)
                : need_q ? (mg ? k_align_lane_na<true, false, true> : k_align_lane_na<true, false, false>)
                         : (mg ? k_align_lane_na<false, false, true> : k_align_lane_na<false, false, false>);
        int na_cu = 0;
        PA_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&na_cu, na, kBlock, 0));
        const unsigned ngrid = (unsigned)std::max<uint64_t>(
            1, std::min<uint64_t>(want, (uint64_t)std::max(1, na_cu) * (uint64_t)cus));
        KernelTimer kt(prof, st, PA_PROF_LANE_NA);
        hipLaunchKernelGGL(na, dim3(ngrid), dim3(kBlock), 0, st, b);
        PA_HIP(hipGetLastError());
    }
    return PA_OK;
}

template <int NW>
pa_status launch_fast_wpl(const AlignArgs &a, int wpl, hipStream_t st) {
    size_t shm = fast_lds_bytes(a.G, wpl, (a.prm.flags & (F_MRQ | F_MKQ)) != 0);
    const bool dense = a.G <= 64;  // membership masks exist (k_class_masks)
    switch (wpl) {
        case 1: return dense ? launch_fast<NW, 1, true>(a, shm, st) : launch_fast<NW, 1, false>(a, shm, st);
        case 2: return dense ? launch_fast<NW, 2, true>(a, shm, st) : launch_fast<NW, 2, false>(a, shm, st);
        default: return dense ? launch_fast<NW, 4, true>(a, shm, st) : launch_fast<NW, 4, false>(a, shm, st);
    }
}

template <int NW>
void launch_exact(const ExactArgs &x, unsigned grid, hipStream_t st) {
    hipLaunchKernelGGL(k_align_exact<NW>, dim3(grid), dim3(kBlock), 0, st, x);
}

void launch_exact_nw(int nw, const ExactArgs &x, unsigned grid, hipStream_t st) {
    switch (nw) {
        case 1: launch_exact<1>(x, grid, st); break;
        case 2: launch_exact<2>(x, grid, st); break;
        case 3: launch_exact<3>(x, grid, st); break;
        case 4: launch_exact<4>(x, grid, st); break;
        case 5: launch_exact<5>(x, grid, st); break;
        case 6: launch_exact<6>(x, grid, st); break;
        case 7: launch_exact<7>(x, grid, st); break;
        default: launch_exact<8>(x, grid, st); break;
    }
}

constexpr unsigned kExactGrid = 512;

AlignArgs make_args(const pa_index *idx, const pa_reads *r, const pa::DevParams &p, uint64_t base) {
    AlignArgs a{};
    a.table = idx->table;
    a.cap = idx->cap;
    a.home = idx->home;
    a.G = idx->n_genomes;
    a.k = (int)std::max<int64_t>(idx->k, 0);
    a.class_genomes = idx->class_genomes;
    a.class_mask = idx->class_mask;
    a.tile_cls = idx->tile_cls;
    a.tile_pk = idx->tile_pk;
    a.goff = idx->goff;
    a.tile_lw = idx->tile_cls ? idx->tile_lw : nullptr;
    a.tile_nb = idx->tile_cls ? idx->tile_nb : nullptr;
    a.nb_spec = idx->nb_spec;
    a.nb_split = idx->tile_nb1 ? idx->nb_split : ~0ull;
    a.nb_base1 = idx->tile_nb1 ? (uint64_t)(uintptr_t)idx->tile_nb1 - idx->nb_split * (idx->nb_spec ? 8 : 4) : 0;
    a.nbbig_ld = (const uint32_t *)(a.tile_nb ? a.tile_nb : (const void *)a.tile_lw);  // (a valid word 0 either way)
    a.nbbig_mask = 0;
    a.gblk = idx->tile_gblk;
    a.bloom = idx->tile_cls ? idx->bloom : nullptr;
    a.bloom_lg = idx->bloom_lg;
    a.tile_rcp = idx->tile_cls ? idx->tile_rcp : nullptr;
    a.mm_bits = idx->tile_cls ? idx->mm_bits : nullptr;
    a.mm_lg = idx->mm_lg;
    if (const char *e = std::getenv("PA_MM_BITS")) if (e[0] == '0') a.mm_bits = nullptr;
    a.tile_rcnb = idx->tile_cls ? idx->tile_rcnb : nullptr;
    if (const char *e = std::getenv("PA_NA_RCNB")) if (e[0] == '0') a.tile_rcnb = nullptr;
    if (const char *e = std::getenv("PA_NA_RCWALK")) if (e[0] == '0') a.tile_rcp = nullptr;
    a.tile_n = idx->tile_cls ? idx->tile_n : 0;
    a.walk_rounds = 1;
    a.tpos_local = idx->tpos_local;
    a.lane_maxpend = 96;
    if (const char *e = std::getenv("PA_LANE_MAXPEND")) a.lane_maxpend = (uint32_t)std::atoi(e);
    a.lane_noanchor = a.bloom != nullptr;  // (without the filter every window costs a table line)
    if (const char *e = std::getenv("PA_LANE_NOANCHOR")) a.lane_noanchor = e[0] == '1';
    if (const char *e = std::getenv("PA_WALK_ROUNDS")) a.walk_rounds = std::atoi(e);
    if (const char *e = std::getenv("PA_DBG_MODE")) a.dbg_mode = std::atoi(e);
    a.seq = r->seq;
    a.qual = r->qual;
    a.off = r->off;
    a.n = r->n;
    a.base = base;
    a.prm = p;
    return a;
}

pa_status prepare_exact(pa_index *idx, const pa_reads *r, ExactArgs &x, unsigned &grid) {
    const uint32_t wcap = std::max<uint32_t>(1, r->max_len);
    uint32_t dh = 64;
    while (dh < 2 * wcap) dh <<= 1;
    const uint64_t stride = exact_ws_stride(wcap, dh, idx->n_genomes);
    grid = kExactGrid;
    while (grid > 16 && (uint64_t)grid * stride > (1ull << 31)) grid >>= 1;
    PA_TRY(pa::ensure_workspace(idx, (size_t)grid * stride));
    x.ws = (unsigned char *)idx->ws.ptr;
    x.ws_stride = stride;
    x.wcap = wcap;
    x.dh = dh;
    return PA_OK;
}

__global__ void k_fill_first(unsigned long long *p, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = (unsigned long long)PA_NO_FIRST_KEY;
}

}  // namespace

namespace pa {

pa_status result_reset(pa_result *res, hipStream_t st) {
    const uint64_t G = res->n_genomes;
    PA_HIP(hipMemsetAsync(res->sum_block, 0, (6 + 2 * G) * 8, st));
    if (G) {
        hipLaunchKernelGGL(k_fill_first, dim3((unsigned)((G + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                           (unsigned long long *)res->min_block, G);
        PA_HIP(hipGetLastError());
    }
    return PA_OK;
}

pa_status ensure_workspace(pa_index *idx, size_t bytes) {
    if (idx->ws.bytes >= bytes) return PA_OK;
    pa::dev_free(idx->ws.ptr);
    idx->ws.ptr = nullptr;
    idx->ws.bytes = 0;
    hipError_t e = pa::dev_malloc(&idx->ws.ptr, bytes);
    if (e != hipSuccess) {
        set_error(std::string("workspace allocation failed: ") + hipGetErrorString(e));
        return PA_ENOMEM;
    }
    idx->ws.bytes = bytes;
    return PA_OK;
}

pa_status ensure_qmask(pa_index *idx, uint64_t n) {
    if (idx->qmask_cap >= n) return PA_OK;
    pa::dev_free(idx->qmask);
    pa::dev_free(idx->qdrop);
    idx->qmask = nullptr;
    idx->qdrop = nullptr;
    idx->qmask_cap = 0;
    PA_HIP(pa::dev_malloc(&idx->qmask, n * sizeof(uint4)));
    PA_HIP(pa::dev_malloc(&idx->qdrop, n));
    idx->qmask_cap = n;
    return PA_OK;
}

pa_status reserve_queues(pa_index *idx, uint64_t n) {
    if (!idx->seg_cnt) PA_HIP(pa::dev_malloc(&idx->seg_cnt, (uint64_t)kSegMaxWaves * 4));
    n += kSegSlack;
    if (idx->queue_cap >= n) return PA_OK;
    pa::dev_free(idx->queue);
    pa::dev_free(idx->queue_hard);
    pa::dev_free(idx->queue_na);
    pa::dev_free(idx->queue_na2);
    pa::dev_free(idx->queue_na_keys);
    pa::dev_free(idx->queue_rc);
    pa::dev_free(idx->queue_rc_anc);
    idx->queue = idx->queue_hard = idx->queue_na = idx->queue_na2 = idx->queue_rc = nullptr;
    idx->queue_na_keys = idx->queue_rc_anc = nullptr;
    idx->queue_cap = 0;
    PA_HIP(pa::dev_malloc(&idx->queue, n * 4));
    PA_HIP(pa::dev_malloc(&idx->queue_hard, n * 4));
    PA_HIP(pa::dev_malloc(&idx->queue_na, n * 4));
    PA_HIP(pa::dev_malloc(&idx->queue_na2, n * 4));
    PA_HIP(pa::dev_malloc(&idx->queue_na_keys, n * 16));
    PA_HIP(pa::dev_malloc(&idx->queue_rc, n * 4));
    PA_HIP(pa::dev_malloc(&idx->queue_rc_anc, n * 8));
    // [0] the lane kernel's reads without a seed, [1] k_rc_seeds' walkable ones, [2] the rest (k_align_lane_na)
    if (!idx->na_count) PA_HIP(pa::dev_malloc(&idx->na_count, 24));
    idx->queue_cap = n;
    return PA_OK;
}

// Smallest quality byte of all reads and smallest read length (grid-stride).
// The quality bytes are read as 16-B vectors (the unaligned head and tail of
// the range byte by byte), the byte minimum kept as packed 16-bit minima of
// the even and odd bytes (v_pk_min_u16: one op per two bytes); four vectors in
// flight per thread.  (Round 5: byte loads, 1.15 TB/s.)
__global__ __launch_bounds__(256) void k_reads_qstats(const uint8_t *__restrict__ qual,
                                                      const uint64_t *__restrict__ off, uint64_t n, uint32_t *out) {
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t b0 = off[0], b1 = off[n];
    // [a0, a1): the part of [b0, b1) whose addresses are whole 16-B vectors
    const uint64_t mis = (uint64_t)(uintptr_t)qual & 15;
    const uint64_t a0 = min(b1, ((b0 + mis + 15) & ~15ull) - mis), a1 = max(a0, ((b1 + mis) & ~15ull) - mis);
    uint32_t qm = 255, lm = 0xFFFFFFFFu;
    if (tid < 16) {  // the head and tail bytes outside the whole vectors
        if (b0 + tid < a0) qm = min(qm, (uint32_t)qual[b0 + tid]);
        if (a1 + tid < b1) qm = min(qm, (uint32_t)qual[a1 + tid]);
    }
    us2 mlo = {255, 255}, mhi = {255, 255};
    const uint4 *vp = (const uint4 *)(qual + a0);  // (16-B aligned)
    const uint64_t nv = (a1 - a0) >> 4;
    auto fold = [&](const uint4 x) {
        const uint32_t d[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t lo = d[j] & 0x00FF00FFu, hi = (d[j] >> 8) & 0x00FF00FFu;
            mlo = __builtin_elementwise_min(mlo, __builtin_bit_cast(us2, lo));
            mhi = __builtin_elementwise_min(mhi, __builtin_bit_cast(us2, hi));
        }
    };
    uint64_t v = tid;
    for (; v + 3 * stride < nv; v += 4 * stride) {
        const uint4 x0 = vp[v], x1 = vp[v + stride], x2 = vp[v + 2 * stride], x3 = vp[v + 3 * stride];
        fold(x0), fold(x1), fold(x2), fold(x3);
    }
    for (; v < nv; v += stride) fold(vp[v]);
    qm = min(qm, (uint32_t)min(min(mlo.x, mlo.y), min(mhi.x, mhi.y)));
    for (uint64_t r = tid; r < n; r += stride) lm = min(lm, (uint32_t)min<uint64_t>(off[r + 1] - off[r], 0xFFFFFFFFull));
    for (int o = 32; o > 0; o >>= 1) {
        qm = min(qm, (uint32_t)__shfl_down(qm, o));
        lm = min(lm, (uint32_t)__shfl_down(lm, o));
    }
    // one atomic pair per block (same-address atomics serialise: a pair per
    // wave of 4096 blocks cost more than the loads)
    __shared__ uint32_t red[2][4];
    if ((threadIdx.x & 63) == 0) red[0][threadIdx.x >> 6] = qm, red[1][threadIdx.x >> 6] = lm;
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicMin(&out[0], min(min(red[0][0], red[0][1]), min(red[0][2], red[0][3])));
        atomicMin(&out[1], min(min(red[1][0], red[1][1]), min(red[1][2], red[1][3])));
    }
}

// The batch's smallest quality byte and read length (pa_reads.q_min / len_min),
// measured when the reads are made (upload, synthesis; the FASTQ parser takes
// them from its own pass).
pa_status reads_measure(pa_reads *r, hipStream_t st) {
    r->q_min = 255;
    r->len_min = 0;
    if (!r->qual || r->n == 0) return PA_OK;
    uint32_t *d = nullptr, h[2] = {255, 0xFFFFFFFFu};
    PA_HIP(pa::dev_malloc(&d, 8));
    hipError_t e = hipMemcpyAsync(d, h, 8, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) {
        const unsigned qgrid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(2048, (r->n_bases >> 14) + 1));
        hipLaunchKernelGGL(k_reads_qstats, dim3(qgrid), dim3(256), 0, st, r->qual, r->off, r->n, d);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    pa::dev_free(d);
    PA_HIP(e);
    r->q_min = (int32_t)h[0];
    r->len_min = (int64_t)h[1];
    return PA_OK;
}

// Quality thresholds no read can fail, dropped from the pass: every read's mean
// and every window's mean are >= the smallest quality byte, so with
// --min-read-quality / --min-kmer-quality <= that byte nothing is filtered
// (src/kmer.py:420, 587: strict <) -- e.g. C3's literal 20 / 25 against
// FASTQ qualities >= '!' (33), quirk 5.  Reads of length 0 keep the read test.
pa_status effective_params(const pa_reads *r, const DevParams &p, DevParams &out, hipStream_t st) {
    out = p;
    if (!(p.flags & (F_MRQ | F_MKQ)) || !r->qual || r->n == 0 || std::getenv("PA_NO_QELIDE")) return PA_OK;
    if (r->q_min < 0) PA_TRY(reads_measure(const_cast<pa_reads *>(r), st));  // (not measured at creation)
    if ((p.flags & F_MRQ) && r->len_min > 0 && p.mrq <= r->q_min) out.flags &= ~F_MRQ;
    if ((p.flags & F_MKQ) && p.mkq <= r->q_min) out.flags &= ~F_MKQ;
    return PA_OK;
}

pa_status align(pa_index *idx, const pa_reads *r, const DevParams &p_in, uint64_t base, pa_result *acc,
                hipStream_t st) {
    if (r->n == 0) return PA_OK;
    if (r->n >= 0xFFFFFFFFull) {  // (read indices of a batch are 32-bit in the queues and lane kernels)
        set_error("pa_align: a batch holds at most 2^32 - 2 reads (split it; read_index_base keeps the order)");
        return PA_EUNSUPPORTED;
    }
    PA_TRY(index_note_reads(idx, r->n, st));  // (the neighbour bits, once enough reads came)
    PA_TRY(reserve_queues(idx, r->n));
    DevParams p;
    PA_TRY(effective_params(r, p_in, p, st));
    AlignArgs a = make_args(idx, r, p, base);
    const uint32_t G = idx->n_genomes;
    a.stats = (unsigned long long *)acc->sum_block;
    a.uniq = (unsigned long long *)acc->sum_block + 6;
    a.amb = a.uniq + G;
    a.first = (unsigned long long *)acc->min_block;
    a.queue = idx->queue;
    a.qcount = (unsigned long long *)idx->counters;
    a.deferred_total = (unsigned long long *)idx->counters + 1;
    a.dbg = (unsigned long long *)idx->counters + 4;
    PA_HIP(hipMemsetAsync(idx->counters, 0, 8, st));
#ifdef PA_STATS
    PA_HIP(hipMemsetAsync(a.dbg, 0, 224, st));
#endif
    ExactArgs x{};
    unsigned egrid = 0;
    PA_TRY(prepare_exact(idx, r, x, egrid));
    x.a = a;
    x.detail = 0;
    const bool fast_ok = idx->k > 0 && idx->nw <= 4 && idx->n_kmers > 0;  // (k <= 127: the wave kernel's keys)
    // the lane kernel first (single-word keys on a tiled index); PA_NO_LANE=1 skips it
    const char *no_lane = std::getenv("PA_NO_LANE");
    const bool lane_ok = fast_ok && idx->nw <= 3 && a.tile_n > 0 && a.tile_lw && !(no_lane && no_lane[0] == '1');
    if (fast_ok) {
        const uint32_t wmax = r->max_len >= idx->k ? (uint32_t)(r->max_len - idx->k + 1) : 0;
        const int wpl = wmax <= 64 ? 1 : wmax <= 128 ? 2 : 4;  // longer reads are deferred by WPL=4
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (idx->profile) {
            PA_HIP(hipEventCreate(&e0));
            PA_HIP(hipEventCreate(&e1));
            PA_HIP(hipEventRecord(e0, st));
        }
        if (lane_ok) {
            if ((a.prm.flags & F_MG) && a.prm.mg >= 2) {
                const uint64_t n_words = a.tile_n / 64 + 8;  // (padded: the 250-bp walk reads five words from any position)
                if (!idx->tile_big) PA_HIP(pa::dev_malloc(&idx->tile_big, n_words * 8));
                if (idx->tile_big_mg != a.prm.mg) {
                    hipLaunchKernelGGL(k_tile_big, dim3((unsigned)std::min<uint64_t>((n_words + 3) / 4, 1u << 20)),
                                       dim3(256), 0, st, idx->tile_cls, a.tile_n, a.G, idx->class_genomes,
                                       (int32_t)a.prm.mg, idx->tile_big, n_words);
                    PA_HIP(hipGetLastError());
                    idx->tile_big_mg = a.prm.mg;
                }
                a.tile_big = idx->tile_big;
                // the neighbour bits' set-size half for this mg (12 B per base;
                // only with the 24-B neighbour bits, and when it fits)
                if (idx->tile_nb && idx->nb_spec && !idx->tile_nb1 && !std::getenv("PA_NO_NBBIG")) {
                    const uint64_t nw = 3 * a.tile_n;
                    if (!idx->tile_nbbig) {
                        size_t free_b = 0, total_b = 0;
                        if (pa::dev_mem_info(&free_b, &total_b) == hipSuccess && nw * 4 + (8ull << 30) < free_b &&
                            pa::dev_malloc(&idx->tile_nbbig, nw * 4 + 64) == hipSuccess) {
                            idx->tile_nbbig_mg = -1;
                            idx->device_bytes += nw * 4 + 64;  // (pa_index_get_info reports the real footprint)
                        } else
                            idx->tile_nbbig = nullptr;
                        (void)hipGetLastError();
                    }
                    if (idx->tile_nbbig && idx->tile_nbbig_mg != a.prm.mg) {
                        hipLaunchKernelGGL(k_nb_big, dim3((unsigned)std::min<uint64_t>((nw + 255) / 256, 1u << 20)),
                                           dim3(256), 0, st, idx->tile_pk, (const uint64_t *)idx->tile_nb, nw, (int)idx->k,
                                           (const Slot<1> *)idx->table, idx->home, a.G, idx->class_genomes,
                                           (int32_t)a.prm.mg, idx->tile_nbbig);
                        PA_HIP(hipGetLastError());
                        idx->tile_nbbig_mg = a.prm.mg;
                    }
                    a.tile_nbbig = idx->tile_nbbig;
                    if (a.tile_nbbig) a.nbbig_ld = a.tile_nbbig, a.nbbig_mask = ~0ull;
                    // interleaved with the neighbour words (48 B per base, when it fits; PA_NO_NBM=1: none)
                    if (idx->tile_nbbig && !std::getenv("PA_NO_NBM")) {
                        if (!idx->tile_nbm) {
                            size_t free_b = 0, total_b = 0;
                            if (pa::dev_mem_info(&free_b, &total_b) == hipSuccess && nw * 16 + (8ull << 30) < free_b &&
                                pa::dev_malloc(&idx->tile_nbm, nw * 16 + 64) == hipSuccess) {
                                idx->tile_nbm_mg = -1;
                                idx->device_bytes += nw * 16 + 64;
                            } else
                                idx->tile_nbm = nullptr;
                            (void)hipGetLastError();
                        }
                        if (idx->tile_nbm && idx->tile_nbm_mg != a.prm.mg) {
                            hipLaunchKernelGGL(k_nb_merge, dim3((unsigned)std::min<uint64_t>((nw + 255) / 256, 1u << 20)),
                                               dim3(256), 0, st, (const uint64_t *)idx->tile_nb, idx->tile_nbbig, nw,
                                               idx->tile_nbm);
                            PA_HIP(hipGetLastError());
                            idx->tile_nbm_mg = a.prm.mg;
                        }
                        a.tile_nbm = idx->tile_nbm;
                    }
                }
            }
            // every present neighbour's set size vs mg known from the bits
            a.mg_nb = (a.prm.flags & F_MG) && a.tile_nb && a.nb_spec && (a.prm.mg < 2 || a.tile_nbbig) &&
                      !std::getenv("PA_NO_MGNB");
            a.queue_hard = idx->queue_hard;
            a.queue_hard_count = (unsigned long long *)idx->counters + 3;
            PA_HIP(hipMemsetAsync(idx->counters + 3, 0, 8, st));
            if (a.prm.flags & (F_MRQ | F_MKQ)) {  // the quality filters of every read, up front
                if (idx->k > 95) {  // (k_quality_masks realigns by k >> 2 <= 23: lane_ok implies k <= 95)
                    set_error("internal: quality pre-pass for k > 95");
                    return PA_EINTERNAL;
                }
                PA_TRY(ensure_qmask(idx, r->n));
                KernelTimer kt(idx, st, PA_PROF_QUALITY);
                hipLaunchKernelGGL(idx->k > 63 ? k_quality_masks<true> : k_quality_masks<false>, dim3((unsigned)std::min<uint64_t>((r->n + 255) / 256, 65536)),
                                   dim3(256), 0, st, r->qual, r->off, r->n, (int)idx->k, (int64_t)a.prm.mrq,
                                   (int64_t)a.prm.mkq, a.prm.flags & (F_MRQ | F_MKQ), idx->qmask, idx->qdrop);
                PA_HIP(hipGetLastError());
                a.qmask = idx->qmask;
                a.qdrop = idx->qdrop;
            }
            // reads without a seed in the index: k_align_lane_na (with a Bloom filter; PA_LANE_NOANCHOR=0/1)
            bool na = a.bloom != nullptr;
            if (const char *e = std::getenv("PA_LANE_NOANCHOR")) na = e[0] == '1';
            if (idx->nw > 3) na = false;  // (two- and three-word keys: k_align_lane_naw)
            a.queue_na = na ? idx->queue_na : nullptr;
            a.queue_na_count = idx->na_count;
            // their reverse-complement seeds (k_rc_seeds -> k_align_lane_rc):
            // with the reverse-complement plane (PA_NA_RCWALK=0: none)
            const bool rcw = na && a.tile_rcp && a.bloom;
            a.queue_na_keys = rcw ? idx->queue_na_keys : nullptr;
            a.queue_rc = idx->queue_rc;
            a.queue_rc_anc = idx->queue_rc_anc;
            a.queue_rc_count = idx->na_count + 1;
            a.seg_cnt = idx->seg_cnt;
            a.queue_cap = idx->queue_cap;
            a.queue_na2 = idx->queue_na2;
            a.queue_na2_count = idx->na_count + 2;
            a.na_min = 32768;  // (PA_NA_MIN: tests)
            if (const char *e = std::getenv("PA_NA_MIN")) a.na_min = std::strtoull(e, nullptr, 10);
            if (na) PA_HIP(hipMemsetAsync(idx->na_count, 0, 24, st));
            // the 250-bp shape when any read is longer than the 150-bp one
            // takes: 176 bases or 128 windows (round 6: reads of 159-176 bases
            // at k = 31 went whole to the wave kernel, 0.15 G reads/s)
            const bool long_reads = r->max_len > (uint32_t)kLaneMaxLen ||
                                    (r->max_len >= idx->k && r->max_len - idx->k + 1 > (uint32_t)kLaneMaxW);
            PA_TRY(launch_lane(a, st, idx, long_reads, idx->nw));
            a.rlist = idx->queue_hard;
            a.rlist_count = a.queue_hard_count;
        }
        {
            KernelTimer kt(idx, st, PA_PROF_WAVE);
            PA_TRY(idx->nw == 1   ? launch_fast_wpl<1>(a, wpl, st)
                   : idx->nw == 2 ? launch_fast_wpl<2>(a, wpl, st)
                   : idx->nw == 3 ? launch_fast_wpl<3>(a, wpl, st)
                                  : launch_fast_wpl<4>(a, wpl, st));
        }
        if (idx->profile) {
            PA_HIP(hipEventRecord(e1, st));
            idx->ev_start.push_back(e0);
            idx->ev_stop.push_back(e1);
        }
        x.a = a;
        x.use_queue = 1;
    } else {
        x.use_queue = 0;
    }
    {
        KernelTimer kt(idx, st, PA_PROF_EXACT);
        launch_exact_nw(idx->nw, x, egrid, st);
        PA_HIP(hipGetLastError());
    }
#ifdef PA_STATS
    unsigned long long d[32];
    PA_HIP(hipMemcpyAsync(d, idx->counters, 256, hipMemcpyDeviceToHost, st));
    PA_HIP(hipStreamSynchronize(st));
    fprintf(stderr, "[pa_stats] reads %llu lane-hard %llu exact %llu | wave kernel: windows %llu probed %llu walk %llu anchors %llu\n",
            (unsigned long long)r->n, d[3], d[0], d[4], d[5], d[6], d[7]);
    fprintf(stderr, "[pa_stats] lane hard reasons: long %llu mkq %llu bad %llu no-anchor %llu range %llu mismatches %llu rep %llu found %llu pending %llu\n",
            d[8], d[9], d[10], d[11], d[12], d[13], d[14], d[15], d[16]);
    fprintf(stderr, "[pa_stats] lane: cooperative probes %llu re-anchors %llu neighbour words %llu | pending: invalid %llu "
            "2+ mismatches %llu neighbour present %llu\n", d[18], d[19], d[20], d[21], d[22], d[23]);
    fprintf(stderr, "[pa_stats] lane found: shared-neighbour+specific %llu second-walk specific %llu probed-shared+specific %llu"
            " | unique by bound %llu, by off-walk counts %llu | probes past the Bloom filter %llu\n", d[24], d[25], d[26], d[27], d[28],
            d[29]);
    fprintf(stderr, "[pa_stats] lane seeds: anchor ranked among stretches %llu, second seed round %llu\n", d[30], d[31]);
#endif
    return PA_OK;
}

pa_status align_detail(pa_index *idx, const pa_reads *r, const DevParams &p, uint8_t *type, uint32_t *qf,
                       uint32_t *hr, uint64_t *list_off, uint32_t *lists, uint64_t list_cap, uint64_t *list_total,
                       hipStream_t st) {
    const uint64_t n = r->n;
    if (list_off) list_off[0] = 0;
    if (list_total) *list_total = 0;
    if (n == 0) return PA_OK;
    ExactArgs x{};
    unsigned egrid = 0;
    PA_TRY(prepare_exact(idx, r, x, egrid));
    x.a = make_args(idx, r, p, 0);
    x.use_queue = 0;
    uint8_t *d_type = nullptr;
    uint32_t *d_qf = nullptr, *d_hr = nullptr, *d_len = nullptr, *d_lists = nullptr;
    uint64_t *d_off = nullptr;
    PA_HIP(pa::dev_malloc(&d_type, n));
    PA_HIP(pa::dev_malloc(&d_qf, n * 4));
    PA_HIP(pa::dev_malloc(&d_hr, n * 4));
    PA_HIP(pa::dev_malloc(&d_len, n * 4));
    x.type_out = d_type;
    x.qf_out = d_qf;
    x.hr_out = d_hr;
    x.len_out = d_len;
    x.detail = 1;
    launch_exact_nw(idx->nw, x, egrid, st);
    PA_HIP(hipGetLastError());
    std::vector<uint32_t> lens(n);
    PA_HIP(hipMemcpyAsync(lens.data(), d_len, n * 4, hipMemcpyDeviceToHost, st));
    PA_HIP(hipMemcpyAsync(type, d_type, n, hipMemcpyDeviceToHost, st));
    PA_HIP(hipMemcpyAsync(qf, d_qf, n * 4, hipMemcpyDeviceToHost, st));
    PA_HIP(hipMemcpyAsync(hr, d_hr, n * 4, hipMemcpyDeviceToHost, st));
    PA_HIP(hipStreamSynchronize(st));
    std::vector<uint64_t> offs(n + 1, 0);
    for (uint64_t i = 0; i < n; i++) offs[i + 1] = offs[i] + lens[i];
    const uint64_t total = offs[n];
    if (list_total) *list_total = total;
    if (list_off) std::memcpy(list_off, offs.data(), (n + 1) * 8);
    pa_status rc = PA_OK;
    if (lists && total > 0) {
        if (list_cap < total) {
            set_error("pa_align_detail: list_cap smaller than the required list length");
            rc = PA_EINVAL;
        } else {
            PA_HIP(pa::dev_malloc(&d_off, (n + 1) * 8));
            PA_HIP(pa::dev_malloc(&d_lists, total * 4));
            PA_HIP(hipMemcpyAsync(d_off, offs.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
            x.detail = 2;
            x.list_off = d_off;
            x.lists = d_lists;
            launch_exact_nw(idx->nw, x, egrid, st);
            PA_HIP(hipGetLastError());
            PA_HIP(hipMemcpyAsync(lists, d_lists, total * 4, hipMemcpyDeviceToHost, st));
            PA_HIP(hipStreamSynchronize(st));
        }
    }
    pa::dev_free(d_type); pa::dev_free(d_qf); pa::dev_free(d_hr); pa::dev_free(d_len); pa::dev_free(d_off); pa::dev_free(d_lists);
    return rc;
}

}  // namespace pa

namespace {
__global__ void k_warm_align() {}
}  // namespace

namespace pa {
// Loads this file's code object (a first launch from a module loads it): the
// CLI's runtime-start thread calls it so that the load overlaps host work.
void warm_align(hipStream_t st) { hipLaunchKernelGGL(k_warm_align, dim3(1), dim3(64), 0, st); }
}  // namespace pa
