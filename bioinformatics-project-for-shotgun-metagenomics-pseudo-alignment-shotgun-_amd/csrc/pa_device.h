// Device-side building blocks shared by the index-build and align kernels.
//
// K-mer keys.  A k-mer is packed 2 bits per base (A=0 C=1 G=2 T=3), first base
// in the most significant bits, into NW = k/32 + 1 64-bit words.  The top word
// holds 2k - 64*(NW-1) < 64 bits, so an all-ones top word is never a key and
// serves as the empty-slot sentinel of the hash table.  This is the HBM form of
// the reference's `Dict[str, ...]` keys (src/kmer.py:130); bases other than
// ACGT poison every window that contains them (the reference skips k-mers with
// 'N' at src/kmer.py:145, and reads can only hold ACGT, src/records.py:262).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pa_home.h"

namespace pad {

constexpr uint64_t EMPTY = ~0ull;        // empty slot (top key word)
constexpr uint64_t BUSY = ~0ull - 1;     // slot being written (multi-word inserts)
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t PA_TILE_REP = 0x80000000u;  // tile_cls flag: the k-mer repeats within the next 255 positions
// compact tile (uint16 per position) of the lane kernel

template <int NW>
struct Key {
    uint64_t w[NW];
};

// Hash-table slot: packed key + class id + tile position.  `tpos` is the
// smallest concatenated-genome window position holding the key (the start of
// its first occurrence in FASTA order), or NONE when the index has no genome
// tiling (see the tile arrays in pa_internal.h and the walk in pa_fast.h).
template <int NW>
struct Slot {
    uint64_t key[NW];
    uint32_t cls;
    uint32_t tpos;
};

// The one-substitution neighbour words of an index (tile_nb), in one piece or
// two: a reference whose words find no single free range in the slab pool
// (C5's 107 GiB after EXTSIM) takes them in two halves instead of stalling on
// the driver's reclaim of freed memory.  Word i lies at base0 + i * wb below
// `split`, at base1 + i * wb from there (base1 biased by -split * wb on the
// host); one piece: split = ~0.
struct NbW {
    uint64_t base0, base1, split;
    template <typename T>
    __device__ __forceinline__ T *word(uint64_t i) const {
        return (T *)((i < split ? base0 : base1) + i * sizeof(T));
    }
};

// Class ids are < 2^31 (the build refuses more genome-set entries), so bit 31
// of a slot's cls is free: for references of 2^32 .. 2^33 bases it holds bit
// 32 of the key's concatenated first position (k_tpos_concat), whose low bits
// are slot.tpos.  Every use of a slot's class goes through cls_of.
constexpr uint32_t kClsMask = 0x7FFFFFFFu;
__device__ __forceinline__ uint32_t cls_of(uint32_t cls) { return cls & kClsMask; }

// Number of genomes of a class: cls < G is a singleton, otherwise the class id
// is G + the offset of its [size, genomes...] record.
__device__ __forceinline__ uint32_t class_size_of(uint32_t cls, uint32_t G, const uint32_t *class_genomes) {
    cls = cls_of(cls);
    return cls < G ? 1u : class_genomes[cls - G];
}

// Concatenated-genome position of a key's first occurrence from its slot's
// (raw) cls and tpos: with `local` (references of >= 2^33 bases, or
// PA_TPOS_HI=0) tpos is genome-local, in the key's first genome (its specific
// genome, or the first of its genome set: records are [size, ascending
// genomes...]), which costs the caller two dependent loads; otherwise tpos is
// the position's low 32 bits and bit 31 of cls its bit 32.
__device__ __forceinline__ uint64_t first_pos(uint32_t cls, uint32_t tpos, uint32_t G, const uint32_t *class_genomes,
                                              const uint64_t *goff, bool local) {
    if (!local) return ((uint64_t)(cls >> 31) << 32) | tpos;
    cls = cls_of(cls);
    const uint32_t g = cls < G ? cls : class_genomes[cls - G + 1];
    return goff[g] + tpos;
}

__device__ __forceinline__ uint64_t fmix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

template <int NW>
__device__ __forceinline__ uint64_t key_hash(const Key<NW> &k) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
#pragma unroll
    for (int j = 0; j < NW; j++) h = fmix64(h ^ k.w[j]);
    return h;
}

// Home slot by multiply-high range reduction (table size need not be 2^n).
// For cap < 2^32 (every table up to 64 GiB) the same value from three 32-bit
// multiplies instead of seven: with h = hi 2^32 + lo, floor(h cap / 2^64) =
// floor((hi cap + floor(lo cap / 2^32)) / 2^32).
__device__ __forceinline__ uint64_t home_slot(uint64_t h, uint64_t cap) {
    if (cap >> 32) return __umul64hi(h, cap);
    const uint32_t c = (uint32_t)cap;
    const uint64_t x = (uint64_t)(uint32_t)(h >> 32) * c + __umulhi((uint32_t)h, c);
    return x >> 32;
}

__device__ __forceinline__ uint32_t base_code(uint32_t ch) {
    return ch == 'A' ? 0u : ch == 'C' ? 1u : ch == 'G' ? 2u : ch == 'T' ? 3u : 4u;
}

// Append one base (2-bit code) to a rolling key, keeping 2k bits.
template <int NW>
__device__ __forceinline__ void key_push(Key<NW> &k, uint32_t c, uint64_t mask0) {
#pragma unroll
    for (int j = 0; j < NW - 1; j++) k.w[j] = (k.w[j] << 2) | (k.w[j + 1] >> 62);
    k.w[NW - 1] = (k.w[NW - 1] << 2) | (uint64_t)c;
    k.w[0] &= mask0;
}

__device__ __forceinline__ uint64_t mask0_of(int k, int nw) {
    int bits = 2 * k - 64 * (nw - 1);
    return bits >= 64 ? ~0ull : ((1ull << bits) - 1);
}

// 64 bits of a MSB-first 2-bit packed base array starting at bit `o`.
__device__ __forceinline__ uint64_t get64(const uint64_t *p, uint32_t o) {
    uint32_t q = o >> 6, r = o & 63;
    uint64_t hi = p[q] << r;
    return r ? (hi | (p[q + 1] >> (64 - r))) : hi;
}

// 64 bits at a 64-bit bit offset (packed genomes exceed 2^32 bits).
__device__ __forceinline__ uint64_t get64_at(const uint64_t *p, uint64_t o) {
    const uint64_t q = o >> 6;
    const uint32_t r = (uint32_t)(o & 63);
    const uint64_t hi = p[q] << r;
    return r ? (hi | (p[q + 1] >> (64 - r))) : hi;
}

// Key of the window starting at base w of a packed read.
template <int NW>
__device__ __forceinline__ Key<NW> extract_key(const uint64_t *packed, uint32_t w, int k) {
    Key<NW> key;
    const int w0bits = 2 * k - 64 * (NW - 1);
    // k a multiple of 32 leaves the top word empty (a 64-bit shift would be undefined)
    key.w[0] = w0bits ? (get64(packed, 2 * w) >> (64 - w0bits)) : 0;
#pragma unroll
    for (int j = 1; j < NW; j++) key.w[j] = get64(packed, 2 * w + w0bits + 64 * (j - 1));
    return key;
}

// Bits [w, w+k) of a LSB-first position bitmap (k < 64).
__device__ __forceinline__ uint64_t window_bits(const uint64_t *bm, uint32_t w, int k) {
    uint32_t q = w >> 6, r = w & 63;
    uint64_t v = bm[q] >> r;
    if (r) v |= bm[q + 1] << (64 - r);
    return k >= 64 ? v : v & ((1ull << k) - 1);
}

// Any of the k bits from bit w on set (k up to the widest key, 64 at a time).
// (Round 5: the wave kernel tested min(k, 64) bits -- and for k >= 64 a
// shifted-out mask -- so a window of k > 63 with a non-ACGT base past its
// first 64 positions was looked up with the base as a code.)
__device__ __forceinline__ bool window_any(const uint64_t *bm, uint32_t w, int k) {
    for (int o = 0; o < k; o += 64)
        if (window_bits(bm, w + (uint32_t)o, k - o)) return true;
    return false;
}

// Where a key starts probing: multiply-high range reduction of its hash over
// the table's capacity.  PA_HOME_ALIGN = 4 homes every key at the start of its
// aligned 4-slot group (the probes read whole groups, so a search then never
// wastes the slots before its home): modelled to cut a wave's seed round trips
// from ~1.9 to ~1.03 at C2's load (scripts/probe_model.py), measured on MI355X
// 1-3 % SLOWER on C2 / c2mix / C4 / C5 (profiles/r04/ab_home_align.txt) -- the
// lanes' extra round trips are hidden by the other waves, while bucketed homes
// crowd the probes of a group -- so homes stay slot-granular.  (A
// minimizer-region variant -- keys of one super-k-mer homed in one region --
// measured 1.7-3x slower on C2 and was removed; the genome walk of pa_fast.h /
// pa_lane.h gets the locality instead.)
#ifndef PA_HOME_ALIGN
#define PA_HOME_ALIGN 1
#endif
constexpr uint64_t kHomeAlign = PA_HOME_ALIGN;
static_assert(kHomeAlign == 1 || kHomeAlign == 2 || kHomeAlign == 4, "tables are whole 4-slot groups");
template <int NW>
__device__ __forceinline__ uint64_t home_of(const Key<NW> &, uint64_t h, const HomeCfg &c) {
    return home_slot(h, c.cap / kHomeAlign) * kHomeAlign;
}

// Ordered clusters.  Once built, every run of occupied slots is put in the
// order of its keys' homes (k_table_order, pa_index.hip): the layout linear
// probing gives when the keys arrive in home order -- the same occupied slots,
// every key at or after its home with no EMPTY slot between.  A search for a
// key homed at h then also ends at the first slot j holding a key that is less
// displaced than the searched one would be there (homed after h, counted
// cyclically): the key cannot lie further.  Absent keys no longer run to the
// end of their cluster, which at C5's load (0.48) cuts a wave's probe rounds
// from ~4.5 to ~2.1 (scripts/probe_model.py: the slowest of a wave's ~128
// probes sets the wave's pace).  The probes test the LAST slot of each group
// they read (the cluster's homes rise along it), only on the path that would
// read another group.  PA_TABLE_ORDER=0 builds tables without the pass, and
// no probe may then use the test.
#ifndef PA_TABLE_ORDER
#define PA_TABLE_ORDER 1
#endif
constexpr bool kTableOrdered = PA_TABLE_ORDER != 0;

template <int NW>
__device__ __forceinline__ bool probe_past_key(const Key<NW> &rk, const Key<NW> &me, uint64_t j, const HomeCfg &hc) {
    if constexpr (!kTableOrdered) return false;
    const uint64_t hr = home_of<NW>(rk, key_hash(rk), hc), hm = home_of<NW>(me, key_hash(me), hc);
    const uint64_t dr = j >= hr ? j - hr : j + hc.cap - hr;
    const uint64_t dm = j >= hm ? j - hm : j + hc.cap - hm;
    return dr < dm;
}
template <int NW>
__device__ __forceinline__ bool probe_past(const Slot<NW> &r, const Key<NW> &me, uint64_t j, const HomeCfg &hc) {
    Key<NW> rk;
#pragma unroll
    for (int t = 0; t < NW; t++) rk.w[t] = r.key[t];
    return probe_past_key<NW>(rk, me, j, hc);
}

// Read-only probe from a home slot (tables are immutable once built).  ORD:
// the table's clusters are ordered (every probe after the build; the build's
// own passes before k_table_order run with ORD = false).
template <int NW, bool ORD = false>
__device__ __forceinline__ bool table_find(const Slot<NW> *__restrict__ t, uint64_t cap, const Key<NW> &k,
                                           uint64_t home, uint64_t &slot, uint32_t &cls, uint32_t &tpos) {
    uint64_t pos = home;
    for (;;) {
        const Slot<NW> s = t[pos];
        if (s.key[0] == EMPTY) return false;
        bool eq = true;
#pragma unroll
        for (int j = 0; j < NW; j++) eq &= (s.key[j] == k.w[j]);
        if (eq) {
            slot = pos;
            cls = s.cls;
            tpos = s.tpos;
            return true;
        }
        if constexpr (ORD && kTableOrdered) {
            Key<NW> rk;
#pragma unroll
            for (int j = 0; j < NW; j++) rk.w[j] = s.key[j];
            const uint64_t hr = home_of<NW>(rk, key_hash(rk), HomeCfg{cap});
            if ((pos >= hr ? pos - hr : pos + cap - hr) < (pos >= home ? pos - home : pos + cap - home)) return false;
        }
        pos = (pos + 1 == cap) ? 0 : pos + 1;
    }
}

// NP single-word probes in flight together, a whole 64-B line (4 slots) per
// step: tables are whole lines (cap % 4 == 0), so a search costs ~1-2 round
// trips even at a high load factor, where slot-by-slot probing (table_find)
// pays one dependent load per slot.  Bit i of `found` / cls[i]: key i's result
// (keys outside `act` are not looked up; classes without the position bit).
template <int NP>
__device__ __forceinline__ uint32_t probe_lines(const Slot<1> *__restrict__ t, const HomeCfg &hc,
                                                const uint64_t (&key)[NP], uint32_t (&cls)[NP],
                                                uint32_t act = (1u << NP) - 1) {
    uint64_t pos[NP];
#pragma unroll
    for (int i = 0; i < NP; i++) {
        Key<1> kk;
        kk.w[0] = key[i];
        pos[i] = home_of<1>(kk, key_hash(kk), hc);
    }
    uint32_t found = 0;
    while (act) {
        Slot<1> s[NP][4];
#pragma unroll
        for (int i = 0; i < NP; i++)
            if ((act >> i) & 1u) {
                const uint64_t b = pos[i] & ~3ull;
#pragma unroll
                for (int h = 0; h < 4; h++) s[i][h] = t[b + h];
            }
#pragma unroll
        for (int i = 0; i < NP; i++) {
            if (!((act >> i) & 1u)) continue;
            const uint64_t b = pos[i] & ~3ull;
            bool done = false;
#pragma unroll
            for (int h = 0; h < 4; h++) {
                if (done || b + h < pos[i]) continue;
                if (s[i][h].key[0] == EMPTY) {
                    done = true;
                } else if (s[i][h].key[0] == key[i]) {
                    done = true;
                    found |= 1u << i;
                    cls[i] = cls_of(s[i][h].cls);
                }
            }
            if (!done) {
                Key<1> kk;
                kk.w[0] = key[i];
                done = probe_past<1>(s[i][3], kk, b + 3, hc);
            }
            if (done) act &= ~(1u << i);
            pos[i] = (b + 4 == hc.cap) ? 0 : b + 4;
        }
    }
    return found;
}

// Bloom filter of the table's single-word keys (the lane kernels' prefilter
// for the windows they must look up): 2^lg 64-bit words (lg <= 33: up to
// 64 GiB; C2 takes lg = 24, C4 / C5 the HBM form up to 1/8 of free memory),
// one word per key and kBloomK bits in it (kBloomK 6-bit fields of the key's
// 32-bit mix).  No false negatives: a key whose bits are not all set is not in
// the table.  Four bits per key: with a run of ~9 keys sharing a block (below)
// the blocks' load varies so much that more bits per key stopped paying --
// modelled on C2: 0.98 false positives per 120 windows with 4, 1.04 with 6.
#ifndef PA_BLOOM_K
#define PA_BLOOM_K 4
#endif
constexpr int kBloomK = PA_BLOOM_K;
static_assert(kBloomK >= 1 && kBloomK <= 5, "the fields and the block-word bits share 32 bits");
// The key's mix: bits 0 .. 6 kBloomK - 1 the fields, the top bits the word
// within its block.  The high word multiplied into the low one, then one
// xorshift-multiply round (two 32-bit multiplies; the 64-bit mix it replaced
// took three 64-bit ones.  The high half of a single multiply, tried in r3, is
// monotone in its input: the fields correlate, c2rc's na kernel 2.63 -> 3.0 ms).
__device__ __forceinline__ uint32_t bloom_key_mix(uint64_t key) {
    uint32_t h = ((uint32_t)(key >> 32) * 0x9E3779B1u) ^ (uint32_t)key;
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    return h;
}
__device__ __forceinline__ uint64_t bloom_bits(uint32_t h) {
    uint64_t m = 0;
#pragma unroll
    for (int i = 0; i < kBloomK; i++) m |= 1ull << ((h >> (6 * i)) & 63);
    return m;
}

// Minimizer-blocked layout: the filter's words pair up into 16-B BLOCKS; the block of a k-mer (k <= 31) is chosen by its
// minimizer -- the 15-mer (the whole k-mer below 15) of smallest order among
// its k - 14 -- so that the windows of a read that share a minimizer (runs of
// ~9 on random sequence) share one block, which k_align_lane_na loads once per
// run; the word within the block (the top bits of the key's mix) and the
// kBloomK bits by the key's own mix.  The minimizer order is two full-rate ops on the
// 15-mer (a 24-bit multiply, no 32-bit one), the block the top bits of one
// multiply of the minimum.
constexpr int kBloomBW = 2;  // 64-bit words per block (32-B blocks: A/B r3, slower -- they spilled)
constexpr int kBloomLgBW = 1;
__device__ __forceinline__ uint32_t mm_order(uint32_t x) {
    return __umul24(x ^ (x >> 15), 0xB5297Bu) ^ (x >> 9);
}
__device__ __forceinline__ uint64_t bloom_block(uint32_t mn, uint32_t lg) {  // (lg - kBloomLgBW bits; lg <= 33)
    return (uint64_t)((mn * 0x9E3779B1u) >> (32 + kBloomLgBW - lg));
}
__device__ __forceinline__ uint32_t key_minimizer(uint64_t key, int k) {
    const int mm = k < 15 ? k : 15;
    const uint64_t mmask = (1ull << (2 * mm)) - 1;
    uint32_t best = ~0u;
    for (int i = 0; i + mm <= k; i++) best = min(best, mm_order((uint32_t)((key >> (2 * i)) & mmask)));
    return best;
}
// The same for a k known at compile time (15 <= K <= 31), unrolled: each
// 15-mer one funnel shift of the key's two halves (the rolled loop above
// costs ~14 VALU per 15-mer, this ~6)
template <int K>
__device__ __forceinline__ uint32_t key_minimizer_c(uint64_t key) {
    static_assert(K >= 15 && K <= 31, "15-mers inside a single-word key");
    const uint32_t lo = (uint32_t)key, hi = (uint32_t)(key >> 32);
    uint32_t best = ~0u;
#pragma unroll
    for (int i = 0; i + 15 <= K; i++) {
        const uint32_t x = (2 * i < 32 ? __builtin_amdgcn_alignbit(hi, lo, 2 * i) : hi >> (2 * i - 32)) & 0x3FFFFFFFu;
        best = min(best, mm_order(x));
    }
    return best;
}
// The Bloom word of a key and its bits.
__device__ __forceinline__ void bloom_word(uint64_t key, int k, uint32_t lg, uint64_t &w, uint64_t &m) {
    const uint32_t h = bloom_key_mix(key);
    m = bloom_bits(h);
    const uint32_t mn = k == 31 ? key_minimizer_c<31>(key) : key_minimizer(key, k);
    w = (bloom_block(mn, lg) << kBloomLgBW) | (h >> (32 - kBloomLgBW));
}
// The build-time filter of k_nb_build / k_nb_first (its own filter, freed
// after): blocked by a minimizer of a cheaper order -- the 15-mer XOR a fixed
// random pattern, one VALU op instead of mm_order's four -- since those kernels
// compute ~93 of them per window and are VALU-bound as much as memory-bound.
constexpr uint32_t kNbOrderXor = 0x2B7E1516u & 0x3FFFFFFFu;
__device__ __forceinline__ uint32_t key_minimizer_nb(uint64_t key, int k) {
    const int mm = k < 15 ? k : 15;
    const uint64_t mmask = (1ull << (2 * mm)) - 1;
    const uint32_t lo = (uint32_t)key, hi = (uint32_t)(key >> 32);
    uint32_t best = ~0u;
    if (k == 31) {
#pragma unroll
        for (int i = 0; i < 17; i++) {
            const uint32_t x = (2 * i < 32 ? __builtin_amdgcn_alignbit(hi, lo, 2 * i) : hi >> (2 * i - 32)) & 0x3FFFFFFFu;
            best = min(best, x ^ kNbOrderXor);
        }
        return best ^ kNbOrderXor;
    }
    for (int i = 0; i + mm <= k; i++) best = min(best, (uint32_t)((key >> (2 * i)) & mmask) ^ kNbOrderXor);
    return best ^ kNbOrderXor;
}
__device__ __forceinline__ void bloom_word_nb(uint64_t key, int k, uint32_t lg, uint64_t &w, uint64_t &m) {
    const uint32_t h = bloom_key_mix(key);
    m = bloom_bits(h);
    w = (bloom_block(key_minimizer_nb(key, k), lg) << kBloomLgBW) | (h >> (32 - kBloomLgBW));
}
// The Bloom word of a two-word key (31 < k <= 63, the lane path of long k):
// the block by a hash of the key (no minimizer runs: a read's windows off the
// walk are probed one by one), the bits by its mix as above.
__device__ __forceinline__ void bloom_word2(const Key<2> &key, uint32_t lg, uint64_t &w, uint64_t &m) {
    const uint32_t h = bloom_key_mix(key.w[1] ^ (key.w[0] * 0x9E3779B97F4A7C15ull));
    m = bloom_bits(h);
    const uint64_t b = fmix64(key.w[1] ^ (key.w[0] * 0xC2B2AE3D27D4EB4Full) ^ 0x5851F42D4C957F2Dull);
    w = ((b >> (64 - (lg - kBloomLgBW))) << kBloomLgBW) | (h >> (32 - kBloomLgBW));
}
// The same for a three-word key (63 < k <= 95: the lane path of the
// reference's demo k = 75, src/RUN_LOG:28-61).
__device__ __forceinline__ void bloom_word3(const Key<3> &key, uint32_t lg, uint64_t &w, uint64_t &m) {
    const uint64_t x = key.w[2] ^ (key.w[1] * 0x9E3779B97F4A7C15ull) ^ (key.w[0] * 0xD6E8FEB86659FD93ull);
    const uint32_t h = bloom_key_mix(x);
    m = bloom_bits(h);
    const uint64_t b = fmix64(x ^ (key.w[1] * 0xC2B2AE3D27D4EB4Full) ^ 0x5851F42D4C957F2Dull);
    w = ((b >> (64 - (lg - kBloomLgBW))) << kBloomLgBW) | (h >> (32 - kBloomLgBW));
}
// The key of the genome window at 2-bit position t (the words key_push leaves:
// the last 32 bases in w[NW - 1], the first 2k - 64 (NW - 1) bits in w[0]).
template <int NW>
__device__ __forceinline__ Key<NW> genome_key(const uint64_t *pk, uint64_t t, int k) {
    Key<NW> K;
    const int hb = 2 * k - 64 * (NW - 1);
#pragma unroll
    for (int j = 1; j < NW; j++) K.w[j] = get64_at(pk, 2 * t + 2 * k - 64 * (NW - j));
    K.w[0] = NW == 1 ? (get64_at(pk, 2 * t) >> (64 - 2 * k)) : (hb ? get64_at(pk, 2 * t) >> (64 - hb) : 0ull);
    return K;
}
// The key with base j of its window (0: the first) replaced by its b-th other
// base ((base + 1 + b) & 3).
template <int NW>
__device__ __forceinline__ Key<NW> key_sub(Key<NW> K, int j, int k, int b) {
    const int bs = 2 * (k - 1 - j);  // the base's bit offset from the key's end
    const int wi = NW - 1 - bs / 64, bo = bs % 64;
    uint64_t c = 0;
#pragma unroll
    for (int q = 0; q < NW; q++)
        if (q == wi) c = (K.w[q] >> bo) & 3;
    const uint64_t x = (c ^ ((c + 1 + (uint64_t)b) & 3)) << bo;
#pragma unroll
    for (int q = 0; q < NW; q++)
        if (q == wi) K.w[q] ^= x;
    return K;
}

// Minimizer presence bitmap (mm_bits, 2^lg bits): bit mm_bit(mn) is set for
// the minimizer of every key (k_mm_build) -- a prefilter small enough to stay
// in the L2 that answers a whole minimizer run of absent windows.
__device__ __forceinline__ uint32_t mm_bit(uint32_t mn, uint32_t lg) { return (mn * 0x85EBCA77u) >> (32 - lg); }
// A key's test against its (loaded) 16-B block.
__device__ __forceinline__ bool bloom_block_has(const uint4 &b, uint32_t h) {
    const bool w1 = (h >> 31) != 0;
    const uint64_t wv = w1 ? (((uint64_t)b.w << 32) | b.z) : (((uint64_t)b.y << 32) | b.x);
    const uint64_t bm = bloom_bits(h);
    return (wv & bm) == bm;
}

// ---- reverse complements (2-bit codes: complement = code ^ 3) ----------------

// The 32 2-bit groups of x in reverse order.
__device__ __forceinline__ uint64_t rev_groups64(uint64_t x) {
    const uint64_t y = __builtin_bitreverse64(x);
    return ((y >> 1) & 0x5555555555555555ull) | ((y & 0x5555555555555555ull) << 1);
}
// Reverse complement of a single-word key of k <= 31 bases.
__device__ __forceinline__ uint64_t rc_key(uint64_t key, int k) { return rev_groups64(~key) >> (64 - 2 * k); }

// ---- wavefront (64-lane) helpers ------------------------------------------

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    uint32_t lo = __shfl_xor((unsigned)(uint32_t)v, m);
    uint32_t hi = __shfl_xor((unsigned)(uint32_t)(v >> 32), m);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    uint32_t lo = __shfl((unsigned)(uint32_t)v, src);
    uint32_t hi = __shfl((unsigned)(uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}

// Wave reductions on DPP (VALU lane moves; no LDS round trips).  row_shr 1/2/4/8
// leave each 16-lane row's total in its lane 15, row_bcast 15/31 carry row
// totals up to lane 63, which readlane broadcasts.  Callers must have all 64
// lanes active (every call site is in wave-uniform control flow).
#define PA_DPP(old, v, ctrl, rmask) __builtin_amdgcn_update_dpp((old), (v), (ctrl), (rmask), 0xf, false)
#define PA_DPP_STEPS(OP, IDENT, v)                          \
    v = OP(v, (uint32_t)PA_DPP(IDENT, (int)v, 0x111, 0xf)); \
    v = OP(v, (uint32_t)PA_DPP(IDENT, (int)v, 0x112, 0xf)); \
    v = OP(v, (uint32_t)PA_DPP(IDENT, (int)v, 0x114, 0xf)); \
    v = OP(v, (uint32_t)PA_DPP(IDENT, (int)v, 0x118, 0xf)); \
    v = OP(v, (uint32_t)PA_DPP(IDENT, (int)v, 0x142, 0xa)); \
    v = OP(v, (uint32_t)PA_DPP(IDENT, (int)v, 0x143, 0xc));

__device__ __forceinline__ uint32_t op_add(uint32_t a, uint32_t b) { return a + b; }
__device__ __forceinline__ uint32_t op_max(uint32_t a, uint32_t b) { return a > b ? a : b; }

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    PA_DPP_STEPS(op_add, 0, v);
    return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
    PA_DPP_STEPS(op_max, 0, v);
    return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ uint64_t dpp64(uint64_t v, int ctrl_sel) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    switch (ctrl_sel) {  // constant-folded: the DPP control must be an immediate
        case 0: lo = PA_DPP(0, (int)lo, 0x111, 0xf); hi = PA_DPP(0, (int)hi, 0x111, 0xf); break;
        case 1: lo = PA_DPP(0, (int)lo, 0x112, 0xf); hi = PA_DPP(0, (int)hi, 0x112, 0xf); break;
        case 2: lo = PA_DPP(0, (int)lo, 0x114, 0xf); hi = PA_DPP(0, (int)hi, 0x114, 0xf); break;
        case 3: lo = PA_DPP(0, (int)lo, 0x118, 0xf); hi = PA_DPP(0, (int)hi, 0x118, 0xf); break;
        case 4: lo = PA_DPP(0, (int)lo, 0x142, 0xa); hi = PA_DPP(0, (int)hi, 0x142, 0xa); break;
        default: lo = PA_DPP(0, (int)lo, 0x143, 0xc); hi = PA_DPP(0, (int)hi, 0x143, 0xc); break;
    }
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
    uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, lane);
    uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_max64(uint64_t v) {
#pragma unroll
    for (int s = 0; s < 6; s++) {
        const uint64_t o = dpp64(v, s);
        v = o > v ? o : v;
    }
    return readlane64(v, 63);
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int s = 0; s < 6; s++) v += dpp64(v, s);
    return readlane64(v, 63);
}

// OR across each 32-lane half of the wave; the result is valid in lanes 31 and 63.
__device__ __forceinline__ uint64_t half_or64(uint64_t v) {
#pragma unroll
    for (int s = 0; s < 5; s++) v |= dpp64(v, s);
    return v;
}

// Inclusive prefix sum across the 64 lanes.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t o = __shfl_up(v, d);
        if (lane >= d) v += o;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v) { return wave_incl_scan(v) - v; }

// ---- coherent scratch access (bypass the per-CU L1) ------------------------

template <typename T>
__device__ __forceinline__ T ld_agent(const T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_agent(T *p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace pad
