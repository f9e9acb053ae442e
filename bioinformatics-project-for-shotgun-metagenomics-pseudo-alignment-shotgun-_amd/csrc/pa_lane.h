// k_align_lane: one READ per lane -- the first pass of
// PseudoAlignment.align_reads_from_container (src/kmer.py:482-526, 563-620) for
// single-word keys on a tiled index.
//
// Included by pa_align.hip inside its anonymous namespace (uses AlignArgs,
// count_genome, first_key, F_* flags, kBlock).
//
// Why a lane per read: the wave-per-read kernel (pa_fast.h) spends most of its
// issue slots on wave-wide bookkeeping (ballots, reductions, LDS hashes) for a
// read whose windows are, almost always, one stretch of one genome.  Here each
// lane takes a whole read and proves that case cheaply:
//   1. lane_prep: the read is 2-bit packed (16-B loads, SWAR codes) into the
//      lane's LDS row; with a quality filter, the read's mean test and the
//      128-bit mask of the windows failing --min-kmer-quality come from the
//      k_quality_masks pre-pass;
//   2. five seed windows (first ... last) are probed in two rounds: the first
//      and the last, then the middle three only if neither is specific.  A
//      found seed gives the read's position on the concatenated genomes (the
//      key's first occurrence) -- the anchor; with only multi-genome seeds, up
//      to three distinct stretches are compared with the read and the one with
//      the fewest mismatching bases is walked;
//   3. lane_walk: the read XOR the genome words of the walk block gives the
//      mismatching bases; the flag planes give 128-bit masks of indexed /
//      specific / local-repeat windows; a window with exactly one mismatch is
//      settled by its neighbour bits (tile_nb, four words per round trip);
//   4. enough walked specific k-mers decide the read by a bound, without any
//      probe (k_align_lane's loop);
//   5. lane_probe_wave: the other windows (two or more mismatches, unindexed
//      genome windows, present specific neighbours) are probed by the whole
//      wave together -- each lane lists its windows, the lists are concatenated
//      in LDS, the Bloom filter drops surely absent keys and every lane probes
//      four entries per pass.  A found specific k-mer off the walk re-anchors
//      the read: it is walked again later, in a per-wave batch of 64 such reads.
// If every included k-mer is a walked window of genome g (no local repeat among
// them, the walk inside g), the reference's decision collapses: no specific
// k-mer -> AMBIGUOUS with an empty list (src/kmer.py:458-461); else exactly one
// genome -> UNIQUE g (src/kmer.py:453), and the p-check cannot demote (every
// included k-mer contains g; src/kmer.py:464-480).  Any other read -- no
// anchor, a local repeat, a non-ACGT base, a second re-anchoring, a read longer
// than the lane limits -- is queued whole for the wave kernel, which handles
// every case exactly.  A read none of whose seeds is in the index (a reverse-
// complemented read, a read of an unindexed organism) is queued for
// k_align_lane_na, which checks all its windows against the Bloom filter
// lane by lane (such reads fill whole waves there, so the per-lane loops stay
// balanced) -- nothing found: UNMAPPED; only multi-genome k-mers: AMBIGUOUS; a
// specific one: the wave kernel.

constexpr uint64_t kPosMask = (1ull << 40) - 1;  // concatenated positions (< 2^40 bases) in packed anchors
// Lane-path read shapes, by NM = 64-bit words of a read's window masks:
//   NM = 2: up to 128 windows and 176 bases (the 150-bp reads of the benchmark);
//   NM = 4: up to 256 windows and 272 bases (250-bp reads), a kernel variant of
//           its own (more registers: 3 waves per SIMD)
template <int NM>
struct LaneShape {
    static constexpr int MAXW = 64 * NM;             // windows
    static constexpr int NWD = NM == 2 ? 6 : 9;      // 64-bit words of the packed read (32 bases each)
    static constexpr int MAXLEN = 32 * NWD - 16;     // bases (the 16-B staging shift stays inside NWD words)
    static constexpr int NB = NM + 1;                // flag-plane words of the walk blocks a read spans
};
constexpr int kLaneMaxW = LaneShape<2>::MAXW;      // (the 150-bp shape: k_align_lane_na / _rc)
constexpr int kLaneMaxLen = LaneShape<2>::MAXLEN;
constexpr int kLaneWords = LaneShape<2>::NWD;
#ifndef PA_LANE_MAXMIS
#define PA_LANE_MAXMIS 40
#endif
constexpr uint32_t kLaneMaxMis = PA_LANE_MAXMIS;  // mismatching bases against the anchor stretch (else the wave kernel)
#ifndef PA_LANE_PROBES
#define PA_LANE_PROBES 4  // unwalked windows probed per lane and cooperative pass
#endif
#ifndef PA_LANE_SEEDS
#define PA_LANE_SEEDS 5   // seed windows probed per read (first ... last, evenly spread)
#endif
#ifndef PA_SEED_SLOTS
#define PA_SEED_SLOTS 2  // table slots per probe step of the seed probes
#endif
#ifndef PA_LANE_RANK_WORDS
#define PA_LANE_RANK_WORDS 6  // 2-bit words of the read its candidate stretches are ranked on (6: all)
#endif
#ifndef PA_LANE_SLOTS
#define PA_LANE_SLOTS 1   // table slots per probe step in the cooperative passes
#endif
constexpr int kPassEntries = 64 * PA_LANE_PROBES;
// Per-workgroup LDS unique counters up to this many genomes (8 B each: the
// count and the smallest batch-local read index, < 2^32); above it the lane
// kernel counts in global memory (two device-scope atomics per unique read, on
// the same G lines from every CU).  1664: a block's counters and its four
// waves' LaneWave<2> (27 KB) fit 40 KB, four blocks per CU in 160 KB -- the
// 4 waves per SIMD of the plain variant.  (Round 4 kept 512 at 12 B each: C5's
// 1200 kept genomes counted in global memory.)
#ifndef PA_TWO_WINQ
#define PA_TWO_WINQ 1  // the two-genome decision in the --min-kmer-quality variants too
#endif
#ifndef PA_LANE_LDS_GENOMES
#define PA_LANE_LDS_GENOMES 1664
#endif
constexpr uint32_t kLaneLdsGenomeCap = PA_LANE_LDS_GENOMES;

// Per-wave LDS of the lane kernel.
template <int NM>
struct __align__(16) LaneWave {
    uint64_t R[64][LaneShape<NM>::NWD + 1];  // every lane's packed read (+ a zero word), for keys of listed windows
    unsigned long long cand[64];     // a found specific unwalked window per lane: (window << 40) | position
    uint32_t flags[64];              // bits 16..: specific k-mers found off the walk, 2..15: unspecific ones,
                                     //   bit 1: the specific ones are of two or more genomes
    uint32_t hr[64];                 // unwalked windows filtered by --max-genomes
    uint32_t gsp[64];                // 1 + the genome of the specific k-mers found off the walk (0: none)
    uint16_t list[kPassEntries];     // pass entries: (lane << 8) | window
    uint32_t again_r[128];           // reads to walk again from a specific k-mer found off their walk,
    unsigned long long again_a[128]; //   and that anchor: (window << 40) | position
};

enum : int {
    LANE_UNIQUE = 0, LANE_AMB = 1, LANE_UNMAPPED = 2, LANE_DROP = 3, LANE_HARD = 4, LANE_WALK = 5, LANE_AGAIN = 6,
    LANE_NOANCHOR = 7  // no seed in the index: k_align_lane_na takes the read
};

// Word q of a register array by a runtime index (selects; no scratch).
template <int N>
__device__ __forceinline__ uint64_t word_at(const uint64_t (&v)[N], uint32_t q) {
    uint64_t r = 0;
#pragma unroll
    for (int i = 0; i < N; i++) r = (q == (uint32_t)i) ? v[i] : r;
    return r;
}

// 64 bits of the MSB-first packed words starting at bit o.
template <int N>
__device__ __forceinline__ uint64_t bits_at(const uint64_t (&v)[N], uint32_t o) {
    const uint32_t q = o >> 6, r = o & 63;
    const uint64_t hi = word_at(v, q) << r;
    return r ? (hi | (word_at(v, q + 1) >> (64 - r))) : hi;
}

// Genome containing concatenated position t (t < tile_n): a binary search over
// goff between the genomes holding positions (t >> 16) << 16 and the next
// 2^16-th (gblk) -- one genome, or two, for genomes longer than 64 kb.
__device__ __forceinline__ uint32_t genome_of(const uint64_t *goff, const uint32_t *gblk, uint64_t t) {
    uint32_t lo = gblk[t >> 16], hi = gblk[(t >> 16) + 1] + 1;  // goff[lo] <= t < goff[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (goff[mid] <= t)
            lo = mid;
        else
            hi = mid;
    }
    return lo;
}

// Up to NP table probes of one lane in flight together, NS slots (an aligned
// NS x 16-B group) per step; linear-probing order is kept exactly.  ORD: end a
// search at a key homed after the searched one (probe_past) -- off in the lane
// kernels (PA_LANE_ORD=1 turns it on for the cooperative probes): its hashes
// cost the 128-VGPR plain variant 200 B/lane of scratch.  The ordered table
// still shortens their searches of present keys.
#ifndef PA_LANE_ORD
#define PA_LANE_ORD 0
#endif
constexpr bool kLaneOrd = PA_LANE_ORD != 0 && kTableOrdered;
template <int NP, int NS = 2, bool ORD = false>
__device__ __forceinline__ void lane_probe(const AlignArgs &a, const uint64_t (&key)[NP], uint32_t act,
                                           uint32_t &found, uint32_t (&cls)[NP], uint32_t (&tpos)[NP]) {
    const Slot<1> *table = (const Slot<1> *)a.table;
    uint64_t pos[NP];
#pragma unroll
    for (int i = 0; i < NP; i++) {
        pos[i] = 0;
        if (bit(act, i)) {  // (skipped by the wave when no lane has key i)
            Key<1> kk;
            kk.w[0] = key[i];
            pos[i] = home_of<1>(kk, key_hash(kk), a.home);
        }
    }
    found = 0;
    while (act) {
        Slot<1> s[NP][NS];
        uint64_t last[NP];
#pragma unroll
        for (int i = 0; i < NP; i++)
            if (bit(act, i)) {
                const uint64_t b = pos[i] & ~(uint64_t)(NS - 1);
#pragma unroll
                for (int h = 0; h < NS; h++) s[i][h] = table[b + h];
            }
#pragma unroll
        for (int i = 0; i < NP; i++) {
            if (!bit(act, i)) continue;
            const uint64_t b = pos[i] & ~(uint64_t)(NS - 1);
            bool done = false;
#pragma unroll
            for (int h = 0; h < NS; h++) {
                if (done || b + h < pos[i]) continue;
                if (s[i][h].key[0] == EMPTY) {
                    done = true;
                } else if (s[i][h].key[0] == key[i]) {
                    done = true;
                    found |= 1u << i;
                    cls[i] = s[i][h].cls;
                    tpos[i] = s[i][h].tpos;
                }
            }
            if (done) act &= ~(1u << i);
            if (ORD && !done) last[i] = s[i][NS - 1].key[0];
            pos[i] = (b + NS == a.cap) ? 0 : b + NS;
        }
        if constexpr (ORD) {  // ordered clusters: a key homed after this one ends its search
#pragma unroll
            for (int i = 0; i < NP; i++)
                if (bit(act, i)) {
                    Key<1> r, me;
                    r.w[0] = last[i];
                    me.w[0] = key[i];
                    if (probe_past_key<1>(r, me, pos[i] == 0 ? a.cap - 1 : pos[i] - 1, a.home)) act &= ~(1u << i);
                }
        }
    }
}

// The same for keys of NW words (the lane path of 31 < k <= 63: NW = 2).
template <int NP, int NS, int NW, bool ORD = false>
__device__ __forceinline__ void lane_probe_k(const AlignArgs &a, const Key<NW> (&key)[NP], uint32_t act,
                                             uint32_t &found, uint32_t (&cls)[NP], uint32_t (&tpos)[NP]) {
    const Slot<NW> *table = (const Slot<NW> *)a.table;
    uint64_t pos[NP];
#pragma unroll
    for (int i = 0; i < NP; i++) pos[i] = bit(act, i) ? home_of<NW>(key[i], key_hash(key[i]), a.home) : 0;
    found = 0;
    while (act) {
        Slot<NW> s[NP][NS];
        Key<NW> last[NP];
#pragma unroll
        for (int i = 0; i < NP; i++)
            if (bit(act, i)) {
                const uint64_t b = pos[i] & ~(uint64_t)(NS - 1);
#pragma unroll
                for (int h = 0; h < NS; h++) s[i][h] = table[b + h];
            }
#pragma unroll
        for (int i = 0; i < NP; i++) {
            if (!bit(act, i)) continue;
            const uint64_t b = pos[i] & ~(uint64_t)(NS - 1);
            bool done = false;
#pragma unroll
            for (int h = 0; h < NS; h++) {
                if (done || b + h < pos[i]) continue;
                if (s[i][h].key[0] == EMPTY) {
                    done = true;
                    continue;
                }
                bool eq = true;
#pragma unroll
                for (int j = 0; j < NW; j++) eq &= s[i][h].key[j] == key[i].w[j];
                if (eq) {
                    done = true;
                    found |= 1u << i;
                    cls[i] = s[i][h].cls;
                    tpos[i] = s[i][h].tpos;
                }
            }
            if (done) act &= ~(1u << i);
            if (ORD && !done)
#pragma unroll
                for (int j = 0; j < NW; j++) last[i].w[j] = s[i][NS - 1].key[j];
            pos[i] = (b + NS == a.cap) ? 0 : b + NS;
        }
        if constexpr (ORD) {
#pragma unroll
            for (int i = 0; i < NP; i++)
                if (bit(act, i) && probe_past_key<NW>(last[i], key[i], pos[i] == 0 ? a.cap - 1 : pos[i] - 1, a.home))
                    act &= ~(1u << i);
        }
    }
}

#ifdef PA_STATS
#define LANE_HARD_WHY(i) atomicAdd(&a.dbg[4 + (i)], 1ull)
#else
#define LANE_HARD_WHY(i) ((void)0)
#endif

// Lane state of one read between the phases of k_align_lane.  The packed read
// itself lives in the lane's LDS row (LW.R[lane]): every lane of the wave needs
// it for the keys of listed windows, and rolled loops over LDS words keep the
// register footprint (and so the occupancy) of this latency-bound kernel low.
template <int NM>
struct LaneRead {
    int kind;                          // LANE_* (LANE_WALK: still resolving)
    uint32_t len, W;
    uint64_t anc;                      // anchor: (window << 40) | first occurrence (concatenated
                                       // position < 2^40, as the again lists hold it: one register pair)
    uint32_t acls;                     //   its class
    uint32_t g, nspec, nincl, hr;      // walk results (anchor genome, counts)
    uint64_t P[NM];                    // unwalked windows (bit w of word w / 64)
    uint64_t F[NM];                    // windows failing --min-kmer-quality (never looked up)
    uint32_t qf;                       // their number (src/kmer.py:420-423)
    uint32_t uoff;                     // walk windows whose k-mer is off the walk, present and multi-genome (neighbour bits)
};

// 64 bits of an LDS row of MSB-first packed words starting at bit o.
__device__ __forceinline__ uint64_t row_bits(const uint64_t *row, uint32_t o) {
    const uint32_t q = o >> 6, r = o & 63;
    const uint64_t hi = row[q] << r;
    return r ? (hi | (row[q + 1] >> (64 - r))) : hi;
}

// The key of window w of a packed row: k bases from bit 2 w, laid out as
// key_push builds them (the last 32 bases in the low word; for NW >= 2 the
// first k - 32 (NW - 1) in the top one, zero at k = 32 (NW - 1)).
template <int NW>
__device__ __forceinline__ Key<NW> row_key(const uint64_t *row, uint32_t w, int k) {
    Key<NW> K;
    if constexpr (NW == 1) {
        K.w[0] = row_bits(row, 2 * w) >> (64 - 2 * k);
    } else {
        static_assert(NW == 2 || NW == 3, "lane-path keys: one to three words");
#pragma unroll
        for (int j = 1; j < NW; j++) K.w[j] = row_bits(row, 2 * w + 2 * k - 64 * (NW - j));
        const int hb = 2 * k - 64 * (NW - 1);
        K.w[0] = hb ? row_bits(row, 2 * w) >> (64 - hb) : 0ull;
    }
    return K;
}

// Bytes [lo, hi) of a dword at staged position p0 that belong to the read.
__device__ __forceinline__ uint32_t in_read_mask(uint32_t p0, uint32_t shift, uint32_t len) {
    const uint32_t lo = shift > p0 ? shift - p0 : 0u, hi = shift + len > p0 ? shift + len - p0 : 0u;
    return (hi >= 4 ? 0xFFFFFFFFu : ((1u << (8 * hi)) - 1)) & (lo >= 4 ? 0u : (0xFFFFFFFFu << (8 * lo)));
}


// The walk blocks (k_tile_walk) from position A on: the 2-bit words of the
// read's span -- gw[i] = the genome's bases from A' = A & ~31 on, word i -- and,
// with PLANES, the flag planes of blocks A >> 6 .. +2.  Three 32-B blocks, a
// fourth only when the read reaches into it (every load issued before any is
// used): 1.6 128-B lines per read on average.
template <bool PLANES, int NWD = kLaneWords, int NB = 3>
__device__ __forceinline__ void lane_blocks(const AlignArgs &a, uint64_t A, uint32_t len, uint64_t (&gw)[NWD + 1],
                                            uint64_t (&pa3)[NB], uint64_t (&pb3)[NB]) {
    const uint64_t *lb = a.tile_lw + 4 * (A >> 6);
    const uint32_t r0 = (uint32_t)(A & 63), o = r0 >> 5, last = r0 + len - 1;
#pragma unroll
    for (int i = 0; i <= NWD; i++) {  // only the words holding bases of the read
        const uint32_t w = o + (uint32_t)i;
        gw[i] = 32 * w <= last ? lb[4 * (w >> 1) + (w & 1)] : 0ull;
    }
    if (PLANES) {
#pragma unroll
        for (int i = 0; i < NB; i++) {
            const ulonglong2 p = *(const ulonglong2 *)(lb + 4 * i + 2);
            pa3[i] = p.x;
            pb3[i] = p.y;
        }
    }
}

// Mismatching bases between the read (LDS row, len bases) and the genome
// words gw of the walk blocks from concatenated position A on (lane_blocks).
template <int NWD = kLaneWords>
__device__ __forceinline__ uint32_t lane_count_mismatches(const uint64_t *row, uint32_t len, uint64_t A,
                                                          const uint64_t (&gw)[NWD + 1]) {
    const uint32_t gr = (uint32_t)(2 * A & 63);
    uint32_t n = 0;
    // the read's last word holds len - 32 * qlast bases: one mask (not one per word)
    const uint32_t qlast = (len - 1) >> 5, rl = len - 32 * qlast;
    const uint64_t tail = rl >= 32 ? ~0ull : ~0ull << (64 - 2 * rl);
#pragma unroll
    for (int i = 0; i < NWD; i++) {
        if (32 * i >= (int)len) break;
        const uint64_t gwi = gr ? ((gw[i] << gr) | (gw[i + 1] >> (64 - gr))) : gw[i];
        uint64_t d = row[i] ^ gwi;
        if ((uint32_t)i == qlast) d &= tail;
        n += __popcll((d | (d >> 1)) & 0x5555555555555555ull);
    }
    return n;
}

// ~0u when the read does not fit the tile from A on.
__device__ __forceinline__ bool lane_fits(const AlignArgs &a, uint32_t len, int64_t A) {
    return A >= 0 && (uint64_t)A + len <= a.tile_n;
}

// Phase 1: qualities, packing (into the lane's LDS row), seeds -> anchor (a
// read walked again: the given anchor, cd != ~0).
template <int NM, bool NEED_Q, bool WIN_Q, bool SEEDS = true, int NW = 1>
__device__ __forceinline__ void lane_prep(const AlignArgs &a, uint64_t r, unsigned long long cd, uint64_t *row,
                                          LaneRead<NM> &S) {
    using SH = LaneShape<NM>;
    static_assert(NM == 2 || !WIN_Q, "the window-quality masks cover 128 windows");
    constexpr int NWD = SH::NWD;
    S.kind = LANE_HARD;
    S.hr = S.nspec = S.nincl = 0;
#pragma unroll
    for (int i = 0; i < NM; i++) S.F[i] = 0;
    S.qf = 0;
    S.uoff = 0;
    const int k = a.k;
    const uint32_t flags = a.prm.flags;
    const uint64_t o = a.off[r];
    const uint32_t len = (uint32_t)(a.off[r + 1] - o);
    const uint64_t o0 = o & ~15ull;
    const uint32_t shift = (uint32_t)(o & 15);
    S.len = len;
    if (len > (uint32_t)SH::MAXLEN) return (void)LANE_HARD_WHY(0);
    // ---- qualities: the read's mean test (src/kmer.py:399, 587) and the windows
    // failing --min-kmer-quality (src/kmer.py:404-408, 420-423), made for every
    // read up front by k_quality_masks
    if (NEED_Q) {
        if (a.qdrop[r]) {
            S.kind = LANE_DROP;  // dropped, not unmapped (src/kmer.py:587-589)
            return;
        }
        if (WIN_Q) {
            const uint4 m = a.qmask[r];
            S.F[0] = (uint64_t)m.x | ((uint64_t)m.y << 32);
            S.F[NM - 1] = (uint64_t)m.z | ((uint64_t)m.w << 32);  // (NM == 2 here)
            S.qf = (uint32_t)(__popcll(S.F[0]) + __popcll(S.F[NM - 1]));
        }
    }
    if (len < (uint32_t)k) {
        S.kind = LANE_UNMAPPED;  // no windows (src/kmer.py:91-92, 516-517)
        return;
    }
    const uint32_t W = len - k + 1;
    S.W = W;
    if (W > (uint32_t)SH::MAXW) return (void)LANE_HARD_WHY(0);
    // ---- 2-bit pack: staged word q (32 bases from the 16-B aligned start) from
    // chunks 2q, 2q+1; row word q-1 = the read's bases from 0 on, shifted
    const uint4 *sp = (const uint4 *)(a.seq + o0);
    const uint32_t s2 = 2 * shift;
    uint32_t bad = 0;
    uint64_t prev = 0;
    // every chunk load of the read issued before any is used (one round trip;
    // the 250-bp shape: three, of six chunks each -- its registers);
    // chunks past the read read as "AAAA" (code 0, valid)
    constexpr int CG = NM == 2 ? 2 * NWD : 6;  // chunks per round trip
#pragma unroll
    for (int g0 = 0; g0 < 2 * NWD; g0 += CG) {
    uint4 ch[CG];
#pragma unroll
    for (int c = 0; c < CG; c++)
        ch[c] = (g0 + c < 2 * NWD && 16u * (g0 + c) < shift + len)
                    ? sp[g0 + c]
                    : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
#pragma unroll
    for (int q = g0 / 2; q < (g0 + CG) / 2 && q < NWD; q++) {
        uint64_t P = 0;
        if (32u * q < shift + len) {
            const uint4 v0 = ch[2 * q - g0], v1 = ch[2 * q + 1 - g0];
            const uint32_t d[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const uint32_t cd = swar_codes(d[e]);
#ifdef PA_PACK_MASKED
                bad |= swar_bad_bytes(d[e], cd) & in_read_mask(32 * q + 4 * e, shift, len);
#else
                bad |= swar_bad_bytes(d[e], cd);  // (bytes of the neighbouring reads too: checked below)
#endif
                P |= (uint64_t)swar_pack_byte(cd) << (56 - 8 * e);
            }
        }
        if (q > 0) row[q - 1] = s2 ? ((prev << s2) | (P >> (64 - s2))) : prev;
        prev = P;
    }
    }
    row[NWD - 1] = prev << s2;  // (staged word NWD would be zero: shift + len <= 32 NWD - 1)
#ifndef PA_PACK_MASKED
    // a non-ACGT byte in the staged chunks, most likely outside the read (the
    // buffer's padding after the last read): only the read's own bytes count
    // (the chunks loaded again: nothing stays live across the packing)
    if (bad) {
        bad = 0;
#pragma unroll 1
        for (int c = 0; c < 2 * NWD; c++) {
            if (16u * c >= shift + len) break;
            const uint4 v = sp[c];
            const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; e++)
                bad |= swar_bad_bytes(d[e], swar_codes(d[e])) & in_read_mask(16u * c + 4 * e, shift, len);
        }
    }
#endif
    // (row[NWD], the zero word past the read, is cleared once per kernel:
    // a store here kept a 64-bit zero live through the whole loop and spilled it)
    if (bad) return (void)LANE_HARD_WHY(2);  // non-ACGT base: the wave kernel poisons its windows
#if defined(PA_STATS) || defined(PA_DISSECT)
    if (a.dbg_mode == 13) {  // timing dissection: stop after the packing
        S.kind = LANE_AMB;
        return;
    }
#endif
    if (!SEEDS) {  // (k_align_lane_na: the read packed, its window masks made; no seeds)
        S.kind = LANE_WALK;
        return;
    }
    if (cd != ~0ull) {  // walked again: from the specific k-mer found off the first walk
        S.anc = cd;
        S.acls = NONE;  // genome from the position
        S.kind = LANE_WALK;
        return;
    }
    const int sh = 64 - 2 * k;
    // ---- seeds: NSEED windows spread evenly from the first to the last; a
    // specific one (its genome is the read's) is preferred as the anchor
    constexpr int NSEED = PA_LANE_SEEDS;
    // (seed i's window, recomputed where needed rather than kept in registers)
    auto sw = [W](int i) { return (uint32_t)(((uint64_t)(W - 1) * (uint32_t)i) / (NSEED - 1)); };
    uint64_t skey[NW == 1 ? NSEED : 1];  // (single-word keys)
    Key<NW> skk[NW == 1 ? 1 : NSEED];    // (two- and three-word keys, 31 < k <= 95)
    if constexpr (NW == 1) {
#pragma unroll
        for (int i = 0; i < NSEED; i++) skey[i] = row_bits(row, 2 * sw(i)) >> sh;
    } else {
        (void)sh;
#pragma unroll
        for (int i = 0; i < NSEED; i++) skk[i] = row_key<NW>(row, sw(i), k);
    }
#ifndef PA_LANE_SEED_ROUNDS
#define PA_LANE_SEED_ROUNDS 2
#endif
    // two rounds: the first and the last seed, then -- only if neither is a
    // specific k-mer -- the middle ones (a random 64-B line per probe is what
    // bounds this kernel)
    uint32_t sfound = 0, scls[NSEED], stp32[NSEED];
    {
#ifndef PA_LANE_SEED_R1
#define PA_LANE_SEED_R1 (1u | (1u << (NSEED - 1)))  // the first round's seeds
#endif
        constexpr uint32_t all = (1u << NSEED) - 1, outer = PA_LANE_SEED_R1;
        uint32_t act = PA_LANE_SEED_ROUNDS > 1 ? outer : all;
#pragma unroll 1
        for (int round = 0; round < 2 && act; round++) {
            uint32_t f;
            if constexpr (NW == 1)
                lane_probe<NSEED, PA_SEED_SLOTS>(a, skey, act, f, scls, stp32);
            else
                lane_probe_k<NSEED, NW == 3 ? 1 : PA_SEED_SLOTS, NW>(a, skk, act, f, scls, stp32);  // (NW 3: registers)
            sfound |= f;
            bool spec = false;
#pragma unroll
            for (int i = 0; i < NSEED; i++) spec |= bit(f, i) && cls_of(scls[i]) < a.G && stp32[i] != NONE;
#ifndef PA_LANE_R2_ONLY_UNSEEDED
#define PA_LANE_R2_ONLY_UNSEEDED 0  // 1 (A/B): the second round only when the first found no seed at all --
                                    // C4 3.94 -> 1.95, C2 3.71 -> 1.91 G reads/s (round 6, profiles/r06/ab_r2u.txt):
                                    // a stretch named by a shared outer seed is a family's first member, and the
                                    // walk on it sends most such reads to the wave kernel
#endif
            act = (round == 0 && act != all && !spec && (!PA_LANE_R2_ONLY_UNSEEDED || f == 0)) ? all & ~outer : 0u;
#if defined(PA_STATS) || defined(PA_DISSECT)
            if (a.dbg_mode == 14) act = 0;  // timing dissection: one seed round
#endif
#ifdef PA_STATS
            if (act) atomicAdd(&a.dbg[27], 1ull);
#endif
        }
    }
    uint64_t stp[NSEED];  // first occurrences, concatenated positions (NONE64: none)
#pragma unroll
    for (int i = 0; i < NSEED; i++) {
        stp[i] = bit(sfound, i) && stp32[i] != NONE ? first_pos(scls[i], stp32[i], a.G, a.class_genomes, a.goff, a.tpos_local)
                                                     : ~0ull;
        scls[i] = cls_of(scls[i]);  // (the position bit used)
    }
    int at = -1;
#pragma unroll
    for (int pass = 0; pass < 2; pass++)
#pragma unroll
        for (int i = 0; i < NSEED; i++)
            if (at < 0 && stp[i] != ~0ull && (pass == 1 || scls[i] < a.G)) at = i;
    if (at < 0) {  // no anchor: no seed k-mer is in the index
        if (a.queue_na) S.kind = LANE_NOANCHOR;
        // the reverse complements of the outer seeds -- R' windows 0 and W - 1
        // of the read's reverse complement R' -- for k_rc_seeds (S.P[0] / S.P[1]:
        // walk fields, unused by such a read)
        if constexpr (NW == 1) {
            S.P[0] = rc_key(skey[NSEED - 1], k);
            S.P[1] = rc_key(skey[0], k);
        }
        return (void)LANE_HARD_WHY(3);
    }
    S.anc = stp[0] | ((uint64_t)sw(0) << 40);
    S.acls = scls[0];
#pragma unroll
    for (int i = 1; i < NSEED; i++)
        if (at == i) {
            S.anc = stp[i] | ((uint64_t)sw(i) << 40);
            S.acls = scls[i];
        }
    // no specific seed: the first occurrence of a multi-genome seed k-mer may
    // lie in a sibling of the read's genome (a family member), whose variants
    // would leave many windows unwalked.  Other found seeds may point to other
    // stretches: walk the one with the fewest mismatching bases (up to three)
    if (S.acls >= a.G) {
        // distinct candidate stretches (selects only: no runtime register indexing)
        const int64_t e0 = (int64_t)(S.anc & kPosMask) - (int64_t)(S.anc >> 40);
        int64_t e1 = INT64_MIN, e2 = INT64_MIN;
        uint64_t t1 = 0, t2 = 0;
        uint32_t w1 = 0, c1 = 0, w2 = 0, c2 = 0;
#pragma unroll
        for (int i = 0; i < NSEED; i++) {
            const int64_t Ai = (int64_t)stp[i] - sw(i);
            if (stp[i] == ~0ull || Ai == e0 || Ai == e1 || e2 != INT64_MIN) continue;
            if (e1 == INT64_MIN) {
                e1 = Ai;
                t1 = stp[i], w1 = sw(i), c1 = scls[i];
            } else {
                e2 = Ai;
                t2 = stp[i], w2 = sw(i), c2 = scls[i];
            }
        }
        if (e1 != INT64_MIN) {
#ifdef PA_STATS
            atomicAdd(&a.dbg[26], 1ull);
#endif
            // the stretches' walk blocks loaded together (one round trip, not one
            // per stretch), ranked on the read's first kRankWords x 32 bases:
            // the choice only steers the walk (any stretch gives the exact
            // result), and the genome words of three whole reads in flight
            // made the kernel spill.  The 250-bp shape ranks on 160 of its
            // bases (round 6: c2l250 1.58 -> 1.65 G reads/s vs 96; all 250:
            // 28 B/lane of scratch, 1.63)
#ifndef PA_LANE_RANK_WORDS4
#define PA_LANE_RANK_WORDS4 5
#endif
            constexpr int NR = NM == 2 ? PA_LANE_RANK_WORDS : PA_LANE_RANK_WORDS4;  // (the 250-bp shape: its registers)
            const uint32_t rlen = len < 32u * NR ? len : 32u * NR;
            const bool f0 = lane_fits(a, len, e0), f1 = lane_fits(a, len, e1), f2 = e2 != INT64_MIN && lane_fits(a, len, e2);
            uint64_t g0[NR + 1], g1[NR + 1], g2[NR + 1], u3[3];
            lane_blocks<false, NR>(a, f0 ? (uint64_t)e0 : 0, rlen, g0, u3, u3);
            lane_blocks<false, NR>(a, f1 ? (uint64_t)e1 : 0, rlen, g1, u3, u3);
            lane_blocks<false, NR>(a, f2 ? (uint64_t)e2 : 0, rlen, g2, u3, u3);
            const uint32_t m0 = f0 ? lane_count_mismatches<NR>(row, rlen, (uint64_t)e0, g0) : ~0u;
            const uint32_t m1 = f1 ? lane_count_mismatches<NR>(row, rlen, (uint64_t)e1, g1) : ~0u;
            const uint32_t m2 = f2 ? lane_count_mismatches<NR>(row, rlen, (uint64_t)e2, g2) : ~0u;
            uint32_t bj = 0, best = m0;
            if (m1 < best) best = m1, bj = 1;
            if (m2 < best) best = m2, bj = 2;
            if (bj == 1) {
                S.anc = t1 | ((uint64_t)w1 << 40), S.acls = c1;
            } else if (bj == 2) {
                S.anc = t2 | ((uint64_t)w2 << 40), S.acls = c2;
            }
        }
    }
    S.kind = LANE_WALK;
}

template <int NM>
__device__ __forceinline__ uint64_t lane_any(const uint64_t (&m)[NM]) {
    uint64_t x = 0;
#pragma unroll
    for (int i = 0; i < NM; i++) x |= m[i];
    return x;
}
template <int NM>
__device__ __forceinline__ uint32_t lane_popc(const uint64_t (&m)[NM]) {
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < NM; i++) x += (uint32_t)__popcll(m[i]);
    return x;
}

// Bits lo .. hi (inclusive, 0 <= lo <= hi < 64 NM) as NM mask words (constant
// word indices: selects, no scratch).
template <int NM>
__device__ __forceinline__ void range_mask(int32_t lo, int32_t hi, uint64_t (&r)[NM]) {
#pragma unroll
    for (int i = 0; i < NM; i++) {
        const int32_t b = 64 * i, l = lo - b, h = hi - b;
        r[i] = (h < 0 || l > 63) ? 0ull
                                 : ((l <= 0 ? ~0ull : (~0ull << l)) & (h >= 63 ? ~0ull : ((2ull << h) - 1)));
    }
}

// m |= v << sft over NM words, v a 32-bit word (sft may be negative: its low
// bits fall below window 0).
template <int NM>
__device__ __forceinline__ void or_at(uint64_t (&m)[NM], uint64_t v, int32_t sft) {
#pragma unroll
    for (int i = 0; i < NM; i++) {
        const int32_t s = sft - 64 * i;
        m[i] |= (s >= 64 || s <= -32) ? 0ull : (s >= 0 ? v << s : v >> (-s));
    }
}

// The NM words of planes p (NB = NM + 1 words from block A >> 6 on), shifted
// down by fr = A & 63: bit w <-> genome position A + w.
template <int NM>
__device__ __forceinline__ void shifted_planes(const uint64_t (&p)[NM + 1], uint32_t fr, uint64_t (&out)[NM]) {
#pragma unroll
    for (int i = 0; i < NM; i++) out[i] = fr ? (p[i] >> fr) | (p[i + 1] << (64 - fr)) : p[i];
}

// Phase 2: walk from the anchor; walked windows resolve from the tile, the
// others are left in S.P for the cooperative probes.  The 150-bp shape (NM =
// 2) in named words: the NM-general form (lane_walk_long) needs ~10 more
// VGPRs here, and the kernel then spills at 4 waves per SIMD.
template <bool WIN_Q, bool MG, int NW = 1>
__device__ __forceinline__ void lane_walk_150(const AlignArgs &a, const uint64_t *row, LaneRead<2> &S) {
    const int k = a.k;
    uint32_t W = S.W, len = S.len;
    // (opaque here: the masks made from len and W -- per-word tails, window
    // ranges -- are then made in each walk, not hoisted out of the kernel's
    // read loop and kept, spilled, through the probe phases)
    asm volatile("" : "+v"(W), "+v"(len));
    const uint64_t atp = S.anc & kPosMask;
    const int64_t A = (int64_t)atp - (int64_t)(S.anc >> 40);  // genome position of window 0
    const bool in_tile = A >= 0 && (uint64_t)A + W <= a.tile_n;
    const uint64_t Ac = in_tile ? (uint64_t)A : 0;
    // every load of the walk is issued before anything waits: the walk blocks
    // of the read's span -- its genome words and the flag planes of windows
    // 0..127 (bit w <-> genome position A + w; tile_lw is padded) -- and the
    // anchor genome's range
    const uint32_t gr = (uint32_t)(2 * Ac & 63);
    uint64_t gw[kLaneWords + 1], pa3[3], pb3[3];
    lane_blocks<true>(a, Ac, len, gw, pa3, pb3);
    const uint32_t g = S.acls < a.G ? S.acls : genome_of(a.goff, a.gblk, atp);
    S.g = g;
    const uint64_t gs = a.goff[g], ge = a.goff[g + 1];
    // every window of the read must lie inside the anchor genome
    if (!in_tile || A < (int64_t)gs || (uint64_t)A + W - 1 + k > ge) {
        S.kind = LANE_HARD;
        return (void)LANE_HARD_WHY(4);
    }
    const uint32_t fr = (uint32_t)(Ac & 63);
    const uint64_t PA0 = fr ? (pa3[0] >> fr) | (pa3[1] << (64 - fr)) : pa3[0];
    const uint64_t PA1 = fr ? (pa3[1] >> fr) | (pa3[2] << (64 - fr)) : pa3[1];
    const uint64_t PB0 = fr ? (pb3[0] >> fr) | (pb3[1] << (64 - fr)) : pb3[0];
    const uint64_t PB1 = fr ? (pb3[1] >> fr) | (pb3[2] << (64 - fr)) : pb3[1];
    const uint64_t IX0 = PA0 | PB0, IX1 = PA1 | PB1;  // indexed genome windows
    // ---- mismatching bases against the genome from A on.  U: windows with a
    // mismatch, V: windows with two or more; with the neighbour bits (tile_nb)
    // a window with exactly one mismatch is resolved by its bit (NP: the bits set).
    // A mismatch inside no indexed window (an N run of the genome, where the
    // read has some base) changes nothing that is decided here -- unindexed
    // windows are probed anyway -- and does not count toward the cap
    uint64_t U0 = 0, U1 = 0, V0 = 0, V1 = 0, NP0 = 0, NP1 = 0, NS0 = 0, NS1 = 0, NG0 = 0, NG1 = 0;
    uint32_t nmis = 0;
    const bool has_nb = a.tile_nb != nullptr;
    uint64_t epk = 0;  // positions e of the mismatches to look up in the neighbour bits (8 bits each, <= 8)
    uint32_t cpk = 0;  //   their substitution index (cr - cg - 1) & 3 (2 bits each)
    uint32_t nnb = 0;
    const uint32_t qlast = (len - 1) >> 5, rl = len - 32 * qlast;  // the last word holds rl bases
    const uint64_t tail = rl >= 32 ? ~0ull : ~0ull << (64 - 2 * rl);
#pragma unroll
    for (int i = 0; i < kLaneWords; i++) {
        if (32 * i >= (int)len) break;
        const uint64_t gwi = gr ? ((gw[i] << gr) | (gw[i + 1] >> (64 - gr))) : gw[i];
        uint64_t d = row[i] ^ gwi;
        if ((uint32_t)i == qlast) d &= tail;
        uint64_t m = (d | (d >> 1)) & 0x5555555555555555ull;  // one bit per mismatching base
        while (m) {
            const uint32_t j = __builtin_clzll(m) >> 1, e = 32 * i + j;
            m &= ~(1ull << (62 - 2 * j));
            const int32_t lo = (int32_t)e - k + 1 < 0 ? 0 : (int32_t)e - k + 1;
            const int32_t hi = (int32_t)e < (int32_t)W - 1 ? (int32_t)e : (int32_t)W - 1;
            if (lo > hi) continue;
            const uint64_t r0 = lo < 64 ? ((~0ull << lo) & (hi >= 63 ? ~0ull : ((2ull << hi) - 1))) : 0ull;
            const uint64_t r1 =
                hi >= 64 ? ((lo <= 64 ? ~0ull : (~0ull << (lo - 64))) & (hi >= 127 ? ~0ull : ((2ull << (hi - 64)) - 1)))
                         : 0ull;
            if (!((r0 & IX0) | (r1 & IX1))) continue;
            if (++nmis > 8) {
                // past the neighbour-bit budget (a sibling's stretch, not a few
                // sequencing errors): its windows are probed; the walked ones
                // still hold (a found specific k-mer re-anchors the read)
                if (nmis > kLaneMaxMis) {
                    S.kind = LANE_HARD;
                    return (void)LANE_HARD_WHY(5);
                }
                V0 |= r0;
                V1 |= r1;
                U0 |= r0;
                U1 |= r1;
                continue;
            }
            V0 |= U0 & r0;
            V1 |= U1 & r1;
            U0 |= r0;
            U1 |= r1;
            if (has_nb) {  // the neighbour word of the genome base at A + e and the read's base there
                const uint32_t cg = (uint32_t)(gwi >> (62 - 2 * j)) & 3u, cr = (uint32_t)(row[i] >> (62 - 2 * j)) & 3u;
                epk |= (uint64_t)e << (8 * nnb);
                cpk |= ((cr - cg - 1) & 3u) << (2 * nnb);
                nnb++;
            }
        }
    }
    // the neighbour words, four loads in flight at a time (one round trip for
    // up to four mismatches, not one per mismatch)
#pragma unroll 1
    for (uint32_t b0 = 0; b0 < nnb; b0 += 4) {
        uint64_t nv[4];
        uint32_t ng[4];
        int32_t sf[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t q = b0 + u < nnb ? b0 + u : b0;  // (a repeated load past the last)
            const uint32_t e = (uint32_t)(epk >> (8 * q)) & 255u, c = (cpk >> (2 * q)) & 3u;
            const uint64_t ni = 3 * ((uint64_t)A + e) + c;
            // (one 8-B load either way, 4-B aligned, no branch: the 12-B form's
            // 32-bit words loaded under a branch waited one by one)
            uint64_t v8;
            if constexpr (NW == 3) {  // (three-word keys: the position's summary bit of this substitution)
                const uint64_t p = (uint64_t)A + e;
                v8 = (((const uint32_t *)a.tile_nb)[p >> 3] >> (4 * (p & 7) + c)) & 1u;
                nv[u] = v8;
            } else if constexpr (NW == 2) {  // (two-word keys: 64-bit words of present neighbours, k <= 63 windows)
                v8 = ((const uint64_t *)a.tile_nb)[ni];
                nv[u] = v8;
            } else if (MG && a.tile_nbm) {  // (the words and the set-size bits in one 16-B record)
                const uint4 v = a.tile_nbm[ni];
                nv[u] = (uint64_t)v.x | ((uint64_t)v.y << 32);
                ng[u] = v.z;
            } else {
                __builtin_memcpy(&v8, (const char *)((ni < a.nb_split ? (uint64_t)(uintptr_t)a.tile_nb : a.nb_base1) +
                                                     (a.nb_spec ? 8 * ni : 4 * ni)), 8);
                nv[u] = a.nb_spec ? v8 : (uint64_t)(uint32_t)v8;
            }
            if (MG && (NW != 1 || !a.tile_nbm)) {  // --max-genomes >= 2: present with a set > mg (no branch around the load)
                const uint32_t gv = a.nbbig_ld[ni & a.nbbig_mask];
                ng[u] = a.tile_nbbig ? gv : 0u;
            } else if (!MG) {
                ng[u] = 0u;
            }
            sf[u] = b0 + u < nnb ? (int32_t)e - k + 1 : 1000;  // bit q of the word <-> window e - k + 1 + q
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (sf[u] == 1000) continue;
            // present, present and specific (the 32-bit form: present only)
            const int32_t sft = sf[u];
            if constexpr (NW == 3) {  // (a set summary bit: every window holding the mismatch may be present)
                if (nv[u]) {
                    const int32_t lo = sft < 0 ? 0 : sft, hi = sft + k - 1 < (int32_t)W - 1 ? sft + k - 1 : (int32_t)W - 1;
                    if (lo <= hi) {
                        NP0 |= lo < 64 ? ((~0ull << lo) & (hi >= 63 ? ~0ull : ((2ull << hi) - 1))) : 0ull;
                        NP1 |= hi >= 64 ? ((lo <= 64 ? ~0ull : (~0ull << (lo - 64))) &
                                           (hi >= 127 ? ~0ull : ((2ull << (hi - 64)) - 1)))
                                        : 0ull;
                    }
                }
                NS0 = NP0;
                NS1 = NP1;
                continue;
            }
            if constexpr (NW == 2) {  // (present only; up to 63 windows: bits reach the second word from any sft > 0)
                const uint64_t nbw = nv[u];
                if (sft >= 0) {
                    NP0 |= sft < 64 ? nbw << sft : 0ull;
                    NP1 |= sft >= 64 ? nbw << (sft - 64) : (sft > 0 ? nbw >> (64 - sft) : 0ull);
                } else {
                    NP0 |= nbw >> (-sft);
                }
                NS0 = NP0;
                NS1 = NP1;
                continue;
            }
            const uint64_t nbw = nv[u] & 0xFFFFFFFFull, nbs = a.nb_spec ? nv[u] >> 32 : nbw, nbg = ng[u];
#ifdef PA_STATS
            atomicAdd(&a.dbg[16], 1ull);
#endif
            if (sft >= 0) {
                NP0 |= sft < 64 ? nbw << sft : 0ull;
                NP1 |= sft >= 64 ? nbw << (sft - 64) : (sft > 32 ? nbw >> (64 - sft) : 0ull);
                NS0 |= sft < 64 ? nbs << sft : 0ull;
                NS1 |= sft >= 64 ? nbs << (sft - 64) : (sft > 32 ? nbs >> (64 - sft) : 0ull);
                NG0 |= sft < 64 ? nbg << sft : 0ull;
                NG1 |= sft >= 64 ? nbg << (sft - 64) : (sft > 32 ? nbg >> (64 - sft) : 0ull);
            } else {
                NP0 |= nbw >> (-sft);
                NS0 |= nbs >> (-sft);
                NG0 |= nbg >> (-sft);
            }
        }
    }
    if (!has_nb) {
        NP0 = NS0 = ~0ull;  // every mismatching window is probed
        NP1 = NS1 = ~0ull;
    }
    // a window with one mismatch whose k-mer is present but multi-genome needs
    // no probe: it only makes the read ambiguous (if no specific k-mer is
    // included) or sends it to the wave kernel (if one is).  Under
    // --max-genomes its set size decides whether it is included at all or
    // counted as highly redundant (src/kmer.py:425-427): known from the bits
    // when a.mg_nb (NB: present with a set larger than mg -- every present one
    // for mg <= 0, every multi-genome one for mg == 1, the per-mg bits
    // tile_nbbig above), else the present neighbours are probed
    const bool has_mg = MG;  // (a.prm.flags & F_MG)
    const int32_t mgv = a.prm.mg;
    const bool mgk = has_mg && a.mg_nb;
    const uint64_t NB0 = !mgk ? 0ull : (mgv <= 0 ? NP0 : (mgv == 1 ? NP0 & ~NS0 : NG0));
    const uint64_t NB1 = !mgk ? 0ull : (mgv <= 0 ? NP1 : (mgv == 1 ? NP1 & ~NS1 : NG1));
    const uint64_t NQ0 = !has_mg ? NS0 : (mgk ? NS0 & ~NB0 : NP0), NQ1 = !has_mg ? NS1 : (mgk ? NS1 & ~NB1 : NP1);
    // ---- walked windows: 128-bit masks from the planes.  valid: an indexed
    // genome window, spec: its k-mer is specific (to g, the genome it lies in),
    // rep: it may repeat inside the read
    const uint64_t in0 = W >= 64 ? ~0ull : ((1ull << W) - 1);
    const uint64_t in1 = W <= 64 ? 0ull : (W >= 128 ? ~0ull : ((1ull << (W - 64)) - 1));
    // windows failing the k-mer quality filter are never looked up (src/kmer.py:420-423)
    const uint64_t live0 = WIN_Q ? in0 & ~S.F[0] : in0, live1 = WIN_Q ? in1 & ~S.F[1] : in1;
    const uint64_t valid0 = IX0 & live0, valid1 = IX1 & live1;
    // probe: not an indexed genome window, or a mismatch that the neighbour
    // bits do not settle (two or more in the window, or the neighbour present)
    const uint64_t P0 = (live0 & ~valid0) | (valid0 & U0 & (V0 | NQ0));
    const uint64_t P1 = (live1 & ~valid1) | (valid1 & U1 & (V1 | NQ1));
    S.uoff = (uint32_t)(__popcll(valid0 & U0 & ~V0 & NP0 & ~NQ0 & ~NB0) + __popcll(valid1 & U1 & ~V1 & NP1 & ~NQ1 & ~NB1));
    const uint32_t hr_off = (uint32_t)(__popcll(valid0 & U0 & ~V0 & NB0) + __popcll(valid1 & U1 & ~V1 & NB1));
    const uint64_t walked0 = valid0 & ~U0, walked1 = valid1 & ~U1;
#ifdef PA_STATS
    atomicAdd(&a.dbg[17], (unsigned long long)(__popcll(live0 & ~valid0) + __popcll(live1 & ~valid1)));
    atomicAdd(&a.dbg[18], (unsigned long long)(__popcll(valid0 & U0 & V0) + __popcll(valid1 & U1 & V1)));
    atomicAdd(&a.dbg[19], (unsigned long long)(__popcll(valid0 & U0 & NQ0 & ~V0) + __popcll(valid1 & U1 & NQ1 & ~V1)));
#endif
    if ((walked0 & PB0 & ~PA0) | (walked1 & PB1 & ~PA1)) {  // a k-mer that may repeat inside the read
        S.kind = LANE_HARD;
        return (void)LANE_HARD_WHY(6);
    }
    const uint64_t spec0 = PA0 & PB0, spec1 = PA1 & PB1;
    // highly redundant walked windows (src/kmer.py:425-427): set size > mg.  A
    // specific k-mer has size 1, a multi-genome one at least 2, so only mg >= 2
    // needs the sizes of the multi-genome windows (one bit plane per mg)
    uint64_t big0 = 0, big1 = 0;
    if (has_mg) {
        const int32_t mg = a.prm.mg;
        if (mg < 1) {
            big0 = walked0;
            big1 = walked1;
        } else if (mg == 1) {
            big0 = walked0 & ~spec0;
            big1 = walked1 & ~spec1;
        } else {  // the plane "set size > mg" of this mg (k_tile_big)
            const uint64_t *bp = a.tile_big + (Ac >> 6);
            const uint64_t b0 = bp[0], b1 = bp[1], b2 = bp[2];
            big0 = walked0 & ~spec0 & (fr ? (b0 >> fr) | (b1 << (64 - fr)) : b0);
            big1 = walked1 & ~spec1 & (fr ? (b1 >> fr) | (b2 << (64 - fr)) : b1);
        }
    }
    const uint64_t incl0 = walked0 & ~big0, incl1 = walked1 & ~big1;
    const uint32_t hr = (uint32_t)(__popcll(big0) + __popcll(big1));
    const uint32_t nincl = (uint32_t)(__popcll(incl0) + __popcll(incl1));
    // a specific k-mer at a position inside genome g is specific to g
    const uint32_t nspec = (uint32_t)(__popcll(incl0 & spec0) + __popcll(incl1 & spec1));
    S.nspec = nspec;
    S.nincl = nincl;
    S.hr = hr + hr_off;  // windows, repeats included (quirk 4)
    S.P[0] = P0;
    S.P[1] = P1;
    // a read with very many unwalked windows is left to the wave kernel
    if ((uint32_t)(__popcll(P0) + __popcll(P1)) > a.lane_maxpend) {
        S.kind = LANE_HARD;
        return (void)LANE_HARD_WHY(8);
    }
}

// Phase 2 for the 250-bp shape as two walks of the 150-bp shape: windows 0 ..
// 127 (bases 0 .. 126 + k) from the anchor's genome position A, then windows
// 128 .. W - 1 (bases 128 ..) from A + 128, each with lane_walk_150's
// registers (the NM-general walk below held ~40 more and spilled 68-76
// B/lane).  The halves' walked windows are distinct k-mers exactly as one
// walk's are: a window whose k-mer starts again within 255 positions -- any
// other window of the read -- carries the local-repeat flag and sends the read
// to the wave kernel; so their counts add, and their unwalked windows are the
// read's (P words 0-1 and 2-3).  Both halves are placed in the anchor's genome.
#ifndef PA_LANE_HALVES
#define PA_LANE_HALVES 1
#endif
template <bool MG>
__device__ __forceinline__ void lane_walk_halves(const AlignArgs &a, const uint64_t *row, LaneRead<4> &S) {
    const int64_t A = (int64_t)(S.anc & kPosMask) - (int64_t)(S.anc >> 40);  // genome position of window 0
    const uint32_t len = S.len, W = S.W;
    S.nspec = S.nincl = S.hr = S.uoff = 0;
    S.P[2] = S.P[3] = 0;
    // (one copy of the walk in a loop, not two inlined ones: the copies' loop
    // invariants were hoisted side by side and spilled)
#pragma unroll 1
    for (uint32_t h = 0; h < 2; h++) {
        LaneRead<2> H;
        H.kind = LANE_WALK;
        H.F[0] = H.F[1] = 0;
        if (h == 0) {
            H.len = W > 128 ? 127 + (uint32_t)a.k : len;
            H.W = W > 128 ? 128u : W;
            H.anc = S.anc;
            H.acls = S.acls;
        } else {
            H.len = len - 128;
            H.W = W - 128;
            H.anc = (uint64_t)(A + 128);  // (window 0 of the second half at A + 128; A >= 0: the first half checked it)
            H.acls = S.g;                 // (the first half's genome: a genome id < G)
        }
        lane_walk_150<false, MG, 1>(a, row + 4 * h, H);
        if (h == 0) S.g = H.g;
        S.kind = H.kind;
        S.nspec += H.nspec, S.nincl += H.nincl, S.hr += H.hr, S.uoff += H.uoff;
        if (h == 0) {
            S.P[0] = H.P[0], S.P[1] = H.P[1];
        } else {
            S.P[2] = H.P[0], S.P[3] = H.P[1];
        }
        if (S.kind != LANE_WALK || W <= 128) break;
    }
}

// Phase 2 for the 250-bp shape (NM = 4; lane_walk_150 below states the steps):
// the same walk over NM-word window masks (PA_LANE_HALVES=0; else
// lane_walk_halves).
template <int NM, bool WIN_Q, bool MG>
__device__ __forceinline__ void lane_walk_long(const AlignArgs &a, const uint64_t *row, LaneRead<NM> &S) {
    using SH = LaneShape<NM>;
    constexpr int NWD = SH::NWD;
    const int k = a.k;
    const uint32_t W = S.W, len = S.len;
    const uint64_t atp = S.anc & kPosMask;
    const int64_t A = (int64_t)atp - (int64_t)(S.anc >> 40);  // genome position of window 0
    const bool in_tile = A >= 0 && (uint64_t)A + W <= a.tile_n;
    const uint64_t Ac = in_tile ? (uint64_t)A : 0;
    // every load of the walk is issued before anything waits: the walk blocks
    // of the read's span -- its genome words and the flag planes of windows
    // 0 .. 64 NM - 1 (bit w <-> genome position A + w; tile_lw is padded) --
    // and the anchor genome's range
    const uint32_t gr = (uint32_t)(2 * Ac & 63);
    uint64_t gw[NWD + 1], pa3[NM + 1], pb3[NM + 1];
    lane_blocks<true, NWD, NM + 1>(a, Ac, len, gw, pa3, pb3);
    const uint32_t g = S.acls < a.G ? S.acls : genome_of(a.goff, a.gblk, atp);
    S.g = g;
    const uint64_t gs = a.goff[g], ge = a.goff[g + 1];
    // every window of the read must lie inside the anchor genome
    if (!in_tile || A < (int64_t)gs || (uint64_t)A + W - 1 + k > ge) {
        S.kind = LANE_HARD;
        return (void)LANE_HARD_WHY(4);
    }
    const uint32_t fr = (uint32_t)(Ac & 63);
    uint64_t PA[NM], PB[NM];  // (indexed genome windows: PA | PB, recomputed where used -- registers)
    shifted_planes<NM>(pa3, fr, PA);
    shifted_planes<NM>(pb3, fr, PB);
    // ---- mismatching bases against the genome from A on.  U: windows with a
    // mismatch, V: windows with two or more; with the neighbour bits (tile_nb)
    // a window with exactly one mismatch is resolved by its bit (NP: the bits set).
    // A mismatch inside no indexed window (an N run of the genome, where the
    // read has some base) changes nothing that is decided here -- unindexed
    // windows are probed anyway -- and does not count toward the cap
    uint64_t U[NM], V[NM], NP[NM], NS[NM], NG[NM];
#pragma unroll
    for (int i = 0; i < NM; i++) U[i] = V[i] = NP[i] = NS[i] = NG[i] = 0;
    uint32_t nmis = 0;
    const bool has_nb = a.tile_nb != nullptr;
    uint64_t epk = 0;  // positions e of the mismatches to look up in the neighbour bits (low 8 bits each, <= 8)
    uint32_t ehi = 0;  //   and bit 8 of each (positions up to 271)
    uint32_t cpk = 0;  //   their substitution index (cr - cg - 1) & 3 (2 bits each)
    uint32_t nnb = 0;
    const uint32_t qlast = (len - 1) >> 5, rl = len - 32 * qlast;  // the last word holds rl bases
    const uint64_t tail = rl >= 32 ? ~0ull : ~0ull << (64 - 2 * rl);
#pragma unroll
    for (int i = 0; i < NWD; i++) {
        if (32 * i >= (int)len) break;
        const uint64_t gwi = gr ? ((gw[i] << gr) | (gw[i + 1] >> (64 - gr))) : gw[i];
        uint64_t d = row[i] ^ gwi;
        if ((uint32_t)i == qlast) d &= tail;
        uint64_t m = (d | (d >> 1)) & 0x5555555555555555ull;  // one bit per mismatching base
        while (m) {
            const uint32_t j = __builtin_clzll(m) >> 1, e = 32 * i + j;
            m &= ~(1ull << (62 - 2 * j));
            const int32_t lo = (int32_t)e - k + 1 < 0 ? 0 : (int32_t)e - k + 1;
            const int32_t hi = (int32_t)e < (int32_t)W - 1 ? (int32_t)e : (int32_t)W - 1;
            if (lo > hi) continue;
            uint64_t rr[NM];
            range_mask<NM>(lo, hi, rr);
            uint64_t hit = 0;
#pragma unroll
            for (int q = 0; q < NM; q++) hit |= rr[q] & (PA[q] | PB[q]);
            if (!hit) continue;
            if (++nmis > 8) {
                // past the neighbour-bit budget (a sibling's stretch, not a few
                // sequencing errors): its windows are probed; the walked ones
                // still hold (a found specific k-mer re-anchors the read)
                if (nmis > kLaneMaxMis) {
                    S.kind = LANE_HARD;
                    return (void)LANE_HARD_WHY(5);
                }
#pragma unroll
                for (int q = 0; q < NM; q++) {
                    V[q] |= rr[q];
                    U[q] |= rr[q];
                }
                continue;
            }
#pragma unroll
            for (int q = 0; q < NM; q++) {
                V[q] |= U[q] & rr[q];
                U[q] |= rr[q];
            }
            if (has_nb) {  // the neighbour word of the genome base at A + e and the read's base there
                const uint32_t cg = (uint32_t)(gwi >> (62 - 2 * j)) & 3u, cr = (uint32_t)(row[i] >> (62 - 2 * j)) & 3u;
                epk |= (uint64_t)(e & 255u) << (8 * nnb);
                ehi |= (e >> 8) << nnb;
                cpk |= ((cr - cg - 1) & 3u) << (2 * nnb);
                nnb++;
            }
        }
    }
    // the neighbour words, four loads in flight at a time (one round trip for
    // up to four mismatches, not one per mismatch)
#pragma unroll 1
    for (uint32_t b0 = 0; b0 < nnb; b0 += 4) {
        uint64_t nv[4];
        uint32_t ng[4];
        int32_t sf[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t q = b0 + u < nnb ? b0 + u : b0;  // (a repeated load past the last)
            const uint32_t e = ((uint32_t)(epk >> (8 * q)) & 255u) | (((ehi >> q) & 1u) << 8), c = (cpk >> (2 * q)) & 3u;
            const uint64_t ni = 3 * ((uint64_t)A + e) + c;
            // (one 8-B load either way, 4-B aligned, no branch: the 12-B form's
            // 32-bit words loaded under a branch waited one by one)
            uint64_t v8;
            __builtin_memcpy(&v8, (const char *)((ni < a.nb_split ? (uint64_t)(uintptr_t)a.tile_nb : a.nb_base1) +
                                                 (a.nb_spec ? 8 * ni : 4 * ni)), 8);
            nv[u] = a.nb_spec ? v8 : (uint64_t)(uint32_t)v8;
            if (MG) {  // --max-genomes >= 2: present with a set > mg (no branch around the load)
                const uint32_t gv = a.nbbig_ld[ni & a.nbbig_mask];
                ng[u] = a.tile_nbbig ? gv : 0u;
            } else {
                ng[u] = 0u;
            }
            sf[u] = b0 + u < nnb ? (int32_t)e - k + 1 : 1000;  // bit q of the word <-> window e - k + 1 + q
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (sf[u] == 1000) continue;
            // present, present and specific (the 32-bit form: present only)
            const uint64_t nbw = nv[u] & 0xFFFFFFFFull, nbs = a.nb_spec ? nv[u] >> 32 : nbw, nbg = ng[u];
#ifdef PA_STATS
            atomicAdd(&a.dbg[16], 1ull);
#endif
            const int32_t sft = sf[u];
            or_at<NM>(NP, nbw, sft);
            or_at<NM>(NS, nbs, sft);
            if (MG) or_at<NM>(NG, nbg, sft);
        }
    }
    if (!has_nb) {
#pragma unroll
        for (int q = 0; q < NM; q++) NP[q] = NS[q] = ~0ull;  // every mismatching window is probed
    }
    // a window with one mismatch whose k-mer is present but multi-genome needs
    // no probe: it only makes the read ambiguous (if no specific k-mer is
    // included) or sends it to the wave kernel (if one is).  Under
    // --max-genomes its set size decides whether it is included at all or
    // counted as highly redundant (src/kmer.py:425-427): known from the bits
    // when a.mg_nb (NB: present with a set larger than mg -- every present one
    // for mg <= 0, every multi-genome one for mg == 1, the per-mg bits
    // tile_nbbig above), else the present neighbours are probed
    const bool has_mg = MG;  // (a.prm.flags & F_MG)
    const int32_t mgv = a.prm.mg;
    const bool mgk = has_mg && a.mg_nb;
    // ---- walked windows: masks from the planes.  valid: an indexed genome
    // window, spec: its k-mer is specific (to g, the genome it lies in), rep:
    // it may repeat inside the read
    uint64_t P[NM], walked[NM];
    uint32_t uoff = 0, hr_off = 0, npend = 0;
    uint64_t reps = 0;
#pragma unroll
    for (int q = 0; q < NM; q++) {
        const int32_t wl = (int32_t)W - 64 * q;
        const uint64_t in = wl >= 64 ? ~0ull : (wl <= 0 ? 0ull : ((1ull << wl) - 1));
        const uint64_t NB = !mgk ? 0ull : (mgv <= 0 ? NP[q] : (mgv == 1 ? NP[q] & ~NS[q] : NG[q]));
        const uint64_t NQ = !has_mg ? NS[q] : (mgk ? NS[q] & ~NB : NP[q]);
        // windows failing the k-mer quality filter are never looked up (src/kmer.py:420-423)
        const uint64_t live = WIN_Q ? in & ~S.F[q] : in;
        const uint64_t valid = (PA[q] | PB[q]) & live;
        // probe: not an indexed genome window, or a mismatch that the neighbour
        // bits do not settle (two or more in the window, or the neighbour present)
        P[q] = (live & ~valid) | (valid & U[q] & (V[q] | NQ));
        uoff += (uint32_t)__popcll(valid & U[q] & ~V[q] & NP[q] & ~NQ & ~NB);
        hr_off += (uint32_t)__popcll(valid & U[q] & ~V[q] & NB);
        walked[q] = valid & ~U[q];
        reps |= walked[q] & PB[q] & ~PA[q];
        npend += (uint32_t)__popcll(P[q]);
#ifdef PA_STATS
        atomicAdd(&a.dbg[17], (unsigned long long)__popcll(live & ~valid));
        atomicAdd(&a.dbg[18], (unsigned long long)__popcll(valid & U[q] & V[q]));
        atomicAdd(&a.dbg[19], (unsigned long long)__popcll(valid & U[q] & NQ & ~V[q]));
#endif
    }
    S.uoff = uoff;
    if (reps) {  // a k-mer that may repeat inside the read
        S.kind = LANE_HARD;
        return (void)LANE_HARD_WHY(6);
    }
    // highly redundant walked windows (src/kmer.py:425-427): set size > mg.  A
    // specific k-mer has size 1, a multi-genome one at least 2, so only mg >= 2
    // needs the sizes of the multi-genome windows (one bit plane per mg)
    uint32_t hr = 0, nincl = 0, nspec = 0;
    uint64_t bb[NM + 1];
    if (has_mg && a.prm.mg >= 2) {  // the plane "set size > mg" of this mg (k_tile_big)
        const uint64_t *bp = a.tile_big + (Ac >> 6);
#pragma unroll
        for (int q = 0; q <= NM; q++) bb[q] = bp[q];
    }
#pragma unroll
    for (int q = 0; q < NM; q++) {
        const uint64_t spec = PA[q] & PB[q];
        uint64_t big = 0;
        if (has_mg) {
            const int32_t mg = a.prm.mg;
            if (mg < 1)
                big = walked[q];
            else if (mg == 1)
                big = walked[q] & ~spec;
            else
                big = walked[q] & ~spec & (fr ? (bb[q] >> fr) | (bb[q + 1] << (64 - fr)) : bb[q]);
        }
        const uint64_t incl = walked[q] & ~big;
        hr += (uint32_t)__popcll(big);
        nincl += (uint32_t)__popcll(incl);
        // a specific k-mer at a position inside genome g is specific to g
        nspec += (uint32_t)__popcll(incl & spec);
        S.P[q] = P[q];
    }
    S.nspec = nspec;
    S.nincl = nincl;
    S.hr = hr + hr_off;  // windows, repeats included (quirk 4)
    // a read with very many unwalked windows is left to the wave kernel
    if (npend > a.lane_maxpend * (uint32_t)(NM / 2)) {
        S.kind = LANE_HARD;
        return (void)LANE_HARD_WHY(8);
    }
}

// Phase 3 (whole wave): probe windows Q of the walking lanes; `reset`
// clears the lanes' outcomes first (LW.flags / hr / cand accumulate otherwise).
// TWO: also note the genome of the specific k-mers found (LW.hr, flags bit 1),
// for k_align_lane's two-genome decision
template <int NM, int NW = 1, bool TWO = false>
__device__ __forceinline__ void lane_probe_wave(const AlignArgs &a, LaneWave<NM> &LW, const LaneRead<NM> &S,
                                                const uint64_t (&Qin)[NM], bool reset) {
    const int lane = lane_id();
    const int sh = 64 - 2 * a.k;
    const bool walking = S.kind == LANE_WALK;
    if (reset) {
        LW.flags[lane] = 0;
        LW.hr[lane] = 0;
        if (TWO) LW.gsp[lane] = 0;
        LW.cand[lane] = ~0ull;
    }
    uint64_t Q[NM];
    uint32_t c = 0;
#pragma unroll
    for (int q = 0; q < NM; q++) {
        Q[q] = walking ? Qin[q] : 0ull;
        c += (uint32_t)__popcll(Q[q]);
    }
    const uint32_t incl = wave_incl_scan(c);
    const uint32_t pre = incl - c;
    const uint32_t total = __shfl(incl, 63);
#ifdef PA_STATS
    if (lane == 0 && total) atomicAdd(&a.dbg[14], (unsigned long long)total);
#endif
    for (uint32_t base = 0; base < total; base += kPassEntries) {
        // this pass's entries of the lane: global indices [max(pre, base), min(pre + c, base + 256))
        const uint32_t lo = max(pre, base), hi = min(pre + c, base + (uint32_t)kPassEntries);
        for (uint32_t e = lo; e < hi; e++) {
            uint32_t w = 0;
            if constexpr (NM == 2) {
                if (Q[0]) {
                    w = __builtin_ctzll(Q[0]);
                    Q[0] &= Q[0] - 1;
                } else {
                    w = 64 + __builtin_ctzll(Q[1]);
                    Q[1] &= Q[1] - 1;
                }
            } else {
                bool got = false;
#pragma unroll
                for (int q = 0; q < NM; q++) {
                    if (!got && Q[q]) {
                        w = 64 * q + __builtin_ctzll(Q[q]);
                        Q[q] &= Q[q] - 1;
                        got = true;
                    }
                }
            }
            LW.list[e - base] = (uint16_t)((lane << 8) | w);
        }
        wave_sync();
        const uint32_t cnt = min(total - base, (uint32_t)kPassEntries);
        constexpr int NPR = PA_LANE_PROBES;
        uint64_t key4[NW == 1 ? NPR : 1];  // (single-word keys)
        Key<NW> kk4[NW == 1 ? 1 : NPR];    // (two-word keys)
        uint32_t tag4[NPR], act = 0;
        // entry 64 i + lane: with fewer than 64 (NPR - 1) entries the last keys
        // of every lane are idle, and their hashing and probing is skipped
#pragma unroll
        for (int i = 0; i < NPR; i++) {
            const uint32_t e = 64 * i + lane;
            if constexpr (NW == 1) key4[i] = 0;
            else kk4[i] = Key<NW>{};
            tag4[i] = 0;
            if (e < cnt) {
                const uint32_t t = LW.list[e];
                const uint64_t *row = LW.R[t >> 8];
                if constexpr (NW == 1) {
                    const uint32_t o = 2 * (t & 255), q = o >> 6, rr = o & 63;
                    const uint64_t hi64 = row[q] << rr;
                    key4[i] = (rr ? (hi64 | (row[q + 1] >> (64 - rr))) : hi64) >> sh;
                } else {
                    kk4[i] = row_key<NW>(row, t & 255, a.k);
                }
                tag4[i] = t;
                act |= 1u << i;
            }
        }
        if (a.bloom) {  // windows whose key is surely absent are not probed
            uint64_t bw[NPR], bm[NPR];
#pragma unroll
            for (int i = 0; i < NPR; i++) {
                bw[i] = ~0ull;
                bm[i] = 0;
                if (64u * i < cnt) {  // (uniform)
                    uint64_t wi;
                    if constexpr (NW == 1)
                        bloom_word(key4[i], a.k, a.bloom_lg, wi, bm[i]);
                    else if constexpr (NW == 2)
                        bloom_word2(kk4[i], a.bloom_lg, wi, bm[i]);
                    else
                        bloom_word3(kk4[i], a.bloom_lg, wi, bm[i]);
                    bw[i] = a.bloom[bit(act, i) ? wi : 0ull];  // (no branch around the load: they issue together)
                    if (!bit(act, i)) bm[i] = 0;
                }
            }
#pragma unroll
            for (int i = 0; i < NPR; i++)
                if ((bw[i] & bm[i]) != bm[i]) act &= ~(1u << i);
#ifdef PA_STATS
            atomicAdd(&a.dbg[25], (unsigned long long)__popc(act));
#endif
        }
        uint32_t f, c4[NPR], t4[NPR];
        if constexpr (NW == 1)
            lane_probe<NPR, PA_LANE_SLOTS, kLaneOrd>(a, key4, act, f, c4, t4);
        else
            lane_probe_k<NPR, PA_LANE_SLOTS, NW, kLaneOrd>(a, kk4, act, f, c4, t4);
#pragma unroll
        for (int i = 0; i < NPR; i++) {
            if (!bit(f, i)) continue;
            const uint32_t o = tag4[i] >> 8, w = tag4[i] & 255;
            const uint32_t cl = cls_of(c4[i]);
            if ((a.prm.flags & F_MG) && (int64_t)class_size_of(cl, a.G, a.class_genomes) > (int64_t)a.prm.mg) {
                atomicAdd(&LW.hr[o], 1u);  // highly redundant: counted, never included
            } else if (cl >= a.G) {
                atomicAdd(&LW.flags[o], 4u);  // unspecific: counted in bits 2..
            } else {
                atomicAdd(&LW.flags[o], 1u << 16);
                if (TWO) {  // (specific: the class is the genome) one genome, or bit 1
                    const uint32_t was = atomicCAS(&LW.gsp[o], 0u, cl + 1);
                    if (was != 0u && was != cl + 1) atomicOr(&LW.flags[o], 2u);
                }
                atomicMin(&LW.cand[o], ((unsigned long long)w << 40) | first_pos(c4[i], t4[i], a.G, a.class_genomes,
                                                                               a.goff, a.tpos_local));
            }
        }
        wave_sync();  // the list is rewritten by the next pass
    }
}

// Waves per SIMD the register allocation must allow.  The kernel is bound by
// the latency of random table / tile reads, so occupancy pays as long as the
// spills stay out of the walk: without --max-genomes and the window-quality
// mask (MG, WIN_Q false: C2) it needs ~145 VGPRs and runs at 4 waves per SIMD
// (128 VGPRs, 32 B/lane of scratch outside the walk loops; round-2 A/B on C2:
// 3.48 vs 3.36 G reads/s at 3).  With them (C3) it needs ~170 and spills
// 100-140 B/lane at 4, so it runs at 3 (no scratch).
#ifndef PA_LANE_WAVES
#define PA_LANE_WAVES 4
#endif

#ifndef PA_LANE_WAVES_Q
#define PA_LANE_WAVES_Q 4  // (--min-kmer-quality: 128 VGPRs, 12 B/lane of scratch; c3raw +1 % vs 3 waves at 140 VGPRs)
#endif
#ifndef PA_LANE_WAVES_LONG
#define PA_LANE_WAVES_LONG 4  // the 250-bp shape (NM = 4, two 150-bp walks: 128 VGPRs, no scratch; c2l250 1.57 vs 1.45 G reads/s at 3 waves)
#endif
#ifndef PA_LANE_WAVES_MG
#define PA_LANE_WAVES_MG 4  // --max-genomes (C3): 128 VGPRs, no scratch once the walk's len / W are opaque (round 4: 146-151 at 3)
#endif
#ifndef PA_LANE_WAVES_W
#define PA_LANE_WAVES_W 3  // two- and three-word keys (~168 VGPRs; at 4 they spill 84-180 B/lane)
#endif
template <bool NEED_Q, bool WIN_Q, bool MG, int NM = 2, int NW = 1>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(
    NM == 4 ? PA_LANE_WAVES_LONG
            : (NW >= 2 ? PA_LANE_WAVES_W : (WIN_Q ? PA_LANE_WAVES_Q : (MG ? PA_LANE_WAVES_MG : PA_LANE_WAVES))))))
void k_align_lane(AlignArgs a) {
    using LW_t = LaneWave<NM>;
    constexpr int NWD = LaneShape<NM>::NWD;
    extern __shared__ __align__(16) unsigned char smem[];
    const uint32_t G = a.G;
    const int lane = lane_id();
    const bool lds = G <= kLaneLdsGenomeCap;
    const size_t cnt_bytes = lds ? ((size_t)G * 8 + 15) / 16 * 16 : 0;
    uint32_t *first = (uint32_t *)smem;  // the smallest batch-local index of a unique read of g (first_key rank 0)
    uint32_t *uniq = first + (lds ? G : 0);
    // (the wave's index read from lane 0: the LDS base is then a scalar, not a VGPR held all kernel long)
    LW_t &LW = ((LW_t *)(smem + cnt_bytes))[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];
    if (lds) {
        for (uint32_t i = threadIdx.x; i < G; i += kBlock) {
            first[i] = ~0u;
            uniq[i] = 0;
        }
        __syncthreads();
    }
    // Register budget: this kernel runs at 3-4 waves per SIMD (PA_LANE_WAVES), so the
    // loop's bookkeeping lives in SGPRs (wave-uniform: chunk cursor, read
    // counts by ballot) and LDS (per-lane window counters), not in VGPRs.
    uint32_t n_uniq = 0, n_amb = 0, n_unm = 0, n_drop = 0;  // wave totals (scalar)
    // window counters of the settled reads, wave totals (scalar): summed
    // across the wave per chunk (a per-lane LDS slot kept its address live in
    // a VGPR all kernel long, and it spilled)
    uint64_t n_hr = 0, n_qf = 0;
    LW.R[lane][NWD] = 0;  // the zero word past every read (lane_prep writes words 0 .. NWD - 1)
    // Each wave takes chunks of 64 consecutive reads; a read whose walk finds a
    // specific k-mer off it is walked again from that k-mer, but later, with 63
    // others (a list per wave), so that the 3 % of such reads do not hold whole
    // waves for a second walk.  Every decision below is wave-uniform.
    const uint64_t n_chunks = (a.n + 63) / 64, wave_stride = (uint64_t)gridDim.x * kWaves;
    uint64_t chunk = (uint64_t)blockIdx.x * kWaves + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // this wave's segment of the seedless reads' queue (a.na_seg): entries
    // seg_base ... seg_base + seg_na (scalar)
    const uint32_t wave_id = (uint32_t)chunk;
    const uint64_t seg_base = (uint64_t)wave_id * a.seg_cap;
    uint32_t seg_na = 0;
    uint32_t n_again = 0;  // entries in LW.again_r / again_a
    while (true) {
        uint32_t r = ~0u;  // (a batch holds < 2^32 reads: pa::align)
        unsigned long long cd = ~0ull;
        bool again_batch = false;
        if (n_again >= 64 || (chunk >= n_chunks && n_again > 0)) {
            const uint32_t take = n_again < 64 ? n_again : 64;
            if ((uint32_t)lane < take) {
                r = LW.again_r[n_again - take + lane];
                cd = LW.again_a[n_again - take + lane];
            }
            n_again -= take;
            again_batch = true;
        } else if (chunk < n_chunks) {
            r = chunk * 64 + lane < a.n ? (uint32_t)(chunk * 64 + lane) : ~0u;
            chunk += wave_stride;
        } else {
            break;
        }
        LaneRead<NM> S;
        S.kind = LANE_UNMAPPED + 100;  // (past the end: counted nowhere)
        wave_sync();  // the previous read's rows (and the taken list entries) are done with
        // (the lane's row address made again at each use, through an opaque
        // copy of the lane id: kept live across the phases it was spilled)
        auto my_row = [&]() -> uint64_t * {
            uint32_t l = (uint32_t)lane;
            asm volatile("" : "+v"(l));
            return LW.R[l];
        };
        if (r != ~0u) lane_prep<NM, NEED_Q, WIN_Q, true, NW>(a, r, cd, my_row(), S);
#if defined(PA_STATS) || defined(PA_DISSECT)
        if (a.dbg_mode == 10 && S.kind == LANE_WALK) S.kind = LANE_AMB;  // timing dissection: stop after the seeds
#endif
#pragma unroll 1
        for (int attempt = again_batch ? 1 : 0; attempt < 2; attempt++) {
            if (S.kind == LANE_WALK) {
                if constexpr (NM == 2)
                    lane_walk_150<WIN_Q, MG, NW>(a, my_row(), S);
                else
                    if constexpr (NM == 4 && !WIN_Q && NW == 1 && PA_LANE_HALVES)
                        lane_walk_halves<MG>(a, my_row(), S);
                    else
                        lane_walk_long<NM, WIN_Q, MG>(a, my_row(), S);
            }
#if defined(PA_STATS) || defined(PA_DISSECT)
            if (a.dbg_mode == 11 && S.kind == LANE_WALK) S.kind = LANE_AMB;  // stop after the walk
#endif
            if (!__ballot(S.kind == LANE_WALK)) break;
            // Enough walked specific k-mers decide the read whatever the windows
            // off the walk hold.  X = windows whose k-mer may be in the index off
            // the walk (unwalked, not known absent).  Any other genome h has at
            // most X specific k-mers and at most (nincl - nspec) + X in total,
            // while g has at least nspec and nincl (src/kmer.py:444-480): with
            // nspec >= X + max(m, 1) g is the strict top and unique, and with
            // X - nspec <= p no genome's total exceeds g's by more than p.
            // Under --max-genomes the filtered_hr_kmers count needs the set size
            // of every window found off the walk: only when every one is known
            // from the bits (a.mg_nb, nothing left to probe).
            if (S.kind == LANE_WALK && S.nspec > 0 && (!MG || (a.mg_nb && !lane_any(S.P)))) {
                const int64_t X = (int64_t)(lane_popc(S.P) + S.uoff);
                const int64_t ns = (int64_t)S.nspec;
                if (ns >= X + (a.prm.m > 0 ? a.prm.m : 1) && (a.prm.p < 0 || X - ns <= a.prm.p)) {
                    S.kind = LANE_UNIQUE;
#ifdef PA_STATS
                    atomicAdd(&a.dbg[23], 1ull);
#endif
                }
            }
            // a multi-genome k-mer off the walk next to walked specific ones
            // under --max-genomes (its set size decides): the wave kernel, without probing
            if (S.kind == LANE_WALK && S.uoff && S.nspec > 0 && MG && !a.mg_nb) {
                S.kind = LANE_HARD;
                LANE_HARD_WHY(7);
                LANE_HARD_WHY(16);
            }
            lane_probe_wave<NM, NW, PA_TWO_WINQ || !WIN_Q>(a, LW, S, S.P, true);
            if (S.kind == LANE_WALK) {
                const uint32_t fl = LW.flags[lane];
                const uint32_t nsoff = fl >> 16;  // specific k-mers off the walk (windows)
                // Specific k-mers of one other genome h off the walk, fewer than
                // g's walked ones: with ns = nspec (distinct: no local repeat
                // among the walked windows) and c = nsoff >= h's distinct
                // specific k-mers, ns >= c + max(m, 1) makes g the strict top
                // and unique (src/kmer.py:446-456); any genome's total is then
                // at most (nincl - nspec) + noff + c and g's at least nincl, so
                // with noff + c - ns <= p the p-check cannot demote
                // (src/kmer.py:464-480).  (A specific k-mer of g itself off the
                // walk may repeat a walked one: not decided here.)
                bool two = false;
                if ((PA_TWO_WINQ || !WIN_Q) && (!MG || a.mg_nb) && nsoff && !(fl & 2u) && LW.gsp[lane] != S.g + 1) {
                    const int64_t ns = (int64_t)S.nspec, c = (int64_t)nsoff;
                    const int64_t noff = (int64_t)(((fl >> 2) & 0x3FFFu) + S.uoff);
                    two = ns >= c + (a.prm.m > 0 ? a.prm.m : 1) && (a.prm.p < 0 || noff + c - ns <= a.prm.p);
                }
                if (two) {
                    S.kind = LANE_UNIQUE;
                    if (MG) S.hr += LW.hr[lane];
#ifdef PA_STATS
                    atomicAdd(&a.dbg[24], 1ull);  // (with the one-genome case below)
#endif
                } else if (nsoff) {  // a specific k-mer off the walk: walk again from it (once)
#if defined(PA_STATS) || defined(PA_DISSECT)
                    if (a.dbg_mode == 12) S.kind = LANE_AMB;  // timing dissection: no second walk
#endif
                    if (S.kind != LANE_WALK) {
                    } else if (attempt == 0) {  // later, in a batch of such reads
#ifdef PA_STATS
                        atomicAdd(&a.dbg[15], 1ull);
#endif
                        S.kind = LANE_AGAIN;
                    } else {
                        S.kind = LANE_HARD;
                        LANE_HARD_WHY(7);
                        LANE_HARD_WHY(17);
                    }
                } else {
                    if (MG) S.hr += LW.hr[lane];
                    const uint32_t noff = ((fl >> 2) & 0x3FFFu) + S.uoff;  // unspecific k-mers off the walk
                    if (noff) {
                        // Only g has specific k-mers (the walked ones; none off the
                        // walk), so the specific map is {g} and the read is UNIQUE g
                        // (src/kmer.py:452-454) unless the total counts demote it:
                        // any h has at most (nincl - nspec) + noff distinct included
                        // k-mers, g at least nincl, so with noff - nspec <= p no total
                        // exceeds g's by more than p (src/kmer.py:471-474).  Under
                        // --max-genomes only when the uoff windows' set sizes are known.
                        if (S.nspec > 0 && (!MG || a.mg_nb) &&
                            (a.prm.p < 0 || (int64_t)noff - (int64_t)S.nspec <= (int64_t)a.prm.p)) {
                            S.kind = LANE_UNIQUE;
#ifdef PA_STATS
                            atomicAdd(&a.dbg[24], 1ull);
#endif
                        } else if (S.nspec > 0) {
                            S.kind = LANE_HARD;
                            LANE_HARD_WHY(7);
                            LANE_HARD_WHY(18);
                        } else {
                            S.kind = LANE_AMB;
                        }
                    } else {
                        S.kind = S.nincl == 0 ? LANE_UNMAPPED : (S.nspec == 0 ? LANE_AMB : LANE_UNIQUE);
                    }
                }
            }
        }
        if (S.kind == LANE_WALK) S.kind = LANE_HARD;  // (a second re-anchoring is not attempted)
        const bool hard = S.kind == LANE_HARD;
        const uint64_t hb = __ballot(hard);
        if (hb) {  // one queue allocation per wave
            uint64_t qbase = 0;
            if (lane == __builtin_ctzll(hb)) qbase = atomicAdd(a.queue_hard_count, (unsigned long long)__popcll(hb));
            qbase = shfl64(qbase, __builtin_ctzll(hb));
            if (hard) a.queue_hard[qbase + lanes_below(hb)] = r;
        }
        const bool na = S.kind == LANE_NOANCHOR;
        const uint64_t nab = __ballot(na);
        if (NM == 2 && a.na_seg) {  // into this wave's segment, with the keys k_rc_seeds probes
            if (na) {
                const uint64_t e = seg_base + seg_na + lanes_below(nab);
                a.queue_na[e] = r;
                a.queue_na_keys[2 * e] = S.P[0];
                a.queue_na_keys[2 * e + 1] = S.P[1];
            }
            seg_na += (uint32_t)__popcll(nab);
        } else if (nab) {  // one queue allocation per wave
            uint64_t qbase = 0;
            if (lane == __builtin_ctzll(nab)) qbase = atomicAdd(a.queue_na_count, (unsigned long long)__popcll(nab));
            qbase = shfl64(qbase, __builtin_ctzll(nab));
            if (na) {
                a.queue_na[qbase + lanes_below(nab)] = r;
                if (a.queue_na_keys) {
                    a.queue_na_keys[2 * (qbase + lanes_below(nab))] = S.P[0];
                    a.queue_na_keys[2 * (qbase + lanes_below(nab)) + 1] = S.P[1];
                }
            }
        }
        const bool again = S.kind == LANE_AGAIN;
        const uint64_t ab = __ballot(again);
        if (ab) {  // (at most 63 + 64 entries: a batch is taken once 64 wait)
            if (again) {
                LW.again_r[n_again + lanes_below(ab)] = r;
                LW.again_a[n_again + lanes_below(ab)] = LW.cand[lane];
            }
            n_again += (uint32_t)__popcll(ab);
        }
        if (S.kind == LANE_UNIQUE) {
            if (lds) {
                atomicAdd(&uniq[S.g], 1u);
                if (r < first[S.g]) atomicMin(&first[S.g], r);
            } else {
                atomicAdd(&a.uniq[S.g], 1ull);
                atomicMin(&a.first[S.g], (unsigned long long)first_key(a.base + r, 0));
            }
        }
        n_uniq += (uint32_t)__popcll(__ballot(S.kind == LANE_UNIQUE));
        n_amb += (uint32_t)__popcll(__ballot(S.kind == LANE_AMB));
        n_unm += (uint32_t)__popcll(__ballot(S.kind == LANE_UNMAPPED));
        n_drop += (uint32_t)__popcll(__ballot(S.kind == LANE_DROP));
        const bool settled = S.kind == LANE_UNIQUE || S.kind == LANE_AMB || S.kind == LANE_UNMAPPED;
        if (MG) n_hr += wave_sum(settled ? S.hr : 0u);
        if (WIN_Q) n_qf += wave_sum(settled ? S.qf : 0u);
    }
    if (lane == 0) {
        if (NM == 2 && a.na_seg) {  // every wave of the grid writes its segment's count
            a.seg_cnt[wave_id] = seg_na;
            if (seg_na) atomicAdd(a.queue_na_count, (unsigned long long)seg_na);
        }
        if (n_uniq) atomicAdd(&a.stats[0], (unsigned long long)n_uniq);
        if (n_amb) atomicAdd(&a.stats[1], (unsigned long long)n_amb);
        if (n_unm) atomicAdd(&a.stats[2], (unsigned long long)n_unm);
        if (n_drop) atomicAdd(&a.stats[3], (unsigned long long)n_drop);
        if (n_hr && MG) atomicAdd(&a.stats[5], (unsigned long long)n_hr);
        if (WIN_Q && n_qf) atomicAdd(&a.stats[4], (unsigned long long)n_qf);
    }
    if (lds) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < G; i += kBlock) {
            if (uniq[i]) atomicAdd(&a.uniq[i], (unsigned long long)uniq[i]);
            if (first[i] != ~0u) atomicMin(&a.first[i], (unsigned long long)first_key(a.base + first[i], 0));
        }
    }
}

constexpr size_t lane_lds_bytes(uint32_t G, int NM = 2) {
    return (G <= kLaneLdsGenomeCap ? ((size_t)G * 8 + 15) / 16 * 16 : 0) +
           (size_t)kWaves * (NM == 4 ? sizeof(LaneWave<4>) : sizeof(LaneWave<2>));
}

// k_align_lane_na: the reads k_align_lane found no seed for, one per lane.
// Every window of the read (but those failing --min-kmer-quality) is looked up
// -- the Bloom filter first, then the table for the few it lets through
// (src/kmer.py:410-429).  No k-mer found: UNMAPPED; found ones all
// multi-genome (or above --max-genomes, counted as highly redundant):
// AMBIGUOUS with an empty list (no specific k-mer, src/kmer.py:458-461); a
// specific one: the read is queued for the wave kernel.
//
// The Bloom test of windows w0 .. w0 + NAG - 1 (w0 a multiple of 16, k <= 31;
// bit j of act: look window w0 + j up).  The group's bases are 128 bits of
// the lane's LDS row, realigned once (a multiple of 32 bits), so every
// window's key and every 15-mer is a shift by a constant; the group's 15-mer
// orders are computed once (NAG + k - 15 of them) and each window's minimizer
// is a sliding minimum.  A window's block is the minimizer's
// (pa_device.h), so the windows of one minimizer run read ONE 16-B block,
// loaded where the run starts (~14 loads per 150-bp read instead of one per
// window) and carried in `cur` to the next group.  Returns the windows the
// filter lets through.
#ifndef PA_NA_GROUP
#define PA_NA_GROUP 8
#endif
__device__ __forceinline__ uint64_t bits128(uint64_t x0, uint64_t x1, int s) {  // (s constant after unrolling)
    return s == 0 ? x0 : ((x0 << s) | (x1 >> (64 - s)));
}
// CARRY false: a group on its own (k_align_lane_rc's cooperative passes): all
// its 15-mer orders computed, its first run loaded, no LDS carry.
template <int NAG, int KC, bool CARRY = true>  // KC: k known at compile time (31, the benchmark k), else 0
__device__ __forceinline__ uint32_t bloom_group(const AlignArgs &a, const uint64_t *row, uint32_t w0, uint32_t act,
                                                bool fresh, uint32_t &prev_blk, uint4 &cur, bool &cur_mm,
                                                uint4 (*hc)[kBlock]) {
    static_assert(NAG == 8 || NAG == 16, "a group's bases are 128 bits from a multiple of 16");
    const int k = KC ? KC : a.k, sh = 64 - 2 * k;
    const int mm = k < 15 ? k : 15;
    const int S = k - mm + 1;  // 15-mers per window (<= 17)
    // the group's bases from window w0 on (bits 2 w0 .. 2 w0 + 127 of the row;
    // 2 w0 is a multiple of 2 NAG, the same in every lane of the wave)
    const uint32_t o = 2 * w0, q = o >> 6, r = o & 63;
    uint64_t X0 = row[q], X1 = row[q + 1];
    if (r) {
        const uint64_t X2 = row[q + 2];
        X0 = (X0 << r) | (X1 >> (64 - r));
        X1 = (X1 << r) | (X2 >> (64 - r));
    }
    // (every h[p] computed: the ones past the group's last 15-mer are never
    // selected below, and branching on them cost more than computing them).
    // The previous group's last sixteen are this group's first sixteen (hc),
    // so a group after the first computes NAG of them, one per window.
    // (hc: the lane's sixteen in LDS, [i][thread]: no bank conflicts)
    uint32_t h[NAG + 16];
    const uint32_t t = threadIdx.x;
    if (CARRY) {
#pragma unroll
        for (int i = 0; i < 4; i++) {  // (the caller stores a read's first sixteen before its first group)
            const uint4 v = hc[i][t];
            h[4 * i] = v.x, h[4 * i + 1] = v.y, h[4 * i + 2] = v.z, h[4 * i + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int p = 0; p < 16; p++) h[p] = mm_order((uint32_t)(bits128(X0, X1, 2 * p) >> (64 - 2 * mm)));
    }
#pragma unroll
    for (int p = 16; p < NAG + 16; p++) h[p] = mm_order((uint32_t)(bits128(X0, X1, 2 * p) >> (64 - 2 * mm)));
    if (CARRY) {
#pragma unroll
        for (int i = 0; i < 4; i++)
            hc[i][t] = make_uint4(h[NAG + 4 * i], h[NAG + 4 * i + 1], h[NAG + 4 * i + 2], h[NAG + 4 * i + 3]);
    }
    // each window's minimum: with S >= 9 every window j < 8 holds 15-mers 7
    // and 8 .. j + S - 1, so it is min(suffix minimum from j to 7, prefix
    // minimum from 7 to j + S - 1)
    uint32_t mn[NAG];
    if (KC && S >= NAG + 1) {  // (k = 31: S = 17; any other k takes the direct minimum below)
        uint32_t sfx[NAG], pfx[17];
        sfx[NAG - 1] = pfx[0] = h[NAG - 1];
#pragma unroll
        for (int j = NAG - 2; j >= 0; j--) sfx[j] = min(h[j], sfx[j + 1]);
#pragma unroll
        for (int t = 1; t < 17; t++) pfx[t] = min(pfx[t - 1], h[NAG - 1 + t]);
#pragma unroll
        for (int j = 0; j < NAG; j++) {
            mn[j] = min(sfx[j], pfx[j + S - NAG]);
        }
    } else {
#pragma unroll
        for (int j = 0; j < NAG; j++) {
            uint32_t best = ~0u;
#pragma unroll
            for (int i = 0; i < 17; i++)
                if (i < S) best = h[j + i] < best ? h[j + i] : best;
            mn[j] = best;
        }
    }
    (void)k;
    // run starts (a new block) and their loads, all issued before any is used
    const uint4 *blocks = (const uint4 *)a.bloom;
    uint32_t blk[NAG], news = 0;
#pragma unroll
    for (int j = 0; j < NAG; j++) {
        blk[j] = (uint32_t)bloom_block(mn[j], a.bloom_lg);
        const uint32_t before = j ? blk[j - 1] : prev_blk;
        news |= (blk[j] != before || (j == 0 && fresh)) ? 1u << j : 0u;
    }
    // minimizer presence (a.mm_bits, a bitmap small enough for the L2): a run
    // whose minimizer is no key's has none of its windows in the index -- an
    // unindexed organism's reads have almost none -- and loads no block.  A
    // run going on from the previous group keeps that group's answer (cur_mm)
    uint32_t pres = (1u << NAG) - 1;
    if (a.mm_bits) {
        uint32_t mw[NAG], mh[NAG];
#pragma unroll
        for (int j = 0; j < NAG; j++) {
            mh[j] = mm_bit(mn[j], a.mm_lg);
            mw[j] = a.mm_bits[bit(news, j) ? mh[j] >> 5 : 0u];  // (loads issue together)
        }
        bool p = cur_mm;
        pres = 0;
#pragma unroll
        for (int j = 0; j < NAG; j++) {
            if (bit(news, j)) p = ((mw[j] >> (mh[j] & 31)) & 1u) != 0;
            pres |= p ? 1u << j : 0u;
        }
        cur_mm = p;
        act &= pres;
    }
    // (no load for a run none of whose windows is looked up; the group's last
    // run may go on in the next group, which then tests against `cur`)
    uint32_t need = 0;
    {
        bool any = bit(pres, NAG - 1);
#pragma unroll
        for (int j = NAG - 1; j >= 0; j--) {
            any = any || bit(act, j);
            if (bit(news, j)) {
                need |= any ? 1u << j : 0u;
                any = false;
            }
        }
    }
    prev_blk = blk[NAG - 1];
    // (a run without a load has no window to test: it ends inside the group).
    // Every slot loads -- the unneeded ones block 0, an L1 hit -- so that the
    // loads issue back to back with one wait (a load under a branch waits
    // inside it); eight at a time (eight blocks in registers, not sixteen)
#pragma unroll
    for (int b0 = 0; b0 < NAG; b0 += 8) {
        uint4 V[8];
#pragma unroll
        for (int j = 0; j < 8; j++) V[j] = blocks[bit(need, b0 + j) ? blk[b0 + j] : 0u];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (bit(need, b0 + j)) cur = V[j];
            if (!bit(act, b0 + j)) continue;
            const uint32_t hk = bloom_key_mix(bits128(X0, X1, 2 * (b0 + j)) >> sh);
            if (!bloom_block_has(cur, hk)) act &= ~(1u << (b0 + j));
        }
    }
    return act;
}

// The first sixteen 15-mer orders of a Bloom group at window w0 (a multiple of
// the group size): a read's first group, or the first after groups skipped.
__device__ __forceinline__ void na_hc_init(const uint64_t *row, uint32_t w0, int k, uint4 (*hc)[kBlock]) {
    const int mm = k < 15 ? k : 15;
    const uint32_t o = 2 * w0, q = o >> 6, r = o & 63;
    uint64_t X0 = row[q], X1 = row[q + 1];
    if (r) {
        const uint64_t X2 = row[q + 2];
        X0 = (X0 << r) | (X1 >> (64 - r));
        X1 = (X1 << r) | (X2 >> (64 - r));
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint32_t v[4];
#pragma unroll
        for (int e = 0; e < 4; e++) v[e] = mm_order((uint32_t)(bits128(X0, X1, 2 * (4 * i + e)) >> (64 - 2 * mm)));
        hc[i][threadIdx.x] = make_uint4(v[0], v[1], v[2], v[3]);
    }
}

// Reverse-strand walk of a read with no seed in the index (k <= 31).  Such a
// read is most often the reverse complement of a stretch of some genome (about
// half of a real FASTQ): its reverse complement R' is then walked like a
// forward read -- a seed (R' window 0, the reverse complement of the read's
// last window; else R' window W - 1, of its first) gives the anchor A, R' is
// compared with the genome words of the walk blocks from A on.  Read window w
// is the reverse complement of R' window w' = W - 1 - w, and where the genome
// window at A + w' is indexed:
//   * R' window w' equals it: read window w is absent unless the
//     reverse-complement plane (k_tile_rcp) has its bit set;
//   * R' window w' differs from it in exactly one base: the reverse-complement
//     neighbour bits (tile_rcnb) say whether read window w is present;
// every other window (two or more mismatches, more than 8 mismatching bases,
// an unindexed genome window, a bit set) is left to look up.  Returns in
// lk0 / lk1 the read's windows still to look up and true; false when no
// anchor is found or R' differs from the stretch in more than kRcMaxMis bases.
// Exact: it only removes windows shown absent.
constexpr uint32_t kRcMaxMis = 16;
__device__ __forceinline__ bool na_rc_walk(const AlignArgs &a, const uint64_t *row, uint32_t len, uint32_t W,
                                           uint64_t seed, uint64_t &lk0, uint64_t &lk1) {
    const int k = a.k;
    // seed = P | s << 63: R' window 0 (s = 0) or W - 1 (s = 1) is at P (k_rc_seeds)
    const int64_t A = (int64_t)(seed & ~(1ull << 63)) - ((seed >> 63) ? (int64_t)(W - 1) : 0);
    if (A < 0 || (uint64_t)A + len > a.tile_n) return false;
    const uint64_t Au = (uint64_t)A;
    uint64_t gw[kLaneWords + 1], pa3[3], pb3[3];
    lane_blocks<true>(a, Au, len, gw, pa3, pb3);
    const uint64_t *rp = a.tile_rcp + (Au >> 6);
    const uint64_t q0 = rp[0], q1 = rp[1], q2 = rp[2];
    const uint32_t fr = (uint32_t)(Au & 63);
    auto shifted = [fr](uint64_t x0, uint64_t x1) { return fr ? (x0 >> fr) | (x1 << (64 - fr)) : x0; };
    const uint64_t IX0 = shifted(pa3[0], pa3[1]) | shifted(pb3[0], pb3[1]);  // indexed genome windows
    const uint64_t IX1 = shifted(pa3[1], pa3[2]) | shifted(pb3[1], pb3[2]);
    const uint32_t gr = (uint32_t)(2 * Au & 63);
    const uint32_t qlast = (len - 1) >> 5, rl = len - 32 * qlast;
    const uint64_t tail = rl >= 32 ? ~0ull : ~0ull << (64 - 2 * rl);
    const bool has_nb = a.tile_rcnb != nullptr;
    uint64_t U0 = 0, U1 = 0, V0 = 0, V1 = 0, NP0 = 0, NP1 = 0;
    uint64_t epk = 0;  // positions e of the mismatches to look up in the neighbour bits (8 bits each, <= 8)
    uint32_t cpk = 0;  //   their substitution index (cr - cg - 1) & 3 (2 bits each)
    uint32_t nnb = 0, nmis = 0;
#pragma unroll
    for (int i = 0; i < kLaneWords; i++) {
        if (32 * i >= (int)len) break;
        // R' word i: the read's bases len - 1 - 32 i down to len - 32 - 32 i,
        // complemented (bases before the read's start read as zeros: past the
        // end of R', masked by `tail`)
        const int32_t o = (int32_t)len - 32 - 32 * i;
        const uint64_t c = o >= 0 ? row_bits(row, 2 * (uint32_t)o) : row[0] >> (-2 * o);
        const uint64_t rw = rev_groups64(~c);
        const uint64_t gwi = gr ? ((gw[i] << gr) | (gw[i + 1] >> (64 - gr))) : gw[i];
        uint64_t d = rw ^ gwi;
        if ((uint32_t)i == qlast) d &= tail;
        uint64_t m = (d | (d >> 1)) & 0x5555555555555555ull;
        while (m) {
            const uint32_t j = __builtin_clzll(m) >> 1, e = 32 * i + j;
            m &= ~(1ull << (62 - 2 * j));
            const int32_t lo = (int32_t)e - k + 1 < 0 ? 0 : (int32_t)e - k + 1;
            const int32_t hi = (int32_t)e < (int32_t)W - 1 ? (int32_t)e : (int32_t)W - 1;
            if (lo > hi) continue;
            const uint64_t r0 = lo < 64 ? ((~0ull << lo) & (hi >= 63 ? ~0ull : ((2ull << hi) - 1))) : 0ull;
            const uint64_t r1 =
                hi >= 64 ? ((lo <= 64 ? ~0ull : (~0ull << (lo - 64))) & (hi >= 127 ? ~0ull : ((2ull << (hi - 64)) - 1)))
                         : 0ull;
            if (++nmis > kRcMaxMis) return false;
            V0 |= U0 & r0;
            V1 |= U1 & r1;
            U0 |= r0;
            U1 |= r1;
            if (has_nb && nnb < 8 && ((r0 & IX0) | (r1 & IX1))) {
                const uint32_t cg = (uint32_t)(gwi >> (62 - 2 * j)) & 3u, cr = (uint32_t)(rw >> (62 - 2 * j)) & 3u;
                epk |= (uint64_t)e << (8 * nnb);
                cpk |= ((cr - cg - 1) & 3u) << (2 * nnb);
                nnb++;
            } else {
                V0 |= r0;  // (no bits for it: its windows are looked up)
                V1 |= r1;
            }
        }
    }
    // the neighbour words of the mismatches, four loads in flight at a time
#pragma unroll 1
    for (uint32_t b0 = 0; b0 < nnb; b0 += 4) {
        uint32_t nv[4];
        int32_t sf[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t q = b0 + u < nnb ? b0 + u : b0;
            const uint32_t e = (uint32_t)(epk >> (8 * q)) & 255u, c = (cpk >> (2 * q)) & 3u;
            nv[u] = a.tile_rcnb[3 * (Au + e) + c];
            sf[u] = b0 + u < nnb ? (int32_t)e - k + 1 : 1000;  // bit q of the word <-> window e - k + 1 + q
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (sf[u] == 1000) continue;
            const uint64_t nbw = nv[u];
            const int32_t sft = sf[u];
            if (sft >= 0) {
                NP0 |= sft < 64 ? nbw << sft : 0ull;
                NP1 |= sft >= 64 ? nbw << (sft - 64) : (sft > 32 ? nbw >> (64 - sft) : 0ull);
            } else {
                NP0 |= nbw >> (-sft);
            }
        }
    }
    const uint64_t RP0 = shifted(q0, q1), RP1 = shifted(q1, q2);
    const uint64_t in0 = W >= 64 ? ~0ull : ((1ull << W) - 1);
    const uint64_t in1 = W <= 64 ? 0ull : (W >= 128 ? ~0ull : ((1ull << (W - 64)) - 1));
    // R' windows to look up: unindexed genome windows; equal ones whose plane
    // bit is set; one mismatch and the neighbour present; two or more
    const uint64_t N0 = in0 & (~IX0 | (~U0 & RP0) | (U0 & (V0 | NP0)));
    const uint64_t N1 = in1 & (~IX1 | (~U1 & RP1) | (U1 & (V1 | NP1)));
    // read window w = W - 1 - w': the 128-bit mask reversed, shifted down by 128 - W
    uint64_t lo = __builtin_bitreverse64(N1), hi = __builtin_bitreverse64(N0);
    const uint32_t s = 128 - W;
    if (s >= 64) {
        lo = hi >> (s - 64);
        hi = 0;
    } else if (s) {
        lo = (lo >> s) | (hi << (64 - s));
        hi >>= s;
    }
    lk0 = lo;
    lk1 = hi;
    return true;
}

// The table probes of a lane's remaining windows (bit w of pm0 | pm1 << 64:
// Bloom false positives, the rare present k-mer): each lane its own next NPB
// windows, so a wave probes as often as its lane with the most (~1.3 rounds
// on c2rc, where probing per group took ~30: some lane has a false positive in
// almost every group).  spec: a specific k-mer found (the read goes to the
// wave kernel); noff: multi-genome ones; hr: above --max-genomes.
#ifndef PA_NA_PROBES
#define PA_NA_PROBES 4
#endif
template <bool MG>
__device__ __forceinline__ void na_probe_rest(const AlignArgs &a, const uint64_t *row, uint64_t pm0, uint64_t pm1,
                                              bool &spec, uint32_t &noff, uint32_t &hr) {
    const int sh = 64 - 2 * a.k;
    constexpr int NPB = PA_NA_PROBES;
#pragma unroll 1
    while ((pm0 | pm1) && !spec) {
        uint64_t key[NPB];
        uint32_t act8 = 0;
#pragma unroll
        for (int j = 0; j < NPB; j++) {
            const bool lo = pm0 != 0;
            const uint64_t m = lo ? pm0 : pm1;
            const uint32_t w = (lo ? 0u : 64u) + (uint32_t)__builtin_ctzll(m | (1ull << 63));
            act8 |= m ? 1u << j : 0u;
            key[j] = m ? row_bits(row, 2 * w) >> sh : 0ull;
            if (lo) pm0 &= pm0 - 1;
            else pm1 &= pm1 - 1;
        }
        uint32_t f, cl[NPB], tp[NPB];
        lane_probe<NPB>(a, key, act8, f, cl, tp);
#pragma unroll
        for (int j = 0; j < NPB; j++) {
            if (!bit(f, j)) continue;
            if (MG && (int64_t)class_size_of(cl[j], a.G, a.class_genomes) > (int64_t)a.prm.mg) hr++;
            else if (cls_of(cl[j]) >= a.G) noff++;
            else spec = true;
        }
    }
}

#ifndef PA_NA_WAVES
#define PA_NA_WAVES 4  // (c2mix: 1.31 vs 1.26 G reads/s at 3, 28 B/lane of scratch)
#endif
template <bool NEED_Q, bool WIN_Q, bool MG>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(PA_NA_WAVES))) void k_align_lane_na(AlignArgs a) {
    __shared__ uint64_t rows[kBlock][kLaneWords + 1];
    __shared__ uint4 hcarry[4][kBlock];  // per lane: the last Bloom group's last sixteen 15-mer orders
    rows[threadIdx.x][kLaneWords] = 0;  // the zero word past every read (lane_prep writes words 0 .. kLaneWords - 1)
    const int lane = lane_id();
    const int sh = 64 - 2 * a.k;
    const uint64_t n = *a.queue_na_count;
    // a few such reads cost a ~0.2 ms chain of dependent loads here (one lane
    // walks ~120 windows) but next to nothing among the wave kernel's reads:
    // below a.na_min (32 k) they are handed to it
    const bool forward = n < a.na_min;
    uint32_t n_amb = 0, n_unm = 0;   // wave totals (scalar)
    uint32_t hr_sum = 0, qf_sum = 0;  // per lane
    for (uint64_t c0 = (uint64_t)blockIdx.x * kBlock + (threadIdx.x & ~63u); c0 < n;
         c0 += (uint64_t)gridDim.x * kBlock) {
        const uint64_t i = c0 + lane;
        LaneRead<2> S;
        S.kind = LANE_UNMAPPED + 100;  // (past the end: counted nowhere)
        uint32_t r = 0;
        if (i < n) {
            r = a.queue_na[i];
            if (forward) S.kind = LANE_HARD;
            else lane_prep<2, NEED_Q, WIN_Q, false>(a, r, ~0ull, rows[threadIdx.x], S);
        }
        if (S.kind == LANE_WALK) {
            const uint64_t *row = rows[threadIdx.x];
            const uint32_t W = S.W;
            bool spec = false;
            uint32_t noff = 0, hr = 0;
            constexpr int NAG = PA_NA_GROUP;
            uint32_t prev_blk = 0;
            uint4 cur = make_uint4(0, 0, 0, 0);
            bool cur_mm = true;
            // the windows to look up (bit w of pm0 | pm1 << 64): every window
            // (W <= kLaneMaxW = 128) but those failing --min-kmer-quality, less
            // those the Bloom filter shows absent.  A group with none is
            // skipped; the next group then starts a new minimizer run
            uint64_t pm0 = 0, pm1 = 0;
            bool fresh = true;
#pragma unroll 1
            for (uint32_t w0 = 0; w0 < W; w0 += NAG) {
                uint32_t act = 0;
#pragma unroll
                for (int j = 0; j < NAG; j++) {
                    const uint32_t w = w0 + j;
                    const bool filt = WIN_Q && (((w < 64 ? S.F[0] >> w : S.F[1] >> (w - 64)) & 1ull) != 0);
                    act |= (w < W && !filt) ? 1u << j : 0u;
                }
                if (!act) {
                    fresh = true;
                    continue;
                }
                if (a.bloom) {  // keys surely absent are not looked up
                    if (fresh) na_hc_init(row, w0, a.k, hcarry);  // (the group's first sixteen 15-mer orders)
                    act = a.k == 31 ? bloom_group<NAG, 31>(a, row, w0, act, fresh, prev_blk, cur, cur_mm, hcarry)
                                    : bloom_group<NAG, 0>(a, row, w0, act, fresh, prev_blk, cur, cur_mm, hcarry);
                }
                fresh = false;
                if (w0 < 64) pm0 |= (uint64_t)act << w0;
                else pm1 |= (uint64_t)act << (w0 - 64);
            }
            // then the table for the rest (Bloom false positives, the rare
            // present k-mer)
            na_probe_rest<MG>(a, row, pm0, pm1, spec, noff, hr);
            S.kind = spec ? LANE_HARD : (noff ? LANE_AMB : LANE_UNMAPPED);
            if (!spec) {
                hr_sum += hr;
                qf_sum += S.qf;
            }
        }
        const bool hard = S.kind == LANE_HARD;
        const uint64_t hb = __ballot(hard);
        if (hb) {
            uint64_t qbase = 0;
            if (lane == __builtin_ctzll(hb)) qbase = atomicAdd(a.queue_hard_count, (unsigned long long)__popcll(hb));
            qbase = shfl64(qbase, __builtin_ctzll(hb));
            if (hard) a.queue_hard[qbase + lanes_below(hb)] = r;
        }
        n_amb += (uint32_t)__popcll(__ballot(S.kind == LANE_AMB));
        n_unm += (uint32_t)__popcll(__ballot(S.kind == LANE_UNMAPPED));
    }
    const uint32_t hr_w = wave_sum(hr_sum);
    const uint32_t qf_w = WIN_Q ? wave_sum(qf_sum) : 0u;
    if (lane == 0) {
        if (n_amb) atomicAdd(&a.stats[1], (unsigned long long)n_amb);
        if (n_unm) atomicAdd(&a.stats[2], (unsigned long long)n_unm);
        if (MG && hr_w) atomicAdd(&a.stats[5], (unsigned long long)hr_w);
        if (WIN_Q && qf_w) atomicAdd(&a.stats[4], (unsigned long long)qf_w);
    }
}

// k_align_lane_naw: k_align_lane_na for keys of two and three words (31 < k
// <= 95): the reads none of whose seeds is in the index -- at k = 75 with 150-bp
// reads 7 % of them at 0.5 % errors, since an error in windows 56 .. 74 and
// another past 74 leave no seed (often no window at all) clean.  Every window
// (but those failing --min-kmer-quality) is tested against the Bloom filter,
// eight loads in flight (a window's word is chosen by its key's hash:
// bloom_word2 / bloom_word3), then the table for the few it lets through;
// nothing found: UNMAPPED, only multi-genome k-mers: AMBIGUOUS with an empty
// list, a specific one: the wave kernel (src/kmer.py:410-461).
template <bool NEED_Q, bool WIN_Q, bool MG, int NW>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(PA_NA_WAVES))) void k_align_lane_naw(AlignArgs a) {
    static_assert(NW == 2 || NW == 3, "multi-word keys");
    __shared__ uint64_t rows[kBlock][kLaneWords + 1];
    rows[threadIdx.x][kLaneWords] = 0;
    const int lane = lane_id();
    const uint64_t n = *a.queue_na_count;
    const bool forward = n < a.na_min;  // (few such reads: on to the wave kernel, as k_align_lane_na)
    uint32_t n_amb = 0, n_unm = 0;
    uint32_t hr_sum = 0, qf_sum = 0;
    for (uint64_t c0 = (uint64_t)blockIdx.x * kBlock + (threadIdx.x & ~63u); c0 < n;
         c0 += (uint64_t)gridDim.x * kBlock) {
        const uint64_t i = c0 + lane;
        LaneRead<2> S;
        S.kind = LANE_UNMAPPED + 100;  // (past the end: counted nowhere)
        uint32_t r = 0;
        if (i < n) {
            r = a.queue_na[i];
            if (forward) S.kind = LANE_HARD;
            else lane_prep<2, NEED_Q, WIN_Q, false, NW>(a, r, ~0ull, rows[threadIdx.x], S);
        }
        if (S.kind == LANE_WALK) {
            const uint64_t *row = rows[threadIdx.x];
            const uint32_t W = S.W;
            uint64_t pm0 = 0, pm1 = 0;  // windows the filter lets through
            if (!a.bloom) {  // (no filter, PA_LANE_NOANCHOR=1 forced: every window is looked up)
                pm0 = W >= 64 ? ~0ull : ((1ull << W) - 1);
                pm1 = W <= 64 ? 0ull : (W >= 128 ? ~0ull : ((1ull << (W - 64)) - 1));
                if (WIN_Q) {
                    pm0 &= ~S.F[0];
                    pm1 &= ~S.F[1];
                }
            }
#pragma unroll 1
            for (uint32_t w0 = 0; a.bloom && w0 < W; w0 += 8) {
                uint64_t bw[8], bm[8];
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const uint32_t w = w0 + j;
                    const bool filt = WIN_Q && (((w < 64 ? S.F[0] >> w : S.F[1] >> (w - 64)) & 1ull) != 0);
                    bm[j] = 0;
                    uint64_t wi = 0;
                    if (w < W && !filt) {
                        const Key<NW> K = row_key<NW>(row, w, a.k);
                        if constexpr (NW == 2)
                            bloom_word2(K, a.bloom_lg, wi, bm[j]);
                        else
                            bloom_word3(K, a.bloom_lg, wi, bm[j]);
                    }
                    bw[j] = a.bloom[wi];  // (every load issued before any is tested)
                }
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const uint32_t w = w0 + j;
                    if (bm[j] && (bw[j] & bm[j]) == bm[j]) {
                        if (w < 64) pm0 |= 1ull << w;
                        else pm1 |= 1ull << (w - 64);
                    }
                }
            }
            bool spec = false;
            uint32_t noff = 0, hr = 0;
#pragma unroll 1
            while ((pm0 | pm1) && !spec) {
                Key<NW> key[4];
                uint32_t act4 = 0;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const bool lo = pm0 != 0;
                    const uint64_t m = lo ? pm0 : pm1;
                    const uint32_t w = (lo ? 0u : 64u) + (uint32_t)__builtin_ctzll(m | (1ull << 63));
                    act4 |= m ? 1u << j : 0u;
                    key[j] = m ? row_key<NW>(row, w, a.k) : Key<NW>{};
                    if (lo) pm0 &= pm0 - 1;
                    else pm1 &= pm1 - 1;
                }
                uint32_t f, cl[4], tp[4];
                lane_probe_k<4, 1, NW>(a, key, act4, f, cl, tp);
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    if (!bit(f, j)) continue;
                    if (MG && (int64_t)class_size_of(cl[j], a.G, a.class_genomes) > (int64_t)a.prm.mg) hr++;
                    else if (cls_of(cl[j]) >= a.G) noff++;
                    else spec = true;
                }
            }
            S.kind = spec ? LANE_HARD : (noff ? LANE_AMB : LANE_UNMAPPED);
            if (!spec) {
                hr_sum += hr;
                qf_sum += S.qf;
            }
        }
        const bool hard = S.kind == LANE_HARD;
        const uint64_t hb = __ballot(hard);
        if (hb) {
            uint64_t qbase = 0;
            if (lane == __builtin_ctzll(hb)) qbase = atomicAdd(a.queue_hard_count, (unsigned long long)__popcll(hb));
            qbase = shfl64(qbase, __builtin_ctzll(hb));
            if (hard) a.queue_hard[qbase + lanes_below(hb)] = r;
        }
        n_amb += (uint32_t)__popcll(__ballot(S.kind == LANE_AMB));
        n_unm += (uint32_t)__popcll(__ballot(S.kind == LANE_UNMAPPED));
    }
    const uint32_t hr_w = wave_sum(hr_sum);
    const uint32_t qf_w = WIN_Q ? wave_sum(qf_sum) : 0u;
    if (lane == 0) {
        if (n_amb) atomicAdd(&a.stats[1], (unsigned long long)n_amb);
        if (n_unm) atomicAdd(&a.stats[2], (unsigned long long)n_unm);
        if (MG && hr_w) atomicAdd(&a.stats[5], (unsigned long long)hr_w);
        if (WIN_Q && qf_w) atomicAdd(&a.stats[4], (unsigned long long)qf_w);
    }
}

// k_rc_seeds: the reverse-complement seeds of the reads k_align_lane found no
// seed for (their keys come with the queue: a.queue_na_keys, made while the
// read was packed), kSeedReads reads per thread: a read with one
// in the index goes to k_align_lane_rc (a.queue_rc, with the seed's first
// occurrence), any other -- an unindexed organism, errors at both ends -- to
// k_align_lane_na (a.queue_na2).  Classifying here, without loading or packing
// the read, keeps the reads k_align_lane_rc cannot walk out of its waves (it
// took ~0.2 ns per such read to load, pack and reject it).
constexpr int kSeedReads = 4;  // reads per thread (their probes in flight together)
constexpr uint32_t kSegGroup = 4;  // (a.na_seg) k_align_lane queue segments per block, taken as one run
__global__ __launch_bounds__(kBlock) void k_rc_seeds(AlignArgs a) {
    // queue slots are taken per block (LDS counters, one global atomic per
    // queue and block of kBlock * kSeedReads reads): one atomic per wave
    // serialised on the two counters took longer than the probes (1.0-1.7 ms
    // for 5 M reads)
    __shared__ uint32_t cnt[2];
    __shared__ unsigned long long base[2];
    const uint64_t n_all = *a.queue_na_count;
    const bool forward = n_all < a.na_min;  // (few such reads: all on to k_align_lane_na, which hands them on)
    constexpr uint64_t kChunk = (uint64_t)kBlock * kSeedReads;
    // the reads: one flat queue_na, or (a.na_seg) k_align_lane's per-wave
    // segments of it, kSegGroup segments per block taken as one run (entry i
    // of segment sg at sg * seg_cap + i; a block per segment cost C4 ~40 us
    // of block starts and queue atomics for its few seedless reads)
    const bool segd = a.na_seg != 0;
    const uint32_t nunits = segd ? (a.nseg + kSegGroup - 1) / kSegGroup : 1u;
#pragma unroll 1
    for (uint32_t u = segd ? blockIdx.x : 0u; u < nunits; u += segd ? gridDim.x : 1u) {
    uint32_t pc[kSegGroup + 1];  // the group's segments' entries, running sums
    pc[0] = 0;
#pragma unroll
    for (uint32_t g = 0; g < kSegGroup; g++)
        pc[g + 1] = pc[g] + (segd && u * kSegGroup + g < a.nseg ? a.seg_cnt[u * kSegGroup + g] : 0u);
    const uint64_t n = segd ? (uint64_t)pc[kSegGroup] : n_all;
    auto qi = [&](uint64_t i) -> uint64_t {  // the queue index of the run's entry i
        if (!segd) return i;
        uint32_t g = 0, b0 = 0;
#pragma unroll
        for (uint32_t h = 1; h < kSegGroup; h++)
            if (i >= pc[h]) g = h, b0 = pc[h];
        return (uint64_t)(u * kSegGroup + g) * a.seg_cap + (i - b0);
    };
    for (uint64_t c0 = segd ? 0ull : (uint64_t)blockIdx.x * kChunk; c0 < n;
         c0 += segd ? kChunk : (uint64_t)gridDim.x * kChunk) {
        if (threadIdx.x < 2) cnt[threadIdx.x] = 0;
        __syncthreads();
        // R' window 0 first (found for ~86 % of reverse-strand reads at 0.5 %
        // errors), R' window W - 1 only where it is absent: 1.1 table lines
        // per such read instead of 2 (an unindexed organism's read takes 2)
        uint64_t sk[kSeedReads];
        uint32_t act = 0;
#pragma unroll
        for (int j = 0; j < kSeedReads; j++) {
            const uint64_t i = c0 + (uint64_t)j * kBlock + threadIdx.x;
            sk[j] = 0;
            if (i < n && !forward) {
                sk[j] = a.queue_na_keys[2 * qi(i)];
                act |= 1u << j;
            }
        }
        uint32_t f0, f1, cl[kSeedReads], tp[kSeedReads];
        lane_probe<kSeedReads>(a, sk, act, f0, cl, tp);
        uint64_t seed[kSeedReads];
        uint32_t walk = 0, slot[kSeedReads], act1 = 0;
#pragma unroll
        for (int j = 0; j < kSeedReads; j++) {
            const uint64_t i = c0 + (uint64_t)j * kBlock + threadIdx.x;
            seed[j] = 0;
            if (bit(f0, j) && tp[j] != NONE) {
                walk |= 1u << j;
                seed[j] = first_pos(cl[j], tp[j], a.G, a.class_genomes, a.goff, a.tpos_local);
            } else if (bit(act, j)) {
                sk[j] = a.queue_na_keys[2 * qi(i) + 1];
                act1 |= 1u << j;
            }
        }
        if (__ballot(act1 != 0)) {
            lane_probe<kSeedReads>(a, sk, act1, f1, cl, tp);
#pragma unroll
            for (int j = 0; j < kSeedReads; j++)
                if (bit(act1, j) && bit(f1, j) && tp[j] != NONE) {
                    walk |= 1u << j;
                    seed[j] = first_pos(cl[j], tp[j], a.G, a.class_genomes, a.goff, a.tpos_local) | (1ull << 63);
                }
        }
#pragma unroll
        for (int j = 0; j < kSeedReads; j++) {
            const uint64_t i = c0 + (uint64_t)j * kBlock + threadIdx.x;
            slot[j] = i < n ? atomicAdd(&cnt[bit(walk, j) ? 0 : 1], 1u) : 0u;
        }
        __syncthreads();
        if (threadIdx.x < 2 && cnt[threadIdx.x])
            base[threadIdx.x] = atomicAdd(threadIdx.x == 0 ? a.queue_rc_count : a.queue_na2_count,
                                          (unsigned long long)cnt[threadIdx.x]);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kSeedReads; j++) {
            const uint64_t i = c0 + (uint64_t)j * kBlock + threadIdx.x;
            if (i >= n) continue;
            const uint32_t r = a.queue_na[qi(i)];
            if (bit(walk, j)) {
                a.queue_rc[base[0] + slot[j]] = r;
                a.queue_rc_anc[base[0] + slot[j]] = seed[j];
            } else {
                a.queue_na2[base[1] + slot[j]] = r;
            }
        }
        __syncthreads();  // (cnt / base are reset by the next chunk)
    }
    }
}

// k_align_lane_rc: the reads k_align_lane found no seed for and k_rc_seeds a
// reverse-complement one (a.queue_rc), walked on the reverse strand
// (na_rc_walk) -- about half of a real FASTQ is the reverse complement of
// some genome stretch, and the forward-only lookups of the reference
// (src/kmer.py:419-429) must show every one of its windows absent.  A walked
// read needs the Bloom filter only for the few windows the walk leaves (N
// runs of the genome, two mismatches in one window, a bit set); a read it
// cannot walk goes on to k_align_lane_na (a.queue_na2), which tests every
// window.  The reads' counts vary a lot (0 ... 120 windows),
// so the Bloom groups are tested by the whole wave together: every lane lists
// its read's groups with a window to look up, the lists are concatenated in
// LDS and each pass takes 64 groups, one per lane (bloom_group without the
// carry: each group's 15-mer orders computed on their own).  Then each lane
// probes its read's remaining windows (na_probe_rest) and settles it as
// k_align_lane_na does.
constexpr int kRcGroups = kLaneMaxW / 8;  // Bloom groups of 8 windows per read
template <bool NEED_Q, bool WIN_Q, bool MG>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(PA_NA_WAVES))) void k_align_lane_rc(AlignArgs a) {
    __shared__ uint64_t rows[kBlock][kLaneWords + 1];
    __shared__ uint32_t glist[kWaves][64 * kRcGroups];      // (lane << 16) | (group << 8) | windows of the group
    __shared__ unsigned long long pmask[kBlock][2];          // per lane: windows the Bloom filter lets through
    rows[threadIdx.x][kLaneWords] = 0;
    const int lane = lane_id();
    const uint32_t wv = threadIdx.x >> 6, wbase = threadIdx.x & ~63u;
    const uint64_t n = *a.queue_rc_count;
    uint32_t n_amb = 0, n_unm = 0;
    uint32_t hr_sum = 0, qf_sum = 0;
    for (uint64_t c0 = (uint64_t)blockIdx.x * kBlock + wbase; c0 < n; c0 += (uint64_t)gridDim.x * kBlock) {
        const uint64_t i = c0 + lane;
        LaneRead<2> S;
        S.kind = LANE_UNMAPPED + 100;  // (past the end: counted nowhere)
        uint32_t r = 0;
        uint64_t seed = 0;
        if (i < n) {
            r = a.queue_rc[i];
            seed = a.queue_rc_anc[i];
            lane_prep<2, NEED_Q, WIN_Q, false>(a, r, ~0ull, rows[threadIdx.x], S);
        }
        const uint64_t *row = rows[threadIdx.x];
        uint32_t gm = 0;  // groups with a window to look up
        uint64_t lk0 = 0, lk1 = 0;
        if (S.kind == LANE_WALK) {
            if (na_rc_walk(a, row, S.len, S.W, seed, lk0, lk1)) {
                if (WIN_Q) {  // windows failing --min-kmer-quality are never looked up
                    lk0 &= ~S.F[0];
                    lk1 &= ~S.F[1];
                }
                if (a.bloom) {
#pragma unroll
                    for (int g = 0; g < kRcGroups; g++)
                        gm |= (((g < 8 ? lk0 >> (8 * g) : lk1 >> (8 * g - 64)) & 0xFFull) != 0) ? 1u << g : 0u;
                }
            } else {
                S.kind = LANE_NOANCHOR;
            }
        }
        // the wave's groups, concatenated
        const uint32_t c = (uint32_t)__popc(gm);
        const uint32_t incl = wave_incl_scan(c);
        const uint32_t total = __shfl(incl, 63);
        // (without a Bloom filter every listed window is probed)
        pmask[threadIdx.x][0] = a.bloom ? 0ull : lk0;
        pmask[threadIdx.x][1] = a.bloom ? 0ull : lk1;
        {
            uint32_t e = incl - c, m = gm;
            while (m) {
                const uint32_t g = (uint32_t)__builtin_ctz(m);
                m &= m - 1;
                const uint32_t wins = (uint32_t)((g < 8 ? lk0 >> (8 * g) : lk1 >> (8 * g - 64)) & 0xFFull);
                glist[wv][e++] = ((uint32_t)lane << 16) | (g << 8) | wins;
            }
        }
        wave_sync();
        // every pass: 64 groups, one per lane (k <= 31 on this path)
#pragma unroll 1
        for (uint32_t base = 0; base < total; base += 64) {
            const uint32_t e = base + lane;
            if (e < total) {
                const uint32_t t = glist[wv][e];
                const uint32_t l = t >> 16, g = (t >> 8) & 255u, act = t & 255u;
                uint32_t pb = 0;
                uint4 cur = make_uint4(0, 0, 0, 0);
                bool cm = true;
                const uint32_t got =
                    a.k == 31 ? bloom_group<8, 31, false>(a, rows[wbase + l], 8 * g, act, true, pb, cur, cm, nullptr)
                              : bloom_group<8, 0, false>(a, rows[wbase + l], 8 * g, act, true, pb, cur, cm, nullptr);
                if (got) atomicOr(&pmask[wbase + l][g >> 3], (unsigned long long)got << (8 * (g & 7)));
            }
        }
        wave_sync();
        if (S.kind == LANE_WALK) {
            bool spec = false;
            uint32_t noff = 0, hr = 0;
            na_probe_rest<MG>(a, row, pmask[threadIdx.x][0], pmask[threadIdx.x][1], spec, noff, hr);
            S.kind = spec ? LANE_HARD : (noff ? LANE_AMB : LANE_UNMAPPED);
            if (!spec) {
                hr_sum += hr;
                qf_sum += S.qf;
            }
        }
        const bool hard = S.kind == LANE_HARD;
        const uint64_t hb = __ballot(hard);
        if (hb) {
            uint64_t qbase = 0;
            if (lane == __builtin_ctzll(hb)) qbase = atomicAdd(a.queue_hard_count, (unsigned long long)__popcll(hb));
            qbase = shfl64(qbase, __builtin_ctzll(hb));
            if (hard) a.queue_hard[qbase + lanes_below(hb)] = r;
        }
        const bool rest = S.kind == LANE_NOANCHOR;  // on to k_align_lane_na
        const uint64_t nb = __ballot(rest);
        if (nb) {
            uint64_t qbase = 0;
            if (lane == __builtin_ctzll(nb)) qbase = atomicAdd(a.queue_na2_count, (unsigned long long)__popcll(nb));
            qbase = shfl64(qbase, __builtin_ctzll(nb));
            if (rest) a.queue_na2[qbase + lanes_below(nb)] = r;
        }
        n_amb += (uint32_t)__popcll(__ballot(S.kind == LANE_AMB));
        n_unm += (uint32_t)__popcll(__ballot(S.kind == LANE_UNMAPPED));
        wave_sync();  // (the group list and the rows are rewritten by the next chunk)
    }
    const uint32_t hr_w = wave_sum(hr_sum);
    const uint32_t qf_w = WIN_Q ? wave_sum(qf_sum) : 0u;
    if (lane == 0) {
        if (n_amb) atomicAdd(&a.stats[1], (unsigned long long)n_amb);
        if (n_unm) atomicAdd(&a.stats[2], (unsigned long long)n_unm);
        if (MG && hr_w) atomicAdd(&a.stats[5], (unsigned long long)hr_w);
        if (WIN_Q && qf_w) atomicAdd(&a.stats[4], (unsigned long long)qf_w);
    }
}
