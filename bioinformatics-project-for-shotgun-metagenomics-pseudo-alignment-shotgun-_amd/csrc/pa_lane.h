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
//   1. the read is 2-bit packed in registers (16-B loads, SWAR codes);
//   2. three seed windows (first, middle, last) are probed in the hash table;
//      a found seed gives the read's position on the concatenated genomes
//      (the key's first occurrence, slot.tpos) -- the anchor;
//   3. the read's packed bases XOR the genome's from the anchor on give the
//      mismatching bases; every window without a mismatch whose genome window
//      is indexed resolves to tile_cls[anchor + w], exactly the table's class;
//   4. the other windows (sequencing errors, N in the genome) are probed; they
//      must all be absent.
// If so, every included k-mer occurs in the anchor genome g, the walked
// windows hold no k-mer twice (no PA_TILE_REP flag, the windows of one read are
// < 127 apart), every specific k-mer is specific to g, and the reference's
// decision collapses: no specific k-mer -> AMBIGUOUS with an empty list
// (src/kmer.py:458-461); else exactly one genome -> UNIQUE g (src/kmer.py:453),
// and the p-check cannot demote (every included k-mer contains g, so no genome
// exceeds g's total; src/kmer.py:464-480).  Any other read -- a found
// non-walked window, a local repeat, no anchor, a non-ACGT base, a k-mer
// quality filter that can bite, a read longer than the lane limits -- is
// queued whole for the wave kernel, which handles every case exactly.

constexpr int kLaneMaxW = 128;    // windows per read on the lane path
constexpr int kLaneMaxLen = 176;  // bases per read on the lane path
constexpr int kLaneChunks = 12;   // 16-B chunks covering shift + kLaneMaxLen bases
constexpr int kLaneWords = 6;     // 64-bit words of the packed read (32 bases each)

enum : int { LANE_UNIQUE = 0, LANE_AMB = 1, LANE_UNMAPPED = 2, LANE_DROP = 3, LANE_HARD = 4 };

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

// Genome containing concatenated position t (binary search over goff).
__device__ __forceinline__ uint32_t genome_of(const uint64_t *goff, uint32_t G, uint64_t t) {
    uint32_t lo = 0, hi = G;  // goff[lo] <= t < goff[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (goff[mid] <= t)
            lo = mid;
        else
            hi = mid;
    }
    return lo;
}

// Up to NP table probes of one lane in flight together, two slots (one 32-B
// aligned pair) per step; linear-probing order is kept exactly.
template <int NP>
__device__ __forceinline__ void lane_probe(const AlignArgs &a, const uint64_t (&key)[NP], uint32_t act,
                                           uint32_t &found, uint32_t (&cls)[NP], uint32_t (&tpos)[NP]) {
    const Slot<1> *table = (const Slot<1> *)a.table;
    uint64_t pos[NP];
#pragma unroll
    for (int i = 0; i < NP; i++) {
        Key<1> kk;
        kk.w[0] = key[i];
        pos[i] = bit(act, i) ? home_of<1>(kk, key_hash(kk), a.home) : 0;
    }
    found = 0;
    while (act) {
        Slot<1> s[NP][2];
#pragma unroll
        for (int i = 0; i < NP; i++)
            if (bit(act, i)) {
                const uint64_t b = pos[i] & ~1ull;
                s[i][0] = table[b];
                s[i][1] = table[b + 1];
            }
#pragma unroll
        for (int i = 0; i < NP; i++) {
            if (!bit(act, i)) continue;
            const uint64_t b = pos[i] & ~1ull;
            bool done = false;
#pragma unroll
            for (int h = 0; h < 2; h++) {
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
            pos[i] = (b + 2 == a.cap) ? 0 : b + 2;
        }
    }
}

struct LaneOut {
    int kind;
    uint32_t genome;  // LANE_UNIQUE
    uint32_t hr;      // windows filtered by --max-genomes
};

#ifdef PA_STATS
#define LANE_HARD_WHY(i) atomicAdd(&a.dbg[4 + (i)], 1ull)
#else
#define LANE_HARD_WHY(i) ((void)0)
#endif

template <bool NEED_Q>
__device__ __forceinline__ LaneOut lane_read(const AlignArgs &a, uint64_t r) {
    LaneOut out{LANE_HARD, 0, 0};
    const int k = a.k;
    const uint32_t flags = a.prm.flags;
    const uint64_t o = a.off[r];
    const uint32_t len = (uint32_t)(a.off[r + 1] - o);
    const uint64_t o0 = o & ~15ull;
    const uint32_t shift = (uint32_t)(o & 15);
    const uint32_t nch = (shift + len + 15) >> 4;
    if (len > (uint32_t)kLaneMaxLen) return LANE_HARD_WHY(0), out;
    // ---- qualities: read mean (src/kmer.py:399, 587) and the k-mer filter bound
    if (NEED_Q) {
        const uint4 *qp = (const uint4 *)(a.qual + o0);
        uint32_t sum = 0, qmin = 255;
#pragma unroll
        for (int c = 0; c < kLaneChunks; c++) {
            if (c >= (int)nch) break;
            const uint4 v = qp[c];
            const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; e++) {
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const uint32_t p = 16 * c + 4 * e + b;
                    const uint32_t q = (d[e] >> (8 * b)) & 255u;
                    const bool in = p >= shift && p < shift + len;
                    sum += in ? q : 0u;
                    qmin = in ? min(qmin, q) : qmin;
                }
            }
        }
        if ((flags & F_MRQ) && (int64_t)sum < (int64_t)a.prm.mrq * (int64_t)len) {
            out.kind = LANE_DROP;  // dropped, not unmapped (src/kmer.py:587-589)
            return out;
        }
        // a window's mean is >= the read's minimum: if that passes, no window can fail
        if ((flags & F_MKQ) && len >= (uint32_t)k && (int64_t)qmin < (int64_t)a.prm.mkq) return LANE_HARD_WHY(1), out;
    }
    if (len < (uint32_t)k) {
        out.kind = LANE_UNMAPPED;  // no windows (src/kmer.py:91-92, 516-517)
        return out;
    }
    const uint32_t W = len - k + 1;
    if (W > (uint32_t)kLaneMaxW) return LANE_HARD_WHY(0), out;
    // ---- 2-bit pack (staged coordinates: base p of the 16-B aligned stretch)
    uint64_t P[kLaneWords + 1];
    uint32_t bad = 0;
    const uint4 *sp = (const uint4 *)(a.seq + o0);
#pragma unroll
    for (int c = 0; c < kLaneChunks; c++) {
        uint32_t half = 0;
        if (c < (int)nch) {
            const uint4 v = sp[c];
            const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const uint32_t cd = swar_codes(d[e]);
                const uint32_t p0 = 16 * c + 4 * e;
                const uint32_t lo = shift > p0 ? shift - p0 : 0u, hi = shift + len > p0 ? shift + len - p0 : 0u;
                const uint32_t inr =
                    (hi >= 4 ? 0xFFFFFFFFu : ((1u << (8 * hi)) - 1)) & (lo >= 4 ? 0u : (0xFFFFFFFFu << (8 * lo)));
                bad |= swar_bad_bytes(d[e], cd) & inr;
                half |= swar_pack_byte(cd) << (24 - 8 * e);
            }
        }
        if (c & 1)
            P[c >> 1] |= half;
        else
            P[c >> 1] = (uint64_t)half << 32;
    }
    P[kLaneWords] = 0;
    if (bad) return LANE_HARD_WHY(2), out;  // non-ACGT base: the wave kernel poisons its windows
    // the read's words from base 0 on
    uint64_t R[kLaneWords];
#pragma unroll
    for (int i = 0; i < kLaneWords; i++) {
        const uint32_t s2 = 2 * shift;
        R[i] = s2 ? ((P[i] << s2) | (P[i + 1] >> (64 - s2))) : P[i];
    }
    const int sh = 64 - 2 * k;
    // ---- seeds: first, middle, last window
    const uint32_t sw[3] = {0u, (W - 1) >> 1, W - 1};
    uint64_t skey[3];
#pragma unroll
    for (int i = 0; i < 3; i++) skey[i] = bits_at(R, 2 * sw[i]) >> sh;
    uint32_t sfound, scls[3], stp[3];
    lane_probe<3>(a, skey, 7u, sfound, scls, stp);
    int at = -1;
#pragma unroll
    for (int pass = 0; pass < 2; pass++)
#pragma unroll
        for (int i = 0; i < 3; i++)
            if (at < 0 && bit(sfound, i) && stp[i] != NONE && (pass == 1 || scls[i] < a.G)) at = i;
    if (at < 0) return LANE_HARD_WHY(3), out;  // no anchor
    uint32_t atp = stp[0], acls = scls[0], aw = sw[0];
#pragma unroll
    for (int i = 1; i < 3; i++)
        if (at == i) {
            atp = stp[i];
            acls = scls[i];
            aw = sw[i];
        }
    // ---- walk from the anchor; a found window off the walk (the read's own
    // genome when a multi-genome seed placed it in another family member) becomes
    // the anchor of a second walk
    uint32_t nspec = 0, nincl = 0, hr = 0, g = 0;
#pragma unroll 1
    for (int attempt = 0;; attempt++) {
        const int64_t A = (int64_t)atp - (int64_t)aw;  // genome position of window 0
        g = acls < a.G ? acls : genome_of(a.goff, a.G, atp);
        const uint64_t gs = a.goff[g], ge = a.goff[g + 1];
        // every window of the read must lie inside the anchor genome
        if (A < (int64_t)gs || (uint64_t)A + W - 1 + k > ge) return LANE_HARD_WHY(4), out;
        // ---- mismatching bases against the genome from A on
        uint64_t mm[kLaneWords];
#pragma unroll
        for (int i = 0; i < kLaneWords; i++) {
            uint64_t d = 0;
            if (32 * i < (int)len) {
                d = R[i] ^ get64_at(a.tile_pk, 2 * (uint64_t)A + 64u * i);
                const uint32_t rest = len - 32 * i;  // bases of the read in this word
                if (rest < 32) d &= ~0ull << (64 - 2 * rest);
            }
            mm[i] = (d | (d >> 1)) & 0x5555555555555555ull;  // one bit per mismatching base
        }
        // windows touching a mismatch: [e - k + 1, e] for every mismatching base e
        uint64_t U0 = 0, U1 = 0;  // windows 0-63, 64-127
        uint32_t nmis = 0;
#pragma unroll
        for (int i = 0; i < kLaneWords; i++) {
            uint64_t m = mm[i];
            while (m) {
                const uint32_t e = 32 * i + (__builtin_clzll(m) >> 1);
                m &= ~(1ull << (62 - 2 * (e & 31)));
                if (++nmis > 8) return LANE_HARD_WHY(5), out;  // a wrong stretch, not a few errors
                const int32_t lo = (int32_t)e - k + 1 < 0 ? 0 : (int32_t)e - k + 1;
                const int32_t hi = (int32_t)e < (int32_t)W - 1 ? (int32_t)e : (int32_t)W - 1;
                if (lo > hi) continue;
                // bits [lo, hi] of the 128-bit mask
                const uint64_t m0 = lo < 64 ? ((~0ull << lo) & (hi >= 63 ? ~0ull : ((2ull << hi) - 1))) : 0ull;
                const uint64_t m1 = hi >= 64 ? ((lo <= 64 ? ~0ull : (~0ull << (lo - 64))) &
                                                (hi >= 127 ? ~0ull : ((2ull << (hi - 64)) - 1)))
                                             : 0ull;
                U0 |= m0;
                U1 |= m1;
            }
        }
        // ---- walked windows: classes from the tile
        const bool has_mg = flags & F_MG;
        nspec = nincl = hr = 0;
        uint64_t P0 = 0, P1 = 0;  // windows to probe
        uint32_t last_c = NONE, last_big = 0;
        const uint32_t *tc = a.tile_cls + A;
        for (uint32_t w = 0; w < W; w++) {
            const bool unmatched = w < 64 ? ((U0 >> w) & 1) : ((U1 >> (w - 64)) & 1);
            const uint32_t v = unmatched ? NONE : tc[w];
            if (v == NONE) {
                if (w < 64)
                    P0 |= 1ull << w;
                else
                    P1 |= 1ull << (w - 64);
                continue;
            }
            if (v & PA_TILE_REP) return LANE_HARD_WHY(6), out;  // the k-mer may repeat inside the read
            if (has_mg) {
                if (v != last_c) {
                    last_c = v;
                    last_big = (int64_t)class_size_of(v, a.G, a.class_genomes) > (int64_t)a.prm.mg;
                }
                if (last_big) {
                    hr++;  // highly redundant (src/kmer.py:425-427)
                    continue;
                }
            }
            nincl++;
            if (v < a.G) {
                if (v != g) return out;  // (cannot happen inside genome g; kept as a guard)
                nspec++;
            }
        }
        // a read with many unwalked windows is cheaper in the wave kernel (a lane
        // would probe them one after the other while the rest of its wave waits)
        if ((uint32_t)(__popcll(P0) + __popcll(P1)) > a.lane_maxpend) return LANE_HARD_WHY(8), out;
        // ---- the other windows: absent, or found off the walk.  A found
        // specific k-mer names the read's genome: walk again from it (once).
        // Found unspecific k-mers alone keep the decision simple only if no
        // specific k-mer is included at all -- then the read is AMBIGUOUS with
        // an empty list whatever the sets (src/kmer.py:458-461).
        bool reanchor = false, off_multi = false;
        while (P0 | P1) {
            uint64_t key4[4];
            uint32_t w4[4], act = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                key4[i] = 0;
                w4[i] = 0;
                if (P0 | P1) {
                    uint32_t w;
                    if (P0) {
                        w = __builtin_ctzll(P0);
                        P0 &= P0 - 1;
                    } else {
                        w = 64 + __builtin_ctzll(P1);
                        P1 &= P1 - 1;
                    }
                    key4[i] = bits_at(R, 2 * w) >> sh;
                    w4[i] = w;
                    act |= 1u << i;
                }
            }
            uint32_t f, c4[4], t4[4];
            lane_probe<4>(a, key4, act, f, c4, t4);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                if (!bit(f, i)) continue;
                const uint32_t c = c4[i];
                if (has_mg && (int64_t)class_size_of(c, a.G, a.class_genomes) > (int64_t)a.prm.mg) {
                    hr++;  // highly redundant: counted, never included
                } else if (c >= a.G) {
                    off_multi = true;
                } else if (!reanchor) {
                    if (attempt > 0 || t4[i] == NONE) return LANE_HARD_WHY(7), out;
                    reanchor = true;
                    atp = t4[i];
                    acls = c;
                    aw = w4[i];
                }
            }
        }
        if (reanchor) continue;
        if (off_multi) {
            if (nspec > 0) return LANE_HARD_WHY(7), out;
            nincl++;  // (only its being nonzero matters below)
        }
        break;
    }
    out.hr = hr;
    if (nincl == 0)
        out.kind = LANE_UNMAPPED;
    else if (nspec == 0)
        out.kind = LANE_AMB;  // only unspecific k-mers: AMBIGUOUS, empty list
    else {
        out.kind = LANE_UNIQUE;
        out.genome = g;
    }
    return out;
}

template <bool NEED_Q>
__global__ __launch_bounds__(kBlock) void k_align_lane(AlignArgs a) {
    extern __shared__ __align__(16) unsigned char smem[];
    const uint32_t G = a.G;
    const bool lds = G <= kLdsGenomeCap;
    unsigned long long *first = (unsigned long long *)smem;
    uint32_t *uniq = (uint32_t *)(first + (lds ? G : 0));
    if (lds) {
        for (uint32_t i = threadIdx.x; i < G; i += kBlock) {
            first[i] = (unsigned long long)PA_NO_FIRST_KEY;
            uniq[i] = 0;
        }
        __syncthreads();
    }
    uint32_t n_uniq = 0, n_amb = 0, n_unm = 0, n_drop = 0, n_hr = 0;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t n_iter = (a.n + stride - 1) / stride;  // uniform trip count (wave-aggregated queueing)
    for (uint64_t it = 0; it < n_iter; it++) {
        const uint64_t r = it * stride + (uint64_t)blockIdx.x * kBlock + threadIdx.x;
        LaneOut res{LANE_UNMAPPED + 100, 0, 0};
        if (r < a.n) res = lane_read<NEED_Q>(a, r);
        const bool hard = res.kind == LANE_HARD;
        const uint64_t hb = __ballot(hard);
        if (hb) {  // one queue allocation per wave
            uint64_t base = 0;
            if (lane_id() == __builtin_ctzll(hb)) base = atomicAdd(a.queue_hard_count, (unsigned long long)__popcll(hb));
            base = shfl64(base, __builtin_ctzll(hb));
            if (hard) a.queue_hard[base + lanes_below(hb)] = (uint32_t)r;
        }
        if (res.kind == LANE_UNIQUE) {
            const uint64_t key = first_key(a.base + r, 0);
            if (lds) {
                atomicAdd(&uniq[res.genome], 1u);
                if (key < first[res.genome]) atomicMin(&first[res.genome], (unsigned long long)key);
            } else {
                atomicAdd(&a.uniq[res.genome], 1ull);
                atomicMin(&a.first[res.genome], (unsigned long long)key);
            }
        }
        n_uniq += res.kind == LANE_UNIQUE;
        n_amb += res.kind == LANE_AMB;
        n_unm += res.kind == LANE_UNMAPPED;
        n_drop += res.kind == LANE_DROP;
        n_hr += (res.kind <= LANE_UNMAPPED) ? res.hr : 0u;
    }
    n_uniq = wave_sum(n_uniq);
    n_amb = wave_sum(n_amb);
    n_unm = wave_sum(n_unm);
    n_drop = wave_sum(n_drop);
    n_hr = wave_sum(n_hr);
    if (lane_id() == 0) {
        if (n_uniq) atomicAdd(&a.stats[0], (unsigned long long)n_uniq);
        if (n_amb) atomicAdd(&a.stats[1], (unsigned long long)n_amb);
        if (n_unm) atomicAdd(&a.stats[2], (unsigned long long)n_unm);
        if (n_drop) atomicAdd(&a.stats[3], (unsigned long long)n_drop);
        if (n_hr && (a.prm.flags & F_MG)) atomicAdd(&a.stats[5], (unsigned long long)n_hr);
    }
    if (lds) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < G; i += kBlock) {
            if (uniq[i]) atomicAdd(&a.uniq[i], (unsigned long long)uniq[i]);
            if (first[i] != (unsigned long long)PA_NO_FIRST_KEY) atomicMin(&a.first[i], first[i]);
        }
    }
}
