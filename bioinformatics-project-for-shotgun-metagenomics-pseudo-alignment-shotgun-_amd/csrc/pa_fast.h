// k_align_fast<NW, WPL, DENSE>: the hot path of
// PseudoAlignment.align_reads_from_container (src/kmer.py:410-480, 563-620).
// Included by pa_align.hip inside its anonymous namespace (uses AlignArgs,
// WgCounters, count_genome, first_key, F_* flags).
//
// Work decomposition: one wavefront per read; every wave owns a CONTIGUOUS chunk
// of reads (sequential offsets and bytes), and while it classifies read r it
// already has the sequence (and quality) dwords of read r+1 in flight, plus the
// offset of read r+2 -- the latency left exposed per read is the table probes.
//
// Register discipline: per-lane predicates are kept as bits of 32-bit integers
// (VGPRs).  `bool x[N]` arrays become 64-bit lane masks in SGPR pairs on AMDGPU,
// and a handful of them spilled ~90 SGPRs into VGPR lanes.
//
// LDS per wave (WPL = 2: 8 KiB): the packed read, its non-ACGT bitmap, the
// staged raw dwords, a 64-bit-key hash (distinct table slots; later the
// multi-genome-set list or the p-check genome hash), a 32-bit-key hash (the
// read's genome sets) and, for the dense path, per-genome specific counts.
//
// Decision paths (template DENSE, chosen per launch):
//   DENSE (G <= 64): lane g owns genome g; specific counts scatter into gcnt/gmin,
//     multi-genome sets contribute through 64-bit membership masks loaded in
//     parallel; everything else is lane arithmetic, DPP reductions, readlanes.
//   hash (G > 64): per-read LDS genome hash; reads whose genome union overflows
//     it are deferred to k_align_exact.

#ifndef PA_HS_PER_WPL
#define PA_HS_PER_WPL 128
#endif
template <int WPL>
struct FastCfg {
    static constexpr int HS = PA_HS_PER_WPL * WPL;     // hash entries per wave (>= windows)
    static constexpr int E = HS / 64;                  // entries owned per lane
    static constexpr int LCAP = 64 * WPL + 64;         // longest read handled (k <= 63)
    static constexpr int NDW = (LCAP + 8 + 255) / 256; // staged dwords per lane
    static constexpr int PW = NDW * 8 + 2;             // packed words (32 staged bases each)
    static constexpr int BW = NDW * 4 + 2;             // non-ACGT bitmap words (64 staged bases each)
};

template <int WPL>
struct __align__(16) WaveLds {
    using C = FastCfg<WPL>;
    uint64_t packed[C::PW];   // the staged bytes 2-bit packed, MSB-first (staged base p at bit 2p)
    uint64_t diff[C::PW];     // packed XOR the anchor genome stretch (genome walk)
    uint64_t poison[C::BW];   // LSB-first bitmap of non-ACGT staged bases
    uint64_t hA_key[C::HS];   // distinct k-mers: key (k <= 31) or table slot; then multi-set masks / p-check genome ids
    uint32_t hA_v[C::HS];     // distinct k-mers: first window; then counts
    uint32_t hA_v2[C::HS];    // first windows
    uint32_t hB_key[C::HS];   // genome set (class id)
    uint32_t hB_cnt[C::HS];   // distinct k-mers of the set
    uint32_t hB_min[C::HS];   // first window of the set
    uint32_t gcnt[64];        // dense path: specific k-mers per genome
    uint32_t gmin[64];        //   and the first window of each
};

template <int WPL>
struct __align__(16) WaveQual {  // only allocated when a quality filter is set
    using C = FastCfg<WPL>;
    uint32_t stage[C::NDW * 64];
    uint32_t pref[C::LCAP + 4];
};

__device__ __forceinline__ uint32_t lds_hash_slot(uint64_t key, uint32_t mask) {
    return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 40) & mask;
}

__device__ __forceinline__ uint32_t lds_insert64(uint64_t *keys, uint32_t hs, uint64_t key) {
    uint32_t p = lds_hash_slot(key, hs - 1);
    for (;;) {
        uint64_t old = atomicCAS((unsigned long long *)&keys[p], (unsigned long long)EMPTY, (unsigned long long)key);
        if (old == EMPTY || old == key) return p;
        p = (p + 1) & (hs - 1);
    }
}

__device__ __forceinline__ uint32_t lds_insert32(uint32_t *keys, uint32_t hs, uint32_t key) {
    uint32_t p = lds_hash_slot(key, hs - 1);
    for (;;) {
        uint32_t old = atomicCAS(&keys[p], NONE, key);
        if (old == NONE || old == key) return p;
        p = (p + 1) & (hs - 1);
    }
}

// Bounded insert for the p-check genome hash; returns hs on overflow.
__device__ __forceinline__ uint32_t lds_insert64_bounded(uint64_t *keys, uint32_t hs, uint64_t key) {
    uint32_t p = lds_hash_slot(key, hs - 1);
    for (uint32_t it = 0; it < hs; it++) {
        uint64_t old = atomicCAS((unsigned long long *)&keys[p], (unsigned long long)EMPTY, (unsigned long long)key);
        if (old == EMPTY || old == key) return p;
        p = (p + 1) & (hs - 1);
    }
    return hs;
}

// Stage NDW dwords per lane covering [o, o + LCAP + 4) (allocations are padded).
template <int WPL>
__device__ __forceinline__ void load_stage(const uint8_t *base, uint64_t o, uint32_t (&d)[FastCfg<WPL>::NDW]) {
    const uint32_t *p = (const uint32_t *)(base + (o & ~3ull));
#pragma unroll
    for (int j = 0; j < FastCfg<WPL>::NDW; j++) d[j] = p[lane_id() + 64 * j];
}

enum : int { OUT_UNIQUE = 0, OUT_AMB = 1, OUT_DEFER = 2, OUT_UNMAPPED = 3, OUT_DROP = 4 };

struct ReadTotals {      // per-lane window counters + read counters (the same in every lane) of a wave
    uint32_t qf = 0, hr = 0;
    uint32_t unique = 0, mapped = 0, unm = 0, drop = 0;
#ifdef PA_STATS
    uint32_t d_win = 0, d_probe = 0, d_walk = 0, d_anchor = 0;
#endif
};

__device__ __forceinline__ bool bit(uint32_t m, int i) { return (m >> i) & 1u; }

// ---- dense decision (G <= 64): lane g owns genome g ------------------------
// L.gcnt / L.gmin hold the specific counts / first windows per genome.  The
// multi-genome sets of the read (membership mask, distinct k-mers, first window
// in L.hA_key / hA_v / hA_v2) are only needed for the p-check, so they come from
// `multi()` on demand (it returns their number); `settled(gstar)` may first
// prove that no genome can exceed G*'s total by more than p.
template <int WPL, typename SettledFn, typename MultiFn>
__device__ __forceinline__ int dense_core(const AlignArgs &a, const WgCounters &wc, WaveLds<WPL> &L, uint64_t r,
                                          bool has_multi, SettledFn settled, MultiFn multi) {
    const int lane = lane_id();
    const uint32_t G = a.G;
    const uint32_t cnt = L.gcnt[lane], smin = L.gmin[lane];
    const uint64_t specb = __ballot(cnt > 0);
    const uint32_t nspec = (uint32_t)__popcll(specb);
    const uint64_t read_idx = a.base + r;
    if (nspec == 0) return OUT_AMB;  // AMBIGUOUS with an empty genome list
    // top = most specific k-mers, ties to the first inserted (smallest first window)
    const uint64_t key = cnt > 0 ? (((uint64_t)cnt << 32) | (NONE - smin)) : 0;
    const uint64_t top = wave_max64(key);
    const int gstar = __builtin_ctzll(__ballot(key == top));
    const uint32_t topcnt = (uint32_t)(top >> 32);
    const uint32_t second = wave_max(lane == gstar ? 0u : cnt);
    const bool unique = nspec == 1 || (int64_t)topcnt >= (int64_t)second + a.prm.m;
    if (!unique) {
        uint32_t rank = 0;
        for (uint64_t m = specb; m; m &= m - 1) rank += __builtin_amdgcn_readlane(smin, __builtin_ctzll(m)) < smin;
        if (cnt > 0) count_genome(a, wc, lane, false, 1, first_key(read_idx, rank));
        return OUT_AMB;
    }
    const uint32_t nmulti = (a.prm.p < 0 || !has_multi || settled(gstar)) ? 0u : multi();
    if (nmulti == 0) {
        if (lane == 0) count_genome(a, wc, gstar, true, 1, first_key(read_idx, 0));
        return OUT_UNIQUE;
    }
    // p-validation: totals over specific + unspecific k-mers (src/kmer.py:464-480)
    uint32_t t = cnt, tmin = cnt > 0 ? smin : NONE;
    for (uint32_t j = 0; j < nmulti; j++) {
        const uint64_t msk = L.hA_key[j];
        if ((msk >> lane) & 1) {
            t += L.hA_v[j];
            tmin = min(tmin, L.hA_v2[j]);
        }
    }
    const uint32_t tstar = __builtin_amdgcn_readlane(t, gstar);
    const uint32_t maxtot = wave_max(t);
    if ((int64_t)maxtot - (int64_t)tstar > a.prm.p) {
        const bool q = (uint32_t)lane < G && t >= tstar;
        const uint64_t qb = __ballot(q);
        const uint64_t me = ((uint64_t)tmin << 32) | (uint32_t)lane;
        uint32_t rank = 1;
        for (uint64_t m = qb; m; m &= m - 1) {
            const int s = __builtin_ctzll(m);
            rank += ((((uint64_t)__builtin_amdgcn_readlane(tmin, s)) << 32) | (uint32_t)s) < me;
        }
        if (q) count_genome(a, wc, lane, false, lane == gstar ? 2 : 1, first_key(read_idx, lane == gstar ? 0 : rank));
        return OUT_AMB;
    }
    if (lane == 0) count_genome(a, wc, gstar, true, 1, first_key(read_idx, 0));
    return OUT_UNIQUE;
}

// Collect the multi-genome sets grouped in the 32-bit-key hash (hB) into the
// list dense_core reads; returns their number.
template <int WPL>
__device__ __forceinline__ uint32_t dense_multi_list(const AlignArgs &a, WaveLds<WPL> &L) {
    using C = FastCfg<WPL>;
    const int lane = lane_id();
    uint32_t nmulti = 0;
#pragma unroll
    for (int e = 0; e < C::E; e++) {
        const int i = lane + 64 * e;
        const uint32_t c = L.hB_key[i];
        const uint32_t is_multi = (c != NONE && c >= a.G) ? 1u : 0u;
        const uint64_t bm = __ballot(is_multi);
        if (is_multi) {
            const uint32_t at = nmulti + lanes_below(bm);
            L.hA_key[at] = a.class_mask[c - a.G];
            L.hA_v[at] = L.hB_cnt[i];
            L.hA_v2[at] = L.hB_min[i];
        }
        nmulti += (uint32_t)__popcll(bm);
    }
    wave_sync();
    return nmulti;
}

// Decision from the genome-set hash hB (every distinct k-mer grouped by set).
template <int WPL>
__device__ __forceinline__ int decide_dense(const AlignArgs &a, const WgCounters &wc, WaveLds<WPL> &L, uint64_t r) {
    using C = FastCfg<WPL>;
    const int lane = lane_id();
#pragma unroll
    for (int e = 0; e < C::E; e++) {
        const int i = lane + 64 * e;
        const uint32_t c = L.hB_key[i];
        if (c < a.G) {  // NONE >= G
            L.gcnt[c] = L.hB_cnt[i];
            L.gmin[c] = L.hB_min[i];
        }
    }
    // hA (distinct k-mer slots) is dead from here on: the multi list may reuse it
    const uint32_t nmulti = dense_multi_list<WPL>(a, L);
    return dense_core<WPL>(a, wc, L, r, nmulti > 0, [](int) { return false; }, [&]() { return nmulti; });
}

// ---- hash decision (G > 64) --------------------------------------------------
template <int WPL>
__device__ __forceinline__ int decide_hash(const AlignArgs &a, const WgCounters &wc, WaveLds<WPL> &L, uint64_t r) {
    using C = FastCfg<WPL>;
    const int lane = lane_id();
    const uint32_t G = a.G;
    uint32_t specm = 0, multim = 0;  // bit e: entry lane + 64e is a singleton / multi-genome set
    uint32_t nspec = 0, nmulti = 0;
    uint64_t top_l = 0;
#pragma unroll
    for (int e = 0; e < C::E; e++) {
        const int i = lane + 64 * e;
        const uint32_t c = L.hB_key[i];
        const uint32_t sp = c < G ? 1u : 0u, mu = (c != NONE && c >= G) ? 1u : 0u;
        specm |= sp << e;
        multim |= mu << e;
        nspec += (uint32_t)__popcll(__ballot(sp));
        nmulti += (uint32_t)__popcll(__ballot(mu));
        if (sp) {
            const uint64_t t = ((uint64_t)L.hB_cnt[i] << 48) | ((uint64_t)(0xFFFFu - L.hB_min[i]) << 32) | c;
            top_l = t > top_l ? t : top_l;
        }
    }
    const uint64_t read_idx = a.base + r;
    if (nspec == 0) return OUT_AMB;
    const uint64_t top = wave_max64(top_l);
    const uint32_t gstar = (uint32_t)top, topcnt = (uint32_t)(top >> 48);
    uint32_t sec_l = 0;
#pragma unroll
    for (int e = 0; e < C::E; e++)
        if (bit(specm, e) && L.hB_key[lane + 64 * e] != gstar) sec_l = max(sec_l, L.hB_cnt[lane + 64 * e]);
    const uint32_t second = wave_max(sec_l);
    const bool unique = nspec == 1 || (int64_t)topcnt >= (int64_t)second + a.prm.m;
    if (!unique) {
        uint32_t mymin[C::E], rank[C::E];
#pragma unroll
        for (int e = 0; e < C::E; e++) {
            mymin[e] = bit(specm, e) ? L.hB_min[lane + 64 * e] : NONE;
            rank[e] = 0;
        }
#pragma unroll
        for (int f = 0; f < C::E; f++) {
            for (uint64_t m = __ballot(bit(specm, f)); m; m &= m - 1) {
                const uint32_t other = L.hB_min[__builtin_ctzll(m) + 64 * f];
#pragma unroll
                for (int e = 0; e < C::E; e++) rank[e] += other < mymin[e];
            }
        }
#pragma unroll
        for (int e = 0; e < C::E; e++)
            if (bit(specm, e)) count_genome(a, wc, L.hB_key[lane + 64 * e], false, 1, first_key(read_idx, rank[e]));
        return OUT_AMB;
    }
    if (a.prm.p < 0 || nmulti == 0) {
        if (lane == 0) count_genome(a, wc, gstar, true, 1, first_key(read_idx, 0));
        return OUT_UNIQUE;
    }
    // p-validation over an LDS genome hash
    wave_sync();
#pragma unroll
    for (int e = 0; e < C::E; e++) {
        const int i = lane + 64 * e;
        L.hA_key[i] = EMPTY;
        L.hA_v[i] = 0;
        L.hA_v2[i] = NONE;
    }
    wave_sync();
    uint32_t ovf = 0;
    const uint32_t limit = (C::HS * 3) / 4;
#pragma unroll
    for (int e = 0; e < C::E; e++)
        if (bit(specm, e)) {
            const int i = lane + 64 * e;
            const uint32_t p = lds_insert64_bounded(L.hA_key, C::HS, L.hB_key[i]);
            if (p >= (uint32_t)C::HS) {
                ovf = 1;
            } else {
                atomicAdd(&L.hA_v[p], L.hB_cnt[i]);
                atomicMin(&L.hA_v2[p], L.hB_min[i]);
            }
        }
#pragma unroll
    for (int f = 0; f < C::E; f++) {
        for (uint64_t m = __ballot(bit(multim, f)); m; m &= m - 1) {  // wave-uniform walk over multi sets
            const uint32_t i = __builtin_ctzll(m) + 64 * f;
            const uint32_t c = L.hB_key[i], cnt = L.hB_cnt[i], mw = L.hB_min[i];
            const uint32_t *rec = a.class_genomes + (c - G);  // [size, genomes...]
            const uint32_t sz = rec[0];
            if (sz > limit) {
                ovf = 1;
                break;
            }
            for (uint32_t j = lane; j < sz; j += 64) {
                const uint32_t p = lds_insert64_bounded(L.hA_key, C::HS, rec[1 + j]);
                if (p >= (uint32_t)C::HS) {
                    ovf = 1;
                } else {
                    atomicAdd(&L.hA_v[p], cnt);
                    atomicMin(&L.hA_v2[p], mw);
                }
            }
        }
    }
    wave_sync();
    uint32_t claimed = 0;
#pragma unroll
    for (int e = 0; e < C::E; e++) claimed += (uint32_t)__popcll(__ballot(L.hA_key[lane + 64 * e] != EMPTY));
    if (__ballot(ovf) || claimed > limit) {
        // the read's genome union does not fit the wave's LDS: the exact kernel takes it
        if (lane == 0) a.queue[atomicAdd(a.qcount, 1ull)] = (uint32_t)r;
        return OUT_DEFER;
    }
    uint32_t ts_l = 0, mx_l = 0;
#pragma unroll
    for (int e = 0; e < C::E; e++) {
        const int i = lane + 64 * e;
        if (L.hA_key[i] == EMPTY) continue;
        mx_l = max(mx_l, L.hA_v[i]);
        if (L.hA_key[i] == gstar) ts_l = L.hA_v[i];
    }
    const uint32_t tstar = wave_max(ts_l), maxtot = wave_max(mx_l);
    if ((int64_t)maxtot - (int64_t)tstar > a.prm.p) {
        uint32_t qm = 0;
        uint64_t me[C::E];
        uint32_t rank[C::E];
#pragma unroll
        for (int e = 0; e < C::E; e++) {
            const int i = lane + 64 * e;
            qm |= (L.hA_key[i] != EMPTY && L.hA_v[i] >= tstar ? 1u : 0u) << e;
            me[e] = ((uint64_t)L.hA_v2[i] << 32) | (uint32_t)L.hA_key[i];
            rank[e] = 1;
        }
#pragma unroll
        for (int f = 0; f < C::E; f++) {
            for (uint64_t m = __ballot(bit(qm, f)); m; m &= m - 1) {
                const uint32_t i = __builtin_ctzll(m) + 64 * f;
                const uint64_t other = ((uint64_t)L.hA_v2[i] << 32) | (uint32_t)L.hA_key[i];
#pragma unroll
                for (int e = 0; e < C::E; e++) rank[e] += other < me[e];
            }
        }
#pragma unroll
        for (int e = 0; e < C::E; e++) {
            if (!bit(qm, e)) continue;
            const uint32_t g = (uint32_t)me[e];
            if (g == gstar)
                count_genome(a, wc, g, false, 2, first_key(read_idx, 0));
            else
                count_genome(a, wc, g, false, 1, first_key(read_idx, rank[e]));
        }
        return OUT_AMB;
    }
    if (lane == 0) count_genome(a, wc, gstar, true, 1, first_key(read_idx, 0));
    return OUT_UNIQUE;
}

// ---- one read --------------------------------------------------------------------
//
// Per-lane window state: window j of the lane is read window lane + 64 j; bit j
// of `pend` / `inc` = unresolved / included.
template <int NW, int WPL>
struct Windows {
    Key<NW> key[WPL];
    uint64_t slot[NW == 1 ? 1 : WPL];  // table slot = k-mer identity for multi-word keys
    uint32_t cls[WPL];
    uint32_t pend, inc, qf, hr;
    uint32_t walk;  // windows resolved by the genome walk
    uint32_t ga;    // genome of the walk's anchor when its seed was specific, else NONE
};

// ASCII -> 2-bit codes of four bases at once: ((c >> 1) ^ (c >> 2)) & 3 maps
// A C G T to 0 1 2 3; a byte is a base iff "ACGT"[code] gives it back.
__device__ __forceinline__ uint32_t swar_codes(uint32_t x) { return ((x >> 1) ^ (x >> 2)) & 0x03030303u; }
__device__ __forceinline__ uint32_t swar_bad_bytes(uint32_t x, uint32_t codes) {
    const uint32_t d = x ^ __builtin_amdgcn_perm(0u, 0x54474341u, codes);  // byte lookup in "ACGT"
    return ((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu | d) & 0x80808080u;           // high bit of every nonzero byte
}
// Four codes (byte i = base i) -> one byte, first base in the top bits.
__device__ __forceinline__ uint32_t swar_pack_byte(uint32_t codes) {
    return (codes * ((1u << 30) | (1u << 20) | (1u << 10) | 1u)) >> 24;
}

// Stage, filter and pack one read; window keys, ok bits and filter counts go to
// `S`.  Staged coordinates: the read's bytes start `shift` bytes into the
// staging buffer, so read window w is staged (and packed) position w + shift.
// Returns false if the read has no windows to resolve (dropped by
// --min-read-quality).
template <int NW, int WPL, bool DENSE>
__device__ __forceinline__ bool prep_read(const AlignArgs &a, WaveLds<WPL> &L, WaveQual<WPL> *Q, bool need_q,
                                          uint32_t shift, uint32_t len, const uint32_t (&sd)[FastCfg<WPL>::NDW],
                                          const uint32_t (&qd)[FastCfg<WPL>::NDW], Windows<NW, WPL> &S,
                                          ReadTotals &tot) {
    using C = FastCfg<WPL>;
    const int lane = lane_id();
    const int k = a.k;
    const uint32_t flags = a.prm.flags;
    const uint32_t W = (len >= (uint32_t)k) ? len - k + 1 : 0;
    wave_sync();  // the previous read is done with the LDS
    if (need_q) {
#pragma unroll
        for (int j = 0; j < C::NDW; j++) Q->stage[lane + 64 * j] = qd[j];
    }
    // per-read LDS state of the dense decision
    if (DENSE && NW == 1) {
        L.gcnt[lane] = 0;
        L.gmin[lane] = NONE;
#pragma unroll
        for (int e = 0; e < C::E; e++) L.hA_key[C::E * lane + e] = EMPTY;  // contiguous: wide stores
    }
    // ---- 2-bit pack (4 bases per lane and staged dword) + non-ACGT test
    uint32_t badany = 0;
    uint8_t *pk8 = (uint8_t *)L.packed;
#pragma unroll
    for (int j = 0; j < C::NDW; j++) {
        const uint32_t x = sd[j];
        const uint32_t cd = swar_codes(x);
        const uint32_t p0 = 4u * (lane + 64 * j);  // staged position of the dword's first byte
        uint32_t bad = swar_bad_bytes(x, cd);
        // only bytes inside the read count
        const uint32_t lo = shift > p0 ? shift - p0 : 0u, hi = shift + len > p0 ? shift + len - p0 : 0u;
        const uint32_t inr = (hi >= 4 ? 0xFFFFFFFFu : ((1u << (8 * hi)) - 1)) & (lo >= 4 ? 0u : (0xFFFFFFFFu << (8 * lo)));
        badany |= bad & inr;
        pk8[(lane + 64 * j) ^ 7] = (uint8_t)swar_pack_byte(cd);
    }
    if (lane < 2) L.packed[C::PW - 2 + lane] = 0;
    const bool any_bad = __ballot(badany != 0) != 0;
    if (any_bad) {  // rare: reads are ACGT by grammar (src/records.py:262); mark every bad base
        if (lane < C::BW) L.poison[lane] = 0;
        wave_sync();
#pragma unroll
        for (int j = 0; j < C::NDW; j++) {
            const uint32_t x = sd[j];
            const uint32_t p0 = 4u * (lane + 64 * j);
            const uint32_t lo = shift > p0 ? shift - p0 : 0u, hi = shift + len > p0 ? shift + len - p0 : 0u;
            const uint32_t inr =
                (hi >= 4 ? 0xFFFFFFFFu : ((1u << (8 * hi)) - 1)) & (lo >= 4 ? 0u : (0xFFFFFFFFu << (8 * lo)));
            const uint32_t bad = swar_bad_bytes(x, swar_codes(x)) & inr;
            const uint32_t nib = ((bad >> 7) & 1u) | ((bad >> 14) & 2u) | ((bad >> 21) & 4u) | ((bad >> 28) & 8u);
            if (nib) atomicOr((uint32_t *)L.poison + (p0 >> 5), nib << (p0 & 31));
        }
    }
    wave_sync();
    // ---- raw-ASCII quality prefix sums (src/kmer.py:399, 408)
    if (need_q) {  // (not `if (Q)`: a null test of an LDS pointer miscompiles)
        const uint8_t *qb = (const uint8_t *)Q->stage + shift;
        uint32_t carry = 0;
        for (uint32_t c0 = 0; c0 < len; c0 += 64) {
            const uint32_t i = c0 + lane;
            const uint32_t s = wave_incl_scan(i < len ? (uint32_t)qb[i] : 0u) + carry;
            Q->pref[i + 1] = s;
            carry = __shfl(s, 63);
        }
        if (lane == 0) Q->pref[0] = 0;
        wave_sync();
        if ((flags & F_MRQ) && (int64_t)Q->pref[len] < (int64_t)a.prm.mrq * (int64_t)len) {
            return false;  // dropped, not unmapped (src/kmer.py:587-589)
        }
    }
    // ---- windows: quality gate, key (src/kmer.py:419-429)
    const int64_t mkq_k = (int64_t)a.prm.mkq * k;
    S.pend = S.inc = S.qf = S.hr = S.walk = 0;
    S.ga = NONE;
#pragma unroll
    for (int j = 0; j < WPL; j++) {
        const uint32_t w = lane + 64 * j;
        uint32_t ok = w < W ? 1u : 0u;
        if (ok && (flags & F_MKQ) && (int64_t)(Q->pref[w + k] - Q->pref[w]) < mkq_k) {
            S.qf++;
            ok = 0;
        }
        if (ok && any_bad && window_any(L.poison, w + shift, k)) ok = 0;
        S.key[j] = extract_key<NW>(L.packed, w + shift, k);
        S.pend |= ok << j;
    }
    return true;
}

// Resolve the windows of a read (its global-memory phase).
template <int NW, int WPL>
__device__ __forceinline__ void resolve_read(const AlignArgs &a, WaveLds<WPL> &L, uint32_t shift,
                                             Windows<NW, WPL> &S, ReadTotals &tot) {
    using C = FastCfg<WPL>;
    const int lane = lane_id();
    const int k = a.k;
    const uint32_t flags = a.prm.flags;
    const Slot<NW> *table = (const Slot<NW> *)a.table;
    // a window whose k-mer is in the index: --max-genomes gate, else included
    auto resolve = [&](int j, uint32_t c) {
        c = cls_of(c);  // (a slot's raw class: without its position bit)
        S.cls[j] = c;
        if ((flags & F_MG) && (int64_t)class_size_of(c, a.G, a.class_genomes) > (int64_t)a.prm.mg)
            S.hr++;  // highly redundant k-mer (src/kmer.py:425-427)
        else
            S.inc |= 1u << j;
    };
    // hash-table probes of the windows in m, all of a lane's in flight together;
    // returns the windows found (first-occurrence positions in tp)
    auto probe = [&](uint32_t m, uint32_t (&tp)[WPL]) -> uint32_t {
        uint32_t found = 0;
#ifdef PA_STATS
        tot.d_probe += __popc(m);
#endif
        uint64_t pos[WPL];
#pragma unroll
        for (int j = 0; j < WPL; j++)
            if (bit(m, j)) pos[j] = home_of<NW>(S.key[j], key_hash(S.key[j]), a.home);
        while (__ballot(m != 0)) {
            Slot<NW> s[WPL];
#pragma unroll
            for (int j = 0; j < WPL; j++)
                if (bit(m, j)) s[j] = table[pos[j]];
#pragma unroll
            for (int j = 0; j < WPL; j++) {
                if (!bit(m, j)) continue;
                if (s[j].key[0] == EMPTY) {
                    m &= ~(1u << j);
                    continue;
                }
                bool eq = true;
#pragma unroll
                for (int t = 0; t < NW; t++) eq &= (s[j].key[t] == S.key[j].w[t]);
                if (eq) {
                    m &= ~(1u << j);
                    found |= 1u << j;
                    tp[j] = s[j].tpos;
                    if constexpr (NW > 1) S.slot[j] = pos[j];
                    resolve(j, s[j].cls);
                } else if (probe_past<NW>(s[j], S.key[j], pos[j], a.home)) {
                    m &= ~(1u << j);  // ordered clusters: homed after this key, so it is absent
                } else {
                    pos[j] = (pos[j] + 1 == a.cap) ? 0 : pos[j] + 1;
                }
            }
        }
        return found;
    };
    uint32_t tp[WPL];
    if constexpr (NW == 1) {
        // One lane per probe: keys are re-extracted from the packed read in LDS,
        // so the probing lanes need not own the windows they probe.
        // Linear probing a 64-B line (4 slots) per step: cap is a multiple of 4
        // and the table 64-B aligned, so the slots from pos to the line's end
        // come in one memory request, and most searches -- hits and misses --
        // end in their first line.
        auto probe_one = [&](bool act, uint32_t w, uint32_t &cls, uint32_t &tpos) -> bool {
            const Key<1> key = extract_key<1>(L.packed, w + shift, k);
            uint64_t pos = act ? home_of<1>(key, key_hash(key), a.home) : 0;
            bool found = false;
            while (__ballot(act)) {
                if (act) {
                    const uint64_t base = pos & ~3ull;
                    Slot<1> s[4];
#pragma unroll
                    for (int i = 0; i < 4; i++) s[i] = table[base + i];
                    bool done = false;
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        if (done || base + i < pos) continue;
                        if (s[i].key[0] == EMPTY) {
                            done = true;
                        } else if (s[i].key[0] == key.w[0]) {
                            done = true;
                            found = true;
                            cls = s[i].cls;
                            tpos = s[i].tpos;
                        }
                    }
                    if (!done) done = probe_past<1>(s[3], key, base + 3, a.home);
                    act = !done;
                    pos = (base + 4 == a.cap) ? 0 : base + 4;
                }
            }
            return found;
        };
        // ---- genome walk: probe three seed windows (first, middle, last pending);
        // a found seed places the read on the concatenated genomes (its key's
        // first occurrence) and every pending window is checked against the
        // genome at the same offset -- the read's packed bases XOR the genome's
        // (a few words) plus one contiguous tile_cls load, instead of a random
        // probe per window.  A window counts as resolved only if its k bases equal
        // the genome's and an indexed window starts there, so its class is
        // exactly the table's.  Seeds stay pending: the walk (or the final
        // probes) resolves them like any other window.
        const int sh = 64 - 2 * k;
#pragma unroll 1
        for (int round = 0; round < a.walk_rounds; round++) {
            uint64_t pb[WPL];
#pragma unroll
            for (int j = 0; j < WPL; j++) pb[j] = __ballot(bit(S.pend, j));
            int wf = -1, wl = -1;
#pragma unroll
            for (int j = 0; j < WPL; j++)
                if (pb[j] && wf < 0) wf = 64 * j + __builtin_ctzll(pb[j]);
#pragma unroll
            for (int j = WPL - 1; j >= 0; j--)
                if (pb[j] && wl < 0) wl = 64 * j + 63 - __builtin_clzll(pb[j]);
            if (wf < 0) break;
            const int mid = (wf + wl) >> 1;
            int wm = wl;
#pragma unroll
            for (int j = WPL - 1; j >= 0; j--) {
                const int lo = mid - 64 * j;
                const uint64_t m = lo <= 0 ? pb[j] : (lo >= 64 ? 0ull : (pb[j] & (~0ull << lo)));
                if (m) wm = 64 * j + __builtin_ctzll(m);
            }
            const uint32_t sw = lane == 0 ? (uint32_t)wf : lane == 1 ? (uint32_t)wm : (uint32_t)wl;
            uint32_t scls = NONE, stp = NONE;
#ifdef PA_STATS
            tot.d_probe += lane < 3 ? 1u : 0u;
#endif
            const bool sf = probe_one(lane < 3, sw, scls, stp) && stp != NONE;
            // anchor: a specific seed (its genome is the read's), else any found one
            const uint64_t b1 = __ballot(sf && cls_of(scls) < a.G), b2 = __ballot(sf);
            if (!b2) continue;
            const int l = (int)__builtin_ctzll(b1 ? b1 : b2);
            const uint32_t ga = b1 ? cls_of(__builtin_amdgcn_readlane(scls, l)) : NONE;
            const uint32_t lcls = __builtin_amdgcn_readlane(scls, l), ltp = __builtin_amdgcn_readlane(stp, l);
            const int64_t A = (int64_t)first_pos(lcls, ltp, a.G, a.class_genomes, a.goff, a.tpos_local) -
                              (int64_t)__builtin_amdgcn_readlane(sw, l);
            const int64_t g0 = A - (int64_t)shift;  // genome position of staged base 0
            if (g0 < 0) continue;
            // walk bits (and the anchor genome) only in round 0 and only inside the
            // anchor genome's own range: a read may match across a genome boundary
            uint64_t gs = 0, ge = 0;
            if (round == 0 && ga != NONE) {
                S.ga = ga;
                gs = a.goff[ga];
                ge = a.goff[ga + 1];
            }
#ifdef PA_STATS
            if (lane == 0) tot.d_anchor++;
#endif
            // diff words: staged packed bases XOR the genome from g0 on (tile_pk is padded)
            if (lane < C::PW - 1) L.diff[lane] = L.packed[lane] ^ get64_at(a.tile_pk, 2 * (uint64_t)g0 + 64u * lane);
            uint32_t tc[WPL];
#pragma unroll
            for (int j = 0; j < WPL; j++) {
                tc[j] = NONE;
                const uint64_t t = (uint64_t)(A + lane + 64 * j);
                if (bit(S.pend, j) && t < a.tile_n) {
                    const uint32_t v = a.tile_cls[t];
                    tc[j] = v == NONE ? NONE : (v & ~PA_TILE_REP);
                }
            }
            wave_sync();
#pragma unroll
            for (int j = 0; j < WPL; j++)
                if (tc[j] != NONE && (get64(L.diff, 2 * (lane + 64 * j + shift)) >> sh) == 0) {
#ifdef PA_STATS
                    tot.d_walk++;
#endif
                    S.pend &= ~(1u << j);
                    const uint64_t t = (uint64_t)(A + lane + 64 * j);
                    if (t >= gs && t < ge) S.walk |= 1u << j;
                    resolve(j, tc[j]);
                }
        }
        // ---- remaining windows: compact them onto the lanes, one probe per lane
        uint32_t *list = L.hA_v, *res = L.hA_v2;  // free until the decision
        uint32_t npend = 0;
#pragma unroll
        for (int j = 0; j < WPL; j++) {
            const uint64_t b = __ballot(bit(S.pend, j));
            if (bit(S.pend, j)) list[npend + lanes_below(b)] = lane + 64 * j;
            npend += (uint32_t)__popcll(b);
        }
        if (npend == 0) return;
        wave_sync();
#ifdef PA_STATS
        tot.d_probe += lane < (int)npend ? 1u : 0u;
#endif
        for (uint32_t base = 0; base < npend; base += 64) {
            const bool act = base + lane < npend;
            const uint32_t w = act ? list[base + lane] : 0u;
            uint32_t c = NONE, t = NONE;
            probe_one(act, w, c, t);  // not found: c stays NONE (never a class id)
            if (act) res[w] = c;
        }
        wave_sync();
#pragma unroll
        for (int j = 0; j < WPL; j++)
            if (bit(S.pend, j)) {
                const uint32_t c = res[lane + 64 * j];
                if (c != NONE) resolve(j, c);
            }
        S.pend = 0;
        return;
    }
    probe(S.pend, tp);  // multi-word keys: every window probes
    S.pend = 0;
}

// Distinct k-mers, genome sets and the decision: the hash path (any NW, any G).
template <int NW, int WPL, bool DENSE>
__device__ __forceinline__ int decide_general(const AlignArgs &a, const WgCounters &wc, WaveLds<WPL> &L,
                                              const Windows<NW, WPL> &S, uint64_t r) {
    using C = FastCfg<WPL>;
    const int lane = lane_id();
    const uint32_t incm = S.inc;
    // ---- clear the hashes
#pragma unroll
    for (int e = 0; e < C::E; e++) {
        const int i = lane + 64 * e;
        L.hA_key[i] = EMPTY;
        L.hA_v[i] = NONE;
        L.hB_key[i] = NONE;
        L.hB_cnt[i] = 0;
        L.hB_min[i] = NONE;
    }
    if (DENSE) {
        L.gcnt[lane] = 0;
        L.gmin[lane] = NONE;
    }
    wave_sync();
    // ---- distinct k-mers: first window per k-mer (quirk 3); the identity is the
    // key itself for single-word keys, the table slot otherwise
    uint32_t hp[WPL];
#pragma unroll
    for (int j = 0; j < WPL; j++)
        if (bit(incm, j)) {
            uint64_t id;
            if constexpr (NW == 1)
                id = S.key[j].w[0];
            else
                id = S.slot[j];
            hp[j] = lds_insert64(L.hA_key, C::HS, id);
            atomicMin(&L.hA_v[hp[j]], (uint32_t)(lane + 64 * j));
        }
    wave_sync();
    // ---- group the distinct k-mers by genome set
#pragma unroll
    for (int j = 0; j < WPL; j++)
        if (bit(incm, j) && L.hA_v[hp[j]] == (uint32_t)(lane + 64 * j)) {
            const uint32_t p = lds_insert32(L.hB_key, C::HS, S.cls[j]);
            atomicAdd(&L.hB_cnt[p], 1u);
            atomicMin(&L.hB_min[p], (uint32_t)(lane + 64 * j));
        }
    wave_sync();
    if (DENSE)
        return decide_dense<WPL>(a, wc, L, r);
    else
        return decide_hash<WPL>(a, wc, L, r);
}

// Dense decision for single-word keys.  Distinct k-mers (quirk 3) by one LDS
// hash insert per window: the window whose insert lands counts its k-mer once,
// every window of a k-mer still takes part in the first-window minimum (all of
// them share its genome set, so the minimum over all windows is the minimum
// over the k-mer's first windows).  Specific k-mers go straight to their
// genome's counter and first window; the multi-genome sets are grouped only
// when the p-check needs them.
template <int WPL>
__device__ __forceinline__ int decide_dense_fast(const AlignArgs &a, const WgCounters &wc, WaveLds<WPL> &L,
                                                 const Windows<1, WPL> &S, uint64_t r) {
    using C = FastCfg<WPL>;
    const int lane = lane_id();
    const uint32_t incm = S.inc;
    uint32_t firstm = 0, multim = 0;
#pragma unroll
    for (int j = 0; j < WPL; j++)
        if (bit(incm, j)) {
            const uint64_t key = S.key[j].w[0];
            uint32_t p = lds_hash_slot(key, C::HS - 1);
            for (;;) {
                const uint64_t old = atomicCAS((unsigned long long *)&L.hA_key[p], (unsigned long long)EMPTY,
                                               (unsigned long long)key);
                if (old == EMPTY) firstm |= 1u << j;
                if (old == EMPTY || old == key) break;
                p = (p + 1) & (C::HS - 1);
            }
            const uint32_t c = S.cls[j];
            if (c < a.G) {
                if (bit(firstm, j)) atomicAdd(&L.gcnt[c], 1u);
                atomicMin(&L.gmin[c], (uint32_t)(lane + 64 * j));
            } else {
                multim |= 1u << j;
            }
        }
    const bool has_multi = __ballot(multim != 0) != 0;
    wave_sync();
#ifdef PA_STATS
    if (a.dbg_mode == 4) return OUT_AMB;
#endif
    // p-check bound: total[g] - total[G*] <= #distinct k-mers whose set lacks G*;
    // if that is <= p no demotion is possible (src/kmer.py:469-480).  Windows the
    // genome walk resolved lie in the anchor genome, so when that is G* they
    // contain it without a look at their set.
    auto settled = [&](int gstar) -> bool {
        uint32_t lack = 0;
#pragma unroll
        for (int j = 0; j < WPL; j++)
            if (bit(firstm, j)) {
                const uint32_t c = S.cls[j];
                bool has;
                if (c < a.G)
                    has = c == (uint32_t)gstar;
                else if (bit(S.walk, j) && S.ga == (uint32_t)gstar)
                    has = true;
                else
                    has = (a.class_mask[c - a.G] >> gstar) & 1;
                lack += has ? 0u : 1u;
            }
        return (int64_t)wave_sum(lack) <= (int64_t)a.prm.p;
    };
    return dense_core<WPL>(a, wc, L, r, has_multi, settled, [&]() -> uint32_t {
#pragma unroll
        for (int e = 0; e < C::E; e++) {
            const int i = lane + 64 * e;
            L.hB_key[i] = NONE;
            L.hB_cnt[i] = 0;
            L.hB_min[i] = NONE;
        }
        wave_sync();
#pragma unroll
        for (int j = 0; j < WPL; j++)
            if (bit(multim, j)) {
                const uint32_t p = lds_insert32(L.hB_key, C::HS, S.cls[j]);
                if (bit(firstm, j)) atomicAdd(&L.hB_cnt[p], 1u);
                atomicMin(&L.hB_min[p], (uint32_t)(lane + 64 * j));
            }
        wave_sync();
        return dense_multi_list<WPL>(a, L);
    });
}

template <int NW, int WPL, bool DENSE>
__device__ __forceinline__ int classify_read(const AlignArgs &a, const WgCounters &wc, WaveLds<WPL> &L,
                                             WaveQual<WPL> *Q, bool need_q, uint64_t r, uint32_t shift, uint32_t len,
                                             const uint32_t (&sd)[FastCfg<WPL>::NDW],
                                             const uint32_t (&qd)[FastCfg<WPL>::NDW], Windows<NW, WPL> &S,
                                             ReadTotals &tot) {
    if (!prep_read<NW, WPL, DENSE>(a, L, Q, need_q, shift, len, sd, qd, S, tot)) return OUT_DROP;
#ifdef PA_STATS
    tot.d_win += __popc(S.pend);
    if (a.dbg_mode == 2) return OUT_UNMAPPED;
#endif
    resolve_read<NW, WPL>(a, L, shift, S, tot);
#ifdef PA_STATS
    if (a.dbg_mode == 3) return OUT_UNMAPPED;
#endif
    if (!__ballot(S.inc != 0)) return OUT_UNMAPPED;  // no k-mer references (src/kmer.py:516-517)
    if constexpr (DENSE && NW == 1)
        return decide_dense_fast<WPL>(a, wc, L, S, r);
    else
        return decide_general<NW, WPL, DENSE>(a, wc, L, S, r);
}

// One read; the read counters are updated in one place from the outcome (LLVM
// merges per-branch increments of different fields into an indexed store,
// which moves the counters to scratch memory).
template <int NW, int WPL, bool DENSE>
__device__ __forceinline__ void fast_read(const AlignArgs &a, const WgCounters &wc, WaveLds<WPL> &L,
                                          WaveQual<WPL> *Q, bool need_q, uint64_t r, uint32_t shift, uint32_t len,
                                          const uint32_t (&sd)[FastCfg<WPL>::NDW],
                                          const uint32_t (&qd)[FastCfg<WPL>::NDW], ReadTotals &tot) {
    Windows<NW, WPL> S;
    const int out = classify_read<NW, WPL, DENSE>(a, wc, L, Q, need_q, r, shift, len, sd, qd, S, tot);
    // a dropped read has no window counts; a deferred one is counted by the exact kernel
    const bool counted = out != OUT_DROP && out != OUT_DEFER;
    tot.qf += counted ? S.qf : 0u;
    tot.hr += counted ? S.hr : 0u;
    tot.unique += out == OUT_UNIQUE ? 1u : 0u;
    tot.mapped += (out == OUT_UNIQUE || out == OUT_AMB) ? 1u : 0u;
    tot.unm += out == OUT_UNMAPPED ? 1u : 0u;
    tot.drop += out == OUT_DROP ? 1u : 0u;
}

#ifndef PA_FAST_MIN_WAVES
#define PA_FAST_MIN_WAVES 1
#endif
template <int NW, int WPL, bool DENSE>
__global__ __launch_bounds__(kBlock, PA_FAST_MIN_WAVES) void k_align_fast(AlignArgs a) {
    using C = FastCfg<WPL>;
    extern __shared__ __align__(16) unsigned char smem[];
    const int lane = lane_id();
    const int wid = threadIdx.x >> 6;
    const uint32_t G = a.G;
    const bool need_q = a.prm.flags & (F_MRQ | F_MKQ);

    WgCounters wc;
    wc.lds = G <= kLdsGenomeCap;
    const uint32_t Gl = wc.lds ? ((G + 1) & ~1u) : 0;
    wc.first = (unsigned long long *)smem;
    wc.uniq = (uint32_t *)(wc.first + Gl);
    wc.amb = wc.uniq + Gl;
    unsigned char *wave_base = smem + ((size_t)Gl * 16 + 15) / 16 * 16;
    WaveLds<WPL> &L = ((WaveLds<WPL> *)wave_base)[wid];
    WaveQual<WPL> *Q = ((WaveQual<WPL> *)(wave_base + kWaves * sizeof(WaveLds<WPL>))) + wid;  // used iff need_q
    for (uint32_t i = threadIdx.x; i < Gl; i += kBlock) {
        wc.first[i] = (unsigned long long)PA_NO_FIRST_KEY;
        wc.uniq[i] = 0;
        wc.amb[i] = 0;
    }
    __syncthreads();

    // contiguous chunk of reads (or of the read list) for this wave; the bytes of
    // the next read are loaded while the current one is classified
    const uint64_t nq = a.rlist ? (uint64_t)*a.rlist_count : a.n;
    const uint64_t nw = (uint64_t)gridDim.x * kWaves, gw = (uint64_t)blockIdx.x * kWaves + wid;
    const uint64_t qb = nq * gw / nw, qe = nq * (gw + 1) / nw;
    ReadTotals tot;
    if (qb < qe) {
        uint64_t r = a.rlist ? a.rlist[qb] : qb;
        uint64_t o_cur = a.off[r], o_end = a.off[r + 1];
        uint32_t sd[C::NDW], qd[C::NDW];
        load_stage<WPL>(a.seq, o_cur, sd);
        if (need_q) load_stage<WPL>(a.qual, o_cur, qd);
        for (uint64_t q = qb; q < qe; q++) {
            uint64_t r_n = 0, o_n = 0, e_n = 0;
            uint32_t sn[C::NDW], qn[C::NDW];
            if (q + 1 < qe) {  // prefetch the next read while this one is classified
                r_n = a.rlist ? a.rlist[q + 1] : q + 1;
                o_n = a.off[r_n];
                e_n = a.off[r_n + 1];
                load_stage<WPL>(a.seq, o_n, sn);
                if (need_q) load_stage<WPL>(a.qual, o_n, qn);
            }
            const uint32_t len = (uint32_t)(o_end - o_cur);
            const uint32_t W = (len >= (uint32_t)a.k) ? len - a.k + 1 : 0;
            if (W > 64u * WPL || len > (uint32_t)(C::LCAP - 8)) {
                if (lane == 0) a.queue[atomicAdd(a.qcount, 1ull)] = (uint32_t)r;  // the exact kernel takes it
            } else {
                fast_read<NW, WPL, DENSE>(a, wc, L, Q, need_q, r, (uint32_t)(o_cur & 3), len, sd, qd, tot);
            }
            r = r_n;
            o_cur = o_n;
            o_end = e_n;
#pragma unroll
            for (int j = 0; j < C::NDW; j++) {
                sd[j] = sn[j];
                qd[j] = qn[j];
            }
        }
    }
    // ---- flush
    const uint32_t qf_w = wave_sum(tot.qf), hr_w = wave_sum(tot.hr);
    const bool has_mkq = a.prm.flags & F_MKQ, has_mg = a.prm.flags & F_MG;
#ifdef PA_STATS
    {
        const uint32_t s0 = wave_sum(tot.d_win), s1 = wave_sum(tot.d_probe), s2 = wave_sum(tot.d_walk),
                       s3 = wave_sum(tot.d_anchor);
        if (lane == 0) {
            atomicAdd(&a.dbg[0], (unsigned long long)s0);
            atomicAdd(&a.dbg[1], (unsigned long long)s1);
            atomicAdd(&a.dbg[2], (unsigned long long)s2);
            atomicAdd(&a.dbg[3], (unsigned long long)s3);
        }
    }
#endif
    if (lane == 0) {
        if (tot.unique) atomicAdd(&a.stats[0], (unsigned long long)tot.unique);
        if (tot.mapped > tot.unique) atomicAdd(&a.stats[1], (unsigned long long)(tot.mapped - tot.unique));
        if (tot.unm) atomicAdd(&a.stats[2], (unsigned long long)tot.unm);
        if (tot.drop) atomicAdd(&a.stats[3], (unsigned long long)tot.drop);
        if (qf_w && has_mkq) atomicAdd(&a.stats[4], (unsigned long long)qf_w);
        if (hr_w && has_mg) atomicAdd(&a.stats[5], (unsigned long long)hr_w);
    }
    if (wc.lds) {
        __syncthreads();
        for (uint32_t g = threadIdx.x; g < G; g += kBlock) {
            if (wc.uniq[g]) atomicAdd(&a.uniq[g], (unsigned long long)wc.uniq[g]);
            if (wc.amb[g]) atomicAdd(&a.amb[g], (unsigned long long)wc.amb[g]);
            if (wc.first[g] != (unsigned long long)PA_NO_FIRST_KEY) atomicMin(&a.first[g], wc.first[g]);
        }
    }
}

template <int WPL>
constexpr size_t fast_wave_bytes(bool need_q) {
    return sizeof(WaveLds<WPL>) + (need_q ? sizeof(WaveQual<WPL>) : 0);
}
