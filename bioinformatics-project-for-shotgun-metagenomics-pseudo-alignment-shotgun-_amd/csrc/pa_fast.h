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

template <int WPL>
struct FastCfg {
    static constexpr int HS = 128 * WPL;               // hash entries per wave (>= 2 x windows)
    static constexpr int E = HS / 64;                  // entries owned per lane
    static constexpr int LCAP = 64 * WPL + 64;         // longest read handled (k <= 63)
    static constexpr int NDW = (LCAP + 8 + 255) / 256; // staged dwords per lane
    static constexpr int PW = LCAP / 32 + 2;           // packed words
    static constexpr int BW = LCAP / 64 + 2;           // non-ACGT bitmap words
};

template <int WPL>
struct __align__(16) WaveLds {
    using C = FastCfg<WPL>;
    uint64_t packed[C::PW];
    uint64_t poison[C::BW];
    uint64_t hA_key[C::HS];   // distinct k-mers: table slot; then multi-set masks / p-check genome ids
    uint32_t stage[C::NDW * 64];
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

struct ReadTotals {      // per-lane window counters + lane-0 read counters of a wave
    uint32_t qf = 0, hr = 0;
    uint32_t unique = 0, amb = 0, unm = 0, drop = 0;
};

__device__ __forceinline__ bool bit(uint32_t m, int i) { return (m >> i) & 1u; }

// ---- dense decision (G <= 64): lane g owns genome g ------------------------
template <int WPL>
__device__ __forceinline__ void decide_dense(const AlignArgs &a, const WgCounters &wc, WaveLds<WPL> &L, uint64_t r,
                                             uint32_t qf, uint32_t hr, ReadTotals &tot) {
    using C = FastCfg<WPL>;
    const int lane = lane_id();
    const uint32_t G = a.G;
    uint32_t nmulti = 0;
#pragma unroll
    for (int e = 0; e < C::E; e++) {
        const int i = lane + 64 * e;
        const uint32_t c = L.hB_key[i];
        const uint32_t is_multi = (c != NONE && c >= G) ? 1u : 0u;
        if (c < G) {  // NONE >= G
            L.gcnt[c] = L.hB_cnt[i];
            L.gmin[c] = L.hB_min[i];
        }
        const uint64_t bm = __ballot(is_multi);
        if (is_multi) {
            const uint32_t at = nmulti + lanes_below(bm);
            L.hA_key[at] = a.class_mask[c - G];
            L.hA_v[at] = L.hB_cnt[i];
            L.hA_v2[at] = L.hB_min[i];
        }
        nmulti += (uint32_t)__popcll(bm);
    }
    wave_sync();
    const uint32_t cnt = L.gcnt[lane], smin = L.gmin[lane];
    const uint64_t specb = __ballot(cnt > 0);
    const uint32_t nspec = (uint32_t)__popcll(specb);
    const uint64_t read_idx = a.base + r;
    tot.qf += qf;
    tot.hr += hr;
    if (nspec == 0) {
        if (lane == 0) tot.amb++;  // AMBIGUOUS with an empty genome list
        return;
    }
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
        if (lane == 0) tot.amb++;
        return;
    }
    if (a.prm.p < 0 || nmulti == 0) {
        if (lane == 0) {
            count_genome(a, wc, gstar, true, 1, first_key(read_idx, 0));
            tot.unique++;
        }
        return;
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
        if (lane == 0) tot.amb++;
    } else if (lane == 0) {
        count_genome(a, wc, gstar, true, 1, first_key(read_idx, 0));
        tot.unique++;
    }
}

// ---- hash decision (G > 64) --------------------------------------------------
template <int WPL>
__device__ __forceinline__ void decide_hash(const AlignArgs &a, const WgCounters &wc, WaveLds<WPL> &L, uint64_t r,
                                            uint32_t qf, uint32_t hr, ReadTotals &tot) {
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
    tot.qf += qf;  // committed from here on unless the read is deferred below
    tot.hr += hr;
    if (nspec == 0) {
        if (lane == 0) tot.amb++;
        return;
    }
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
        if (lane == 0) tot.amb++;
        return;
    }
    if (a.prm.p < 0 || nmulti == 0) {
        if (lane == 0) {
            count_genome(a, wc, gstar, true, 1, first_key(read_idx, 0));
            tot.unique++;
        }
        return;
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
        tot.qf -= qf;
        tot.hr -= hr;
        if (lane == 0) a.queue[atomicAdd(a.qcount, 1ull)] = (uint32_t)r;
        return;
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
        if (lane == 0) tot.amb++;
    } else if (lane == 0) {
        count_genome(a, wc, gstar, true, 1, first_key(read_idx, 0));
        tot.unique++;
    }
}

// ---- one read ------------------------------------------------------------------
template <int NW, int WPL, bool DENSE>
__device__ __forceinline__ void fast_read(const AlignArgs &a, const WgCounters &wc, WaveLds<WPL> &L,
                                          WaveQual<WPL> *Q, bool need_q, uint64_t r, uint32_t shift,
                                          uint32_t len, ReadTotals &tot) {
    using C = FastCfg<WPL>;
    const int lane = lane_id();
    const int k = a.k;
    const uint32_t flags = a.prm.flags;
    const uint8_t *sb = (const uint8_t *)L.stage + shift;
    const uint32_t W = (len >= (uint32_t)k) ? len - k + 1 : 0;

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
            if (lane == 0) tot.drop++;  // dropped, not unmapped (src/kmer.py:587-589)
            return;
        }
    }
    // ---- 2-bit pack + non-ACGT bitmap; clear the hashes
    for (uint32_t c0 = 0; c0 < len; c0 += 64) {
        const uint32_t i = c0 + lane;
        const uint32_t code = i < len ? base_code(sb[i]) : 0u;
        const uint64_t bad = __ballot(code > 3);
        const uint64_t v = half_or64((uint64_t)(code & 3) << (62 - 2 * (lane & 31)));
        if ((lane & 31) == 31) L.packed[c0 / 32 + (lane >> 5)] = v;
        if (lane == 0) L.poison[c0 / 64] = bad;
    }
    if (lane < 2) {
        const uint32_t nc = (len + 63) / 64;
        L.packed[nc * 2 + lane] = 0;
        if (lane == 0) L.poison[nc] = 0;
    }
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
    // ---- windows: quality gate, key, probe (src/kmer.py:419-429)
    const Slot<NW> *table = (const Slot<NW> *)a.table;
    const int64_t mkq_k = (int64_t)a.prm.mkq * k;
    Key<NW> key[WPL];
    uint64_t pos[WPL];
    uint32_t cls[WPL];
    uint32_t pendm = 0, incm = 0;  // bit j: window lane + 64j still probing / included
    uint32_t qf = 0, hr = 0;
#pragma unroll
    for (int j = 0; j < WPL; j++) {
        const uint32_t w = lane + 64 * j;
        uint32_t ok = w < W ? 1u : 0u;
        if (ok && (flags & F_MKQ) && (int64_t)(Q->pref[w + k] - Q->pref[w]) < mkq_k) {
            qf++;
            ok = 0;
        }
        if (ok && window_bits(L.poison, w, k) != 0) ok = 0;
        if (ok) {
            key[j] = extract_key<NW>(L.packed, w, k);
            pos[j] = home_of<NW>(key[j], key_hash(key[j]), a.home);
        }
        pendm |= ok << j;
    }
    while (__ballot(pendm != 0)) {  // all probes of the lane in flight together
        Slot<NW> s[WPL];
#pragma unroll
        for (int j = 0; j < WPL; j++)
            if (bit(pendm, j)) s[j] = table[pos[j]];
#pragma unroll
        for (int j = 0; j < WPL; j++) {
            if (!bit(pendm, j)) continue;
            if (s[j].key[0] == EMPTY) {
                pendm &= ~(1u << j);
                continue;
            }
            bool eq = true;
#pragma unroll
            for (int t = 0; t < NW; t++) eq &= (s[j].key[t] == key[j].w[t]);
            if (eq) {
                pendm &= ~(1u << j);
                cls[j] = s[j].cls;
                if ((flags & F_MG) && (int64_t)s[j].csize > (int64_t)a.prm.mg)
                    hr++;  // highly redundant k-mer (src/kmer.py:425-427)
                else
                    incm |= 1u << j;
            } else {
                pos[j] = (pos[j] + 1 == a.cap) ? 0 : pos[j] + 1;
            }
        }
    }
    if (!__ballot(incm != 0)) {
        tot.qf += qf;
        tot.hr += hr;
        if (lane == 0) tot.unm++;  // no k-mer references -> UNMAPPED (src/kmer.py:516-517)
        return;
    }
    // ---- distinct k-mers: first window per table slot (quirk 3)
    uint32_t hp[WPL];
#pragma unroll
    for (int j = 0; j < WPL; j++)
        if (bit(incm, j)) {
            hp[j] = lds_insert64(L.hA_key, C::HS, pos[j]);
            atomicMin(&L.hA_v[hp[j]], (uint32_t)(lane + 64 * j));
        }
    wave_sync();
    // ---- group the distinct k-mers by genome set
#pragma unroll
    for (int j = 0; j < WPL; j++)
        if (bit(incm, j) && L.hA_v[hp[j]] == (uint32_t)(lane + 64 * j)) {
            const uint32_t p = lds_insert32(L.hB_key, C::HS, cls[j]);
            atomicAdd(&L.hB_cnt[p], 1u);
            atomicMin(&L.hB_min[p], (uint32_t)(lane + 64 * j));
        }
    wave_sync();
    if (DENSE)
        decide_dense<WPL>(a, wc, L, r, qf, hr, tot);
    else
        decide_hash<WPL>(a, wc, L, r, qf, hr, tot);
}

template <int NW, int WPL, bool DENSE>
__global__ __launch_bounds__(kBlock) void k_align_fast(AlignArgs a) {
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

    // contiguous chunk of reads for this wave
    const uint64_t nw = (uint64_t)gridDim.x * kWaves, gw = (uint64_t)blockIdx.x * kWaves + wid;
    const uint64_t rb = a.n * gw / nw, re = a.n * (gw + 1) / nw;
    ReadTotals tot;
    if (rb < re) {
        uint64_t o_cur = a.off[rb], o_nxt = a.off[rb + 1];
        uint32_t sd[C::NDW], qd[C::NDW];
        load_stage<WPL>(a.seq, o_cur, sd);
        if (need_q) load_stage<WPL>(a.qual, o_cur, qd);
        for (uint64_t r = rb; r < re; r++) {
            const uint64_t o_nn = (r + 2 <= a.n) ? a.off[r + 2] : o_nxt;
            uint32_t sn[C::NDW], qn[C::NDW];
            if (r + 1 < re) {  // prefetch the next read while this one is classified
                load_stage<WPL>(a.seq, o_nxt, sn);
                if (need_q) load_stage<WPL>(a.qual, o_nxt, qn);
            }
            const uint32_t len = (uint32_t)(o_nxt - o_cur);
            const uint32_t W = (len >= (uint32_t)a.k) ? len - a.k + 1 : 0;
            if (W > 64u * WPL || len > (uint32_t)(C::LCAP - 8)) {
                if (lane == 0) a.queue[atomicAdd(a.qcount, 1ull)] = (uint32_t)r;
            } else {
                wave_sync();
#pragma unroll
                for (int j = 0; j < C::NDW; j++) {
                    L.stage[lane + 64 * j] = sd[j];
                    if (need_q) Q->stage[lane + 64 * j] = qd[j];
                }
                wave_sync();
                fast_read<NW, WPL, DENSE>(a, wc, L, Q, need_q, r, (uint32_t)(o_cur & 3), len, tot);
            }
            o_cur = o_nxt;
            o_nxt = o_nn;
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
    if (lane == 0) {
        if (tot.unique) atomicAdd(&a.stats[0], (unsigned long long)tot.unique);
        if (tot.amb) atomicAdd(&a.stats[1], (unsigned long long)tot.amb);
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
