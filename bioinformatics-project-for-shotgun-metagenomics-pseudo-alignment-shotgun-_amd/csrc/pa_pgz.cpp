// pa_pgz.cpp -- parallel inflate of ordinary gzip files (one deflate stream per
// member, as `gzip` writes them), for the readers' `.gz` input
// (src/data_file.py:123-125: gzip.open(...).read()).
//
// A deflate stream has no index: block boundaries are known only to a decoder
// that started at the beginning.  The stream is cut into chunks of compressed
// bytes, one per host thread, and (phase A) every chunk but the first finds
// the first position in its range where a dynamic-Huffman block header parses
// and the block decodes to its end-of-block code.  Phase B decodes each chunk
// from there until the block that starts where the next chunk's search landed.
// A back-reference may reach up to 32 KiB before the chunk's start -- bytes
// only the previous chunk knows -- so a chunk decodes into 16-bit symbols over
// a window of 32 768 MARKERS (symbol 256 + j: byte j of the window); once the
// chunks are validated in order (chunk i must stop exactly where chunk i + 1
// started, else the batch ends at chunk i and the next batch starts there, with
// its window known), each chunk's window is the previous chunk's resolved tail
// and its markers are replaced in parallel.  The member's CRC-32 (combined from
// per-chunk CRCs) and size are checked against its trailer.  Anything that is
// not a clean gzip stream -- a decode error, a bad trailer -- gives
// PA_ENOTCANON, so the caller takes the exact path (the reference's error).
//
// Exactness: chunk 0 of every batch starts at a boundary a sequential decode
// reached, with its real window; a later chunk's output is used only if the
// previous chunk's decode ended exactly at its start, i.e. the same decode a
// sequential inflater would make from there; and the CRC-32 of the whole text
// is checked.
#include <sys/mman.h>
#include <zlib.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "pa_gz.h"
#include "pa_internal.h"
#include "pa_pgz.h"

namespace pa {

namespace {

constexpr uint32_t kWin = 32768;  // deflate window

// ---- bits ---------------------------------------------------------------------

struct Bits {
    const uint8_t *p;
    uint64_t n;  // bytes
    // 57+ bits from bit position bp on (zeros past the end)
    inline uint64_t peek(uint64_t bp) const {
        const uint64_t b = bp >> 3;
        uint64_t v;
        if (b + 8 <= n) {
            std::memcpy(&v, p + b, 8);
        } else {
            v = 0;
            for (uint64_t i = 0; b + i < n && i < 8; i++) v |= (uint64_t)p[b + i] << (8 * i);
        }
        return v >> (bp & 7);
    }
};

// ---- canonical Huffman decoding tables ------------------------------------------
// entry: nbits (8) | kind (2) << 8 | subbits (4) << 10 | value << 14
enum : uint32_t { K_SYM = 0, K_SUB = 1, K_BAD = 2 };
inline uint32_t ent(uint32_t nbits, uint32_t kind, uint32_t subbits, uint32_t value) {
    return nbits | (kind << 8) | (subbits << 10) | (value << 14);
}

struct Huff {
    int pb = 0;                  // primary index bits
    std::vector<uint32_t> t;     // primary table then subtables
    // Build from code lengths; false if over-subscribed, or incomplete where
    // deflate does not allow it (allow_single: one code of length 1, the
    // distance code of a block with a single distance)
    bool build(const uint8_t *len, int n, int pbits, bool allow_incomplete_single) {
        pb = pbits;
        uint32_t count[16] = {0};
        for (int i = 0; i < n; i++) count[len[i]]++;
        count[0] = 0;
        int left = 1, maxlen = 0, used = 0;
        for (int l = 1; l <= 15; l++) {
            left <<= 1;
            left -= (int)count[l];
            if (left < 0) return false;  // over-subscribed
            if (count[l]) maxlen = l;
            used += (int)count[l];
        }
        if (left > 0) {  // incomplete
            if (!(allow_incomplete_single && used == 1 && count[1] == 1)) {
                if (used != 0) return false;
            }
        }
        const uint32_t psize = 1u << pb;
        t.assign(psize, ent(0, K_BAD, 0, 0));
        if (used == 0) return true;
        // canonical codes
        uint32_t next[16] = {0};
        uint32_t code = 0;
        for (int l = 1; l <= 15; l++) {
            code = (code + count[l - 1]) << 1;
            next[l] = code;
        }
        const int sb = maxlen > pb ? maxlen - pb : 0;  // subtable bits (one size for all)
        std::vector<int32_t> sub_of(psize, -1);
        for (int s = 0; s < n; s++) {
            const int l = len[s];
            if (!l) continue;
            const uint32_t c = next[l]++;
            uint32_t r = 0;  // bit-reversed code (deflate reads codes MSB first from an LSB-first stream)
            for (int i = 0; i < l; i++) r |= ((c >> i) & 1u) << (l - 1 - i);
            if (l <= pb) {
                for (uint32_t k = r; k < psize; k += 1u << l) t[k] = ent((uint32_t)l, K_SYM, 0, (uint32_t)s);
            } else {
                const uint32_t pre = r & (psize - 1);
                if (sub_of[pre] < 0) {
                    sub_of[pre] = (int32_t)t.size();
                    t.resize(t.size() + (1u << sb), ent(0, K_BAD, 0, 0));
                    t[pre] = ent((uint32_t)pb, K_SUB, (uint32_t)sb, (uint32_t)sub_of[pre]);
                }
                const uint32_t rest = r >> pb, rl = (uint32_t)(l - pb);
                for (uint32_t k = rest; k < (1u << sb); k += 1u << rl)
                    t[(uint32_t)sub_of[pre] + k] = ent(rl, K_SYM, 0, (uint32_t)s);
            }
        }
        return true;
    }
    // symbol at bit window w (LSB first); nbits consumed; -1 if invalid
    inline int decode(uint64_t w, uint32_t &nb) const {
        uint32_t e = t[w & ((1u << pb) - 1)];
        if (((e >> 8) & 3) == K_SUB) {
            const uint32_t sb = (e >> 10) & 15;
            const uint32_t e2 = t[(e >> 14) + ((uint32_t)(w >> pb) & ((1u << sb) - 1))];
            if (((e2 >> 8) & 3) != K_SYM) return -1;
            nb = (uint32_t)pb + (e2 & 255);
            return (int)(e2 >> 14);
        }
        if (((e >> 8) & 3) != K_SYM) return -1;
        nb = e & 255;
        return (int)(e >> 14);
    }
};

const uint16_t kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                               35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
const uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
const uint16_t kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193,
                                257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
const uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
const uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct Tables {
    Huff lit, dist;
};

const Tables &fixed_tables() {
    static Tables *f = [] {
        auto *x = new Tables();
        uint8_t l[288];
        for (int i = 0; i < 144; i++) l[i] = 8;
        for (int i = 144; i < 256; i++) l[i] = 9;
        for (int i = 256; i < 280; i++) l[i] = 7;
        for (int i = 280; i < 288; i++) l[i] = 8;
        x->lit.build(l, 288, 10, false);
        uint8_t d[32];  // (30 and 31 complete the code; the decoder rejects them)
        for (int i = 0; i < 32; i++) d[i] = 5;
        x->dist.build(d, 32, 8, false);
        return x;
    }();
    return *f;
}

// The header of a dynamic block from bit bp on (past BFINAL / BTYPE): its
// tables, bp advanced; false if it is not a valid header.
bool read_dynamic(const Bits &in, uint64_t &bp, Tables &tb) {
    uint64_t w = in.peek(bp);
    const int hlit = (int)(w & 31) + 257, hdist = (int)((w >> 5) & 31) + 1, hclen = (int)((w >> 10) & 15) + 4;
    if (hlit > 286 || hdist > 30) return false;
    bp += 14;
    uint8_t cl[19] = {0};
    w = in.peek(bp);
    for (int i = 0; i < hclen; i++) cl[kClOrder[i]] = (uint8_t)((w >> (3 * i)) & 7);
    bp += 3 * (uint64_t)hclen;
    // the code-length code must be complete
    {
        int left = 1;
        uint32_t cnt[8] = {0};
        for (int i = 0; i < 19; i++) cnt[cl[i]]++;
        for (int l = 1; l <= 7; l++) {
            left = (left << 1) - (int)cnt[l];
            if (left < 0) return false;
        }
        if (left != 0) return false;
    }
    Huff clh;
    if (!clh.build(cl, 19, 7, false)) return false;
    uint8_t lens[286 + 30];
    int i = 0;
    const int total = hlit + hdist;
    while (i < total) {
        w = in.peek(bp);
        uint32_t nb;
        const int s = clh.decode(w, nb);
        if (s < 0) return false;
        bp += nb;
        w >>= nb;
        if (s < 16) {
            lens[i++] = (uint8_t)s;
        } else if (s == 16) {
            if (i == 0) return false;
            const int r = 3 + (int)(w & 3);
            bp += 2;
            if (i + r > total) return false;
            const uint8_t v = lens[i - 1];
            for (int j = 0; j < r; j++) lens[i++] = v;
        } else {
            const int r = s == 17 ? 3 + (int)(w & 7) : 11 + (int)(w & 127);
            bp += s == 17 ? 3 : 7;
            if (i + r > total) return false;
            for (int j = 0; j < r; j++) lens[i++] = 0;
        }
    }
    if (lens[256] == 0) return false;  // no end-of-block code
    if (!tb.lit.build(lens, hlit, 10, true)) return false;
    if (!tb.dist.build(lens + hlit, hdist, 8, true)) return false;
    return true;
}

// Growable buffer of 16-bit symbols (no zero fill on growth: the decoder
// writes every element it keeps).
struct SymBuf {
    uint16_t *p = nullptr;
    size_t n = 0, cap = 0;
    SymBuf() = default;
    SymBuf(const SymBuf &) = delete;
    SymBuf &operator=(const SymBuf &) = delete;
    ~SymBuf() { std::free(p); }
    bool reserve(size_t c) {
        if (c <= cap) return true;
        void *q = std::realloc(p, c * sizeof(uint16_t));
        if (!q) return false;
        p = (uint16_t *)q;
        cap = c;
        return true;
    }
    size_t size() const { return n; }
    uint16_t operator[](size_t i) const { return p[i]; }
};

// One chunk's decoder state: 16-bit symbols (bytes, or 256 + j: byte j of the
// unknown window before the chunk), the first kWin of them that window.
struct Chunk {
    uint64_t start = ~0ull;   // bit position of its first block (~0: none found)
    uint64_t end = 0;         // bit position where it stopped (a block boundary)
    bool ok = false;          // start found / decode clean
    bool final_seen = false;  // the member's last block ended inside it (end = past that block)
    SymBuf out;
};

enum BlockRes { B_OK = 0, B_ERR = 1 };

// Decode one block (header at bp) into out; bp advanced past it.  out_cap
// bounds the symbols (a false block start can decode a long run of garbage).
BlockRes decode_block(const Bits &in, uint64_t &bp, SymBuf &out, bool &final_blk, Tables &tb, uint64_t out_cap) {
    uint64_t w = in.peek(bp);
    final_blk = (w & 1) != 0;
    const uint32_t type = (uint32_t)((w >> 1) & 3);
    bp += 3;
    if (type == 0) {  // stored
        bp = (bp + 7) & ~7ull;
        if ((bp >> 3) + 4 > in.n) return B_ERR;
        const uint8_t *q = in.p + (bp >> 3);
        const uint32_t len = (uint32_t)q[0] | ((uint32_t)q[1] << 8), nlen = (uint32_t)q[2] | ((uint32_t)q[3] << 8);
        if ((len ^ 0xFFFFu) != nlen) return B_ERR;
        if ((bp >> 3) + 4 + len > in.n) return B_ERR;
        if (!out.reserve(out.n + len + 1024)) return B_ERR;
        for (uint32_t i = 0; i < len; i++) out.p[out.n + i] = q[4 + i];
        out.n += len;
        bp += 8ull * (4 + len);
        return B_OK;
    }
    if (type == 3) return B_ERR;
    const Tables *T = &fixed_tables();
    if (type == 2) {
        if (!read_dynamic(in, bp, tb)) return B_ERR;
        T = &tb;
    }
    const Huff &L = T->lit, &D = T->dist;
    size_t o = out.n;
    if (!out.reserve(std::max<size_t>(out.cap, o + 65536))) return B_ERR;
    uint16_t *op = out.p;
    size_t cap = out.cap;
    const uint64_t limit_bits = 8 * in.n + 64;
    BlockRes res = B_OK;
    for (;;) {
        if (o + 516 > cap) {
            if (cap > out_cap || !out.reserve(2 * cap)) {
                res = B_ERR;
                break;
            }
            op = out.p;
            cap = out.cap;
        }
        if (bp > limit_bits) {
            res = B_ERR;
            break;
        }
        w = in.peek(bp);
        uint32_t nb;
        const int s = L.decode(w, nb);
        if (s < 0) {
            res = B_ERR;
            break;
        }
        if (s < 256) {
            op[o++] = (uint16_t)s;
            bp += nb;
            // a second literal from the same bits when it is one
            w >>= nb;
            uint32_t nb2;
            const int s2 = L.decode(w, nb2);
            if (s2 >= 0 && s2 < 256) {
                op[o++] = (uint16_t)s2;
                bp += nb2;
            }
            continue;
        }
        if (s == 256) {
            bp += nb;
            break;
        }
        if (s > 285) {
            res = B_ERR;
            break;
        }
        w >>= nb;
        uint32_t used = nb;
        const int li = s - 257;
        const uint32_t le = kLenExtra[li];
        const uint32_t len = kLenBase[li] + (uint32_t)(w & ((1u << le) - 1));
        w >>= le;
        used += le;
        uint32_t nd;
        const int ds = D.decode(w, nd);
        if (ds < 0 || ds > 29) {
            res = B_ERR;
            break;
        }
        w >>= nd;
        used += nd;
        const uint32_t de = kDistExtra[ds];
        const uint32_t dist = kDistBase[ds] + (uint32_t)(w & ((1u << de) - 1));
        used += de;
        bp += used;
        if (dist > o) {
            res = B_ERR;
            break;
        }
        const uint16_t *src = op + o - dist;
        uint16_t *dst = op + o;
        if (dist >= len) {
            std::memcpy(dst, src, (size_t)len * 2);
        } else {
            for (uint32_t i = 0; i < len; i++) dst[i] = src[i];
        }
        o += len;
    }
    out.n = o;
    return res;
}

// Phase A: the first bit position in [b0, b1) where a dynamic block header
// parses and the block decodes cleanly to its end, or ~0.
uint64_t find_block(const Bits &in, uint64_t b0, uint64_t b1) {
    Tables tb;
    SymBuf scratch;
    for (uint64_t b = b0; b < b1; b++) {
        const uint64_t w = in.peek(b);
        if (((w >> 1) & 3) != 2) continue;                             // BTYPE = dynamic
        if (((w >> 3) & 31) > 29 || ((w >> 8) & 31) > 29) continue;  // HLIT <= 286, HDIST <= 30
        // the code-length code's lengths must form a complete code
        {
            const int hclen = (int)((w >> 13) & 15) + 4;
            const uint64_t v = in.peek(b + 17);
            uint32_t cnt[8] = {0};
            for (int i = 0; i < hclen; i++) cnt[(v >> (3 * i)) & 7]++;
            int left = 1;
            bool bad = false;
            for (int l = 1; l <= 7 && !bad; l++) {
                left = (left << 1) - (int)cnt[l];
                bad = left < 0;
            }
            if (bad || left != 0) continue;
        }
        uint64_t bp = b;
        bool fin = false;
        if (!scratch.reserve(kWin + 65536)) return ~0ull;
        scratch.n = kWin;  // (markers: any back-reference is in range; their values do not matter here)
        if (decode_block(in, bp, scratch, fin, tb, 16ull << 20) == B_OK) return b;
    }
    return ~0ull;
}

}  // namespace

// ---- the stream ------------------------------------------------------------------

struct Pgz {
    Bits in{};
    const uint8_t *map = nullptr;
    uint64_t map_len = 0;
    int threads = 1;
    uint64_t chunk_bytes = 4ull << 20;
    // the current member
    uint64_t bp = 0;              // next block (a boundary a sequential decode reached)
    uint8_t window[kWin];         // the last kWin bytes of text before bp
    uint32_t window_len = 0;      // how many of them exist (member start: 0)
    uint32_t crc = 0;             // CRC-32 of the member's text so far
    uint64_t isize = 0;           // its length
    bool in_member = false;
    bool eof = false;
    // text decoded, not yet handed out
    std::vector<uint8_t> pend;
    uint64_t pend_pos = 0;
    std::string err;
};

namespace {

// Parse a gzip member header at byte o; the deflate start byte, or false.
bool member_header(const Pgz &g, uint64_t o, uint64_t &data) {
    const uint8_t *m = g.map;
    const uint64_t n = g.map_len;
    if (n - o < 18 || m[o] != 0x1f || m[o + 1] != 0x8b || m[o + 2] != 8) return false;
    const uint32_t flg = m[o + 3];
    if (flg & 0xE0) return false;
    uint64_t p = o + 10;
    if (flg & 4) {  // FEXTRA
        if (p + 2 > n) return false;
        p += 2 + ((uint32_t)m[p] | ((uint32_t)m[p + 1] << 8));
    }
    if (flg & 8) {  // FNAME
        while (p < n && m[p]) p++;
        p++;
    }
    if (flg & 16) {  // FCOMMENT
        while (p < n && m[p]) p++;
        p++;
    }
    if (flg & 2) p += 2;  // FHCRC
    if (p >= n) return false;
    data = p;
    return true;
}

// Markers of `c` replaced from `win` (the kWin bytes before the chunk, wl of them real).
bool resolve(const Chunk &c, const uint8_t *win, uint32_t wl, uint8_t *dst) {
    const uint16_t *s = c.out.p + kWin;
    const size_t n = c.out.size() - kWin;
    uint32_t badm = 0;
    for (size_t i = 0; i < n; i++) {
        const uint16_t v = s[i];
        if (v < 256) {
            dst[i] = (uint8_t)v;
        } else {
            const uint32_t j = v - 256u;
            badm |= (uint32_t)(j < kWin - wl);  // a byte before the member's text
            dst[i] = win[j];
        }
    }
    return badm == 0;
}

// Decode from the stream position on: one batch of chunks; appends text to g.pend.
pa_status next_batch(Pgz &g) {
    const uint64_t byte0 = g.bp >> 3;
    const uint64_t avail = g.map_len > byte0 ? g.map_len - byte0 : 0;
    int T = std::max(1, g.threads);
    const uint64_t span = std::min<uint64_t>(avail, (uint64_t)T * g.chunk_bytes);
    T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)T, span / (g.chunk_bytes / 2) + 1));
    std::vector<Chunk> ch(T);
    ch[0].start = g.bp;
    ch[0].ok = true;
    std::vector<uint64_t> lo(T + 1);
    for (int i = 0; i <= T; i++) lo[i] = 8 * (byte0 + span * (uint64_t)i / (uint64_t)T);
    // phase A: block starts of chunks 1 .. T-1
    {
        std::vector<std::thread> th;
        for (int i = 1; i < T; i++)
            th.emplace_back([&, i] {
                const uint64_t s = find_block(g.in, lo[i], lo[i + 1]);
                ch[i].start = s;
                ch[i].ok = s != ~0ull;
            });
        for (auto &x : th) x.join();
    }
    // each found chunk decodes up to the next found start (a chunk with none is absorbed)
    std::vector<uint64_t> stop(T, ~0ull);
    for (int i = 0; i < T; i++)
        for (int j = i + 1; j < T; j++)
            if (ch[j].ok) {
                stop[i] = ch[j].start;
                break;
            }
    // the last chunk (or one with no later start) stops at the first boundary past the batch
    const uint64_t batch_end = lo[T];
    // phase B
    auto decode_chunk = [&](int i) {
        Chunk &c = ch[i];
        if (!c.ok) return;
        if (!c.out.reserve(kWin + (1u << 20))) {
            c.ok = false;
            return;
        }
        c.out.n = kWin;
        if (i == 0) {  // the real window
            for (uint32_t j = 0; j < kWin; j++) c.out.p[j] = j < kWin - g.window_len ? (uint16_t)(256 + j) : g.window[j];
        } else {
            for (uint32_t j = 0; j < kWin; j++) c.out.p[j] = (uint16_t)(256 + j);
        }
        uint64_t bp = c.start;
        Tables tb;
        const uint64_t lim = stop[i] != ~0ull ? stop[i] : batch_end;
        // Symbols a chunk may decode before it is given up.  Chunk 0 starts at a
        // boundary a sequential decode reached: its text is real, and only
        // input above 64:1 fails it (the caller then inflates with zlib).  The
        // others start where phase A found a header, possibly a false start:
        // they are held to 16x their compressed bits (FASTQ deflates ~4:1),
        // 16-64 M symbols -- one that stops there leaves its range to chunk 0
        // of the next batch, so the cap bounds the batch's host memory (T x
        // 2 x 128 MB at most) without failing any input.
        const uint64_t cbytes = (lim - c.start) / 8;
        const uint64_t cap = i == 0 ? std::max<uint64_t>(256ull << 20, 64 * cbytes + (1u << 20))
                                    : std::min<uint64_t>(64ull << 20, std::max<uint64_t>(16ull << 20, 16 * cbytes + (1u << 20)));
        while (bp < lim) {
            bool fin = false;
            if (decode_block(g.in, bp, c.out, fin, tb, cap) != B_OK) {
                c.ok = false;
                break;
            }
            if (fin) {
                c.final_seen = true;
                break;
            }
        }
        c.end = bp;
    };
    {
        std::vector<std::thread> th;
        for (int i = 1; i < T; i++) th.emplace_back(decode_chunk, i);
        decode_chunk(0);
        for (auto &x : th) x.join();
    }
    if (!ch[0].ok) {
        g.err = "deflate data error";
        return PA_ENOTCANON;
    }
    // validation in order: a chunk is used when the previous used one stopped
    // exactly where its decode began (a chunk whose search found nothing was
    // decoded by its predecessor)
    std::vector<int> idx{0};
    for (int a = 0, b = 1; b < T; b++) {
        if (ch[a].final_seen) break;
        if (ch[b].start == ~0ull) continue;
        if (!ch[b].ok || ch[a].end != ch[b].start) break;
        idx.push_back(b);
        a = b;
    }
    // resolve in order: each chunk's window is the previous text's last kWin bytes
    uint8_t win[kWin];
    uint32_t wl = g.window_len;
    std::memcpy(win, g.window, kWin);
    std::vector<uint64_t> dst_off(idx.size() + 1, 0);
    for (size_t u = 0; u < idx.size(); u++) dst_off[u + 1] = dst_off[u] + (ch[idx[u]].out.size() - kWin);
    const uint64_t base = g.pend.size();
    g.pend.resize(base + dst_off.back());
    std::vector<std::vector<uint8_t>> wins(idx.size(), std::vector<uint8_t>(kWin));
    std::vector<uint32_t> wls(idx.size());
    for (size_t u = 0; u < idx.size(); u++) {
        std::memcpy(wins[u].data(), win, kWin);
        wls[u] = wl;
        // the new window: the last kWin bytes after this chunk (its tail resolved now)
        const Chunk &c = ch[idx[u]];
        const size_t n = c.out.size() - kWin;
        uint8_t nw[kWin];
        const size_t keep = n >= kWin ? 0 : kWin - n;  // bytes of the old window that stay
        if (keep) std::memcpy(nw, win + (kWin - keep), keep);
        for (size_t j = keep; j < kWin; j++) {
            const uint16_t v = c.out[kWin + n - (kWin - j)];
            nw[j] = v < 256 ? (uint8_t)v : win[v - 256u];
        }
        std::memcpy(win, nw, kWin);
        wl = (uint32_t)std::min<uint64_t>(kWin, (uint64_t)wl + n);
    }
    std::vector<int> okr(idx.size(), 1);
    std::vector<uint32_t> crcs(idx.size(), 0);
    {
        std::vector<std::thread> th;
        auto work = [&](size_t u) {
            uint8_t *d = g.pend.data() + base + dst_off[u];
            okr[u] = resolve(ch[idx[u]], wins[u].data(), wls[u], d);
            const uint64_t n = dst_off[u + 1] - dst_off[u];
            uLong c = crc32(0L, Z_NULL, 0);
            for (uint64_t o = 0; o < n; o += 1u << 30) c = crc32(c, d + o, (uInt)std::min<uint64_t>(n - o, 1u << 30));
            crcs[u] = (uint32_t)c;
        };
        for (size_t u = 1; u < idx.size(); u++) th.emplace_back(work, u);
        if (!idx.empty()) work(0);
        for (auto &x : th) x.join();
    }
    for (size_t u = 0; u < idx.size(); u++) {
        if (!okr[u]) {
            g.err = "deflate back-reference before the member's start";
            return PA_ENOTCANON;
        }
        const uint64_t n = dst_off[u + 1] - dst_off[u];
        g.crc = (uint32_t)crc32_combine(g.crc, crcs[u], (z_off_t)n);
        g.isize += n;
    }
    std::memcpy(g.window, win, kWin);
    g.window_len = wl;
    const Chunk &last = ch[idx.back()];
    g.bp = last.end;
    if (last.final_seen) {  // the member's trailer: CRC-32 and size
        const uint64_t t = (g.bp + 7) >> 3;
        if (t + 8 > g.map_len) {
            g.err = "truncated gzip member";
            return PA_ENOTCANON;
        }
        const uint8_t *q = g.map + t;
        const uint32_t crc = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
        const uint32_t isz = (uint32_t)q[4] | ((uint32_t)q[5] << 8) | ((uint32_t)q[6] << 16) | ((uint32_t)q[7] << 24);
        if (crc != g.crc || isz != (uint32_t)g.isize) {
            g.err = "gzip member CRC-32 or size mismatch";
            return PA_ENOTCANON;
        }
        g.in_member = false;
        uint64_t o = t + 8;
        if (o >= g.map_len) {
            g.eof = true;
        } else {  // another member (gzip.open reads them all)
            uint64_t data = 0;
            if (!member_header(g, o, data)) {
                g.err = "trailing bytes after the last gzip member";
                return PA_ENOTCANON;
            }
            g.bp = 8 * data;
            g.window_len = 0;
            g.crc = 0;
            g.isize = 0;
            g.in_member = true;
        }
    } else if (g.bp >= 8 * g.map_len) {
        g.err = "truncated deflate stream";
        return PA_ENOTCANON;
    }
    return PA_OK;
}

}  // namespace

pa_status pgz_open(const uint8_t *map, uint64_t len, int threads, Pgz **out) {
    *out = nullptr;
    auto *g = new Pgz();
    g->map = map;
    g->map_len = len;
    g->in.p = map;
    g->in.n = len;
    g->threads = std::max(1, threads);
    if (const char *e = std::getenv("PA_PGZ_CHUNK_KB")) g->chunk_bytes = std::max<uint64_t>(64, std::strtoull(e, nullptr, 10)) << 10;
    uint64_t data = 0;
    if (!member_header(*g, 0, data)) {
        delete g;
        set_error("not a gzip member header");
        return PA_ENOTCANON;
    }
    g->bp = 8 * data;
    g->in_member = true;
    *out = g;
    return PA_OK;
}

pa_status pgz_read(Pgz *g, uint8_t *dst, uint64_t n, uint64_t *got, bool *eof) {
    *got = 0;
    while (*got < n) {
        if (g->pend_pos < g->pend.size()) {
            const uint64_t k = std::min<uint64_t>(n - *got, g->pend.size() - g->pend_pos);
            std::memcpy(dst + *got, g->pend.data() + g->pend_pos, k);
            g->pend_pos += k;
            *got += k;
            continue;
        }
        g->pend.clear();
        g->pend_pos = 0;
        if (g->eof) break;
        const pa_status s = next_batch(*g);
        if (s != PA_OK) {
            set_error("gzip: " + g->err);
            return s;
        }
    }
    *eof = g->eof && g->pend_pos >= g->pend.size();
    return PA_OK;
}

void pgz_close(Pgz *g) { delete g; }

}  // namespace pa

// pa_gz_inflate_file (include/pa.h): inflate a whole gzip file with `threads`
// threads into dst (cap bytes); the text length in *n.  A text of exactly cap
// bytes fits: at tot == cap one more read into a scratch byte tells the end
// from more text (the zlib path sets its end flag only after a read of 0 bytes).
extern "C" pa_status pa_gz_inflate_file(const char *path, int threads, uint8_t *dst, uint64_t cap, uint64_t *n) {
    pa::Gz *g = nullptr;
    const pa_status s = pa::gz_open(path, threads, &g);
    if (s != PA_OK) return s;
    uint64_t tot = 0;
    bool eof = false;
    while (!eof) {
        uint64_t got = 0;
        if (tot >= cap) {
            uint8_t probe = 0;
            // (BGZF refuses a 1-byte window while a member is left: PA_EINVAL, more text)
            const pa_status r = pa::gz_read(g, &probe, 1, &got, &eof);
            if (r != PA_OK && r != PA_EINVAL) {
                pa::gz_close(g);
                return r;
            }
            if (r == PA_OK && got == 0 && eof) break;
            pa::gz_close(g);
            pa::set_error("pa_gz_inflate_file: buffer too small");
            return PA_EINVAL;
        }
        const pa_status r = pa::gz_read(g, dst + tot, cap - tot, &got, &eof);
        if (r != PA_OK) {
            pa::gz_close(g);
            return r;
        }
        tot += got;
    }
    pa::gz_close(g);
    *n = tot;
    return PA_OK;
}
