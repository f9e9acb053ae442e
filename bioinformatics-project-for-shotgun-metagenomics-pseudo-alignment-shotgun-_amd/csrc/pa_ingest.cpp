// pa_ingest.cpp -- multi-threaded FASTA / FASTQ ingest for the reference grammar.
//
// The reference parses whole files with two regular expressions
// (src/records.py:141-199 scan + :212-233 FASTA + :245-302 FASTQ, loaded by
// src/data_file.py:117-158 as UTF-8 text with universal newlines).  This file
// parses the CANONICAL subset of that grammar -- the form every well-formed
// file has -- at memory speed on host threads, straight into the column
// buffers the align path uploads (sequence / quality bytes + uint64 offsets):
//
//   FASTA  optional leading whitespace; records ">" header-line "\n" genome
//          section, a record starting at every ">" that begins a line; header
//          bytes 0x21-0x7E, space, tab (at least one); the genome section is
//          everything up to the next record (at least one byte before the line
//          break that precedes it) of A C G T N and whitespace, whitespace
//          removed; the description is the header stripped.
//   FASTQ  optional leading line breaks, then exactly four lines per record:
//          "@" header (as above), A C G T sequence, "+", qualities 0x21-0x7E of
//          the sequence's length; one optional final line break; ids unique.
//   Both   CRLF line ends are accepted; files are read the reference's way,
//          with universal newlines (a CRLF is one line break, a final lone CR
//          ends the text), text handed over in memory is taken as is (the
//          regexes' own \r?\n); any other CR, any byte >= 0x80, or anything
//          else outside the subset returns PA_ENOTCANON.
//
// On PA_ENOTCANON the Python layer parses the same text with the exact
// regex grammar (records.py), which then reports the reference's own error
// (DuplicateRecordError, UnparsedDataError, InvalidRecordData, ...) or
// accepts the text the way the reference does.  Inside the subset both
// parsers yield identical records; tests/test_host.py checks that on the
// reference's parser fixtures and on generated files.
//
// Threads: FASTQ -- line counts per chunk, a prefix over chunks gives each
// chunk the role (line index mod 4) of its first line, then every chunk parses
// the records whose header line it holds; duplicate ids are found by hashing
// (each thread owns one hash partition).  FASTA -- record starts found per
// chunk, genome sections split into pieces that are validated and compacted in
// parallel.  Export copies the pieces into caller buffers in parallel.

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "pa_gz.h"
#include "pa_internal.h"

namespace {

using std::vector;

// byte classes
enum : uint8_t { C_HDR = 1, C_ACGT = 2, C_N = 4, C_WS = 8, C_QUAL = 16 };

struct Classes {
    uint8_t t[256];
    Classes() {
        memset(t, 0, sizeof(t));
        for (int c = 0x21; c <= 0x7E; c++) t[c] |= C_HDR | C_QUAL;
        t[(int)' '] |= C_HDR | C_WS;
        t[(int)'\t'] |= C_HDR | C_WS;
        for (int c : {'\n', '\v', '\f', '\r'}) t[c] |= C_WS;
        for (int c : {'A', 'C', 'G', 'T'}) t[c] |= C_ACGT;
        t[(int)'N'] |= C_N;
    }
};
const Classes kCls;

inline bool is_strip_ws(uint8_t c) { return c == ' ' || c == '\t'; }

uint64_t hash_bytes(const uint8_t *p, size_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)n;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        h = (h ^ w) * 0xFF51AFD7ED558CCDull;
        h ^= h >> 32;
    }
    uint64_t w = 0;
    memcpy(&w, p + i, n - i);
    h = (h ^ w) * 0xC4CEB9FE1A85EC53ull;
    h ^= h >> 29;
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 32;
    return h;
}

template <class F>
void parallel_for(int nt, F &&f) {
    if (nt <= 1) {
        f(0);
        return;
    }
    vector<std::thread> th;
    th.reserve(nt);
    for (int t = 0; t < nt; t++) th.emplace_back([&, t] { f(t); });
    for (auto &x : th) x.join();
}

// One piece of parsed output (a chunk's records, or a piece of a genome).
struct Piece {
    vector<uint8_t> seq, qual;
    vector<uint64_t> lens;   // FASTQ: per record
    std::string names;       // FASTQ: ids joined by '\n'
    vector<uint64_t> name_end;
    vector<uint64_t> hashes; // FASTQ: id hashes
    bool ok = true;
};

}  // namespace

struct pa_seqset {
    int kind = 0;  // 0 FASTA, 1 FASTQ
    uint64_t n_records = 0, n_bases = 0;
    vector<Piece> pieces;
    // FASTA: record r's genome is pieces [rec_piece[r], rec_piece[r + 1])
    vector<uint64_t> rec_piece;
    std::string names;  // all names, '\n'-joined (FASTA), built at parse
    int threads = 1;
};

namespace {

// Trailing CR of a line [b, e) (CRLF) -> e - 1; a CR elsewhere in the line is
// left for the byte-class checks (no class but C_WS holds it).
// (only for a line that ends at a LF: a CR at the end of the text is no line end)
inline const uint8_t *line_end_nocr(const uint8_t *b, const uint8_t *e, const uint8_t *text_end) {
    return (e < text_end && e > b && e[-1] == '\r') ? e - 1 : e;
}

bool valid_header(const uint8_t *b, const uint8_t *e) {  // "@"/">" excluded
    if (e <= b) return false;
    for (const uint8_t *p = b; p < e; p++)
        if (!(kCls.t[*p] & C_HDR)) return false;
    return true;
}

void strip_into(const uint8_t *b, const uint8_t *e, std::string &out) {
    while (b < e && is_strip_ws(*b)) b++;
    while (e > b && is_strip_ws(e[-1])) e--;
    out.append((const char *)b, (size_t)(e - b));
}

// ---------------------------------------------------------------- FASTQ

pa_status parse_fastq(const uint8_t *T, uint64_t L, int nt, bool universal, pa_seqset *S) {
    uint64_t pos = 0;
    while (pos < L && (T[pos] == '\n' || (T[pos] == '\r' && pos + 1 < L && T[pos + 1] == '\n'))) pos++;
    if (pos >= L || T[pos] != '@') return PA_ENOTCANON;
    // one optional final line break (with universal newlines a final lone CR is one too)
    uint64_t end = L;
    if (end > pos && T[end - 1] == '\n') {
        end--;
        if (end > pos && T[end - 1] == '\r') end--;
    } else if (universal && end > pos && T[end - 1] == '\r') {
        end--;
    }
    const uint8_t *B = T + pos;
    const uint64_t BL = end - pos;
    // chunks starting at line starts
    nt = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)nt, BL / (1 << 16) + 1));
    vector<uint64_t> cs(nt + 1);
    cs[0] = 0;
    cs[nt] = BL;
    for (int t = 1; t < nt; t++) {
        uint64_t c = BL * t / nt;
        const void *nl = memchr(B + c, '\n', BL - c);
        cs[t] = nl ? (uint64_t)((const uint8_t *)nl - B) + 1 : BL;
        if (cs[t] < cs[t - 1]) cs[t] = cs[t - 1];
    }
    vector<uint64_t> nls(nt, 0);
    parallel_for(nt, [&](int t) {
        uint64_t n = 0;
        const uint8_t *p = B + cs[t], *e = B + cs[t + 1];
        while (p < e) {
            const void *q = memchr(p, '\n', (size_t)(e - p));
            if (!q) break;
            n++;
            p = (const uint8_t *)q + 1;
        }
        nls[t] = n;
    });
    vector<uint64_t> first_line(nt + 1, 0);
    for (int t = 0; t < nt; t++) first_line[t + 1] = first_line[t] + nls[t];
    const uint64_t lines = first_line[nt] + 1;
    if (lines % 4) return PA_ENOTCANON;
    S->pieces.assign(nt, Piece());
    parallel_for(nt, [&](int t) {
        Piece &P = S->pieces[t];
        const uint8_t *p = B + cs[t], *e_all = B + BL;
        const uint8_t *chunk_end = B + cs[t + 1];
        uint64_t li = first_line[t];
        if (cs[t] == cs[t + 1]) return;
        auto next_line = [&](const uint8_t *&q, const uint8_t *&le) -> bool {  // [q, le) = line; q -> next
            if (q > e_all) return false;
            const void *nl = memchr(q, '\n', (size_t)(e_all - q));
            le = nl ? (const uint8_t *)nl : e_all;
            return true;
        };
        // skip to the first header line of this chunk
        while (li % 4 && p < chunk_end) {
            const uint8_t *le;
            next_line(p, le);
            p = le + 1;
            li++;
        }
        const uint64_t approx = (uint64_t)(chunk_end - p) / 2 + 64;  // sequence ~ quality ~ 1/2 of the text
        P.seq.reserve(approx);
        P.qual.reserve(approx);
        while (p < chunk_end) {
            const uint8_t *l0b = p, *l0e, *l1b, *l1e, *l2b, *l2e, *l3b, *l3e;
            next_line(l0b, l0e);
            l1b = l0e + 1;
            if (l1b > e_all || !next_line(l1b, l1e)) { P.ok = false; return; }
            l2b = l1e + 1;
            if (l2b > e_all || !next_line(l2b, l2e)) { P.ok = false; return; }
            l3b = l2e + 1;
            if (l3b > e_all || !next_line(l3b, l3e)) { P.ok = false; return; }
            p = l3e + 1;
            l0e = line_end_nocr(l0b, l0e, e_all);
            l1e = line_end_nocr(l1b, l1e, e_all);
            l2e = line_end_nocr(l2b, l2e, e_all);
            l3e = line_end_nocr(l3b, l3e, e_all);
            // @header
            if (l0e - l0b < 2 || *l0b != '@' || !valid_header(l0b + 1, l0e)) { P.ok = false; return; }
            // sequence
            const uint64_t n = (uint64_t)(l1e - l1b);
            if (n == 0 || (uint64_t)(l3e - l3b) != n) { P.ok = false; return; }
            uint8_t acc = C_ACGT, accq = C_QUAL;
            for (const uint8_t *q = l1b; q < l1e; q++) acc &= kCls.t[*q];
            for (const uint8_t *q = l3b; q < l3e; q++) accq &= kCls.t[*q];
            if (!(acc & C_ACGT) || !(accq & C_QUAL)) { P.ok = false; return; }
            // "+" (the dots variant keeps a space section: left to the exact parser)
            if (l2e - l2b != 1 || *l2b != '+') { P.ok = false; return; }
            P.seq.insert(P.seq.end(), l1b, l1e);
            P.qual.insert(P.qual.end(), l3b, l3e);
            P.lens.push_back(n);
            const size_t nb = P.names.size();
            strip_into(l0b + 1, l0e, P.names);
            P.hashes.push_back(hash_bytes((const uint8_t *)P.names.data() + nb, P.names.size() - nb));
            P.names.push_back('\n');
            P.name_end.push_back(P.names.size() - 1);
        }
    });
    for (auto &P : S->pieces)
        if (!P.ok) return PA_ENOTCANON;
    uint64_t n = 0, nb = 0;
    for (auto &P : S->pieces) {
        n += P.lens.size();
        nb += P.seq.size();
    }
    if (n == 0) return PA_ENOTCANON;
    // duplicate ids: every thread owns the hashes with (h % nt2 == t)
    vector<std::pair<uint32_t, uint32_t>> where;  // (piece, record in piece) by global record index
    where.reserve(n);
    vector<uint64_t> hashes;
    hashes.reserve(n);
    for (uint32_t pi = 0; pi < S->pieces.size(); pi++)
        for (uint32_t r = 0; r < S->pieces[pi].hashes.size(); r++) {
            where.emplace_back(pi, r);
            hashes.push_back(S->pieces[pi].hashes[r]);
        }
    auto name_of = [&](uint64_t i, const char *&b, size_t &len) {
        const Piece &P = S->pieces[where[i].first];
        const uint32_t r = where[i].second;
        const uint64_t s = r ? P.name_end[r - 1] + 1 : 0;
        b = P.names.data() + s;
        len = P.name_end[r] - s;
    };
    const int nt2 = std::max(1, nt);
    std::atomic<bool> dup{false};
    parallel_for(nt2, [&](int t) {
        uint64_t cnt = 0;
        for (uint64_t i = 0; i < n; i++) cnt += (hashes[i] % nt2) == (uint64_t)t;
        uint64_t cap = 16;
        while (cap < 2 * cnt) cap <<= 1;
        vector<uint64_t> tab(cap, ~0ull);  // global record index
        for (uint64_t i = 0; i < n && !dup.load(std::memory_order_relaxed); i++) {
            const uint64_t h = hashes[i];
            if (h % nt2 != (uint64_t)t) continue;
            uint64_t j = (h >> 7) & (cap - 1);
            for (;;) {
                const uint64_t o = tab[j];
                if (o == ~0ull) {
                    tab[j] = i;
                    break;
                }
                if (hashes[o] == h) {
                    const char *a, *b;
                    size_t la, lb;
                    name_of(i, a, la);
                    name_of(o, b, lb);
                    if (la == lb && memcmp(a, b, la) == 0) {
                        dup = true;
                        break;
                    }
                }
                j = (j + 1) & (cap - 1);
            }
        }
    });
    if (dup) return PA_ENOTCANON;  // the exact parser raises DuplicateRecordError in the reference's order
    S->n_records = n;
    S->n_bases = nb;
    for (auto &P : S->pieces) {
        vector<uint64_t>().swap(P.hashes);
    }
    return PA_OK;
}

// ---------------------------------------------------------------- FASTA

pa_status parse_fasta(const uint8_t *T, uint64_t L, int nt, bool universal, pa_seqset *S) {
    // leading whitespace, then '>' at a line start
    uint64_t pos = 0;
    while (pos < L && (kCls.t[T[pos]] & C_WS)) pos++;
    if (pos >= L || T[pos] != '>' || (pos > 0 && T[pos - 1] != '\n')) return PA_ENOTCANON;
    // record starts: '>' at line starts (found per chunk)
    nt = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)nt, (L - pos) / (1 << 20) + 1));
    vector<vector<uint64_t>> starts(nt);
    parallel_for(nt, [&](int t) {
        const uint64_t b = pos + (L - pos) * t / nt, e = pos + (L - pos) * (t + 1) / nt;
        const uint8_t *p = T + b;
        while (p < T + e) {
            const void *q = memchr(p, '>', (size_t)(T + e - p));
            if (!q) break;
            const uint64_t i = (uint64_t)((const uint8_t *)q - T);
            if (i == pos || (i > 0 && T[i - 1] == '\n')) starts[t].push_back(i);
            // a '>' elsewhere is caught by the section / header checks
            p = (const uint8_t *)q + 1;
        }
    });
    vector<uint64_t> rs;
    for (auto &v : starts) rs.insert(rs.end(), v.begin(), v.end());
    const uint64_t R = rs.size();
    rs.push_back(L);
    // headers and genome sections
    vector<uint64_t> gs(R), ge(R);
    std::string names;
    for (uint64_t r = 0; r < R; r++) {
        const uint8_t *hb = T + rs[r] + 1, *rend = T + rs[r + 1];
        const void *nl = memchr(hb, '\n', (size_t)(rend - hb));
        if (!nl) return PA_ENOTCANON;  // header without a line break (or at EOF)
        const uint8_t *he = line_end_nocr(hb, (const uint8_t *)nl, T + L);
        if (!valid_header(hb, he)) return PA_ENOTCANON;
        strip_into(hb, he, names);
        names.push_back('\n');
        gs[r] = (uint64_t)((const uint8_t *)nl - T) + 1;
        ge[r] = rs[r + 1];
        // at least one character before the line break that precedes the next
        // record, as the reference sees the text: with universal newlines (a
        // file) a CRLF is one line break; in raw text the CR is a genome char
        uint64_t body_end = ge[r];
        if (r + 1 < R) {
            body_end--;
            if (universal && body_end > gs[r] && T[body_end - 1] == '\r') body_end--;
        }
        if (body_end <= gs[r]) return PA_ENOTCANON;
    }
    // genome pieces: sections split at ~8 MiB
    constexpr uint64_t kPiece = 8ull << 20;
    vector<uint64_t> pb, pe;
    S->rec_piece.assign(R + 1, 0);
    for (uint64_t r = 0; r < R; r++) {
        S->rec_piece[r] = pb.size();
        for (uint64_t b = gs[r]; b < ge[r]; b += kPiece) {
            pb.push_back(b);
            pe.push_back(std::min(ge[r], b + kPiece));
        }
    }
    S->rec_piece[R] = pb.size();
    const uint64_t np = pb.size();
    S->pieces.assign(np, Piece());
    std::atomic<uint64_t> next{0};
    parallel_for(std::max(1, std::min<int>(S->threads, (int)np)), [&](int) {
        for (;;) {
            const uint64_t i = next.fetch_add(1);
            if (i >= np) break;
            Piece &P = S->pieces[i];
            const uint8_t *p = T + pb[i], *e = T + pe[i];
            P.seq.resize((size_t)(e - p));
            uint8_t *o = P.seq.data();
            uint8_t bad = 0;
            for (; p < e; p++) {
                const uint8_t c = kCls.t[*p];
                bad |= (c & (C_ACGT | C_N | C_WS)) ? 0 : 1;
                // a CR not followed by LF would be a line break to the reference
                if (*p == '\r' && (p + 1 >= T + L || p[1] != '\n')) bad = 1;
                *o = *p;
                o += (c & (C_ACGT | C_N)) ? 1 : 0;
            }
            P.seq.resize((size_t)(o - P.seq.data()));
            P.ok = !bad;
        }
    });
    uint64_t nb = 0;
    for (auto &P : S->pieces) {
        if (!P.ok) return PA_ENOTCANON;
        nb += P.seq.size();
    }
    S->n_records = R;
    S->n_bases = nb;
    S->names.swap(names);
    return PA_OK;
}

pa_status parse(int kind, const uint8_t *T, uint64_t L, int threads, bool universal, pa_seqset **out) {
    if (!out || (kind != PA_FASTA && kind != PA_FASTQ) || (!T && L)) {
        pa::set_error("pa_parse: bad arguments");
        return PA_EINVAL;
    }
    *out = nullptr;  // (bytes >= 0x80 have no class: non-ASCII text is rejected by the class checks)
    pa_seqset *S = new (std::nothrow) pa_seqset();
    if (!S) return PA_ENOMEM;
    S->kind = kind;
    S->threads = std::max(1, std::min(threads, 256));
    pa_status st;
    try {
        st = kind == PA_FASTQ ? parse_fastq(T, L, S->threads, universal, S)
                              : parse_fasta(T, L, S->threads, universal, S);
    } catch (const std::bad_alloc &) {
        st = PA_ENOMEM;
    }
    if (st != PA_OK) {
        if (st == PA_ENOTCANON) pa::set_error("text is outside the canonical FASTA/FASTQ subset");
        if (st == PA_ENOMEM) pa::set_error("pa_parse: out of host memory");
        delete S;
        return st;
    }
    *out = S;
    return PA_OK;
}

}  // namespace

extern "C" {

pa_status pa_parse_text(int32_t kind, const char *text, uint64_t len, int32_t threads, int32_t universal_newlines,
                        pa_seqset **out) {
    return parse(kind, (const uint8_t *)text, len, threads, universal_newlines != 0, out);
}

pa_status pa_parse_file(int32_t kind, const char *path, int32_t threads, pa_seqset **out) {
    if (!path || !out) {
        pa::set_error("pa_parse_file: bad arguments");
        return PA_EINVAL;
    }
    const size_t pl = strlen(path);
    const bool gz = pl >= 3 && strcmp(path + pl - 3, ".gz") == 0;
    if (gz) {  // (pa_gz.cpp: a BGZF file is inflated on all threads; not gzip data: PA_ENOTCANON)
        pa::Gz *f = nullptr;
        const pa_status os = pa::gz_open(path, threads, &f);
        if (os != PA_OK) return os;
        vector<uint8_t> buf;
        size_t n = 0;
        buf.resize(std::max<uint64_t>(64ull << 20, pa::gz_text_size(f)));
        bool eof = false;
        while (!eof) {
            if (buf.size() - n < (16 << 20)) buf.resize(buf.size() * 2);
            uint64_t got = 0;
            const pa_status rs = pa::gz_read(f, buf.data() + n, buf.size() - n, &got, &eof);
            if (rs != PA_OK) {
                pa::gz_close(f);
                return rs == PA_ENOTCANON ? PA_EIO : rs;  // (the Python layer takes the exact path on PA_EIO)
            }
            n += (size_t)got;
            if (got == 0 && !eof) break;
        }
        pa::gz_close(f);
        return parse(kind, buf.data(), n, threads, true, out);
    }
    const int fd = open(path, O_RDONLY);
    if (fd < 0) {
        pa::set_error(std::string("cannot open ") + path);
        return PA_EIO;
    }
    struct stat st;
    if (fstat(fd, &st) != 0) {
        close(fd);
        pa::set_error(std::string("cannot stat ") + path);
        return PA_EIO;
    }
    const uint64_t L = (uint64_t)st.st_size;
    if (L == 0) {
        close(fd);
        return parse(kind, nullptr, 0, threads, true, out);
    }
    void *m = mmap(nullptr, L, PROT_READ, MAP_PRIVATE, fd, 0);  // pages fault in on the parsing threads
    close(fd);
    if (m == MAP_FAILED) {
        pa::set_error(std::string("cannot map ") + path);
        return PA_EIO;
    }
    madvise(m, L, MADV_SEQUENTIAL);
    const pa_status s = parse(kind, (const uint8_t *)m, L, threads, true, out);
    munmap(m, L);
    return s;
}

pa_status pa_seqset_sizes(const pa_seqset *s, uint64_t *n_records, uint64_t *n_bases, uint64_t *name_bytes) {
    if (!s) return PA_EINVAL;
    if (n_records) *n_records = s->n_records;
    if (n_bases) *n_bases = s->n_bases;
    if (name_bytes) {
        uint64_t b = s->names.size();
        for (auto &P : s->pieces) b += P.names.size();
        *name_bytes = b;
    }
    return PA_OK;
}

pa_status pa_seqset_export(const pa_seqset *s, uint8_t *seq, uint8_t *qual, uint64_t *off, char *names) {
    if (!s || !off) return PA_EINVAL;
    const uint64_t np = s->pieces.size();
    vector<uint64_t> base(np + 1, 0), nbase(np + 1, 0), rbase(np + 1, 0);
    for (uint64_t i = 0; i < np; i++) {
        base[i + 1] = base[i] + s->pieces[i].seq.size();
        nbase[i + 1] = nbase[i] + s->pieces[i].names.size();
        rbase[i + 1] = rbase[i] + s->pieces[i].lens.size();
    }
    std::atomic<uint64_t> next{0};
    parallel_for(std::max(1, std::min<int>(s->threads, (int)np)), [&](int) {
        for (;;) {
            const uint64_t i = next.fetch_add(1);
            if (i >= np) break;
            const Piece &P = s->pieces[i];
            if (seq && !P.seq.empty()) memcpy(seq + base[i], P.seq.data(), P.seq.size());
            if (qual && !P.qual.empty()) memcpy(qual + base[i], P.qual.data(), P.qual.size());
            if (names && !P.names.empty()) memcpy(names + nbase[i], P.names.data(), P.names.size());
            if (s->kind == PA_FASTQ) {
                uint64_t o = base[i];
                uint64_t *w = off + rbase[i];
                for (uint64_t r = 0; r < P.lens.size(); r++) {
                    w[r] = o;
                    o += P.lens[r];
                }
            }
        }
    });
    if (s->kind == PA_FASTQ) {
        off[s->n_records] = base[np];
    } else {
        for (uint64_t r = 0; r <= s->n_records; r++) off[r] = base[s->rec_piece[r]];
        if (names && !s->names.empty()) memcpy(names, s->names.data(), s->names.size());
    }
    return PA_OK;
}

void pa_seqset_free(pa_seqset *s) { delete s; }

}  // extern "C"
