// pa_gz.cpp -- gzip input of the readers (src/data_file.py:117-128: a ".gz"
// FASTA/FASTQ file is read through gzip.open(...).read()).
//
// A BGZF file (bgzip, the usual compressed FASTQ of sequencing pipelines) is a
// series of gzip members of at most 64 KiB of text, each recording its
// compressed size in a "BC" extra field and its text size and CRC-32 in its
// trailer.  Its members are located without inflating anything, so they are
// inflated on all host threads at once, each straight into its place in the
// caller's buffer, and each checked against its CRC-32 and size.  Any other
// gzip file (one member, as `gzip` writes) is inflated on all host threads by
// pa_pgz.cpp (block boundaries found by search, 32-KiB windows resolved once
// the previous chunk is known; PA_PGZ=0: zlib on one thread).
// Data that is not what gzip.open would read cleanly -- a bad CRC, a truncated
// member, bytes after the last one -- gives PA_ENOTCANON, so the caller takes
// the exact path, which raises the reference's own error.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "pa_gz.h"
#include "pa_internal.h"
#include "pa_pgz.h"

namespace pa {

struct GzMember {
    uint64_t coff;   // compressed data (raw deflate) offset in the file
    uint32_t clen;   // its length
    uint32_t isize;  // text bytes
    uint32_t crc;    // CRC-32 of the text
    uint64_t uoff;   // text offset in the decompressed stream
};

struct Gz {
    std::string path;
    int threads = 1;
    // BGZF: the file mapped and its members
    bool bgzf = false;
    const uint8_t *map = nullptr;
    uint64_t map_len = 0;
    std::vector<GzMember> members;
    uint64_t next = 0;  // next member to hand out
    uint64_t total = 0;
    // any other gzip file: parallel inflate of the mapped file, or zlib
    Pgz *pgz = nullptr;
    gzFile gz = nullptr;
    bool eof = false;
};

namespace {

inline uint32_t le16(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
inline uint32_t le32(const uint8_t *p) { return le16(p) | (le16(p + 2) << 16); }

// The members of a BGZF file, or false if the file is not one (then zlib reads it).
bool bgzf_index(const uint8_t *m, uint64_t len, std::vector<GzMember> &out) {
    uint64_t o = 0, u = 0;
    while (o < len) {
        if (len - o < 28 || m[o] != 0x1f || m[o + 1] != 0x8b || m[o + 2] != 8 || m[o + 3] != 4) return false;
        const uint32_t xlen = le16(m + o + 10);
        if (12ull + xlen + 8 > len - o) return false;
        uint32_t bsize = 0;
        for (uint32_t x = 0; x + 4 <= xlen;) {  // the extra subfields: SI1 SI2 LEN data
            const uint8_t *sf = m + o + 12 + x;
            const uint32_t sl = le16(sf + 2);
            if (sf[0] == 66 && sf[1] == 67 && sl == 2) bsize = le16(sf + 4) + 1;
            x += 4 + sl;
        }
        if (bsize == 0 || bsize < 12 + xlen + 8 || bsize > len - o) return false;
        GzMember g;
        g.coff = o + 12 + xlen;
        g.clen = bsize - 12 - xlen - 8;
        g.crc = le32(m + o + bsize - 8);
        g.isize = le32(m + o + bsize - 4);
        g.uoff = u;
        if (g.isize > (1u << 16)) return false;  // (BGZF blocks hold at most 64 KiB)
        out.push_back(g);
        u += g.isize;
        o += bsize;
    }
    return !out.empty();
}

bool inflate_member(z_stream &z, const uint8_t *src, const GzMember &g, uint8_t *dst) {
    if (inflateReset(&z) != Z_OK) return false;
    z.next_in = const_cast<Bytef *>(src + g.coff);
    z.avail_in = g.clen;
    z.next_out = dst;
    z.avail_out = g.isize;
    const int r = inflate(&z, Z_FINISH);
    if (r != Z_STREAM_END || z.avail_out != 0) return false;
    return (uint32_t)crc32(0L, dst, g.isize) == g.crc;
}

}  // namespace

pa_status gz_open(const char *path, int threads, Gz **out) {
    *out = nullptr;
    auto *g = new Gz();
    g->path = path;
    g->threads = std::max(1, threads);
    const int fd = open(path, O_RDONLY);
    struct stat st;
    if (fd < 0 || fstat(fd, &st) != 0) {
        if (fd >= 0) close(fd);
        delete g;
        set_error(std::string("cannot open ") + path);
        return PA_EIO;
    }
    const uint64_t len = (uint64_t)st.st_size;
    void *m = len ? mmap(nullptr, len, PROT_READ, MAP_PRIVATE, fd, 0) : MAP_FAILED;
    close(fd);
    if (m != MAP_FAILED) {
        madvise(m, len, MADV_SEQUENTIAL);
        if (bgzf_index((const uint8_t *)m, len, g->members)) {
            g->bgzf = true;
            g->map = (const uint8_t *)m;
            g->map_len = len;
            g->total = g->members.back().uoff + g->members.back().isize;
            *out = g;
            return PA_OK;
        }
        g->members.clear();
        const char *e = std::getenv("PA_PGZ");
        Pgz *p = nullptr;
        if (!(e && e[0] == '0') && pgz_open((const uint8_t *)m, len, g->threads, &p) == PA_OK) {
            g->pgz = p;
            g->map = (const uint8_t *)m;
            g->map_len = len;
            *out = g;
            return PA_OK;
        }
        munmap(m, len);
    }
    g->gz = gzopen(path, "rb");
    if (!g->gz) {
        delete g;
        set_error(std::string("cannot open ") + path);
        return PA_EIO;
    }
    gzbuffer(g->gz, 1 << 20);
    if (gzdirect(g->gz)) {  // not gzip data: the exact path raises the reference's BadGzipFile
        gzclose(g->gz);
        delete g;
        set_error(std::string("not a gzip file: ") + path);
        return PA_ENOTCANON;
    }
    *out = g;
    return PA_OK;
}

bool gz_is_bgzf(const Gz *g) { return g && g->bgzf; }
uint64_t gz_text_size(const Gz *g) { return g && g->bgzf ? g->total : 0; }

pa_status gz_read(Gz *g, uint8_t *dst, uint64_t n, uint64_t *got, bool *eof) {
    *got = 0;
    if (g->pgz) return pgz_read(g->pgz, dst, n, got, eof);
    if (!g->bgzf) {
        uint64_t k = 0;
        while (k < n) {
            const int r = gzread(g->gz, dst + k, (unsigned)std::min<uint64_t>(n - k, 1u << 30));
            if (r < 0) {  // a damaged file: the exact path (Python gzip) raises the reference's error
                set_error("gzip data error in " + g->path);
                return PA_ENOTCANON;
            }
            if (r == 0) {
                g->eof = true;
                break;
            }
            k += (uint64_t)r;
        }
        if (!g->eof && gzeof(g->gz)) g->eof = true;
        *got = k;
        *eof = g->eof;
        return PA_OK;
    }
    // whole members only, as many as fit (the caller's windows are >= 64 KiB)
    const uint64_t m0 = g->next, base = m0 < g->members.size() ? g->members[m0].uoff : g->total;
    uint64_t m1 = m0;
    while (m1 < g->members.size() && g->members[m1].uoff + g->members[m1].isize - base <= n) m1++;
    if (m1 == m0 && m0 < g->members.size()) {
        set_error("gzip window smaller than one BGZF member");
        return PA_EINVAL;
    }
    const uint64_t cnt = m1 - m0;
    std::atomic<int> bad{0};
    const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)g->threads, cnt / 8));
    auto work = [&](int t) {
        z_stream z{};
        if (inflateInit2(&z, -15) != Z_OK) {
            bad = 1;
            return;
        }
        for (uint64_t i = m0 + cnt * t / T; i < m0 + cnt * (t + 1) / T && !bad; i++) {
            const GzMember &mb = g->members[i];
            if (!inflate_member(z, g->map, mb, dst + (mb.uoff - base))) bad = 1;
        }
        inflateEnd(&z);
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; t++) th.emplace_back(work, t);
    work(0);
    for (auto &x : th) x.join();
    if (bad) {
        set_error("gzip data error (BGZF member CRC or size) in " + g->path);
        return PA_ENOTCANON;
    }
    g->next = m1;
    *got = (m1 < g->members.size() ? g->members[m1].uoff : g->total) - base;
    *eof = m1 >= g->members.size();
    return PA_OK;
}

void gz_close(Gz *g) {
    if (!g) return;
    if (g->pgz) pgz_close(g->pgz);
    if (g->map) munmap(const_cast<uint8_t *>(g->map), g->map_len);
    if (g->gz) gzclose(g->gz);
    delete g;
}

}  // namespace pa
