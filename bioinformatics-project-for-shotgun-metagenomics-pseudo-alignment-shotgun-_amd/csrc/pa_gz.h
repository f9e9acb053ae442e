// gzip input of the readers (pa_gz.cpp): BGZF member-parallel inflate, zlib
// for any other gzip file.  Internal to libpa.so.
#pragma once

#include <stdint.h>

#include "../../include/pa.h"

namespace pa {
struct Gz;
// PA_EIO: the file cannot be read; PA_ENOTCANON: not gzip data (the exact
// path raises the reference's error).
pa_status gz_open(const char *path, int threads, Gz **out);
// The next text bytes, up to n (BGZF: whole members, n >= 64 KiB); *eof once
// the stream is done.  PA_ENOTCANON: damaged data (the exact path raises).
pa_status gz_read(Gz *g, uint8_t *dst, uint64_t n, uint64_t *got, bool *eof);
bool gz_is_bgzf(const Gz *g);
uint64_t gz_text_size(const Gz *g);  // BGZF: the whole text's size, else 0
void gz_close(Gz *g);
}  // namespace pa
