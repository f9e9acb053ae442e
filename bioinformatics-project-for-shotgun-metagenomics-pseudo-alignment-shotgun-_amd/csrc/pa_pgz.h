// Parallel inflate of ordinary (non-BGZF) gzip files: pa_pgz.cpp.
#pragma once

#include <stdint.h>

#include "../../include/pa.h"

namespace pa {
struct Pgz;
// The member(s) of the gzip file mapped at [map, map + len) (kept mapped by the caller).
pa_status pgz_open(const uint8_t *map, uint64_t len, int threads, Pgz **out);
// Up to n bytes of text; eof once every member is inflated and checked.
pa_status pgz_read(Pgz *g, uint8_t *dst, uint64_t n, uint64_t *got, bool *eof);
void pgz_close(Pgz *g);
}  // namespace pa
