// Hash-table home-slot parameters, shared by host (index metadata) and device.
#pragma once

#include <stdint.h>

namespace pad {

// Where a key starts probing: with m > 0 the home slot lies in a region of R
// slots chosen by the key's minimizer (see home_of in pa_device.h); m == 0 is
// plain multiply-high hashing over all cap slots.
struct HomeCfg {
    uint64_t cap;    // slots (a multiple of R when m > 0)
    uint64_t nreg;   // cap / R
    uint32_t R;      // region size in slots (power of two)
    int k, m;        // m == 0: plain hashing
};

}  // namespace pad
