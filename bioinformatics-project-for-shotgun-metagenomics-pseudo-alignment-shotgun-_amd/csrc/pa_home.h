// Hash-table home-slot parameters, shared by host (index metadata) and device.
#pragma once

#include <stdint.h>

namespace pad {

// Where a key starts probing (home_of in pa_device.h): multiply-high hashing
// over all cap slots.  nreg / R / k / m are kept for the layout of the struct
// (m is always 0).
struct HomeCfg {
    uint64_t cap;    // slots (a multiple of R when m > 0)
    uint64_t nreg;   // cap / R
    uint32_t R;      // region size in slots (power of two)
    int k, m;        // m == 0: plain hashing
};

}  // namespace pad
