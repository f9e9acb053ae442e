// Hash-table home-slot parameters, shared by host (index metadata) and device.
#pragma once

#include <stdint.h>

namespace pad {

// Where a key starts probing (home_of in pa_device.h): multiply-high hashing
// over all cap slots.
struct HomeCfg {
    uint64_t cap;  // slots (a whole number of 64-B lines)
};

}  // namespace pad
