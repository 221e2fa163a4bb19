// Control block of a persistent launch with bounded in-kernel waits
// (heat_flow.hip, heat_tile_res.hip): device words zeroed by one memset per
// call (tickets, completion words, abort word, give-up records) and a pinned
// host word the kernels set when a wait gives up -- sticky, read after the
// stream is synchronised. One block per launch family and device
// (persist_ws_for): the family's launches on a device are serialised on
// their stream, and a device switch never reuses another device's memory.
#pragma once

#include "cme213/common.h"

namespace cme {

struct PersistWs {
    unsigned* dev = nullptr;
    size_t words = 0;              // allocated device words (a multiple of 4: 16-B padded)
    unsigned* timeout = nullptr;  // pinned, host-coherent

    // at least `need` device words (grown, never shrunk) and the pinned word
    int reserve(size_t need) {
        need = ((need + 3) / 4) * 4;
        if (words < need) {
            if (dev) CME_TRY(hipFree(dev));
            dev = nullptr;
            words = 0;
            CME_TRY(hipMalloc(&dev, need * 4));
            words = need;
        }
        if (!timeout) {
            CME_TRY(hipHostMalloc(&timeout, 16, hipHostMallocCoherent));
            *timeout = 0u;
        }
        return 0;
    }

    // the sticky give-up word (0 before any launch); reset clears it
    unsigned take_timeout(bool reset) {
        const unsigned v = timeout ? *timeout : 0u;
        if (reset && timeout) *timeout = 0u;
        return v;
    }
};

// The control block of launch family F on the current device (up to 64).
template <int F>
PersistWs& persist_ws_for() {
    static PersistWs blocks[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    return blocks[dev & 63];
}

}  // namespace cme
