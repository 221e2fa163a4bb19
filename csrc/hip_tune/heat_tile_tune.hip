// Tuning arms of the LDS-resident tile pass (csrc/hip/heat_tile.h): tile
// shape and workgroup size, fp64 order 8 (the hw5 shapes), exact and FMA.
//   cfg 0: 64 x 64, 256 threads   1: 64 x 64, 512   2: 64 x 64, 1024
//   cfg 3: 64 x 32, 256           4: 64 x 32, 512   5: 128 x 32, 512
//   cfg 6: 32 x 64, 256           7: 128 x 64, 1024
#include "../hip/heat_tile.h"

using namespace cme;

namespace {
template <int NS, bool FMA>
int tile_cfg(const double* p, double* c, int pitch, int gy, Region g, int cfg, double xc, double yc, hipStream_t s) {
    using namespace cme_tile;
    switch (cfg) {
        case 0: return launch_tile<double, 8, NS, FMA, 64, 64, 256>(p, c, pitch, gy, g, xc, yc, s);
        case 1: return launch_tile<double, 8, NS, FMA, 64, 64, 512>(p, c, pitch, gy, g, xc, yc, s);
        case 2: return launch_tile<double, 8, NS, FMA, 64, 64, 1024>(p, c, pitch, gy, g, xc, yc, s);
        case 3: return launch_tile<double, 8, NS, FMA, 64, 32, 256>(p, c, pitch, gy, g, xc, yc, s);
        case 4: return launch_tile<double, 8, NS, FMA, 64, 32, 512>(p, c, pitch, gy, g, xc, yc, s);
        case 5:
            if constexpr (NS <= 2) return launch_tile<double, 8, NS, FMA, 128, 32, 512>(p, c, pitch, gy, g, xc, yc, s);
            return (int)hipErrorInvalidValue;
        case 6: return launch_tile<double, 8, NS, FMA, 32, 64, 256>(p, c, pitch, gy, g, xc, yc, s);
        case 7:
            if constexpr (NS <= 1) return launch_tile<double, 8, NS, FMA, 128, 64, 1024>(p, c, pitch, gy, g, xc, yc, s);
            return (int)hipErrorInvalidValue;
        default: return (int)hipErrorInvalidValue;
    }
}
template <bool FMA>
int tile_ns(const double* p, double* c, int pitch, int gy, Region g, int ns, int cfg, double xc, double yc,
            hipStream_t s) {
    switch (ns) {
        case 1: return tile_cfg<1, FMA>(p, c, pitch, gy, g, cfg, xc, yc, s);
        case 2: return tile_cfg<2, FMA>(p, c, pitch, gy, g, cfg, xc, yc, s);
        case 3: return tile_cfg<3, FMA>(p, c, pitch, gy, g, cfg, xc, yc, s);
        case 4: return tile_cfg<4, FMA>(p, c, pitch, gy, g, cfg, xc, yc, s);
        default: return (int)hipErrorInvalidValue;
    }
}
}  // namespace

// `iters` timesteps of the whole interior g from a into b (ping-pong), ns
// steps per tile pass (the remainder as one shorter pass); *final_idx = 1
// if the result is in b.
CME_EXPORT int cme_heat_tile_tune(double* a, double* b, int pitch, int gy, int xb, int xe, int yb, int ye, int ns,
                                  int fma, int cfg, int iters, double xcfl, double ycfl, int* final_idx,
                                  void* stream) {
    const Region g{xb, xe, yb, ye};
    double* buf[2] = {a, b};
    int cur = 0;
    for (int i = 0; i < iters;) {
        const int k = iters - i < ns ? iters - i : ns;
        const int rc = fma ? tile_ns<true>(buf[cur], buf[cur ^ 1], pitch, gy, g, k, cfg, xcfl, ycfl, as_stream(stream))
                           : tile_ns<false>(buf[cur], buf[cur ^ 1], pitch, gy, g, k, cfg, xcfl, ycfl,
                                            as_stream(stream));
        if (rc) return rc;
        cur ^= 1;
        i += k;
    }
    *final_idx = cur;
    return 0;
}

// One ns-step pass of the production tile shape (64 x 64, 1024 threads) with
// per-workgroup phase timestamps (heat_tile.h trace: entry, load, each step,
// stores; 8 words per workgroup, 100 MHz wall clock).
// nts: non-temporal output stores.
CME_EXPORT int cme_heat_tile_trace(const double* a, double* b, int pitch, int gy, int xb, int xe, int yb, int ye,
                                   int ns, int fma, int nts, double xcfl, double ycfl, unsigned long long* trace,
                                   void* stream) {
    using namespace cme_tile;
    const Region g{xb, xe, yb, ye};
    hipStream_t s = as_stream(stream);
#define CME_TT(NS)                                                                                                 \
    if (nts)                                                                                                      \
        return fma ? launch_tile<double, 8, NS, true, 64, 64, 1024, true>(a, b, pitch, gy, g, xcfl, ycfl, s, trace) \
                   : launch_tile<double, 8, NS, false, 64, 64, 1024, true>(a, b, pitch, gy, g, xcfl, ycfl, s,      \
                                                                              trace);                              \
    return fma ? launch_tile<double, 8, NS, true, 64, 64, 1024>(a, b, pitch, gy, g, xcfl, ycfl, s, trace)       \
               : launch_tile<double, 8, NS, false, 64, 64, 1024>(a, b, pitch, gy, g, xcfl, ycfl, s, trace)
    switch (ns) {
        case 2: CME_TT(2);
        case 3: CME_TT(3);
        case 4: CME_TT(4);
        default: return (int)hipErrorInvalidValue;
    }
#undef CME_TT
}
