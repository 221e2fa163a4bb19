// LDS-resident temporal blocking for SMALL heat grids (the hw5 shapes,
// hw/hw5/2dHeat_solution.cpp:501-535: 1000^2 / 2000^2, order 8, fp64).
//
// Why a separate pass: the streaming passes (heat2d.hip streamN, heat_pipe.hip)
// give every wave a 224-480-column strip and walk it down the rows. A 1000^2
// grid has 2-5 such strips, so filling 1024 SIMDs means chunks of a handful
// of rows, each paying 2(NS-1)B warm-up rows -- the pass is latency- and
// recompute-bound at ~17 us for three steps (profiles/hw5_default_path_r3.jsonl)
// while its arithmetic is ~1.5 us. Here a 1024-thread workgroup owns a 2-D
// output tile (64 x TY points): it loads the tile plus an NS*B-deep halo into
// LDS ONCE, runs NS timesteps entirely in LDS (each step over a region B
// narrower per side than the one before -- the dependency cone), and writes
// only the tile. 1000^2 is 256 tiles of 64 x 64: one workgroup per CU.
//
// Inside a step each thread owns a column PAIR (one 16-B LDS word of fp64,
// 8-B of fp32) and a band of rows; it walks the band with a (2B+1)-row
// register window for the y-neighbours (a compile-time ring: the row loop is
// unrolled by 2B+1, so no register shifts) and reads the x-neighbours as
// B (+1) aligned pairs from LDS. Every point is evaluated by the shared
// expression of heat_stencil.h (exact or FMA), so a pass is bitwise equal to
// NS single steps. Points outside the region g (the Dirichlet ghost cells)
// are never written: both LDS buffers start with the same loaded values, so
// every step reads their fixed BC values.
#include "heat_tile.h"

using namespace cme;

namespace {

constexpr int kTileThreads = 1024;  // 16 waves: 4 per SIMD (tune_tile.py cfg 2)

// Tile shapes: fp64 64 x 64 (1000^2 = 256 tiles, one workgroup per CU; LDS
// 2 x (64 + 2NSB)^2 x 8 B = 102 / 124 / 147 KB at NS = 2 / 3 / 4); fp32
// 64 x 64 as well (half the LDS: two workgroups per CU up to NS = 4).
// Output tiles go out with non-temporal stores: the kernel boundary after a
// pass shrinks (3.8 -> 3.2 us) and a 1000^2 pass runs 19.8 -> 18.7 us exact,
// 17.1 -> 16.1 FMA (benchmarks/trace_tile.py, profiles/heat_tile_r4.md).
template <typename T, int ORDER, bool FMA>
int tile_ns(const T* p, T* c, int pitch, int gy, Region g, int ns, T xcfl, T ycfl, hipStream_t s) {
    switch (ns) {
        case 1: return cme_tile::launch_tile<T, ORDER, 1, FMA, 64, 64, kTileThreads, true>(p, c, pitch, gy, g, xcfl, ycfl, s);
        case 2: return cme_tile::launch_tile<T, ORDER, 2, FMA, 64, 64, kTileThreads, true>(p, c, pitch, gy, g, xcfl, ycfl, s);
        case 3: return cme_tile::launch_tile<T, ORDER, 3, FMA, 64, 64, kTileThreads, true>(p, c, pitch, gy, g, xcfl, ycfl, s);
        case 4: return cme_tile::launch_tile<T, ORDER, 4, FMA, 64, 64, kTileThreads, true>(p, c, pitch, gy, g, xcfl, ycfl, s);
        default: return (int)hipErrorInvalidValue;
    }
}

template <typename T>
int tile_pass(const T* p, T* c, int pitch, int gy, Region g, int order, int ns, int fma, T xcfl, T ycfl,
              hipStream_t s) {
    if (fma) {
        switch (order) {
            case 2: return tile_ns<T, 2, true>(p, c, pitch, gy, g, ns, xcfl, ycfl, s);
            case 4: return tile_ns<T, 4, true>(p, c, pitch, gy, g, ns, xcfl, ycfl, s);
            case 8: return tile_ns<T, 8, true>(p, c, pitch, gy, g, ns, xcfl, ycfl, s);
        }
    } else {
        switch (order) {
            case 2: return tile_ns<T, 2, false>(p, c, pitch, gy, g, ns, xcfl, ycfl, s);
            case 4: return tile_ns<T, 4, false>(p, c, pitch, gy, g, ns, xcfl, ycfl, s);
            case 8: return tile_ns<T, 8, false>(p, c, pitch, gy, g, ns, xcfl, ycfl, s);
        }
    }
    return (int)hipErrorInvalidValue;
}

}  // namespace

// One ns-step (1-4) pass of region g = [xb, xe) x [yb, ye) (every cell of
// the buffers outside g holds the same fixed value in prev and curr -- the
// whole-interior case of heat_run) from prev into curr.
CME_EXPORT int cme_heat_tile_f32(const float* prev, float* curr, int pitch, int gy, int xb, int xe, int yb, int ye,
                                 int order, int nsteps, float xcfl, float ycfl, int fma, void* stream) {
    return tile_pass<float>(prev, curr, pitch, gy, Region{xb, xe, yb, ye}, order, nsteps, fma, xcfl, ycfl,
                            as_stream(stream));
}

CME_EXPORT int cme_heat_tile_f64(const double* prev, double* curr, int pitch, int gy, int xb, int xe, int yb, int ye,
                                 int order, int nsteps, double xcfl, double ycfl, int fma, void* stream) {
    return tile_pass<double>(prev, curr, pitch, gy, Region{xb, xe, yb, ye}, order, nsteps, fma, xcfl, ycfl,
                             as_stream(stream));
}

CME_REGISTER_KERNEL(heat_tile4_fma_f64_o8, kTileThreads, cme_tile::heat_tile_kernel<double, 8, 4, true, 64, 64, kTileThreads>);
CME_REGISTER_KERNEL(heat_tile2_f64_o8, kTileThreads, cme_tile::heat_tile_kernel<double, 8, 2, false, 64, 64, kTileThreads>);
CME_REGISTER_KERNEL(heat_tile4_fma_f32_o8, kTileThreads, cme_tile::heat_tile_kernel<float, 8, 4, true, 64, 64, kTileThreads>);
