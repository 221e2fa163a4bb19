// Compute-region descriptors shared by the multi-step heat kernels
// (heat2d.hip: stream2 / streamN; heat_pipe.hip: the wave-pipelined pass).
#pragma once

namespace cme {

constexpr int cgcd(int a, int b) { return b == 0 ? a : cgcd(b, a % b); }

// A rectangle of cells [xb, xe) x [yb, ye) of a device grid.
struct Region {
    int xb, xe, yb, ye;
};

// Up to eight output regions per launch (a distributed subdomain's border
// strips go out as ONE launch, or its deep interior AND border strips in the
// fused schedule); every region shares the intermediate-step region passed
// next to it.
constexpr int kMaxS2Regions = 8;
struct S2Regions {
    int n;
    int xb[kMaxS2Regions], xe[kMaxS2Regions], yb[kMaxS2Regions], ye[kMaxS2Regions];
    int strips[kMaxS2Regions], chunk[kMaxS2Regions];
    int wave_end[kMaxS2Regions];  // cumulative wave (or workgroup-task) counts
};

// Output columns of one 64-lane strip of an NS-step pass (4 columns per lane;
// step k is valid on lanes k..63-k, x-neighbours arrive through DPP).
template <int NS>
struct StripN {
    static constexpr int kOut = (64 - 2 * NS) * 4;
};

// Output columns of one strip of the wave-pipelined pass: WPR waves side by
// side per timestep role (64*WPR lanes of VW columns). VW = 4: NS lanes lost
// per side (one lane per step, exact at order 8). VW = 8 (wide lanes): the
// whole lanes covering the NS*B columns each side loses over NS steps.
template <int NS, int WPR, int VW = 4, int B = 4>
struct PipeOut {
    static constexpr int kMargin = VW == 4 ? NS : (NS * B + VW - 1) / VW;
    static constexpr int kOut = (64 * WPR - 2 * kMargin) * VW;
};

// Fused-schedule gate of the pipelined pass: workgroups of regions
// [from, n) wait until *flag >= val (wrap-safe) before reading their input
// -- the halo exchange of the previous pass signals the flag from the comm
// stream (dist_heat.hip). Bounded: a wait past the spin limit sets *timeout
// (pinned host word) and proceeds. flag == nullptr: no gate. `spins`: polls
// before giving up (~2^24: tens of seconds; CME_DIST_GATE_SPINS lowers it so
// a test can force the timeout path).
struct PipeGate {
    const unsigned* flag = nullptr;
    unsigned val = 0;
    int from = 0;
    unsigned* timeout = nullptr;
    unsigned spins = 1u << 24;
    // profiling only (hip_tune/heat_pipe_tune.hip cme_heat_pipe_trace): per
    // task {start, end} wall clock (100 MHz) and {HW_ID, XCC_ID, region}
    unsigned long long* trace = nullptr;
};

}  // namespace cme
