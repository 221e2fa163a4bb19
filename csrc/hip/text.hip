// Text analytics for the Vigenere assignment (hw3) and generic histograms
// (slides/Lecture12 "sparse/dense histogram", Lecture21 atomics).
//
//  histogram_u8   : byte histogram over [lo, lo+nbins), per-wave private LDS
//                   sub-histograms (cuts same-address LDS atomic contention)
//                   merged once per block into global counts
//  digraphs       : 26x26 counts of non-overlapping letter pairs
//                   (hw/hw3/solution/solve_cipher_solution.cu:131-151)
//  residue_hist   : per-residue letter histograms [period][26]
//                   (the strided_range + sort + reduce_by_key of :185-200)
//  match_count    : kappa index of coincidence numerators for a batch of
//                   shifts, sum_i [t[i] == t[i+s]] (the inner_product with
//                   equal_to, :156-179), text tile + halo staged in LDS
//  sanitize       : lowercase + keep [a-z] (the remove_copy_if over a
//                   transform_iterator, create_cipher.cu:111-113) as a
//                   reduce-then-scan stream compaction
//  vigenere       : periodic shift with wrap-around, encode or decode
#include "cme213/common.h"
#include "cme213/wave.h"

using namespace cme;

namespace {

__global__ __launch_bounds__(256) void histogram_u8_kernel(const uint8_t* __restrict__ in, long long n, int lo,
                                                           int nbins, int* __restrict__ out) {
    extern __shared__ int sh[];  // [4 waves][nbins]
    const int wid = threadIdx.x / kWave;
    for (int i = threadIdx.x; i < 4 * nbins; i += 256) sh[i] = 0;
    __syncthreads();
    int* h = sh + wid * nbins;
    const long long stride = (long long)gridDim.x * 256 * 4;
    for (long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += stride) {
        uint32_t w;
        if (i + 3 < n) {
            w = *reinterpret_cast<const uint32_t*>(in + i);
        } else {
            w = 0;
            for (int j = 0; j < 4; ++j) w |= (i + j < n ? (uint32_t)in[i + j] : 0xffu) << (8 * j);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (i + j >= n) break;
            const int b = (int)((w >> (8 * j)) & 0xffu) - lo;
            if (b >= 0 && b < nbins) atomicAdd(&h[b], 1);
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < nbins; b += 256) {
        const int c = sh[b] + sh[nbins + b] + sh[2 * nbins + b] + sh[3 * nbins + b];
        if (c) atomicAdd(&out[b], c);
    }
}

__global__ __launch_bounds__(256) void digraph_kernel(const uint8_t* __restrict__ in, long long npairs,
                                                      int* __restrict__ out) {
    __shared__ int h[676];
    for (int i = threadIdx.x; i < 676; i += 256) h[i] = 0;
    __syncthreads();
    for (long long p = blockIdx.x * 256LL + threadIdx.x; p < npairs; p += (long long)gridDim.x * 256) {
        const int a = (int)in[2 * p] - 'a', b = (int)in[2 * p + 1] - 'a';
        if (a >= 0 && a < 26 && b >= 0 && b < 26) atomicAdd(&h[a * 26 + b], 1);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 676; i += 256)
        if (h[i]) atomicAdd(&out[i], h[i]);
}

__global__ __launch_bounds__(256) void residue_hist_kernel(const uint8_t* __restrict__ in, long long n, int period,
                                                           int* __restrict__ out, int use_lds) {
    extern __shared__ int sh[];
    const int nb = period * 26;
    if (use_lds) {
        for (int i = threadIdx.x; i < nb; i += 256) sh[i] = 0;
        __syncthreads();
    }
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const int c = (int)in[i] - 'a';
        if (c < 0 || c >= 26) continue;
        const int bin = (int)(i % period) * 26 + c;
        if (use_lds) atomicAdd(&sh[bin], 1);
        else atomicAdd(&out[bin], 1);
    }
    if (use_lds) {
        __syncthreads();
        for (int i = threadIdx.x; i < nb; i += 256)
            if (sh[i]) atomicAdd(&out[i], sh[i]);
    }
}

// counts[s - s0] += #{i : t[i] == t[i+s]} for s in [s0, s0+ns), ns <= 1024:
// A = t[t0, t0+T), B = t[t0+s0, t0+s0+T+ns) staged in LDS.
constexpr int kMcTile = 4096;
__global__ __launch_bounds__(256) void match_count_kernel(const uint8_t* __restrict__ t, long long n, int s0, int ns,
                                                          unsigned long long* __restrict__ counts) {
    __shared__ uint8_t A[kMcTile];
    __shared__ uint8_t Bh[kMcTile + 1024];
    const long long t0 = (long long)blockIdx.x * kMcTile;
    for (int i = threadIdx.x; i < kMcTile; i += 256) A[i] = t0 + i < n ? t[t0 + i] : 0;
    for (int i = threadIdx.x; i < kMcTile + ns; i += 256) {
        const long long g = t0 + s0 + i;
        Bh[i] = g < n ? t[g] : 0;
    }
    __syncthreads();
    const int lane = lane_id();
    for (int s = s0 + threadIdx.x / kWave; s < s0 + ns; s += 4) {
        unsigned c = 0;
        const int d = s - s0;
        for (int j = lane; j < kMcTile; j += kWave)
            if (t0 + j + s < n) c += A[j] == Bh[j + d];
        const unsigned tot = wave_reduce(c);
        if (lane == 0 && tot) atomicAdd(&counts[d], (unsigned long long)tot);
    }
}

__device__ __forceinline__ bool keep_letter(uint8_t c, uint8_t* low) {
    const uint8_t l = (c >= 'A' && c <= 'Z') ? (uint8_t)(c + 32) : c;
    *low = l;
    return l >= 'a' && l <= 'z';
}

__global__ __launch_bounds__(256) void sanitize_count_kernel(const uint8_t* __restrict__ in, long long n,
                                                             long long chunk, int* __restrict__ part) {
    __shared__ int lds[4];
    const long long b0 = (long long)blockIdx.x * chunk;
    const long long b1 = b0 + chunk < n ? b0 + chunk : n;
    int c = 0;
    for (long long i = b0 + threadIdx.x; i < b1; i += 256) {
        uint8_t l;
        c += keep_letter(in[i], &l);
    }
    const int r = block_reduce<4>(c, lds, OpAdd());
    if (threadIdx.x == 0) part[blockIdx.x] = r;
}

__global__ __launch_bounds__(1024) void exclusive_scan_small_kernel(int* part, int m, int* total) {
    __shared__ int lds[16];
    int carry = 0;
    for (int base = 0; base < m; base += 1024) {
        const int i = base + threadIdx.x;
        int v = i < m ? part[i] : 0;
        int tot;
        int ex = block_exclusive_scan<16>(v, lds, tot, OpAdd());
        if (i < m) part[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(256) void sanitize_write_kernel(const uint8_t* __restrict__ in, long long n,
                                                             long long chunk, const int* __restrict__ part,
                                                             uint8_t* __restrict__ out) {
    __shared__ int lds[4];
    const long long b0 = (long long)blockIdx.x * chunk;
    const long long b1 = b0 + chunk < n ? b0 + chunk : n;
    long long base = part[blockIdx.x];
    for (long long t0 = b0; t0 < b1; t0 += 256) {
        const long long i = t0 + threadIdx.x;
        uint8_t l = 0;
        const int k = i < b1 ? keep_letter(in[i], &l) : 0;
        int tot;
        const int ex = block_exclusive_scan<4>(k, lds, tot, OpAdd());
        if (k) out[base + ex] = l;
        base += tot;
    }
}

__global__ __launch_bounds__(256) void vigenere_kernel(const uint8_t* __restrict__ in, long long n,
                                                       const int* __restrict__ shifts, int period, int sign,
                                                       uint8_t* __restrict__ out) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        int c = (int)in[i] + sign * shifts[i % period];
        while (c > 'z') c -= 26;
        while (c < 'a') c += 26;
        out[i] = (uint8_t)c;
    }
}

}  // namespace

CME_EXPORT int cme_histogram_u8(const uint8_t* in, long long n, int lo, int nbins, int* out, void* stream) {
    if (nbins <= 0 || nbins > 256) return (int)hipErrorInvalidValue;
    hipStream_t s = as_stream(stream);
    CME_TRY(hipMemsetAsync(out, 0, nbins * sizeof(int), s));
    hipLaunchKernelGGL(histogram_u8_kernel, dim3(stream_grid(cdiv(n, 4), 256, 4)), dim3(256), 4 * nbins * sizeof(int),
                       s, in, n, lo, nbins, out);
    CME_LAUNCH_STATUS();
}

CME_EXPORT int cme_digraphs(const uint8_t* in, long long n, int* out, void* stream) {
    hipStream_t s = as_stream(stream);
    CME_TRY(hipMemsetAsync(out, 0, 676 * sizeof(int), s));
    const long long np = n / 2;
    if (np) hipLaunchKernelGGL(digraph_kernel, dim3(stream_grid(np, 256, 2)), dim3(256), 0, s, in, np, out);
    CME_LAUNCH_STATUS();
}

CME_EXPORT int cme_residue_hist(const uint8_t* in, long long n, int period, int* out, void* stream) {
    hipStream_t s = as_stream(stream);
    const size_t nb = (size_t)period * 26;
    CME_TRY(hipMemsetAsync(out, 0, nb * sizeof(int), s));
    const int use_lds = nb * sizeof(int) <= 48 * 1024;
    hipLaunchKernelGGL(residue_hist_kernel, dim3(stream_grid(n, 256, 2)), dim3(256), use_lds ? nb * sizeof(int) : 0,
                       s, in, n, period, out, use_lds);
    CME_LAUNCH_STATUS();
}

// counts: uint64 [ns], shifts s0 .. s0+ns-1 (s0 >= 1), batches of 1024.
CME_EXPORT int cme_match_count(const uint8_t* t, long long n, int s0, int ns, unsigned long long* counts,
                               void* stream) {
    hipStream_t s = as_stream(stream);
    CME_TRY(hipMemsetAsync(counts, 0, ns * sizeof(unsigned long long), s));
    for (int b = 0; b < ns; b += 1024) {
        const int cnt = ns - b < 1024 ? ns - b : 1024;
        hipLaunchKernelGGL(match_count_kernel, dim3(cdiv(n, kMcTile)), dim3(256), 0, s, t, n, s0 + b, cnt,
                           counts + b);
    }
    CME_LAUNCH_STATUS();
}

// Lowercase + keep letters. part: >= 1025 ints of scratch. *count_out (device)
// receives the number of letters kept.
CME_EXPORT int cme_sanitize(const uint8_t* in, long long n, uint8_t* out, int* part, int* count_out, void* stream) {
    hipStream_t s = as_stream(stream);
    const int blocks = n < 1024 * 4096LL ? (int)cdiv(n, 4096) : 1024;
    const long long chunk = (n + blocks - 1) / blocks;
    hipLaunchKernelGGL(sanitize_count_kernel, dim3(blocks), dim3(256), 0, s, in, n, chunk, part);
    hipLaunchKernelGGL(exclusive_scan_small_kernel, dim3(1), dim3(1024), 0, s, part, blocks, count_out);
    hipLaunchKernelGGL(sanitize_write_kernel, dim3(blocks), dim3(256), 0, s, in, n, chunk, part, out);
    CME_LAUNCH_STATUS();
}

CME_EXPORT int cme_vigenere(const uint8_t* in, long long n, const int* shifts, int period, int sign, uint8_t* out,
                            void* stream) {
    hipLaunchKernelGGL(vigenere_kernel, dim3(stream_grid(n, 256)), dim3(256), 0, as_stream(stream), in, n, shifts,
                       period, sign, out);
    CME_LAUNCH_STATUS();
}

// kernels in the occupancy / resource report (cme_kernel_query)
CME_REGISTER_KERNEL(histogram_u8, 256, histogram_u8_kernel);
CME_REGISTER_KERNEL(match_count, 256, match_count_kernel);
CME_REGISTER_KERNEL(vigenere, 256, vigenere_kernel);
