// Fixed-order summation of slot partials: the reduction step of the deterministic mode
// (sg2_set_deterministic, sg2_common.h).  The kernels write each contribution they would otherwise add with a
// float atomic to its own slot; det_sum adds the slots in an order that depends only on the shapes:
//   out[g * go + i] += sum_{s < S} ws[g * gw + s * ss + i]
// One workgroup per (64 consecutive i, g): lane row r (0..3) sums s = r, r + 4, r + 8, ... in increasing s (eight
// independent loads in flight per lane, added in s order), then the four row sums are added in row order; each load
// instruction of a wave reads 64 consecutive floats of one slot.  When that leaves too few workgroups (a few outputs
// summed over thousands of slots), a first launch sums chunks of consecutive s the same way into a temporary and a
// second adds the chunk sums in chunk order.
#include "sg2_common.h"

#include <cstdio>
#include <cstdlib>

namespace sg2 {
namespace {

constexpr int kRows = 4, kLanes = 64, kUnroll = 8;

__global__ __launch_bounds__(256) void det_sum_kernel(float* out, int64_t go, const float* ws, int64_t gw, int64_t ss,
                                                      int64_t S, int64_t n, int64_t chunk, int64_t to, int assign) {
    // blockIdx.z: a chunk of `chunk` consecutive s (one chunk: the whole sum); assign: out = instead of out +=
    __shared__ float part[kRows][kLanes];
    const int il = threadIdx.x & (kLanes - 1), r = threadIdx.x / kLanes;
    const int64_t i = (int64_t)blockIdx.x * kLanes + il;
    const int64_t g = blockIdx.y;
    const int64_t s0 = (int64_t)blockIdx.z * chunk, s1 = s0 + chunk < S ? s0 + chunk : S;
    float acc = 0.f;
    if (i < n) {
        const float* w = ws + g * gw + i;
        int64_t s = s0 + r;
        for (; s + (kUnroll - 1) * kRows < s1; s += kUnroll * kRows) {
            float v[kUnroll];
#pragma unroll
            for (int k = 0; k < kUnroll; ++k) v[k] = w[(s + k * kRows) * ss];
#pragma unroll
            for (int k = 0; k < kUnroll; ++k) acc += v[k];
        }
        for (; s < s1; s += kRows) acc += w[s * ss];
    }
    part[r][il] = acc;
    __syncthreads();
    if (r == 0 && i < n) {
        const float v = ((part[0][il] + part[1][il]) + part[2][il]) + part[3][il];
        float* o = out + g * go + (int64_t)blockIdx.z * to + i;
        if (assign) *o = v;
        else *o += v;
    }
}

}  // namespace

hipError_t det_sum(float* out, int64_t go, const float* ws, int64_t gw, int64_t ss, int G, int64_t S, int64_t n,
                   DetArena& arena, hipStream_t st) {
    if (G <= 0 || n <= 0 || S <= 0) return hipSuccess;
    if (G > 65535) return hipErrorInvalidValue;
    const int64_t bx = cdiv(n, kLanes);
    // few outputs over a long sum (a bias or dot reduction over every pixel block): first chunks of the s range in
    // parallel into a temporary, then their sums in chunk order (both steps fixed by the shapes alone)
    static const bool trace = getenv("SG2_DET_TRACE") != nullptr;   // diagnostics: one line per call (tools/)
    const int64_t S0 = S;
    int64_t K = 1;
    if (bx * G < 512 && S > 16 * kRows) K = std::min<int64_t>(std::min<int64_t>(cdiv(S, 16 * kRows), 1024),
                                                              cdiv(512, bx * G));
    if (K > 1) {
        const int64_t chunk = cdiv(S, K);
        K = cdiv(S, chunk);
        float* tmp = arena.get((int64_t)G * K * n);
        if (!tmp) {             // (no single-launch fallback: the summation order must follow from the shapes alone)
            set_error("deterministic scratch too small (det_sum)");
            return hipErrorOutOfMemory;
        }
        {
            det_sum_kernel<<<dim3((unsigned)bx, (unsigned)G, (unsigned)K), 256, 0, st>>>(tmp, K * n, ws, gw, ss, S, n,
                                                                                       chunk, n, 1);
            ws = tmp;
            gw = K * n;
            ss = n;
            S = K;
        }
    }
    if (trace) fprintf(stderr, "DETSUM G=%d n=%lld S=%lld K=%lld\n", G, (long long)n, (long long)S0,
                       (long long)K);
    det_sum_kernel<<<dim3((unsigned)bx, (unsigned)G, 1), 256, 0, st>>>(out, go, ws, gw, ss, S, n, S, 0, 0);
    return hipGetLastError();
}

}  // namespace sg2
