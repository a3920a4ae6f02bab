// Fixed-order summation of slot partials: the reduction step of the deterministic mode
// (sg2_set_deterministic, sg2_common.h).  The kernels write each contribution they would otherwise add with a
// float atomic to its own slot; det_sum adds the slots in an order that depends only on the shapes:
//   out[g * go + i] += sum_{s < S} ws[g * gw + s * ss + i]
// as sums of runs of kRun consecutive s (in s order), then sums of runs of those partial sums, and so on.
// One lane per (g, i[, run]); lanes of a wavefront read consecutive i, so each step is a coalesced stream.
#include "sg2_common.h"

namespace sg2 {
namespace {

constexpr int kRun = 64;

// tmp[(g * K + k) * n + i] = sum_{s in run k} ws[g * gw + s * ss + i]   (K = ceil(S / kRun))
__global__ __launch_bounds__(256) void det_runs_kernel(float* tmp, const float* ws, int64_t gw, int64_t ss, int G,
                                                       int64_t S, int64_t n, int64_t K) {
    const int64_t total = (int64_t)G * K * n;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = t % n;
        const int64_t gk = t / n;
        const int64_t k = gk % K, g = gk / K;
        const int64_t s0 = k * kRun, s1 = s0 + kRun < S ? s0 + kRun : S;
        const float* w = ws + g * gw + i;
        float acc = 0.f;
        for (int64_t s = s0; s < s1; ++s) acc += w[s * ss];
        tmp[t] = acc;
    }
}

// out[g * go + i] += sum_{s < S} ws[g * gw + s * ss + i]   (S <= kRun)
__global__ __launch_bounds__(256) void det_final_kernel(float* out, int64_t go, const float* ws, int64_t gw,
                                                        int64_t ss, int G, int64_t S, int64_t n) {
    const int64_t total = (int64_t)G * n;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = t % n, g = t / n;
        const float* w = ws + g * gw + i;
        float acc = 0.f;
        for (int64_t s = 0; s < S; ++s) acc += w[s * ss];
        out[g * go + i] += acc;
    }
}

inline int grid_for(int64_t total) { return (int)std::min<int64_t>(cdiv(total, 256), 256 * 64); }

}  // namespace

hipError_t det_sum(float* out, int64_t go, const float* ws, int64_t gw, int64_t ss, int G, int64_t S, int64_t n,
                   DetArena& arena, hipStream_t st) {
    if (G <= 0 || n <= 0 || S <= 0) return hipSuccess;
    while (S > kRun) {
        const int64_t K = cdiv(S, kRun);
        float* tmp = arena.get((int64_t)G * K * n);
        if (!tmp) {
            set_error("deterministic scratch too small (det_sum)");
            return hipErrorOutOfMemory;
        }
        det_runs_kernel<<<grid_for((int64_t)G * K * n), 256, 0, st>>>(tmp, ws, gw, ss, G, S, n, K);
        ws = tmp;
        gw = K * n;
        ss = n;
        S = K;
    }
    det_final_kernel<<<grid_for((int64_t)G * n), 256, 0, st>>>(out, go, ws, gw, ss, G, S, n);
    return hipGetLastError();
}

}  // namespace sg2
