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

constexpr int kRows = 4, kLanes = 64, kUnroll = 8, kMaxDetJobs = 4;

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

// Few slots over many outputs (a weight gradient's pixel splits: S <= kVecS over millions of i): a lane owns four
// consecutive i (16-byte loads) and adds s = 0, 1, ..., S - 1 in order.  The 4-row form leaves three of its four
// lane rows idle at S = 1 and issues one 4-byte load per lane per slot (1.2-2.5 TB/s at S <= 4).
constexpr int kVecS = 16;

__global__ __launch_bounds__(256) void det_sum_vec4_kernel(float* out, int64_t go, const float* ws, int64_t gw,
                                                           int64_t ss, int64_t S, int64_t n4, int assign) {
    const int64_t i4 = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t g = blockIdx.y;
    if (i4 >= n4) return;
    const float4* w = (const float4*)(ws + g * gw) + i4;
    const int64_t ss4 = ss / 4;
    float4 acc = w[0];
    int64_t s = 1;
    for (; s + 7 < S; s += 8) {
        float4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = w[(s + k) * ss4];
#pragma unroll
        for (int k = 0; k < 8; ++k) { acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w; }
    }
    for (; s < S; ++s) {
        const float4 v = w[s * ss4];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    float4* o = (float4*)(out + g * go) + i4;
    if (assign) {
        *o = acc;
        return;
    }
    float4 r = *o;
    r.x += acc.x; r.y += acc.y; r.z += acc.z; r.w += acc.w;
    *o = r;
}

// Several independent sums in one launch (the pairs of sums one kernel's slots feed, e.g. sg2_layer_bwd's bias and
// demodulation gradients): workgroup b belongs to the job whose block range holds it and runs det_sum_kernel's body
// for that job's (i block, g, chunk).
struct DetJob {
    float* out;
    const float* ws;
    int64_t go, gw, ss, S, n, chunk, to;
    int assign, bx, G, K, begin;
};
struct DetJobs {
    DetJob j[kMaxDetJobs];
    int count;
};

__global__ __launch_bounds__(256) void det_sum_multi_kernel(DetJobs jobs) {
    __shared__ float part[kRows][kLanes];
    int jb = 0;
    while (jb + 1 < jobs.count && (int)blockIdx.x >= jobs.j[jb + 1].begin) ++jb;
    const DetJob& J = jobs.j[jb];
    const int l = (int)blockIdx.x - J.begin;
    const int bxi = l % J.bx, rest = l / J.bx;
    const int64_t g = rest % J.G, z = rest / J.G;
    const int il = threadIdx.x & (kLanes - 1), r = threadIdx.x / kLanes;
    const int64_t i = (int64_t)bxi * kLanes + il;
    const int64_t s0 = z * J.chunk, s1 = s0 + J.chunk < J.S ? s0 + J.chunk : J.S;
    float acc = 0.f;
    if (i < J.n) {
        const float* w = J.ws + g * J.gw + i;
        int64_t s = s0 + r;
        for (; s + (kUnroll - 1) * kRows < s1; s += kUnroll * kRows) {
            float v[kUnroll];
#pragma unroll
            for (int k = 0; k < kUnroll; ++k) v[k] = w[(s + k * kRows) * J.ss];
#pragma unroll
            for (int k = 0; k < kUnroll; ++k) acc += v[k];
        }
        for (; s < s1; s += kRows) acc += w[s * J.ss];
    }
    part[r][il] = acc;
    __syncthreads();
    if (r == 0 && i < J.n) {
        const float v = ((part[0][il] + part[1][il]) + part[2][il]) + part[3][il];
        float* o = J.out + g * J.go + z * J.to + i;
        if (J.assign) *o = v;
        else *o += v;
    }
}

// det_sum into the parameter layout of a convolution weight gradient: the slots hold [A][KK][B] partials (the
// kernels' K-major layout), out is [A][B][KK] (torch's [O, I, kh, kw]), or [B][A][KK] with swap (a transposed
// convolution's weight, whose gradient is the call with g and x exchanged).  A workgroup owns one a and 64
// consecutive b: it sums the KK x 64 slot tile (reads coalesced along b, s in order), transposes it through LDS and
// adds it to out with writes coalesced along (b, tap) -- the first form wrote four scattered floats a lane, 48 us a
// 512 x 512 x 3 x 3 call.
constexpr int kOikkB = 64, kOikkMaxKK = 9;

__global__ __launch_bounds__(256) void det_sum_oikk_kernel(float* out, const float* ws, int64_t S, int64_t nel, int KK,
                                                           int B, int A, int swap, int assign) {
    __shared__ float tile[kOikkMaxKK][kOikkB + 1];
    const int a = blockIdx.y, b0 = blockIdx.x * kOikkB;
    const int nb = min(kOikkB, B - b0);
    for (int e = threadIdx.x; e < KK * kOikkB; e += 256) {
        const int t = e / kOikkB, bl = e - t * kOikkB;
        float acc = 0.f;
        if (bl < nb) {
            const float* w = ws + ((int64_t)a * KK + t) * B + b0 + bl;
            int64_t s = 0;
            for (; s + 7 < S; s += 8) {
                float v[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = w[(s + k) * nel];
#pragma unroll
                for (int k = 0; k < 8; ++k) acc += v[k];
            }
            for (; s < S; ++s) acc += w[s * nel];
        }
        tile[t][bl] = acc;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < nb * KK; e += 256) {
        const int bl = e / KK, t = e - bl * KK;
        float* o = out + (swap ? (int64_t)(b0 + bl) * A + a : (int64_t)a * B + b0 + bl) * KK + t;
        *o = assign ? tile[t][bl] : *o + tile[t][bl];
    }
}

}  // namespace

hipError_t det_sum(float* out, int64_t go, const float* ws, int64_t gw, int64_t ss, int G, int64_t S, int64_t n,
                   DetArena& arena, hipStream_t st, int assign) {
    if (G <= 0 || n <= 0 || S <= 0) return hipSuccess;
    if (G > 65535) return hipErrorInvalidValue;
    static const bool trace = getenv("SG2_DET_TRACE") != nullptr;   // diagnostics: one line per call (tools/)
    const int64_t S0 = S;
    const int64_t bx = cdiv(n, kLanes);
    if (S <= kVecS && n % 4 == 0 && go % 4 == 0 && gw % 4 == 0 && ss % 4 == 0 && (uintptr_t)out % 16 == 0 &&
        (uintptr_t)ws % 16 == 0 && bx * G >= 512) {
        if (trace) fprintf(stderr, "DETSUM G=%d n=%lld S=%lld K=%lld\n", G, (long long)n, (long long)S, 1LL);
        det_sum_vec4_kernel<<<dim3((unsigned)cdiv(n / 4, 256), (unsigned)G, 1), 256, 0, st>>>(out, go, ws, gw, ss, S,
                                                                                             n / 4, assign);
        return hipGetLastError();
    }
    // few outputs over a long sum (a bias or dot reduction over every pixel block): first chunks of the s range in
    // parallel into a temporary, then their sums in chunk order (both steps fixed by the shapes alone)
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
    det_sum_kernel<<<dim3((unsigned)bx, (unsigned)G, 1), 256, 0, st>>>(out, go, ws, gw, ss, S, n, S, 0, assign);
    return hipGetLastError();
}

hipError_t det_sum_oikk(float* out, const float* ws, int64_t S, int A, int KK, int B, int swap, hipStream_t st,
                        int assign) {
    const int64_t nel = (int64_t)A * KK * B;
    if (nel == 0 || S <= 0) return hipSuccess;
    if (KK > kOikkMaxKK || A > 65535) return hipErrorInvalidValue;
    det_sum_oikk_kernel<<<dim3((unsigned)cdiv(B, kOikkB), (unsigned)A), 256, 0, st>>>(out, ws, S, nel, KK, B, A, swap,
                                                                                                   assign);
    return hipGetLastError();
}

hipError_t det_sum_multi(const DetSumJob* jobs, int count, DetArena& arena, hipStream_t st) {
    static const bool trace = getenv("SG2_DET_TRACE") != nullptr;
    if (count <= 0) return hipSuccess;
    if (count > kMaxDetJobs) return hipErrorInvalidValue;
    DetJobs first{}, second{};
    int nb1 = 0, nb2 = 0;
    for (int q = 0; q < count; ++q) {
        const DetSumJob& in = jobs[q];
        if (in.G <= 0 || in.n <= 0 || in.S <= 0) continue;
        if (in.G > 65535) return hipErrorInvalidValue;
        const int64_t bx = cdiv(in.n, kLanes);
        int64_t K = 1;
        if (bx * in.G < 512 && in.S > 16 * kRows)
            K = std::min<int64_t>(std::min<int64_t>(cdiv(in.S, 16 * kRows), 1024), cdiv(512, bx * in.G));
        const float* ws = in.ws;
        int64_t gw = in.gw, ss = in.ss, S = in.S;
        if (K > 1) {
            const int64_t chunk = cdiv(in.S, K);
            K = cdiv(in.S, chunk);
            float* tmp = arena.get((int64_t)in.G * K * in.n);
            if (!tmp) { set_error("deterministic scratch too small (det_sum)"); return hipErrorOutOfMemory; }
            DetJob& j = first.j[first.count++];
            j = DetJob{tmp, in.ws, K * in.n, in.gw, in.ss, in.S, in.n, chunk, in.n, 1, (int)bx, in.G, (int)K, nb1};
            nb1 += (int)(bx * in.G * K);
            ws = tmp; gw = K * in.n; ss = in.n; S = K;
        }
        if (trace) fprintf(stderr, "DETSUM G=%d n=%lld S=%lld K=%lld\n", in.G, (long long)in.n, (long long)in.S,
                           (long long)K);
        DetJob& j = second.j[second.count++];
        j = DetJob{in.out, ws, in.go, gw, ss, S, in.n, S, 0, in.assign, (int)bx, in.G, 1, nb2};
        nb2 += (int)(bx * in.G);
    }
    if (first.count) det_sum_multi_kernel<<<nb1, 256, 0, st>>>(first);
    if (second.count) det_sum_multi_kernel<<<nb2, 256, 0, st>>>(second);
    return hipGetLastError();
}

}  // namespace sg2
