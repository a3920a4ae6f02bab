// Fused bias + activation (+ gain, clamp) and its first/second-order gradients.
// Semantics: SG3/torch_utils/ops/bias_act.py:21-207 and the plugin contract bias_act.cpp:32-90.
// HBM-bound elementwise kernel: one 16-byte vector (4 f32 / 8 f16|bf16) per lane per step,
// grid-stride over the flat tensor; bias index = (i / step_b) % size_b.
#include "sg2_common.h"

namespace sg2 {
namespace {

constexpr float kSeluScale = 1.0507009873554804934193349852946f;
constexpr float kSeluAlpha = 1.6732632423543772848170429916717f;

template <int ACT>
__device__ __forceinline__ float act_fwd(float v, float alpha) {
    if (ACT == 1) return v;
    if (ACT == 2) return v > 0.f ? v : 0.f;
    if (ACT == 3) return v > 0.f ? v : v * alpha;
    if (ACT == 4) return tanhf(v);
    if (ACT == 5) return 1.f / (1.f + __expf(-v));
    if (ACT == 6) return v >= 0.f ? v : __expf(v) - 1.f;
    if (ACT == 7) return v >= 0.f ? kSeluScale * v : (kSeluScale * kSeluAlpha) * (__expf(v) - 1.f);
    if (ACT == 8) return v > 20.f ? v : log1pf(__expf(v));
    if (ACT == 9) return v / (1.f + __expf(-v));
    return v;
}

// d act / d x expressed through yy = y / gain (or through xs = x + b for swish), times g.
template <int ACT>
__device__ __forceinline__ float act_d1(float g, float yy, float xs, float alpha) {
    if (ACT == 1) return g;
    if (ACT == 2) return yy > 0.f ? g : 0.f;
    if (ACT == 3) return yy > 0.f ? g : g * alpha;
    if (ACT == 4) return g * (1.f - yy * yy);
    if (ACT == 5) return g * yy * (1.f - yy);
    if (ACT == 6) return yy >= 0.f ? g : g * (yy + 1.f);
    if (ACT == 7) return yy >= 0.f ? g * kSeluScale : g * (yy + kSeluScale * kSeluAlpha);
    if (ACT == 8) return g * (1.f - __expf(-yy));
    if (ACT == 9) {
        if (xs > 40.f) return g;
        float e = __expf(xs), d = e + 1.f;
        return g * e * (xs + d) / (d * d);
    }
    return g;
}

// second derivative term, times g.
template <int ACT>
__device__ __forceinline__ float act_d2(float g, float yy, float xs) {
    if (ACT == 4) return g * (1.f - yy * yy) * (-2.f * yy);
    if (ACT == 5) return g * yy * (1.f - yy) * (1.f - 2.f * yy);
    if (ACT == 6) return yy >= 0.f ? 0.f : g * (yy + 1.f);
    if (ACT == 7) return yy >= 0.f ? 0.f : g * (yy + kSeluScale * kSeluAlpha);
    if (ACT == 8) { float e = __expf(-yy); return g * e * (1.f - e); }
    if (ACT == 9) {
        if (xs > 40.f) return 0.f;
        float e = __expf(xs), d = e + 1.f;
        return g * e * (xs * (2.f - d) + 2.f * d) / (d * d * d);
    }
    return 0.f;
}

template <typename T> struct Vec;
template <> struct Vec<float> { static constexpr int N = 4; };
template <> struct Vec<f16_t> { static constexpr int N = 8; };
template <> struct Vec<bf16_t> { static constexpr int N = 8; };

struct BAParams {
    void* y;
    const void* x;
    const void* b;
    const void* xref;
    const void* yref;
    const void* dy;
    uint32_t numel, size_b, step_b;
    float alpha, gain, clamp;
};

template <typename T, int ACT, int GRAD>
__global__ __launch_bounds__(256) void bias_act_kernel(BAParams p) {
    constexpr int V = Vec<T>::N;
    typedef T vecT __attribute__((ext_vector_type(V)));
    const T* x = (const T*)p.x;
    const T* b = (const T*)p.b;
    const T* xr = (const T*)p.xref;
    const T* yr = (const T*)p.yref;
    const T* dyp = (const T*)p.dy;
    T* y = (T*)p.y;
    const float inv_gain = p.gain != 0.f ? 1.f / p.gain : 0.f;
    const uint32_t nvec = p.numel / V;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < nvec + (p.numel % V ? 1 : 0); v += stride) {
        const uint32_t base = v * V;
        const bool full = base + V <= p.numel;
        float xv[V], xrv[V], yrv[V], dyv[V], bv[V];
        if (full) {
            vecT t = *(const vecT*)(x + base);
#pragma unroll
            for (int j = 0; j < V; ++j) xv[j] = (float)t[j];
            if (xr) { t = *(const vecT*)(xr + base);
#pragma unroll
                for (int j = 0; j < V; ++j) xrv[j] = (float)t[j]; }
            if (yr) { t = *(const vecT*)(yr + base);
#pragma unroll
                for (int j = 0; j < V; ++j) yrv[j] = (float)t[j]; }
            if (dyp) { t = *(const vecT*)(dyp + base);
#pragma unroll
                for (int j = 0; j < V; ++j) dyv[j] = (float)t[j]; }
        } else {
#pragma unroll
            for (int j = 0; j < V; ++j) {
                uint32_t i = base + j < p.numel ? base + j : p.numel - 1;
                xv[j] = (float)x[i];
                if (xr) xrv[j] = (float)xr[i];
                if (yr) yrv[j] = (float)yr[i];
                if (dyp) dyv[j] = (float)dyp[i];
            }
        }
#pragma unroll
        for (int j = 0; j < V; ++j) {
            if (!xr) xrv[j] = 0.f;
            if (!yr) yrv[j] = 0.f;
            if (!dyp) dyv[j] = 1.f;
            bv[j] = b ? (float)b[((base + j) / p.step_b) % p.size_b] : 0.f;
        }
        T out[V];
#pragma unroll
        for (int j = 0; j < V; ++j) {
            float r;
            if (GRAD == 0) {
                r = act_fwd<ACT>(xv[j] + bv[j], p.alpha) * p.gain;
                if (p.clamp >= 0.f) r = fminf(fmaxf(r, -p.clamp), p.clamp);
            } else {
                const float xs = xrv[j] + bv[j];
                float yref = yrv[j];
                if (ACT == 9) yref = act_fwd<9>(xs, 0.f) * p.gain;
                const float yy = yref * inv_gain;
                r = (GRAD == 1 ? act_d1<ACT>(xv[j], yy, xs, p.alpha) : act_d2<ACT>(xv[j], yy, xs)) * p.gain * dyv[j];
                if (p.clamp >= 0.f && !(yref > -p.clamp && yref < p.clamp)) r = 0.f;
            }
            out[j] = (T)r;
        }
        if (full) {
            vecT t;
#pragma unroll
            for (int j = 0; j < V; ++j) t[j] = out[j];
            *(vecT*)(y + base) = t;
        } else {
            for (int j = 0; j < V; ++j)
                if (base + j < p.numel) y[base + j] = out[j];
        }
    }
}

template <typename T, int GRAD>
int launch_grad(const BAParams& p, int act, hipStream_t s) {
    constexpr int V = Vec<T>::N;
    const int64_t nvec = cdiv(p.numel, V);
    const int grid = (int)std::min<int64_t>(cdiv(nvec, 256), 256 * 16);
    switch (act) {
#define CASE(A) case A: bias_act_kernel<T, A, GRAD><<<grid, 256, 0, s>>>(p); break;
        CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(9)
#undef CASE
        default: set_error("sg2_bias_act: unknown activation id"); return -1;
    }
    return launch_status("sg2_bias_act");
}

}  // namespace
}  // namespace sg2

extern "C" int sg2_bias_act(void* y, const void* x, const void* b, const void* xref, const void* yref, const void* dy,
                            int dtype, int64_t numel, int64_t size_b, int64_t step_b, int grad, int act,
                            float alpha, float gain, float clamp, void* stream) {
    using namespace sg2;
    SG2_CHECK(y != nullptr && x != nullptr, "sg2_bias_act: x and y must be non-null");
    SG2_CHECK(numel >= 0 && numel <= INT32_MAX, "sg2_bias_act: x is too large");
    SG2_CHECK(grad >= 0 && grad <= 2, "sg2_bias_act: grad must be 0, 1 or 2");
    SG2_CHECK(b == nullptr || (size_b > 0 && step_b > 0), "sg2_bias_act: bad bias geometry");
    SG2_CHECK(act >= 1 && act <= 9, "sg2_bias_act: unknown activation id");
    if (numel == 0) return 0;
    BAParams p{y, x, b, xref, yref, dy, (uint32_t)numel, (uint32_t)(b ? size_b : 1), (uint32_t)(b ? step_b : 1),
               alpha, gain, clamp};
    hipStream_t s = as_stream(stream);
    SG2_DISPATCH(dtype, T, {
        if (grad == 0) return launch_grad<T, 0>(p, act, s);
        if (grad == 1) return launch_grad<T, 1>(p, act, s);
        return launch_grad<T, 2>(p, act, s);
    });
    return 0;
}
