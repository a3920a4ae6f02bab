// ADA geometric transform of a batch in one launch (sg2_aug_geom).
//
// The reference builds each sample's 3x3 transform from its random draws with a few dozen tiny torch ops per
// augmentation call -- stack / cos / sin / where / matmul per enabled op, then the corner margins, the reflect-pad
// compensation and the up / down-sampling conjugations (SG3/training/augment_mi.py:214-318) -- about a hundred
// launches of microseconds each, four calls per step.  Here the draws stay torch draws in the reference's order
// (an RNG tape reproduces them) and one workgroup composes every sample's matrix, reduces the batch's margins
// (a max: order-independent, so the result is deterministic) and writes what the geometric stage consumes: the
// sampling theta [N, 2, 3], the reflect-pad margins, the up-sampling extents and the logical up-sampled size.
// Every transform is affine (last row 0 0 1), so a matrix is its top two rows; each composition takes the same
// f32 products and sums, in the same order, as the reference's 3x3 matmul (the zero terms aside).
#include "sg2_common.h"

#include <math.h>

namespace sg2 {
namespace {

struct Aff {   // [[a b c] [d e f] [0 0 1]]
    float a, b, c, d, e, f;
};

// G @ M
__device__ __forceinline__ Aff mul(const Aff& G, const Aff& M) {
    return Aff{G.a * M.a + G.b * M.d, G.a * M.b + G.b * M.e, G.a * M.c + G.b * M.f + G.c,
               G.d * M.a + G.e * M.d, G.d * M.b + G.e * M.e, G.d * M.c + G.e * M.f + G.f};
}
__device__ __forceinline__ Aff scale(float sx, float sy) { return Aff{sx, 0.f, 0.f, 0.f, sy, 0.f}; }
__device__ __forceinline__ Aff translate(float tx, float ty) { return Aff{1.f, 0.f, tx, 0.f, 1.f, ty}; }
__device__ __forceinline__ Aff rotate(float th) {   // rotate2d(th): [[cos, sin(-th)], [sin, cos]]
    return Aff{cosf(th), sinf(-th), 0.f, sinf(th), cosf(th), 0.f};
}

__device__ Aff compose(const sg2_aug_geom_args& a, int i, float p) {
    const float* const* D = a.draw;
    Aff G{1.f, 0.f, 0.f, 0.f, 1.f, 0.f};
    const int n = a.n;
    if (a.xflip > 0.f) {                       // scale2d_inv(1 - 2 i, 1)
        float v = floorf(D[0][i] * 2.f);
        v = D[1][i] < a.xflip * p ? v : 0.f;
        G = mul(G, scale(1.f / (1.f - 2.f * v), 1.f));
    }
    if (a.rotate90 > 0.f) {                    // rotate2d_inv(-pi/2 i) = rotate2d(pi/2 i)
        float v = floorf(D[2][i] * 4.f);
        v = D[3][i] < a.rotate90 * p ? v : 0.f;
        G = mul(G, rotate(-(-(float)M_PI / 2.f * v)));
    }
    if (a.xint > 0.f) {                        // translate2d_inv(round(tx w), round(ty h))
        const bool on = D[5][i] < a.xint * p;
        const float tx = on ? (D[4][2 * i] * 2.f - 1.f) * a.xint_max : 0.f;
        const float ty = on ? (D[4][2 * i + 1] * 2.f - 1.f) * a.xint_max : 0.f;
        G = mul(G, translate(-rintf(tx * (float)a.w), -rintf(ty * (float)a.h)));
    }
    if (a.scale > 0.f) {                       // scale2d_inv(s, s)
        float s = exp2f(D[6][i] * a.scale_std);
        s = D[7][i] < a.scale * p ? s : 1.f;
        G = mul(G, scale(1.f / s, 1.f / s));
    }
    const float p_rot = 1.f - sqrtf(fminf(fmaxf(1.f - a.rotate * p, 0.f), 1.f));
    if (a.rotate > 0.f) {                      // rotate2d_inv(-th) = rotate2d(th)
        float th = (D[8][i] * 2.f - 1.f) * (float)M_PI * a.rotate_max;
        th = D[9][i] < p_rot ? th : 0.f;
        G = mul(G, rotate(-(-th)));
    }
    if (a.aniso > 0.f) {                       // scale2d_inv(s, 1 / s)
        float s = exp2f(D[10][i] * a.aniso_std);
        s = D[11][i] < a.aniso * p ? s : 1.f;
        const float inv = 1.f / s;
        G = mul(G, scale(1.f / s, 1.f / inv));
    }
    if (a.rotate > 0.f) {
        float th = (D[12][i] * 2.f - 1.f) * (float)M_PI * a.rotate_max;
        th = D[13][i] < p_rot ? th : 0.f;
        G = mul(G, rotate(-(-th)));
    }
    if (a.xfrac > 0.f) {                       // translate2d_inv(tx w, ty h)
        const bool on = D[15][i] < a.xfrac * p;
        const float tx = on ? D[14][2 * i] * a.xfrac_std : 0.f;
        const float ty = on ? D[14][2 * i + 1] * a.xfrac_std : 0.f;
        G = mul(G, translate(-(tx * (float)a.w), -(ty * (float)a.h)));
    }
    (void)n;
    return G;
}

constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void aug_geom_kernel(sg2_aug_geom_args a, float* theta, int* margins,
                                                            int* lims, int* dyn_hw) {
    __shared__ float red[4][kThreads];
    __shared__ float fin[4];                   // mx0, my0, mx1, my1 as floats
    const int tid = threadIdx.x;
    const float p = *a.p;
    const float cx = (float)((a.w - 1) / 2.0), cy = (float)((a.h - 1) / 2.0);
    float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};   // max of -x, -y, x, y over the corners
    for (int i = tid; i < a.n; i += kThreads) {
        const Aff G = compose(a, i, p);
        float* t = theta + 6 * i;
        t[0] = G.a; t[1] = G.b; t[2] = G.c; t[3] = G.d; t[4] = G.e; t[5] = G.f;
        const float px[4] = {-cx, cx, cx, -cx}, py[4] = {-cy, -cy, cy, cy};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float x = G.a * px[k] + G.b * py[k] + G.c;
            const float y = G.d * px[k] + G.e * py[k] + G.f;
            m[0] = fmaxf(m[0], -x);
            m[1] = fmaxf(m[1], -y);
            m[2] = fmaxf(m[2], x);
            m[3] = fmaxf(m[3], y);
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) red[k][tid] = m[k];
    __syncthreads();
    for (int s = kThreads / 2; s > 0; s >>= 1) {
        if (tid < s)
#pragma unroll
            for (int k = 0; k < 4; ++k) red[k][tid] = fmaxf(red[k][tid], red[k][tid + s]);
        __syncthreads();
    }
    if (tid == 0) {
        const float lo[4] = {a.pad_x, a.pad_y, a.pad_x, a.pad_y};          // (hz_pad * 2 - cx, .. - cy)
        const float hi[4] = {(float)(a.w - 1), (float)(a.h - 1), (float)(a.w - 1), (float)(a.h - 1)};
        int mi[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float v = red[k][0] + lo[k];
            v = fminf(fmaxf(v, 0.f), hi[k]);
            mi[k] = (int)ceilf(v);
            margins[k] = mi[k];
            fin[k] = (float)mi[k];
        }
        const int hd = mi[1] + mi[3] + a.h, wd = mi[0] + mi[2] + a.w;
        const int l[8] = {hd + 32, 2 * wd + 32, 2 * hd + 32, 2 * wd + 32, 2 * hd + 96, wd + 32, hd + 32, wd + 32};
#pragma unroll
        for (int k = 0; k < 8; ++k) lims[k] = l[k];
        dyn_hw[0] = (int)((((float)a.h + fin[1]) + fin[3]) * 2.f);
        dyn_hw[1] = (int)((((float)a.w + fin[0]) + fin[2]) * 2.f);
    }
    __syncthreads();
    const float tx = (fin[0] - fin[2]) / 2.f, ty = (fin[1] - fin[3]) / 2.f;
    const float dyn_h = (((float)a.h + fin[1]) + fin[3]) * 2.f, dyn_w = (((float)a.w + fin[0]) + fin[2]) * 2.f;
    const float sx = 2.f / dyn_w, sy = 2.f / dyn_h;
    for (int i = tid; i < a.n; i += kThreads) {
        float* t = theta + 6 * i;
        float g[6] = {t[0], t[1], t[2], t[3], t[4], t[5]};
        g[2] = g[2] + tx;                                   // translate2d((mx0 - mx1) / 2, (my0 - my1) / 2) @ G
        g[5] = g[5] + ty;
        g[2] = g[2] * 2.f;                                  // scale2d(2, 2) @ G @ scale2d_inv(2, 2)
        g[5] = g[5] * 2.f;
        g[2] = g[0] * 0.5f + g[1] * 0.5f + (g[2] - 0.5f);   // translate2d(-.5, -.5) @ G @ translate2d_inv(-.5, -.5)
        g[5] = g[3] * 0.5f + g[4] * 0.5f + (g[5] - 0.5f);
        t[0] = g[0] * sx * a.inv_sx;                        // scale2d(2 / dyn_w, 2 / dyn_h) @ G @ scale2d_inv(2 / W, 2 / H)
        t[1] = g[1] * sx * a.inv_sy;
        t[2] = g[2] * sx;
        t[3] = g[3] * sy * a.inv_sx;
        t[4] = g[4] * sy * a.inv_sy;
        t[5] = g[5] * sy;
    }
}

}  // namespace
}  // namespace sg2

extern "C" int sg2_aug_geom(float* theta, int* margins, int* lims, int* dyn_hw, const sg2_aug_geom_args* args,
                            void* stream) {
    using namespace sg2;
    SG2_CHECK(theta && margins && lims && dyn_hw && args && args->p, "sg2_aug_geom: null pointer");
    const sg2_aug_geom_args& a = *args;
    SG2_CHECK(a.n > 0 && a.h > 1 && a.w > 1, "sg2_aug_geom: empty batch or image");
    const bool need[8] = {a.xflip > 0.f, a.rotate90 > 0.f, a.xint > 0.f, a.scale > 0.f,
                          a.rotate > 0.f, a.aniso > 0.f, a.rotate > 0.f, a.xfrac > 0.f};
    for (int k = 0; k < 8; ++k)
        SG2_CHECK(!need[k] || (a.draw[2 * k] && a.draw[2 * k + 1]), "sg2_aug_geom: a draw of an enabled op is null");
    aug_geom_kernel<<<1, kThreads, 0, as_stream(stream)>>>(a, theta, margins, lims, dyn_hw);
    return launch_status("sg2_aug_geom");
}
