// Bilinear grid sampling (zeros padding, align_corners = False) and its input gradient.
// Replaces aten::grid_sampler_2d / grid_sampler_2d_backward as used by
// SG3/torch_utils/ops/grid_sample_gradfix.py:28-83 inside the ADA pipe (augment_mi.py:317-318).
// The gradient w.r.t. the grid is never needed on the training path (the grid is built from
// random augmentation parameters), and the backward-of-backward is the forward itself.
//
// One lane per output pixel; the four corner weights are computed once and reused across channels.
// Backward scatters with float atomics into a float32 buffer (images are 1-3 channels, so the
// atomic traffic is ~4 x 4 B per output pixel per channel).
#include <cstdlib>

#include "sg2_common.h"

namespace sg2 {
namespace {

struct GSParams {
    const void* in;
    void* out;
    const float* grid;
    const float* theta;  // optional [N, 2, 3]: the grid is affine_grid(theta, align_corners=False), built inline
    int N, C, Hi, Wi, Ho, Wo;
    int64_t is_n, is_c, is_h, is_w;
    int64_t os_n, os_c, os_h, os_w;
    const int* dyn_hw;   // optional device [2]: logical input height / width (<= Hi, Wi of the buffer)
    int gather_wide;     // deterministic gather: scan one pixel beyond the rounded-out box (SG2_GATHER_WIDE, tests)
};

struct Corners {
    int x0, y0;
    float w00, w01, w10, w11;  // w[yy][xx]
};

// affine_grid, align_corners = False: base coordinate of pixel j at its centre, (2j + 1) / W - 1
__device__ __forceinline__ float base_coord(int j, int W) { return (float)(2 * j + 1) / (float)W - 1.f; }

__device__ __forceinline__ Corners corners_g(float gx, float gy, int Hi, int Wi);

__device__ __forceinline__ Corners corners_affine(const float* t, float bx, float by, int Hi, int Wi) {
    return corners_g(t[0] * bx + t[1] * by + t[2], t[3] * bx + t[4] * by + t[5], Hi, Wi);
}

__device__ __forceinline__ Corners corners(const GSParams& p, int n, int oy, int ox, int Hi, int Wi) {
    if (p.theta) return corners_affine(p.theta + n * 6, base_coord(ox, p.Wo), base_coord(oy, p.Ho), Hi, Wi);
    const float* g = p.grid + (((int64_t)n * p.Ho + oy) * p.Wo + ox) * 2;
    return corners_g(g[0], g[1], Hi, Wi);
}

__device__ __forceinline__ Corners corners_g(float gx, float gy, int Hi, int Wi) {
    const float ix = ((gx + 1.f) * Wi - 1.f) * 0.5f;
    const float iy = ((gy + 1.f) * Hi - 1.f) * 0.5f;
    Corners c;
    const float fx = floorf(ix), fy = floorf(iy);
    c.x0 = (int)fx;
    c.y0 = (int)fy;
    const float ax = ix - fx, ay = iy - fy;
    const float bx = (fx + 1.f) - ix, by = (fy + 1.f) - iy;
    c.w00 = bx * by;
    c.w01 = ax * by;
    c.w10 = bx * ay;
    c.w11 = ax * ay;
    return c;
}

template <typename T>
__global__ __launch_bounds__(256) void grid_sample_fwd_kernel(GSParams p) {
    const unsigned total = (unsigned)p.N * p.Ho * p.Wo;       // (host-checked < 2^31: 32-bit index math)
    const T* in = (const T*)p.in;
    T* out = (T*)p.out;
    const int Hi = p.dyn_hw ? p.dyn_hw[0] : p.Hi, Wi = p.dyn_hw ? p.dyn_hw[1] : p.Wi;
    for (unsigned idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
        const unsigned r = idx / (unsigned)p.Wo;
        const int ox = (int)(idx - r * (unsigned)p.Wo);
        const int n = (int)(r / (unsigned)p.Ho);
        const int oy = (int)(r - (unsigned)n * (unsigned)p.Ho);
        const Corners k = corners(p, n, oy, ox, Hi, Wi);
        const bool vx0 = k.x0 >= 0 && k.x0 < Wi, vx1 = k.x0 + 1 >= 0 && k.x0 + 1 < Wi;
        const bool vy0 = k.y0 >= 0 && k.y0 < Hi, vy1 = k.y0 + 1 >= 0 && k.y0 + 1 < Hi;
        for (int c = 0; c < p.C; ++c) {
            const T* b = in + n * p.is_n + c * p.is_c;
            float acc = 0.f;
            if (vy0 && vx0) acc += (float)b[k.y0 * p.is_h + k.x0 * p.is_w] * k.w00;
            if (vy0 && vx1) acc += (float)b[k.y0 * p.is_h + (k.x0 + 1) * p.is_w] * k.w01;
            if (vy1 && vx0) acc += (float)b[(k.y0 + 1) * p.is_h + k.x0 * p.is_w] * k.w10;
            if (vy1 && vx1) acc += (float)b[(k.y0 + 1) * p.is_h + (k.x0 + 1) * p.is_w] * k.w11;
            out[n * p.os_n + c * p.os_c + (int64_t)oy * p.os_h + (int64_t)ox * p.os_w] = (T)acc;
        }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void grid_sample_bwd_kernel(GSParams p) {
    const unsigned total = (unsigned)p.N * p.Ho * p.Wo;
    const T* gout = (const T*)p.in;   // gradient w.r.t. output (layout os_*)
    float* gin = (float*)p.out;       // gradient w.r.t. input  (layout is_*)
    const int Hi = p.dyn_hw ? p.dyn_hw[0] : p.Hi, Wi = p.dyn_hw ? p.dyn_hw[1] : p.Wi;
    for (unsigned idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
        const unsigned r = idx / (unsigned)p.Wo;
        const int ox = (int)(idx - r * (unsigned)p.Wo);
        const int n = (int)(r / (unsigned)p.Ho);
        const int oy = (int)(r - (unsigned)n * (unsigned)p.Ho);
        const Corners k = corners(p, n, oy, ox, Hi, Wi);
        const bool vx0 = k.x0 >= 0 && k.x0 < Wi, vx1 = k.x0 + 1 >= 0 && k.x0 + 1 < Wi;
        const bool vy0 = k.y0 >= 0 && k.y0 < Hi, vy1 = k.y0 + 1 >= 0 && k.y0 + 1 < Hi;
        for (int c = 0; c < p.C; ++c) {
            const float g = (float)gout[n * p.os_n + c * p.os_c + (int64_t)oy * p.os_h + (int64_t)ox * p.os_w];
            float* b = gin + n * p.is_n + c * p.is_c;
            if (vy0 && vx0) atomicAdd(b + k.y0 * p.is_h + k.x0 * p.is_w, g * k.w00);
            if (vy0 && vx1) atomicAdd(b + k.y0 * p.is_h + (k.x0 + 1) * p.is_w, g * k.w01);
            if (vy1 && vx0) atomicAdd(b + (k.y0 + 1) * p.is_h + k.x0 * p.is_w, g * k.w10);
            if (vy1 && vx1) atomicAdd(b + (k.y0 + 1) * p.is_h + (k.x0 + 1) * p.is_w, g * k.w11);
        }
    }
}

// Deterministic form of grid_sample_bwd_kernel for the affine grid (sg2_set_deterministic): one lane per INPUT
// pixel gathers, in a fixed order, the output pixels whose bilinear footprint covers it.  The affine map
// ix = a00 ox + a01 oy + c0, iy = a10 ox + a11 oy + c1 (input pixels per output pixel, from theta) is inverted
// per sample; the output pixels with floor(ix) in {X - 1, X} and floor(iy) in {Y - 1, Y} lie in the preimage of
// [X - 1, X + 1) x [Y - 1, Y + 1), whose bounding box (plus a 2-pixel margin for rounding) is scanned row by
// row.  Each candidate's corners are recomputed with the forward's own float arithmetic (corners()), so the
// contributions are exactly the scatter kernel's products, summed in scan order.
template <typename T>
__global__ __launch_bounds__(256) void grid_sample_bwd_gather_kernel(GSParams p) {
    const int Hi = p.dyn_hw ? p.dyn_hw[0] : p.Hi, Wi = p.dyn_hw ? p.dyn_hw[1] : p.Wi;
    const int hl = p.dyn_hw ? min(p.Hi, Hi + 96) : p.Hi, wl = p.dyn_hw ? min(p.Wi, Wi + 96) : p.Wi;
    const unsigned total = (unsigned)p.N * hl * wl;
    const T* gout = (const T*)p.in;
    float* gin = (float*)p.out;
    for (unsigned idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
        const unsigned r = idx / (unsigned)wl;
        const int X = (int)(idx - r * (unsigned)wl);
        const int n = (int)(r / (unsigned)hl);
        const int Y = (int)(r - (unsigned)n * (unsigned)hl);
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        if (X < Wi && Y < Hi) {
            float t[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) t[j] = p.theta[n * 6 + j];
            // d(ix)/d(ox) etc. and the offset, in double for the inversion only
            const double rwo = 1.0 / p.Wo, rho = 1.0 / p.Ho;
            const double a00 = (double)t[0] * Wi * rwo, a01 = (double)t[1] * Wi * rho;
            const double a10 = (double)t[3] * Hi * rwo, a11 = (double)t[4] * Hi * rho;
            // ix at (ox, oy) = ((t0 bx + t1 by + t2 + 1) Wi - 1) / 2 with bx = (2 ox + 1) / Wo - 1
            const double c0 = (((double)t[0] * (rwo - 1.0) + (double)t[1] * (rho - 1.0) + t[2] + 1.0) * Wi - 1.0) * 0.5;
            const double c1 = (((double)t[3] * (rwo - 1.0) + (double)t[4] * (rho - 1.0) + t[5] + 1.0) * Hi - 1.0) * 0.5;
            const double det = a00 * a11 - a01 * a10;
            // a (near-)singular map: scan the whole output (the bounds below clamp to it)
            double oxmin = -1e30, oxmax = 1e30, oymin = -1e30, oymax = 1e30;
            if (fabs(det) > 1e-12) {
                const double rdet = 1.0 / det;
                oxmin = 1e30; oxmax = -1e30; oymin = 1e30; oymax = -1e30;
                for (int cy = 0; cy < 2; ++cy)
                    for (int cx = 0; cx < 2; ++cx) {
                        const double u = (X - 1 + 2 * cx) - c0, v = (Y - 1 + 2 * cy) - c1;
                        const double ox = (a11 * u - a01 * v) * rdet, oy = (-a10 * u + a00 * v) * rdet;
                        oxmin = fmin(oxmin, ox); oxmax = fmax(oxmax, ox);
                        oymin = fmin(oymin, oy); oymax = fmax(oymax, oy);
                    }
            }
            // clamped in double before the int conversion (a huge or NaN bound is undefined as an int)
            auto cl = [](double v, int hi) { return v > -4.0 ? (v < hi + 4.0 ? v : hi + 4.0) : -4.0; };
            // The output pixels inside the exact preimage, widened by kGatherEps output pixels: the forward's float
            // ix / iy differ from the exact map by ~1e-4 input pixels at these sizes (|ix| < 2^11, a few roundings
            // of 2^-24), and the map's gain is >= 1/4 for any transform the pipe draws, so a pixel whose float
            // corner is (X, Y) or its up / left neighbour lies within 1e-3 output pixels of the preimage.  (The
            // first form scanned a whole pixel beyond the rounded-out box: 5 x 5 candidates per input pixel at a
            // near-identity map instead of 2-3 per axis.)
            constexpr double kGatherEps = 1.0 / 64;
            int ox0 = max(0, (int)ceil(cl(oxmin - kGatherEps, p.Wo))), ox1 = min(p.Wo - 1, (int)floor(cl(oxmax + kGatherEps, p.Wo)));
            int oy0 = max(0, (int)ceil(cl(oymin - kGatherEps, p.Ho))), oy1 = min(p.Ho - 1, (int)floor(cl(oymax + kGatherEps, p.Ho)));
            if (p.gather_wide) {
                ox0 = max(0, (int)floor(cl(oxmin, p.Wo)) - 1); ox1 = min(p.Wo - 1, (int)ceil(cl(oxmax, p.Wo)) + 1);
                oy0 = max(0, (int)floor(cl(oymin, p.Ho)) - 1); oy1 = min(p.Ho - 1, (int)ceil(cl(oymax, p.Ho)) + 1);
            }
            for (int oy = oy0; oy <= oy1; ++oy) {
                const float by = base_coord(oy, p.Ho);
                for (int ox = ox0; ox <= ox1; ++ox) {
                    const Corners k = corners_affine(t, base_coord(ox, p.Wo), by, Hi, Wi);
                    const int dx = X - k.x0, dy = Y - k.y0;           // 0 or 1 when (X, Y) is a corner
                    if ((unsigned)dx > 1u || (unsigned)dy > 1u) continue;
                    const float w = dy ? (dx ? k.w11 : k.w10) : (dx ? k.w01 : k.w00);
                    for (int c = 0; c < p.C && c < 4; ++c)
                        acc[c] += (float)gout[n * p.os_n + c * p.os_c + (int64_t)oy * p.os_h + (int64_t)ox * p.os_w] * w;
                }
            }
        }
        for (int c = 0; c < p.C && c < 4; ++c) gin[n * p.is_n + c * p.is_c + (int64_t)Y * p.is_h + (int64_t)X * p.is_w] = acc[c];
    }
}

// Reflect padding with margins held in device memory (so the ADA pipe needs no host sync): the
// padded image of logical size (H + my0 + my1) x (W + mx0 + mx1) is written at the origin of a static
// [N, C, Hs, Ws] buffer, zeros elsewhere (exactly what upfirdn2d's implicit zero padding sees).
// Margins never exceed the image size minus one (augment_mi.py:295-296), so one reflection suffices.
__device__ __forceinline__ int reflect1(int k, int L) { return k < 0 ? -k : (k >= L ? 2 * (L - 1) - k : k); }

__global__ __launch_bounds__(256) void reflect_pad_kernel(float* y, const float* x, const int* m, int N, int C, int H,
                                                          int W, int Hs, int Ws) {
    // the grid strides over the region a consumer reads only (the padded image plus 64 rows / columns of zeros,
    // upfirdn2d.hip UpfParams::lim), with 32-bit index math (the host checks N C Hs Ws < 2^31)
    const int mx0 = m[0], my0 = m[1], mx1 = m[2], my1 = m[3];
    const int Hd = H + my0 + my1, Wd = W + mx0 + mx1;
    const int hl = min(Hs, Hd + 64), wl = min(Ws, Wd + 64);
    const unsigned total = (unsigned)N * C * hl * wl;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const unsigned r = i / (unsigned)wl;
        const int px = (int)(i - r * (unsigned)wl);
        const unsigned nc = r / (unsigned)hl;
        const int py = (int)(r - nc * (unsigned)hl);
        float v = 0.f;
        if (py < Hd && px < Wd) v = x[((int64_t)nc * H + reflect1(py - my0, H)) * W + reflect1(px - mx0, W)];
        y[((int64_t)nc * Hs + py) * Ws + px] = v;
    }
}

// Adjoint of reflect_pad_kernel: every source pixel gathers the (up to 3 x 3) padded positions that
// reflect onto it.
__global__ __launch_bounds__(256) void reflect_pad_adj_kernel(float* gx, const float* gy, const int* m, int N, int C,
                                                              int H, int W, int Hs, int Ws) {
    const int mx0 = m[0], my0 = m[1], mx1 = m[2], my1 = m[3];
    const int64_t total = (int64_t)N * C * H * W;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int ix = (int)(i % W);
        const int iy = (int)((i / W) % H);
        const int64_t nc = i / ((int64_t)W * H);
        int ys[3], xs[3], ny = 0, nx = 0;
        ys[ny++] = my0 + iy;
        if (iy >= 1 && iy <= my0) ys[ny++] = my0 - iy;
        if (iy <= H - 2 && iy >= H - 1 - my1) ys[ny++] = my0 + 2 * (H - 1) - iy;
        xs[nx++] = mx0 + ix;
        if (ix >= 1 && ix <= mx0) xs[nx++] = mx0 - ix;
        if (ix <= W - 2 && ix >= W - 1 - mx1) xs[nx++] = mx0 + 2 * (W - 1) - ix;
        const float* b = gy + nc * Hs * Ws;
        float acc = 0.f;
        for (int a = 0; a < ny; ++a)
            for (int c = 0; c < nx; ++c) acc += b[(int64_t)ys[a] * Ws + xs[c]];
        gx[i] = acc;
    }
}

// Zero rows < dyn_h + band and cols < dyn_w + band of the [N, C, Hi, Wi] gradient buffer (strides is_*): the grid
// strides over the region only (32-bit index math; the region of the static buffer is < 2^31 elements).
__global__ __launch_bounds__(256) void zero_region_kernel(float* g, GSParams p, const int* dyn_hw, int band) {
    const int hl = min(p.Hi, dyn_hw[0] + band), wl = min(p.Wi, dyn_hw[1] + band);
    const unsigned total = (unsigned)p.N * p.C * hl * wl;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const unsigned r = i / (unsigned)wl;
        const int x = (int)(i - r * (unsigned)wl);
        const unsigned nc = r / (unsigned)hl;
        const int y = (int)(r - nc * (unsigned)hl);
        const int c = (int)(nc % (unsigned)p.C), n = (int)(nc / (unsigned)p.C);
        g[n * p.is_n + c * p.is_c + (int64_t)y * p.is_h + (int64_t)x * p.is_w] = 0.f;
    }
}

int fill(GSParams& p, const int64_t* in_size, const int64_t* in_stride, const int64_t* out_size,
         const int64_t* out_stride) {
    SG2_CHECK(in_size && in_stride && out_size && out_stride, "sg2_grid_sample: null size/stride");
    p.N = (int)in_size[0]; p.C = (int)in_size[1]; p.Hi = (int)in_size[2]; p.Wi = (int)in_size[3];
    SG2_CHECK(out_size[0] == p.N && out_size[1] == p.C, "sg2_grid_sample: batch/channel mismatch");
    p.Ho = (int)out_size[2]; p.Wo = (int)out_size[3];
    p.is_n = in_stride[0]; p.is_c = in_stride[1]; p.is_h = in_stride[2]; p.is_w = in_stride[3];
    p.os_n = out_stride[0]; p.os_c = out_stride[1]; p.os_h = out_stride[2]; p.os_w = out_stride[3];
    return 0;
}

}  // namespace
}  // namespace sg2

namespace sg2 {
namespace {
int gs_fwd(void* out, const void* in, const float* grid, const float* theta, int dtype, const int64_t* in_size,
           const int64_t* in_stride, const int64_t* out_size, const int64_t* out_stride, const int* dyn_hw,
           void* stream) {
    SG2_CHECK(out && in && (grid || theta), "sg2_grid_sample_fwd: null pointer");
    GSParams p;
    p.in = in; p.out = out; p.grid = grid; p.theta = theta; p.dyn_hw = dyn_hw;
    if (fill(p, in_size, in_stride, out_size, out_stride)) return -1;
    const int64_t total = (int64_t)p.N * p.Ho * p.Wo;
    if (total == 0 || p.C == 0) return 0;
    SG2_CHECK(total < INT32_MAX && (int64_t)p.N * p.Hi * p.Wi < INT32_MAX, "sg2_grid_sample_fwd: too many pixels");
    const int g = (int)std::min<int64_t>(cdiv(total, 256), 256 * 32);
    SG2_DISPATCH(dtype, T, { grid_sample_fwd_kernel<T><<<g, 256, 0, as_stream(stream)>>>(p); });
    return launch_status("sg2_grid_sample_fwd");
}

int gs_bwd(float* gin, const void* gout, const float* grid, const float* theta, int dtype, const int64_t* in_size,
           const int64_t* in_stride, const int64_t* out_size, const int64_t* out_stride, const int* dyn_hw,
           void* stream) {
    SG2_CHECK(gin && gout && (grid || theta), "sg2_grid_sample_bwd: null pointer");
    GSParams p;
    p.in = gout; p.out = gin; p.grid = grid; p.theta = theta; p.dyn_hw = dyn_hw;
    { const char* e = getenv("SG2_GATHER_WIDE"); p.gather_wide = e ? atoi(e) : 0; }
    if (fill(p, in_size, in_stride, out_size, out_stride)) return -1;
    // zero the float32 input-gradient buffer (dense over the strided extent)
    const int64_t extent = (p.N - 1) * p.is_n + (p.C - 1) * p.is_c + (p.Hi - 1) * p.is_h + (p.Wi - 1) * p.is_w + 1;
    hipStream_t s = as_stream(stream);
    const bool gather = det_on() && theta;
    if (dyn_hw && gather) {
        // the deterministic gather writes every element of the region below (its band included): no zeroing
        SG2_CHECK(p.C <= 4, "sg2_affine_grid_sample_bwd: deterministic mode supports C <= 4");
    } else if (dyn_hw) {
        // only the region a consumer of the dynamically sized gradient reads: the logical image plus a
        // band (upfirdn2d.hip kZeroBand and the adjoint FIR's reach)
        SG2_CHECK((int64_t)p.N * p.C * p.Hi * p.Wi < INT32_MAX, "sg2_grid_sample_bwd: gradient buffer too large");
        const int64_t tot = (int64_t)p.N * p.C * p.Hi * p.Wi;
        const int g = (int)std::min<int64_t>(cdiv(tot, 256), 256 * 64);
        zero_region_kernel<<<g, 256, 0, s>>>(gin, p, dyn_hw, 96);
        int rc = launch_status("sg2_grid_sample_bwd zero");
        if (rc) return rc;
    } else {
        hipError_t e = zero_fill(gin, extent * sizeof(float), s);
        if (e != hipSuccess) { set_error("sg2_grid_sample_bwd: memset failed"); return (int)e; }
    }
    const int64_t total = (int64_t)p.N * p.Ho * p.Wo;
    if (total == 0 || p.C == 0) return 0;
    SG2_CHECK(total < INT32_MAX && (int64_t)p.N * p.Hi * p.Wi < INT32_MAX, "sg2_grid_sample_bwd: too many pixels");
    if (gather) {
        SG2_CHECK(p.C <= 4, "sg2_affine_grid_sample_bwd: deterministic mode supports C <= 4");
        const int64_t tot_in = (int64_t)p.N * p.Hi * p.Wi;
        static const int gmax = [] { const char* e = getenv("SG2_GATHER_GRID"); return e ? atoi(e) : 256 * 64; }();
        const int gi = (int)std::min<int64_t>(cdiv(tot_in, 256), gmax);
        SG2_DISPATCH(dtype, T, { grid_sample_bwd_gather_kernel<T><<<gi, 256, 0, s>>>(p); });
        return launch_status("sg2_affine_grid_sample_bwd (deterministic gather)");
    }
    const int g = (int)std::min<int64_t>(cdiv(total, 256), 256 * 32);
    SG2_DISPATCH(dtype, T, { grid_sample_bwd_kernel<T><<<g, 256, 0, s>>>(p); });
    return launch_status("sg2_grid_sample_bwd");
}
}  // namespace
}  // namespace sg2

extern "C" int sg2_grid_sample_fwd(void* out, const void* in, const float* grid, int dtype, const int64_t* in_size,
                                   const int64_t* in_stride, const int64_t* out_size, const int64_t* out_stride,
                                   const int* dyn_hw, void* stream) {
    return sg2::gs_fwd(out, in, grid, nullptr, dtype, in_size, in_stride, out_size, out_stride, dyn_hw, stream);
}

extern "C" int sg2_grid_sample_bwd(float* gin, const void* gout, const float* grid, int dtype, const int64_t* in_size,
                                   const int64_t* in_stride, const int64_t* out_size, const int64_t* out_stride,
                                   const int* dyn_hw, void* stream) {
    return sg2::gs_bwd(gin, gout, grid, nullptr, dtype, in_size, in_stride, out_size, out_stride, dyn_hw, stream);
}

extern "C" int sg2_affine_grid_sample_fwd(void* out, const void* in, const float* theta, int dtype,
                                          const int64_t* in_size, const int64_t* in_stride, const int64_t* out_size,
                                          const int64_t* out_stride, const int* dyn_hw, void* stream) {
    return sg2::gs_fwd(out, in, nullptr, theta, dtype, in_size, in_stride, out_size, out_stride, dyn_hw, stream);
}

extern "C" int sg2_affine_grid_sample_bwd(float* gin, const void* gout, const float* theta, int dtype,
                                          const int64_t* in_size, const int64_t* in_stride, const int64_t* out_size,
                                          const int64_t* out_stride, const int* dyn_hw, void* stream) {
    return sg2::gs_bwd(gin, gout, nullptr, theta, dtype, in_size, in_stride, out_size, out_stride, dyn_hw, stream);
}

extern "C" int sg2_reflect_pad_dyn(float* y, const float* x, const int* margins, int N, int C, int H, int W, int Hs,
                                   int Ws, int adjoint, void* stream) {
    using namespace sg2;
    SG2_CHECK(y && x && margins, "sg2_reflect_pad_dyn: null pointer");
    SG2_CHECK(N >= 0 && C >= 0 && H > 0 && W > 0 && Hs >= 3 * H - 2 && Ws >= 3 * W - 2,
              "sg2_reflect_pad_dyn: the static buffer must hold the largest padded image (3H-2 x 3W-2)");
    const int64_t total = adjoint ? (int64_t)N * C * H * W : (int64_t)N * C * Hs * Ws;
    if (total == 0) return 0;
    SG2_CHECK(adjoint || total < INT32_MAX, "sg2_reflect_pad_dyn: static buffer too large");
    static const int gmax = [] { const char* e = getenv("SG2_PAD_GRID"); return e ? atoi(e) : 256 * 64; }();
    const int g = (int)std::min<int64_t>(cdiv(total, 256), gmax);
    if (adjoint) reflect_pad_adj_kernel<<<g, 256, 0, as_stream(stream)>>>(y, x, margins, N, C, H, W, Hs, Ws);
    else reflect_pad_kernel<<<g, 256, 0, as_stream(stream)>>>(y, x, margins, N, C, H, W, Hs, Ws);
    return launch_status("sg2_reflect_pad_dyn");
}
