// upfirdn2d: zero-insertion upsample -> pad/crop -> 2-D FIR -> decimate.
// Semantics: SG3/torch_utils/ops/upfirdn2d.py:118-211 (plugin contract upfirdn2d.cpp:16-98).
//
// Output sample o (per axis) reads upsampled-padded positions u = o*down - pad0 + t, t in [0, f);
// only u divisible by `up` carry input samples x[u/up], so per output row the valid taps are
// t = t0 + k*up with t0 = (-(o*down - pad0)) mod up.  Filter taps are staged once per workgroup in
// LDS; the weight of tap t is f[f-1-t] (convolution) or f[t] (flip = correlation).
//
// Two kernels:
//  * upfirdn_nhwc_vec: channels-last activations with C % V == 0 (the network's feature maps);
//    each lane owns one 16-byte channel vector of one output pixel, so every tap read is a
//    coalesced 16-byte load and neighbouring taps hit L1/L2.  Its specialisations: upfirdn_nhwc_f4 /
//    upfirdn_nhwc_f4s (4x4, up 1: LDS-staged tiles, column strips) and upfirdn_nhwc_up2 (4x4, up 2, down 1:
//    a 2 x 2 output cell per lane from one 3 x 3 input neighbourhood).
//  * upfirdn_generic : any 4-D strides (images, NCHW tensors, odd channel counts).
#include <cstdlib>

#include "sg2_common.h"

namespace sg2 {
namespace {

constexpr int kMaxTaps = 1024;

struct UpfParams {
    const void* x;
    void* y;
    const float* f;
    int N, C, H, W;           // input
    int OH, OW;               // output
    int64_t xs_n, xs_c, xs_h, xs_w;
    int64_t ys_n, ys_c, ys_h, ys_w;
    int fw, fh;
    int upx, upy, downx, downy, padx0, pady0;
    int flip;
    float gain;
    // fused layer epilogue (nhwc_vec kernel only; include/sg2hip.h sg2_epilogue)
    const float* out_scale;   // [N, C]
    const void* noise;        // [N, OH, OW]
    const float* bias;        // [C]
    const void* residual;     // like y
    void* aux;                // like y
    float noise_gain, alpha, egain, clamp;
    int act, aux_mode, epi;
    // optional device int[2] output extent (rows, cols) of a dynamically sized image in a static buffer
    // (the ADA pipe): outputs below it are computed, outputs in the kZeroBand rows/cols beyond it are
    // written as zeros (their exact value: the image's support ends inside the extent), the rest of the
    // static buffer is left untouched -- no consumer reads it.  Generic kernel only.
    const int* lim;
    int xcd;                  // f4 kernel: XCD-contiguous block order (default on)
};

constexpr int kZeroBand = 32;

__device__ __forceinline__ int floordiv(int a, int b) { return (a >= 0) ? a / b : -((-a + b - 1) / b); }

// Tap geometry along one axis for output coordinate o.
__device__ __forceinline__ void axis_taps(int o, int down, int pad0, int up, int& t0, int& i0) {
    const int z = o * down - pad0;
    int r = (-z) % up;
    if (r < 0) r += up;
    t0 = r;
    i0 = floordiv(z + r, up);
}

__device__ __forceinline__ void stage_filter(float* sf, const UpfParams& p) {
    const int n = p.fw * p.fh;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        // store in "tap order": sf[ty*fw+tx] = weight applied to tap (ty, tx)
        const int ty = i / p.fw, tx = i % p.fw;
        const int sy = p.flip ? ty : p.fh - 1 - ty;
        const int sx = p.flip ? tx : p.fw - 1 - tx;
        sf[i] = p.f[sy * p.fw + sx] * p.gain;
    }
    __syncthreads();
}

template <typename T>
__global__ __launch_bounds__(256) void upfirdn_generic(UpfParams p) {
    __shared__ float sf[kMaxTaps];
    stage_filter(sf, p);
    const T* x = (const T*)p.x;
    T* y = (T*)p.y;
    const int64_t total = (int64_t)p.N * p.C * p.OH * p.OW;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        int64_t r = idx;
        const int ox = (int)(r % p.OW); r /= p.OW;
        const int oy = (int)(r % p.OH); r /= p.OH;
        const int c = (int)(r % p.C); r /= p.C;
        const int n = (int)r;
        if (p.lim) {
            const int ly = p.lim[0], lx = p.lim[1];
            if (oy >= ly + kZeroBand || ox >= lx + kZeroBand) continue;
            if (oy >= ly || ox >= lx) {
                y[n * p.ys_n + c * p.ys_c + (int64_t)oy * p.ys_h + (int64_t)ox * p.ys_w] = (T)0.f;
                continue;
            }
        }
        int ty0, iy0, tx0, ix0;
        axis_taps(oy, p.downy, p.pady0, p.upy, ty0, iy0);
        axis_taps(ox, p.downx, p.padx0, p.upx, tx0, ix0);
        const T* xb = x + n * p.xs_n + c * p.xs_c;
        float acc = 0.f;
        for (int ty = ty0, iy = iy0; ty < p.fh; ty += p.upy, ++iy) {
            if (iy < 0 || iy >= p.H) continue;
            const T* xr = xb + iy * p.xs_h;
            for (int tx = tx0, ix = ix0; tx < p.fw; tx += p.upx, ++ix) {
                if (ix < 0 || ix >= p.W) continue;
                acc += (float)xr[ix * p.xs_w] * sf[ty * p.fw + tx];
            }
        }
        y[n * p.ys_n + c * p.ys_c + (int64_t)oy * p.ys_h + (int64_t)ox * p.ys_w] = (T)acc;
    }
}

// Tap geometry along one axis with the up / down factors known at compile time (0: runtime, axis_taps).
template <int UP, int DOWN>
__device__ __forceinline__ void axis_taps_c(int o, int down, int pad0, int up, int& t0, int& i0) {
    if (UP == 1 && DOWN != 0) { t0 = 0; i0 = o * DOWN - pad0; }
    else if (UP == 2 && DOWN != 0) { const int z = o * DOWN - pad0; t0 = z & 1; i0 = (z + t0) >> 1; }
    else axis_taps(o, down, pad0, up, t0, i0);
}

// One separable pass (filter along x only, or along y only; the other axis is the identity): the two
// launches of every 1-D-filter upfirdn2d (upfirdn2d.py:190-193), e.g. the ADA pipe's 12-tap sym6
// up/down-sampling of single-channel images.  The grid strides over (output row, 256-column tile) pairs
// inside the computed extent (with a device-side lim the skipped part of the static buffer costs no
// workgroups); the pair index is uniform, its decode 32-bit scalar math.  UP / DOWN: the pass's factors when
// known at compile time (the ADA pipe's up-2 and down-2 passes), which turns the per-lane tap geometry into
// shifts.  Reads are coalesced along x and the horizontal pass's neighbouring taps hit L1.
template <typename T, bool HORIZ, int KT, int UP, int DOWN>
__global__ __launch_bounds__(256) void upfirdn_1d(UpfParams p) {
    // KT: taps per output (ceil(F / up)), unrolled so all of a lane's loads are in flight together.
    __shared__ float sf[64];
    const int F = HORIZ ? p.fw : p.fh;
    for (int t = threadIdx.x; t < F; t += 256) sf[t] = p.f[p.flip ? t : F - 1 - t] * p.gain;
    __syncthreads();
    const int ly = p.lim ? p.lim[0] : p.OH, lx = p.lim ? p.lim[1] : p.OW;      // computed extent
    const int rows = min(p.OH, ly + (p.lim ? kZeroBand : 0)), cols = min(p.OW, lx + (p.lim ? kZeroBand : 0));
    const int tiles = (cols + 255) / 256;
    const int total = p.N * p.C * rows * tiles;
    const int up = HORIZ ? p.upx : p.upy, down = HORIZ ? p.downx : p.downy, L = HORIZ ? p.W : p.H;
    for (int b = blockIdx.x; b < total; b += gridDim.x) {
        const int row = b / tiles;
        const int ox = (b - row * tiles) * 256 + threadIdx.x;
        const int oy = row % rows, nc = row / rows;
        if (ox >= cols) continue;
        const int c = nc % p.C, n = nc / p.C;
        T* yp = (T*)p.y + n * p.ys_n + c * p.ys_c + (int64_t)oy * p.ys_h + (int64_t)ox * p.ys_w;
        if (oy >= ly || ox >= lx) { *yp = (T)0.f; continue; }
        const T* xb = (const T*)p.x + n * p.xs_n + c * p.xs_c;
        int t0, i0;
        if (HORIZ) axis_taps_c<UP, DOWN>(ox, down, p.padx0, up, t0, i0);
        else axis_taps_c<UP, DOWN>(oy, down, p.pady0, up, t0, i0);
        const T* xl = HORIZ ? xb + (int64_t)oy * p.xs_h : xb + (int64_t)ox * p.xs_w;
        const int64_t st = HORIZ ? p.xs_w : p.xs_h;
        const int upk = UP ? UP : up;
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < KT; ++k) {
            const int t = t0 + k * upk, i = i0 + k;
            const bool ok = t < F && i >= 0 && i < L;
            const float v = (float)xl[(int64_t)(ok ? i : 0) * st];
            acc += ok ? v * sf[t < F ? t : 0] : 0.f;
        }
        *yp = (T)acc;
    }
}

// The horizontal pass with UP, DOWN in {1, 2}: a workgroup stages the input span of its 256 outputs of one row
// (256 * DOWN / UP + KT values) in LDS with coalesced loads, then each lane reads its KT taps from LDS (the
// global form issues KT strided loads per output: at DOWN = 2 each wave load spans twice the cache lines).
template <typename T, int UP, int DOWN, int KT, int TWD = 256>
__global__ __launch_bounds__(256) void upfirdn_1d_hlds(UpfParams p) {
    // TWD: outputs per row segment; a workgroup takes 256 / TWD consecutive rows of one (n, c) plane (narrow
    // outputs, e.g. the 313-wide down-2 pass, idle fewer lanes in 128-wide segments)
    constexpr int ROWS = 256 / TWD;
    constexpr int SPAN = ((TWD - 1) * DOWN + UP - 1) / UP + KT + 1;
    __shared__ float sf[64];
    __shared__ float sx[ROWS][SPAN];
    const int F = p.fw;
    for (int t = threadIdx.x; t < KT * UP; t += 256) sf[t] = t < F ? p.f[p.flip ? t : F - 1 - t] * p.gain : 0.f;
    __syncthreads();
    float fr[KT * UP];                                 // the taps in registers, zero past the filter
#pragma unroll
    for (int t = 0; t < KT * UP; ++t) fr[t] = t < F ? sf[t] : 0.f;
    const int ly = p.lim ? p.lim[0] : p.OH, lx = p.lim ? p.lim[1] : p.OW;      // computed extent
    const int rows = min(p.OH, ly + (p.lim ? kZeroBand : 0)), cols = min(p.OW, lx + (p.lim ? kZeroBand : 0));
    const int tiles = (cols + TWD - 1) / TWD, rgroups = (rows + ROWS - 1) / ROWS;
    const int total = p.N * p.C * rgroups * tiles;
    const int rr = threadIdx.x / TWD, col = threadIdx.x % TWD;
    for (int b = blockIdx.x; b < total; b += gridDim.x) {
        const int rg = b / tiles;
        const int ox0 = (b - rg * tiles) * TWD, ox = ox0 + col;
        const int oy0 = (rg % rgroups) * ROWS, nc = rg / rgroups;
        const int c = nc % p.C, n = nc / p.C;
        int tb, base;
        axis_taps_c<UP, DOWN>(ox0, DOWN, p.padx0, UP, tb, base);                 // the span's first input
        const T* xp = (const T*)p.x + n * p.xs_n + c * p.xs_c;
        __syncthreads();                                                        // (the previous pair's reads)
        for (int e = threadIdx.x; e < ROWS * SPAN; e += 256) {
            const int r = e / SPAN, m = e - r * SPAN;
            const int i = base + m, y = oy0 + r;
            sx[r][m] = (i >= 0 && i < p.W && y < rows) ? (float)xp[(int64_t)y * p.xs_h + (int64_t)i * p.xs_w] : 0.f;
        }
        __syncthreads();
        const int oy = oy0 + rr;
        if (ox >= cols || oy >= rows) continue;
        T* yp = (T*)p.y + n * p.ys_n + c * p.ys_c + (int64_t)oy * p.ys_h + (int64_t)ox * p.ys_w;
        if (oy >= ly || ox >= lx) { *yp = (T)0.f; continue; }
        int t0, i0;
        axis_taps_c<UP, DOWN>(ox, DOWN, p.padx0, UP, t0, i0);
        const float* w = &sx[rr][i0 - base];
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < KT; ++k)      // tap t0 + k UP: registers at UP = 1; at UP = 2 (t0 alternates between
            acc += w[k] * (UP == 1 ? fr[k] : sf[t0 + k * UP]);   // lanes) LDS, faster than a per-tap select
        *yp = (T)acc;
    }
}

// The vertical pass with UP, DOWN in {1, 2}: a lane owns column ox and a run of R consecutive output rows.
// The run reads SPAN input rows; each is loaded once and feeds every output of the run it is a tap of, with the
// (input row, output, tap) pattern fixed at compile time: output j reads rows dj + k with tap tj + k UP, where
// (dj, tj) depend only on the parity P of the run's first z = oy0 DOWN - pad0 (VRunPat; at UP = 2 an even R keeps P
// the same for every run of a launch).  So the taps stay in registers and every tap is one FMA -- the
// first form tested each (row, output) pair with a uniform branch and an LDS read of its tap (77 branches, LDS
// latency on the FMA chain).  Per output, taps are added in increasing k, as upfirdn_1d does.
template <int UP, int DOWN, int P>
struct VRunPat {
    static constexpr int dj(int j) { return UP == 1 ? j * DOWN : (P == 0 ? (j + 1) / 2 : j / 2); }
    static constexpr int tj(int j) { return UP == 1 ? 0 : (P == 0 ? (j & 1) : 1 - (j & 1)); }
};

template <int UP, int DOWN, int KT, int R, int SPAN, int P>
__device__ __forceinline__ void vrun_acc(const float (&win)[SPAN], const float (&fr)[KT * UP], float (&acc)[R]) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
#pragma unroll
        for (int k = 0; k < KT; ++k) acc[j] += win[VRunPat<UP, DOWN, P>::dj(j) + k] * fr[VRunPat<UP, DOWN, P>::tj(j) + k * UP];
    }
}

template <typename T, int UP, int DOWN, int KT, int R>
__global__ __launch_bounds__(256) void upfirdn_1d_vrun(UpfParams p) {
    static_assert(UP == 1 || R % 2 == 0, "even runs keep the phase fixed");
    constexpr int SPAN = ((R - 1) * DOWN + UP - 1) / UP + KT;
    __shared__ float sf[64];
    const int F = p.fh;
    for (int t = threadIdx.x; t < F; t += 256) sf[t] = p.f[p.flip ? t : F - 1 - t] * p.gain;
    __syncthreads();
    float fr[KT * UP];                                 // the taps in registers, zero past the filter
#pragma unroll
    for (int t = 0; t < KT * UP; ++t) fr[t] = t < F ? sf[t] : 0.f;
    const int ly = p.lim ? p.lim[0] : p.OH, lx = p.lim ? p.lim[1] : p.OW;      // computed extent
    const int rows = min(p.OH, ly + (p.lim ? kZeroBand : 0)), cols = min(p.OW, lx + (p.lim ? kZeroBand : 0));
    const int tiles = (cols + 255) / 256, runs = (rows + R - 1) / R;
    const int total = p.N * p.C * runs * tiles;
    for (int b = blockIdx.x; b < total; b += gridDim.x) {
        const int run = b / tiles;
        const int ox = (b - run * tiles) * 256 + threadIdx.x;
        const int oy0 = (run % runs) * R, nc = run / runs;
        if (ox >= cols) continue;
        const int c = nc % p.C, n = nc / p.C;
        const T* xb = (const T*)p.x + n * p.xs_n + c * p.xs_c + (int64_t)ox * p.xs_w;
        T* yb = (T*)p.y + n * p.ys_n + c * p.ys_c + (int64_t)ox * p.ys_w;
        const int z0 = oy0 * DOWN - p.pady0;
        const int ph = UP == 2 ? (z0 & 1) : 0;
        const int base = UP == 2 ? (z0 + ph) >> 1 : z0;              // input row of output 0's tap 0
        float win[SPAN];
#pragma unroll
        for (int m = 0; m < SPAN; ++m) {
            const int i = base + m;
            const bool ok = i >= 0 && i < p.H;
            const float v = (float)xb[(int64_t)(ok ? i : 0) * p.xs_h];
            win[m] = ok ? v : 0.f;
        }
        float acc[R];
#pragma unroll
        for (int j = 0; j < R; ++j) acc[j] = 0.f;
        if (ph) vrun_acc<UP, DOWN, KT, R, SPAN, 1>(win, fr, acc);
        else vrun_acc<UP, DOWN, KT, R, SPAN, 0>(win, fr, acc);
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const int oy = oy0 + j;
            if (oy >= rows) break;
            yb[(int64_t)oy * p.ys_h] = (oy >= ly || ox >= lx) ? (T)0.f : (T)acc[j];
        }
    }
}

template <typename T> struct VecN { static constexpr int N = 8; };
template <> struct VecN<float> { static constexpr int N = 4; };

// Shared epilogue of the vectorised kernels: z = clamp(act(c * out_scale + noise * g + bias) * gain),
// y = round(z) + residual, aux = c or z.
template <typename T, int V, typename vecT>
__device__ __forceinline__ void store_out(const UpfParams& p, T* y, const float* acc, int n, int oy, int ox, int cv) {
    const int64_t dst = n * p.ys_n + (int64_t)oy * p.ys_h + (int64_t)ox * p.ys_w + cv * V;
    vecT o;
    if (p.epi) {
        const float nv = p.noise ? (float)((const T*)p.noise)[((int64_t)n * p.OH + oy) * p.OW + ox] * p.noise_gain : 0.f;
        vecT ax, rv;
        if (p.residual) rv = *(const vecT*)((const T*)p.residual + dst);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const int c = cv * V + j;
            float v = acc[j];
            if (p.out_scale) v *= p.out_scale[(int64_t)n * p.C + c];
            v += nv;
            if (p.bias) v += (float)(T)p.bias[c];     // bias rounded to the activation dtype
            if (p.act == 1) v = v > 0.f ? v : v * p.alpha;
            v *= p.egain;
            if (p.clamp >= 0.f) v = fminf(fmaxf(v, -p.clamp), p.clamp);
            ax[j] = (T)(p.aux_mode == 1 ? acc[j] : v);
            o[j] = (T)v;
            if (p.residual) o[j] = (T)((float)o[j] + (float)rv[j]);
        }
        if (p.aux_mode) *(vecT*)((T*)p.aux + dst) = ax;
    } else {
#pragma unroll
        for (int j = 0; j < V; ++j) o[j] = (T)acc[j];
    }
    *(vecT*)(y + dst) = o;
}


// channels-last, C % V == 0, xs_c == ys_c == 1.  IDX: the flat output index type -- unsigned 32-bit when
// N*OH*OW*C/V < 2^31 (the host checks), where the 64-bit divisions and remainders that split it into
// (n, oy, ox, cv) cost ~4x the rest of the lane's work (the up-2 adjoint FIRs of the D skips).
template <typename T, typename IDX>
__global__ __launch_bounds__(256) void upfirdn_nhwc_vec(UpfParams p) {
    constexpr int V = VecN<T>::N;
    typedef T vecT __attribute__((ext_vector_type(V)));
    __shared__ float sf[kMaxTaps];
    stage_filter(sf, p);
    const T* x = (const T*)p.x;
    T* y = (T*)p.y;
    const IDX CV = (IDX)(p.C / V), OW = (IDX)p.OW, OH = (IDX)p.OH;
    const IDX total = (IDX)((int64_t)p.N * p.OH * p.OW * (p.C / V));
    for (IDX idx = (IDX)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (IDX)gridDim.x * blockDim.x) {
        IDX r = idx;
        const int cv = (int)(r % CV); r /= CV;
        const int ox = (int)(r % OW); r /= OW;
        const int oy = (int)(r % OH); r /= OH;
        const int n = (int)r;
        int ty0, iy0, tx0, ix0;
        axis_taps(oy, p.downy, p.pady0, p.upy, ty0, iy0);
        axis_taps(ox, p.downx, p.padx0, p.upx, tx0, ix0);
        const T* xb = x + n * p.xs_n + cv * V;
        float acc[V];
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] = 0.f;
        for (int ty = ty0, iy = iy0; ty < p.fh; ty += p.upy, ++iy) {
            if (iy < 0 || iy >= p.H) continue;
            const T* xr = xb + iy * p.xs_h;
            for (int tx = tx0, ix = ix0; tx < p.fw; tx += p.upx, ++ix) {
                if (ix < 0 || ix >= p.W) continue;
                const float wt = sf[ty * p.fw + tx];
                const vecT v = *(const vecT*)(xr + ix * p.xs_w);
#pragma unroll
                for (int j = 0; j < V; ++j) acc[j] += (float)v[j] * wt;
            }
        }
        store_out<T, V, vecT>(p, y, acc, n, oy, ox, cv);
    }
}

// f16 operand (low / high half of a packed pair) times an f32 weight plus an f32 accumulator in one
// v_fma_mix_f32: the exact f16 -> f32 conversion and a single-rounding FMA, bitwise what cvt + fma give.
__device__ __forceinline__ float fma_mix_lo(unsigned h2, float w, float acc) {
    float r;
    asm volatile("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h2), "v"(w), "v"(acc));
    return r;
}
__device__ __forceinline__ float fma_mix_hi(unsigned h2, float w, float acc) {
    float r;
    asm volatile("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h2), "v"(w), "v"(acc));
    return r;
}

// 4x4 filter, up = 2, down = 1 on both axes, channels-last (the adjoint of every down-2 FIR: the D skips'
// input gradients; upsample2d): a lane owns one channel vector of a 2 x 2 output cell (2 cy + py, 2 cx + px).
// Each output reads 2 x 2 input pixels and the cell's four outputs read inside one 3 x 3 neighbourhood,
// so the lane issues its 9 loads at once (vs 16 dependent ones for four upfirdn_nhwc_vec iterations) and
// all index math is 32-bit (the host checks the cell count).
template <typename T>
__global__ __launch_bounds__(256) void upfirdn_nhwc_up2(UpfParams p) {
    constexpr int V = VecN<T>::N;
    typedef T vecT __attribute__((ext_vector_type(V)));
    __shared__ float sf[16];
    if (threadIdx.x < 16) {
        const int ty = threadIdx.x >> 2, tx = threadIdx.x & 3;
        sf[threadIdx.x] = p.f[(p.flip ? ty : 3 - ty) * 4 + (p.flip ? tx : 3 - tx)] * p.gain;
    }
    __syncthreads();
    const unsigned CV = p.C / V, CW = (p.OW + 1) >> 1, CH = (p.OH + 1) >> 1;
    const unsigned total = (unsigned)p.N * CH * CW * CV;
    const unsigned idx = blockIdx.x * 256u + threadIdx.x;
    if (idx >= total) return;
    unsigned r = idx;
    const int cv = (int)(r % CV); r /= CV;
    const int cx = (int)(r % CW); r /= CW;
    const int cy = (int)(r % CH);
    const int n = (int)(r / CH);
    // per output row / column of the cell: first tap and its input index (axis_taps), relative to the first
    int ty[2], iy[2], tx[2], ix[2];
    axis_taps(2 * cy, 1, p.pady0, 2, ty[0], iy[0]);
    axis_taps(2 * cy + 1, 1, p.pady0, 2, ty[1], iy[1]);
    axis_taps(2 * cx, 1, p.padx0, 2, tx[0], ix[0]);
    axis_taps(2 * cx + 1, 1, p.padx0, 2, tx[1], ix[1]);
    const int y0 = min(iy[0], iy[1]), x0 = min(ix[0], ix[1]);
    const T* xb = (const T*)p.x + n * p.xs_n + cv * V;
    vecT xv[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            const int yy = y0 + a, xx = x0 + b;
            const bool ok = yy >= 0 && yy < p.H && xx >= 0 && xx < p.W;
            xv[a][b] = ok ? *(const vecT*)(xb + yy * p.xs_h + xx * p.xs_w) : vecT{};
        }
#pragma unroll
    for (int py = 0; py < 2; ++py) {
        const int oy = 2 * cy + py;
        if (oy >= p.OH) continue;
        const int dy = iy[py] - y0;
#pragma unroll
        for (int px = 0; px < 2; ++px) {
            const int ox = 2 * cx + px;
            if (ox >= p.OW) continue;
            const int dx = ix[px] - x0;
            float acc[V];
#pragma unroll
            for (int j = 0; j < V; ++j) acc[j] = 0.f;
            // taps (ty + 2 a, tx + 2 b) on inputs (iy + a, ix + b), a, b in {0, 1}, in upfirdn_nhwc_vec's order
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                const int t1 = ty[py] + 2 * a;
                if (t1 >= 4) continue;
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    const int t2 = tx[px] + 2 * b;
                    if (t2 >= 4) continue;
                    const float w = sf[t1 * 4 + t2];
                    const vecT v = dy ? (dx ? xv[1 + a][1 + b] : xv[1 + a][b]) : (dx ? xv[a][1 + b] : xv[a][b]);
                    if constexpr (std::is_same<T, f16_t>::value) {
                        typedef unsigned u32v __attribute__((ext_vector_type(V / 2)));
                        const u32v u = __builtin_bit_cast(u32v, v);
#pragma unroll
                        for (int q = 0; q < V / 2; ++q) {
                            acc[2 * q] = fma_mix_lo(u[q], w, acc[2 * q]);
                            acc[2 * q + 1] = fma_mix_hi(u[q], w, acc[2 * q + 1]);
                        }
                    } else {
#pragma unroll
                        for (int j = 0; j < V; ++j) acc[j] += (float)v[j] * w;
                    }
                }
            }
            store_out<T, V, vecT>(p, (T*)p.y, acc, n, oy, ox, cv);
        }
    }
}

// 4x4 filter, up = 1, down = DOWN (1 or 2) on both axes, channels-last: the resample filter of every
// G/D layer.  A workgroup owns a TW x TH output tile x CG channel vectors: it stages the
// ((TH-1)*DOWN + 4) x ((TW-1)*DOWN + 4) input patch once in LDS with coalesced loads (CG consecutive
// lanes = one pixel's CG*16 bytes; ~1.4 global loads per output vector at DOWN 1 instead of 16 L1
// requests), then each lane reads its 16 taps back with conflict-free ds_read_b128.  CG = 4 keeps the
// patch at 25 KB (DOWN 1, 32 x 8) / 39 KB (DOWN 2, 16 x 8) so several workgroups share a CU.
template <typename T, int DOWN, int TW, int TH, int CG>
__global__ __launch_bounds__(256) void upfirdn_nhwc_f4(UpfParams p) {
    constexpr int V = VecN<T>::N;
    constexpr int F = 4;                              // CG channel vectors per workgroup
    constexpr int IW = (TW - 1) * DOWN + F, IH = (TH - 1) * DOWN + F, NIN = IW * IH * CG;
    typedef T vecT __attribute__((ext_vector_type(V)));
    __shared__ float sf[F * F];
    extern __shared__ __attribute__((aligned(16))) char tile_raw[];
    vecT* tile = (vecT*)tile_raw;                     // [IH][IW][CG]
    const int tid = threadIdx.x;
    if (tid < F * F) {
        const int ty = tid / F, tx = tid % F;
        sf[tid] = p.f[(p.flip ? ty : F - 1 - ty) * F + (p.flip ? tx : F - 1 - tx)] * p.gain;
    }
    const int CV = p.C / V;
    const int ngroups = (CV + CG - 1) / CG;
    const int tiles_x = (p.OW + TW - 1) / TW, tiles_y = (p.OH + TH - 1) / TH;
    int64_t b = blockIdx.x;
    // XCD-contiguous renumbering (SG2_FIR_XCD=0 disables, for A/B): workgroups are dealt to the 8 XCDs round
    // robin, so without it the channel groups of one tile -- which split each pixel's cache lines -- and
    // neighbouring tiles -- which share halo rows -- land in different L2s
    const int64_t nb = gridDim.x;
    if ((nb & 7) == 0 && p.xcd) b = (b & 7) * (nb >> 3) + (b >> 3);
    const int cg = (int)(b % ngroups); b /= ngroups;
    const int tx0 = (int)(b % tiles_x) * TW; b /= tiles_x;
    const int ty0 = (int)(b % tiles_y) * TH; b /= tiles_y;
    const int n = (int)b;
    const int cv0 = cg * CG;
    const T* xb = (const T*)p.x + n * p.xs_n;
    const int iy0 = ty0 * DOWN - p.pady0, ix0 = tx0 * DOWN - p.padx0;
    for (int i = tid; i < NIN; i += 256) {
        const int c = i % CG, px = i / CG;
        const int ry = px / IW, rx = px - ry * IW;
        const int iy = iy0 + ry, ix = ix0 + rx;
        const bool ok = iy >= 0 && iy < p.H && ix >= 0 && ix < p.W && cv0 + c < CV;
        vecT v = *(const vecT*)(xb + (int64_t)(ok ? iy : 0) * p.xs_h + (int64_t)(ok ? ix : 0) * p.xs_w +
                                (ok ? cv0 + c : 0) * V);
#pragma unroll
        for (int j = 0; j < V; ++j) v[j] = ok ? v[j] : (T)0.f;
        tile[i] = v;
    }
    __syncthreads();
    const int c = tid % CG;
    if (cv0 + c >= CV) return;
#pragma unroll
    for (int pass = 0; pass < TW * TH * CG / 256; ++pass) {
        const int pix = tid / CG + pass * (256 / CG);
        const int oy = ty0 + pix / TW, ox = tx0 + pix % TW;
        if (oy >= p.OH || ox >= p.OW) continue;
        float acc[V];
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] = 0.f;
        const vecT* base = tile + ((pix / TW) * DOWN * IW + (pix % TW) * DOWN) * CG + c;
#pragma unroll
        for (int ky = 0; ky < F; ++ky)
#pragma unroll
            for (int kx = 0; kx < F; ++kx) {
                const float w = sf[ky * F + kx];
                const vecT v = base[(ky * IW + kx) * CG];
                if constexpr (std::is_same<T, f16_t>::value) {   // conversion + FMA in one v_fma_mix_f32
                    typedef unsigned u32v __attribute__((ext_vector_type(V / 2)));
                    const u32v u = __builtin_bit_cast(u32v, v);
#pragma unroll
                    for (int q = 0; q < V / 2; ++q) {
                        acc[2 * q] = fma_mix_lo(u[q], w, acc[2 * q]);
                        acc[2 * q + 1] = fma_mix_hi(u[q], w, acc[2 * q + 1]);
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < V; ++j) acc[j] += (float)v[j] * w;
                }
            }
        store_out<T, V, vecT>(p, (T*)p.y, acc, n, oy, ox, cv0 + c);
    }
}

// One lane's column strip of the f4s kernel: every input row is read from LDS once and feeds the
// up-to-4 output rows that use it; an output row is stored as soon as its last input row is in.  The
// layer epilogue (store_out's semantics) is resolved to per-lane constants once, so the per-row store
// is branch-free apart from the uniform noise/residual/aux pointer tests.
// SEP: the 4x4 taps are an exact outer product wf[ky][kx] = fy[ky] * fx[kx] (the [1,3,3,1] resample
// filter): every input row is filtered horizontally once (4 FMAs) and the output rows combine those
// row sums vertically (4 FMAs), 9.5 FMAs per output vector instead of 16.  For fp16 the horizontal FMAs
// take their operand straight from the packed halves (v_fma_mix_f32: the exact f16 -> f32 conversion and
// the FMA in one instruction, where cvt + v_pk_fma_f32 costs 1.5 per tap and element).
// EPI = false (no layer epilogue): the rounded FIR sum is stored as is, none of the epilogue arithmetic runs.
template <typename T, int V, typename vecT, int TW, int TH, int CG, bool SEP, bool EPI>
__device__ __forceinline__ void fir4_strip(const UpfParams& p, const vecT* base, const float* wf, const float* fy,
                                           const float* fx, int n, int ty0, int ox, int cv) {
    constexpr int F = 4, IW = TW + F - 1, IH = TH + F - 1;
    float os[V], bj[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        const int c = cv * V + j;
        os[j] = (p.epi && p.out_scale) ? p.out_scale[(int64_t)n * p.C + c] : 1.f;
        bj[j] = (p.epi && p.bias) ? (float)(T)p.bias[c] : 0.f;   // bias rounded to the activation dtype
    }
    const float slope = (p.epi && p.act == 1) ? p.alpha : 1.f;
    const float eg = p.epi ? p.egain : 1.f;
    const bool clamp_on = p.epi && p.clamp >= 0.f;
    const float cl = p.clamp;
    const bool noise = p.epi && p.noise, resid = p.epi && p.residual;
    const int aux_mode = p.epi ? p.aux_mode : 0;
    float acc[TH][V];
#pragma unroll
    for (int o = 0; o < TH; ++o)
#pragma unroll
        for (int j = 0; j < V; ++j) acc[o][j] = 0.f;
#pragma unroll
    for (int ry = 0; ry < IH; ++ry) {
        vecT v[F];
#pragma unroll
        for (int kx = 0; kx < F; ++kx) v[kx] = base[(ry * IW + kx) * CG];
        if constexpr (SEP) {
            float h[V];
            if constexpr (std::is_same<T, f16_t>::value) {
                typedef unsigned u32v __attribute__((ext_vector_type(V / 2)));
#pragma unroll
                for (int j = 0; j < V; ++j) h[j] = 0.f;
#pragma unroll
                for (int kx = 0; kx < F; ++kx) {
                    const u32v u = __builtin_bit_cast(u32v, v[kx]);
#pragma unroll
                    for (int q = 0; q < V / 2; ++q) {
                        h[2 * q] = fma_mix_lo(u[q], fx[kx], h[2 * q]);
                        h[2 * q + 1] = fma_mix_hi(u[q], fx[kx], h[2 * q + 1]);
                    }
                }
            } else {
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    h[j] = 0.f;
#pragma unroll
                    for (int kx = 0; kx < F; ++kx) h[j] += (float)v[kx][j] * fx[kx];
                }
            }
#pragma unroll
            for (int ky = 0; ky < F; ++ky) {
                const int o = ry - ky;
                if (o < 0 || o >= TH) continue;
#pragma unroll
                for (int j = 0; j < V; ++j) acc[o][j] += h[j] * fy[ky];
            }
        } else {
#pragma unroll
            for (int ky = 0; ky < F; ++ky) {
                const int o = ry - ky;                // output row fed by input row ry through tap row ky
                if (o < 0 || o >= TH) continue;
#pragma unroll
                for (int kx = 0; kx < F; ++kx)
#pragma unroll
                    for (int j = 0; j < V; ++j) acc[o][j] += (float)v[kx][j] * wf[ky * F + kx];
            }
        }
        const int od = ry - (F - 1);                  // output row completed by input row ry
        if (od < 0) continue;
        const int oy = ty0 + od;
        const int64_t dst = n * p.ys_n + (int64_t)oy * p.ys_h + (int64_t)ox * p.ys_w + cv * V;
        if constexpr (!EPI) {
            vecT o;
#pragma unroll
            for (int j = 0; j < V; ++j) o[j] = (T)acc[od][j];
            *(vecT*)((T*)p.y + dst) = o;
            __builtin_amdgcn_sched_barrier(0);
            continue;
        }
        const float nv = noise ? (float)((const T*)p.noise)[((int64_t)n * p.OH + oy) * p.OW + ox] * p.noise_gain : 0.f;
        vecT o, ax;
#pragma unroll
        for (int j = 0; j < V; ++j) {
            float z = acc[od][j] * os[j] + nv + bj[j];
            z = (z > 0.f ? z : z * slope) * eg;
            if (clamp_on) z = fminf(fmaxf(z, -cl), cl);
            o[j] = (T)z;
            ax[j] = (T)(aux_mode == 1 ? acc[od][j] : z);
        }
        if (resid) {
            const vecT rv = *(const vecT*)((const T*)p.residual + dst);
#pragma unroll
            for (int j = 0; j < V; ++j) o[j] = (T)((float)o[j] + (float)rv[j]);
        }
        if (aux_mode) *(vecT*)((T*)p.aux + dst) = ax;
        *(vecT*)((T*)p.y + dst) = o;
        __builtin_amdgcn_sched_barrier(0);            // keeps the next rows' LDS reads below this store
    }
}

// 4x4 filter, up = down = 1, channels-last: the FIR of every G up-layer and D down-layer pad-FIR.
// A workgroup owns a TW x TH output tile x CG = 8 channel vectors (a whole 128-byte line of each
// pixel, so no line is split between workgroups on different XCDs); CG = 4 with TW = 64 for 16-bit C = 32
// (C5's 1024^2 layers: a 64-byte pixel, where 8-vector groups left half the lanes idle).  All loads of the
// (TH+3) x (TW+3) input patch are issued before the first LDS write (one latency per tile, ~13
// 16-byte loads in flight per lane).  Each lane then owns one column x one channel vector and slides
// down the strip: every input row is read from LDS once (4 ds_read_b128) and feeds the up-to-4 output
// rows that use it, 5.5 LDS reads per output instead of 16.  Blocks are renumbered so each XCD walks a
// contiguous run of tiles (neighbouring tiles share halo rows in that XCD's L2).
template <typename T, int TW, int TH, int CG = 8>
__global__ __launch_bounds__(256, 2) void upfirdn_nhwc_f4s(UpfParams p) {
    constexpr int V = VecN<T>::N, F = 4;
    constexpr int IW = TW + F - 1, IH = TH + F - 1, NIN = IW * IH * CG;
    constexpr int NL = (NIN + 255) / 256;
    static_assert(TW * CG == 256, "one lane per (column, channel vector)");
    typedef T vecT __attribute__((ext_vector_type(V)));
    extern __shared__ __attribute__((aligned(16))) char tile_raw[];
    vecT* tile = (vecT*)tile_raw;                     // [IH][IW][CG]
    const int tid = threadIdx.x;
    float wf[F * F];
#pragma unroll
    for (int t = 0; t < F * F; ++t) {
        const int ty = t / F, tx = t % F;
        wf[t] = p.f[(p.flip ? ty : F - 1 - ty) * F + (p.flip ? tx : F - 1 - tx)] * p.gain;
    }
    const int CV = p.C / V;
    const int ngroups = (CV + CG - 1) / CG;
    const int tiles_x = (p.OW + TW - 1) / TW, tiles_y = (p.OH + TH - 1) / TH;
    int64_t b = blockIdx.x;
    const int64_t nb = gridDim.x;
    if ((nb & 7) == 0) b = (b & 7) * (nb >> 3) + (b >> 3);   // XCD-contiguous tile runs
    // the last tile of a row/column is shifted back inside the image (host guarantees OH >= TH,
    // OW >= TW): every strip is whole and branch-free; the overlap is written twice with equal values
    const int tx0 = min((int)(b % tiles_x) * TW, p.OW - TW); b /= tiles_x;
    const int ty0 = min((int)(b % tiles_y) * TH, p.OH - TH); b /= tiles_y;
    const int cg = (int)(b % ngroups); b /= ngroups;
    const int n = (int)b;
    const int cv0 = cg * CG;
    const T* xb = (const T*)p.x + n * p.xs_n;
    const int iy0 = ty0 - p.pady0, ix0 = tx0 - p.padx0;
    vecT r[NL];
#pragma unroll
    for (int l = 0; l < NL; ++l) {
        const int i = tid + l * 256;
        const int c = i % CG, px = i / CG;
        const int ry = px / IW, rx = px - ry * IW;
        const int iy = iy0 + ry, ix = ix0 + rx;
        const bool ok = i < NIN && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W && cv0 + c < CV;
        r[l] = *(const vecT*)(xb + (int64_t)(ok ? iy : 0) * p.xs_h + (int64_t)(ok ? ix : 0) * p.xs_w +
                              (ok ? cv0 + c : 0) * V);
#pragma unroll
        for (int j = 0; j < V; ++j) r[l][j] = ok ? r[l][j] : (T)0.f;
    }
#pragma unroll
    for (int l = 0; l < NL; ++l)
        if (l < NL - 1 || tid + l * 256 < NIN) tile[tid + l * 256] = r[l];
    __syncthreads();
    const int c = tid % CG, col = tid / CG;
    if (cv0 + c >= CV) return;
    // exact rank-1 test of the taps (uniform): wf = fy (x) fx with fy[ky] = wf[ky][0] / wf[0][0], fx = wf[0][:]
    float fy[F], fx[F];
    bool sep = wf[0] != 0.f;
#pragma unroll
    for (int k = 0; k < F; ++k) {
        fx[k] = wf[k];
        fy[k] = sep ? wf[k * F] / wf[0] : 0.f;
    }
#pragma unroll
    for (int t = 0; t < F * F; ++t) sep = sep && (fy[t / F] * fx[t % F] == wf[t]);
    const vecT* tb = tile + col * CG + c;
    if (sep) {
        if (p.epi) fir4_strip<T, V, vecT, TW, TH, CG, true, true>(p, tb, wf, fy, fx, n, ty0, tx0 + col, cv0 + c);
        else fir4_strip<T, V, vecT, TW, TH, CG, true, false>(p, tb, wf, fy, fx, n, ty0, tx0 + col, cv0 + c);
    } else {
        if (p.epi) fir4_strip<T, V, vecT, TW, TH, CG, false, true>(p, tb, wf, fy, fx, n, ty0, tx0 + col, cv0 + c);
        else fir4_strip<T, V, vecT, TW, TH, CG, false, false>(p, tb, wf, fy, fx, n, ty0, tx0 + col, cv0 + c);
    }
}

template <typename T>
int launch(const UpfParams& p, bool vec, hipStream_t s) {
    static const bool fir_old = getenv("SG2_FIR_OLD") != nullptr;
    if (!fir_old && vec && p.upx == 1 && p.upy == 1 && p.downx == 1 && p.downy == 1 && p.fw == 4 && p.fh == 4 &&
        p.OH >= 8 && (p.OW % 32 == 0 || p.OW >= 224) && !(p.residual && p.residual == p.y)) {
        // (narrow ragged widths, e.g. the 65- and 33-wide pad-FIR of D, waste up to half the shifted last
        // column tile: they stay on upfirdn_nhwc_f4)
        constexpr int TW = 32, TH = 8;
        const char* e32 = getenv("SG2_FIR_C32");      // A/B: 0 = the 8-vector groups (read per launch: tests)
        const bool c32_off = e32 && e32[0] == '0';
        if (!c32_off && p.C / VecN<T>::N == 4 && (p.OW % 64 == 0 || p.OW >= 224)) {   // 16-bit C = 32
            constexpr int TW4 = 64, CG4 = 4;
            const int64_t blocks4 = (int64_t)p.N * cdiv(p.OH, TH) * cdiv(p.OW, TW4);
            if (blocks4 < INT32_MAX) {
                const size_t lds = (size_t)(TH + 3) * (TW4 + 3) * CG4 * 16;
                auto k = upfirdn_nhwc_f4s<T, TW4, TH, CG4>;
                static bool set4 = false;
                if (!set4) { (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); set4 = true; }
                k<<<(unsigned)blocks4, 256, lds, s>>>(p);
                return launch_status("sg2_upfirdn2d");
            }
        }
        const int64_t blocks = (int64_t)p.N * cdiv(p.OH, TH) * cdiv(p.OW, TW) * cdiv(p.C / VecN<T>::N, 8);
        if (blocks < INT32_MAX) {
            const size_t lds = (size_t)(TH + 3) * (TW + 3) * 8 * 16;
            auto k = upfirdn_nhwc_f4s<T, TW, TH>;
            static bool set = false;
            if (!set) { (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); set = true; }
            k<<<(unsigned)blocks, 256, lds, s>>>(p);
            return launch_status("sg2_upfirdn2d");
        }
    }
    if (vec && p.upx == 1 && p.upy == 1 && p.downx == p.downy && (p.downy == 1 || p.downy == 2) && p.fw == 4 &&
        p.fh == 4) {
        constexpr int CG = 4;
        const int d = p.downy;
        const int TW = d == 1 ? 32 : 16, TH = 8;
        const int64_t blocks = (int64_t)p.N * cdiv(p.OH, TH) * cdiv(p.OW, TW) * cdiv(p.C / VecN<T>::N, CG);
        if (blocks < INT32_MAX) {
            const size_t lds = (size_t)((TH - 1) * d + 4) * ((TW - 1) * d + 4) * CG * 16;
            if (d == 1) {
                auto k = upfirdn_nhwc_f4<T, 1, 32, 8, CG>;
                static bool set1 = false;
                if (!set1) { (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); set1 = true; }
                k<<<(unsigned)blocks, 256, lds, s>>>(p);
            } else {
                auto k = upfirdn_nhwc_f4<T, 2, 16, 8, CG>;
                static bool set2 = false;
                if (!set2) { (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); set2 = true; }
                k<<<(unsigned)blocks, 256, lds, s>>>(p);
            }
            return launch_status("sg2_upfirdn2d");
        }
    }
    if (vec && p.upx == 2 && p.upy == 2 && p.downx == 1 && p.downy == 1 && p.fw == 4 && p.fh == 4 &&
        !getenv("SG2_UPF_UP2_OFF")) {
        const int64_t cells = (int64_t)p.N * ((p.OH + 1) / 2) * ((p.OW + 1) / 2) * (p.C / VecN<T>::N);
        if (cells < INT32_MAX - 256) {
            upfirdn_nhwc_up2<T><<<(unsigned)cdiv(cells, 256), 256, 0, s>>>(p);
            return launch_status("sg2_upfirdn2d");
        }
    }
    if (!vec && !p.epi) {
        const bool horiz = p.fh == 1 && p.upy == 1 && p.downy == 1 && p.pady0 == 0 && p.OH == p.H && p.fw <= 64;
        const bool vert = p.fw == 1 && p.upx == 1 && p.downx == 1 && p.padx0 == 0 && p.OW == p.W && p.fh <= 64;
        const int up = horiz ? p.upx : p.upy, down = horiz ? p.downx : p.downy, F = horiz ? p.fw : p.fh;
        const int kt = (F + up - 1) / up;
        const int64_t pairs = (int64_t)p.N * p.C * p.OH * cdiv(p.OW, 256);
        if ((horiz || vert) && kt <= 16 && pairs < INT32_MAX) {
            static const int gmax = [] { const char* e = getenv("SG2_U1D_GRID"); return e ? atoi(e) : 4096; }();   // 16 a CU (r06aj A/B)
            const unsigned g = (unsigned)std::min<int64_t>(pairs, gmax);
            const bool ada_up = up == 2 && down == 1 && kt == 6, ada_down = up == 1 && down == 2 && kt == 12;
            static const int vr = [] { const char* e = getenv("SG2_U1D_VRUN"); return e ? atoi(e) : 4; }();
            static const bool hl = [] { const char* e = getenv("SG2_U1D_HLDS"); return e ? atoi(e) != 0 : true; }();
            static const int htw = [] { const char* e = getenv("SG2_U1D_HTW"); return e ? atoi(e) : 128; }();
            if (vert && vr == 4 && ada_up) upfirdn_1d_vrun<T, 2, 1, 6, 4><<<g, 256, 0, s>>>(p);
            else if (vert && vr == 4 && ada_down) upfirdn_1d_vrun<T, 1, 2, 12, 4><<<g, 256, 0, s>>>(p);
            else if (vert && vr == 8 && ada_up) upfirdn_1d_vrun<T, 2, 1, 6, 8><<<g, 256, 0, s>>>(p);
            else if (vert && vr == 8 && ada_down) upfirdn_1d_vrun<T, 1, 2, 12, 8><<<g, 256, 0, s>>>(p);
            else if (horiz && hl && ada_up && htw == 128) upfirdn_1d_hlds<T, 2, 1, 6, 128><<<g, 256, 0, s>>>(p);
            else if (horiz && hl && ada_down && htw == 128) upfirdn_1d_hlds<T, 1, 2, 12, 128><<<g, 256, 0, s>>>(p);
            else if (horiz && hl && ada_up) upfirdn_1d_hlds<T, 2, 1, 6><<<g, 256, 0, s>>>(p);
            else if (horiz && hl && ada_down) upfirdn_1d_hlds<T, 1, 2, 12><<<g, 256, 0, s>>>(p);
            else if (horiz && ada_up) upfirdn_1d<T, true, 6, 2, 1><<<g, 256, 0, s>>>(p);
            else if (horiz && ada_down) upfirdn_1d<T, true, 12, 1, 2><<<g, 256, 0, s>>>(p);
            else if (ada_up) upfirdn_1d<T, false, 6, 2, 1><<<g, 256, 0, s>>>(p);
            else if (ada_down) upfirdn_1d<T, false, 12, 1, 2><<<g, 256, 0, s>>>(p);
            else {
#define U1D(KT_) { if (horiz) upfirdn_1d<T, true, KT_, 0, 0><<<g, 256, 0, s>>>(p); \
                   else upfirdn_1d<T, false, KT_, 0, 0><<<g, 256, 0, s>>>(p); }
                if (kt <= 4) U1D(4) else if (kt <= 8) U1D(8) else U1D(16)
#undef U1D
            }
            return launch_status("sg2_upfirdn2d");
        }
    }
    const int64_t work = vec ? (int64_t)p.N * p.OH * p.OW * (p.C / VecN<T>::N) : (int64_t)p.N * p.C * p.OH * p.OW;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(work, 256), 256 * 32));
    if (vec && work < INT32_MAX && (int64_t)grid * 256 < INT32_MAX)
        upfirdn_nhwc_vec<T, unsigned><<<grid, 256, 0, s>>>(p);
    else if (vec)
        upfirdn_nhwc_vec<T, int64_t><<<grid, 256, 0, s>>>(p);
    else
        upfirdn_generic<T><<<grid, 256, 0, s>>>(p);
    return launch_status("sg2_upfirdn2d");
}

}  // namespace
}  // namespace sg2

extern "C" int sg2_upfirdn2d_fused(void* y, const void* x, const float* f, int dtype, const int64_t* in_size,
                                   const int64_t* in_stride, const int64_t* out_size, const int64_t* out_stride,
                                   int fw, int fh, int upx, int upy, int downx, int downy, int padx0, int padx1,
                                   int pady0, int pady1, int flip, float gain, const sg2_epilogue* epi,
                                   void* stream) {
    using namespace sg2;
    SG2_CHECK(x && y && f && in_size && in_stride && out_size && out_stride, "sg2_upfirdn2d: null argument");
    SG2_CHECK(upx >= 1 && upy >= 1 && downx >= 1 && downy >= 1, "sg2_upfirdn2d: up/down must be >= 1");
    SG2_CHECK(fw >= 1 && fh >= 1 && fw * fh <= kMaxTaps, "sg2_upfirdn2d: filter too large");
    UpfParams p;
    p.x = x; p.y = y; p.f = f;
    p.N = (int)in_size[0]; p.C = (int)in_size[1]; p.H = (int)in_size[2]; p.W = (int)in_size[3];
    p.OH = (int)out_size[2]; p.OW = (int)out_size[3];
    SG2_CHECK(out_size[0] == p.N && out_size[1] == p.C, "sg2_upfirdn2d: batch/channel mismatch");
    const int64_t eh = ((int64_t)p.H * upy + pady0 + pady1 - fh + downy) / downy;
    const int64_t ew = ((int64_t)p.W * upx + padx0 + padx1 - fw + downx) / downx;
    SG2_CHECK(p.H * upy + pady0 + pady1 >= fh && p.W * upx + padx0 + padx1 >= fw,
              "sg2_upfirdn2d: upsampled buffer must be at least the size of the filter");
    SG2_CHECK(eh == p.OH && ew == p.OW, "sg2_upfirdn2d: output size mismatch");
    p.xs_n = in_stride[0]; p.xs_c = in_stride[1]; p.xs_h = in_stride[2]; p.xs_w = in_stride[3];
    p.ys_n = out_stride[0]; p.ys_c = out_stride[1]; p.ys_h = out_stride[2]; p.ys_w = out_stride[3];
    p.fw = fw; p.fh = fh; p.upx = upx; p.upy = upy; p.downx = downx; p.downy = downy;
    p.padx0 = padx0; p.pady0 = pady0; p.flip = flip; p.gain = gain; p.lim = nullptr;
    { const char* e = getenv("SG2_FIR_XCD"); p.xcd = e ? atoi(e) : 1; }
    p.out_scale = nullptr; p.noise = nullptr; p.bias = nullptr; p.residual = nullptr; p.aux = nullptr;
    p.noise_gain = 0.f; p.alpha = 0.f; p.egain = 1.f; p.clamp = -1.f; p.act = 0; p.aux_mode = 0; p.epi = 0;
    if (epi) {
        SG2_CHECK(epi->act == 0 || epi->act == 1, "sg2_upfirdn2d: epilogue act must be 0 or 1");
        SG2_CHECK(epi->aux_mode >= 0 && epi->aux_mode <= 2 && (epi->aux_mode == 0 || epi->aux),
                  "sg2_upfirdn2d: bad epilogue aux output");
        p.out_scale = epi->out_scale; p.noise = epi->noise; p.bias = epi->bias; p.residual = epi->residual;
        p.aux = epi->aux; p.noise_gain = epi->noise_gain; p.alpha = epi->alpha; p.egain = epi->gain;
        p.clamp = epi->clamp; p.act = epi->act; p.aux_mode = epi->aux_mode; p.epi = 1;
    }
    if ((int64_t)p.N * p.C * p.OH * p.OW == 0) return 0;
    hipStream_t s = as_stream(stream);
    SG2_DISPATCH(dtype, T, {
        constexpr int V = VecN<T>::N;
        const bool vec = p.xs_c == 1 && p.ys_c == 1 && p.C % V == 0 && p.C >= V &&
                         ((uintptr_t)x % 16 == 0) && ((uintptr_t)y % 16 == 0) &&
                         p.xs_w % V == 0 && p.xs_h % V == 0 && p.xs_n % V == 0 &&
                         p.ys_w % V == 0 && p.ys_h % V == 0 && p.ys_n % V == 0;
        SG2_CHECK(vec || !p.epi, "sg2_upfirdn2d: the fused epilogue needs NHWC activations with C % 8 == 0");
        return launch<T>(p, vec, s);
    });
    return 0;
}

extern "C" int sg2_upfirdn2d_lim(void* y, const void* x, const float* f, int dtype, const int64_t* in_size,
                                 const int64_t* in_stride, const int64_t* out_size, const int64_t* out_stride, int fw,
                                 int fh, int upx, int upy, int downx, int downy, int padx0, int padx1, int pady0,
                                 int pady1, int flip, float gain, const int* lim, void* stream) {
    using namespace sg2;
    SG2_CHECK(x && y && f && in_size && in_stride && out_size && out_stride, "sg2_upfirdn2d: null argument");
    SG2_CHECK(upx >= 1 && upy >= 1 && downx >= 1 && downy >= 1, "sg2_upfirdn2d: up/down must be >= 1");
    SG2_CHECK(fw >= 1 && fh >= 1 && fw * fh <= kMaxTaps, "sg2_upfirdn2d: filter too large");
    UpfParams p{};
    p.x = x; p.y = y; p.f = f; p.lim = lim;
    p.N = (int)in_size[0]; p.C = (int)in_size[1]; p.H = (int)in_size[2]; p.W = (int)in_size[3];
    p.OH = (int)out_size[2]; p.OW = (int)out_size[3];
    SG2_CHECK(out_size[0] == p.N && out_size[1] == p.C, "sg2_upfirdn2d: batch/channel mismatch");
    const int64_t eh = ((int64_t)p.H * upy + pady0 + pady1 - fh + downy) / downy;
    const int64_t ew = ((int64_t)p.W * upx + padx0 + padx1 - fw + downx) / downx;
    SG2_CHECK(eh == p.OH && ew == p.OW, "sg2_upfirdn2d: output size mismatch");
    p.xs_n = in_stride[0]; p.xs_c = in_stride[1]; p.xs_h = in_stride[2]; p.xs_w = in_stride[3];
    p.ys_n = out_stride[0]; p.ys_c = out_stride[1]; p.ys_h = out_stride[2]; p.ys_w = out_stride[3];
    p.fw = fw; p.fh = fh; p.upx = upx; p.upy = upy; p.downx = downx; p.downy = downy;
    p.padx0 = padx0; p.pady0 = pady0; p.flip = flip; p.gain = gain; p.egain = 1.f; p.clamp = -1.f;
    if ((int64_t)p.N * p.C * p.OH * p.OW == 0) return 0;
    hipStream_t s = as_stream(stream);
    SG2_DISPATCH(dtype, T, { return launch<T>(p, false, s); });
    return 0;
}

extern "C" int sg2_upfirdn2d(void* y, const void* x, const float* f, int dtype, const int64_t* in_size,
                             const int64_t* in_stride, const int64_t* out_size, const int64_t* out_stride, int fw,
                             int fh, int upx, int upy, int downx, int downy, int padx0, int padx1, int pady0,
                             int pady1, int flip, float gain, void* stream) {
    return sg2_upfirdn2d_fused(y, x, f, dtype, in_size, in_stride, out_size, out_stride, fw, fh, upx, upy, downx,
                               downy, padx0, padx1, pady0, pady1, flip, gain, nullptr, stream);
}
