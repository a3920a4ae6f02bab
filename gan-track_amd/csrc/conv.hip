// Dense 2-D convolutions of the StyleGAN2 G/D on MFMA (gfx950), NHWC activations.
//
// Replaces the cuDNN convolutions the reference reaches through
// SG3/torch_utils/ops/conv2d_resample.py:29-41 -> conv2d_gradfix.py:37-45 (F.conv2d,
// F.conv_transpose2d) and their autograd weight gradients.
//
// Forward / data-gradient: implicit GEMM.  M = output pixels of one output phase, N = Cout,
// K = taps x Cin.  A transposed stride-S convolution is split into S*S output phases; inside a phase
// every output pixel uses the same taps, so the GEMM has no zero-inserted work
// (2*N*Cout*Cin*KH*KW*H*W FLOPs in total, the SURVEY 8(d) count).
//   A[m][k] = x[n, q*is + tap.dy, q*is + tap.dx, c]     (gathered, zero outside the image)
//   B[k][o] = w[o][tap][c]                               (packed weight, K-contiguous per o)
// Block tile BM x BN, 4 waves in 2 x 2, each wave (BM/2) x (BN/2) of 16x16 MFMA tiles:
//   f16/bf16: v_mfma_f32_16x16x32_{f16,bf16}, K-stage 32 elements
//   f32     : v_mfma_f32_16x16x4_f32 (exact f32), K-stage 16 elements
// Both operand tiles are register-staged global->LDS with two LDS buffers: the next stage's 16-byte
// global loads are issued before the current stage's MFMAs, and written to the other buffer after.
// Small-M layers (low resolutions) split K over blocks and reduce with f32 atomics.
//
// Weight gradient: dw[a][tap][b] = sum_m g[m][a] * x[in(m,tap)][b]; GEMM over K = pixels with both
// operands pixel-major in LDS; the 16-bit fragments are read with ds_read_b64_tr_b16 (hardware
// transpose), f32 fragments with plain ds_read_b32.  Split over pixels, f32 atomic reduction.
//
// f32 layers (the 4^2..16^2 blocks, num_fp16_res=4) run by default as a three-way bf16 split ("S3"):
// each f32 operand is staged into LDS as x = h + m + l (three bf16 planes, exact for normal
// numbers), and the GEMM takes the six products h*h, h*m, m*h, h*l, l*h, m*m on the bf16 MFMA with
// f32 accumulation.  The dropped terms (m*l, l*m, l*l) are O(2^-24) of each product, the size of
// one f32 rounding, so the result has f32 accuracy (the reference disables TF32,
// training_loop_mi_multimodal.py:169-170, and this keeps that contract) at 6 x 16 = 96 cycles per
// 32-deep K step instead of 8 x 32 = 256 for v_mfma_f32_16x16x4_f32.  SG2_F32_EXACT=1 selects the
// f32-input MFMA path instead.
#include "sg2_common.h"

#include <algorithm>
#include <type_traits>

namespace sg2 {
namespace {

constexpr int kMaxTaps = 64;
constexpr int kMaxPhases = 4;

struct Tap { int8_t dy, dx, w, pad_; };

struct Phase {
    int QH, QW, M;           // phase grid, M = N*QH*QW
    int osy, osx, oy0, ox0;  // output coordinate = q*os + o0
    int tap0, ntaps, nk;     // taps [tap0, tap0 + ntaps) of the shared table; nk = ntaps * nck
};

// Fused epilogue (mirror of sg2_epilogue in include/sg2hip.h).
struct Epi {
    const float* out_scale;  // [N, Cout]
    const void* noise;       // [N, OH, OW] (T)
    const float* bias;       // [Cout]
    const void* residual;    // [N, OH, OW, Cout] (T), added after rounding the activation
    void* aux;               // [N, OH, OW, Cout] (T): aux_mode 1 = conv result, 2 = activation before residual
    const void* dot_src;     // [N, OH, OW, Cout] (T): dot_out[n, o] += sum_p c * dot_src
    float* dot_out;          // [N, Cout] float, zeroed by the host
    float* det_dot;          // deterministic mode: the dot's contributions by slot instead of atomics --
                             // [N * OH * OW][Cout] per-element products (conv_fwd / finalize), or
                             // [gridDim.x][N][Cout] workgroup partials (conv1x1_smallk_dot)
    float noise_gain, alpha, gain, clamp;
    int act, aux_mode, on;
};

struct ConvArgs {
    const void* x;
    const void* w;
    void* y;       // T output (non-split)
    float* acc;    // f32 output for split-K (zeroed)
    const float* in_scale;   // [N, Cin] modulation of the A operand, or null
    Epi e;
    int N, H, W, Cin, Cout, OH, OW;
    int isy, isx;            // input coordinate  = q*is + tap.d
    int wtaps;               // taps per output channel in the packed weight (KH*KW)
    int nck;                 // ceil(Cin / BK)
    int splits, kper;        // K split: kper chunks per split
    int64_t det_stride;      // deterministic mode: split s stores its partial sums at acc + s * det_stride
    int64_t xpl, wpl;        // SG2_F32S3 operands: elements between the h / m / l bf16 planes of x and w
    Phase ph[kMaxPhases];
    Tap taps[kMaxTaps];
};

template <typename T> struct Traits;
template <> struct Traits<float> {
    static constexpr int BK = 16, V = 4;
};
// K-stage of a kernel instance: 32 (one bf16 MFMA K) for the split-f32 form
template <typename T, bool S3> struct KStage { static constexpr int BK = Traits<T>::BK; };
template <> struct KStage<float, true> { static constexpr int BK = 32; };

constexpr int S3LD = 32;              // bf16 plane row pitch (elements, 64 B rows, XOR-swizzled: swz64)

// 16-byte piece q of a 64-byte LDS row r (one 32-element K slice of an A or B tile row): fragment reads of
// 16 consecutive rows hit 16 distinct bank slots in each of ds_read_b128's lane groups
// (tools/lds_swizzle_check.py; the 80-byte padded rows used before conflicted 2-way, SQ_LDS_BANK_CONFLICT
// ~45% of LDS cycles, profiles/r02_v2_pmc_diag.txt).
__device__ __forceinline__ int swz64(int r, int q) { return r * 64 + ((q ^ ((r >> 1) & 2)) << 4); }

// x = h + m + l, three bf16 pieces (exact for normal f32; round-to-nearest at each step)
__device__ __forceinline__ void split3(float x, bf16_t& h, bf16_t& m, bf16_t& l) {
    h = (bf16_t)x;
    float r = x - (float)h;
    m = (bf16_t)r;
    r -= (float)m;
    l = (bf16_t)r;
}

// split3 of four values on packed math: v_cvt_pk_bf16_f32 (round-to-nearest-even, as split3) and
// v_pk_add_f32 residuals, ~4.5 VALU ops per element instead of ~7.5
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef bf16_t bf16x2_t __attribute__((ext_vector_type(2)));
typedef bf16_t bf16x4_s3 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x2_t bf16x2_to_f32(unsigned u) {
    return f32x2_t{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}
__device__ __forceinline__ void split3x4(float x0, float x1, float x2, float x3, bf16x4_s3& h, bf16x4_s3& m,
                                         bf16x4_s3& l) {
    unsigned hu[2], mu[2], lu[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        f32x2_t r = q ? f32x2_t{x2, x3} : f32x2_t{x0, x1};
        hu[q] = __builtin_bit_cast(unsigned, __builtin_convertvector(r, bf16x2_t));
        r = r - bf16x2_to_f32(hu[q]);
        mu[q] = __builtin_bit_cast(unsigned, __builtin_convertvector(r, bf16x2_t));
        r = r - bf16x2_to_f32(mu[q]);
        lu[q] = __builtin_bit_cast(unsigned, __builtin_convertvector(r, bf16x2_t));
    }
    typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
    h = __builtin_bit_cast(bf16x4_s3, u32x2_t{hu[0], hu[1]});
    m = __builtin_bit_cast(bf16x4_s3, u32x2_t{mu[0], mu[1]});
    l = __builtin_bit_cast(bf16x4_s3, u32x2_t{lu[0], lu[1]});
}

// sg2_split3: planes[p * n + i] = piece p of x[i] * scale[n_of(i), i % C]; 8 elements a lane (one 32-byte load, three
// 16-byte stores), the same arithmetic as the kernels' in-loop split (split3x4: round-to-nearest-even residuals)
__global__ __launch_bounds__(256) void split3_kernel(bf16_t* planes, const float* x, int64_t n, int C, int64_t pix_per_n,
                                                     const float* scale) {
    const int64_t groups = n / 8;
    for (int64_t gi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; gi < groups; gi += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = gi * 8;
        const float4 v0 = *(const float4*)(x + i), v1 = *(const float4*)(x + i + 4);
        float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        if (scale) {
            const int64_t pix = i / C;
            const int c = (int)(i - pix * C);
            const float* sp = scale + (pix / pix_per_n) * C + c;
            const float4 s0 = *(const float4*)sp, s1 = *(const float4*)(sp + 4);
            const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = __fmul_rn(v[j], sv[j]);   // the rounded product, as the kernels' staging
        }
        bf16x4_s3 h0, m0, l0, h1, m1, l1;
        split3x4(v[0], v[1], v[2], v[3], h0, m0, l0);
        split3x4(v[4], v[5], v[6], v[7], h1, m1, l1);
        *(bf16x8*)(planes + i) = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
        *(bf16x8*)(planes + n + i) = __builtin_shufflevector(m0, m1, 0, 1, 2, 3, 4, 5, 6, 7);
        *(bf16x8*)(planes + 2 * n + i) = __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7);
    }
}

// acc += a * b over the six significant products of the split operands (small terms first)
__device__ __forceinline__ f32x4 mfma_s3(const bf16x8* a, const bf16x8* b, f32x4 c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], c, 0, 0, 0);
}

// f32 exact mode (SG2_F32_EXACT=1): the f32-input MFMA kernels instead of the bf16 split.  Read per launch
// (an A/B switch that diagnostics flip between calls; one getenv beside a kernel launch)
inline bool f32_exact() {
    const char* e = getenv("SG2_F32_EXACT");
    return e != nullptr && e[0] == '1';
}
template <> struct Traits<f16_t> {
    static constexpr int BK = 32, V = 8;
};
template <> struct Traits<bf16_t> {
    static constexpr int BK = 32, V = 8;
};

typedef short s16x8 __attribute__((ext_vector_type(8)));

template <typename T>
using v8_t = typename std::conditional<std::is_same<T, bf16_t>::value, bf16x8, f16x8>::type;

template <typename T>
__device__ __forceinline__ f32x4 mfma16v(v8_t<T> a, v8_t<T> b, f32x4 c) {
    if constexpr (std::is_same<T, bf16_t>::value)
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

template <typename T>
__device__ __forceinline__ f32x4 mfma16(const T* pa, const T* pb, f32x4 c) {
    if constexpr (std::is_same<T, bf16_t>::value) {
        bf16x8 a = *(const bf16x8*)pa, b = *(const bf16x8*)pb;
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    } else {
        f16x8 a = *(const f16x8*)pa, b = *(const f16x8*)pb;
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    }
}

template <typename T, bool VEC>
struct Loader {
    // A 16-byte chunk of one tile row.  The load itself is unconditional (callers pass a clamped,
    // always-valid row pointer); masking is a select applied when the registers are written to LDS,
    // so no branch sits between the prefetch and the MFMAs (see conv3x3.hip).
    typedef T vecT __attribute__((ext_vector_type(Traits<T>::V)));
    static __device__ __forceinline__ vecT load(const T* row, int c, int Cin) {
        constexpr int V = Traits<T>::V;
        if (VEC) return *(const vecT*)(row + (c < Cin ? c : 0));
        vecT v;
#pragma unroll
        for (int j = 0; j < V; ++j) v[j] = row[(c + j < Cin) ? c + j : 0];
        return v;
    }
    static __device__ __forceinline__ vecT mask(vecT v, int c, int Cin, bool valid) {
        constexpr int V = Traits<T>::V;
#pragma unroll
        for (int j = 0; j < V; ++j) v[j] = (valid && c + j < Cin) ? v[j] : (T)0.f;
        return v;
    }
};

// The fused epilogue of one output element: z = clamp(act(c * out_scale + noise * g + bias) * gain).
template <typename T>
__device__ __forceinline__ float epi_full(const Epi& e, float c, int n, int o, int64_t pix, int Cout) {
    float v = c;
    if (e.out_scale) v *= e.out_scale[(int64_t)n * Cout + o];
    if (e.noise) v += (float)((const T*)e.noise)[pix] * e.noise_gain;
    if (e.bias) v += (float)(T)e.bias[o];        // bias rounded to the activation dtype, as the reference
    if (e.act == 1) v = v > 0.f ? v : v * e.alpha;
    v *= e.gain;
    if (e.clamp >= 0.f) v = fminf(fmaxf(v, -e.clamp), e.clamp);
    return v;
}

// Implicit-GEMM convolution.  grid = (M tiles, Cout tiles, phases * splits).
// 1x1 convolution with a tiny input depth (Cin <= 4: D's fromrgb on 1-channel images): an outer
// product, HBM-bound on the Cout-wide output, so no GEMM tiling -- a lane owns one pixel x 8 output
// channels, reads Cin inputs and 8 x Cin weights, applies the fused epilogue and writes 16 / 32 bytes.
// Same operand rounding as conv_fwd_kernel (x * in_scale rounded to T before the product).
// CK: Cin as a compile-time count (1..4; fromRGB has Cin = img_channels): CK FMAs per output, not four
template <typename T, int CK>
__global__ __launch_bounds__(256) void conv1x1_smallk_kernel(ConvArgs a) {
    typedef T vec8 __attribute__((ext_vector_type(8)));
    const int OG = a.Cout / 8, HW = a.H * a.W;      // the host guarantees 256 % OG == 0: o0 is fixed per lane
    const int64_t total = (int64_t)a.N * HW * OG;
    const T* x = (const T*)a.x;
    const T* w = (const T*)a.w;
    const int o0 = (int)(((int64_t)blockIdx.x * 256 + threadIdx.x) % OG) * 8;
    float wv[8][CK], bj[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int k = 0; k < CK; ++k) wv[j][k] = (float)w[(o0 + j) * CK + k];
        bj[j] = (a.e.on && a.e.bias) ? (float)(T)a.e.bias[o0 + j] : 0.f;
    }
    const bool on = a.e.on;
    const float slope = (on && a.e.act == 1) ? a.e.alpha : 1.f, eg = on ? a.e.gain : 1.f;
    const bool clamp_on = on && a.e.clamp >= 0.f;
    const float cl = a.e.clamp;
    const int aux_mode = on ? a.e.aux_mode : 0;
    const bool i32 = total + (int64_t)gridDim.x * 256 < INT32_MAX;   // 32-bit divisions when they fit
    for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
        const int64_t pix = i32 ? (int64_t)((unsigned)idx / (unsigned)OG) : idx / OG;
        const int n = i32 ? (int)((unsigned)pix / (unsigned)HW) : (int)(pix / HW);
        float xv[CK];
#pragma unroll
        for (int c = 0; c < CK; ++c) {
            float v = (float)x[pix * CK + c];
            if (a.in_scale) v = (float)(T)(v * a.in_scale[(int64_t)n * CK + c]);
            xv[c] = v;
        }
        const float nv = (on && a.e.noise) ? (float)((const T*)a.e.noise)[pix] * a.e.noise_gain : 0.f;
        vec8 yo, ao, rv;
        const bool resid = on && a.e.residual;
        if (resid) rv = *(const vec8*)((const T*)a.e.residual + pix * a.Cout + o0);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float c = 0.f;
#pragma unroll
            for (int k = 0; k < CK; ++k) c += xv[k] * wv[j][k];
            float v = c;
            if (on && a.e.out_scale) v *= a.e.out_scale[(int64_t)n * a.Cout + o0 + j];
            v = v + nv + bj[j];                       // epi_full order: scale, noise, bias, act, gain, clamp
            v = (v > 0.f ? v : v * slope) * eg;
            if (clamp_on) v = fminf(fmaxf(v, -cl), cl);
            ao[j] = (T)(aux_mode == 1 ? c : v);
            if (resid) v = (float)(T)v + (float)rv[j];
            yo[j] = (T)v;
        }
        if (aux_mode) *(vec8*)((T*)a.e.aux + pix * a.Cout + o0) = ao;
        *(vec8*)((T*)a.y + pix * a.Cout + o0) = yo;
    }
}

// The same product with the per-(n, o) dot reduction of a dgrad (toRGB's input gradient with its
// modulation gradient: dot_out[n, o] = sum_p round(c) * dot_src[n, p, o]).  grid = (blocks per sample, N):
// a workgroup owns SK_ITERS x (256 / OG) consecutive pixels of ONE sample, so a lane accumulates its 8
// channels' products in registers, the workgroup combines them in LDS and adds Cout floats to dot_out
// (instead of the implicit GEMM padding K = Cin to 32 and reducing through per-element atomics).
constexpr int SK_ITERS = 16;
template <typename T, int CK>   // CK = Cin (1..4), as in conv1x1_smallk
__global__ __launch_bounds__(256) void conv1x1_smallk_dot_kernel(ConvArgs a) {
    typedef T vec8 __attribute__((ext_vector_type(8)));
    __shared__ float red[2048];
    const int OG = a.Cout / 8, HW = a.H * a.W, PPI = 256 / OG;   // host: 256 % OG == 0
    const int n = blockIdx.y;
    const T* x = (const T*)a.x;
    const T* w = (const T*)a.w;
    const int o0 = (threadIdx.x % OG) * 8;
    float wv[8][CK], bj[8], dacc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int k = 0; k < CK; ++k) wv[j][k] = (float)w[(o0 + j) * CK + k];
        bj[j] = (a.e.on && a.e.bias) ? (float)(T)a.e.bias[o0 + j] : 0.f;
        dacc[j] = 0.f;
    }
    for (int i = threadIdx.x; i < a.Cout; i += 256) red[i] = 0.f;
    const bool on = a.e.on;
    const float slope = (on && a.e.act == 1) ? a.e.alpha : 1.f, eg = on ? a.e.gain : 1.f;
    const bool clamp_on = on && a.e.clamp >= 0.f;
    const float cl = a.e.clamp;
    const int aux_mode = on ? a.e.aux_mode : 0;
    float isc[CK], osc[8];
#pragma unroll
    for (int c = 0; c < CK; ++c) isc[c] = a.in_scale ? a.in_scale[(int64_t)n * CK + c] : 1.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) osc[j] = (on && a.e.out_scale) ? a.e.out_scale[(int64_t)n * a.Cout + o0 + j] : 1.f;
    const int p_begin = blockIdx.x * SK_ITERS * PPI;
#pragma unroll 4
    for (int it = 0; it < SK_ITERS; ++it) {
        const int p = p_begin + it * PPI + threadIdx.x / OG;
        if (p >= HW) break;
        const int64_t pix = (int64_t)n * HW + p;
        float xv[CK];
#pragma unroll
        for (int c = 0; c < CK; ++c) {
            float v = (float)x[pix * CK + c];
            if (a.in_scale) v = (float)(T)(v * isc[c]);
            xv[c] = v;
        }
        const float nv = (on && a.e.noise) ? (float)((const T*)a.e.noise)[pix] * a.e.noise_gain : 0.f;
        const vec8 ds = *(const vec8*)((const T*)a.e.dot_src + pix * a.Cout + o0);
        vec8 yo, ao, rv;
        const bool resid = on && a.e.residual;
        if (resid) rv = *(const vec8*)((const T*)a.e.residual + pix * a.Cout + o0);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float c = 0.f;
#pragma unroll
            for (int k = 0; k < CK; ++k) c += xv[k] * wv[j][k];
            dacc[j] += (float)(T)c * (float)ds[j];
            float v = c * osc[j];
            v = v + nv + bj[j];
            v = (v > 0.f ? v : v * slope) * eg;
            if (clamp_on) v = fminf(fmaxf(v, -cl), cl);
            ao[j] = (T)(aux_mode == 1 ? c : v);
            if (resid) v = (float)(T)v + (float)rv[j];
            yo[j] = (T)v;
        }
        if (aux_mode) *(vec8*)((T*)a.e.aux + pix * a.Cout + o0) = ao;
        *(vec8*)((T*)a.y + pix * a.Cout + o0) = yo;
    }
    __syncthreads();
    if (a.e.det_dot) {
        // rows of PPI lanes' partials, summed in row order; one slot per workgroup
        det_rows_store(red, a.Cout, threadIdx.x / OG, o0, dacc);
        __syncthreads();
        for (int i = threadIdx.x; i < a.Cout; i += 256)
            a.e.det_dot[((int64_t)blockIdx.x * gridDim.y + n) * a.Cout + i] = det_rows_sum(red, a.Cout, PPI, i);
        return;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) atomicAdd(&red[o0 + j], dacc[j]);
    __syncthreads();
    for (int i = threadIdx.x; i < a.Cout; i += 256) atomicAdd(a.e.dot_out + (int64_t)n * a.Cout + i, red[i]);
}

// 1x1 convolution with a tiny output depth (Cout <= 4: G's toRGB, Cin % 8 == 0): a dot product per
// pixel, HBM-bound on the Cin-wide input.  Eight lanes share a pixel, each summing every eighth
// 8-channel chunk (16-byte loads, x * in_scale rounded to T as in conv_fwd_kernel), three xor shuffles
// combine them and the group's first lane applies the epilogue.
template <typename T>
__global__ __launch_bounds__(256) void conv1x1_smallo_kernel(ConvArgs a) {
    typedef T vec8 __attribute__((ext_vector_type(8)));
    const int HW = a.H * a.W, NCH = a.Cin / 8, g = threadIdx.x & 7;
    const int64_t npix = (int64_t)a.N * HW;
    const T* x = (const T*)a.x;
    const T* w = (const T*)a.w;
    const bool on = a.e.on;
    const bool i32 = npix < INT32_MAX;   // 32-bit division when it fits (the 64-bit one is ~40 instructions)
    for (int64_t pix = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 3; pix < npix; pix += (int64_t)gridDim.x * 32) {
        const int n = i32 ? (int)((unsigned)pix / (unsigned)HW) : (int)(pix / HW);
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        for (int ch = g; ch < NCH; ch += 8) {
            vec8 v = *(const vec8*)(x + pix * a.Cin + ch * 8);
            if (a.in_scale) {
                const float4 s0 = *(const float4*)(a.in_scale + (int64_t)n * a.Cin + ch * 8);
                const float4 s1 = *(const float4*)(a.in_scale + (int64_t)n * a.Cin + ch * 8 + 4);
                const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = (T)((float)v[j] * sc[j]);
            }
#pragma unroll
            for (int o = 0; o < 4; ++o) {
                if (o >= a.Cout) break;
                const vec8 wv = *(const vec8*)(w + (int64_t)o * a.Cin + ch * 8);
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[o] += (float)v[j] * (float)wv[j];
            }
        }
#pragma unroll
        for (int o = 0; o < 4; ++o) {
            acc[o] += __shfl_xor(acc[o], 1);
            acc[o] += __shfl_xor(acc[o], 2);
            acc[o] += __shfl_xor(acc[o], 4);
        }
        if (g == 0) {
            for (int o = 0; o < a.Cout; ++o) {
                const float c = acc[o];
                float v = on ? epi_full<T>(a.e, c, n, o, pix, a.Cout) : c;
                if (on && a.e.aux_mode) ((T*)a.e.aux)[pix * a.Cout + o] = (T)(a.e.aux_mode == 1 ? c : v);
                if (on && a.e.residual) v = (float)(T)v + (float)((const T*)a.e.residual)[pix * a.Cout + o];
                ((T*)a.y)[pix * a.Cout + o] = (T)v;
            }
        }
    }
}

// P3 (with S3): the operands arrive pre-split (SG2_F32S3, sg2_split3): three bf16 planes in HBM, loaded as whole
// 16-byte pieces (8 elements a lane) straight into the LDS planes -- no split VALU in the K loop, and each element
// is split once per call instead of once per workgroup that stages it.
template <typename T, int BM, int BN, bool VEC, bool SPLIT, bool SI, bool S3, bool P3 = false>
__global__ __launch_bounds__(256, S3 ? 2 : 3) void conv_fwd_kernel(ConvArgs a) {
    static_assert(!S3 || std::is_same<T, float>::value, "the split form is for f32 operands");
    static_assert(!P3 || (S3 && VEC && !SI), "pre-split operands: the split form, vector loads, scale folded in");
    constexpr int BK = KStage<T, S3>::BK, V = P3 ? 8 : Traits<T>::V;
    constexpr int LPR = BK / V;          // lanes per tile row
    constexpr int RPP = 256 / LPR;       // rows per load pass
    constexpr int PA = BM / RPP, PB = BN / RPP;
    constexpr int LDK = sizeof(T) == 2 ? BK : BK + V;   // 16-bit: 64-byte swizzled rows; f32: padded rows
    constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
    typedef typename Loader<T, VEC>::vecT vecT;

    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    T* lds = (T*)smem_raw;               // [2][(BM + BN) * LDK], reused by the epilogue
    constexpr int BUF = (BM + BN) * LDK;
    // split form: [2][3 planes][(BM + BN) rows][S3LD] bf16
    bf16_t* lds3 = (bf16_t*)smem_raw;
    constexpr int PLANE = (BM + BN) * S3LD, BUF3 = 3 * PLANE;

    const int phase = blockIdx.z / a.splits, split = blockIdx.z - phase * a.splits;
    const int QH = a.ph[phase].QH, QW = a.ph[phase].QW, M = a.ph[phase].M;
    const int tap0 = a.ph[phase].tap0, nk = a.ph[phase].nk;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    if (m0 >= M) return;                 // phases have slightly different M; the whole block leaves

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const T* __restrict__ x = (const T*)a.x;
    const T* __restrict__ w = (const T*)a.w;

    // --- per-thread load geometry (fixed across K) ---
    const int lrow = tid / LPR, lcol = (tid % LPR) * V;
    // 32-bit element offsets (the host checks numel < 2^31): the row base is computed once, each K step
    // adds a uniform tap offset, so the per-row cost of a prefetch is a bounds test and one add
    int a_n[PA], a_qy[PA], a_qx[PA], a_base[PA], b_base[PB];
    bool a_ok[PA], b_ok[PB];
#pragma unroll
    for (int i = 0; i < PA; ++i) {
        const int m = m0 + lrow + i * RPP;
        a_ok[i] = m < M;
        const int mm = a_ok[i] ? m : 0;
        const int per = QH * QW;
        a_n[i] = mm / per;
        const int r = mm - a_n[i] * per;
        a_qy[i] = (r / QW) * a.isy;
        a_qx[i] = (r % QW) * a.isx;
        a_base[i] = ((a_n[i] * a.H + a_qy[i]) * a.W + a_qx[i]) * a.Cin;
    }
    const int wrow = a.wtaps * a.Cin;
#pragma unroll
    for (int i = 0; i < PB; ++i) {
        const int o = n0 + lrow + i * RPP;
        b_ok[i] = o < a.Cout;
        b_base[i] = (b_ok[i] ? o : 0) * wrow;
    }

    const int k_begin = split * a.kper;
    const int k_end = min(nk, k_begin + a.kper);

    const __amdgpu_buffer_rsrc_t rx = make_rsrc(x, P3 ? 6 * a.xpl : (int64_t)a.N * a.H * a.W * a.Cin * (int64_t)sizeof(T));
    const __amdgpu_buffer_rsrc_t rw = make_rsrc(w, P3 ? 6 * a.wpl : (int64_t)a.Cout * wrow * (int64_t)sizeof(T));
    const int xplb = (int)(2 * a.xpl), wplb = (int)(2 * a.wpl);   // plane strides in bytes (P3)
    bf16x8 r3a[P3 ? PA : 1][3], r3b[P3 ? PB : 1][3];
    vecT ra[PA], rb[PB];
    bool ra_ok[PA], rb_ok[PB];
    float rsc[SI ? PA : 1][V];
    int cur_c = 0;
    auto gload = [&](int kc) {
        const int t = kc / a.nck;
        const int c = (kc - t * a.nck) * BK + lcol;
        cur_c = c;
        const Tap tp = a.taps[tap0 + t];
        const int dy = tp.dy, dx = tp.dx, wt = tp.w;
        const int tapoff = (dy * a.W + dx) * a.Cin;
        if constexpr (P3) {
#pragma unroll
            for (int i = 0; i < PA; ++i) {
                const int iy = a_qy[i] + dy, ix = a_qx[i] + dx;
                const bool ok = a_ok[i] && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W && c < a.Cin;
                const int off = ok ? (a_base[i] + tapoff + c) * 2 : -1;
#pragma unroll
                for (int p = 0; p < 3; ++p) r3a[i][p] = buf_load16<bf16x8>(rx, ok ? off + p * xplb : -1);
            }
            const int woff = wt * a.Cin;
#pragma unroll
            for (int i = 0; i < PB; ++i) {
                const bool ok = b_ok[i] && c < a.Cin;
                const int off = ok ? (b_base[i] + woff + c) * 2 : -1;
#pragma unroll
                for (int p = 0; p < 3; ++p) r3b[i][p] = buf_load16<bf16x8>(rw, ok ? off + p * wplb : -1);
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < PA; ++i) {
            const int iy = a_qy[i] + dy, ix = a_qx[i] + dx;
            const bool ok = a_ok[i] && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
            ra_ok[i] = ok;
            if constexpr (VEC)   // out-of-range buffer offset: the hardware returns zeros, no mask
                ra[i] = buf_load16<vecT>(rx, ok && c < a.Cin ? (a_base[i] + tapoff + c) * (int)sizeof(T) : -1);
            else
                ra[i] = Loader<T, VEC>::load(x + (ok ? a_base[i] + tapoff : 0), c, a.Cin);
            if (SI) {
                const float* sp = a.in_scale + (int64_t)a_n[i] * a.Cin;
                if constexpr (VEC) {   // c % V == 0 and Cin % V == 0: whole float4s (clamped to the row start)
                    const float* q = sp + (c < a.Cin ? c : 0);
#pragma unroll
                    for (int j = 0; j < V; j += 4) {
                        const float4 f = *(const float4*)(q + j);
                        rsc[i][j] = f.x; rsc[i][j + 1] = f.y; rsc[i][j + 2] = f.z; rsc[i][j + 3] = f.w;
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < V; ++j) rsc[i][j] = sp[c + j < a.Cin ? c + j : 0];
                }
            }
        }
        const int woff = wt * a.Cin;
#pragma unroll
        for (int i = 0; i < PB; ++i) {
            rb_ok[i] = b_ok[i];
            if constexpr (VEC)
                rb[i] = buf_load16<vecT>(rw, b_ok[i] && c < a.Cin ? (b_base[i] + woff + c) * (int)sizeof(T) : -1);
            else
                rb[i] = Loader<T, VEC>::load(w + b_base[i] + woff, c, a.Cin);
        }
    };
    typedef bf16_t bf16x4_t __attribute__((ext_vector_type(4)));
    // split-f32 staging: row r of the buffer (A rows first, then B) gets the three planes of v
    auto store3 = [&](int buf, int r, const vecT& v) {
        bf16x4_t h, m, l;
        split3x4((float)v[0], (float)v[1], (float)v[2], (float)v[3], h, m, l);
        bf16_t* p = (bf16_t*)((char*)(lds3 + buf * BUF3) + swz64(r, lcol >> 3) + (lcol & 7) * 2);
        *(bf16x4_t*)p = h;
        *(bf16x4_t*)(p + PLANE) = m;
        *(bf16x4_t*)(p + 2 * PLANE) = l;
    };
    auto sstore = [&](int buf) {
        if constexpr (P3) {   // whole 16-byte pieces of each plane, the same swizzled rows as store3
            char* P = (char*)(lds3 + buf * BUF3);
#pragma unroll
            for (int i = 0; i < PA; ++i)
#pragma unroll
                for (int p = 0; p < 3; ++p) *(bf16x8*)(P + p * PLANE * 2 + swz64(lrow + i * RPP, lcol >> 3)) = r3a[i][p];
#pragma unroll
            for (int i = 0; i < PB; ++i)
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    *(bf16x8*)(P + p * PLANE * 2 + swz64(BM + lrow + i * RPP, lcol >> 3)) = r3b[i][p];
            return;
        }
        T* As = lds + buf * BUF;
        T* Bs = As + BM * LDK;
#pragma unroll
        for (int i = 0; i < PA; ++i) {
            vecT v = VEC ? ra[i] : Loader<T, VEC>::mask(ra[i], cur_c, a.Cin, ra_ok[i]);
            if (SI) {
#pragma unroll
                for (int j = 0; j < V; ++j) v[j] = (T)__fmul_rn((float)v[j], rsc[i][j]);   // rounded product (no fma contraction)
            }
            if constexpr (S3) store3(buf, lrow + i * RPP, v);
            else if constexpr (sizeof(T) == 2) *(vecT*)((char*)As + swz64(lrow + i * RPP, lcol >> 3)) = v;
            else *(vecT*)(As + (lrow + i * RPP) * LDK + lcol) = v;
        }
#pragma unroll
        for (int i = 0; i < PB; ++i) {
            const vecT v = VEC ? rb[i] : Loader<T, VEC>::mask(rb[i], cur_c, a.Cin, rb_ok[i]);
            if constexpr (S3) store3(buf, BM + lrow + i * RPP, v);
            else if constexpr (sizeof(T) == 2) *(vecT*)((char*)Bs + swz64(lrow + i * RPP, lcol >> 3)) = v;
            else *(vecT*)(Bs + (lrow + i * RPP) * LDK + lcol) = v;
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto compute = [&](int cur) {
        const T* As = lds + cur * BUF + (wm * WM) * LDK;
        const T* Bs = lds + cur * BUF + BM * LDK + (wn * WN) * LDK;
        if constexpr (S3) {
            const char* P = (const char*)(lds3 + cur * BUF3);
            const int fl = swz64(lane & 15, lane >> 4);          // + 64 * (16-aligned row): the same swizzle
            bf16x8 af[TM][3], bfr[TN][3];
#pragma unroll
            for (int q = 0; q < 3; ++q) {
#pragma unroll
                for (int i = 0; i < TM; ++i)
                    af[i][q] = *(const bf16x8*)(P + q * PLANE * 2 + (wm * WM + i * 16) * 64 + fl);
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    bfr[j][q] = *(const bf16x8*)(P + q * PLANE * 2 + (BM + wn * WN + j * 16) * 64 + fl);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j] = mfma_s3(af[i], bfr[j], acc[i][j]);
        } else if constexpr (std::is_same<T, float>::value) {
#pragma unroll
            for (int kk = 0; kk < BK; kk += 4) {
                float af[TM], bfr[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) af[i] = As[(i * 16 + (lane & 15)) * LDK + kk + (lane >> 4)];
#pragma unroll
                for (int j = 0; j < TN; ++j) bfr[j] = Bs[(j * 16 + (lane & 15)) * LDK + kk + (lane >> 4)];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
            }
        } else {
            const int fl = swz64(lane & 15, lane >> 4);          // rows 16-aligned: the same swizzle
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = mfma16<T>((const T*)((const char*)As + i * 16 * 64 + fl),
                                          (const T*)((const char*)Bs + j * 16 * 64 + fl), acc[i][j]);
        }
    };
    if (k_begin < k_end) {
        if constexpr (S3) {
            // one LDS buffer (the three bf16 planes of a K tile are 61 KB): two workgroups per CU, the
            // next tile's global loads in flight during this tile's MFMAs
            gload(k_begin);
            for (int kc = k_begin; kc < k_end; ++kc) {
                const bool more = kc + 1 < k_end;
                sstore(0);
                __syncthreads();
                if (more) gload(kc + 1);
                compute(0);
                __syncthreads();
            }
        } else {
            gload(k_begin);
            sstore(0);
            __syncthreads();
            for (int kc = k_begin; kc < k_end; ++kc) {
                const int cur = (kc - k_begin) & 1;
                const bool more = kc + 1 < k_end;
                if (more) gload(kc + 1);
                compute(cur);
                if (more) sstore(cur ^ 1);
                __syncthreads();
            }
        }
    }

    // --- epilogue ---
    const int per = QH * QW;
    const int osy = a.ph[phase].osy, osx = a.ph[phase].osx, oy0 = a.ph[phase].oy0, ox0 = a.ph[phase].ox0;
    if (SPLIT || std::is_same<T, float>::value) {
        // f32 tiles / split-K partial sums: direct stores (the split-K epilogue runs in the finalize kernel)
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm * WM + i * 16 + 4 * (lane >> 4) + r;
                if (m >= M) continue;
                const int n = m / per;
                const int rr = m - n * per;
                const int oy = (rr / QW) * osy + oy0, ox = (rr % QW) * osx + ox0;
                const int64_t pix = ((int64_t)n * a.OH + oy) * a.OW + ox;
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int o = n0 + wn * WN + j * 16 + (lane & 15);
                    if (o >= a.Cout) continue;
                    const float c = acc[i][j][r];
                    if (SPLIT) {
                        if (a.det_stride) a.acc[split * a.det_stride + pix * a.Cout + o] = c;
                        else atomicAdd(a.acc + pix * a.Cout + o, c);
                    } else {
                        float v = c;
                        if (a.e.dot_out) {
                            const float pr = c * (float)((const T*)a.e.dot_src)[pix * a.Cout + o];
                            if (a.e.det_dot) a.e.det_dot[pix * a.Cout + o] = pr;
                            else atomicAdd(a.e.dot_out + (int64_t)n * a.Cout + o, pr);
                        }
                        if (a.e.on) {
                            v = epi_full<T>(a.e, c, n, o, pix, a.Cout);
                            if (a.e.aux_mode == 1) ((T*)a.e.aux)[pix * a.Cout + o] = (T)c;
                            if (a.e.aux_mode == 2) ((T*)a.e.aux)[pix * a.Cout + o] = (T)v;
                            if (a.e.residual) v = (float)(T)v + (float)((const T*)a.e.residual)[pix * a.Cout + o];
                        }
                        ((T*)a.y)[pix * a.Cout + o] = (T)v;
                    }
                }
            }
        }
        return;
    }
    // 16-bit: epilogue math in registers, tile transposed through LDS (64 columns at a time, inside
    // the main loop's LDS budget so occupancy is unchanged), 16-byte row stores
    constexpr int EH = 64, NHALF = BN / EH, OS = EH + 8, CPR = EH / 8;
    T* ot = lds;                 // [BM][OS]
    T* xt = lds + BM * OS;       // [BM][OS] aux tile (also holds c for the dot reduction)
    float* red = (float*)(lds + 2 * BM * OS);   // [EH] dot partial sums
    const bool want_aux = a.e.on && a.e.aux_mode != 0;
    const bool want_dot = a.e.dot_out != nullptr;
    const bool det_dot = a.e.det_dot != nullptr;
    const bool keep_c = want_aux || want_dot;
    // the dot reduction goes through LDS when the whole tile belongs to one sample
    const int n_first = m0 / per, n_last = (min(m0 + BM, M) - 1) / per;
    const bool dot_uniform = n_first == n_last;
    float bj[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int o = min(n0 + wn * WN + j * 16 + (lane & 15), a.Cout - 1);
        bj[j] = (a.e.on && a.e.bias) ? (float)(T)a.e.bias[o] : 0.f;
    }
    typedef T vec8o __attribute__((ext_vector_type(8)));
    const bool cvec = (a.Cout % 8) == 0;
#pragma unroll
    for (int h = 0; h < NHALF; ++h) {
        if (h) __syncthreads();                      // the previous half's stores have read the tile
        if (wn * WN >= h * EH && wn * WN < (h + 1) * EH) {
#pragma unroll
            for (int i = 0; i < TM; ++i) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int ml = wm * WM + i * 16 + 4 * (lane >> 4) + r;
                    const int m = min(m0 + ml, M - 1);
                    const int n = m / per;
                    const int rr = m - n * per;
                    const int oy = (rr / QW) * osy + oy0, ox = (rr % QW) * osx + ox0;
                    const int64_t pix = ((int64_t)n * a.OH + oy) * a.OW + ox;
                    const float nv = (a.e.on && a.e.noise) ? (float)((const T*)a.e.noise)[pix] * a.e.noise_gain : 0.f;
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        const int ol = wn * WN + j * 16 + (lane & 15);
                        const int o = min(n0 + ol, a.Cout - 1);
                        const float c = acc[i][j][r];
                        float v = c;
                        if (a.e.on) {
                            if (a.e.out_scale) v *= a.e.out_scale[(int64_t)n * a.Cout + o];
                            v += nv + bj[j];
                            if (a.e.act == 1) v = v > 0.f ? v : v * a.e.alpha;
                            v *= a.e.gain;
                            if (a.e.clamp >= 0.f) v = fminf(fmaxf(v, -a.e.clamp), a.e.clamp);
                        }
                        ot[ml * OS + ol - h * EH] = (T)v;
                        if (keep_c) xt[ml * OS + ol - h * EH] = (T)(a.e.aux_mode == 2 ? v : c);
                    }
                }
            }
        }
        if (want_dot && tid < EH) red[tid] = 0.f;
        __syncthreads();
        float dacc[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) dacc[e] = 0.f;
#pragma unroll
        for (int k = 0; k < BM * CPR / 256; ++k) {
            const int idx = tid + k * 256;
            const int ml = idx / CPR, c8 = (idx % CPR) * 8;
            const int m = m0 + ml, o = n0 + h * EH + c8;
            if (m >= M || o >= a.Cout) continue;
            if (want_dot) {
                const int n = m / per;
                const int rr = m - n * per;
                const int oy = (rr / QW) * osy + oy0, ox = (rr % QW) * osx + ox0;
                const int64_t src = (((int64_t)n * a.OH + oy) * a.OW + ox) * a.Cout + o;
                for (int e = 0; e < 8 && o + e < a.Cout; ++e) {
                    const float pr = (float)xt[ml * OS + c8 + e] * (float)((const T*)a.e.dot_src)[src + e];
                    if (det_dot) a.e.det_dot[src + e] = pr;
                    else if (dot_uniform) dacc[e] += pr;
                    else atomicAdd(a.e.dot_out + (int64_t)n * a.Cout + o + e, pr);
                }
            }
            const int n = m / per;
            const int rr = m - n * per;
            const int oy = (rr / QW) * osy + oy0, ox = (rr % QW) * osx + ox0;
            const int64_t dst = (((int64_t)n * a.OH + oy) * a.OW + ox) * a.Cout + o;
            if (cvec) {
                vec8o v = *(const vec8o*)(ot + ml * OS + c8);
                if (a.e.on && a.e.residual) {
                    const vec8o rv = *(const vec8o*)((const T*)a.e.residual + dst);
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] = (T)((float)v[e] + (float)rv[e]);
                }
                *(vec8o*)((T*)a.y + dst) = v;
                if (want_aux) *(vec8o*)((T*)a.e.aux + dst) = *(const vec8o*)(xt + ml * OS + c8);
            } else {
                for (int e = 0; e < 8 && o + e < a.Cout; ++e) {
                    float v = (float)ot[ml * OS + c8 + e];
                    if (a.e.on && a.e.residual) v += (float)((const T*)a.e.residual)[dst + e];
                    ((T*)a.y)[dst + e] = (T)v;
                    if (want_aux) ((T*)a.e.aux)[dst + e] = xt[ml * OS + c8 + e];
                }
            }
        }
        if (want_dot && dot_uniform && !det_dot) {
            const int c8 = (tid % CPR) * 8;
#pragma unroll
            for (int e = 0; e < 8; ++e) atomicAdd(&red[c8 + e], dacc[e]);
            __syncthreads();
            const int o = n0 + h * EH + tid;
            if (tid < EH && o < a.Cout) atomicAdd(a.e.dot_out + (int64_t)n_first * a.Cout + o, red[tid]);
        }
    }
}

// Split-K finalize: f32 partial sums -> T with the fused epilogue.
template <typename T>
__global__ void conv_finalize_kernel(T* y, float* src, const float* slots, int nslots, Epi e, int64_t n_el, int Cout,
                                     int64_t pix_per_n, int clean) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_el; i += (int64_t)gridDim.x * blockDim.x) {
        float c;
        if (slots) {                             // deterministic mode: the splits' partial sums in split order
            c = 0.f;
            for (int k = 0; k < nslots; ++k) c += slots[(int64_t)k * n_el + i];
        } else {
            c = src[i];
            if (clean) src[i] = 0.f;             // leave the workspace zeroed for the next split-K call
        }
        float v = c;
        if (e.dot_out) {
            const int64_t pix = i / Cout;
            const int o = (int)(i - pix * Cout);
            const float pr = c * (float)((const T*)e.dot_src)[i];
            if (e.det_dot) e.det_dot[i] = pr;
            else atomicAdd(e.dot_out + (pix / pix_per_n) * Cout + o, pr);
        }
        if (e.on) {
            const int64_t pix = i / Cout;
            const int o = (int)(i - pix * Cout);
            const int n = (int)(pix / pix_per_n);
            v = epi_full<T>(e, c, n, o, pix, Cout);
            if (e.aux_mode == 1) ((T*)e.aux)[i] = (T)c;
            if (e.aux_mode == 2) ((T*)e.aux)[i] = (T)v;
            if (e.residual) v = (float)(T)v + (float)((const T*)e.residual)[i];
        }
        y[i] = (T)v;
    }
}

template <typename T, int BM, int BN, bool S3>
size_t fwd_lds_bytes() {
    constexpr int BK = Traits<T>::BK, V = Traits<T>::V;
    if (S3) return 3 * (size_t)(BM + BN) * S3LD * sizeof(bf16_t);   // one buffer (conv_fwd_kernel S3 loop)
    const size_t main = 2 * (size_t)(BM + BN) * (sizeof(T) == 2 ? BK : BK + V) * sizeof(T);
    const size_t epi = std::is_same<T, float>::value ? 0 : 2 * (size_t)BM * (64 + 8) * sizeof(T) + 64 * sizeof(float);
    return std::max(main, epi);
}

template <typename T, int BM, int BN, bool VEC, bool SPLIT, bool SI, bool S3, bool P3 = false>
int launch_fwd_k(ConvArgs& a, dim3 grid, hipStream_t s) {
    auto kern = conv_fwd_kernel<T, BM, BN, VEC, SPLIT, SI, S3, P3>;
    const size_t lds = fwd_lds_bytes<T, BM, BN, S3>();
    static bool attr_set = false;   // benign race: idempotent attribute
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr_set = true;
    }
    kern<<<grid, 256, lds, s>>>(a);
    return launch_status("sg2_conv2d");
}

template <typename T, int BM, int BN>
int launch_fwd(ConvArgs& a, bool vec, hipStream_t s) {
    int maxM = 0;
    int nph = 0;
    for (int i = 0; i < kMaxPhases; ++i)
        if (a.ph[i].M > 0) { maxM = std::max(maxM, a.ph[i].M); nph = i + 1; }
    dim3 grid((unsigned)cdiv(maxM, BM), (unsigned)cdiv(a.Cout, BN), (unsigned)(nph * a.splits));
    constexpr bool F32 = std::is_same<T, float>::value;
    if (F32 && a.xpl) {      // pre-split operands (SG2_F32S3)
        if (a.splits > 1) return launch_fwd_k<T, BM, BN, true, true, false, F32, F32>(a, grid, s);
        return launch_fwd_k<T, BM, BN, true, false, false, F32, F32>(a, grid, s);
    }
    if (F32 && !f32_exact()) {
#define LF(V_, S_) return a.in_scale ? launch_fwd_k<T, BM, BN, V_, S_, true, F32>(a, grid, s) \
                                     : launch_fwd_k<T, BM, BN, V_, S_, false, F32>(a, grid, s)
        if (a.splits > 1) { if (vec) LF(true, true); else LF(false, true); }
        if (vec) LF(true, false); else LF(false, false);
#undef LF
    }
#define LF(V_, S_) return a.in_scale ? launch_fwd_k<T, BM, BN, V_, S_, true, false>(a, grid, s) \
                                     : launch_fwd_k<T, BM, BN, V_, S_, false, false>(a, grid, s)
    if (a.splits > 1) { if (vec) LF(true, true); else LF(false, true); }
    if (vec) LF(true, false); else LF(false, false);
#undef LF
}

// ------------------------------------------------------------------------------------ wgrad

struct WgradArgs {
    int oikk;            // sg2_conv2d_wgrad_oikk: the final slot sum writes dw as [A][B][KH][KW] (2: [B][A][KH][KW])
    const void* g;   // [N, OH, OW, A]
    const void* x;   // [N, H, W, B]
    float* dw;       // [A][KK][B]
    const float* b_scale;   // optional [N, B]: x operand multiplied by b_scale[n, b]
    const float* a_scale;   // optional [N, A]: g operand multiplied by a_scale[n, a]
    int N, A, OH, OW, B, H, W, KH, KW, stride, pady, padx;
    int M;           // N*OH*OW
    int kper;        // pixels per split (multiple of BK)
    int splits;
    float alpha;     // dw += alpha * (partial sums): a layer's weight gain folded in
    float* det;      // deterministic mode: partial sums by slot (split / lane row), summed by det_sum
    int64_t gpl, xpl;   // SG2_F32S3 operands: elements between the h / m / l bf16 planes of g and x
};

template <typename T>
__device__ __forceinline__ v8_t<T> frag_tr(const T* base, int ld, int k0, int c0, int lane) {
    // element j = base[(k0 + 8*(lane>>4) + j) * ld + c0 + (lane & 15)],  j = 0..7  (ds_read_b64_tr_b16)
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const T* p0 = base + (k0 + 8 * g + q) * ld + c0 + 4 * p;
    const T* p1 = p0 + 4 * ld;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p0);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p1);
    s16x8 r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(v8_t<T>, r);
}

// Weight gradient of a 1x1 convolution with a tiny input depth (B <= 4, fromrgb): dw[a][b] =
// sum_p g[p,a] x[p,b] is a reduction of the A-wide gradient over all pixels, HBM-bound on g.  A lane
// owns 8 output channels (fixed, as the grid stride is a multiple of A/8) and accumulates over its
// pixels in registers; the block reduces through LDS and adds once per element to dw (zeroed).
// BT: B as a compile-time count (1..4; the fromRGB weight gradient has B = img_channels); IDX: 32-bit index
// math when it fits; the g operand's modulation row a_scale[n, a0 .. a0 + 7] is re-read only when the sample
// changes (re-reading it per pixel doubled the load traffic, as in wgrad1x1_smalla).
template <typename T, int BT, typename IDX>
__global__ __launch_bounds__(256) void wgrad1x1_smallb_kernel(WgradArgs a) {
    typedef T vec8 __attribute__((ext_vector_type(8)));
    __shared__ float red[2048];                       // [A][B], A * B <= 2048
    const IDX OG = (IDX)(a.A / 8);
    for (int i = threadIdx.x; i < a.A * BT; i += 256) red[i] = 0.f;
    __syncthreads();
    const IDX total = (IDX)((int64_t)a.M * (a.A / 8));
    const IDX per = (IDX)(a.OH * a.OW);
    const T* g = (const T*)a.g;
    const T* x = (const T*)a.x;
    IDX idx = (IDX)blockIdx.x * 256 + threadIdx.x;
    const int a0 = (int)(idx % OG) * 8;
    float acc[8][BT];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int k = 0; k < BT; ++k) acc[j][k] = 0.f;
    int cur_n = -1;
    float as[8];
    for (; idx < total; idx += (IDX)gridDim.x * 256) {
        const IDX pix = idx / OG;
        const int n = (int)(pix / per);
        const vec8 gv = *(const vec8*)(g + (int64_t)pix * a.A + a0);
        float xv[BT];
#pragma unroll
        for (int k = 0; k < BT; ++k) {
            float v = (float)x[(int64_t)pix * BT + k];
            if (a.b_scale) v = (float)(T)(v * a.b_scale[(int64_t)n * BT + k]);
            xv[k] = v;
        }
        if (a.a_scale && n != cur_n) {
#pragma unroll
            for (int j = 0; j < 8; ++j) as[j] = a.a_scale[(int64_t)n * a.A + a0 + j];
            cur_n = n;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float gj = (float)gv[j];
            if (a.a_scale) gj = (float)(T)(gj * as[j]);
#pragma unroll
            for (int k = 0; k < BT; ++k) acc[j][k] += gj * xv[k];
        }
    }
    if (a.det) {
        // one slot per row of OG lanes (every lane of a row owns 8 distinct a): [row][A][B]
        const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / (a.A / 8);
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int k = 0; k < BT; ++k) a.det[row * a.A * BT + (a0 + j) * BT + k] = acc[j][k] * a.alpha;
        return;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int k = 0; k < BT; ++k) atomicAdd(&red[(a0 + j) * BT + k], acc[j][k]);
    __syncthreads();
    for (int i = threadIdx.x; i < a.A * BT; i += 256) atomicAdd(a.dw + i, red[i] * a.alpha);
}

// Mirror for a tiny output depth (A <= 4, toRGB): the lane owns 8 input channels b of the wide x.
// AT: A as a compile-time count (1..4; the toRGB weight gradient has A = img_channels), so a pixel costs A FMAs
// per element rather than four; IDX: unsigned 32-bit index math when M * B / 8 < 2^31 (the host checks) --
// the 64-bit divisions that split the flat index into (pixel, sample) cost more than the FMAs.
template <typename T, int AT, typename IDX>
__global__ __launch_bounds__(256) void wgrad1x1_smalla_kernel(WgradArgs a) {
    typedef T vec8 __attribute__((ext_vector_type(8)));
    __shared__ float red[2048];                       // [A][B], A * B <= 2048
    const IDX BG = (IDX)(a.B / 8);
    for (int i = threadIdx.x; i < AT * a.B; i += 256) red[i] = 0.f;
    __syncthreads();
    const IDX total = (IDX)((int64_t)a.M * (a.B / 8));
    const IDX per = (IDX)(a.OH * a.OW);
    const T* g = (const T*)a.g;
    const T* x = (const T*)a.x;
    IDX idx = (IDX)blockIdx.x * 256 + threadIdx.x;
    const int b0 = (int)(idx % BG) * 8;
    float acc[AT][8];
#pragma unroll
    for (int k = 0; k < AT; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
    // U pixels per trip with all their loads issued first (one 16-byte load in flight per lane left the
    // kernel latency-bound at ~1.4 TB/s); the accumulation order is the plain loop's
    constexpr int U = 4;
    const IDX stride = (IDX)gridDim.x * 256;
    // the x operand's modulation row b_scale[n, b0 .. b0 + 7] is re-read only when the sample changes
    int cur_n = -1;
    float bs[8];
    auto body = [&](const vec8& xv, const float* graw, IDX pix) {
        const int n = (int)(pix / per);
        if (a.b_scale && n != cur_n) {
#pragma unroll
            for (int j = 0; j < 8; ++j) bs[j] = a.b_scale[(int64_t)n * a.B + b0 + j];
            cur_n = n;
        }
        float gk[AT];
#pragma unroll
        for (int k = 0; k < AT; ++k) {
            float v = graw[k];
            if (a.a_scale) v = (float)(T)(v * a.a_scale[(int64_t)n * AT + k]);
            gk[k] = v;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float xj = (float)xv[j];
            if (a.b_scale) xj = (float)(T)(xj * bs[j]);
#pragma unroll
            for (int k = 0; k < AT; ++k) acc[k][j] += gk[k] * xj;
        }
    };
    for (; idx + (U - 1) * stride < total; idx += U * stride) {
        vec8 xv[U];
        float gr[U][AT];
        IDX pix[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            pix[u] = (idx + u * stride) / BG;
            xv[u] = *(const vec8*)(x + (int64_t)pix[u] * a.B + b0);
#pragma unroll
            for (int k = 0; k < AT; ++k) gr[u][k] = (float)g[(int64_t)pix[u] * AT + k];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) body(xv[u], gr[u], pix[u]);
    }
    for (; idx < total; idx += stride) {
        const IDX pix = idx / BG;
        float gr[AT];
#pragma unroll
        for (int k = 0; k < AT; ++k) gr[k] = (float)g[(int64_t)pix * AT + k];
        body(*(const vec8*)(x + (int64_t)pix * a.B + b0), gr, pix);
    }
    if (a.det) {
        const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / (a.B / 8);
#pragma unroll
        for (int k = 0; k < AT; ++k)
#pragma unroll
            for (int j = 0; j < 8; ++j) a.det[row * AT * a.B + k * a.B + b0 + j] = acc[k][j] * a.alpha;
        return;
    }
#pragma unroll
    for (int k = 0; k < AT; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) atomicAdd(&red[k * a.B + b0 + j], acc[k][j]);
    __syncthreads();
    for (int i = threadIdx.x; i < AT * a.B; i += 256) atomicAdd(a.dw + i, red[i] * a.alpha);
}

template <typename T, int BM, int BN, bool VEC, bool S3, bool P3 = false>
__global__ __launch_bounds__(256, S3 ? 2 : 1) void conv_wgrad_kernel(WgradArgs a) {
    static_assert(!S3 || std::is_same<T, float>::value, "the split form is for f32 operands");
    static_assert(!P3 || (S3 && VEC), "pre-split operands: the split form with vector loads");
    constexpr int BK = KStage<T, S3>::BK, V = P3 ? 8 : Traits<T>::V;
    constexpr int LDA = BM + V, LDB = BN + V;   // padded pixel-major rows
    constexpr int LPA = BM / V, LPB = BN / V;   // lanes per row
    constexpr int RPA = 256 / LPA, RPB = 256 / LPB;
    constexpr int PA = (BK + RPA - 1) / RPA, PB = (BK + RPB - 1) / RPB;
    constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
    typedef typename Loader<T, VEC>::vecT vecT;
    // split form: [2][3 planes][BK][LDA3 + LDB3] bf16, pixel-major, read with ds_read_b64_tr_b16
    constexpr int LDA3 = BM + 8, LDB3 = BN + 8, PL3 = BK * (LDA3 + LDB3);
    // S3: one buffer (52 KB of bf16 planes; the loop below is single-buffered), three workgroups per CU
    constexpr size_t BYTES = S3 ? 3 * (size_t)PL3 * 2 : 2 * (size_t)BK * (LDA + LDB) * sizeof(T);

    __shared__ __attribute__((aligned(16))) char lds_raw[BYTES];
    typedef T Row[BK * (LDA + LDB)];
    Row* lds = (Row*)lds_raw;
    bf16_t* lds3 = (bf16_t*)lds_raw;
    typedef bf16_t bf16x4_t __attribute__((ext_vector_type(4)));
    auto store3 = [&](int buf, int off, const vecT& v) {
        bf16x4_t h, m, l;
        split3x4((float)v[0], (float)v[1], (float)v[2], (float)v[3], h, m, l);
        bf16_t* p = lds3 + buf * 3 * PL3 + off;
        *(bf16x4_t*)p = h;
        *(bf16x4_t*)(p + PL3) = m;
        *(bf16x4_t*)(p + 2 * PL3) = l;
    };

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int a0 = blockIdx.x * BM, b0 = blockIdx.y * BN;
    const int tap = blockIdx.z / a.splits, split = blockIdx.z % a.splits;
    const int ky = tap / a.KW, kx = tap % a.KW;
    const T* __restrict__ g = (const T*)a.g;
    const T* __restrict__ x = (const T*)a.x;
    const __amdgpu_buffer_rsrc_t rgw = make_rsrc(g, P3 ? 6 * a.gpl : (int64_t)a.M * a.A * (int64_t)sizeof(T));
    const __amdgpu_buffer_rsrc_t rxw = make_rsrc(x, P3 ? 6 * a.xpl : (int64_t)a.N * a.H * a.W * a.B * (int64_t)sizeof(T));
    const int gplb = (int)(2 * a.gpl), xplb = (int)(2 * a.xpl);
    bf16x8 r3a[P3 ? PA : 1][3], r3b[P3 ? PB : 1][3];

    const int ga_row = tid / LPA, ga_col = (tid % LPA) * V;
    const int xb_row = tid / LPB, xb_col = (tid % LPB) * V;
    const int p_begin = split * a.kper;
    const int p_end = min(a.M, p_begin + a.kper);

    vecT ra[PA], rb[PB];
    bool ra_ok[PA], rb_ok[PB];
    float rsc[PB][V], asc[PA][V];
    auto gload = [&](int p0) {
        if constexpr (P3) {   // scales folded into the planes by sg2_split3
#pragma unroll
            for (int i = 0; i < PA; ++i) {
                const int r = ga_row + i * RPA;
                const int m = p0 + r;
                const bool ok = r < BK && m < p_end && a0 + ga_col < a.A;
                const int off = ok ? (m * a.A + a0 + ga_col) * 2 : -1;
#pragma unroll
                for (int q = 0; q < 3; ++q) r3a[i][q] = buf_load16<bf16x8>(rgw, ok ? off + q * gplb : -1);
            }
#pragma unroll
            for (int i = 0; i < PB; ++i) {
                const int r = xb_row + i * RPB;
                const int m = p0 + r;
                bool ok = r < BK && m < p_end;
                const int mm = ok ? m : 0;
                const int per = a.OH * a.OW;
                const int n = mm / per;
                const int rr = mm - n * per;
                const int iy = (rr / a.OW) * a.stride + ky - a.pady, ix = (rr % a.OW) * a.stride + kx - a.padx;
                ok = ok && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W && b0 + xb_col < a.B;
                const int off = ok ? (((n * a.H + iy) * a.W + ix) * a.B + b0 + xb_col) * 2 : -1;
#pragma unroll
                for (int q = 0; q < 3; ++q) r3b[i][q] = buf_load16<bf16x8>(rxw, ok ? off + q * xplb : -1);
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < PA; ++i) {
            const int r = ga_row + i * RPA;
            const int m = p0 + r;
            const bool ok = r < BK && m < p_end;
            ra_ok[i] = ok;
            if constexpr (VEC) {
                ra[i] = buf_load16<vecT>(rgw, ok && a0 + ga_col < a.A ? (m * a.A + a0 + ga_col) * (int)sizeof(T) : -1);
            } else {
                const T* row = g + (int64_t)(ok ? m : 0) * a.A;
                ra[i] = Loader<T, VEC>::load(row, a0 + ga_col, a.A);
            }
            if (a.a_scale) {
                const int n = (ok ? m : 0) / (a.OH * a.OW);
                const float* sp = a.a_scale + (int64_t)n * a.A;
                if constexpr (VEC) {
                    const float* q = sp + (a0 + ga_col < a.A ? a0 + ga_col : 0);
#pragma unroll
                    for (int j = 0; j < V; j += 4) {
                        const float4 f = *(const float4*)(q + j);
                        asc[i][j] = f.x; asc[i][j + 1] = f.y; asc[i][j + 2] = f.z; asc[i][j + 3] = f.w;
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < V; ++j) {
                        const int c = a0 + ga_col + j;
                        asc[i][j] = sp[c < a.A ? c : 0];
                    }
                }
            }
        }
#pragma unroll
        for (int i = 0; i < PB; ++i) {
            const int r = xb_row + i * RPB;
            const int m = p0 + r;
            bool ok = r < BK && m < p_end;
            int n = 0, iy = 0, ix = 0;
            {
                const int mm = ok ? m : 0;
                const int per = a.OH * a.OW;
                n = mm / per;
                const int rr = mm - n * per;
                iy = (rr / a.OW) * a.stride + ky - a.pady;
                ix = (rr % a.OW) * a.stride + kx - a.padx;
                ok = ok && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
            }
            rb_ok[i] = ok;
            if constexpr (VEC) {
                rb[i] = buf_load16<vecT>(rxw, ok && b0 + xb_col < a.B
                                                  ? (((n * a.H + iy) * a.W + ix) * a.B + b0 + xb_col) * (int)sizeof(T) : -1);
            } else {
                const T* row = x + (((int64_t)n * a.H + (ok ? iy : 0)) * a.W + (ok ? ix : 0)) * a.B;
                rb[i] = Loader<T, VEC>::load(row, b0 + xb_col, a.B);
            }
            if (a.b_scale) {
                const float* sp = a.b_scale + (int64_t)n * a.B;
                if constexpr (VEC) {
                    const float* q = sp + (b0 + xb_col < a.B ? b0 + xb_col : 0);
#pragma unroll
                    for (int j = 0; j < V; j += 4) {
                        const float4 f = *(const float4*)(q + j);
                        rsc[i][j] = f.x; rsc[i][j + 1] = f.y; rsc[i][j + 2] = f.z; rsc[i][j + 3] = f.w;
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < V; ++j) {
                        const int b = b0 + xb_col + j;
                        rsc[i][j] = sp[b < a.B ? b : 0];
                    }
                }
            }
        }
    };
    auto sstore = [&](int buf) {
        if constexpr (P3) {
#pragma unroll
            for (int i = 0; i < PA; ++i) {
                const int r = ga_row + i * RPA;
                if (r < BK) {
#pragma unroll
                    for (int q = 0; q < 3; ++q) *(bf16x8*)(lds3 + buf * 3 * PL3 + q * PL3 + r * LDA3 + ga_col) = r3a[i][q];
                }
            }
#pragma unroll
            for (int i = 0; i < PB; ++i) {
                const int r = xb_row + i * RPB;
                if (r < BK) {
#pragma unroll
                    for (int q = 0; q < 3; ++q)
                        *(bf16x8*)(lds3 + buf * 3 * PL3 + q * PL3 + BK * LDA3 + r * LDB3 + xb_col) = r3b[i][q];
                }
            }
            return;
        }
        T* As = lds[buf];
        T* Bs = lds[buf] + BK * LDA;
#pragma unroll
        for (int i = 0; i < PA; ++i) {
            const int r = ga_row + i * RPA;
            vecT v = VEC ? ra[i] : Loader<T, VEC>::mask(ra[i], a0 + ga_col, a.A, ra_ok[i]);
            if (a.a_scale) {
#pragma unroll
                for (int j = 0; j < V; ++j) v[j] = (T)__fmul_rn((float)v[j], asc[i][j]);
            }
            if constexpr (S3) {
                if (r < BK) store3(buf, r * LDA3 + ga_col, v);
            } else {
                if (r < BK) *(vecT*)(As + r * LDA + ga_col) = v;
            }
        }
#pragma unroll
        for (int i = 0; i < PB; ++i) {
            const int r = xb_row + i * RPB;
            vecT v = VEC ? rb[i] : Loader<T, VEC>::mask(rb[i], b0 + xb_col, a.B, rb_ok[i]);
            if (a.b_scale) {
#pragma unroll
                for (int j = 0; j < V; ++j) v[j] = (T)__fmul_rn((float)v[j], rsc[i][j]);   // rounded product (no fma contraction)
            }
            if constexpr (S3) {
                if (r < BK) store3(buf, BK * LDA3 + r * LDB3 + xb_col, v);
            } else {
                if (r < BK) *(vecT*)(Bs + r * LDB + xb_col) = v;
            }
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto compute = [&](int cur) {
        const T* As = lds[cur];
        const T* Bs = lds[cur] + BK * LDA;
        if constexpr (S3) {
            const bf16_t* P = lds3 + cur * 3 * PL3;
            bf16x8 af[TM][3], bfr[TN][3];
#pragma unroll
            for (int q = 0; q < 3; ++q) {
#pragma unroll
                for (int i = 0; i < TM; ++i) af[i][q] = frag_tr<bf16_t>(P + q * PL3, LDA3, 0, wm * WM + i * 16, lane);
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    bfr[j][q] = frag_tr<bf16_t>(P + q * PL3 + BK * LDA3, LDB3, 0, wn * WN + j * 16, lane);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j] = mfma_s3(af[i], bfr[j], acc[i][j]);
        } else if constexpr (std::is_same<T, float>::value) {
#pragma unroll
            for (int kk = 0; kk < BK; kk += 4) {
                float af[TM], bfr[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) af[i] = As[(kk + (lane >> 4)) * LDA + wm * WM + i * 16 + (lane & 15)];
#pragma unroll
                for (int j = 0; j < TN; ++j) bfr[j] = Bs[(kk + (lane >> 4)) * LDB + wn * WN + j * 16 + (lane & 15)];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
            }
        } else {
            v8_t<T> af[TM], bfr[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) af[i] = frag_tr<T>(As, LDA, 0, wm * WM + i * 16, lane);
#pragma unroll
            for (int j = 0; j < TN; ++j) bfr[j] = frag_tr<T>(Bs, LDB, 0, wn * WN + j * 16, lane);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j] = mfma16v<T>(af[i], bfr[j], acc[i][j]);
        }
    };
    if (p_begin < p_end) {
        if constexpr (S3) {
            gload(p_begin);
            for (int p0 = p_begin; p0 < p_end; p0 += BK) {
                const bool more = p0 + BK < p_end;
                sstore(0);
                __syncthreads();
                if (more) gload(p0 + BK);
                compute(0);
                __syncthreads();
            }
        } else {
            gload(p_begin);
            sstore(0);
            __syncthreads();
            int it = 0;
            for (int p0 = p_begin; p0 < p_end; p0 += BK, ++it) {
                const int cur = it & 1;
                const bool more = p0 + BK < p_end;
                if (more) gload(p0 + BK);
                compute(cur);
                if (more) sstore(cur ^ 1);
                __syncthreads();
            }
        }
    }

    const int KK = a.KH * a.KW;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int ar = a0 + wm * WM + i * 16 + 4 * (lane >> 4) + r;
            if (ar >= a.A) continue;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int bc = b0 + wn * WN + j * 16 + (lane & 15);
                if (bc >= a.B) continue;
                const int64_t di = ((int64_t)ar * KK + tap) * a.B + bc;
                if (a.det) a.det[(int64_t)split * a.A * KK * a.B + di] = acc[i][j][r] * a.alpha;
                else atomicAdd(a.dw + di, acc[i][j][r] * a.alpha);
            }
        }
}

template <typename T, int BM, int BN>
int launch_wgrad(WgradArgs& a, bool vec, hipStream_t s) {
    constexpr bool F32 = std::is_same<T, float>::value;
    const bool s3 = F32 && (a.gpl || !f32_exact());
    const int BK = s3 ? KStage<float, true>::BK : Traits<T>::BK;
    const int mt = (int)cdiv(a.A, BM), nt = (int)cdiv(a.B, BN);
    const int KK = a.KH * a.KW;
    const int chunks = (int)cdiv(a.M, BK);
    // workgroups the pixel split aims at (every workgroup adds a BM x BN partial per tap: float atomics, or a slot
    // of the fixed-order sum); SG2_CWGRAD_WGS overrides (tuning runs).  1024 since the parameter-layout slot sum
    // (fewer slots to sum): bench 777.3 / 778.7 img/s at 2048, 781.5 / 781.2 at 1024, 768-1536 level, 512 lower
    // (profiles/r06be, r06bf)
    static const int target = [] { const char* e = getenv("SG2_CWGRAD_WGS"); return e ? std::max(1, atoi(e)) : 1024; }();
    int splits = (int)std::max<int64_t>(1, std::min<int64_t>(chunks / 8, cdiv(target, (int64_t)mt * nt * KK)));
    a.kper = (int)cdiv(chunks, splits) * BK;
    a.splits = (int)cdiv(a.M, a.kper);
    DetArena arena;
    const int64_t nel = (int64_t)a.A * KK * a.B;
    if (det_on()) SG2_DET_GET(a.det, arena, a.splits * nel, "sg2_conv2d_wgrad");
    dim3 grid(mt, nt, KK * a.splits);
    if (F32 && a.gpl) {      // pre-split operands (SG2_F32S3)
        conv_wgrad_kernel<T, BM, BN, true, F32, F32><<<grid, 256, 0, s>>>(a);
    } else if (s3) {
        if (vec) conv_wgrad_kernel<T, BM, BN, true, F32><<<grid, 256, 0, s>>>(a);
        else conv_wgrad_kernel<T, BM, BN, false, F32><<<grid, 256, 0, s>>>(a);
    } else {
        if (vec) conv_wgrad_kernel<T, BM, BN, true, false><<<grid, 256, 0, s>>>(a);
        else conv_wgrad_kernel<T, BM, BN, false, false><<<grid, 256, 0, s>>>(a);
    }
    int rc = launch_status("sg2_conv2d_wgrad");
    if (rc || !a.det) return rc;
    hipError_t e = a.oikk ? det_sum_oikk(a.dw, a.det, a.splits, a.A, KK, a.B, a.oikk == 2, s, det_assign())
                          : det_sum(a.dw, 0, a.det, 0, nel, 1, a.splits, nel, arena, s, det_assign());
    if (e) { set_error("sg2_conv2d_wgrad: det_sum"); return (int)e; }
    return 0;
}

int floordiv_h(int a, int b) { return (a >= 0) ? a / b : -((-a + b - 1) / b); }

}  // namespace

// wgrad3x3.hip: halo weight gradient (3x3 / 1x1, stride 1 or 2, 16-bit)
bool wgrad_halo_ok(int dtype, int KH, int KW, int stride, int pad_y, int pad_x, int OW, int A, int B);
int wgrad3x3_launch(float* dw, const void* g, const void* x, const float* gscale, const float* xscale, int dtype,
                    int N, int A, int OH, int OW, int B, int H, int W, int KH, int KW, int stride, int pad_y,
                    int pad_x, float alpha, hipStream_t s);
}  // namespace sg2

extern "C" int sg2_conv2d_fused(void* y, const void* x, const void* w, int dtype, int N, int Cin, int H, int W,
                                int Cout, int OH, int OW, int KH, int KW, int stride, int pad_y, int pad_x,
                                int transpose, const float* in_scale, const sg2_epilogue* epi, float* workspace,
                                int64_t workspace_elems, void* stream) {
    using namespace sg2;
    SG2_CHECK(y && x && w, "sg2_conv2d: null pointer");
    SG2_CHECK(N > 0 && Cin > 0 && H > 0 && W > 0 && Cout > 0 && OH > 0 && OW > 0, "sg2_conv2d: empty shape");
    SG2_CHECK(KH >= 1 && KW >= 1 && KH * KW <= kMaxTaps, "sg2_conv2d: kernel too large");
    SG2_CHECK(stride >= 1 && stride <= 4, "sg2_conv2d: unsupported stride");
    SG2_CHECK(pad_y > -64 && pad_y < 64 && pad_x > -64 && pad_x < 64, "sg2_conv2d: padding out of range");
    SG2_CHECK((int64_t)N * OH * OW * Cout < INT32_MAX && (int64_t)N * H * W * Cin * 4 < INT32_MAX &&
                  (int64_t)KH * KW * Cin * Cout * 4 < INT32_MAX,
              "sg2_conv2d: tensor too large (32-bit byte offsets of the buffer loads)");
    if (epi) {
        SG2_CHECK(epi->act == 0 || epi->act == 1, "sg2_conv2d: epilogue act must be 0 (linear) or 1 (lrelu)");
        SG2_CHECK(epi->aux_mode >= 0 && epi->aux_mode <= 2 && (epi->aux_mode == 0 || epi->aux),
                  "sg2_conv2d: bad epilogue aux output");
    }
    hipStream_t s = as_stream(stream);
    // SG2_F32S3: x and w are sg2_split3 planes (h, m, l), everything else f32
    const bool p3 = dtype == SG2_F32S3;
    if (p3) {
        SG2_CHECK(in_scale == nullptr, "sg2_conv2d: SG2_F32S3 operands carry their modulation (sg2_split3 scale)");
        SG2_CHECK(Cin % 8 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)w % 16 == 0,
                  "sg2_conv2d: SG2_F32S3 needs Cin % 8 == 0 and 16-byte aligned planes");
        SG2_CHECK((int64_t)N * H * W * Cin * 6 < INT32_MAX && (int64_t)Cout * KH * KW * Cin * 6 < INT32_MAX,
                  "sg2_conv2d: SG2_F32S3 planes too large (32-bit byte offsets)");
        dtype = SG2_F32;
    }

    ConvArgs base{};
    base.x = x; base.w = w; base.y = y; base.acc = nullptr; base.in_scale = in_scale;
    if (p3) { base.xpl = (int64_t)N * H * W * Cin; base.wpl = (int64_t)Cout * KH * KW * Cin; }
    base.N = N; base.H = H; base.W = W; base.Cin = Cin; base.Cout = Cout; base.OH = OH; base.OW = OW;
    base.wtaps = KH * KW;
    if (epi) {
        Epi& e = base.e;
        e.out_scale = epi->out_scale; e.noise = epi->noise; e.bias = epi->bias; e.residual = epi->residual;
        e.aux = epi->aux; e.noise_gain = epi->noise_gain; e.alpha = epi->alpha; e.gain = epi->gain;
        e.clamp = epi->clamp; e.act = epi->act; e.aux_mode = epi->aux_mode; e.on = 1;
        e.dot_src = epi->dot_src; e.dot_out = epi->dot_out;
        SG2_CHECK((e.dot_src == nullptr) == (e.dot_out == nullptr), "sg2_conv2d: dot_src and dot_out go together");
        SG2_CHECK(!(e.dot_out && e.aux_mode == 2), "sg2_conv2d: the dot reduction needs aux_mode 0 or 1");
        if (e.dot_out) {
            hipError_t er = zero_acc(e.dot_out, (size_t)N * Cout * sizeof(float), s);
            if (er != hipSuccess) { set_error("sg2_conv2d: memset failed"); return (int)er; }
        }
    }
    // Output phases (one for a plain conv; stride^2 for a transposed conv, launched 4 at a time).
    struct PhaseDef { Phase p; int ntaps; Tap taps[kMaxTaps]; };
    PhaseDef defs[16];
    int nph = 0;
    if (!transpose) {
        PhaseDef& d = defs[nph++];
        d.p = Phase{};
        d.p.QH = OH; d.p.QW = OW; d.p.osy = d.p.osx = 1; d.p.oy0 = d.p.ox0 = 0;
        SG2_CHECK((int64_t)(OH - 1) * stride - pad_y + KH - 1 >= 0, "sg2_conv2d: bad geometry");
        d.ntaps = 0;
        for (int ky = 0; ky < KH; ++ky)
            for (int kx = 0; kx < KW; ++kx)
                d.taps[d.ntaps++] = Tap{(int8_t)(ky - pad_y), (int8_t)(kx - pad_x), (int8_t)(ky * KW + kx), 0};
        base.isy = base.isx = stride;
    } else {
        // y[oy] = sum_{iy,ky: oy = iy*S + ky - P} x[iy] w[ky]  ->  phase py = oy mod S
        for (int py = 0; py < stride; ++py)
            for (int px = 0; px < stride; ++px) {
                PhaseDef& d = defs[nph];
                d.p = Phase{};
                d.p.QH = (OH - py + stride - 1) / stride;
                d.p.QW = (OW - px + stride - 1) / stride;
                if (d.p.QH <= 0 || d.p.QW <= 0) continue;
                d.p.osy = d.p.osx = stride; d.p.oy0 = py; d.p.ox0 = px;
                d.ntaps = 0;
                for (int ky = 0; ky < KH; ++ky) {
                    const int ny = py + pad_y - ky;
                    if (((ny % stride) + stride) % stride) continue;
                    for (int kx = 0; kx < KW; ++kx) {
                        const int nx = px + pad_x - kx;
                        if (((nx % stride) + stride) % stride) continue;
                        d.taps[d.ntaps++] = Tap{(int8_t)floordiv_h(ny, stride), (int8_t)floordiv_h(nx, stride),
                                                (int8_t)(ky * KW + kx), 0};
                    }
                }
                ++nph;
            }
        base.isy = base.isx = 1;
    }

    int rc = 0;
    if (!p3 && KH == 1 && KW == 1 && stride == 1 && pad_y == 0 && pad_x == 0 && OH == H && OW == W && Cout <= 4 &&
        Cin % 8 == 0 && Cin >= 8 && !base.e.dot_out && (uintptr_t)x % 16 == 0 && (uintptr_t)w % 16 == 0 &&
        (uintptr_t)in_scale % 16 == 0 && dtype != SG2_F32) {
        const int64_t groups = (int64_t)N * H * W;
        const int g = (int)std::min<int64_t>(cdiv(groups * 8, 256), 256 * 64);
        SG2_DISPATCH(dtype, T, { conv1x1_smallo_kernel<T><<<g, 256, 0, s>>>(base); });
        return launch_status("sg2_conv2d (1x1, small Cout)");
    }
    // (a 1x1 stride-1 transposed conv is the same product with the caller's transposed pack: dgrad of toRGB)
    if (!p3 && KH == 1 && KW == 1 && stride == 1 && pad_y == 0 && pad_x == 0 && OH == H && OW == W &&
        Cin <= 4 && Cout % 8 == 0 && 256 % (Cout / 8) == 0 && (uintptr_t)y % 32 == 0 &&
        (!base.e.aux || (uintptr_t)base.e.aux % 32 == 0) && (!base.e.residual || (uintptr_t)base.e.residual % 32 == 0) &&
        (!base.e.dot_out || (uintptr_t)base.e.dot_src % 16 == 0)) {
        if (base.e.dot_out) {
            const int ppb = SK_ITERS * (256 / (Cout / 8));
            dim3 g((unsigned)cdiv((int64_t)H * W, ppb), (unsigned)N);
            DetArena arena;
            if (det_on()) SG2_DET_GET(base.e.det_dot, arena, (int64_t)g.x * N * Cout, "sg2_conv2d (1x1, small Cin, dot)");
            SG2_DISPATCH(dtype, T, {
                if (Cin == 1) conv1x1_smallk_dot_kernel<T, 1><<<g, 256, 0, s>>>(base);
                else if (Cin == 2) conv1x1_smallk_dot_kernel<T, 2><<<g, 256, 0, s>>>(base);
                else if (Cin == 3) conv1x1_smallk_dot_kernel<T, 3><<<g, 256, 0, s>>>(base);
                else conv1x1_smallk_dot_kernel<T, 4><<<g, 256, 0, s>>>(base);
            });
            int rc1 = launch_status("sg2_conv2d (1x1, small Cin, dot)");
            if (rc1 || !base.e.det_dot) return rc1;
            hipError_t e = det_sum(base.e.dot_out, 0, base.e.det_dot, 0, (int64_t)N * Cout, 1, g.x, (int64_t)N * Cout,
                                   arena, s, det_assign());
            if (e) { set_error("sg2_conv2d: det_sum"); return (int)e; }
            return 0;
        }
        const int64_t total = (int64_t)N * H * W * (Cout / 8);
        const int g = (int)std::min<int64_t>(cdiv(total, 256), 256 * 64);
        SG2_DISPATCH(dtype, T, {
            if (Cin == 1) conv1x1_smallk_kernel<T, 1><<<g, 256, 0, s>>>(base);
            else if (Cin == 2) conv1x1_smallk_kernel<T, 2><<<g, 256, 0, s>>>(base);
            else if (Cin == 3) conv1x1_smallk_kernel<T, 3><<<g, 256, 0, s>>>(base);
            else conv1x1_smallk_kernel<T, 4><<<g, 256, 0, s>>>(base);
        });
        return launch_status("sg2_conv2d (1x1, small Cin)");
    }
    SG2_DISPATCH(dtype, T, {
        constexpr int V = Traits<T>::V;
        const int BK = (std::is_same<T, float>::value && (p3 || !f32_exact())) ? KStage<float, true>::BK : Traits<T>::BK;
        const bool vec = p3 || ((Cin % V == 0) && ((uintptr_t)x % 16 == 0) && ((uintptr_t)w % 16 == 0) &&
                                ((uintptr_t)in_scale % 16 == 0));
        const bool wide = Cout > 64;
        const int BN_ = wide ? 128 : 64;
        base.nck = (Cin + BK - 1) / BK;
        // split-K when the grid is too small to fill 256 CUs
        int64_t blocks = 0;
        int maxnk = 1;
        for (int i = 0; i < nph; ++i) {
            const int M = N * defs[i].p.QH * defs[i].p.QW;
            blocks += cdiv(M, 128) * cdiv(Cout, BN_);
            maxnk = std::max(maxnk, defs[i].ntaps * base.nck);
        }
        int splits = 1;
        const int64_t total_out = (int64_t)N * OH * OW * Cout;
        // split-K target 512 workgroups (tools/split_ab.py, profiles/r02_split_ab.log: f32 16^2 / 8^2 / 4^2 fwd
        // 0.281 / 0.103 / 0.056 ms at 1024 -> 0.263 / 0.083 / 0.044 at 512); SG2_CONV_SPLIT_WGS overrides
        static const int target = [] { const char* e = getenv("SG2_CONV_SPLIT_WGS"); return e ? std::max(1, atoi(e)) : 512; }();
        if (blocks < 512 && workspace != nullptr && workspace_elems >= total_out)
            splits = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(target, blocks), maxnk / 4));
        const bool split = splits > 1;
        const bool clean = workspace_clean();
        // deterministic mode: split s writes its partial sums to slot s (every output element of every slot: the
        // splits cover all K steps' tiles), and the finalize adds the slots in split order; the dot's per-element
        // products go to det_dot
        DetArena arena;
        float* det_acc = nullptr;
        float* acc_src = workspace;
        if (det_on()) {
            if (base.e.dot_out) SG2_DET_GET(base.e.det_dot, arena, total_out, "sg2_conv2d");
            if (split) SG2_DET_GET(det_acc, arena, (int64_t)splits * total_out, "sg2_conv2d");
        }
        if (split && !clean && !det_acc) {
            hipError_t e = zero_fill(acc_src, total_out * sizeof(float), s);
            if (e != hipSuccess) { set_error("sg2_conv2d: memset failed"); return (int)e; }
        }
        for (int g0 = 0; g0 < nph && rc == 0; g0 += kMaxPhases) {
            ConvArgs a = base;
            a.acc = split ? (det_acc ? det_acc : workspace) : nullptr;
            a.det_stride = det_acc ? total_out : 0;
            a.splits = splits;
            a.kper = (int)cdiv(maxnk, splits);
            int nt = 0;
            for (int i = 0; i < kMaxPhases; ++i) {
                a.ph[i] = Phase{};
                if (g0 + i >= nph) continue;
                const PhaseDef& d = defs[g0 + i];
                a.ph[i] = d.p;
                a.ph[i].M = N * d.p.QH * d.p.QW;
                a.ph[i].tap0 = nt;
                a.ph[i].ntaps = d.ntaps;
                a.ph[i].nk = d.ntaps * base.nck;
                for (int t = 0; t < d.ntaps; ++t) a.taps[nt++] = d.taps[t];
            }
            if (wide) rc = launch_fwd<T, 128, 128>(a, vec, s);
            else rc = launch_fwd<T, 128, 64>(a, vec, s);
        }
        if (rc == 0 && split) {
            const int g = (int)std::min<int64_t>(cdiv(total_out, 256), 4096);
            conv_finalize_kernel<T><<<g, 256, 0, s>>>((T*)y, acc_src, det_acc, det_acc ? splits : 0, base.e, total_out,
                                                      Cout, (int64_t)OH * OW, (int)clean);
            rc = launch_status("sg2_conv2d finalize");
        }
        if (rc == 0 && base.e.det_dot) {
            hipError_t e = det_sum(base.e.dot_out, Cout, base.e.det_dot, (int64_t)OH * OW * Cout, Cout, N,
                                   (int64_t)OH * OW, Cout, arena, s, det_assign());
            if (e) { set_error("sg2_conv2d: det_sum"); return (int)e; }
        }
    });
    return rc;
}

extern "C" int sg2_conv2d(void* y, const void* x, const void* w, int dtype, int N, int Cin, int H, int W, int Cout,
                          int OH, int OW, int KH, int KW, int stride, int pad_y, int pad_x, int transpose,
                          float* workspace, int64_t workspace_elems, void* stream) {
    return sg2_conv2d_fused(y, x, w, dtype, N, Cin, H, W, Cout, OH, OW, KH, KW, stride, pad_y, pad_x, transpose,
                            nullptr, nullptr, workspace, workspace_elems, stream);
}

namespace sg2 {
int conv2d_wgrad_impl(float* dw, const void* g, const void* x, int dtype, int N, int A, int OH, int OW, int B, int H,
                      int W, int KH, int KW, int stride, int pad_y, int pad_x, const float* g_scale,
                      const float* x_scale, float alpha, void* stream, int oikk);
}

extern "C" int sg2_conv2d_wgrad(float* dw, const void* g, const void* x, int dtype, int N, int A, int OH, int OW, int B,
                                int H, int W, int KH, int KW, int stride, int pad_y, int pad_x, const float* g_scale,
                                const float* x_scale, float alpha, void* stream) {
    return sg2::conv2d_wgrad_impl(dw, g, x, dtype, N, A, OH, OW, B, H, W, KH, KW, stride, pad_y, pad_x, g_scale,
                                  x_scale, alpha, stream, 0);
}

extern "C" int sg2_conv2d_wgrad_oikk(float* dw, const void* g, const void* x, int dtype, int N, int A, int OH, int OW,
                                     int B, int H, int W, int KH, int KW, int stride, int pad_y, int pad_x, float alpha,
                                     int swap_ab, void* stream) {
    using namespace sg2;
    SG2_CHECK(dtype == SG2_F32S3 && det_on() && B % 4 == 0 && KH * KW <= 9 && A <= 65535,
              "sg2_conv2d_wgrad_oikk: SG2_F32S3 operands in deterministic mode, B % 4 == 0, KH KW <= 9");
    return conv2d_wgrad_impl(dw, g, x, dtype, N, A, OH, OW, B, H, W, KH, KW, stride, pad_y, pad_x, nullptr, nullptr,
                             alpha, stream, swap_ab ? 2 : 1);
}

int sg2::conv2d_wgrad_impl(float* dw, const void* g, const void* x, int dtype, int N, int A, int OH, int OW, int B,
                           int H, int W, int KH, int KW, int stride, int pad_y, int pad_x, const float* g_scale,
                           const float* x_scale, float alpha, void* stream, int oikk) {
    using namespace sg2;
    SG2_CHECK(dw && g && x, "sg2_conv2d_wgrad: null pointer");
    SG2_CHECK(N > 0 && A > 0 && B > 0 && OH > 0 && OW > 0 && H > 0 && W > 0, "sg2_conv2d_wgrad: empty shape");
    SG2_CHECK(KH >= 1 && KW >= 1 && KH * KW <= 64, "sg2_conv2d_wgrad: kernel too large");
    SG2_CHECK((int64_t)N * OH * OW * A * 4 < INT32_MAX && (int64_t)N * H * W * B * 4 < INT32_MAX,
              "sg2_conv2d_wgrad: tensor too large (32-bit byte offsets of the buffer loads)");
    hipStream_t s = as_stream(stream);
    const bool p3 = dtype == SG2_F32S3;
    if (p3) {
        SG2_CHECK(!g_scale && !x_scale, "sg2_conv2d_wgrad: SG2_F32S3 operands carry their scales (sg2_split3)");
        SG2_CHECK(A % 8 == 0 && B % 8 == 0 && (uintptr_t)g % 16 == 0 && (uintptr_t)x % 16 == 0,
                  "sg2_conv2d_wgrad: SG2_F32S3 needs A, B % 8 == 0 and 16-byte aligned planes");
        SG2_CHECK((int64_t)N * OH * OW * A * 6 < INT32_MAX && (int64_t)N * H * W * B * 6 < INT32_MAX,
                  "sg2_conv2d_wgrad: SG2_F32S3 planes too large (32-bit byte offsets)");
    }
    hipError_t e = zero_acc(dw, (int64_t)A * KH * KW * B * sizeof(float), s);
    if (e != hipSuccess) { set_error("sg2_conv2d_wgrad: memset failed"); return (int)e; }
    WgradArgs a{};
    a.g = g; a.x = x; a.dw = dw; a.b_scale = x_scale; a.a_scale = g_scale;
    a.N = N; a.A = A; a.OH = OH; a.OW = OW; a.B = B; a.H = H; a.W = W; a.KH = KH; a.KW = KW;
    a.stride = stride; a.pady = pad_y; a.padx = pad_x; a.alpha = alpha;
    a.M = N * OH * OW;
    a.oikk = oikk;
    if (p3) {
        a.gpl = (int64_t)N * OH * OW * A;
        a.xpl = (int64_t)N * H * W * B;
        int rc = 0;
        if (A > 64 && B > 64) rc = launch_wgrad<float, 128, 128>(a, true, s);
        else if (A > 64) rc = launch_wgrad<float, 128, 64>(a, true, s);
        else if (B > 64) rc = launch_wgrad<float, 64, 128>(a, true, s);
        else rc = launch_wgrad<float, 64, 64>(a, true, s);
        return rc;
    }
    if (KH == 1 && KW == 1 && stride == 1 && pad_y == 0 && pad_x == 0 && OH == H && OW == W && B <= 4 &&
        A % 8 == 0 && 256 % (A / 8) == 0 && A * B <= 2048 && (uintptr_t)g % 16 == 0) {
        const int g_ = (int)std::min<int64_t>(cdiv((int64_t)a.M * (A / 8), 256), 1024);
        DetArena arena;
        const int64_t rows = (int64_t)g_ * 256 / (A / 8);
        if (det_on()) SG2_DET_GET(a.det, arena, rows * A * B, "sg2_conv2d_wgrad (1x1, small B)");
        const bool i32 = (int64_t)a.M * (A / 8) + (int64_t)g_ * 256 < INT32_MAX;
#define WGB(BT_) { if (i32) wgrad1x1_smallb_kernel<T, BT_, unsigned><<<g_, 256, 0, s>>>(a); \
                   else wgrad1x1_smallb_kernel<T, BT_, int64_t><<<g_, 256, 0, s>>>(a); }
        SG2_DISPATCH(dtype, T, { if (B == 1) WGB(1) else if (B == 2) WGB(2) else if (B == 3) WGB(3) else WGB(4) });
#undef WGB
        int rc1 = launch_status("sg2_conv2d_wgrad (1x1, small B)");
        if (rc1 || !a.det) return rc1;
        e = det_sum(dw, 0, a.det, 0, (int64_t)A * B, 1, rows, (int64_t)A * B, arena, s, det_assign());
        if (e) { set_error("sg2_conv2d_wgrad: det_sum"); return (int)e; }
        return 0;
    }
    if (KH == 1 && KW == 1 && stride == 1 && pad_y == 0 && pad_x == 0 && OH == H && OW == W && A <= 4 &&
        B % 8 == 0 && 256 % (B / 8) == 0 && A * B <= 2048 && (uintptr_t)x % 16 == 0) {
        const int g_ = (int)std::min<int64_t>(cdiv((int64_t)a.M * (B / 8), 256), 1024);
        DetArena arena;
        const int64_t rows = (int64_t)g_ * 256 / (B / 8);
        if (det_on()) SG2_DET_GET(a.det, arena, rows * A * B, "sg2_conv2d_wgrad (1x1, small A)");
        const bool i32 = (int64_t)a.M * (B / 8) + (int64_t)g_ * 256 < INT32_MAX;
#define WG1(AT_) { if (i32) wgrad1x1_smalla_kernel<T, AT_, unsigned><<<g_, 256, 0, s>>>(a); \
                   else wgrad1x1_smalla_kernel<T, AT_, int64_t><<<g_, 256, 0, s>>>(a); }
        SG2_DISPATCH(dtype, T, { if (A == 1) WG1(1) else if (A == 2) WG1(2) else if (A == 3) WG1(3) else WG1(4) });
#undef WG1
        int rc1 = launch_status("sg2_conv2d_wgrad (1x1, small A)");
        if (rc1 || !a.det) return rc1;
        e = det_sum(dw, 0, a.det, 0, (int64_t)A * B, 1, rows, (int64_t)A * B, arena, s, det_assign());
        if (e) { set_error("sg2_conv2d_wgrad: det_sum"); return (int)e; }
        return 0;
    }
    const bool halo = wgrad_halo_ok(dtype, KH, KW, stride, pad_y, pad_x, OW, A, B) && (uintptr_t)x % 16 == 0 &&
                      (uintptr_t)g % 16 == 0;
    if (halo) return wgrad3x3_launch(dw, g, x, g_scale, x_scale, dtype, N, A, OH, OW, B, H, W, KH, KW, stride, pad_y,
                                     pad_x, alpha, s);
    int rc = 0;
    SG2_DISPATCH(dtype, T, {
        constexpr int V = Traits<T>::V;
        const bool vec = (A % V == 0) && (B % V == 0) && ((uintptr_t)x % 16 == 0) && ((uintptr_t)g % 16 == 0) &&
                         ((uintptr_t)g_scale % 16 == 0) && ((uintptr_t)x_scale % 16 == 0);
        if (A > 64 && B > 64) rc = launch_wgrad<T, 128, 128>(a, vec, s);
        else if (A > 64) rc = launch_wgrad<T, 128, 64>(a, vec, s);
        else if (B > 64) rc = launch_wgrad<T, 64, 128>(a, vec, s);
        else rc = launch_wgrad<T, 64, 64>(a, vec, s);
    });
    return rc;
}

extern "C" int sg2_split3(void* planes, const float* x, int64_t n, int C, int64_t pix_per_n, const float* scale,
                          void* stream) {
    using namespace sg2;
    SG2_CHECK(planes && x, "sg2_split3: null pointer");
    SG2_CHECK(C > 0 && C % 8 == 0 && n % C == 0 && pix_per_n > 0, "sg2_split3: C % 8 == 0 and n a multiple of C");
    SG2_CHECK((uintptr_t)planes % 16 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)scale % 16 == 0,
              "sg2_split3: 16-byte alignment required");
    if (n == 0) return 0;
    const int g = (int)std::min<int64_t>(cdiv(n / 8, 256), 256 * 64);
    split3_kernel<<<g, 256, 0, as_stream(stream)>>>((bf16_t*)planes, x, n, C, pix_per_n, scale);
    return launch_status("sg2_split3");
}
