// 3x3 / stride 1 / pad 1 convolution with an LDS halo tile, for the 16-bit layers (f16 / bf16,
// the 32^2 .. 256^2 blocks of G and D) -- the bulk of the training FLOPs.
//
// Why a second kernel next to the generic implicit GEMM (conv.hip): the generic kernel gathers the
// A operand per tap from global memory, so every input pixel is fetched 9 times.  Here a workgroup
// owns a TH x TW tile of output pixels of one sample and BN = 64 output channels; per 32-channel
// chunk of the input it stages the (TH+2) x (TW+2) halo ONCE in LDS plus the chunk's 9 x 64 x 32
// weights, then runs all 9 taps as MFMAs reading shifted windows of the halo:
//   per chunk and wave (64 pixels x 64 channels): 9 taps x 16 v_mfma_f32_16x16x32 = 144 MFMAs
//   against 9 x 8 ds_read_b128 fragment reads; halo pixel rows padded to 80 B so the 16 rows of a
//   fragment read hit 16 distinct 16-byte bank slots (conflict free).
// The two LDS buffers are filled through registers: the next chunk's global loads are issued
// before the current chunk's MFMAs and written after them (one barrier per chunk).
//
// Fused prologue / epilogue (the StyleGAN2 modulated-conv layer, networks_stylegan2.py:309-328):
//   A operand : x[n,y,x,c] * in_scale[n,c]                       (modulation, optional)
//   raw out   : c = conv(.)                                      (optional second output, for backward)
//   epilogue  : z = c * out_scale[n,o] + noise[n,y,x] * noise_gain + bias[o]  (demod + noise + bias)
//               y = clamp(act(z) * gain, +-clamp), act in {linear, lrelu(alpha)}
#include "sg2_common.h"

#include <algorithm>
#include <atomic>
#include <type_traits>

namespace sg2 {
namespace {

constexpr int CK = 32;              // input channels per chunk (= MFMA K)
constexpr int BN = 64;              // output channels per workgroup
constexpr int PX = CK;              // LDS pixel / weight-row stride in elements (64 B, XOR-swizzled: swz64)

// 16-byte piece q of LDS row p (a halo pixel or a weight row of one 32-channel chunk): a fragment read of
// 16 consecutive rows then hits 16 distinct bank slots in each of ds_read_b128's lane groups for any
// starting row (tools/lds_swizzle_check.py; the 80-byte padded rows used before conflicted 2-way).
__device__ __forceinline__ int swz64(int p, int q) { return p * 64 + ((q ^ ((p >> 1) & 2)) << 4); }

struct Conv3Args {
    const void* x;
    const void* w;          // packed [Cout][9][Cin]
    void* y;
    void* y_raw;            // optional: conv result before the epilogue
    const float* in_scale;  // [N, Cin] or null
    const float* out_scale; // [N, Cout] or null
    const void* noise;      // [N, H, W] (dtype T) or null
    const float* bias;      // [Cout] or null
    const void* dot_src;    // optional [N,H,W,Cout] (dtype T): dot_out[n,o] += sum_p c * dot_src
    float* dot_out;         // [N, Cout] float accum
    float noise_gain, alpha, gain, clamp;
    int act;                // 0 linear, 1 lrelu
    int N, H, W, Cin, Cout;
    int tiles_x, tiles_y;
    int OH, OW;             // output size (= H, W at stride 1; the stride-2 pad-0 form: (H - 3) / 2 + 1)
    const void* residual;   // optional [N,OH,OW,Cout] (dtype T): y = round(act(...)) + residual (the D resnet add)
    int raw_act;            // y_raw receives the activated value before the residual add (the activation
                            // gradient's input) instead of the raw conv output
    float* det_dot;         // deterministic mode: the dot's partial sums by slot (det_sum adds them per sample):
                            // halo kernel [tile][Cout], one per 256-pixel tile; c64p [N][det_maxb][8 waves][64]
    int edge_rx, edge_cy;   // up-2 edge split: per image, tiles of the last cell row / column (0: no split)
    int det_maxb;           // c64p, deterministic mode: workgroups that can share one sample (slot rows per sample)
};

// Output channel of MFMA row P of a 64-channel tile (see the C = 64 kernels below)
__device__ __forceinline__ int p_chan(int P) { return (P >> 5) * 32 + 8 * ((P & 15) >> 2) + 4 * ((P >> 4) & 1) + (P & 3); }

template <typename T>
using v8 = typename std::conditional<std::is_same<T, bf16_t>::value, bf16x8, f16x8>::type;

template <typename T>
__device__ __forceinline__ f32x4 mma(v8<T> a, v8<T> b, f32x4 c) {
    if constexpr (std::is_same<T, bf16_t>::value)
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// TW: tile width (pixels); TH = 256 / TW.  4 waves, each owns 64 consecutive tile pixels x 64 channels.
// NBUF = 2: double-buffered chunks (1 workgroup / CU); NBUF = 1: single buffer, 2 workgroups / CU
// overlap each other's staging (better when Cin spans only a couple of chunks).
// S = 2: the stride-2, padding-0 3x3 conv (conv2d_resample's down-2 plan after its FIR, :94-109; the D
// blocks' conv1 and the input gradient of the G up layers) on a 32 x 4 output tile: the (2 TW + 1) x
// (2 TH + 1) input halo is stored column-deinterleaved (a halo row = its even columns, then its odd ones),
// so a fragment read of 16 output pixels (input columns 2 apart) is 16 consecutive swizzled LDS rows.
// DIR (round 5; S = 1, Cout % 64 == 0): the MFMA operands swapped (weights as A, pixels as B) and the weight rows
// staged in p_chan order, so a lane's accumulators hold 8 consecutive output channels of one pixel and the epilogue
// stores 16 bytes per lane straight from registers -- no output tile through LDS, no epilogue barrier (the dot
// reduction: 16-lane shuffles, LDS atomics, one global atomic per channel).
template <typename T, int TW, bool SCALE_IN, bool EPI, int NBUF, int S = 1, bool DIR = false>
__global__ __launch_bounds__(256, 3 - NBUF) void conv3x3_halo_kernel(Conv3Args a) {   // NBUF = 1: two workgroups per CU
    static_assert(!DIR || S == 1, "the direct epilogue is the stride-1 form");
    constexpr int TH = S == 1 ? 256 / TW : 4;
    constexpr int PXW = TW * TH / 4, NFR = PXW / 16;                 // pixels and 16-pixel fragments per wave
    constexpr int HW_ = S * (TW - 1) + 3, HH = S * (TH - 1) + 3, HP = HW_ * HH;   // halo pixels
    constexpr int HEV = (HW_ + 1) / 2;                                // even columns of a halo row (S = 2)
    constexpr int HALO = HP * PX;                                      // elements per halo buffer
    constexpr int WTS = 9 * BN * PX;                                   // elements per weight buffer
    constexpr int NH = (HP * 4 + 255) / 256;                          // halo 16-B loads per thread
    constexpr int NW = (9 * BN * 4) / 256;                            // weight 16-B loads per thread (= 9)
    typedef T vec8 __attribute__((ext_vector_type(8)));

    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    T* smem = (T*)smem_raw;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tile = blockIdx.x;
    const int n = tile / (a.tiles_x * a.tiles_y);
    const int tr = tile - n * a.tiles_x * a.tiles_y;
    const int ty0 = (tr / a.tiles_x) * TH, tx0 = (tr % a.tiles_x) * TW;
    const int o0 = blockIdx.y * BN;
    const T* __restrict__ x = (const T*)a.x;
    const T* __restrict__ w = (const T*)a.w;
    const int nchunks = (a.Cin + CK - 1) / CK;

    // ---- staging geometry ----
    int h_src[NH], h_dst[NH];
    bool h_ok[NH];
#pragma unroll
    for (int i = 0; i < NH; ++i) {
        const int idx = tid + i * 256;             // (pixel, 16-byte quarter)
        const int p = idx >> 2, q = idx & 3;
        const int hy = p / HW_, hx = p - hy * HW_;
        const int iy = S == 1 ? ty0 - 1 + hy : 2 * ty0 + hy, ix = S == 1 ? tx0 - 1 + hx : 2 * tx0 + hx;
        h_ok[i] = p < HP && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
        h_src[i] = h_ok[i] ? ((n * a.H + iy) * a.W + ix) : 0;     // pixel index
        const int pl = S == 1 ? p : hy * HW_ + ((hx & 1) ? HEV + (hx >> 1) : (hx >> 1));   // LDS row
        h_dst[i] = p < HP ? swz64(pl, q) : -1;     // byte offset
    }
    const int hq = (tid & 3) * 8;
    int w_src[NW], w_dst[NW];
    bool w_ok[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const int idx = tid + i * 256;             // (tap, o, quarter)
        const int r = idx >> 2;                    // 0 .. 9*BN-1
        const int tap = r / BN, o = r - tap * BN;
        w_ok[i] = o0 + o < a.Cout;
        w_src[i] = (w_ok[i] ? (o0 + (DIR ? p_chan(o) : o)) : 0) * 9 + tap;   // row index in [Cout*9]
        w_dst[i] = swz64(tap * BN + o, idx & 3);   // byte offset
    }

    // Loads are unconditional (out-of-image / out-of-range lanes read a valid dummy address) and the
    // zero-fill + modulation happen at the LDS write, after the MFMAs: a branch around a load would
    // make hipcc drain vmcnt per load and serialise the prefetch against the math.
    // Raw buffer loads: an out-of-image pixel, a row past Cout or a channel past Cin gets offset -1,
    // which reads zeros (sg2_common.h make_rsrc), so the LDS write needs no select.
    const __amdgpu_buffer_rsrc_t rxb = make_rsrc(x, (int64_t)a.N * a.H * a.W * a.Cin * (int64_t)sizeof(T));
    const __amdgpu_buffer_rsrc_t rwb = make_rsrc(w, (int64_t)a.Cout * 9 * a.Cin * (int64_t)sizeof(T));
    vec8 rh[NH], rw[NW];
    float4 sc0, sc1;
    auto gload = [&](int chunk) {
        const int c = chunk * CK + hq;
        const bool cok = c < a.Cin;
        const int cc = cok ? c : 0;
#pragma unroll
        for (int i = 0; i < NH; ++i)
            rh[i] = buf_load16<vec8>(rxb, h_ok[i] && cok ? (h_src[i] * a.Cin + c) * (int)sizeof(T) : -1);
#pragma unroll
        for (int i = 0; i < NW; ++i)
            rw[i] = buf_load16<vec8>(rwb, w_ok[i] && cok ? (w_src[i] * a.Cin + c) * (int)sizeof(T) : -1);
        if (SCALE_IN) {
            const float* sc = a.in_scale + (int64_t)n * a.Cin + cc;
            sc0 = *(const float4*)sc;
            sc1 = *(const float4*)(sc + 4);
        }
    };
    auto sstore = [&](int buf) {
        T* hb = smem + buf * (HALO + WTS);
        T* wb = hb + HALO;
        const float scl[8] = {sc0.x, sc0.y, sc0.z, sc0.w, sc1.x, sc1.y, sc1.z, sc1.w};
#pragma unroll
        for (int i = 0; i < NH; ++i) {
            if (h_dst[i] < 0) continue;
            vec8 v = rh[i];
            if (SCALE_IN) {   // x * s.to(x.dtype) (networks_stylegan2.py:69): s rounded first, one rounding after
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = (T)((float)v[j] * (float)(T)scl[j]);
            }
            *(vec8*)((char*)hb + h_dst[i]) = v;
        }
#pragma unroll
        for (int i = 0; i < NW; ++i) *(vec8*)((char*)wb + w_dst[i]) = rw[i];
    };

    // ---- per-lane fragment bases ----
    const int lq = lane >> 4, l16 = lane & 15;
    int a_pos[NFR];
#pragma unroll
    for (int i = 0; i < NFR; ++i) {
        const int m = wave * PXW + i * 16 + l16;
        const int py = m / TW, px = m - py * TW;
        a_pos[i] = S * py * HW_ + px;              // LDS row of tap (0,0)
    }
    const int b_lane = swz64(l16, lq);             // + (tap * BN + j * 16) * 64: the same swizzle

    f32x4 acc[NFR][4];
#pragma unroll
    for (int i = 0; i < NFR; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    gload(0);
    sstore(0);
    __syncthreads();
    for (int ch = 0; ch < nchunks; ++ch) {
        const int cur = NBUF == 2 ? (ch & 1) : 0;
        const bool more = ch + 1 < nchunks;
        if (more) gload(ch + 1);
        const char* hb = (const char*)(smem + cur * (HALO + WTS));
        const char* wb = hb + HALO * sizeof(T) + b_lane;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                const int tap = ky * 3 + kx;
                // S = 2: input column 2 px + kx of the deinterleaved halo row
                const int toff = ky * HW_ + (S == 1 ? kx : ((kx & 1) ? HEV : (kx >> 1)));
                v8<T> af[NFR], bfr[4];
#pragma unroll
                for (int i = 0; i < NFR; ++i) af[i] = *(const v8<T>*)(hb + swz64(a_pos[i] + toff, lq));
#pragma unroll
                for (int j = 0; j < 4; ++j) bfr[j] = *(const v8<T>*)(wb + (tap * BN + j * 16) * 64);
#pragma unroll
                for (int i = 0; i < NFR; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[i][j] = DIR ? mma<T>(bfr[j], af[i], acc[i][j]) : mma<T>(af[i], bfr[j], acc[i][j]);
            }
        }
        if (NBUF == 1 && more) __syncthreads();   // everyone done reading before the overwrite
        if (more) sstore(NBUF == 2 ? (cur ^ 1) : 0);
        __syncthreads();
    }

    if constexpr (DIR) {
        // lane (l16, q): pixel wave PXW + 16 i + l16 of the tile, channels o0 + 32 h + 8 q + e (e = 4 jj + r)
        float dsc[2][8], bsc[2][8];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int o = o0 + 32 * h + 8 * lq + e;
                dsc[h][e] = (EPI && a.out_scale) ? a.out_scale[(int64_t)n * a.Cout + o] : 1.f;
                bsc[h][e] = (EPI && a.bias) ? (float)(T)a.bias[o] : 0.f;
            }
        typedef T vec8d __attribute__((ext_vector_type(8)));
        const bool want_dot = a.dot_out != nullptr, atom = want_dot && !a.det_dot;
        float* red = (float*)smem;                 // dot partial sums (the halo buffer is free after the loop):
                                                   // [BN] (atomic mode), [4 waves][BN] (deterministic mode)
        if (atom) {
            if (tid < BN) red[tid] = 0.f;
            __syncthreads();
        }
        float dacc[2][8];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int e = 0; e < 8; ++e) dacc[h][e] = 0.f;
        T* y = (T*)a.y;
        T* yr = (T*)a.y_raw;
        const T* dsrc = (const T*)a.dot_src;
        const T* nz = (const T*)a.noise;
#pragma unroll
        for (int i = 0; i < NFR; ++i) {
            const int m = wave * PXW + i * 16 + l16;
            const int py = m / TW, px = m - py * TW;
            const int oy = ty0 + py, ox = tx0 + px;
            const bool ok = oy < a.OH && ox < a.OW;
            const int64_t pix = ((int64_t)n * a.OH + (ok ? oy : 0)) * a.OW + (ok ? ox : 0);
            const float nv = (EPI && nz) ? (float)nz[pix] * a.noise_gain : 0.f;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                vec8d yv, rv;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    float v = acc[i][2 * h + (e >> 2)][e & 3];
                    rv[e] = (T)v;
                    if (EPI) {
                        v = v * dsc[h][e] + nv + bsc[h][e];
                        if (a.act == 1) v = v > 0.f ? v : v * a.alpha;
                        v *= a.gain;
                        if (a.clamp >= 0.f) v = fminf(fmaxf(v, -a.clamp), a.clamp);
                    }
                    yv[e] = (T)v;
                }
                if (!ok) continue;
                const int64_t dst = pix * a.Cout + o0 + 32 * h + 8 * lq;
                *(vec8d*)(y + dst) = yv;
                if (yr) *(vec8d*)(yr + dst) = rv;
                if (want_dot) {
                    const vec8d sv = *(const vec8d*)(dsrc + dst);
#pragma unroll
                    for (int e = 0; e < 8; ++e) dacc[h][e] += (float)rv[e] * (float)sv[e];
                }
            }
        }
        if (want_dot) {
            // the 16 pixel lanes of a channel group by shuffles; then the 4 waves: LDS atomics + one global atomic
            // per channel, or (deterministic mode) wave partials added in wave order into the tile's slot
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    float v = dacc[h][e];
                    v += __shfl_xor(v, 1);
                    v += __shfl_xor(v, 2);
                    v += __shfl_xor(v, 4);
                    v += __shfl_xor(v, 8);
                    if (l16 == 0) {
                        if (atom) atomicAdd(&red[32 * h + 8 * lq + e], v);
                        else red[wave * BN + 32 * h + 8 * lq + e] = v;
                    }
                }
            __syncthreads();
            if (tid < BN) {
                if (atom) atomicAdd(&a.dot_out[(int64_t)n * a.Cout + o0 + tid], red[tid]);
                else a.det_dot[(int64_t)tile * a.Cout + o0 + tid] = ((red[tid] + red[BN + tid]) + red[2 * BN + tid]) +
                                                                     red[3 * BN + tid];
            }
        }
        return;
    }
    // ---- epilogue: fused math in registers, transpose through LDS, 16-byte row stores ----
    // per-lane channel parameters (n is fixed per workgroup).  (Fetching these and the noise before
    // the main loop raised register pressure past two workgroups per CU: measured slower.)
    float dsc[4], bsc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int o = o0 + j * 16 + (lane & 15);
        const int oc = o < a.Cout ? o : 0;
        dsc[j] = (EPI && a.out_scale) ? a.out_scale[(int64_t)n * a.Cout + oc] : 1.f;
        bsc[j] = (EPI && a.bias) ? (float)(T)a.bias[oc] : 0.f;   // the reference adds the bias rounded to x.dtype
    }
    constexpr int OS = BN + 8;                 // LDS row stride (elements) of the output tile
    constexpr int NPX = 4 * PXW;               // tile pixels
    T* ot = smem;                              // y tile  [NPX][OS]
    T* rt = smem + NPX * OS;                   // raw tile [NPX][OS] (y_raw and/or dot)
    float* red = (float*)(smem + 2 * NPX * OS);   // [BN] dot partial sums
    const T* nz = (const T*)a.noise;
    const bool want_raw = a.y_raw != nullptr;
    const bool want_dot = a.dot_out != nullptr;
    const bool keep_raw = want_raw || want_dot;
    if (want_dot && tid < BN) red[tid] = 0.f;
#pragma unroll
    for (int i = 0; i < NFR; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = wave * PXW + i * 16 + 4 * (lane >> 4) + r;
            float nv = 0.f;
            if (EPI && nz) {
                const int py = m / TW, px = m - py * TW;
                const int oy = min(ty0 + py, a.OH - 1), ox = min(tx0 + px, a.OW - 1);
                nv = (float)nz[((int64_t)n * a.OH + oy) * a.OW + ox] * a.noise_gain;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float v = acc[i][j][r];
                if (keep_raw) rt[m * OS + j * 16 + (lane & 15)] = (T)v;
                if (EPI) {
                    v = v * dsc[j] + nv + bsc[j];
                    if (a.act == 1) v = v > 0.f ? v : v * a.alpha;
                    v *= a.gain;
                    if (a.clamp >= 0.f) v = fminf(fmaxf(v, -a.clamp), a.clamp);
                }
                ot[m * OS + j * 16 + (lane & 15)] = (T)v;
            }
        }
    }
    __syncthreads();
    typedef T vec8o __attribute__((ext_vector_type(8)));
    T* y = (T*)a.y;
    T* yr = (T*)a.y_raw;
    const T* dsrc = (const T*)a.dot_src;
    const bool cvec = (a.Cout % 8) == 0;
    float dacc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) dacc[e] = 0.f;
    const int c8 = (tid & 7) * 8;              // fixed per thread (256 % 8 == 0)
#pragma unroll
    for (int k = 0; k < NPX / 32; ++k) {        // NPX pixels x 8 chunks of 8 channels / 256 threads
        const int idx = tid + k * 256;
        const int m = idx >> 3;
        const int py = m / TW, px = m - py * TW;
        const int oy = ty0 + py, ox = tx0 + px;
        const int o = o0 + c8;
        if (oy >= a.OH || ox >= a.OW || o >= a.Cout) continue;
        const int64_t dst = (((int64_t)n * a.OH + oy) * a.OW + ox) * a.Cout + o;
        if (cvec) {
            vec8o yo = *(const vec8o*)(ot + m * OS + c8);
            if (a.residual) {
                if (want_raw && a.raw_act) *(vec8o*)(yr + dst) = yo;
                const vec8o rr = *(const vec8o*)((const T*)a.residual + dst);
#pragma unroll
                for (int e = 0; e < 8; ++e) yo[e] = (T)((float)yo[e] + (float)rr[e]);   // round(v) + residual, rounded
            }
            *(vec8o*)(y + dst) = yo;
            if (want_raw && !a.raw_act) *(vec8o*)(yr + dst) = *(const vec8o*)(rt + m * OS + c8);
            if (want_dot) {
                const vec8o sv = *(const vec8o*)(dsrc + dst);
                const vec8o rv = *(const vec8o*)(rt + m * OS + c8);
#pragma unroll
                for (int e = 0; e < 8; ++e) dacc[e] += (float)rv[e] * (float)sv[e];
            }
        } else {
            for (int e = 0; e < 8 && o + e < a.Cout; ++e) {
                T yo = ot[m * OS + c8 + e];
                if (want_raw) yr[dst + e] = a.raw_act ? yo : rt[m * OS + c8 + e];
                if (a.residual) yo = (T)((float)yo + (float)((const T*)a.residual)[dst + e]);
                y[dst + e] = yo;
                if (want_dot) dacc[e] += (float)rt[m * OS + c8 + e] * (float)dsrc[dst + e];
            }
        }
    }
    if (want_dot && !a.det_dot) {
#pragma unroll
        for (int e = 0; e < 8; ++e) atomicAdd(&red[c8 + e], dacc[e]);
        __syncthreads();
        if (tid < BN && o0 + tid < a.Cout) atomicAdd(&a.dot_out[(int64_t)n * a.Cout + o0 + tid], red[tid]);
    } else if (want_dot) {
        // deterministic mode: the 32 threads of a channel octet in thread order (the tiles are free now), into the
        // tile's slot
        float* part = (float*)smem;                // [32][BN]
        __syncthreads();
#pragma unroll
        for (int e = 0; e < 8; ++e) part[(tid >> 3) * BN + c8 + e] = dacc[e];
        __syncthreads();
        if (tid < BN && o0 + tid < a.Cout) {
            float v = 0.f;
            for (int r = 0; r < 32; ++r) v += part[r * BN + tid];
            a.det_dot[(int64_t)tile * a.Cout + o0 + tid] = v;
        }
    }
}

template <typename T, int TW, bool SI, bool EPI, int NBUF, int S = 1, bool DIR = false>
int launch3_k(const Conv3Args& a, hipStream_t s) {
    constexpr int TH = S == 1 ? 256 / TW : 4;
    size_t lds = NBUF * (size_t)((S * (TW - 1) + 3) * (S * (TH - 1) + 3) * PX + 9 * BN * PX) * sizeof(T);
    if (!DIR) lds = std::max(lds, (size_t)2 * TW * TH * (BN + 8) * sizeof(T) + BN * sizeof(float));   // epilogue tiles
    auto kern = conv3x3_halo_kernel<T, TW, SI, EPI, NBUF, S, DIR>;
    static bool attr_set = false;   // benign race: idempotent attribute
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr_set = true;
    }
    dim3 grid(a.N * a.tiles_x * a.tiles_y, (a.Cout + BN - 1) / BN);
    if (a.dot_out && det_on()) {     // the dot's tile partials by slot, summed per sample in tile order
        Conv3Args b = a;
        DetArena arena;
        const int tps = a.tiles_x * a.tiles_y;
        SG2_DET_GET(b.det_dot, arena, (int64_t)grid.x * a.Cout, "sg2_conv3x3");
        kern<<<grid, 256, lds, s>>>(b);
        if (int rc = launch_status("sg2_conv3x3")) return rc;
        hipError_t e = det_sum(a.dot_out, a.Cout, b.det_dot, (int64_t)tps * a.Cout, a.Cout, a.N, tps, a.Cout, arena, s,
                               det_assign());
        if (e) { set_error("sg2_conv3x3: det_sum"); return (int)e; }
        return 0;
    }
    kern<<<grid, 256, lds, s>>>(a);
    return launch_status("sg2_conv3x3");
}

template <typename T, int TW, bool SI, bool EPI, int NBUF, int S = 1>
int launch3(const Conv3Args& a, hipStream_t s) {
    if constexpr (S == 1) {
        // the direct epilogue (SG2_HALO_DIRECT=0: the LDS-transposed one); read per launch: tests switch it
        const char* e = getenv("SG2_HALO_DIRECT");
        if ((!e || atoi(e) != 0) && a.Cout % BN == 0 && ((uintptr_t)a.y % 16) == 0 && ((uintptr_t)a.y_raw % 16) == 0 &&
            ((uintptr_t)a.dot_src % 16) == 0)
            return launch3_k<T, TW, SI, EPI, NBUF, 1, true>(a, s);
    }
    return launch3_k<T, TW, SI, EPI, NBUF, S, false>(a, s);
}

// ---------------------------------------------------------------------------------------------------
// Persistent, weights-resident variant for the 64 -> 64 channel layers (the 256^2 layer of the Claro
// network, 512^2 at cbase 32768; forward and dgrad).  The generic halo kernel above restages the 9 x 64 x 64
// weights (74 KB) for every 256-pixel tile, and its per-tile prologue / epilogue are exposed: with Cin = 64
// a tile is only two chunks of MFMAs.  Here one workgroup of 8 waves per CU keeps all weights in LDS for
// the whole launch and walks a contiguous run of 32 x 16 pixel tiles (vertically neighbouring tiles share
// halo rows through the CU's L2):
//   * wave w owns tile rows 2w, 2w+1 (64 pixels) x all 64 output channels: per tap and chunk 4 pixel and
//     4 weight fragments feed 16 MFMAs (0.5 ds_read_b128 per MFMA; 2 waves per SIMD, so one wave's LDS
//     reads and epilogue overlap the other's MFMAs);
//   * LDS is unpadded and XOR-swizzled: the 16-byte piece q of position p (a halo pixel or a weight row,
//     64 B per 32-channel chunk) sits at p * 64 + ((q ^ ((p >> 1) & 2)) << 4).  A fragment read (16
//     consecutive positions, 4 pieces) then hits 16 distinct 16-byte bank slots in each of ds_read_b128's
//     four lane groups ({0-3,12-15,20-27}, ...) for ANY starting position -- the tap shifts included --
//     where the 80-byte padded rows of the halo kernel conflict 2-way (SQ_LDS_BANK_CONFLICT = half the
//     LDS cycles, profiles/r02_v1_pmc_diag.txt).  The staging stores (8 lanes = 2 positions) stay
//     contiguous 128-byte blocks;
//   * the tile's two 32-channel chunks live in a double buffer: the next chunk's global loads (the next
//     tile's first chunk, during the current tile's second) are issued before the current chunk's MFMAs,
//     one barrier per chunk, no per-tile prologue;
//   * the epilogue's operands (noise, demod scales, dot source) are loaded before the tile's last chunk of
//     MFMAs, and the MFMA operands are swapped (weights as A, pixels as B) so a lane's accumulator holds 4
//     consecutive output channels of one pixel: 8-byte stores straight from registers, no LDS transpose;
//     the dot epilogue (dgrad's ds = sum_p c * x) keeps its per-(n, channel) partial sums in registers
//     across the run's tiles of one sample and flushes them once per sample;
//   * the modulation x * s is applied at the LDS store as a 16-bit multiply by s rounded to the
//     activation dtype -- the reference's `x * styles.to(x.dtype)` (networks_stylegan2.py:69) bit for bit.
#ifndef SG2_DIAG
#define SG2_DIAG 0          // timing-only builds (tools/c64p_diag.sh): 1 no MFMA, 2 no output stores, 4 no halo loads,
                            // 8 both chunks load the first 64 B of each pixel line, 16 epilogue tables as constants,
                            // 32 no modulation multiply at the LDS store, 64 no style-scale loads,
                            // 128 no noise / demod loads, 256 no noise / demod LDS table stores
#endif
constexpr int P_TW = 32, P_TH = 16, P_C = 64;
constexpr int P_HW = P_TW + 2, P_HH = P_TH + 2, P_HP = P_HW * P_HH;      // 34 x 18 halo positions
constexpr int P_POS = CK * 2;                                             // bytes per position and chunk
constexpr int P_WB = 2 * 9 * P_C * P_POS;                                 // weights: 73,728 B
constexpr int P_HB = P_HP * P_POS;                                        // one halo buffer: 39,168 B
constexpr int P_EB = (2 * P_C + P_TW * P_TH) * 4 + 16;                     // epilogue tables (f32), a dummy slot
constexpr size_t P_LDS = (size_t)P_WB + 2 * P_HB + P_EB;                  // 154,624 B
static_assert(P_WB % 256 == 0 && P_HB % 256 == 0, "swizzle assumes 256-byte aligned regions");

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// Output channel of MFMA row m (0..15) of channel tile j (A-operand row P = 16 j + m): tiles 2jj, 2jj+1 give
// lane group q the 8 consecutive channels 32 jj + 8 q .. +7 (rows 4q..4q+3 of each), so the epilogue stores
// 16 bytes per lane and pixel instead of 8 (a store-issue-bound tail: MI355X_MICROARCH.md latency table).
__device__ __forceinline__ int swz(int pos, int q) { return pos * P_POS + ((q ^ ((pos >> 1) & 2)) << 4); }

template <typename T, bool SCALE_IN, bool EPI, bool DOT>
__global__ __launch_bounds__(512, 1) void conv3x3_c64p_kernel(Conv3Args a, int tiles_total) {
    constexpr int NT = 512;
    constexpr int NH = (P_HP * 4 + NT - 1) / NT;         // halo 16-B loads per thread per chunk (5)
    constexpr int NWL = 2 * 9 * P_C * 4 / NT;            // weight 16-B loads per thread (9)
    typedef T vec8 __attribute__((ext_vector_type(8)));
    typedef T vec4 __attribute__((ext_vector_type(4)));
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    char* wlds = smem_raw;                               // [2 chunks][9 taps][64 rows] x 64 B, swizzled
    char* hlds = smem_raw + P_WB;                        // [2 buffers][612 positions] x 64 B, swizzled
    float* blds = (float*)(smem_raw + P_WB + 2 * P_HB);  // gain * bias[64]
    float* dlds = blds + P_C;                            // the tile's gain * demod[n, 64]
    float* nlds = dlds + P_C;                            // the tile's gain * noise_gain * noise[512 pixels]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tiles_x = a.W / P_TW, tiles_y = a.H / P_TH;
    const int per_n = tiles_x * tiles_y;
    const int t_begin = (int)((int64_t)blockIdx.x * tiles_total / gridDim.x);
    const int t_end = (int)((int64_t)(blockIdx.x + 1) * tiles_total / gridDim.x);
    if (t_begin >= t_end) return;
    const __amdgpu_buffer_rsrc_t rxb = make_rsrc(a.x, (int64_t)a.N * a.H * a.W * P_C * (int64_t)sizeof(T));
    const __amdgpu_buffer_rsrc_t rwb = make_rsrc(a.w, (int64_t)P_C * 9 * P_C * (int64_t)sizeof(T));

    // ---- weights: both chunks, once; bias ----
#pragma unroll
    for (int k = 0; k < NWL; ++k) {
        const int idx = tid + k * NT;
        const int c = idx / (9 * P_C * 4), rem = idx - c * 9 * P_C * 4;
        const int r = rem >> 2, q = rem & 3, tap = r / P_C, row = r - tap * P_C;
        const int o = p_chan(row);
        const vec8 v = buf_load16<vec8>(rwb, ((o * 9 + tap) * P_C + c * CK + q * 8) * (int)sizeof(T));
        *(vec8*)(wlds + swz((c * 9 + tap) * P_C + row, q)) = v;
    }
    if (tid < P_C) blds[tid] = (EPI && a.bias) ? (float)(T)a.bias[tid] * a.gain : 0.f;

    // ---- halo staging geometry (fixed per thread; the tile origin varies) ----
    int h_dy[NH], h_dx[NH], h_dst[NH];
#pragma unroll
    for (int i = 0; i < NH; ++i) {
        const int idx = tid + i * NT, p = idx >> 2, q = idx & 3;
        h_dy[i] = p / P_HW - 1;
        h_dx[i] = p % P_HW - 1;
        h_dst[i] = p < P_HP ? swz(p, q) : -1;
    }
    const int hq = (tid & 3) * 8;
    vec8 rh[NH];
    float4 s0, s1;                                       // the chunk's 8 style scales (rounded to T at the store)
    const __amdgpu_buffer_rsrc_t rsc = make_rsrc(a.in_scale, SCALE_IN ? (int64_t)a.N * P_C * 4 : 0);
    auto tile_of = [&](int t, int& n, int& ty0, int& tx0) {
        n = t / per_n;
        const int tr = t - n * per_n;
        ty0 = (tr / tiles_x) * P_TH;
        tx0 = (tr % tiles_x) * P_TW;
    };
    auto gload = [&](int t, int c) {
        int n, ty0, tx0;
        tile_of(t, n, ty0, tx0);
#pragma unroll
        for (int i = 0; i < NH; ++i) {
            const int iy = ty0 + h_dy[i], ix = tx0 + h_dx[i];
            // bitwise &: no short-circuit branches (each would split the load sequence)
            const bool ok = (tid + i * NT < P_HP * 4) & ((unsigned)iy < (unsigned)a.H) & ((unsigned)ix < (unsigned)a.W);
            if (!(SG2_DIAG & 4)) rh[i] = buf_load16<vec8>(rxb, ok ? (((n * a.H + iy) * a.W + ix) * P_C + ((SG2_DIAG & 8) ? 0 : c) * CK + hq) * (int)sizeof(T) : -1);
            else rh[i] = vec8{};
        }
        if (SCALE_IN && !(SG2_DIAG & 64)) {
            s0 = buf_load16<float4>(rsc, (n * P_C + c * CK + hq) * 4);
            s1 = buf_load16<float4>(rsc, (n * P_C + c * CK + hq + 4) * 4);
        } else if (SCALE_IN) {
            s0 = float4{1.f, 1.f, 1.f, 1.f};
            s1 = s0;
        }
    };
    auto sstore = [&](int buf) {
        char* hb = hlds + buf * P_HB;
        const vec8 sv8 = vec8{(T)s0.x, (T)s0.y, (T)s0.z, (T)s0.w, (T)s1.x, (T)s1.y, (T)s1.z, (T)s1.w};
#pragma unroll
        for (int i = 0; i < NH; ++i) {
            vec8 v = rh[i];
            if (SCALE_IN && !(SG2_DIAG & 32)) {
                if constexpr (std::is_same<T, f16_t>::value) {
                    v = v * sv8;                         // v_pk_mul_f16: round(x * round(s)), as the reference
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) v[j] = (T)((float)v[j] * (float)sv8[j]);
                }
            }
            // the ragged last round writes a dummy slot instead of branching round the store (a branch
            // leaves the skipped load pending for the waitcnt pass, which then drains vmcnt at the loop top)
            char* dst = h_dst[i] >= 0 ? hb + h_dst[i] : smem_raw + P_LDS - 16;
            *(vec8*)dst = v;
        }
    };

    // MFMA operand addressing (lane: row / pixel = lane & 15, 16-byte piece q = lane >> 4)
    const int l16 = lane & 15, q = lane >> 4;
    const int w_lane = swz(l16, q);                      // + (chunk * 9 + tap) * 4096 + j * 1024 (same swizzle)
    int hp[4];                                           // halo position of pixel fragment i at tap (0, 0)
#pragma unroll
    for (int i = 0; i < 4; ++i) hp[i] = (2 * wave + (i >> 1)) * P_HW + (i & 1) * 16 + l16;
    const int oq8 = 8 * q;                               // channel of acc[.][j][r] is 32 (j / 2) + oq8 + 4 (j % 2) + r
    const float lr_alpha = (EPI && a.act == 1) ? a.alpha : 1.f;   // lrelu as max(v, alpha v), 0 <= alpha <= 1
    const float clampv = (EPI && a.clamp >= 0.f) ? a.clamp : __builtin_inff();
    const float ngain = a.noise_gain * a.gain;
    const float dgain = a.gain;
    T e_noise;                                           // this thread's pixel of the tile's noise
    float e_d;                                           // this thread's (tid < 64) demodulation scale

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float dacc[2][8];                                    // dot partial sums of the current sample
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int e = 0; e < 8; ++e) dacc[jj][e] = 0.f;

    const int64_t npix = (int64_t)a.N * a.H * a.W;
    const __amdgpu_buffer_rsrc_t ryb = make_rsrc(a.y, npix * P_C * (int64_t)sizeof(T));
    const __amdgpu_buffer_rsrc_t ryr = make_rsrc(a.y_raw, a.y_raw ? npix * P_C * (int64_t)sizeof(T) : 0);
    const bool has_raw = __builtin_amdgcn_readfirstlane(a.y_raw != nullptr);
    const __amdgpu_buffer_rsrc_t rnz = make_rsrc(a.noise, a.noise ? npix * (int64_t)sizeof(T) : 0);
    const __amdgpu_buffer_rsrc_t ros = make_rsrc(a.out_scale, a.out_scale ? (int64_t)a.N * P_C * 4 : 0);
    const int e_row = tid / P_TW, e_col = tid % P_TW;
    const __amdgpu_buffer_rsrc_t rds = make_rsrc(a.dot_src, a.dot_src ? npix * P_C * (int64_t)sizeof(T) : 0);
    gload(t_begin, 0);
    __syncthreads();                                     // weights in LDS
    sstore(0);
    __syncthreads();
    for (int t = t_begin; t < t_end; ++t) {
        int n, ty0, tx0;
        tile_of(t, n, ty0, tx0);
        vec8 dv[4][2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {                   // chunk c of tile t lives in halo buffer c
            // no branch around a load (hipcc would drain vmcnt right after it): the last tile's "next
            // chunk" re-reads the tile itself, and absent epilogue operands read zeros (empty buffers)
            gload(c == 0 ? t : min(t + 1, t_end - 1), c ^ 1);
            if (c == 0 && EPI && !(SG2_DIAG & 128)) {
                // the tile's noise and demodulation scales: into LDS with the chunk's halo store
                e_noise = buf_load2<T>(rnz, ((n * a.H + ty0 + e_row) * a.W + tx0 + e_col) * (int)sizeof(T));
                e_d = buf_load4f(ros, (n * P_C + (tid & (P_C - 1))) * 4);
            } else if (c == 0 && EPI) {
                e_noise = (T)0.5f;
                e_d = 0.9f;
            }
            if (c == 1 && DOT) {
                // the dot source of pixel fragments 0, 1 in flight during the last chunk's MFMAs (2, 3 are
                // loaded at the epilogue's start: the registers for all four would spill)
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int pix = (n * a.H + ty0 + 2 * wave + (i >> 1)) * a.W + tx0 + (i & 1) * 16 + l16;
#pragma unroll
                    for (int jj = 0; jj < 2; ++jj) dv[i][jj] = buf_load16<vec8>(rds, (pix * P_C + jj * 32 + oq8) * (int)sizeof(T));
                }
            }
            __builtin_amdgcn_sched_barrier(0);         // all loads issued before the MFMAs
            const char* hb = hlds + c * P_HB;
            const char* wb = wlds + c * 9 * P_C * P_POS + w_lane;
#pragma unroll
            for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    const int tap = ky * 3 + kx;
                    v8<T> pf[4], wf[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) wf[j] = *(const v8<T>*)(wb + (tap * P_C + j * 16) * P_POS);
#pragma unroll
                    for (int i = 0; i < 4; ++i) pf[i] = *(const v8<T>*)(hb + swz(hp[i] + ky * P_HW + kx, q));
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            if (!(SG2_DIAG & 1)) acc[i][j] = mma<T>(wf[j], pf[i], acc[i][j]);
                            else acc[i][j][0] += (float)wf[j][0] * (float)pf[i][0];
                        }
                }
            }
            // keep the scheduler from hoisting the staging store's math (which waits for the in-flight halo
            // loads) or the epilogue above the MFMAs
            __builtin_amdgcn_sched_barrier(0);
            if (c == 1) {
                // ---- epilogue of tile t from the accumulators: lane = 4 channels x 1 pixel ----
                // the gain folded in: gain * lrelu(z) = lrelu(gain * z) for gain > 0 (host-checked)
                if (DOT) {
#pragma unroll
                    for (int i = 2; i < 4; ++i) {
                        const int pix = (n * a.H + ty0 + 2 * wave + (i >> 1)) * a.W + tx0 + (i & 1) * 16 + l16;
#pragma unroll
                        for (int jj = 0; jj < 2; ++jj) dv[i][jj] = buf_load16<vec8>(rds, (pix * P_C + jj * 32 + oq8) * (int)sizeof(T));
                    }
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int64_t pix = ((int64_t)n * a.H + ty0 + 2 * wave + (i >> 1)) * a.W + tx0 + (i & 1) * 16 + l16;
                    const float nv = (EPI && !(SG2_DIAG & 16)) ? nlds[(2 * wave + (i >> 1)) * P_TW + (i & 1) * 16 + l16] : 0.f;
#pragma unroll
                    for (int jj = 0; jj < 2; ++jj) {
                        const int ch = jj * 32 + oq8;            // channels ch .. ch + 7: acc[i][2jj][.], acc[i][2jj+1][.]
                        const int64_t dst = pix * P_C + ch;
                        float bb[8], dd[8];
                        if (EPI && (SG2_DIAG & 16)) {
#pragma unroll
                            for (int e = 0; e < 8; ++e) { bb[e] = 0.1f * (e + 1); dd[e] = 1.f - 0.01f * e; }
                        } else if (EPI) {
                            const float4 b0 = *(const float4*)(blds + ch), b1 = *(const float4*)(blds + ch + 4);
                            const float4 d0 = *(const float4*)(dlds + ch), d1 = *(const float4*)(dlds + ch + 4);
                            bb[0] = b0.x; bb[1] = b0.y; bb[2] = b0.z; bb[3] = b0.w; bb[4] = b1.x; bb[5] = b1.y; bb[6] = b1.z; bb[7] = b1.w;
                            dd[0] = d0.x; dd[1] = d0.y; dd[2] = d0.z; dd[3] = d0.w; dd[4] = d1.x; dd[5] = d1.y; dd[6] = d1.z; dd[7] = d1.w;
                        }
                        vec8 yv, rv;
                        // (the raw output is only rounded where something consumes it; a packed-f32 form of
                        // this loop measured the same: profiles/r02_v7_c64p_variants.log)
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            const float cv = acc[i][2 * jj + (e >> 2)][e & 3];
                            if (DOT) rv[e] = (T)cv;
                            float v = cv;
                            if (EPI) {
                                v = fmaf(v, dd[e], nv + bb[e]);
                                v = fmaxf(v, v * lr_alpha);
                                v = __builtin_amdgcn_fmed3f(v, -clampv, clampv);
                            }
                            yv[e] = (T)v;
                            if (DOT) dacc[jj][e] += (float)rv[e] * (float)dv[i][jj][e];
                        }
                        if (!(SG2_DIAG & 2)) {
                            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, yv), ryb, (int)(dst * sizeof(T)), 0, 0);
                            // a uniform (scalar) branch: a dropped store still costs its issue slot
                            if (has_raw) {
                                if (!DOT) {
#pragma unroll
                                    for (int e = 0; e < 8; ++e) rv[e] = (T)acc[i][2 * jj + (e >> 2)][e & 3];
                                }
                                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, rv), ryr, (int)(dst * sizeof(T)), 0, 0);
                            }
                        } else if (yv[0] == (T)12345.f && yv[1] == (T)-7.f) {
                            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, yv), ryb, (int)(dst * sizeof(T)), 0, 0);
                        }
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
                }
                if (DOT && (t + 1 == t_end || (t + 1) / per_n != n)) {
                    // this run is done with sample n: sum over the 16 lanes holding the same channels
                    // (lane % 16 = pixel), one atomic per channel and wave
#pragma unroll
                    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            float v = dacc[jj][e];
                            v += __shfl_xor(v, 1);
                            v += __shfl_xor(v, 2);
                            v += __shfl_xor(v, 4);
                            v += __shfl_xor(v, 8);
                            if (l16 == 0) {
                                if (a.det_dot) {
                                    // deterministic mode: this wave's slot of (sample n, workgroup offset within the
                                    // workgroups that can cover n: blockIdx.x - first of them)
                                    const int64_t blo = ((int64_t)(n * per_n + 1) * gridDim.x + tiles_total - 1) / tiles_total - 1;
                                    a.det_dot[(((int64_t)n * a.det_maxb + (blockIdx.x - blo)) * 8 + wave) * P_C + jj * 32 + oq8 + e] = v;
                                } else {
                                    atomicAdd(&a.dot_out[(int64_t)n * P_C + jj * 32 + oq8 + e], v);
                                }
                            }
                            dacc[jj][e] = 0.f;
                        }
                }
            }
            sstore(c ^ 1);
            if (c == 0 && EPI && !(SG2_DIAG & 256)) {
                nlds[tid] = (float)e_noise * ngain;
                if (tid < P_C) dlds[tid] = a.out_scale ? e_d * dgain : dgain;
            }
            __syncthreads();
        }
    }
}

template <typename T, bool SI, bool EPI, bool DOT>
int launch_c64p(const Conv3Args& a, hipStream_t s, int tiles, int grid) {
    auto kern = conv3x3_c64p_kernel<T, SI, EPI, DOT>;
    static bool attr_set = false;   // benign race: idempotent attribute
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)P_LDS);
        attr_set = true;
    }
    if (DOT && det_on()) {
        // deterministic mode: slots [N][maxb][8 waves][64] (maxb: the most workgroups one sample's tiles spread
        // over, offsets from the first that can cover it -- the kernel's formula), zeroed (a sample's later
        // offsets may be unused), summed per sample in slot order
        const int per_n = (a.W / P_TW) * (a.H / P_TH);
        int maxb = 1;
        for (int b = 0; b < grid; ++b) {
            const int t0 = (int)((int64_t)b * tiles / grid), t1 = (int)((int64_t)(b + 1) * tiles / grid);
            if (t0 >= t1) continue;
            for (int n = t0 / per_n; n <= (t1 - 1) / per_n; ++n) {
                const int64_t blo = ((int64_t)(n * per_n + 1) * grid + tiles - 1) / tiles - 1;
                maxb = std::max(maxb, (int)(b - blo) + 1);
            }
        }
        Conv3Args b = a;
        DetArena arena;
        const int64_t nslot = (int64_t)maxb * 8 * P_C;
        SG2_DET_GET(b.det_dot, arena, a.N * nslot, "sg2_conv3x3 (c64 persistent)");
        b.det_maxb = maxb;
        hipError_t e = zero_fill(b.det_dot, a.N * nslot * sizeof(float), s);
        if (e) { set_error("sg2_conv3x3 (c64 persistent): zero"); return (int)e; }
        kern<<<grid, 512, P_LDS, s>>>(b, tiles);
        if (int rc = launch_status("sg2_conv3x3 (c64 persistent)")) return rc;
        e = det_sum(a.dot_out, P_C, b.det_dot, nslot, P_C, a.N, (int64_t)maxb * 8, P_C, arena, s, det_assign());
        if (e) { set_error("sg2_conv3x3 (c64 persistent): det_sum"); return (int)e; }
        return 0;
    }
    kern<<<grid, 512, P_LDS, s>>>(a, tiles);
    return launch_status("sg2_conv3x3 (c64 persistent)");
}

template <typename T, bool SI, bool EPI>
int launch_c64p_dot(const Conv3Args& a, hipStream_t s, int tiles, int grid) {
    return a.dot_out ? launch_c64p<T, SI, EPI, true>(a, s, tiles, grid) : launch_c64p<T, SI, EPI, false>(a, s, tiles, grid);
}

int num_cus() {
    static const int n = [] {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return 256;
        return v > 0 ? v : 256;
    }();
    return n;
}

// ---------------------------------------------------------------------------------------------------
// Ring form of the 64 -> 64 channel layer (round 3; the 256^2 layer of the Claro network, 512^2 at cbase 32768).
// The persistent kernel above keeps the 74 KB of weights in LDS, which leaves room for only two 39 KB halo
// chunks: one being read by the MFMAs, one in flight, and every byte of it staged through registers by the
// computing waves (load -> wait -> modulate -> ds_write), so each CU had ~39 KB of HBM reads in flight and the
// memory phases added to the MFMA phase instead of hiding under it.  Here:
//   * the weights live in REGISTERS: wave w owns output channels 32 (w & 1) .. +31 (two A fragments per tap and
//     chunk: 36 x 16 B = 144 VGPRs), so the whole LDS is a 3-slot ring of 32 x 8 pixel tiles (10 x 40 halo
//     positions of whole 128-byte pixel lines, 51,200 B a slot) -- two tiles (~100 KB) in flight per CU;
//   * the halo arrives by LDS-DMA (buffer_load ... lds, 16 B a lane, one 1 KiB wave-instruction = 8 whole pixel
//     lines), issued two tiles ahead, with no register and no LDS-store pass; out-of-image pixels are buffer
//     out-of-range loads, which land as zeros.  The DMA destination is lane-linear, so the bank swizzle sits in
//     the SOURCE address: the 16-byte piece j of position p is stored at j ^ (((p >> 1) & 3) << 1) (conflict-free
//     ds_read_b128 of 16 consecutive positions at any tap shift; the 40-position row pitch keeps p mod 8 a
//     function of the lane and kx only, so each read is a per-lane base + an immediate offset);
//   * the modulation x * s moves onto the weights: once per sample each wave multiplies its register-resident
//     fragments by s rounded to T (round(W * round(s)) where the reference rounds x * round(s): a product
//     rounded once either way);
//   * the tile's noise and demodulation scales arrive by a 1 KiB LDS-DMA into a 4-deep epilogue ring;
//   * one barrier per tile and counted vmcnt waits (never 0 in the loop);
//   * (default form, TH = 4) two workgroups of 4 waves per CU, each on its own 32 x 4 tiles with a 2-slot ring,
//     so that a SIMD's two waves belong to workgroups that drift apart: one's MFMAs run beside the other's
//     epilogue VALU, stores and barrier wait (measured: the memory streams alone -- the halo DMA 0.053 ms, the
//     stores at 7 TB/s, tools/membench.py -- are well under the kernel time; its one-workgroup 8-wave form
//     spent the difference with both waves of a SIMD in the same phase).
// Wave w: rows 2 (w >> 1), +1 of the tile (4 pixel fragments of 16) x its 32 channels: per tap and chunk 4
// ds_read_b128 (pixels) feed 8 MFMAs (weights from registers).
constexpr int R_TW = 32, R_PITCH = 40;
constexpr int R_EPI = 1024, R_NEPI = 4;               // noise [TH x 32] T at 0, demod [64] f32 at 512
// Two forms (template TH): TH = 8 -- 32 x 8 tiles, 8 waves, one workgroup per CU, a 3-slot ring (two tiles in
// flight); TH = 4 -- 32 x 4 tiles, 4 waves, TWO workgroups per CU, each with a 2-slot ring.  The waves of a
// workgroup meet at one barrier per tile, so in the one-workgroup form a SIMD's two waves reach their MFMA,
// epilogue and barrier phases together; two workgroups drift apart and one's MFMAs run beside the other's
// epilogue, stores and barrier wait.
template <int TH, int WR> struct Ring {
    static constexpr int NW = 2 * TH / WR;                            // waves: 2 channel halves x TH / WR row groups
    static constexpr int NSLOT = TH == 8 ? 3 : 2;
    static constexpr int HPOS = (TH + 2) * R_PITCH;                   // halo positions (34 used per row)
    static constexpr int SLOT = HPOS * 128;                           // 51,200 / 30,720 B
    static constexpr int HALO_I = HPOS / 8;                           // halo DMA wave-instructions per tile
    static constexpr int DMA = (HALO_I + 1 + NW - 1) / NW;            // per wave and tile (+ the epilogue table)
    static constexpr size_t LDS = (size_t)NSLOT * SLOT + R_NEPI * R_EPI + 64 * 4 + 16;   // + gain * bias [64], a broadcast word
    static constexpr int WGS_PER_CU = TH == 8 ? 1 : 2;
    static_assert(LDS * WGS_PER_CU <= 160 * 1024, "ring LDS");
    static_assert((DMA - 1) * NW <= HALO_I && DMA * NW > HALO_I, "the last DMA round holds the epilogue table");
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;
#ifndef SG2_RDIAG
#define SG2_RDIAG 0         // timing-only builds of the ring kernel (tools/ring_diag.sh): 16 no loads, 32 no stores, 64 no MFMA
                            // (128: the pad lanes load the pixels that follow, the round-3 first form;
                            //  256: whole-line store addressing with the data misplaced)
#endif

#if SG2_RDIAG & 512
// Diagnostic build only (tools/ring_stamps.py): per wave, the summed cycles of each loop phase of the ring kernel
// from s_memtime stamps (issue DMAs | MFMAs issued | epilogue + stores issued | DMA wait | barrier), the first and
// last stamp and the hardware wave id, written once at the end by lane 0 (vector stores; nothing in the loop).
constexpr int RST_WAVES = 4096, RST_F = 10;
__device__ unsigned long long g_ring_stamps[RST_WAVES * RST_F];
__device__ __forceinline__ unsigned long long ring_stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#endif

__device__ __forceinline__ unsigned lds_addr(const void* p) {    // byte address in LDS of a __shared__ pointer
    return (unsigned)(uintptr_t)(__attribute__((address_space(3))) const char*)p;
}

template <int N>
__device__ __forceinline__ void wait_vm() {           // s_waitcnt vmcnt(N) (gfx9 encoding), expcnt / lgkmcnt untouched
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// STG & 16: a dynamic tail within each sample.  The ring kernel is persistent with a static split of the tiles, and
// the CUs do not run at one speed (the in-kernel clock differs by ~8 % between XCDs under this load and the
// slowest workgroup of a launch ended ~17 % after the median one, tools/ring_stamps.py).  Here the workgroups of a
// sample (grid / N of them, dealt round-robin over the XCDs) keep static runs of `dyn.s_per_wg` tiles and take the
// sample's remaining tiles in chunks of two vertically adjacent tiles from the sample's device-scope counter: a
// workgroup grabs its next chunk one tile before it needs it (one returning atomic by one lane, broadcast through
// LDS at the tile's barrier) and leaves when the counter passes the sample's last chunk.  Every chunk is in the
// workgroup's own sample, so its weights stay modulated (a chunk of another sample re-modulated them: tried, the
// reloads cost more than the balance gained).  The last workgroup of a sample to leave resets the sample's counter
// pair for the next launch.  Which workgroup runs a tile never changes its result (no cross-tile reductions).
struct RingDyn {
    int* q;             // [grab counter per sample][N], then [done counter per sample][N] (zero between launches)
    int s_per_wg;       // static tiles per workgroup (>= 2)
    int wg_per_n;       // workgroups per sample (grid = N wg_per_n)
    int nchunks;        // dynamic chunks of 2 tiles per sample after its static runs
    // a dynamic tile's coordinates without runtime divisions: x / d = umulhi(x, m_d) for x d < 2^32
    // (m_d = floor(2^32 / d) + 1; d >= 2), band = 1 << band_sh
    unsigned m_pern, m_pband;
    int band_sh;
};
constexpr int RQ_SLOTS = 64, RQ_MAXN = 4096;
__device__ int g_ring_q[RQ_SLOTS * 2 * RQ_MAXN];

template <typename T, bool SI, bool EPI, bool RAW, int R_TH, int WR, bool PIPE, int STG>
__global__ __launch_bounds__((Ring<R_TH, WR>::NW) * 64, (Ring<R_TH, WR>::WGS_PER_CU)) void conv3x3_c64r_kernel(Conv3Args a, int tiles_total, int band, RingDyn dyn) {
    typedef T vec8 __attribute__((ext_vector_type(8)));
    typedef Ring<R_TH, WR> RG;
    constexpr int NF = 2 * WR;                        // pixel fragments (16 px) per wave
    constexpr int R_NSLOT = RG::NSLOT, R_SLOT = RG::SLOT, R_HALO_I = RG::HALO_I, R_DMA = RG::DMA, NW = RG::NW;
    constexpr int S = (RAW ? 2 : 1) * 2 * WR;         // buffer stores per wave and tile
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    char* epil = smem_raw + R_NSLOT * R_SLOT;
    float* blds = (float*)(epil + R_NEPI * R_EPI);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l16 = lane & 15, q = lane >> 4;
    const int h = wave & 1, wr = wave >> 1;           // channel half, tile row group (rows WR wr .. + WR - 1)
    constexpr bool DYN = (STG & 16) != 0;
    const int dyn_n = DYN ? (int)blockIdx.x / dyn.wg_per_n : 0;                       // the workgroup's sample
    const int dyn_per_n = DYN ? tiles_total / a.N : 0;
    const int t_begin = DYN ? dyn_n * dyn_per_n + ((int)blockIdx.x - dyn_n * dyn.wg_per_n) * dyn.s_per_wg
                            : (int)((int64_t)blockIdx.x * tiles_total / gridDim.x);
    const int t_end = DYN ? t_begin + dyn.s_per_wg : (int)((int64_t)(blockIdx.x + 1) * tiles_total / gridDim.x);
    const int dyn_base = DYN ? dyn_n * dyn_per_n + dyn.wg_per_n * dyn.s_per_wg : 0;
    if (t_begin >= t_end) return;
    // tile t -> (n, ty, tx): samples, bands of `band` tile rows, column-major inside a band (vertical neighbours,
    // which share two halo rows, are consecutive in a CU's run).  Lane j of tinfo0 / tinfo1 holds tile
    // t_begin + j / + 64 + j packed, so a tile's coordinates are one v_readlane in the loop, not three runtime
    // divisions (the host sends at most 128 tiles per workgroup here)
    auto pack_tile = [&](int t) -> int {
        const int tiles_x = a.W / R_TW, per_n = tiles_x * (a.H / R_TH), per_band = band * tiles_x;
        const int n = t / per_n, r = t - n * per_n, b = r / per_band, rb = r - b * per_band, col = rb / band;
        return (n << 20) | ((b * band + rb - col * band) << 10) | col;
    };
    const int tinfo0 = t_begin + lane < t_end ? pack_tile(t_begin + lane) : 0;
    const int tinfo1 = t_begin + 64 + lane < t_end ? pack_tile(t_begin + 64 + lane) : 0;
    // a dynamic tile (uniform t): the same packing by multiply-high (RingDyn), ~6 scalar instructions where the three
    // signed divisions took ~90
    auto pack_tile_dyn = [&](int t) -> int {
        const int tiles_x = a.W / R_TW, per_n = tiles_x * (a.H / R_TH), per_band = tiles_x << dyn.band_sh;
        const int n = (int)__builtin_amdgcn_readfirstlane(__umulhi((unsigned)t, dyn.m_pern)), r = t - n * per_n;
        const int b = (int)__builtin_amdgcn_readfirstlane(__umulhi((unsigned)r, dyn.m_pband)), rb = r - b * per_band;
        const int col = rb >> dyn.band_sh;
        return (n << 20) | (((b << dyn.band_sh) + rb - (col << dyn.band_sh)) << 10) | col;
    };
    auto tile_of = [&](int t, int& n, int& ty, int& tx) {
        const int j = t - t_begin;
        int v;
        if (DYN && (unsigned)j >= (unsigned)(t_end - t_begin)) v = pack_tile_dyn(t);   // a dynamic tile
        else v = j < 64 ? __builtin_amdgcn_readlane(tinfo0, j) : __builtin_amdgcn_readlane(tinfo1, j - 64);
        n = (int)((unsigned)v >> 20);      // unsigned: a sample index >= 2048 sets bit 31
        ty = ((v >> 10) & 1023) * R_TH;
        tx = (v & 1023) * R_TW;
    };
    // (the host checked N H W 64 sizeof(T) < 2^31; readfirstlane keeps the descriptors provably uniform -- a
    // descriptor hipcc cannot prove uniform is rebuilt per lane in a readfirstlane loop around every load)
    const int xbytes = __builtin_amdgcn_readfirstlane(a.N * a.H * a.W * 64 * (int)sizeof(T));
    const __amdgpu_buffer_rsrc_t rxb = make_rsrc(a.x, xbytes);
    const __amdgpu_buffer_rsrc_t rwb = make_rsrc(a.w, 64 * 9 * 64 * (int)sizeof(T));
    const __amdgpu_buffer_rsrc_t rsc = make_rsrc(a.in_scale, SI ? __builtin_amdgcn_readfirstlane(a.N * 64 * 4) : 0);
    const __amdgpu_buffer_rsrc_t ryb = make_rsrc(a.y, xbytes);
    const __amdgpu_buffer_rsrc_t ryr = make_rsrc(a.y_raw, RAW ? xbytes : 0);

    // ---- weights: this wave's 2 x 9 x 2 A fragments, modulated by the sample's styles ----
    vec8 wf[2][9][2];
    auto load_weights = [&](int n) {
        float4 s4[2][2];
        if (SI) {
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) s4[c][hh] = buf_load16<float4>(rsc, (n * 64 + c * 32 + q * 8 + hh * 4) * 4);
        }
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            const int o = p_chan(16 * (2 * h + jj) + l16);
#pragma unroll
            for (int tap = 0; tap < 9; ++tap)
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    vec8 v = buf_load16<vec8>(rwb, ((o * 9 + tap) * 64 + c * 32 + q * 8) * (int)sizeof(T));
                    if (SI) {
                        const float4 x0 = s4[c][0], x1 = s4[c][1];
                        const vec8 sv = vec8{(T)x0.x, (T)x0.y, (T)x0.z, (T)x0.w, (T)x1.x, (T)x1.y, (T)x1.z, (T)x1.w};
                        if constexpr (std::is_same<T, f16_t>::value) {
                            v = v * sv;                // v_pk_mul_f16: round(w * round(s))
                        } else {
#pragma unroll
                            for (int e = 0; e < 8; ++e) v[e] = (T)((float)v[e] * (float)sv[e]);
                        }
                    }
                    wf[jj][tap][c] = v;
                }
        }
    };
    int cur_n;
    {
        int ty, tx;
        tile_of(t_begin, cur_n, ty, tx);
    }
    load_weights(cur_n);
    if (tid < 64) blds[tid] = (EPI && a.bias) ? (float)(T)a.bias[tid] * a.gain : 0.f;

    // ---- LDS-DMA issue: wave w owns instructions i = u * NW + w, u < R_DMA ----
    const bool has_noise = EPI && a.noise != nullptr, has_d = EPI && a.out_scale != nullptr;
    const char* epi_src0 = has_noise ? (const char*)a.noise : (has_d ? (const char*)a.out_scale : (const char*)a.x);
    const char* epi_src1 = has_d ? (const char*)a.out_scale : epi_src0;
    // Instruction i < 50 loads halo row hy = i / 5, columns (i % 5) * 8 + lane / 8 (8 whole pixel lines); the
    // stored piece lane % 8 holds global piece j = (lane % 8) ^ swizzle, a function of the lane only (the column
    // group adds a multiple of 8).  Row validity is wave-uniform; column validity per lane.
    const int lx = lane >> 3;
    const int hlane = lx * 128 + (((lane & 7) ^ (((lx >> 1) & 3) << 1)) * 16);
    // epilogue table: lanes 0-31 the tile's noise (row (lane / 4) mod TH, 16-byte piece lane % 4; with TH = 4 lanes
    // 16-31 repeat rows 0-3 into the unused rows 4-7 of the table), lanes 32-63 the sample's demodulation scales
    // (16 bytes a lane; lanes 48-63 repeat 32-47 into the unused tail of the table)
    // (without noise the first half reads the start of whichever buffer stands in for it: always in bounds)
    const int elane = lane < 32 ? (has_noise ? (((lane >> 2) % R_TH) * a.W + (lane & 3) * 8) * (int)sizeof(T) : 0)
                                : ((lane - 32) & 15) * 16;
    auto issue = [&](int t, int slot, int eslot) {
        if (SG2_RDIAG & 16) return;                   // timing-only build: no loads
        int n, ty, tx;
        tile_of(t, n, ty, tx);
#pragma unroll
        for (int u = 0; u < R_DMA; ++u) {
            const int i = u * NW + wave;              // wave-uniform; u < R_DMA - 1: always a halo instruction
            if (u < R_DMA - 1 || i < R_HALO_I) {
                const int hy = i / 5, cg = i - hy * 5;
                const int iy = ty - 1 + hy, ix0 = tx - 1 + cg * 8;
                // uniform row base; a row outside the image gets a negative base (every lane out of range: zeros).
                // Per lane the image's left / right border column reads zeros, and the pad lanes (column 34 .. 39
                // of the halo row, never read) read nothing: an out-of-range lane moves no bytes (15 % of the
                // halo's requests)
                const int base = (unsigned)iy < (unsigned)a.H ? ((n * a.H + iy) * a.W + ix0) * 128 : -(1 << 30);
                const bool kill = ((tx == 0) & (cg == 0) & (lx == 0)) | ((tx + R_TW == a.W) & (cg == 4) & (lx == 1)) |
                                  (!(SG2_RDIAG & 128) & (cg == 4) & (lx >= 2));
                const int off = kill ? -1 : base + hlane;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rxb, (lds_ptr_t)(smem_raw + slot * R_SLOT + i * 1024), 16, off, 0, 0, 0);
            } else {                                  // the epilogue table (duplicates write the same bytes)
                const char* nb = has_noise ? epi_src0 + (int64_t)((n * a.H + ty) * a.W + tx) * (int)sizeof(T) : epi_src0;
                const char* db = has_d ? epi_src1 + n * 256 : epi_src1;
                const char* src = (lane < 32 ? nb : db) + elane;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                                 (lds_ptr_t)(epil + eslot * R_EPI), 16, 0, 0);
            }
        }
    };

    // STG & 4 (TH = 4, 4 waves): the same DMAs with the tile-independent parts of their addresses hoisted out of the
    // loop and every column group a compile-time constant of the instruction: wave w loads halo row w (column groups
    // 0..4), then waves 0 / 1 row 4 / 5 column groups 0..2 and waves 2 / 3 row 4 / 5 column groups 3, 4 and the
    // epilogue table (both: duplicates write the same bytes).  Per DMA: one scalar add for the row base (twice a
    // tile), one vector add, a select on the border columns only -- where the generic issue above spends ~20
    // instructions (a runtime division, the row-validity branch and the per-lane kill logic) on each.
    const int rs_w = a.W * 128;
    auto issue_fast_at = [&](int n, int ty, int tx, int slot, int eslot) {
        if constexpr (R_TH == 4 && NW == 4) {
            if (SG2_RDIAG & 16) return;
            const int base0 = ((n * a.H + ty - 1) * a.W + tx - 1) * 128;     // halo row 0, column -1
            const int rowA = wave, rowB = 4 + (wave & 1);
            // an invalid row: every lane out of range (INT_MIN + < 8 KiB stays above any buffer of < 2^31 - 2^16 B)
            const int bA = (rowA == 0 && ty == 0) ? (int)0x80000000 : base0 + rowA * rs_w;
            const int bB = (rowB == R_TH + 1 && ty + R_TH == a.H) ? (int)0x80000000 : base0 + rowB * rs_w;
            const bool killL = (tx == 0) & (lx == 0);
            const bool killR = (!(SG2_RDIAG & 128) & (lx >= 2)) | ((tx + R_TW == a.W) & (lx == 1));
            char* sb = smem_raw + slot * R_SLOT;
            auto dma = [&](int b, int row, int cg) {
                int off = b + cg * 1024 + hlane;
                if (cg == 0) off = killL ? -1 : off;
                if (cg == 4) off = killR ? -1 : off;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rxb, (lds_ptr_t)(sb + (row * 5 + cg) * 1024), 16, off, 0, 0, 0);
            };
#pragma unroll
            for (int cg = 0; cg < 5; ++cg) dma(bA, rowA, cg);
            if (wave < 2) {
#pragma unroll
                for (int cg = 0; cg < 3; ++cg) dma(bB, rowB, cg);
            } else {
                dma(bB, rowB, 3);
                dma(bB, rowB, 4);
                const char* nb = has_noise ? epi_src0 + (int64_t)((n * a.H + ty) * a.W + tx) * (int)sizeof(T) : epi_src0;
                const char* db = has_d ? epi_src1 + n * 256 : epi_src1;
                const char* src = (lane < 32 ? nb : db) + elane;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                                 (lds_ptr_t)(epil + eslot * R_EPI), 16, 0, 0);
            }
        }
    };
    auto issue_any = [&](int t, int slot, int eslot) {
        if constexpr ((STG & 4) != 0) {
            int n, ty, tx;
            tile_of(t, n, ty, tx);
            issue_fast_at(n, ty, tx, slot, eslot);
        } else {
            issue(t, slot, eslot);
        }
    };

    // MFMA B-fragment addressing: pixel fragment i of the wave at tap (ky, kx), chunk c reads position
    // (2 wr + (i >> 1) + ky) * 40 + (i & 1) * 16 + l16 + kx, piece c * 4 + q (swizzled as at the DMA)
    int boff[3][2];
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int x = l16 + kx;
            boff[kx][c] = (WR * wr * R_PITCH + x) * 128 + 16 * ((c * 4 + q) ^ (((x >> 1) & 3) << 1));
        }

    const float lr_alpha = (EPI && a.act == 1) ? a.alpha : 1.f;
    const float clampv = (EPI && a.clamp >= 0.f) ? a.clamp : __builtin_inff();
    const float ngain = a.noise_gain * a.gain;
    const int ch0 = 32 * h + 8 * q;                   // this lane's 8 output channels

    // The epilogue tables are read by inline-asm ds_reads: an LDS-DMA writes this ring, so hipcc would put an
    // s_waitcnt vmcnt(0) before any ds_read it can see here, draining the tiles in flight.  The ring discipline
    // (the DMA of the tile was waited for and a barrier passed) is what orders these reads.  Branch-free: a
    // missing noise / demod table is read anyway (its DMA read a stand-in buffer) and selected away.
    auto epi_table = [&](int eslot, float (&bb)[8], float (&dd)[8], float (&nz)[NF]) {
        if (!EPI) return;
        const unsigned et = lds_addr(epil + eslot * R_EPI);
        float4 b0, b1, d0, d1;
        asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\t"
                     "ds_read_b128 %2, %5 offset:512\n\tds_read_b128 %3, %5 offset:528\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(b0), "=&v"(b1), "=&v"(d0), "=&v"(d1)
                     : "v"(lds_addr(blds + ch0)), "v"(et + ch0 * 4));
        const float bq[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        const float dq[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            bb[e] = bq[e];
            dd[e] = has_d ? dq[e] * a.gain : a.gain;
        }
        // pixel (WR wr + (i >> 1)) * 32 + (i & 1) * 16 + l16 of the table: byte offset 32 i from na
        const unsigned na = et + (WR * wr * R_TW + l16) * (unsigned)sizeof(T);
#pragma unroll
        for (int g = 0; g < NF / 4; ++g) {
            unsigned r0, r1, r2, r3;
            asm volatile("ds_read_u16 %0, %4\n\tds_read_u16 %1, %4 offset:32\n\tds_read_u16 %2, %4 offset:64\n\t"
                         "ds_read_u16 %3, %4 offset:96\n\ts_waitcnt lgkmcnt(0)"
                         : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3) : "v"(na + 128 * g));
            const unsigned rr[4] = {r0, r1, r2, r3};
#pragma unroll
            for (int j = 0; j < 4; ++j)
                nz[4 * g + j] = has_noise ? (float)__builtin_bit_cast(T, (unsigned short)rr[j]) * ngain : 0.f;
        }
    };
    // the epilogue math and stores of one tile from its accumulators: pure VALU + buffer stores, no branch, so
    // in the pipelined form it shares a basic block (and the scheduler's interleave) with the next tile's MFMAs
    auto epi_store = [&](f32x4 (&A)[NF][2], int n, int ty, int tx, const float (&bb)[8], const float (&dd)[8],
                         const float (&nz)[NF]) {
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int r = WR * wr + (i >> 1), px = (i & 1) * 16 + l16;
            const int pix = (n * a.H + ty + r) * a.W + tx + px;
            vec8 yv, rv;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float cv = A[i][e >> 2][e & 3];
                if (RAW) rv[e] = (T)cv;
                float v = cv;
                if (EPI) {
                    v = fmaf(v, dd[e], nz[i] + bb[e]);
                    v = fmaxf(v, v * lr_alpha);
                    v = __builtin_amdgcn_fmed3f(v, -clampv, clampv);
                }
                yv[e] = (T)v;
            }
            int dst = (pix * 64 + ch0) * (int)sizeof(T) | -(int)((SG2_RDIAG & 32) != 0);   // timing-only build: dropped
            if (SG2_RDIAG & 256)   // timing-only build: the same bytes as whole-line stores (8 px x 128 B an instruction)
                dst = (((n * a.H + ty + WR * wr + h) * a.W + tx + i * 8 + (lane >> 3)) * 64 + (lane & 7) * 8) * (int)sizeof(T);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, yv), ryb, dst, 0, 0);
            if (RAW) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, rv), ryr, dst, 0, 0);
        }
    };
    // STG: the same epilogue with whole-line stores.  The tile's outputs go through the slot its MFMAs just
    // consumed (free until the next iteration's DMA into it, which follows the loop's last barrier): each wave
    // writes its 16-byte pieces (8 channels of a pixel) into a [128 px][128 B] image, piece c of pixel P at
    // c ^ (P & 7) (conflict-free ds_write_b128 and ds_read_b128), then reads back whole 128-byte pixel lines, 8
    // pixels per wave-instruction, and stores those.  Measured with a timing build (RDIAG 256): the half-line
    // stores' texture-address cost beside the halo DMAs was 11 % of the launch.  Two more barriers (four with
    // the raw output, staged in a second round).
    auto epi_store_staged = [&](f32x4 (&A)[NF][2], int slot, int n, int ty, int tx, const float (&bb)[8],
                                const float (&dd)[8], const float (&nz)[NF]) {
        if constexpr (WR == 2) {                      // (staged stores: two rows per wave pair)
        const unsigned sb = lds_addr(smem_raw + slot * R_SLOT);
        u32x4 yq[NF], rq[NF];
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            vec8 yv, rv;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float cv = A[i][e >> 2][e & 3];
                if (RAW) rv[e] = (T)cv;
                float v = cv;
                if (EPI) {
                    v = fmaf(v, dd[e], nz[i] + bb[e]);
                    v = fmaxf(v, v * lr_alpha);
                    v = __builtin_amdgcn_fmed3f(v, -clampv, clampv);
                }
                yv[e] = (T)v;
            }
            yq[i] = __builtin_bit_cast(u32x4, yv);
            rq[i] = __builtin_bit_cast(u32x4, rv);
        }
        auto stage_store = [&](const u32x4 (&v)[NF], const __amdgpu_buffer_rsrc_t& rout) {
#pragma unroll
            for (int i = 0; i < NF; ++i) {
                const int P = (2 * wr + (i >> 1)) * R_TW + (i & 1) * 16 + l16;
                const unsigned off = sb + P * 128 + (((4 * h + q) ^ (P & 7)) << 4);
                asm volatile("ds_write_b128 %0, %1" :: "v"(off), "v"(v[i]) : "memory");
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_s_barrier();
            const int c = lane & 7, row = 2 * wr + h;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int px = 8 * j + (lane >> 3), P = row * R_TW + px;
                u32x4 w;
                asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(w) : "v"(sb + P * 128 + ((c ^ (P & 7)) << 4)));
                const int pix = (n * a.H + ty + row) * a.W + tx + px;
                __builtin_amdgcn_raw_buffer_store_b128(w, rout, (pix * 64 + c * 8) * (int)sizeof(T), 0, 0);
            }
        };
        __builtin_amdgcn_s_waitcnt(0xc07f);           // every wave is done reading the slot's halo
        __builtin_amdgcn_s_barrier();
        stage_store(yq, ryb);
        if (RAW) {
            __builtin_amdgcn_s_barrier();             // the y image has been read back
            stage_store(rq, ryr);
        }
        }
    };
    auto mfma_tile = [&](f32x4 (&A)[NF][2], const char* hb) {
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    v8<T> pf[NF];
#pragma unroll
                    for (int i = 0; i < NF; ++i)
                        pf[i] = *(const v8<T>*)(hb + boff[kx][c] + (((i >> 1) + ky) * R_PITCH + (i & 1) * 16) * 128);
                    const bool first = c == 0 && ky == 0 && kx == 0;   // the tile's first tap starts each chain at 0
#pragma unroll
                    for (int i = 0; i < NF; ++i)
#pragma unroll
                        for (int jj = 0; jj < 2; ++jj) {
                            if (SG2_RDIAG & 64) A[i][jj][0] = (first ? 0.f : A[i][jj][0]) + (float)pf[i][jj] * (float)wf[jj][ky * 3 + kx][c][i];   // timing-only build
                            else A[i][jj] = mma<T>(wf[jj][ky * 3 + kx][c], pf[i], first ? f32x4{0.f, 0.f, 0.f, 0.f} : A[i][jj]);
                        }
                }
    };

    // ---- prologue: tiles 0 .. NSLOT - 2 in flight, wait for tile 0 ----
    issue_any(t_begin, 0, 0);
    if (R_NSLOT == 3) {
        issue_any(min(t_begin + 1, t_end - 1), 1, 1);
        wait_vm<R_DMA>();
    } else {
        wait_vm<0>();
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);               // lgkmcnt(0): the bias table
    __builtin_amdgcn_s_barrier();

    int k = 0;
#if SG2_RDIAG & 512
    unsigned long long st_sum[5] = {0, 0, 0, 0, 0}, st_first = ring_stamp(), st_prev = st_first;
    const unsigned long long rt_first = __builtin_amdgcn_s_memrealtime();
    auto st = [&](int ph) { const unsigned long long t = ring_stamp(); st_sum[ph] += t - st_prev; st_prev = t; };
#define RING_STAMP(ph) st(ph)
#else
#define RING_STAMP(ph) ((void)0)
#endif
    if constexpr (DYN) {
        static_assert(R_NSLOT == 2 && !PIPE, "dynamic tail: the 2-slot form");
        int* qlds = (int*)(blds + 64);               // the broadcast word (16 bytes past the bias table)
        int* qn = dyn.q + dyn_n;                      // this sample's grab counter
        f32x4 acc[NF][2];
        int cur = t_begin, rend = t_end, gv = 0;
        int cn, cty, ctx;                                 // the current tile's coordinates (carried from its issue)
        tile_of(cur, cn, cty, ctx);
        for (;; ++k) {
            int nxt;
            if (cur + 1 < rend) {
                nxt = cur + 1;
            } else {
                unsigned qv;
                asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(qv) : "v"(lds_addr(qlds)));
                const int qc = __builtin_amdgcn_readfirstlane((int)qv);
                nxt = qc < dyn.nchunks ? dyn_base + 2 * qc : -1;
            }
            const bool grab = cur + 2 == rend;            // second-to-last tile of its run / chunk: grab the next chunk
            if (grab && wave == 0 && lane == 0) gv = __hip_atomic_fetch_add(qn, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int slot = k % R_NSLOT;
            const int n = cn, ty = cty, tx = ctx;
            if (nxt >= 0) tile_of(nxt, cn, cty, ctx);
            if constexpr ((STG & 4) != 0) issue_fast_at(cn, cty, ctx, (k + 1) % R_NSLOT, (k + 1) % R_NEPI);
            else issue(nxt >= 0 ? nxt : cur, (k + 1) % R_NSLOT, (k + 1) % R_NEPI);
            RING_STAMP(0);
            mfma_tile(acc, smem_raw + slot * R_SLOT);
            RING_STAMP(1);
            float bb[8], dd[8], nz[NF];
            epi_table(k % R_NEPI, bb, dd, nz);
            epi_store(acc, n, ty, tx, bb, dd, nz);
            RING_STAMP(2);
            if (grab && wave == 0) {
                const int g0 = __builtin_amdgcn_readfirstlane(gv);
                asm volatile("ds_write_b32 %0, %1" :: "v"(lds_addr(qlds)), "v"(g0) : "memory");
            }
            wait_vm<S>();
            RING_STAMP(3);
            __builtin_amdgcn_s_waitcnt(0xc07f);       // lgkmcnt(0): this tile's LDS reads (and the q write) are done
            __builtin_amdgcn_s_barrier();
            RING_STAMP(4);
            if (nxt < 0) break;
            if (nxt != cur + 1) rend = nxt + 2;        // a new chunk
            cur = nxt;
        }
    } else if constexpr (!PIPE) {
        f32x4 acc[NF][2];
        for (int t = t_begin; t < t_end; ++t, ++k) {
            const int slot = k % R_NSLOT;
            issue_any(min(t + R_NSLOT - 1, t_end - 1), (k + R_NSLOT - 1) % R_NSLOT, (k + R_NSLOT - 1) % R_NEPI);
            int n, ty, tx;
            tile_of(t, n, ty, tx);
            if (SI && n != cur_n) {                   // a new sample: re-modulate the weights (rare)
                cur_n = n;
                load_weights(n);
            }
            RING_STAMP(0);
            mfma_tile(acc, smem_raw + slot * R_SLOT);
            RING_STAMP(1);
            float bb[8], dd[8], nz[NF];
            epi_table(k % R_NEPI, bb, dd, nz);
            if constexpr (STG == 1) epi_store_staged(acc, slot, n, ty, tx, bb, dd, nz);
            else epi_store(acc, n, ty, tx, bb, dd, nz);
            RING_STAMP(2);
            // tile t + 1's DMAs must have landed: everything but the youngest ops of this wave.  3 slots: t + 1
            // was issued one iteration ago, younger are this iteration's DMAs and stores and the previous
            // iteration's stores; 2 slots: t + 1 was issued at the top of this iteration, younger are this
            // iteration's stores
            if (R_NSLOT == 2) wait_vm<S>();
            else if (k == 0) wait_vm<R_DMA + S>();
            else wait_vm<R_DMA + 2 * S>();
            RING_STAMP(3);
            __builtin_amdgcn_s_waitcnt(0xc07f);       // lgkmcnt(0): this tile's LDS reads are done
            __builtin_amdgcn_s_barrier();
            RING_STAMP(4);
        }
    } else {
        // Pipelined epilogue (3-slot form): iteration k runs tile k's MFMAs into one accumulator set and tile
        // k - 1's epilogue from the other in the same basic block, so the epilogue's VALU and stores issue
        // between MFMAs instead of after them.  The epilogue table of tile k - 1 (its epilogue-ring slot is
        // rewritten three iterations later) is read at the top of the iteration.
        static_assert(!PIPE || R_NSLOT == 3, "pipelined epilogue: 3-slot ring");
        f32x4 acc0[NF][2], acc1[NF][2];
        int t = t_begin, pn = 0, pty = 0, ptx = 0;
        auto step = [&](auto has_prev, f32x4 (&Acur)[NF][2], f32x4 (&Aprev)[NF][2]) {
            constexpr bool HP = decltype(has_prev)::value;
            const int slot = k % R_NSLOT;
            issue(min(t + R_NSLOT - 1, t_end - 1), (k + R_NSLOT - 1) % R_NSLOT, (k + R_NSLOT - 1) % R_NEPI);
            int n, ty, tx;
            tile_of(t, n, ty, tx);
            if (SI && n != cur_n) {
                cur_n = n;
                load_weights(n);
            }
            float bb[8], dd[8], nz[NF];
            if (HP) epi_table((k + R_NEPI - 1) % R_NEPI, bb, dd, nz);
            mfma_tile(Acur, smem_raw + slot * R_SLOT);
            if (HP) epi_store(Aprev, pn, pty, ptx, bb, dd, nz);
            // tile t + 1's DMAs (issued one iteration ago) must have landed; younger: the stores of the previous
            // iteration (none at k = 1), this iteration's DMAs and its stores (none at k = 0)
            if (k == 0) wait_vm<R_DMA>();
            else if (k == 1) wait_vm<R_DMA + S>();
            else wait_vm<R_DMA + 2 * S>();
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_s_barrier();
            pn = n; pty = ty; ptx = tx;
            ++k; ++t;
        };
        step(std::false_type{}, acc0, acc1);
        bool last0 = true;                            // which set holds the last tile's sums
        while (t < t_end) {
            step(std::true_type{}, acc1, acc0);
            last0 = false;
            if (t >= t_end) break;
            step(std::true_type{}, acc0, acc1);
            last0 = true;
        }
        float bb[8], dd[8], nz[NF];
        epi_table((k + R_NEPI - 1) % R_NEPI, bb, dd, nz);
        if (last0) epi_store(acc0, pn, pty, ptx, bb, dd, nz);
        else epi_store(acc1, pn, pty, ptx, bb, dd, nz);
    }
    wait_vm<0>();                                     // no LDS-DMA may outlive the workgroup
    if constexpr (DYN) {
        // every grab of this workgroup has returned: count it out of its sample; the sample's last one resets the
        // sample's pair for the next launch
        if (wave == 0 && lane == 0) {
            int* dn = dyn.q + a.N + dyn_n;
            const int d = __hip_atomic_fetch_add(dn, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (d == dyn.wg_per_n - 1) {
                __hip_atomic_exchange(dyn.q + dyn_n, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_exchange(dn, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
#if SG2_RDIAG & 512
    {
        const int gw = blockIdx.x * NW + wave;
        if (lane == 0 && gw < RST_WAVES) {
            unsigned long long* o = g_ring_stamps + gw * RST_F;
            for (int ph = 0; ph < 5; ++ph) o[ph] = st_sum[ph];
            o[5] = st_first;
            o[6] = st_prev;
            o[7] = ((unsigned long long)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)) << 32) |
                   (unsigned)(__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11)) << 16 | (t_end - t_begin));
            o[8] = rt_first;
            o[9] = __builtin_amdgcn_s_memrealtime();
        }
    }
#endif
#undef RING_STAMP
}

int* ring_queue_slot() {
    // One counter table per launch in flight: a rotating slot of g_ring_q, each left zero by its launch's
    // workgroups (device globals start zeroed).  The symbol's address is per device, so it is looked up per device.
    // Two launches that share a slot must not run at once: the dynamic tail relies on launches being serialized per
    // slot -- the library's launches of one process are issued to one stream at a time (the trainer's phases, and
    // their graph replays, run in stream order), and RQ_SLOTS launches separate two users of a slot.
    static std::atomic<int*> base[64];
    static std::atomic<unsigned> next{0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    int* b = base[dev].load(std::memory_order_acquire);
    if (!b) {
        if (hipGetSymbolAddress((void**)&b, HIP_SYMBOL(g_ring_q)) != hipSuccess) return nullptr;
        base[dev].store(b, std::memory_order_release);
    }
    return b + 2 * RQ_MAXN * (next.fetch_add(1, std::memory_order_relaxed) % RQ_SLOTS);
}

// The dynamic tail's plan (form 49): static tiles per workgroup, chunk count and the reciprocals of the tile
// decode.  false when the shape cannot take it (the caller then launches the static form 46).
// SG2_RING_DYN: percent of a sample's tiles handed out dynamically (default 12), a whole number of 2-tile chunks.
bool ring_dyn_plan(const Conv3Args& a, int tiles, int grid, int band, RingDyn& dyn) {
    static const int pct = [] { const char* e = getenv("SG2_RING_DYN"); return e ? std::max(0, std::min(50, atoi(e))) : 12; }();
    if (grid % a.N || a.N > RQ_MAXN || (band != 1 && band != 2 && band != 4)) return false;
    const int per_n = tiles / a.N, gpn = grid / a.N;
    const int per_band = band * (a.W / R_TW);
    if (per_n / gpn < 8 || per_n < 2 || per_band < 2 || (int64_t)tiles * per_n >= (1ll << 32)) return false;
    int sp = std::max(2, (int)((int64_t)per_n * (100 - pct) / (100 * (int64_t)gpn)));
    while (sp > 2 && (per_n - gpn * sp) % 2) --sp;
    if (gpn * sp > per_n || (per_n - gpn * sp) % 2) return false;
    dyn.s_per_wg = sp;
    dyn.wg_per_n = gpn;
    dyn.nchunks = (per_n - gpn * sp) / 2;
    dyn.m_pern = (unsigned)((1ull << 32) / (unsigned)per_n + 1);
    dyn.m_pband = (unsigned)((1ull << 32) / (unsigned)per_band + 1);
    dyn.band_sh = band == 4 ? 2 : (band == 2 ? 1 : 0);
    return true;
}

template <typename T, bool SI, bool EPI, bool RAW, int TH, int WR, bool PIPE, int STG>
int launch_c64r(const Conv3Args& a, hipStream_t s, int tiles, int grid, int band) {
    typedef Ring<TH, WR> RG;
    auto kern = conv3x3_c64r_kernel<T, SI, EPI, RAW, TH, WR, PIPE, STG>;
    static bool attr_set = false;   // benign race: idempotent attribute
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)RG::LDS);
        attr_set = true;
    }
    RingDyn dyn{nullptr, 0, 0, 0, 0u, 0u, 0};
    if ((STG & 16) != 0) {     // the caller (launch_c64r_form) checked ring_dyn_plan
        if (!ring_dyn_plan(a, tiles, grid, band, dyn) || !(dyn.q = ring_queue_slot())) {
            set_error("sg2_conv3x3 (c64 ring): dynamic tail unavailable");
            return -1;
        }
    }
    kern<<<grid, RG::NW * 64, RG::LDS, s>>>(a, tiles, band, dyn);
    return launch_status("sg2_conv3x3 (c64 ring)");
}

template <typename T, bool SI, bool EPI, int TH, int WR, bool PIPE = false, int STG = 0>
int launch_c64r_raw(const Conv3Args& a, hipStream_t s, int tiles, int grid, int band) {
    return a.y_raw ? launch_c64r<T, SI, EPI, true, TH, WR, PIPE, STG>(a, s, tiles, grid, band)
                   : launch_c64r<T, SI, EPI, false, TH, WR, PIPE, STG>(a, s, tiles, grid, band);
}

// form: 4 = 32 x 4 tiles, two workgroups of 4 waves per CU; 46 = form 4 with the hoisted DMA issue (issue_fast,
// the default); 8 = 32 x 8 tiles, one workgroup of 8 waves;
// 44 = form 4 with whole-line stores staged through the consumed slot; 84 = 32 x 8 tiles, one workgroup of 4
// waves with 4 rows each (one wave per SIMD, 512 registers).  (The PIPE
// template form -- tile k - 1's epilogue beside tile k's MFMAs -- spills at 512 registers with the weights in
// VGPRs and is not instantiated.)
template <typename T, bool SI, bool EPI>
int launch_c64r_form(const Conv3Args& a, hipStream_t s, int form) {
    const int th = (form == 4 || form == 44 || form == 46 || form == 49) ? 4 : 8;
    const int tiles = a.N * (a.H / th) * (a.W / R_TW);
    const int ty = a.H / th;
    const int band = ty % 4 == 0 ? 4 : (ty % 2 == 0 ? 2 : 1);
    if (form == 4) return launch_c64r_raw<T, SI, EPI, 4, 2>(a, s, tiles, 2 * num_cus(), band);
    if (form == 44) return launch_c64r_raw<T, SI, EPI, 4, 2, false, 1>(a, s, tiles, 2 * num_cus(), band);

    if (form == 46) return launch_c64r_raw<T, SI, EPI, 4, 2, false, 4>(a, s, tiles, 2 * num_cus(), band);
    if (form == 49) {     // the dynamic tail where its plan exists (whole samples per workgroup group, >= 8 tiles
                          // per workgroup, an even dynamic remainder ...), else the static form 46
        const int grid = 2 * num_cus();
        RingDyn probe{nullptr, 0, 0, 0, 0u, 0u, 0};
        if (ring_dyn_plan(a, tiles, grid, band, probe))
            return launch_c64r_raw<T, SI, EPI, 4, 2, false, 20>(a, s, tiles, grid, band);
        return launch_c64r_raw<T, SI, EPI, 4, 2, false, 4>(a, s, tiles, grid, band);
    }


    if (form == 84) return launch_c64r_raw<T, SI, EPI, 8, 4>(a, s, tiles, num_cus(), band);
    return launch_c64r_raw<T, SI, EPI, 8, 2>(a, s, tiles, num_cus(), band);
}

// ---------------------------------------------------------------------------------------------------
// Ring form of the 32 -> 32 channel layer (the 1024^2 layers of the cbase-32768 networks, BASELINE C5), round 5.
// The C = 64 ring above in 64-byte positions: a pixel line is 32 channels (64 B), so one 1 KiB LDS-DMA
// wave-instruction brings 16 halo positions (4 lanes a position) and one 16-byte output store per lane and
// fragment writes 16 consecutive whole pixels (1 KiB contiguous).  The generic halo kernel ran this layer with half
// of every output-channel tile idle (64-wide tiles of 32 channels) at 0.17 of HBM.
//   * tile 32 x 8 pixels, 4 waves, wave w: rows 2w, 2w+1 (4 fragments of 16 pixels) x all 32 output channels;
//     per tap 4 ds_read_b128 (pixels) feed 8 MFMAs, weights (2 A fragments a tap, one 32-channel chunk: 72 VGPRs)
//     in registers, re-modulated when the run crosses into a new sample;
//   * halo slot: 10 rows x 40 positions of 64 B (34 used a row; the pitch keeps position mod 4 a function of the lane
//     and the tap column: per-lane base + immediate reads), XOR-swizzled as swz64 on the DMA source address;
//     25 DMA pieces a tile (16 consecutive positions each, rows crossed per lane), 2-slot ring, two workgroups per
//     CU; the pieces' per-lane halo offsets and border classes are computed once, a tile adds its base and masks
//     the border lanes (out-of-range loads read zeros);
//   * epilogue ring (noise 8 x 32 and demod 32 of a tile in one 1 KiB DMA) and the epilogue math of the C = 64 form.
constexpr int Q_TW = 32, Q_TH = 8, Q_PITCH = 40, Q_HPOS = (Q_TH + 2) * Q_PITCH;   // 400 positions
constexpr int Q_SLOT = Q_HPOS * 64;                                                // 25,600 B
constexpr int Q_PIECES = Q_HPOS / 16;                                              // 25
constexpr int Q_DMA = 7;                                                           // per wave: 28 slots >= 25 + 1
constexpr int Q_NEPI = 4, Q_EPI = 1024;
constexpr size_t Q_LDS = 2 * (size_t)Q_SLOT + Q_NEPI * Q_EPI + 32 * 4;

template <typename T, bool SI, bool EPI, bool RAW>
__global__ __launch_bounds__(256, 2) void conv3x3_c32r_kernel(Conv3Args a, int tiles_total, int band) {
    typedef T vec8 __attribute__((ext_vector_type(8)));
    constexpr int NF = 4;
    constexpr int S = (RAW ? 2 : 1) * NF;             // buffer stores per wave and tile
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    char* epil = smem_raw + 2 * Q_SLOT;
    float* blds = (float*)(epil + Q_NEPI * Q_EPI);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l16 = lane & 15, q = lane >> 4;
    const int t_begin = (int)((int64_t)blockIdx.x * tiles_total / gridDim.x);
    const int t_end = (int)((int64_t)(blockIdx.x + 1) * tiles_total / gridDim.x);
    if (t_begin >= t_end) return;
    auto pack_tile = [&](int t) -> int {
        const int tiles_x = a.W / Q_TW, per_n = tiles_x * (a.H / Q_TH), per_band = band * tiles_x;
        const int n = t / per_n, r = t - n * per_n, b = r / per_band, rb = r - b * per_band, col = rb / band;
        return (n << 20) | ((b * band + rb - col * band) << 10) | col;
    };
    const int tinfo0 = t_begin + lane < t_end ? pack_tile(t_begin + lane) : 0;
    const int tinfo1 = t_begin + 64 + lane < t_end ? pack_tile(t_begin + 64 + lane) : 0;
    auto tile_of = [&](int t, int& n, int& ty, int& tx) {
        const int j = t - t_begin;
        const int v = j < 64 ? __builtin_amdgcn_readlane(tinfo0, j) : __builtin_amdgcn_readlane(tinfo1, j - 64);
        n = (int)((unsigned)v >> 20);
        ty = ((v >> 10) & 1023) * Q_TH;
        tx = (v & 1023) * Q_TW;
    };
    const int xbytes = __builtin_amdgcn_readfirstlane(a.N * a.H * a.W * 32 * (int)sizeof(T));
    const __amdgpu_buffer_rsrc_t rxb = make_rsrc(a.x, xbytes);
    const __amdgpu_buffer_rsrc_t rwb = make_rsrc(a.w, 32 * 9 * 32 * (int)sizeof(T));
    const __amdgpu_buffer_rsrc_t rsc = make_rsrc(a.in_scale, SI ? __builtin_amdgcn_readfirstlane(a.N * 32 * 4) : 0);
    const __amdgpu_buffer_rsrc_t ryb = make_rsrc(a.y, xbytes);
    const __amdgpu_buffer_rsrc_t ryr = make_rsrc(a.y_raw, RAW ? xbytes : 0);

    // ---- weights: 2 x 9 A fragments (rows: output channels p_chan(16 jj + m), cols: the 32 input channels) ----
    vec8 wf[2][9];
    auto load_weights = [&](int n) {
        float4 s4[2];
        if (SI) {
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) s4[hh] = buf_load16<float4>(rsc, (n * 32 + q * 8 + hh * 4) * 4);
        }
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            const int o = p_chan(16 * jj + l16);
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                vec8 v = buf_load16<vec8>(rwb, ((o * 9 + tap) * 32 + q * 8) * (int)sizeof(T));
                if (SI) {
                    const float4 x0 = s4[0], x1 = s4[1];
                    const vec8 sv = vec8{(T)x0.x, (T)x0.y, (T)x0.z, (T)x0.w, (T)x1.x, (T)x1.y, (T)x1.z, (T)x1.w};
                    if constexpr (std::is_same<T, f16_t>::value) {
                        v = v * sv;                    // round(w * round(s)), as the C = 64 ring
                    } else {
#pragma unroll
                        for (int e = 0; e < 8; ++e) v[e] = (T)((float)v[e] * (float)sv[e]);
                    }
                }
                wf[jj][tap] = v;
            }
        }
    };
    int cur_n;
    {
        int ty, tx;
        tile_of(t_begin, cur_n, ty, tx);
    }
    load_weights(cur_n);
    if (tid < 32) blds[tid] = (EPI && a.bias) ? (float)(T)a.bias[tid] * a.gain : 0.f;

    // ---- DMA geometry: wave w issues pieces i = u * 4 + w (u < Q_DMA); piece i < 25: halo positions 16 i + lane / 4
    // (4 lanes a position), i = 25 + ...: the epilogue table ----
    const bool has_noise = EPI && a.noise != nullptr, has_d = EPI && a.out_scale != nullptr;
    const char* epi_src0 = has_noise ? (const char*)a.noise : (has_d ? (const char*)a.out_scale : (const char*)a.x);
    const char* epi_src1 = has_d ? (const char*)a.out_scale : epi_src0;
    int hoff[Q_DMA], hcls[Q_DMA];                     // per piece: this lane's halo offset (bytes) and border class
#pragma unroll
    for (int u = 0; u < Q_DMA; ++u) {
        const int i = u * 4 + wave;
        const int p = 16 * i + (lane >> 2);
        const int hy = p / Q_PITCH, hx = p - hy * Q_PITCH;
        const int j = (lane & 3) ^ ((p >> 1) & 2);    // swz64 on the source side (lane-linear destination)
        hoff[u] = (hy * a.W + hx) * 64 + j * 16;
        hcls[u] = (hy == 0 ? 1 : 0) | (hy == Q_TH + 1 ? 2 : 0) | (hx == 0 ? 4 : 0) | (hx == Q_TW + 1 ? 8 : 0) |
                  (hx >= Q_TW + 2 ? 16 : 0) | (i >= Q_PIECES ? 16 : 0);
    }
    // epilogue table: lanes 0-31 the tile's noise (row lane / 4, 16-byte piece lane % 4 of the row's 64 B), lanes
    // 32-63 the sample's 32 demodulation scales (128 B; lanes 40-63 repeat 32-39)
    const int elane = lane < 32 ? (has_noise ? ((lane >> 2) * a.W * (int)sizeof(T) + (lane & 3) * 16) : 0)
                                : ((lane - 32) & 7) * 16;
    auto issue = [&](int t, int slot, int eslot) {
        int n, ty, tx;
        tile_of(t, n, ty, tx);
        const int tbase = ((n * a.H + ty - 1) * a.W + tx - 1) * 64;
        const int flags = (ty == 0 ? 1 : 0) | (ty + Q_TH == a.H ? 2 : 0) | (tx == 0 ? 4 : 0) | (tx + Q_TW == a.W ? 8 : 0) | 16;
        char* sb = smem_raw + slot * Q_SLOT;
#pragma unroll
        for (int u = 0; u < Q_DMA; ++u) {
            const int i = u * 4 + wave;               // wave-uniform
            if (i < Q_PIECES) {
                const int off = (hcls[u] & flags) ? -1 : tbase + hoff[u];
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rxb, (lds_ptr_t)(sb + i * 1024), 16, off, 0, 0, 0);
            } else if (i == Q_PIECES || u == Q_DMA - 1) {   // (the last round: every wave past the halo loads the
                // table -- duplicates write the same bytes -- so each wave issues Q_DMA instructions a tile)
                const char* nb = has_noise ? epi_src0 + (int64_t)((n * a.H + ty) * a.W + tx) * (int)sizeof(T) : epi_src0;
                const char* db = has_d ? epi_src1 + n * 128 : epi_src1;
                const char* src = (lane < 32 ? nb : db) + elane;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                                 (lds_ptr_t)(epil + eslot * Q_EPI), 16, 0, 0);
            }
        }
    };

    // B fragment i at tap (ky, kx): position (2 wave + (i >> 1) + ky) * 40 + (i & 1) * 16 + l16 + kx, piece q
    int boff[3];
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
        const int x = l16 + kx;
        boff[kx] = (2 * wave * Q_PITCH + x) * 64 + ((q ^ ((x >> 1) & 2)) << 4);
    }
    const float lr_alpha = (EPI && a.act == 1) ? a.alpha : 1.f;
    const float clampv = (EPI && a.clamp >= 0.f) ? a.clamp : __builtin_inff();
    const float ngain = a.noise_gain * a.gain;
    const int ch0 = 8 * q;                            // this lane's 8 output channels

    auto epi_table = [&](int eslot, float (&bb)[8], float (&dd)[8], float (&nz)[NF]) {
        if (!EPI) return;
        const unsigned et = lds_addr(epil + eslot * Q_EPI);
        float4 b0, b1, d0, d1;
        asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\t"
                     "ds_read_b128 %2, %5 offset:512\n\tds_read_b128 %3, %5 offset:528\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(b0), "=&v"(b1), "=&v"(d0), "=&v"(d1)
                     : "v"(lds_addr(blds + ch0)), "v"(et + ch0 * 4));
        const float bq[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        const float dq[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            bb[e] = bq[e];
            dd[e] = has_d ? dq[e] * a.gain : a.gain;
        }
        // pixel (2 wave + (i >> 1)) * 32 + (i & 1) * 16 + l16: byte 32 i from na
        const unsigned na = et + (2 * wave * Q_TW + l16) * (unsigned)sizeof(T);
        unsigned r0, r1, r2, r3;
        asm volatile("ds_read_u16 %0, %4\n\tds_read_u16 %1, %4 offset:32\n\tds_read_u16 %2, %4 offset:64\n\t"
                     "ds_read_u16 %3, %4 offset:96\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3) : "v"(na));
        const unsigned rr[4] = {r0, r1, r2, r3};
#pragma unroll
        for (int j = 0; j < 4; ++j) nz[j] = has_noise ? (float)__builtin_bit_cast(T, (unsigned short)rr[j]) * ngain : 0.f;
    };
    auto epi_store = [&](f32x4 (&A)[NF][2], int n, int ty, int tx, const float (&bb)[8], const float (&dd)[8],
                         const float (&nz)[NF]) {
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int r = 2 * wave + (i >> 1), px = (i & 1) * 16 + l16;
            const int pix = (n * a.H + ty + r) * a.W + tx + px;
            vec8 yv, rv;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float cv = A[i][e >> 2][e & 3];
                if (RAW) rv[e] = (T)cv;
                float v = cv;
                if (EPI) {
                    v = fmaf(v, dd[e], nz[i] + bb[e]);
                    v = fmaxf(v, v * lr_alpha);
                    v = __builtin_amdgcn_fmed3f(v, -clampv, clampv);
                }
                yv[e] = (T)v;
            }
            const int dst = (pix * 32 + ch0) * (int)sizeof(T);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, yv), ryb, dst, 0, 0);
            if (RAW) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, rv), ryr, dst, 0, 0);
        }
    };
    auto mfma_tile = [&](f32x4 (&A)[NF][2], const char* hb) {
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                v8<T> pf[NF];
#pragma unroll
                for (int i = 0; i < NF; ++i)
                    pf[i] = *(const v8<T>*)(hb + boff[kx] + (((i >> 1) + ky) * Q_PITCH + (i & 1) * 16) * 64);
                const bool first = ky == 0 && kx == 0;
#pragma unroll
                for (int i = 0; i < NF; ++i)
#pragma unroll
                    for (int jj = 0; jj < 2; ++jj)
                        A[i][jj] = mma<T>(wf[jj][ky * 3 + kx], pf[i], first ? f32x4{0.f, 0.f, 0.f, 0.f} : A[i][jj]);
            }
    };

    issue(t_begin, 0, 0);
    wait_vm<0>();
    __builtin_amdgcn_s_waitcnt(0xc07f);               // lgkmcnt(0): the bias table
    __builtin_amdgcn_s_barrier();
    f32x4 acc[NF][2];
    int k = 0;
    for (int t = t_begin; t < t_end; ++t, ++k) {
        const int slot = k & 1;
        issue(min(t + 1, t_end - 1), slot ^ 1, (k + 1) % Q_NEPI);
        int n, ty, tx;
        tile_of(t, n, ty, tx);
        if (SI && n != cur_n) {                       // a new sample: re-modulate the weights
            cur_n = n;
            load_weights(n);
        }
        mfma_tile(acc, smem_raw + slot * Q_SLOT);
        float bb[8], dd[8], nz[NF];
        epi_table(k % Q_NEPI, bb, dd, nz);
        epi_store(acc, n, ty, tx, bb, dd, nz);
        wait_vm<S>();                                 // tile t + 1's DMAs landed (younger: this tile's stores)
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_s_barrier();
    }
    wait_vm<0>();                                     // no LDS-DMA may outlive the workgroup
}

template <typename T, bool SI, bool EPI, bool RAW>
int launch_c32r(const Conv3Args& a, hipStream_t s, int tiles, int grid, int band) {
    auto kern = conv3x3_c32r_kernel<T, SI, EPI, RAW>;
    static bool attr_set = false;   // benign race: idempotent attribute
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)Q_LDS);
        attr_set = true;
    }
    kern<<<grid, 256, Q_LDS, s>>>(a, tiles, band);
    return launch_status("sg2_conv3x3 (c32 ring)");
}

template <typename T, bool SI, bool EPI>
int launch_c32r_raw(const Conv3Args& a, hipStream_t s) {
    const int tiles = a.N * (a.H / Q_TH) * (a.W / Q_TW);
    const int ty = a.H / Q_TH;
    const int band = ty % 4 == 0 ? 4 : (ty % 2 == 0 ? 2 : 1);
    const int grid = 2 * num_cus();
    return a.y_raw ? launch_c32r<T, SI, EPI, true>(a, s, tiles, grid, band)
                   : launch_c32r<T, SI, EPI, false>(a, s, tiles, grid, band);
}

// ---------------------------------------------------------------------------------------------------
// Stride-2 / pad-0 3x3 conv of the wide discriminator down layers (conv2d_resample's down-2 plan after its FIR,
// :94-109: the D blocks' conv1 at 128^2 .. 32^2 outputs, Cin 64 .. 256 -> Cout = 2 Cin), round 5.  The 32 x 4 halo
// form above restages a tile's 9 x 64 x 32 weights per 128 output pixels and ran these shapes at 0.10-0.18 of the
// MFMA peak, the generic implicit GEMM (register-staged gathers) at 0.12-0.24 (profiles/r02_s2_ab.log).  Here an
// implicit GEMM whose operands arrive by LDS-DMA, nothing staged through registers:
//   * workgroup tile: 256 output pixels (linear over n, oy, ox) x 128 output channels; 4 waves of 128 x 64
//     (8 pixel fragments x 4 channel fragments: 32 MFMAs and 12 ds_read_b128 per wave and K step);
//   * K = 9 taps x Cin in 32-channel steps, tap-minor (consecutive steps read neighbouring input pixels); per step
//     the workgroup stages the 256 pixels' tap inputs (64 B each) and 128 weight rows into one of G_NS = 3 LDS slots
//     by 24 wave-instructions of 1 KiB (6 per wave, issued two steps ahead, one barrier per step); the 16-byte
//     pieces are swizzled on the source side (swz64), so fragment reads of 16 consecutive rows are conflict-free;
//     the weight rows are loaded in p_chan order, so a lane's accumulators hold 8 consecutive output channels of
//     one pixel (16-byte stores straight from registers);
//   * XCD-aware order: workgroup i runs on XCD i % 8 and takes tile (i % 8) * (grid / 8) + i / 8, so neighbouring
//     tiles -- which share input rows -- meet in one L2.
// Epilogue in registers: demod scale, bias (rounded to T), lrelu, gain, clamp (the halo kernel's order), then the
// residual add (the D resnet's skip: round(round(v) + residual)) with y_raw = the raw conv output or (raw_act) the
// activated value before the add.
constexpr int G_BM = 256, G_BN = 128, G_NS = 3;
constexpr int G_SLOT = (G_BM + G_BN) * 64;                  // 24 KiB
constexpr int G_DMA = (G_BM + G_BN) / 16 / 4;               // wave-instructions per wave and step (6)
constexpr int G_ADMA = G_BM / 16 / 4;                       // of which pixel rows (4)
constexpr size_t G_LDS = (size_t)G_NS * G_SLOT;

template <typename T, bool EPI>
__global__ __launch_bounds__(256, 2) void conv3x3_s2g_kernel(Conv3Args a, int m_tiles, int n_tiles) {
    typedef T vec8 __attribute__((ext_vector_type(8)));
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l16 = lane & 15, q = lane >> 4;
    const int t = (int)(blockIdx.x % 8) * (int)(gridDim.x / 8) + (int)(blockIdx.x / 8);
    if (t >= m_tiles * n_tiles) return;
    const int mt = t / n_tiles, nt = t - mt * n_tiles;
    const int OHW = a.OH * a.OW, M = a.N * OHW;
    const int m0 = mt * G_BM, n0 = nt * G_BN;
    const int nk = 9 * (a.Cin / 32);
    const __amdgpu_buffer_rsrc_t rxb = make_rsrc(a.x, (int64_t)a.N * a.H * a.W * a.Cin * 2);
    const __amdgpu_buffer_rsrc_t rwb = make_rsrc(a.w, (int64_t)a.Cout * 9 * a.Cin * 2);

    // DMA lanes: instruction u of wave w fills slot rows (4 u + w) * 16 + lane / 4, piece lane % 4 (u < G_ADMA:
    // pixel rows, else weight rows); the lane reads source piece (lane % 4) ^ ((row >> 1) & 2)
    int dbase[G_DMA];
#pragma unroll
    for (int u = 0; u < G_DMA; ++u) {
        const int r = (u * 4 + wave) * 16 + (lane >> 2);
        const int j = (lane & 3) ^ ((r >> 1) & 2);
        if (u < G_ADMA) {
            const int m = m0 + r;
            if (m < M) {
                const int n = m / OHW, rem = m - n * OHW, oy = rem / a.OW, ox = rem - oy * a.OW;
                dbase[u] = (((n * a.H + 2 * oy) * a.W + 2 * ox) * a.Cin + j * 8) * 2;
            } else {
                dbase[u] = -1;
            }
        } else {
            dbase[u] = ((n0 + p_chan(r - G_BM)) * 9 * a.Cin + j * 8) * 2;
        }
    }
    auto issue = [&](int step, int slot) {
        const int tap = step % 9, c = step / 9;
        const int ky = tap / 3, kx = tap - ky * 3;
        const int aoff = ((ky * a.W + kx) * a.Cin + c * 32) * 2, boff = (tap * a.Cin + c * 32) * 2;
        char* sb = smem_raw + slot * G_SLOT;
#pragma unroll
        for (int u = 0; u < G_DMA; ++u) {
            if (u < G_ADMA) {
                const int off = dbase[u] < 0 ? -1 : dbase[u] + aoff;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rxb, (lds_ptr_t)(sb + (u * 4 + wave) * 1024), 16, off, 0, 0, 0);
            } else {
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rwb, (lds_ptr_t)(sb + (u * 4 + wave) * 1024), 16, dbase[u] + boff,
                                                         0, 0, 0);
            }
        }
    };

    const int wm = wave >> 1, wn = wave & 1;
    const int sw = ((q ^ ((l16 >> 1) & 2)) << 4) + l16 * 64;    // a fragment row's lane offset (row base % 16 == 0)
    f32x4 acc[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int st = 0; st < G_NS - 1; ++st)
        if (st < nk) issue(st, st);
    for (int step = 0; step < nk; ++step) {
        if (step + G_NS - 2 < nk) wait_vm<(G_NS - 2) * G_DMA>();
        else wait_vm<0>();
        __builtin_amdgcn_s_waitcnt(0xc07f);           // lgkmcnt(0)
        __builtin_amdgcn_s_barrier();                 // every wave's DMAs of this step landed; the oldest slot is free
        if (step + G_NS - 1 < nk) issue(step + G_NS - 1, (step + G_NS - 1) % G_NS);
        const char* sb = smem_raw + (step % G_NS) * G_SLOT + sw;
        v8<T> wf[4], pf[8];
#pragma unroll
        for (int jc = 0; jc < 4; ++jc) wf[jc] = *(const v8<T>*)(sb + (G_BM + wn * 64 + jc * 16) * 64);
#pragma unroll
        for (int jp = 0; jp < 8; ++jp) pf[jp] = *(const v8<T>*)(sb + (wm * 128 + jp * 16) * 64);
#pragma unroll
        for (int jp = 0; jp < 8; ++jp)
#pragma unroll
            for (int jc = 0; jc < 4; ++jc) acc[jc][jp] = mma<T>(wf[jc], pf[jp], acc[jc][jp]);
    }

    // ---- epilogue: lane (l16, q) holds, per pixel fragment jp and channel pair h, channels
    // n0 + (2 wn + h) * 32 + 8 q .. + 7 of pixel m0 + wm * 128 + 16 jp + l16 ----
    float bsc[2][8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int ch0 = n0 + (2 * wn + h) * 32 + 8 * q;
#pragma unroll
        for (int e = 0; e < 8; ++e) bsc[h][e] = (EPI && a.bias) ? (float)(T)a.bias[ch0 + e] : 0.f;
    }
    const float alpha = (EPI && a.act == 1) ? a.alpha : 1.f;
    const float clampv = (EPI && a.clamp >= 0.f) ? a.clamp : __builtin_inff();
    T* y = (T*)a.y;
    T* yr = (T*)a.y_raw;
    const T* res = (const T*)a.residual;
#pragma unroll
    for (int jp = 0; jp < 8; ++jp) {
        const int m = m0 + wm * 128 + jp * 16 + l16;
        if (m >= M) continue;
        const int n = m / OHW;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int ch0 = n0 + (2 * wn + h) * 32 + 8 * q;
            const int64_t dst = (int64_t)m * a.Cout + ch0;
            vec8 yv, rv;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                float v = acc[2 * h + (e >> 2)][jp][e & 3];
                rv[e] = (T)v;
                if (EPI) {
                    const float d = a.out_scale ? a.out_scale[(int64_t)n * a.Cout + ch0 + e] : 1.f;
                    v = v * d + bsc[h][e];
                    v = v > 0.f ? v : v * alpha;
                    v *= a.gain;
                    v = fminf(fmaxf(v, -clampv), clampv);
                }
                yv[e] = (T)v;
            }
            if (res) {
                if (yr && a.raw_act) *(vec8*)(yr + dst) = yv;
                const vec8 rr = *(const vec8*)(res + dst);
#pragma unroll
                for (int e = 0; e < 8; ++e) yv[e] = (T)((float)yv[e] + (float)rr[e]);
            }
            *(vec8*)(y + dst) = yv;
            if (yr && !(res && a.raw_act)) *(vec8*)(yr + dst) = rv;
        }
    }
}

template <typename T, bool EPI>
int launch_s2g(const Conv3Args& a, hipStream_t s) {
    const int M = a.N * a.OH * a.OW;
    const int m_tiles = (M + G_BM - 1) / G_BM, n_tiles = a.Cout / G_BN;
    const int grid = (m_tiles * n_tiles + 7) / 8 * 8;
    auto kern = conv3x3_s2g_kernel<T, EPI>;
    static bool attr_set = false;   // benign race: idempotent attribute
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G_LDS);
        attr_set = true;
    }
    kern<<<grid, 256, G_LDS, s>>>(a, m_tiles, n_tiles);
    return launch_status("sg2_conv3x3_s2 (s2g)");
}

template <typename T>
int dispatch(Conv3Args& a, hipStream_t s, int stride) {
    const bool si = a.in_scale != nullptr;
    const bool epi = a.out_scale || a.noise || a.bias || a.act != 0 || a.gain != 1.f || a.clamp >= 0.f;
    if (a.dot_out) {
        hipError_t e = zero_acc(a.dot_out, (size_t)a.N * a.Cout * sizeof(float), s);
        if (e != hipSuccess) { set_error("sg2_conv3x3: memset failed"); return (int)e; }
    }
    if (stride == 2) {
        // the wide down layers: the LDS-DMA implicit GEMM (SG2_S2G=0: off)
        const char* eg = getenv("SG2_S2G");          // read per launch: tests switch it in one process
        if ((!eg || atoi(eg) != 0) && !si && !a.noise && !a.dot_out && a.Cin % 32 == 0 && a.Cout % G_BN == 0 &&
            a.OW >= 32 && (int64_t)a.N * a.OH * a.OW * a.Cout * 2 < 0x7fff0000ll &&
            ((uintptr_t)a.y % 16) == 0 && ((uintptr_t)a.y_raw % 16) == 0 && ((uintptr_t)a.residual % 16) == 0 &&
            (!epi || a.gain > 0.f)) {
            if (epi) return launch_s2g<T, true>(a, s);
            return launch_s2g<T, false>(a, s);
        }
        // 32 x 4 output tiles, two workgroups per CU
        a.tiles_x = (a.OW + 31) / 32;
        a.tiles_y = (a.OH + 3) / 4;
        if (si) { if (epi) return launch3<T, 32, true, true, 1, 2>(a, s); return launch3<T, 32, true, false, 1, 2>(a, s); }
        if (epi) return launch3<T, 32, false, true, 1, 2>(a, s);
        return launch3<T, 32, false, false, 1, 2>(a, s);
    }
    static const bool persist = [] { const char* e = getenv("SG2_HALO_PERSIST"); return !e || atoi(e) != 0; }();
    {
        // the C = 32 ring (SG2_C32_RING=0: off)
        const char* e32 = getenv("SG2_C32_RING");     // read per launch: tests switch it in one process
        const bool ring32 = !e32 || atoi(e32) != 0;
        const int tiles = a.H % Q_TH == 0 && a.W % Q_TW == 0 ? a.N * (a.H / Q_TH) * (a.W / Q_TW) : 0;
        const int grid = 2 * num_cus();
        if (ring32 && !a.dot_out && a.Cin == 32 && a.Cout == 32 && tiles >= 2 * grid && tiles <= 128 * grid &&
            a.N < 4096 && a.H / Q_TH < 1024 && a.W / Q_TW < 1024 &&
            (int64_t)a.N * a.H * a.W * 32 * (int64_t)sizeof(T) < 0x7fff0000ll &&
            ((uintptr_t)a.y % 16) == 0 && ((uintptr_t)a.y_raw % 16) == 0 && ((uintptr_t)a.noise % 16) == 0 &&
            ((uintptr_t)a.out_scale % 16) == 0 && ((uintptr_t)a.in_scale % 16) == 0 && (a.W * (int)sizeof(T)) % 16 == 0 &&
            (!epi || (a.gain > 0.f && (a.act == 0 || (a.alpha >= 0.f && a.alpha <= 1.f))))) {
            if (si) { if (epi) return launch_c32r_raw<T, true, true>(a, s); return launch_c32r_raw<T, true, false>(a, s); }
            if (epi) return launch_c32r_raw<T, false, true>(a, s);
            return launch_c32r_raw<T, false, false>(a, s);
        }
    }
    // SG2_C64_RING: 0 off, else the ring form (launch_c64r_form: 49 default -- form 4 with the hoisted DMA issue
    // and the per-sample dynamic tail, 0.146-0.150 ms on the bench launch against 0.154-0.156 for 46 (hoisted issue
    // only) and 0.161 for 4, profiles/r05_ring_forms.txt --, 46, 4, 44, 8, 84)
    const char* ring_env = getenv("SG2_C64_RING");   // read per launch: tests switch forms in one process
    const int ring = ring_env ? atoi(ring_env) : 49;
    const int rth = (ring == 4 || ring == 44 || ring == 46 || ring == 49) ? 4 : 8;
    if (ring && !a.dot_out && a.Cin == P_C && a.Cout == P_C && a.H % rth == 0 && a.W % R_TW == 0 &&
        ((uintptr_t)a.y % 16) == 0 && ((uintptr_t)a.y_raw % 16) == 0 && ((uintptr_t)a.noise % 16) == 0 &&
        ((uintptr_t)a.out_scale % 16) == 0 && ((uintptr_t)a.in_scale % 16) == 0 &&
        (!epi || (a.gain > 0.f && (a.act == 0 || (a.alpha >= 0.f && a.alpha <= 1.f))))) {
        const int tiles = a.N * (a.H / rth) * (a.W / R_TW);
        const int grid = (rth == 4 ? 2 : 1) * num_cus();
        // (the fast DMA issue marks an invalid halo row with base INT_MIN: the image must stay below 2^31 - 2^16 B)
        if (tiles >= 2 * grid && tiles <= 128 * grid && a.N < 4096 && a.H / rth < 1024 && a.W / R_TW < 1024 &&
            (int64_t)a.N * a.H * a.W * 64 * (int64_t)sizeof(T) < 0x7fff0000ll) {
            const int form = (ring == 84 || ring == 44 || ring == 46 || ring == 49) ? ring : rth;
            if (si) { if (epi) return launch_c64r_form<T, true, true>(a, s, form); return launch_c64r_form<T, true, false>(a, s, form); }
            if (epi) return launch_c64r_form<T, false, true>(a, s, form);
            return launch_c64r_form<T, false, false>(a, s, form);
        }
    }
    // (the persistent kernel's epilogue folds the gain into the demod / noise / bias terms and evaluates lrelu
    // as max(v, alpha v): it needs gain > 0 and 0 <= alpha <= 1, the StyleGAN2 settings)
    if (persist && a.Cin == P_C && a.Cout == P_C && a.H % P_TH == 0 && a.W % P_TW == 0 &&
        (!epi || (a.gain > 0.f && (a.act == 0 || (a.alpha >= 0.f && a.alpha <= 1.f))))) {
        const int tiles = a.N * (a.H / P_TH) * (a.W / P_TW);
        if (tiles >= 2 * num_cus()) {
            const int grid = num_cus();
            if (si) { if (epi) return launch_c64p_dot<T, true, true>(a, s, tiles, grid); return launch_c64p_dot<T, true, false>(a, s, tiles, grid); }
            if (epi) return launch_c64p_dot<T, false, true>(a, s, tiles, grid);
            return launch_c64p_dot<T, false, false>(a, s, tiles, grid);
        }
    }
    const int TW = a.W >= 32 ? 32 : 16;
    a.tiles_x = (a.W + TW - 1) / TW;
    a.tiles_y = (a.H + (256 / TW) - 1) / (256 / TW);
    static const int force_nbuf = [] { const char* e = getenv("SG2_HALO_NBUF"); return e ? atoi(e) : 0; }();
    // one LDS buffer per workgroup: two workgroups per CU (2 waves / SIMD) hide each other's staging and
    // load latency; measured 1.3-1.4x faster than a double-buffered single workgroup per CU at C >= 128
    // (gpurun_out/nbuf.log; SG2_HALO_NBUF=2 selects the double-buffered form)
    const int nbuf = force_nbuf ? force_nbuf : 1;
#define L3(TWV, SIV, EPIV) return nbuf == 1 ? launch3<T, TWV, SIV, EPIV, 1>(a, s) : launch3<T, TWV, SIV, EPIV, 2>(a, s)
    if (TW == 32) {
        if (si) { if (epi) L3(32, true, true); else L3(32, true, false); }
        else { if (epi) L3(32, false, true); else L3(32, false, false); }
    } else {
        if (si) { if (epi) L3(16, true, true); else L3(16, true, false); }
        else { if (epi) L3(16, false, true); else L3(16, false, false); }
    }
#undef L3
}

// ---------------------------------------------------------------------------------------------------
// Stride-2 transposed 3x3 convolution, padding 0 (conv2d_resample's up-2 plan, conv2d_resample.py:112-129:
// the G up layers' conv_transpose2d, and the input gradient of the D down layers' stride-2 conv):
//   y[n, 2i + ky, 2j + kx, o] += sum_c x[n, i, j, c] (* s[n, c]) W[o][ky][kx][c],   y: (2H+1) x (2W+1)
// The generic implicit GEMM runs this as four output phases, each a separate GEMM of 1, 2, 2 or 4 taps:
// the input is fetched once per phase and a phase's K is only taps x Cin, so its workgroups are bound by
// prologue and epilogue.  Here a workgroup owns a 16 x 8 tile of output CELLS (cell (i, j) = the 2 x 2
// output pixels 2i + py, 2j + px) x 64 output channels: per 32-channel chunk it stages the 17 x 9 input
// halo (cell (i, j) reads inputs (i - 1 .. i, j - 1 .. j)) and the chunk's 9 x 64 x 32 weights once, and
// every wave accumulates all nine taps into the four phase accumulators of its 2 x 16 cells:
//   per tap: 2 pixel and 4 weight fragments, 8 MFMAs into phase (ky & 1, kx & 1).
// LDS rows are the swizzled 64-byte rows of swz64.  The epilogue transposes each phase through LDS and
// stores whole 128-byte pixel lines (64 channels).  Two workgroups per CU, single-buffered LDS (the same
// staging discipline as conv3x3_halo_kernel NBUF = 1).
constexpr int U_TW = 16, U_TH = 8, U_CELLS = U_TW * U_TH;              // 128 cells
constexpr int U_HW = U_TW + 1, U_HH = U_TH + 1, U_HP = U_HW * U_HH;   // 17 x 9 = 153 input positions
constexpr int U_HB = ((U_HP * 64 + 255) / 256) * 256;                  // halo bytes (256-aligned: swz64)
constexpr int U_WB = 9 * BN * 64;                                      // weight bytes per chunk
constexpr int U_OS = BN + 8;                                           // epilogue tile row (elements)
constexpr size_t U_LDS = (size_t)U_HB + U_WB;                          // 46,848 B
static_assert((size_t)U_CELLS * U_OS * 2 <= U_LDS, "epilogue tile fits the staging buffer");

// Edge split (EDGE > 0): with H % 8 == W % 16 == 0 the 16 x 8 tiles cover cells 0 .. H-1 x 0 .. W-1 exactly and
// the last cell row (i = H: output row 2H only, from input row H-1 through the ky = 2 taps) and column (j = W:
// output column 2W, the kx = 2 taps) run as 128 x 1 (EDGE 1) and 1 x 128 (EDGE 2) strips of three taps each.  At
// 32^2 inputs the ragged 16 x 8 tiling of 33 x 33 cells ran 15 tiles of nine taps per image; split it is 8 + 2/3.
template <int EDGE> struct UpGeom {
    static constexpr int TW = EDGE == 0 ? U_TW : (EDGE == 1 ? 128 : 1);       // cells per tile row
    static constexpr int HR = EDGE == 1 ? 1 : (EDGE == 0 ? U_TH : 128) + 1;    // staged halo rows
    static constexpr int HC = EDGE == 2 ? 1 : TW + 1;                          // staged halo columns
    static constexpr int HP = HR * HC;
    static constexpr int NT = EDGE == 0 ? 9 : 3;                               // taps
    __device__ static constexpr int tap(int t) { return EDGE == 0 ? t : (EDGE == 1 ? 6 + t : 2 + 3 * t); }
};
static_assert(((UpGeom<1>::HP * 64 + 255) / 256) * 256 + 3 * BN * 64 <= U_LDS &&
              ((UpGeom<2>::HP * 64 + 255) / 256) * 256 + 3 * BN * 64 <= U_LDS, "edge strips fit the staging buffer");

template <typename T, bool SCALE_IN, int EDGE>
__device__ __forceinline__ void up2_tile(const Conv3Args& a, int n, int i0, int j0, char* smem_raw) {
    using G = UpGeom<EDGE>;
    constexpr int NH = (G::HP * 4 + 255) / 256;               // halo 16-B loads per thread
    constexpr int NW = (G::NT * BN * 4) / 256;                // weight 16-B loads per thread
    constexpr int HB = ((G::HP * 64 + 255) / 256) * 256;
    typedef T vec8 __attribute__((ext_vector_type(8)));
    char* hl = smem_raw;                                      // [HP rows] x 64 B
    char* wl = smem_raw + HB;                                 // [NT taps][64 rows] x 64 B

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int o0 = blockIdx.y * BN;
    const int OH = 2 * a.H + 1, OW = 2 * a.W + 1;
    const int nchunks = a.Cin / CK;
    const __amdgpu_buffer_rsrc_t rxb = make_rsrc(a.x, (int64_t)a.N * a.H * a.W * a.Cin * (int64_t)sizeof(T));
    const __amdgpu_buffer_rsrc_t rwb = make_rsrc(a.w, (int64_t)a.Cout * 9 * a.Cin * (int64_t)sizeof(T));
    const int hq = (tid & 3) * 8;

    vec8 rh[NH], rw[NW];
    float4 sc0, sc1;
    auto gload = [&](int chunk) {
        const int c = chunk * CK + hq;
#pragma unroll
        for (int k = 0; k < NH; ++k) {
            const int p = (tid + k * 256) >> 2;
            const int iy = i0 - 1 + p / G::HC, ix = j0 - 1 + p % G::HC;
            const bool ok = (p < G::HP) & ((unsigned)iy < (unsigned)a.H) & ((unsigned)ix < (unsigned)a.W);
            rh[k] = buf_load16<vec8>(rxb, ok ? (((n * a.H + iy) * a.W + ix) * a.Cin + c) * (int)sizeof(T) : -1);
        }
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            const int r = (tid + k * 256) >> 2, t = r / BN, o = r - t * BN;
            rw[k] = buf_load16<vec8>(rwb, o0 + o < a.Cout ? (((o0 + o) * 9 + G::tap(t)) * a.Cin + c) * (int)sizeof(T)
                                                          : -1);
        }
        if (SCALE_IN) {
            const float* sc = a.in_scale + (int64_t)n * a.Cin + c;
            sc0 = *(const float4*)sc;
            sc1 = *(const float4*)(sc + 4);
        }
    };
    auto sstore = [&]() {
        const float scl[8] = {sc0.x, sc0.y, sc0.z, sc0.w, sc1.x, sc1.y, sc1.z, sc1.w};
#pragma unroll
        for (int k = 0; k < NH; ++k) {
            const int p = (tid + k * 256) >> 2;
            if (k * 256 + 256 > G::HP * 4 && p >= G::HP) continue;   // the ragged last round only
            vec8 v = rh[k];
            if (SCALE_IN) {   // x * s.to(x.dtype) (networks_stylegan2.py:69): s rounded first, one rounding after
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = (T)((float)v[e] * (float)(T)scl[e]);
            }
            *(vec8*)(hl + swz64(p, tid & 3)) = v;
        }
#pragma unroll
        for (int k = 0; k < NW; ++k) *(vec8*)(wl + swz64((tid + k * 256) >> 2, tid & 3)) = rw[k];
    };

    const int lq = lane >> 4, l16 = lane & 15;
    const int b_lane = swz64(l16, lq);                        // + (tap * 64 + j * 16) * 64: the same swizzle
    f32x4 acc[4][2][4];                                       // [phase (ky & 1) * 2 + (kx & 1)][cell group][co tile]
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[f][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    gload(0);
    sstore();
    __syncthreads();
    for (int ch = 0; ch < nchunks; ++ch) {
        const bool more = ch + 1 < nchunks;
        if (more) gload(ch + 1);
#pragma unroll
        for (int t = 0; t < G::NT; ++t) {
            const int tap = G::tap(t), ky = tap / 3, kx = tap % 3, ph = (ky & 1) * 2 + (kx & 1);
            v8<T> af[2], bfr[4];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                // cell m = 16 (2 wave + i) + l16 of the tile reads halo row (cell row + 1 - ky / 2), column
                // (cell column + 1 - kx / 2); the edge strips stage only the row / column their taps read
                const int m = (2 * wave + i) * 16 + l16, cy = m / G::TW, cx = m % G::TW;
                const int hy = EDGE == 1 ? 0 : cy + 1 - (ky >> 1), hx = EDGE == 2 ? 0 : cx + 1 - (kx >> 1);
                af[i] = *(const v8<T>*)(hl + swz64(hy * G::HC + hx, lq));
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) bfr[j] = *(const v8<T>*)(wl + b_lane + (t * BN + j * 16) * 64);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[ph][i][j] = mma<T>(af[i], bfr[j], acc[ph][i][j]);
        }
        if (more) {
            __syncthreads();                                  // everyone done reading before the overwrite
            sstore();
        }
        __syncthreads();
    }

    // ---- epilogue: per phase, the 128 x 64 tile through LDS, whole 128-byte pixel lines out ----
    T* ot = (T*)smem_raw;                                     // [128 cells][U_OS]
    T* y = (T*)a.y;
    const int c8 = (tid & 7) * 8;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
        const int py = ph >> 1, px = ph & 1;
        if ((EDGE == 1 && py) || (EDGE == 2 && px)) continue;  // output row 2H + 1 / column 2W + 1: none
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = (2 * wave + i) * 16 + 4 * lq + r;       // cell of accumulator row 4 lq + r
#pragma unroll
                for (int j = 0; j < 4; ++j) ot[m * U_OS + j * 16 + l16] = (T)acc[ph][i][j][r];
            }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 4; ++k) {                         // 128 cells x 8 channel vectors / 256 threads
            const int m = (tid >> 3) + k * 32;
            const int oy = 2 * (i0 + m / G::TW) + py, ox = 2 * (j0 + m % G::TW) + px;
            // (the column strip leaves the corner cell (H, W) to the row strip)
            if (oy < (EDGE == 2 ? 2 * a.H : OH) && ox < OW && o0 + c8 < a.Cout)
                *(vec8*)(y + (((int64_t)n * OH + oy) * OW + ox) * a.Cout + o0 + c8) = *(const vec8*)(ot + m * U_OS + c8);
        }
        __syncthreads();
    }
}

template <typename T, bool SCALE_IN>
__global__ __launch_bounds__(256, 2) void conv3x3_up2_kernel(Conv3Args a) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const int per_n = a.tiles_x * a.tiles_y;
    int b = blockIdx.x;
    if (b < a.N * per_n) {
        const int n = b / per_n, tr = b - n * per_n;
        up2_tile<T, SCALE_IN, 0>(a, n, (tr / a.tiles_x) * U_TH, (tr % a.tiles_x) * U_TW, smem_raw);
        return;
    }
    b -= a.N * per_n;
    if (b < a.N * a.edge_rx) {                                // cells (H, 128 t ..)
        const int n = b / a.edge_rx;
        up2_tile<T, SCALE_IN, 1>(a, n, a.H, (b - n * a.edge_rx) * 128, smem_raw);
        return;
    }
    b -= a.N * a.edge_rx;
    const int n = b / a.edge_cy;                              // cells (128 t .., W)
    up2_tile<T, SCALE_IN, 2>(a, n, (b - n * a.edge_cy) * 128, a.W, smem_raw);
}

template <typename T, bool SI>
int launch_up2(Conv3Args& a, hipStream_t s) {
    auto kern = conv3x3_up2_kernel<T, SI>;
    static bool attr_set = false;   // benign race: idempotent attribute
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)U_LDS);
        attr_set = true;
    }
    const char* e = getenv("SG2_UP2_EDGE");          // read per launch: tests switch it in one process
    const bool split = !(e && e[0] == '0') && a.H % U_TH == 0 && a.W % U_TW == 0;
    a.tiles_x = split ? a.W / U_TW : (a.W + 1 + U_TW - 1) / U_TW;
    a.tiles_y = split ? a.H / U_TH : (a.H + 1 + U_TH - 1) / U_TH;
    a.edge_rx = split ? (a.W + 1 + 127) / 128 : 0;
    a.edge_cy = split ? (a.H + 127) / 128 : 0;
    dim3 grid(a.N * (a.tiles_x * a.tiles_y + a.edge_rx + a.edge_cy), (a.Cout + BN - 1) / BN);
    kern<<<grid, 256, U_LDS, s>>>(a);
    return launch_status("sg2_conv3x3_up2");
}

}  // namespace
}  // namespace sg2

namespace sg2 {
namespace {
int conv3x3_entry(void* y, void* y_raw, const void* x, const void* w, int dtype, int N, int Cin, int H, int W,
                  int Cout, const float* in_scale, const float* out_scale, const void* noise, float noise_gain,
                  const float* bias, int act, float alpha, float gain, float clamp, const void* dot_src,
                  float* dot_out, void* stream, int stride, const void* residual = nullptr, int raw_act = 0);
}
}

extern "C" int sg2_conv3x3(void* y, void* y_raw, const void* x, const void* w, int dtype, int N, int Cin, int H, int W,
                           int Cout, const float* in_scale, const float* out_scale, const void* noise, float noise_gain,
                           const float* bias, int act, float alpha, float gain, float clamp, const void* dot_src,
                           float* dot_out, void* stream) {
    return sg2::conv3x3_entry(y, y_raw, x, w, dtype, N, Cin, H, W, Cout, in_scale, out_scale, noise, noise_gain, bias,
                              act, alpha, gain, clamp, dot_src, dot_out, stream, 1);
}

extern "C" int sg2_conv3x3_s2(void* y, void* y_raw, const void* x, const void* w, int dtype, int N, int Cin, int H,
                              int W, int Cout, const float* in_scale, const float* out_scale, const void* noise,
                              float noise_gain, const float* bias, int act, float alpha, float gain, float clamp,
                              const void* residual, int raw_act, const void* dot_src, float* dot_out, void* stream) {
    using namespace sg2;
    SG2_CHECK(H >= 3 && W >= 3, "sg2_conv3x3_s2: input smaller than the kernel");
    SG2_CHECK(residual == nullptr || ((uintptr_t)residual % 16) == 0, "sg2_conv3x3_s2: 16-byte alignment required");
    return sg2::conv3x3_entry(y, y_raw, x, w, dtype, N, Cin, H, W, Cout, in_scale, out_scale, noise, noise_gain, bias,
                              act, alpha, gain, clamp, dot_src, dot_out, stream, 2, residual, raw_act);
}

namespace sg2 {
namespace {
int conv3x3_entry(void* y, void* y_raw, const void* x, const void* w, int dtype, int N, int Cin, int H, int W,
                  int Cout, const float* in_scale, const float* out_scale, const void* noise, float noise_gain,
                  const float* bias, int act, float alpha, float gain, float clamp, const void* dot_src,
                  float* dot_out, void* stream, int stride, const void* residual, int raw_act) {
    SG2_CHECK(y && x && w, "sg2_conv3x3: null pointer");
    SG2_CHECK(N > 0 && Cin > 0 && H > 0 && W > 0 && Cout > 0, "sg2_conv3x3: empty shape");
    SG2_CHECK(dtype == SG2_F16 || dtype == SG2_BF16, "sg2_conv3x3: f16/bf16 only");
    SG2_CHECK(Cin % 8 == 0, "sg2_conv3x3: Cin must be a multiple of 8");
    SG2_CHECK(((uintptr_t)x % 16) == 0 && ((uintptr_t)w % 16) == 0, "sg2_conv3x3: 16-byte alignment required");
    SG2_CHECK(act == 0 || act == 1, "sg2_conv3x3: act must be 0 (linear) or 1 (lrelu)");
    SG2_CHECK((dot_src == nullptr) == (dot_out == nullptr), "sg2_conv3x3: dot_src and dot_out go together");
    SG2_CHECK((int64_t)N * H * W * Cin * 2 < INT32_MAX && (int64_t)Cout * 9 * Cin * 2 < INT32_MAX,
              "sg2_conv3x3: tensor too large (32-bit byte offsets of the buffer loads)");
    Conv3Args a{};
    a.x = x; a.w = w; a.y = y; a.y_raw = y_raw; a.in_scale = in_scale; a.out_scale = out_scale; a.noise = noise;
    a.bias = bias; a.dot_src = dot_src; a.dot_out = dot_out; a.noise_gain = noise_gain; a.alpha = alpha; a.gain = gain; a.clamp = clamp; a.act = act;
    a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout;
    a.residual = residual; a.raw_act = raw_act;
    a.OH = stride == 1 ? H : (H - 3) / 2 + 1;
    a.OW = stride == 1 ? W : (W - 3) / 2 + 1;
    hipStream_t s = as_stream(stream);
    // deterministic mode: the kernels that take a dot (halo, persistent C = 64) write their partial sums to slots
    // and sum them per sample in a fixed order (launch3_k, launch_c64p)
    return dtype == SG2_F16 ? dispatch<f16_t>(a, s, stride) : dispatch<bf16_t>(a, s, stride);
}
}  // namespace
}  // namespace sg2

extern "C" int sg2_conv3x3_up2(void* y, const void* x, const void* w, int dtype, int N, int Cin, int H, int W, int Cout,
                               const float* in_scale, void* stream) {
    using namespace sg2;
    SG2_CHECK(y && x && w, "sg2_conv3x3_up2: null pointer");
    SG2_CHECK(N > 0 && Cin > 0 && H > 0 && W > 0 && Cout > 0, "sg2_conv3x3_up2: empty shape");
    SG2_CHECK(dtype == SG2_F16 || dtype == SG2_BF16, "sg2_conv3x3_up2: f16/bf16 only");
    SG2_CHECK(Cin % CK == 0 && Cout % 8 == 0, "sg2_conv3x3_up2: Cin must be a multiple of 32, Cout of 8");
    SG2_CHECK(((uintptr_t)x % 16) == 0 && ((uintptr_t)w % 16) == 0 && ((uintptr_t)y % 16) == 0,
              "sg2_conv3x3_up2: 16-byte alignment required");
    SG2_CHECK((int64_t)N * H * W * Cin * 2 < INT32_MAX && (int64_t)Cout * 9 * Cin * 2 < INT32_MAX,
              "sg2_conv3x3_up2: tensor too large (32-bit byte offsets of the buffer loads)");
    Conv3Args a{};
    a.x = x; a.w = w; a.y = y; a.in_scale = in_scale;
    a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout;
    hipStream_t s = as_stream(stream);
    if (dtype == SG2_F16) return in_scale ? launch_up2<f16_t, true>(a, s) : launch_up2<f16_t, false>(a, s);
    return in_scale ? launch_up2<bf16_t, true>(a, s) : launch_up2<bf16_t, false>(a, s);
}

#if SG2_RDIAG & 512
extern "C" int sg2_diag_ring_stamps(void* dst, long long bytes) {
    const size_t n = sizeof(sg2::g_ring_stamps) < (size_t)bytes ? sizeof(sg2::g_ring_stamps) : (size_t)bytes;
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(sg2::g_ring_stamps), n, 0, hipMemcpyDeviceToHost);
}
#endif

