// Small kernels of the training step: demodulation coefficients and their gradient, conv weight packs,
// fp16 range pre-normalisation, and the optimiser step (multi-tensor Adam with the gradient sanitation
// fused in front, the G_ema lerp).  All HBM- or latency-bound.
#include "sg2_common.h"

#include <algorithm>

namespace sg2 {
namespace {

// Demodulation with the per-(o, i) weight energy kept for the backward: wsq[o,i] = sum_k w^2 (written when
// wsq_out != null), d[n,o] = rsqrt(sum_i s[n,i]^2 wsq[o,i] + eps).  One workgroup per o; after wsq is in
// LDS, eight lanes per sample reduce a row of s each (32 samples per pass, no block barrier per sample).
__global__ __launch_bounds__(256) void demod_fwd_kernel(float* d, float* wsq_out, const float* s, const float* w,
                                                        int N, int O, int I, int KK, float eps) {
    __shared__ float wsq[1024];
    const int o = blockIdx.x;
    for (int i = threadIdx.x; i < I; i += 256) {
        const float* wr = w + ((int64_t)o * I + i) * KK;
        float acc = 0.f;
        for (int k = 0; k < KK; ++k) acc += wr[k] * wr[k];
        wsq[i] = acc;
        if (wsq_out) wsq_out[(int64_t)o * I + i] = acc;
    }
    __syncthreads();
    // 8 lanes per sample, 32 samples per pass: a lane sums a contiguous 1/8 of the row of s (all its loads
    // independent), then three xor shuffles combine the eighths
    const int seg = threadIdx.x & 7, len = (I + 7) / 8, i0 = seg * len, i1 = min(I, i0 + len);
    for (int n0 = 0; n0 < N; n0 += 32) {
        const int n = n0 + (threadIdx.x >> 3);
        float acc = 0.f;
        if (n < N) {
            const float* sr = s + (int64_t)n * I;
#pragma unroll 8
            for (int i = i0; i < i1; ++i) {
                const float v = sr[i];
                acc += v * v * wsq[i];
            }
        }
        acc += __shfl_xor(acc, 1);
        acc += __shfl_xor(acc, 2);
        acc += __shfl_xor(acc, 4);
        if (seg == 0 && n < N) d[(int64_t)n * O + o] = rsqrtf(acc + eps);
    }
}

// Backward of demod_fwd: with gu[n,o] = -1/2 dd[n,o] d[n,o]^3,
//   gw[o,i,k] = 2 w[o,i,k] sum_n gu[n,o] s[n,i]^2     (workgroup per o)
//   gs[n,i]   = 2 s[n,i]   sum_o gu[n,o] wsq[o,i]      (workgroup per (n, 64 i); four o-quarters reduced in LDS)
__global__ __launch_bounds__(256) void demod_bwd_w_kernel(float* gw, const float* dd, const float* d, const float* s,
                                                          const float* w, int N, int O, int I, int KK) {
    __shared__ float gu[1024];
    const int o = blockIdx.x;
    for (int n = threadIdx.x; n < N; n += 256) {
        const float dv = d[(int64_t)n * O + o];
        gu[n] = -0.5f * dd[(int64_t)n * O + o] * dv * dv * dv;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < I; i += 256) {
        float acc = 0.f;
        for (int n = 0; n < N; ++n) {
            const float v = s[(int64_t)n * I + i];
            acc += gu[n] * v * v;
        }
        const float* wr = w + ((int64_t)o * I + i) * KK;
        float* gr = gw + ((int64_t)o * I + i) * KK;
        for (int k = 0; k < KK; ++k) gr[k] = 2.f * wr[k] * acc;
    }
}

__global__ __launch_bounds__(256) void demod_bwd_s_kernel(float* gs, const float* dd, const float* d, const float* s,
                                                          const float* wsq, int N, int O, int I) {
    __shared__ float gu[1024];
    __shared__ float part[4][64];
    const int n = blockIdx.x, i = blockIdx.y * 64 + (threadIdx.x & 63), q = threadIdx.x >> 6;
    for (int o = threadIdx.x; o < O; o += 256) {
        const float dv = d[(int64_t)n * O + o];
        gu[o] = -0.5f * dd[(int64_t)n * O + o] * dv * dv * dv;
    }
    __syncthreads();
    float acc = 0.f;
    if (i < I) {
        // 16 independent loads in flight per lane (L2-latency bound otherwise)
        float a4[4] = {0.f, 0.f, 0.f, 0.f};
        int o = q;
        for (; o + 60 < O; o += 64) {
#pragma unroll
            for (int u = 0; u < 16; ++u) a4[u & 3] += gu[o + 4 * u] * wsq[(int64_t)(o + 4 * u) * I + i];
        }
        for (; o < O; o += 4) a4[0] += gu[o] * wsq[(int64_t)o * I + i];
        acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
    }
    part[q][threadIdx.x & 63] = acc;
    __syncthreads();
    if (q == 0 && i < I)
        gs[(int64_t)n * I + i] = 2.f * s[(int64_t)n * I + i] * (part[0][threadIdx.x] + part[1][threadIdx.x] +
                                                                 part[2][threadIdx.x] + part[3][threadIdx.x]);
}

// Multi-tensor kernels of the optimiser step.  A launch walks a block table: entry = (segment << 40) | start,
// one workgroup per SEG_CHUNK elements of one segment (a parameter tensor), so a whole module's ~100
// tensors of very different sizes are one launch with no idle lanes beyond each tensor's last chunk.
constexpr int SEG_CHUNK = 4096;     // 256 lanes x 16 elements

// torch.optim.Adam (foreach arithmetic, no weight decay, amsgrad off) on every parameter of one exchanged
// gradient, with the reference's sanitation in front (training_loop_mi_multimodal.py:345-347):
//   g = nan_to_num(grad * gscale, nan=0, posinf=1e5, neginf=-1e5)
//   m = lerp(m, g, 1 - b1); v = v * b2 + (1 - b2) * g * g
//   p += -step_size * (m / (sqrt(v) / bc2_sqrt + eps))
// seg[s] = {param address, offset of the segment in grad/m/v, numel}; coef[s] = {step_size, bc2_sqrt}.
// write_grad: store the sanitised g back (the caller's .grad views then hold the exchanged gradient).
__global__ __launch_bounds__(256) void adam_multi_kernel(const int64_t* __restrict__ seg, const float* __restrict__ coef,
                                                         const int64_t* __restrict__ blocks, float* __restrict__ grad,
                                                         float* __restrict__ m, float* __restrict__ v, float b1, float b2,
                                                         float eps, float gscale, int write_grad) {
    const int64_t e = blocks[blockIdx.x];
    const int s = (int)(e >> 40);
    const int64_t start = e & ((1LL << 40) - 1);
    float* __restrict__ p = reinterpret_cast<float*>(seg[3 * s]);
    const int64_t off = seg[3 * s + 1], n = seg[3 * s + 2];
    const float step_size = coef[2 * s], bc2_sqrt = coef[2 * s + 1];
    const float w = 1.f - b1;
    const int64_t end = start + SEG_CHUNK < n ? start + SEG_CHUNK : n;
    for (int64_t i = start + threadIdx.x; i < end; i += 256) {
        float g = grad[off + i] * gscale;
        if (g != g) g = 0.f;
        else if (isinf(g)) g = g > 0.f ? 1e5f : -1e5f;
        if (write_grad) grad[off + i] = g;
        float mi = m[off + i];
        mi = w < 0.5f ? mi + w * (g - mi) : g - (g - mi) * (1.f - w);      // torch lerp
        float vi = v[off + i] * b2;
        vi = vi + (1.f - b2) * g * g;                                      // addcmul
        m[off + i] = mi;
        v[off + i] = vi;
        const float denom = sqrtf(vi) / bc2_sqrt + eps;
        p[i] = p[i] + (-step_size) * (mi / denom);                         // addcdiv
    }
}

// G_ema update (training_loop_mi_multimodal.py:363-364): dst = src.lerp(dst, beta), torch's lerp formula.
// seg[s] = {dst address, src address, numel}.
__global__ __launch_bounds__(256) void lerp_multi_kernel(const int64_t* __restrict__ seg,
                                                         const int64_t* __restrict__ blocks, float beta) {
    const int64_t e = blocks[blockIdx.x];
    const int s = (int)(e >> 40);
    const int64_t start = e & ((1LL << 40) - 1);
    float* __restrict__ dst = reinterpret_cast<float*>(seg[3 * s]);
    const float* __restrict__ src = reinterpret_cast<const float*>(seg[3 * s + 1]);
    const int64_t n = seg[3 * s + 2];
    const int64_t end = start + SEG_CHUNK < n ? start + SEG_CHUNK : n;
    for (int64_t i = start + threadIdx.x; i < end; i += 256) {
        const float a = src[i], b = dst[i];
        dst[i] = beta < 0.5f ? a + beta * (b - a) : b - (b - a) * (1.f - beta);
    }
}


// Conv weight pack: out[a][k][b] = in[a*sa + b*sb + k'*sk] (k' = K-1-k when flip), cast to Tout.  One lane
// per output element: the stores are coalesced runs of b, the gathered loads of a wavefront touch the same
// cache lines as its neighbours' (the other taps of the same rows), so the input is read from HBM once.
// Every lane issues its single load at once -- no serial per-lane loop, which left small packs
// latency-bound.  Replaces the strided-permute copy of _pack_conv / _pack_convT.
template <typename Tin, typename Tout>
__global__ __launch_bounds__(256) void pack_weight_kernel(Tout* __restrict__ out, const Tin* __restrict__ in, int A,
                                                          int B, int K, int64_t sa, int64_t sb, int64_t sk, int flip,
                                                          float scale) {
    const unsigned e = blockIdx.x * 256u + threadIdx.x;      // 32-bit index math (A*B*K < 2^31, host-checked)
    if (e >= (unsigned)A * B * K) return;
    const unsigned r = e / (unsigned)B, b = e - r * B;
    const unsigned a = r / (unsigned)K, k = r - a * K;
    const int kk = flip ? K - 1 - (int)k : (int)k;
    // (weight * gain).to(dtype): one f32 product, one rounding -- as the reference's `self.weight * self.weight_gain`
    // (the empty asm keeps the f32 product: fmul + fptrunc would otherwise become one v_fma_mix with a
    // single rounding, not torch's f32 product then cast)
    float v = to_f32(in[(int64_t)a * sa + (int64_t)b * sb + kk * sk]) * scale;
    asm volatile("" : "+v"(v));
    out[e] = from_f32<Tout>(v);
}

// Every conv-weight pack of a training phase in one launch per 64 packs (sg2_pack_weight_multi): workgroup b
// serves elements [(b - blk0[d]) 1024, + 1024) of descriptor d with blk0[d] <= b < blk0[d + 1], and does for each what
// pack_weight_kernel does for that descriptor -- the same element map, product and rounding, so each pack is
// bitwise the single-launch pack.  The phase's packs (~40 per phase, 158 launches per step) were each a
// few-microsecond launch.
__device__ __forceinline__ float ld_any(const void* p, int64_t i, int dt) {
    return dt == SG2_F32 ? ((const float*)p)[i] : dt == SG2_F16 ? (float)((const f16_t*)p)[i] : (float)((const bf16_t*)p)[i];
}
__device__ __forceinline__ void st_any(void* p, unsigned i, int dt, float v) {
    if (dt == SG2_F32) ((float*)p)[i] = v;
    else if (dt == SG2_F16) ((f16_t*)p)[i] = (f16_t)v;
    else ((bf16_t*)p)[i] = (bf16_t)v;
}
// The table travels in the kernel arguments (scalar loads through the constant cache): a workgroup finds its
// descriptor by a binary search over block0 there, with no dependent global loads before its element loads.
// Row mode (B * K <= PACK_ROW_MAX, every conv of the networks): one workgroup per output row a -- the row's
// B x K inputs read in input order (a conv weight's [Cin][kh][kw] slab is contiguous: whole-line loads), the
// scaled f32 values staged in LDS, then out[a][k][b] written in output order (whole-line stores).  The element
// mode (1024 elements per workgroup, 4 per lane) gathered 9-apart elements per wave load and ran at ~0.5 TB/s
// (222 us per phase table, profiles/r05 step breakdown).
constexpr int PACK_PER_LAUNCH = 64, PACK_EPT = 4, PACK_ROW_MAX = 8192;
struct PackDescK {
    void* out;
    const void* in;
    int sa, sb, sk, A, B, K, block0;
    float scale;
    unsigned char out_dt, in_dt, flip, rows;
};
struct PackTable {
    PackDescK d[PACK_PER_LAUNCH];
    int n;
};
__global__ __launch_bounds__(256) void pack_weight_multi_kernel(const PackTable t) {
    const int b = blockIdx.x;
    int lo = 0, hi = t.n - 1;                      // last d with block0 <= b (wave-uniform: scalar loads)
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (t.d[mid].block0 <= b) lo = mid; else hi = mid - 1;
    }
    const PackDescK& d = t.d[lo];
    if (d.rows) {
        __shared__ float row[PACK_ROW_MAX];
        const int a = b - d.block0, L = d.B * d.K;
        const int64_t base = (int64_t)a * d.sa;
        for (int i = threadIdx.x; i < L; i += 256) {
            const int bb = i / d.K, k = i - bb * d.K;
            float x = ld_any(d.in, base + (int64_t)bb * d.sb + (int64_t)k * d.sk, d.in_dt) * d.scale;
            asm volatile("" : "+v"(x));          // (as pack_weight_kernel: the f32 product, then one rounding)
            row[i] = x;
        }
        __syncthreads();
        const unsigned ob = (unsigned)a * (unsigned)L;
        for (int e = threadIdx.x; e < L; e += 256) {
            const int k = e / d.B, bb = e - k * d.B;
            const int kk = d.flip ? d.K - 1 - k : k;
            st_any(d.out, ob + e, d.out_dt, row[bb * d.K + kk]);
        }
        return;
    }
    const unsigned total = (unsigned)d.A * d.B * d.K;
    const unsigned e0 = (unsigned)(b - d.block0) * (256u * PACK_EPT) + threadIdx.x;
    float v[PACK_EPT];
#pragma unroll
    for (int j = 0; j < PACK_EPT; ++j) {
        const unsigned e = e0 + j * 256u;
        const unsigned ec = e < total ? e : total - 1;     // (a clamped index: loads stay in bounds, no branch)
        const unsigned r = ec / (unsigned)d.B, bb = ec - r * d.B;
        const unsigned a = r / (unsigned)d.K, k = r - a * d.K;
        const int kk = d.flip ? d.K - 1 - (int)k : (int)k;
        v[j] = ld_any(d.in, (int64_t)a * d.sa + (int64_t)bb * d.sb + (int64_t)kk * d.sk, d.in_dt) * d.scale;
    }
#pragma unroll
    for (int j = 0; j < PACK_EPT; ++j) {
        const unsigned e = e0 + j * 256u;
        float x = v[j];
        asm volatile("" : "+v"(x));              // (as pack_weight_kernel: the f32 product, then one rounding)
        if (e < total) st_any(d.out, e, d.out_dt, x);
    }
}

// Row-wise infinity-norm pre-normalisation of the fp16 modulated layers (networks_stylegan2.py:52-54):
// n = max_i |t[r,i]|; mode 0: y = t * ((1/n) * c) (the weight: torch's scalar / tensor is a reciprocal and a
// scale), mode 1: y = t / n (the styles).  One workgroup per row, the row reread from L2 for the store.
// max that propagates NaN (torch's amax / norm(inf) does; fmaxf would drop it)
__device__ __forceinline__ float nanmax(float a, float b) { return (a != a || b != b) ? __builtin_nanf("") : fmaxf(a, b); }

__device__ __forceinline__ float block_reduce(float v, float* red, bool is_max) {
    for (int off = 32; off > 0; off >>= 1) {
        const float o = __shfl_xor(v, off);
        v = is_max ? nanmax(v, o) : v + o;
    }
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return is_max ? nanmax(nanmax(red[0], red[1]), nanmax(red[2], red[3])) : (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void infnorm_fwd_kernel(float* __restrict__ y, float* __restrict__ nrm,
                                                          const float* __restrict__ t, int L, float c, int mode) {
    __shared__ float red[4];
    const float* tr = t + (int64_t)blockIdx.x * L;
    float m = 0.f;
    for (int i = threadIdx.x; i < L; i += 256) m = nanmax(m, fabsf(tr[i]));
    m = block_reduce(m, red, true);
    if (threadIdx.x == 0) nrm[blockIdx.x] = m;
    float* yr = y + (int64_t)blockIdx.x * L;
    const float k = (1.0f / m) * c;
    for (int i = threadIdx.x; i < L; i += 256) yr[i] = mode == 0 ? tr[i] * k : tr[i] / m;
}

// First-order gradient: dt = dy * k + [|t| == n] sgn(t) g_n / cnt, g_n = -(k / n) sum_i dy t, with k = c / n
// (mode 0) or 1 / n (mode 1; the direct term as dy / n); cnt = the number of maxima (torch's
// infinity-norm backward splits the gradient evenly between ties).
__global__ __launch_bounds__(256) void infnorm_bwd_kernel(float* __restrict__ dt, const float* __restrict__ dy,
                                                          const float* __restrict__ t, const float* __restrict__ nrm,
                                                          int L, float c, int mode) {
    __shared__ float red[4];
    const int64_t base = (int64_t)blockIdx.x * L;
    const float n = nrm[blockIdx.x];
    float s1 = 0.f, cnt = 0.f;
    for (int i = threadIdx.x; i < L; i += 256) {
        const float tv = t[base + i];
        s1 += dy[base + i] * tv;
        cnt += (fabsf(tv) == n || tv != tv) ? 1.f : 0.f;
    }
    s1 = block_reduce(s1, red, false);
    cnt = block_reduce(cnt, red, false);
    const float k = mode == 0 ? (1.0f / n) * c : 1.0f / n;
    const float gm = -(k / n) * s1 / cnt;
    for (int i = threadIdx.x; i < L; i += 256) {
        const float tv = t[base + i], g = dy[base + i];
        float d = mode == 0 ? g * k : g / n;
        if (fabsf(tv) == n || tv != tv) d += (tv > 0.f ? gm : (tv < 0.f ? -gm : (tv != tv ? tv : 0.f)));
        dt[base + i] = d;
    }
}

// Second order of the path-length pass (networks_stylegan2._DemodVJP / _InfNormVJP): the backward of the
// first-order gradients above, each from its closed form, so that a differentiated gradient costs one or two
// launches instead of the ~25 torch elementwise / reduction launches of its composed form.
//
// demod: with sg = s * g and v[n,o] = sum_i sg[n,i] wsq[o,i] (workgroup per o; wsq row in LDS, 8 lanes/sample)
//   g_dd = -d^3 v,   g_d = -3 dd d^2 v,   g_w[o,i,k] = -2 w[o,i,k] sum_n dd d^3 sg[n,i]
// (the styles' part, g_s = 2 g (u @ wsq) with u = -dd d^3 / 2, is demod_bwd_s_kernel with s := g).
__global__ __launch_bounds__(256) void demod_vjp_o_kernel(float* g_dd, float* g_d, float* g_w, const float* g,
                                                          const float* dd, const float* d, const float* s,
                                                          const float* w, const float* wsq, int N, int O, int I,
                                                          int KK) {
    __shared__ float wr[1024];
    __shared__ float z[1024];
    const int o = blockIdx.x;
    for (int i = threadIdx.x; i < I; i += 256) wr[i] = wsq[(int64_t)o * I + i];
    for (int n = threadIdx.x; n < N; n += 256) {
        const float dv = d[(int64_t)n * O + o];
        z[n] = dd[(int64_t)n * O + o] * dv * dv * dv;
    }
    __syncthreads();
    if (g_dd || g_d) {
        const int seg = threadIdx.x & 7, len = (I + 7) / 8, i0 = seg * len, i1 = min(I, i0 + len);
        for (int n0 = 0; n0 < N; n0 += 32) {
            const int n = n0 + (threadIdx.x >> 3);
            float acc = 0.f;
            if (n < N) {
                const float* sr = s + (int64_t)n * I;
                const float* gr = g + (int64_t)n * I;
#pragma unroll 8
                for (int i = i0; i < i1; ++i) acc += sr[i] * gr[i] * wr[i];
            }
            acc += __shfl_xor(acc, 1);
            acc += __shfl_xor(acc, 2);
            acc += __shfl_xor(acc, 4);
            if (seg == 0 && n < N) {
                const int64_t e = (int64_t)n * O + o;
                const float dv = d[e];
                if (g_dd) g_dd[e] = -(dv * dv * dv) * acc;
                if (g_d) g_d[e] = -3.f * dd[e] * dv * dv * acc;
            }
        }
    }
    if (g_w) {
        for (int i = threadIdx.x; i < I; i += 256) {
            float acc = 0.f;
            for (int n = 0; n < N; ++n) acc += z[n] * s[(int64_t)n * I + i] * g[(int64_t)n * I + i];
            const float* wk = w + ((int64_t)o * I + i) * KK;
            float* gk = g_w + ((int64_t)o * I + i) * KK;
            for (int k = 0; k < KK; ++k) gk[k] = -2.f * wk[k] * acc;
        }
    }
}

// infnorm: with e = sgn(t) [|t| = n] / cnt, ge = sum g e, gdy = sum g dy, P = sum dy t (workgroup per row),
//   g_dy = c (g - t ge / n) / n,   g_t = e (2 c P ge / n^3 - c gdy / n^2) - dy c ge / n^2
// (c = the mode-0 scale, 1 for the styles).
__global__ __launch_bounds__(256) void infnorm_vjp_kernel(float* __restrict__ g_dy, float* __restrict__ g_t,
                                                          const float* __restrict__ g, const float* __restrict__ dy,
                                                          const float* __restrict__ t, const float* __restrict__ nrm,
                                                          int L, float c) {
    __shared__ float red[4];
    const int64_t base = (int64_t)blockIdx.x * L;
    const float n = nrm[blockIdx.x];
    float cnt = 0.f, ge = 0.f, gdy = 0.f, P = 0.f;
    for (int i = threadIdx.x; i < L; i += 256) {
        const float tv = t[base + i], gv = g[base + i], dv = dy[base + i];
        if (fabsf(tv) == n || tv != tv) {
            cnt += 1.f;
            ge += tv > 0.f ? gv : (tv < 0.f ? -gv : (tv != tv ? tv : 0.f));
        }
        gdy += gv * dv;
        P += dv * tv;
    }
    cnt = block_reduce(cnt, red, false);
    ge = block_reduce(ge, red, false) / cnt;
    gdy = block_reduce(gdy, red, false);
    P = block_reduce(P, red, false);
    const float n2 = n * n;
    const float a = 2.f * c * P * ge / (n2 * n) - c * gdy / n2, b = c * ge / n2;
    for (int i = threadIdx.x; i < L; i += 256) {
        const float tv = t[base + i], gv = g[base + i], dv = dy[base + i];
        if (g_dy) g_dy[base + i] = c * (gv - tv * (ge / n)) / n;
        if (g_t) {
            float e = 0.f;
            if (fabsf(tv) == n || tv != tv) e = (tv > 0.f ? 1.f : (tv < 0.f ? -1.f : (tv != tv ? tv : 0.f))) / cnt;
            g_t[base + i] = e * a - dv * b;
        }
    }
}

}  // namespace

__global__ void zero_fill_kernel(unsigned char* p, size_t bytes) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t head = (16 - ((uintptr_t)p & 15)) & 15;
    if (head > bytes) head = bytes;
    for (size_t k = i; k < head; k += stride) p[k] = 0;
    const size_t nv = (bytes - head) / 16;
    uint4* v = reinterpret_cast<uint4*>(p + head);
    for (size_t k = i; k < nv; k += stride) v[k] = make_uint4(0u, 0u, 0u, 0u);
    for (size_t k = head + nv * 16 + i; k < bytes; k += stride) p[k] = 0;
}

hipError_t zero_fill(void* p, size_t bytes, hipStream_t s) {
    if (bytes == 0) return hipSuccess;
    const int g = (int)std::min<int64_t>(cdiv((int64_t)(bytes / 16 + 1), 256), 2048);
    zero_fill_kernel<<<g, 256, 0, s>>>(static_cast<unsigned char*>(p), bytes);
    return hipGetLastError();
}
}  // namespace sg2

extern "C" int sg2_demod_fwd(float* d, float* wsq, const float* s, const float* w, int N, int O, int I, int KK,
                             float eps, void* stream) {
    using namespace sg2;
    SG2_CHECK(d && s && w, "sg2_demod_fwd: null pointer");
    SG2_CHECK(I <= 1024 && I > 0 && O > 0 && N > 0 && KK > 0, "sg2_demod_fwd: unsupported shape");
    demod_fwd_kernel<<<O, 256, 0, as_stream(stream)>>>(d, wsq, s, w, N, O, I, KK, eps);
    return launch_status("sg2_demod_fwd");
}

extern "C" int sg2_demod_bwd(float* gs, float* gw, const float* dd, const float* d, const float* s, const float* w,
                             const float* wsq, int N, int O, int I, int KK, void* stream) {
    using namespace sg2;
    SG2_CHECK(dd && d && s && w, "sg2_demod_bwd: null pointer");
    SG2_CHECK(!gs || wsq, "sg2_demod_bwd: gs needs wsq");
    SG2_CHECK(I <= 1024 && O <= 1024 && N <= 1024 && I > 0 && O > 0 && N > 0 && KK > 0,
              "sg2_demod_bwd: unsupported shape");
    hipStream_t st = as_stream(stream);
    if (gw) {
        demod_bwd_w_kernel<<<O, 256, 0, st>>>(gw, dd, d, s, w, N, O, I, KK);
        int rc = launch_status("sg2_demod_bwd");
        if (rc) return rc;
    }
    if (gs) {
        demod_bwd_s_kernel<<<dim3(N, (I + 63) / 64), 256, 0, st>>>(gs, dd, d, s, wsq, N, O, I);
        return launch_status("sg2_demod_bwd");
    }
    return 0;
}

extern "C" int sg2_demod_vjp_bwd(float* g_dd, float* g_d, float* g_w, float* g_s, const float* g, const float* dd,
                                 const float* d, const float* s, const float* w, const float* wsq, int N, int O, int I,
                                 int KK, void* stream) {
    using namespace sg2;
    SG2_CHECK(g && dd && d && s && w && wsq, "sg2_demod_vjp_bwd: null pointer");
    SG2_CHECK(I <= 1024 && O <= 1024 && N <= 1024 && I > 0 && O > 0 && N > 0 && KK > 0,
              "sg2_demod_vjp_bwd: unsupported shape");
    hipStream_t st = as_stream(stream);
    if (g_dd || g_d || g_w) {
        demod_vjp_o_kernel<<<O, 256, 0, st>>>(g_dd, g_d, g_w, g, dd, d, s, w, wsq, N, O, I, KK);
        int rc = launch_status("sg2_demod_vjp_bwd");
        if (rc) return rc;
    }
    if (g_s) {
        demod_bwd_s_kernel<<<dim3(N, (I + 63) / 64), 256, 0, st>>>(g_s, dd, d, g, wsq, N, O, I);
        return launch_status("sg2_demod_vjp_bwd");
    }
    return 0;
}

extern "C" int sg2_infnorm_vjp_bwd(float* g_dy, float* g_t, const float* g, const float* dy, const float* t,
                                   const float* nrm, int rows, int L, float c, void* stream) {
    using namespace sg2;
    SG2_CHECK(g && dy && t && nrm, "sg2_infnorm_vjp_bwd: null pointer");
    SG2_CHECK(rows >= 0 && L > 0, "sg2_infnorm_vjp_bwd: bad shape");
    if (rows == 0 || (!g_dy && !g_t)) return 0;
    infnorm_vjp_kernel<<<rows, 256, 0, as_stream(stream)>>>(g_dy, g_t, g, dy, t, nrm, L, c);
    return launch_status("sg2_infnorm_vjp_bwd");
}

extern "C" int sg2_adam_multi(const int64_t* seg, const float* coef, const int64_t* blocks, int nblocks,
                              float* grad, float* exp_avg, float* exp_avg_sq, float beta1, float beta2, float eps,
                              float grad_scale, int write_grad, void* stream) {
    using namespace sg2;
    SG2_CHECK(seg && coef && blocks && grad && exp_avg && exp_avg_sq, "sg2_adam_multi: null pointer");
    SG2_CHECK(nblocks >= 0, "sg2_adam_multi: nblocks < 0");
    if (nblocks == 0) return 0;
    adam_multi_kernel<<<nblocks, 256, 0, as_stream(stream)>>>(seg, coef, blocks, grad, exp_avg, exp_avg_sq, beta1,
                                                               beta2, eps, grad_scale, write_grad);
    return launch_status("sg2_adam_multi");
}

extern "C" int sg2_lerp_multi(const int64_t* seg, const int64_t* blocks, int nblocks, float beta, void* stream) {
    using namespace sg2;
    SG2_CHECK(seg && blocks, "sg2_lerp_multi: null pointer");
    SG2_CHECK(nblocks >= 0, "sg2_lerp_multi: nblocks < 0");
    if (nblocks == 0) return 0;
    lerp_multi_kernel<<<nblocks, 256, 0, as_stream(stream)>>>(seg, blocks, beta);
    return launch_status("sg2_lerp_multi");
}

extern "C" int sg2_pack_weight(void* out, int out_dtype, const void* in, int in_dtype, int A, int B, int K,
                               int64_t sa, int64_t sb, int64_t sk, int flip, float scale, void* stream) {
    using namespace sg2;
    SG2_CHECK(out && in, "sg2_pack_weight: null pointer");
    SG2_CHECK(A > 0 && B > 0 && K >= 1 && K <= 9 && (int64_t)A * B * K < (1LL << 31),
              "sg2_pack_weight: unsupported shape (K <= 9, A*B*K < 2^31)");
    hipStream_t s = as_stream(stream);
    if (B * K <= PACK_ROW_MAX && sa >= 0 && sb >= 0 && sk >= 0 && sa < (1LL << 31) && sb < (1LL << 31) && sk < (1LL << 31) &&
        (in_dtype == SG2_F32 || in_dtype == SG2_F16 || in_dtype == SG2_BF16) &&
        (out_dtype == SG2_F32 || out_dtype == SG2_F16 || out_dtype == SG2_BF16)) {   // the row-mode kernel
        PackTable t{};
        t.n = 1;
        t.d[0] = PackDescK{out, in, (int)sa, (int)sb, (int)sk, A, B, K, 0, scale, (unsigned char)out_dtype,
                           (unsigned char)in_dtype, (unsigned char)(flip != 0), 1};
        pack_weight_multi_kernel<<<A, 256, 0, s>>>(t);
        return launch_status("sg2_pack_weight");
    }
    const unsigned grid = (unsigned)cdiv((int64_t)A * B * K, 256);
    SG2_DISPATCH(in_dtype, Tin, SG2_DISPATCH(out_dtype, Tout,
        pack_weight_kernel<Tin, Tout><<<grid, 256, 0, s>>>((Tout*)out, (const Tin*)in, A, B, K, sa, sb, sk, flip, scale)));
    return launch_status("sg2_pack_weight");
}

extern "C" int sg2_pack_weight_multi(const sg2_pack_desc* descs, int n, void* stream) {
    using namespace sg2;
    SG2_CHECK(descs != nullptr && n > 0, "sg2_pack_weight_multi: empty table");
    hipStream_t s = as_stream(stream);
    for (int i0 = 0; i0 < n; i0 += PACK_PER_LAUNCH) {
        PackTable t{};
        t.n = std::min(PACK_PER_LAUNCH, n - i0);
        int blk = 0;
        for (int j = 0; j < t.n; ++j) {
            const sg2_pack_desc& d = descs[i0 + j];
            SG2_CHECK(d.out && d.in && d.A > 0 && d.B > 0 && d.K >= 1 && d.K <= 9 &&
                      (int64_t)d.A * d.B * d.K < (1LL << 31) && d.sa < (1LL << 31) && d.sb < (1LL << 31) &&
                      d.sk < (1LL << 31) && d.sa >= 0 && d.sb >= 0 && d.sk >= 0,
                      "sg2_pack_weight_multi: unsupported descriptor (K <= 9, A*B*K < 2^31, 32-bit strides)");
            SG2_CHECK((d.in_dtype == SG2_F32 || d.in_dtype == SG2_F16 || d.in_dtype == SG2_BF16) &&
                      (d.out_dtype == SG2_F32 || d.out_dtype == SG2_F16 || d.out_dtype == SG2_BF16),
                      "sg2_pack_weight_multi: unsupported dtype");
            const bool rows = d.B * d.K <= PACK_ROW_MAX;
            t.d[j] = PackDescK{d.out, d.in, (int)d.sa, (int)d.sb, (int)d.sk, d.A, d.B, d.K, blk, d.scale,
                               (unsigned char)d.out_dtype, (unsigned char)d.in_dtype, (unsigned char)(d.flip != 0),
                               (unsigned char)rows};
            blk += rows ? d.A : (int)cdiv((int64_t)d.A * d.B * d.K, 256 * PACK_EPT);
        }
        pack_weight_multi_kernel<<<blk, 256, 0, s>>>(t);
        const int rc = launch_status("sg2_pack_weight_multi");
        if (rc) return rc;
    }
    return 0;
}

extern "C" int sg2_infnorm_fwd(float* y, float* nrm, const float* t, int rows, int L, float c, int mode,
                               void* stream) {
    using namespace sg2;
    SG2_CHECK(y && nrm && t, "sg2_infnorm_fwd: null pointer");
    SG2_CHECK(rows > 0 && L > 0 && (mode == 0 || mode == 1), "sg2_infnorm_fwd: bad arguments");
    infnorm_fwd_kernel<<<rows, 256, 0, as_stream(stream)>>>(y, nrm, t, L, c, mode);
    return launch_status("sg2_infnorm_fwd");
}

extern "C" int sg2_infnorm_bwd(float* dt, const float* dy, const float* t, const float* nrm, int rows, int L, float c,
                               int mode, void* stream) {
    using namespace sg2;
    SG2_CHECK(dt && dy && t && nrm, "sg2_infnorm_bwd: null pointer");
    SG2_CHECK(rows > 0 && L > 0 && (mode == 0 || mode == 1), "sg2_infnorm_bwd: bad arguments");
    infnorm_bwd_kernel<<<rows, 256, 0, as_stream(stream)>>>(dt, dy, t, nrm, L, c, mode);
    return launch_status("sg2_infnorm_bwd");
}

// ------------------------------------------------------------------------------------ statistic moments
// training_stats.report (SG3/torch_utils/training_stats.py:55-99: count, sum and sum of squares of a reported
// value, added into its float64 row) in one launch instead of ~7 (flatten / square / two sums / stack / cast /
// two adds).  One workgroup: strided double partials, then a fixed-order tree -- deterministic.  mode 1: the
// moments of sign(v) (the ADA heuristic's Loss/signs/*, without the separate sign launch).
namespace sg2 {
namespace {
__global__ __launch_bounds__(256) void moments_kernel(double* row, const float* v, int64_t n, int mode) {
    __shared__ double s1[256], s2[256];
    const int tid = threadIdx.x;
    double a = 0.0, b = 0.0;
    for (int64_t i = tid; i < n; i += 256) {
        float x = v[i];
        if (mode == 1) x = x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f);   // torch.sign: (0 < x) - (x < 0): 0 and NaN -> 0
        const double d = (double)x;
        a += d;
        b += d * d;
    }
    s1[tid] = a;
    s2[tid] = b;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (tid < s) {
            s1[tid] += s1[tid + s];
            s2[tid] += s2[tid + s];
        }
        __syncthreads();
    }
    if (tid == 0) {
        row[0] += (double)n;
        row[1] += s1[0];
        row[2] += s2[0];
    }
}
}  // namespace
}  // namespace sg2

extern "C" int sg2_moments(double* row, const float* v, int64_t n, int mode, void* stream) {
    using namespace sg2;
    SG2_CHECK(row && v, "sg2_moments: null pointer");
    SG2_CHECK(n > 0 && (mode == 0 || mode == 1), "sg2_moments: n > 0, mode 0 or 1");
    moments_kernel<<<1, 256, 0, as_stream(stream)>>>(row, v, n, mode);
    return launch_status("sg2_moments");
}
