// Fused first-order backward of a StyleGAN2 layer epilogue, one HBM pass.
//
// Forward (networks_stylegan2.py:309-328 / :172-181):  z = c * d[n,o] + noise[n,p] + b[o]
//                                                      y = clamp(lrelu(z) * gain, +-clamp)
// Given dy this kernel produces, reading dy, y (and c) once:
//   dz          = dy * gain * (y > 0 ? 1 : alpha) * [|y| < clamp]   (bias_act.cu grad=1 semantics)
//   dc[n,p,o]   = dz * d[n,o]          (written; the input of the dgrad / wgrad convolutions)
//   db[o]      += sum_{n,p} dz          (float atomics, one per channel per workgroup)
//   dd[n,o]    += sum_p dz * c          (demodulation-coefficient gradient)
//   dnoise[n,p] = sum_o dz              (noise-strength gradient; written, each pixel owned by one WG)
// Replaces: bias_act grad kernel + db reduction + noise reduction + (dz*c).sum + dz*d of the
// composed reference path (five to seven passes over the activation).
// NHWC layout: a lane owns 8 consecutive channels of one pixel (16-byte loads, 32 for f32); C % 8 == 0.
#include "sg2_common.h"

namespace sg2 {
namespace {

struct LBArgs {
    const void* dy;
    const void* y;
    const void* c;       // optional
    const float* d;      // optional [N, C]
    void* dc;            // output [N,HW,C]
    float* db;           // optional [C] accum
    float* dd;           // optional [N, C] accum
    float* dnoise;       // optional [N, HW] written
    int N, HW, C;
    int pix_per_block;
    float alpha, gain, clamp;
    int act;             // 0 linear, 1 lrelu
    float* det_db;       // deterministic mode: [gridDim.y * gridDim.x][C] slot partials of db
    float* det_dd;       // deterministic mode: [gridDim.x][N * C] slot partials of dd
};

template <typename T>
__global__ __launch_bounds__(256) void layer_bwd_kernel(LBArgs a) {
    typedef T vec8 __attribute__((ext_vector_type(8)));
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int LP = a.C / 8;                       // lanes per pixel
    const int PPP = 256 / LP;                     // pixels per pass (threads beyond LP*PPP idle)
    float* s_db = sm;                             // [C]
    float* s_dd = sm + a.C;                       // [C]
    float* s_dn = sm + 2 * a.C;                   // [pix_per_block]
    float* part = sm + 2 * a.C + a.pix_per_block; // deterministic mode: [PPP][C] per-thread partials
    const bool det = a.det_db || a.det_dd;
    const int tid = threadIdx.x;
    const int n = blockIdx.y;
    const int p0 = blockIdx.x * a.pix_per_block;
    const int p1 = min(a.HW, p0 + a.pix_per_block);
    for (int i = tid; i < 2 * a.C + a.pix_per_block; i += 256) sm[i] = 0.f;
    __syncthreads();

    const int cg = tid % LP, pl = tid / LP;
    const bool active = pl < PPP;
    const int c0 = cg * 8;
    float dv[8], adb[8], add[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        dv[j] = (a.d && active) ? a.d[(int64_t)n * a.C + c0 + j] : 1.f;
        adb[j] = 0.f;
        add[j] = 0.f;
    }
    T* dcp = (T*)a.dc;
    // U pixels per lane per iteration, all loads issued first (raw buffer loads: a pixel past the block
    // reads zeros); the noise gradient sums the LP lanes of a pixel with xor shuffles when LP is a power
    // of two <= 64 (C <= 512), else through LDS atomics.
    constexpr int U = 4;
    constexpr int V = 16 / sizeof(T) < 8 ? 16 / sizeof(T) : 8;   // elements per 16-byte load
    constexpr int NL = 8 / V;                                     // 16-byte loads per 8 channels
    typedef T vecv __attribute__((ext_vector_type(V)));
    const int64_t bytes = (int64_t)a.N * a.HW * a.C * (int64_t)sizeof(T);
    const __amdgpu_buffer_rsrc_t rdy = make_rsrc(a.dy, bytes), ry = make_rsrc(a.y, bytes),
                                 rc = make_rsrc(a.c ? a.c : a.dy, bytes);
    const bool has_c = a.c != nullptr;
    const bool shfl = (LP & (LP - 1)) == 0 && LP <= 64;
    if (active) {
        for (int pb = p0 + pl; pb < p1; pb += PPP * U) {
            vecv g[U][NL], yv[U][NL], cv[U][NL];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int p = pb + u * PPP;
                const int boff = p < p1 ? (int)((((int64_t)n * a.HW + p) * a.C + c0) * (int64_t)sizeof(T)) : -1;
#pragma unroll
                for (int l = 0; l < NL; ++l) {
                    const int o = boff < 0 ? -1 : boff + 16 * l;
                    g[u][l] = buf_load16<vecv>(rdy, o);
                    yv[u][l] = buf_load16<vecv>(ry, o);
                    if (has_c) cv[u][l] = buf_load16<vecv>(rc, o);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int p = pb + u * PPP;
                float psum = 0.f;
                vecv o[NL];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int l = j / V, e = j % V;
                    const float yy = (float)yv[u][l][e];
                    float dz = (float)g[u][l][e] * a.gain;
                    if (a.act == 1 && !(yy > 0.f)) dz *= a.alpha;
                    if (a.clamp >= 0.f && !(yy > -a.clamp && yy < a.clamp)) dz = 0.f;
                    adb[j] += dz;
                    psum += dz;
                    if (has_c) add[j] += dz * (float)cv[u][l][e];
                    o[l][e] = (T)(dz * dv[j]);
                }
                if (p < p1) {
#pragma unroll
                    for (int l = 0; l < NL; ++l)
                        *(vecv*)(dcp + ((int64_t)n * a.HW + p) * a.C + c0 + l * V) = o[l];
                }
                if (a.dnoise) {
                    if (shfl) {
                        for (int m = 1; m < LP; m <<= 1) psum += __shfl_xor(psum, m);
                        if (cg == 0 && p < p1) a.dnoise[(int64_t)n * a.HW + p] = psum;
                    } else if (p < p1) {
                        atomicAdd(&s_dn[p - p0], psum);
                    }
                }
            }
        }
    }
    if (det) {
        // fixed order: thread partials by row, rows in order, then one slot per workgroup (det_sum)
        const int slot = blockIdx.y * gridDim.x + blockIdx.x;
        if (a.db) {
            if (active) det_rows_store(part, a.C, pl, c0, adb);
            __syncthreads();
            for (int i = tid; i < a.C; i += 256) a.det_db[(int64_t)slot * a.C + i] = det_rows_sum(part, a.C, PPP, i);
            __syncthreads();
        }
        if (a.dd) {
            if (active) det_rows_store(part, a.C, pl, c0, add);
            __syncthreads();
            for (int i = tid; i < a.C; i += 256)
                a.det_dd[((int64_t)blockIdx.x * a.N + n) * a.C + i] = det_rows_sum(part, a.C, PPP, i);
        }
        __syncthreads();
    } else {
        if (a.db || a.dd) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (!active) break;
                if (a.db) atomicAdd(&s_db[c0 + j], adb[j]);
                if (a.dd) atomicAdd(&s_dd[c0 + j], add[j]);
            }
        }
        __syncthreads();
        for (int i = tid; i < a.C; i += 256) {
            if (a.db) atomicAdd(&a.db[i], s_db[i]);
            if (a.dd) atomicAdd(&a.dd[(int64_t)n * a.C + i], s_dd[i]);
        }
    }
    if (a.dnoise && !shfl)
        for (int p = p0 + tid; p < p1; p += 256) a.dnoise[(int64_t)n * a.HW + p] = s_dn[p - p0];
}

// out[n, c] = sum_p a[n, p, c] * b[n, p, c] over the pixels of NHWC tensors, f32 accumulation: the
// modulation / demodulation gradients of the path-length pass (sum_p dz*c, sum_p dxs*x), which autograd
// would run as a full-size multiply plus a reduction.  Same lane layout as layer_bwd_kernel.
template <typename T>
__global__ __launch_bounds__(256) void dot_hw_kernel(float* out, const T* a, const T* b, int HW, int C,
                                                     int pix_per_block, float* det_ws) {
    typedef T vec8 __attribute__((ext_vector_type(8)));
    extern __shared__ __attribute__((aligned(16))) float red[];   // [C] (deterministic mode: [PPP][C])
    const int LP = C / 8, PPP = 256 / LP;
    const int tid = threadIdx.x, n = blockIdx.y;
    const int p0 = blockIdx.x * pix_per_block, p1 = min(HW, p0 + pix_per_block);
    for (int i = tid; i < C; i += 256) red[i] = 0.f;
    __syncthreads();
    const int cg = tid % LP, pl = tid / LP;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    if (pl < PPP) {
        for (int p = p0 + pl; p < p1; p += PPP) {
            const int64_t off = ((int64_t)n * HW + p) * C + cg * 8;
            const vec8 av = *(const vec8*)(a + off), bv = *(const vec8*)(b + off);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] += (float)(T)((float)av[j] * (float)bv[j]);   // product rounded as torch's
        }
        if (det_ws) {
            det_rows_store(red, C, pl, cg * 8, acc);
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) atomicAdd(&red[cg * 8 + j], acc[j]);
        }
    }
    __syncthreads();
    if (det_ws) {
        // slot per workgroup: [blockIdx.x][N][C]
        for (int i = tid; i < C; i += 256)
            det_ws[((int64_t)blockIdx.x * gridDim.y + n) * C + i] = det_rows_sum(red, C, PPP, i);
        return;
    }
    for (int i = tid; i < C; i += 256) atomicAdd(&out[(int64_t)n * C + i], red[i]);
}

// out = act'(a * sa[n,c] + b * sb[n,c]; y) (the act' factor only when y is given), dot[n,c] += sum_p a * e:
// the elementwise steps of the layers' create_graph VJP nodes (torch_utils/ops/modconv.py _LayerVJP) in one
// pass each -- G = g_dx * s + g_ds * x with the modulation gradient's sum_p g_dx * dxs, the input-gradient
// sum gxc + g_ds * dxs, and act'(A d + g_dd * c; y) -- where autograd runs two to four full-size passes.
// f32 arithmetic, one rounding to T.  Same lane layout as layer_bwd_kernel.
struct AxArgs {
    void* out;
    const void *a, *b, *y, *e;
    const float *sa, *sb;
    float* dot;
    int N, HW, C, pix_per_block, act;
    float alpha, gain, clamp;
    float* det_dot;      // deterministic mode: [gridDim.x][N][C] slot partials of dot
};

template <typename T>
__global__ __launch_bounds__(256) void vjp_axpy_kernel(AxArgs a) {
    constexpr int V = 16 / sizeof(T) < 8 ? 16 / sizeof(T) : 8;   // elements per 16-byte load
    constexpr int NL = 8 / V;
    typedef T vecv __attribute__((ext_vector_type(V)));
    extern __shared__ __attribute__((aligned(16))) float red[];   // [C] when dot (deterministic mode: [PPP][C])
    const int LP = a.C / 8, PPP = 256 / LP;
    const int tid = threadIdx.x, n = blockIdx.y;
    const int p0 = blockIdx.x * a.pix_per_block, p1 = min(a.HW, p0 + a.pix_per_block);
    if (a.dot) {
        for (int i = tid; i < a.C; i += 256) red[i] = 0.f;
        __syncthreads();
    }
    const int cg = tid % LP, pl = tid / LP, c0 = cg * 8;
    const bool active = pl < PPP;
    float sa[8], sb[8], acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        sa[j] = (a.sa && active) ? a.sa[(int64_t)n * a.C + c0 + j] : 1.f;
        sb[j] = (a.sb && active) ? a.sb[(int64_t)n * a.C + c0 + j] : 1.f;
        acc[j] = 0.f;
    }
    const int64_t bytes = (int64_t)a.N * a.HW * a.C * (int64_t)sizeof(T);
    const __amdgpu_buffer_rsrc_t ra = make_rsrc(a.a, bytes), rb = make_rsrc(a.b ? a.b : a.a, bytes),
                                 ry = make_rsrc(a.y ? a.y : a.a, bytes), re = make_rsrc(a.e ? a.e : a.a, bytes);
    const bool hb = a.b != nullptr, hy = a.y != nullptr, he = a.e != nullptr && a.dot != nullptr;
    T* out = (T*)a.out;
    constexpr int U = 4;
    if (active) {
        for (int pb = p0 + pl; pb < p1; pb += PPP * U) {
            vecv av[U][NL], bv[U][NL], yv[U][NL], ev[U][NL];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int p = pb + u * PPP;
                const int boff = p < p1 ? (int)((((int64_t)n * a.HW + p) * a.C + c0) * (int64_t)sizeof(T)) : -1;
#pragma unroll
                for (int l = 0; l < NL; ++l) {
                    const int o = boff < 0 ? -1 : boff + 16 * l;
                    av[u][l] = buf_load16<vecv>(ra, o);
                    if (hb) bv[u][l] = buf_load16<vecv>(rb, o);
                    if (hy) yv[u][l] = buf_load16<vecv>(ry, o);
                    if (he) ev[u][l] = buf_load16<vecv>(re, o);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int p = pb + u * PPP;
                vecv o[NL];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int l = j / V, k = j % V;
                    const float x = (float)av[u][l][k];
                    float v = x * sa[j];
                    if (hb) v = fmaf((float)bv[u][l][k], sb[j], v);
                    if (hy) {
                        const float yy = (float)yv[u][l][k];
                        v *= a.gain;
                        if (a.act == 1 && !(yy > 0.f)) v *= a.alpha;
                        if (a.clamp >= 0.f && !(yy > -a.clamp && yy < a.clamp)) v = 0.f;
                    }
                    if (he) acc[j] = fmaf(x, (float)ev[u][l][k], acc[j]);
                    o[l][k] = (T)v;
                }
                if (p < p1) {
#pragma unroll
                    for (int l = 0; l < NL; ++l) *(vecv*)(out + ((int64_t)n * a.HW + p) * a.C + c0 + l * V) = o[l];
                }
            }
        }
        if (he) {
            if (a.det_dot) {
                det_rows_store(red, a.C, pl, c0, acc);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) atomicAdd(&red[c0 + j], acc[j]);
            }
        }
    }
    if (he) {
        __syncthreads();
        if (a.det_dot) {
            for (int i = tid; i < a.C; i += 256)
                a.det_dot[((int64_t)blockIdx.x * a.N + n) * a.C + i] = det_rows_sum(red, a.C, PPP, i);
            return;
        }
        for (int i = tid; i < a.C; i += 256) atomicAdd(&a.dot[(int64_t)n * a.C + i], red[i]);
    }
}

}  // namespace
}  // namespace sg2

extern "C" int sg2_vjp_axpy(void* out, const void* a, const float* sa, const void* b, const float* sb, const void* y,
                            int act, float alpha, float gain, float clamp, const void* e, float* dot, int dtype, int N,
                            int HW, int C, void* stream) {
    using namespace sg2;
    SG2_CHECK(out && a, "sg2_vjp_axpy: null pointer");
    SG2_CHECK((e == nullptr) == (dot == nullptr), "sg2_vjp_axpy: e and dot go together");
    SG2_CHECK(C % 8 == 0 && C <= 2048 && C >= 8, "sg2_vjp_axpy: C must be a multiple of 8 (<= 2048)");
    SG2_CHECK(dtype == SG2_F16 || dtype == SG2_BF16 || dtype == SG2_F32, "sg2_vjp_axpy: bad dtype");
    SG2_CHECK(act == 0 || act == 1, "sg2_vjp_axpy: act must be linear or lrelu");
    if ((int64_t)N * HW == 0) return 0;
    SG2_CHECK((int64_t)N * HW * C * 4 < INT32_MAX, "sg2_vjp_axpy: tensor too large (32-bit buffer offsets)");
    hipStream_t s = as_stream(stream);
    if (dot) {
        hipError_t err = zero_acc(dot, (int64_t)N * C * sizeof(float), s);
        if (err) { set_error("sg2_vjp_axpy: memset failed"); return err; }
    }
    AxArgs x{};
    x.out = out; x.a = a; x.b = b; x.y = y; x.e = e; x.sa = sa; x.sb = sb; x.dot = dot;
    x.N = N; x.HW = HW; x.C = C; x.act = act; x.alpha = alpha; x.gain = gain; x.clamp = clamp;
    const int PPP = std::max(1, 256 / (C / 8));
    x.pix_per_block = std::min(HW, PPP * 16);
    dim3 grid((unsigned)cdiv(HW, x.pix_per_block), (unsigned)N);
    DetArena arena;
    if (dot && det_on()) SG2_DET_GET(x.det_dot, arena, (int64_t)grid.x * N * C, "sg2_vjp_axpy");
    const size_t lds = dot ? (x.det_dot ? (size_t)PPP * C : (size_t)C) * sizeof(float) : 0;
    if (dtype == SG2_F16) vjp_axpy_kernel<f16_t><<<grid, 256, lds, s>>>(x);
    else if (dtype == SG2_BF16) vjp_axpy_kernel<bf16_t><<<grid, 256, lds, s>>>(x);
    else vjp_axpy_kernel<float><<<grid, 256, lds, s>>>(x);
    int rc = launch_status("sg2_vjp_axpy");
    if (rc || !x.det_dot) return rc;
    hipError_t err = det_sum(dot, 0, x.det_dot, 0, (int64_t)N * C, 1, grid.x, (int64_t)N * C, arena, s, det_assign());
    if (err) { set_error("sg2_vjp_axpy: det_sum"); return err; }
    return 0;
}

extern "C" int sg2_layer_bwd(void* dc, float* db, float* dd, float* dnoise, const void* dy, const void* y,
                             const void* c, const float* d, int dtype, int N, int HW, int C, int act, float alpha,
                             float gain, float clamp, void* stream) {
    using namespace sg2;
    SG2_CHECK(dc && dy && y, "sg2_layer_bwd: null pointer");
    SG2_CHECK(C % 8 == 0 && C <= 2048 && C >= 8, "sg2_layer_bwd: C must be a multiple of 8 (<= 2048)");
    SG2_CHECK(dtype == SG2_F16 || dtype == SG2_BF16 || dtype == SG2_F32, "sg2_layer_bwd: bad dtype");
    SG2_CHECK(act == 0 || act == 1, "sg2_layer_bwd: act must be linear or lrelu");
    if ((int64_t)N * HW == 0) return 0;
    SG2_CHECK((int64_t)N * HW * C * 4 < INT32_MAX, "sg2_layer_bwd: tensor too large (32-bit buffer offsets)");
    hipStream_t s = as_stream(stream);
    if (db && dd == db + C) {   // adjacent accumulators (the Python wrapper's layout): one memset
        hipError_t e = zero_acc(db, ((int64_t)N + 1) * C * sizeof(float), s);
        if (e) { set_error("memset"); return e; }
    } else {
        if (db) { hipError_t e = zero_acc(db, C * sizeof(float), s); if (e) { set_error("memset"); return e; } }
        if (dd) { hipError_t e = zero_acc(dd, (int64_t)N * C * sizeof(float), s); if (e) { set_error("memset"); return e; } }
    }
    LBArgs a{};
    a.dy = dy; a.y = y; a.c = c; a.d = d; a.dc = dc; a.db = db; a.dd = dd; a.dnoise = dnoise;
    a.N = N; a.HW = HW; a.C = C; a.alpha = alpha; a.gain = gain; a.clamp = clamp; a.act = act;
    const int LP = C / 8;
    const int PPP = std::max(1, 256 / LP);
    // ~16 passes per workgroup; enough workgroups to cover the chip
    a.pix_per_block = std::min(HW, PPP * 16);
    dim3 grid((unsigned)cdiv(HW, a.pix_per_block), (unsigned)N);
    DetArena arena;
    const bool det = det_on() && (db || dd);
    if (det_on() && dnoise) SG2_CHECK(LP <= 64, "sg2_layer_bwd: deterministic mode needs C <= 512 with dnoise");
    if (det && db) SG2_DET_GET(a.det_db, arena, (int64_t)grid.x * N * C, "sg2_layer_bwd");
    if (det && dd) SG2_DET_GET(a.det_dd, arena, (int64_t)grid.x * N * C, "sg2_layer_bwd");
    const size_t lds = (2 * C + a.pix_per_block + (det ? PPP * C : 0)) * sizeof(float);
    if (dtype == SG2_F16) layer_bwd_kernel<f16_t><<<grid, 256, lds, s>>>(a);
    else if (dtype == SG2_BF16) layer_bwd_kernel<bf16_t><<<grid, 256, lds, s>>>(a);
    else layer_bwd_kernel<float><<<grid, 256, lds, s>>>(a);
    int rc = launch_status("sg2_layer_bwd");
    if (rc || !det) return rc;
    hipError_t err = hipSuccess;
    DetSumJob jobs[2];
    int nj = 0;
    if (db) jobs[nj++] = DetSumJob{db, 0, a.det_db, 0, C, 1, (int64_t)grid.x * N, C, det_assign()};
    if (dd) jobs[nj++] = DetSumJob{dd, 0, a.det_dd, 0, (int64_t)N * C, 1, grid.x, (int64_t)N * C, det_assign()};
    err = det_sum_multi(jobs, nj, arena, s);
    if (err) { set_error("sg2_layer_bwd: det_sum"); return err; }
    return 0;
}

extern "C" int sg2_dot_hw(float* out, const void* a, const void* b, int dtype, int N, int HW, int C, void* stream) {
    using namespace sg2;
    SG2_CHECK(out && a && b, "sg2_dot_hw: null pointer");
    SG2_CHECK(C % 8 == 0 && C >= 8 && C <= 2048, "sg2_dot_hw: C must be a multiple of 8 (<= 2048)");
    SG2_CHECK(dtype == SG2_F16 || dtype == SG2_BF16, "sg2_dot_hw: f16/bf16 only");
    SG2_CHECK(((uintptr_t)a % 16) == 0 && ((uintptr_t)b % 16) == 0, "sg2_dot_hw: 16-byte alignment required");
    if ((int64_t)N * HW == 0) return 0;
    hipStream_t s = as_stream(stream);
    hipError_t e = zero_fill(out, (int64_t)N * C * sizeof(float), s);
    if (e) { set_error("sg2_dot_hw: memset failed"); return e; }
    const int PPP = std::max(1, 256 / (C / 8));
    const int ppb = std::min(HW, PPP * 32);
    dim3 grid((unsigned)cdiv(HW, ppb), (unsigned)N);
    DetArena arena;
    float* det_ws = nullptr;
    if (det_on()) SG2_DET_GET(det_ws, arena, (int64_t)grid.x * N * C, "sg2_dot_hw");
    const size_t lds = (det_ws ? (size_t)PPP * C : (size_t)C) * sizeof(float);
    if (dtype == SG2_F16)
        dot_hw_kernel<f16_t><<<grid, 256, lds, s>>>(out, (const f16_t*)a, (const f16_t*)b, HW, C, ppb, det_ws);
    else dot_hw_kernel<bf16_t><<<grid, 256, lds, s>>>(out, (const bf16_t*)a, (const bf16_t*)b, HW, C, ppb, det_ws);
    int rc = launch_status("sg2_dot_hw");
    if (rc || !det_ws) return rc;
    e = det_sum(out, 0, det_ws, 0, (int64_t)N * C, 1, grid.x, (int64_t)N * C, arena, s);
    if (e) { set_error("sg2_dot_hw: det_sum"); return e; }
    return 0;
}
