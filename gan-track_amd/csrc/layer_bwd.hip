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
    const T* dyp = (const T*)a.dy;
    const T* yp = (const T*)a.y;
    const T* cp = (const T*)a.c;
    T* dcp = (T*)a.dc;
    if (active) {
        for (int p = p0 + pl; p < p1; p += PPP) {
            const int64_t off = ((int64_t)n * a.HW + p) * a.C + c0;
            const vec8 g = *(const vec8*)(dyp + off);
            const vec8 yv = *(const vec8*)(yp + off);
            vec8 cv;
            if (cp) cv = *(const vec8*)(cp + off);
            vec8 o;
            float psum = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float yy = (float)yv[j];
                float dz = (float)g[j] * a.gain;
                if (a.act == 1 && !(yy > 0.f)) dz *= a.alpha;
                if (a.clamp >= 0.f && !(yy > -a.clamp && yy < a.clamp)) dz = 0.f;
                adb[j] += dz;
                psum += dz;
                if (cp) add[j] += dz * (float)cv[j];
                o[j] = (T)(dz * dv[j]);
            }
            *(vec8*)(dcp + off) = o;
            if (a.dnoise) atomicAdd(&s_dn[p - p0], psum);
        }
    }
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
    if (a.dnoise)
        for (int p = p0 + tid; p < p1; p += 256) a.dnoise[(int64_t)n * a.HW + p] = s_dn[p - p0];
}

}  // namespace
}  // namespace sg2

extern "C" int sg2_layer_bwd(void* dc, float* db, float* dd, float* dnoise, const void* dy, const void* y,
                             const void* c, const float* d, int dtype, int N, int HW, int C, int act, float alpha,
                             float gain, float clamp, void* stream) {
    using namespace sg2;
    SG2_CHECK(dc && dy && y, "sg2_layer_bwd: null pointer");
    SG2_CHECK(C % 8 == 0 && C <= 2048 && C >= 8, "sg2_layer_bwd: C must be a multiple of 8 (<= 2048)");
    SG2_CHECK(dtype == SG2_F16 || dtype == SG2_BF16 || dtype == SG2_F32, "sg2_layer_bwd: bad dtype");
    SG2_CHECK(act == 0 || act == 1, "sg2_layer_bwd: act must be linear or lrelu");
    if ((int64_t)N * HW == 0) return 0;
    hipStream_t s = as_stream(stream);
    if (db) { hipError_t e = hipMemsetAsync(db, 0, C * sizeof(float), s); if (e) { set_error("memset"); return e; } }
    if (dd) { hipError_t e = hipMemsetAsync(dd, 0, (int64_t)N * C * sizeof(float), s); if (e) { set_error("memset"); return e; } }
    LBArgs a{};
    a.dy = dy; a.y = y; a.c = c; a.d = d; a.dc = dc; a.db = db; a.dd = dd; a.dnoise = dnoise;
    a.N = N; a.HW = HW; a.C = C; a.alpha = alpha; a.gain = gain; a.clamp = clamp; a.act = act;
    const int LP = C / 8;
    const int PPP = std::max(1, 256 / LP);
    // ~16 passes per workgroup; enough workgroups to cover the chip
    a.pix_per_block = std::min(HW, PPP * 16);
    dim3 grid((unsigned)cdiv(HW, a.pix_per_block), (unsigned)N);
    const size_t lds = (2 * C + a.pix_per_block) * sizeof(float);
    if (dtype == SG2_F16) layer_bwd_kernel<f16_t><<<grid, 256, lds, s>>>(a);
    else if (dtype == SG2_BF16) layer_bwd_kernel<bf16_t><<<grid, 256, lds, s>>>(a);
    else layer_bwd_kernel<float><<<grid, 256, lds, s>>>(a);
    return launch_status("sg2_layer_bwd");
}
