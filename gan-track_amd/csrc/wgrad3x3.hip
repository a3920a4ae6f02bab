// Weight gradient of the 3x3 / stride 1 / pad 1 convolution with an LDS halo tile (16-bit layers).
//
//   dw[a][tap][b] = sum_{n,y,x} g[n,y,x,a] * x[n, y+ky-1, x+kx-1, b] * s[n,b]      (s optional)
//
// The generic weight-gradient kernel (conv.hip) runs one GEMM per tap, so it re-reads g and the
// shifted x nine times and does only 4 MFMAs per barrier at C = 64.  Here a workgroup owns a
// 64 (a) x 64 (b) channel block and walks a range of 256-pixel tiles (TW x TH of one sample):
// per tile it stages g[256 px][64] and the (TH+2) x (TW+2) halo of x[.][64] in LDS once, then every
// wave accumulates ALL nine taps of its 32 x 32 (a, b) sub-block:
//   per 16-pixel k-step: 1 A fragment (g) + 9 B fragments (x shifted by the tap) through
//   ds_read_b64_tr_b16, 9 v_mfma_f32_32x32x16 -- 144 MFMAs per tile and wave.
// The pixel dimension is the GEMM's K, so partial sums over tiles stay in registers (9 x 16 f32 per
// lane) and leave through one float atomic per (a, tap, b) per workgroup at the end.
// The next tile's global loads are issued before the current tile's MFMAs (register staging).
// Replaces the cuDNN weight gradient of the reference's 3x3 convolutions
// (SG3/torch_utils/ops/conv2d_gradfix.py:37-45 -> autograd of F.conv2d).
#include "sg2_common.h"

#include <algorithm>
#include <type_traits>

namespace sg2 {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x8w __attribute__((ext_vector_type(8)));

constexpr int BC = 64;          // channels per block in a and in b
constexpr int LD = BC + 8;      // LDS row pitch (elements) of both tiles

struct W3Args {
    const void* g;        // [N,H,W,A]
    const void* x;        // [N,H,W,B]
    const float* scale;   // [N,B] or null
    float* dw;            // [A][9][B], accumulated
    int N, H, W, A, B;
    int tiles_x, tiles_y, tiles;   // per sample / total
    int tiles_per_block;
};

template <typename T>
using v8w = typename std::conditional<std::is_same<T, bf16_t>::value, bf16x8, f16x8>::type;

template <typename T>
__device__ __forceinline__ f32x16 mma32(v8w<T> a, v8w<T> b, f32x16 c) {
    if constexpr (std::is_same<T, bf16_t>::value)
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// 32x32x16 operand fragment from a row-major (pixel-major) LDS tile: lane l gets column c0 + (l & 31)
// at rows r(8 * (l >> 5) + j), j = 0..7, where the 8 rows of each half are consecutive starting at
// row0[half].  ds_read_b64_tr_b16 transposes a 4-row x 16-column block inside each 16-lane group.
template <typename T>
__device__ __forceinline__ v8w<T> frag32(const T* tile, int row0, int c0, int lane) {
    const int G = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const T* p0 = tile + (row0 + q) * LD + c0 + 16 * (G & 1) + 4 * p;
    const T* p1 = p0 + 4 * LD;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p0);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p1);
    s16x8w r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(v8w<T>, r);
}

template <typename T, int TW>
__global__ __launch_bounds__(256) void wgrad3x3_kernel(W3Args a) {
    constexpr int TH = 256 / TW;
    constexpr int HWD = TW + 2, HP = HWD * (TH + 2);     // halo width / pixels
    constexpr int GCH = 8;                               // g: 256 px x 8 chunks / 256 threads
    constexpr int XCH = (HP * 8 + 255) / 256;            // x halo chunks per thread
    typedef T vec8 __attribute__((ext_vector_type(8)));

    __shared__ __attribute__((aligned(16))) T gs[256 * LD];
    __shared__ __attribute__((aligned(16))) T xs[HP * LD];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wa = wave >> 1, wb = wave & 1;            // 32 x 32 sub-block of the 64 x 64
    const int a0 = blockIdx.x * BC, b0 = blockIdx.y * BC;
    const int t_begin = blockIdx.z * a.tiles_per_block;
    const int t_end = min(a.tiles, t_begin + a.tiles_per_block);
    const T* __restrict__ gp = (const T*)a.g;
    const T* __restrict__ xp = (const T*)a.x;
    const int cc = (tid & 7) * 8;                       // channel chunk of this thread (fixed)
    const bool a_ok = a0 + cc < a.A, b_ok = b0 + cc < a.B;

    vec8 rg[GCH], rx[XCH];
    bool okg[GCH], okx[XCH];
    float sc[8];
    auto gload = [&](int t) {
        const int per = a.tiles_x * a.tiles_y;
        const int n = t / per, r = t - n * per;
        const int ty0 = (r / a.tiles_x) * TH, tx0 = (r % a.tiles_x) * TW;
#pragma unroll
        for (int i = 0; i < GCH; ++i) {
            const int px = (tid >> 3) + i * 32;          // tile pixel
            const int oy = ty0 + px / TW, ox = tx0 + px % TW;
            const bool ok = a_ok && oy < a.H && ox < a.W;
            okg[i] = ok;
            const int64_t off = ((int64_t)(n * a.H + (ok ? oy : 0)) * a.W + (ok ? ox : 0)) * a.A + (a_ok ? a0 + cc : 0);
            rg[i] = *(const vec8*)(gp + off);
        }
#pragma unroll
        for (int i = 0; i < XCH; ++i) {
            const int hp = (tid >> 3) + i * 32;
            const int iy = ty0 - 1 + hp / HWD, ix = tx0 - 1 + hp % HWD;
            const bool ok = b_ok && hp < HP && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
            okx[i] = ok;
            const int64_t off = ((int64_t)(n * a.H + (ok ? iy : 0)) * a.W + (ok ? ix : 0)) * a.B + (b_ok ? b0 + cc : 0);
            rx[i] = *(const vec8*)(xp + off);
        }
        if (a.scale) {
#pragma unroll
            for (int j = 0; j < 8; ++j) sc[j] = a.scale[(int64_t)n * a.B + (b_ok ? b0 + cc + j : 0)];
        }
    };
    auto sstore = [&]() {
#pragma unroll
        for (int i = 0; i < GCH; ++i) {
            vec8 v = rg[i];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = okg[i] ? v[j] : (T)0.f;
            *(vec8*)(gs + ((tid >> 3) + i * 32) * LD + cc) = v;
        }
#pragma unroll
        for (int i = 0; i < XCH; ++i) {
            const int hp = (tid >> 3) + i * 32;
            vec8 v = rx[i];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float f = okx[i] ? (float)v[j] : 0.f;
                if (a.scale) f *= sc[j];
                v[j] = (T)f;
            }
            if (hp < HP) *(vec8*)(xs + hp * LD + cc) = v;
        }
    };

    f32x16 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[t][j] = 0.f;

    if (t_begin < t_end) {
        gload(t_begin);
        sstore();
        __syncthreads();
        for (int t = t_begin; t < t_end; ++t) {
            const bool more = t + 1 < t_end;
            if (more) gload(t + 1);
#pragma unroll 2
            for (int k0 = 0; k0 < 256; k0 += 16) {
                // this lane's 8 pixels: k0 + 8 * (lane >> 5) + j, all in one tile row
                const int pr = k0 + 8 * ((lane >> 4) >> 1);
                const int py = pr / TW, px = pr % TW;
                const v8w<T> fa = frag32<T>(gs, pr, wa * 32, lane);
#pragma unroll
                for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                    for (int kx = 0; kx < 3; ++kx) {
                        const v8w<T> fb = frag32<T>(xs, (py + ky) * HWD + px + kx, wb * 32, lane);
                        acc[ky * 3 + kx] = mma32<T>(fa, fb, acc[ky * 3 + kx]);
                    }
            }
            __syncthreads();
            if (more) {
                sstore();
                __syncthreads();
            }
        }
    }

    // acc[tap][j]: a = a0 + 32 wa + 8 (j / 4) + 4 (lane >> 5) + (j % 4), b = b0 + 32 wb + (lane & 31)
    const int b = b0 + wb * 32 + (lane & 31);
    if (b < a.B) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int ar = a0 + wa * 32 + 8 * (j >> 2) + 4 * (lane >> 5) + (j & 3);
            if (ar >= a.A) continue;
#pragma unroll
            for (int t = 0; t < 9; ++t) atomicAdd(a.dw + ((int64_t)ar * 9 + t) * a.B + b, acc[t][j]);
        }
    }
}

}  // namespace

// Called by sg2_conv2d_wgrad for 16-bit 3x3 / s1 / p1 problems with A % 8 == 0, B % 8 == 0 and
// 16-byte aligned operands (dw already zeroed).
int wgrad3x3_launch(float* dw, const void* g, const void* x, const float* scale, int dtype, int N, int A, int H, int W,
                    int B, hipStream_t s) {
    W3Args a{};
    a.g = g; a.x = x; a.scale = scale; a.dw = dw;
    a.N = N; a.H = H; a.W = W; a.A = A; a.B = B;
    const int TW = W >= 32 ? 32 : 16;
    a.tiles_x = (int)cdiv(W, TW);
    a.tiles_y = (int)cdiv(H, 256 / TW);
    a.tiles = N * a.tiles_x * a.tiles_y;
    const int cb = (int)(cdiv(A, BC) * cdiv(B, BC));
    // ~512 workgroups (2 per CU over the launch), at least 4 tiles each
    int splits = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(512, cb), a.tiles / 4));
    a.tiles_per_block = (int)cdiv(a.tiles, splits);
    splits = (int)cdiv(a.tiles, a.tiles_per_block);
    dim3 grid((unsigned)cdiv(A, BC), (unsigned)cdiv(B, BC), (unsigned)splits);
    if (dtype == SG2_F16) {
        if (TW == 32) wgrad3x3_kernel<f16_t, 32><<<grid, 256, 0, s>>>(a);
        else wgrad3x3_kernel<f16_t, 16><<<grid, 256, 0, s>>>(a);
    } else {
        if (TW == 32) wgrad3x3_kernel<bf16_t, 32><<<grid, 256, 0, s>>>(a);
        else wgrad3x3_kernel<bf16_t, 16><<<grid, 256, 0, s>>>(a);
    }
    return launch_status("sg2_conv2d_wgrad (3x3 halo)");
}

}  // namespace sg2
