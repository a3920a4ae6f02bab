// Weight gradient of the 3x3 convolutions (stride 1 or 2, and the transposed stride-2 convolution
// of the up layers) with an LDS halo tile, for the 16-bit layers.
//
//   dw[a][ky][kx][b] = sum_{n,oy,ox} g[n,oy,ox,a] u[n,a] * x[n, oy*S + ky - P, ox*S + kx - P, b] s[n,b]
//   (u = g_scale, s = x_scale: a layer's modulation, optional)
//
// Split by output phase: with S = 2, tap k reads x at (o + shift) * S + phase where
// (k - P) = shift * S + phase; for one phase the taps' shifts lie in {-1, 0, 1}.  So each phase is a
// "stride-1 halo" problem on the phase sub-grid of x: a workgroup owns a 64 (a) x 64 (b) channel block
// and walks a range of 256-pixel tiles of the g grid (TW x TH of one sample).  Per tile it stages
// g[256 px][64] and the (TH+2) x (TW+2) halo of the x phase sub-grid in LDS once; every wave then
// accumulates ALL the phase's taps for its 32 x 32 (a, b) sub-block:
//   per 16-pixel k-step: 1 A fragment (g) + NT B fragments (x shifted by the tap) through
//   ds_read_b64_tr_b16, NT v_mfma_f32_32x32x16.
// Pixels are the GEMM's K, so the partial sums stay in registers (NT x 16 f32 per lane) across tiles
// and leave through one float atomic per (a, tap, b) per workgroup.  The next tile's global loads are
// issued before the current tile's MFMAs (register staging).
// The generic per-tap weight-gradient kernel (conv.hip) re-reads g and x once per tap and does only 4
// MFMAs per barrier at C = 64; this one reads them once per phase.
// Replaces the cuDNN weight gradients of the reference's convolutions
// (SG3/torch_utils/ops/conv2d_gradfix.py:37-45 -> autograd of F.conv2d / F.conv_transpose2d).
#include "sg2_common.h"

#include <algorithm>
#include <type_traits>

namespace sg2 {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x8w __attribute__((ext_vector_type(8)));

constexpr int BC = 64;          // channels per block in a and in b
constexpr int LDP = BC + 8;     // padded LDS row pitch (elements), SWZ = false
// SWZ = true: 128-B unpadded rows whose 32-channel halves swap when bit 1 of the row is set, so the four
// rows of a ds_read_b64_tr_b16 block hit disjoint banks (rows r and r + 2 share a bank half and always
// differ in that bit); 75.5 KB of LDS instead of 86 KB
template <bool SWZ> struct Lay {
    static constexpr int LD = SWZ ? BC : LDP;
    static __device__ __forceinline__ int off(int row, int col) {
        return row * LD + (SWZ ? (col ^ (((row >> 1) & 1) << 5)) : col);
    }
};

struct PTap { int8_t dy, dx, out, pad_; };   // shift on the phase grid, output tap index
typedef __attribute__((address_space(3))) void* lds_ptr_w;

struct W3Args {
    const void* g;        // [N,GH,GW,A]
    const void* x;        // [N,XH,XW,B]
    const float* gscale;  // [N,A] or null
    const float* xscale;  // [N,B] or null
    float* dw;            // [A][KK][B], accumulated
    int N, GH, GW, XH, XW, A, B, KK;
    int S, PY, PX;        // stride and phase: x coordinate = (g coordinate + shift) * S + phase
    int tiles_x, tiles_y, tiles;
    int tiles_per_block;
    float alpha;          // dw += alpha * partial sums (a layer's weight gain)
    PTap taps[9];
    float* det;           // deterministic mode: [gridDim.z][A][KK][B] workgroup partials (det_sum adds them)
    int det_slots;
};

// dw[i] += v, or (deterministic mode) the workgroup's slot of i
__device__ __forceinline__ void w3_add(const W3Args& a, int64_t i, float v) {
    if (a.det) a.det[(int64_t)blockIdx.z * a.A * a.KK * a.B + i] = v;
    else atomicAdd(a.dw + i, v);
}

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
// at rows row0 + j, j = 0..7, where row0 already includes the 8 * (l >> 5) half offset.
// ds_read_b64_tr_b16 transposes a 4-row x 16-column block inside each 16-lane group.
template <typename T, bool SWZ>
__device__ __forceinline__ v8w<T> frag32(const T* tile, int row0, int c0, int lane) {
    const int G = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const T* p0 = tile + Lay<SWZ>::off(row0 + q, c0 + 16 * (G & 1) + 4 * p);
    const T* p1 = p0 + 4 * Lay<SWZ>::LD;       // row + 4 keeps the swizzle bit
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p0);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p1);
    s16x8w r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(v8w<T>, r);
}

template <typename T, int TW, int NT, bool SWZ>
__global__ __launch_bounds__(256) void wgrad3x3_kernel(W3Args a) {
    constexpr int LD = Lay<SWZ>::LD;
    constexpr int TH = 256 / TW;
    constexpr int HWD = TW + 2, HP = HWD * (TH + 2);     // halo width / pixels (g-grid coordinates)
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
    float gsc[8], xsc[8];
    // 32-bit offsets into raw buffer loads (out-of-range pixels read as zeros: no mask in sstore)
    const __amdgpu_buffer_rsrc_t rgb = make_rsrc(gp, (int64_t)a.N * a.GH * a.GW * a.A * (int64_t)sizeof(T));
    const __amdgpu_buffer_rsrc_t rxb = make_rsrc(xp, (int64_t)a.N * a.XH * a.XW * a.B * (int64_t)sizeof(T));
    auto gload = [&](int t) {
        const int per = a.tiles_x * a.tiles_y;
        const int n = t / per, r = t - n * per;
        const int ty0 = (r / a.tiles_x) * TH, tx0 = (r % a.tiles_x) * TW;
#pragma unroll
        for (int i = 0; i < GCH; ++i) {
            const int px = (tid >> 3) + i * 32;          // tile pixel
            const int oy = ty0 + px / TW, ox = tx0 + px % TW;
            const bool ok = a_ok && oy < a.GH && ox < a.GW;
            rg[i] = buf_load16<vec8>(rgb, ok ? (((n * a.GH + oy) * a.GW + ox) * a.A + a0 + cc) * (int)sizeof(T) : -1);
        }
#pragma unroll
        for (int i = 0; i < XCH; ++i) {
            const int hp = (tid >> 3) + i * 32;
            const int iy = (ty0 - 1 + hp / HWD) * a.S + a.PY, ix = (tx0 - 1 + hp % HWD) * a.S + a.PX;
            const bool ok = b_ok && hp < HP && (unsigned)iy < (unsigned)a.XH && (unsigned)ix < (unsigned)a.XW;
            rx[i] = buf_load16<vec8>(rxb, ok ? (((n * a.XH + iy) * a.XW + ix) * a.B + b0 + cc) * (int)sizeof(T) : -1);
        }
        if (a.gscale) {
#pragma unroll
            for (int j = 0; j < 8; ++j) gsc[j] = a.gscale[n * a.A + (a_ok ? a0 + cc + j : 0)];
        }
        if (a.xscale) {
#pragma unroll
            for (int j = 0; j < 8; ++j) xsc[j] = a.xscale[n * a.B + (b_ok ? b0 + cc + j : 0)];
        }
    };
    auto scale8 = [](vec8 v, const float* sc) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (T)((float)v[j] * sc[j]);
        return v;
    };
    auto sstore = [&]() {
#pragma unroll
        for (int i = 0; i < GCH; ++i)
            *(vec8*)(gs + Lay<SWZ>::off((tid >> 3) + i * 32, cc)) = a.gscale ? scale8(rg[i], gsc) : rg[i];
#pragma unroll
        for (int i = 0; i < XCH; ++i) {
            const int hp = (tid >> 3) + i * 32;
            if (hp < HP) *(vec8*)(xs + Lay<SWZ>::off(hp, cc)) = a.xscale ? scale8(rx[i], xsc) : rx[i];
        }
    };

    int toff[NT];   // halo row offset of each tap
#pragma unroll
    for (int t = 0; t < NT; ++t) toff[t] = (a.taps[t].dy + 1) * HWD + a.taps[t].dx + 1;

    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[t][j] = 0.f;

    if (t_begin < t_end) {
        gload(t_begin);
        sstore();
        __syncthreads();
        for (int t = t_begin; t < t_end; ++t) {
            const bool more = t + 1 < t_end;
            if (more) gload(t + 1);
            // rolling prefetch: B fragment tp of the next k-step is read into fb[tp] as soon as this
            // step's MFMA tp has consumed it, so every MFMA's operands were read a whole step earlier (the
            // compiler otherwise funnels the B reads through one register quad and waits before each MFMA)
            auto rowk = [&](int k0) { return k0 + 8 * ((lane >> 4) >> 1); };   // this lane's 8 pixels: one tile row
            auto hbk = [&](int k0) { const int pr = rowk(k0); return (pr / TW) * HWD + pr % TW; };
            v8w<T> fa = frag32<T, SWZ>(gs, rowk(0), wa * 32, lane), fb[NT];
#pragma unroll
            for (int tp = 0; tp < NT; ++tp) fb[tp] = frag32<T, SWZ>(xs, hbk(0) + toff[tp], wb * 32, lane);
#pragma unroll 2
            for (int k0 = 0; k0 < 256; k0 += 16) {
                const bool nx = k0 + 16 < 256;
                const int kn = nx ? k0 + 16 : k0;
                const v8w<T> fan = frag32<T, SWZ>(gs, rowk(kn), wa * 32, lane);
                const int hn = hbk(kn);
#pragma unroll
                for (int tp = 0; tp < NT; ++tp) {
                    acc[tp] = mma32<T>(fa, fb[tp], acc[tp]);
                    fb[tp] = frag32<T, SWZ>(xs, hn + toff[tp], wb * 32, lane);
                }
                fa = fan;
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
            for (int t = 0; t < NT; ++t)
                w3_add(a, ((int64_t)ar * a.KK + a.taps[t].out) * a.B + b, acc[t][j] * a.alpha);
        }
    }
}

// LDS-DMA form of the stride-1 kernel (round 3).  The kernel above stages each tile through registers
// (19 16-byte loads a lane, then a ds_write pass behind a barrier, during which the matrix pipe idles) and
// reads a padded 144-byte-pitch image whose ds_read_b64_tr_b16 row quads conflict 2-way (SQ_LDS_BANK_CONFLICT
// 0.45 of the LDS cycles).  Here:
//   * g and the x halo arrive by LDS-DMA (buffer_load ... lds, 1 KiB = 8 whole 128-byte pixel rows a
//     wave-instruction) into a double-buffered image: tile t + 1 is in flight while tile t's MFMAs run, one
//     barrier a tile, no staging registers (2 x 77 KB of LDS, one workgroup per CU as before);
//   * rows are unpadded and their 32-channel halves swap when bit 1 of the row is set (Lay<true>): the four rows
//     of a transposing read hit four disjoint bank quarters.  The DMA destination is lane-linear, so the swap
//     sits in the SOURCE address: lane l loads piece (l & 7) ^ (4 ((l >> 4) & 1)) of its row.  The halo rows
//     have a pitch of TW + 4 pixels (a multiple of 4; two pad columns never read), so bit 1 of a fragment row is
//     a function of the lane and the tap column only and every fragment read is a per-lane base plus an
//     immediate offset (the k-step loop is fully unrolled);
//   * the modulation (g_scale / x_scale, one value per channel and sample) leaves the inner loop: with a scale the
//     host gives each workgroup tiles of ONE sample, and the partial sums are multiplied by u[n, a] s[n, b] at
//     the final atomics.  The reference rounds x * round(s) to 16 bits before its GEMM; this keeps the product
//     in f32 (the difference is below the 16-bit rounding of the inputs).
// Stride 1, one phase holding every tap (3x3 pad 1, or 1x1 pad 0).
template <int TW> struct WDma {
    static constexpr int TH = 256 / TW, HWD = TW + 4, HP = HWD * (TH + 2);
    static_assert(HP % 8 == 0, "whole DMA instructions");
    static constexpr int GI = 256 / 8, XI = HP / 8;            // DMA wave-instructions per tile (g, x)
    static constexpr int GB = 256 * 128, STAGE = GB + HP * 128;
    static constexpr size_t LDS = 2 * (size_t)STAGE;
    static_assert(LDS <= 160 * 1024, "wgrad DMA LDS");
};

__device__ __forceinline__ unsigned lds_off_w(const void* p) {
    return (unsigned)(uintptr_t)(__attribute__((address_space(3))) const char*)p;
}

template <typename T>
__device__ __forceinline__ v8w<T> ld_frag(unsigned addr) {     // rows r .. r + 3 at addr, r + 4 .. r + 7 at + 512
    typedef __attribute__((address_space(3))) s16x4* lp;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(uintptr_t)addr);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(uintptr_t)(addr + 512));
    s16x8w r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(v8w<T>, r);
}

template <typename T, int TW, int NT, bool SC>
__global__ __launch_bounds__(256) void wgrad3x3_dma_kernel(W3Args a) {
    typedef WDma<TW> L;
    constexpr int TH = L::TH, HWD = L::HWD, HP = L::HP;
    constexpr int SZ = (int)sizeof(T);
    static_assert(SZ == 2, "16-bit");
    extern __shared__ __attribute__((aligned(16))) char wsm[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wa = wave >> 1, wb = wave & 1;
    const int a0 = blockIdx.x * BC, b0 = blockIdx.y * BC;
    const int t_begin = blockIdx.z * a.tiles_per_block;
    const int t_end = min(a.tiles, t_begin + a.tiles_per_block);
    if (t_begin >= t_end) return;
    const int GH = a.GH, GW = a.GW, XH = a.XH, XW = a.XW, A = a.A, B = a.B, tiles_x = a.tiles_x;
    const int per = tiles_x * a.tiles_y;
    const __amdgpu_buffer_rsrc_t rgb = make_rsrc(a.g, (int64_t)a.N * GH * GW * A * SZ);
    const __amdgpu_buffer_rsrc_t rxb = make_rsrc(a.x, (int64_t)a.N * XH * XW * B * SZ);
    const int l3 = lane >> 3;
    const int pj = (lane & 7) ^ (((lane >> 4) & 1) << 2);      // source piece of this lane (swizzle, see above)
    const bool gok = a0 + 8 * pj < A, xok = b0 + 8 * pj < B;   // out-of-block channels read zeros
    const int gch = (a0 + 8 * pj) * SZ, xch = (b0 + 8 * pj) * SZ;
    const unsigned lbase = lds_off_w(wsm);

    auto issue = [&](int t, int stage) {
        const int n = t / per, r = t - n * per;
        const int ty0 = (r / tiles_x) * TH, tx0 = (r - (r / tiles_x) * tiles_x) * TW;
        char* sb = wsm + stage * L::STAGE;
#pragma unroll
        for (int u = 0; u < L::GI / 4; ++u) {
            const int px = 8 * (u * 4 + wave) + l3;
            const int oy = ty0 + px / TW, ox = tx0 + px % TW;
            int off = ((n * GH + oy) * GW + ox) * A * SZ + gch;
            off = (gok && oy < GH && ox < GW) ? off : -1;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rgb, (lds_ptr_w)(sb + (u * 4 + wave) * 1024), 16, off, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < (L::XI + 3) / 4; ++u) {
            const int i = u * 4 + wave;                        // wave-uniform
            if (u < L::XI / 4 || i < L::XI) {
                const int hp = 8 * i + l3, hy = hp / HWD, hx = hp - hy * HWD;
                const int iy = ty0 - 1 + hy, ix = tx0 - 1 + hx;
                int off = ((n * XH + iy) * XW + ix) * B * SZ + xch;
                off = (xok && hx < TW + 2 && (unsigned)iy < (unsigned)XH && (unsigned)ix < (unsigned)XW) ? off : -1;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rxb, (lds_ptr_w)(sb + L::GB + i * 1024), 16, off, 0, 0, 0);
            }
        }
    };

    // fragment addressing (frag32 above, with the row arithmetic taken out): a 16-lane group G reads a 4-row
    // quad, lane li = 4 q + p at row + q, columns 4 p .. + 3 of its 16-column block.  Bit 1 of the row is bit 1
    // of q for g (rows k0 + 8 (lane >> 5) + q, k0 a multiple of 16) and of q + tap column for x (rows
    // (py + dy) HWD + px + dx + q with HWD and px multiples of 4).
    const int G = lane >> 4, q = (lane & 15) >> 2, p = lane & 3, hh = lane >> 5;
    const unsigned colA = ((wa * 32 + 16 * (G & 1) + 4 * p) * SZ) ^ (((q >> 1) & 1) << 6);
    const unsigned abase = (8 * hh + q) * 128 + colA;
    unsigned bbase[3];
#pragma unroll
    for (int dx = 0; dx < 3; ++dx)
        bbase[dx] = L::GB + (8 * hh + dx + q) * 128 + (((wb * 32 + 16 * (G & 1) + 4 * p) * SZ) ^ ((((dx + q) >> 1) & 1) << 6));
    auto tap_dy = [](int tp) { return NT == 9 ? tp / 3 : 1; };
    auto tap_dx = [](int tp) { return NT == 9 ? tp % 3 : 1; };

    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[t][j] = 0.f;
    const int b = b0 + wb * 32 + (lane & 31);

    issue(t_begin, 0);
    __builtin_amdgcn_s_waitcnt(0x0f70);                        // vmcnt(0): this wave's DMAs of the first tile
    __builtin_amdgcn_s_barrier();
    int k = 0;
    for (int t = t_begin; t < t_end; ++t, ++k) {
        const int stage = k & 1;
        if (t + 1 < t_end) issue(t + 1, stage ^ 1);            // the other stage was released by the last barrier
        const unsigned sa = lbase + stage * L::STAGE + abase;
        unsigned sb[3];
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) sb[dx] = lbase + stage * L::STAGE + bbase[dx];
        // k-step ks: g rows 16 ks.., x rows (py + dy) HWD + px0 + ...; next step's fragments read before this
        // step's MFMAs
        auto xoff = [&](int ks, int tp) {
            const int k0 = 16 * ks, py = k0 / TW, px0 = k0 % TW;
            return ((py + tap_dy(tp)) * HWD + px0) * 128;
        };
        // rolling prefetch: fragment tp of step ks + 1 is read as soon as step ks's MFMA tp has consumed it
        v8w<T> fa = ld_frag<T>(sa), fb[NT];
#pragma unroll
        for (int tp = 0; tp < NT; ++tp) fb[tp] = ld_frag<T>(sb[tap_dx(tp)] + xoff(0, tp));
        // (fully unrolled: every fragment read is base + immediate, and the compiler keeps the x fragments that a
        // later step reads again at another tap row in registers)
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) {
            const int kn = ks + 1 < 16 ? ks + 1 : ks;
            const v8w<T> fan = ld_frag<T>(sa + 16 * kn * 128);
#pragma unroll
            for (int tp = 0; tp < NT; ++tp) {
                acc[tp] = mma32<T>(fa, fb[tp], acc[tp]);
                if (ks + 1 < 16) fb[tp] = ld_frag<T>(sb[tap_dx(tp)] + xoff(kn, tp));
            }
            fa = fan;
        }
        // the next tile's DMAs (this wave's only outstanding vector-memory ops) have landed, and every wave is
        // done reading this stage before the next iteration's DMAs overwrite it
        __builtin_amdgcn_s_waitcnt(0x0070);                    // vmcnt(0) lgkmcnt(0)
        __builtin_amdgcn_s_barrier();
    }
    // SC: the host keeps every workgroup's tiles inside one sample, so the modulation u[n, a] s[n, b] is one
    // factor per (a, b) on the whole sum
    const int n0 = t_begin / per;
    const float sx = (SC && a.xscale) ? a.xscale[n0 * B + min(b, B - 1)] : 1.f;
    if (b < B) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int ar = a0 + wa * 32 + 8 * (j >> 2) + 4 * hh + (j & 3);
            if (ar >= A) continue;
            const float f = a.alpha * sx * ((SC && a.gscale) ? a.gscale[n0 * A + ar] : 1.f);
#pragma unroll
            for (int t = 0; t < NT; ++t)
                w3_add(a, ((int64_t)ar * a.KK + (NT == 9 ? t : 0)) * B + b, acc[t][j] * f);
        }
    }
}

// Stride-2 / pad-0 3x3 weight gradient in ONE launch (the discriminator's down-2 layers after their FIR
// and the transposed convs of the up layers): x coordinate = 2 g + k.  Where the phase split above runs
// four launches that each re-stage the whole of g and feed 1-4 MFMAs per A fragment, this kernel stages
// a 16 x 8 g tile and the (2*8+1) x (2*16+1) x region it reads ONCE, with each x row stored
// column-deinterleaved (its even columns, then its odd ones): the 8 consecutive g pixels of a fragment
// then read x columns 2 px + kx as 8 consecutive LDS rows for every tap, so all nine taps accumulate per
// A fragment (9 MFMAs per 16-pixel k-step, as the stride-1 kernel).
template <typename T, bool SWZ>
__global__ __launch_bounds__(256) void wgrad3x3_s2_kernel(W3Args a) {
    constexpr int LD = Lay<SWZ>::LD;
    constexpr int TW = 16, TH = 8, NP = TW * TH;          // g tile
    constexpr int XW = 2 * TW + 1, XH = 2 * TH + 1, XEV = TW + 1, HP = XW * XH;   // x region (561 px)
    constexpr int GCH = NP * 8 / 256;                     // 4 g loads per thread
    constexpr int XCH = (HP * 8 + 255) / 256;             // 18 x loads per thread
    typedef T vec8 __attribute__((ext_vector_type(8)));

    __shared__ __attribute__((aligned(16))) T gs[NP * LD];
    __shared__ __attribute__((aligned(16))) T xs[HP * LD];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wa = wave >> 1, wb = wave & 1;
    const int a0 = blockIdx.x * BC, b0 = blockIdx.y * BC;
    const int t_begin = blockIdx.z * a.tiles_per_block;
    const int t_end = min(a.tiles, t_begin + a.tiles_per_block);
    const T* __restrict__ gp = (const T*)a.g;
    const T* __restrict__ xp = (const T*)a.x;
    const int cc = (tid & 7) * 8;
    const bool a_ok = a0 + cc < a.A, b_ok = b0 + cc < a.B;

    vec8 rg[GCH], rx[XCH];
    float gsc[8], xsc[8];
    const __amdgpu_buffer_rsrc_t rgb = make_rsrc(gp, (int64_t)a.N * a.GH * a.GW * a.A * (int64_t)sizeof(T));
    const __amdgpu_buffer_rsrc_t rxb = make_rsrc(xp, (int64_t)a.N * a.XH * a.XW * a.B * (int64_t)sizeof(T));
    auto gload = [&](int t) {
        const int per = a.tiles_x * a.tiles_y;
        const int n = t / per, r = t - n * per;
        const int ty0 = (r / a.tiles_x) * TH, tx0 = (r % a.tiles_x) * TW;
#pragma unroll
        for (int i = 0; i < GCH; ++i) {
            const int px = (tid >> 3) + i * 32;
            const int oy = ty0 + px / TW, ox = tx0 + px % TW;
            const bool ok = a_ok && oy < a.GH && ox < a.GW;
            rg[i] = buf_load16<vec8>(rgb, ok ? (((n * a.GH + oy) * a.GW + ox) * a.A + a0 + cc) * (int)sizeof(T) : -1);
        }
#pragma unroll
        for (int i = 0; i < XCH; ++i) {
            const int hp = (tid >> 3) + i * 32;           // x region pixel, row-major (natural column order)
            const int iy = 2 * ty0 + hp / XW, ix = 2 * tx0 + hp % XW;
            const bool ok = b_ok && hp < HP && iy < a.XH && ix < a.XW;
            rx[i] = buf_load16<vec8>(rxb, ok ? (((n * a.XH + iy) * a.XW + ix) * a.B + b0 + cc) * (int)sizeof(T) : -1);
        }
        if (a.gscale) {
#pragma unroll
            for (int j = 0; j < 8; ++j) gsc[j] = a.gscale[n * a.A + (a_ok ? a0 + cc + j : 0)];
        }
        if (a.xscale) {
#pragma unroll
            for (int j = 0; j < 8; ++j) xsc[j] = a.xscale[n * a.B + (b_ok ? b0 + cc + j : 0)];
        }
    };
    auto scale8 = [](vec8 v, const float* sc) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (T)((float)v[j] * sc[j]);
        return v;
    };
    auto sstore = [&]() {
#pragma unroll
        for (int i = 0; i < GCH; ++i)
            *(vec8*)(gs + Lay<SWZ>::off((tid >> 3) + i * 32, cc)) = a.gscale ? scale8(rg[i], gsc) : rg[i];
#pragma unroll
        for (int i = 0; i < XCH; ++i) {
            const int hp = (tid >> 3) + i * 32;
            const int hy = hp / XW, hx = hp - hy * XW;
            const int row = hy * XW + ((hx & 1) ? XEV + (hx >> 1) : (hx >> 1));   // deinterleaved
            if (hp < HP) *(vec8*)(xs + Lay<SWZ>::off(row, cc)) = a.xscale ? scale8(rx[i], xsc) : rx[i];
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
            // rolling prefetch of the next k-step's fragments (see wgrad3x3_kernel)
            auto rowk = [&](int k0) { return k0 + 8 * ((lane >> 4) >> 1); };   // 8 pixels of one tile row
            auto xrow = [&](int k0, int ky, int kx) {
                const int pr = rowk(k0), py = pr / TW, px = pr % TW;
                return (2 * py + ky) * XW + ((kx & 1) ? XEV : 0) + px + (kx >> 1);
            };
            v8w<T> fa = frag32<T, SWZ>(gs, rowk(0), wa * 32, lane), fb[9];
#pragma unroll
            for (int t = 0; t < 9; ++t) fb[t] = frag32<T, SWZ>(xs, xrow(0, t / 3, t % 3), wb * 32, lane);
#pragma unroll 2
            for (int k0 = 0; k0 < NP; k0 += 16) {
                const int kn = k0 + 16 < NP ? k0 + 16 : k0;
                const v8w<T> fan = frag32<T, SWZ>(gs, rowk(kn), wa * 32, lane);
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    acc[t] = mma32<T>(fa, fb[t], acc[t]);
                    fb[t] = frag32<T, SWZ>(xs, xrow(kn, t / 3, t % 3), wb * 32, lane);
                }
                fa = fan;
            }
            __syncthreads();
            if (more) {
                sstore();
                __syncthreads();
            }
        }
    }

    const int b = b0 + wb * 32 + (lane & 31);
    if (b < a.B) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int ar = a0 + wa * 32 + 8 * (j >> 2) + 4 * (lane >> 5) + (j & 3);
            if (ar >= a.A) continue;
#pragma unroll
            for (int t = 0; t < 9; ++t) w3_add(a, ((int64_t)ar * 9 + t) * a.B + b, acc[t][j] * a.alpha);
        }
    }
}

// Pipelined form of the stride-2 kernel above (round 5).  That kernel holds a 99 KB single LDS buffer, so one
// workgroup (one wave per SIMD, 390 registers) runs per CU and every tile ends with compute, barrier, staging
// store, barrier: the matrix pipe idles through the store and both barriers (mfma_util 0.25, and the LDS bank
// conflicts it shows -- 0.40 of the LDS cycles -- are not what bounds it: the swizzled layout removes them and
// is 5 % slower, profiles/r05_pmc_wgrad.txt).  Here the g tile is 16 x 6 (96 pixels; the x region 33 x 13) and the
// LDS holds two stages (2 x 75.6 KB): tile t's MFMAs read stage t & 1 while tile t + 1's registers are stored
// into the other stage between its third and fourth k-step, the loads of tile t + 2 are issued right after that
// store, and ONE barrier ends the tile.
template <typename T>
__global__ __launch_bounds__(256) void wgrad3x3_s2p_kernel(W3Args a) {
    constexpr int LD = LDP;
    constexpr int TW = 16, TH = 6, NP = TW * TH;          // g tile (96 px, 6 k-steps of 16)
    constexpr int XW = 2 * TW + 1, XH = 2 * TH + 1, XEV = TW + 1, HP = XW * XH;   // x region (429 px)
    constexpr int GCH = NP * 8 / 256;                     // 3 g loads per thread
    constexpr int XCH = (HP * 8 + 255) / 256;             // 14 x loads per thread
    constexpr int STAGE = (NP + HP) * LD;                 // elements per stage
    typedef T vec8 __attribute__((ext_vector_type(8)));
    extern __shared__ __attribute__((aligned(16))) char smem_w[];
    T* const st0 = (T*)smem_w;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wa = wave >> 1, wb = wave & 1;
    const int a0 = blockIdx.x * BC, b0 = blockIdx.y * BC;
    const int t_begin = blockIdx.z * a.tiles_per_block;
    const int t_end = min(a.tiles, t_begin + a.tiles_per_block);
    const T* __restrict__ gp = (const T*)a.g;
    const T* __restrict__ xp = (const T*)a.x;
    const int cc = (tid & 7) * 8;
    const bool a_ok = a0 + cc < a.A, b_ok = b0 + cc < a.B;

    vec8 rg[GCH], rx[XCH];
    float gsc[8], xsc[8];
    const __amdgpu_buffer_rsrc_t rgb = make_rsrc(gp, (int64_t)a.N * a.GH * a.GW * a.A * (int64_t)sizeof(T));
    const __amdgpu_buffer_rsrc_t rxb = make_rsrc(xp, (int64_t)a.N * a.XH * a.XW * a.B * (int64_t)sizeof(T));
    auto gload = [&](int t) {
        const int per = a.tiles_x * a.tiles_y;
        const int n = t / per, r = t - n * per;
        const int ty0 = (r / a.tiles_x) * TH, tx0 = (r % a.tiles_x) * TW;
#pragma unroll
        for (int i = 0; i < GCH; ++i) {
            const int px = (tid >> 3) + i * 32;
            const int oy = ty0 + px / TW, ox = tx0 + px % TW;
            const bool ok = a_ok && oy < a.GH && ox < a.GW;
            rg[i] = buf_load16<vec8>(rgb, ok ? (((n * a.GH + oy) * a.GW + ox) * a.A + a0 + cc) * (int)sizeof(T) : -1);
        }
#pragma unroll
        for (int i = 0; i < XCH; ++i) {
            const int hp = (tid >> 3) + i * 32;
            const int iy = 2 * ty0 + hp / XW, ix = 2 * tx0 + hp % XW;
            const bool ok = b_ok && hp < HP && iy < a.XH && ix < a.XW;
            rx[i] = buf_load16<vec8>(rxb, ok ? (((n * a.XH + iy) * a.XW + ix) * a.B + b0 + cc) * (int)sizeof(T) : -1);
        }
        if (a.gscale) {
#pragma unroll
            for (int j = 0; j < 8; ++j) gsc[j] = a.gscale[n * a.A + (a_ok ? a0 + cc + j : 0)];
        }
        if (a.xscale) {
#pragma unroll
            for (int j = 0; j < 8; ++j) xsc[j] = a.xscale[n * a.B + (b_ok ? b0 + cc + j : 0)];
        }
    };
    auto scale8 = [](vec8 v, const float* sc) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (T)((float)v[j] * sc[j]);
        return v;
    };
    auto sstore = [&](T* gs, T* xs) {
#pragma unroll
        for (int i = 0; i < GCH; ++i)
            *(vec8*)(gs + Lay<false>::off((tid >> 3) + i * 32, cc)) = a.gscale ? scale8(rg[i], gsc) : rg[i];
#pragma unroll
        for (int i = 0; i < XCH; ++i) {
            const int hp = (tid >> 3) + i * 32;
            const int hy = hp / XW, hx = hp - hy * XW;
            const int row = hy * XW + ((hx & 1) ? XEV + (hx >> 1) : (hx >> 1));   // deinterleaved
            if (hp < HP) *(vec8*)(xs + Lay<false>::off(row, cc)) = a.xscale ? scale8(rx[i], xsc) : rx[i];
        }
    };

    f32x16 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[t][j] = 0.f;

    auto rowk = [&](int k0) { return k0 + 8 * ((lane >> 4) >> 1); };
    auto xrow = [&](int k0, int ky, int kx) {
        const int pr = rowk(k0), py = pr / TW, px = pr % TW;
        return (2 * py + ky) * XW + ((kx & 1) ? XEV : 0) + px + (kx >> 1);
    };
    if (t_begin < t_end) {
        gload(t_begin);
        sstore(st0, st0 + NP * LD);
        if (t_begin + 1 < t_end) gload(t_begin + 1);
        __syncthreads();
        int k = 0;
        for (int t = t_begin; t < t_end; ++t, ++k) {
            T* const gs = st0 + (k & 1) * STAGE;
            T* const xs = gs + NP * LD;
            T* const gn = st0 + ((k + 1) & 1) * STAGE;
            v8w<T> fa = frag32<T, false>(gs, rowk(0), wa * 32, lane), fb[9];
#pragma unroll
            for (int tp = 0; tp < 9; ++tp) fb[tp] = frag32<T, false>(xs, xrow(0, tp / 3, tp % 3), wb * 32, lane);
#pragma unroll
            for (int k0 = 0; k0 < NP; k0 += 16) {
                const int kn = k0 + 16 < NP ? k0 + 16 : k0;
                const v8w<T> fan = frag32<T, false>(gs, rowk(kn), wa * 32, lane);
#pragma unroll
                for (int tp = 0; tp < 9; ++tp) {
                    acc[tp] = mma32<T>(fa, fb[tp], acc[tp]);
                    fb[tp] = frag32<T, false>(xs, xrow(kn, tp / 3, tp % 3), wb * 32, lane);
                }
                fa = fan;
                if (k0 == 32 && t + 1 < t_end) {       // mid-tile: stage tile t + 1, then fetch tile t + 2
                    sstore(gn, gn + NP * LD);
                    if (t + 2 < t_end) gload(t + 2);
                }
            }
            __syncthreads();
        }
    }

    const int b = b0 + wb * 32 + (lane & 31);
    if (b < a.B) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int ar = a0 + wa * 32 + 8 * (j >> 2) + 4 * (lane >> 5) + (j & 3);
            if (ar >= a.A) continue;
#pragma unroll
            for (int t = 0; t < 9; ++t) w3_add(a, ((int64_t)ar * 9 + t) * a.B + b, acc[t][j] * a.alpha);
        }
    }
}
constexpr size_t W3P_LDS = 2 * (size_t)((16 * 6) + 33 * 13) * LDP * 2;    // 151,200 B (16-bit elements)

template <typename T>
void launch_w3p(const W3Args& a, dim3 grid, hipStream_t s) {
    auto kern = wgrad3x3_s2p_kernel<T>;
    static bool attr_set = false;   // benign race: idempotent attribute
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)W3P_LDS);
        attr_set = true;
    }
    kern<<<grid, 256, W3P_LDS, s>>>(a);
}

template <typename T, int TW, int NT>
void launch_w3(const W3Args& a, dim3 grid, hipStream_t s) {
    static const bool swz = [] { const char* e = getenv("SG2_WGRAD_SWZ"); return e != nullptr && e[0] == '1'; }();
    if (swz) wgrad3x3_kernel<T, TW, NT, true><<<grid, 256, 0, s>>>(a);
    else wgrad3x3_kernel<T, TW, NT, false><<<grid, 256, 0, s>>>(a);
}

template <typename T, int TW, int NT, bool SC>
void launch_wdma(const W3Args& a, dim3 grid, hipStream_t s) {
    auto kern = wgrad3x3_dma_kernel<T, TW, NT, SC>;
    static bool attr_set = false;   // benign race: idempotent attribute
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)WDma<TW>::LDS);
        attr_set = true;
    }
    kern<<<grid, 256, WDma<TW>::LDS, s>>>(a);
}

template <typename T, int TW>
int dispatch_nt(const W3Args& a, dim3 grid, int nt, hipStream_t s) {
    switch (nt) {
        case 1: launch_w3<T, TW, 1>(a, grid, s); break;
        case 2: launch_w3<T, TW, 2>(a, grid, s); break;
        case 4: launch_w3<T, TW, 4>(a, grid, s); break;
        case 9: launch_w3<T, TW, 9>(a, grid, s); break;
        default: set_error("sg2_conv2d_wgrad: unsupported tap count per phase"); return -1;
    }
    return 0;
}

int floordiv_w(int a, int b) { return (a >= 0) ? a / b : -((-a + b - 1) / b); }

// workgroups per launch the K (pixel) split aims at: one per CU (these kernels hold one workgroup per CU);
// every workgroup adds its 64 x 9 x 64 partial sums with float atomics, so more workgroups cost atomics
// (512: +10-25% time, 1024: +40-60%; profiles/r02_wgrad_wgs.log).  SG2_WGRAD_WGS overrides (tuning).
int wgrad_wgs() {
    static const int v = [] { const char* e = getenv("SG2_WGRAD_WGS"); return e ? std::max(1, atoi(e)) : 256; }();
    return v;
}

}  // namespace

// Is the halo weight gradient applicable?  (3x3 or 1x1 kernel, stride 1 or 2, every tap's shift on
// its phase grid within [-1, 1], 16-bit, channels multiples of 8, g grid at least 16 wide.)
bool wgrad_halo_ok(int dtype, int KH, int KW, int stride, int pad_y, int pad_x, int OW, int A, int B) {
    if (dtype == SG2_F32 || KH != KW || (KH != 3 && KH != 1) || stride < 1 || stride > 2) return false;
    if (A % 8 || B % 8 || OW < 16) return false;
    for (int k = 0; k < KH; ++k) {
        const int sy = floordiv_w(k - pad_y, stride), sx = floordiv_w(k - pad_x, stride);
        if (sy < -1 || sy > 1 || sx < -1 || sx > 1) return false;
    }
    return true;
}

namespace {
int wgrad3x3_run(W3Args& a, DetArena& arena, float* dw, const void* g, const void* x, const float* gscale,
                 const float* xscale, int dtype, int N, int A, int OH, int OW, int B, int H, int W, int KH, int KW,
                 int stride, int pad_y, int pad_x, float alpha, hipStream_t s);
}

// dw already zeroed.  One launch per output phase that has taps.  Deterministic mode: every launch writes its
// workgroups' partial sums to slots (blockIdx.z) of one zeroed [splits][A][KK][B] array, added in slot order
// into dw at the end.
int wgrad3x3_launch(float* dw, const void* g, const void* x, const float* gscale, const float* xscale, int dtype,
                    int N, int A, int OH, int OW, int B, int H, int W, int KH, int KW, int stride, int pad_y,
                    int pad_x, float alpha, hipStream_t s) {
    W3Args a{};
    DetArena arena;
    int rc = wgrad3x3_run(a, arena, dw, g, x, gscale, xscale, dtype, N, A, OH, OW, B, H, W, KH, KW, stride, pad_y,
                          pad_x, alpha, s);
    if (rc || !a.det) return rc;
    const int64_t nel = (int64_t)A * KH * KW * B;
    hipError_t e = det_sum(dw, 0, a.det, 0, nel, 1, a.det_slots, nel, arena, s, det_assign());
    if (e) { set_error("sg2_conv2d_wgrad: det_sum"); return (int)e; }
    return 0;
}

namespace {
// det mode: allocate the slot array for `slots` workgroup splits.  A launch that writes every tap of its
// workgroup's (a, b) block (all taps in one phase) fills its slot completely; `zero` (several phase launches, each
// writing its own taps) zeroes the array first.
int w3_det_slots(W3Args& a, DetArena& arena, int slots, hipStream_t s, bool zero = false) {
    if (!det_on()) return 0;
    const int64_t n = (int64_t)slots * a.A * a.KK * a.B;
    SG2_DET_GET(a.det, arena, n, "sg2_conv2d_wgrad (halo)");
    a.det_slots = slots;
    if (!zero) return 0;
    hipError_t e = zero_fill(a.det, n * sizeof(float), s);
    if (e) { set_error("sg2_conv2d_wgrad: zero"); return (int)e; }
    return 0;
}

int wgrad3x3_run(W3Args& a, DetArena& arena, float* dw, const void* g, const void* x, const float* gscale,
                 const float* xscale, int dtype, int N, int A, int OH, int OW, int B, int H, int W, int KH, int KW,
                 int stride, int pad_y, int pad_x, float alpha, hipStream_t s) {
    a.g = g; a.x = x; a.gscale = gscale; a.xscale = xscale; a.dw = dw; a.alpha = alpha;
    a.N = N; a.GH = OH; a.GW = OW; a.XH = H; a.XW = W; a.A = A; a.B = B; a.KK = KH * KW; a.S = stride;
    static const bool s2_on = [] { const char* e = getenv("SG2_WGRAD_S2"); return !e || atoi(e) != 0; }();
    if (s2_on && stride == 2 && KH == 3 && KW == 3 && pad_y == 0 && pad_x == 0) {
        // all nine taps in one launch: the pipelined 16 x 6 form for g grids of 64^2 and up, where it measured
        // 1-14 % faster, the 16 x 8 wgrad3x3_s2_kernel below them, where the pipelined form was 6-7 % slower
        // (tools/wgrad_s2p_ab.py, profiles/r05_wgrad_s2p_ab.txt); SG2_WGRAD_S2P=1 / 0 forces either
        const char* ep = getenv("SG2_WGRAD_S2P");     // read per call: tests switch it in one process
        const bool pipe = ep ? atoi(ep) != 0 : (OH >= 64 && OW >= 64);
        a.tiles_x = (int)cdiv(OW, 16);
        a.tiles_y = (int)cdiv(OH, pipe ? 6 : 8);
        a.tiles = N * a.tiles_x * a.tiles_y;
        const int cb = (int)(cdiv(A, BC) * cdiv(B, BC));
        int splits = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(wgrad_wgs(), cb), a.tiles / 4));
        a.tiles_per_block = (int)cdiv(a.tiles, splits);
        splits = (int)cdiv(a.tiles, a.tiles_per_block);
        dim3 grid((unsigned)cdiv(A, BC), (unsigned)cdiv(B, BC), (unsigned)splits);
        if (int rc = w3_det_slots(a, arena, (int)grid.z, s)) return rc;
        static const bool swz = [] { const char* e = getenv("SG2_WGRAD_SWZ"); return e != nullptr && e[0] == '1'; }();
        if (pipe) {
            if (dtype == SG2_F16) launch_w3p<f16_t>(a, grid, s);
            else launch_w3p<bf16_t>(a, grid, s);
        } else if (dtype == SG2_F16) {
            if (swz) wgrad3x3_s2_kernel<f16_t, true><<<grid, 256, 0, s>>>(a);
            else wgrad3x3_s2_kernel<f16_t, false><<<grid, 256, 0, s>>>(a);
        } else {
            if (swz) wgrad3x3_s2_kernel<bf16_t, true><<<grid, 256, 0, s>>>(a);
            else wgrad3x3_s2_kernel<bf16_t, false><<<grid, 256, 0, s>>>(a);
        }
        return launch_status("sg2_conv2d_wgrad (halo, stride 2)");
    }
    const int TW = OW >= 32 ? 32 : 16;
    a.tiles_x = (int)cdiv(OW, TW);
    a.tiles_y = (int)cdiv(OH, 256 / TW);
    a.tiles = N * a.tiles_x * a.tiles_y;
    const int cb = (int)(cdiv(A, BC) * cdiv(B, BC));
    // ~512 workgroups per launch, at least 4 tiles each
    int splits = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(wgrad_wgs(), cb), a.tiles / 4));
    a.tiles_per_block = (int)cdiv(a.tiles, splits);
    splits = (int)cdiv(a.tiles, a.tiles_per_block);
    dim3 grid((unsigned)cdiv(A, BC), (unsigned)cdiv(B, BC), (unsigned)splits);
    // stride 1 with every tap in one phase: the LDS-DMA kernel (SG2_WGRAD_DMA=0 keeps the register-staged one)
    // With a modulation scale every workgroup's tile range must lie inside one sample: tiles_per_block a divisor
    // of the tiles per sample (at most doubling the workgroups), else the register-staged kernel runs.
    static const int dma_on = [] { const char* e = getenv("SG2_WGRAD_DMA"); return e ? atoi(e) : 1; }();
    const bool scaled = gscale || xscale;
    const int per_n = a.tiles_x * a.tiles_y;
    bool sc_ok = !scaled;
    if (scaled && dma_on) {
        int tpb = std::min(a.tiles_per_block, per_n);
        while (tpb > 1 && per_n % tpb) --tpb;
        if (tpb * 2 >= a.tiles_per_block && tpb >= 4) {
            a.tiles_per_block = tpb;
            grid.z = (unsigned)cdiv(a.tiles, tpb);
            sc_ok = true;
        }
    }
    if (dma_on && sc_ok && stride == 1 && ((KH == 3 && pad_y == 1 && pad_x == 1) || (KH == 1 && pad_y == 0 && pad_x == 0))) {
        for (int ky = 0; ky < KH; ++ky)
            for (int kx = 0; kx < KW; ++kx)
                a.taps[ky * KW + kx] = PTap{(int8_t)(ky - pad_y), (int8_t)(kx - pad_x), (int8_t)(ky * KW + kx), 0};
        a.PY = 0; a.PX = 0;
        if (int rc = w3_det_slots(a, arena, (int)grid.z, s)) return rc;
        const int sel = ((gscale || xscale) ? 1 : 0) | (KH == 3 ? 2 : 0) | (TW == 32 ? 4 : 0) | (dtype == SG2_F16 ? 8 : 0);
        switch (sel) {
#define SG2_WDMA_2(B_, T_, TW_, NT_)                                   \
            case B_: launch_wdma<T_, TW_, NT_, false>(a, grid, s); break; \
            case B_ + 1: launch_wdma<T_, TW_, NT_, true>(a, grid, s); break;
            SG2_WDMA_2(0, bf16_t, 16, 1)
            SG2_WDMA_2(2, bf16_t, 16, 9)
            SG2_WDMA_2(4, bf16_t, 32, 1)
            SG2_WDMA_2(6, bf16_t, 32, 9)
            SG2_WDMA_2(8, f16_t, 16, 1)
            SG2_WDMA_2(10, f16_t, 16, 9)
            SG2_WDMA_2(12, f16_t, 32, 1)
            SG2_WDMA_2(14, f16_t, 32, 9)
#undef SG2_WDMA_2
        }
        return launch_status("sg2_conv2d_wgrad (halo, LDS-DMA)");
    }
    if (int rc = w3_det_slots(a, arena, (int)grid.z, s, stride > 1)) return rc;
    for (int py = 0; py < stride; ++py)
        for (int px = 0; px < stride; ++px) {
            int nt = 0;
            for (int ky = 0; ky < KH; ++ky) {
                const int ry = ky - pad_y;
                if (((ry % stride) + stride) % stride != py) continue;
                for (int kx = 0; kx < KW; ++kx) {
                    const int rx = kx - pad_x;
                    if (((rx % stride) + stride) % stride != px) continue;
                    a.taps[nt++] = PTap{(int8_t)floordiv_w(ry, stride), (int8_t)floordiv_w(rx, stride),
                                        (int8_t)(ky * KW + kx), 0};
                }
            }
            if (nt == 0) continue;
            a.PY = py; a.PX = px;
            int rc;
            if (dtype == SG2_F16) rc = TW == 32 ? dispatch_nt<f16_t, 32>(a, grid, nt, s) : dispatch_nt<f16_t, 16>(a, grid, nt, s);
            else rc = TW == 32 ? dispatch_nt<bf16_t, 32>(a, grid, nt, s) : dispatch_nt<bf16_t, 16>(a, grid, nt, s);
            if (rc) return rc;
            rc = launch_status("sg2_conv2d_wgrad (halo)");
            if (rc) return rc;
        }
    return 0;
}
}  // namespace

}  // namespace sg2
