// Memory-path microbenchmarks for the 256^2 x 64-channel layer's traffic (tools/membench.py): what the chip does
// with the ring kernel's access patterns, without its math.  Not part of the product library.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}

// (1) plain streaming copy, 16 B a lane, whole lines: the HBM read+write baseline
extern "C" __global__ void __launch_bounds__(256) k_copy(const u32x4* __restrict__ x, u32x4* __restrict__ y, int n16) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) y[i] = x[i];
}

// (2) stores only, the ring kernel's epilogue shape: lane (l16, q) of wave w writes 16 B at pixel l16 of a
// 16-pixel fragment, channel bytes (h * 32 + q * 8) * 2 -- 64-byte half lines; h = wave & 1
extern "C" __global__ void __launch_bounds__(512) k_store_half(u32x4* y, int npix) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = wave & 1, wr = wave >> 1;
    const __amdgpu_buffer_rsrc_t r = rsrc(y, npix * 128);
    const u32x4 v = {1u, 2u, 3u, 4u};
    for (int t = blockIdx.x; t * 256 < npix; t += gridDim.x) {
        for (int i = 0; i < 4; ++i) {
            const int pix = t * 256 + (wr * 2 + (i >> 1)) * 32 + (i & 1) * 16 + (lane & 15);
            __builtin_amdgcn_raw_buffer_store_b128(v, r, (pix * 64 + h * 32 + (lane >> 4) * 8) * 2, 0, 0);
        }
    }
}

// (3) stores only, whole lines: lane (p8, q8) writes 16 B of pixel p8's 128-B line
extern "C" __global__ void __launch_bounds__(512) k_store_full(u32x4* y, int npix) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const __amdgpu_buffer_rsrc_t r = rsrc(y, npix * 128);
    const u32x4 v = {1u, 2u, 3u, 4u};
    for (int t = blockIdx.x; t * 256 < npix; t += gridDim.x) {
        for (int i = 0; i < 4; ++i) {
            const int pix = t * 256 + wave * 32 + i * 8 + (lane >> 3);
            __builtin_amdgcn_raw_buffer_store_b128(v, r, (pix * 64 + (lane & 7) * 8) * 2, 0, 0);
        }
    }
}

// (4) the ring's halo stream alone: 32 x 8 tiles, 10 x 40-position halos by LDS-DMA into a 3-slot ring, two tiles
// in flight, one barrier per tile, wave w issuing 7 wave-instructions a tile -- no math, no stores.  kill_pad: the
// pad positions (columns 34 .. 39) read nothing (out of range) instead of the pixels that follow.
template <bool KILL_PAD, int NSLOT>
__global__ void __launch_bounds__(512) k_halo(const void* x, int N, int H, int W, int tiles_total, float* sink) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int t_begin = (int)((int64_t)blockIdx.x * tiles_total / gridDim.x);
    const int t_end = (int)((int64_t)(blockIdx.x + 1) * tiles_total / gridDim.x);
    const __amdgpu_buffer_rsrc_t r = rsrc(x, N * H * W * 128);
    const int lx = lane >> 3, hlane = lx * 128 + (((lane & 7) ^ (((lx >> 1) & 3) << 1)) * 16);
    const int tiles_x = W / 32, per_n = tiles_x * (H / 8);
    auto issue = [&](int t, int slot) {
        const int n = t / per_n, rr = t - n * per_n, ty = (rr / tiles_x) * 8, tx = (rr % tiles_x) * 32;
#pragma unroll
        for (int u = 0; u < 7; ++u) {
            const int i = u * 8 + wave;
            if (i < 50) {
                const int hy = i / 5, cg = i - hy * 5, iy = ty - 1 + hy, ix0 = tx - 1 + cg * 8;
                const int base = (unsigned)iy < (unsigned)H ? ((n * H + iy) * W + ix0) * 128 : -(1 << 30);
                const bool kill = ((tx == 0) & (cg == 0) & (lx == 0)) | ((tx + 32 == W) & (cg == 4) & (lx == 1)) |
                                  (KILL_PAD & (cg == 4) & (lx >= 2));
                __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(smem + slot * 51200 + i * 1024), 16,
                                                         kill ? -1 : base + hlane, 0, 0, 0);
            }
        }
    };
    issue(t_begin, 0);
    if (NSLOT > 2) issue(min(t_begin + 1, t_end - 1), 1);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_s_barrier();
    float acc = 0.f;
    int k = 0;
    for (int t = t_begin; t < t_end; ++t, ++k) {
        issue(min(t + NSLOT - 1, t_end - 1), (k + NSLOT - 1) % NSLOT);
        acc += *(const float*)(smem + (k % NSLOT) * 51200 + threadIdx.x * 16);
        if (NSLOT > 2) __builtin_amdgcn_s_waitcnt(0x3f70 | 7);   // vmcnt(7): the newest tile's DMAs stay in flight
        else __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_s_barrier();
    }
    __builtin_amdgcn_s_waitcnt(0);
    if (acc == 12345.f) sink[0] = acc;
}

extern "C" int run_halo(int kill_pad, int nslot, const void* x, int N, int H, int W, float* sink, int grid, hipStream_t s) {
    const int tiles = N * (H / 8) * (W / 32);
    const size_t lds = nslot * 51200;
    if (kill_pad && nslot == 3) {
        hipFuncSetAttribute((const void*)k_halo<true, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        k_halo<true, 3><<<grid, 512, lds, s>>>(x, N, H, W, tiles, sink);
    } else if (nslot == 3) {
        hipFuncSetAttribute((const void*)k_halo<false, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        k_halo<false, 3><<<grid, 512, lds, s>>>(x, N, H, W, tiles, sink);
    } else {
        hipFuncSetAttribute((const void*)k_halo<true, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        k_halo<true, 2><<<grid, 512, lds, s>>>(x, N, H, W, tiles, sink);
    }
    return (int)hipGetLastError();
}
extern "C" int run_copy(const void* x, void* y, int n16, int grid, hipStream_t s) {
    k_copy<<<grid, 256, 0, s>>>((const u32x4*)x, (u32x4*)y, n16);
    return (int)hipGetLastError();
}
extern "C" int run_store(int full, void* y, int npix, int grid, hipStream_t s) {
    if (full) k_store_full<<<grid, 512, 0, s>>>((u32x4*)y, npix);
    else k_store_half<<<grid, 512, 0, s>>>((u32x4*)y, npix);
    return (int)hipGetLastError();
}
