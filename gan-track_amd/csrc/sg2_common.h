// Shared helpers for the sg2hip kernels (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/sg2hip.h"

typedef _Float16 f16_t;
typedef __bf16 bf16_t;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef bf16_t bf16x8 __attribute__((ext_vector_type(8)));
typedef f16_t f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

namespace sg2 {

// Per-host-thread error message (sg2_last_error).
void set_error(const std::string& msg);

#define SG2_CHECK(cond, msg)                     \
    do {                                         \
        if (!(cond)) {                           \
            ::sg2::set_error(std::string(msg));  \
            return -1;                           \
        }                                        \
    } while (0)

// Zeroing of an entry point's float accumulator outputs (dot_out, dw, db / dd).  While the host thread has
// sg2_set_zeroed_accumulators(1) in effect the caller has zeroed them itself (one fill for all of a layer's
// accumulators instead of a memset per call), and this is a no-op.
bool accumulators_prezeroed();
// sg2_set_clean_workspace(1): the split-K workspace passed to the conv entry points is zero on entry, and the
// call leaves it zero (its finalize clears what it read) -- no memset per split-K call.
bool workspace_clean();
// Zero `bytes` bytes at p on stream s with a kernel.  Not hipMemsetAsync: the library's memsets captured into
// a phase graph (accumulators allocated inside the capture, memsets issued from the backward) took effect on
// the first replay only, so every later replay added into the previous one's sums (tools/greg_replay_check.py:
// second replay inf / NaN, 7e-7 with this kernel).  A stand-alone memset node replays correctly
// (tools/memset_graph_check.py); kernel nodes replay every time.
hipError_t zero_fill(void* p, size_t bytes, hipStream_t s);
inline hipError_t zero_acc(void* p, size_t bytes, hipStream_t s) {
    return accumulators_prezeroed() ? hipSuccess : zero_fill(p, bytes, s);
}

inline int launch_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error(std::string(what) + ": " + hipGetErrorString(e));
        return (int)e;
    }
    return 0;
}

// Raw buffer loads (stride 0, num_records = the tensor's bytes, < 2 GB): an offset past the end (-1 as
// unsigned) returns zeros, which replaces the bounds select after a conditional load.  gfx9 dword3.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0,
                                             (int)(bytes < 0x7fffffffLL ? bytes : 0x7fffffffLL), 0x00020000);
}
template <typename vecT>
__device__ __forceinline__ vecT buf_load16(__amdgpu_buffer_rsrc_t r, int byte_off) {
    return __builtin_bit_cast(vecT, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}

template <typename T>
__device__ __forceinline__ T buf_load2(__amdgpu_buffer_rsrc_t r, int byte_off) {   // one 16-bit element
    return __builtin_bit_cast(T, (unsigned short)__builtin_amdgcn_raw_buffer_load_b16(r, byte_off, 0, 0));
}
__device__ __forceinline__ float buf_load4f(__amdgpu_buffer_rsrc_t r, int byte_off) {   // one f32
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
}
template <typename vecT>
__device__ __forceinline__ vecT buf_load8(__amdgpu_buffer_rsrc_t r, int byte_off) {   // 8 bytes
    return __builtin_bit_cast(vecT, __builtin_amdgcn_raw_buffer_load_b64(r, byte_off, 0, 0));
}

template <typename T> __device__ __forceinline__ float to_f32(T v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f32(float v) { return (T)v; }

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace sg2

// Dispatch on the runtime dtype code.
#define SG2_DISPATCH(dtype, T, ...)                                  \
    switch (dtype) {                                                 \
        case SG2_F32: { typedef float T; __VA_ARGS__; break; }       \
        case SG2_F16: { typedef f16_t T; __VA_ARGS__; break; }       \
        case SG2_BF16: { typedef bf16_t T; __VA_ARGS__; break; }     \
        default: ::sg2::set_error("unsupported dtype"); return -1;   \
    }
