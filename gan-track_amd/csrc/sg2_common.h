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
bool det_on();
// In deterministic mode every accumulator output that zero_acc clears is written by exactly one fixed-order slot sum
// of the same entry call, which then assigns (det_assign) instead of adding into zeros: no fill launch (a 4.6 us
// launch each, 45 per training step, profiles/r06bj_zero_fill_sites.txt).  A caller's pre-zeroed buffer
// (sg2_set_zeroed_accumulators: possibly accumulating several calls) is added into as before.
bool det_assign_on();   // SG2_DET_ASSIGN=0: the former fill + add (an A/B switch)
inline hipError_t zero_acc(void* p, size_t bytes, hipStream_t s) {
    return (accumulators_prezeroed() || (det_on() && det_assign_on())) ? hipSuccess : zero_fill(p, bytes, s);
}
inline int det_assign() { return (accumulators_prezeroed() || !det_assign_on()) ? 0 : 1; }

// Deterministic mode (sg2_set_deterministic, process-wide).  Every float accumulation that the fast path
// makes with atomics (split-K partial sums, weight-gradient pixel splits, per-channel dot / bias / demod
// reductions, the grid-sample scatter) is made instead by writing each contribution to a slot of the registered
// scratch and summing the slots in a fixed order (det_sum): results are bitwise reproducible run to run.
// Within a workgroup, LDS float atomics are replaced by per-thread partials summed in thread order.
bool det_on();
// A per-call bump allocator over the registered scratch (floats).  get() returns nullptr (and sets the error)
// when the scratch is exhausted; entry points then return -1.
class DetArena {
 public:
    DetArena();
    float* get(int64_t n_floats);
 private:
    float* base_;
    int64_t cap_, off_;
};
// out[g * go + i] += sum_{s < S} ws[g * gw + s * ss + i] for g < G (<= 65535), i < n: a fixed-order sum (four
// interleaved row sums over s, s = r mod 4 in increasing s, added in row order; at S <= 16 over many outputs, s in
// increasing order four outputs a lane; det.hip), one launch, or two (a chunk pass into `arena`) for few outputs
// over many slots.
hipError_t det_sum(float* out, int64_t go, const float* ws, int64_t gw, int64_t ss, int G, int64_t S, int64_t n,
                   DetArena& arena, hipStream_t st, int assign = 0);   // assign: out = instead of out +=
// Up to four independent det_sum calls in (at most) two launches: the chunk passes of those that need one
// together, then the final sums together; each job's order is det_sum's.
struct DetSumJob {
    float* out;
    int64_t go;
    const float* ws;
    int64_t gw, ss;
    int G;
    int64_t S, n;
    int assign;     // out = instead of out +=
};
hipError_t det_sum_multi(const DetSumJob* jobs, int count, DetArena& arena, hipStream_t st);
// out[a][b][t] (swap: out[b][a][t]) += sum_{s < S} ws[s][a][t][b] (t < KK, B % 4 == 0): a weight gradient's slots
// into torch's [O, I, kh, kw] layout (sg2_conv2d_wgrad_oikk).
hipError_t det_sum_oikk(float* out, const float* ws, int64_t S, int A, int KK, int B, int swap, hipStream_t st,
                        int assign = 0);
#define SG2_DET_GET(ptr, arena, n, what)                                                        \
    do {                                                                                       \
        (ptr) = (arena).get(n);                                                                \
        if (!(ptr)) {                                                                          \
            ::sg2::set_error(std::string(what) + ": deterministic scratch too small");        \
            return -1;                                                                         \
        }                                                                                      \
    } while (0)

// Deterministic replacement of a workgroup's LDS float atomics `red[c0 + j] += v[j]` by threads laid out as
// (row, c0): each thread stores its 8 partials in its row of part[rows][C]; after a barrier, det_rows_sum(i)
// adds channel i over the rows in row order.
__device__ __forceinline__ void det_rows_store(float* part, int C, int row, int c0, const float* v) {
#pragma unroll
    for (int j = 0; j < 8; ++j) part[row * C + c0 + j] = v[j];
}
__device__ __forceinline__ float det_rows_sum(const float* part, int C, int rows, int i) {
    float s = 0.f;
    for (int r = 0; r < rows; ++r) s += part[r * C + i];
    return s;
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
