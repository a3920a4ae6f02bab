/*
 * sg2hip -- C-ABI of the MI355X (gfx950) kernels of the StyleGAN2-ADA training hot path.
 *
 * The library (libsg2hip.so, built from gan-track_amd/csrc) replaces the reference's two
 * pybind11 CUDA plugins and the cuDNN convolutions reached through conv2d_gradfix:
 *
 *   reference (ltronchin/Gan-track, src/models/stylegan3 = SG3/)          replaced by
 *   SG3/torch_utils/ops/bias_act.cpp:32   bias_act(x,b,xref,yref,dy,grad,dim,act,alpha,gain,clamp)
 *                                                                          -> sg2_bias_act
 *   SG3/torch_utils/ops/upfirdn2d.cpp:16  upfirdn2d(x,f,upx,upy,downx,downy,padx0,padx1,pady0,pady1,flip,gain)
 *                                                                          -> sg2_upfirdn2d
 *   SG3/torch_utils/ops/conv2d_gradfix.py:37-45 (F.conv2d / F.conv_transpose2d, cuDNN)
 *                                                                          -> sg2_conv2d (fwd + dgrad)
 *   autograd weight gradient of those convolutions (cuDNN wgrad)          -> sg2_conv2d_wgrad
 *   SG3/torch_utils/ops/grid_sample_gradfix.py:28-65 (aten grid_sampler_2d fwd/bwd)
 *                                                                          -> sg2_grid_sample_fwd / _bwd
 *   SG3/training/networks_stylegan2.py:59-63 demodulation coefficients    -> sg2_demod_fwd / _bwd
 *   SG3/training/training_loop_mi_multimodal.py:341-351 (flat grad, /N, nan_to_num, torch.optim.Adam)
 *                                                                          -> sg2_adam_multi
 *   SG3/training/training_loop_mi_multimodal.py:358-366 (G_ema lerp)      -> sg2_lerp_multi
 *
 * Conventions
 *  - Every pointer is a device pointer; the library never allocates or frees device memory.
 *  - Mutable state: three mode switches, set between launches and read by every later launch --
 *      sg2_set_deterministic (PROCESS-WIDE: the caller's scratch arena for fixed-order slot reductions; process-
 *        wide because autograd runs a deterministic scope's backward on its own device thread),
 *      sg2_set_zeroed_accumulators, sg2_set_clean_workspace (PER HOST THREAD),
 *    plus the per-thread sg2_last_error() message.  Otherwise the kernels are re-entrant and capturable into a
 *    hipGraph; do not change the process-wide deterministic arena while another thread is launching.
 *  - `stream` is a hipStream_t (pass the caller's current stream; NULL = default stream).
 *  - dtype codes: SG2_F32 = 0, SG2_F16 = 1, SG2_BF16 = 2 (arithmetic is always f32 internally).
 *  - 4-D activations are NHWC in memory (torch channels_last); sizes are given as [N, C, H, W]
 *    like the reference, strides (in elements) as [sN, sC, sH, sW] where a function accepts strides.
 *  - Return value: 0 = success, < 0 = invalid argument (see sg2_last_error()), > 0 = hipError_t of
 *    the launch.  The Python wrapper raises RuntimeError with sg2_last_error() -- the same behaviour
 *    as the reference's TORCH_CHECK / AT_CUDA_CHECK.
 */
#ifndef SG2HIP_H
#define SG2HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SG2_ABI_VERSION 9

enum sg2_dtype { SG2_F32 = 0, SG2_F16 = 1, SG2_BF16 = 2, SG2_F32S3 = 3 };

/* SG2_F32S3 (ABI 5): float32 operands handed over PRE-SPLIT as three bf16 planes h, m, l (x = h + m + l, exact
 * for normal floats; sg2_split3), each plane the tensor's element order, the planes back to back.  Accepted as
 * the operand dtype of sg2_conv2d / sg2_conv2d_fused (x and w; the output, epilogue and workspace are float32;
 * Cin % 8 == 0; in_scale must be folded into x's planes) and of sg2_conv2d_wgrad (g and x; A, B % 8 == 0;
 * scales folded in).  The f32 convolutions then run the split form's six bf16 MFMA products on operands split
 * once per call instead of once per workgroup that stages them.
 *
 * planes[p * n + i] = piece p of x[i] * scale[(i / C) / pix_per_n, i % C]   (scale NULL = 1; x f32, n elements,
 * C % 8 == 0, 16-byte aligned) */
int sg2_split3(void* planes, const float* x, int64_t n, int C, int64_t pix_per_n, const float* scale, void* stream);

/* ABI version of the loaded library (SG2_ABI_VERSION). */
int sg2_abi_version(void);

/* Message of the last failing call on this host thread ("" if none). */
const char* sg2_last_error(void);

/* Fused bias + activation + gain + clamp, and its 1st/2nd order gradients.
 * Replaces SG3/torch_utils/ops/bias_act.cpp:32 (kernel semantics bias_act.cu:23-147).
 *   y[i] = f(x[i], b[(i / step_b) % size_b], ...) for i < numel.
 *   grad = 0: y = clamp(act(x + b) * gain)
 *   grad = 1: y = x * act'(...) * gain masked by |yref| < clamp     (x holds dL/dy)
 *   grad = 2: second-order term (needs dy, the first-order incoming gradient)
 * b / xref / yref / dy may be NULL (absent, like the reference's empty tensor).
 * act: 1 linear, 2 relu, 3 lrelu, 4 tanh, 5 sigmoid, 6 elu, 7 selu, 8 softplus, 9 swish
 * (the reference's cuda_idx, bias_act.py:21-31).  clamp < 0 disables clamping. */
int sg2_bias_act(void* y, const void* x, const void* b, const void* xref, const void* yref, const void* dy,
                 int dtype, int64_t numel, int64_t size_b, int64_t step_b, int grad, int act, float alpha,
                 float gain, float clamp, void* stream);

/* Upsample (zero insertion), pad/crop, 2-D FIR, downsample.
 * Replaces SG3/torch_utils/ops/upfirdn2d.cpp:16 (semantics upfirdn2d.py:118-211).
 *   in/out sizes [N, C, H, W], strides in elements (any layout); f is a float32 [fh, fw] filter
 *   (row-major, device).  flip = 0: true convolution (filter flipped), 1: correlation.
 *   Output size must equal ((in*up + pad0 + pad1 - f) / down) + 1 per axis. */
int sg2_upfirdn2d(void* y, const void* x, const float* f, int dtype, const int64_t* in_size,
                  const int64_t* in_stride, const int64_t* out_size, const int64_t* out_stride, int fw, int fh,
                  int upx, int upy, int downx, int downy, int padx0, int padx1, int pady0, int pady1, int flip,
                  float gain, void* stream);

/* sg2_upfirdn2d of a dynamically sized image held at the origin of a static buffer (the ADA pipe's padded
 * image, augment_mi.py:288-321, whose size is data dependent): lim = device int[2] output extent (rows,
 * cols).  Outputs inside it are computed, outputs within 32 rows / cols beyond it are written as zeros
 * (exact when the image's support ends inside the extent), the rest of y is left unwritten.  Generic
 * (any-stride) kernel. */
int sg2_upfirdn2d_lim(void* y, const void* x, const float* f, int dtype, const int64_t* in_size,
                      const int64_t* in_stride, const int64_t* out_size, const int64_t* out_stride, int fw, int fh,
                      int upx, int upy, int downx, int downy, int padx0, int padx1, int pady0, int pady1, int flip,
                      float gain, const int* lim, void* stream);

/* sg2_upfirdn2d followed by the fused layer epilogue (sg2_epilogue, defined below) -- the FIR of
 * an up-2 synthesis layer with its demodulation, noise, bias, lrelu and clamp
 * (networks_stylegan2.py:68-76 + :325-327).  epi may be NULL; with an epilogue the activations
 * must be NHWC with C % 8 == 0 (C % 4 for f32). */
typedef struct sg2_epilogue sg2_epilogue;
int sg2_upfirdn2d_fused(void* y, const void* x, const float* f, int dtype, const int64_t* in_size,
                        const int64_t* in_stride, const int64_t* out_size, const int64_t* out_stride, int fw, int fh,
                        int upx, int upy, int downx, int downy, int padx0, int padx1, int pady0, int pady1, int flip,
                        float gain, const sg2_epilogue* epi, void* stream);

/* Dense 2-D convolution on NHWC activations (implicit GEMM on MFMA).
 *   transpose = 0: y = conv2d(x, w, stride, padding)            (torch.nn.functional.conv2d)
 *                  w packed [Cout][KH][KW][Cin]  (= OIHW weight in channels_last memory)
 *   transpose = 1: y = conv_transpose2d(x, w, stride, padding)  (torch.nn.functional.conv_transpose2d)
 *                  w packed [Cout][KH][KW][Cin]  (= the [Cin, Cout, KH, KW] torch weight permuted (1,2,3,0))
 *   x [N, H, W, Cin], y [N, OH, OW, Cout] (OH/OW explicit: output_padding is implied).
 *   workspace: float32 scratch of >= N*OH*OW*Cout elements, or NULL (then no split-K is used). */
int sg2_conv2d(void* y, const void* x, const void* w, int dtype, int N, int Cin, int H, int W, int Cout,
               int OH, int OW, int KH, int KW, int stride, int pad_y, int pad_x, int transpose,
               float* workspace, int64_t workspace_elems, void* stream);

/* Fused epilogue of sg2_conv2d_fused (all pointers optional):
 *   z   = clamp(act(c * out_scale[n,o] + noise[n,oy,ox] * noise_gain + bias[o]) * gain, +-clamp)
 *   y   = round(z) + residual[n,oy,ox,o]          (residual: the resnet skip of the D block)
 *   aux = c (aux_mode 1) or z (aux_mode 2)        (saved for the fused backward)
 *   dot_out[n,o] = sum_{oy,ox} c * dot_src        (the modulation gradient when the call is a dgrad)
 * Replaces the fma / bias_act / add passes the reference runs after each conv
 * (networks_stylegan2.py:68-76, :172-181, :621-627). */
struct sg2_epilogue {
    const float* out_scale;  /* [N, Cout] float32 */
    const void* noise;       /* [N, OH, OW], activation dtype */
    const float* bias;       /* [Cout] float32, added rounded to the activation dtype (the reference's b.to(x.dtype)) */
    const void* residual;    /* [N, OH, OW, Cout] NHWC, activation dtype */
    void* aux;               /* [N, OH, OW, Cout] NHWC, activation dtype */
    float noise_gain, alpha, gain, clamp;   /* clamp < 0: off */
    int act;                 /* 0 linear, 1 lrelu(alpha) */
    int aux_mode;            /* 0 none, 1 conv result c, 2 activation z */
    const void* dot_src;     /* [N, OH, OW, Cout] or NULL (sg2_conv2d_fused only; needs aux_mode 0 or 1) */
    float* dot_out;          /* [N, Cout] float32: sum over pixels of c * dot_src, zeroed by the call */
};

/* sg2_conv2d with the A operand modulated by in_scale[n, ci] (float32 [N, Cin], or NULL) and the
 * fused epilogue above (epi may be NULL = plain convolution).  Transposed convolutions run all their
 * stride x stride output phases in one launch (up to 4 phases per launch). */
int sg2_conv2d_fused(void* y, const void* x, const void* w, int dtype, int N, int Cin, int H, int W, int Cout,
                     int OH, int OW, int KH, int KW, int stride, int pad_y, int pad_x, int transpose,
                     const float* in_scale, const sg2_epilogue* epi, float* workspace, int64_t workspace_elems,
                     void* stream);

/* 3x3 / stride 1 / pad 1 convolution of 16-bit NHWC activations with an LDS halo tile, optional
 * modulation of the input and the fused StyleGAN2 layer epilogue (networks_stylegan2.py:309-328):
 *   c      = conv(x[n,:,:,ci] * in_scale[n,ci], w)          w packed [Cout][3][3][Cin], Cin % 8 == 0
 *   y_raw  = c                                              (optional second output, may be NULL)
 *   y      = clamp(act(c * out_scale[n,o] + noise[n,y,x] * noise_gain + bias[o]) * gain, +-clamp)
 * in_scale / out_scale / bias are float32 (NULL = off); noise has the activation dtype, [N,H,W]
 * (NULL = off); act 0 = linear, 1 = lrelu(alpha); clamp < 0 = off.  dtype: SG2_F16 or SG2_BF16.
 * dot_src / dot_out (both or neither): dot_out[n,o] = sum_{y,x} c[n,y,x,o] * dot_src[n,y,x,o] (float,
 * zeroed by the call) -- the modulation gradient of the layer when this kernel runs its dgrad. */
int sg2_conv3x3(void* y, void* y_raw, const void* x, const void* w, int dtype, int N, int Cin, int H, int W,
                int Cout, const float* in_scale, const float* out_scale, const void* noise, float noise_gain,
                const float* bias, int act, float alpha, float gain, float clamp, const void* dot_src,
                float* dot_out, void* stream);

/* While on (per host thread), the entry points below skip zeroing their float accumulator outputs --
 * sg2_conv2d_fused / sg2_conv3x3 / sg2_conv3x3_s2 dot_out, sg2_conv2d_wgrad dw, sg2_layer_bwd db / dd --
 * because the caller zeroed them (one fill for all of a layer's accumulators instead of one memset per
 * call).  Default off. */
void sg2_set_zeroed_accumulators(int on);

/* While on (per host thread), the split-K f32 workspace passed to sg2_conv2d / sg2_conv2d_fused is zero on
 * entry and is left zero on return (the finalize pass clears what it read), so a split-K call issues no
 * memset.  The caller keeps one persistent zeroed workspace per stream.  Default off. */
void sg2_set_clean_workspace(int on);

/* Deterministic mode (process-wide, so that autograd's backward threads see it; scratch NULL = off, the
 * default).  While a device scratch buffer is
 * registered, every float accumulation the entry points otherwise make with atomics -- split-K partial sums,
 * weight-gradient pixel splits, dot_out / db / dd reductions, the grid-sample input-gradient scatter -- is made
 * by writing each contribution to a slot of the scratch and summing the slots in a fixed order, so results
 * are bitwise reproducible.  Calls made while it is on must be stream-ordered (they share the scratch); a call
 * whose partial sums do not fit returns -1 ("deterministic scratch too small").  The explicit-grid
 * sg2_grid_sample_bwd keeps its atomics (only the affine form has the gather used here).  Since round 6 this is
 * the training iteration's default arithmetic (Trainer(deterministic=True) registers a 2 GiB scratch around every
 * phase's forward and backward): the slot reductions (per-tile dot slots, split sums folded into the split-K
 * finalize, one-launch det_sum) measured faster than the float atomics on the bench step. */
void sg2_set_deterministic(void* scratch, int64_t bytes);

/* Stride-2 / pad-0 form of sg2_conv3x3 (conv2d_resample.py:139-142 with down = 2: the discriminator's
 * down-2 3x3 layers after their FIR pre-filter, and the input gradient of the up-2 synthesis layers):
 * x [N, H, W, Cin] -> y [N, (H-3)/2+1, (W-3)/2+1, Cout]; same epilogue and dot as sg2_conv3x3, plus
 *   residual  [N, OH, OW, Cout] (dtype, NULL = off): y = round(epilogue) + residual, rounded
 *             (the resnet add of DiscriminatorBlock, networks_stylegan2.py:621-627)
 *   raw_act   1: y_raw receives the epilogue value before the residual add (the activation gradient's
 *             input) instead of the raw conv. */
int sg2_conv3x3_s2(void* y, void* y_raw, const void* x, const void* w, int dtype, int N, int Cin, int H, int W,
                   int Cout, const float* in_scale, const float* out_scale, const void* noise, float noise_gain,
                   const float* bias, int act, float alpha, float gain, float clamp, const void* residual,
                   int raw_act, const void* dot_src, float* dot_out, void* stream);

/* Stride-2 transposed 3x3 convolution, padding 0, 16-bit (conv2d_resample.py:112-129, the up-2 plan's
 * conv_transpose2d; also the input gradient of a stride-2 3x3 convolution):
 *   y[n, 2i+ky, 2j+kx, o] = sum_{c, (i,j) -> (2i+ky, 2j+kx)} x[n, i, j, c] (* s[n, c]) w[o][ky][kx][c]
 * x [N, H, W, Cin] NHWC, y [N, 2H+1, 2W+1, Cout] NHWC (overwritten), w packed [Cout][3][3][Cin] (the
 * conv_transpose2d weight [Cin, Cout, 3, 3] read as [Cout][Cin] without a tap flip), in_scale [N, Cin] f32
 * or NULL (the modulation x * s rounded as the reference's x * s.to(x.dtype)).  Cin % 32 == 0, Cout % 8 == 0. */
int sg2_conv3x3_up2(void* y, const void* x, const void* w, int dtype, int N, int Cin, int H, int W, int Cout,
                    const float* in_scale, void* stream);

/* Weight gradient of sg2_conv2d (transpose = 0 form):
 *   dw[a][ky][kx][b] = sum_{n,oy,ox} g[n,oy,ox,a] * u[n,a] * x[n, oy*stride+ky-pad_y, ox*stride+kx-pad_x, b] * s[n,b]
 *   u = g_scale [N, A], s = x_scale [N, B] float32 (a layer's modulation), or NULL for 1.
 *   g [N, OH, OW, A] NHWC, x [N, H, W, B] NHWC; dw is float32 [A][KH][KW][B], overwritten.
 *   The conv_transpose2d weight gradient is the same call with (g, x) = (x_of_convT, dy).
 *   alpha scales the result (dw = alpha * sum ...): a layer's weight gain, the backward of the reference's
 *   `self.weight * self.weight_gain` (networks_stylegan2.py:173) folded in (ABI 3). */
int sg2_conv2d_wgrad(float* dw, const void* g, const void* x, int dtype, int N, int A, int OH, int OW, int B,
                     int H, int W, int KH, int KW, int stride, int pad_y, int pad_x, const float* g_scale,
                     const float* x_scale, float alpha, void* stream);

/* sg2_conv2d_wgrad with dw written as float32 [A][B][KH][KW] -- torch's [O, I, kh, kw] parameter layout, so the
 * gradient reaches the parameter without a layout copy -- or, swap_ab != 0, as [B][A][KH][KW] (a transposed
 * convolution's weight, whose gradient is the call with g and x exchanged) (ABI 9).  SG2_F32S3 operands (the f32
 * layers) in deterministic mode only, B % 4 == 0, KH * KW <= 9: its fixed-order slot sum writes the transposed
 * layout. */
int sg2_conv2d_wgrad_oikk(float* dw, const void* g, const void* x, int dtype, int N, int A, int OH, int OW, int B,
                          int H, int W, int KH, int KW, int stride, int pad_y, int pad_x, float alpha, int swap_ab,
                          void* stream);

/* Fused first-order backward of the layer epilogue z = c*d + noise + b, y = clamp(act(z)*gain):
 *   dc = dz * d;  db[o] = sum dz;  dd[n,o] = sum_p dz*c;  dnoise[n,p] = sum_o dz
 * where dz = dy * act'(y) * gain masked by |y| < clamp.  dy, y, c, dc: [N, HW, C] NHWC (any dtype),
 * C % 8 == 0.  c / d / db / dd / dnoise may be NULL; db and dd are zeroed by the call. */
int sg2_layer_bwd(void* dc, float* db, float* dd, float* dnoise, const void* dy, const void* y, const void* c,
                  const float* d, int dtype, int N, int HW, int C, int act, float alpha, float gain, float clamp,
                  void* stream);

/* The elementwise steps of the layers' create_graph VJP (path-length / R1 passes; the reference runs them as
 * autograd's mul / add / bias_act-grad nodes, SG3/training/networks_stylegan2.py:59-89 and bias_act.py:154-207):
 *   out[n,p,c] = act'(a * sa[n,c] + b * sb[n,c]; y)      (sa / sb NULL = 1, b NULL = off, y NULL = no act')
 *   dot[n,c]   = sum_p a[n,p,c] * e[n,p,c]                (e and dot both or neither; dot zeroed by the call)
 * act' = the bias_act gradient given the output y: * gain, * alpha where y <= 0 (lrelu), 0 where |y| >= clamp
 * (clamp < 0 = off).  a, b, y, e, out: [N, HW, C] NHWC of dtype (f16 / bf16 / f32), C % 8 == 0; f32
 * arithmetic, one rounding. */
int sg2_vjp_axpy(void* out, const void* a, const float* sa, const void* b, const float* sb, const void* y, int act,
                 float alpha, float gain, float clamp, const void* e, float* dot, int dtype, int N, int HW, int C,
                 void* stream);

/* out[n, c] = sum_p a[n, p, c] * b[n, p, c] (f32 accumulation; a, b: [N, HW, C] NHWC f16/bf16, C % 8 == 0;
 * out zeroed by the call).  The reductions (dz * c).sum([2, 3]) and (dxs * x).sum([2, 3]) of the
 * modulated-conv backward (SG3/training/networks_stylegan2.py:59-70 under autograd) without the
 * full-size product in HBM. */
int sg2_dot_hw(float* out, const void* a, const void* b, int dtype, int N, int HW, int C, void* stream);

/* Bilinear grid sample, zeros padding, align_corners = False (the only mode the reference uses,
 * grid_sample_gradfix.py:9-12).  in [N,C,Hi,Wi] any strides; grid float32 [N,Ho,Wo,2] contiguous;
 * out [N,C,Ho,Wo] any strides. */
int sg2_grid_sample_fwd(void* out, const void* in, const float* grid, int dtype, const int64_t* in_size,
                        const int64_t* in_stride, const int64_t* out_size, const int64_t* out_stride,
                        const int* dyn_hw, void* stream);

/* Gradient of sg2_grid_sample_fwd w.r.t. its input: gin (float32, [N,C,Hi,Wi] with in_stride) is
 * zero-filled then accumulated. */
int sg2_grid_sample_bwd(float* gin, const void* gout, const float* grid, int dtype, const int64_t* in_size,
                        const int64_t* in_stride, const int64_t* out_size, const int64_t* out_stride,
                        const int* dyn_hw, void* stream);

/* The same two ops with the sampling grid built inline from theta (float32 [N,2,3] contiguous) as
 * torch.nn.functional.affine_grid(theta, [N,C,Ho,Wo], align_corners=False) would build it: the fusion of
 * SG3/training/augment_mi.py:317-318 (affine_grid + grid_sample_gradfix.grid_sample), which never
 * materialises the [N,Ho,Wo,2] grid in HBM. */
int sg2_affine_grid_sample_fwd(void* out, const void* in, const float* theta, int dtype, const int64_t* in_size,
                               const int64_t* in_stride, const int64_t* out_size, const int64_t* out_stride,
                               const int* dyn_hw, void* stream);
int sg2_affine_grid_sample_bwd(float* gin, const void* gout, const float* theta, int dtype, const int64_t* in_size,
                               const int64_t* in_stride, const int64_t* out_size, const int64_t* out_stride,
                               const int* dyn_hw, void* stream);

/* dyn_hw (all grid-sample calls; may be NULL): device int[2], the logical input height / width when
 * `in` is a larger static buffer whose valid region starts at the origin -- the ADA pipe's padded image
 * whose size depends on device-side margins (augment_mi.py:288-318), sampled without a host sync. */

/* Reflect padding with device-side margins (augment_mi.py:301): margins = device int[4] {mx0, my0,
 * mx1, my1} (each <= size - 1).  adjoint = 0: y [N,C,Hs,Ws] (NCHW, f32) = reflect-padded x [N,C,H,W]
 * at the origin, zeros elsewhere; Hs >= 3H-2, Ws >= 3W-2.  adjoint = 1: y [N,C,H,W] = the adjoint
 * (gather of the reflected positions) of x [N,C,Hs,Ws]. */
int sg2_reflect_pad_dyn(float* y, const float* x, const int* margins, int N, int C, int H, int W, int Hs, int Ws,
                        int adjoint, void* stream);

/* ADA geometric transforms of a batch in one launch (ABI 6; replaces the per-op matrix algebra of
 * SG3/training/augment_mi.py:214-318 -- stack / sin / cos / where / matmul per enabled op, the corner margins
 * and the pad / up-sampling conjugations).  draw[2k], draw[2k+1]: the value draw and the choice draw of op k
 * in the reference's order -- 0 xflip (rand[N], rand[N]), 1 rotate90 (rand[N], rand[N]), 2 xint (rand[N,2],
 * rand[N,1]), 3 scale (randn[N], rand[N]), 4 rotate (rand[N], rand[N]), 5 aniso (randn[N], rand[N]), 6 the
 * second rotate, 7 xfrac (randn[N,2], rand[N,1]); NULL for an op whose probability is 0.  p: device f32
 * scalar, the augmentation probability.  pad_x / pad_y: f32(2 hz_pad - (W-1)/2) / (.. (H-1)/2); inv_sx /
 * inv_sy: f32(1 / (2 / Wup)) / f32(1 / (2 / Hup)) of the up-sampled static buffer (the reference's Python
 * floats).  Writes theta [N,2,3] (the grid-sample transform), margins int[4] (mx0, my0, mx1, my1: the
 * reflect pad), lims int[8] (the up-sampling extents) and dyn_hw int[2] (the logical up-sampled size). */
typedef struct sg2_aug_geom_args {
    const float* draw[16];
    const float* p;
    float xflip, rotate90, xint, xint_max, scale, rotate, aniso, xfrac;
    float scale_std, rotate_max, aniso_std, xfrac_std;
    float pad_x, pad_y, inv_sx, inv_sy;
    int n, h, w;
} sg2_aug_geom_args;
int sg2_aug_geom(float* theta, int* margins, int* lims, int* dyn_hw, const sg2_aug_geom_args* args, void* stream);

/* training_stats.report in one launch (ABI 6; SG3/torch_utils/training_stats.py:55-99): row[0] += n,
 * row[1] += sum v, row[2] += sum v^2 over the n f32 values v (mode 1: of sign(v)), accumulated in float64 in a
 * fixed order.  row: device double[3], the statistic's row of the caller's moment table. */
int sg2_moments(double* row, const float* v, int64_t n, int mode, void* stream);

/* Demodulation coefficients d[n,o] = rsqrt(sum_i s[n,i]^2 * wsq[o,i] + eps), wsq[o,i] = sum_k w[o,i,k]^2
 * (SG3/training/networks_stylegan2.py:59-63, summation regrouped); s [N,I] f32, w [O,I*KK] f32.  Also
 * writes wsq [O, I] (may be NULL) for the backward. */
int sg2_demod_fwd(float* d, float* wsq, const float* s, const float* w, int N, int O, int I, int KK, float eps,
                  void* stream);

/* Gradient of sg2_demod_fwd (first order): with gu = -dd * d^3 / 2,
 *   gw[o,i,k] = 2 w[o,i,k] sum_n gu[n,o] s[n,i]^2,   gs[n,i] = 2 s[n,i] sum_o gu[n,o] wsq[o,i].
 * gs / gw may be NULL (gs needs wsq).  The reference gets these from autograd of
 * networks_stylegan2.py:59-63. */
int sg2_demod_bwd(float* gs, float* gw, const float* dd, const float* d, const float* s, const float* w,
                  const float* wsq, int N, int O, int I, int KK, void* stream);

/* Backward of sg2_demod_bwd's styles gradient gs = 2 s (u @ wsq), u = -dd d^3 / 2 (ABI 7; the path-length pass
 * differentiates it once more -- the reference by autograd of networks_stylegan2.py:59-63 under create_graph):
 * given g = dL/dgs [N,I],
 *   g_dd = -d^3 v,  g_d = -3 dd d^2 v  (v = (s g) @ wsq^T),   g_w[o,i,k] = 2 w (u^T @ 2 s g)[o,i],
 *   g_s = 2 g (u @ wsq).
 * Any output may be NULL; w [O,I*KK], wsq [O,I] as written by sg2_demod_fwd. */
int sg2_demod_vjp_bwd(float* g_dd, float* g_d, float* g_w, float* g_s, const float* g, const float* dd,
                      const float* d, const float* s, const float* w, const float* wsq, int N, int O, int I, int KK,
                      void* stream);

/* Convolution weight pack (replaces the strided-permute copies that feed every conv launch,
 * conv2d_gradfix.py _pack_conv / _pack_convT; the reference feeds cuDNN the [O,I,kh,kw] weight
 * directly, networks_stylegan2.py:70/176):  out[a][k][b] = in[a*sa + b*sb + k'*sk], k' = K-1-k when
 * flip != 0, else k.  Strides in elements; in/out dtypes SG2_F32/F16/BF16 (cast in the same pass); K <= 9.
 * [O,I,kh,kw] -> [O][kh][kw][I]: A=O, B=I, K=kh*kw, sa=I*K, sb=K, sk=1.
 * Each element is multiplied by `scale` in f32 before the cast (ABI 3): a layer's weight gain, the
 * reference's `self.weight * self.weight_gain` (networks_stylegan2.py:173) in the same pass. */
int sg2_pack_weight(void* out, int out_dtype, const void* in, int in_dtype, int A, int B, int K, int64_t sa,
                    int64_t sb, int64_t sk, int flip, float scale, void* stream);

/* Many packs in one launch per 64 (ABI 8): `descs` is a HOST array of n sg2_pack_desc (copied into the launch's
 * kernel arguments, so the call can be captured into a hipGraph; block0 is ignored).  Each pack is bitwise what
 * sg2_pack_weight computes for the same arguments; strides must fit 32 bits.  Used by conv2d_gradfix.pack_cache to
 * pack all of a training phase's conv weights at the phase start. */
typedef struct sg2_pack_desc {
    void* out;
    const void* in;
    int64_t sa, sb, sk;
    int out_dtype, in_dtype, A, B, K, flip;
    float scale;
    int block0;
} sg2_pack_desc;
int sg2_pack_weight_multi(const sg2_pack_desc* descs, int n, void* stream);

/* fp16 range pre-normalisation, row-wise (SG3/training/networks_stylegan2.py:52-54): t [rows, L] f32,
 * n[r] = max_i |t[r,i]| (written to nrm [rows]); mode 0: y = t * ((1/n) * c)  (the weight, c = 1/sqrt(fan_in)),
 * mode 1: y = t / n  (the styles). */
int sg2_infnorm_fwd(float* y, float* nrm, const float* t, int rows, int L, float c, int mode, void* stream);

/* First-order gradient of sg2_infnorm_fwd w.r.t. t (torch's infinity-norm backward: the norm's gradient split
 * evenly between tied maxima). */
int sg2_infnorm_bwd(float* dt, const float* dy, const float* t, const float* nrm, int rows, int L, float c, int mode,
                    void* stream);

/* Backward of sg2_infnorm_bwd (ABI 7; the path-length pass's second order through the fp16 pre-normalisation,
 * reference: autograd of networks_stylegan2.py:52-54 under create_graph).  With the first-order gradient
 * dt = c dy / n - c P e / n^2, P = sum dy t, e = sgn(t) [|t| = n] / cnt, and g = dL/ddt [rows, L]:
 *   g_dy = c (g - t (g.e) / n) / n,   g_t = c (2 P (g.e) e / n^3 - ((g.dy) e + (g.e) dy) / n^2).
 * c = the mode-0 scale (1 for mode 1); either output may be NULL. */
int sg2_infnorm_vjp_bwd(float* g_dy, float* g_t, const float* g, const float* dy, const float* t, const float* nrm,
                        int rows, int L, float c, void* stream);

/* Multi-tensor launches of the optimiser step.  A segment is one parameter tensor; `blocks` [nblocks] lists
 * the work items as (segment << 40) | start, one per 4096 elements of a segment (start = 0, 4096, ...),
 * so one launch covers a whole module.  Tables are device int64 / float arrays built by the caller. */

/* torch.optim.Adam (no weight decay, amsgrad off; foreach arithmetic) of every parameter in one exchanged
 * flat gradient, with the reference's sanitation in front (training_loop_mi_multimodal.py:341-351):
 *   g = nan_to_num(grad * grad_scale, nan=0, posinf=1e5, neginf=-1e5)      (grad_scale = 1/num_gpus)
 *   m = m.lerp(g, 1-beta1);  v = v*beta2 + (1-beta2)*g*g;  p += -step_size * m / (sqrt(v)/bc2_sqrt + eps)
 * seg [nseg][3] = {float* param, offset of the segment in grad / exp_avg / exp_avg_sq, numel};
 * coef [nseg][2] f32 = {step_size = lr / (1 - beta1^step), bc2_sqrt = sqrt(1 - beta2^step)} (the caller's
 * per-parameter step counts, as torch keeps them).  write_grad != 0 stores the sanitised g back. */
int sg2_adam_multi(const int64_t* seg, const float* coef, const int64_t* blocks, int nblocks, float* grad,
                   float* exp_avg, float* exp_avg_sq, float beta1, float beta2, float eps, float grad_scale,
                   int write_grad, void* stream);

/* dst = src.lerp(dst, beta) per segment (the G_ema update, training_loop_mi_multimodal.py:363-364);
 * seg [nseg][3] = {float* dst, const float* src, numel}. */
int sg2_lerp_multi(const int64_t* seg, const int64_t* blocks, int nblocks, float beta, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SG2HIP_H */
