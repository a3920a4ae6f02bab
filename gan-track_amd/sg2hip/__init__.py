"""ctypes binding of libsg2hip.so -- the C-ABI declared in include/sg2hip.h.

The product path has no fallback: if the library is missing, or a tensor is not on a ROCm
device, every op raises.  (The reference's ops silently fall back to slow `_ref` paths on CPU,
SG3/torch_utils/ops/upfirdn2d.py:160-162; here that would hide a broken build, so it is an error.)
"""
import contextlib
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('SG2HIP_LIB', os.path.join(_HERE, 'libsg2hip.so'))

F32, F16, BF16, F32S3 = 0, 1, 2, 3
_DTYPES = {torch.float32: F32, torch.float16: F16, torch.bfloat16: BF16}

_c_i64p = ctypes.POINTER(ctypes.c_int64)


class Epilogue(ctypes.Structure):
    """sg2_epilogue (include/sg2hip.h)."""
    _fields_ = [('out_scale', ctypes.c_void_p), ('noise', ctypes.c_void_p), ('bias', ctypes.c_void_p),
                ('residual', ctypes.c_void_p), ('aux', ctypes.c_void_p), ('noise_gain', ctypes.c_float),
                ('alpha', ctypes.c_float), ('gain', ctypes.c_float), ('clamp', ctypes.c_float),
                ('act', ctypes.c_int), ('aux_mode', ctypes.c_int), ('dot_src', ctypes.c_void_p),
                ('dot_out', ctypes.c_void_p)]

class AugGeomArgs(ctypes.Structure):
    """sg2_aug_geom_args (include/sg2hip.h)."""
    _fields_ = [('draw', ctypes.c_void_p * 16), ('p', ctypes.c_void_p)] + \
        [(k, ctypes.c_float) for k in ('xflip', 'rotate90', 'xint', 'xint_max', 'scale', 'rotate', 'aniso', 'xfrac',
                                       'scale_std', 'rotate_max', 'aniso_std', 'xfrac_std', 'pad_x', 'pad_y',
                                       'inv_sx', 'inv_sy')] + \
        [(k, ctypes.c_int) for k in ('n', 'h', 'w')]


_vp = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64
_f = ctypes.c_float

# name -> argtypes (restype is int for all entry points except sg2_last_error)
SIGNATURES = {
    'sg2_abi_version': [],
    'sg2_bias_act': [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i64, _i64, _i64, _i, _i, _f, _f, _f, _vp],
    'sg2_upfirdn2d': [_vp, _vp, _vp, _i, _c_i64p, _c_i64p, _c_i64p, _c_i64p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i,
                      _i, _f, _vp],
    'sg2_conv2d': [_vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _i64, _vp],
    'sg2_conv2d_fused': [_vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp,
                         ctypes.POINTER(Epilogue), _vp, _i64, _vp],
    'sg2_conv3x3': [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _f, _vp, _i, _f, _f, _f, _vp, _vp,
                    _vp],
    'sg2_set_zeroed_accumulators': [_i],
    'sg2_set_clean_workspace': [_i],
    'sg2_set_deterministic': [_vp, _i64],
    'sg2_split3': [_vp, _vp, _i64, _i, _i64, _vp, _vp],
    'sg2_conv3x3_s2': [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _f, _vp, _i, _f, _f, _f, _vp, _i,
                       _vp, _vp, _vp],
    'sg2_conv3x3_up2': [_vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp],
    'sg2_conv2d_wgrad': [_vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _f, _vp],
    'sg2_conv2d_wgrad_oikk': [_vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _f, _i, _vp],
    'sg2_upfirdn2d_lim': [_vp, _vp, _vp, _i, _c_i64p, _c_i64p, _c_i64p, _c_i64p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i,
                          _i, _f, _vp, _vp],
    'sg2_upfirdn2d_fused': [_vp, _vp, _vp, _i, _c_i64p, _c_i64p, _c_i64p, _c_i64p, _i, _i, _i, _i, _i, _i, _i, _i, _i,
                            _i, _i, _f, ctypes.POINTER(Epilogue), _vp],
    'sg2_layer_bwd': [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _f, _f, _f, _vp],
    'sg2_dot_hw': [_vp, _vp, _vp, _i, _i, _i, _i, _vp],
    'sg2_vjp_axpy': [_vp, _vp, _vp, _vp, _vp, _vp, _i, _f, _f, _f, _vp, _vp, _i, _i, _i, _i, _vp],
    'sg2_grid_sample_fwd': [_vp, _vp, _vp, _i, _c_i64p, _c_i64p, _c_i64p, _c_i64p, _vp, _vp],
    'sg2_grid_sample_bwd': [_vp, _vp, _vp, _i, _c_i64p, _c_i64p, _c_i64p, _c_i64p, _vp, _vp],
    'sg2_affine_grid_sample_fwd': [_vp, _vp, _vp, _i, _c_i64p, _c_i64p, _c_i64p, _c_i64p, _vp, _vp],
    'sg2_affine_grid_sample_bwd': [_vp, _vp, _vp, _i, _c_i64p, _c_i64p, _c_i64p, _c_i64p, _vp, _vp],
    'sg2_reflect_pad_dyn': [_vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp],
    'sg2_aug_geom': [_vp, _vp, _vp, _vp, ctypes.POINTER(AugGeomArgs), _vp],
    'sg2_moments': [_vp, _vp, _i64, _i, _vp],
    'sg2_demod_fwd': [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _f, _vp],
    'sg2_demod_bwd': [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp],
    'sg2_demod_vjp_bwd': [_vp] * 10 + [_i, _i, _i, _i, _vp],
    'sg2_adam_multi': [_vp, _vp, _vp, _i, _vp, _vp, _vp, _f, _f, _f, _f, _i, _vp],
    'sg2_lerp_multi': [_vp, _vp, _i, _f, _vp],
    'sg2_infnorm_fwd': [_vp, _vp, _vp, _i, _i, _f, _i, _vp],
    'sg2_infnorm_bwd': [_vp, _vp, _vp, _vp, _i, _i, _f, _i, _vp],
    'sg2_infnorm_vjp_bwd': [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _f, _vp],
    'sg2_pack_weight': [_vp, _i, _vp, _i, _i, _i, _i, _i64, _i64, _i64, _i, _f, _vp],
    'sg2_pack_weight_multi': [_vp, _i, _vp],
}
ABI_VERSION = 9

_lib = None


def lib():
    """Load (once) and return the ctypes handle; raises if the HIP build is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f'sg2hip: {LIB_PATH} not found -- build it with `python -c "import __graft_entry__ as '
                               f'g; g.build()"` (hipcc --offload-arch=gfx950); there is no CPU fallback')
        L = ctypes.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = ctypes.c_int
        L.sg2_last_error.argtypes = []
        L.sg2_last_error.restype = ctypes.c_char_p
        L.sg2_set_zeroed_accumulators.restype = None
        L.sg2_set_clean_workspace.restype = None
        L.sg2_set_deterministic.restype = None
        if L.sg2_abi_version() != ABI_VERSION:
            raise RuntimeError(f'sg2hip: ABI version mismatch ({L.sg2_abi_version()} != {ABI_VERSION})')
        _lib = L
    return _lib


@contextlib.contextmanager
def clean_workspace(on=True):
    """Calls inside take their split-K workspace as zeroed and leave it zeroed (sg2_set_clean_workspace)."""
    if not on:
        yield
        return
    L = lib()
    L.sg2_set_clean_workspace(1)
    try:
        yield
    finally:
        L.sg2_set_clean_workspace(0)


_det_scratch = {}
_det_retired = []
_det_state = (0, 0)     # the registration in force: (scratch pointer, bytes); (0, 0) = float-atomic mode


def det_active():
    """Whether the deterministic reductions are in force on this process (sg2_set_deterministic)."""
    return _det_state[0] != 0


def _det_register(ptr, nbytes):
    global _det_state
    lib().sg2_set_deterministic(ctypes.c_void_p(ptr), ctypes.c_int64(nbytes))
    _det_state = (ptr, nbytes)


@contextlib.contextmanager
def deterministic(on=True, scratch_mb=2048, device=None):
    """Bitwise-reproducible mode (sg2_set_deterministic): inside, every float accumulation the kernels would make
    with atomics is made through slots of a device scratch buffer summed in a fixed order -- the arithmetic the
    training iteration runs by default (training/trainer.py Trainer(deterministic=True)).  on=False selects the
    float-atomic reductions inside (an A/B mode).  The mode in force before is restored on exit.  The scratch
    (`scratch_mb` MiB, allocated once per device and kept) must not be used by two streams at once: run the calls
    inside on one stream."""
    prev = _det_state
    if on:
        dev = torch.device('cuda', torch.cuda.current_device()) if device is None else torch.device(device)
        buf = _det_scratch.get(dev)
        if buf is None or buf.numel() * 4 < scratch_mb << 20:
            if buf is not None:
                _det_retired.append(buf)     # a captured graph may still write the old scratch
            buf = _det_scratch[dev] = torch.empty([scratch_mb << 18], dtype=torch.float32, device=dev)
        _det_register(buf.data_ptr(), buf.numel() * 4)
    else:
        _det_register(0, 0)
    try:
        yield
    finally:
        _det_register(*prev)


@contextlib.contextmanager
def zeroed_accumulators(on=True):
    """Calls inside skip zeroing their float accumulator outputs (sg2_set_zeroed_accumulators): the
    caller passed buffers it zeroed itself, one fill for all of a layer's accumulators."""
    if not on:
        yield
        return
    L = lib()
    L.sg2_set_zeroed_accumulators(1)
    try:
        yield
    finally:
        L.sg2_set_zeroed_accumulators(0)


def check(rc, what):
    if rc != 0:
        msg = lib().sg2_last_error().decode(errors='replace')
        raise RuntimeError(f'{what} failed ({rc}): {msg}')


def dtype_code(t):
    try:
        return _DTYPES[t.dtype]
    except KeyError:
        raise RuntimeError(f'sg2hip: unsupported dtype {t.dtype}') from None


def require_device(*tensors):
    for t in tensors:
        if t is not None and (not isinstance(t, torch.Tensor) or t.device.type != 'cuda'):
            raise RuntimeError('sg2hip ops run only on ROCm device tensors (no CPU fallback); got '
                               f'{type(t).__name__} on {getattr(t, "device", None)}')


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def i64arr(vals):
    return (ctypes.c_int64 * len(vals))(*[int(v) for v in vals])
