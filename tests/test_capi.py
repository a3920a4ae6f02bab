"""C-ABI boundary checks that need no GPU: the library loads, exports every symbol include/sg2hip.h
declares with the ABI version the binding expects, and argument errors come back as negative
status codes with a message (no device work is issued)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'sg2hip.h')


def header_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r'^\s*(?:int|void|const char\*)\s+(sg2_\w+)\s*\(', text, flags=re.M)))


def test_header_parses():
    syms = header_symbols()
    assert 'sg2_conv2d' in syms and 'sg2_upfirdn2d' in syms and 'sg2_bias_act' in syms
    assert len(syms) >= 10


def test_library_exports_header_symbols():
    import sg2hip
    lib = sg2hip.lib()
    for s in header_symbols():
        assert hasattr(lib, s), s
    assert set(header_symbols()) - {'sg2_last_error'} == set(sg2hip.SIGNATURES), 'binding and header disagree'
    assert lib.sg2_abi_version() == sg2hip.ABI_VERSION


def test_argument_errors_are_reported():
    import sg2hip
    lib = sg2hip.lib()
    rc = lib.sg2_bias_act(None, None, None, None, None, None, 0, 10, 1, 1, 0, 3, 0.2, 1.0, -1.0, None)
    assert rc < 0
    assert b'non-null' in lib.sg2_last_error()
    rc = lib.sg2_conv2d(None, None, None, 0, 1, 1, 1, 1, 1, 1, 1, 3, 3, 1, 1, 1, 0, None, 0, None)
    assert rc < 0
    rc = lib.sg2_bias_act(ctypes.c_void_p(16), ctypes.c_void_p(16), None, None, None, None, 0, 10, 1, 1, 0, 42,
                          0.2, 1.0, -1.0, None)
    assert rc < 0 and b'activation' in lib.sg2_last_error()


def test_ops_refuse_cpu_tensors():
    import torch
    from torch_utils.ops import bias_act, upfirdn2d, conv2d_gradfix, grid_sample_gradfix
    x = torch.zeros(1, 2, 4, 4)
    with pytest.raises(RuntimeError):
        bias_act.bias_act(x, act='lrelu')
    with pytest.raises(RuntimeError):
        upfirdn2d.upfirdn2d(x, None)
    with pytest.raises(RuntimeError):
        conv2d_gradfix.conv2d(x, torch.zeros(3, 2, 3, 3))
    with pytest.raises(RuntimeError):
        grid_sample_gradfix.grid_sample(x, torch.zeros(1, 4, 4, 2))
