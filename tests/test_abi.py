"""The C-ABI library loads and exports every symbol include/nicnes.h declares; config validation
and layout queries work without a GPU (no compute calls here)."""
import ctypes
import os
import re

import numpy as np

import nicnes
from nicnes import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(REPO, 'include', 'nicnes.h')).read()
    return sorted(set(re.findall(r'^\s*(?:int|int64_t|const char\*)\s+(nicnes_\w+)\(', src, re.M)))


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(_lib.EXPORTS) == syms


def test_param_count_and_offsets_match_reference_layout():
    L = _lib.lib()
    cfg = _lib.NicnesConfig(9487, 128, 128, 2048, 16, 128, 640, 512, 1 << 27, 0)
    assert L.nicnes_param_count(ctypes.byref(cfg)) == 2865808     # src/algorithm/tools/utils.py:180
    off = (ctypes.c_int64 * 10)()
    assert L.nicnes_param_offsets(ctypes.byref(cfg), off) == 0
    assert list(off) == [0, 262144, 262272, 1476736, 2691200, 2700688, 2782608, 2783248, 2865168, 2865808]


def test_unsupported_configs_rejected_before_touching_the_gpu():
    L = _lib.lib()
    h = ctypes.c_void_p()
    bad = [
        _lib.NicnesConfig(9487, 64, 128, 2048, 16, 128, 640, 512, 1 << 27, 0),    # E != 128
        _lib.NicnesConfig(9487, 128, 128, 2000, 16, 128, 640, 512, 1 << 27, 0),   # F % 128
        _lib.NicnesConfig(9488, 128, 128, 2048, 16, 128, 640, 512, 1 << 27, 0),   # V+1 % 4
        _lib.NicnesConfig(20000, 128, 128, 2048, 16, 128, 640, 512, 1 << 27, 0),  # ids >= 2^14
        _lib.NicnesConfig(9487, 128, 128, 2048, 17, 128, 640, 512, 1 << 27, 0),   # seq_length > 16
    ]
    for cfg in bad:
        assert L.nicnes_create(ctypes.byref(cfg), 0, ctypes.byref(h)) == _lib.ERR_UNSUPPORTED
    assert L.nicnes_create(None, 0, ctypes.byref(h)) == _lib.ERR_INVALID


def test_null_handle_calls_fail_cleanly():
    L = _lib.lib()
    assert L.nicnes_evaluate(None, 0, 0, 1, 0.01, None, None, None) == _lib.ERR_INVALID
    assert L.nicnes_last_error(None) == b'null handle'
    assert L.nicnes_destroy(None) == 0


def test_check_raises_with_message():
    try:
        _lib.check(_lib.ERR_UNSUPPORTED, None, 'x')
    except _lib.NicnesError as e:
        assert 'not supported' in str(e)
    else:
        raise AssertionError


def test_product_does_not_import_the_oracle():
    pkg = os.path.join(REPO, 'nes-img-captioning_amd')
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(('.py', '.cpp', '.hip', '.h')):
                txt = open(os.path.join(root, f)).read()
                assert 'import oracle' not in txt and 'from oracle' not in txt, f
                assert 'nicnes_oracle' not in txt, f


def test_pack_ngram_layout():
    assert nicnes.pack_ngram((5,)) == (1 << 56) | (5 << 42)
    assert nicnes.pack_ngram((1, 2, 3, 4)) == (4 << 56) | (1 << 42) | (2 << 28) | (3 << 14) | 4
    keys, vals = nicnes.df_table_arrays({('3', '4'): 2.0, (1,): 5.0})
    assert keys.dtype == np.uint64 and np.all(np.diff(keys.astype(np.float64)) > 0)
    assert list(vals) == [5.0, 2.0]
