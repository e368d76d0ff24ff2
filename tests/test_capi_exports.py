"""CPU: the C-ABI library loads and exports every function include/h264mi.h declares (no compute
calls -- there is no GPU here)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, 'include', 'h264mi.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    names = re.findall(r'^[A-Za-z_][\w \*]*?\b([a-z_][a-z0-9_]*)\s*\(', src, flags=re.M)
    return sorted(set(n for n in names if n not in ('if', 'while', 'sizeof')))


def test_header_declares_reference_surface():
    names = declared_functions()
    for f in ('init_encoder', 'force_key_frame', 'init_decoder', 'deinit_decoder', 'encode_frame',
              'encode_frame_yuv_i420', 'decode_frame_optimized', 'decode_frame_yuv_i420', 'free_buffer'):
        assert f in names, f
    assert len(names) > 30


def test_library_exports_every_declared_symbol(libpath):
    L = ctypes.CDLL(libpath)
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing


def test_python_bindings_cover_header(libpath):
    import h264mi
    L = h264mi.lib()
    for n in declared_functions():
        assert hasattr(L, n), n


def test_version_string(libpath):
    L = ctypes.CDLL(libpath)
    L.h264mi_version.restype = ctypes.c_char_p
    assert L.h264mi_version().startswith(b'h264mi')
