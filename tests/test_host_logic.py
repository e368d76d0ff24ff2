"""CPU: host-side pieces that need no GPU -- the synthetic input generator, the Emscripten-style
Module arena, and the decoder-side NAL splitting used by the C-ABI geometry peek."""
import hashlib
import os

import numpy as np
import pytest


def test_synthetic_stream_deterministic():
    from h264mi.synth import SyntheticStream
    a = SyntheticStream(5, 176, 144)
    b = SyntheticStream(5, 176, 144)
    f0, f1 = a.frame(3), b.frame(3)
    assert f0.dtype == np.uint8 and f0.size == 176 * 144 * 3 // 2
    assert np.array_equal(f0, f1)
    assert not np.array_equal(a.frame(0), a.frame(1))          # motion
    assert not np.array_equal(SyntheticStream(6, 176, 144).frame(0), f0)  # per-stream seed


def test_synthetic_stream_motion_is_translation():
    """frame t is the texture window at offset (3t mod 64, 2t mod 64): consecutive frames differ by
    a (3, 2) pixel shift away from the wrap, which is what the encoder's ME must find"""
    from h264mi.synth import SyntheticStream
    g = SyntheticStream(0, 64, 64)
    y0 = g.frame(1)[:64 * 64].reshape(64, 64)
    y1 = g.frame(2)[:64 * 64].reshape(64, 64)
    assert np.array_equal(y1[:-2, :-3], y0[2:, 3:])


class _FakeLib:
    """stand-in for the ctypes library so the Module arena logic is testable without a GPU"""
    def __getattr__(self, name):
        raise AttributeError(name)


def _module(monkeypatch):
    import h264mi
    monkeypatch.setattr(h264mi, 'lib', lambda: _FakeLib())
    return h264mi.Module(heap_bytes=1 << 16)


def test_module_malloc_free_reuse(monkeypatch):
    m = _module(monkeypatch)
    a = m._malloc(100)
    b = m._malloc(50)
    assert a != b and a % 16 == 0 and b % 16 == 0 and b >= a + 100
    m._free(a)
    c = m._malloc(64)   # first fit into the freed block
    assert c == a
    m.setValue(b, -12345, 'i32')
    assert m.getValue(b, 'i32') == -12345
    assert m.HEAPU8[b:b + 4] == (-12345).to_bytes(4, 'little', signed=True)


def test_module_exhaustion(monkeypatch):
    import pytest
    m = _module(monkeypatch)
    with pytest.raises(MemoryError):
        m._malloc(1 << 20)


def test_module_cwrap_rejects_unexported(monkeypatch):
    import pytest
    m = _module(monkeypatch)
    with pytest.raises(KeyError):
        m.cwrap('not_a_wrapper_function', 'number', [])


def test_code_object_has_no_ashr_pk(libpath, tmp_path):
    """hipcc (ROCm 7.2, gfx950) mis-lowers "shift, saturate to u8, pack two bytes" to v_ashr_pk_u8_i32
    with its upper 16 bits assumed zero; the sources use the clamp-first form. Guard:
    the built gfx950 code object must not contain the instruction."""
    import shutil
    import subprocess
    llvm = '/opt/rocm/lib/llvm/bin'
    if not os.path.exists(os.path.join(llvm, 'llvm-objdump')):
        pytest.skip('ROCm LLVM tools not installed')
    fb, co = tmp_path / 'fb.bin', tmp_path / 'gfx950.co'
    subprocess.run([os.path.join(llvm, 'llvm-objcopy'), '--dump-section', f'.hip_fatbin={fb}', libpath, str(tmp_path / 'x.so')], check=True)
    subprocess.run([os.path.join(llvm, 'clang-offload-bundler'), '--unbundle', '--type=o', f'--input={fb}',
                    '--targets=hipv4-amdgcn-amd-amdhsa--gfx950', f'--output={co}'], check=True)
    dis = subprocess.run([os.path.join(llvm, 'llvm-objdump'), '-d', '--mcpu=gfx950', str(co)], capture_output=True, text=True, check=True).stdout
    assert 'enc_mb_kernel' in dis
    assert 'v_ashr_pk' not in dis
