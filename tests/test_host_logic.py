"""CPU: host-side pieces that need no GPU -- the synthetic input generator, the Emscripten-style
Module arena, and the decoder-side NAL splitting used by the C-ABI geometry peek."""
import hashlib

import numpy as np


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
