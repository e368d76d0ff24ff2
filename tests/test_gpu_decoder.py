"""GPU: decoder parity through the C-ABI (init_decoder / decode_frame_yuv_i420 /
decode_frame_optimized / deinit_decoder): pictures identical to the oracle decoder's on oracle
streams, plus the wrapper's pool and error semantics."""
import ctypes
import json
import os

import numpy as np
import pytest

from golden.make_golden import CASES, case_inputs, sha

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
FX = {c['name']: c for c in json.load(open(os.path.join(HERE, 'golden', 'oracle_fixtures.json')))['cases']}


def gpu_decode(L, idx, nal, w, h, rgba=False):
    a = np.frombuffer(nal, np.uint8).copy() if nal else np.zeros(1, np.uint8)
    out = np.zeros(w * h * 4, np.uint8)
    gw, gh = ctypes.c_int(-1), ctypes.c_int(-1)
    f = L.decode_frame_optimized if rgba else L.decode_frame_yuv_i420
    f(idx, a.ctypes.data, len(nal), out.ctypes.data, ctypes.byref(gw), ctypes.byref(gh))
    n = gw.value * gh.value * (4 if rgba else 3) // (1 if rgba else 2)
    return gw.value, gh.value, out[:n]


@pytest.mark.parametrize('case', CASES, ids=[c[0] for c in CASES])
def test_decoder_matches_oracle(gpu_lib, oracle, case):
    name, w, h, br, n, force_every, kind = case
    L = gpu_lib
    frames, _ = case_inputs(oracle, w, h, n, kind)
    oe, od = oracle.encoder(w, h, br), oracle.decoder()
    assert L.init_decoder(2) == 0
    for t in range(n):
        if force_every and t % force_every == 0 and t > 0:
            oe.force_idr()
        nal = oe.encode(frames[t])
        if not nal:  # frame skipped by the rate control: no access unit
            continue
        rc, pic, _, _ = od.decode(nal)
        gw, gh, got = gpu_decode(L, 2, nal, w, h)
        assert (gw, gh) == (w, h)
        assert np.array_equal(got, pic), f'{name} frame {t}'
        assert sha(got) == FX[name]['dec_sha256'][t]
    L.deinit_decoder(2)


def test_decoder_rgba_matches_oracle(gpu_lib, oracle):
    from h264mi.synth import SyntheticStream
    w, h = 352, 288
    L = gpu_lib
    g = SyntheticStream(9, w, h)
    oe, od = oracle.encoder(w, h, 1500000), oracle.decoder()
    oe.set_frame_skip(False)  # every frame coded
    assert L.init_decoder(5) == 0
    for t in range(4):
        nal = oe.encode(np.ascontiguousarray(g.frame(t)))
        _, pic, _, _ = od.decode(nal)
        gw, gh, got = gpu_decode(L, 5, nal, w, h, rgba=True)
        assert (gw, gh) == (w, h)
        assert np.array_equal(got, oracle.i420_to_rgba(pic, w, h)), t
    L.deinit_decoder(5)


def test_committed_stream(gpu_lib, oracle):
    data = open(os.path.join(HERE, 'golden', 'synth3_qcif_3f.h264'), 'rb').read()
    starts = [k for k in range(len(data) - 3) if data[k:k + 4] == b'\x00\x00\x00\x01']
    cuts = [0] + [k for k in starts if data[k + 4] & 31 == 1] + [len(data)]
    L = gpu_lib
    od = oracle.decoder()
    assert L.init_decoder(0) == 0
    for a, b in zip(cuts[:-1], cuts[1:]):
        _, pic, _, _ = od.decode(data[a:b])
        gw, gh, got = gpu_decode(L, 0, data[a:b], 176, 144)
        assert (gw, gh) == (176, 144) and np.array_equal(got, pic)
    L.deinit_decoder(0)


def test_decoder_pool_semantics(gpu_lib):
    L = gpu_lib
    assert L.init_decoder(-1) == -1 and L.init_decoder(32) == -1     # openh264_wrapper.cpp:255
    gw, gh, _ = gpu_decode(L, 31, b'\x00\x00\x00\x01\x09\x10', 16, 16)  # uninitialised slot: no-op
    assert (gw, gh) == (0, 0)
    assert L.init_decoder(31) == 0
    gw, gh, _ = gpu_decode(L, 31, b'', 16, 16)
    assert (gw, gh) == (0, 0)
    L.deinit_decoder(31)
    L.deinit_decoder(31)  # double deinit is harmless


def test_decoder_garbage_then_recovery(gpu_lib, oracle):
    """damaged access units produce no picture or the frame-copy concealment of the last picture
    (ERROR_CON_FRAME_COPY) and the decoder resumes at the next IDR; the parse kernel must survive
    arbitrary payloads"""
    from h264mi.synth import SyntheticStream
    w, h = 176, 144
    L = gpu_lib
    assert L.init_decoder(7) == 0
    oe, od = oracle.encoder(w, h, 300000), oracle.decoder()
    g = SyntheticStream(1, w, h)
    first = oe.encode(np.ascontiguousarray(g.frame(0)))
    _, pic, _, _ = od.decode(first)
    gw, gh, got = gpu_decode(L, 7, first, w, h)
    assert (gw, gh) == (w, h) and np.array_equal(got, pic)
    sps_pps = first[:first.index(b'\x00\x00\x00\x01\x65')]
    rng = np.random.default_rng(0)
    for k in range(12):
        junk = bytes(rng.integers(0, 256, 40 + 211 * k, dtype=np.uint8))
        hdr = b'\x00\x00\x00\x01' + (b'\x65' if k % 2 == 0 else b'\x41')
        gw, gh, _ = gpu_decode(L, 7, (sps_pps if k % 3 == 0 else b'') + hdr + junk, w, h)
        # random payloads almost never form a valid slice; either way the call must return
        assert (gw, gh) in ((0, 0), (w, h))
    oe.force_idr()
    nal = oe.encode(np.ascontiguousarray(g.frame(1)))
    _, pic, _, _ = od.decode(nal)
    gw, gh, got = gpu_decode(L, 7, nal, w, h)
    assert (gw, gh) == (w, h) and np.array_equal(got, pic)
    L.deinit_decoder(7)


def test_decoder_frame_copy_concealment(gpu_lib, oracle):
    """ERROR_CON_FRAME_COPY (openh264_wrapper.cpp:269): a damaged access unit -- here a truncated
    P slice and a picture split into slices (outside the Baseline subset both decoders accept) --
    is concealed by a copy of the last picture, which stays the reference, exactly as in the oracle
    decoder; the following frames decode against it (drifted, identically in both decoders). The
    wrapper outputs a picture only when DecodeFrameNoDelay returns 0 (openh264_wrapper.cpp:407,
    :435) and OpenH264 flags a concealed frame with a non-zero status, so the C-ABI reports 0 x 0
    for the concealed access units themselves."""
    from h264mi.synth import SyntheticStream
    from streamgen import p_frame
    w, h = 176, 144
    L = gpu_lib
    assert L.init_decoder(9) == 0
    oe, od = oracle.encoder(w, h, 300000), oracle.decoder()
    oe.set_frame_skip(False)  # every frame coded
    g = SyntheticStream(4, w, h)
    units = [oe.encode(np.ascontiguousarray(g.frame(t))) for t in range(6)]
    units[2] = units[2][:len(units[2]) // 2]                                        # truncated slice
    units[4] = p_frame(11, 9, 4, 8, np.random.default_rng(4), first_mb=33)          # second slice only
    concealed = 0
    for k, u in enumerate(units):
        rc, pic, _, _ = od.decode(u)
        gw, gh, got = gpu_decode(L, 9, u, w, h)
        assert rc in (1, 2), k
        if rc == 2:
            concealed += 1
            assert (gw, gh) == (0, 0), f'frame {k}: a concealed access unit is not output'
        else:
            assert (gw, gh) == (w, h) and np.array_equal(got, pic), f'frame {k} (oracle rc {rc})'
    assert concealed == 2
    L.deinit_decoder(9)
    # nothing to conceal before the first picture: no output
    assert L.init_decoder(9) == 0
    od2 = oracle.decoder()
    rc, _, _, _ = od2.decode(units[1])
    assert rc <= 0
    assert gpu_decode(L, 9, units[1], w, h)[:2] == (0, 0)
    L.deinit_decoder(9)


@pytest.mark.parametrize('max_mvd,dbk', [(24, 0), (160, 0), (400, 1)], ids=['mvd24', 'mvd160', 'mvd400-nodbk'])
def test_long_vectors_vs_oracle(gpu_lib, oracle, max_mvd, dbk):
    """Hand-built P pictures with arbitrary motion vectors (references far outside the picture and
    outside the reconstruction kernel's LDS window) decode exactly as the oracle decoder does."""
    import ctypes
    import numpy as np
    from h264mi.synth import SyntheticStream
    from streamgen import p_frame
    w, h = 176, 144
    idr = oracle.encoder(w, h, 400000).encode(np.ascontiguousarray(SyntheticStream(3, w, h).frame(0)))
    rng = np.random.default_rng(max_mvd)
    units = [idr] + [p_frame(11, 9, t, 2 * t, rng, max_mvd=max_mvd, dbk_idc=dbk) for t in range(1, 6)]
    od = oracle.decoder()
    L = gpu_lib
    assert L.init_decoder(5) == 0
    out = np.zeros(w * h * 3 // 2, np.uint8)
    gw, gh = ctypes.c_int(), ctypes.c_int()
    for k, u in enumerate(units):
        rc, ref, _, _ = od.decode(u)
        assert rc == 1, k
        buf = np.frombuffer(u, np.uint8).copy()
        L.decode_frame_yuv_i420(5, buf.ctypes.data, len(u), out.ctypes.data, ctypes.byref(gw), ctypes.byref(gh))
        assert (gw.value, gh.value) == (w, h), k
        assert np.array_equal(out, ref), f'frame {k}'
    L.deinit_decoder(5)
