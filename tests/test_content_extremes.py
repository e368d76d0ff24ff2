"""Content and rate extremes, fixture-free: flat pictures (P_Skip everywhere), white noise at
100 Mbps (rate control walks the QP down, at most 3 per frame, from the table IDR QP 24: large
levels, CAVLC level_prefix escapes) and at 50 kbps (QP pinned at OpenH264's camera maximum 42), motion beyond the +-16 search range, scene cuts between unrelated
textures, and saturated 0/255 blocks (clipping in prediction and reconstruction).

At 50 kbps the rate control also skips frames (0-byte access units).

-m "not gpu": the oracle decoder reproduces the oracle encoder's reconstruction on every coded frame.
-m gpu: through the C-ABI, GPU encoder bytes == oracle encoder bytes and GPU decoder pictures ==
oracle decoder pictures, frame by frame. Bit-exact (integer path, no tolerance)."""
import ctypes

import numpy as np
import pytest

W, H, N = 352, 288, 8

# name, bitrate, content
CASES = [
    ('flat', 1000000, 'flat'),
    ('noise_100m', 100000000, 'noise'),
    ('noise_50k', 50000, 'noise'),
    ('fast_motion', 2000000, 'fast'),
    ('scene_cut', 2000000, 'cut'),
    ('saturated', 4000000, 'sat'),
]


def content_frames(kind, w=W, h=H, n=N):
    """Seeded tight I420 frames of the named content."""
    rng = np.random.default_rng(7)
    fs = w * h * 3 // 2
    out = []
    if kind == 'flat':
        out = [np.full(fs, 128 if t % 2 == 0 else 131, np.uint8) for t in range(n)]
    elif kind == 'noise':
        out = [rng.integers(0, 256, fs, dtype=np.uint8) for _ in range(n)]
    elif kind in ('fast', 'cut'):
        from h264mi.synth import SyntheticStream
        a = SyntheticStream(3, w + 48 * n, h) if kind == 'fast' else SyntheticStream(3, w, h)
        b = SyntheticStream(11, w, h)
        for t in range(n):
            if kind == 'cut':  # alternate two unrelated textures every frame
                out.append(np.ascontiguousarray((a if t % 2 == 0 else b).frame(t)))
            else:  # a window sliding 40 luma samples per frame over one wide picture
                big = a.frame(0)
                bw = w + 48 * n
                y = big[:bw * h].reshape(h, bw)[:, 40 * t:40 * t + w]
                u = big[bw * h:bw * h + (bw // 2) * (h // 2)].reshape(h // 2, bw // 2)[:, 20 * t:20 * t + w // 2]
                v = big[bw * h + (bw // 2) * (h // 2):].reshape(h // 2, bw // 2)[:, 20 * t:20 * t + w // 2]
                out.append(np.ascontiguousarray(np.concatenate([y.ravel(), u.ravel(), v.ravel()])))
    elif kind == 'sat':
        for t in range(n):
            blk = rng.integers(0, 2, (h // 8, w // 8), dtype=np.uint8) * 255
            y = np.repeat(np.repeat(blk, 8, 0), 8, 1)
            c = np.repeat(np.repeat(blk, 4, 0), 4, 1)  # the co-sited 4x4 chroma blocks
            out.append(np.ascontiguousarray(np.concatenate([y.ravel(), c.ravel(), (255 - c).ravel()]).astype(np.uint8)))
    assert len(out) == n and all(f.size == fs and f.dtype == np.uint8 for f in out)
    return out


@pytest.mark.parametrize('case', CASES, ids=[c[0] for c in CASES])
def test_oracle_roundtrip_extremes(oracle, case):
    name, br, kind = case
    oe, od = oracle.encoder(W, H, br), oracle.decoder()
    qps, skipped = [], 0
    for t, f in enumerate(content_frames(kind)):
        nal = oe.encode(f)
        if not nal:  # skipped by rate control: the reference stays, nothing to decode
            assert t > 0, name
            skipped += 1
            continue
        qps.append(oe.last_qp())
        rc, pic, dw, dh = od.decode(nal)
        assert rc == 1 and (dw, dh) == (W, H), (name, t, rc)
        assert np.array_equal(pic, oe.recon()), f'{name}: oracle decoder != encoder reconstruction at frame {t}'
    if name == 'noise_100m':  # IDR at the table QP, then down the frame window's lower bound (-3)
        assert qps[0] == 24 and min(qps) <= 18 and qps == sorted(qps, reverse=True), qps
    if name == 'noise_50k':  # the buffer overflows: frames are skipped; without skipping QP pins at 42
        assert skipped > 0, (qps, skipped)
        oe2 = oracle.encoder(W, H, br)
        oe2.set_frame_skip(False)
        for f in content_frames(kind):
            assert len(oe2.encode(f)) > 0
            qps.append(oe2.last_qp())
        assert max(qps) == 42, qps
    if name in ('flat', 'noise_100m', 'saturated'):
        assert skipped == 0, (name, skipped)


@pytest.mark.gpu
@pytest.mark.parametrize('case', CASES, ids=[c[0] for c in CASES])
def test_gpu_encode_decode_extremes(gpu_lib, oracle, case):
    name, br, kind = case
    L = gpu_lib
    assert L.init_encoder(W, H, br) == 0
    assert L.init_decoder(5) == 0
    oe, od = oracle.encoder(W, H, br), oracle.decoder()
    p = ctypes.POINTER(ctypes.c_ubyte)()
    sz = ctypes.c_int(0)
    out = np.zeros(W * H * 3 // 2, np.uint8)
    gw, gh = ctypes.c_int(-1), ctypes.c_int(-1)
    for t, f in enumerate(content_frames(kind)):
        L.encode_frame_yuv_i420(f.ctypes.data, W, H, ctypes.byref(p), ctypes.byref(sz))
        got = ctypes.string_at(p, sz.value) if sz.value > 0 else b''
        ref = oe.encode(f)
        assert got == ref, f'{name} frame {t}: GPU {len(got)} B vs oracle {len(ref)} B'
        if not ref:  # frame skipped by both rate controls
            continue
        _, pic, _, _ = od.decode(ref)
        a = np.frombuffer(got, np.uint8).copy()
        L.decode_frame_yuv_i420(5, a.ctypes.data, len(got), out.ctypes.data, ctypes.byref(gw), ctypes.byref(gh))
        assert (gw.value, gh.value) == (W, H), (name, t)
        assert np.array_equal(out, pic), f'{name} frame {t}: GPU decoded picture != oracle'
    L.deinit_decoder(5)
