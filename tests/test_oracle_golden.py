"""CPU: the oracle (TEST INFRASTRUCTURE) against the committed fixtures, and its internal
consistency (decoder output == encoder reconstruction, every frame)."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

from golden.make_golden import CASES, colour_case, run_case, sha

HERE = os.path.dirname(os.path.abspath(__file__))
FX = json.load(open(os.path.join(HERE, 'golden', 'oracle_fixtures.json')))


@pytest.mark.parametrize('case', CASES, ids=[c[0] for c in CASES])
def test_oracle_matches_fixture(oracle, case):
    got = run_case(oracle, *case)  # also asserts decode == recon per frame
    ref = next(c for c in FX['cases'] if c['name'] == case[0])
    for k in ('nal_sizes', 'nal_sha256', 'dec_sha256', 'recon_sha256', 'qp'):
        assert got[k] == ref[k], (case[0], k)


def test_colour_fixture(oracle):
    assert colour_case(oracle) == FX['colour']


def test_committed_stream_decodes(oracle):
    data = open(os.path.join(HERE, 'golden', 'synth3_qcif_3f.h264'), 'rb').read()
    # access units: cut before every non-IDR slice (stream = [SPS PPS IDR] [P] [P])
    starts = [k for k in range(len(data) - 3) if data[k:k + 4] == b'\x00\x00\x00\x01']
    cuts = [0] + [k for k in starts if data[k + 4] & 31 == 1] + [len(data)]
    aus = [data[a:b] for a, b in zip(cuts[:-1], cuts[1:])]
    dec = oracle.decoder()
    hashes = []
    for au in aus:
        rc, pic, w, h = dec.decode(au)
        assert rc == 1 and (w, h) == (176, 144)
        hashes.append(sha(pic))
    assert len(hashes) == 3 and len(set(hashes)) == 3


OH = json.load(open(os.path.join(HERE, 'golden', 'openh264_tables.json')))


@pytest.mark.parametrize('name', sorted(OH['tables']))
def test_openh264_tables_pinned(oracle, name):
    """The oracle's OpenH264 tables (quantiser MF / FF, lambda, rate-control tables) equal the copies the
    reference's own scripts/h264.wasm holds (tools/wasm_tables.py reads them as bytes)."""
    t = OH['tables'][name]
    n = int(np.prod(t['shape']))
    buf = (ctypes.c_double * n)()
    oracle.L.h264o_table.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    assert oracle.L.h264o_table(name.encode(), buf) == n
    assert list(buf) == list(np.array(t['values'], dtype=np.float64).reshape(-1)), name


def test_openh264_rc_constants_pinned(oracle):
    """The rate-control constants the oracle applies are the immediates of the instructions the fixture
    cites (camera QP range, default frame rate, frame QP windows, IDR bit ratio, skip-buffer ratio)."""
    c = OH['code_constants']
    out = (ctypes.c_int32 * 8)()
    oracle.L.h264o_rc_constants(out)
    want = [c['default_max_frame_rate']['value'], c['camera_min_qp']['value'], c['camera_max_qp']['value'],
            c['frame_delta_qp_lower']['value'], c['frame_delta_qp_upper']['value'], c['idr_frame_qp_window']['value'],
            c['default_idr_bitrate_ratio']['value'], c['skip_buffer_ratio']['value']]
    assert list(out) == want


def idr_params_from_fixture(w, h, br):
    """RcCalculateIdrQp (h264.wasm func 1226) restated in Python from the fixture alone: the oracle's C
    restatement must agree with it for every geometry / bitrate."""
    t, c = OH['tables'], OH['code_constants']
    fps = np.float32(c['default_max_frame_rate']['value'])
    bpp = br / float(np.float32(np.float32(fps * np.float32(w)) * np.float32(h)))
    area = w * h
    cls = 0 if area < c['area_90p']['value'] else 1 if area < c['area_180p']['value'] else 2 if area < c['area_360p']['value'] else 3
    i = 1 - c['default_fix_rc_overshoot']['value']
    while i < 4 and not t['rc_bpp']['values'][cls][i] >= bpp:
        i += 1
    lo, hi = c['camera_min_qp']['value'], c['camera_max_qp']['value']
    mx, mn = (min(max(v, lo), hi) for v in t['rc_qp_range']['values'][i])
    return min(max(t['rc_init_qp']['values'][cls][i], mn), mx), mn, mx


@pytest.mark.parametrize('w,h', [(176, 144), (352, 288), (640, 360), (1280, 720), (1920, 1080), (208, 120), (3840, 2160)])
@pytest.mark.parametrize('br', [100000, 300000, 1000000, 2000000, 8000000, 30000000, 200000000])
def test_rc_idr_qp_vs_fixture(oracle, w, h, br):
    a, b = ctypes.c_int(), ctypes.c_int()
    oracle.L.h264o_rc_idr_params.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    q = oracle.L.h264o_rc_idr_params(w, h, br, ctypes.byref(a), ctypes.byref(b))
    assert (q, a.value, b.value) == idr_params_from_fixture(w, h, br)


def test_rc_idr_qp_known_points(oracle):
    """the wrapper's operating points (1 Mbps, encoder_worker.js:96) and the 8 Mbps bench line"""
    L = oracle.L
    assert L.h264o_rc_init_qp(1920, 1080, 1000000) == 36
    assert L.h264o_rc_init_qp(1280, 720, 1000000) == 34
    assert L.h264o_rc_init_qp(1280, 720, 8000000) == 28
    assert L.h264o_rc_init_qp(176, 144, 300000) == 34


def test_rc_update_direction(oracle):
    """the step on the last frame's bits (this project's rule), inside OpenH264's camera range [12, 42]"""
    L = oracle.L
    br = 1000000
    target = br // 60
    assert L.h264o_rc_next_qp(30, 10 * target, br, 0) > 30
    assert L.h264o_rc_next_qp(30, target // 10, br, 0) < 30
    assert L.h264o_rc_next_qp(42, 100 * target, br, 0) == 42
    assert L.h264o_rc_next_qp(12, 0, br, 0) == 12


def test_rc_row_plan(oracle):
    """MB-row (GOM) QP plan: rows costlier than the mean get +1 / +2, cheap rows -1"""
    f = oracle.L.h264o_rc_row_delta
    f.argtypes = [ctypes.c_int64, ctypes.c_int64]
    assert [f(b, 1000) for b in (0, 499, 500, 1000, 1250, 1251, 2000, 2001)] == [-1, -1, 0, 0, 0, 1, 1, 2]
    assert f(5, 0) == 0


def test_frame_skip_and_row_qp_in_stream(oracle):
    """at a bitrate far below the content's cost, non-IDR frames are skipped (0 bytes) while the
    virtual buffer holds more than half a second of bits; coded P frames carry mb_qp_delta != 0
    (per-row QPs) and still decode to the encoder's reconstruction; with skipping off every frame
    is coded"""
    from h264mi.synth import SyntheticStream
    w, h = 352, 288
    g = SyntheticStream(2, w, h)
    frames = [np.ascontiguousarray(g.frame(t)) for t in range(10)]
    oe, od = oracle.encoder(w, h, 200000), oracle.decoder()
    sizes, qps_seen = [], set()
    for f in frames:
        nal = oe.encode(f)
        sizes.append(len(nal))
        if nal:
            rc, pic, _, _ = od.decode(nal)
            assert rc == 1 and np.array_equal(pic, oe.recon())
            mi = np.zeros((w // 16) * (h // 16) * 8, np.int32)
            oracle.L.h264o_dec_mbinfo(od.d, mi.ctypes.data)
            qps_seen |= set(mi.reshape(-1, 8)[:, 1].tolist())
    assert sizes[0] > 0 and 0 in sizes and oracle.L.h264o_enc_frames_skipped(oe.e) == sizes.count(0)
    assert len(qps_seen) > 1, qps_seen   # more than one QPY within pictures: mb_qp_delta was coded
    oe2 = oracle.encoder(w, h, 200000)
    oracle.L.h264o_enc_set_frame_skip(oe2.e, 0)
    assert all(len(oe2.encode(f)) > 0 for f in frames)


def test_motion_search_stages_exercised(oracle):
    """the fixture workloads reach every integer-search stage the GPU is held bit-exact on: start
    points won by a neighbour's vector, cross searches, and cross searches that move the vector"""
    from h264mi.synth import SyntheticStream
    tot = np.zeros(3, np.int64)
    for sid, (w, h, br) in enumerate([(352, 288, 2000000), (640, 360, 1000000), (352, 288, 30000000)]):
        g = SyntheticStream(sid, w, h)
        oe = oracle.encoder(w, h, br)
        oe.set_frame_skip(False)
        for t in range(5):
            oe.encode(np.ascontiguousarray(g.frame(t)))
        st = np.zeros(3, np.int32)
        oracle.L.h264o_enc_me_stats(oe.e, st.ctypes.data)
        tot += st
    assert (tot > 0).all(), tot


def test_parameter_sets_are_baseline(oracle):
    buf = np.zeros(64, np.uint8)
    n = oracle.L.h264o_write_sps(1920, 1080, buf.ctypes.data)
    sps = bytes(buf[:n])
    assert sps[:5] == b'\x00\x00\x00\x01\x67'   # 4-byte start code, nal_ref_idc 3, SPS
    assert sps[5] == 66                          # profile_idc Baseline
    n = oracle.L.h264o_write_pps(buf.ctypes.data)
    assert bytes(buf[:5]) == b'\x00\x00\x00\x01\x68'
