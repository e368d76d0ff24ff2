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


def test_rc_init_qp_thresholds(oracle):
    """frame-level RC: initial QP from bits per pixel thresholds"""
    L = oracle.L
    qps = [L.h264o_rc_init_qp(1920, 1080, br) for br in (100000, 1000000, 8000000, 30000000, 200000000)]
    assert all(12 <= q <= 51 for q in qps)
    assert qps == sorted(qps, reverse=True)  # more bits -> lower QP


def test_rc_update_direction(oracle):
    L = oracle.L
    br = 1000000
    target = br // 30
    assert L.h264o_rc_next_qp(30, 10 * target, br, 0) > 30
    assert L.h264o_rc_next_qp(30, target // 10, br, 0) < 30
    assert L.h264o_rc_next_qp(51, 100 * target, br, 0) == 51
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
    oe, od = oracle.encoder(w, h, 60000), oracle.decoder()
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
    oe2 = oracle.encoder(w, h, 60000)
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
