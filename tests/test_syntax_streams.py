"""CPU: the full-syntax test-stream generator (tests/streamgen.py SyntaxGen) against the oracle
decoder. Every macroblock the generator writes -- P_L0_16x16 / 16x8 / 8x16, P_8x8 with all four
sub_mb_types, P_Skip runs, I_NxN, I_16x16, I_PCM, mb_qp_delta across its whole range -- is parsed by
the oracle with the same type, QPY and coded_block_pattern (h264o_dec_mbinfo), under cropping,
non-zero chroma_qp_index_offset, deblocking offsets / idc 2, num_ref_idx_active_override and a
ref_pic_list_modification. These streams are what tests/test_gpu_syntax.py decodes on the GPU."""
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, 'oracle', 'build', 'libh264_oracle.so')

CASES = [  # (mbw, mbh, crop_right, crop_bottom, chroma_qp_index_offset, pic_init_qp, seed)
    (11, 9, 0, 0, 0, 26, 1),
    (11, 9, 4, 2, -7, 20, 2),
    (11, 9, 0, 0, 12, 34, 3),
    (5, 3, 2, 0, -12, 8, 4),
]
SLICES = [dict(), dict(qp_delta=4, dbk=(0, 3, -2), override=True), dict(qp_delta=-9, dbk=(2, -6, 6), reorder=True),
          dict(dbk=(1, 0, 0), override=True, reorder=True)]


def _stream(oracle, case):
    from streamgen import SyntaxGen
    mbw, mbh, cr, cb, cqp, iqp, seed = case
    g = SyntaxGen(SO, mbw, mbh, seed, crop_right=cr, crop_bottom=cb, cqp=cqp, init_qp=iqp)
    units, logs = [g.idr()], []
    logs.append(g.log)
    for kw in SLICES:
        units.append(g.p(**kw))
        logs.append(g.log)
    return units, logs


@pytest.mark.parametrize('case', CASES, ids=[f'{c[0]}x{c[1]}_crop{c[2]}{c[3]}_cqp{c[4]}' for c in CASES])
def test_oracle_parses_every_generated_macroblock(oracle, case):
    units, logs = _stream(oracle, case)
    d = oracle.decoder()
    mbw, mbh = case[0], case[1]
    seen_types, wraps = set(), 0
    for k, (u, log) in enumerate(zip(units, logs)):
        rc, pic, w, h = d.decode(u)
        assert rc == 1, f'unit {k}'
        assert (w, h) == (mbw * 16 - 2 * case[2], mbh * 16 - 2 * case[3])
        mi = np.zeros(mbw * mbh * 8, np.int32)
        oracle.L.h264o_dec_mbinfo(d.d, mi.ctypes.data)
        got = [tuple(int(x) for x in r[:3]) for r in mi.reshape(-1, 8)]
        assert got == log, f'unit {k}: first mismatch at MB {next(i for i, (a, b) in enumerate(zip(got, log)) if a != b)}'
        seen_types |= {t for t, _, _ in log}
        wraps += sum(1 for a, b in zip(log, log[1:]) if abs(a[1] - b[1]) > 26)
    if mbw * mbh >= 99:
        assert seen_types == {0, 1, 2, 3, 4, 5, 6, 7}, seen_types   # every mb type class
        assert wraps > 0                                             # QP wrapped across 0 / 51


@pytest.mark.parametrize('poc', [(1, 0), (1, 1), (2, 0)], ids=['poc1', 'poc1_always_zero', 'poc2'])
def test_oracle_poc_types(oracle, poc):
    """POC types 1 (with and without delta_pic_order_always_zero_flag) and 2: the slice header's POC
    fields are parsed by the SPS's rules, every macroblock as generated"""
    from streamgen import SyntaxGen
    g = SyntaxGen(SO, 11, 9, 7, poc_type=poc[0], dpoaz=poc[1])
    d = oracle.decoder()
    units = []
    for k in range(3):
        units.append(((g.idr() if k == 0 else g.p()), g.log))
    for k, (u, log) in enumerate(units):
        rc, _, _, _ = d.decode(u)
        assert rc == 1, f'unit {k}'
        mi = np.zeros(11 * 9 * 8, np.int32)
        oracle.L.h264o_dec_mbinfo(d.d, mi.ctypes.data)
        assert [tuple(int(x) for x in r[:3]) for r in mi.reshape(-1, 8)] == log, f'unit {k}'


def test_oracle_non_reference_picture(oracle):
    """nal_ref_idc 0 (a non-reference P picture): decoded and output, without dec_ref_pic_marking(), and
    not used as the next P picture's reference: the P picture after it decodes to the same
    samples whether or not the non-reference picture was decoded first"""
    from streamgen import SyntaxGen
    g = SyntaxGen(SO, 11, 9, 8)
    idr, pn, p2 = g.idr(), g.p(ref_idc=0), g.p()
    a, b = oracle.decoder(), oracle.decoder()
    assert a.decode(idr)[0] == 1 and b.decode(idr)[0] == 1
    rc, pic_n, _, _ = a.decode(pn)
    assert rc == 1
    ra, pa, _, _ = a.decode(p2)
    rb, pb, _, _ = b.decode(p2)
    assert ra == rb == 1 and np.array_equal(pa, pb)
    assert not np.array_equal(pic_n, pa)


# slice layouts (first_mb_in_slice of each slice, per-slice overrides) for an 11 x 9 picture: slices that
# start mid-row (the top-left / top-right neighbours of their second row lie in the previous slice),
# several slices in one row, a one-MB slice, I slices inside a P picture, disable_deblocking_filter_idc
# 0 / 1 / 2 per slice with different offsets and QPs
MULTI = [
    [dict(first=0), dict(first=37)],
    [dict(first=0, dbk=(2, 2, -2)), dict(first=5, qp_delta=3, dbk=(0, -4, 4)), dict(first=16, intra=True, dbk=(2, 0, 0)),
     dict(first=17), dict(first=60, qp_delta=-6, dbk=(1, 0, 0)), dict(first=98)],
    [dict(first=k) for k in range(0, 99, 7)],
]


def _multi_units(seed, layout, mbw=11, mbh=9):
    from streamgen import SyntaxGen
    g = SyntaxGen(SO, mbw, mbh, seed)
    units = [(g.idr(slices=layout), g.log)]
    for _ in range(3):
        units.append((g.p(slices=layout), g.log))
    return g, units


@pytest.mark.parametrize('layout', range(len(MULTI)))
def test_oracle_multislice_pictures(oracle, layout):
    """multi-slice IDR and P pictures (f4): every macroblock parses as generated -- CAVLC contexts, intra
    mode prediction and P_Skip / motion vector prediction use neighbours of the same slice only -- and
    the pictures decode (all macroblocks covered exactly once)"""
    _, units = _multi_units(20 + layout, MULTI[layout])
    d = oracle.decoder()
    for k, (u, log) in enumerate(units):
        rc, _, _, _ = d.decode(u)
        assert rc == 1, f'unit {k}'
        mi = np.zeros(11 * 9 * 8, np.int32)
        oracle.L.h264o_dec_mbinfo(d.d, mi.ctypes.data)
        assert [tuple(int(x) for x in r[:3]) for r in mi.reshape(-1, 8)] == log, f'unit {k}'


def _split_nals(au):
    starts = [k for k in range(len(au) - 3) if au[k:k + 4] == b'\x00\x00\x00\x01']
    return [au[a:b] for a, b in zip(starts, starts[1:] + [len(au)])]


def test_oracle_arbitrary_slice_order(oracle):
    """the slices of a picture in any order (ASO, allowed in Baseline) decode to the same picture"""
    _, units = _multi_units(31, MULTI[1])
    fwd, rev = oracle.decoder(), oracle.decoder()
    for k, (u, _) in enumerate(units):
        nals = _split_nals(u)
        head = [n for n in nals if n[4] & 31 in (7, 8)]
        sl = [n for n in nals if n[4] & 31 in (1, 5)]
        r1, p1, _, _ = fwd.decode(u)
        r2, p2, _, _ = rev.decode(b''.join(head + sl[::-1]))
        assert r1 == r2 == 1 and np.array_equal(p1, p2), f'unit {k}'


def test_oracle_incomplete_or_overlapping_picture_concealed(oracle):
    """a picture with a slice missing, or with a slice repeated, is damaged: concealed by the last
    picture (frame copy, rc 2), which stays the reference"""
    _, units = _multi_units(32, MULTI[0])
    d = oracle.decoder()
    rc, ref_pic, _, _ = d.decode(units[0][0])
    assert rc == 1
    sl = _split_nals(units[1][0])
    rc, pic, _, _ = d.decode(sl[0])                    # second slice missing
    assert rc == 2 and np.array_equal(pic, ref_pic)
    rc, pic, _, _ = d.decode(sl[0] + sl[0] + sl[1])    # first slice twice
    assert rc == 2 and np.array_equal(pic, ref_pic)
    rc, _, _, _ = d.decode(units[1][0])                # the complete picture still decodes on the IDR
    assert rc == 1
