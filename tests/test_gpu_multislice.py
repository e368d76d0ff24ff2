"""GPU: multi-slice pictures. DecodeFrameNoDelay (openh264_wrapper.cpp:407, :435)
decodes any Baseline picture the glue hands it (scripts/decoder_worker.js:179, 189), not only the
wrapper encoder's single-slice ones: pictures of several slices -- starting mid-row, several per row,
one-MB slices, I slices inside P pictures, per-slice QP and disable_deblocking_filter_idc 0 / 1 / 2 with
different filter offsets -- in stream order and in arbitrary slice order (ASO), at QCIF-like and 1080p
sizes, through the C-ABI (a slot decoder parses a picture's slices on 8 concurrent waves) and the batch
decoder with 1 and 4 slice waves per picture. Every picture == the oracle decoder's
(tests/test_syntax_streams.py pins the streams' syntax against the oracle's parse); a picture with a
slice missing or repeated is concealed (no picture at the C-ABI, 0 x 0) and the stream decodes on."""
import numpy as np
import pytest

from test_gpu_decoder import gpu_decode
from test_syntax_streams import MULTI, SO, _multi_units, _split_nals

pytestmark = pytest.mark.gpu


def _reorder(u):
    nals = _split_nals(u)
    return b''.join([n for n in nals if n[4] & 31 in (7, 8)] + [n for n in nals if n[4] & 31 in (1, 5)][::-1])


@pytest.mark.parametrize('aso', [False, True], ids=['in-order', 'reversed'])
@pytest.mark.parametrize('layout', range(len(MULTI)))
def test_multislice_capi_vs_oracle(gpu_lib, oracle, layout, aso):
    _, units = _multi_units(20 + layout, MULTI[layout])
    od = oracle.decoder()
    L = gpu_lib
    assert L.init_decoder(15) == 0
    for k, (u, _) in enumerate(units):
        if aso:
            u = _reorder(u)
        rc, pic, _, _ = od.decode(u)
        assert rc == 1
        gw, gh, got = gpu_decode(L, 15, u, 176, 144)
        assert (gw, gh) == (176, 144) and np.array_equal(got, pic), f'unit {k}: {int(np.count_nonzero(got != pic))} samples differ'
    L.deinit_decoder(15)


def test_multislice_damaged_pictures_concealed(gpu_lib, oracle):
    _, units = _multi_units(32, MULTI[0])
    od = oracle.decoder()
    L = gpu_lib
    assert L.init_decoder(16) == 0
    u0 = units[0][0]
    assert od.decode(u0)[0] == 1
    gw, gh, got0 = gpu_decode(L, 16, u0, 176, 144)
    assert (gw, gh) == (176, 144)
    sl = _split_nals(units[1][0])
    for bad in (sl[0], sl[0] + sl[0] + sl[1]):  # a slice missing; a slice twice
        rc, _, _, _ = od.decode(bad)
        assert rc == 2
        gw, gh, _ = gpu_decode(L, 16, bad, 176, 144)
        assert (gw, gh) == (0, 0)
    rc, pic, _, _ = od.decode(units[1][0])
    gw, gh, got = gpu_decode(L, 16, units[1][0], 176, 144)
    assert rc == 1 and (gw, gh) == (176, 144) and np.array_equal(got, pic)
    L.deinit_decoder(16)


def _layout_1080p():
    # 8160 MBs: slices of uneven length, mostly starting mid-row, one I slice, idc 2 on some
    firsts = [0, 50, 1000, 1001, 2345, 4100, 4219, 6000, 7777, 8159]
    out = []
    for i, f in enumerate(firsts):
        d = dict(first=f)
        if i % 3 == 1:
            d['dbk'] = (2, (i % 5) - 2, 2 - (i % 5))
        if i == 4:
            d['intra'] = True
        if i % 4 == 2:
            d['qp_delta'] = -3
        out.append(d)
    return out


@pytest.mark.parametrize('waves', [1, 4])
def test_multislice_1080p_batch_and_capi(gpu_lib, oracle, waves):
    """1920x1080 (cropped from 1088) multi-slice IDR + 2 P pictures: the C-ABI decoder and the batch
    decoder (waves slice waves per picture, both P pictures in one call) == the oracle"""
    import torch
    import h264mi
    from streamgen import SyntaxGen
    g = SyntaxGen(SO, 120, 68, seed=41 + waves, crop_bottom=4, cqp=-2, init_qp=28)
    lay = _layout_1080p()
    units = [g.idr(slices=lay), g.p(slices=lay), g.p(slices=lay, order=list(range(len(lay)))[::-1])]
    od = oracle.decoder()
    pics = []
    for u in units:
        rc, pic, _, _ = od.decode(u)
        assert rc == 1
        pics.append(pic)
    L = gpu_lib
    assert L.init_decoder(17) == 0
    for k, u in enumerate(units):
        gw, gh, got = gpu_decode(L, 17, u, 1920, 1080)
        assert (gw, gh) == (1920, 1080) and np.array_equal(got, pics[k]), f'C-ABI unit {k}'
    L.deinit_decoder(17)
    dec = h264mi.BatchDecoder(1920, 1080, 1, max_frames=2)
    dec.set_slice_waves(waves)
    dev = [torch.from_numpy(np.frombuffer(u, np.uint8).copy()).cuda() for u in units]
    out = torch.zeros((3, 1920 * 1080 * 3 // 2), dtype=torch.uint8, device='cuda')
    dec.decode_frames([dev[0].data_ptr()], nal_sizes=[len(units[0])], out_ptrs=[out[0].data_ptr()])
    dec.decode_frames([dev[1].data_ptr(), dev[2].data_ptr()], nal_sizes=[len(units[1]), len(units[2])],
                      out_ptrs=[out[1].data_ptr(), out[2].data_ptr()])
    rc, got = dec.status()
    assert rc == 0 and got == [1]
    host = out.cpu().numpy()
    for k in range(3):
        assert np.array_equal(host[k], pics[k]), f'batch unit {k}'
    dec.close()
