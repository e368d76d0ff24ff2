"""GPU: the decoder on streams that carry the whole Baseline macroblock-layer syntax an OpenH264
stream can contain (openh264_wrapper.cpp:407, :435 hand DecodeFrameNoDelay any such stream), not only
what this project's encoder emits: P_L0_16x16 / 16x8 / 8x16, P_8x8 with every sub_mb_type, P_Skip,
I_NxN, I_16x16, I_PCM, mb_qp_delta over its whole range with wrap-around, coded residuals of every
block class (escape-coded levels at low QP), cropping, chroma_qp_index_offset != 0, deblocking
offsets and idc 2, num_ref_idx_active_override and ref_pic_list_modification (tests/streamgen.py
SyntaxGen; tests/test_syntax_streams.py pins the streams' syntax against the oracle's parse).
Every picture == the oracle decoder's picture, through the C-ABI and through the batch decoder.

Also BASELINE.json configs[3] (1920x1080 decode-only, 8 concurrent decoders): 8 decoder instances
of one oracle-encoded 1080p stream, 16 frames, each picture == the oracle's; and the app.js fan-out
of one GPU-encoded 1080p stream to 8 decoders through the device NAL ring."""
import os

import numpy as np
import pytest

from test_gpu_decoder import gpu_decode
from test_syntax_streams import CASES, SLICES, SO

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('case', CASES, ids=[f'{c[0]}x{c[1]}_crop{c[2]}{c[3]}_cqp{c[4]}' for c in CASES])
def test_full_syntax_vs_oracle(gpu_lib, oracle, case):
    from test_syntax_streams import _stream
    units, _ = _stream(oracle, case)
    od = oracle.decoder()
    L = gpu_lib
    assert L.init_decoder(12) == 0
    w, h = case[0] * 16 - 2 * case[2], case[1] * 16 - 2 * case[3]
    for k, u in enumerate(units):
        rc, pic, _, _ = od.decode(u)
        assert rc == 1
        for rgba in (False,):
            gw, gh, got = gpu_decode(L, 12, u, w, h, rgba=rgba)
            assert (gw, gh) == (w, h), f'unit {k}'
            assert np.array_equal(got, pic), f'unit {k}: {int(np.count_nonzero(got != pic))} samples differ'
    L.deinit_decoder(12)


@pytest.mark.parametrize('poc', [(1, 0), (1, 1), (2, 0)], ids=['poc1', 'poc1_always_zero', 'poc2'])
def test_poc_types_and_non_reference_vs_oracle(gpu_lib, oracle, poc):
    """POC types 1 and 2 (the slice header's POC fields by the SPS's rules): every picture == the
    oracle's; non-reference P pictures (nal_ref_idc 0, no dec_ref_pic_marking) are decoded and output
    but do not become the reference -- the P picture after them predicts from the last reference
    picture, two non-reference pictures in a row included"""
    from streamgen import SyntaxGen
    g = SyntaxGen(SO, 11, 9, 21, poc_type=poc[0], dpoaz=poc[1])
    units = [g.idr(), g.p(), g.p(ref_idc=0), g.p(), g.p(ref_idc=0), g.p(ref_idc=0), g.p()]
    od = oracle.decoder()
    L = gpu_lib
    assert L.init_decoder(14) == 0
    for k, u in enumerate(units):
        rc, pic, _, _ = od.decode(u)
        gw, gh, got = gpu_decode(L, 14, u, 176, 144)
        assert rc == 1 and (gw, gh) == (176, 144) and np.array_equal(got, pic), f'unit {k}'
    L.deinit_decoder(14)


def test_full_syntax_1080p_vs_oracle(gpu_lib, oracle):
    """the same syntax at 1920x1080 (cropped from 1088), chroma_qp_index_offset 3: IDR + 2 P pictures,
    through the C-ABI (one frame per call) and the frame-batched decoder (both P frames in one call)"""
    import torch
    import h264mi
    from streamgen import SyntaxGen
    g = SyntaxGen(SO, 120, 68, seed=11, crop_bottom=4, cqp=3, init_qp=24)
    units = [g.idr(), g.p(dbk=(0, -2, 3), override=True), g.p(qp_delta=5, dbk=(2, 1, -1), reorder=True)]
    od = oracle.decoder()
    pics = []
    for u in units:
        rc, pic, _, _ = od.decode(u)
        assert rc == 1
        pics.append(pic)
    L = gpu_lib
    assert L.init_decoder(13) == 0
    for k, u in enumerate(units):
        gw, gh, got = gpu_decode(L, 13, u, 1920, 1080)
        assert (gw, gh) == (1920, 1080) and np.array_equal(got, pics[k]), f'C-ABI unit {k}'
    L.deinit_decoder(13)
    dec = h264mi.BatchDecoder(1920, 1080, 1, max_frames=2)
    dev = [torch.from_numpy(np.frombuffer(u, np.uint8).copy()).cuda() for u in units]
    dec.decode_frames([dev[0].data_ptr()], nal_sizes=[len(units[0])])
    dec.decode_frames([dev[1].data_ptr(), dev[2].data_ptr()], nal_sizes=[len(units[1]), len(units[2])])
    rc, got = dec.status()
    assert rc == 0 and got == [1]
    assert dec.picture_i420(0) == pics[2].tobytes()
    dec.close()


def _oracle_1080p_stream(oracle, nf, br=1000000, sid=0):
    from h264mi.synth import SyntheticStream
    g = SyntheticStream(sid, 1920, 1080)
    oe, od = oracle.encoder(1920, 1080, br), oracle.decoder()
    oe.set_frame_skip(False)  # every frame coded (at 1 Mbps this content would overflow the RC buffer)
    units, pics = [], []
    for t in range(nf):
        u = oe.encode(np.ascontiguousarray(g.frame(t)))
        rc, pic, _, _ = od.decode(u)
        assert rc == 1
        units.append(u)
        pics.append(hash_pic(pic.tobytes()))
    return units, pics


def hash_pic(b):
    import hashlib
    return hashlib.sha256(b).hexdigest()


def test_config4_eight_concurrent_1080p_decoders(gpu_lib, oracle):
    """BASELINE.json configs[3]: one 1080p IPPP stream (oracle-encoded, 16 frames) decoded by 8
    concurrent decoder instances on one GPU (one batch decoder of 8 streams, 4 frames per call);
    after every call each decoder's picture == the oracle's picture of that frame"""
    import torch
    import h264mi
    nf, S, G = 16, 8, 4
    units, pics = _oracle_1080p_stream(oracle, nf)
    dev = [torch.from_numpy(np.frombuffer(u, np.uint8).copy()).cuda() for u in units]
    sizes = [torch.tensor([len(u)], dtype=torch.int32, device='cuda') for u in units]
    dec = h264mi.BatchDecoder(1920, 1080, S, max_frames=G)
    for t0 in range(0, nf, G):
        dec.decode_frames([dev[t].data_ptr() for t in range(t0, t0 + G) for _ in range(S)],
                          size_ptrs=[sizes[t].data_ptr() for t in range(t0, t0 + G) for _ in range(S)])
        rc, got = dec.status()
        assert rc == 0 and got == [1] * S
        for s in range(S):
            assert hash_pic(dec.picture_i420(s)) == pics[t0 + G - 1], f'decoder {s} frame {t0 + G - 1}'
    dec.close()


def test_config4_ring_fanout_1080p(gpu_lib, oracle):
    """app.js fan-out at 1080p: the GPU encoder publishes each frame once to the device NAL ring with
    ref_count 8; 8 decoders (own HIP streams) decode straight from the slot and release it; every
    picture == the oracle decoder's picture of the oracle's stream (the GPU stream is byte-identical)"""
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    nf, D = 6, 8
    units, pics = _oracle_1080p_stream(oracle, nf, sid=3)
    g = SyntheticStream(3, 1920, 1080)
    es = torch.cuda.Stream()
    dss = [torch.cuda.Stream() for _ in range(D)]
    enc = h264mi.BatchEncoder(1920, 1080, 1000000, 1, stream=es)
    enc.set_frame_skip(False)
    decs = [h264mi.BatchDecoder(1920, 1080, 1, stream=dss[k]) for k in range(D)]
    ring = h264mi.NalRing(slots=4, slot_bytes=1 << 21)
    for t in range(nf):
        f = torch.from_numpy(np.ascontiguousarray(g.frame(t))).cuda()
        torch.cuda.synchronize()
        with torch.cuda.stream(es):
            enc.encode(f)
            tk = ring.publish(enc, 0, D)
            ev = torch.cuda.Event()
            ev.record(es)
        for k in range(D):
            with torch.cuda.stream(dss[k]):
                dss[k].wait_event(ev)
                decs[k].decode_frames([ring.nal_ptr(tk)], size_ptrs=[ring.size_ptr(tk)])
                ring.release(tk, stream=dss[k])
        torch.cuda.synchronize()
        assert enc.nal_bytes(0, enc.nal_sizes()[0]) == units[t], f'frame {t}: GPU stream != oracle stream'
        for k in range(D):
            rc, got = decs[k].status()
            assert rc == 0 and got == [1]
            assert hash_pic(decs[k].picture_i420(0)) == pics[t], f'frame {t} decoder {k}'
    st = ring.stats()
    assert (st['published'], st['dropped_busy'], st['dropped_size']) == (nf, 0, 0)
    assert st['ref_counts'] == [0] * 4
    for d in decs:
        d.close()
    ring.close()
    enc.close()


# macroblock contents that steer the asm P-slice run (cavlc_blk.inc p_mb_run) down each of its paths:
# mix, fixed coded_block_pattern, TotalCoeff choices of the generated blocks
ASM_KINDS = [
    ('skip', {'skip': 1}, None, None),
    ('p16_cbp0', {'p16': 1}, 0, None),
    ('p16_chroma_dc', {'p16': 1}, 0x10, [0, 1, 2, 3, 4]),
    ('p16_chroma_quiet', {'p16': 1}, 0x20, [0, 0, 0, 1]),      # quiet planes: empty blocks, tc 1 (short / long total_zeros)
    ('p16_chroma_mixed', {'p16': 1}, 0x20, [0, 1, 2]),         # quiet planes that bail out, generic planes
    ('p16_luma_dense', {'p16': 1}, 0x2f, [2, 4, 6, 16]),
    ('p16_skip_i16', {'p16': 3, 'skip': 2, 'i16': 1}, None, None),  # runs, I_16x16 in P slices (DC + AC blocks)
    ('p16_other_types', {'p16': 3, 'p16x8': 1, 'p8x8': 1, 'i4': 1, 'pcm': 0.3}, None, None),  # exits to the C++ loop
]


@pytest.mark.parametrize('kind', ASM_KINDS, ids=[k[0] for k in ASM_KINDS])
def test_asm_p_run_paths_vs_oracle(gpu_lib, oracle, kind):
    """P slices of one macroblock content each (CIF, IDR + 3 P pictures): every picture == the oracle
    decoder's, through the C-ABI"""
    from streamgen import SyntaxGen
    name, mix, cbp, tcs = kind
    g = SyntaxGen(SO, 22, 18, 31 + len(name))
    g.tc_choice = tcs
    units = [g.idr()] + [g.p(mix, cbp_fixed=cbp) for _ in range(3)]
    od = oracle.decoder()
    L = gpu_lib
    assert L.init_decoder(15) == 0
    for k, u in enumerate(units):
        rc, pic, _, _ = od.decode(u)
        assert rc == 1
        gw, gh, got = gpu_decode(L, 15, u, 352, 288)
        assert (gw, gh) == (352, 288) and np.array_equal(got, pic), f'{name} unit {k}'
    L.deinit_decoder(15)
