"""GPU: BASELINE.json configs at their stated spans and both bitrates (configs 2 and 3
"1 Mbps and 8 Mbps"; the glue's own bitrate is 1 Mbps, scripts/encoder_worker.js:96), frame by frame
against the oracle through the C-ABI the reference's glue binds (init_encoder / force_key_frame /
encode_frame_yuv_i420 / init_decoder / decode_frame_yuv_i420, openh264_wrapper.cpp:198-464), plus the
config-4 fan-out with EVERY frame's picture checked (batched calls carry 4 frames).

Parity is with the oracle (the CPU restatement); OpenH264 parity is unpinned."""
import ctypes
import os
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _enc(L, f, w, h):
    p = ctypes.POINTER(ctypes.c_ubyte)()
    sz = ctypes.c_int(0)
    L.encode_frame_yuv_i420(f.ctypes.data, w, h, ctypes.byref(p), ctypes.byref(sz))
    return ctypes.string_at(p, sz.value) if sz.value > 0 else b''


def _dec(L, idx, nal, w, h, out):
    a = np.frombuffer(nal, np.uint8).copy()
    gw, gh = ctypes.c_int(-1), ctypes.c_int(-1)
    L.decode_frame_yuv_i420(idx, a.ctypes.data, len(nal), out.ctypes.data, ctypes.byref(gw), ctypes.byref(gh))
    return gw.value, gh.value


def _run_capi(L, oracle, w, h, br, nf, i_only, sid=0):
    """encode nf frames through the C-ABI and the oracle (same synthetic input), decode every coded
    frame through the C-ABI decoder and the oracle decoder; returns (sizes, qps)"""
    from h264mi.synth import SyntheticStream
    g = SyntheticStream(sid, w, h)
    assert L.init_encoder(w, h, br) == 0
    assert L.init_decoder(0) == 0
    oe, od = oracle.encoder(w, h, br), oracle.decoder()
    out = np.zeros(w * h * 3 // 2, np.uint8)
    sizes, qps = [], []
    for t in range(nf):
        f = np.ascontiguousarray(g.frame(t))
        if i_only:
            L.force_key_frame()
            oe.force_idr()
        got, ref = _enc(L, f, w, h), oe.encode(f)
        assert got == ref, f'{w}x{h} {br} bps frame {t}: GPU {len(got)} B vs oracle {len(ref)} B'
        sizes.append(len(ref))
        qps.append(oe.last_qp())
        if not ref:
            continue
        rc, pic, ow, oh = od.decode(ref)
        assert rc == 1
        gw, gh = _dec(L, 0, got, w, h, out)
        assert (gw, gh) == (ow, oh) == (w, h), f'frame {t}: decoded {gw}x{gh}'
        assert np.array_equal(out, pic), f'{w}x{h} {br} bps frame {t}: GPU picture != oracle picture'
    L.deinit_decoder(0)
    return sizes, qps


def test_config3_1080p_ippp_8mbps_60_frames(gpu_lib, oracle):
    """configs[2] at its stated span (60 frames IPPP, 1 IDR + 59 P) at 8 Mbps (frame
    skipping on, as the wrapper's encoder): NAL bytes and decoded pictures == oracle frame by frame, with
    the QP inside OpenH264's camera range [12, 42] and the IDR at the table QP"""
    sizes, qps = _run_capi(gpu_lib, oracle, 1920, 1080, 8000000, 60, False)
    # the IDR (~490 KB at QP 30) fills the skip buffer (bitrate / 2, drained bitrate / 60 per frame): the
    # rate control drops some P frames after it, then codes the rest (GPU == oracle, skips included)
    assert sum(1 for n in sizes[1:] if n > 0) >= 10, sizes  # P frames really coded
    assert qps[0] == 30 and max(qps) <= 42, qps


def test_config3_1080p_ippp_1mbps_rc_skipping(gpu_lib, oracle):
    """configs[2] at its 60-frame span and the glue's 1 Mbps with the wrapper's frame skipping (OpenH264's
    RC_BITRATE_MODE restated from h264.wasm): the IDR overfills the skip buffer, frames are
    skipped (0-byte access units) until the cap on the run of skipped frames -- (round(fullness / bits per frame)
    + 1) >> 1 >= the run, CheckFrameSkipBasedMaxbr -- forces a P frame through at frame 40. GPU == oracle frame
    by frame, the skips and the forced P frame included; every coded frame decodes to the oracle's picture."""
    sizes, qps = _run_capi(gpu_lib, oracle, 1920, 1080, 1000000, 60, False)
    assert qps[0] == 36, qps  # RcCalculateIdrQp at 1 Mbps, 60 fps default: bpp 0.008 -> QP 36 in [28, 40]
    assert sizes[0] > 0 and all(n == 0 for n in sizes[1:40]) and sizes[40] > 0, sizes
    assert qps[40] == 36  # the first P frame takes the IDR's QP (RcCalculatePictureQp, iPFrameNum 0)


def test_rc_state_batch_vs_oracle(gpu_lib, oracle):
    """the device rate control's whole state (skip decision, QP and window, target and remaining bits, buffer
    fullness, run of skips, frame complexity, VGOP counters) == the oracle's after every frame, 1080p, two
    streams at 8 Mbps with skipping on (coded / skipped alternation after the IDR's overspend) and a forced
    IDR at frame 9 (the intra R-Q model's QP)"""
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    w, h, br, S, nf = 1920, 1080, 8000000, 2, 14
    gs = [SyntheticStream(s, w, h) for s in range(S)]
    enc = h264mi.BatchEncoder(w, h, br, S)
    oes = [oracle.encoder(w, h, br) for _ in range(S)]
    coded = 0
    for t in range(nf):
        fr = [np.ascontiguousarray(g.frame(t)) for g in gs]
        if t == 9:
            enc.force_idr()
            for oe in oes:
                oe.force_idr()
        enc.encode(torch.from_numpy(np.stack(fr)).cuda())
        n = enc.nal_sizes()
        for s in range(S):
            ref = oes[s].encode(fr[s])
            assert n[s] == len(ref) and (n[s] == 0 or enc.nal_bytes(s, n[s]) == ref), f'frame {t} stream {s}'
            assert enc.rc_state(s) == oes[s].rc_state(), f'frame {t} stream {s}'
            coded += n[s] > 0
    assert 2 * S <= coded < S * nf  # both coded and skipped frames were exercised
    enc.close()


@pytest.mark.parametrize('br', [1000000, 8000000], ids=['1mbps', '8mbps'])
def test_config2_720p_i_only_30_frames(gpu_lib, oracle, br):
    """configs[1]: 1280x720, force_key_frame before every frame (all IDR), 30 frames, 1 and 8 Mbps"""
    sizes, qps = _run_capi(gpu_lib, oracle, 1280, 720, br, 30, True)
    assert all(n > 0 for n in sizes), sizes


def test_encoder_1080p_p_frames_skip_off(gpu_lib, oracle):
    """1080p IPPP at 1 Mbps with frame skipping off (bench.py's setting): 6 frames, all coded (P frames
    included), batch encoder bytes == oracle bytes"""
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    w, h, br = 1920, 1080, 1000000
    g = SyntheticStream(0, w, h)
    enc = h264mi.BatchEncoder(w, h, br, 1)
    enc.set_frame_skip(False)
    oe = oracle.encoder(w, h, br)
    oe.set_frame_skip(False)
    for t in range(6):
        f = np.ascontiguousarray(g.frame(t))
        enc.encode(torch.from_numpy(f).cuda())
        n = enc.nal_sizes()[0]
        ref = oe.encode(f)
        assert n > 0 and enc.nal_bytes(0, n) == ref, f'frame {t}'
    enc.close()


def _oracle_stream(oracle, w, h, br, nf, sid=0):
    from h264mi.synth import SyntheticStream
    g = SyntheticStream(sid, w, h)
    oe, od = oracle.encoder(w, h, br), oracle.decoder()
    oe.set_frame_skip(False)
    units, pics = [], []
    for t in range(nf):
        u = oe.encode(np.ascontiguousarray(g.frame(t)))
        rc, pic, _, _ = od.decode(u)
        assert rc == 1
        units.append(u)
        pics.append(hashlib.sha256(pic.tobytes()).hexdigest())
    return units, pics


@pytest.mark.parametrize('br', [1000000, 8000000], ids=['1mbps', '8mbps'])
def test_config4_every_frame_8_decoders(gpu_lib, oracle, br):
    """configs[3] at its stated span: one 1080p IPPP stream of 60 frames decoded by 8 concurrent decoders,
    4 frames per call; EVERY frame's picture of every decoder (per-frame outputs of the batched call) ==
    the oracle's picture"""
    import torch
    import h264mi
    w, h, nf, S, G = 1920, 1080, 60, 8, 4
    units, pics = _oracle_stream(oracle, w, h, br, nf)
    dev = [torch.from_numpy(np.frombuffer(u, np.uint8).copy()).cuda() for u in units]
    F = w * h * 3 // 2
    out = torch.zeros((nf, S, F), dtype=torch.uint8, device='cuda')
    got = torch.full((nf, S), -1, dtype=torch.int32, device='cuda')
    dec = h264mi.BatchDecoder(w, h, S, max_frames=G)
    for t0 in range(0, nf, G):
        fr = range(t0, t0 + G)
        dec.decode_frames([dev[t].data_ptr() for t in fr for _ in range(S)], nal_sizes=[len(units[t]) for t in fr for _ in range(S)],
                          out_ptrs=[out[t, s].data_ptr() for t in fr for s in range(S)],
                          got_ptrs=[got[t, s].data_ptr() for t in fr for s in range(S)])
    rc, _ = dec.status()
    assert rc == 0
    assert got.cpu().eq(1).all()
    host = out.cpu().numpy()
    for t in range(nf):
        for s in range(S):
            assert hashlib.sha256(host[t, s].tobytes()).hexdigest() == pics[t], f'frame {t} decoder {s}'
    dec.close()


def test_capi_decoder_memory_1080p(gpu_lib, oracle):
    """a C-ABI decoder slot (one call in flight: two slot groups, one parse stream) holds well under
    64 MB at 1080p; a pipelined batch decoder's default ring is larger"""
    import h264mi
    L = gpu_lib
    inst = L.h264mi_instance_create()
    w, h = 1920, 1080
    units, _ = _oracle_stream(oracle, w, h, 8000000, 1)
    a = np.frombuffer(units[0], np.uint8).copy()
    out = np.zeros(w * h * 3 // 2, np.uint8)
    gw, gh = ctypes.c_int(), ctypes.c_int()
    L.h264mi_i_init_decoder.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.h264mi_i_decode_frame_yuv_i420.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_void_p]
    assert L.h264mi_i_init_decoder(inst, 3) == 0
    L.h264mi_i_decode_frame_yuv_i420(inst, 3, a.ctypes.data, len(a), out.ctypes.data, ctypes.byref(gw), ctypes.byref(gh))
    assert (gw.value, gh.value) == (w, h)
    capi = L.h264mi_i_decoder_device_bytes(inst, 3)
    L.h264mi_instance_destroy(inst)
    dec = h264mi.BatchDecoder(w, h, 1)
    batch = dec.device_bytes()
    dec.close()
    assert 0 < capi < 64 << 20, capi
    assert batch > capi, (batch, capi)


@pytest.mark.parametrize('w,h,br,skip,S,nf', [(1920, 1080, 8000000, False, 2, 6), (1920, 1080, 20000000, True, 2, 5),
                                              (1280, 720, 2000000, False, 2, 5), (352, 288, 500000, False, 4, 6)],
                         ids=['1080p_8m', '1080p_20m_skip', '720p_odd_gom', 'cif_narrow'])
def test_exact_gom_rc_vs_oracle(gpu_lib, oracle, w, h, br, skip, S, nf):
    """OpenH264's GOM rate control exactly (h264mi_enc_set_gom_exact; oracle h264o_enc_set_gom_exact): every P
    frame's GOM takes its QP from the bits of every MB coded before it (WelsRcMbInitGom, h264.wasm func 1215).
    GPU bytes, RC state and every GOM's {QP, slice bits before it, target bits} == oracle, GOMs of 2 MB rows (1080p, 720p whose last GOM has one row) and of 1 row
    (352x288: fewer than 31 MBs wide); the MB QPs really vary inside pictures"""
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    gs = [SyntheticStream(5 + s, w, h) for s in range(S)]
    enc = h264mi.BatchEncoder(w, h, br, S)
    enc.set_gom_exact(True)
    enc.set_frame_skip(skip)
    oes = [oracle.encoder(w, h, br) for _ in range(S)]
    od = oracle.decoder()
    qps = set()
    for oe in oes:
        oe.set_gom_exact(True)
        oe.set_frame_skip(skip)
    for t in range(nf):
        fr = [np.ascontiguousarray(g.frame(t)) for g in gs]
        enc.encode(torch.from_numpy(np.stack(fr)).cuda())
        n = enc.nal_sizes()
        for s in range(S):
            ref = oes[s].encode(fr[s])
            assert n[s] == len(ref) and (n[s] == 0 or enc.nal_bytes(s, n[s]) == ref), f'frame {t} stream {s}'
            assert enc.rc_state(s) == oes[s].rc_state(), f'frame {t} stream {s}'
            if t > 0 and ref and not enc.rc_state(s)['skipped']:  # per GOM: QP, bits before it, target, last MB
                assert enc.gom_state(s) == oes[s].gom_state(), f'frame {t} stream {s}'
            if s == 0 and ref:
                rc, _, _, _ = od.decode(ref)
                assert rc == 1
                mi = np.zeros(((w + 15) // 16) * ((h + 15) // 16) * 8, np.int32)
                oracle.L.h264o_dec_mbinfo(od.d, mi.ctypes.data)
                if t > 0:
                    qps.add(len(set(mi.reshape(-1, 8)[:, 1].tolist())))
    assert max(qps) > 1, qps
    enc.close()


@pytest.mark.parametrize('sgrp', [1, 3])
def test_stream_grouped_tickets_same_bytes(gpu_lib, sgrp):
    """enc_mb_kernel's stream-grouped ticket order (H264MI_ENC_SGRP, EncLaunch::sgrp: the streams of a per-XCD queue
    taken sgrp at a time, the last group smaller with 3) changes only when rows run: 32 streams (4 per queue) give
    the same NAL bytes and reconstructions as the default order over an IDR and P frames"""
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    w, h, S, nf = 352, 288, 32, 4
    gs = [SyntheticStream(s, w, h) for s in range(S)]
    clip = [torch.from_numpy(np.stack([np.ascontiguousarray(g.frame(t)) for g in gs])).cuda() for t in range(nf)]
    outs = []
    for v in (None, str(sgrp)):
        if v is None:
            os.environ.pop('H264MI_ENC_SGRP', None)
        else:
            os.environ['H264MI_ENC_SGRP'] = v
        try:
            enc = h264mi.BatchEncoder(w, h, 500000, S)
        finally:
            os.environ.pop('H264MI_ENC_SGRP', None)
        enc.set_frame_skip(False)
        got = []
        for t in range(nf):
            enc.encode(clip[t])
            n = enc.nal_sizes()
            got.append([enc.nal_bytes(s, n[s]) for s in range(S)])
        outs.append(got)
        enc.close()
    assert outs[0] == outs[1]


@pytest.mark.parametrize('w,h', [(16, 16), (48, 16), (16, 48), (32, 32), (80, 48), (176, 144)])
def test_intra_decision_geometries_vs_oracle(gpu_lib, oracle, w, h):
    """OpenH264's intra mode decision (the I16x16 / chroma mode orders by neighbour flags, the
    VAA gate, WelsMdI4x4Fast's fast and table paths by block availability) at picture edges: one-MB-wide and
    one-MB-high pictures (no top-right, no left or no top anywhere), every frame an IDR, content from flat to
    noise (VAA variance below and above 149) at two rates; GPU bytes == oracle bytes"""
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    rng = np.random.default_rng(w * 131 + h)
    fs = w * h * 3 // 2
    g = SyntheticStream(9, w, h)
    clips = []
    for t in range(4):
        flat = np.full(fs, 90 + 7 * t, np.uint8)
        noise = rng.integers(0, 256, fs, dtype=np.uint8)
        tex = np.ascontiguousarray(g.frame(t))
        clips.append(np.stack([flat if t == 0 else tex, noise]))
    for br in (300000, 4000000):
        enc = h264mi.BatchEncoder(w, h, br, 2)
        enc.set_frame_skip(False)
        oes = [oracle.encoder(w, h, br) for _ in range(2)]
        for oe in oes:
            oe.set_frame_skip(False)
        for t in range(4):
            enc.force_idr(-1)
            enc.encode(torch.from_numpy(clips[t]).cuda())
            n = enc.nal_sizes()
            for s in range(2):
                oes[s].force_idr()
                ref = oes[s].encode(clips[t][s])
                assert n[s] == len(ref) and enc.nal_bytes(s, n[s]) == ref, (br, t, s)
        enc.close()


def test_p_slice_decisions_16_streams_vs_oracle(gpu_lib, oracle):
    """OpenH264's P-slice decisions (the P_Skip judge, its double check, WelsMdFirstIntraMode with
    Intra4x4 MBs in P slices) on the lean encoder build with per-XCD ticket queues (16 streams of 1080p: every
    workgroup's judge accumulators, the intra MBs' early decision and top-right polls under real contention -- a
    judge word cleared while a late wave still read it diverged 1 stream in 16 here before the accumulators were
    double-buffered): NAL bytes == oracle for 3 frames, and the frames hold intra MBs in P slices"""
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    w, h, br, S = 1920, 1080, 1000000, 16
    gs = [SyntheticStream(s, w, h) for s in range(S)]
    enc = h264mi.BatchEncoder(w, h, br, S)
    enc.set_frame_skip(False)
    oes = [oracle.encoder(w, h, br) for _ in range(S)]
    for oe in oes:
        oe.set_frame_skip(False)
    for t in range(3):
        frames = np.stack([np.ascontiguousarray(g.frame(t)) for g in gs])
        enc.encode(torch.from_numpy(frames).cuda())
        n = enc.nal_sizes()
        for s in range(S):
            ref = oes[s].encode(frames[s])
            assert n[s] == len(ref) and enc.nal_bytes(s, n[s]) == ref, f'frame {t} stream {s}'
    st = np.zeros(6, np.int32)
    oracle.L.h264o_enc_me_stats(oes[0].e, st.ctypes.data)
    assert st[3] > 0 and st[5] > 0, st  # judges run, intra MBs in P slices
    enc.close()
