"""GPU: the device-resident batch API (many streams per launch, NAL units and sizes in HBM,
frame-batched decoding) -- decoder picture == encoder reconstruction for every stream, stream
bytes == oracle bytes for EVERY stream of the launch (each against its own oracle encoder), at the bench
configuration's full 1080p size."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tools'))


@pytest.mark.parametrize('args', [
    (176, 144, 300000, 2, 5, 1, 1),      # per-frame decode_dev
    (176, 144, 300000, 3, 9, 0, 1),      # per-frame decode (host sizes)
    (352, 288, 2000000, 2, 10, 1, 4),    # 4-frame batches, device sizes, ragged tail
    (208, 120, 500000, 3, 7, 0, 3),      # cropped geometry, host sizes
    (1920, 1080, 1000000, 4, 6, 1, 3),   # bench geometry
    (352, 288, 2000000, 3, 9, 1, 3, 16),    # reserved decode lane: parse on 16 masked CUs, wavefronts on the rest
    (1920, 1080, 1000000, 4, 6, 1, 2, 16),  # the same at the bench geometry
    (1920, 1080, 1000000, 32, 3, 1, 3, 32),  # the bench's own launch: 32 streams, 32 parse CUs, every stream vs its oracle
    (176, 144, 300000, 2, 5, 1, 1, 0, 0),      # reconstruction after the parse launch (streamed off)
    (1920, 1080, 1000000, 4, 6, 1, 2, 16, 0),  # reserved decode lane, streamed off
    (1920, 1080, 1000000, 2, 5, 1, 1, 0, 1),   # streamed forced without a reserved lane (2 streams: few waves wait)
    # the bench's timed regime (frames 5..24 incl. the frame-22 scene change): 4 streams x 25 frames, 1080p, 1 Mbps, skipping
    # off, 4-frame calls on the reserved lane; bytes == oracle and decoded picture == oracle reconstruction, every frame
    (1920, 1080, 1000000, 4, 25, 1, 4, 16, None, 1),
], ids=['qcif-dev', 'qcif-host', 'cif-batch4', 'crop-batch3', '1080p-batch3', 'cif-lanes16', '1080p-lanes16', '1080p-s32-lanes32',
        'qcif-unstreamed', '1080p-lanes16-unstreamed', '1080p-streamed-forced', '1080p-s4-25frames-bench-window'])
def test_batch_encode_decode(gpu_lib, args):
    """streamed reconstruction (the first frame of each call row by row behind its slice data) is on in
    the lanes cases and wherever the library's automatic choice takes it; the *-unstreamed cases pin the
    launch-after-parse order"""
    import batch_check
    assert batch_check.main(*args)


def test_color_host_entry_points(gpu_lib, oracle):
    import ctypes
    from golden.make_golden import rgba_frame
    L = gpu_lib
    for w, h in ((64, 48), (1920, 1080)):
        rgba = rgba_frame(w, h, 3)
        out = np.zeros(w * h * 3 // 2, np.uint8)
        assert L.h264mi_rgba_to_i420_host(rgba.ctypes.data, w, h, out.ctypes.data) == 0
        assert np.array_equal(out, oracle.rgba_to_i420(rgba, w, h))
        yuv = np.random.default_rng(w).integers(0, 256, w * h * 3 // 2, dtype=np.uint8)
        o2 = np.zeros(w * h * 4, np.uint8)
        assert L.h264mi_i420_to_rgba_host(yuv.ctypes.data, w, h, o2.ctypes.data) == 0
        assert np.array_equal(o2, oracle.i420_to_rgba(yuv, w, h))
    assert L.h264mi_rgba_to_i420_host(rgba.ctypes.data, 63, 48, out.ctypes.data) == -1   # odd width


def test_module_facade_replays_worker_sequence(gpu_lib, oracle):
    """The Emscripten-Module-shaped facade, driven like encoder_worker.js / decoder_worker.js:
    _malloc the frame, copy into HEAPU8, encode, read the out pointer with getValue, decode into a
    heap buffer, compare with the oracle."""
    import h264mi
    from h264mi.synth import SyntheticStream
    w, h = 176, 144
    M = h264mi.Module(heap_bytes=8 << 20)
    init_encoder = M.cwrap('init_encoder', 'number', ['number', 'number', 'number'])
    encode = M.cwrap('encode_frame_yuv_i420', None, ['number'] * 5)
    init_decoder = M.cwrap('init_decoder', 'number', ['number'])
    decode = M.cwrap('decode_frame_yuv_i420', None, ['number'] * 6)
    assert init_encoder(w, h, 300000) == 0 and init_decoder(1) == 0
    fsz = w * h * 3 // 2
    src, outpp, outsz = M._malloc(fsz), M._malloc(4), M._malloc(4)
    dst, wp, hp, nalp = M._malloc(fsz), M._malloc(4), M._malloc(4), M._malloc(1 << 20)
    oe, od = oracle.encoder(w, h, 300000), oracle.decoder()
    g = SyntheticStream(2, w, h)
    for t in range(3):
        f = np.ascontiguousarray(g.frame(t))
        M.HEAPU8[src:src + fsz] = f.tobytes()
        encode(src, w, h, outpp, outsz)
        off, n = M.getValue(outpp, 'i32'), M.getValue(outsz, 'i32')
        nal = bytes(M.HEAPU8[off:off + n])
        assert nal == oe.encode(f)
        if n == 0:  # skipped by the rate control (the worker posts no frame, encoder_worker.js:167)
            continue
        M.HEAPU8[nalp:nalp + n] = nal
        decode(1, nalp, n, dst, wp, hp)
        assert (M.getValue(wp), M.getValue(hp)) == (w, h)
        _, pic, _, _ = od.decode(nal)
        assert bytes(M.HEAPU8[dst:dst + fsz]) == pic.tobytes()


@pytest.mark.parametrize('use_event', [False, True], ids=['stream-ordered', 'ready-event'])
def test_pipelined_two_stream_decode(gpu_lib, use_event):
    """bench.py's pipeline without host synchronisation: the encoder codes groups of G frames on one
    HIP stream and stages their NAL units; the decoder takes each group on a second stream (ordered
    by wait_event, or by ready_event) while the next group is being encoded. After the last group
    every stream's decoded picture must equal the encoder's reconstruction and no stream may report
    an error (a parse of not-yet-written staging data fails one or the other)."""
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    w, h, S, G, groups = 352, 288, 3, 4, 5
    F = w * h * 3 // 2
    clip = torch.empty((G * groups, S * F), dtype=torch.uint8, device='cuda')
    for s in range(S):
        g = SyntheticStream(10 + s, w, h)
        clip[:, s * F:(s + 1) * F].copy_(torch.from_numpy(np.stack([g.frame(t) for t in range(G * groups)])))
    torch.cuda.synchronize()
    es, ds = torch.cuda.Stream(), torch.cuda.Stream()
    enc = h264mi.BatchEncoder(w, h, 2000000, S, stream=es)
    enc.set_frame_skip(False)
    dec = h264mi.BatchDecoder(w, h, S, stream=ds, max_frames=G)
    slot = 1 << 20
    stage = [torch.empty((G, S * slot), dtype=torch.uint8, device='cuda') for _ in range(2)]
    stage_sz = [torch.zeros((G, S), dtype=torch.int32, device='cuda') for _ in range(2)]
    ev_enc = [torch.cuda.Event() for _ in range(2)]
    ev_dec = [torch.cuda.Event() for _ in range(2)]
    t = 0
    for gi in range(groups):
        b = gi & 1
        with torch.cuda.stream(es):
            es.wait_event(ev_dec[b])
            for j in range(G):
                enc.encode(clip[t])
                enc.copy_nals(stage[b][j], slot, stage_sz[b][j])
                t += 1
            ev_enc[b].record(es)
        with torch.cuda.stream(ds):
            ptrs = [stage[b].data_ptr() + j * S * slot + s * slot for j in range(G) for s in range(S)]
            szp = [stage_sz[b].data_ptr() + 4 * (j * S + s) for j in range(G) for s in range(S)]
            if use_event:
                dec.decode_frames(ptrs, size_ptrs=szp, ready_event=ev_enc[b])
            else:
                ds.wait_event(ev_enc[b])
                dec.decode_frames(ptrs, size_ptrs=szp)
            ev_dec[b].record(ds)
    torch.cuda.synchronize()
    rc, got = dec.status()
    assert rc == 0 and all(got)
    n = dec.cw * dec.ch * 3 // 2
    for s in range(S):
        a_, b_ = np.empty(n, np.uint8), np.empty(n, np.uint8)
        h264mi._hip_memcpy_d2h(a_.ctypes.data, enc.recon_ptr(s), n)
        h264mi._hip_memcpy_d2h(b_.ctypes.data, dec.picture_ptr(s), n)
        assert np.array_equal(a_, b_), f'stream {s}'


@pytest.mark.parametrize('mode', ['satisfied', 'timeout'])
def test_recon_gate(gpu_lib, mode):
    """h264mi_dec_set_recon_gate is a scheduling hint: a call whose frames wait on an encoder's rows counter
    (already past the target, or never reaching it: the bounded wait gives up) decodes exactly as an ungated call;
    the counter advances by S * mbh per encoder frame step"""
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    w, h, S, G = 176, 144, 2, 4
    mbh = (h + 15) // 16
    gens = [SyntheticStream(20 + s, w, h) for s in range(S)]
    enc = h264mi.BatchEncoder(w, h, 500000, S)
    enc.set_frame_skip(False)
    dec = h264mi.BatchDecoder(w, h, S, max_frames=G)
    slot = 1 << 20
    stage = torch.empty((G, S * slot), dtype=torch.uint8, device='cuda')
    stage_sz = torch.zeros((G, S), dtype=torch.int32, device='cuda')
    for j in range(G):
        enc.encode(torch.from_numpy(np.concatenate([g.frame(j) for g in gens])).cuda())
        enc.copy_nals(stage[j], slot, stage_sz[j])
    torch.cuda.synchronize()
    cnt = np.zeros(1, np.uint32)
    h264mi._hip_memcpy_d2h(cnt.ctypes.data, enc.rows_counter(), 4)
    assert int(cnt[0]) == G * S * mbh
    target = 0 if mode == 'satisfied' else G * S * mbh + 1000  # never reached: each frame waits its limit
    dec.set_recon_gate(enc.rows_counter(), target, S * mbh, G, limit_us=2000)
    ptrs = [stage.data_ptr() + j * S * slot + s * slot for j in range(G) for s in range(S)]
    szp = [stage_sz.data_ptr() + 4 * (j * S + s) for j in range(G) for s in range(S)]
    dec.decode_frames(ptrs, size_ptrs=szp)
    torch.cuda.synchronize()
    rc, got = dec.status()
    assert rc == 0 and all(got)
    n = dec.cw * dec.ch * 3 // 2
    for s in range(S):
        a_, b_ = np.empty(n, np.uint8), np.empty(n, np.uint8)
        h264mi._hip_memcpy_d2h(a_.ctypes.data, enc.recon_ptr(s), n)
        h264mi._hip_memcpy_d2h(b_.ctypes.data, dec.picture_ptr(s), n)
        assert np.array_equal(a_, b_), f'stream {s}'
    enc.close()
    dec.close()
