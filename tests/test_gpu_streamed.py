"""GPU: streamed reconstruction -- the first frame of each decode call is reconstructed row
by row behind its slice data (the parse wave publishes each finished MB row; the reconstruction rows wait
for theirs) instead of after the parse launch. Forced on (h264mi_dec_set_streamed(1)), with the bench's
reserved decode lane and without it, every picture == the oracle decoder's, including damaged access
units: a slice cut short aborts the frame's wavefront from the parse side and the picture is concealed
(no picture, the reference stays), and the stream decodes on. Multi-slice pictures (rows handed over when
every slice is done) are covered by test_gpu_multislice.py's batch decoder, which the library's automatic
choice streams (one 1080p stream)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _units(oracle, w, h, br, seed, n):
    from h264mi.synth import SyntheticStream
    g = SyntheticStream(seed, w, h)
    e = oracle.encoder(w, h, br)
    e.set_frame_skip(False)
    return [e.encode(np.ascontiguousarray(g.frame(t))) for t in range(n)]


@pytest.mark.parametrize('lanes', [0, 16], ids=['shared-cus', 'reserved-lane'])
def test_streamed_reconstruction_vs_oracle_with_damage(gpu_lib, oracle, lanes):
    import torch
    import h264mi
    w, h, S, n = 1920, 1080, 2, 6
    units = [_units(oracle, w, h, 2000000, 40 + s, n) for s in range(S)]
    # stream 1, frame 2: the slice data cut in half (the parse fails part-way through the picture);
    # stream 0, frame 4: a few bytes flipped in the middle of the slice data
    units[1][2] = units[1][2][:len(units[1][2]) // 2]
    u = bytearray(units[0][4])
    for k in range(len(u) // 2, len(u) // 2 + 6):
        u[k] ^= 0x5A
    units[0][4] = bytes(u)
    ods = [oracle.decoder() for _ in range(S)]
    st = h264mi.masked_stream(0, lanes, True) if lanes else None
    dec = h264mi.BatchDecoder(w, h, S, stream=st, max_frames=1)
    if lanes:
        dec.set_parse_cus(0, lanes)
    dec.set_streamed(1)
    assert dec.streamed() == 1
    F = w * h * 3 // 2
    out = torch.zeros((S, F), dtype=torch.uint8, device='cuda')
    got = torch.zeros(S, dtype=torch.int32, device='cuda')
    for t in range(n):
        dev = [torch.from_numpy(np.frombuffer(units[s][t], np.uint8).copy()).cuda() for s in range(S)]
        torch.cuda.synchronize()
        dec.decode_frames([d.data_ptr() for d in dev], nal_sizes=[len(units[s][t]) for s in range(S)],
                          out_ptrs=[out[s].data_ptr() for s in range(S)], got_ptrs=[got[s:s + 1].data_ptr() for s in range(S)])
        if st is not None:
            st.synchronize()
        torch.cuda.synchronize()
        g = got.cpu().tolist()
        host = out.cpu().numpy()
        for s in range(S):
            rc, pic, _, _ = ods[s].decode(units[s][t])
            assert (g[s] == 1) == (rc == 1), f'frame {t} stream {s}: got {g[s]}, oracle rc {rc}'
            if rc == 1:
                assert np.array_equal(host[s], pic), f'frame {t} stream {s}: {int(np.count_nonzero(host[s] != pic))} samples differ'
    assert g == [1, 1]  # both streams decode on after their damaged frames
    dec.close()
    if st is not None:
        h264mi.destroy_stream(st)


def test_streamed_budget_from_device(gpu_lib):
    """automatic streaming's wave budget comes from the device (a quarter of dec_recon_kernel's resident wave
    slots: CUs x its blocks per CU); a decoder whose reconstruction waves exceed the budget falls back to
    unstreamed reconstruction, one that fits is streamed (the fixed 1024 did not follow the device)"""
    import torch
    import h264mi
    L = h264mi.lib()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    default = L.h264mi_dec_set_streamed_budget(0)
    assert 0 < default <= cus * 4 * 8 // 4, (default, cus)  # at most a quarter of 8 waves per SIMD
    try:
        assert L.h264mi_dec_set_streamed_budget(8) == 8
        dec = h264mi.BatchDecoder(176, 144, 1)  # 2 x 9 MB rows = 18 waves > 8: unstreamed
        assert dec.streamed() == 0
        dec.close()
        assert L.h264mi_dec_set_streamed_budget(0) == default
        dec = h264mi.BatchDecoder(176, 144, 1)  # 18 waves fit the device budget: streamed
        assert dec.streamed() == 1
        dec.close()
    finally:
        L.h264mi_dec_set_streamed_budget(0)
