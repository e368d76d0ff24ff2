"""Debug driver for the batch (device-resident) API: S streams encoded by BatchEncoder and decoded by
BatchDecoder. With group G = 1 every frame is decoded right after it is encoded (decode or
decode_dev); with G > 1 frames are staged and decoded G at a time (decode_frames). Checks per
decode call: decoder status, decoder picture == encoder reconstruction (every stream), and EVERY
stream's bytes == the bytes of that stream's own oracle encoder (seed s) for every frame. lanes > 0: encoder and reconstruction on streams masked off
CU bits [0, lanes), entropy decoding (4 parse streams) on those CUs -- the bench's reserved decode lane.
streamed: h264mi_dec_set_streamed mode (None: 1 with lanes -- the reconstruction stream is off the parse CUs --,
else -1, the library's automatic choice). pic: also every stream's decoded picture (cropped) == its oracle
encoder's reconstruction, after every call. The S oracle encoders run in threads (ctypes drops the GIL).
usage: batch_check.py w h br S nf [dev=1] [G=1] [lanes=0] [streamed] [pic=0]"""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))


def _crop_i420(a, cw, ch, w, h):
    y = a[:cw * ch].reshape(ch, cw)[:h, :w]
    u = a[cw * ch:cw * ch * 5 // 4].reshape(ch // 2, cw // 2)[:h // 2, :w // 2]
    v = a[cw * ch * 5 // 4:cw * ch * 3 // 2].reshape(ch // 2, cw // 2)[:h // 2, :w // 2]
    return np.concatenate([y.ravel(), u.ravel(), v.ravel()])


def main(w, h, br, S, nf, dev=1, G=1, lanes=0, streamed=None, pic=0):
    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(max_workers=min(S, 16))
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    O = ctypes.CDLL(os.path.join(ROOT, 'oracle/build/libh264_oracle.so'))
    O.h264o_enc_create.restype = ctypes.c_void_p
    oes = [ctypes.c_void_p(O.h264o_enc_create(w, h, br)) for _ in range(S)]  # one oracle encoder per stream
    for oe in oes:
        O.h264o_enc_set_frame_skip(oe, 0)  # the batch pipeline under test decodes every frame
    F = w * h * 3 // 2
    gens = [SyntheticStream(s, w, h) for s in range(S)]
    st = h264mi.masked_stream(0, lanes, True) if lanes else None
    enc = h264mi.BatchEncoder(w, h, br, S, stream=st)
    enc.set_frame_skip(False)
    dec = h264mi.BatchDecoder(w, h, S, stream=st, max_frames=G)
    if lanes:
        dec.set_parse_streams(4)
        dec.set_parse_cus(0, lanes)
    dec.set_streamed((1 if lanes else -1) if streamed is None else streamed)
    print(f'streamed reconstruction: {dec.streamed()}', flush=True)
    outs = [np.zeros(w * h * 4, np.uint8) for _ in range(S)]
    slot = 1 << 21
    stage = torch.empty((G, S * slot), dtype=torch.uint8, device='cuda')
    stage_sz = torch.zeros((G, S), dtype=torch.int32, device='cuda')
    ok = True
    t = 0
    while t < nf:
        n = min(G, nf - t)
        same = [True] * S
        sizes = None
        for j in range(n):
            host = np.concatenate([g.frame(t + j) for g in gens])
            with torch.cuda.stream(st) if st is not None else torch.cuda.stream(torch.cuda.current_stream()):
                enc.encode(torch.from_numpy(host).cuda())
            sizes = enc.nal_sizes()

            def oenc(s):
                return O.h264o_enc_encode(oes[s], host[s * F:(s + 1) * F].ctypes.data_as(ctypes.c_void_p), outs[s].ctypes.data_as(ctypes.c_void_p),
                                          ctypes.c_int(outs[s].size))
            for s, m in enumerate(pool.map(oenc, range(S))):
                same[s] = same[s] and enc.nal_bytes(s, sizes[s]) == outs[s][:m].tobytes()
            if G > 1:
                enc.copy_nals(stage[j], slot, stage_sz[j])
        if G == 1:
            if dev:
                dec.decode_dev(enc.nal_ptrs(), enc.nal_size_ptrs())
            else:
                dec.decode(enc.nal_ptrs(), sizes)
        else:
            torch.cuda.synchronize()
            if st is not None:
                st.synchronize()
            ptrs = [stage.data_ptr() + j * S * slot + s * slot for j in range(n) for s in range(S)]
            if dev:
                szp = [stage_sz.data_ptr() + 4 * (j * S + s) for j in range(n) for s in range(S)]
                dec.decode_frames(ptrs, size_ptrs=szp)
            else:
                dec.decode_frames(ptrs, nal_sizes=stage_sz[:n].cpu().flatten().tolist())
        rc, got = dec.status()
        eq = []
        for s in range(S):
            cw, ch = dec.cw, dec.ch
            a = np.empty(cw * ch * 3 // 2, np.uint8)
            b = np.empty_like(a)
            h264mi._hip_memcpy_d2h(a.ctypes.data, enc.recon_ptr(s), a.size)
            h264mi._hip_memcpy_d2h(b.ctypes.data, dec.picture_ptr(s), b.size)
            eq.append(bool(np.array_equal(a, b)))
            if pic:
                r = np.empty(w * h * 3 // 2, np.uint8)
                O.h264o_enc_recon(oes[s], r.ctypes.data_as(ctypes.c_void_p))
                eq[-1] = eq[-1] and bool(np.array_equal(_crop_i420(b, cw, ch, w, h), r))
            if not eq[-1] and s == 0:
                d = np.nonzero(a != b)[0]
                print('   stream0 first diff', d[0], 'count', len(d), 'luma' if d[0] < cw * ch else 'chroma',
                      (d[0] % cw, d[0] // cw) if d[0] < cw * ch else '')
        print(f'frames {t}..{t + n - 1}: last sizes {sizes} oracle-bytes-equal(every stream)={same} dec rc={rc} got={got} '
              f'recon==dec {eq}', flush=True)
        ok = ok and all(same) and rc == 0 and all(got) and all(eq)
        t += n
    pool.shutdown()
    for oe in oes:
        O.h264o_enc_destroy(oe)
    return ok


if __name__ == '__main__':
    a = [int(x) for x in sys.argv[1:]]
    sys.exit(0 if main(*a) else 1)
