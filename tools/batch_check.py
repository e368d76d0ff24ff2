"""Debug driver for the batch (device-resident) API: S streams encoded by BatchEncoder, decoded by
BatchDecoder (decode or decode_dev), per frame: decoder status, decoder picture == encoder recon,
and stream 0's bytes == oracle bytes.   usage: batch_check.py w h br S nf [dev=1]"""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))


def main(w, h, br, S, nf, dev=1):
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    O = ctypes.CDLL(os.path.join(ROOT, 'oracle/build/libh264_oracle.so'))
    O.h264o_enc_create.restype = ctypes.c_void_p
    oe = ctypes.c_void_p(O.h264o_enc_create(w, h, br))
    F = w * h * 3 // 2
    gens = [SyntheticStream(s, w, h) for s in range(S)]
    enc = h264mi.BatchEncoder(w, h, br, S)
    dec = h264mi.BatchDecoder(w, h, S)
    out = np.zeros(w * h * 4, np.uint8)
    ok = True
    for t in range(nf):
        host = np.concatenate([g.frame(t) for g in gens])
        frames = torch.from_numpy(host).cuda()
        enc.encode(frames)
        sizes = enc.nal_sizes()
        if dev:
            dec.decode_dev(enc.nal_ptrs(), enc.nal_size_ptrs())
        else:
            dec.decode(enc.nal_ptrs(), sizes)
        rc, got = dec.status()
        n = O.h264o_enc_encode(oe, host[:F].ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(out.size))
        same0 = enc.nal_bytes(0, sizes[0]) == out[:n].tobytes()
        eq = []
        for s in range(S):
            cw, ch = dec.cw, dec.ch
            a = np.empty(cw * ch * 3 // 2, np.uint8)
            b = np.empty_like(a)
            h264mi._hip_memcpy_d2h(a.ctypes.data, enc.recon_ptr(s), a.size)
            h264mi._hip_memcpy_d2h(b.ctypes.data, h264mi.lib().h264mi_dec_picture_ptr(dec._d, s), b.size)
            eq.append(bool(np.array_equal(a, b)))
            if not eq[-1] and s == 0:
                d = np.nonzero(a != b)[0]
                print('   stream0 first diff', d[0], 'count', len(d), 'luma' if d[0] < cw * ch else 'chroma',
                      (d[0] % cw, d[0] // cw) if d[0] < cw * ch else '')
        print(f'frame {t}: sizes {sizes} oracle0 {n} same0={same0} dec rc={rc} got={got} recon==dec {eq}', flush=True)
        ok = ok and same0 and rc == 0 and all(got) and all(eq)
    return ok


if __name__ == '__main__':
    a = [int(x) for x in sys.argv[1:]]
    sys.exit(0 if main(*a) else 1)
