"""Debug/parity driver: encode synthetic frames with the oracle, decode the Annex-B stream with
libh264mi (GPU, C-ABI decode_frame_yuv_i420 / decode_frame_optimized) and with the oracle decoder,
compare the pictures byte for byte."""
import ctypes, sys, os, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))
from h264mi.synth import SyntheticStream

def main(w, h, br, nf, force_every=0, rgba=0):
    O = ctypes.CDLL(os.path.join(ROOT, 'oracle/build/libh264_oracle.so'))
    O.h264o_enc_create.restype = ctypes.c_void_p
    O.h264o_dec_create.restype = ctypes.c_void_p
    G = ctypes.CDLL(os.path.join(ROOT, 'openh264-wasm_amd/lib/libh264mi.so'))
    e = ctypes.c_void_p(O.h264o_enc_create(w, h, br))
    d = ctypes.c_void_p(O.h264o_dec_create())
    assert G.init_decoder(3) == 0
    S = SyntheticStream(1, w, h)
    out = np.zeros(w * h * 4 + 8192, np.uint8)
    ref = np.zeros(w * h * 3 // 2, np.uint8)
    got = np.zeros(w * h * 4, np.uint8)
    W = ctypes.c_int(); H = ctypes.c_int(); gw = ctypes.c_int(); gh = ctypes.c_int()
    ok = True
    for t in range(nf):
        f = np.ascontiguousarray(S.frame(t))
        if force_every and t % force_every == 0 and t > 0:
            O.h264o_enc_force_idr(e)
        n = O.h264o_enc_encode(e, f.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(out.size))
        r = O.h264o_dec_decode(d, out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(n), ref.ctypes.data_as(ctypes.c_void_p), ctypes.byref(W), ctypes.byref(H))
        t0 = time.time()
        if rgba:
            G.decode_frame_optimized(3, out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(n), got.ctypes.data_as(ctypes.c_void_p), ctypes.byref(gw), ctypes.byref(gh))
            exp = np.zeros(w * h * 4, np.uint8)
            O.h264o_i420_to_rgba(ref.ctypes.data_as(ctypes.c_void_p), ref[w*h:].ctypes.data_as(ctypes.c_void_p), ref[w*h+w*h//4:].ctypes.data_as(ctypes.c_void_p),
                                 w, h, w, w // 2, exp.ctypes.data_as(ctypes.c_void_p))
            same = (gw.value, gh.value) == (w, h) and np.array_equal(got[:w*h*4], exp)
        else:
            G.decode_frame_yuv_i420(3, out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(n), got.ctypes.data_as(ctypes.c_void_p), ctypes.byref(gw), ctypes.byref(gh))
            same = (gw.value, gh.value) == (w, h) and np.array_equal(got[:w*h*3//2], ref)
        dt = time.time() - t0
        print(f'frame {t}: {n} B, oracle dec {r} {W.value}x{H.value}, gpu {gw.value}x{gh.value}, match={same}, gpu call {dt*1e3:.2f} ms', flush=True)
        if not same:
            ok = False
            if not rgba and gw.value:
                diff = np.nonzero(got[:w*h*3//2] != ref)[0]
                i0 = diff[0]
                if i0 < w*h: print('  first diff luma at', (i0 % w, i0 // w), 'mb', ((i0 % w)//16, (i0//w)//16), 'n diff', len(diff))
                else: print('  first diff chroma at', i0 - w*h, 'n diff', len(diff))
            break
    return ok

if __name__ == '__main__':
    a = [int(x) for x in sys.argv[1:]]
    sys.exit(0 if main(*a) else 1)
