"""Debug: per-MB decisions of the GPU encoder (batch API, 1 stream) vs the CPU oracle, frame by frame.
Prints the first frame whose MB records differ and up to 12 differing MBs (type, qp, cbp, mv,
i16mode, cmode, sum of TotalCoeff).   usage: mb_diff.py w h br nf [seed]"""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))


def main(w, h, br, nf, seed=0):
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    O = ctypes.CDLL(os.path.join(ROOT, 'oracle/build/libh264_oracle.so'))
    O.h264o_enc_create.restype = ctypes.c_void_p
    oe = ctypes.c_void_p(O.h264o_enc_create(w, h, br))
    g = SyntheticStream(seed, w, h)
    enc = h264mi.BatchEncoder(w, h, br, 1)
    L = h264mi.lib()
    mbw, mbh = (w + 15) // 16, (h + 15) // 16
    n = mbw * mbh
    out = np.zeros(w * h * 4, np.uint8)
    for t in range(nf):
        f = np.ascontiguousarray(g.frame(t))
        enc.encode(torch.from_numpy(f).cuda())
        sz = enc.nal_sizes()[0]
        m = O.h264o_enc_encode(oe, f.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(out.size))
        oi = np.zeros(n * 8, np.int32)
        O.h264o_enc_mbinfo(oe, oi.ctypes.data_as(ctypes.c_void_p))
        oi = oi.reshape(n, 8)
        raw = np.zeros(n * 128, np.uint8)
        L.h264mi_enc_mbinfo(enc._e, 0, raw.ctypes.data)
        raw = raw.reshape(n, 128)
        gi = np.zeros((n, 8), np.int32)
        gi[:, 0] = raw[:, 0]; gi[:, 1] = raw[:, 1]; gi[:, 2] = raw[:, 2]; gi[:, 5] = raw[:, 3]; gi[:, 6] = raw[:, 4]
        mv = raw[:, 60:124].copy().view(np.int16).reshape(n, 16, 2)
        gi[:, 3] = mv[:, 0, 0]; gi[:, 4] = mv[:, 0, 1]
        gi[:, 7] = raw[:, 28:52].astype(np.int32).sum(1)
        same = enc.nal_bytes(0, sz) == out[:m].tobytes()
        bad = np.nonzero((gi != oi).any(1))[0]
        print(f'frame {t}: gpu {sz} B oracle {m} B bytes-equal={same} differing MBs {len(bad)}', flush=True)
        if len(bad):
            for i in bad[:12]:
                print(f'  mb ({i % mbw},{i // mbw}) gpu {gi[i].tolist()} oracle {oi[i].tolist()}')
            return False
    return True


if __name__ == '__main__':
    a = [int(x) for x in sys.argv[1:]]
    sys.exit(0 if main(*a) else 1)
