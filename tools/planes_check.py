"""Debug: the encoder's padded motion-search planes (G, b, h, j, Cb, Cr) vs a numpy restatement
(8.4.2.2.1 with edge replication) computed from the encoder's deblocked reference, after each frame.
usage: planes_check.py w h br nf"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))
LPX, LPY, CPX, CPY = 40, 32, 20, 16


def ref_planes(ref, cw, ch):
    Y = ref[:cw * ch].reshape(ch, cw).astype(np.int64)
    ys = np.clip(np.arange(-LPY - 3, ch + LPY + 3), 0, ch - 1)
    xs = np.clip(np.arange(-LPX - 3, cw + LPX + 3), 0, cw - 1)
    G = Y[ys][:, xs]  # margin 3 around the padded plane
    t = lambda a, k, ax: np.take(a, np.arange(k, k + a.shape[ax] - 5), axis=ax)
    b1 = t(G, 0, 1) - 5 * t(G, 1, 1) + 20 * t(G, 2, 1) + 20 * t(G, 3, 1) - 5 * t(G, 4, 1) + t(G, 5, 1)  # centred at x+2 -> cols -LPX-1..
    h1 = t(G, 0, 0) - 5 * t(G, 1, 0) + 20 * t(G, 2, 0) + 20 * t(G, 3, 0) - 5 * t(G, 4, 0) + t(G, 5, 0)
    j1 = t(b1, 0, 0) - 5 * t(b1, 1, 0) + 20 * t(b1, 2, 0) + 20 * t(b1, 3, 0) - 5 * t(b1, 4, 0) + t(b1, 5, 0)
    H, W = ch + 2 * LPY, cw + 2 * LPX
    g = G[3:3 + H, 3:3 + W]
    b = np.clip((b1[3:3 + H, 1:1 + W] + 16) >> 5, 0, 255)
    hh = np.clip((h1[1:1 + H, 3:3 + W] + 16) >> 5, 0, 255)
    j = np.clip((j1[1:1 + H, 1:1 + W] + 512) >> 10, 0, 255)
    return [p.astype(np.uint8) for p in (g, b, hh, j)]


def main(w, h, br, nf):
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    g = SyntheticStream(0, w, h)
    enc = h264mi.BatchEncoder(w, h, br, 1)
    L = h264mi.lib()
    cw, ch = ((w + 15) // 16) * 16, ((h + 15) // 16) * 16
    lsz, csz = (cw + 2 * LPX) * (ch + 2 * LPY), (cw // 2 + 2 * CPX) * (ch // 2 + 2 * CPY)
    ok = True
    for t in range(nf):
        enc.encode(torch.from_numpy(np.ascontiguousarray(g.frame(t))).cuda())
        enc.nal_sizes()
        buf = np.zeros(4 * lsz + 2 * csz, np.uint8)
        assert L.h264mi_enc_ref_planes(enc._e, 0, buf.ctypes.data) == 0
        ref = np.empty(cw * ch * 3 // 2, np.uint8)
        h264mi._hip_memcpy_d2h(ref.ctypes.data, enc.recon_ptr(0), ref.size)
        want = ref_planes(ref, cw, ch)
        for k, name in enumerate('Gbhj'):
            got = buf[k * lsz:(k + 1) * lsz].reshape(ch + 2 * LPY, cw + 2 * LPX)
            d = np.argwhere(got != want[k])
            if len(d):
                ok = False
                print(f'frame {t} plane {name}: {len(d)} diffs, first (row,col) padded {d[0].tolist()} got {got[tuple(d[0])]} want {want[k][tuple(d[0])]}')
        for k in range(2):
            C = ref[cw * ch + k * (cw * ch // 4): cw * ch + (k + 1) * (cw * ch // 4)].reshape(ch // 2, cw // 2)
            wantc = C[np.clip(np.arange(-CPY, ch // 2 + CPY), 0, ch // 2 - 1)][:, np.clip(np.arange(-CPX, cw // 2 + CPX), 0, cw // 2 - 1)]
            got = buf[4 * lsz + k * csz: 4 * lsz + (k + 1) * csz].reshape(ch // 2 + 2 * CPY, cw // 2 + 2 * CPX)
            if not np.array_equal(got, wantc):
                ok = False
                print(f'frame {t} chroma {k}: {int((got != wantc).sum())} diffs')
        print(f'frame {t}: planes ok={ok}', flush=True)
    return ok


if __name__ == '__main__':
    sys.exit(0 if main(*[int(x) for x in sys.argv[1:]]) else 1)
