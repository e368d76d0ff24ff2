"""dec_recon_kernel section profile (H264MI_RECON_PROF=1): S streams of 1080p IPPP encoded on the GPU
and decoded frame by frame; prints cycles per MB per section (summed over rows, per MB).
usage: recon_prof.py [w h br S nf]"""
import os, sys
os.environ['H264MI_RECON_PROF'] = '1'
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))


def main(w=1920, h=1080, br=1000000, S=8, nf=6):
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    gens = [SyntheticStream(s, w, h) for s in range(S)]
    enc = h264mi.BatchEncoder(w, h, br, S)
    dec = h264mi.BatchDecoder(w, h, S)
    L = h264mi.lib()
    names = ['-', 'prefetch', 'wait-above', 'resolve', 'levels+ctx', 'residual', 'luma-pred', 'chroma', 'outputs']
    prev = np.zeros(16, np.uint64)
    nmb = ((w + 15) // 16) * ((h + 15) // 16) * S
    for t in range(nf):
        enc.encode(torch.from_numpy(np.concatenate([g.frame(t) for g in gens])).cuda())
        sizes = enc.nal_sizes()
        dec.decode_dev(enc.nal_ptrs(), enc.nal_size_ptrs())
        dec.status()
        cur = np.zeros(16, np.uint64)
        L.h264mi_dec_recon_profile(dec._d, cur.ctypes.data)
        d = (cur - prev).astype(np.float64) / nmb
        prev = cur
        print(f'frame {t}: {sizes[0]} B; recon cycles/MB: total {d[1:9].sum():.0f} | ' +
              ', '.join(f'{names[k]} {d[k]:.0f}' for k in range(1, 9)), flush=True)


if __name__ == '__main__':
    main(*[int(x) for x in sys.argv[1:]])
