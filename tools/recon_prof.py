"""dec_recon_kernel section profile (H264MI_RECON_PROF=1): S streams of 1080p IPPP encoded on the GPU and
decoded one frame per call; prints the kernel's section cycles per reconstructed macroblock (summed over
all row waves) and the launch time per frame.  usage: recon_prof.py [w h br S nf]"""
import os, sys
os.environ['H264MI_RECON_PROF'] = '1'
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))

NAMES = ['-', 'prefetch', 'row-above wait', 'record resolution', 'levels + neighbours', 'residuals',
         'luma prediction', 'chroma', 'outputs + window']


def main(w=1920, h=1080, br=1000000, S=32, nf=8):
    import ctypes, time, torch
    import h264mi
    from h264mi.synth import SyntheticStream
    gens = [SyntheticStream(s, w, h) for s in range(S)]
    enc = h264mi.BatchEncoder(w, h, br, S)
    enc.set_frame_skip(False)
    dec = h264mi.BatchDecoder(w, h, S, groups=2, parse_streams=1)
    dec.set_timing(True)
    L = h264mi.lib()
    prev = np.zeros(16, np.uint64)
    mbs = S * ((w + 15) // 16) * ((h + 15) // 16)
    for t in range(nf):
        frames = torch.from_numpy(np.concatenate([g.frame(t) for g in gens])).cuda()
        enc.encode(frames)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dec.decode_dev(enc.nal_ptrs(), enc.nal_size_ptrs())
        rc, got = dec.status()
        dt = time.perf_counter() - t0
        cur = np.zeros(16, np.uint64)
        L.h264mi_dec_recon_profile(dec._d, cur.ctypes.data)
        d = (cur - prev).astype(np.int64)
        prev = cur
        tot = int(d[1:9].sum())
        print(f'frame {t}: rc={rc} call {dt * 1e3:.2f} ms; cycles per MB {tot / mbs:.0f}: ' +
              ', '.join(f'{NAMES[k]} {d[k] / mbs:.0f}' for k in range(1, 9)), flush=True)
    ms, n = dec.kernel_time(0)
    print(f'dec_recon_kernel: {ms / max(n, 1):.3f} ms per launch over {n} launches ({S} streams)')


if __name__ == '__main__':
    main(*[int(x) for x in sys.argv[1:]])
