"""Encoder alone (no decoder beside it): S streams of 1080p IPPP at 1 Mbps, frame skipping off, nf
frames; for rocprofv3 kernel traces of the encoder's kernels without the decode pipeline's
interference.   usage: enc_only.py [S nf]"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))


def main(S=32, nf=8):
    import torch, h264mi
    from h264mi.synth import SyntheticStream
    gens = [SyntheticStream(s, 1920, 1080) for s in range(S)]
    enc = h264mi.BatchEncoder(1920, 1080, 1000000, S)
    enc.set_frame_skip(False)
    clip = [torch.from_numpy(np.concatenate([g.frame(t) for g in gens])).cuda() for t in range(4)]
    torch.cuda.synchronize()
    for t in range(nf):
        t0 = time.perf_counter()
        enc.encode(clip[t % 4])
        torch.cuda.synchronize()
        print(f'frame {t}: {(time.perf_counter() - t0) * 1e3:.2f} ms', flush=True)
    enc.close()


if __name__ == '__main__':
    main(*[int(x) for x in sys.argv[1:]])
