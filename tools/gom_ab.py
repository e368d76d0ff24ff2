#!/usr/bin/env python3
"""A/B of the encoder's P-frame QP rule at the metric geometry: this project's MB-row plan (default) against
OpenH264's exact GOM rate control (h264mi_enc_set_gom_exact), encode only, frame skipping off, S streams of
1920x1080 at 1 Mbps, frames resident on the GPU (a clip of 4 frames per stream, IPPP across the wrap).
Prints one JSON line per (S, mode): frames/s over the timed frames and enc_mb_kernel's ms per launch.

  python tools/gom_ab.py [--streams 32,128,256] [--frames 16] [--warmup 4]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--streams', default='32,128,256')
    ap.add_argument('--frames', type=int, default=16)
    ap.add_argument('--warmup', type=int, default=4)
    ap.add_argument('--width', type=int, default=1920)
    ap.add_argument('--height', type=int, default=1080)
    ap.add_argument('--bitrate', type=int, default=1000000)
    ap.add_argument('--clip', type=int, default=4)
    a = ap.parse_args()
    import numpy as np
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    W, H = a.width, a.height
    base = [np.stack([np.ascontiguousarray(SyntheticStream(s, W, H).frame(t)) for t in range(a.clip)]) for s in range(8)]
    for S in [int(x) for x in a.streams.split(',')]:
        # streams s and s + 8 share content (the 8 generated clips), offset in time so they differ per frame
        clip = torch.from_numpy(np.stack([np.roll(base[s % 8], s // 8, axis=0) for s in range(S)], axis=1)).cuda()
        for exact in (False, True):
            enc = h264mi.BatchEncoder(W, H, a.bitrate, S)
            enc.set_frame_skip(False)
            enc.set_gom_exact(exact)
            for t in range(a.warmup):
                enc.encode(clip[t % a.clip])
            enc.nal_sizes()
            torch.cuda.synchronize()
            enc.set_timing(True)
            t0 = time.perf_counter()
            for t in range(a.warmup, a.warmup + a.frames):
                enc.encode(clip[t % a.clip])
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            kt = enc.kernel_time()
            enc.set_timing(False)
            sizes = enc.nal_sizes()
            print(json.dumps({'streams': S, 'mode': 'gom_exact' if exact else 'row_plan', 'frames_per_s': S * a.frames / dt,
                              'ms_per_frame_step': 1e3 * dt / a.frames, 'kernel_ms': kt, 'last_sizes_mean': float(np.mean(sizes))}), flush=True)
            enc.close()
        del clip
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
