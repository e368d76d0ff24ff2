"""Generate tests/golden/oracle_fixtures.json (+ a small Annex-B stream) from the CPU oracle.

These are ORACLE REGRESSION FIXTURES: they pin the oracle's own output (NAL bytes, decoded pictures,
colour conversions) so that any change to the oracle -- or a GPU result that disagrees with the
committed numbers -- is caught. They are not OpenH264 golden vectors: the reference holds none and
its prebuilt h264.wasm is never executed here, so encoder parity against OpenH264 is "parity
unpinned" (DESIGN.md §3). Decoding is pinned by the normative H.264 process the oracle decoder
restates. Run:  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))

# name, w, h, bitrate, frames, force_every, input
CASES = [
    ('qcif_300k', 176, 144, 300000, 6, 0, 'synth'),
    ('cif_2m_idr3', 352, 288, 2000000, 7, 3, 'synth'),
    ('crop_208x120', 208, 120, 500000, 4, 0, 'synth'),
    ('config1_640x360_1m', 640, 360, 1000000, 8, 0, 'synth'),
    ('config2_720p_ionly_8m', 1280, 720, 8000000, 2, 1, 'synth'),
    ('qcif_rgba', 176, 144, 400000, 4, 0, 'rgba'),
    ('cif_30m_idr4', 352, 288, 30000000, 5, 4, 'synth'),
]


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def rgba_frame(w, h, t):
    """Seeded RGBA test picture (smooth + detail) for the encode_frame path."""
    rng = np.random.default_rng(1000 + t)
    base = rng.integers(0, 256, (h // 2, w // 2, 4), dtype=np.uint8)
    img = np.repeat(np.repeat(base, 2, 0), 2, 1).astype(np.uint16)
    img = (img + np.roll(img, 1, 1)) // 2
    return np.ascontiguousarray(img.astype(np.uint8))


def case_inputs(oracle, w, h, n, kind, seed=0):
    from h264mi.synth import SyntheticStream
    if kind == 'synth':
        g = SyntheticStream(seed, w, h)
        return [np.ascontiguousarray(g.frame(t)) for t in range(n)], None
    rgbas = [rgba_frame(w, h, t) for t in range(n)]
    return [oracle.rgba_to_i420(r, w, h) for r in rgbas], rgbas


def run_case(oracle, name, w, h, br, n, force_every, kind):
    frames, _ = case_inputs(oracle, w, h, n, kind)
    enc = oracle.encoder(w, h, br)
    dec = oracle.decoder()
    out = {'name': name, 'w': w, 'h': h, 'bitrate': br, 'frames': n, 'force_every': force_every, 'input': kind,
           'nal_sizes': [], 'nal_sha256': [], 'dec_sha256': [], 'recon_sha256': [], 'qp': []}
    for t, f in enumerate(frames):
        if force_every and t % force_every == 0 and t > 0:
            enc.force_idr()
        nal = enc.encode(f)
        if not nal:  # frame skipped by rate control: nothing to decode
            for k in ('nal_sha256', 'dec_sha256', 'recon_sha256'):
                out[k].append(None)
            out['nal_sizes'].append(0)
            out['qp'].append(None)
            continue
        rc, pic, dw, dh = dec.decode(nal)
        assert rc == 1 and (dw, dh) == (w, h), (name, t, rc)
        recon = enc.recon()
        assert np.array_equal(pic, recon), f'{name}: oracle decoder != oracle encoder reconstruction at frame {t}'
        out['nal_sizes'].append(len(nal))
        out['nal_sha256'].append(sha(nal))
        out['dec_sha256'].append(sha(pic))
        out['recon_sha256'].append(sha(recon))
        out['qp'].append(enc.last_qp())
    return out


def colour_case(oracle):
    w, h = 64, 48
    rgba = rgba_frame(w, h, 7)
    i420 = oracle.rgba_to_i420(rgba, w, h)
    rng = np.random.default_rng(5)
    yuv = rng.integers(0, 256, w * h * 3 // 2, dtype=np.uint8)
    back = oracle.i420_to_rgba(yuv, w, h)
    return {'w': w, 'h': h, 'rgba_to_i420_sha256': sha(i420), 'i420_to_rgba_sha256': sha(back),
            'rgba_to_i420_head': i420[:16].tolist(), 'i420_to_rgba_head': back[:16].tolist()}


def main():
    from _oracle import Oracle
    oracle = Oracle(os.path.join(ROOT, 'oracle', 'build', 'libh264_oracle.so'))
    fx = {'note': 'oracle regression fixtures (see make_golden.py docstring); parity vs OpenH264 unpinned',
          'cases': [run_case(oracle, *c) for c in CASES], 'colour': colour_case(oracle)}
    with open(os.path.join(HERE, 'oracle_fixtures.json'), 'w') as f:
        json.dump(fx, f, indent=1)
    # one small Annex-B stream kept verbatim for decoder regression tests (I + P frames)
    frames, _ = case_inputs(oracle, 176, 144, 3, 'synth', seed=3)
    enc = oracle.encoder(176, 144, 200000)
    enc.set_frame_skip(False)  # three coded pictures (the rate control would skip the P frames at this bitrate)
    stream = b''.join(enc.encode(f) for f in frames)
    with open(os.path.join(HERE, 'synth3_qcif_3f.h264'), 'wb') as f:
        f.write(stream)
    print('wrote', len(fx['cases']), 'cases;', len(stream), 'byte stream')


if __name__ == '__main__':
    main()
