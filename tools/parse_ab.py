"""A/B of parse-kernel variants on steady-state bench frames: stream 0 of the bench (1920x1080, 1 Mbps,
frame skipping off) is encoded once on the GPU, then each variant (openh264-wasm_amd/lib/variants/<name>.so,
or 'cur' for lib/libh264mi.so) decodes frames 0..N-1 one call at a time in a child process; prints the
dec_parse_kernel time (HIP events) summed over frames 8..N-1 and the decoded-picture hash (must agree).
usage: parse_ab.py <outdir> <name>... [--frames N]"""
import hashlib, json, os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))
W, H = 1920, 1080
BR = int(os.environ.get('PARSE_AB_BR', '1000000'))


def encode(path, nf):
    import torch, h264mi
    from h264mi.synth import SyntheticStream
    g = SyntheticStream(0, W, H)
    enc = h264mi.BatchEncoder(W, H, BR, 1)
    enc.set_frame_skip(False)
    units = []
    for t in range(nf):
        enc.encode(torch.from_numpy(np.ascontiguousarray(g.frame(t))).cuda())
        n = enc.nal_sizes()[0]
        units.append(np.frombuffer(enc.nal_bytes(0, n), np.uint8))
    np.savez(path, *units)


def decode(path):
    import torch, h264mi
    units = list(np.load(path).values())
    dec = h264mi.BatchDecoder(W, H, 1, max_frames=1, groups=2, parse_streams=1)
    dev = [torch.from_numpy(u.copy()).cuda() for u in units]
    torch.cuda.synchronize()
    per, hs = [], hashlib.sha256()
    for t, u in enumerate(dev):
        dec.set_timing(True)
        dec.decode([u.data_ptr()], [u.numel()])
        rc, got = dec.status()
        ms, n = dec.kernel_time(1)
        per.append(ms)
        hs.update(dec.picture_i420(0))
    print(json.dumps({'parse_ms': per, 'hash': hs.hexdigest()[:16]}))


def main():
    if sys.argv[1] == '--child':
        return decode(sys.argv[2])
    out = sys.argv[1]
    names = [a for a in sys.argv[2:] if not a.startswith('--')]
    nf = int(sys.argv[sys.argv.index('--frames') + 1]) if '--frames' in sys.argv else 24
    names = [n for n in names if not n.isdigit()]
    os.makedirs(out, exist_ok=True)
    path = os.path.join(out, 'units.npz')
    encode(path, nf)
    for name in names:
        env = dict(os.environ)
        if name != 'cur':
            env['H264MI_LIB'] = os.path.join(ROOT, 'openh264-wasm_amd', 'lib', 'variants', name + '.so')
        r = subprocess.run([sys.executable, __file__, '--child', path], capture_output=True, text=True, env=env, timeout=300)
        try:
            d = json.loads([l for l in r.stdout.splitlines() if l.startswith('{')][-1])
        except Exception:
            print(name, 'FAILED', r.stdout[-500:], r.stderr[-1500:], flush=True)
            continue
        p = d['parse_ms']
        print(f"{name:12s} parse ms frames 8..: {sum(p[8:]):8.2f}  (per frame {np.mean(p[8:]):.2f})  IDR {p[0]:.2f}  hash {d['hash']}", flush=True)


if __name__ == '__main__':
    main()
