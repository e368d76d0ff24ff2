"""Debug: C-ABI encode of n frames vs the oracle, first differing byte per frame (GPU box).
usage: enc_diff.py [w h bitrate n]"""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd')); sys.path.insert(0, os.path.join(ROOT, 'tests'))
import h264mi
from h264mi.synth import SyntheticStream
from _oracle import Oracle
w, h, br, n = [int(x) for x in sys.argv[1:5]] if len(sys.argv) > 4 else (176, 144, 300000, 3)
L = h264mi.lib()
o = Oracle(os.path.join(ROOT, 'oracle', 'build', 'libh264_oracle.so'))
oe = o.encoder(w, h, br)
assert L.init_encoder(w, h, br) == 0
g = SyntheticStream(0, w, h)
for t in range(n):
    f = np.ascontiguousarray(g.frame(t))
    p = ctypes.POINTER(ctypes.c_ubyte)(); sz = ctypes.c_int(0)
    L.encode_frame_yuv_i420(f.ctypes.data, w, h, ctypes.byref(p), ctypes.byref(sz))
    got = ctypes.string_at(p, sz.value) if sz.value > 0 else b''
    ref = oe.encode(f)
    if got == ref:
        print(f'frame {t}: equal ({len(got)} B)')
        continue
    d = next((i for i in range(min(len(got), len(ref))) if got[i] != ref[i]), min(len(got), len(ref)))
    print(f'frame {t}: GPU {len(got)} B oracle {len(ref)} B first diff at {d}')
    print('  gpu', got[max(0, d - 8):d + 24].hex())
    print('  ref', ref[max(0, d - 8):d + 24].hex())
