"""debug aid: GPU vs oracle per-row QPs of exact-GOM P frames (prints the first differing rows)"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd')); sys.path.insert(0, os.path.join(ROOT, 'tests'))
import torch
import h264mi
from h264mi.synth import SyntheticStream
from _oracle import Oracle
O = Oracle(os.path.join(ROOT, 'oracle', 'build', 'libh264_oracle.so'))
w, h, br, S, nf = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
gs = [SyntheticStream(5 + s, w, h) for s in range(S)]
enc = h264mi.BatchEncoder(w, h, br, S); enc.set_gom_exact(True); enc.set_frame_skip(False)
oes = [O.encoder(w, h, br) for _ in range(S)]
for oe in oes: oe.set_gom_exact(True); oe.set_frame_skip(False)
mbw, mbh = (w + 15) // 16, (h + 15) // 16
def rowqps(nal):
    d = O.decoder(); 
    return None
decs_o = [O.decoder() for _ in range(S)]; decs_g = [O.decoder() for _ in range(S)]
for t in range(nf):
    fr = [np.ascontiguousarray(g.frame(t)) for g in gs]
    enc.encode(torch.from_numpy(np.stack(fr)).cuda())
    n = enc.nal_sizes()
    for s in range(S):
        ref = oes[s].encode(fr[s]); got = enc.nal_bytes(s, n[s]) if n[s] else b''
        ro = decs_o[s].decode(ref); rg = decs_g[s].decode(got)
        mo = np.zeros(mbw * mbh * 8, np.int32); mg = np.zeros(mbw * mbh * 8, np.int32)
        O.L.h264o_dec_mbinfo(decs_o[s].d, mo.ctypes.data); O.L.h264o_dec_mbinfo(decs_g[s].d, mg.ctypes.data)
        qo = mo.reshape(mbh, mbw, 8)[:, :, 1]; qg = mg.reshape(mbh, mbw, 8)[:, :, 1]
        if got != ref:
            fd = next((i for i in range(min(len(got), len(ref))) if got[i] != ref[i]), -1)
            print(f'first differing byte {fd} of {len(ref)}')
            print(f'frame {t} stream {s}: {len(got)} vs {len(ref)} B; rc gpu {enc.rc_state(s)} oracle {oes[s].rc_state()}')
            for r in range(mbh):
                if not np.array_equal(qo[r], qg[r]) or not np.array_equal(mo.reshape(mbh, mbw, 8)[r], mg.reshape(mbh, mbw, 8)[r]):
                    print(' row', r, 'qp oracle', qo[r].tolist(), '\n        gpu   ', qg[r].tolist())
                    print('   type o', mo.reshape(mbh, mbw, 8)[r, :, 0].tolist(), '\n        g', mg.reshape(mbh, mbw, 8)[r, :, 0].tolist())
                    break
            go, gg = oes[s].gom_state(), enc.gom_state(s)
            for g in range(len(go)):
                print(' gom', g, 'oracle', go[g], 'gpu', gg[g], '' if go[g] == gg[g] else '<<')
            sys.exit(0)
print('no difference')
