"""How the asm P-slice run meets the chroma AC planes of a stream (oracle decoder, CPU): per plane of
a P_L0_16x16 MB with coded_block_pattern chroma 2, the path p_mb_run takes -- '1111' (four empty
blocks, every nC < 2), 'quiet' (every neighbour TotalCoeff 0/1 and every block 0/1), 'quiet-bail'
(quiet neighbours, a block with TotalCoeff > 1), 'generic'.   usage: chroma_planes.py [bitrate] [frames]"""
import collections, ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests')); sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))


def main(br=1000000, nf=24):
    from _oracle import Oracle
    from h264mi.synth import SyntheticStream
    O = Oracle(os.path.join(ROOT, 'oracle', 'build', 'libh264_oracle.so'))
    O.L.h264o_dec_nnz.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    g = SyntheticStream(0, 1920, 1080)
    oe, od = O.encoder(1920, 1080, br), O.decoder()
    oe.set_frame_skip(False)
    mbw, mbh = 120, 68
    mi = np.zeros(mbw * mbh * 8, np.int32)
    nz = np.zeros(mbw * mbh * 24, np.uint8)
    tot = collections.Counter()
    tcs = collections.Counter()
    for t in range(nf):
        u = oe.encode(np.ascontiguousarray(g.frame(t)))
        od.decode(u)
        if t < 8:
            continue
        O.L.h264o_dec_mbinfo(od.d, mi.ctypes.data)
        O.L.h264o_dec_nnz(od.d, nz.ctypes.data)
        m = mi.reshape(mbh, mbw, 8)
        z = nz.reshape(mbh, mbw, 24).astype(int)
        for y in range(mbh):
            for x in range(mbw):
                if m[y, x, 0] != 2 or (m[y, x, 2] >> 4) != 2:
                    continue
                for pl in range(2):
                    b = z[y, x, 16 + 4 * pl:20 + 4 * pl]   # blocks 0..3 (2x2 raster)
                    tcs.update(b.tolist())
                    # neighbours: left MB blocks 1, 3; upper MB blocks 2, 3 (skip / no-chroma MBs: 0; edge: n/a)
                    l = z[y, x - 1, 16 + 4 * pl:20 + 4 * pl][[1, 3]] if x > 0 else np.array([255, 255])
                    tp = z[y - 1, x, 16 + 4 * pl:20 + 4 * pl][[2, 3]] if y > 0 else np.array([255, 255])
                    nb = list(l) + list(tp)
                    quiet_nb = all(v <= 1 for v in nb)
                    if all(v == 0 for v in b) and l[0] + tp[0] <= 2 and l[1] <= 2 and tp[1] <= 2:
                        tot['1111'] += 1
                    elif quiet_nb and all(v <= 1 for v in b):
                        tot['quiet'] += 1
                    elif quiet_nb:
                        tot['quiet-bail'] += 1
                    else:
                        tot['generic'] += 1
    n = sum(tot.values())
    print(f'{br} bps, frames 8..{nf - 1}: planes {n}', {k: round(v / n, 3) for k, v in tot.most_common()})
    m = sum(tcs.values())
    print('  chroma AC TotalCoeff', {k: round(v / m, 3) for k, v in sorted(tcs.items())[:8]})


if __name__ == '__main__':
    main(*[int(a) for a in sys.argv[1:]])
