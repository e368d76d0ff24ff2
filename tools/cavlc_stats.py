"""Residual-block statistics of the bench's 1080p frames (one stream, the oracle encoder and decoder on the
CPU): per macroblock the blocks of each class, the non-empty ones, levels beyond the trailing ones and the
run_before codes decoded -- what the slice-data chain spends its instructions on.
Builds tools/cavlc_stats.c with the oracle sources into /tmp.   usage: cavlc_stats.py [bitrate]"""
import ctypes, os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))


def build():
    out, o = '/tmp/h264mi_cavlc_stats.so', os.path.join(ROOT, 'oracle')
    dec = open(os.path.join(o, 'h264o_dec.c')).read().replace('cavlc_read_block(r,', 'stat_rb(r,')
    src = '/tmp/h264mi_cavlc_stats_dec.c'
    open(src, 'w').write('int stat_rb(void *r, short *coef, int maxnum, int nc);\n' + dec)
    subprocess.check_call(['gcc', '-O2', '-fPIC', '-shared', '-w', '-I' + o, '-o', out, os.path.join(ROOT, 'tools', 'cavlc_stats.c'),
                           os.path.join(o, 'h264o_common.c'), os.path.join(o, 'h264o_enc.c'), src])
    return out


def main(br=1000000, frames=(0, 1, 10, 21, 22, 23)):
    from _oracle import Oracle
    from h264mi.synth import SyntheticStream
    o = Oracle(build())
    o.L.h264o_stat_get.argtypes = [ctypes.c_void_p]
    g = SyntheticStream(0, 1920, 1080)
    e = o.encoder(1920, 1080, br)
    e.set_frame_skip(False)
    d = o.decoder()
    nmb = 120 * 68
    for t in range(max(frames) + 1):
        u = e.encode(np.ascontiguousarray(g.frame(t)))
        o.L.h264o_stat_reset()
        d.decode(u)
        s = np.zeros((3, 40), np.int64)
        o.L.h264o_stat_get(s.ctypes.data)
        if t not in frames:
            continue
        print(f'frame {t}: {len(u)} B')
        for k, nm in enumerate(['16 coefficients (P luma, I16 DC)', 'AC, 15 coefficients', 'chroma DC']):
            b, ne, tc, t1, lv, rn, tz0 = s[k][:7]
            q = max(ne, 1)
            print(f'  {nm:33s} per MB: blocks {b / nmb:5.2f} non-empty {ne / nmb:5.2f} levels {lv / nmb:5.2f} runs {rn / nmb:5.2f}'
                  f' | per non-empty block: TotalCoeff {tc / q:4.2f} trailing ones {t1 / q:4.2f} total_zeros 0: {tz0 / q:4.2f}')


if __name__ == '__main__':
    main(*[int(x) for x in sys.argv[1:2]])
