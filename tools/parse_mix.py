"""Parse cost by macroblock content: synthetic 1080p P slices of one kind each (tests/streamgen.py
SyntaxGen, pinned by the oracle's parse), decoded one call at a time on the GPU; prints the
dec_parse_kernel time per slice and per macroblock (--prof: the section timers of H264MI_PARSE_PROF=1 as
cycles per macroblock instead).   usage: parse_mix.py [--prof]"""
import os, sys
import numpy as np
PROF = '--prof' in sys.argv
CNT = bool(os.environ.get('H264MI_LIB', '').endswith('_cnt.so'))  # the -DH264MI_ASM_CNT build
import ctypes
if PROF:
    os.environ['H264MI_PARSE_PROF'] = '1'
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))

KINDS = [  # name, mix, cbp_fixed, TotalCoeff choices
    ('skip', {'skip': 1}, None, None),
    ('p16_cbp0', {'p16': 1}, 0, None),
    ('p16_chroma_dc', {'p16': 1}, 0x10, [0, 1]),
    ('p16_chroma_ac_quiet', {'p16': 1}, 0x20, [0, 0, 0, 1]),
    ('p16_luma1_quiet', {'p16': 1}, 0x01, [0, 1]),
    ('p16_luma15_tc2', {'p16': 1}, 0x0f, [1, 2, 3]),
    ('p16_all_tc4', {'p16': 1}, 0x2f, [2, 4, 6]),
    ('i16', {'i16': 1}, None, None),
    # scene-change-like I_16x16 content in P slices (bench frame 22 at 1 Mbps: cbp 47, ~90 % of the luma AC
    # blocks empty, chroma AC blocks half empty): DC only, luma AC only, chroma only, both
    ('i16_cbp0', {'i16': 1}, 0x00, [0, 1, 2, 3]),
    ('i16_luma_sparse', {'i16': 1}, 0x0f, [0] * 9 + [1]),
    ('i16_chroma_half', {'i16': 1}, 0x20, [0, 0, 1, 1, 2]),
    ('i16_cbp47_scene', {'i16': 1}, 0x2f, [0] * 9 + [1]),
    # chroma AC only (P_L0_16x16, cbp 0x20), every coefficient +-1 (mag1) or 2..3 (mag2): the cost per block kind
    ('cac_tc1_mag1', {'p16': 1}, 0x20, [1]),
    ('cac_tc2_mag1', {'p16': 1}, 0x20, [2]),
    ('cac_tc3_mag1', {'p16': 1}, 0x20, [3]),
    ('cac_tc1_mag2', {'p16': 1}, 0x20, [1]),
    ('cac_half_mag1', {'p16': 1}, 0x20, [0, 1, 2]),
    ('i4', {'i4': 1}, None, None),
]


def main():
    import torch, h264mi
    from streamgen import SyntaxGen
    so = os.path.join(ROOT, 'oracle', 'build', 'libh264_oracle.so')
    nmb = 120 * 68
    dec = h264mi.BatchDecoder(1920, 1080, 1, groups=2, parse_streams=1)
    L = h264mi.lib()
    NSL = dec.ring_groups()
    names = ['ring-fill', 'skip-runs', 'mb-hdr', 'residual-rest', 'record', 'qp+ctx', 'luma', 'chromaDC', 'chromaAC']
    only = sys.argv[sys.argv.index('--kind') + 1] if '--kind' in sys.argv else None
    if CNT:
        L.h264mi_debug_asm_counts.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.h264mi_debug_asm_counts((ctypes.c_uint64 * 16)(), 1)
    for name, mix, cbp, tcs in KINDS:
        if only and name not in only.split(','):
            continue
        g = SyntaxGen(so, 120, 68, 5)
        g.tc_choice = tcs
        g.i16_cbp = cbp if name.startswith('i16_') else None
        g.mag_choice = [1] if name.endswith('_mag1') else ([2, 3] if name.endswith('_mag2') else None)
        units = [g.idr()] + [g.p(mix, cbp_fixed=cbp) for _ in range(3)]
        dev = [torch.from_numpy(np.frombuffer(u, np.uint8).copy()).cuda() for u in units]
        ms = []
        prev = np.zeros(NSL * 16, np.uint64)
        for j, u in enumerate(dev):
            dec.set_timing(True)
            dec.decode([u.data_ptr()], [u.numel()])
            rc, got = dec.status()
            t, n = dec.kernel_time(1)
            ms.append(t)
            if PROF:
                cur = np.zeros(NSL * 16, np.uint64)
                L.h264mi_dec_parse_profile(dec._d, cur.ctypes.data)
                d = (cur - prev).reshape(-1, 16).sum(0)
                prev = cur
                if j == len(dev) - 1:
                    print(f'{name:22s} cycles/MB ' + ', '.join(f'{names[k - 3]} {int(d[k]) / nmb:.0f}' for k in range(3, 12)) +
                          f' | total {int(d[3:12].sum()) / nmb:.0f} (slice {int(d[1]) / nmb:.0f})', flush=True)
        if CNT:  # event counts of the asm MB run per P macroblock (H264MI_ASM_CNT build, tools/README.md)
            c = (ctypes.c_uint64 * 16)()
            L.h264mi_debug_asm_counts(c, 1)
            ev = ['plane', 'pq', 'quiet', 'q-bail', 'blk', 'gen', 'nz1', 'core2', 't23', 'q4', 'mb', 'i16dc', 't1s']
            print(f'{name:22s} events per MB: ' + ', '.join(f'{ev[k]} {c[k] / (3 * nmb):.2f}' for k in range(13)), flush=True)
        p = float(np.mean(ms[1:]))
        print(f'{name:22s} {np.mean([len(u) for u in units[1:]]):9.0f} B  parse {p:7.3f} ms  {p * 1e6 / nmb:7.1f} ns/MB  '
              f'({p * 2.4e6 / nmb:6.0f} cycles/MB at 2.4 GHz) rc {rc}', flush=True)


if __name__ == '__main__':
    main()
