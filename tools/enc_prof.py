"""enc_mb_kernel section profile (H264MI_ENC_PROF=1): S streams 1080p IPPP, prints cycles per MB
per section summed over all waves, for I and P frames. Needs a profiling build of the library loaded with
H264MI_LIB (the default build compiles the counters out): -DH264MI_ENC_PROF_BUILD, or -DH264MI_ENC_PROF_DETAIL
for the finer per-wave slots (tools/gpu_prof_rows.sh builds on that one).   usage: enc_prof.py [w h br S nf]"""
import os, sys
os.environ['H264MI_ENC_PROF'] = '1'
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))


def main(w=1920, h=1080, br=1000000, S=8, nf=6):
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    gens = [SyntheticStream(s, w, h) for s in range(S)]
    enc = h264mi.BatchEncoder(w, h, br, S)
    enc.set_frame_skip(False)  # every frame coded, as in bench.py
    L = h264mi.lib()
    fine = bool(os.environ.get('H264MI_ENC_FINE_BUILD'))  # a -DH264MI_ENC_FINE library: slots 11..15 are finer sections
    names = ['row-start-wait', 'wait-above', 'loads+ctx', 'pskip-test', 'int-ME', 'subpel', 'intra-alt', 'p16-resid', 'I4-search',
             'I-resid', 'outputs', 'F:pskip-pred', 'F:ME-first', 'F:satd-half', 'F:sel+satd-q', 'F:p16-pred']
    if not fine:  # default build: each wave's own busy time inside the pskip-test section (not part of the total)
        names[11:15] = ['(w0 int-ME busy)', '(w1 pskip busy)', '(w2 pskip busy)', '(w3 pskip busy)']
    in_total = list(range(16)) if fine else list(range(11)) + [15]
    prev = np.zeros(64, np.uint64)
    enc.set_timing(True)
    kprev = 0.0
    nmb = ((w + 15) // 16) * ((h + 15) // 16) * S
    if os.environ.get('H264MI_ENC_PROF_ROW'):  # one MB row profiled: per MB of that row
        nmb = ((w + 15) // 16) * S
    for t in range(nf):
        frames = torch.from_numpy(np.concatenate([g.frame(t) for g in gens])).cuda()
        enc.encode(frames)
        sizes = enc.nal_sizes()
        cur = np.zeros(64, np.uint64)
        L.h264mi_enc_profile(enc._e, cur.ctypes.data)
        d = (cur - prev).astype(np.float64) / nmb
        prev = cur
        kms, _ = enc.kernel_time()
        print(f'frame {t}: enc_mb {kms - kprev:.3f} ms (with profiling)', flush=True)
        kprev = kms
        print(f'frame {t}: {sizes[0]} B; cycles/MB: total {d[in_total].sum():.0f} | ' +
              ', '.join(f'{names[k]} {d[k]:.0f}' for k in range(0, 16) if d[k] > 0), flush=True)
        print('   per wave: outputs busy to the barrier | of which up to the prefetch commit: ' +
              ', '.join(f'w{k} {d[32 + k]:.0f} | {d[36 + k]:.0f}' for k in range(4)), flush=True)
        print('   outputs, per wave (to the end of its first store group): ' + ', '.join(f'w{k} {d[52 + k]:.0f}' for k in range(4)), flush=True)
        # phase beside the integer search, from its start (sums over the MBs that took it, per MB of the frame)
        print('   search phase, per wave (test or ME start | first mode or diamond | last task): ' +
              ', '.join(f'w{k} {d[40 + k]:.0f} | {d[44 + k]:.0f} | {d[48 + k]:.0f}' for k in range(4)), flush=True)
        dn = ['-', 'tile+prefetch', 'top-wait', 'bS+params', 'filter', 'stores+flush']
        print(f'   deblock cycles/MB: total {d[17:22].sum():.0f} | ' + ', '.join(f'{dn[k]} {d[16 + k]:.0f}' for k in range(1, 6)), flush=True)


if __name__ == '__main__':
    main(*[int(x) for x in sys.argv[1:]])
