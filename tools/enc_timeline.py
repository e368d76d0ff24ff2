"""enc_mb_kernel per-ticket timeline (H264MI_ENC_TL=1): S streams 1080p IPPP at the bench's bitrate, frames 0..nf-1;
for each frame: the launch span, the encoder rows' and deblocking rows' start / end distribution, and how many
tickets were live over time (which bounds the kernel: residency, the wavefront ramp, or the deblocking tail).
With the per-XCD ticket queues (the default when S % 8 == 0; H264MI_ENC_XQ=0 turns them off) the kernel records
ticket t of XCD queue q at slot q * 2 (S / 8) mbh + t; the slots are put back in the one-queue order (encoder row r
of stream s at r S + s, its deblocking row at S mbh + r S + s) before anything is summarised.
usage: enc_timeline.py [w h br S nf]"""
import os, sys
os.environ['H264MI_ENC_TL'] = '1'
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))


def main(w=1920, h=1080, br=1000000, S=32, nf=6):
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    gens = [SyntheticStream(s, w, h) for s in range(S)]
    enc = h264mi.BatchEncoder(w, h, br, S)
    enc.set_frame_skip(False)
    L = h264mi.lib()
    mbh = (h + 15) // 16
    n = 4 * S * mbh
    for t in range(nf):
        enc.encode(torch.from_numpy(np.concatenate([g.frame(t) for g in gens])).cuda())
        torch.cuda.synchronize()
        tl = np.zeros(n, np.uint64)
        assert L.h264mi_enc_timeline(enc._e, tl.ctypes.data, n) == 0
        tl = tl.reshape(-1, 2).astype(np.int64)
        if S % 8 == 0 and os.environ.get('H264MI_ENC_XQ', '1') != '0' and int(os.environ.get('H264MI_DBK_LAG', '0')) <= 0:
            Sq, per = S // 8, 2 * (S // 8) * mbh
            slot = np.arange(2 * S * mbh)
            q, tq = slot // per, slot % per
            tb, s = tq // Sq, (tq % Sq) * 8 + q
            canon = np.where(tb < mbh, tb * S + s, S * mbh + (tb - mbh) * S + s)
            out = np.empty_like(tl)
            out[canon] = tl[:2 * S * mbh]
            tl = out
        t0 = tl[:, 0].min()
        st, en = (tl[:, 0] - t0) / 100.0, (tl[:, 1] - t0) / 100.0  # microseconds (100 MHz)
        E, D = slice(0, S * mbh), slice(S * mbh, 2 * S * mbh)
        span = en.max()
        print(f'frame {t}: span {span:.0f} us | enc rows: start p50 {np.median(st[E]):.0f} max {st[E].max():.0f}, '
              f'life mean {np.mean(en[E] - st[E]):.0f} (row 0 {np.mean((en[E] - st[E])[:S]):.0f}), end max {en[E].max():.0f} | '
              f'dbk rows: start min {st[D].min():.0f} p50 {np.median(st[D]):.0f}, life mean {np.mean(en[D] - st[D]):.0f}, '
              f'end max {en[D].max():.0f}', flush=True)
        # live tickets over time (10 buckets)
        edges = np.linspace(0, span, 11)
        live_e = [int(((st[E] <= x) & (en[E] > x)).sum()) for x in edges[:-1] + span / 20]
        live_d = [int(((st[D] <= x) & (en[D] > x)).sum()) for x in edges[:-1] + span / 20]
        print(f'   live enc rows by decile: {live_e}\n   live dbk rows by decile: {live_d}', flush=True)
        # per-row lifetime by MB row index (mean over streams) for a few rows
        life = (en[E] - st[E]).reshape(mbh, S).mean(axis=1)
        print('   enc row life by row (us): ' + ' '.join(f'{r}:{life[r]:.0f}' for r in (0, 1, 2, 8, 16, 31, 32, 33, 48, 63, 64, 67)), flush=True)
        sr = st[E].reshape(mbh, S).mean(axis=1)
        print('   enc row start by row (us): ' + ' '.join(f'{r}:{sr[r]:.0f}' for r in (0, 1, 2, 8, 16, 31, 32, 33, 48, 63, 64, 67)), flush=True)


if __name__ == '__main__':
    main(*[int(x) for x in sys.argv[1:]])
