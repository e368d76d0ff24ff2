"""Debug aid (GPU box): 1080p 1 Mbps skip-off batch encode of a few synthetic streams against the oracle; per frame, the
first stream whose NAL bytes differ, whether the oracle decoder reproduces the GPU encoder's reconstruction from the GPU
bytes (bitstream self-consistency), and the first MB whose luma reconstruction differs from the oracle's, with the
oracle's MB types around it.   usage: python tools/debug/intra_p_diff.py [sid ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))


def main():
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    from _oracle import Oracle
    O = Oracle(os.path.join(ROOT, 'oracle', 'build', 'libh264_oracle.so'))
    sids = [int(a) for a in sys.argv[1:]] or [2, 15, 37]
    w, h, br, nf = 1920, 1080, 1000000, int(os.environ.get('NF', '25'))
    S = len(sids)
    gs = [SyntheticStream(s, w, h) for s in sids]
    enc = h264mi.BatchEncoder(w, h, br, S)
    enc.set_frame_skip(False)
    dec = h264mi.BatchDecoder(w, h, S, max_frames=1, groups=2)
    oes = [O.encoder(w, h, br) for _ in sids]
    ods = [O.decoder() for _ in sids]
    for oe in oes:
        oe.set_frame_skip(False)
    cw, ch = 1920, 1088
    mbw = cw // 16
    for t in range(nf):
        frames = np.stack([np.ascontiguousarray(g.frame(t)) for g in gs])
        enc.encode(torch.from_numpy(frames).cuda())
        torch.cuda.synchronize()
        n = enc.nal_sizes()
        # the GPU decoder on the GPU bytes, against the GPU encoder's reconstruction
        dec.decode_frames([enc.nal_ptr(i) for i in range(S)], nal_sizes=list(n))
        torch.cuda.synchronize()
        drc, dgot = dec.status()
        for i, s in enumerate(sids):
            ref = oes[i].encode(frames[i])
            got = enc.nal_bytes(i, n[i])
            rec = np.empty(cw * ch * 3 // 2, np.uint8)
            h264mi._hip_memcpy_d2h(rec.ctypes.data, enc.recon_ptr(i), rec.size)
            rec_y = rec[:cw * ch].reshape(ch, cw)[:h, :w]
            orec = np.empty(w * h * 3 // 2, np.uint8)
            O.L.h264o_enc_recon(oes[i].e, orec.ctypes.data)
            orec_y = orec[:w * h].reshape(h, w)
            mi = np.zeros(mbw * 68 * 8, np.int32)
            O.L.h264o_enc_mbinfo(oes[i].e, mi.ctypes.data)
            mi = mi.reshape(-1, 8)
            types = np.bincount(mi[:, 0], minlength=4)[:4].tolist()
            same = got == ref
            # bitstream self-consistency: the oracle decoder on the GPU bytes against the GPU reconstruction
            dec_ok = None
            rc, pic, _, _ = ods[i].decode(got) if got else (0, None, 0, 0)
            if pic is not None:
                dec_ok = bool(np.array_equal(pic[:w * h].reshape(h, w), rec_y))
            dpic = np.empty(cw * ch * 3 // 2, np.uint8)
            h264mi._hip_memcpy_d2h(dpic.ctypes.data, dec.picture_ptr(i), dpic.size)
            gdec_ok = bool(np.array_equal(dpic, rec))
            msg = f'frame {t} stream {s}: bytes {"==" if same else "!="} oracle ({len(got)} / {len(ref)}), oracle types {types}, ' \
                  f'oracle-decoded GPU bytes == GPU recon: {dec_ok}, GPU-decoded == GPU recon: {gdec_ok} (rc {drc})'
            if not np.array_equal(rec_y, orec_y):
                d = np.argwhere(rec_y != orec_y)
                y, x = d[0]
                mb = (y // 16) * mbw + x // 16
                msg += f'; first recon diff at MB ({x // 16}, {y // 16}) oracle record {mi[mb].tolist()}, left {mi[mb - 1].tolist()}'
            print(msg, flush=True)
    enc.close()
    dec.close()


if __name__ == '__main__':
    main()
