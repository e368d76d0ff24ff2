"""Parse-kernel section profile: S streams of 1080p IPPP encoded on the GPU and decoded with
H264MI_PARSE_PROF=1; prints cycles per section per frame.   usage: parse_prof.py [w h br S nf]"""
import ctypes, os, sys
LOAD = '--load' in sys.argv  # an 8-stream encoder runs on another HIP stream while decoding (the bench's mix)
if LOAD:
    sys.argv.remove('--load')
PMC = '--pmc' in sys.argv  # plain kernel (no section timers), for rocprofv3 counter passes
if PMC:
    sys.argv.remove('--pmc')
else:
    os.environ['H264MI_PARSE_PROF'] = '1'
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))


def main(w=1920, h=1080, br=1000000, S=4, nf=8):
    import torch, time
    import h264mi
    from h264mi.synth import SyntheticStream
    gens = [SyntheticStream(s, w, h) for s in range(S)]
    enc = h264mi.BatchEncoder(w, h, br, S)
    enc.set_frame_skip(False)  # every frame coded, as in bench.py
    dec = h264mi.BatchDecoder(w, h, S, groups=2, parse_streams=1)
    if LOAD:
        es = torch.cuda.Stream()
        lenc = h264mi.BatchEncoder(w, h, br, 8, stream=es)
        lenc.set_frame_skip(False)
        lgen = [SyntheticStream(100 + s, w, h) for s in range(8)]
        lclip = [torch.from_numpy(np.concatenate([g.frame(t) for g in lgen])).cuda() for t in range(4)]
    L = h264mi.lib()
    names = ['-', '-', '-', 'ring-fill', 'skip-runs', 'mb-hdr', 'residual-rest', 'record', 'qp+ctx', 'luma', 'chromaDC', 'chromaAC']
    NSL = S * dec.ring_groups()  # frame slots of a max_frames=1 decoder
    prev = np.zeros(NSL * 16, np.uint64)
    for t in range(nf):
        frames = torch.from_numpy(np.concatenate([g.frame(t) for g in gens])).cuda()
        enc.encode(frames)
        sizes = enc.nal_sizes()
        torch.cuda.synchronize()
        if LOAD:
            with torch.cuda.stream(es):
                for k in range(12):
                    lenc.encode(lclip[k % 4])
        t0 = time.perf_counter()
        dec.decode_dev(enc.nal_ptrs(), enc.nal_size_ptrs())
        rc, got = dec.status()
        dt = time.perf_counter() - t0
        if PMC:
            print(f'frame {t}: {sizes[0]} B rc={rc} decode {dt*1e3:.2f} ms', flush=True)
            continue
        if os.environ.get('H264MI_LIB', '').endswith('_cnt.so'):  # asm MB-run events per MB (H264MI_ASM_CNT build)
            c = (ctypes.c_uint64 * 16)()
            L.h264mi_debug_asm_counts.argtypes = [ctypes.c_void_p, ctypes.c_int]
            L.h264mi_debug_asm_counts(c, 1)
            ev = ['plane', 'pq', 'quiet', 'q-bail', 'blk', 'gen', 'nz1', 'core2', 't23', 'q4', 'mb', 'i16dc', 't1s']
            nmb = S * ((w + 15) // 16) * ((h + 15) // 16)
            print(f'frame {t}: events per MB ' + ', '.join(f'{ev[k]} {c[k] / nmb:.2f}' for k in range(13)), flush=True)
        cur = np.zeros(NSL * 16, np.uint64)
        L.h264mi_dec_parse_profile(dec._d, cur.ctypes.data)
        d = (cur - prev).reshape(-1, S, 16).sum(0)[0]
        prev = cur
        tot = int(d[3:12].sum())
        mhz = d[1] / d[0] * 100 if d[0] else 0
        print(f'frame {t}: {sizes[0]} B rc={rc} decode {dt*1e3:.2f} ms; stream0 cycles total {tot/1e6:.2f} M: ' +
              ', '.join(f'{names[k]} {int(d[k])/1e6:.2f}M' for k in range(3, 12)) +
              f'; slice {int(d[0]) / 1e5:.2f} ms at {mhz:.0f} MHz; AC blocks generic {int(d[12])} (sum tc {int(d[15])}), planes skipped {int(d[13])}, blocks skipped {int(d[14])}', flush=True)


if __name__ == '__main__':
    main(*[int(x) for x in sys.argv[1:]])
