"""CPU baseline for bench.py: the oracle (oracle/, the CPU restatement of the reference path --
TEST INFRASTRUCTURE, loaded here only as the baseline being timed and as the parity checker) run on
host cores, one single-threaded stream per worker process (the wrapper runs OpenH264 single-threaded,
SURVEY.md §2, openh264_wrapper.cpp:198-228 leaves threading off). Prints one JSON line.

Modes (what one timed frame is, matching bench.py's configs):
  encdec  1 IDR untimed, then P frames encoded + decoded        (metric, configs 3 and 5)
  enc_i   every frame forced IDR, encoded                         (config 2)
  dec     the stream is encoded untimed, then its P frames decoded (config 4)
--window-last T: frames 0..T of the bench's streams through the oracle (encoded + decoded), timed over the GPU's
own window --window-first..T (like-for-like content: the GPU's timed frames include the synthetic scene change
at frame 22) and hashed at frame T (the timed pipeline's last frame, checked after the timed region).
Also (--hash K): sha256 of the oracle's NAL bytes and decoded pictures of the first K frames of stream 0
-- or, with --hash-streams N, of each of streams F..F+N-1 (--hash-first F; one oracle encoder and decoder
per stream, in parallel worker processes) -- which bench.py compares with the bytes and pictures of the
timed pipeline's own streams (parity at the bench's own size and stream count).
Run as a child process before the parent touches the GPU.
"""
import argparse, ctypes, hashlib, json, os, sys, time
import multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def gom_exact():
    """the P-frame QP rule of the GPU encoders this baseline is compared with: OpenH264's exact GOM rate control
    when H264MI_GOM_EXACT=1 (bench.py --gom-exact; the library reads the same variable), else the MB-row plan"""
    v = os.environ.get('H264MI_GOM_EXACT', '0').strip()
    return 1 if v.isdigit() and int(v) != 0 else 0  # as the library's atoi(...) != 0 for plain digits


def worker(args):
    stream, w, h, bitrate, nframes, mode, nhash = args
    sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))
    import numpy as np
    from h264mi.synth import SyntheticStream
    O = ctypes.CDLL(os.path.join(ROOT, 'oracle', 'build', 'libh264_oracle.so'))
    O.h264o_enc_create.restype = ctypes.c_void_p
    O.h264o_dec_create.restype = ctypes.c_void_p
    vp = ctypes.c_void_p
    S = SyntheticStream(stream, w, h)
    frames = [np.ascontiguousarray(S.frame(t)) for t in range(nframes)]
    e = vp(O.h264o_enc_create(w, h, bitrate))
    O.h264o_enc_set_frame_skip(e, 0)  # as bench.py's GPU encoder: every frame coded
    O.h264o_enc_set_gom_exact(e, gom_exact())
    d = vp(O.h264o_dec_create())
    out = np.zeros(w * h * 4, np.uint8)
    pic = np.zeros(w * h * 3 // 2, np.uint8)
    W, H = ctypes.c_int(), ctypes.c_int()
    hashes = []

    def enc(f):
        n = O.h264o_enc_encode(e, f.ctypes.data_as(vp), out.ctypes.data_as(vp), ctypes.c_int(out.size))
        return n

    def dec(buf, n):
        return O.h264o_dec_decode(d, buf.ctypes.data_as(vp), ctypes.c_int(n), pic.ctypes.data_as(vp), ctypes.byref(W), ctypes.byref(H))

    timed = 0.0
    counted = 0
    t_enc = 0.0  # encdec: the encode share of `timed` (north_star prices the GPU against encode FPS)
    if mode == 'dec':
        units = []
        for f in frames:
            n = enc(f)
            units.append(out[:n].copy())
        for t, u in enumerate(units):
            t0 = time.perf_counter()
            dec(u, u.size)
            dt = time.perf_counter() - t0
            if t > 0:
                timed += dt; counted += 1
            if t < nhash:
                hashes.append({'nal': hashlib.sha256(u.tobytes()).hexdigest(), 'pic': hashlib.sha256(pic.tobytes()).hexdigest()})
    else:
        for t, f in enumerate(frames):
            t0 = time.perf_counter()
            if mode == 'enc_i':
                O.h264o_enc_force_idr(e)
            n = enc(f)
            t1 = time.perf_counter()
            if mode == 'encdec':
                dec(out, n)
            dt = time.perf_counter() - t0
            if mode == 'enc_i' or t > 0:
                timed += dt; counted += 1
                t_enc += t1 - t0
            if t < nhash:
                if mode != 'encdec':
                    dec(out, n)
                hashes.append({'nal': hashlib.sha256(out[:n].tobytes()).hexdigest(), 'pic': hashlib.sha256(pic.tobytes()).hexdigest()})
    O.h264o_enc_destroy(e)
    O.h264o_dec_destroy(d)
    return timed, counted, hashes, t_enc


def worker_window(args):
    """One stream through frames 0..T (input frame t % clip, IPPP, skipping off; every frame forced IDR in
    enc_i mode), every frame encoded and -- except in enc_i mode -- decoded by the oracle. Returns the time of
    the encode and decode calls of frames first..T (the GPU's timed window: like-for-like content) and the
    sha256 of frame T's NAL bytes and decoded picture (the timed pipeline's last frame, checked after the
    timed region), and the pid of the process that ran it (window() adds busy time per real process)."""
    stream, w, h, bitrate, T, clip, mode, first = args
    sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))
    import numpy as np
    from h264mi.synth import SyntheticStream
    O = ctypes.CDLL(os.path.join(ROOT, 'oracle', 'build', 'libh264_oracle.so'))
    O.h264o_enc_create.restype = ctypes.c_void_p
    O.h264o_dec_create.restype = ctypes.c_void_p
    vp = ctypes.c_void_p
    S = SyntheticStream(stream, w, h)
    frames = [np.ascontiguousarray(S.frame(t)) for t in range(min(clip, T + 1))]
    e = vp(O.h264o_enc_create(w, h, bitrate))
    O.h264o_enc_set_frame_skip(e, 0)
    O.h264o_enc_set_gom_exact(e, gom_exact())
    d = vp(O.h264o_dec_create())
    out = np.zeros(w * h * 4, np.uint8)
    pic = np.zeros(w * h * 3 // 2, np.uint8)
    W, H = ctypes.c_int(), ctypes.c_int()
    t_enc = t_dec = 0.0
    n = 0
    for t in range(T + 1):
        f = frames[t % clip]
        t0 = time.perf_counter()
        if mode == 'enc_i':
            O.h264o_enc_force_idr(e)
        n = O.h264o_enc_encode(e, f.ctypes.data_as(vp), out.ctypes.data_as(vp), ctypes.c_int(out.size))
        t1 = time.perf_counter()
        if mode != 'enc_i':
            O.h264o_dec_decode(d, out.ctypes.data_as(vp), ctypes.c_int(n), pic.ctypes.data_as(vp), ctypes.byref(W), ctypes.byref(H))
        t2 = time.perf_counter()
        if t >= first:
            t_enc += t1 - t0
            t_dec += t2 - t1
    last = {'frame': T, 'nal': hashlib.sha256(out[:n].tobytes()).hexdigest(),
            'pic': hashlib.sha256(pic.tobytes()).hexdigest() if mode != 'enc_i' else None}
    O.h264o_enc_destroy(e)
    O.h264o_dec_destroy(d)
    return stream, t_enc, t_dec, T + 1 - first, last, os.getpid()


def window(streams, w, h, bitrate, T, clip, mode, first, procs):
    """worker_window over the given streams on `procs` processes; each process's busy time is the sum over
    the streams it really ran (the pool hands jobs out dynamically: accounted by the worker's pid), the rate is
    all timed frames / the busiest process (as run())"""
    jobs = [(sid, w, h, bitrate, T, clip, mode, first) for sid in streams]
    with mp.get_context('spawn').Pool(max(1, min(procs, len(jobs)))) as pool:
        res = pool.map(worker_window, jobs, chunksize=1)
    busy, busy_e = {}, {}
    for r in res:
        busy[r[5]] = busy.get(r[5], 0.0) + r[1] + r[2]
        busy_e[r[5]] = busy_e.get(r[5], 0.0) + r[1]
    per, per_e = list(busy.values()), list(busy_e.values())
    counted = sum(r[3] for r in res)
    return {'value': counted / max(per) if max(per) > 0 else None, 'encode_only': counted / max(per_e) if max(per_e) > 0 else None,
            'unit': 'frames/s', 'cores': len(per), 'frames': f'{first}..{T}', 'streams': len(jobs), 'timed_frames': counted,
            'sample': f'streams {streams[0]}..{streams[-1]} x frames {first}..{T} (the GPU timed window, same synthetic '
                      f'inputs, input frame t % {clip}) encoded' + ('' if mode == 'enc_i' else ' + decoded') +
                      f' by the oracle on {len(per)} processes; value = timed frames / busiest process'}, \
        {str(r[0]): r[4] for r in res}


def host_cores():
    """The CPU share this process may use: the affinity mask, capped by OMP_NUM_THREADS when the
    environment sets it (the GPU box sets 16 = its CPU share; nproc there shows the whole host)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else (os.cpu_count() or 1)
    omp = os.environ.get('OMP_NUM_THREADS')
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def run(procs, w, h, bitrate, frames, mode, nhash=0):
    ctx = mp.get_context('spawn')
    jobs = [(s, w, h, bitrate, frames, mode, nhash if s == 0 else 0) for s in range(procs)]
    t0 = time.perf_counter()
    if procs == 1:
        res = [worker(jobs[0])]
    else:
        with ctx.Pool(procs) as pool:
            res = pool.map(worker, jobs)
    wall = time.perf_counter() - t0
    counted = sum(r[1] for r in res)
    busy = max(r[0] for r in res)
    busy_enc = max(r[3] for r in res)
    return counted / busy, counted, busy, wall, res[0][2], (counted / busy_enc if busy_enc > 0 else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--width', type=int, default=1920)
    ap.add_argument('--height', type=int, default=1080)
    ap.add_argument('--bitrate', type=int, default=1000000)
    ap.add_argument('--frames', type=int, default=7, help='frames per process (the first, IDR, is untimed except in enc_i)')
    ap.add_argument('--mode', default='encdec', choices=['encdec', 'enc_i', 'dec'])
    ap.add_argument('--procs', type=int, default=0, help='0: the host CPU share (host_cores())')
    ap.add_argument('--hash', type=int, default=0, help='sha256 of stream 0 frames 0..K-1 (NAL bytes, decoded picture)')
    ap.add_argument('--hash-stream', type=int, default=0, help='synthetic stream id whose frames are hashed')
    ap.add_argument('--hash-only', action='store_true', help='only the parity hashes (no timing; N > 1 ranks)')
    ap.add_argument('--hash-streams', type=int, default=0, help='hash the first K frames of N streams (--hash-first ..)')
    ap.add_argument('--hash-first', type=int, default=0, help='first synthetic stream id of --hash-streams')
    ap.add_argument('--window-last', type=int, default=-1,
                    help='T: run frames 0..T of --hash-streams streams (from --hash-first), time frames --window-first..T '
                         '(the GPU timed window) and hash frame T (the timed pipeline\'s last frame)')
    ap.add_argument('--window-first', type=int, default=0)
    ap.add_argument('--window-streams', type=int, default=0, help='streams in the window job (0: --hash-streams)')
    ap.add_argument('--clip', type=int, default=60, help='input frame t is synthetic frame t % clip (bench.py --clip)')
    a = ap.parse_args()
    allc = a.procs or host_cores()
    streams_hashes = None
    if a.hash_streams > 0 and a.hash > 0:
        jobs = [(sid, a.width, a.height, a.bitrate, a.hash, a.mode, a.hash) for sid in range(a.hash_first, a.hash_first + a.hash_streams)]
        with mp.get_context('spawn').Pool(min(allc, len(jobs))) as pool:
            streams_hashes = {str(j[0]): r[2] for j, r in zip(jobs, pool.map(worker, jobs))}
    win, last = None, None
    if a.window_last >= 0:
        ns = a.window_streams or a.hash_streams or 1
        win, last = window(list(range(a.hash_first, a.hash_first + ns)), a.width, a.height, a.bitrate, a.window_last, a.clip,
                           a.mode, a.window_first, allc)
    if a.hash_only:
        if streams_hashes is not None:
            print(json.dumps({'parity_hashes_streams': streams_hashes, 'parity_last': last, 'window': win}))
            return
        _, _, hashes, _ = worker((a.hash_stream, a.width, a.height, a.bitrate, a.hash, a.mode, a.hash))
        print(json.dumps({'parity_hashes': hashes, 'stream': a.hash_stream}))
        return
    v1, n1, b1, w1, hashes, e1 = run(1, a.width, a.height, a.bitrate, a.frames, a.mode, a.hash)
    vn, nn, bn, wn, _, en = run(allc, a.width, a.height, a.bitrate, a.frames, a.mode) if allc > 1 else (v1, n1, b1, w1, None, e1)
    what = {'encdec': 'P frames encoded+decoded', 'enc_i': 'IDR frames encoded', 'dec': 'P frames decoded'}[a.mode]
    d = {'value': vn, 'unit': 'frames/s', 'cores': allc, 'kind': 'port', 'value_1core': v1,
         'build': 'oracle/build/libh264_oracle.so, gcc -O3 -march=x86-64-v3',
         'sample': f'{allc} procs x 1 stream x {a.frames} frames {a.width}x{a.height} at {a.bitrate} bps '
                   f'({what}; {nn} timed frames, slowest process {bn:.2f} s); 1-core: {n1} frames in {b1:.2f} s',
         'wall_s': round(w1 + wn, 2), 'parity_hashes': hashes, 'parity_hashes_streams': streams_hashes,
         'window': win, 'parity_last': last}
    if a.mode == 'encdec':  # the encode share of the same timed frames (north_star: "host-CPU encode FPS")
        d['encode_only'] = {'value': en, 'value_1core': e1, 'unit': 'frames/s', 'cores': allc,
                            'sample': 'encode calls of the same timed P frames (decode time excluded)'}
    print(json.dumps(d))


if __name__ == '__main__':
    main()
