#!/usr/bin/env python
"""bench.py -- BASELINE.json metric "1080p30 frames/sec encode+decode per GPU" on MI355X.

Parity: the GPU's NAL bytes and decoded pictures are checked against the oracle (oracle/, the CPU
restatement of the reference path) on the bench's own geometry and bitrate: the first frames of every
stream (captured in the warmup) and the last timed frame of every stream (captured after the timed
region); parity with OpenH264 itself is partial. A failed check prints value null and exits 1.

Default workload (the metric; at N > 1 also BASELINE.json configs[4]'s NAL gather): every rank owns
S streams (default 128: the GPU's 1080p30 throughput comes from concurrent independent streams, SURVEY.md
§7; at 128 streams a frame step of all of them takes ~24 ms, inside the 33 ms of a 30 fps frame
interval, so every stream runs in real time; 32 streams give ~20 % less, DESIGN.md §5 Capacity). One
step = one frame of each of them: GPU encode (libh264mi batch encoder,
IPPP, intra period 0, the wrapper's parameters, 1 Mbps) and GPU decode of exactly the NAL units
produced, plus (N > 1) the gather of those NAL units to rank 0 over RCCL. Frames are encoded on one
HIP stream and decoded in groups of G on another (entropy decoding of a group runs concurrently),
overlapped with encoding. Inputs are synthetic I420 clips resident in HBM before the timed region.
value = frames encoded+decoded by all ranks / max-over-ranks wall time of K steps.

Other BASELINE.json configs (one JSON line each, N = 1):
  --config 2  1280x720, every frame IDR (force_key_frame), encode; S streams
  --config 3  1920x1080 IPPP encode+decode, one stream
  --config 4  1920x1080 decode only: 8 concurrent decoders of one 1080p stream (the app.js fan-out)
  --config 5  1920x1080 IPPP encode+decode, 4 streams per GPU (32 over 8 GPUs), NAL gather at N > 1

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C] [--streams S] [--group G]
  --gpus N > 1 without a torch.distributed launcher: bench.py starts `torch.distributed.run` with N
  ranks itself (a child process, before this process touches the GPU) and exits with its code.
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# BASELINE.json's metric names "bit-exact vs OpenH264"; what this build can show is parity with the oracle
# (the CPU restatement) -- OpenH264 parity is unpinned, so the line does not claim it
METRIC = '1080p30 frames/sec encode+decode per GPU'
PARITY_NOTE = 'NAL bytes and decoded pictures == oracle (CPU restatement) at this config; OpenH264 parity unpinned'


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=240)
    ap.add_argument('--warmup', type=int, default=16)
    ap.add_argument('--config', type=int, default=0, choices=[0, 2, 3, 4, 5], help='0 = the metric workload')
    ap.add_argument('--streams', type=int, default=0,
                    help='streams per GPU (default: 32 for the metric; config 3: 1, config 4: 8 decoders, config 5: 4)')
    ap.add_argument('--width', type=int, default=0)
    ap.add_argument('--height', type=int, default=0)
    ap.add_argument('--bitrate', type=int, default=1000000)
    ap.add_argument('--clip', type=int, default=60, help='frames per stream kept resident (IPPP continues across wrap)')
    ap.add_argument('--group', type=int, default=0,
                    help='frames per stream per decode call (frame-parallel entropy decoding); default 4, 16 for the '
                         'decode-only config (no encoder latency to hide: more slices in flight)')
    ap.add_argument('--tail-streamed', type=int, default=1, choices=[0, 1],
                    help='reconstruct the frame-by-frame tail calls streamed (h264mi_dec_set_streamed 1: each frame\'s '
                         'reconstruction rows follow its slice data instead of waiting for the whole parse launch); '
                         'only with the reserved decode lane, whose CUs the waiting waves cannot take')
    ap.add_argument('--no-decode', action='store_true',
                    help='diagnostics: encode only (the metric line then counts encoded frames; not the metric)')
    ap.add_argument('--recon-gate-frac', type=float, default=1.0,
                    help='with --recon-gate: the fraction of the encoder launch\'s MB rows that must have started')
    ap.add_argument('--recon-gate', type=int, default=0, choices=[0, 1],
                    help='start each decoded frame\'s reconstruction once the encoder launch running two frames later has '
                         'started all its MB rows (h264mi_dec_set_recon_gate on h264mi_enc_rows_counter): the reconstruction '
                         'then fills the encoder launch\'s tail instead of sharing its densest part')
    ap.add_argument('--no-tail-frames', dest='tail_frames', action='store_false',
                    help='decode the last group of a run as one call too (default: frame by frame)')
    ap.add_argument('--stages', type=int, default=4, help='NAL staging buffers (groups in flight between encoder and decoder)')
    ap.add_argument('--parse-streams', type=int, default=3, help='HIP streams the decoder rotates entropy decoding over')
    ap.add_argument('--parse-cus', type=int, default=-1,
                    help='CUs reserved for entropy decoding (CU mask bits [0, n) for the parse streams, the rest for the '
                         'encoder / reconstruction streams); 0 = shared; default when encoding and decoding: 20 per 128 '
                         'slices per call (>= 128), else 24; 0 for decode-only')
    ap.add_argument('--recon-cus', type=int, default=0,
                    help='CUs reserved for the reconstruction stream (mask bits [parse_cus, parse_cus + n)); the encoder '
                         'keeps the rest. 0 = reconstruction shares the encoder\'s CUs')
    ap.add_argument('--enc-groups', type=int, default=0,
                    help='the streams are encoded by this many encoders (S / groups streams each) on their own HIP '
                         'streams, so that one group\'s wavefront ramp overlaps another\'s frame')
    ap.add_argument('--dec-groups', type=int, default=1,
                    help='the streams are decoded by this many decoders (S / groups streams each), each reconstructing '
                         'on its own HIP stream')
    ap.add_argument('--streamed', type=int, default=-1, choices=[-1, 0, 1],
                    help='streamed reconstruction (h264mi_dec_set_streamed; -1: the library\'s automatic choice, which '
                         'leaves a 32-stream decoder unstreamed: its 4352 waiting reconstruction waves would hold the CUs '
                         'the encoder needs while a long slice parses -- profiles/round4/timeline_streamed_tail.txt)')
    ap.add_argument('--gom-exact', action='store_true',
                    help='P-frame QPs by OpenH264\'s exact GOM rate control (H264MI_GOM_EXACT=1 for the encoders and the '
                         'oracle); default: this project\'s MB-row plan (DESIGN.md §3.6)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-frames', type=int, default=7)
    ap.add_argument('--parity-frames', type=int, default=4, help='frames of stream 0 checked against the oracle before timing')
    ap.add_argument('--no-traffic', action='store_true', help='skip the rocprofv3 --pmc passes that measure roofline.traffic')
    ap.add_argument('--traffic-probe', action='store_true', help=argparse.SUPPRESS)  # child of measure_traffic()
    a = ap.parse_args()
    if a.gom_exact:  # before any child process starts and before the library is loaded
        os.environ['H264MI_GOM_EXACT'] = '1'
    if a.config == 2:
        a.width, a.height = a.width or 1280, a.height or 720
    a.width, a.height = a.width or 1920, a.height or 1080
    # the metric workload: 128 streams per GPU (round 6, profiles/round6/sweep_streams.txt: 32 streams 4296-4320
    # frames/s, 64 4820, 96 5079, 128 5108-5323, 192 5275, 256 5181-5362 -- the pipeline fills the chip from ~128)
    a.streams = a.streams or {2: 8, 3: 1, 4: 8, 5: 4}.get(a.config, 128)
    a.group = a.group or (16 if a.config == 4 else 4)
    # one encoder: two of 16 streams each on their own HIP streams measured within noise of it (3826-3922 vs
    # 3738-3902 frames/s over 8 runs, profiles/round4/ab_enc_groups*.txt) and halve the per-launch roofline
    a.enc_groups = a.enc_groups or 1
    if a.parse_cus < 0:  # a reserved decode lane pays only beside the encoder's wavefronts
        # a slice wave takes a quarter of a CU's LDS (four per CU). Round 5, after the reconstruction's
        # latency work (profiles/round5/sweep_parse_cus_final.txt): the 128 slices of a 32-stream, 4-frame call
        # run best on the fewest CUs that take them in two rounds -- 16 CUs 4517-4546 frames/s, 20 4512-4521,
        # 24 4501, 32 4485-4492, 40 4211-4230; 12 and 8 (three and four rounds) drop to 3655. 20 keeps a round's
        # margin: 20 CUs per 128 slices, in steps of 4 (smaller calls keep the earlier 24)
        # Round 6 at 512 and 1024 slices (128 / 256 streams): 32 CUs (four slice waves each: 4 and 8 full rounds)
        # beat 24 (5108 / 5181), 28 (5091), 36 (4904), 40 (4969 / 5107), 48 (4984) and 80 (4309 / 4336)
        sl = a.streams * a.group
        a.parse_cus = ((20 if sl <= 128 else 24 if sl < 512 else 32) if sl >= 128 else 24) if a.config in (0, 3, 5) else 0
    # Hardware queues per process: the pipeline drives the encoder stream, the reconstruction stream and
    # the decoder's entropy-decoding streams (runtime_dec.inc); with HIP's default of 4 queues parse
    # streams share queues and their kernels serialise. Set before the HIP runtime initialises.
    need = max(8, a.dec_groups * (a.parse_streams + 1) + 3 + a.enc_groups)
    if int(os.environ.get('GPU_MAX_HW_QUEUES', '4') or 4) < need:
        os.environ['GPU_MAX_HW_QUEUES'] = str(min(need, 32))
    return a


def relaunch(a):
    """--gpus N > 1 outside a distributed launcher: run N ranks as a child torch.distributed.run
    (nothing here has touched the GPU) and return its exit code."""
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={a.gpus}',
           '--master-addr', '127.0.0.1', '--master-port', str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=dict(os.environ)).returncode


# the reference's only published numbers (a screenshot: wasm OpenH264 at 854x480, 1 Mbps)
# scaled by macroblock count to 1080p give, per core of that machine, ~79 encodes/s and ~41.7
# encode+decode frames/s. An estimate of OpenH264's CPU speed, not a measurement (OpenH264 itself is
# never run here).
OPENH264_1080P_PER_CORE = {'encdec': 41.7, 'encode': 79.0}


def openh264_estimate(a, cores):
    """the screenshot-implied OpenH264 rate on the box's cores for the metric's 1080p IPPP encode+decode
    configs (None for the I-only and decode-only configs, which the screenshot does not price)"""
    if a.config not in (0, 3, 5) or (a.width, a.height) != (1920, 1080) or not cores:
        return None
    return {'value': OPENH264_1080P_PER_CORE['encdec'] * cores, 'encode_only': OPENH264_1080P_PER_CORE['encode'] * cores,
            'unit': 'frames/s', 'cores': cores, 'kind': 'estimate',
            'basis': 'BASELINE.md §1: screenshot-implied per-core 1080p rates of the reference\'s wasm OpenH264 '
                     '(41.7 encode+decode, 79 encode-only frames/s per core) x the box\'s cores, assuming linear '
                     'scaling over independent streams; an estimate, not a measurement'}


def window_args(a, mode):
    """the CPU leg's window job: frames 0..T (T = the timed pipeline's last frame) of the bench's streams through
    the oracle, timed over the GPU's own window (warmup..T) and hashed at T. Every stream while T + 1 <= 96
    frames (32 x 25 1080p frames take ~12 s on 16 host cores); longer runs check as many streams as the host
    has cores (one stream's serial chain per core) so that the default bench stays within minutes."""
    if mode == 'dec':
        return []
    T = a.warmup + a.steps - 1
    # N > 1: every rank's CPU leg runs on the one host beside the others', so each checks the last frame of its
    # first 32 streams (frames 0..parity_frames-1 of all of them are checked regardless)
    ns = (a.streams if getattr(a, 'world', 1) == 1 else min(a.streams, 32)) if T + 1 <= 96 else min(a.streams, 16)
    return ['--window-last', str(T), '--window-first', str(a.warmup), '--window-streams', str(ns), '--clip', str(a.clip)]


def cpu_baseline(a, mode):
    """the CPU leg (a child process, before this process touches the GPU): the timed baseline, plus the
    oracle's hashes of the first parity_frames frames of every stream the timed pipeline encodes and of
    its last timed frame (window_args)"""
    cmd = [sys.executable, os.path.join(ROOT, 'tools', 'cpu_baseline.py'), '--width', str(a.width), '--height', str(a.height),
           '--bitrate', str(a.bitrate), '--frames', str(a.cpu_frames), '--mode', mode, '--hash', str(a.parity_frames)]
    if mode != 'dec':
        cmd += ['--hash-streams', str(a.streams)] + window_args(a, mode)
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        d = json.loads([l for l in r.stdout.splitlines() if l.startswith('{')][-1])
        return d
    except Exception as e:  # reported, never silently replaced
        return {'value': None, 'unit': 'frames/s', 'cores': None, 'kind': 'port', 'sample': f'failed: {e!r}', 'parity_hashes': None}


TRAFFIC_FRAMES, TRAFFIC_SKIP = 12, 2  # probe frames; dispatches excluded from the average (IDR, first P)


def traffic_probe(a):
    """child of measure_traffic(), run under rocprofv3 --pmc. Encoding configs: the bench's encoder alone
    (S streams, geometry, bitrate, frame skipping off) for TRAFFIC_FRAMES frames; enc_mb_kernel dispatch
    k = frame k. Config 4: one stream encoded, then decoded frame by frame by S decoders; dec_recon_kernel
    dispatch k = frame k of all S decoders."""
    import numpy as np
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    W, H, S = a.width, a.height, a.streams
    if a.config == 4:
        g = SyntheticStream(0, W, H)
        enc = h264mi.BatchEncoder(W, H, a.bitrate, 1)
        enc.set_frame_skip(False)
        dec = h264mi.BatchDecoder(W, H, S)
        for t in range(TRAFFIC_FRAMES):
            enc.encode(torch.from_numpy(np.ascontiguousarray(g.frame(t))).cuda())
            n = enc.nal_sizes()[0]
            dec.decode([enc.nal_ptr(0)] * S, [n] * S)
            dec.status()
        dec.close()
        enc.close()
        return
    gens = [SyntheticStream(s, W, H) for s in range(S)]
    enc = h264mi.BatchEncoder(W, H, a.bitrate, S)
    enc.set_frame_skip(False)
    for t in range(TRAFFIC_FRAMES):
        if a.config == 2:
            enc.force_idr(-1)
        enc.encode(torch.from_numpy(np.concatenate([g.frame(t) for g in gens])).cuda())
    torch.cuda.synchronize()
    enc.close()


def measure_traffic(a):
    """HBM bytes per launch of the line's dominant kernel (a.traffic_kernel: enc_mb_kernel, or
    dec_recon_kernel for config 4), measured in this run: two rocprofv3 --pmc passes (FETCH_SIZE, then
    WRITE_SIZE: they do not fit one pass) over a child that runs the bench's encoder (decoders), started
    before this process touches the GPU. gfx950 (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts half the
    bytes of wide streaming reads, so read bytes = 2 x FETCH_SIZE; both counters are KiB."""
    kname = a.traffic_kernel
    import csv
    import glob
    import shutil
    import tempfile
    if not shutil.which('rocprofv3'):
        return None, 'rocprofv3 not found'
    vals = {}
    work = tempfile.mkdtemp(prefix='h264mi_pmc_', dir='/tmp')
    env = dict(os.environ, TMPDIR='/tmp')
    for ctr in ('FETCH_SIZE', 'WRITE_SIZE'):
        d = os.path.join(work, ctr)
        cmd = ['rocprofv3', '--pmc', ctr, '-d', d, '-o', 'run', '--output-format', 'csv', '--', sys.executable,
               os.path.abspath(__file__), '--traffic-probe', '--config', str(a.config),
               '--streams', str(a.streams // max(1, a.enc_groups) if kname == 'enc_mb_kernel' else a.streams),
               '--width', str(a.width), '--height', str(a.height), '--bitrate', str(a.bitrate)]
        try:
            subprocess.run(cmd, cwd='/tmp', env=env, capture_output=True, text=True, timeout=180)
        except Exception as e:  # reported, never replaced by a stored figure
            return None, f'{ctr} pass failed: {e!r}'
        per = {}
        for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
            for r in csv.DictReader(open(f)):
                if kname in r['Kernel_Name'] and r['Counter_Name'] == ctr:
                    per[int(r['Dispatch_Id'])] = per.get(int(r['Dispatch_Id']), 0.0) + float(r['Counter_Value'])
        ks = sorted(per)[TRAFFIC_SKIP:]
        if not ks:
            return None, f'{ctr}: no {kname} dispatches recorded'
        vals[ctr] = sum(per[k] for k in ks) / len(ks)
    shutil.rmtree(work, ignore_errors=True)
    hbm = (2 * vals['FETCH_SIZE'] + vals['WRITE_SIZE']) * 1024
    raw = (vals['FETCH_SIZE'] + vals['WRITE_SIZE']) * 1024
    a.traffic_raw = raw
    return hbm, (f'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes in this run over {kname} dispatches '
                 f'{TRAFFIC_SKIP}..{TRAFFIC_FRAMES - 1} of the bench ' + ('decoders' if kname == 'dec_recon_kernel' else 'encoder') + '; bytes = (2 x FETCH_SIZE + WRITE_SIZE) KiB x 1024 '
                 f'(read {2 * vals["FETCH_SIZE"] * 1024 / 1e6:.1f} MB, written {vals["WRITE_SIZE"] * 1024 / 1e6:.1f} MB). '
                 f'The doubling is the guide\'s gfx950 correction for wide streaming reads; this kernel also does narrow '
                 f'loads, so 2 x FETCH_SIZE is an upper bound on its reads and the raw counters ({raw / 1e6:.1f} MB) a lower bound')


PARSE_SQ = ('SQ_WAVE_CYCLES', 'SQ_INSTS_SALU', 'SQ_INSTS_VALU', 'SQ_INSTS_BRANCH', 'SQ_INSTS_SMEM', 'SQ_INSTS_LDS',
            'SQ_WAIT_ANY', 'SQ_ACTIVE_INST_ANY')  # one pass: 8 SQ counters (the block's limit)


def measure_parse_mix(a):
    """dec_parse_kernel's instruction mix and issue rate, measured in this run: one rocprofv3
    --pmc pass over a short child bench of the same workload (--steps 4 --warmup 4, no CPU leg, no PMC of its
    own; the first dispatch, the IDR's I slices, is left out). A slice is one wave whose CAVLC chain issues at
    most one instruction per quad-cycle (~4.3 cycles per independent SALU op on gfx950), so
    issue_frac = instructions / SQ_WAVE_CYCLES (quad-cycles) is the fraction of that per-wave issue bound the
    slices reach; the rest is dependency latency (taken branches, readlane -> SALU, LDS) and waits."""
    import csv
    import glob
    import shutil
    import tempfile
    if not shutil.which('rocprofv3'):
        return {'note': 'rocprofv3 not found'}
    work = tempfile.mkdtemp(prefix='h264mi_pmc_parse_', dir='/tmp')
    cmd = ['rocprofv3', '--pmc', *PARSE_SQ, '-d', work, '-o', 'run', '--output-format', 'csv', '--', sys.executable,
           os.path.abspath(__file__), '--no-cpu-baseline', '--no-traffic', '--steps', '4', '--warmup', '4', '--clip', '8',
           '--config', str(a.config), '--streams', str(a.streams), '--width', str(a.width), '--height', str(a.height),
           '--bitrate', str(a.bitrate), '--group', str(a.group), '--parse-cus', str(a.parse_cus),
           '--parse-streams', str(a.parse_streams), '--enc-groups', str(a.enc_groups), '--dec-groups', str(a.dec_groups)]
    try:
        subprocess.run(cmd, cwd='/tmp', env=dict(os.environ, TMPDIR='/tmp'), capture_output=True, text=True, timeout=240)
    except Exception as e:  # reported, never replaced by a stored figure
        shutil.rmtree(work, ignore_errors=True)
        return {'note': f'PMC pass failed: {e!r}'}
    per = {}
    for f in glob.glob(os.path.join(work, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if 'dec_parse_kernel' in r['Kernel_Name']:
                d = per.setdefault(int(r['Dispatch_Id']), {})
                d[r['Counter_Name']] = d.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    shutil.rmtree(work, ignore_errors=True)
    ks = sorted(per)[1:]
    if not ks:
        return {'note': 'no dec_parse_kernel dispatches recorded'}
    t = {c: sum(per[k].get(c, 0.0) for k in ks) for c in PARSE_SQ}
    insts = sum(t[c] for c in PARSE_SQ[1:6])
    wc = t['SQ_WAVE_CYCLES'] or 1.0
    return {'dispatches': len(ks), 'instructions': insts, 'wave_quad_cycles': t['SQ_WAVE_CYCLES'],
            'issue_frac': insts / wc, 'salu_share': t['SQ_INSTS_SALU'] / max(insts, 1.0),
            'branch_share': t['SQ_INSTS_BRANCH'] / max(insts, 1.0), 'active_frac': t['SQ_ACTIVE_INST_ANY'] / wc,
            'wait_frac': t['SQ_WAIT_ANY'] / wc,
            'note': 'rocprofv3 --pmc ' + ' '.join(PARSE_SQ) + ' over dec_parse_kernel dispatches 2.. of a 4 + 4-step child '
                    'bench of this workload; instructions = SALU + VALU + BRANCH + SMEM + LDS; issue_frac = instructions '
                    '/ SQ_WAVE_CYCLES (quad-cycles: 1.0 = one instruction per 4 cycles per wave, the per-wave issue bound)'}


def oracle_hashes(a, mode, first):
    """the oracle's sha256 of the first frames of this rank's streams first..first+S-1 (N > 1 ranks;
    child process, no GPU): {str(stream id): [{'nal', 'pic'}, ...]}"""
    cmd = [sys.executable, os.path.join(ROOT, 'tools', 'cpu_baseline.py'), '--width', str(a.width), '--height', str(a.height),
           '--bitrate', str(a.bitrate), '--mode', mode, '--hash', str(a.parity_frames), '--hash-first', str(first),
           '--hash-streams', str(a.streams), '--hash-only'] + window_args(a, mode)
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        d = json.loads([l for l in r.stdout.splitlines() if l.startswith('{')][-1])
        return d['parity_hashes_streams'], d.get('parity_last')
    except Exception:
        return {}, None  # reported as a failed parity check (no hashes)


def gpu_parity(a, oracle_hashes, i_only=False, sid=0):
    """Stream sid's first frames on the GPU (fresh encoder + decoder, the bench's geometry and bitrate)
    vs the oracle's sha256 of the same frames: NAL bytes and decoded pictures."""
    import numpy as np
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    if not oracle_hashes:
        return False, 'no oracle hashes (CPU baseline leg failed or skipped)'
    g = SyntheticStream(sid, a.width, a.height)
    enc = h264mi.BatchEncoder(a.width, a.height, a.bitrate, 1)
    enc.set_frame_skip(False)  # as the timed encoder (see bench_encode)
    dec = h264mi.BatchDecoder(a.width, a.height, 1)
    ok = True
    for t, want in enumerate(oracle_hashes):
        f = torch.from_numpy(np.ascontiguousarray(g.frame(t))).cuda()
        if i_only:
            enc.force_idr(0)
        enc.encode(f)
        n = enc.nal_sizes()[0]
        nal = enc.nal_bytes(0, n)
        dec.decode([enc.nal_ptr(0)], [n])
        rc, got = dec.status()
        pic = dec.picture_i420(0) if rc == 0 and got[0] else b''
        ok = ok and hashlib.sha256(nal).hexdigest() == want['nal'] and hashlib.sha256(pic).hexdigest() == want['pic']
    enc.close()
    dec.close()
    return ok, f'stream {sid} frames 0..{len(oracle_hashes) - 1}: ' + ('pass' if ok else 'FAIL')


def all_stream_parity(captured, shashes, sids, a, decoded):
    """frames 0..K-1 of every stream of the timed pipeline (captured during its warmup) vs the oracle's
    sha256 of the same synthetic streams: NAL bytes, and decoded pictures when the pipeline decodes"""
    K = a.parity_frames
    if not captured:
        return False, f'not checked (warmup {a.warmup} < {K} frames, or no capture)'
    bad = []
    for s, sid in enumerate(sids):
        want = shashes.get(str(sid)) or []
        got = captured.get(s) or []
        ok = len(want) == K and len(got) == K and all(
            g['nal'] == w['nal'] and (not decoded or g['pic'] == w['pic']) for g, w in zip(got, want))
        if not ok:
            bad.append(sid)
    what = 'NAL bytes' + (' and decoded pictures' if decoded else '')
    msg = f'{len(sids)} streams x {K} frames of the timed pipeline ({what}) vs the oracle: '
    return not bad, msg + ('pass' if not bad else f'FAIL (streams {bad[:8]})')


def last_frame_parity(got, want, sids, decoded):
    """the timed pipeline's last frame of every stream the CPU leg ran (all streams unless the run is long;
    window_args) after the timed region: NAL bytes (and decoded pictures) vs the oracle's sha256"""
    if not want:
        return False, 'last timed frame: not checked (no oracle hashes)'
    if got is None:
        return False, 'last timed frame: not captured'
    bad, n, T = [], 0, None
    for s, sid in enumerate(sids):
        w = want.get(str(sid))
        if w is None:
            continue
        n += 1
        T = w['frame']
        g = got[s]
        if g['nal'] != w['nal'] or (decoded and g['pic'] != w['pic']):
            bad.append(sid)
    what = 'NAL bytes' + (' and decoded pictures' if decoded else '')
    msg = f'last timed frame {T} of {n} streams ({what}, after the timed region) vs the oracle: '
    return n > 0 and not bad, msg + ('pass' if n and not bad else f'FAIL (streams {bad[:8]})')


def timed(run_steps, K, W, dist, sync):
    run_steps(W)
    sync()
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    run_steps(K)
    sync()
    if dist:
        dist.barrier()
    return time.perf_counter() - t0


def main():
    a = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if a.gpus > 1 and 'RANK' not in os.environ:
        sys.exit(relaunch(a))
    if a.gpus != world:
        print(f'bench.py: --gpus {a.gpus} but WORLD_SIZE {world}', file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    a.world = world
    if a.traffic_probe:
        return traffic_probe(a)
    mode = {2: 'enc_i', 4: 'dec'}.get(a.config, 'encdec')
    # CPU baseline + oracle parity hashes first, in child processes, before this process touches the GPU.
    # At N > 1 every rank takes the oracle's hashes of its own first stream (no timing).
    cpu, hashes, shashes, last = None, None, None, None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(a, mode)
        hashes = cpu.get('parity_hashes')
        shashes = cpu.get('parity_hashes_streams')
        last = cpu.get('parity_last')
    elif world > 1 and not a.no_cpu_baseline:
        shashes, last = oracle_hashes(a, mode, rank * a.streams)
    a.traffic_kernel = 'dec_recon_kernel' if a.config == 4 else 'enc_mb_kernel'
    a.traffic_measured = (None, 'not measured (--no-traffic or N > 1)')
    a.parse_mix = None
    if rank == 0 and world == 1 and not a.no_traffic:
        a.traffic_measured = measure_traffic(a)
        if a.config in (0, 3, 5) and not a.no_decode:
            a.parse_mix = measure_parse_mix(a)
    import numpy as np
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    from h264mi.shard import NalGather, stream_ids
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)
    W, H, S, G = a.width, a.height, a.streams, a.group
    F = W * H * 3 // 2
    sync = torch.cuda.synchronize
    res = {}
    if a.config == 4:
        res = bench_decode_only(a, torch, np, h264mi, SyntheticStream, dev, sync)
    else:
        # parity: the timed pipeline's own encoder and decoder, every stream, frames 0..K-1 (captured in
        # the warmup, which starts at frame 0) against the oracle's hashes of the same streams
        cap = a.parity_frames if shashes is not None and a.warmup >= a.parity_frames else 0
        res = bench_encode(a, torch, np, h264mi, SyntheticStream, NalGather, stream_ids, dev, sync, dist, world, rank, cap)
    parity_ok, parity_msg = True, 'skipped (--no-cpu-baseline)'
    if a.config == 4 and hashes is not None:
        # decode-only: the bench's stream 0 (its decoders all decode that stream) from a fresh encoder +
        # decoder after the timed region
        parity_ok, parity_msg = gpu_parity(a, hashes, sid=0)
    elif shashes is not None:
        parity_ok, parity_msg = all_stream_parity(res.pop('captured', None), shashes, stream_ids(rank, a.streams), a,
                                                  decoded=a.config != 2)
        lok, lmsg = last_frame_parity(res.pop('last_frame', None), last, stream_ids(rank, a.streams), decoded=a.config != 2)
        parity_ok, parity_msg = parity_ok and lok, parity_msg + '; ' + lmsg
        if world > 1:
            parity_msg = f'rank {rank}: ' + parity_msg
    res.pop('captured', None)
    parity_ok = parity_ok and res.pop('selfcheck_ok')
    elapsed = res.pop('elapsed')
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt[0])
        ok = torch.tensor([1 if parity_ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        parity_ok = bool(ok.item())
        if shashes is not None:
            nl = int(window_args(a, mode)[5]) if window_args(a, mode) else 0
            parity_msg = (f'all {world} ranks x {a.streams} streams x frames 0..{a.parity_frames - 1} and the last timed frame '
                          f'{a.warmup + a.steps - 1} of the first {nl} streams of each rank, of the timed pipeline vs the oracle: '
                          + ('pass' if parity_ok else 'FAIL'))
    frames = res.pop('frames_per_rank') * world
    value = frames / elapsed
    if rank == 0:
        vs = None
        if cpu is not None:
            cpu = {k: cpu.get(k) for k in ('value', 'unit', 'cores', 'kind', 'sample', 'value_1core', 'build', 'encode_only',
                                           'window') if k in cpu}
            if cpu.get('window') and cpu['window'].get('value'):
                # like-for-like: the restatement over the GPU's own timed frames of the same streams is
                # the line's baseline; the short early-frame sample (frames 1..cpu_frames-1) is kept beside it
                w_ = cpu.pop('window')
                cpu['early_frames'] = {k: cpu.pop(k) for k in ('value', 'sample', 'value_1core', 'encode_only') if k in cpu}
                cpu.update({'value': w_['value'], 'cores': w_['cores'], 'sample': w_['sample'],
                            'encode_only': {'value': w_['encode_only'], 'unit': 'frames/s', 'cores': w_['cores'],
                                            'sample': 'encode calls of the same timed frames (decode time excluded)'},
                            'window_frames': w_['frames'], 'window_streams': w_['streams']})
            est = openh264_estimate(a, cpu.get('cores'))
            if est is not None:
                cpu['openh264_estimate'] = est
                vs = value / est['value'] if parity_ok else None
                cpu['ratios'] = {'value_over_openh264_estimate': vs,
                                 'value_over_openh264_encode_estimate': value / est['encode_only'] if parity_ok else None,
                                 'value_over_restatement': value / cpu['value'] if parity_ok and cpu.get('value') else None}
        out = {
            'metric': METRIC + ' (parity vs oracle; OpenH264 parity unpinned)',
            'value': value if parity_ok else None, 'unit': 'frames/s', 'n_gpus': world, 'steps': a.steps, 'warmup': a.warmup,
            'ms_per_step': elapsed / a.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': vs, 'dtype': 'u8', 'data': 'synthetic',
            'config': res.pop('config'),
            'roofline': res.pop('roofline'),
            'cpu_baseline': cpu,
            'parity': {'vs_oracle': parity_msg, 'selfcheck': res.pop('selfcheck'), 'note': PARITY_NOTE},
        }
        out.update(res)
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()
    if not parity_ok:
        sys.exit(1)


def roofline(kernel, alg_bytes, ms_total, launches, a, note=None):
    kavg = ms_total / max(launches, 1)
    achieved = alg_bytes / (kavg / 1e3) / 1e9 if kavg > 0 else 0.0
    traffic, tnote = a.traffic_measured if kernel == a.traffic_kernel else (None, 'no PMC pass for this kernel')
    raw = getattr(a, 'traffic_raw', None) if traffic else None
    r = {'bound': 'hbm', 'kernel': kernel, 'achieved': achieved, 'peak': HBM_PEAK_GBPS, 'unit': 'GB/s',
         'frac': achieved / HBM_PEAK_GBPS, 'traffic': traffic, 'alg_bytes_per_launch': alg_bytes, 'avg_launch_ms': kavg,
         'launches': launches, 'traffic_note': tnote,
         'traffic_range': [raw, traffic] if traffic else None,
         'traffic_x_alg': traffic / alg_bytes if traffic else None}
    if note:
        r['note'] = note
    return r


def bench_encode(a, torch, np, h264mi, SyntheticStream, NalGather, stream_ids, dev, sync, dist, world, rank, capture=0):
    """configs 0 (metric), 2 (I-only encode), 3 (one stream), 5 (4 streams): encode (+ decode). capture = K:
    the warmup keeps every stream's NAL units and decoded pictures of frames 0..K-1 (parity check)"""
    W, H, S, G = a.width, a.height, a.streams, a.group
    F = W * H * 3 // 2
    i_only = a.config == 2
    decode = not i_only and not a.no_decode
    clip = torch.empty((a.clip, S * F), dtype=torch.uint8, device=dev)
    for i, sid in enumerate(stream_ids(rank, S)):
        g = SyntheticStream(sid, W, H)
        clip[:, i * F:(i + 1) * F].copy_(torch.from_numpy(np.stack([g.frame(t) for t in range(a.clip)])))
    sync()
    # The encoder codes frame t of all S streams on `es` (P frames chain through its reconstruction,
    # so it is sequential in time) and copies each frame's NAL units to a staging slot; the decoder,
    # on `ds`, takes G frames per call, entropy-decoding all G x S slices concurrently before
    # reconstructing them in order. NB staging buffers keep NB groups in flight: encoding group g+1
    # overlaps the entropy decoding of g and the reconstruction of g-1.
    EG, DG = a.enc_groups, a.dec_groups
    assert EG >= 1 and S % EG == 0 and DG >= 1 and S % DG == 0, '--enc-groups / --dec-groups must divide the streams'
    Sg, Sd = S // EG, S // DG
    if a.parse_cus > 0 and a.recon_cus > 0:  # three lanes: entropy decoding, reconstruction, encoder
        hi = a.parse_cus + a.recon_cus
        ess, dss = [h264mi.masked_stream(0, hi, True) for _ in range(EG)], [h264mi.masked_stream(a.parse_cus, hi, False) for _ in range(DG)]
    elif a.parse_cus > 0:  # wavefront streams off the CUs reserved for entropy decoding
        ess, dss = [h264mi.masked_stream(0, a.parse_cus, True) for _ in range(EG)], [h264mi.masked_stream(0, a.parse_cus, True) for _ in range(DG)]
    else:
        ess, dss = [torch.cuda.Stream(device=dev) for _ in range(EG)], [torch.cuda.Stream(device=dev) for _ in range(DG)]
    # EG encoders of Sg streams each, one HIP stream each (stream s = group s // Sg, index s % Sg)
    encs = [h264mi.BatchEncoder(W, H, a.bitrate, Sg, stream=e) for e in ess]
    # frame skipping off: every step codes a frame (at 1 Mbps the synthetic 1080p content overflows
    # the rate control's buffer and most frames would be dropped)
    for enc in encs:
        enc.set_frame_skip(False)
    # DG decoders of Sd streams each (stream s = decoder s // Sd, index s % Sd), each reconstructing on its
    # own HIP stream; their entropy decoding shares the reserved parse CUs
    decs = [h264mi.BatchDecoder(W, H, Sd, stream=d, max_frames=G) for d in dss] if decode else []
    for dec in decs:
        if a.parse_streams != 3:
            dec.set_parse_streams(a.parse_streams)
        if a.parse_cus > 0:
            dec.set_parse_cus(0, a.parse_cus)
        dec.set_streamed(a.streamed)
    streamed_mode = all(dec.streamed() for dec in decs) if decs else False
    slot = 1 << 21  # bytes per staged access unit (a 1080p IDR at 1 Mbps is ~100 KB)
    NB = max(2, a.stages)
    stage = [torch.empty((G, S * slot), dtype=torch.uint8, device=dev) for _ in range(NB)]
    stage_sz = [torch.zeros((G, S), dtype=torch.int32, device=dev) for _ in range(NB)]
    ev_enc = [[torch.cuda.Event() for _ in range(EG)] for _ in range(NB)]
    ev_dec = [[torch.cuda.Event() for _ in range(DG)] for _ in range(NB)]
    gather = NalGather(dist, torch, S, slot, G, rank, world, dev) if world > 1 else None
    # the size all-gather and the sends of a group are ordered after the encoder's staging of that group
    # only (a stream of their own), never after its decode: NalGather's host reads are one group late
    gs = torch.cuda.Stream(device=dev) if gather is not None else None
    state = {'t': 0, 'g': 0}
    cap_nal = []  # (stage copy, sizes copy) of frames 0..capture-1
    cap_pic = torch.empty((capture, S, W * H * 3 // 2), dtype=torch.uint8, device=dev) if capture and decode else None

    R_enc = (S // EG) * ((H + 15) // 16)  # MB-row workgroups per encoder launch (h264mi_enc_rows_counter steps)

    def run_group(n, tail=False):
        b = state['g'] % NB
        t0 = state['t']
        for k, (enc, es) in enumerate(zip(encs, ess)):
            with torch.cuda.stream(es):
                for e in ev_dec[b]:
                    es.wait_event(e)  # the decoders have finished with this staging buffer
                if gather is not None and gather.done_event(b) is not None:
                    es.wait_event(gather.done_event(b))  # and the NAL gather's sends of it
                for j in range(n):
                    if i_only:
                        enc.force_idr(-1)
                    enc.encode(clip[(t0 + j) % a.clip][k * Sg * F:(k + 1) * Sg * F])
                    enc.copy_nals(stage[b][j][k * Sg * slot:(k + 1) * Sg * slot], slot, stage_sz[b][j][k * Sg:(k + 1) * Sg])
                ev_enc[b][k].record(es)
        state['t'] = t0 + n
        state['last'] = (b, n - 1)
        for d, ds in enumerate(dss):
            with torch.cuda.stream(ds):
                for e in ev_enc[b]:
                    ds.wait_event(e)
                if d == 0:
                    for j in range(n):
                        if t0 + j < capture:
                            cap_nal.append((stage[b][j].clone(), stage_sz[b][j].clone()))
                if decode:
                    base = stage[b].data_ptr()
                    ss = range(d * Sd, (d + 1) * Sd)
                    ptrs = [base + j * S * slot + s * slot for j in range(n) for s in ss]
                    szp = [stage_sz[b].data_ptr() + 4 * (j * S + s) for j in range(n) for s in ss]
                    outp = None
                    if t0 < capture:  # every frame's picture of the first frames (parity capture, warmup only)
                        outp = [cap_pic[t0 + j, s].data_ptr() if t0 + j < capture else 0 for j in range(n) for s in ss]
                    if a.recon_gate and not tail:
                        # frame t0 + j reconstructs once encoder launch t0 + n + j has started all its rows (launch k
                        # = frame k of this run); only launches this segment will still enqueue
                        cnt = max(0, min(n, state['seg_end'] - (t0 + n)))
                        if cnt:
                            decs[d].set_recon_gate(encs[0].rows_counter(), (t0 + n) * R_enc + int(a.recon_gate_frac * R_enc), R_enc, cnt)
                    decs[d].decode_frames(ptrs, size_ptrs=szp, ready_event=ev_enc[b], out_ptrs=outp)
                ev_dec[b][d].record(ds)
        if gather is not None:
            with torch.cuda.stream(gs):
                for e in ev_enc[b]:
                    gs.wait_event(e)
                gather.submit(stage[b], stage_sz[b], n, b)  # sizes gathered once per group; sends of the previous group
        state['g'] += 1

    tail_streamed = bool(a.tail_streamed and decs and a.parse_cus > 0 and a.tail_frames)

    def set_tail(on):  # the tail's reconstruction streamed behind its slice data (a forced, gated launch)
        if tail_streamed:
            for dec in decs:
                dec.set_streamed(1 if on else a.streamed)

    def run_steps(k):
        state['seg_end'] = state['t'] + k
        # groups of G frames; the last group of a run is decoded frame by frame, so the pipeline drains
        # at frame granularity (each of its frames is entropy-decoded as soon as it is encoded, instead of
        # after the whole group), and those calls reconstruct streamed: the drain is the tail's slowest slice
        # (the frame-22 scene change, ~35 ms of one wave's CAVLC chain) plus the reconstructions queued
        # behind it, and a streamed reconstruction finishes with its parse instead of ~3 ms after it
        while k > 0:
            n = min(G, k)
            if k <= G and a.tail_frames:
                set_tail(True)
                for _ in range(n):
                    run_group(1, tail=True)
                set_tail(False)
            else:
                run_group(n)
            k -= n
        if gather is not None:
            gather.flush()

    # warmup, then the self-check: decoder output == encoder reconstruction, every stream
    run_steps(a.warmup)
    sync()
    captured = None
    if capture:
        captured = {s: [] for s in range(S)}
        pics = cap_pic.cpu().numpy() if cap_pic is not None else None
        for t, (nb, sz) in enumerate(cap_nal):
            szh = sz.cpu().tolist()
            host = nb.cpu().numpy()
            for s in range(S):
                e = {'nal': hashlib.sha256(host[s * slot:s * slot + szh[s]].tobytes()).hexdigest()}
                if pics is not None:
                    e['pic'] = hashlib.sha256(pics[t, s].tobytes()).hexdigest()
                captured[s].append(e)
        del pics
        cap_nal.clear()
        cap_pic = None
    selfcheck_ok = True
    if decode:
        for dec in decs:
            rc, got = dec.status()
            selfcheck_ok = selfcheck_ok and rc == 0 and all(got)
        nb = decs[0].cw * decs[0].ch * 3 // 2
        for s in range(S):
            x, y = np.empty(nb, np.uint8), np.empty(nb, np.uint8)
            h264mi._hip_memcpy_d2h(x.ctypes.data, encs[s // Sg].recon_ptr(s % Sg), nb)
            h264mi._hip_memcpy_d2h(y.ctypes.data, decs[s // Sd].picture_ptr(s % Sd), nb)
            selfcheck_ok = selfcheck_ok and bool(np.array_equal(x, y))
    for enc in encs:
        enc.set_timing(True)
    for dec in decs:
        dec.set_timing(True)
    elapsed = timed(run_steps, a.steps, 0, dist, sync)
    ems, en = [sum(x) for x in zip(*[enc.kernel_time() for enc in encs])]
    kern = {'enc_mb_kernel': {'avg_ms': ems / max(en, 1), 'launches': en}}
    # after the timed region: every stream's last timed frame (NAL units in the last staging slot, the decoders'
    # current pictures) for the oracle check, and the decoder == reconstruction self-check again
    sync()
    lb, lj = state['last']
    szl = stage_sz[lb][lj].cpu().tolist()
    hostl = stage[lb][lj].cpu().numpy()
    last_frame = [{'nal': hashlib.sha256(hostl[s * slot:s * slot + szl[s]].tobytes()).hexdigest(),
                   'pic': hashlib.sha256(decs[s // Sd].picture_i420(s % Sd)).hexdigest() if decode else None} for s in range(S)]
    del hostl
    if decode:
        for dec in decs:
            rc, got = dec.status()
            selfcheck_ok = selfcheck_ok and rc == 0 and all(got)
        nb = decs[0].cw * decs[0].ch * 3 // 2
        for s in range(S):
            x, y = np.empty(nb, np.uint8), np.empty(nb, np.uint8)
            h264mi._hip_memcpy_d2h(x.ctypes.data, encs[s // Sg].recon_ptr(s % Sg), nb)
            h264mi._hip_memcpy_d2h(y.ctypes.data, decs[s // Sd].picture_ptr(s % Sd), nb)
            selfcheck_ok = selfcheck_ok and bool(np.array_equal(x, y))
    gather_check = None
    if gather is not None:  # the last group's units as rank 0 received them == what every rank staged
        sync()
        b = (state['g'] - 1) % NB
        n = len(gather.received[-1]) // (world * S)
        szs = stage_sz[b][:n].cpu().reshape(-1).tolist()
        host = stage[b][:n].reshape(-1).cpu()
        mine = [hashlib.sha256(bytes(host[u * slot:u * slot + szs[u]].numpy())).hexdigest() for u in range(n * S)]
        allh = [None] * world
        dist.all_gather_object(allh, mine)
        if rank == 0:
            rx = gather.rx[:world * n * S * slot].cpu()
            sz = gather.received[-1]
            got = [hashlib.sha256(bytes(rx[u * slot:u * slot + sz[u]].numpy())).hexdigest() for u in range(world * n * S)]
            gather_check = got == [h for r in range(world) for h in allh[r]]
        gather_check = {'ok': gather_check, 'units': world * n * S, 'host_waits': gather.host_waits}
    if decode:
        rms, rn = [sum(x) for x in zip(*[dec.kernel_time(0) for dec in decs])]
        pms, pn = [sum(x) for x in zip(*[dec.kernel_time(1) for dec in decs])]
        kern['dec_recon_kernel'] = {'avg_ms': rms / max(rn, 1), 'launches': rn}
        kern['dec_parse_kernel'] = {'avg_ms': pms / max(pn, 1), 'launches': pn, 'slices_per_launch': Sd * G,
                                    # the parse launches' summed duration over the timed region's wall time (they run
                                    # beside the encoder and the reconstruction on reserved CUs, so this is not additive)
                                    'busy_share_of_timed_wall': pms / (elapsed * 1e3) if elapsed > 0 else None,
                                    'sq': a.parse_mix}
        if os.environ.get('H264MI_PARSE_PROF'):  # diagnostic: the slices' own duration (wave start to end)
            dec = decs[0]
            nsl = Sd * G * dec.ring_groups()
            prof = np.zeros(nsl * 16, np.uint64)
            h264mi.lib().h264mi_dec_parse_profile(dec._d, prof.ctypes.data)
            kern['dec_parse_kernel']['slice_ms_mean_all_calls'] = float(prof.reshape(-1, 16)[:, 0].sum()) / 1e5 / max(1, (a.warmup + a.steps) * S)
    sizes = [x for enc in encs for x in enc.nal_sizes()]
    for enc in encs:
        enc.close()
    for dec in decs:
        dec.close()
    if a.parse_cus > 0:
        for st in ess + dss:
            h264mi.destroy_stream(st)
    # roofline of the dominant kernel (enc_mb_kernel): algorithmic bytes per launch = S streams x
    # (read source F + read reference F + write reconstruction F) for a P frame, 2F for an IDR
    # 
    alg = Sg * (2 if i_only else 3) * F  # per launch: one encoder group's streams
    work = {0: 'IPPP encode+decode (intra period 0)', 2: 'I-only encode (force_key_frame before every frame)',
            3: 'IPPP encode+decode (intra period 0), one stream', 5: 'IPPP encode+decode (intra period 0)'}[a.config]
    cfg = {'workload': f'{W}x{H} {work}, {S} streams per GPU, {a.bitrate} bps, wrapper encoder params'
                       + (f' (encoded by {EG} encoders of {Sg} streams on their own HIP streams)' if EG > 1 else '')
                       + (f', decode batches of {G} frames' if decode else '') + ('; NAL gather to rank 0 at N>1' if a.config in (0, 5) else ''),
           'baseline_config': {0: f'metric (configs[2] x {S} streams)', 2: 'configs[1]', 3: 'configs[2]', 5: 'configs[4]'}[a.config],
           'width': W, 'height': H, 'streams_per_gpu': S, 'bitrate': a.bitrate, 'group': G, 'frame_skip': False,
           'p_frame_qp': 'OpenH264 exact GOM' if a.gom_exact else 'MB-row plan (DESIGN.md §3.6)',
           'parse_cus': a.parse_cus, 'recon_cus': a.recon_cus, 'parse_streams': a.parse_streams,
           'streamed_recon': streamed_mode, 'tail_streamed': tail_streamed, 'recon_gate': bool(a.recon_gate), 'enc_groups': EG, 'dec_groups': DG,
           'parallelism': f'streams x{world} (weak)'}
    if gather_check is not None:
        selfcheck_ok = selfcheck_ok and gather_check['ok'] is not False
    return {'elapsed': elapsed, 'frames_per_rank': S * a.steps, 'config': cfg, 'captured': captured, 'last_frame': last_frame,
            'roofline': roofline('enc_mb_kernel', alg, ems, en, a), 'kernels': kern,
            'nal_gather': gather_check,
            'selfcheck_ok': selfcheck_ok,
            'selfcheck': ('decoder output == encoder reconstruction for every stream, after the warmup and after the timed '
                          'region: ' + ('pass' if selfcheck_ok else 'FAIL'))
            if decode else 'n/a (encode only)',
            'last_nal_bytes': sizes}


def bench_decode_only(a, torch, np, h264mi, SyntheticStream, dev, sync):
    """config 4: 8 concurrent decoders of one 1080p stream (app.js fans one encoded stream out to
    numStreams decoders). The stream (stream 0, a.clip frames, IPPP) is encoded untimed; the timed
    steps decode frame t in all S decoders (wrapping to the next IDR-started pass of the clip)."""
    W, H, S, G = a.width, a.height, a.streams, a.group
    F = W * H * 3 // 2
    g = SyntheticStream(0, W, H)
    enc = h264mi.BatchEncoder(W, H, a.bitrate, 1)
    enc.set_frame_skip(False)  # a.clip coded frames
    slot = 1 << 21
    n = a.clip
    units = torch.empty((n, slot), dtype=torch.uint8, device=dev)
    usz = torch.zeros((n,), dtype=torch.int32, device=dev)
    for t in range(n):
        if t == 0:
            enc.force_idr(0)
        enc.encode(torch.from_numpy(np.ascontiguousarray(g.frame(t))).to(dev))
        enc.copy_nals(units[t], slot, usz[t:t + 1])
    sync()
    nbytes = usz.cpu().tolist()
    ds = h264mi.masked_stream(0, a.parse_cus, True) if a.parse_cus > 0 else torch.cuda.Stream(device=dev)
    dec = h264mi.BatchDecoder(W, H, S, stream=ds, max_frames=G)
    if a.parse_streams != 3:
        dec.set_parse_streams(a.parse_streams)
    if a.parse_cus > 0:
        dec.set_parse_cus(0, a.parse_cus)
    dec.set_streamed(a.streamed)
    state = {'t': 0}

    def run_steps(k):
        with torch.cuda.stream(ds):
            while k > 0:
                m = min(G, k, n - state['t'] % n)  # a call never wraps past the clip end (the next call starts at the IDR)
                t0 = state['t'] % n
                ptrs = [units[t0 + j].data_ptr() for j in range(m) for _ in range(S)]
                szp = [usz[t0 + j:t0 + j + 1].data_ptr() for j in range(m) for _ in range(S)]
                dec.decode_frames(ptrs, size_ptrs=szp)
                state['t'] += m
                k -= m

    run_steps(a.warmup)
    sync()
    rc, got = dec.status()
    ok = rc == 0 and all(got)
    pics = [dec.picture_i420(s) for s in range(S)]
    ok = ok and all(p == pics[0] for p in pics)
    dec.set_timing(True)
    elapsed = timed(run_steps, a.steps, 0, None, sync)
    rms, rn = dec.kernel_time(0)
    pms, pn = dec.kernel_time(1)
    dec.close()
    enc.close()
    if a.parse_cus > 0:
        h264mi.destroy_stream(ds)
    alg = S * 2 * F  # decode P: read reference F + write picture F, per stream
    cfg = {'workload': f'{W}x{H} decode only: {S} concurrent decoders of one IPPP stream ({a.bitrate} bps, '
                       f'{sum(nbytes) // n} B/frame mean), decode batches of {G} frames',
           'baseline_config': 'configs[3]', 'width': W, 'height': H, 'decoders': S, 'bitrate': a.bitrate, 'group': G,
           'parallelism': 'decoders x1'}
    return {'elapsed': elapsed, 'frames_per_rank': S * a.steps, 'config': cfg,
            'roofline': roofline('dec_recon_kernel', alg, rms, rn, a,
                                 note='by GPU time dec_parse_kernel dominates: one wave per slice walks the serial CAVLC '
                                      'chain (latency-bound, no meaningful HBM roofline)'),
            'kernels': {'dec_recon_kernel': {'avg_ms': rms / max(rn, 1), 'launches': rn},
                        'dec_parse_kernel': {'avg_ms': pms / max(pn, 1), 'launches': pn, 'slices_per_launch': S * G}},
            'selfcheck_ok': ok, 'selfcheck': 'all decoders produce the same picture: ' + ('pass' if ok else 'FAIL')}


if __name__ == '__main__':
    main()
