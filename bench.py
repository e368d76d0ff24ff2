#!/usr/bin/env python
"""bench.py -- BASELINE.json metric "1080p30 frames/sec encode+decode per GPU; bit-exact vs OpenH264".

Workload (config 4's 8 concurrent 1080p streams per MI355X, doing the metric's encode+decode; at
N > 1 weak-scaled with config 5's NAL gather): every rank owns S streams (default 8). One step =
one frame of each of them: GPU encode (libh264mi batch encoder, IPPP, intra period 0, the wrapper's
parameters, 1 Mbps) and GPU decode of exactly the NAL units produced, plus (N > 1) the gather of
those NAL units to rank 0 over RCCL. Frames are encoded in groups of G and each group is decoded by
one frame-batched call (concurrent entropy decoding), overlapped with encoding of the next group.
Inputs are synthetic 1080p I420 clips resident in HBM before the timed region.
value = frames encoded+decoded by all ranks / max-over-ranks wall time of K steps.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--streams S] [--group G]
  (N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N)
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=480)
    ap.add_argument('--warmup', type=int, default=32)
    ap.add_argument('--streams', type=int, default=8, help='streams per GPU (config 4: 8 concurrent 1080p streams on one MI355X)')
    ap.add_argument('--width', type=int, default=1920)
    ap.add_argument('--height', type=int, default=1080)
    ap.add_argument('--bitrate', type=int, default=1000000)
    ap.add_argument('--clip', type=int, default=60, help='frames per stream kept resident (IPPP continues across wrap)')
    ap.add_argument('--group', type=int, default=16, help='frames per stream per decode call (frame-parallel entropy decoding)')
    ap.add_argument('--stages', type=int, default=3, help='NAL staging buffers (groups in flight between encoder and decoder)')
    ap.add_argument('--encode-only', action='store_true', help='diagnostic: skip decoding (not the metric)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--lanes', type=int, default=1, help='encoder lanes: the streams split over this many encoders, each on its own HIP stream')
    ap.add_argument('--enc-priority', type=int, default=0, help='HIP stream priority of the encoder stream (-1 = high)')
    ap.add_argument('--cpu-frames', type=int, default=16)
    ap.add_argument('--cpu-procs', type=int, default=16)
    ap.add_argument('--traffic', default=os.path.join(ROOT, 'profiles', 'round1', 'pmc_enc_mb.json'))
    return ap.parse_args()


def cpu_baseline(a):
    procs = min(a.cpu_procs, os.cpu_count() or 1)
    cmd = [sys.executable, os.path.join(ROOT, 'tools', 'cpu_baseline.py'), '--width', str(a.width), '--height', str(a.height),
           '--bitrate', str(a.bitrate), '--frames', str(a.cpu_frames), '--procs', str(procs)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        line = [l for l in r.stdout.splitlines() if l.startswith('{')][-1]
        d = json.loads(line)
        return {k: d[k] for k in ('value', 'unit', 'cores', 'kind', 'sample')}
    except Exception as e:  # reported, never silently replaced
        return {'value': None, 'unit': 'frames/s', 'cores': procs, 'kind': 'port', 'sample': f'failed: {e!r}'}


def main():
    a = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if a.gpus != world and world > 1:
        print(f'warning: --gpus {a.gpus} but WORLD_SIZE {world}', file=sys.stderr)
    # CPU baseline first, in child processes, before this process touches the GPU (rank 0, N = 1)
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(a)

    import numpy as np
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    from h264mi.shard import gather_nals_to_rank0, stream_ids
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)
    W, H, S = a.width, a.height, a.streams
    F = W * H * 3 // 2
    # ---- synthetic clips, resident in HBM: clip[t] = S frames back to back
    clip = torch.empty((a.clip, S * F), dtype=torch.uint8, device=dev)
    for i, sid in enumerate(stream_ids(rank, S)):
        g = SyntheticStream(sid, W, H)
        host = np.stack([g.frame(t) for t in range(a.clip)])
        clip[:, i * F:(i + 1) * F].copy_(torch.from_numpy(host))
    torch.cuda.synchronize()
    # Two HIP streams: the encoder runs on `es`, the decoder on `ds`. The encoder codes a group of G
    # frames per stream (P frames chain through its reconstruction, so it is sequential in time) and
    # copies each frame's NAL units into a staging slot; the decoder then takes the whole group in one
    # call, entropy-decoding all G x S slices concurrently before reconstructing them in order. NB
    # staging buffers keep NB groups in flight: encoding group g+1 overlaps the entropy decoding of
    # group g and the reconstruction of group g-1 (with two buffers the encoder would wait for the
    # reconstruction of g-1 before starting g+1, serialising encode -> parse -> reconstruct).
    L = a.lanes if a.lanes > 0 and S % a.lanes == 0 else 1
    SL = S // L
    ess = [torch.cuda.Stream(device=dev, priority=a.enc_priority) for _ in range(L)]
    ds = torch.cuda.Stream(device=dev)
    G = a.group
    encs = [h264mi.BatchEncoder(W, H, a.bitrate, SL, stream=ess[l]) for l in range(L)]
    dec = h264mi.BatchDecoder(W, H, S, stream=ds, max_frames=G)
    slot = 1 << 21  # bytes per staged access unit (a 1080p IDR at 1 Mbps is ~100 KB)
    NB = max(2, a.stages)
    stage = [torch.empty((G, S * slot), dtype=torch.uint8, device=dev) for _ in range(NB)]
    stage_sz = [torch.zeros((G, S), dtype=torch.int32, device=dev) for _ in range(NB)]
    ev_enc = [[torch.cuda.Event() for _ in range(L)] for _ in range(NB)]
    ev_dec = [torch.cuda.Event() for _ in range(NB)]
    rx = torch.empty(world * S * slot, dtype=torch.uint8, device=dev) if world > 1 and rank == 0 else None

    state = {'t': 0, 'g': 0}

    def run_group(n):
        """encode n frames of every stream, then decode them as one batch (async)"""
        b = state['g'] % NB
        t0 = state['t']
        for l in range(L):  # lane l codes streams [l*SL, (l+1)*SL) on its own HIP stream
            es = ess[l]
            with torch.cuda.stream(es):
                es.wait_event(ev_dec[b])  # the decoder has finished reading this staging buffer
                for j in range(n):
                    enc = encs[l]
                    enc.encode(clip[(t0 + j) % a.clip][l * SL * F:(l + 1) * SL * F])
                    enc.copy_nals(stage[b][j][l * SL * slot:], slot, stage_sz[b][j][l * SL:])
                ev_enc[b][l].record(es)
        state['t'] = t0 + n
        if a.encode_only:
            with torch.cuda.stream(ds):
                for l in range(L):
                    ds.wait_event(ev_enc[b][l])
                ev_dec[b].record(ds)
            state['g'] += 1
            return
        with torch.cuda.stream(ds):
            for l in range(L):
                ds.wait_event(ev_enc[b][l])
            base = stage[b].data_ptr()
            ptrs = [base + j * S * slot + s * slot for j in range(n) for s in range(S)]
            szp = [stage_sz[b].data_ptr() + 4 * (j * S + s) for j in range(n) for s in range(S)]
            dec.decode_frames(ptrs, size_ptrs=szp, ready_event=ev_enc[b])  # parse waits for every lane
            if world > 1:
                for j in range(n):
                    gather_nals_to_rank0(dist, torch, stage[b][j], stage_sz[b][j], S, slot, rank, world, rx)
            ev_dec[b].record(ds)
        state['g'] += 1

    def run_steps(k):
        while k > 0:
            n = min(G, k)
            run_group(n)
            k -= n

    run_steps(a.warmup)
    torch.cuda.synchronize()
    # ---- parity self-check before timing: decoder output == encoder reconstruction, every stream
    rc, got = dec.status()
    parity_ok = rc == 0 and all(got)
    for s in range(S):
        n = dec.cw * dec.ch * 3 // 2
        a_, b_ = np.empty(n, np.uint8), np.empty(n, np.uint8)
        h264mi._hip_memcpy_d2h(a_.ctypes.data, encs[s // SL].recon_ptr(s % SL), n)
        h264mi._hip_memcpy_d2h(b_.ctypes.data, dec.picture_ptr(s), n)
        parity_ok = parity_ok and bool(np.array_equal(a_, b_))
    # ---- timed region
    for enc in encs:
        enc.set_timing(True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(a.steps)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kt = [enc.kernel_time() for enc in encs]
    kms, nl = sum(k[0] for k in kt), sum(k[1] for k in kt)
    for enc in encs:
        enc.set_timing(False)
    sizes = [x for enc in encs for x in enc.nal_sizes()]
    if dist:
        tt = torch.tensor([elapsed, kms / max(nl, 1)], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, kavg = float(tt[0]), float(tt[1])
        ok = torch.tensor([1 if parity_ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        parity_ok = bool(ok.item())
    else:
        kavg = kms / max(nl, 1)
    frames = S * world * a.steps
    value = frames / elapsed
    # roofline of the dominant kernel (enc_mb_kernel): algorithmic bytes per launch = S streams x
    # (read source F + read reference F + write reconstruction F) for a P frame
    alg_bytes = SL * 3 * F
    achieved = alg_bytes / (kavg / 1e3) / 1e9
    traffic = None
    if os.path.exists(a.traffic):
        try:
            tj = json.load(open(a.traffic))
            if tj.get('width') == W and tj.get('height') == H and tj.get('streams') == S:
                traffic = tj.get('hbm_bytes_per_launch')
        except Exception:
            traffic = None
    if rank == 0:
        out = {
            'metric': '1080p30 frames/sec encode+decode per GPU; bit-exact vs OpenH264',
            'value': value, 'unit': 'frames/s', 'n_gpus': world, 'steps': a.steps, 'warmup': a.warmup,
            'ms_per_step': elapsed / a.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'u8', 'data': 'synthetic',
            'config': {'workload': f'{W}x{H} IPPP encode+decode (intra period 0), {S} streams per GPU, '
                                   f'{a.bitrate} bps, wrapper encoder params, decode batches of {G} frames; '
                                   f'NAL gather to rank 0 at N>1' + (f'; {L} encoder lanes of {SL} streams' if L > 1 else ''),
                       'width': W, 'height': H, 'streams_per_gpu': S, 'bitrate': a.bitrate, 'group': G, 'encoder_lanes': L,
                       'parallelism': f'streams x{world} (weak)'},
            'roofline': {'bound': 'hbm', 'kernel': 'enc_mb_kernel', 'achieved': achieved, 'peak': HBM_PEAK_GBPS,
                         'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBPS, 'traffic': traffic,
                         'alg_bytes_per_launch': alg_bytes, 'avg_launch_ms': kavg},
            'cpu_baseline': cpu,
            'parity_selfcheck': 'decoder output == encoder reconstruction for every stream: ' + ('pass' if parity_ok else 'FAIL'),
            'last_nal_bytes': sizes,
        }
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
