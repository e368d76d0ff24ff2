"""CPU: the N>1 path -- streams sharded across ranks, per-frame gather of staged NAL units to rank 0
(all-gather of byte counts + exact-size point-to-point sends) -- on gloo with world_size 2."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from h264mi.shard import gather_nals_to_rank0, stream_ids
        S, slot = 3, 64
        ids = stream_ids(rank, S)
        buf = torch.zeros(S * slot, dtype=torch.uint8)
        sizes = torch.zeros(S, dtype=torch.int32)
        for i, sid in enumerate(ids):
            n = 5 + 7 * sid  # distinct ragged sizes; stream 0 of rank 0 is short
            buf[i * slot:i * slot + n] = torch.arange(n, dtype=torch.uint8) + sid
            sizes[i] = n
        rx = torch.zeros(world * S * slot, dtype=torch.uint8) if rank == 0 else None
        sz = gather_nals_to_rank0(dist, torch, buf, sizes, S, slot, rank, world, rx)
        if rank == 0:
            ok = sz == [5 + 7 * s for s in range(world * S)]
            for s in range(world * S):
                n = 5 + 7 * s
                ok = ok and torch.equal(rx[s * slot:s * slot + n], torch.arange(n, dtype=torch.uint8) + s)
            q.put(bool(ok))
    finally:
        dist.destroy_process_group()


def test_gather_world2():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'openh264-wasm_amd'))
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True


def test_stream_ids_partition():
    from h264mi.shard import stream_ids
    allids = [i for r in range(8) for i in stream_ids(r, 4)]
    assert allids == list(range(32))  # config 5: 32 streams over 8 GPUs
