"""GPU: the multi-GPU NAL gather's device packing (h264mi_nal_pack / h264mi_nal_unpack, csrc/gather.inc):
a group's staged access units leave a rank as one contiguous message (unit u at the sum of the sizes before
it) and rank 0 scatters each received message back into slots. Ragged sizes with empty units and every
byte alignment of the packed offsets, against numpy."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('n,slot', [(1, 64), (37, 4096), (128, 1 << 16)])
def test_pack_unpack_round_trip(gpu_lib, n, slot):
    import torch
    rng = np.random.default_rng(n)
    sizes = rng.integers(0, slot + 1, n).astype(np.int32)
    sizes[rng.random(n) < 0.2] = 0
    if n > 1:
        sizes[1] = slot  # a full slot
    src = torch.from_numpy(rng.integers(0, 256, n * slot, dtype=np.uint8)).cuda()
    sz = torch.from_numpy(sizes).cuda()
    tot = int(sizes.sum())
    packed = torch.zeros(max(tot, 1) + 64, dtype=torch.uint8, device='cuda')
    st = torch.cuda.current_stream().cuda_stream
    assert gpu_lib.h264mi_nal_pack(packed.data_ptr(), src.data_ptr(), slot, sz.data_ptr(), n, st) == 0
    host = src.cpu().numpy()
    want = np.concatenate([host[u * slot:u * slot + int(b)] for u, b in enumerate(sizes)] + [np.zeros(0, np.uint8)])
    got = packed.cpu().numpy()
    assert np.array_equal(got[:tot], want) and not got[tot:].any()
    back = torch.zeros(n * slot, dtype=torch.uint8, device='cuda')
    assert gpu_lib.h264mi_nal_unpack(back.data_ptr(), packed.data_ptr(), slot, sz.data_ptr(), n, st) == 0
    b = back.cpu().numpy()
    for u, k in enumerate(sizes):
        assert np.array_equal(b[u * slot:u * slot + k], host[u * slot:u * slot + k]) and not b[u * slot + k:(u + 1) * slot].any()
    assert gpu_lib.h264mi_nal_pack(packed.data_ptr(), src.data_ptr(), slot, sz.data_ptr(), 0, st) == -1


class _ThreadDist:
    """An in-process stand-in for torch.distributed between threads that share one GPU: all_gather and
    batch_isend_irecv move the bytes with device copies (after a device synchronisation, so each rank's own
    stream order is respected). Everything NalGather does on CUDA around the transport -- the device packing,
    the side stream, the pinned host copies of the sizes, rank 0's unpacking by the gathered device sizes -- is
    the real code path (the branch bench.py's N > 1 metric takes)."""

    class P2POp:
        def __init__(self, op, tensor, peer):
            self.op, self.tensor, self.peer = op, tensor, peer

    def __init__(self, world):
        import threading
        self.world, self.cv, self.gathers, self.mail = world, threading.Condition(), {}, {}
        self.isend, self.irecv = 'send', 'recv'
        self.local = threading.local()

    def _rank(self):
        return self.local.rank

    def all_gather(self, parts, t, async_op=False):
        import torch
        me = self._rank()
        with self.cv:
            key = len([k for k in self.gathers if k[1] == me])
            self.gathers[(key, me)] = t
            self.cv.notify_all()

        class W:
            def wait(w):
                with self.cv:
                    assert self.cv.wait_for(lambda: all((key, r) in self.gathers for r in range(self.world)), timeout=60)
                torch.cuda.synchronize()
                for r in range(self.world):
                    parts[r].copy_(self.gathers[(key, r)])
        return W()

    def batch_isend_irecv(self, ops):
        import torch
        me = self._rank()
        reqs = []
        for o in ops:
            if o.op == 'send':
                torch.cuda.synchronize()  # the packed bytes are complete on the sender's stream
                with self.cv:
                    self.mail.setdefault((me, o.peer), []).append(o.tensor)
                    self.cv.notify_all()
                reqs.append(type('W', (), {'wait': lambda w: None})())
            else:
                with self.cv:
                    assert self.cv.wait_for(lambda: self.mail.get((o.peer, me)), timeout=60)
                    src = self.mail[(o.peer, me)].pop(0)
                o.tensor.copy_(src)
                reqs.append(type('W', (), {'wait': lambda w: None})())
        return reqs


def test_nal_gather_cuda_path_two_ranks(gpu_lib, oracle):
    """NalGather's CUDA branch end to end in one process: two threads as ranks 0 and 1 on one GPU, each staging
    real access units (352x288, skipped frames included) on its own stream, groups of 3 frames; rank 0's rx
    holds every unit of both ranks byte for byte and each group crossed as one packed message"""
    import threading
    import torch
    from h264mi.shard import NalGather, stream_ids
    from h264mi.synth import SyntheticStream
    world, S, G, slot, nframes, w, h = 2, 2, 3, 1 << 17, 7, 352, 288
    units = {}
    for sid in range(world * S):
        e = oracle.encoder(w, h, 200000 + 50000 * sid)
        g = SyntheticStream(sid, w, h)
        units[sid] = [e.encode(np.ascontiguousarray(g.frame(t))) for t in range(nframes)]
    fd = _ThreadDist(world)
    result, errors = {}, []

    def run(rank):
        try:
            fd.local.rank = rank
            torch.cuda.set_device(0)
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                gat = NalGather(fd, torch, S, slot, G, rank, world, 'cuda')
                stage = [torch.zeros((G, S * slot), dtype=torch.uint8, device='cuda') for _ in range(3)]
                stage_sz = [torch.zeros((G, S), dtype=torch.int32, device='cuda') for _ in range(3)]
                got, t, gi = [], 0, 0
                while t < nframes:
                    n, b = min(G, nframes - t), gi % 3
                    for j in range(n):
                        for i, sid in enumerate(stream_ids(rank, S)):
                            u = units[sid][t + j]
                            if u:
                                stage[b][j, i * slot:i * slot + len(u)].copy_(torch.frombuffer(bytearray(u), dtype=torch.uint8))
                            stage_sz[b][j, i] = len(u)
                    gat.submit(stage[b], stage_sz[b], n, b)
                    if rank == 0 and len(gat.received) > len(got):
                        torch.cuda.synchronize()
                        got.append((gat.rx.cpu().numpy().copy(), gat.received[-1]))
                    t, gi = t + n, gi + 1
                gat.flush()
                torch.cuda.synchronize()
                if rank == 0:
                    got.append((gat.rx.cpu().numpy().copy(), gat.received[-1]))
                    result['got'], result['messages'] = got, gat.messages
                else:
                    result['messages1'] = gat.messages
        except Exception as ex:  # surfaced below
            errors.append(repr(ex))

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for x in th:
        x.start()
    for x in th:
        x.join(120)
    assert not errors, errors
    groups = result['got']
    assert len(groups) == 3 and result['messages'] == 3 and result['messages1'] == 3
    t0 = 0
    for rx, sz in groups:
        n = len(sz) // (world * S)
        for r in range(world):
            for j in range(n):
                for i in range(S):
                    u = (r * n + j) * S + i
                    want = units[r * S + i][t0 + j]
                    assert sz[u] == len(want) and bytes(rx[u * slot:u * slot + sz[u]]) == want, (t0 + j, r, i)
        t0 += n
    assert t0 == nframes
