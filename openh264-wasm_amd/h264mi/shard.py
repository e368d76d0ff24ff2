"""Multi-GPU sharding of independent streams.

Streams are independent encoders/decoders, so they shard across ranks with no data-path
collective: rank r owns global streams [r*S, (r+1)*S). The only exchange is the gather of encoded
NAL units to rank 0 (BASELINE.json configs[4]): an all-gather of the int32 byte counts, then
exact-size point-to-point sends of each staged access unit (a gatherv over RCCL/xGMI; gloo on CPU).
"""


def stream_ids(rank, streams_per_rank):
    return list(range(rank * streams_per_rank, (rank + 1) * streams_per_rank))


def gather_nals_to_rank0(dist, torch, nal_buf, sizes, S, slot, rank, world, rx=None):
    """One frame, synchronous: nal_buf holds S staged access units (stream s at [s*slot, s*slot +
    sizes[s])); sizes is an int32 tensor of S byte counts on nal_buf's device. On rank 0, rx (world *
    S * slot bytes) receives every rank's units at [(r*S+s)*slot, ...). Returns the world*S byte counts
    (host list) on every rank. Used by tests; the pipelined path is NalGather."""
    parts = [torch.empty_like(sizes) for _ in range(world)]
    dist.all_gather(parts, sizes)
    sz = torch.cat(parts).cpu().tolist()
    _post(dist, nal_buf.reshape(-1), sz, S, 1, slot, rank, world, rx, wait=True)
    return sz


def _post(dist, buf, sz, S, n, slot, rank, world, rx, wait):
    """point-to-point sends (rank > 0) / receives (rank 0) of n frames x S units; buf holds frame j's
    stream s at (j*S + s)*slot; sz[r*n*S + j*S + s] = its bytes; rx on rank 0 gets (r, j, s) at
    ((r*n + j)*S + s)*slot"""
    ops = []
    if rank == 0:
        if rx is not None:
            rx[:n * S * slot].copy_(buf[:n * S * slot])
        for r in range(1, world):
            for u in range(n * S):
                b = sz[r * n * S + u]
                if b > 0:
                    o = (r * n * S + u) * slot
                    ops.append(dist.P2POp(dist.irecv, rx[o:o + b], r))
    else:
        for u in range(n * S):
            b = sz[rank * n * S + u]
            if b > 0:
                ops.append(dist.P2POp(dist.isend, buf[u * slot:u * slot + b], 0))
    reqs = dist.batch_isend_irecv(ops) if ops else []
    if wait:
        for q in reqs:
            q.wait()
    return reqs


class NalGather:
    """Pipelined NAL gather for bench.py: one size all-gather per GROUP of n frames (not per frame),
    and the exact-size sends of group g posted while group g+1 is being encoded, so the host never
    waits on the group the GPU is working on. Call submit() on the decoder's stream after a group's
    units are staged, flush() at the end; done_event(b) is recorded once group g's sends (staging
    buffer b) are complete: the encoder waits on it before reusing the buffer."""

    def __init__(self, dist, torch, S, slot, G, rank, world, device):
        self.dist, self.torch, self.S, self.slot, self.G = dist, torch, S, slot, G
        self.rank, self.world = rank, world
        self.rx = torch.empty(world * G * S * slot, dtype=torch.uint8, device=device) if rank == 0 else None
        self.cuda = device is not None and torch.device(device).type == 'cuda'
        self.pending = None  # (buf, gathered sizes, work, n, buffer id)
        self.events = {}
        self.received = []   # per group: world*n*S byte counts (host), for tests / accounting

    def done_event(self, b):
        return self.events.get(b)

    def submit(self, buf, sizes, n, b=None):
        """buf: (G, S*slot) uint8 staging tensor, sizes: (G, S) int32 byte counts; frames 0..n-1 valid"""
        t = self.torch
        flat = sizes[:n].reshape(-1).contiguous()
        parts = [t.empty_like(flat) for _ in range(self.world)]
        work = self.dist.all_gather(parts, flat, async_op=True)
        prev, self.pending = self.pending, (buf, parts, work, n, b)
        if prev is not None:
            self._finish(prev)

    def flush(self):
        if self.pending is not None:
            p, self.pending = self.pending, None
            self._finish(p)

    def _finish(self, p):
        buf, parts, work, n, b = p
        work.wait()
        sz = self.torch.cat(parts).cpu().tolist()  # host sync on an EARLIER group's sizes only
        reqs = _post(self.dist, buf.reshape(-1), sz, self.S, n, self.slot, self.rank, self.world, self.rx, wait=False)
        for q in reqs:
            q.wait()  # on CUDA: orders the current stream after the transfers (no host block)
        if self.cuda and b is not None:
            ev = self.events.get(b) or self.torch.cuda.Event()
            ev.record()
            self.events[b] = ev
        self.received.append(sz)
