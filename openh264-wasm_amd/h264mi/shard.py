"""Multi-GPU sharding of independent streams.

Streams are independent encoders/decoders, so they shard across ranks with no data-path
collective: rank r owns global streams [r*S, (r+1)*S). The only exchange is the gather of encoded
NAL units to rank 0 (BASELINE.json configs[4]): an all-gather of the int32 byte counts, then one
exact-size point-to-point message per rank and group (a gatherv over RCCL/xGMI; gloo on CPU): each rank
packs its group's staged units into one contiguous buffer on the device (h264mi_nal_pack: unit u at the
sum of the sizes before it), rank 0 unpacks every received buffer back into slots (h264mi_nal_unpack).
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


def _pack_host(torch, buf, sizes, slot):
    """CPU tensors (gloo): the units of buf (unit u at u * slot, sizes[u] bytes) concatenated in order"""
    parts = [buf[u * slot:u * slot + b] for u, b in enumerate(sizes) if b > 0]
    return torch.cat(parts) if parts else buf[:0]


def _post_packed(dist, torch, packed, sz, m, slot, rank, world, rx, rxp):
    """one message per rank: rank r > 0 sends its m units packed (sum of its sizes bytes); rank 0 receives
    rank r's into rxp[r] (packed). Returns the requests."""
    ops = []
    if rank == 0:
        for r in range(1, world):
            tot = sum(max(b, 0) for b in sz[r * m:(r + 1) * m])
            if tot > 0:
                ops.append(dist.P2POp(dist.irecv, rxp[r][:tot], r))
    else:
        tot = sum(max(b, 0) for b in sz[rank * m:(rank + 1) * m])
        if tot > 0:
            ops.append(dist.P2POp(dist.isend, packed[:tot], 0))
    return dist.batch_isend_irecv(ops) if ops else []


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
    """Pipelined NAL gather for bench.py: one size all-gather per GROUP of n frames (not per frame), and
    the exact-size sends of group g posted when group g+1 is submitted, so the host never waits on the
    group it has just submitted. Each rank sends its group as ONE packed message (h264mi_nal_pack on the
    device at submit time, behind the staging); rank 0 unpacks each rank's message into the slot layout of
    rx (h264mi_nal_unpack) with the gathered sizes, which stay on the device.

    On CUDA, call submit() on a stream that is ordered after the group's staging only (bench.py: a
    gather stream that waits for the encoder's staging event), never after the decoder: the collective
    then depends on nothing but the encoder. The gathered byte counts are copied into pinned host memory
    on a side stream behind the collective (non-blocking) with an event; the host reads them one group
    later, when that event has long completed. done_event(b) is recorded once the sends of staging
    buffer b are complete: the encoder waits on it before reusing the buffer. flush() at the end."""

    def __init__(self, dist, torch, S, slot, G, rank, world, device):
        self.dist, self.torch, self.S, self.slot, self.G = dist, torch, S, slot, G
        self.rank, self.world = rank, world
        self.rx = torch.empty(world * G * S * slot, dtype=torch.uint8, device=device) if rank == 0 else None
        # rank 0: one packed receive buffer per sending rank (a group's units of one rank fit G * S slots)
        self.rxp = [None] + [torch.empty(G * S * slot, dtype=torch.uint8, device=device) for _ in range(1, world)] \
            if rank == 0 else None
        self.cuda = device is not None and torch.device(device).type == 'cuda'
        self.side = torch.cuda.Stream(device=device) if self.cuda else None
        self.messages = 0  # point-to-point messages this rank posted (sends or receives)
        if self.cuda:
            from . import lib
            self._L = lib()
        self.pending = None  # (buf, host sizes, ready event, n, buffer id)
        self.events = {}
        self.received = []   # per group: world*n*S byte counts (host), for tests / accounting
        self.host_waits = 0  # times _finish found the earlier group's sizes not yet on the host (diagnostic)

    def done_event(self, b):
        return self.events.get(b)

    def submit(self, buf, sizes, n, b=None):
        """buf: (G, S*slot) uint8 staging tensor, sizes: (G, S) int32 byte counts; frames 0..n-1 valid"""
        t = self.torch
        flat = sizes[:n].reshape(-1).contiguous()
        m = flat.numel()
        parts = [t.empty_like(flat) for _ in range(self.world)]
        work = self.dist.all_gather(parts, flat, async_op=True)
        packed = None
        if self.cuda and self.rank > 0:  # this rank's units, packed on the device behind the staging
            packed = t.empty(m * self.slot, dtype=t.uint8, device=buf.device)
            st = t.cuda.current_stream()
            if self._L.h264mi_nal_pack(packed.data_ptr(), buf.data_ptr(), self.slot, flat.data_ptr(), m, st.cuda_stream) != 0:
                raise RuntimeError('h264mi_nal_pack failed')
        if self.cuda:
            host = t.empty(self.world * m, dtype=flat.dtype, pin_memory=True)
            self.side.wait_stream(t.cuda.current_stream())
            with t.cuda.stream(self.side):
                work.wait()  # device-side: the side stream waits for the collective, the host does not
                for r, q in enumerate(parts):
                    host[r * m:(r + 1) * m].copy_(q, non_blocking=True)
                ready = t.cuda.Event()
                ready.record(self.side)
            for q in parts:
                q.record_stream(self.side)
            pend = (buf, host, ready, n, b, packed, parts)
        else:
            pend = (buf, (parts, work), None, n, b, None, None)
        prev, self.pending = self.pending, pend
        if prev is not None:
            self._finish(prev)

    def flush(self):
        if self.pending is not None:
            p, self.pending = self.pending, None
            self._finish(p)

    def _finish(self, p):
        buf, host, ready, n, b, packed, dparts = p
        t = self.torch
        m = n * self.S
        if ready is not None:
            if not ready.query():
                self.host_waits += 1
            ready.synchronize()  # an EARLIER group's gathered sizes (normally complete already)
            sz = host.tolist()
        else:
            parts, work = host
            work.wait()
            sz = t.cat(parts).tolist()
        flat = buf.reshape(-1)
        if packed is None and self.rank > 0:  # gloo: pack on the host
            packed = _pack_host(t, flat, sz[self.rank * m:(self.rank + 1) * m], self.slot)
        if self.rank == 0:
            self.rx[:m * self.slot].copy_(flat[:m * self.slot])
        reqs = _post_packed(self.dist, t, packed, sz, m, self.slot, self.rank, self.world, self.rx, self.rxp)
        self.messages += len(reqs)
        for q in reqs:
            q.wait()  # on CUDA: orders the current stream after the transfers (no host block)
        if self.rank == 0:  # each rank's packed units back into rx's slots, by the gathered sizes
            if self.cuda and self.world > 1:
                st = t.cuda.current_stream()
                st.wait_event(ready)  # the gathered device sizes are complete (the side stream waited on them)
                for q in dparts:
                    q.record_stream(st)
            for r in range(1, self.world):
                dst = self.rx[r * m * self.slot:(r + 1) * m * self.slot]
                if self.cuda:
                    st = t.cuda.current_stream()
                    if self._L.h264mi_nal_unpack(dst.data_ptr(), self.rxp[r].data_ptr(), self.slot, dparts[r].data_ptr(), m,
                                                 st.cuda_stream) != 0:
                        raise RuntimeError('h264mi_nal_unpack failed')
                else:
                    o = 0
                    for u, nb in enumerate(sz[r * m:(r + 1) * m]):
                        if nb > 0:
                            dst[u * self.slot:u * self.slot + nb].copy_(self.rxp[r][o:o + nb])
                            o += nb
        if self.cuda and b is not None:
            ev = self.events.get(b) or self.torch.cuda.Event()
            ev.record()
            self.events[b] = ev
        self.received.append(sz)
