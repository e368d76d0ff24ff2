"""Multi-GPU sharding of independent streams.

Streams are independent encoders/decoders, so they shard across ranks with no data-path
collective: rank r owns global streams [r*S, (r+1)*S). The only exchange is the per-frame gather of
encoded NAL units to rank 0 (config 5): an all-gather of the int32 byte counts, then exact-size
point-to-point sends of each stream's staged access unit (a gatherv over RCCL/xGMI; gloo on CPU).
"""


def stream_ids(rank, streams_per_rank):
    return list(range(rank * streams_per_rank, (rank + 1) * streams_per_rank))


def gather_nals_to_rank0(dist, torch, nal_buf, sizes, S, slot, rank, world, rx=None):
    """nal_buf: uint8 tensor holding S staged access units (stream s at [s*slot, s*slot+sizes[s]));
    sizes: int32 tensor of S byte counts (same device as nal_buf). On rank 0, rx (uint8 tensor of
    world*S*slot bytes) receives every rank's units at [(r*S+s)*slot, ...). Returns the world*S byte
    counts (host list) on every rank."""
    parts = [torch.empty_like(sizes) for _ in range(world)]
    dist.all_gather(parts, sizes)
    sz = torch.cat(parts).cpu().tolist()
    ops = []
    if rank == 0:
        if rx is not None:
            rx[:S * slot].copy_(nal_buf[:S * slot])
        for r in range(1, world):
            for s in range(S):
                n = sz[r * S + s]
                if n > 0:
                    ops.append(dist.P2POp(dist.irecv, rx[(r * S + s) * slot:(r * S + s) * slot + n], r))
    else:
        for s in range(S):
            n = sz[rank * S + s]
            if n > 0:
                ops.append(dist.P2POp(dist.isend, nal_buf[s * slot:s * slot + n], 0))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return sz
