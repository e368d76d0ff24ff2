"""GPU: the device-resident NAL ring -- the reference's SharedArrayBuffer frame
pool (app.js:52-53, :292-310) with encoder_worker.js:163-202 publish semantics (drop when too large,
drop when the buffer is still referenced, else copy + size + ref_count = numStreams) and
decoder_worker.js:138-164 release semantics (one Atomics.sub per consumer), decided on the device.

The semantics are checked against a host model of the JS (`JsPool`, below) driven by the same
sequence of publishes and releases; the decoded pictures against the oracle decoder."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class JsPool:
    """encoder_worker.js:163-202 / decoder_worker.js:138-164 restated on the host, with this
    library's one documented difference: ticket t uses slot t % slots (the JS keeps
    currentBufferIndex on a drop)."""

    def __init__(self, slots, slot_bytes):
        self.slots, self.max = slots, slot_bytes
        self.size, self.ref = [0] * slots, [0] * slots
        self.data = [b''] * slots
        self.published = self.busy = self.too_big = 0
        self.tickets = {}

    def publish(self, t, nal, consumers):
        b = t % self.slots
        if len(nal) <= 0:                   # encoder_worker.js:167-169
            self.tickets[t] = 0
        elif len(nal) > self.max:           # :170-173
            self.too_big += 1
            self.tickets[t] = 0
        elif self.ref[b] > 0:               # :177-182
            self.busy += 1
            self.tickets[t] = 0
        else:                               # :185-190
            self.data[b], self.size[b], self.ref[b] = nal, len(nal), consumers
            self.published += 1
            self.tickets[t] = len(nal)

    def release(self, t):                   # decoder_worker.js:145, :164
        if self.tickets[t] > 0:
            self.ref[t % self.slots] -= 1


def _dev_i32(ptr):
    import h264mi
    v = np.zeros(1, np.int32)
    h264mi._hip_memcpy_d2h(v.ctypes.data, ptr, 4)
    return int(v[0])


def _dev_bytes(ptr, n):
    import h264mi
    v = np.zeros(n, np.uint8)
    if n:
        h264mi._hip_memcpy_d2h(v.ctypes.data, ptr, n)
    return v.tobytes()


def _frames(w, h, n, seed):
    import torch
    from h264mi.synth import SyntheticStream
    g = SyntheticStream(seed, w, h)
    return [torch.from_numpy(np.ascontiguousarray(g.frame(t))).cuda() for t in range(n)]


def test_ring_drop_semantics_match_js_pool(gpu_lib):
    """Busy-slot drops, oversized drops, release accounting and the host's lag guard, against JsPool."""
    import torch
    import h264mi
    w, h = 176, 144
    enc = h264mi.BatchEncoder(w, h, 300000, 1)
    enc.set_frame_skip(False)  # the ring semantics under test need a unit per frame
    frames = _frames(w, h, 8, 3)
    ring = h264mi.NalRing(slots=2, slot_bytes=1 << 16)
    model = JsPool(2, 1 << 16)
    nals = []

    def publish(t_expected, consumers=2):
        t = ring.publish(enc, 0, consumers)
        assert t == t_expected
        torch.cuda.synchronize()
        nal = enc.nal_bytes(0, enc.nal_sizes()[0])
        nals.append(nal)
        model.publish(t, nal, consumers)
        return t

    def release(t):
        ring.release(t)
        model.release(t)

    for t in range(3):                       # t0, t1 land; t2 finds slot 0 referenced -> dropped
        enc.encode(frames[t])
        publish(t)
    release(0), release(0)                   # both consumers of t0 done
    enc.encode(frames[3]); publish(3)        # slot 1 still referenced by t1 -> dropped
    enc.encode(frames[4]); publish(4)        # slot 0 free -> lands
    torch.cuda.synchronize()
    st = ring.stats()
    assert (st['published'], st['dropped_busy'], st['dropped_size']) == (model.published, model.busy, model.too_big) == (3, 2, 0)
    assert st['ref_counts'] == model.ref == [2, 2]
    for t in (1, 2, 3, 4):                   # t0's size word now belongs to t4
        assert _dev_i32(ring.size_ptr(t)) == model.tickets[t]
    assert _dev_bytes(ring.nal_ptr(4), model.tickets[4]) == nals[4] == model.data[0]
    assert _dev_bytes(ring.nal_ptr(1), model.tickets[1]) == nals[1] == model.data[1]
    enc.encode(frames[5])
    with pytest.raises(RuntimeError):        # t5 would reuse t1's size word before t1 is released
        ring.publish(enc, 0, 2)
    for t in (1, 2, 3):
        release(t), release(t)
    with pytest.raises(RuntimeError):        # a third release of t1: more releases than consumers
        ring.release(1)
    publish(5)
    torch.cuda.synchronize()
    assert ring.stats()['ref_counts'] == model.ref == [2, 2]
    ring.close()

    small = h264mi.NalRing(slots=4, slot_bytes=64)   # every coded frame is larger than a slot
    enc.encode(frames[6])
    t = small.publish(enc, 0, 1)
    torch.cuda.synchronize()
    st = small.stats()
    assert (st['published'], st['dropped_busy'], st['dropped_size']) == (0, 0, 1)
    assert _dev_i32(small.size_ptr(t)) == 0 and st['ref_counts'] == [0] * 4
    small.release(t)
    torch.cuda.synchronize()
    assert small.stats()['ref_counts'] == [0] * 4
    small.close()
    enc.close()


def test_ring_fanout_zero_copy_decoders(gpu_lib, oracle):
    """app.js fan-out: one encoder publishes each frame once with ref_count = numStreams; every
    decoder (own HIP stream, own instance) decodes straight from the slot and releases it. With the
    pool large enough nothing drops, every slot ends unreferenced, and each decoder's pictures are
    the oracle decoder's."""
    import torch
    import h264mi
    w, h, n, D = 352, 288, 6, 3
    frames = _frames(w, h, n, 11)
    es = torch.cuda.Stream()
    dss = [torch.cuda.Stream() for _ in range(D)]
    enc = h264mi.BatchEncoder(w, h, 1000000, 1, stream=es)
    enc.set_frame_skip(False)  # every frame coded and published
    decs = [h264mi.BatchDecoder(w, h, 1, stream=dss[k]) for k in range(D)]
    ring = h264mi.NalRing(slots=4, slot_bytes=1 << 20)
    od = oracle.decoder()
    oe = oracle.encoder(w, h, 1000000)
    oe.set_frame_skip(False)
    for t in range(n):
        with torch.cuda.stream(es):
            es.wait_stream(torch.cuda.current_stream())
            enc.encode(frames[t])
            tk = ring.publish(enc, 0, D)
            ev = torch.cuda.Event()
            ev.record(es)
        for k in range(D):
            with torch.cuda.stream(dss[k]):
                dss[k].wait_event(ev)
                decs[k].decode_frames([ring.nal_ptr(tk)], size_ptrs=[ring.size_ptr(tk)])
                ring.release(tk, stream=dss[k])
        torch.cuda.synchronize()
        nal = oe.encode(frames[t].cpu().numpy())
        _, pic, _, _ = od.decode(nal)
        for k in range(D):
            rc, got = decs[k].status()
            assert rc == 0 and got == [1]
            assert decs[k].picture_i420(0) == pic.tobytes(), f'frame {t} decoder {k}'
    st = ring.stats()
    assert (st['published'], st['dropped_busy'], st['dropped_size']) == (n, 0, 0)
    assert st['ref_counts'] == [0] * 4
    for d in decs:
        d.close()
    ring.close()
    enc.close()


def test_ring_wraps_without_host_sync(gpu_lib):
    """Publishes and releases enqueued back to back with NO host synchronisation, on a 2-slot ring
    (ticket t + 4 reuses ticket t's size word): each publish that reuses a size word is ordered on
    the device after every release of the ticket that last used it, so no release reads a word
    that was already overwritten. Drops are timing-dependent (the JS pool's drop-when-busy), but
    every ticket is either published or dropped exactly once and no reference count leaks."""
    import torch
    import h264mi
    w, h, n, D = 176, 144, 14, 2
    frames = _frames(w, h, n, 5)
    es = torch.cuda.Stream()
    dss = [torch.cuda.Stream() for _ in range(D)]
    enc = h264mi.BatchEncoder(w, h, 300000, 1, stream=es)
    enc.set_frame_skip(False)  # the ring semantics under test need a unit per frame
    decs = [h264mi.BatchDecoder(w, h, 1, stream=dss[k]) for k in range(D)]
    ring = h264mi.NalRing(slots=2, slot_bytes=1 << 18)
    torch.cuda.synchronize()
    for t in range(n):
        with torch.cuda.stream(es):
            enc.encode(frames[t])
            tk = ring.publish(enc, 0, D)
            assert tk == t
            ev = torch.cuda.Event()
            ev.record(es)
        for k in range(D):
            with torch.cuda.stream(dss[k]):
                dss[k].wait_event(ev)
                decs[k].decode_frames([ring.nal_ptr(tk)], size_ptrs=[ring.size_ptr(tk)])
                ring.release(tk, stream=dss[k])
    torch.cuda.synchronize()
    st = ring.stats()
    assert st['published'] + st['dropped_busy'] + st['dropped_size'] == n
    assert st['published'] >= 2 and st['dropped_size'] == 0
    assert st['ref_counts'] == [0, 0]
    for d in decs:
        d.close()
    ring.close()
    enc.close()


@pytest.mark.parametrize('code', [2, 3], ids=['after-assembly', 'rbsp-overflow-branch'])
def test_ring_failed_frame_publishes_nothing(gpu_lib, oracle, code):
    """A frame whose kernels fail publishes nothing to the ring -- no truncated or stale access unit
    reaches a consumer -- and the encoder restarts with an IDR (SPS + PPS + IDR slice): the decoder,
    which never saw the failed frame, decodes the stream on. Code 2 fails the frame after
    the slice is assembled; code 3 takes enc_pack_kernel's RBSP-overflow early exit itself (ADVICE r3:
    that exit used to leave the previous frame's size in place)."""
    import torch
    import h264mi
    w, h, n, bad = 176, 144, 5, 2
    frames = _frames(w, h, n, 7)
    enc = h264mi.BatchEncoder(w, h, 300000, 1)
    enc.set_frame_skip(False)  # the ring semantics under test need a unit per frame
    enc.set_frame_skip(False)
    dec = h264mi.BatchDecoder(w, h, 1)
    ring = h264mi.NalRing(slots=4, slot_bytes=1 << 18)
    od = oracle.decoder()
    for t in range(n):
        if t == bad:
            enc.inject_error(0, code)
        enc.encode(frames[t])
        tk = ring.publish(enc, 0, 1)
        torch.cuda.synchronize()
        size = torch.empty(1, dtype=torch.int32)
        h264mi._hip_memcpy_d2h(size.data_ptr(), ring.size_ptr(tk), 4)
        nb = int(size[0])
        if t == bad:
            assert nb == 0, 'a failed frame reached the ring'
            ring.release(tk)
            continue
        assert nb > 0
        unit = torch.empty(nb, dtype=torch.uint8)
        h264mi._hip_memcpy_d2h(unit.data_ptr(), ring.nal_ptr(tk), nb)
        u = bytes(unit.numpy())
        types = [u[i + 4] & 31 for i in range(len(u) - 4) if u[i:i + 4] == b'\x00\x00\x00\x01']
        if t in (0, bad + 1):
            assert types[:3] == [7, 8, 5], (t, types)  # the frame after the failure restarts with an IDR
        else:
            assert types == [1], (t, types)
        dec.decode_frames([ring.nal_ptr(tk)], size_ptrs=[ring.size_ptr(tk)])
        ring.release(tk)
        rc, got = dec.status()
        orc, opic, _, _ = od.decode(u)
        assert rc == 0 and got == [1] and orc == 1
        assert dec.picture_i420(0) == opic.tobytes(), f'frame {t}'
    st = ring.stats()
    assert st['published'] == n - 1 and st['ref_counts'] == [0] * 4
    dec.close()
    ring.close()
    enc.close()
