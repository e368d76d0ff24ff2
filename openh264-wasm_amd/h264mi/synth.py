"""Deterministic synthetic I420 video (SURVEY.md §8(d) 'Synthetic input').

Per stream s: a textured plane from a counter-based hash (lowbias32 of index ^ seed,
seed = 0x9E3779B9 ^ s), 4x4 box-filtered (wrap-around) to mid-frequency content; frame t is a
window at offset (3t mod 64, 2t mod 64) luma pixels (half for chroma), so motion estimation finds
real motion. Chroma planes come from separately seeded textures. A counter-based hash replaces the
survey's sequential xorshift32 so the generator vectorises; the content statistics are the same.
"""
import numpy as np

_M1 = np.uint32(0x7FEB352D)
_M2 = np.uint32(0x846CA68B)


def _mix32(x):
    x = x.astype(np.uint32)
    x ^= x >> np.uint32(16)
    x *= _M1
    x ^= x >> np.uint32(15)
    x *= _M2
    x ^= x >> np.uint32(16)
    return x


def texture(seed, tw, th):
    idx = np.arange(tw * th, dtype=np.uint64)
    raw = (_mix32(((idx * np.uint64(0x9E3779B1)) ^ np.uint64(seed)) & np.uint64(0xFFFFFFFF)) >> np.uint32(24))
    raw = raw.astype(np.int32).reshape(th, tw)
    acc = np.zeros_like(raw)
    for dy in range(4):
        for dx in range(4):
            acc += np.roll(np.roll(raw, -dy, axis=0), -dx, axis=1)
    return (acc >> 4).astype(np.uint8)


class SyntheticStream:
    """Frames of one synthetic stream; textures are generated once."""

    def __init__(self, stream, w, h):
        assert w % 2 == 0 and h % 2 == 0
        self.w, self.h = w, h
        seed = (0x9E3779B9 ^ stream) & 0xFFFFFFFF
        self.ty = texture(seed, w + 64, h + 64)
        self.tu = texture(seed ^ 0x55555555, w // 2 + 32, h // 2 + 32)
        self.tv = texture(seed ^ 0x2AAAAAAA, w // 2 + 32, h // 2 + 32)

    def frame(self, t):
        w, h = self.w, self.h
        ox, oy = (3 * t) % 64, (2 * t) % 64
        y = self.ty[oy:oy + h, ox:ox + w]
        u = self.tu[oy // 2:oy // 2 + h // 2, ox // 2:ox // 2 + w // 2]
        v = self.tv[oy // 2:oy // 2 + h // 2, ox // 2:ox // 2 + w // 2]
        return np.concatenate([y.ravel(), u.ravel(), v.ravel()])


def synthetic_frame(stream, t, w, h):
    return SyntheticStream(stream, w, h).frame(t)
