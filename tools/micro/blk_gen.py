"""Random residual blocks for tools/micro/blk_check.hip: every nC class (neighbour bytes 0..16 and 0xff),
maxNumCoeff 15 and 16, empty / +-1 / small / escape-coded / dense blocks; bits by the oracle's CAVLC
writer (h264o_cavlc_bits). usage: blk_gen.py <seed> <out.bin>
Output: int32 {nblocks, ndwords}, per block int32 {na, nb, maxnum, nbits}, the ring-format dwords (RBSP
byte p at ring byte p^3), int16 expected coefficients [nblocks][16] (scan order, base 1 for maxnum 15)."""
import ctypes, sys
import numpy as np

L = ctypes.CDLL(__file__.rsplit('/', 3)[0] + '/oracle/build/libh264_oracle.so')
L.h264o_cavlc_bits.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]


def nc_of(na, nb):
    both = (na + nb + 1) >> 1
    t = nb if na == 0xff else both
    t = na if nb == 0xff else t
    return 0 if t == 0xff else t


def block(rng, maxnum):
    c = np.zeros(16, np.int16)
    kind = rng.integers(0, 6)
    if kind == 0:
        pass
    elif kind == 1:
        c[rng.integers(0, maxnum)] = rng.choice([-1, 1])
    elif kind == 2:
        for p in rng.choice(maxnum, rng.integers(1, 4), replace=False):
            c[p] = rng.choice([-3, -2, -1, 1, 2, 3])
    elif kind == 3:
        for p in rng.choice(maxnum, rng.integers(1, 6), replace=False):
            c[p] = int(rng.choice([-1, 1])) * int(rng.integers(1, 1000))
    elif kind == 4:
        k = rng.integers(5, maxnum + 1)
        for p in rng.choice(maxnum, k, replace=False):
            c[p] = int(rng.choice([-1, 1])) * int(rng.geometric(0.3))
    else:
        k = rng.integers(1, maxnum + 1)
        for p in rng.choice(maxnum, k, replace=False):
            c[p] = int(rng.choice([-1, 1])) * int(rng.geometric(0.6))
    return c


def main(seed, path):
    rng = np.random.default_rng(seed)
    bits, meta, coefs = [], [], []
    ctx = list(range(17)) + [0xff]
    while True:
        maxnum = int(rng.choice([15, 16]))
        na, nb = int(rng.choice(ctx)), int(rng.choice(ctx))
        c = block(rng, maxnum)
        buf = np.zeros(1024, np.uint8)
        n = L.h264o_cavlc_bits(c[:maxnum].ctypes.data, maxnum, nc_of(na, nb), buf.ctypes.data, 1024)
        assert n > 0
        if len(bits) + n > 8 * 15000:
            break
        bits.extend(buf[:n].tolist())
        meta.append((na, nb, maxnum, n))
        e = np.zeros(16, np.int16)
        e[(1 if maxnum == 15 else 0):][:maxnum] = c[:maxnum]
        coefs.append(e)
    bits.extend([1] + [0] * 7)
    while len(bits) % 32:
        bits.append(0)
    by = np.packbits(np.array(bits, np.uint8))
    ring = by.reshape(-1, 4)[:, ::-1].reshape(-1)
    with open(path, 'wb') as f:
        f.write(np.array([len(meta), len(ring) // 4], np.int32).tobytes())
        f.write(np.array(meta, np.int32).tobytes())
        f.write(ring.tobytes())
        f.write(np.array(coefs, np.int16).tobytes())
    print(f'seed {seed}: {len(meta)} blocks, {len(bits)} bits')


if __name__ == '__main__':
    main(int(sys.argv[1]), sys.argv[2])
