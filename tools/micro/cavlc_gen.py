"""Synthetic CAVLC residual-block streams for tools/micro/cavlc_bench.hip (bits written by the CPU
oracle's h264o_cavlc_bits). usage: cavlc_gen.py <scenario> <out.bin>
Output: int32 header {nblocks, maxnum, nc, ndwords}, then the ring-format dwords (RBSP byte p at
ring byte p^3), then int16 expected coefficients [nblocks][16] (scan order, base 1 for maxnum 15)."""
import ctypes, sys
import numpy as np

L = ctypes.CDLL(__file__.rsplit('/', 3)[0] + '/oracle/build/libh264_oracle.so')
L.h264o_cavlc_bits.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]


def blocks(scn, rng, n):
    out = []
    for _ in range(n):
        c = np.zeros(16, np.int16)
        if scn == 'ac1':      # one +-1 (TotalCoeff 1, one trailing one)
            c[rng.integers(0, 15)] = rng.choice([-1, 1])
        elif scn == 'ac2':    # two coefficients, one may exceed 1
            for p in rng.choice(15, 2, replace=False):
                c[p] = rng.choice([-2, -1, 1, 1, 2])
        elif scn == 'empty':
            pass
        elif scn == 'luma':   # denser 4x4 blocks
            k = rng.integers(1, 9)
            for p in rng.choice(16, k, replace=False):
                c[p] = int(rng.choice([-1, 1])) * int(rng.geometric(0.5))
        out.append(c)
    return out


def main(scn, path):
    rng = np.random.default_rng(7)
    maxnum = 16 if scn == 'luma' else 15
    bits = []
    coefs = []
    for c in blocks(scn, rng, 20000):
        buf = np.zeros(512, np.uint8)
        n = L.h264o_cavlc_bits(c[:maxnum].ctypes.data, maxnum, 0, buf.ctypes.data, 512)
        assert n > 0
        if len(bits) + n > 8 * 16000:
            break
        bits.extend(buf[:n].tolist())
        e = np.zeros(16, np.int16)
        e[(1 if maxnum == 15 else 0):][:maxnum] = c[:maxnum]
        coefs.append(e)
    bits.extend([1] + [0] * 7)
    while len(bits) % 32:
        bits.append(0)
    by = np.packbits(np.array(bits, np.uint8))
    ring = by.reshape(-1, 4)[:, ::-1].reshape(-1)  # byte p at p ^ 3
    hdr = np.array([len(coefs), maxnum, 0, len(ring) // 4], np.int32)
    with open(path, 'wb') as f:
        f.write(hdr.tobytes()); f.write(ring.tobytes()); f.write(np.array(coefs, np.int16).tobytes())
    print(f'{scn}: {len(coefs)} blocks, {len(bits)} bits ({len(bits) / len(coefs):.1f} per block)')


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
