"""Hand-built Baseline P-slice access units for decoder tests (TEST INFRASTRUCTURE).

The encoder under test only emits vectors within +-16 integer pels, so its streams never exercise the
decoder's paths for long vectors (references far outside the picture, blocks whose reference lies
outside the LDS window). This writes P pictures whose macroblocks are P_L0_16x16 with arbitrary mvd
and no residual, or P_Skip runs, on top of the SPS/PPS/IDR access unit of a stream from the
encoder, so that the decoder output can be checked against the oracle decoder (a restatement of the
normative decoding process, 8.4). Syntax: 7.3.3 slice_header, 7.3.4 slice_data, 7.3.5 mb_pred with
the encoder's parameter sets (OpenH264's, DESIGN.md §3.1: log2_max_frame_num 15, POC type 2 -- no POC
field in the slice header --, deblocking_filter_control_present, one reference)."""
import numpy as np


class BitWriter:
    def __init__(self):
        self.bits = []

    def u(self, v, n):
        self.bits += [(v >> (n - 1 - i)) & 1 for i in range(n)]

    def ue(self, v):
        k = v + 1
        n = k.bit_length()
        self.u(0, n - 1)
        self.u(k, n)

    def se(self, v):
        self.ue(2 * v - 1 if v > 0 else -2 * v)

    def rbsp(self):
        b = self.bits + [1]
        b += [0] * (-len(b) % 8)
        return bytes(int(''.join(map(str, b[i:i + 8])), 2) for i in range(0, len(b), 8))


def nal(ref_idc, typ, rbsp):
    out = bytearray(b'\x00\x00\x00\x01')
    out.append((ref_idc << 5) | typ)
    z = 0
    for c in rbsp:
        if z >= 2 and c <= 3:
            out.append(3)
            z = 0
        out.append(c)
        z = z + 1 if c == 0 else 0
    return bytes(out)


def p_frame(mbw, mbh, frame_num, poc_lsb, rng, max_mvd=96, skip_prob=0.2, qp_delta=0, dbk_idc=0, first_mb=0):
    """One P access unit: each MB P_Skip (runs) with probability skip_prob, else P_L0_16x16 with a
    random mvd in [-max_mvd, max_mvd] quarter samples and coded_block_pattern 0. first_mb > 0 makes
    it the second slice of a two-slice picture (MBs first_mb..end). poc_lsb is unused: the encoder's SPS
    has POC type 2 (the order follows frame_num)."""
    w = BitWriter()
    w.ue(first_mb)          # first_mb_in_slice
    w.ue(5)                 # slice_type P (all slices of the picture P)
    w.ue(0)                 # pic_parameter_set_id
    w.u(frame_num & 0x7fff, 15)
    w.u(0, 1)               # num_ref_idx_active_override_flag
    w.u(0, 1)               # ref_pic_list_modification_flag_l0
    w.u(0, 1)               # adaptive_ref_pic_marking_mode_flag
    w.se(qp_delta)          # slice_qp_delta
    w.ue(dbk_idc)           # disable_deblocking_filter_idc
    if dbk_idc != 1:
        w.se(0); w.se(0)    # slice_alpha_c0_offset_div2, slice_beta_offset_div2
    run = 0
    for _ in range(mbw * mbh - first_mb):
        if rng.random() < skip_prob:
            run += 1
            continue
        w.ue(run)           # mb_skip_run
        run = 0
        w.ue(0)             # mb_type P_L0_16x16
        w.se(int(rng.integers(-max_mvd, max_mvd + 1)))
        w.se(int(rng.integers(-max_mvd, max_mvd + 1)))
        w.ue(0)             # coded_block_pattern (inter, codeNum 0 -> 0)
    if run:
        w.ue(run)
    return nal(2, 1, w.rbsp())


# ---------------------------------------------------------------------------------------------
# Full Baseline syntax generator: random but conforming access units that exercise every branch of
# the decoders' macroblock layer (7.3.5): P_L0_16x16 / 16x8 / 8x16, P_8x8 with every sub_mb_type,
# P_Skip runs, I_NxN, I_16x16 (all 24 types), I_PCM, mb_qp_delta over its whole range (including the
# wrap across 0 / 51), coded residuals of every block class with large levels (level_prefix 14 / 15
# escapes) at low QP, num_ref_idx_active_override, a ref_pic_list_modification that resolves to the
# single reference, non-zero chroma_qp_index_offset and deblocking filter offsets. Residual blocks are
# written by the oracle's CAVLC writer (h264o_cavlc_bits); everything else here, from 7.3 syntax.
# Intra prediction modes are drawn only among the modes whose neighbours are available (8.3.1.2,
# 8.3.3, 8.3.4), and levels are bounded by QP so that no dequantised value leaves the 16-bit range
# a conforming stream keeps (8.5.12).

class FastBits:
    def __init__(self):
        self.b = bytearray()

    def u(self, v, n):
        for i in range(n - 1, -1, -1):
            self.b.append((v >> i) & 1)

    def ue(self, v):
        k = v + 1
        n = k.bit_length()
        self.u(0, n - 1)
        self.u(k, n)

    def se(self, v):
        self.ue(2 * v - 1 if v > 0 else -2 * v)

    def align_zero(self):
        while len(self.b) % 8:
            self.b.append(0)

    def raw(self, bits):
        self.b += bits

    def rbsp(self):
        bits = np.frombuffer(bytes(self.b) + b'\x01', np.uint8)
        pad = (-len(bits)) % 8
        bits = np.concatenate([bits, np.zeros(pad, np.uint8)])
        return np.packbits(bits).tobytes()


# T / L / D: the top / left / top-left neighbour samples (8.3.1.2.x, 8.3.3.x, 8.3.4.x); a slice
# boundary can leave the top-left macroblock unavailable while the top and left ones are available
_I4_NEEDS = {0: 'T', 1: 'L', 2: '', 3: 'T', 4: 'TLD', 5: 'TLD', 6: 'TLD', 7: 'T', 8: 'L'}
_I16_NEEDS = {0: 'T', 1: 'L', 2: '', 3: 'TLD'}
_CHROMA_NEEDS = {0: '', 1: 'L', 2: 'T', 3: 'TLD'}
_BLK_ORDER = [0, 1, 4, 5, 2, 3, 6, 7, 8, 9, 12, 13, 10, 11, 14, 15]  # decoding order -> raster 4x4


def _ok(needs, top, left, tl=True):
    return ('T' not in needs or top) and ('L' not in needs or left) and ('D' not in needs or tl)


class SyntaxGen:
    def __init__(self, oracle_so, mbw, mbh, seed, crop_right=0, crop_bottom=0, cqp=0, init_qp=26, poc_type=0, dpoaz=0):
        import ctypes
        self.ct = ctypes
        L = ctypes.CDLL(oracle_so)
        L.h264o_cavlc_bits.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        L.h264o_cbp_code.argtypes = [ctypes.c_int, ctypes.c_int]
        self.L = L
        self.mbw, self.mbh = mbw, mbh
        self.rng = np.random.default_rng(seed)
        self.crop = (crop_right, crop_bottom)
        self.cqp, self.init_qp = cqp, init_qp
        self.poc_type, self.dpoaz = poc_type, dpoaz  # POC type 0 / 1 (delta_pic_order_always_zero_flag) / 2
        self.tc_choice = None  # TotalCoeff distribution of generated blocks (None: the default mix)
        self.frame_num = 0
        self.poc = 0
        self.idr_id = 0
        self._bits = np.zeros(512, np.uint8)

    # ---- parameter sets (7.3.2.1, 7.3.2.2)
    def sps(self):
        w = FastBits()
        w.u(66, 8); w.u(0xC0, 8); w.u(40, 8); w.ue(0)
        w.ue(12)              # log2_max_frame_num_minus4 (16 bits)
        w.ue(self.poc_type)
        if self.poc_type == 0:
            w.ue(12)          # 16-bit lsb
        elif self.poc_type == 1:
            w.u(self.dpoaz, 1); w.se(-1); w.se(0); w.ue(2); w.se(2); w.se(3)
        w.ue(1); w.u(0, 1)
        w.ue(self.mbw - 1); w.ue(self.mbh - 1)
        w.u(1, 1); w.u(1, 1)
        cr, cb = self.crop
        w.u(1 if (cr or cb) else 0, 1)
        if cr or cb:
            w.ue(0); w.ue(cr); w.ue(0); w.ue(cb)
        w.u(0, 1)
        return nal(3, 7, w.rbsp())

    def pps(self):
        w = FastBits()
        w.ue(0); w.ue(0); w.u(0, 1); w.u(0, 1); w.ue(0)
        w.ue(0); w.ue(0)      # num_ref_idx_l0/l1_default_active_minus1
        w.u(0, 1); w.u(0, 2)
        w.se(self.init_qp - 26); w.se(0); w.se(self.cqp)
        w.u(1, 1); w.u(0, 1); w.u(0, 1)
        return nal(3, 8, w.rbsp())

    # ---- helpers
    def _av(self, mx, my, dx, dy):
        """macroblock (mx + dx, my + dy) available to (mx, my): in the picture and in the same slice"""
        x, y = mx + dx, my + dy
        return 0 <= x < self.mbw and y >= 0 and y * self.mbw + x >= self._first

    def _nc(self, nn, avail_mb, mx, my, cur, ras):
        bx, by = ras & 3, ras >> 2
        na = cur[ras - 1] if bx > 0 else (nn[my][mx - 1][ras + 3] if self._av(mx, my, -1, 0) else None)
        nb = cur[ras - 4] if by > 0 else (nn[my - 1][mx][ras + 12] if self._av(mx, my, 0, -1) else None)
        return self._avg(na, nb)

    def _ncc(self, nn, mx, my, cur, pl, blk):
        base = 16 + 4 * pl
        bx, by = blk & 1, blk >> 1
        na = cur[base + blk - 1] if bx > 0 else (nn[my][mx - 1][base + blk + 1] if self._av(mx, my, -1, 0) else None)
        nb = cur[base + blk - 2] if by > 0 else (nn[my - 1][mx][base + blk + 2] if self._av(mx, my, 0, -1) else None)
        return self._avg(na, nb)

    @staticmethod
    def _avg(na, nb):
        if na is not None and nb is not None:
            return (na + nb + 1) >> 1
        return na if na is not None else (nb if nb is not None else 0)

    def _levels(self, maxnum, qp, big_ok=True):
        """coefficients in scan order (maxnum of them) for one block, bounded by QP"""
        rng = self.rng
        lim = max(1, 2048 // (25 << (qp // 6)))
        tc = int(rng.choice(self.tc_choice or [0, 1, 1, 2, 3, 4, 6, 8, maxnum // 2, maxnum]))
        tc = min(tc, maxnum)
        c = np.zeros(maxnum, np.int16)
        if tc:
            pos = rng.choice(maxnum, tc, replace=False)
            mag = rng.choice(getattr(self, 'mag_choice', None) or [1, 1, 1, 2, 3, 5], tc)
            if big_ok and lim > 8 and rng.random() < 0.3:
                mag[int(rng.integers(tc))] = int(rng.integers(8, lim + 1))   # escape codes (level_prefix 14/15)
            mag = np.minimum(mag, lim)
            c[pos] = mag * rng.choice([-1, 1], tc)
        return c

    def _block(self, w, coef, nc):
        n = self.L.h264o_cavlc_bits(coef.ctypes.data, len(coef), nc, self._bits.ctypes.data, self._bits.size)
        assert n > 0
        w.raw(self._bits[:n].tobytes())
        return int(np.count_nonzero(coef))

    def _residual(self, w, nn, mx, my, cur, mtype, cbp, qp, i16):
        qpc = _CHROMA_QP[min(51, max(0, qp + self.cqp))]
        if i16:
            self._block(w, self._levels(16, qp - 6 if qp >= 6 else 0, big_ok=False), self._nc(nn, None, mx, my, cur, 0))
        for k in range(16):
            ras = _BLK_ORDER[k]
            if not (cbp >> (k >> 2)) & 1:
                continue
            coef = self._levels(15 if i16 else 16, qp)
            cur[ras] = self._block(w, coef, self._nc(nn, None, mx, my, cur, ras))
        cbpc = cbp >> 4
        if cbpc:
            for pl in range(2):
                self._block(w, self._levels(4, qpc + 6 if qpc + 6 <= 51 else 51, big_ok=False), -1)
            if cbpc == 2:
                for pl in range(2):
                    for blk in range(4):
                        cur[16 + 4 * pl + blk] = self._block(w, self._levels(15, qpc), self._ncc(nn, mx, my, cur, pl, blk))

    def _qp_delta(self, w, qp):
        rng = self.rng
        r = rng.random()
        if r < 0.5:
            dq = 0
        elif r < 0.8:
            dq = int(rng.integers(-4, 5))
        else:
            dq = int(rng.integers(-26, 26))   # wraps across 0 / 51
        w.se(dq)
        return (qp + dq + 52) % 52

    def _intra(self, w, nn, i4m, kinds, mx, my, qp, in_p, kind):
        """I_NxN / I_16x16 / I_PCM macroblock (mb_type already chosen); returns (qp, nnz row, i4 modes)"""
        rng = self.rng
        cur = [0] * 24
        top_mb, left_mb, tl_mb = self._av(mx, my, 0, -1), self._av(mx, my, -1, 0), self._av(mx, my, -1, -1)
        off = 5 if in_p else 0
        modes = None
        self._last_cbp = 0
        if kind == 'pcm':
            w.ue(off + 25)
            w.align_zero()
            for _ in range(384):
                w.u(int(rng.integers(1, 256)), 8)
            return qp, [16] * 24, None
        cm = int(rng.choice([m for m, nd in _CHROMA_NEEDS.items() if _ok(nd, top_mb, left_mb, tl_mb)]))
        if kind == 'i4':
            w.ue(off + 0)
            modes = [2] * 16
            for k in range(16):
                ras = _BLK_ORDER[k]
                bx, by = ras & 3, ras >> 2
                top = by > 0 or top_mb
                left = bx > 0 or left_mb
                tl = (bx > 0 and by > 0) or (bx == 0 and by > 0 and left_mb) or (bx > 0 and by == 0 and top_mb) or \
                     (bx == 0 and by == 0 and tl_mb)
                # predIntra4x4PredMode (8.3.1.1)
                if (bx == 0 and not left_mb) or (by == 0 and not top_mb):
                    pm = 2
                else:
                    a = modes[ras - 1] if bx > 0 else (i4m[my][mx - 1][ras + 3] if kinds[my][mx - 1] == 'i4' else 2)
                    b = modes[ras - 4] if by > 0 else (i4m[my - 1][mx][ras + 12] if kinds[my - 1][mx] == 'i4' else 2)
                    pm = min(a, b)
                m = int(rng.choice([m for m, nd in _I4_NEEDS.items() if _ok(nd, top, left, tl)]))
                if rng.random() < 0.3 and _ok(_I4_NEEDS[pm], top, left, tl):
                    m = pm
                modes[ras] = m
                if m == pm:
                    w.u(1, 1)
                else:
                    w.u(0, 1)
                    w.u(m if m < pm else m - 1, 3)
            w.ue(cm)
            cbp = int(rng.integers(0, 48))
            self._last_cbp = cbp
            w.ue(self.L.h264o_cbp_code(cbp, 1))
            if cbp:
                qp = self._qp_delta(w, qp)
                self._residual(w, nn, mx, my, cur, 'i4', cbp, qp, False)
            return qp, cur, modes
        # I_16x16
        pm16 = int(rng.choice([m for m, nd in _I16_NEEDS.items() if _ok(nd, top_mb, left_mb, tl_mb)]))
        cbpc = int(rng.integers(0, 3))
        cbpl = 15 if rng.random() < 0.5 else 0
        if getattr(self, 'i16_cbp', None) is not None:  # fixed I_16x16 coded_block_pattern (tools/parse_mix.py)
            cbpc, cbpl = self.i16_cbp >> 4, self.i16_cbp & 15
        self._last_cbp = cbpl | (cbpc << 4)
        w.ue(off + 1 + pm16 + 4 * cbpc + (12 if cbpl else 0))
        w.ue(cm)
        qp = self._qp_delta(w, qp)
        self._residual(w, nn, mx, my, cur, 'i16', cbpl | (cbpc << 4), qp, True)
        return qp, cur, None

    def _header(self, w, first_mb, idr, islice, qp_delta, dbk, override, reorder, ref_idc):
        """slice_header() (7.3.3) -> SliceQPY"""
        rng = self.rng
        w.ue(first_mb)
        w.ue(7 if islice else 5)
        w.ue(0)
        w.u(self.frame_num & 0xffff, 16)
        if idr:
            w.ue(self.idr_id)
        if self.poc_type == 0:
            w.u(self.poc & 0xffff, 16)
        elif self.poc_type == 1 and not self.dpoaz:
            w.se(self._dpoc)                  # delta_pic_order_cnt[0] (the same in every slice)
        if not islice:
            w.u(1 if override else 0, 1)
            if override:
                w.ue(0)                       # num_ref_idx_l0_active_minus1
            w.u(1 if reorder else 0, 1)       # ref_pic_list_modification_flag_l0
            if reorder:
                w.ue(0); w.ue(0)              # subtract 1: picNum of the previous (only) reference
                w.ue(3)
        if idr:
            w.u(0, 1); w.u(0, 1)
        elif ref_idc:                         # dec_ref_pic_marking() only in reference pictures
            w.u(0, 1)
        qp_delta = min(51 - self.init_qp, max(-self.init_qp, qp_delta))  # SliceQPY in 0..51
        w.se(qp_delta)
        idc, fa, fb = dbk
        w.ue(idc)
        if idc != 1:
            w.se(fa); w.se(fb)
        return self.init_qp + qp_delta

    def _slice(self, idr, mix, qp_delta=0, dbk=(0, 0, 0), override=False, reorder=False, max_mvd=24, ref_idc=2, cbp_fixed=None,
               slices=None):
        """one picture; slices = [{'first': first_mb_in_slice, 'qp_delta', 'dbk', 'intra'}, ...] (first 0 first,
        increasing; a key left out takes the picture-wide argument) -> the RBSP of each slice in
        raster order (the single-slice default returns one)"""
        rng = self.rng
        mbw, mbh = self.mbw, self.mbh
        slices = slices or [{'first': 0}]
        assert slices[0]['first'] == 0 and all(a['first'] < b['first'] for a, b in zip(slices, slices[1:]))
        self._dpoc = int(rng.integers(-3, 4))
        nn = [[None] * mbw for _ in range(mbh)]
        i4m = [[None] * mbw for _ in range(mbh)]
        kinds = [[None] * mbw for _ in range(mbh)]
        names = list(mix)
        probs = np.array([mix[k] for k in names], float)
        probs /= probs.sum()
        self.log = []   # per MB: (mb type code as h264o_dec_mbinfo reports it, QPY, coded_block_pattern)
        out = []
        w, run, si, islice, qp = None, 0, -1, idr, 0
        for my in range(mbh):
            for mx in range(mbw):
                addr = my * mbw + mx
                if si + 1 < len(slices) and addr == slices[si + 1]['first']:
                    if w is not None:
                        if run:
                            w.ue(run)
                        out.append(w.rbsp())
                    si += 1
                    sd = slices[si]
                    self._first = addr
                    islice = idr or sd.get('intra', False)
                    w, run = FastBits(), 0
                    qp = self._header(w, addr, idr, islice, sd.get('qp_delta', qp_delta), sd.get('dbk', dbk), override, reorder, ref_idc)
                kind = names[int(rng.choice(len(names), p=probs))]
                if islice and kind in ('skip', 'p16', 'p16x8', 'p8x16', 'p8x8'):
                    kind = 'i4'
                if kind == 'skip':
                    run += 1
                    nn[my][mx], kinds[my][mx] = [0] * 24, 'skip'
                    self.log.append((3, qp, 0))
                    continue
                if not islice:
                    w.ue(run)
                    run = 0
                kinds[my][mx] = kind
                if kind in ('i4', 'i16', 'pcm'):
                    qp, nn[my][mx], i4m[my][mx] = self._intra(w, nn, i4m, kinds, mx, my, qp, not islice, kind)
                    self.log.append(({'i4': 0, 'i16': 1, 'pcm': 7}[kind], qp, self._last_cbp))
                    continue
                cur = [0] * 24
                mt = {'p16': 0, 'p16x8': 1, 'p8x16': 2, 'p8x8': 3}[kind]
                w.ue(mt)
                if mt < 3:
                    for _ in range(1 if mt == 0 else 2):
                        w.se(int(rng.integers(-max_mvd, max_mvd + 1))); w.se(int(rng.integers(-max_mvd, max_mvd + 1)))
                else:
                    subs = [int(rng.integers(0, 4)) for _ in range(4)]
                    for s_ in subs:
                        w.ue(s_)
                    for s_ in subs:
                        for _ in range({0: 1, 1: 2, 2: 2, 3: 4}[s_]):
                            w.se(int(rng.integers(-max_mvd, max_mvd + 1))); w.se(int(rng.integers(-max_mvd, max_mvd + 1)))
                cbp = int(rng.integers(0, 48)) if rng.random() < 0.85 else 0
                if cbp_fixed is not None:
                    cbp = cbp_fixed
                w.ue(self.L.h264o_cbp_code(cbp, 0))
                if cbp:
                    qp = self._qp_delta(w, qp)
                    self._residual(w, nn, mx, my, cur, kind, cbp, qp, False)
                nn[my][mx] = cur
                self.log.append(({'p16': 2, 'p16x8': 4, 'p8x16': 5, 'p8x8': 6}[kind], qp, cbp))
        if run:
            w.ue(run)
        out.append(w.rbsp())
        return out

    def idr(self, mix=None, order=None, **kw):
        """SPS + PPS + IDR picture (I_NxN / I_16x16 / I_PCM); slices=[...] (see _slice) splits it, order
        permutes the slices' NAL units (arbitrary slice order)"""
        self.frame_num, self.poc = 0, 0
        bodies = self._slice(True, mix or {'i4': 5, 'i16': 4, 'pcm': 1}, **kw)
        self.idr_id = (self.idr_id + 1) & 0xffff
        self.frame_num, self.poc = 1, 2
        return self.sps() + self.pps() + b''.join(nal(3, 5, bodies[i]) for i in (order or range(len(bodies))))

    def p(self, mix=None, ref_idc=2, order=None, **kw):
        """one P picture with every macroblock type (ref_idc 0: a non-reference picture); slices=[...]
        (see _slice) splits it, a slice with 'intra' True is an I slice; order permutes the slices"""
        mix = mix or {'skip': 3, 'p16': 3, 'p16x8': 2, 'p8x16': 2, 'p8x8': 3, 'i4': 1, 'i16': 1, 'pcm': 0.3}
        bodies = self._slice(False, mix, ref_idc=ref_idc, **kw)
        if ref_idc:
            self.frame_num = (self.frame_num + 1) & 0xffff
        self.poc += 2
        return b''.join(nal(ref_idc, 1, bodies[i]) for i in (order or range(len(bodies))))


_CHROMA_QP = [i for i in range(30)] + [29, 30, 31, 32, 32, 33, 34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39]
