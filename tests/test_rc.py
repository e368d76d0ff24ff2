"""CPU: OpenH264's frame-level rate control (RC_BITRATE_MODE at the wrapper's parameters) as the oracle restates it
from the reference's h264.wasm, against a second, independent restatement in Python that reads
every constant and table from tests/golden/openh264_tables.json (cut from the wasm bytes by tools/wasm_tables.py):

* RcConvertQStep2Qp with musl's logf (func 483): the oracle's C, this file's numpy float64 / float32 version, and
  the product's device thresholds (libh264mi h264mi_rc_qstep_to_qp, a host function -- no GPU needed) agree on
  every QStep up to 400000;
* the frame-level state machine -- the skip decision with its run cap (func 589 / 1258), post-skip bookkeeping
  (func 1254), the VGOP allocation and picture QP (func 1226), the R-Q model updates (funcs 1218 / 676) and the
  VBV skip check -- driven by the oracle encoder's per-frame slice sizes, average QPs and frame complexities on
  real content, at 1080p 1 / 8 Mbps with skipping on and off, must give the oracle's skip decisions, QPs, QP
  windows, target bits, remaining bits, buffer fullness and run counts frame by frame.
Parity with OpenH264 itself: the functions are restated from its compiled code (no OpenH264 output exists here)."""
import ctypes
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
OH = json.load(open(os.path.join(HERE, 'golden', 'openh264_tables.json')))
T, C = OH['tables'], OH['code_constants']


def cc(name):
    return C[name]['value']


def py_logf(x):
    """musl logf (h264.wasm func 483) from the fixture's table and polynomial, float32 in and out"""
    x = np.float32(x)
    ix = int(np.array([x], np.float32).view(np.uint32)[0])
    if ix == 0x3f800000:
        return np.float32(0.0)
    assert 0x00800000 <= ix < 0x7f800000  # normal positive inputs only (QStep / 100 >= 0.64)
    tab, poly = T['logf_table']['values'], T['logf_poly']['values']
    tmp = (ix - 0x3f330000) & 0xffffffff
    i = (tmp >> 19) & 15
    k = (tmp if tmp < 0x80000000 else tmp - (1 << 32)) >> 23
    iz = (ix - (tmp & 0xff800000)) & 0xffffffff
    z = np.float64(np.array([iz], np.uint32).view(np.float32)[0])
    f = np.float64
    r = z * f(tab[i][0]) + f(-1.0)
    r2 = r * r
    y = (f(poly[1]) * r2 + (f(poly[2]) * r + f(poly[3]))) * r2 + ((f(k) * f(poly[0]) + f(tab[i][1])) + r)
    return np.float32(y)


def py_qstep2qp(q):
    """RcConvertQStep2Qp (func 1226): 0 below the pinned minimum, else trunc(6 logf(q / 100f) / ln2 + 4 + 0.5)"""
    if q < cc('qstep_min'):
        return 0
    t = py_logf(np.float32(np.float32(q) / np.float32(100.0)))
    return int((np.float64(np.float32(t * np.float32(6.0))) / cc('qstep_conv_ln2') + cc('qstep_conv_offset'))
               + cc('qstep_conv_round'))


def test_logf_restatement(oracle):
    """the oracle's logf == this file's restatement bit for bit, and both within an ULP of the true log"""
    rng = np.random.default_rng(3)
    xs = np.concatenate([np.float32(rng.uniform(0.5, 5e6, 3000)), np.float32([1.0, 0.64, 2.0, 100.0])])
    for x in xs:
        a = np.float32(oracle.L.h264o_logf(float(x)))
        assert a == py_logf(x), x
        assert abs(float(a) - np.log(float(x))) <= 2 * np.spacing(np.float32(abs(a)) + np.float32(1e-30)), x


def test_qstep2qp_three_ways(oracle, libpath):
    """oracle (musl-logf form) == Python restatement == the product's thresholds, every QStep 0..400000"""
    lib = ctypes.CDLL(libpath)
    f_o, f_g = oracle.L.h264o_rc_qstep2qp, lib.h264mi_rc_qstep_to_qp
    f_g.argtypes = [ctypes.c_int]
    qs = np.arange(0, 400000)
    o = np.array([f_o(int(q)) for q in qs])
    g = np.array([f_g(int(q)) for q in qs])
    assert np.array_equal(np.minimum(o, 52), g)
    for q in list(range(0, 2000, 7)) + [2016, 22807, 24163, 24164, 399999]:
        assert py_qstep2qp(q) == o[q], q
    # the QStep table round trips: QP k's QStep converts back to k
    assert [int(o[v]) for v in T['rc_qstep']['values'][1:]] == list(range(1, 52))


class PyRc:
    """RC_BITRATE_MODE at the wrapper's parameters, one layer, from the fixture alone"""

    def __init__(self, w, h, br, skip_en=True):
        vary = cc('rc_vary_percentage')
        w16, h16 = (w + 15) // 16 * 16, (h + 15) // 16 * 16
        self.mbw, self.nmb = w16 // 16, (w16 // 16) * (h16 // 16)
        narrow = self.mbw < 31
        self.skip_qp = cc('skip_qp_value_narrow') if narrow else cc('skip_qp_value_wide')
        self.w16, self.h16, self.br, self.vary, self.skip_en = w16, h16, br, vary, skip_en
        self.qmin, self.qmax = cc('camera_min_qp'), cc('camera_max_qp')
        self.weight = T['rc_tl_weight']['values'][0][0]
        self.gop_num = cc('vgop_gops')
        self.idr_num = 0
        self.skip_flag, self.continual, self.fullness = False, 0, 0
        for k in ('remaining', 'vgop_bits', 'remaining_weights', 'gop_index', 'coded_in_vgop', 'target', 'bpf',
                  'pframes', 'intra_mb_count', 'intra_cmplx', 'intra_mean', 'lin', 'mean', 'last_qscale', 'init_qp',
                  'qp', 'min_qp', 'max_qp', 'bits_level', 'avg_qp', 'buf_size', 'min_bits', 'max_bits'):
            setattr(self, k, 0)

    @staticmethod
    def cdiv(a, b):  # C integer division (truncates toward zero)
        q = abs(a) // abs(b)
        return q if (a >= 0) == (b > 0) else -q

    def div_round(self, x, y):  # WELS_DIV_ROUND64
        return x if y == 0 else self.cdiv(x + self.cdiv(y, 2), y)

    def update_bitrate_fps(self):
        fps = np.float32(cc('default_max_frame_rate'))
        self.bpf = int((fps * np.float32(0.5) + np.float32(self.br)) / fps)
        lo = 100 - ((cc('min_bits_base') - self.vary) >> 1)
        div = cc('bits_tl_divisor')
        self.max_bits = (self.bpf * cc('max_bits_ratio') * self.weight + div // 2) // div
        self.min_bits = (self.bpf * lo * self.weight + div // 2) // div
        self.buf_size = (cc('skip_buffer_ratio') * self.br + 50) // 100

    def init_vgop(self):
        t = self.remaining + (self.gop_index - self.gop_num) * self.cdiv(self.vgop_bits, self.gop_num)
        self.remaining = min(t, 0) + (self.bpf << cc('vgop_bits_shift'))
        self.vgop_bits = self.remaining
        self.gop_index = self.coded_in_vgop = 0
        self.remaining_weights = self.gop_num * cc('weight_multiply')

    def judge_skip(self):
        if not self.skip_flag:
            if not self.skip_en:
                return False
            pred = (self.div_round(self.fullness, self.bpf) + 1) >> 1
            self.skip_flag = pred >= self.continual and self.fullness > self.buf_size
            if not self.skip_flag:
                return False
        self.skip_flag = False
        self.continual += 1
        return True

    def post_skip(self):
        self.fullness = max(0, self.fullness - self.bpf)
        self.remaining += self.bpf

    def ratio(self, fc, mean):
        r = fc * 100 if mean == 0 else self.div_round(fc * 100, mean)
        return min(max(r, cc('cmplx_ratio_lo')), cc('cmplx_ratio_hi'))

    def qstep(self, cmplx, ratio):
        v = cmplx * ratio if self.target == 0 else self.div_round(cmplx * ratio, self.target * 100)
        return ((v + (1 << 31)) % (1 << 32)) - (1 << 31)  # wrapped to int32

    def picture_init(self, idr, fc):
        self.continual = 0
        if idr and self.idr_num == 0:
            self.intra_cmplx = self.intra_mb_count = self.intra_mean = 0
            self.pframes = self.lin = self.mean = 0
            self.fullness = self.gop_index = self.vgop_bits = self.remaining = 0
            self.bpf = 0
            self.update_bitrate_fps()
            self.init_vgop()
        if self.gop_index == self.gop_num or idr:
            self.init_vgop()
        self.gop_index += 1
        self.bits_level = 0
        if idr:
            self.target = cc('default_idr_bitrate_ratio') * self.bpf // 100 if self.idr_num else self.bpf << cc('first_idr_target_shift')
        else:
            rw, wt = self.remaining_weights, self.weight
            tb = self.cdiv(self.cdiv(rw, 2) + self.remaining * wt, rw) if rw >= wt else self.remaining
            if tb <= 0 and not self.skip_en:
                self.bits_level = 2
            self.target = min(max(tb, self.min_bits), self.max_bits)
        self.remaining_weights -= self.weight
        if idr:
            fps = np.float32(cc('default_max_frame_rate'))
            bpp = self.br / float(np.float32(np.float32(fps * np.float32(self.w16)) * np.float32(self.h16)))
            area = self.w16 * self.h16
            cls = 0 if area < cc('area_90p') else 1 if area < cc('area_180p') else 2 if area < cc('area_360p') else 3
            i = 1 - cc('default_fix_rc_overshoot')
            while i < 4 and not T['rc_bpp']['values'][cls][i] >= bpp:
                i += 1
            hi_, lo_ = (min(max(v, self.qmin), self.qmax) for v in T['rc_qp_range']['values'][i])
            if self.idr_num == 0:
                q = T['rc_init_qp']['values'][cls][i]
            else:
                if self.nmb != self.intra_mb_count:
                    self.intra_cmplx = self.cdiv(self.intra_cmplx * self.nmb, self.intra_mb_count)
                q = py_qstep2qp(self.qstep(self.intra_cmplx, self.ratio(fc, self.intra_mean)))
            q = min(max(q, lo_), hi_)
            self.init_qp = q
            w_ = cc('idr_frame_qp_window')
            self.min_qp, self.max_qp = min(max(q - w_, lo_), hi_), min(max(q + w_, lo_), hi_)
        else:
            if self.pframes == 0:
                q = self.init_qp
            elif self.bits_level == 2:
                q = self.last_qscale + cc('bits_exceeded_qp_step')
            else:
                q = py_qstep2qp(self.qstep(self.lin, self.ratio(fc, self.mean)))
            self.min_qp = min(max(self.last_qscale - cc('frame_delta_qp_lower'), self.qmin), self.qmax)
            self.max_qp = min(max(self.last_qscale + cc('frame_delta_qp_upper'), self.qmin), self.qmax)
            q = min(max(q, self.min_qp), self.max_qp)
        self.qp = self.last_qscale = q

    def picture_update(self, idr, slice_bytes, avg, fc):
        bits = slice_bytes * 8
        self.last_qscale = self.avg_qp = avg
        qs = T['rc_qstep']['values'][avg]
        new, old = cc('cmplx_decay_new'), cc('cmplx_decay_old')
        if not idr:
            if self.pframes == 0:
                self.mean, self.lin = fc, bits * qs
            else:
                self.mean = self.cdiv(fc * new + self.mean * old + 50, 100)
                self.lin = self.cdiv(self.lin * old + qs * bits * new + 50, 100)
            self.pframes = min(self.pframes, 254) + 1
        else:
            ic = qs * bits
            if self.idr_num == 0:
                self.intra_mean, self.intra_cmplx = fc, ic
            else:
                self.intra_cmplx = self.cdiv(ic * new + self.intra_cmplx * old + 50, 100)
                self.intra_mean = self.cdiv(fc * new + self.intra_mean * old + 50, 100)
            self.intra_mb_count = self.nmb
            self.idr_num = min(self.idr_num, 254) + 1
        self.remaining -= bits
        if self.skip_en:
            self.fullness += bits - self.bpf
            pred = sum(self.min_bits for _ in range(self.coded_in_vgop + 1, 8)) if self.coded_in_vgop <= 6 else 0
            inc = (float(pred - self.remaining) * cc('vbv_percent')) / float(self.bpf << cc('vbv_vgop_shift')) + cc('vbv_percent_diff')
            if (self.fullness > self.buf_size and avg > self.skip_qp) or inc > self.vary:
                self.skip_flag = True
        self.coded_in_vgop += 1


def slice_bytes(nal):
    """bytes of the slice NAL (the access unit minus its parameter-set NALs: another layer for the RC)"""
    starts = [k for k in range(len(nal) - 4) if nal[k:k + 4] == b'\x00\x00\x00\x01']
    for a, b in zip(starts, starts[1:] + [len(nal)]):
        if nal[a + 4] & 31 in (1, 5):
            return b - a
    raise AssertionError('no slice NAL')


@pytest.mark.parametrize('br,skip,force', [(1000000, True, 0), (8000000, True, 0), (1000000, False, 0),
                                           (8000000, False, 0), (8000000, True, 7)],
                         ids=['1m_skip', '8m_skip', '1m_noskip', '8m_noskip', '8m_skip_idr7'])
def test_frame_rc_state_machine_vs_python(oracle, br, skip, force):
    """the oracle's rate control on real 1080p content, frame by frame, == the Python restatement fed with the
    oracle's per-frame slice sizes, average QPs and frame complexities"""
    from h264mi.synth import SyntheticStream
    w, h, n = 1920, 1080, 45 if skip else 24
    g = SyntheticStream(1, w, h)
    oe = oracle.encoder(w, h, br)
    oe.set_frame_skip(skip)
    py = PyRc(w, h, br, skip)
    coded_p = 0
    for t in range(n):
        idr = t == 0 or (force and t % force == 0)
        if force and t % force == 0 and t > 0:
            oe.force_idr()
        nal = oe.encode(np.ascontiguousarray(g.frame(t)))
        st = oe.rc_state()
        skipped = py.judge_skip() and not idr
        assert skipped == bool(st['skipped']) == (len(nal) == 0), (t, st)
        if skipped:
            py.post_skip()
        else:
            py.picture_init(idr, st['cmplx'])
            assert (py.qp, py.min_qp, py.max_qp, py.target) == (st['qp'], st['min_qp'], st['max_qp'], st['target']), (t, st)
            py.picture_update(idr, slice_bytes(nal), st['avg_qp'], st['cmplx'])
            coded_p += not idr
        got = {'remaining': py.remaining, 'fullness': py.fullness, 'continual': py.continual,
               'skip_flag': int(py.skip_flag), 'remaining_weights': py.remaining_weights, 'coded_in_vgop': py.coded_in_vgop}
        assert got == {k: st[k] for k in got}, (t, got, st)
    assert coded_p > 0


def test_run_cap_codes_p_frames_at_the_wrappers_operating_point(oracle):
    """1080p at the wrapper's 1 Mbps with skipping on: the IDR fills the buffer, and the cap on the run of skipped
    frames (predicted skips >= the run) forces a P frame through after 39 skips (round 5's rule skipped all)"""
    from h264mi.synth import SyntheticStream
    w, h = 1920, 1080
    g = SyntheticStream(0, w, h)
    oe = oracle.encoder(w, h, 1000000)
    sizes = [len(oe.encode(np.ascontiguousarray(g.frame(t)))) for t in range(44)]
    assert sizes[0] > 0 and all(s == 0 for s in sizes[1:40]) and sizes[40] > 0, sizes
