"""Hand-built Baseline P-slice access units for decoder tests (TEST INFRASTRUCTURE).

The encoder under test only emits vectors within +-16 integer pels, so its streams never exercise the
decoder's paths for long vectors (references far outside the picture, blocks whose reference lies
outside the LDS window). This writes P pictures whose macroblocks are P_L0_16x16 with arbitrary mvd
and no residual, or P_Skip runs, on top of the SPS/PPS/IDR access unit of a stream from the
encoder, so that the decoder output can be checked against the oracle decoder (a restatement of the
normative decoding process, 8.4). Syntax: 7.3.3 slice_header, 7.3.4 slice_data, 7.3.5 mb_pred with
the encoder's parameter sets (log2_max_frame_num 16, POC type 0 with 16-bit lsb,
deblocking_filter_control_present, one reference)."""
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
    it the second slice of a two-slice picture (MBs first_mb..end)."""
    w = BitWriter()
    w.ue(first_mb)          # first_mb_in_slice
    w.ue(5)                 # slice_type P (all slices of the picture P)
    w.ue(0)                 # pic_parameter_set_id
    w.u(frame_num & 0xffff, 16)
    w.u(poc_lsb & 0xffff, 16)
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
