#!/usr/bin/env python3
"""Read OpenH264's encoder constants out of the reference's prebuilt scripts/h264.wasm AS BYTES.

The module is never instantiated, translated to something runnable or linked: this script parses the
binary's section headers, maps its passive data segments to linear-memory addresses (the start
function's `i32.const dest; i32.const 0; i32.const size; memory.init seg` sequence, read as a byte
pattern), copies tables out of the data segments, and decodes the immediate operand of a handful of
individual instructions at known file offsets. Nothing is executed.

What it pins: the wrapper links cisco/openh264 (not vendored, no tag),
so these constants are the only part of OpenH264's encoder arithmetic the reference itself holds:

  tables   quantiser MF (int16[52][8]), quantiser rounding FF (int16[58][8]; intra = row qp + 6),
           lambda (int32[52]), rate-control bits-per-pixel thresholds (f64[4][4]), initial IDR QP
           (int32[4][5]), IDR QP range (int32[5][2]), QP -> Qstep (int32[52])
  code     the immediates the RC control flow around those tables uses (camera-content QP limits,
           the default frame rate, the frame-to-frame QP window, ...), each at the file offset of
           the instruction that carries it, with the function it sits in

Where each fact was found (wasm function indices count imports; offsets are file offsets):
  func 1226  WelsRcPictureInitGom with RcCalculateIdrQp / RcCalculatePictureQp inlined
             (bpp search 767012-767140, QP range 767141-767222, initial QP 767244, frame window
             767530/767559, P-frame window 768096-768207)
  func  592  RcInitSequenceParameter (iFrameDeltaQpLower/Upper 401384-401409, skip ratio 401267)
  func  597  parameter validation (iMinQp/iMaxQp defaults 408923-409035)
  func 1023  GetDefaultParams (fMaxFrameRate 690465, bFixRCOverShoot 690589, iIdrBitrateRatio 690580)
  func  280  WelsInitSps: log2_max_frame_num / POC type, default profile, the level search (167923-169382)
  func  640  WelsWriteSpsSyntax + WelsWriteVUI (direct_8x8 level test 439081, VUI ue(16) 442600)
  func  367  WelsInitPps (pic_init_qp / qs 202643)
  func  225  slice init before WelsSliceHeaderWrite (func 1148): num_ref_idx override 120201
  func 1017  the encode loop: slice type / NAL type per frame type (665206, 665253), nal_ref_idc 669837,
             WelsUpdateRefSyntax's reordering commands (673611)
  func 1029  WelsHadamardT4Dc: luma DC Hadamard (x + 1) >> 1 with int16 clip (691446-691537)
  funcs 265/345/534/536  quantiser callers: DC quantised with (int16)(FF[0] << 1), MF[0] >> 1; intra
             rows at FF + 6 rows (345 @190274 load16_u off=96, 536 @283180 i32.const 38992)

  python tools/wasm_tables.py [--wasm PATH] [--out tests/golden/openh264_tables.json]
"""
import argparse
import hashlib
import json
import os
import re
import struct

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
DEFAULT_WASM = '/root/reference/scripts/h264.wasm'
DEFAULT_OUT = os.path.join(ROOT, 'tests', 'golden', 'openh264_tables.json')


def uleb(b, i):
    r = s = 0
    while True:
        x = b[i]
        i += 1
        r |= (x & 0x7f) << s
        s += 7
        if x < 0x80:
            return r, i


def sleb(b, i):
    r = s = 0
    while True:
        x = b[i]
        i += 1
        r |= (x & 0x7f) << s
        s += 7
        if x < 0x80:
            if x & 0x40:
                r -= 1 << s
            return r, i


def sections(b):
    assert b[:8] == b'\x00asm\x01\x00\x00\x00', 'not a wasm v1 module'
    out, i = {}, 8
    while i < len(b):
        sid = b[i]
        n, i = uleb(b, i + 1)
        out[sid] = (i, n)
        i += n
    return out


def data_segments(b, secs):
    """[(file offset, size)] of the data section's segments (all passive in this module)."""
    i, _ = secs[11]
    cnt, i = uleb(b, i)
    segs = []
    for _ in range(cnt):
        flag, i = uleb(b, i)
        if flag == 0:  # active: i32.const expr
            assert b[i] == 0x41
            _, i = sleb(b, i + 1)
            assert b[i] == 0x0b
            i += 1
        elif flag != 1:
            raise ValueError(f'unsupported data segment flag {flag}')
        sz, i = uleb(b, i)
        segs.append((i, sz))
        i += sz
    return segs


MEMORY_INIT = re.compile(rb'\x41([\x80-\xff]*[\x00-\x7f])\x41\x00\x41([\x80-\xff]*[\x00-\x7f])\xfc\x08(.)\x00', re.S)


def segment_addresses(b, secs, segs):
    """linear-memory address of each passive segment, from the memory.init sequence of the start
    function (a byte pattern inside the code section: dest, source offset 0, size, seg)."""
    c0, n = secs[10]
    addr = {}
    for m in MEMORY_INIT.finditer(b, c0, c0 + n):
        dest, _ = sleb(m.group(1) + b'\x00', 0)
        size, _ = sleb(m.group(2) + b'\x00', 0)
        k = m.group(3)[0]
        if k < len(segs) and segs[k][1] == size and k not in addr:
            addr[k] = dest
    if len(addr) != len(segs):
        raise ValueError(f'mapped {len(addr)} of {len(segs)} segments')
    return addr


class Memory:
    """read-only view of the initial linear memory image the data segments describe"""

    def __init__(self, b):
        self.b = b
        self.secs = sections(b)
        self.segs = data_segments(b, self.secs)
        self.addr = segment_addresses(b, self.secs, self.segs)

    def file_offset(self, mem, nbytes):
        for k, (fo, sz) in enumerate(self.segs):
            a = self.addr[k]
            if a <= mem and mem + nbytes <= a + sz:
                return fo + (mem - a)
        raise ValueError(f'address {mem} (+{nbytes}) is not inside one data segment')

    def read(self, mem, fmt, count):
        n = struct.calcsize('<' + fmt) * count
        try:
            fo = self.file_offset(mem, n)
            return list(struct.unpack_from(f'<{count}{fmt}', self.b, fo)), fo
        except ValueError:
            pass
        # a table whose tail is zero: the linker ends the data segment at its last non-zero byte and linear memory
        # starts zeroed, so the bytes past the segment read 0 -- as long as no other segment covers them
        for k, (fo, sz) in enumerate(self.segs):
            a = self.addr[k]
            if a <= mem < a + sz:
                for k2, (_, sz2) in enumerate(self.segs):
                    a2 = self.addr[k2]
                    if k2 != k and a2 < mem + n and a + sz < a2 + sz2:
                        raise ValueError(f'address {mem} (+{n}) spans two data segments')
                raw = self.b[fo + (mem - a):fo + sz] + bytes(n - (a + sz - mem))
                return list(struct.unpack_from(f'<{count}{fmt}', raw, 0)), fo + (mem - a)
        raise ValueError(f'address {mem} (+{n}) is not inside a data segment')


# name: (linear-memory address, struct format, shape, meaning)
TABLES = {
    'quant_ff': (38896, 'h', (58, 8), 'g_kiQuantInterFF: rounding offset per (qp, position); inter rows qp, intra rows qp + 6'),
    'quant_mf': (39824, 'h', (52, 8), 'g_kiQuantMF: level = ((|x| + FF) * MF) >> 16; DC: ((|x| + (FF[0] << 1)) * (MF[0] >> 1)) >> 16'),
    'lambda': (40768, 'i', (52,), 'g_kiQpCostTable: motion / mode cost lambda per QP'),
    'rc_bpp': (43440, 'd', (4, 4), 'RcCalculateIdrQp dBppArray[iBppIndex][i], iBppIndex by luma area <= 28800 / 115200 / 460800 / else'),
    'rc_init_qp': (43568, 'i', (4, 5), 'RcCalculateIdrQp initial IDR QP [iBppIndex][i]'),
    'rc_qp_range': (43648, 'i', (5, 2), 'RcCalculateIdrQp {max, min} QP of the IDR [i]'),
    'rc_qstep': (43696, 'i', (52,), 'g_kiQpToQstepTable (RcConvertQp2QStep): round(100 * 2^((qp - 4) / 6))'),
    'rc_tl_weight': (43376, 'i', (4, 4), 'g_kiTlWeight[iDecompositionStages][temporal id] (RcInitTlWeight, func 702): '
                     'one temporal layer -> row 0, weight 2000 = WEIGHT_MULTIPLY'),
    'logf_table': (73408, 'd', (16, 2), 'musl logf {invc, logc}[16] (func 483, called by RcConvertQStep2Qp in func 1226)'),
    'logf_poly': (73664, 'd', (4,), 'musl logf {Ln2, A[0], A[1], A[2]} (func 483)'),
    # intra mode decision at the wrapper's settings (camera usage, complexity LOW: DESIGN.md §3.3)
    'i16_avail_modes': (42624, 'b', (8, 5), 'g_kiIntra16AvaliMode[neighbour flags & 7]: the I16x16 modes WelsMdI16x16 (func 313) '
                        'tries, in order (0 V, 1 H, 2 DC, 3 P, 4 DC_L, 5 DC_T, 6 DC_128), count in column 4'),
    'i16_mode_map': (40976, 'b', (7,), 'g_kiMapModeI16x16: the syntax mode (Intra16x16PredMode) of each internal mode'),
    'chroma_avail_modes': (42992, 'b', (8, 5), 'g_kiIntraChromaAvailMode[neighbour flags & 7]: the chroma modes '
                           'WelsMdIntraChroma (func 312) tries, in order (0 DC, 1 H, 2 V, 3 P, 4 DC_L, 5 DC_T, 6 DC_128)'),
    'chroma_mode_map': (40983, 'b', (7,), 'g_kiMapModeIntraChroma: the syntax mode (intra_chroma_pred_mode) of each internal mode'),
    'i4_avail_index': (42688, 'b', (16, 16), 'g_kiNeighborIntraToI4x4[MB neighbour flags: 1 left, 2 top, 4 top-left, 8 '
                       'top-right][4x4 block, decoding order]: the block\'s availability index (same bits)'),
    'i4_avail_count': (42672, 'b', (16,), 'g_kiIntra4AvailCount[availability index]: modes WelsMdI4x4Fast (in func 774) tries; '
                       '7 and 9 take its fast search'),
    'i4_avail_modes': (43120, 'b', (16, 16), 'g_kiIntra4AvailMode[availability index]: the Intra4x4 modes in order '
                       '(0..8 the standard\'s, 9 DC_L, 10 DC_T, 11 DC_128)'),
    'i4_mode_map': (42976, 'b', (16,), 'g_kiMapModeI4x4: the syntax mode (Intra4x4PredMode) of each internal mode'),
    # P_Skip judge (oracle pskip_judge, GPU pskip_test_4w / _3w)
    'single_ctr_run': (40656, 'i', (16,), 'WelsCalculateSingleCtr4x4 (func 1011) cost per nonzero level by the run of zeros below '
                       'it in scan order (JVT-O079)'),
    'chroma_qp': (55152, 'B', (52,), 'g_kuiChromaQpTable: chroma QP of min(51, luma QP + chroma_qp_index_offset) (func 534)'),
    'level_limits': (63120, 'i', (17, 8),'g_ksLevelLimits {level_idc, MaxMBPS, MaxFS, MaxDpbMbs, MaxBR, MaxCPB, MinVmv, MaxVmv} '
                     '(WelsInitSps, func 280, walks it in this order)'),
}

# name: (file offset of the instruction, opcode, function, meaning)
CODE_CONSTANTS = {
    'camera_min_qp': (408976, 'i32.const', 597, 'iMinQp when the caller leaves it 0 (camera content)'),
    'camera_max_qp': (408980, 'i32.const', 597, 'iMaxQp when the caller leaves iMinQp 0 (camera content)'),
    'screen_min_qp': (408923, 'i32.const', 597, 'iMinQp default for screen content (unused by the wrapper)'),
    'screen_max_qp': (408927, 'i32.const', 597, 'iMaxQp default for screen content (unused by the wrapper)'),
    'default_max_frame_rate': (690465, 'f32bits', 1023, 'GetDefaultParams fMaxFrameRate (the wrapper never sets it)'),
    'default_fix_rc_overshoot': (690589, 'i32.const', 1023, 'GetDefaultParams bFixRCOverShoot: the IDR bpp search starts at column !flag'),
    'default_idr_bitrate_ratio': (690580, 'i32.const', 1023, 'GetDefaultParams iIdrBitrateRatio (percent)'),
    'frame_delta_qp_lower': (401392, 'i32.const', 592, 'iFrameDeltaQpLower = this - iRcVaryRatio / 100 (ratio 0 by default)'),
    'frame_delta_qp_upper': (401406, 'i32.const', 592, 'iFrameDeltaQpUpper = this - iRcVaryRatio / 50'),
    'skip_buffer_ratio': (401267, 'i32.const', 592, 'iSkipBufferRatio (percent of the bitrate the skip buffer holds)'),
    'idr_frame_qp_window': (767530, 'i32.const', 1226, 'RcCalculateIdrQp iMaxFrameQp = clip(QP + this), iMinFrameQp = clip(QP - this)'),
    'bits_exceeded_qp_step': (767701, 'i32.const', 1226, 'RcCalculatePictureQp: QP = last QP + this when the bits level is exceeded'),
    'cmplx_ratio_hi': (767802, 'i64.const', 1226, 'complexity ratio clamp, high (INT_MULTIPLY 100 + FRAME_CMPLX_RATIO_RANGE)'),
    'cmplx_ratio_lo': (767805, 'i64.const', 1226, 'complexity ratio clamp, low'),
    'area_90p': (766979, 'i32.const', 1226, 'iBppIndex 0 when w * h < this (<= 28800)'),
    'area_180p': (766991, 'i32.const', 1226, 'iBppIndex 1 when w * h < this'),
    'area_360p': (767005, 'i32.const', 1226, 'iBppIndex 2 when w * h < this, else 3'),
    # frame-level rate control (oracle rc_* in h264o_enc.c; GPU enc_bits.inc)
    'rc_vary_percentage': (689577, 'i32.const', 1021, 'InitializeExt: iRcVaryPercentage default (RcInitSequenceParameter '
                           'copies it to iRcVaryPercentage / iRcVaryRatio)'),
    'skip_qp_value_narrow': (401275, 'i32.const', 592, 'iSkipQpValue when the picture is < 31 MBs wide'),
    'skip_qp_value_wide': (401277, 'i32.const', 592, 'iSkipQpValue otherwise (VBV skip needs the average QP above it)'),
    'gom_rows_narrow': (401339, 'i32.const', 592, 'iNumberMbGom = mbw * (this + ...) below 31 MBs wide'),
    'gom_rows_wide': (401341, 'i32.const', 592, 'iNumberMbGom = mbw * (this + (4 - 2) * vary / 100) from 31 MBs wide'),
    'vgop_gops': (462240, 'i32.const', 702, 'RcInitTlWeight: iGopNumberInVGop = this >> iDecompositionStages (VGOP_SIZE)'),
    'vgop_bits_shift': (764394, 'i32.const', 1226, 'RcInitVGop: iRemainingBits += iBitsPerFrame << this (VGOP_SIZE 8)'),
    'weight_multiply': (764433, 'i32.const', 1226, 'RcInitVGop: iRemainingWeights = iGopNumberInVGop * this'),
    'min_bits_base': (458364, 'i32.const', 697, 'RcUpdateBitrateFps: iMinBitsTl ratio = this - ((this - vary) >> 1)'),
    'max_bits_ratio': (458356, 'i64.const', 697, 'RcUpdateBitrateFps: iMaxBitsTl ratio (percent)'),
    'bits_tl_divisor': (458411, 'i64.const', 697, 'RcUpdateBitrateFps: divisor of gop bits x ratio x weight (100 x 2000)'),
    'first_idr_target_shift': (766523, 'i32.const', 1226, 'RcDecideTargetBits: the first IDR targets iBitsPerFrame << this'),
    'continual_skip_reset': (763777, 'i32.const', 1226, 'WelsRcPictureInitGom: iContinualSkipFrames = this on every coded frame'),
    'qstep_min': (767923, 'i32.const', 1226, 'RcConvertQStep2Qp: QP 0 below this QStep'),
    'qstep_conv_ln2': (767435, 'f64.const', 1226, 'RcConvertQStep2Qp: / this (ln 2) after 6 * logf(QStep / 100)'),
    'qstep_conv_offset': (767445, 'f64.const', 1226, 'RcConvertQStep2Qp: + this'),
    'qstep_conv_round': (767455, 'f64.const', 1226, 'RcConvertQStep2Qp: + this, then truncation'),
    'cmplx_decay_new': (450973, 'i64.const', 676, 'RcUpdateFrameComplexity: weight of the new frame (of 100)'),
    'cmplx_decay_old': (450981, 'i64.const', 676, 'RcUpdateFrameComplexity: weight of the running mean / model'),
    'intra_decay_new': (760958, 'i64.const', 1218, 'RcUpdateIntraComplexity: weight of the new IDR'),
    'vbv_percent': (761473, 'f64.const', 1218, 'RcVBufferCalculationSkip: dIncPercent scale'),
    'vbv_percent_diff': (761493, 'f64.const', 1218, 'RcVBufferCalculationSkip: + this (-VGOP_BITS_PERCENTAGE_DIFF)'),
    'vbv_vgop_shift': (761488, 'i32.const', 1218, 'RcVBufferCalculationSkip: divisor iBitsPerFrame << this'),
    'gom_ratio_scale': (759582, 'i64.const', 1215, 'RcCalculateGomQp: iBitsRatio = this * left bits / (target left + 1)'),
    'gom_ratio_up2': (759595, 'i64.const', 1215, 'RcCalculateGomQp: QP + 2 below this ratio'),
    'gom_ratio_up1': (759608, 'i64.const', 1215, 'RcCalculateGomQp: QP + 1 below this ratio'),
    'gom_ratio_down1': (759623, 'i64.const', 1215, 'RcCalculateGomQp: QP - 1 above this ratio'),
    'gom_var_sample_shift': (530814, 'i32.const', 910, 'AnalyzeGomComplexityViaVar: sample count = first-row MBs << this'),
    # intra mode decision (oracle encode_intra_mb / best_chroma_mode; GPU enc_mb_kernel.inc)
    'md_camera_intra_fine_md': (675919, 'i32.const', 1017, 'PreprocessSliceCoding: pfIntraFineMd = table entry 254 '
                                '(func 774, WelsMdIntraFinePartitionVaa) for camera usage with iComplexityMode (param '
                                '+832) 0 -- the wrapper\'s'),
    'md_camera_md_cost_array': (675952, 'i32.const', 1017, 'PreprocessSliceCoding: pfMdCost = the function list + this '
                                '(pfSampleSad; + 112 is pfSampleSatd, the other branch): mode costs are SADs'),
    'md_vaa_i4_threshold': (474996, 'i32.const', 774, 'WelsMdIntraFinePartitionVaa: Intra4x4 is tried only when the source '
                            'MB\'s 4x4-mean variance (func 854) is above this'),
    'md_i4_mode_bits_shift': (475108, 'i32.const', 774, 'WelsMdI4x4Fast: a mode other than the predicted one costs lambda << this'),
    'md_i4_mb_overhead': (476981, 'i32.const', 774, 'WelsMdI4x4Fast: the I4x4 MB costs its blocks + lambda * this'),
    # P_Skip judge: WelsMdInterMb func 746, WelsMdPSkipEnc func 415, PredictSadSkip func 331,
    # WelsTryPUVskip func 534, WelsMdInterSecondaryModesEnc's double check func 399
    'pskip_mb_type_skip': (235007, 'i32.const', 415, 'MB_TYPE_SKIP: the co-located MB of a P reference picture must be of '
                           'this type for its skip SAD to admit the skip'),
    'pskip_try_nb_type_skip': (470843, 'i32.const', 746, 'WelsMdInterMb: without a skipped neighbour the skip is tried only '
                               'when the co-located MB of a P reference picture has this type (or MB_TYPE_BACKGROUND)'),
    'pskip_mv_min': (234693, 'i32.const', 415, 'WelsMdPSkipEnc: no skip when (mv >> 2) + 16 * mb position is below this'),
    'pskip_mv_max_low_bits': (234709, 'i32.const', 415, 'WelsMdPSkipEnc: ... or above (16 * MBs across | this)'),
    'pskip_max_level': (235268, 'i32.const', 415, 'WelsMdPSkipEnc: a luma 4x4 block whose largest |level| exceeds this '
                        'rejects the skip'),
    'pskip_luma_single_ctr_max': (235324, 'i32.const', 415, 'WelsMdPSkipEnc: the MB\'s summed single-coefficient cost of '
                                  'luma blocks may be at most this'),
    'pskip_chroma_single_ctr_max': (281767, 'i32.const', 534, 'WelsTryPUVskip: a chroma plane\'s summed single-coefficient '
                                    'cost may be at most this'),
    'pskip_double_check_type': (217889, 'i32.const', 399, 'WelsMdInterDoubleCheckPskip: only an MB of this type '
                                '(MB_TYPE_16x16) with cbp 0 at the skip vector becomes P_Skip'),
    # stream syntax (oracle h264o_write_sps / h264o_enc_encode)
    'sps_log2_max_frame_num_and_poc_type': (167923, 'i64.const', 280, 'WelsInitSps: one i64 store of '
                                            '{uiLog2MaxFrameNum (low word), uiPocType (high word)}'),
    'sps_default_profile': (168044, 'i32.const', 280, 'WelsInitSps: uiProfileIdc when the layer leaves it 0 (Baseline)'),
    'sps_level_table_address': (168196, 'i32.const', 280, 'WelsInitSps: address of g_ksLevelLimits (tables.level_limits)'),
    'sps_level_maxbr_factor': (168248, 'i32.const', 280, 'WelsInitSps: a level fits when MaxBR * this >= the target bitrate'),
    'sps_level_fallback': (168271, 'i32.const', 280, 'WelsInitSps: level_idc when no level fits'),
    'sps_direct8x8_level_gt': (439081, 'i32.const', 640, 'WelsWriteSpsSyntax: direct_8x8_inference_flag = level_idc > this'),
    'vui_log2_max_mv_length_code': (442600, 'i32.const', 640, 'WelsWriteVUI: the ue(16) code word (17 in 9 bits) of '
                                    'log2_max_mv_length_horizontal / vertical'),
    'pps_pic_init_qp_qs': (202643, 'i32.const', 367, 'WelsInitPps: one u16 store of {iPicInitQp, iPicInitQs} (26, 26)'),
    'p_slice_type_and_nal': (665206, 'i64.const', 1017, 'P frame: one i64 store of {eSliceType (P_SLICE 0), eNalType (1)}'),
    'idr_slice_type_and_nal': (665253, 'i64.const', 1017, 'IDR frame: {eSliceType (I_SLICE 2), eNalType (5)}: slice_type '
                               'is written without the +5'),
    'slice_nal_ref_idc': (669837, 'i32.const', 1017, 'eNalRefIdc of every slice NAL with one temporal layer'),
    'p_num_ref_idx_override': (120201, 'i32.const', 225, 'P slice: bNumRefIdxActiveOverrideFlag (uiNumRefIdxL0Active = 1)'),
    'p_reorder_end_idc': (673611, 'i32.const', 1017, 'WelsUpdateRefSyntax: the second reordering command '
                          '(modification_of_pic_nums_idc 3) after {idc 0, abs_diff_pic_num_minus1}'),
}


def decode_const(b, off, op):
    if op in ('i32.const', 'f32bits'):
        assert b[off] == 0x41, f'no i32.const at {off}'
        v, _ = sleb(b, off + 1)
        if op == 'f32bits':
            v = struct.unpack('<f', struct.pack('<i', v))[0]
        return v
    if op == 'i64.const':
        assert b[off] == 0x42, f'no i64.const at {off}'
        return sleb(b, off + 1)[0]
    if op == 'f64.const':
        assert b[off] == 0x44, f'no f64.const at {off}'
        return struct.unpack_from('<d', b, off + 1)[0]
    raise ValueError(op)


def extract(path):
    b = open(path, 'rb').read()
    mem = Memory(b)
    out = {'source': 'scripts/h264.wasm (reference, prebuilt OpenH264 + wrapper; parsed as bytes, never executed)',
           'sha256': hashlib.sha256(b).hexdigest(), 'bytes': len(b), 'tables': {}, 'code_constants': {},
           'segments': [{'file_offset': fo, 'size': sz, 'address': mem.addr[k]} for k, (fo, sz) in enumerate(mem.segs)]}
    for name, (addr, fmt, shape, meaning) in TABLES.items():
        n = 1
        for d in shape:
            n *= d
        vals, fo = mem.read(addr, fmt, n)
        if len(shape) == 2:
            vals = [vals[r * shape[1]:(r + 1) * shape[1]] for r in range(shape[0])]
        out['tables'][name] = {'address': addr, 'file_offset': fo, 'type': {'b': 'int8', 'B': 'uint8', 'h': 'int16', 'i': 'int32', 'd': 'f64'}[fmt],
                               'shape': list(shape), 'meaning': meaning, 'values': vals}
    for name, (off, op, func, meaning) in CODE_CONSTANTS.items():
        out['code_constants'][name] = {'file_offset': off, 'instruction': op.replace('f32bits', 'i32.const (f32 bits)'),
                                       'function': func, 'meaning': meaning, 'value': decode_const(b, off, op)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--wasm', default=DEFAULT_WASM)
    ap.add_argument('--out', default=DEFAULT_OUT)
    a = ap.parse_args()
    d = extract(a.wasm)
    with open(a.out, 'w') as f:
        json.dump(d, f, indent=1)
        f.write('\n')
    t = d['tables']
    print(f"wrote {a.out}: lambda[51]={t['lambda']['values'][51]} mf[0]={t['quant_mf']['values'][0]} "
          f"ff[57]={t['quant_ff']['values'][57]} camera QP [{d['code_constants']['camera_min_qp']['value']}, "
          f"{d['code_constants']['camera_max_qp']['value']}] fps {d['code_constants']['default_max_frame_rate']['value']}")


if __name__ == '__main__':
    main()
