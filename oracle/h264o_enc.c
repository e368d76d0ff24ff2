/*
 * oracle/h264o_enc.c -- TEST INFRASTRUCTURE ONLY (CPU oracle; see oracle/README.md).
 *
 * CPU restatement of the encoder behind openh264_wrapper.cpp:198-228 (init_encoder) and
 * :358-389 (encode_frame_yuv_i420 -> ISVCEncoder::EncodeFrame). The wrapper's parameters
 * (CAMERA_VIDEO_REAL_TIME, RC_BITRATE_MODE, LOW_COMPLEXITY, iNumRefFrame=1, AQ/background/
 * scene-change off; upstream defaults Baseline/CAVLC, single slice, IDR only on first frame or
 * ForceIntraFrame, loop filter on) fix the syntax; the decision algorithm (rate control, integer
 * diamond ME, half/quarter SATD refinement, I16x16/I4x4/P16x16/P_Skip mode decision) restates
 * OpenH264's upstream approach as specified in DESIGN.md §3. OpenH264 sources are not in the
 * reference and its prebuilt h264.wasm may not be executed here, so parity with OpenH264 itself
 * is UNPINNED; the GPU product is held bit-exact to THIS file.
 */
#include "h264o_api.h"
#include "h264o_common.h"
#include "h264o_tables.h"
#include <stdlib.h>
#include <string.h>

/* Rate-control constants OpenH264 applies at the wrapper's parameters, as its h264.wasm holds them
 * (tests/golden/openh264_tables.json "code_constants"): */
#define RC_FPS 60           /* GetDefaultParams fMaxFrameRate (wasm func 1023); the wrapper never sets it */
#define QP_MIN 12           /* iMinQp / iMaxQp for camera content when the caller leaves iMinQp 0 (func 597) */
#define QP_MAX 42
#define FRAME_DQP_LOWER 3   /* iFrameDeltaQpLower / iFrameDeltaQpUpper at iRcVaryRatio 0 (func 592) */
#define FRAME_DQP_UPPER 5
#define IDR_QP_WINDOW 3     /* RcCalculateIdrQp: the IDR's frame QP window (func 1226) */
/* Stream syntax OpenH264 writes at the wrapper's parameters, read from the same binary's code
 * (tools/wasm_syntax.py pins each instruction): WelsInitSps (func 280) stores
 * uiLog2MaxFrameNum 15 and uiPocType 2 as one i64 constant (file offset 167929), so the slice header
 * carries a 15-bit frame_num and no POC; the level comes from the level limits at the 60 fps frame
 * rate and the target bitrate (level_idc_for below). */
#define LOG2_MAX_FRAME_NUM 15
#ifndef CROSS_THR
#define CROSS_THR 1024  /* cross search when the best integer cost exceeds this */
#endif

struct H264OEnc {
    int w, h, mbw, mbh, cw, ch;
    int bitrate;
    uint8_t *src[3], *rec[3], *ref[3];
    MBInfo *mbs;
    int first, force_idr;
    int frame_num, idr_pic_id, poc;
    int qp;           /* the next frame's QP before its bounds (the bits-ratio step below) */
    int last_qp, last_idr;
    int init_qp, rmin, rmax;  /* RcCalculateIdrQp: first IDR QP and the IDR QP range */
    int idr_num, pframes;     /* IDRs / P frames coded (OpenH264 iIdrNum, iPFrameNum) */
    int qmin, qmax;           /* the coded frame's QP window (iMinFrameQp, iMaxFrameQp): clamps the row QPs */
    int64_t last_bits;
    /* GOM (MB-row) rate control and frame skipping */
    int *rowqp;       /* QP offset plan of the next frame, one per MB row (added to the frame QP) */
    int64_t *rowbits; /* macroblock_layer() bits per MB row of the last coded frame */
    int64_t vbuf;     /* virtual buffer fullness (bits) */
    int skip_en, skipped;
    int stat_cross, stat_cross_moved, stat_nb_start;  /* ME path counters (tests: coverage of the search stages) */
};

/* ---------------- rate control ---------------- */
/* RcCalculateIdrQp restated from the reference's h264.wasm (func 1226, file offsets 766934-767578):
 * bits per pixel = bitrate / (float)(fps * w * h); area class by w * h; the first column i of
 * OH_RC_BPP[class] at or above it (the search starts at column 0: bFixRCOverShoot defaults to 1);
 * IDR QP range = OH_RC_QP_RANGE[i] clipped to [QP_MIN, QP_MAX]; first IDR QP = OH_RC_INIT_QP[class][i]
 * clipped to that range. Writes *rmin / *rmax, returns the first IDR QP. */
int h264o_rc_idr_params(int w, int h, int bitrate, int *rmin, int *rmax) {
    float p = (float)RC_FPS * (float)w;
    p = p * (float)h;
    const double bpp = (double)bitrate / (double)p;
    const int area = w * h;
    const int cls = area < 28801 ? 0 : (area < 115201 ? 1 : (area < 460801 ? 2 : 3));
    int i = 0;
    while (i < 4 && !(OH_RC_BPP[cls][i] >= bpp)) i++;
    const int mx = clip3(QP_MIN, QP_MAX, OH_RC_QP_RANGE[i][0]), mn = clip3(QP_MIN, QP_MAX, OH_RC_QP_RANGE[i][1]);
    *rmin = mn; *rmax = mx;
    return clip3(mn, mx, OH_RC_INIT_QP[cls][i]);
}
int h264o_rc_init_qp(int w, int h, int bitrate) {
    int a, b;
    return h264o_rc_idr_params(w, h, bitrate, &a, &b);
}
/* The next frame's QP before its bounds: this project's step on the bits of the frame just coded
 * against the per-frame target T = bitrate / fps (x4 for an IDR: iIdrBitrateRatio 400). OpenH264
 * derives it from its complexity model instead (RcCalculatePictureQp); not pinned. */
int h264o_rc_next_qp(int qp, int64_t bits, int bitrate, int was_idr) {
    int64_t T = bitrate / RC_FPS;
    if (was_idr) T *= 4;
    int d;
    if (bits > 2 * T) d = 3;
    else if (2 * bits > 3 * T) d = 2;
    else if (100 * bits > 115 * T) d = 1;
    else if (2 * bits < T) d = -2;
    else if (100 * bits < 85 * T) d = -1;
    else d = 0;
    return clip3(QP_MIN, QP_MAX, qp + d);
}
/* The coded frame's QP and window (RcCalculateIdrQp / RcCalculatePictureQp, wasm func 1226):
 * IDR: the first takes the table QP, later ones the step result, clipped to the IDR range; window
 * QP -/+ IDR_QP_WINDOW inside the range. P: the first P frame takes the first IDR's QP, later ones
 * the step result; window [last - FRAME_DQP_LOWER, last + FRAME_DQP_UPPER] inside [QP_MIN, QP_MAX],
 * last = the previous coded frame's QP; the QP is clipped to the window. */
static int rc_frame_qp(H264OEnc *e, int idr) {
    int q;
    if (idr) {
        q = e->idr_num == 0 ? e->init_qp : clip3(e->rmin, e->rmax, e->qp);
        e->qmin = clip3(e->rmin, e->rmax, q - IDR_QP_WINDOW);
        e->qmax = clip3(e->rmin, e->rmax, q + IDR_QP_WINDOW);
        e->idr_num++;
    } else {
        q = e->pframes == 0 ? e->init_qp : e->qp;
        e->qmin = clip3(QP_MIN, QP_MAX, e->last_qp - FRAME_DQP_LOWER);
        e->qmax = clip3(QP_MIN, QP_MAX, e->last_qp + FRAME_DQP_UPPER);
        q = clip3(e->qmin, e->qmax, q);
        e->pframes++;
    }
    return q;
}
/* MB-row ("GOM") QP offsets of the next frame: rows that cost more than the mean in the last coded
 * frame are quantised more coarsely, cheaper rows more finely; the row QP is the frame QP plus the
 * offset, clipped to the frame's window (this project's rule; OpenH264 re-plans GOMs from the bits
 * of the frame being coded, a serial dependency). */
int h264o_rc_row_delta(int64_t row_bits, int64_t mean) {
    if (mean <= 0) return 0;
    if (row_bits > 2 * mean) return 2;
    if (4 * row_bits > 5 * mean) return 1;
    if (2 * row_bits < mean) return -1;
    return 0;
}
static void rc_plan_rows(H264OEnc *e) {
    int64_t sum = 0;
    for (int r = 0; r < e->mbh; r++) sum += e->rowbits[r];
    int64_t mean = sum / e->mbh;
    for (int r = 0; r < e->mbh; r++) e->rowqp[r] = h264o_rc_row_delta(e->rowbits[r], mean);
}
/* oracle RC constants for tests/test_oracle_golden.py (pinned against the h264.wasm fixture) */
void h264o_rc_constants(int32_t out[8]) {
    out[0] = RC_FPS; out[1] = QP_MIN; out[2] = QP_MAX; out[3] = FRAME_DQP_LOWER; out[4] = FRAME_DQP_UPPER;
    out[5] = IDR_QP_WINDOW; out[6] = 400; out[7] = 50;
}
/* the oracle's copy of an OpenH264 table, for the same test: returns the entry count (-1: unknown) */
int h264o_table(const char *name, double *out) {
    int n = 0;
    if (!strcmp(name, "quant_mf")) { for (int i = 0; i < 52 * 8; i++) out[n++] = OH_QUANT_MF[i / 8][i % 8]; }
    else if (!strcmp(name, "quant_ff")) { for (int i = 0; i < 58 * 8; i++) out[n++] = OH_QUANT_FF[i / 8][i % 8]; }
    else if (!strcmp(name, "lambda")) { for (int i = 0; i < 52; i++) out[n++] = LAMBDA[i]; }
    else if (!strcmp(name, "rc_bpp")) { for (int i = 0; i < 16; i++) out[n++] = OH_RC_BPP[i / 4][i % 4]; }
    else if (!strcmp(name, "rc_init_qp")) { for (int i = 0; i < 20; i++) out[n++] = OH_RC_INIT_QP[i / 5][i % 5]; }
    else if (!strcmp(name, "rc_qp_range")) { for (int i = 0; i < 10; i++) out[n++] = OH_RC_QP_RANGE[i / 2][i % 2]; }
    else if (!strcmp(name, "rc_qstep")) { for (int i = 0; i < 52; i++) out[n++] = OH_RC_QSTEP[i]; }
    else if (!strcmp(name, "level_limits")) { for (int i = 0; i < 17 * 6; i++) out[n++] = OH_LEVEL_LIMITS[i / 6][i % 6]; }
    else return -1;
    return n;
}
/* mb_qp_delta carrying QP a from QP_pred b, wrapped into -26..25 (7.4.5) */
static int qp_delta_wrap(int a, int b) { return ((a - b + 26 + 52) % 52) - 26; }
/* level_idc as WelsInitSps chooses it (func 280, file offsets 168119-169382): the first row of the level
 * limits (OH_LEVEL_LIMITS, in the binary's order) whose MaxMBPS covers the MB rate at the layer's frame
 * rate (60 fps: the wrapper leaves fMaxFrameRate at its default; (uint32)(60.0f * (float)MBs)), whose MaxFS
 * covers the frame and 8 * MaxFS covers max(mbw^2, mbh^2), whose MaxDpbMbs covers MBs x num_ref_frames and
 * whose MaxBR * 1200 covers the target bitrate (the bitrate test is skipped when the bitrate is 0); none:
 * 51. Level 1b (idc 9) becomes constraint_set3 + idc 11 for Baseline (*cs3 = 1). */
int h264o_level_idc(int w, int h, int bitrate, int *cs3) {
    const uint32_t mbw = (uint32_t)(w + 15) >> 4, mbh = (uint32_t)(h + 15) >> 4, mbs = mbw * mbh;
    const uint32_t sq = mbw * mbw > mbh * mbh ? mbw * mbw : mbh * mbh, dpb = mbs * 1;
    const uint32_t mbps = (uint32_t)(60.0f * (float)mbs);
    int level = 51;
    *cs3 = 0;
    for (int i = 0; i < 17; i++) {
        const int32_t *L = OH_LEVEL_LIMITS[i];
        if ((uint32_t)L[1] < mbps || (uint32_t)L[2] < mbs || ((uint32_t)L[2] << 3) < sq || (uint32_t)L[3] < dpb) continue;
        if (bitrate && L[4] * 1200 < bitrate) continue;
        level = L[0];
        break;
    }
    if (level == 9) { *cs3 = 1; level = 11; }
    return level;
}

/* ---------------- parameter sets (7.3.2.1 / 7.3.2.2) ---------------- */
/* OpenH264's SPS at the wrapper's parameters: WelsInitSps (func 280) fills it, WelsWriteSpsSyntax +
 * WelsWriteVUI (func 640) write it (DESIGN.md §3.1 lists the file offset of every field):
 * profile 66; constraint_set0 (Baseline) and constraint_set1 (profile <= 77) set, set2 clear (one layer),
 * set3 only for level 1b, four reserved zero bits; level_idc (above); sps id 0 (INCREASING_ID never
 * advances it for a single non-simulcast layer); log2_max_frame_num 15; POC type 2; num_ref_frames 1;
 * gaps 0; frame_mbs_only 1; direct_8x8_inference = level_idc >= 30; cropping right / bottom by half the
 * padding; vui_parameters_present 1 with every flag 0 except bitstream_restriction: motion vectors over
 * picture boundaries 1, max_bytes_per_pic_denom 0, max_bits_per_mb_denom 0, log2_max_mv_length 16 / 16,
 * max_num_reorder_frames 0, max_dec_frame_buffering = num_ref_frames. */
size_t h264o_write_sps(int w, int h, int bitrate, uint8_t *out) {
    int mbw = (w + 15) / 16, mbh = (h + 15) / 16, cs3;
    const int level = h264o_level_idc(w, h, bitrate, &cs3);
    BW b; bw_init(&b);
    bw_put(&b, 66, 8);            /* profile_idc: Baseline */
    bw_put(&b, 0xC0 | (cs3 << 4), 8); /* constraint_set0..3, reserved_zero_4bits */
    bw_put(&b, level, 8);
    bw_ue(&b, 0);                 /* seq_parameter_set_id */
    bw_ue(&b, LOG2_MAX_FRAME_NUM - 4);
    bw_ue(&b, 2);                 /* pic_order_cnt_type */
    bw_ue(&b, 1);                 /* max_num_ref_frames */
    bw_put(&b, 0, 1);             /* gaps_in_frame_num_value_allowed_flag */
    bw_ue(&b, mbw - 1);
    bw_ue(&b, mbh - 1);
    bw_put(&b, 1, 1);             /* frame_mbs_only_flag */
    bw_put(&b, level >= 30, 1);   /* direct_8x8_inference_flag */
    int crop = (mbw * 16 != w) || (mbh * 16 != h);
    bw_put(&b, crop, 1);
    if (crop) { bw_ue(&b, 0); bw_ue(&b, (mbw * 16 - w) / 2); bw_ue(&b, 0); bw_ue(&b, (mbh * 16 - h) / 2); }
    bw_put(&b, 1, 1);             /* vui_parameters_present_flag */
    bw_put(&b, 0, 1); bw_put(&b, 0, 1); bw_put(&b, 0, 1); /* aspect_ratio_info, overscan_info, video_signal_type */
    bw_put(&b, 0, 1); bw_put(&b, 0, 1);                   /* chroma_loc_info, timing_info */
    bw_put(&b, 0, 1); bw_put(&b, 0, 1); bw_put(&b, 0, 1); /* nal_hrd, vcl_hrd, pic_struct */
    bw_put(&b, 1, 1);             /* bitstream_restriction_flag */
    bw_put(&b, 1, 1);             /* motion_vectors_over_pic_boundaries_flag */
    bw_ue(&b, 0); bw_ue(&b, 0);   /* max_bytes_per_pic_denom, max_bits_per_mb_denom */
    bw_ue(&b, 16); bw_ue(&b, 16); /* log2_max_mv_length_horizontal / vertical */
    bw_ue(&b, 0);                 /* max_num_reorder_frames */
    bw_ue(&b, 1);                 /* max_dec_frame_buffering */
    bw_trailing(&b);
    size_t n = nal_write(out, 3, 7, b.buf, b.len);
    bw_free(&b);
    return n;
}
/* OpenH264's PPS (WelsInitPps func 367, WelsWritePpsSyntax func 370): ids 0, CAVLC, one slice group,
 * num_ref_idx defaults 0, no weighted prediction, pic_init_qp / qs 26, chroma_qp_index_offset 0,
 * deblocking_filter_control_present 1, constrained_intra_pred 0, redundant_pic_cnt_present 0 */
size_t h264o_write_pps(uint8_t *out) {
    BW b; bw_init(&b);
    bw_ue(&b, 0); bw_ue(&b, 0);   /* pps id, sps id */
    bw_put(&b, 0, 1);             /* entropy_coding_mode_flag: CAVLC */
    bw_put(&b, 0, 1);             /* bottom_field_pic_order_in_frame_present_flag */
    bw_ue(&b, 0);                 /* num_slice_groups_minus1 */
    bw_ue(&b, 0); bw_ue(&b, 0);   /* num_ref_idx_l0/l1_default_active_minus1 */
    bw_put(&b, 0, 1); bw_put(&b, 0, 2); /* weighted_pred_flag, weighted_bipred_idc */
    bw_se(&b, 0); bw_se(&b, 0); bw_se(&b, 0); /* pic_init_qp/qs_minus26, chroma_qp_index_offset */
    bw_put(&b, 1, 1);             /* deblocking_filter_control_present_flag */
    bw_put(&b, 0, 1);             /* constrained_intra_pred_flag */
    bw_put(&b, 0, 1);             /* redundant_pic_cnt_present_flag */
    bw_trailing(&b);
    size_t n = nal_write(out, 3, 8, b.buf, b.len);
    bw_free(&b);
    return n;
}

/* ---------------- helpers ---------------- */
static void get_nb16(const uint8_t *pl, int stride, int px, int py, int size, int has_top, int has_left, IntraNb *n) {
    memset(n, 0, sizeof(*n));
    n->has_top = has_top; n->has_left = has_left; n->has_tl = has_top && has_left;
    if (has_top) for (int i = 0; i < size; i++) n->top[i] = pl[(py - 1) * stride + px + i];
    if (has_left) for (int i = 0; i < size; i++) n->left[i] = pl[(py + i) * stride + px - 1];
    if (n->has_tl) n->tl = pl[(py - 1) * stride + px - 1];
}
static int i4_tr_avail(int mbx, int mby, int mbw, int ras) {
    int bx = ras & 3, by = ras >> 2;
    if (by == 0) return bx < 3 ? mby > 0 : (mby > 0 && mbx + 1 < mbw);
    if (bx == 3) return 0;
    return RAS2BLK[(by - 1) * 4 + bx + 1] < RAS2BLK[ras];
}
static void get_nb4(const uint8_t *pl, int stride, int mbx, int mby, int mbw, int ras, IntraNb *n) {
    int bx = ras & 3, by = ras >> 2, px = mbx * 16 + bx * 4, py = mby * 16 + by * 4;
    memset(n, 0, sizeof(*n));
    n->has_top = by > 0 || mby > 0;
    n->has_left = bx > 0 || mbx > 0;
    n->has_tl = n->has_top && n->has_left;
    n->has_tr = n->has_top && i4_tr_avail(mbx, mby, mbw, ras);
    if (n->has_top) {
        for (int i = 0; i < 4; i++) n->top[i] = pl[(py - 1) * stride + px + i];
        for (int i = 4; i < 8; i++) n->top[i] = n->has_tr ? pl[(py - 1) * stride + px + i] : n->top[3];
    }
    if (n->has_left) for (int i = 0; i < 4; i++) n->left[i] = pl[(py + i) * stride + px - 1];
    if (n->has_tl) n->tl = pl[(py - 1) * stride + px - 1];
}
/* Intra4x4PredMode prediction (8.3.1.1) */
static int i4_pred_mode(const MBInfo *mbs, const MBInfo *cur, int mbw, int mbx, int mby, int ras) {
    int bx = ras & 3, by = ras >> 2, a, b;
    if (bx > 0) a = cur->i4mode[ras - 1];
    else if (mbx > 0) { const MBInfo *m = &mbs[mby * mbw + mbx - 1]; a = m->type == MBT_I4 ? m->i4mode[ras + 3] : 2; }
    else return 2;
    if (by > 0) b = cur->i4mode[ras - 4];
    else if (mby > 0) { const MBInfo *m = &mbs[(mby - 1) * mbw + mbx]; b = m->type == MBT_I4 ? m->i4mode[ras + 12] : 2; }
    else return 2;
    return imin(a, b);
}
static int satd16x16(const uint8_t *src, int ss, const uint8_t *pred, int ps) {
    int s = 0, d[16];
    for (int by = 0; by < 4; by++)
        for (int bx = 0; bx < 4; bx++) {
            for (int y = 0; y < 4; y++)
                for (int x = 0; x < 4; x++)
                    d[4 * y + x] = src[(4 * by + y) * ss + 4 * bx + x] - pred[(4 * by + y) * ps + 4 * bx + x];
            s += satd4(d);
        }
    return s;
}
static int satd8x8(const uint8_t *src, int ss, const uint8_t *pred, int ps) {
    int s = 0, d[16];
    for (int by = 0; by < 2; by++)
        for (int bx = 0; bx < 2; bx++) {
            for (int y = 0; y < 4; y++)
                for (int x = 0; x < 4; x++)
                    d[4 * y + x] = src[(4 * by + y) * ss + 4 * bx + x] - pred[(4 * by + y) * ps + 4 * bx + x];
            s += satd4(d);
        }
    return s;
}
static int count_nz(const int16_t *c, int n) { int k = 0; for (int i = 0; i < n; i++) k += c[i] != 0; return k; }

/* Luma 4x4 residual: forward transform + quantisation into scan-ordered levels; returns the
 * raster DC coefficient (unquantised) for the I16 path. */
static int luma_block_levels(const uint8_t *src, int ss, const uint8_t *pred, int ps, int qp, int intra, int first,
                             int16_t lv[16]) {
    int d[16], c[16];
    for (int y = 0; y < 4; y++) for (int x = 0; x < 4; x++) d[4 * y + x] = src[y * ss + x] - pred[y * ps + x];
    fdct4(d, c);
    lv[0] = 0;
    for (int k = first; k < 16; k++) lv[k] = (int16_t)quant4(c[ZIGZAG4[k]], qp, ZIGZAG4[k], intra);
    return c[0];
}
/* Chroma residual for one MB: levels + recon into rec planes. pred[pl][64]. */
static void encode_chroma(H264OEnc *e, MBInfo *mb, int mbx, int mby, uint8_t pred[2][64], int intra) {
    int qpc = CHROMA_QP[mb->qp];
    int cs = e->cw / 2, any_ac = 0, any_dc = 0;
    for (int pl = 0; pl < 2; pl++) {
        const uint8_t *src = e->src[1 + pl] + mby * 8 * cs + mbx * 8;
        int dcraw[4];
        for (int blk = 0; blk < 4; blk++) {
            int ox = (blk & 1) * 4, oy = (blk >> 1) * 4;
            dcraw[blk] = luma_block_levels(src + oy * cs + ox, cs, pred[pl] + oy * 8 + ox, 8, qpc, intra, 1, mb->cac[pl][blk]);
            if (count_nz(mb->cac[pl][blk], 16)) any_ac = 1;
        }
        int f0 = dcraw[0] + dcraw[1] + dcraw[2] + dcraw[3], f1 = dcraw[0] - dcraw[1] + dcraw[2] - dcraw[3];
        int f2 = dcraw[0] + dcraw[1] - dcraw[2] - dcraw[3], f3 = dcraw[0] - dcraw[1] - dcraw[2] + dcraw[3];
        mb->cdc[pl][0] = (int16_t)quant_dc4(f0, qpc, intra); mb->cdc[pl][1] = (int16_t)quant_dc4(f1, qpc, intra);
        mb->cdc[pl][2] = (int16_t)quant_dc4(f2, qpc, intra); mb->cdc[pl][3] = (int16_t)quant_dc4(f3, qpc, intra);
        if (count_nz(mb->cdc[pl], 4)) any_dc = 1;
    }
    int cbpc = any_ac ? 2 : (any_dc ? 1 : 0);
    mb->cbp = (mb->cbp & 15) | (cbpc << 4);
    for (int pl = 0; pl < 2; pl++) {
        int dc[4];
        chroma_dc_dequant(mb->cdc[pl], qpc, dc);
        uint8_t *dst = e->rec[1 + pl] + mby * 8 * cs + mbx * 8;
        for (int blk = 0; blk < 4; blk++) {
            int ox = (blk & 1) * 4, oy = (blk >> 1) * 4, coef[16];
            dequant_block(mb->cac[pl][blk], qpc, 1, coef);
            coef[0] = dc[blk];
            idct4_add(coef, dst + oy * cs + ox, cs, pred[pl] + oy * 8 + ox, 8);
            mb->nnz[16 + 4 * pl + blk] = (uint8_t)count_nz(mb->cac[pl][blk], 16);
        }
    }
}
static int best_chroma_mode(H264OEnc *e, int mbx, int mby, IntraNb nb[2], uint8_t pred[2][64]) {
    int cs = e->cw / 2, best = -1, bc = 0;
    uint8_t p[2][64];
    for (int m = 0; m < 4; m++) {
        if (!pred_chroma_avail(&nb[0], m)) continue;
        int c = 0;
        for (int pl = 0; pl < 2; pl++) {
            pred_chroma(&nb[pl], m, p[pl]);
            c += satd8x8(e->src[1 + pl] + mby * 8 * cs + mbx * 8, cs, p[pl], 8);
        }
        if (best < 0 || c < bc) { best = m; bc = c; memcpy(pred, p, sizeof(p)); }
    }
    return best;
}
static void chroma_intra(H264OEnc *e, MBInfo *mb, int mbx, int mby) {
    IntraNb nb[2];
    int cs = e->cw / 2;
    for (int pl = 0; pl < 2; pl++) get_nb16(e->rec[1 + pl], cs, mbx * 8, mby * 8, 8, mby > 0, mbx > 0, &nb[pl]);
    uint8_t pred[2][64];
    mb->cmode = best_chroma_mode(e, mbx, mby, nb, pred);
    encode_chroma(e, mb, mbx, mby, pred, 1);
}

/* I16x16 best mode by SATD (ties -> lower mode index) */
static int i16_best(H264OEnc *e, int mbx, int mby, const IntraNb *nb, int *cost, uint8_t pred[256]) {
    const uint8_t *src = e->src[0] + mby * 16 * e->cw + mbx * 16;
    int best = -1, bc = 0;
    uint8_t p[256];
    for (int m = 0; m < 4; m++) {
        if (!pred16x16_avail(nb, m)) continue;
        pred16x16(nb, m, p);
        int c = satd16x16(src, e->cw, p, 16);
        if (best < 0 || c < bc) { best = m; bc = c; memcpy(pred, p, 256); }
    }
    *cost = bc;
    return best;
}
static void encode_i16(H264OEnc *e, MBInfo *mb, int mbx, int mby, int mode, const uint8_t pred[256]) {
    const uint8_t *src = e->src[0] + mby * 16 * e->cw + mbx * 16;
    uint8_t *dst = e->rec[0] + mby * 16 * e->cw + mbx * 16;
    int qp = mb->qp, dcraw[16], any_ac = 0;
    mb->type = MBT_I16; mb->i16mode = mode;
    for (int ras = 0; ras < 16; ras++) {
        int ox = (ras & 3) * 4, oy = (ras >> 2) * 4;
        dcraw[ras] = luma_block_levels(src + oy * e->cw + ox, e->cw, pred + oy * 16 + ox, 16, qp, 1, 1, mb->luma[ras]);
        if (count_nz(mb->luma[ras], 16)) any_ac = 1;
    }
    /* forward 4x4 Hadamard on the spatial DC matrix, then (x + 1) >> 1 (WelsHadamardT4Dc, wasm func 1029;
     * the int16 clip there never binds for 8-bit input: |x| <= 32640) */
    int t[16], f[16];
    for (int i = 0; i < 4; i++) {
        int a = dcraw[4 * i], b = dcraw[4 * i + 1], c = dcraw[4 * i + 2], d = dcraw[4 * i + 3];
        t[4 * i + 0] = a + b + c + d; t[4 * i + 1] = a + b - c - d; t[4 * i + 2] = a - b - c + d; t[4 * i + 3] = a - b + c - d;
    }
    for (int j = 0; j < 4; j++) {
        int a = t[j], b = t[4 + j], c = t[8 + j], d = t[12 + j];
        f[j] = (a + b + c + d + 1) >> 1; f[4 + j] = (a + b - c - d + 1) >> 1; f[8 + j] = (a - b - c + d + 1) >> 1;
        f[12 + j] = (a - b + c - d + 1) >> 1;
    }
    for (int k = 0; k < 16; k++) mb->lumadc[k] = (int16_t)quant_dc4(f[ZIGZAG4[k]], qp, 1);
    mb->cbp = any_ac ? 15 : 0;
    int dc[16];
    luma_dc_dequant(mb->lumadc, qp, dc);
    for (int ras = 0; ras < 16; ras++) {
        int ox = (ras & 3) * 4, oy = (ras >> 2) * 4, coef[16];
        dequant_block(mb->luma[ras], qp, 1, coef);
        coef[0] = dc[ras];
        idct4_add(coef, dst + oy * e->cw + ox, e->cw, pred + oy * 16 + ox, 16);
        mb->nnz[ras] = (uint8_t)count_nz(mb->luma[ras], 16);
        mb->i4mode[ras] = 2;
    }
}

/* Intra MB decision for I slices: I16x16 vs I4x4. */
static void encode_intra_mb(H264OEnc *e, MBInfo *mb, int mbx, int mby) {
    int lam = LAMBDA[mb->qp];
    IntraNb nb;
    get_nb16(e->rec[0], e->cw, mbx * 16, mby * 16, 16, mby > 0, mbx > 0, &nb);
    uint8_t p16[256];
    int c16;
    int m16 = i16_best(e, mbx, mby, &nb, &c16, p16);
    /* I4x4 trial with progressive reconstruction and exact early termination */
    MBInfo t = *mb;
    t.type = MBT_I4;
    int cost4 = 24 * lam, won = 1;
    const uint8_t *src = e->src[0] + mby * 16 * e->cw + mbx * 16;
    uint8_t *dst = e->rec[0] + mby * 16 * e->cw + mbx * 16;
    for (int blk = 0; blk < 16; blk++) {
        int ras = BLK2RAS[blk], ox = (ras & 3) * 4, oy = (ras >> 2) * 4;
        IntraNb n4;
        get_nb4(e->rec[0], e->cw, mbx, mby, e->mbw, ras, &n4);
        int pm = i4_pred_mode(e->mbs, &t, e->mbw, mbx, mby, ras);
        int best = -1, bc = 0, d[16];
        uint8_t p[16], bp[16];
        for (int m = 0; m < 9; m++) {
            if (!pred4x4_avail(&n4, m)) continue;
            pred4x4(&n4, m, p);
            for (int y = 0; y < 4; y++) for (int x = 0; x < 4; x++) d[4 * y + x] = src[(oy + y) * e->cw + ox + x] - p[4 * y + x];
            int c = satd4(d) + lam * (m == pm ? 1 : 4);
            if (best < 0 || c < bc) { best = m; bc = c; memcpy(bp, p, 16); }
        }
        cost4 += bc;
        if (cost4 >= c16) { won = 0; break; }
        t.i4mode[ras] = (int8_t)best;
        luma_block_levels(src + oy * e->cw + ox, e->cw, bp, 4, mb->qp, 1, 0, t.luma[ras]);
        int coef[16];
        dequant_block(t.luma[ras], mb->qp, 0, coef);
        idct4_add(coef, dst + oy * e->cw + ox, e->cw, bp, 4);
        t.nnz[ras] = (uint8_t)count_nz(t.luma[ras], 16);
    }
    if (won) {
        *mb = t;
        int cbp = 0;
        for (int i8 = 0; i8 < 4; i8++)
            for (int i4 = 0; i4 < 4; i4++) if (t.nnz[BLK2RAS[i8 * 4 + i4]]) cbp |= 1 << i8;
        mb->cbp = cbp;
    } else {
        encode_i16(e, mb, mbx, mby, m16, p16);
    }
    chroma_intra(e, mb, mbx, mby);
}

/* ---------------- P macroblocks ---------------- */
static int sad16_int(H264OEnc *e, int mbx, int mby, int mx, int my) {
    const uint8_t *src = e->src[0] + mby * 16 * e->cw + mbx * 16;
    int X = mbx * 16 + mx, Y = mby * 16 + my, s = 0;
    for (int y = 0; y < 16; y++) {
        int yy = clip3(0, e->ch - 1, Y + y);
        for (int x = 0; x < 16; x++) {
            int xx = clip3(0, e->cw - 1, X + x);
            s += iabs(src[y * e->cw + x] - e->ref[0][yy * e->cw + xx]);
        }
    }
    return s;
}
static int mvbits(int mx, int my, const int mvp[2]) { return se_len(mx - mvp[0]) + se_len(my - mvp[1]); }
static int subpel_cost(H264OEnc *e, int mbx, int mby, int mx, int my, const int mvp[2], int lam) {
    Pic rp = {e->ref[0], e->ref[1], e->ref[2], e->cw, e->ch, e->cw, e->cw / 2};
    uint8_t p[256];
    mc_luma(&rp, mbx * 16, mby * 16, 16, 16, mx, my, p, 16);
    return satd16x16(e->src[0] + mby * 16 * e->cw + mbx * 16, e->cw, p, 16) + lam * mvbits(mx, my, mvp);
}
/* Inter residual of the whole MB with prediction pl/pc; returns 1 if any level is nonzero. */
static int inter_levels(H264OEnc *e, MBInfo *mb, int mbx, int mby, const uint8_t pl[256], uint8_t pc[2][64]) {
    const uint8_t *src = e->src[0] + mby * 16 * e->cw + mbx * 16;
    int any = 0, cbp = 0;
    for (int ras = 0; ras < 16; ras++) {
        int ox = (ras & 3) * 4, oy = (ras >> 2) * 4;
        luma_block_levels(src + oy * e->cw + ox, e->cw, pl + oy * 16 + ox, 16, mb->qp, 0, 0, mb->luma[ras]);
        mb->nnz[ras] = (uint8_t)count_nz(mb->luma[ras], 16);
        if (mb->nnz[ras]) { any = 1; cbp |= 1 << (((ras >> 3) << 1) | ((ras & 3) >> 1)); }
    }
    mb->cbp = cbp;
    /* chroma levels + chroma reconstruction with this prediction */
    encode_chroma(e, mb, mbx, mby, pc, 0);
    if (mb->cbp >> 4) any = 1;
    return any;
}
static void encode_p_mb(H264OEnc *e, MBInfo *mb, int mbx, int mby) {
    int lam = LAMBDA[mb->qp];
    Pic rp = {e->ref[0], e->ref[1], e->ref[2], e->cw, e->ch, e->cw, e->cw / 2};
    int cs = e->cw / 2;
    uint8_t pl[256], pc[2][64];
    int skmv[2], mvp[2];
    pskip_mv(e->mbs, e->mbw, mbx, mby, skmv);
    mvp_16x16(e->mbs, e->mbw, mbx, mby, mvp);
    /* 1. P_Skip test: skip iff every quantised level at the skip MV is zero */
    mc_luma(&rp, mbx * 16, mby * 16, 16, 16, skmv[0], skmv[1], pl, 16);
    mc_chroma(e->ref[1], cs, e->ch / 2, cs, mbx * 8, mby * 8, 8, 8, skmv[0], skmv[1], pc[0], 8);
    mc_chroma(e->ref[2], cs, e->ch / 2, cs, mbx * 8, mby * 8, 8, 8, skmv[0], skmv[1], pc[1], 8);
    MBInfo t = *mb;
    if (!inter_levels(e, &t, mbx, mby, pl, pc)) {
        mb->type = MBT_PSKIP; mb->cbp = 0;
        memset(mb->nnz, 0, sizeof(mb->nnz));
        for (int i = 0; i < 16; i++) { mb->mv[i][0] = (int16_t)skmv[0]; mb->mv[i][1] = (int16_t)skmv[1]; mb->i4mode[i] = 2; }
        for (int i = 0; i < 4; i++) mb->ref[i] = 0;
        uint8_t *dst = e->rec[0] + mby * 16 * e->cw + mbx * 16;
        for (int y = 0; y < 16; y++) memcpy(dst + y * e->cw, pl + 16 * y, 16);
        /* chroma already reconstructed with zero residual == prediction */
        return;
    }
    /* 2. integer ME: start candidates {mvp, (0,0), A, B, C} (the MV predictors'
     * neighbours, integer-rounded), iterated small diamond, then -- when the match is still poor --
     * a cross search along the full horizontal and vertical lines through the best point */
    /* integer search range: +-16 pel around (0,0) */
    const int xmin = -16, xmax = 16, ymin = -16, ymax = 16;
    int cand[5][2], ncand = 0;
    cand[ncand][0] = (mvp[0] + 2) >> 2; cand[ncand][1] = (mvp[1] + 2) >> 2; ncand++;
    cand[ncand][0] = 0; cand[ncand][1] = 0; ncand++;
    {
        const MBInfo *nb[3] = {mbx > 0 ? &e->mbs[mby * e->mbw + mbx - 1] : NULL, mby > 0 ? &e->mbs[(mby - 1) * e->mbw + mbx] : NULL,
                               mby > 0 ? (mbx + 1 < e->mbw ? &e->mbs[(mby - 1) * e->mbw + mbx + 1]
                                                           : (mbx > 0 ? &e->mbs[(mby - 1) * e->mbw + mbx - 1] : NULL)) : NULL};
        for (int i = 0; i < 3; i++) {
            const MBInfo *m = nb[i];
            if (m && !mb_is_intra(m->type)) {
                cand[ncand][0] = (m->mv[0][0] + 2) >> 2; cand[ncand][1] = (m->mv[0][1] + 2) >> 2; ncand++;
            }
        }
    }
    int bx = 0, by = 0, bc = -1;
    for (int i = 0; i < ncand; i++) {
        int cx = clip3(xmin, xmax, cand[i][0]), cy = clip3(ymin, ymax, cand[i][1]);
        int c = sad16_int(e, mbx, mby, cx, cy) + lam * mvbits(4 * cx, 4 * cy, mvp);
        if (bc < 0 || c < bc) { bc = c; bx = cx; by = cy; if (i >= 2) e->stat_nb_start++; }
    }
    static const int DIA[4][2] = {{0, -1}, {-1, 0}, {1, 0}, {0, 1}};
    for (int it = 0; it < 32; it++) {
        int nb = -1, nx = 0, ny = 0;
        for (int k = 0; k < 4; k++) {
            int cx = bx + DIA[k][0], cy = by + DIA[k][1];
            if (cx < xmin || cx > xmax || cy < ymin || cy > ymax) continue;
            int c = sad16_int(e, mbx, mby, cx, cy) + lam * mvbits(4 * cx, 4 * cy, mvp);
            if (nb < 0 || c < nb) { nb = c; nx = cx; ny = cy; }
        }
        if (nb >= 0 && nb < bc) { bc = nb; bx = nx; by = ny; } else break;
    }
    if (bc > CROSS_THR) {  /* horizontal line (x ascending), then vertical line (y ascending) */
        int cbx = bx, cby = by, cbc = bc;
        for (int k = 0; k < 66; k++) {
            int cx = k < 33 ? xmin + k : bx, cy = k < 33 ? by : ymin + (k - 33);
            int c = sad16_int(e, mbx, mby, cx, cy) + lam * mvbits(4 * cx, 4 * cy, mvp);
            if (c < cbc) { cbc = c; cbx = cx; cby = cy; }
        }
        e->stat_cross++;
        if (cbx != bx || cby != by) e->stat_cross_moved++;
        bc = cbc; bx = cbx; by = cby;
    }
    /* 3. half then quarter refinement by SATD */
    static const int SUB[8][2] = {{0, -1}, {0, 1}, {-1, 0}, {1, 0}, {-1, -1}, {1, -1}, {-1, 1}, {1, 1}};
    int mx = 4 * bx, my = 4 * by;
    int sc = subpel_cost(e, mbx, mby, mx, my, mvp, lam);
    for (int step = 2; step >= 1; step--) {
        int cx0 = mx, cy0 = my;
        for (int k = 0; k < 8; k++) {
            int cx = cx0 + step * SUB[k][0], cy = cy0 + step * SUB[k][1];
            int c = subpel_cost(e, mbx, mby, cx, cy, mvp, lam);
            if (c < sc) { sc = c; mx = cx; my = cy; }
        }
    }
    /* 4. intra 16x16 alternative */
    IntraNb nb;
    get_nb16(e->rec[0], e->cw, mbx * 16, mby * 16, 16, mby > 0, mbx > 0, &nb);
    uint8_t p16[256];
    int c16;
    int m16 = i16_best(e, mbx, mby, &nb, &c16, p16);
    if (c16 + 6 * lam < sc) {
        for (int i = 0; i < 4; i++) mb->ref[i] = -1;
        for (int i = 0; i < 16; i++) mb->mv[i][0] = mb->mv[i][1] = 0;
        encode_i16(e, mb, mbx, mby, m16, p16);
        chroma_intra(e, mb, mbx, mby);
        return;
    }
    /* 5. P16x16 */
    mb->type = MBT_P16x16;
    for (int i = 0; i < 16; i++) { mb->mv[i][0] = (int16_t)mx; mb->mv[i][1] = (int16_t)my; mb->i4mode[i] = 2; }
    for (int i = 0; i < 4; i++) mb->ref[i] = 0;
    mb->mvd[0][0] = (int16_t)(mx - mvp[0]); mb->mvd[0][1] = (int16_t)(my - mvp[1]);
    mc_luma(&rp, mbx * 16, mby * 16, 16, 16, mx, my, pl, 16);
    mc_chroma(e->ref[1], cs, e->ch / 2, cs, mbx * 8, mby * 8, 8, 8, mx, my, pc[0], 8);
    mc_chroma(e->ref[2], cs, e->ch / 2, cs, mbx * 8, mby * 8, 8, 8, mx, my, pc[1], 8);
    inter_levels(e, mb, mbx, mby, pl, pc);
    uint8_t *dst = e->rec[0] + mby * 16 * e->cw + mbx * 16;
    for (int ras = 0; ras < 16; ras++) {
        int ox = (ras & 3) * 4, oy = (ras >> 2) * 4, coef[16];
        dequant_block(mb->luma[ras], mb->qp, 0, coef);
        idct4_add(coef, dst + oy * e->cw + ox, e->cw, pl + oy * 16 + ox, 16);
    }
}

/* ---------------- macroblock_layer() writer (7.3.5) ---------------- */
static int cbp_code(int cbp, int intra) {
    const uint8_t *t = intra ? CBP_INTRA_FROM_CODE : CBP_INTER_FROM_CODE;
    for (int i = 0; i < 48; i++) if (t[i] == cbp) return i;
    return 0;
}
static void write_residual(BW *b, H264OEnc *e, MBInfo *mb, int mbx, int mby) {
    int tot;
    if (mb->type == MBT_I16) {
        cavlc_write_block(b, mb->lumadc, 16, nc_luma(e->mbs, mb, e->mbw, mbx, mby, 0), &tot);
        if (mb->cbp & 15)
            for (int blk = 0; blk < 16; blk++) {
                int ras = BLK2RAS[blk];
                cavlc_write_block(b, mb->luma[ras] + 1, 15, nc_luma(e->mbs, mb, e->mbw, mbx, mby, ras), &tot);
            }
    } else {
        for (int i8 = 0; i8 < 4; i8++) {
            if (!(mb->cbp & (1 << i8))) continue;
            for (int i4 = 0; i4 < 4; i4++) {
                int ras = BLK2RAS[i8 * 4 + i4];
                cavlc_write_block(b, mb->luma[ras], 16, nc_luma(e->mbs, mb, e->mbw, mbx, mby, ras), &tot);
            }
        }
    }
    int cbpc = mb->cbp >> 4;
    if (cbpc) {
        for (int pl = 0; pl < 2; pl++) cavlc_write_block(b, mb->cdc[pl], 4, -1, &tot);
        if (cbpc == 2)
            for (int pl = 0; pl < 2; pl++)
                for (int blk = 0; blk < 4; blk++)
                    cavlc_write_block(b, mb->cac[pl][blk] + 1, 15, nc_chroma(e->mbs, mb, e->mbw, mbx, mby, pl, blk), &tot);
    }
}
static void write_mb(BW *b, H264OEnc *e, MBInfo *mb, int mbx, int mby, int pslice, int dqp) {
    int off = pslice ? 5 : 0;
    if (mb->type == MBT_I4) {
        bw_ue(b, off + 0);
        for (int blk = 0; blk < 16; blk++) {
            int ras = BLK2RAS[blk];
            int pm = i4_pred_mode(e->mbs, mb, e->mbw, mbx, mby, ras);
            int m = mb->i4mode[ras];
            if (m == pm) bw_put(b, 1, 1);
            else { bw_put(b, 0, 1); bw_put(b, m < pm ? m : m - 1, 3); }
        }
        bw_ue(b, mb->cmode);
        bw_ue(b, cbp_code(mb->cbp, 1));
        if (mb->cbp) bw_se(b, dqp);
    } else if (mb->type == MBT_I16) {
        bw_ue(b, off + 1 + mb->i16mode + 4 * (mb->cbp >> 4) + 12 * ((mb->cbp & 15) ? 1 : 0));
        bw_ue(b, mb->cmode);
        bw_se(b, dqp);
    } else { /* P16x16 */
        bw_ue(b, 0);
        bw_se(b, mb->mvd[0][0]);
        bw_se(b, mb->mvd[0][1]);
        bw_ue(b, cbp_code(mb->cbp, 0));
        if (mb->cbp) bw_se(b, dqp);
    }
    write_residual(b, e, mb, mbx, mby);
}

/* ---------------- public API ---------------- */
H264OEnc *h264o_enc_create(int w, int h, int bitrate) {
    if (w <= 0 || h <= 0 || (w & 1) || (h & 1)) return NULL;
    H264OEnc *e = (H264OEnc *)calloc(1, sizeof(H264OEnc));
    e->w = w; e->h = h; e->mbw = (w + 15) / 16; e->mbh = (h + 15) / 16;
    e->cw = e->mbw * 16; e->ch = e->mbh * 16;
    e->bitrate = bitrate;
    for (int p = 0; p < 3; p++) {
        size_t n = p ? (size_t)(e->cw / 2) * (e->ch / 2) : (size_t)e->cw * e->ch;
        e->src[p] = (uint8_t *)calloc(n, 1); e->rec[p] = (uint8_t *)calloc(n, 1); e->ref[p] = (uint8_t *)calloc(n, 1);
    }
    e->mbs = (MBInfo *)calloc((size_t)e->mbw * e->mbh, sizeof(MBInfo));
    e->rowqp = (int *)calloc((size_t)e->mbh, sizeof(int));
    e->rowbits = (int64_t *)calloc((size_t)e->mbh, sizeof(int64_t));
    e->first = 1;
    e->skip_en = 1;  /* the wrapper leaves OpenH264's frame skipping on (bEnableFrameSkip default) */
    e->init_qp = h264o_rc_idr_params(w, h, bitrate, &e->rmin, &e->rmax);
    e->qp = e->init_qp;
    e->idr_pic_id = 0;
    return e;
}
void h264o_enc_destroy(H264OEnc *e) {
    if (!e) return;
    for (int p = 0; p < 3; p++) { free(e->src[p]); free(e->rec[p]); free(e->ref[p]); }
    free(e->mbs); free(e->rowqp); free(e->rowbits); free(e);
}
void h264o_enc_set_frame_skip(H264OEnc *e, int enable) { if (e) e->skip_en = enable != 0; }
int h264o_enc_frames_skipped(const H264OEnc *e) { return e ? e->skipped : 0; }
void h264o_enc_me_stats(const H264OEnc *e, int32_t out[3]) {
    out[0] = e->stat_cross; out[1] = e->stat_cross_moved; out[2] = e->stat_nb_start;
}
void h264o_enc_force_idr(H264OEnc *e) { if (e) e->force_idr = 1; }
int h264o_enc_last_qp(const H264OEnc *e) { return e->last_qp; }

/* Source I420 (tight, w x h) -> coded-size planes with edge replication. */
static void load_source(H264OEnc *e, const uint8_t *yuv) {
    const uint8_t *pl[3] = {yuv, yuv + (size_t)e->w * e->h, yuv + (size_t)e->w * e->h + (size_t)(e->w / 2) * (e->h / 2)};
    for (int p = 0; p < 3; p++) {
        int sw = p ? e->w / 2 : e->w, sh = p ? e->h / 2 : e->h, dw = p ? e->cw / 2 : e->cw, dh = p ? e->ch / 2 : e->ch;
        for (int y = 0; y < dh; y++) {
            const uint8_t *s = pl[p] + (size_t)imin(y, sh - 1) * sw;
            uint8_t *d = e->src[p] + (size_t)y * dw;
            memcpy(d, s, sw);
            for (int x = sw; x < dw; x++) d[x] = s[sw - 1];
        }
    }
}

int h264o_enc_encode(H264OEnc *e, const uint8_t *yuv, uint8_t *out, int cap) {
    if (!e || !yuv || !out) return 0;
    int idr = e->first || e->force_idr;
    const int64_t T = e->bitrate / RC_FPS;
    /* frame skip: a non-IDR frame is dropped while the virtual buffer holds more
     * than half a second of bits; nothing else changes (reference, frame_num, POC, QP plan) */
    if (!idr && e->skip_en && e->vbuf > e->bitrate / 2) {
        e->vbuf = e->vbuf > T ? e->vbuf - T : 0;
        e->skipped++;
        return 0;
    }
    load_source(e, yuv);
    e->first = 0; e->force_idr = 0;
    /* uiIdrPicId (a uint16) is incremented before the IDR's parameter sets are written (func 589, file
     * offset 378895), so the first IDR carries 1 when the counter starts at 0 */
    if (idr) { e->frame_num = 0; e->poc = 0; e->idr_pic_id = (e->idr_pic_id + 1) & 0xffff; }
    int qp = rc_frame_qp(e, idr);
    size_t o = 0;
    uint8_t *tmp = (uint8_t *)malloc(64 + (size_t)e->cw * e->ch * 4);
    if (idr) { o += h264o_write_sps(e->w, e->h, e->bitrate, tmp + o); o += h264o_write_pps(tmp + o); }
    BW b; bw_init(&b);
    /* slice_header() 7.3.3 as OpenH264's WelsSliceHeaderWrite (func 1148) writes it with the fields its
     * slice init (func 225) and WelsUpdateRefSyntax (inlined in func 1017) set:
     * slice_type 2 (I) / 0 (P), without the +5; no POC field (type 2); a P slice overrides
     * num_ref_idx_l0_active (1) and reorders its list explicitly: modification_of_pic_nums_idc 0 with
     * abs_diff_pic_num_minus1 = frame_num - ref frame_num - 1 (0: skipped frames do not advance
     * frame_num), then 3; IDR marking {no_output_of_prior_pics 0, long_term_reference 0}, P marking
     * {adaptive_ref_pic_marking_mode 0}; deblocking idc 0 with zero offsets */
    bw_ue(&b, 0);
    bw_ue(&b, idr ? 2 : 0);
    bw_ue(&b, 0);
    bw_put(&b, (uint32_t)e->frame_num, LOG2_MAX_FRAME_NUM);
    if (idr) bw_ue(&b, (uint32_t)e->idr_pic_id);
    if (!idr) {
        bw_put(&b, 1, 1); bw_ue(&b, 0);                   /* num_ref_idx_active_override_flag, l0 active - 1 */
        bw_put(&b, 1, 1); bw_ue(&b, 0); bw_ue(&b, 0); bw_ue(&b, 3); /* ref_pic_list_modification_l0 */
        bw_put(&b, 0, 1);                                  /* adaptive_ref_pic_marking_mode_flag */
    } else {
        bw_put(&b, 0, 1); bw_put(&b, 0, 1);                /* no_output_of_prior_pics, long_term_reference */
    }
    bw_se(&b, qp - 26);
    bw_ue(&b, 0); bw_se(&b, 0); bw_se(&b, 0);
    /* slice_data(): each MB is decided and quantised at its row's QP; an MB that carries
     * mb_qp_delta (I16, or coded_block_pattern != 0) moves the running QP there; any other MB's
     * QPY is the running QP (7.4.5) */
    int skip_run = 0, running = qp;
    for (int mby = 0; mby < e->mbh; mby++) {
        const int qrow = clip3(e->qmin, e->qmax, qp + e->rowqp[mby]);
        e->rowbits[mby] = 0;
        for (int mbx = 0; mbx < e->mbw; mbx++) {
            MBInfo *mb = &e->mbs[mby * e->mbw + mbx];
            memset(mb, 0, sizeof(*mb));
            mb->qp = qrow;
            for (int i = 0; i < 16; i++) mb->i4mode[i] = 2;
            for (int i = 0; i < 4; i++) mb->ref[i] = -1;
            if (idr) encode_intra_mb(e, mb, mbx, mby);
            else encode_p_mb(e, mb, mbx, mby);
            const int carries = mb->type == MBT_I16 || (mb->type != MBT_PSKIP && mb->cbp != 0);
            const int dqp = carries ? qp_delta_wrap(qrow, running) : 0;
            if (carries) running = qrow;
            mb->qp = running;
            if (mb->type == MBT_PSKIP) { skip_run++; continue; }
            if (!idr) { bw_ue(&b, (uint32_t)skip_run); skip_run = 0; }
            const int64_t b0 = bw_bits(&b);
            write_mb(&b, e, mb, mbx, mby, !idr, dqp);
            e->rowbits[mby] += bw_bits(&b) - b0;
        }
    }
    if (skip_run) bw_ue(&b, (uint32_t)skip_run);
    bw_trailing(&b);
    o += nal_write(tmp + o, 3, idr ? 5 : 1, b.buf, b.len);
    bw_free(&b);
    /* loop filter on the reconstruction -> next reference */
    deblock_frame(e->rec[0], e->rec[1], e->rec[2], e->cw, e->cw / 2, e->mbs, e->mbw, e->mbh, 0);
    for (int p = 0; p < 3; p++) { uint8_t *t = e->ref[p]; e->ref[p] = e->rec[p]; e->rec[p] = t; }
    e->last_qp = qp; e->last_idr = idr;
    e->last_bits = (int64_t)o * 8;
    e->vbuf = e->vbuf + e->last_bits > T ? e->vbuf + e->last_bits - T : 0;
    e->qp = h264o_rc_next_qp(qp, e->last_bits, e->bitrate, idr);
    rc_plan_rows(e);
    e->frame_num = (e->frame_num + 1) & ((1 << LOG2_MAX_FRAME_NUM) - 1);
    e->poc += 2;
    int n = (int)o;
    if (n > cap) n = 0; else memcpy(out, tmp, o);
    free(tmp);
    return n;
}
/* Deblocked reconstruction of the last encoded frame, cropped tight I420. */
void h264o_enc_recon(const H264OEnc *e, uint8_t *out) {
    uint8_t *o = out;
    for (int y = 0; y < e->h; y++, o += e->w) memcpy(o, e->ref[0] + (size_t)y * e->cw, e->w);
    for (int p = 1; p < 3; p++)
        for (int y = 0; y < e->h / 2; y++, o += e->w / 2) memcpy(o, e->ref[p] + (size_t)y * (e->cw / 2), e->w / 2);
}
/* Per-MB decisions of the last frame: 8 int32 per MB {type, qp, cbp, mvx, mvy, i16mode, cmode, nnz_sum}. */
void h264o_enc_mbinfo(const H264OEnc *e, int32_t *out) {
    for (int i = 0; i < e->mbw * e->mbh; i++) {
        const MBInfo *m = &e->mbs[i];
        int s = 0; for (int k = 0; k < 24; k++) s += m->nnz[k];
        int32_t *r = out + 8 * i;
        r[0] = m->type; r[1] = m->qp; r[2] = m->cbp; r[3] = m->mv[0][0]; r[4] = m->mv[0][1];
        r[5] = m->i16mode; r[6] = m->cmode; r[7] = s;
    }
}
