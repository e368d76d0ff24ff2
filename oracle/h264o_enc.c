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
#define RC_VARY 10          /* iRcVaryPercentage = iRcVaryRatio (InitializeExt default, func 1021) */
#define FRAME_DQP_LOWER (RC_VARY / -100 + 3)  /* iFrameDeltaQpLower / Upper (RcInitSequenceParameter, func 592) */
#define FRAME_DQP_UPPER (RC_VARY / -50 + 5)
#define IDR_QP_WINDOW 3     /* RcCalculateIdrQp: the IDR's frame QP window (func 1226) */
#define VGOP_SIZE 8         /* RcInitVGop / RcInitTlWeight: iGopNumberInVGop = 8 >> iDecompositionStages */
#define WEIGHT_MULTIPLY 2000
/* intra mode decision (tools/wasm_tables.py CODE_CONSTANTS md_*) */
#define OH_VAA_I4_THRESHOLD 149  /* WelsMdIntraFinePartitionVaa: I4x4 tried when the VAA variance is above this */
#define OH_I4_MODE_BITS_SHIFT 2  /* a mode other than the predicted one costs lambda << 2 */
#define OH_I4_MB_OVERHEAD 24     /* the I4x4 MB costs its blocks + 24 lambda */
/* P_Skip judge (CODE_CONSTANTS pskip_*, TABLES single_ctr_run) */
#define OH_PSKIP_MV_MIN (-29)        /* WelsMdPSkipEnc: (mv >> 2) + 16 * MB position below this: no skip */
#define OH_PSKIP_MV_MAX_LOW 12       /* ... or above (16 * MBs) | this */
#define OH_PSKIP_MAX_LEVEL 1         /* a 4x4 block with a larger |level| rejects the skip */
#define OH_PSKIP_LUMA_CTR_MAX 5      /* the MB's summed single-coefficient cost of luma blocks: at most this */
#define OH_PSKIP_CHROMA_CTR_MAX 6    /* a chroma plane's: at most this */
/* Stream syntax OpenH264 writes at the wrapper's parameters, read from the same binary's code
 * (tools/wasm_tables.py CODE_CONSTANTS pins each instruction): WelsInitSps (func 280) stores
 * uiLog2MaxFrameNum 15 and uiPocType 2 as one i64 constant (sps_log2_max_frame_num_and_poc_type, 167923), so the slice header
 * carries a 15-bit frame_num and no POC; the level comes from the level limits at the 60 fps frame
 * rate and the target bitrate (level_idc_for below). */
#define LOG2_MAX_FRAME_NUM 15
#ifndef CROSS_THR
#define CROSS_THR 1024  /* cross search when the best integer cost exceeds this */
#endif

/* OpenH264's RC_BITRATE_MODE state at the wrapper's parameters (one spatial and one temporal layer, one
 * slice), restated from the reference's h264.wasm. Field comments name the wasm struct offsets the
 * functions below follow: rc+N = SWelsSvcRc (336 bytes per layer), tl+N = its SRCTemporal[0] (48 bytes),
 * sl+N = the slice's SRCSlicing; DESIGN.md §3.6 lists the functions. */
typedef struct {
    /* sequence (RcInitSequenceParameter inlined in func 592 @401199-401452; RcInitTlWeight func 702;
     * RcUpdateBitrateFps func 697) */
    int mbw, nmb, mb_per_gom, gom_count;  /* rc+156 iNumberMbFrame, rc+160 iNumberMbGom, rc+164 iGomSize */
    int skip_qp;            /* rc+188 iSkipQpValue */
    int bitrate, max_bitrate;
    int bpf, max_bpf;       /* rc+40 iBitsPerFrame, rc+44 iMaxBitsPerFrame */
    int min_bits_tl, max_bits_tl;  /* tl+0, tl+4 */
    int buffer_size_skip;   /* rc+228 */
    int tl_weight, gop_num; /* tl+8 iTlayerWeight, rc+180 iGopNumberInVGop */
    int skip_en;            /* param bEnableFrameSkip */
    /* frame skipping (func 589's check, CheckFrameSkipBasedMaxbr func 1258, WelsRcPostFrameSkipping func 1254) */
    int skip_flag;          /* rc+280 bSkipFlag */
    int continual_skip;     /* rc+284 iContinualSkipFrames */
    int skip_frame_num, skip_in_vgop;  /* rc+168, rc+176 */
    int64_t fullness;       /* rc+232 iBufferFullnessSkip */
    /* VGOP bit allocation (RcInitVGop, RcDecideTargetBits; func 1226) */
    int remaining;          /* rc+60 iRemainingBits */
    int vgop_bits;          /* rc+56: the VGOP's starting budget (bFixRCOverShoot) */
    int remaining_weights;  /* rc+112 */
    int gop_index;          /* rc+184 iGopIndexInVGop */
    int frame_coded_in_vgop;/* rc+172 */
    int gop_bits_dq;        /* tl+12 */
    int target;             /* rc+68 iTargetBits */
    int bits_level;         /* rc+72 iCurrentBitsLevel (2 = BITS_EXCEEDED) */
    /* QP (RcCalculateIdrQp / RcCalculatePictureQp, func 1226) */
    int init_qp;            /* rc+8 iInitialQp */
    int global_qp;          /* ctx+244 iGlobalQp: slice QP, the first GOM's QP */
    int last_qscale;        /* rc+224 iLastCalculatedQScale */
    int qstep;              /* rc+212 iQStep */
    int avg_qp;             /* rc+144 iAverageFrameQp */
    int min_frame_qp, max_frame_qp;  /* rc+148, rc+152 */
    /* R-Q models (RcUpdateIntraComplexity, RcUpdateFrameComplexity func 676) */
    int idr_num, intra_mb_count;     /* rc+76, rc+88 */
    int64_t intra_cmplx, intra_cmplx_mean;  /* rc+80, rc+96 */
    int pframe_num;                  /* tl+24 */
    int64_t linear_cmplx, frame_cmplx_mean;  /* tl+16, tl+32 */
    int64_t frame_cmplx;    /* the preprocessing's iFrameComplexity of the frame being coded (rc_complexity) */
    /* GOM (WelsRcMbInitGom func 1215, WelsRcMbInfoUpdateGom func 1206): exact mode only */
    int bits_per_mb;        /* rc+64 iBitsPerMb */
    int target_bits_slice, frame_bits_slice, gom_bits_slice, gom_target_bits;  /* sl+1372, +1380, +1384, +1388 */
    int complexity_index, calc_qp;   /* sl+1348 iComplexityIndexSlice, sl+1352 iCalculatedQpSlice */
    int total_qp, total_mb;          /* sl+1364, sl+1368 */
    uint32_t *gom_sad;      /* rc+132 pCurrentFrameGomSad: the frame's complexity per GOM */
    int mb_seen, last_coded; /* this frame's MBs counted so far, the last one with bits (-1: none) */
    int32_t *gom_trace;     /* per GOM of the last P frame {QP, slice bits before it, target bits, last coded MB + 1} */
} Rc;

struct H264OEnc {
    int w, h, mbw, mbh, cw, ch;
    int bitrate;
    uint8_t *src[3], *rec[3], *ref[3];
    uint8_t *prev_src;  /* luma source of the last coded frame, coded size (the preprocessing's reference picture) */
    MBInfo *mbs;
    int first, force_idr;
    int frame_num, idr_pic_id, poc;
    int last_qp, last_idr;
    Rc rc;
    int gom_exact;    /* MB QPs by OpenH264's GOM rule (h264o_enc_set_gom_exact); else this project's row plan */
    /* this project's MB-row QP plan of P frames */
    int *rowqp;       /* QP offset plan of the next frame, one per MB row (added to the frame QP) */
    int64_t *rowbits; /* macroblock_layer() bits per MB row of the last coded frame */
    int skipped, last_skipped;
    /* per MB, the P_Skip judge's memory (func 734): the skip SAD (luma + chroma SAD of the prediction at the skip
     * vector) of a skipped MB, -1 for any other; this frame's and the reference picture's (last coded frame) */
    int32_t *sksad_cur, *sksad_ref;
    int stat_cross, stat_cross_moved, stat_nb_start, stat_skip_tried, stat_skip_double, stat_intra_p;  /* ME path counters (tests: coverage of the search stages) */
};

/* ---------------- rate control ---------------- */
/* musl logf as h264.wasm func 483 computes it (RcConvertQStep2Qp's log): table-driven, in double, no FMA
 * (oracle/Makefile builds with -ffp-contract=off) */
float h264o_logf(float x) {
    uint32_t ix;
    memcpy(&ix, &x, 4);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x7f800000u <= 0x807fffffu) {  /* 0, subnormal, negative, inf, nan */
        if ((ix << 1) == 0) return -1.0f / 0.0f;
        if (ix == 0x7f800000u) return x;
        if (!((ix << 1) < 0xff000000u && (int32_t)ix >= 0)) return (x - x) / (x - x);
        const float xs = x * 8388608.0f;
        memcpy(&ix, &xs, 4);
        ix -= 192937984u;  /* 23 << 23 */
    }
    const uint32_t tmp = ix - 1060306944u;  /* 0x3f330000 */
    const int i = (int)((tmp >> 19) & 15), k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & 0xff800000u);
    float fz;
    memcpy(&fz, &iz, 4);
    const double r = (double)fz * OH_LOGF_T[i][0] + -1.0, r2 = r * r;
    return (float)(((OH_LOGF_P[1] * r2) + ((OH_LOGF_P[2] * r) + OH_LOGF_P[3])) * r2 +
                   ((((double)k * OH_LOGF_P[0]) + OH_LOGF_T[i][1]) + r));
}
/* RcConvertQStep2Qp (inlined twice in func 1226, 767413-767467 / 767927-767980): QP 0 below QStep 64,
 * else trunc(6 * logf(QStep / 100.0f) / ln 2 + 4 + 0.5) */
int h264o_rc_qstep2qp(int32_t qstep) {
    if (qstep < 64) return 0;
    const float t = h264o_logf((float)(uint32_t)qstep / 100.0f);
    return (int)((((double)(t * 6.0f)) / 0.6931471805599453 + 4.0) + 0.5);
}
/* bits per pixel class and column of RcCalculateIdrQp (func 1226, 766870-767222): the layer's size is the
 * picture rounded up to whole MBs (ParamTranscode, func 585, 373611-373776), bpp = bitrate / (float)(fps * w * h),
 * the first column at or above it from column 0 (bFixRCOverShoot) */
static void rc_idr_class(int w, int h, int bitrate, int *cls, int *col) {
    const int w16 = (w + 15) & ~15, h16 = (h + 15) & ~15;
    const float fps = (float)RC_FPS;
    const double bpp = (double)bitrate / (double)((fps * (float)w16) * (float)h16);
    const int area = w16 * h16;
    *cls = area < 28801 ? 0 : ((unsigned)area < 115201u ? 1 : ((unsigned)area < 460801u ? 2 : 3));
    int i = 0;
    while (i < 4 && !(OH_RC_BPP[*cls][i] >= bpp)) i++;
    *col = i;
}
/* the first IDR's QP and the IDR QP range {*rmin, *rmax} */
int h264o_rc_idr_params(int w, int h, int bitrate, int *rmin, int *rmax) {
    int cls, i;
    rc_idr_class(w, h, bitrate, &cls, &i);
    const int mx = clip3(QP_MIN, QP_MAX, OH_RC_QP_RANGE[i][0]), mn = clip3(QP_MIN, QP_MAX, OH_RC_QP_RANGE[i][1]);
    *rmin = mn; *rmax = mx;
    return clip3(mn, mx, OH_RC_INIT_QP[cls][i]);
}
int h264o_rc_init_qp(int w, int h, int bitrate) {
    int a, b;
    return h264o_rc_idr_params(w, h, bitrate, &a, &b);
}
/* RcInitSequenceParameter (func 592, 401199-401452) at creation; RcInitTlWeight / RcUpdateBitrateFps run at the
 * first IDR. The maximum bitrate is WelsBitRateVerification's (func 278): the caller leaves it unspecified and
 * uiLevelIdc unknown, so it becomes level 5.2's MaxBR x 1200. */
static void rc_init(Rc *rc, int w, int h, int bitrate) {
    uint32_t *g = rc->gom_sad;
    int32_t *gt = rc->gom_trace;
    memset(rc, 0, sizeof(*rc));
    const int w16 = (w + 15) & ~15, h16 = (h + 15) & ~15;
    rc->mbw = w16 >> 4;
    rc->nmb = rc->mbw * (h16 >> 4);
    const int narrow = rc->mbw < 31, g0 = narrow ? 1 : 2, g1 = narrow ? 2 : 4;
    rc->skip_qp = narrow ? 24 : 31;
    rc->mb_per_gom = rc->mbw * ((RC_VARY * (g1 - g0)) / 100 + g0);
    rc->gom_count = (rc->mb_per_gom + rc->nmb - 1) / rc->mb_per_gom;
    rc->bitrate = bitrate;
    rc->max_bitrate = 0;
    for (int i = 0; i < 17; i++) if (OH_LEVEL_LIMITS[i][0] == 52) rc->max_bitrate = OH_LEVEL_LIMITS[i][4] * 1200;
    rc->skip_en = 1;
    rc->gom_sad = g;
    rc->gom_trace = gt;
}
/* RcUpdateBitrateFps (func 697): float per-frame bits at the 60 fps default, the temporal layer's bit bounds
 * (55 % / 150 % of the GOP's bits at iRcVaryRatio 10, weighted), the skip buffer (50 % of the bitrate) */
static void rc_update_bitrate_fps(Rc *rc) {
    const float fps = (float)RC_FPS;
    const int in_bpf = (int)((fps * 0.5f + (float)rc->bitrate) / fps);
    const int64_t gop_bits = in_bpf;  /* << iDecompositionStages (0) */
    rc->max_bits_tl = (int)((gop_bits * 150 * rc->tl_weight + 100000) / 200000);
    rc->min_bits_tl = (int)((gop_bits * (100 - ((100 - RC_VARY) >> 1)) * rc->tl_weight + 100000) / 200000);
    rc->buffer_size_skip = (int)((50 * (int64_t)rc->bitrate + 50) / 100);
    if (rc->bpf >= 2)
        rc->remaining = (int)(((int64_t)((uint32_t)rc->bpf >> 1) + (int64_t)rc->remaining * in_bpf) / (int64_t)(uint32_t)rc->bpf);
    rc->bpf = in_bpf;
    rc->max_bpf = (int)((fps * 0.5f + (float)rc->max_bitrate) / fps);
}
/* RcInitVGop with bFixRCOverShoot (func 1226, 764341-764437 / 765012-765094 / 765431-765497): an overspent VGOP
 * carries its deficit into the next, an underspent one does not carry its surplus */
static void rc_init_vgop(Rc *rc) {
    const int t = rc->remaining + (rc->gop_index - rc->gop_num) * (rc->vgop_bits / rc->gop_num);
    rc->remaining = (t < 0 ? t : 0) + (rc->bpf << 3);
    rc->vgop_bits = rc->remaining;
    rc->gop_index = 0;
    rc->frame_coded_in_vgop = 0;
    rc->remaining_weights = rc->gop_num * WEIGHT_MULTIPLY;
    rc->gop_bits_dq = 0;
    rc->skip_in_vgop = 0;
}
static int64_t cmplx_ratio(int64_t fc, int64_t mean) {  /* WELS_DIV_ROUND64(fc * 100, mean) clipped to 80..120 */
    int64_t r = mean == 0 ? fc * 100 : (fc * 100 + mean / 2) / mean;
    r = r <= 80 ? 80 : r;
    return r >= 120 ? 120 : r;
}
static int32_t qstep_model(int64_t cmplx, int64_t ratio, int target) {  /* WELS_DIV_ROUND64(cmplx * ratio, target * 100) */
    const int64_t v = target == 0 ? cmplx * ratio : ((int64_t)(target * 50) + cmplx * ratio) / (int64_t)(target * 100);
    return (int32_t)(uint32_t)(uint64_t)v;
}
/* Frame skip decision before a frame (WelsEncoderEncodeExt's check, func 589 376000-376503): a flag left by the
 * last update skips at once; otherwise CheckFrameSkipBasedMaxbr (func 1258) skips while the buffer holds more than
 * its size and the run of skipped frames is at most (round(fullness / bits per frame) + 1) >> 1. Its three
 * maximum-bitrate cases need iCheckWindowInterval > 2500 ms, which the wrapper's zero timestamps never reach
 * (UpdateMaxBrCheckWindowStatus, func 1251). bFixRCOverShoot: 1258 only sets the flag (774599-774612).
 * Returns 1 when the frame is skipped unless it is an IDR. */
static int rc_judge_skip(Rc *rc) {
    if (!rc->skip_flag) {
        if (!rc->skip_en) return 0;
        const int64_t r = rc->bpf == 0 ? rc->fullness : (rc->fullness + rc->bpf / 2) / rc->bpf;
        const int pred_tar = ((int32_t)(uint32_t)(uint64_t)r + 1) >> 1;
        rc->skip_flag = pred_tar >= rc->continual_skip && rc->fullness > rc->buffer_size_skip;
        if (!rc->skip_flag) return 0;
    }
    rc->skip_flag = 0;
    rc->continual_skip++;
    return 1;
}
/* WelsRcPostFrameSkipping (func 1254): the skipped frame's bits leave the buffer and return to the VGOP */
static void rc_post_skip(Rc *rc) {
    rc->fullness -= rc->bpf;
    rc->remaining += rc->bpf;
    rc->skip_frame_num++;
    rc->skip_in_vgop++;
    if (rc->fullness < 0) rc->fullness = 0;
}
/* WelsRcPictureInitGom (func 1226) for a coded frame: RcInitRefreshParameter at the first IDR, RcUpdateTemporalZero,
 * RcDecideTargetBits, RcCalculateIdrQp / RcCalculatePictureQp, RcInitSliceInformation, RcInitGomParameters and the
 * slice's RC init (func 225, 120355-120428). rc->frame_cmplx holds the frame's complexity. */
static void rc_picture_init(Rc *rc, int idr, int w, int h) {
    rc->continual_skip = 0;
    if (idr && rc->idr_num == 0) {  /* RcInitRefreshParameter (763796-764694) */
        rc->intra_cmplx = 0; rc->intra_mb_count = 0; rc->intra_cmplx_mean = 0;
        rc->pframe_num = 0; rc->linear_cmplx = 0; rc->frame_cmplx_mean = 0;
        rc->fullness = 0; rc->gop_index = 0; rc->vgop_bits = 0;
        rc->bpf = 0; rc->remaining = 0;
        rc->tl_weight = OH_RC_TL_WEIGHT[0][0];  /* RcInitTlWeight: one temporal layer, decomposition stages 0 */
        rc->gop_num = VGOP_SIZE >> 0;
        rc_update_bitrate_fps(rc);
        rc_init_vgop(rc);
    }
    /* RcUpdateTemporalZero (764840-765777): a new VGOP after iGopNumberInVGop frames and at every IDR */
    if (rc->gop_index == rc->gop_num || idr) rc_init_vgop(rc);
    rc->gop_index++;
    /* RcDecideTargetBits (766402-766725) */
    rc->bits_level = 0;
    if (idr) rc->target = rc->idr_num ? 400 * rc->bpf / 100 : rc->bpf << 2;  /* iIdrBitrateRatio 400 % */
    else {
        const int rw = rc->remaining_weights, wt = rc->tl_weight;
        int tb;
        if (rw >= wt)  /* rw == wt divides too: bFixRCOverShoot */
            tb = rw == 0 ? (int)(uint32_t)((uint64_t)(uint32_t)rc->remaining * (uint64_t)(uint32_t)wt)
                         : (int)(((int64_t)(rw / 2) + (int64_t)rc->remaining * wt) / rw);
        else tb = rc->remaining;
        if (tb <= 0 && !rc->skip_en) rc->bits_level = 2;
        rc->target = clip3(rc->min_bits_tl, rc->max_bits_tl, tb);
    }
    rc->remaining_weights -= rc->tl_weight;
    if (idr) {  /* RcCalculateIdrQp (766790-767604) */
        int cls, i;
        rc_idr_class(w, h, rc->bitrate, &cls, &i);
        const int lo = clip3(QP_MIN, QP_MAX, OH_RC_QP_RANGE[i][1]), hi = clip3(QP_MIN, QP_MAX, OH_RC_QP_RANGE[i][0]);
        int q;
        if (rc->idr_num == 0) q = OH_RC_INIT_QP[cls][i];
        else {
            if (rc->nmb != rc->intra_mb_count) rc->intra_cmplx = rc->intra_cmplx * rc->nmb / rc->intra_mb_count;
            q = h264o_rc_qstep2qp(qstep_model(rc->intra_cmplx, cmplx_ratio(rc->frame_cmplx, rc->intra_cmplx_mean), rc->target));
        }
        q = clip3(lo, hi, q);
        rc->init_qp = q; rc->global_qp = q; rc->last_qscale = q; rc->qstep = OH_RC_QSTEP[q];
        rc->max_frame_qp = clip3(lo, hi, q + IDR_QP_WINDOW);
        rc->min_frame_qp = clip3(lo, hi, q - IDR_QP_WINDOW);
    } else {    /* RcCalculatePictureQp (767612-768334); one temporal layer: no temporal QP delta */
        int q;
        if (rc->pframe_num == 0) q = rc->init_qp;
        else if (rc->bits_level == 2) q = rc->last_qscale + 3;
        else {
            rc->qstep = qstep_model(rc->linear_cmplx, cmplx_ratio(rc->frame_cmplx, rc->frame_cmplx_mean), rc->target);
            q = h264o_rc_qstep2qp(rc->qstep);
        }
        rc->min_frame_qp = clip3(QP_MIN, QP_MAX, rc->last_qscale - FRAME_DQP_LOWER);
        rc->max_frame_qp = clip3(QP_MIN, QP_MAX, rc->last_qscale + FRAME_DQP_UPPER);
        q = clip3(rc->min_frame_qp, rc->max_frame_qp, q);
        rc->last_qscale = q; rc->qstep = OH_RC_QSTEP[q]; rc->global_qp = q;
    }
    /* RcInitSliceInformation / RcInitGomParameters (768342-769173), the slice's RC init (func 225) */
    rc->bits_per_mb = (int)(uint32_t)(uint64_t)(rc->nmb == 0 ? (int64_t)rc->target * 100
                                                            : ((int64_t)(rc->nmb / 2) + (int64_t)rc->target * 100) / rc->nmb);
    rc->avg_qp = 0;
    rc->complexity_index = 0;
    rc->calc_qp = rc->global_qp;
    rc->total_qp = rc->total_mb = 0;
    rc->frame_bits_slice = rc->gom_bits_slice = rc->gom_target_bits = 0;
    rc->mb_seen = 0; rc->last_coded = -1;
    rc->target_bits_slice = (int)(uint32_t)(uint64_t)(((int64_t)rc->nmb * rc->bits_per_mb + 50) / 100);
}
/* WelsRcMbInitGom (func 1215) in exact-GOM mode: at the first MB of every GOM after the first, RcCalculateGomQp
 * moves the QP by the slice's bits so far against the GOM targets (+2 / +1 / -1 at bit ratios 0.8409 / 0.9439 /
 * 1.06; its -2 branch is unreachable), clipped to the frame's window; then RcGomTargetBits shares the remaining
 * bits over the GOMs left by their complexity. Returns the MB's QP. I slices (bEnableGomQp 0 in RC_BITRATE_MODE,
 * 766730-766775): the frame QP. */
static int rc_mb_init_gom(Rc *rc, int mb, int idr) {
    if (idr) return rc->global_qp;
    if (mb % rc->mb_per_gom == 0) {
        if (mb != 0) {  /* iStartMbSlice 0 */
            rc->complexity_index++;
            int d = 2;
            const int left = rc->target_bits_slice - rc->frame_bits_slice;
            if (left > 0) {
                const int64_t tleft = (int64_t)left + rc->gom_bits_slice - rc->gom_target_bits;
                if (tleft > 0) {
                    const uint64_t ratio = (uint64_t)((int64_t)left * 10000) / (uint64_t)(tleft + 1);
                    if (ratio >= 8409) d = ratio < 9439 ? 1 : -(ratio > 10600);
                }
            }
            rc->calc_qp = clip3(rc->min_frame_qp, rc->max_frame_qp, rc->calc_qp + d);
            rc->gom_bits_slice = 0;
        }
        /* RcGomTargetBits (759693-760199) */
        const int last = (rc->nmb - 1) / rc->mb_per_gom, k = rc->complexity_index;
        int left = rc->target_bits_slice - rc->frame_bits_slice;
        if (left <= 0) left = 0;
        else if (last > k) {
            int sum = 0;
            for (int i = k + 1; i <= last; i++) sum += (int)rc->gom_sad[i];
            if (sum == 0) left = (left + (last - k) / 2) / (last - k);
            else left = (int)(uint32_t)(uint64_t)(((int64_t)(sum / 2) + (int64_t)(int32_t)rc->gom_sad[k + 1] * (int64_t)(uint32_t)left) / sum);
        }
        rc->gom_target_bits = left;
        int32_t *t = rc->gom_trace + 4 * k;
        t[0] = rc->calc_qp; t[1] = rc->frame_bits_slice; t[2] = left; t[3] = rc->last_coded + 1;
    }
    return rc->calc_qp;
}
/* WelsRcMbInfoUpdateGom (func 1206): the MB's bits (its mb_skip_run code included) and, when it has any, its QP */
static void rc_mb_update(Rc *rc, int bits, int qp) {
    rc->frame_bits_slice += bits;
    rc->gom_bits_slice += bits;
    if (bits > 0) { rc->total_qp += qp; rc->total_mb++; rc->last_coded = rc->mb_seen; }
    rc->mb_seen++;
}
/* WelsRcPictureInfoUpdateGom (func 1218) after a coded frame: slice_bytes = the slice NAL (start code and
 * emulation prevention included; the parameter sets are another layer). RcUpdatePictureQpBits, the R-Q model
 * (RcUpdateFrameComplexity func 676 / RcUpdateIntraComplexity), the VGOP budget and RcVBufferCalculationSkip. */
static void rc_picture_update(Rc *rc, int idr, int slice_bytes) {
    const int bits = slice_bytes << 3;
    const int avg = (!idr && rc->total_mb > 0) ? (rc->total_mb * 50 + rc->total_qp * 100) / (rc->total_mb * 100) : rc->global_qp;
    rc->last_qscale = avg;
    rc->avg_qp = avg;
    rc->gop_bits_dq += bits;
    if (!idr) {
        const int q = OH_RC_QSTEP[avg];
        if (rc->pframe_num == 0) {
            rc->frame_cmplx_mean = (int64_t)(int32_t)(uint32_t)(uint64_t)rc->frame_cmplx;
            rc->linear_cmplx = (int64_t)bits * q;
        } else {
            rc->frame_cmplx_mean = (rc->frame_cmplx * 20 + rc->frame_cmplx_mean * 80 + 50) / 100;
            rc->linear_cmplx = (rc->linear_cmplx * 80 + (int64_t)q * bits * 20 + 50) / 100;
        }
        rc->pframe_num = (rc->pframe_num >= 254 ? 254 : rc->pframe_num) + 1;
    } else {
        const int64_t ic = (int64_t)OH_RC_QSTEP[avg] * bits;
        if (rc->idr_num == 0) { rc->intra_cmplx_mean = rc->frame_cmplx; rc->intra_cmplx = ic; }
        else {
            rc->intra_cmplx = (ic * 20 + rc->intra_cmplx * 80 + 50) / 100;
            rc->intra_cmplx_mean = (rc->frame_cmplx * 20 + rc->intra_cmplx_mean * 80 + 50) / 100;
        }
        rc->intra_mb_count = rc->nmb;
        rc->idr_num = (rc->idr_num >= 254 ? 254 : rc->idr_num) + 1;
    }
    rc->remaining -= bits;
    if (rc->skip_en) {  /* RcVBufferCalculationSkip (761104-761644) */
        rc->fullness += bits - rc->bpf;
        int64_t pred = 0;
        if (rc->frame_coded_in_vgop <= 6)
            for (int i = rc->frame_coded_in_vgop + 1; i < VGOP_SIZE; i++) pred += rc->min_bits_tl;
        const double inc = ((double)(pred - rc->remaining) * 100.0) / (double)(rc->bpf << 3) + -5.0;
        if ((rc->fullness > rc->buffer_size_skip && rc->avg_qp > rc->skip_qp) || inc > (double)RC_VARY) rc->skip_flag = 1;
    }
    rc->frame_coded_in_vgop++;
}
/* The preprocessing's frame complexity (AnalyzeSpatialPic -> CComplexityAnalysis::Process, func 910) over the
 * coded-size luma picture, one value per GOM of mb_per_gom MBs (written to gom_sad), the frame's = their uint32
 * sum. P (GOM_SAD, GomSampleSad func 909): the four 8x8 SADs (VAACalcSad) of every MB against the last coded
 * frame's source. I (GOM_VAR, VAACalcSadVar): per GOM, uint32 square sum - (uint32 sum)^2 / (MBs of the GOM's
 * first row x 256). */
static int64_t rc_complexity(Rc *rc, const uint8_t *cur, const uint8_t *ref, int stride, int idr) {
    const int mbw = rc->mbw, nmb = rc->nmb;
    uint32_t frame = 0;
    for (int j = 0; j < rc->gom_count; j++) {
        const int start = j * rc->mb_per_gom, end = imin((j + 1) * rc->mb_per_gom, nmb);
        uint32_t sad = 0, sum = 0, sq = 0;
        for (int m = start; m < end; m++) {
            const uint8_t *c = cur + (size_t)(m / mbw) * 16 * stride + (m % mbw) * 16;
            const uint8_t *r = ref + (size_t)(m / mbw) * 16 * stride + (m % mbw) * 16;
            for (int y = 0; y < 16; y++)
                for (int x = 0; x < 16; x++) {
                    const int a = c[y * stride + x], b = r[y * stride + x];
                    sad += (uint32_t)(a > b ? a - b : b - a);
                    sum += (uint32_t)a;
                    sq += (uint32_t)(a * a);
                }
        }
        const uint32_t first_row = (uint32_t)(imin((start / mbw + 1) * mbw, end) - start);
        const uint32_t v = idr ? sq - (sum * sum) / (first_row << 8) : sad;
        rc->gom_sad[j] = v;
        frame += v;
    }
    return (int64_t)frame;
}
/* this project's MB-row QP plan for P frames: rows that cost more than the mean in the last coded
 * frame are quantised more coarsely, cheaper rows more finely, inside the frame's window */
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
/* the intra mode decision's constants for tests/test_oracle_golden.py: {VAA threshold, mode bits shift, I4x4 MB
 * overhead} (pinned against the h264.wasm fixture, tools/wasm_tables.py md_*) */
/* the P_Skip judge's constants (tests check them against the binary's instructions) */
void h264o_pskip_constants(int32_t out[5]) {
    out[0] = OH_PSKIP_MV_MIN; out[1] = OH_PSKIP_MV_MAX_LOW; out[2] = OH_PSKIP_MAX_LEVEL;
    out[3] = OH_PSKIP_LUMA_CTR_MAX; out[4] = OH_PSKIP_CHROMA_CTR_MAX;
}
void h264o_md_constants(int32_t out[3]) {
    out[0] = OH_VAA_I4_THRESHOLD; out[1] = OH_I4_MODE_BITS_SHIFT; out[2] = OH_I4_MB_OVERHEAD;
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
    else if (!strcmp(name, "logf_table")) { for (int i = 0; i < 32; i++) out[n++] = OH_LOGF_T[i / 2][i % 2]; }
    else if (!strcmp(name, "logf_poly")) { for (int i = 0; i < 4; i++) out[n++] = OH_LOGF_P[i]; }
    else if (!strcmp(name, "rc_tl_weight")) { for (int i = 0; i < 16; i++) out[n++] = OH_RC_TL_WEIGHT[i / 4][i % 4]; }
    else if (!strcmp(name, "i16_avail_modes")) { for (int i = 0; i < 40; i++) out[n++] = OH_I16_AVAIL[i / 5][i % 5]; }
    else if (!strcmp(name, "i16_mode_map")) { for (int i = 0; i < 7; i++) out[n++] = OH_I16_MAP[i]; }
    else if (!strcmp(name, "chroma_avail_modes")) { for (int i = 0; i < 40; i++) out[n++] = OH_CHROMA_AVAIL[i / 5][i % 5]; }
    else if (!strcmp(name, "chroma_mode_map")) { for (int i = 0; i < 7; i++) out[n++] = OH_CHROMA_MAP[i]; }
    else if (!strcmp(name, "i4_avail_index")) { for (int i = 0; i < 256; i++) out[n++] = OH_I4_AVAIL_IDX[i / 16][i % 16]; }
    else if (!strcmp(name, "i4_avail_count")) { for (int i = 0; i < 16; i++) out[n++] = OH_I4_COUNT[i]; }
    else if (!strcmp(name, "i4_avail_modes")) { for (int i = 0; i < 256; i++) out[n++] = OH_I4_MODES[i / 16][i % 16]; }
    else if (!strcmp(name, "i4_mode_map")) { for (int i = 0; i < 16; i++) out[n++] = OH_I4_MAP[i]; }
    else if (!strcmp(name, "level_limits")) { for (int i = 0; i < 17 * 6; i++) out[n++] = OH_LEVEL_LIMITS[i / 6][i % 6]; }
    else if (!strcmp(name, "single_ctr_run")) { for (int i = 0; i < 16; i++) out[n++] = OH_SINGLE_CTR[i]; }
    else if (!strcmp(name, "chroma_qp")) { for (int i = 0; i < 52; i++) out[n++] = CHROMA_QP[i]; }
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
/* sum of absolute differences of a w x h block (pfSampleSad: the mode decision's cost at the wrapper's settings) */
static int sad_blk(const uint8_t *src, int ss, const uint8_t *pred, int ps, int w, int h) {
    int s = 0;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) s += iabs(src[y * ss + x] - pred[y * ps + x]);
    return s;
}
/* bits of ue(v) (BsSizeUE) */
static int ue_bits(int v) { int n = 0; while (((unsigned)v + 1) >> (n + 1)) n++; return 2 * n + 1; }
/* the MB's neighbour flags as OpenH264's MB cache holds them (one slice per picture): 1 left, 2 top, 4 top-left,
 * 8 top-right (uiNeighborAvail, func 246 125527) */
static int mb_nb_flags(int mbx, int mby, int mbw) {
    return (mbx > 0) | ((mby > 0) << 1) | ((mbx > 0 && mby > 0) << 2) | ((mby > 0 && mbx + 1 < mbw) << 3);
}
/* WelsMdIntraChroma (h264.wasm func 312) with pfMdCost = SAD: the modes of OH_CHROMA_AVAIL[flags & 7]
 * in that order, cost = SAD(Cb) + SAD(Cr) + lambda * ue bits of the syntax mode, the first minimum wins (strict <).
 * The internal DC_L / DC_T / DC_128 modes are the standard's DC for those neighbours. */
static int best_chroma_mode(H264OEnc *e, int mbx, int mby, IntraNb nb[2], uint8_t pred[2][64], int lam) {
    const int cs = e->cw / 2;
    const int8_t *row = OH_CHROMA_AVAIL[mb_nb_flags(mbx, mby, e->mbw) & 7];
    int best = 0x7fffffff, bm = OH_CHROMA_MAP[row[0]];
    uint8_t p[2][64];
    for (int i = 0; i < row[4]; i++) {
        const int m = OH_CHROMA_MAP[row[i]];
        int c = lam * ue_bits(m);
        for (int pl = 0; pl < 2; pl++) {
            pred_chroma(&nb[pl], m, p[pl]);
            c += sad_blk(e->src[1 + pl] + mby * 8 * cs + mbx * 8, cs, p[pl], 8, 8, 8);
        }
        if (c < best) { best = c; bm = m; memcpy(pred, p, sizeof(p)); }
    }
    return bm;
}
static void chroma_intra(H264OEnc *e, MBInfo *mb, int mbx, int mby) {
    IntraNb nb[2];
    int cs = e->cw / 2;
    for (int pl = 0; pl < 2; pl++) get_nb16(e->rec[1 + pl], cs, mbx * 8, mby * 8, 8, mby > 0, mbx > 0, &nb[pl]);
    uint8_t pred[2][64];
    mb->cmode = best_chroma_mode(e, mbx, mby, nb, pred, LAMBDA[mb->qp]);
    encode_chroma(e, mb, mbx, mby, pred, 1);
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

/* WelsMdI16x16 (h264.wasm func 313) with pfMdCost = SAD: the modes of OH_I16_AVAIL[flags & 7] in that order, cost
 * = SAD + lambda * ue bits of the syntax mode, the first minimum wins. Returns the syntax mode. */
static int i16_best_oh(H264OEnc *e, int mbx, int mby, const IntraNb *nb, int lam, int *cost, uint8_t pred[256]) {
    const uint8_t *src = e->src[0] + mby * 16 * e->cw + mbx * 16;
    const int8_t *row = OH_I16_AVAIL[mb_nb_flags(mbx, mby, e->mbw) & 7];
    int best = 0x7fffffff, bm = OH_I16_MAP[row[0]];
    uint8_t p[256];
    for (int i = 0; i < row[4]; i++) {
        const int m = OH_I16_MAP[row[i]];
        pred16x16(nb, m, p);
        const int c = sad_blk(src, e->cw, p, 16, 16, 16) + lam * ue_bits(m);
        if (c < best) { best = c; bm = m; memcpy(pred, p, 256); }
    }
    *cost = best;
    return bm;
}
/* AnalysisVaaInfoIntra (func 854): the variance of the source MB's sixteen 4x4 means (sum >> 4),
 * sum of squares - (sum^2 >> 4) */
int h264o_vaa_intra_var(const uint8_t *src, int ss) {
    uint32_t sum = 0, sq = 0;
    for (int by = 0; by < 4; by++)
        for (int bx = 0; bx < 4; bx++) {
            uint32_t t = 0;
            for (int y = 0; y < 4; y++) for (int x = 0; x < 4; x++) t += src[(4 * by + y) * ss + 4 * bx + x];
            t = (t & 0xfff0u) >> 4;
            sum += t; sq += t * t;
        }
    return (int)(sq - ((sum * sum) >> 4));
}
/* WelsMdI4x4Fast's choice for one block (inlined in func 774, 475164-476768): c[m] = SAD + (m == predicted mode ?
 * lambda : 4 lambda) for syntax mode m. Blocks whose availability gives 7 or 9 modes take the fast search -- DC, H
 * and V first, then the directional modes beside the better of V / H -- the others try their modes in the table's
 * order; the first minimum wins everywhere (strict <). Returns the mode, *cost its cost. */
int h264o_i4_choose(const int c[9], int avail_index, int *cost) {
    const int cnt = OH_I4_COUNT[avail_index];
    int best, m;
    if (cnt == 7 || cnt == 9) {
        const int hb = c[1] < c[2];
        best = hb ? c[1] : c[2]; m = hb ? 1 : 2;
        if (c[0] < best) { best = c[0]; m = 0; }
        if (c[0] < c[1]) {
            if (cnt == 9) {
                if (c[5] < best) { best = c[5]; m = 5; }
                if (best > c[7]) { best = c[7]; m = 7; }
                if (!(c[0] <= c[7] && c[0] <= c[5])) {
                    if (c[5] < c[7]) { if (c[4] < best) { best = c[4]; m = 4; } }
                    else if (c[3] < best) { best = c[3]; m = 3; }
                }
            } else {
                if (c[4] < best) { best = c[4]; m = 4; }
                if (c[5] < best) { best = c[5]; m = 5; }
            }
        } else {
            if (c[6] < best) { best = c[6]; m = 6; }
            if (best > c[8]) { best = c[8]; m = 8; }
            if (!(c[6] >= c[1] && c[8] >= c[1])) {
                if (c[8] > c[6]) { if (c[4] < best) { best = c[4]; m = 4; } }
                else if (cnt == 9 && c[3] < best) { best = c[3]; m = 3; }
            }
        }
    } else {
        best = 0x7fffffff; m = 2;
        for (int i = 0; i < cnt; i++) {
            const int mm = OH_I4_MAP[OH_I4_MODES[avail_index][i]];
            if (c[mm] < best) { best = c[mm]; m = mm; }
        }
    }
    *cost = best;
    return m;
}
/* WelsMdIntraMb (func 439) for I slices: I16x16 (func 313), then -- WelsMdIntraFinePartitionVaa, func 774 -- the
 * Intra4x4 search only when the source MB's VAA variance is above 149: blocks in decoding order, each coded and
 * reconstructed as chosen (the next block predicts from it), the search stops as soon as the blocks' cost reaches
 * the I16x16 cost, and I4x4 wins when its blocks + 24 lambda cost less. */
static void encode_intra_mb(H264OEnc *e, MBInfo *mb, int mbx, int mby) {
    int lam = LAMBDA[mb->qp];
    IntraNb nb;
    get_nb16(e->rec[0], e->cw, mbx * 16, mby * 16, 16, mby > 0, mbx > 0, &nb);
    uint8_t p16[256];
    int c16;
    int m16 = i16_best_oh(e, mbx, mby, &nb, lam, &c16, p16);
    MBInfo t = *mb;
    t.type = MBT_I4;
    const uint8_t *src = e->src[0] + mby * 16 * e->cw + mbx * 16;
    uint8_t *dst = e->rec[0] + mby * 16 * e->cw + mbx * 16;
    const int flags = mb_nb_flags(mbx, mby, e->mbw);
    int won = 0;
    if (h264o_vaa_intra_var(src, e->cw) > OH_VAA_I4_THRESHOLD) {
        int sum = 0;
        won = 1;
        for (int blk = 0; blk < 16; blk++) {
            int ras = BLK2RAS[blk], ox = (ras & 3) * 4, oy = (ras >> 2) * 4;
            IntraNb n4;
            get_nb4(e->rec[0], e->cw, mbx, mby, e->mbw, ras, &n4);
            const int pm = i4_pred_mode(e->mbs, &t, e->mbw, mbx, mby, ras);
            const int ai = OH_I4_AVAIL_IDX[flags][blk];
            int c[9];
            uint8_t p[16];
            for (int m = 0; m < 9; m++) {
                c[m] = 0x7fffffff;
                if (!pred4x4_avail(&n4, m)) continue;
                pred4x4(&n4, m, p);
                c[m] = sad_blk(src + oy * e->cw + ox, e->cw, p, 4, 4, 4) + (m == pm ? lam : lam << OH_I4_MODE_BITS_SHIFT);
            }
            int bc;
            const int best = h264o_i4_choose(c, ai, &bc);
            sum += bc;
            if (sum >= c16) { won = 0; break; }
            pred4x4(&n4, best, p);
            t.i4mode[ras] = (int8_t)best;
            luma_block_levels(src + oy * e->cw + ox, e->cw, p, 4, mb->qp, 1, 0, t.luma[ras]);
            int coef[16];
            dequant_block(t.luma[ras], mb->qp, 0, coef);
            idct4_add(coef, dst + oy * e->cw + ox, e->cw, p, 4);
            t.nnz[ras] = (uint8_t)count_nz(t.luma[ras], 16);
        }
        if (won && sum + OH_I4_MB_OVERHEAD * lam >= c16) won = 0;
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
/* ---------------- OpenH264's P_Skip judge ---------------- */
/* WelsCalculateSingleCtr4x4 (func 1011): from the last non-zero level down (scan order), each non-zero level adds
 * OH_SINGLE_CTR[the run of zeros below it, to the next non-zero level or to the start] */
int h264o_single_ctr(const int16_t lv[16]) {
    int k = 15, s = 0;
    while (k >= 0 && lv[k] == 0) k--;
    while (k >= 0) {
        int j = k - 1;
        while (j >= 0 && lv[j] == 0) j--;
        s += OH_SINGLE_CTR[k - 1 - j];
        k = j;
    }
    return s;
}
/* WelsMdPSkipEnc's residual test (func 415 235160-235655, WelsTryPUVskip func 534): the luma 4x4 blocks of the MB
 * predicted at the skip vector quantised at the MB's QP (inter rounding, every position; pfQuantizationFour4x4Max,
 * func 1060): a block with a level above 1 rejects, and the single-coefficient costs of the blocks with a level
 * of 1 may sum to at most 5 over the MB; per chroma plane, at the chroma QP: a non-zero quantised 2x2 DC
 * coefficient rejects (pfQuantizationHadamard2x2Skip, func 1050), then each block quantised at every position (its
 * DC coefficient by the AC rule too) may have no level above 1, and the single-coefficient costs of the AC levels
 * (pfScan4x4Ac, func 1012) may sum to at most 6 per plane. Returns 1 when the residual admits the skip. */
static int pskip_residual_ok(H264OEnc *e, int mbx, int mby, int qp, const uint8_t pl[256], uint8_t pc[2][64]) {
    const uint8_t *src = e->src[0] + mby * 16 * e->cw + mbx * 16;
    int ctr = 0;
    for (int ras = 0; ras < 16; ras++) {
        const int ox = (ras & 3) * 4, oy = (ras >> 2) * 4;
        int d[16], c[16], mx = 0;
        int16_t lv[16];
        for (int y = 0; y < 4; y++) for (int x = 0; x < 4; x++) d[4 * y + x] = src[(oy + y) * e->cw + ox + x] - pl[(oy + y) * 16 + ox + x];
        fdct4(d, c);
        for (int k = 0; k < 16; k++) { lv[k] = (int16_t)quant4(c[ZIGZAG4[k]], qp, ZIGZAG4[k], 0); mx = imax(mx, iabs(lv[k])); }
        if (mx > OH_PSKIP_MAX_LEVEL) return 0;
        if (mx == 1) ctr += h264o_single_ctr(lv);
        if (ctr > OH_PSKIP_LUMA_CTR_MAX) return 0;
    }
    const int qpc = CHROMA_QP[qp], cs = e->cw / 2;
    for (int p = 0; p < 2; p++) {
        const uint8_t *cs_src = e->src[1 + p] + mby * 8 * cs + mbx * 8;
        int c4[4][16];
        for (int blk = 0; blk < 4; blk++) {
            const int ox = (blk & 1) * 4, oy = (blk >> 1) * 4;
            int d[16];
            for (int y = 0; y < 4; y++) for (int x = 0; x < 4; x++) d[4 * y + x] = cs_src[(oy + y) * cs + ox + x] - pc[p][(oy + y) * 8 + ox + x];
            fdct4(d, c4[blk]);
        }
        const int a = c4[0][0], b = c4[1][0], cc = c4[2][0], dd = c4[3][0];
        if (quant_dc4(a + b + cc + dd, qpc, 0) || quant_dc4(a - b + cc - dd, qpc, 0) || quant_dc4(a + b - cc - dd, qpc, 0) ||
            quant_dc4(a - b - cc + dd, qpc, 0))
            return 0;
        int pctr = 0;
        for (int blk = 0; blk < 4; blk++) {
            int16_t lv[16], ac[16];
            int mx = 0;
            for (int k = 0; k < 16; k++) { lv[k] = (int16_t)quant4(c4[blk][ZIGZAG4[k]], qpc, ZIGZAG4[k], 0); mx = imax(mx, iabs(lv[k])); }
            if (mx > OH_PSKIP_MAX_LEVEL) return 0;
            if (mx == 1) {
                for (int k = 0; k < 15; k++) ac[k] = lv[k + 1];
                ac[15] = 0;
                pctr += h264o_single_ctr(ac);
                if (pctr > OH_PSKIP_CHROMA_CTR_MAX) return 0;
            }
        }
    }
    return 1;
}
/* PredictSadSkip (func 331) over OpenH264's neighbour cache: index 0 top-left, 1 top, 2 top-right, 3 left; ref the
 * cached reference index (-2 outside the picture, -1 intra, 0 inter), sk 1 if the MB was skipped, sad its skip SAD. C is
 * the top-right MB, the top-left one when the top-right is outside the picture; a neighbour counts with its skip SAD if
 * it was skipped (and inter), else 0. One such neighbour: its SAD; otherwise the median of the three. Without a top or
 * top-left MB: the left MB's. */
int h264o_predict_sad_skip(const int32_t ref[4], const int32_t sk[4], const int32_t sad[4]) {
    int sA = sk[3] ? sad[3] : 0, sB = sk[1] ? sad[1] : 0, sC = sk[2] ? sad[2] : 0;
    int refC = ref[2], skC = sk[2];
    if (refC == -2) {
        refC = ref[0]; skC = sk[0]; sC = sk[0] ? sad[0] : 0;
        if (ref[1] == -2 && refC == -2 && ref[3] != -2) return sA;
    }
    const int f = (ref[3] == 0 ? sk[3] : 0) | ((ref[1] == 0 ? sk[1] : 0) << 1) | ((refC == 0 ? (skC ? 4 : 0) : 0));
    switch (f) {
    case 1: return sA;
    case 2: return sB;
    case 4: return sC;
    default: return sA + sB + sC - imin(sA, imin(sB, sC)) - imax(sA, imax(sB, sC));
    }
}
static int predict_sad_skip(const H264OEnc *e, int mbx, int mby) {
    const int mbw = e->mbw, n = mby * mbw + mbx;
    const int av[4] = {mbx > 0 && mby > 0, mby > 0, mby > 0 && mbx + 1 < mbw, mbx > 0};
    const int nb[4] = {n - mbw - 1, n - mbw, n - mbw + 1, n - 1};
    int32_t ref[4], sk[4], sad[4];
    for (int i = 0; i < 4; i++) {
        const MBInfo *m = av[i] ? &e->mbs[nb[i]] : NULL;
        ref[i] = !m ? -2 : (mb_is_intra(m->type) ? -1 : 0);
        sk[i] = m && m->type == MBT_PSKIP;
        sad[i] = sk[i] ? e->sksad_cur[nb[i]] : 0;
    }
    return h264o_predict_sad_skip(ref, sk, sad);
}
/* WelsMdI16x16's cost (func 313: SAD + lambda x mode bits, the first minimum in the pinned order) of the MB against its
 * reconstructed neighbours -- WelsMdFirstIntraMode's (func 747) first step in P slices */
static int i16_cost_oh(H264OEnc *e, int mbx, int mby, int lam) {
    IntraNb nb;
    uint8_t p16[256];
    int c16;
    get_nb16(e->rec[0], e->cw, mbx * 16, mby * 16, 16, mby > 0, mbx > 0, &nb);
    i16_best_oh(e, mbx, mby, &nb, lam, &c16, p16);
    return c16;
}
static int sad_mb_pred(H264OEnc *e, int mbx, int mby, const uint8_t pl[256], uint8_t pc[2][64]) {
    const int cs = e->cw / 2;
    return sad_blk(e->src[0] + mby * 16 * e->cw + mbx * 16, e->cw, pl, 16, 16, 16) +
           sad_blk(e->src[1] + mby * 8 * cs + mbx * 8, cs, pc[0], 8, 8, 8) + sad_blk(e->src[2] + mby * 8 * cs + mbx * 8, cs, pc[1], 8, 8, 8);
}
static void encode_p_mb(H264OEnc *e, MBInfo *mb, int mbx, int mby) {
    int lam = LAMBDA[mb->qp];
    Pic rp = {e->ref[0], e->ref[1], e->ref[2], e->cw, e->ch, e->cw, e->cw / 2};
    int cs = e->cw / 2;
    uint8_t pl[256], pc[2][64];
    int skmv[2], mvp[2];
    pskip_mv(e->mbs, e->mbw, mbx, mby, skmv);
    mvp_16x16(e->mbs, e->mbw, mbx, mby, mvp);
    /* 1. OpenH264's P_Skip judge (WelsMdInterMb func 746, WelsMdPSkipEnc func 415): tried when a
     * neighbour (left, top, top-left, top-right) was skipped, or, on a P reference picture, the co-located MB was;
     * then, unless the skip vector points too far outside the picture, the skip is taken when the prediction's SAD
     * (luma + chroma) is 0, below the neighbours' predicted skip SAD, or (P reference, co-located MB skipped) below
     * that MB's skip SAD -- else when its residual passes pskip_residual_ok. A taken skip is kept outright when the left,
     * top and top-right MBs were skipped (bKeepSkip); otherwise WelsMdFirstIntraMode (func 747) codes the MB intra
     * when its I16x16 cost (pinned SAD rule, §3.3) is below the skip's luma SAD (bMdUsingSad: the wrapper's
     * complexity 0, func 1143 732160) -- I16x16, or Intra4x4 by the same VAA-gated search as in I slices. */
    const int n = mby * e->mbw + mbx, mbw = e->mbw;
    const int ref_p = !e->last_idr, ref_skip = ref_p && e->sksad_ref[n] >= 0;
    const int try_skip = (mbx > 0 && e->mbs[n - 1].type == MBT_PSKIP) || (mby > 0 && e->mbs[n - mbw].type == MBT_PSKIP) ||
                         (mbx > 0 && mby > 0 && e->mbs[n - mbw - 1].type == MBT_PSKIP) ||
                         (mby > 0 && mbx + 1 < mbw && e->mbs[n - mbw + 1].type == MBT_PSKIP) || ref_skip;
    const int sx = (skmv[0] >> 2) + 16 * mbx, sy = (skmv[1] >> 2) + 16 * mby;
    e->sksad_cur[n] = -1;
    if (try_skip && sx >= OH_PSKIP_MV_MIN && sx <= ((16 * mbw) | OH_PSKIP_MV_MAX_LOW) && sy >= OH_PSKIP_MV_MIN &&
        sy <= ((16 * e->mbh) | OH_PSKIP_MV_MAX_LOW)) {
        mc_luma(&rp, mbx * 16, mby * 16, 16, 16, skmv[0], skmv[1], pl, 16);
        mc_chroma(e->ref[1], cs, e->ch / 2, cs, mbx * 8, mby * 8, 8, 8, skmv[0], skmv[1], pc[0], 8);
        mc_chroma(e->ref[2], cs, e->ch / 2, cs, mbx * 8, mby * 8, 8, 8, skmv[0], skmv[1], pc[1], 8);
        const int tsad = sad_mb_pred(e, mbx, mby, pl, pc);
        const int take = tsad == 0 || tsad < predict_sad_skip(e, mbx, mby) || (ref_skip && tsad < e->sksad_ref[n]) ||
                         pskip_residual_ok(e, mbx, mby, mb->qp, pl, pc);
        e->stat_skip_tried++;
        if (take) e->sksad_cur[n] = tsad;
    }
    if (e->sksad_cur[n] >= 0) {
        const int keep = mbx > 0 && mby > 0 && mbx + 1 < mbw && e->mbs[n - 1].type == MBT_PSKIP && e->mbs[n - mbw].type == MBT_PSKIP &&
                         e->mbs[n - mbw + 1].type == MBT_PSKIP;
        if (!keep && i16_cost_oh(e, mbx, mby, lam) < sad_blk(e->src[0] + mby * 16 * e->cw + mbx * 16, e->cw, pl, 16, 16, 16)) {
            e->sksad_cur[n] = -1;
            e->stat_intra_p++;
            encode_intra_mb(e, mb, mbx, mby);
            return;
        }
    }
    if (e->sksad_cur[n] >= 0) {  /* P_Skip: the reconstruction is the prediction */
        for (int p = 0; p < 2; p++)
            for (int y = 0; y < 8; y++) memcpy(e->rec[1 + p] + (mby * 8 + y) * cs + mbx * 8, pc[p] + 8 * y, 8);
        mb->type = MBT_PSKIP; mb->cbp = 0;
        memset(mb->nnz, 0, sizeof(mb->nnz));
        for (int i = 0; i < 16; i++) { mb->mv[i][0] = (int16_t)skmv[0]; mb->mv[i][1] = (int16_t)skmv[1]; mb->i4mode[i] = 2; }
        for (int i = 0; i < 4; i++) mb->ref[i] = 0;
        uint8_t *dst = e->rec[0] + mby * 16 * e->cw + mbx * 16;
        for (int y = 0; y < 16; y++) memcpy(dst + y * e->cw, pl + 16 * y, 16);
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
    /* 3. WelsMdFirstIntraMode (func 747, called first by WelsMdInterSecondaryModesEnc, func 399): the MB is coded intra
     * when its I16x16 cost (pinned SAD rule) is below the integer search's cost (here this project's search: SAD +
     * lambda x mvd bits) -- I16x16, or Intra4x4 by the VAA-gated search; before the sub-pel refinement, as OpenH264 */
    if (i16_cost_oh(e, mbx, mby, lam) < bc) {
        e->stat_intra_p++;
        encode_intra_mb(e, mb, mbx, mby);
        return;
    }
    /* 4. half then quarter refinement by SATD */
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
    /* 6. WelsMdInterDoubleCheckPskip (func 399 217892-217961): a P16x16 MB with no coded residual at the skip vector
     * is a P_Skip (same reconstruction); its skip SAD for the judge is the prediction's SAD there */
    if (mb->cbp == 0 && mx == skmv[0] && my == skmv[1]) {
        mb->type = MBT_PSKIP;
        e->sksad_cur[n] = sad_mb_pred(e, mbx, mby, pl, pc);
        e->stat_skip_double++;
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
    e->prev_src = (uint8_t *)calloc((size_t)e->cw * e->ch, 1);
    e->sksad_cur = (int32_t *)malloc((size_t)e->mbw * e->mbh * sizeof(int32_t));
    e->sksad_ref = (int32_t *)malloc((size_t)e->mbw * e->mbh * sizeof(int32_t));
    for (int i = 0; i < e->mbw * e->mbh; i++) e->sksad_cur[i] = e->sksad_ref[i] = -1;
    e->rc.gom_sad = (uint32_t *)calloc((size_t)e->mbw * e->mbh, sizeof(uint32_t));
    e->rc.gom_trace = (int32_t *)calloc(4 * (size_t)e->mbw * e->mbh, sizeof(int32_t));
    rc_init(&e->rc, w, h, bitrate);  /* frame skipping on: the wrapper leaves bEnableFrameSkip at its default */
    e->first = 1;
    e->idr_pic_id = 0;
    return e;
}
void h264o_enc_destroy(H264OEnc *e) {
    if (!e) return;
    for (int p = 0; p < 3; p++) { free(e->src[p]); free(e->rec[p]); free(e->ref[p]); }
    free(e->prev_src); free(e->rc.gom_sad); free(e->rc.gom_trace);
    free(e->mbs); free(e->rowqp); free(e->rowbits); free(e->sksad_cur); free(e->sksad_ref); free(e);
}
/* bEnableFrameSkip (on by default, as the wrapper leaves it): off, no frame is skipped, the VBV check is not
 * made, and an exhausted VGOP budget raises the QP instead (BITS_EXCEEDED) */
void h264o_enc_set_frame_skip(H264OEnc *e, int enable) { if (e) e->rc.skip_en = enable != 0; }
void h264o_enc_set_gom_exact(H264OEnc *e, int enable) { if (e) e->gom_exact = enable != 0; }
/* the rate control's state after the last encode call, for tests: {skipped (1 if that call skipped the frame),
 * global QP, average QP, target bits, remaining bits, buffer fullness (low 32 bits), continual skips,
 * frame complexity (low 32 bits), min frame QP, max frame QP, bits per frame, P frames coded, IDRs coded,
 * skip flag, remaining weights, frames coded in the VGOP} */
void h264o_enc_rc_state(const H264OEnc *e, int32_t out[16]) {
    const Rc *r = &e->rc;
    out[0] = e->last_skipped; out[1] = r->global_qp; out[2] = r->avg_qp; out[3] = r->target; out[4] = r->remaining;
    out[5] = (int32_t)r->fullness; out[6] = r->continual_skip; out[7] = (int32_t)r->frame_cmplx; out[8] = r->min_frame_qp;
    out[9] = r->max_frame_qp; out[10] = r->bpf; out[11] = r->pframe_num; out[12] = r->idr_num; out[13] = r->skip_flag;
    out[14] = r->remaining_weights; out[15] = r->frame_coded_in_vgop;
}
/* exact GOM mode: the last P frame's per-GOM {QP, slice bits before it, target bits, last coded MB + 1} (4 int32
 * per GOM, at most cap values); returns the GOM count */
int h264o_enc_gom_state(const H264OEnc *e, int32_t *out, int cap) {
    const int G = e->rc.gom_count;
    for (int i = 0; i < 4 * G && i < cap; i++) out[i] = e->rc.gom_trace[i];
    return G;
}
int h264o_enc_frames_skipped(const H264OEnc *e) { return e ? e->skipped : 0; }
void h264o_enc_me_stats(const H264OEnc *e, int32_t out[6]) {
    out[0] = e->stat_cross; out[1] = e->stat_cross_moved; out[2] = e->stat_nb_start;
    out[3] = e->stat_skip_tried; out[4] = e->stat_skip_double; out[5] = e->stat_intra_p;
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
    Rc *rc = &e->rc;
    /* frame skip (func 589 / 1258 / 1254): a skipped frame leaves the reference, frame_num and
     * the preprocessing's reference picture as they are; an IDR is never skipped */
    e->last_skipped = 0;
    if (rc_judge_skip(rc) && !idr) {
        rc_post_skip(rc);
        e->skipped++;
        e->last_skipped = 1;
        return 0;
    }
    load_source(e, yuv);
    e->first = 0; e->force_idr = 0;
    /* uiIdrPicId (a uint16) is incremented before the IDR's parameter sets are written (func 589, file
     * offset 378895), so the first IDR carries 1 when the counter starts at 0 */
    if (idr) { e->frame_num = 0; e->poc = 0; e->idr_pic_id = (e->idr_pic_id + 1) & 0xffff; }
    rc->frame_cmplx = rc_complexity(rc, e->src[0], e->prev_src, e->cw, idr);
    rc_picture_init(rc, idr, e->w, e->h);
    const int qp = rc->global_qp;
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
        /* this project's row plan: P rows at the frame QP + the row's offset inside the frame's window; an IDR
         * is coded at the frame QP (OpenH264 turns the GOM QP off for I slices in RC_BITRATE_MODE) */
        const int qplan = idr ? qp : clip3(rc->min_frame_qp, rc->max_frame_qp, qp + e->rowqp[mby]);
        e->rowbits[mby] = 0;
        for (int mbx = 0; mbx < e->mbw; mbx++) {
            MBInfo *mb = &e->mbs[mby * e->mbw + mbx];
            const int qrow = e->gom_exact ? rc_mb_init_gom(rc, mby * e->mbw + mbx, idr) : qplan;
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
            if (mb->type == MBT_PSKIP) { skip_run++; rc_mb_update(rc, 0, running); continue; }
            const int64_t bs = bw_bits(&b);
            if (!idr) { bw_ue(&b, (uint32_t)skip_run); skip_run = 0; }
            const int64_t b0 = bw_bits(&b);
            write_mb(&b, e, mb, mbx, mby, !idr, dqp);
            e->rowbits[mby] += bw_bits(&b) - b0;
            rc_mb_update(rc, (int)(bw_bits(&b) - bs), running);
        }
    }
    if (skip_run) bw_ue(&b, (uint32_t)skip_run);
    bw_trailing(&b);
    const size_t o_slice = o;
    o += nal_write(tmp + o, 3, idr ? 5 : 1, b.buf, b.len);
    bw_free(&b);
    { int32_t *t = e->sksad_ref; e->sksad_ref = e->sksad_cur; e->sksad_cur = t; }
    /* loop filter on the reconstruction -> next reference */
    deblock_frame(e->rec[0], e->rec[1], e->rec[2], e->cw, e->cw / 2, e->mbs, e->mbw, e->mbh, 0);
    for (int p = 0; p < 3; p++) { uint8_t *t = e->ref[p]; e->ref[p] = e->rec[p]; e->rec[p] = t; }
    e->last_qp = qp; e->last_idr = idr;
    /* the RC update on the slice NAL's size (func 1218: iLayerSize of the slice layer, 677356 / 683472) */
    rc_picture_update(rc, idr, (int)(o - o_slice));
    rc_plan_rows(e);
    /* the preprocessing's reference picture is the last coded frame's source (UpdateSrcList) */
    memcpy(e->prev_src, e->src[0], (size_t)e->cw * e->ch);
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
