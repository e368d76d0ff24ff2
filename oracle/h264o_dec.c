/*
 * oracle/h264o_dec.c -- TEST INFRASTRUCTURE ONLY (CPU oracle; see oracle/README.md).
 *
 * CPU restatement of the decode path behind openh264_wrapper.cpp:253-280 (init_decoder) and
 * :424-464 (decode_frame_yuv_i420 -> ISVCDecoder::DecodeFrameNoDelay): the normative H.264
 * Baseline decoding process (clauses 7.3 syntax, 8.3 intra, 8.4 inter, 8.5 transform, 8.7 loop
 * filter, 9.2 CAVLC). Scope: CAVLC, frame MBs, any number of slices per picture in any order (ASO;
 * I and P slices mixed in non-IDR pictures), neighbour availability and the loop filter's slice-edge
 * rules per slice, non-reference pictures (decoded and output, the reference kept), one reference
 * frame, all P partition shapes incl. sub-8x8, I_PCM. Out of scope (rejected with an error): FMO,
 * more than one active reference, constrained intra prediction, redundant pictures.
 */
#include "h264o_api.h"
#include "h264o_common.h"
#include "h264o_tables.h"
#include <stdlib.h>
#include <string.h>

struct H264ODec {
    int have_sps, have_pps;
    int mbw, mbh, log2_mfn, poc_type, log2_poc, dpoaz, crop[4], frame_mbs_only;
    int num_ref_default, pic_init_qp, cqp_off, dbk_ctrl, constrained_intra, redundant, bottom_field_poc, weighted;
    int cw, ch;
    uint8_t *cur[3], *ref[3];
    int has_ref;
    MBInfo *mbs;
    uint8_t *done;            /* per MB: decoded in the picture being assembled */
    int pic_open, pic_idr, pic_ref;  /* the access unit's picture: started, IDR, nal_ref_idc != 0 */
};

H264ODec *h264o_dec_create(void) { return (H264ODec *)calloc(1, sizeof(H264ODec)); }
static void free_frames(H264ODec *d) {
    for (int p = 0; p < 3; p++) { free(d->cur[p]); free(d->ref[p]); d->cur[p] = d->ref[p] = NULL; }
    free(d->mbs); d->mbs = NULL;
    free(d->done); d->done = NULL;
}
void h264o_dec_destroy(H264ODec *d) { if (d) { free_frames(d); free(d); } }

static int parse_sps(H264ODec *d, BR *r) {
    int profile = br_get(r, 8);
    br_get(r, 8); br_get(r, 8);
    br_ue(r);
    if (profile == 100 || profile == 110 || profile == 122 || profile == 244 || profile == 44 || profile == 83 ||
        profile == 86 || profile == 118 || profile == 128) return -1; /* High profiles: out of scope */
    int log2_mfn = br_ue(r) + 4;
    int poc_type = br_ue(r), log2_poc = 0, dpoaz = 0;
    if (poc_type == 0) log2_poc = br_ue(r) + 4;
    else if (poc_type == 1) {
        dpoaz = br_get(r, 1); br_se(r); br_se(r);  /* delta_pic_order_always_zero_flag */
        int n = br_ue(r);
        for (int i = 0; i < n; i++) br_se(r);
    }
    br_ue(r);            /* max_num_ref_frames */
    br_get(r, 1);        /* gaps */
    int mbw = br_ue(r) + 1, mbh = br_ue(r) + 1;
    int fmo = br_get(r, 1);
    if (!fmo) return -1;
    br_get(r, 1);        /* direct_8x8_inference */
    int crop[4] = {0, 0, 0, 0};
    if (br_get(r, 1)) for (int i = 0; i < 4; i++) crop[i] = br_ue(r);
    if (r->err || mbw > 1024 || mbh > 1024) return -1;
    if (mbw != d->mbw || mbh != d->mbh || !d->mbs) {
        free_frames(d);
        d->mbw = mbw; d->mbh = mbh; d->cw = mbw * 16; d->ch = mbh * 16;
        for (int p = 0; p < 3; p++) {
            size_t n = p ? (size_t)(d->cw / 2) * (d->ch / 2) : (size_t)d->cw * d->ch;
            d->cur[p] = (uint8_t *)calloc(n, 1); d->ref[p] = (uint8_t *)calloc(n, 1);
        }
        d->mbs = (MBInfo *)calloc((size_t)mbw * mbh, sizeof(MBInfo));
        d->done = (uint8_t *)calloc((size_t)mbw * mbh, 1);
        d->has_ref = 0;
    }
    d->log2_mfn = log2_mfn; d->poc_type = poc_type; d->log2_poc = log2_poc; d->dpoaz = dpoaz;
    memcpy(d->crop, crop, sizeof(crop));
    d->have_sps = 1;
    return 0;
}
static int parse_pps(H264ODec *d, BR *r) {
    br_ue(r); br_ue(r);
    if (br_get(r, 1)) return -1;          /* CABAC: out of scope (Baseline only) */
    d->bottom_field_poc = br_get(r, 1);
    if (br_ue(r) != 0) return -1;         /* FMO */
    d->num_ref_default = br_ue(r) + 1;
    br_ue(r);
    d->weighted = br_get(r, 1);
    br_get(r, 2);
    d->pic_init_qp = 26 + br_se(r);
    br_se(r);
    d->cqp_off = br_se(r);
    d->dbk_ctrl = br_get(r, 1);
    d->constrained_intra = br_get(r, 1);
    d->redundant = br_get(r, 1);
    if (d->constrained_intra || d->weighted) return -1;
    d->have_pps = 1;
    return r->err ? -1 : 0;
}

static void nb16(const uint8_t *pl, int stride, int px, int py, int size, int has_top, int has_left, int has_tl, IntraNb *n) {
    memset(n, 0, sizeof(*n));
    n->has_top = has_top; n->has_left = has_left; n->has_tl = has_tl;
    if (has_top) for (int i = 0; i < size; i++) n->top[i] = pl[(py - 1) * stride + px + i];
    if (has_left) for (int i = 0; i < size; i++) n->left[i] = pl[(py + i) * stride + px - 1];
    if (n->has_tl) n->tl = pl[(py - 1) * stride + px - 1];
}
/* 4x4 block neighbours inside / across the macroblock (6.4.11.4), MBs by slice (mb_nb_avail) */
static int tr_avail(const MBInfo *mbs, int mbx, int mby, int mbw, int ras) {
    int bx = ras & 3, by = ras >> 2;
    if (by == 0) return mb_nb_avail(mbs, mbw, mbx, mby, bx < 3 ? 0 : 1, -1);
    if (bx == 3) return 0;
    return RAS2BLK[(by - 1) * 4 + bx + 1] < RAS2BLK[ras];
}
static void nb4(const MBInfo *mbs, const uint8_t *pl, int stride, int mbx, int mby, int mbw, int ras, IntraNb *n) {
    int bx = ras & 3, by = ras >> 2, px = mbx * 16 + bx * 4, py = mby * 16 + by * 4;
    memset(n, 0, sizeof(*n));
    n->has_top = by > 0 || mb_nb_avail(mbs, mbw, mbx, mby, 0, -1);
    n->has_left = bx > 0 || mb_nb_avail(mbs, mbw, mbx, mby, -1, 0);
    n->has_tl = (bx > 0 && by > 0) ? 1 : mb_nb_avail(mbs, mbw, mbx, mby, bx > 0 ? 0 : -1, by > 0 ? 0 : -1);
    n->has_tr = n->has_top && tr_avail(mbs, mbx, mby, mbw, ras);
    if (n->has_top) {
        for (int i = 0; i < 4; i++) n->top[i] = pl[(py - 1) * stride + px + i];
        for (int i = 4; i < 8; i++) n->top[i] = n->has_tr ? pl[(py - 1) * stride + px + i] : n->top[3];
    }
    if (n->has_left) for (int i = 0; i < 4; i++) n->left[i] = pl[(py + i) * stride + px - 1];
    if (n->has_tl) n->tl = pl[(py - 1) * stride + px - 1];
}
static int pred_mode4(const MBInfo *mbs, const MBInfo *cur, int mbw, int mbx, int mby, int ras) {
    int bx = ras & 3, by = ras >> 2, a, b;
    if (bx > 0) a = cur->i4mode[ras - 1];
    else if (mb_nb_avail(mbs, mbw, mbx, mby, -1, 0)) { const MBInfo *m = &mbs[mby * mbw + mbx - 1]; a = m->type == MBT_I4 ? m->i4mode[ras + 3] : 2; }
    else return 2;
    if (by > 0) b = cur->i4mode[ras - 4];
    else if (mb_nb_avail(mbs, mbw, mbx, mby, 0, -1)) { const MBInfo *m = &mbs[(mby - 1) * mbw + mbx]; b = m->type == MBT_I4 ? m->i4mode[ras + 12] : 2; }
    else return 2;
    return imin(a, b);
}

/* residual() 7.3.5.3 */
static void parse_residual(H264ODec *d, BR *r, MBInfo *mb, int mbx, int mby) {
    memset(mb->nnz, 0, sizeof(mb->nnz));
    memset(mb->luma, 0, sizeof(mb->luma)); memset(mb->lumadc, 0, sizeof(mb->lumadc));
    memset(mb->cdc, 0, sizeof(mb->cdc)); memset(mb->cac, 0, sizeof(mb->cac));
    if (mb->type == MBT_I16) {
        cavlc_read_block(r, mb->lumadc, 16, nc_luma(d->mbs, mb, d->mbw, mbx, mby, 0));
        if (mb->cbp & 15)
            for (int blk = 0; blk < 16; blk++) {
                int ras = BLK2RAS[blk];
                mb->nnz[ras] = (uint8_t)cavlc_read_block(r, mb->luma[ras] + 1, 15, nc_luma(d->mbs, mb, d->mbw, mbx, mby, ras));
            }
    } else {
        for (int i8 = 0; i8 < 4; i8++) {
            if (!(mb->cbp & (1 << i8))) continue;
            for (int i4 = 0; i4 < 4; i4++) {
                int ras = BLK2RAS[i8 * 4 + i4];
                mb->nnz[ras] = (uint8_t)cavlc_read_block(r, mb->luma[ras], 16, nc_luma(d->mbs, mb, d->mbw, mbx, mby, ras));
            }
        }
    }
    int cbpc = mb->cbp >> 4;
    if (cbpc) {
        for (int pl = 0; pl < 2; pl++) cavlc_read_block(r, mb->cdc[pl], 4, -1);
        if (cbpc == 2)
            for (int pl = 0; pl < 2; pl++)
                for (int blk = 0; blk < 4; blk++)
                    mb->nnz[16 + 4 * pl + blk] = (uint8_t)cavlc_read_block(r, mb->cac[pl][blk] + 1, 15,
                                                                           nc_chroma(d->mbs, mb, d->mbw, mbx, mby, pl, blk));
    }
}

/* Reconstruction of one macroblock into d->cur (8.3, 8.4, 8.5). */
static void recon_mb(H264ODec *d, MBInfo *mb, int mbx, int mby) {
    int ys = d->cw, cs = d->cw / 2;
    uint8_t *Y = d->cur[0] + mby * 16 * ys + mbx * 16;
    uint8_t *C[2] = {d->cur[1] + mby * 8 * cs + mbx * 8, d->cur[2] + mby * 8 * cs + mbx * 8};
    int qp = mb->qp, qpc = mb->type == MBT_IPCM ? 0 : CHROMA_QP[clip3(0, 51, qp + d->cqp_off)];
    if (mb->type == MBT_IPCM) {
        for (int y = 0; y < 16; y++) memcpy(Y + y * ys, mb->pcm + 16 * y, 16);
        for (int pl = 0; pl < 2; pl++) for (int y = 0; y < 8; y++) memcpy(C[pl] + y * cs, mb->pcm + 256 + 64 * pl + 8 * y, 8);
        return;
    }
    uint8_t cpred[2][64];
    if (mb_is_intra(mb->type)) {
        if (mb->type == MBT_I4) {
            for (int blk = 0; blk < 16; blk++) {
                int ras = BLK2RAS[blk], ox = (ras & 3) * 4, oy = (ras >> 2) * 4, coef[16];
                IntraNb n; uint8_t p[16];
                nb4(d->mbs, d->cur[0], ys, mbx, mby, d->mbw, ras, &n);
                pred4x4(&n, mb->i4mode[ras], p);
                dequant_block(mb->luma[ras], qp, 0, coef);
                idct4_add(coef, Y + oy * ys + ox, ys, p, 4);
            }
        } else {
            IntraNb n; uint8_t p[256]; int dc[16];
            nb16(d->cur[0], ys, mbx * 16, mby * 16, 16, mb_nb_avail(d->mbs, d->mbw, mbx, mby, 0, -1),
                 mb_nb_avail(d->mbs, d->mbw, mbx, mby, -1, 0), mb_nb_avail(d->mbs, d->mbw, mbx, mby, -1, -1), &n);
            pred16x16(&n, mb->i16mode, p);
            luma_dc_dequant(mb->lumadc, qp, dc);
            for (int ras = 0; ras < 16; ras++) {
                int ox = (ras & 3) * 4, oy = (ras >> 2) * 4, coef[16];
                dequant_block(mb->luma[ras], qp, 1, coef);
                coef[0] = dc[ras];
                idct4_add(coef, Y + oy * ys + ox, ys, p + oy * 16 + ox, 16);
            }
        }
        for (int pl = 0; pl < 2; pl++) {
            IntraNb n;
            nb16(d->cur[1 + pl], cs, mbx * 8, mby * 8, 8, mb_nb_avail(d->mbs, d->mbw, mbx, mby, 0, -1),
                 mb_nb_avail(d->mbs, d->mbw, mbx, mby, -1, 0), mb_nb_avail(d->mbs, d->mbw, mbx, mby, -1, -1), &n);
            pred_chroma(&n, mb->cmode, cpred[pl]);
        }
    } else {
        Pic rp = {d->ref[0], d->ref[1], d->ref[2], d->cw, d->ch, d->cw, cs};
        uint8_t p[256];
        for (int ras = 0; ras < 16; ras++) {
            int ox = (ras & 3) * 4, oy = (ras >> 2) * 4;
            mc_luma(&rp, mbx * 16 + ox, mby * 16 + oy, 4, 4, mb->mv[ras][0], mb->mv[ras][1], p + oy * 16 + ox, 16);
            for (int pl = 0; pl < 2; pl++)
                mc_chroma(d->ref[1 + pl], cs, d->ch / 2, cs, mbx * 8 + ox / 2, mby * 8 + oy / 2, 2, 2, mb->mv[ras][0],
                          mb->mv[ras][1], cpred[pl] + (oy / 2) * 8 + ox / 2, 8);
        }
        for (int ras = 0; ras < 16; ras++) {
            int ox = (ras & 3) * 4, oy = (ras >> 2) * 4, coef[16];
            dequant_block(mb->luma[ras], qp, 0, coef);
            idct4_add(coef, Y + oy * ys + ox, ys, p + oy * 16 + ox, 16);
        }
    }
    for (int pl = 0; pl < 2; pl++) {
        int dc[4];
        chroma_dc_dequant(mb->cdc[pl], qpc, dc);
        for (int blk = 0; blk < 4; blk++) {
            int ox = (blk & 1) * 4, oy = (blk >> 1) * 4, coef[16];
            dequant_block(mb->cac[pl][blk], qpc, 1, coef);
            coef[0] = dc[blk];
            idct4_add(coef, C[pl] + oy * cs + ox, cs, cpred[pl] + oy * 8 + ox, 8);
        }
    }
}

static void set_part(MBInfo *mb, int bx, int by, int pw, int ph, const int mv[2]) {
    for (int y = by; y < by + ph; y += 4)
        for (int x = bx; x < bx + pw; x += 4) {
            int ras = (y >> 2) * 4 + (x >> 2);
            mb->mv[ras][0] = (int16_t)mv[0]; mb->mv[ras][1] = (int16_t)mv[1];
            mb->done4 |= (uint16_t)(1u << ras);
        }
}

/* One slice of the access unit's picture (7.3.3, 7.3.4). The first slice opens the picture; the
 * others must agree with it on IDR-ness and on being a reference picture (7.4.1.2.4). Returns 1 when
 * the slice decoded, -1 on an error (the access unit is then concealed). */
static int decode_slice(H264ODec *d, BR *r, int nal_type, int nal_ref_idc) {
    if (!d->have_sps || !d->have_pps) return -1;
    if (nal_type == 5 && nal_ref_idc == 0) return -1;
    int first_mb = br_ue(r);
    int st = br_ue(r) % 5;           /* 0 P, 2 I */
    br_ue(r);
    const int total = d->mbw * d->mbh;
    if (st != 0 && st != 2) return -1;
    if (first_mb >= total || (nal_type == 5 && st != 2)) return -1;
    if (!d->pic_open) {
        d->pic_open = 1; d->pic_idr = nal_type == 5; d->pic_ref = nal_ref_idc != 0;
        memset(d->done, 0, (size_t)total);
    } else if (d->pic_idr != (nal_type == 5) || d->pic_ref != (nal_ref_idc != 0)) {
        return -1;
    }
    br_get(r, d->log2_mfn);
    if (nal_type == 5) br_ue(r);
    if (d->poc_type == 0) { br_get(r, d->log2_poc); if (d->bottom_field_poc) br_se(r); }
    else if (d->poc_type == 1 && !d->dpoaz) { br_se(r); if (d->bottom_field_poc) br_se(r); }
    if (d->redundant) br_ue(r);
    int nref = d->num_ref_default;
    if (st == 0) {
        if (br_get(r, 1)) nref = br_ue(r) + 1;
        if (br_get(r, 1)) { /* ref_pic_list_modification */
            int op;
            while ((op = br_ue(r)) != 3) { br_ue(r); if (r->err) return -1; }
        }
        if (!d->has_ref) return -1;
    }
    if (nref > 1 && st == 0) return -1;   /* multiple references: out of scope */
    if (nal_ref_idc != 0) {               /* dec_ref_pic_marking() (7.3.3.3): reference pictures only */
        if (nal_type == 5) { br_get(r, 1); br_get(r, 1); }
        else if (br_get(r, 1)) {
            int op;
            while ((op = br_ue(r)) != 0) {
                if (op == 1 || op == 3) br_ue(r);
                if (op == 2) br_ue(r);
                if (op == 3 || op == 6) br_ue(r);
                if (op == 4) br_ue(r);
                if (r->err) return -1;
            }
        }
    }
    int qp = d->pic_init_qp + br_se(r);
    int dbk_idc = 0, dbk_a = 0, dbk_b = 0;
    if (d->dbk_ctrl) {
        dbk_idc = br_ue(r);
        if (dbk_idc > 2) return -1;
        if (dbk_idc != 1) {
            dbk_a = br_se(r) * 2; dbk_b = br_se(r) * 2;
            if (dbk_a < -12 || dbk_a > 12 || dbk_b < -12 || dbk_b > 12) return -1;
        }
    }
    if (r->err || qp < 0 || qp > 51 || d->cqp_off < -12 || d->cqp_off > 12) return -1;
    int addr = first_mb, more = 1;
    /* every MB of the slice carries the slice's identity and loop-filter parameters */
#define H264O_SLICE_MB(mb) do { (mb)->slice_first = first_mb; (mb)->dbk_idc = (int8_t)dbk_idc; (mb)->dbk_a = (int8_t)dbk_a; \
                                (mb)->dbk_b = (int8_t)dbk_b; if (d->done[addr]) return -1; d->done[addr] = 1; } while (0)
    while (more && addr < total) {
        if (st == 0) {
            uint32_t run = br_ue(r);
            if (r->err || run > (uint32_t)(total - addr)) return -1;
            for (uint32_t i = 0; i < run; i++, addr++) {
                int mbx = addr % d->mbw, mby = addr / d->mbw;
                MBInfo *mb = &d->mbs[addr];
                memset(mb, 0, sizeof(*mb));
                H264O_SLICE_MB(mb);
                mb->type = MBT_PSKIP; mb->qp = qp;
                for (int k = 0; k < 16; k++) mb->i4mode[k] = 2;
                for (int k = 0; k < 4; k++) mb->ref[k] = 0;
                int mv[2];
                pskip_mv(d->mbs, d->mbw, mbx, mby, mv);
                for (int k = 0; k < 16; k++) { mb->mv[k][0] = (int16_t)mv[0]; mb->mv[k][1] = (int16_t)mv[1]; }
                recon_mb(d, mb, mbx, mby);
            }
            if (run > 0) more = br_more_rbsp(r);
            if (!more || addr >= total) break;
        }
        int mbx = addr % d->mbw, mby = addr / d->mbw;
        MBInfo *mb = &d->mbs[addr];
        memset(mb, 0, sizeof(*mb));
        H264O_SLICE_MB(mb);
        for (int k = 0; k < 16; k++) mb->i4mode[k] = 2;
        for (int k = 0; k < 4; k++) mb->ref[k] = -1;
        uint32_t mt = br_ue(r);
        int itype = -1;
        if (st == 0) { if (mt >= 5) itype = (int)mt - 5; } else itype = (int)mt;
        if (itype > 25 || (st == 0 && mt > 30)) return -1;
        if (itype == 25) {
            mb->type = MBT_IPCM; mb->qp = qp;
            r->pos = (r->pos + 7) & ~(size_t)7;
            for (int i = 0; i < 384; i++) mb->pcm[i] = (uint8_t)br_get(r, 8);
            memset(mb->nnz, 16, sizeof(mb->nnz));
        } else if (itype >= 0) {
            if (itype == 0) {
                mb->type = MBT_I4;
                for (int blk = 0; blk < 16; blk++) {
                    int ras = BLK2RAS[blk];
                    int pm = pred_mode4(d->mbs, mb, d->mbw, mbx, mby, ras);
                    if (br_get(r, 1)) mb->i4mode[ras] = (int8_t)pm;
                    else { int rem = br_get(r, 3); mb->i4mode[ras] = (int8_t)(rem < pm ? rem : rem + 1); }
                }
                mb->cmode = br_ue(r);
                uint32_t c = br_ue(r);
                if (c > 47) return -1;
                mb->cbp = CBP_INTRA_FROM_CODE[c];
            } else {
                mb->type = MBT_I16;
                mb->i16mode = (itype - 1) % 4;
                mb->cbp = ((((itype - 1) / 4) % 3) << 4) | (itype >= 13 ? 15 : 0);
                mb->cmode = br_ue(r);
            }
            if (mb->cmode > 3) return -1;
        } else {
            /* P macroblock: mb_pred / sub_mb_pred (7.3.5.1, 7.3.5.2) */
            for (int k = 0; k < 4; k++) mb->ref[k] = 0;
            int mvd[16][2], np = 0;
            int px[16], py[16], pw[16], ph[16], shape[16];
            if (mt <= 2) {
                static const int PW[3] = {16, 16, 8}, PH[3] = {16, 8, 16};
                int n = mt == 0 ? 1 : 2;
                mb->type = mt == 0 ? MBT_P16x16 : (mt == 1 ? MBT_P16x8 : MBT_P8x16);
                for (int i = 0; i < n; i++) {
                    px[i] = mt == 2 ? 8 * i : 0; py[i] = mt == 1 ? 8 * i : 0;
                    pw[i] = PW[mt]; ph[i] = PH[mt]; shape[i] = mt == 0 ? 0 : (int)mt;
                }
                np = n;
                for (int i = 0; i < n; i++) { mvd[i][0] = br_se(r); mvd[i][1] = br_se(r); }
            } else {
                mb->type = MBT_P8x8;
                int sub[4];
                for (int i = 0; i < 4; i++) { sub[i] = br_ue(r); if (sub[i] > 3) return -1; mb->sub_type[i] = (int8_t)sub[i]; }
                for (int i = 0; i < 4; i++) {
                    int sw = (sub[i] == 0 || sub[i] == 1) ? 8 : 4, sh = (sub[i] == 0 || sub[i] == 2) ? 8 : 4;
                    for (int y = 0; y < 8; y += sh)
                        for (int x = 0; x < 8; x += sw) {
                            px[np] = (i & 1) * 8 + x; py[np] = (i >> 1) * 8 + y; pw[np] = sw; ph[np] = sh; shape[np] = 0;
                            mvd[np][0] = br_se(r); mvd[np][1] = br_se(r);
                            np++;
                        }
                }
            }
            mb->done4 = 0;
            for (int i = 0; i < np; i++) {
                int mvp[2], mv[2];
                mvp_part(d->mbs, mb, d->mbw, mbx, mby, px[i], py[i], pw[i], ph[i], shape[i], mvp);
                mv[0] = mvp[0] + mvd[i][0]; mv[1] = mvp[1] + mvd[i][1];
                set_part(mb, px[i], py[i], pw[i], ph[i], mv);
            }
            uint32_t c = br_ue(r);
            if (c > 47) return -1;
            mb->cbp = CBP_INTER_FROM_CODE[c];
        }
        if (mb->type != MBT_IPCM) {
            if (mb->cbp || mb->type == MBT_I16) {
                int dq = br_se(r);
                if (dq < -26 || dq > 25) return -1;
                qp = (qp + dq + 52) % 52;
            }
            mb->qp = qp;
            parse_residual(d, r, mb, mbx, mby);
        }
        if (r->err) return -1;
        recon_mb(d, mb, mbx, mby);
        addr++;
        more = br_more_rbsp(r);
    }
#undef H264O_SLICE_MB
    if (more && addr >= total && br_more_rbsp(r)) return -1;  /* slice data past the picture's end */
    return 1;
}

/* tight cropped I420 copy of picture planes pic[] */
static void emit_picture(const H264ODec *d, uint8_t *const pic[3], uint8_t *out, int *w, int *h) {
    int W = d->cw - 2 * (d->crop[0] + d->crop[1]), H = d->ch - 2 * (d->crop[2] + d->crop[3]);
    int x0 = 2 * d->crop[0], y0 = 2 * d->crop[2];
    if (out) {
        uint8_t *o = out;
        for (int y = 0; y < H; y++, o += W) memcpy(o, pic[0] + (size_t)(y0 + y) * d->cw + x0, W);
        for (int p = 1; p < 3; p++)
            for (int y = 0; y < H / 2; y++, o += W / 2) memcpy(o, pic[p] + (size_t)(y0 / 2 + y) * (d->cw / 2) + x0 / 2, W / 2);
    }
    *w = W; *h = H;
}
/* returns 1: picture decoded, 2: damaged access unit concealed (frame copy), 0: no picture, -1: error */
int h264o_dec_decode(H264ODec *d, const uint8_t *data, int size, uint8_t *out, int *w, int *h) {
    *w = *h = 0;
    if (!d || !data || size <= 0) return -1;
    int got_pic = 0, damaged = 0, i = 0;
    d->pic_open = 0;
    while (i + 3 <= size) {
        /* find start code */
        int s = -1;
        for (int k = i; k + 3 <= size; k++)
            if (data[k] == 0 && data[k + 1] == 0 && data[k + 2] == 1) { s = k + 3; break; }
        if (s < 0) break;
        int e = size;
        for (int k = s; k + 3 <= size; k++)
            if (data[k] == 0 && data[k + 1] == 0 && (data[k + 2] == 1 || (data[k + 2] == 0 && k + 3 < size && data[k + 3] == 1))) { e = k; break; }
        int n = e - s;
        while (n > 0 && data[s + n - 1] == 0) n--;
        i = e;
        if (n < 1) continue;
        int hdr = data[s];
        int type = hdr & 31, ref_idc = (hdr >> 5) & 3;
        /* remove emulation prevention bytes */
        uint8_t *rb = (uint8_t *)malloc((size_t)n);
        int m = 0, zeros = 0;
        for (int k = 1; k < n; k++) {
            if (zeros >= 2 && data[s + k] == 3) { zeros = 0; continue; }
            rb[m++] = data[s + k];
            zeros = data[s + k] == 0 ? zeros + 1 : 0;
        }
        BR r = {rb, (size_t)m, 0, 0};
        int rv = 0;
        if (type == 7) rv = parse_sps(d, &r);
        else if (type == 8) rv = parse_pps(d, &r);
        else if (type == 1 || type == 5) {
            rv = decode_slice(d, &r, type, ref_idc);
            if (rv == 1) got_pic = 1;
        }
        free(rb);
        if (rv < 0) { damaged = 1; break; }
    }
    if (damaged) {
        /* ERROR_CON_FRAME_COPY (openh264_wrapper.cpp:269): a damaged access unit is concealed by a
         * copy of the last picture, which stays the reference; with no earlier picture, no output */
        if (!d->has_ref) return -1;
        emit_picture(d, d->ref, out, w, h);
        return 2;
    }
    if (!got_pic) return 0;
    /* every macroblock of the picture decoded exactly once (its slices in any order), else concealed */
    for (int k = 0; k < d->mbw * d->mbh; k++)
        if (!d->done[k]) {
            if (!d->has_ref) return -1;
            emit_picture(d, d->ref, out, w, h);
            return 2;
        }
    /* the loop filter over the whole picture, each MB with its slice's parameters (8.7) */
    deblock_frame(d->cur[0], d->cur[1], d->cur[2], d->cw, d->cw / 2, d->mbs, d->mbw, d->mbh, d->cqp_off);
    emit_picture(d, d->cur, out, w, h);
    if (d->pic_ref) {  /* a reference picture becomes the next P slices' reference; a non-reference one does not */
        for (int p = 0; p < 3; p++) { uint8_t *t = d->ref[p]; d->ref[p] = d->cur[p]; d->cur[p] = t; }
        d->has_ref = 1;
    }
    return 1;
}
/* per MB the 24 TotalCoeff bytes (luma raster 0..15, chroma AC 16..23) of the last picture -- test / analysis */
void h264o_dec_nnz(const H264ODec *d, uint8_t *out) {
    for (int i = 0; i < d->mbw * d->mbh; i++) memcpy(out + 24 * i, d->mbs[i].nnz, 24);
}
void h264o_dec_mbinfo(const H264ODec *d, int32_t *out) {
    for (int i = 0; i < d->mbw * d->mbh; i++) {
        const MBInfo *m = &d->mbs[i];
        int s = 0; for (int k = 0; k < 24; k++) s += m->nnz[k];
        int32_t *r = out + 8 * i;
        r[0] = m->type; r[1] = m->qp; r[2] = m->cbp; r[3] = m->mv[0][0]; r[4] = m->mv[0][1];
        r[5] = m->i16mode; r[6] = m->cmode; r[7] = s;
    }
}

/* ---------------- wrapper colour conversion (openh264_wrapper.cpp:22-40, :150-195) ---------------- */
void h264o_rgba_to_i420(const uint8_t *rgba, int w, int h, uint8_t *out) {
    uint8_t *Y = out, *U = out + (size_t)w * h, *V = U + (size_t)(w / 2) * (h / 2);
    int yi = 0, ui = 0, vi = 0;
    for (int row = 0; row < h; row++)
        for (int col = 0; col < w; col++) {
            const uint8_t *p = rgba + ((size_t)row * w + col) * 4;
            int r = p[0], g = p[1], b = p[2];
            Y[yi++] = (uint8_t)(((66 * r + 129 * g + 25 * b + 128) >> 8) + 16);
            if (!(row & 1) && !(col & 1)) {
                U[ui++] = (uint8_t)((uint8_t)((-38 * r - 74 * g + 112 * b + 128) >> 8) + 128);
                V[vi++] = (uint8_t)((uint8_t)((112 * r - 94 * g - 18 * b + 128) >> 8) + 128);
            }
        }
}
void h264o_i420_to_rgba(const uint8_t *y, const uint8_t *u, const uint8_t *v, int w, int h, int ys, int uvs, uint8_t *out) {
    size_t o = 0;
    for (int row = 0; row < h; row++)
        for (int col = 0; col < w; col++) {
            int c = 298 * (y[row * ys + col] - 16);
            int cb = u[(row / 2) * uvs + col / 2] - 128, cr = v[(row / 2) * uvs + col / 2] - 128;
            out[o++] = (uint8_t)clip1((c + 409 * cr + 128) >> 8);
            out[o++] = (uint8_t)clip1((c - 100 * cb - 208 * cr + 128) >> 8);
            out[o++] = (uint8_t)clip1((c + 516 * cb + 128) >> 8);
            out[o++] = 255;
        }
}

/* ---------------- test-stream writing helpers (tests/streamgen.py) ----------------
 * The CAVLC residual_block writer (9.2, the encoder half's cavlc_write_block) as a bit string of
 * 0/1 bytes, and the coded_block_pattern code (Table 9-4 inverse), so that the hand-built decoder
 * test streams share their VLC tables with the oracle rather than restating them a second time. */
int h264o_cavlc_bits(const int16_t *coef, int maxnum, int nc, uint8_t *bits, int cap) {
    BW b; bw_init(&b);
    int tc = 0;
    cavlc_write_block(&b, coef, maxnum, nc, &tc);
    int n = (int)(b.len * 8) + b.nacc;
    if (n > cap) { bw_free(&b); return -1; }
    for (int i = 0; i < n; i++) {
        int byte = i >> 3;
        bits[i] = byte < (int)b.len ? (uint8_t)((b.buf[byte] >> (7 - (i & 7))) & 1)
                                    : (uint8_t)((b.acc >> (b.nacc - 1 - (i - (int)b.len * 8))) & 1);
    }
    bw_free(&b);
    return n;
}
int h264o_cbp_code(int cbp, int intra) {
    const uint8_t *t = intra ? CBP_INTRA_FROM_CODE : CBP_INTER_FROM_CODE;
    for (int c = 0; c < 48; c++) if (t[c] == cbp) return c;
    return -1;
}
