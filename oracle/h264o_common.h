/*
 * oracle/h264o_common.h -- TEST INFRASTRUCTURE ONLY (CPU oracle; see oracle/README.md).
 *
 * Shared pieces of the CPU restatement: bit writer/reader, 4x4 transforms, quantisation,
 * intra prediction, luma/chroma motion-compensated interpolation, deblocking, CAVLC.
 * Everything is integer arithmetic restating ITU-T H.264 clauses (cited per function) plus the
 * encoder-side choices documented in DESIGN.md §3 (the wrapper's parameters from
 * openh264_wrapper.cpp:207-220 and OpenH264's upstream algorithm as restated there).
 */
#ifndef H264O_COMMON_H
#define H264O_COMMON_H
#include <stdint.h>
#include <stddef.h>

enum { MBT_I4 = 0, MBT_I16 = 1, MBT_P16x16 = 2, MBT_PSKIP = 3, MBT_P16x8 = 4, MBT_P8x16 = 5,
       MBT_P8x8 = 6, MBT_IPCM = 7 };

static inline int mb_is_intra(int t) { return t == MBT_I4 || t == MBT_I16 || t == MBT_IPCM; }
static inline int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
static inline int clip1(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
static inline int iabs(int v) { return v < 0 ? -v : v; }
static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline int median3(int a, int b, int c) { return imax(imin(a, b), imin(imax(a, b), c)); }

/* Per-macroblock state (decisions, motion, coefficient levels). */
typedef struct {
    int type;
    int qp;
    int cbp;             /* luma bits 0..3 (per 8x8), chroma (0..2) << 4 */
    int i16mode;         /* 0 V,1 H,2 DC,3 Plane */
    int cmode;           /* chroma: 0 DC,1 H,2 V,3 Plane */
    int8_t i4mode[16];   /* raster 4x4 index; DC(2) for non-I4 MBs */
    int16_t mv[16][2];   /* per 4x4 raster, quarter-pel */
    int8_t ref[4];       /* per 8x8; -1 for intra */
    uint8_t nnz[24];     /* TotalCoeff: luma raster 0..15, Cb 16..19, Cr 20..23 */
    int16_t mvd[16][2];  /* encoder: mvd per partition (index = first 4x4 raster of partition) */
    int16_t luma[16][16];      /* [raster blk][scan idx] levels (I16: scan 0 unused) */
    int16_t lumadc[16];        /* I16 DC levels, scan order */
    int16_t cdc[2][4];         /* chroma DC levels */
    int16_t cac[2][4][16];     /* chroma AC levels [plane][blk][scan idx], scan 0 unused */
    uint8_t pcm[384];          /* I_PCM samples (decoder) */
    int8_t sub_type[4];        /* P8x8 sub_mb_type (decoder) */
    uint16_t done4;            /* decoder: 4x4 blocks whose motion is already derived (MV pred availability) */
    int32_t slice_first;       /* first_mb_in_slice of the MB's slice (0: single-slice pictures, the encoder) */
    int8_t dbk_idc, dbk_a, dbk_b; /* its slice's disable_deblocking_filter_idc, FilterOffsetA / B */
} MBInfo;

/* Neighbour MB (mbx + dx, mby + dy) of MB (mbx, mby), dy <= 0: available (6.4.8 / 6.4.9) when it is
 * inside the picture and in the same slice. Slices are raster runs (no FMO), so a preceding MB is in
 * the current slice exactly when its address is >= the slice's first_mb_in_slice. */
static inline int mb_nb_avail(const MBInfo *mbs, int mbw, int mbx, int mby, int dx, int dy) {
    const int x = mbx + dx, y = mby + dy;
    if (x < 0 || y < 0 || x >= mbw) return 0;
    return y * mbw + x >= mbs[mby * mbw + mbx].slice_first;
}

/* ---------------- bit writer (MSB first) ---------------- */
typedef struct { uint8_t *buf; size_t cap, len; uint64_t acc; int nacc; } BW;
void bw_init(BW *b);
void bw_free(BW *b);
void bw_put(BW *b, uint32_t v, int n);
void bw_ue(BW *b, uint32_t v);
void bw_se(BW *b, int v);
void bw_trailing(BW *b);          /* rbsp_trailing_bits */
int64_t bw_bits(const BW *b);
int ue_len(uint32_t v);
int se_len(int v);
/* Append NAL: 4-byte start code, header, emulation-prevented RBSP. Returns bytes written. */
size_t nal_write(uint8_t *out, int nal_ref_idc, int nal_type, const uint8_t *rbsp, size_t n);

/* ---------------- bit reader ---------------- */
typedef struct { const uint8_t *buf; size_t len; size_t pos; int err; } BR;
uint32_t br_peek(BR *r, int n);
uint32_t br_get(BR *r, int n);
uint32_t br_ue(BR *r);
int br_se(BR *r);
int br_more_rbsp(BR *r);

/* ---------------- transforms / quant ---------------- */
void fdct4(const int d[16], int c[16]);                 /* forward core transform */
void idct4_add(const int c[16], uint8_t *dst, int stride, const uint8_t *pred, int pstride); /* 8.5.12 */
int quant4(int c, int qp, int pos, int intra);
int quant_dc4(int v, int qp, int intra);
int satd4(const int d[16]);
void dequant_block(const int16_t lvl_scan[16], int qp, int first, int out_raster[16]);
void luma_dc_dequant(const int16_t lvl_scan[16], int qp, int dc_raster[16]);   /* 8.5.10 */
void chroma_dc_dequant(const int16_t lvl[4], int qpc, int dc[4]);            /* 8.5.11 */

/* ---------------- intra prediction ---------------- */
typedef struct {
    uint8_t top[16 + 8]; /* p[x,-1], up to 16 (+8 top-right for 4x4) */
    uint8_t left[16];
    uint8_t tl;
    int has_top, has_left, has_tl, has_tr;
} IntraNb;
void pred4x4(const IntraNb *n, int mode, uint8_t pred[16]);   /* 8.3.1.2 */
int pred4x4_avail(const IntraNb *n, int mode);
void pred16x16(const IntraNb *n, int mode, uint8_t pred[256]); /* 8.3.3 */
int pred16x16_avail(const IntraNb *n, int mode);
void pred_chroma(const IntraNb *n, int mode, uint8_t pred[64]); /* 8.3.4 */
int pred_chroma_avail(const IntraNb *n, int mode);

/* ---------------- inter prediction ---------------- */
typedef struct { const uint8_t *y, *u, *v; int w, h, stride, cstride; } Pic; /* coded size */
void mc_luma(const Pic *ref, int x, int y, int bw, int bh, int mvx, int mvy, uint8_t *dst, int dstride);  /* 8.4.2.2.1 */
void mc_chroma(const uint8_t *plane, int cw, int ch, int cstride, int x, int y, int bw, int bh,
               int mvx, int mvy, uint8_t *dst, int dstride);                                              /* 8.4.2.2.2 */

/* ---------------- motion vector prediction ---------------- */
void mvp_16x16(const MBInfo *mbs, int mbw, int mbx, int mby, int out[2]);          /* 8.4.1.3 */
void pskip_mv(const MBInfo *mbs, int mbw, int mbx, int mby, int out[2]);          /* 8.4.1.1 */
void mvp_part(const MBInfo *mbs, const MBInfo *cur, int mbw, int mbx, int mby, int bx, int by,
              int pw, int ph, int shape, int out[2]);

/* ---------------- deblocking ---------------- */
void deblock_frame(uint8_t *y, uint8_t *u, uint8_t *v, int stride, int cstride, const MBInfo *mbs, int mbw, int mbh,
                  int cqp_off);   /* 8.7; each MB with its slice's dbk_idc / dbk_a / dbk_b */

/* ---------------- CAVLC ---------------- */
int nc_luma(const MBInfo *mbs, const MBInfo *cur, int mbw, int mbx, int mby, int ras);
int nc_chroma(const MBInfo *mbs, const MBInfo *cur, int mbw, int mbx, int mby, int plane, int blk);
void cavlc_write_block(BW *b, const int16_t *coef, int maxnum, int nc, int *total_out);  /* 9.2 */
int cavlc_read_block(BR *r, int16_t *coef, int maxnum, int nc);                         /* 9.2 */

#endif
