/*
 * oracle/h264o_common.c -- TEST INFRASTRUCTURE ONLY (CPU oracle; see oracle/README.md).
 * Restatement of the normative H.264 building blocks used on the reference hot path
 * (OpenH264 EncodeFrame / DecodeFrameNoDelay behind openh264_wrapper.cpp:351,384,407,435).
 */
#include "h264o_common.h"
#include "h264o_tables.h"
#include <stdlib.h>
#include <string.h>

/* ================= bit writer ================= */
void bw_init(BW *b) { b->cap = 4096; b->buf = (uint8_t *)malloc(b->cap); b->len = 0; b->acc = 0; b->nacc = 0; }
void bw_free(BW *b) { free(b->buf); b->buf = NULL; }
static void bw_byte(BW *b, uint8_t x) {
    if (b->len == b->cap) { b->cap *= 2; b->buf = (uint8_t *)realloc(b->buf, b->cap); }
    b->buf[b->len++] = x;
}
void bw_put(BW *b, uint32_t v, int n) {
    if (n <= 0) return;
    if (n < 32) v &= (1u << n) - 1u;
    b->acc = (b->acc << n) | v;
    b->nacc += n;
    while (b->nacc >= 8) { b->nacc -= 8; bw_byte(b, (uint8_t)(b->acc >> b->nacc)); }
}
int ue_len(uint32_t v) { uint64_t k = (uint64_t)v + 1; int l = 0; while ((k >> l) > 1) l++; return 2 * l + 1; }
int se_len(int v) { return ue_len(v > 0 ? (uint32_t)(2 * v - 1) : (uint32_t)(-2 * v)); }
void bw_ue(BW *b, uint32_t v) {
    uint64_t k = (uint64_t)v + 1; int l = 0; while ((k >> l) > 1) l++;
    bw_put(b, 0, l);
    if (l + 1 > 32) { bw_put(b, (uint32_t)(k >> 32), l + 1 - 32); bw_put(b, (uint32_t)k, 32); }
    else bw_put(b, (uint32_t)k, l + 1);
}
void bw_se(BW *b, int v) { bw_ue(b, v > 0 ? (uint32_t)(2 * v - 1) : (uint32_t)(-2 * v)); }
void bw_trailing(BW *b) { bw_put(b, 1, 1); if (b->nacc) bw_put(b, 0, 8 - b->nacc); }
int64_t bw_bits(const BW *b) { return (int64_t)b->len * 8 + b->nacc; }

/* 7.4.1: emulation prevention -- insert 0x03 after two zero bytes when the next byte <= 3. */
size_t nal_write(uint8_t *out, int nal_ref_idc, int nal_type, const uint8_t *rbsp, size_t n) {
    size_t o = 0;
    out[o++] = 0; out[o++] = 0; out[o++] = 0; out[o++] = 1;
    out[o++] = (uint8_t)((nal_ref_idc << 5) | nal_type);
    int zeros = 0;
    for (size_t i = 0; i < n; i++) {
        if (zeros >= 2 && rbsp[i] <= 3) { out[o++] = 3; zeros = 0; }
        out[o++] = rbsp[i];
        zeros = rbsp[i] == 0 ? zeros + 1 : 0;
    }
    return o;
}

/* ================= bit reader ================= */
uint32_t br_peek(BR *r, int n) {
    uint64_t v = 0;
    size_t byte = r->pos >> 3;
    for (int i = 0; i < 5; i++) v = (v << 8) | (byte + i < r->len ? r->buf[byte + i] : 0);
    v <<= (r->pos & 7);            /* 40-bit window, top bit = current */
    return n == 0 ? 0 : (uint32_t)((v >> (40 - n)) & ((n == 32) ? 0xffffffffu : ((1u << n) - 1)));
}
uint32_t br_get(BR *r, int n) {
    if (n == 0) return 0;
    uint32_t v = br_peek(r, n);
    r->pos += n;
    if (r->pos > r->len * 8) r->err = 1;
    return v;
}
uint32_t br_ue(BR *r) {
    int lz = 0;
    while (lz < 32 && br_peek(r, 1) == 0) { r->pos++; lz++; if (r->pos > r->len * 8) { r->err = 1; return 0; } }
    if (lz >= 32) { r->err = 1; return 0; }
    r->pos++;
    uint32_t suf = br_get(r, lz);
    return (uint32_t)(((1ull << lz) - 1) + suf);
}
int br_se(BR *r) { uint32_t k = br_ue(r); return (k & 1) ? (int)((k + 1) >> 1) : -(int)(k >> 1); }
/* 7.2 more_rbsp_data(): true if there is more data before the rbsp_stop_one_bit. */
int br_more_rbsp(BR *r) {
    size_t total = r->len * 8;
    if (r->pos >= total) return 0;
    /* find last 1 bit in buffer */
    size_t last = r->len;
    while (last > 0 && r->buf[last - 1] == 0) last--;
    if (last == 0) return 0;
    uint8_t lb = r->buf[last - 1];
    int tz = 0; while (!((lb >> tz) & 1)) tz++;
    size_t stop = (last - 1) * 8 + (7 - tz);
    return r->pos < stop;
}

/* ================= transforms ================= */
/* forward 4x4 core transform (8.5.12 inverse's informative forward counterpart) */
void fdct4(const int d[16], int c[16]) {
    int t[16];
    for (int i = 0; i < 4; i++) {
        const int *s = d + 4 * i;
        int s0 = s[0] + s[3], s1 = s[1] + s[2], s2 = s[1] - s[2], s3 = s[0] - s[3];
        t[4 * i + 0] = s0 + s1; t[4 * i + 2] = s0 - s1;
        t[4 * i + 1] = 2 * s3 + s2; t[4 * i + 3] = s3 - 2 * s2;
    }
    for (int j = 0; j < 4; j++) {
        int s0 = t[j] + t[12 + j], s1 = t[4 + j] + t[8 + j], s2 = t[4 + j] - t[8 + j], s3 = t[j] - t[12 + j];
        c[j] = s0 + s1; c[8 + j] = s0 - s1; c[4 + j] = 2 * s3 + s2; c[12 + j] = s3 - 2 * s2;
    }
}
/* 8.5.12.2: rows (horizontal) first, then columns; (x + 32) >> 6; add prediction, clip. */
void idct4_add(const int c[16], uint8_t *dst, int stride, const uint8_t *pred, int pstride) {
    int t[16];
    for (int i = 0; i < 4; i++) {
        const int *d = c + 4 * i;
        int e0 = d[0] + d[2], e1 = d[0] - d[2], e2 = (d[1] >> 1) - d[3], e3 = d[1] + (d[3] >> 1);
        t[4 * i + 0] = e0 + e3; t[4 * i + 1] = e1 + e2; t[4 * i + 2] = e1 - e2; t[4 * i + 3] = e0 - e3;
    }
    for (int j = 0; j < 4; j++) {
        int e0 = t[j] + t[8 + j], e1 = t[j] - t[8 + j];
        int e2 = (t[4 + j] >> 1) - t[12 + j], e3 = t[4 + j] + (t[12 + j] >> 1);
        int r0 = e0 + e3, r1 = e1 + e2, r2 = e1 - e2, r3 = e0 - e3;
        dst[0 * stride + j] = (uint8_t)clip1(pred[0 * pstride + j] + ((r0 + 32) >> 6));
        dst[1 * stride + j] = (uint8_t)clip1(pred[1 * pstride + j] + ((r1 + 32) >> 6));
        dst[2 * stride + j] = (uint8_t)clip1(pred[2 * pstride + j] + ((r2 + 32) >> 6));
        dst[3 * stride + j] = (uint8_t)clip1(pred[3 * pstride + j] + ((r3 + 32) >> 6));
    }
}
/* Quantiser: OpenH264's table quantiser (WelsQuant4x4_c; tables from h264.wasm):
 * level = sign(c) * (((|c| + FF) * MF) >> 16), MF = OH_QUANT_MF[qp][pos & 7], FF = OH_QUANT_FF[qp +
 * 6 * intra][pos & 7] (intra rounding rows sit six rows down, wasm funcs 345 / 536). pos: raster. */
int quant4(int c, int qp, int pos, int intra) {
    int a = iabs(c);
    int l = ((a + OH_QUANT_FF[qp + (intra ? 6 : 0)][pos & 7]) * OH_QUANT_MF[qp][pos & 7]) >> 16;
    return c < 0 ? -l : l;
}
/* DC levels (I16x16 luma DC after the Hadamard, chroma 2x2 DC): WelsQuant4x4Dc / WelsHadamardQuant2x2
 * called with (int16)(FF[0] << 1) and MF[0] >> 1 (wasm funcs 265, 345, 534). */
int quant_dc4(int v, int qp, int intra) {
    int a = iabs(v);
    int ff = (int16_t)(OH_QUANT_FF[qp + (intra ? 6 : 0)][0] << 1), mf = OH_QUANT_MF[qp][0] >> 1;
    int l = ((a + ff) * mf) >> 16;
    return v < 0 ? -l : l;
}
/* SATD: (sum |H d H| + 1) >> 1 over a 4x4 difference block. */
int satd4(const int d[16]) {
    int t[16], s = 0;
    for (int i = 0; i < 4; i++) {
        const int *r = d + 4 * i;
        int a0 = r[0] + r[1], a1 = r[0] - r[1], a2 = r[2] + r[3], a3 = r[2] - r[3];
        t[4 * i + 0] = a0 + a2; t[4 * i + 1] = a1 + a3; t[4 * i + 2] = a0 - a2; t[4 * i + 3] = a1 - a3;
    }
    for (int j = 0; j < 4; j++) {
        int a0 = t[j] + t[4 + j], a1 = t[j] - t[4 + j], a2 = t[8 + j] + t[12 + j], a3 = t[8 + j] - t[12 + j];
        s += iabs(a0 + a2) + iabs(a1 + a3) + iabs(a0 - a2) + iabs(a1 - a3);
    }
    return (s + 1) >> 1;
}
/* 8.5.12.1 (flat scaling): d = (c * v) << (qp/6) for positions >= first (scan order input). */
void dequant_block(const int16_t lvl[16], int qp, int first, int out[16]) {
    for (int k = 0; k < 16; k++) out[k] = 0;
    for (int k = first; k < 16; k++) {
        int pos = ZIGZAG4[k];
        out[pos] = lvl[k] * DEQUANT_V[qp % 6][POS_CLASS[pos]] * (1 << (qp / 6));
    }
}
/* 8.5.10: inverse Hadamard of Intra16x16 DC + scaling. Output raster over 4x4 block grid. */
void luma_dc_dequant(const int16_t lvl[16], int qp, int dc[16]) {
    int c[16], t[16];
    for (int k = 0; k < 16; k++) c[ZIGZAG4[k]] = lvl[k];
    for (int i = 0; i < 4; i++) {
        int a = c[4 * i], b = c[4 * i + 1], e = c[4 * i + 2], d = c[4 * i + 3];
        t[4 * i + 0] = a + b + e + d; t[4 * i + 1] = a + b - e - d;
        t[4 * i + 2] = a - b - e + d; t[4 * i + 3] = a - b + e - d;
    }
    int v = DEQUANT_V[qp % 6][0], q6 = qp / 6;
    for (int j = 0; j < 4; j++) {
        int a = t[j], b = t[4 + j], e = t[8 + j], d = t[12 + j];
        int f[4] = {a + b + e + d, a + b - e - d, a - b - e + d, a - b + e - d};
        for (int i = 0; i < 4; i++) {
            int x = f[i] * v;
            dc[4 * i + j] = q6 >= 2 ? x * (1 << (q6 - 2)) : ((x + (1 << (1 - q6))) >> (2 - q6));
        }
    }
}
/* 8.5.11: 2x2 chroma DC inverse transform + scaling. */
void chroma_dc_dequant(const int16_t l[4], int qpc, int dc[4]) {
    int f0 = l[0] + l[1] + l[2] + l[3], f1 = l[0] - l[1] + l[2] - l[3];
    int f2 = l[0] + l[1] - l[2] - l[3], f3 = l[0] - l[1] - l[2] + l[3];
    int v = DEQUANT_V[qpc % 6][0], q6 = qpc / 6;
    dc[0] = (f0 * v * (1 << q6)) >> 1; dc[1] = (f1 * v * (1 << q6)) >> 1;
    dc[2] = (f2 * v * (1 << q6)) >> 1; dc[3] = (f3 * v * (1 << q6)) >> 1;
}

/* ================= intra prediction ================= */
static inline int T4(const IntraNb *n, int i) { return i < 0 ? n->tl : n->top[i]; }
static inline int L4(const IntraNb *n, int i) { return i < 0 ? n->tl : n->left[i]; }
int pred4x4_avail(const IntraNb *n, int m) {
    switch (m) {
    case 0: case 3: case 7: return n->has_top;
    case 1: case 8: return n->has_left;
    case 2: return 1;
    default: return n->has_top && n->has_left && n->has_tl;
    }
}
/* 8.3.1.2.x; n->top[4..7] must already hold the top-right (or replicated p[3,-1]). */
void pred4x4(const IntraNb *n, int m, uint8_t p[16]) {
    for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++) {
            int v = 0;
            switch (m) {
            case 0: v = n->top[x]; break;
            case 1: v = n->left[y]; break;
            case 2:
                if (n->has_top && n->has_left)
                    v = (n->top[0] + n->top[1] + n->top[2] + n->top[3] + n->left[0] + n->left[1] + n->left[2] + n->left[3] + 4) >> 3;
                else if (n->has_left) v = (n->left[0] + n->left[1] + n->left[2] + n->left[3] + 2) >> 2;
                else if (n->has_top) v = (n->top[0] + n->top[1] + n->top[2] + n->top[3] + 2) >> 2;
                else v = 128;
                break;
            case 3:
                if (x == 3 && y == 3) v = (n->top[6] + 3 * n->top[7] + 2) >> 2;
                else v = (n->top[x + y] + 2 * n->top[x + y + 1] + n->top[x + y + 2] + 2) >> 2;
                break;
            case 4:
                if (x > y) v = (T4(n, x - y - 2) + 2 * T4(n, x - y - 1) + T4(n, x - y) + 2) >> 2;
                else if (x < y) v = (L4(n, y - x - 2) + 2 * L4(n, y - x - 1) + L4(n, y - x) + 2) >> 2;
                else v = (n->top[0] + 2 * n->tl + n->left[0] + 2) >> 2;
                break;
            case 5: {
                int z = 2 * x - y;
                if (z >= 0 && !(z & 1)) v = (T4(n, x - (y >> 1) - 1) + T4(n, x - (y >> 1)) + 1) >> 1;
                else if (z >= 0) v = (T4(n, x - (y >> 1) - 2) + 2 * T4(n, x - (y >> 1) - 1) + T4(n, x - (y >> 1)) + 2) >> 2;
                else if (z == -1) v = (n->left[0] + 2 * n->tl + n->top[0] + 2) >> 2;
                else v = (L4(n, y - 1) + 2 * L4(n, y - 2) + L4(n, y - 3) + 2) >> 2;
                break;
            }
            case 6: {
                int z = 2 * y - x;
                if (z >= 0 && !(z & 1)) v = (L4(n, y - (x >> 1) - 1) + L4(n, y - (x >> 1)) + 1) >> 1;
                else if (z >= 0) v = (L4(n, y - (x >> 1) - 2) + 2 * L4(n, y - (x >> 1) - 1) + L4(n, y - (x >> 1)) + 2) >> 2;
                else if (z == -1) v = (n->left[0] + 2 * n->tl + n->top[0] + 2) >> 2;
                else v = (T4(n, x - 1) + 2 * T4(n, x - 2) + T4(n, x - 3) + 2) >> 2;
                break;
            }
            case 7:
                if (!(y & 1)) v = (n->top[x + (y >> 1)] + n->top[x + (y >> 1) + 1] + 1) >> 1;
                else v = (n->top[x + (y >> 1)] + 2 * n->top[x + (y >> 1) + 1] + n->top[x + (y >> 1) + 2] + 2) >> 2;
                break;
            case 8: {
                int z = x + 2 * y;
                if (z < 5 && !(z & 1)) v = (n->left[y + (x >> 1)] + n->left[y + (x >> 1) + 1] + 1) >> 1;
                else if (z < 5) v = (n->left[y + (x >> 1)] + 2 * n->left[y + (x >> 1) + 1] + n->left[y + (x >> 1) + 2] + 2) >> 2;
                else if (z == 5) v = (n->left[2] + 3 * n->left[3] + 2) >> 2;
                else v = n->left[3];
                break;
            }
            }
            p[4 * y + x] = (uint8_t)v;
        }
}
int pred16x16_avail(const IntraNb *n, int m) {
    switch (m) {
    case 0: return n->has_top;
    case 1: return n->has_left;
    case 2: return 1;
    default: return n->has_top && n->has_left && n->has_tl;
    }
}
void pred16x16(const IntraNb *n, int m, uint8_t p[256]) {
    if (m == 0) { for (int y = 0; y < 16; y++) for (int x = 0; x < 16; x++) p[16 * y + x] = n->top[x]; return; }
    if (m == 1) { for (int y = 0; y < 16; y++) for (int x = 0; x < 16; x++) p[16 * y + x] = n->left[y]; return; }
    if (m == 2) {
        int st = 0, sl = 0, v;
        for (int i = 0; i < 16; i++) { st += n->top[i]; sl += n->left[i]; }
        if (n->has_top && n->has_left) v = (st + sl + 16) >> 5;
        else if (n->has_left) v = (sl + 8) >> 4;
        else if (n->has_top) v = (st + 8) >> 4;
        else v = 128;
        memset(p, v, 256);
        return;
    }
    int H = 0, V = 0;
    for (int i = 0; i < 8; i++) {
        H += (i + 1) * (n->top[8 + i] - (6 - i >= 0 ? n->top[6 - i] : n->tl));
        V += (i + 1) * (n->left[8 + i] - (6 - i >= 0 ? n->left[6 - i] : n->tl));
    }
    int a = 16 * (n->left[15] + n->top[15]), b = (5 * H + 32) >> 6, c = (5 * V + 32) >> 6;
    for (int y = 0; y < 16; y++)
        for (int x = 0; x < 16; x++) p[16 * y + x] = (uint8_t)clip1((a + b * (x - 7) + c * (y - 7) + 16) >> 5);
}
int pred_chroma_avail(const IntraNb *n, int m) {
    switch (m) {
    case 0: return 1;
    case 1: return n->has_left;
    case 2: return n->has_top;
    default: return n->has_top && n->has_left && n->has_tl;
    }
}
void pred_chroma(const IntraNb *n, int m, uint8_t p[64]) {
    if (m == 0) {
        for (int by = 0; by < 2; by++)
            for (int bx = 0; bx < 2; bx++) {
                int st = 0, sl = 0, v;
                for (int i = 0; i < 4; i++) { st += n->top[4 * bx + i]; sl += n->left[4 * by + i]; }
                int t = n->has_top, l = n->has_left;
                if ((bx == 0 && by == 0) || (bx == 1 && by == 1)) {
                    if (t && l) v = (st + sl + 4) >> 3; else if (l) v = (sl + 2) >> 2; else if (t) v = (st + 2) >> 2; else v = 128;
                } else if (bx == 1 && by == 0) {
                    if (t) v = (st + 2) >> 2; else if (l) v = (sl + 2) >> 2; else v = 128;
                } else {
                    if (l) v = (sl + 2) >> 2; else if (t) v = (st + 2) >> 2; else v = 128;
                }
                for (int y = 0; y < 4; y++) for (int x = 0; x < 4; x++) p[8 * (4 * by + y) + 4 * bx + x] = (uint8_t)v;
            }
        return;
    }
    if (m == 1) { for (int y = 0; y < 8; y++) for (int x = 0; x < 8; x++) p[8 * y + x] = n->left[y]; return; }
    if (m == 2) { for (int y = 0; y < 8; y++) for (int x = 0; x < 8; x++) p[8 * y + x] = n->top[x]; return; }
    int H = 0, V = 0;
    for (int i = 0; i < 4; i++) {
        H += (i + 1) * (n->top[4 + i] - (2 - i >= 0 ? n->top[2 - i] : n->tl));
        V += (i + 1) * (n->left[4 + i] - (2 - i >= 0 ? n->left[2 - i] : n->tl));
    }
    int a = 16 * (n->left[7] + n->top[7]), b = (34 * H + 32) >> 6, c = (34 * V + 32) >> 6;
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) p[8 * y + x] = (uint8_t)clip1((a + b * (x - 3) + c * (y - 3) + 16) >> 5);
}

/* ================= motion compensation ================= */
static inline int refpx(const Pic *r, int x, int y) {
    return r->y[clip3(0, r->h - 1, y) * r->stride + clip3(0, r->w - 1, x)];
}
static inline int tap6(int a, int b, int c, int d, int e, int f) { return a - 5 * b + 20 * c + 20 * d - 5 * e + f; }
/* 8.4.2.2.1: luma sample interpolation with reference sample clamping (infinite edge extension). */
void mc_luma(const Pic *ref, int x0, int y0, int bw, int bh, int mvx, int mvy, uint8_t *dst, int ds) {
    int fx = mvx & 3, fy = mvy & 3;
    int X = x0 + (mvx >> 2), Y = y0 + (mvy >> 2);
    /* window arrays over (bh+1) x (bw+1) integer positions */
    int W = bw + 1, Hh = bh + 1;
    int G[17 * 17], B[17 * 17], HV[17 * 17], J[17 * 17], b1[22 * 17];
    for (int y = 0; y < Hh; y++)
        for (int x = 0; x < W; x++) {
            int gx = X + x, gy = Y + y;
            G[y * W + x] = refpx(ref, gx, gy);
            int bb = tap6(refpx(ref, gx - 2, gy), refpx(ref, gx - 1, gy), refpx(ref, gx, gy), refpx(ref, gx + 1, gy), refpx(ref, gx + 2, gy), refpx(ref, gx + 3, gy));
            B[y * W + x] = clip1((bb + 16) >> 5);
            int hh = tap6(refpx(ref, gx, gy - 2), refpx(ref, gx, gy - 1), refpx(ref, gx, gy), refpx(ref, gx, gy + 1), refpx(ref, gx, gy + 2), refpx(ref, gx, gy + 3));
            HV[y * W + x] = clip1((hh + 16) >> 5);
        }
    if ((fx == 2 && fy) || (fy == 2 && fx)) {
        /* unclipped b1 over rows Y-2 .. Y+Hh+2 */
        for (int y = -2; y < Hh + 3; y++)
            for (int x = 0; x < W; x++) {
                int gx = X + x, gy = Y + y;
                b1[(y + 2) * W + x] = tap6(refpx(ref, gx - 2, gy), refpx(ref, gx - 1, gy), refpx(ref, gx, gy), refpx(ref, gx + 1, gy), refpx(ref, gx + 2, gy), refpx(ref, gx + 3, gy));
            }
        for (int y = 0; y < Hh; y++)
            for (int x = 0; x < W; x++) {
                int j1 = tap6(b1[(y) * W + x], b1[(y + 1) * W + x], b1[(y + 2) * W + x], b1[(y + 3) * W + x], b1[(y + 4) * W + x], b1[(y + 5) * W + x]);
                J[y * W + x] = clip1((j1 + 512) >> 10);
            }
    }
#define AV(a, b) (((a) + (b) + 1) >> 1)
    for (int y = 0; y < bh; y++)
        for (int x = 0; x < bw; x++) {
            int i = y * W + x, v;
            switch (fy * 4 + fx) {
            case 0: v = G[i]; break;
            case 1: v = AV(G[i], B[i]); break;
            case 2: v = B[i]; break;
            case 3: v = AV(B[i], G[i + 1]); break;
            case 4: v = AV(G[i], HV[i]); break;
            case 5: v = AV(B[i], HV[i]); break;
            case 6: v = AV(B[i], J[i]); break;
            case 7: v = AV(B[i], HV[i + 1]); break;
            case 8: v = HV[i]; break;
            case 9: v = AV(HV[i], J[i]); break;
            case 10: v = J[i]; break;
            case 11: v = AV(J[i], HV[i + 1]); break;
            case 12: v = AV(HV[i], G[i + W]); break;
            case 13: v = AV(HV[i], B[i + W]); break;
            case 14: v = AV(J[i], B[i + W]); break;
            default: v = AV(HV[i + 1], B[i + W]); break;
            }
            dst[y * ds + x] = (uint8_t)v;
        }
#undef AV
}
/* 8.4.2.2.2: chroma eighth-sample bilinear interpolation. (x,y) block origin in chroma samples. */
void mc_chroma(const uint8_t *pl, int cw, int ch, int cs, int x0, int y0, int bw, int bh, int mvx, int mvy,
               uint8_t *dst, int ds) {
    int fx = mvx & 7, fy = mvy & 7;
    int X = x0 + (mvx >> 3), Y = y0 + (mvy >> 3);
    for (int y = 0; y < bh; y++)
        for (int x = 0; x < bw; x++) {
            int xa = clip3(0, cw - 1, X + x), xb = clip3(0, cw - 1, X + x + 1);
            int ya = clip3(0, ch - 1, Y + y), yb = clip3(0, ch - 1, Y + y + 1);
            int A = pl[ya * cs + xa], B = pl[ya * cs + xb], C = pl[yb * cs + xa], D = pl[yb * cs + xb];
            dst[y * ds + x] = (uint8_t)(((8 - fx) * (8 - fy) * A + fx * (8 - fy) * B + (8 - fx) * fy * C + fx * fy * D + 32) >> 6);
        }
}

/* ================= motion vector prediction (8.4.1.3) ================= */
/* Neighbour at luma offset (x,y) relative to current MB origin. cur may be partially filled; the
 * within-MB availability is given by done_mask (bit = raster 4x4 already predicted). */
typedef struct { int avail; int ref; int mv[2]; } NbMv;
static NbMv nb_mv(const MBInfo *mbs, const MBInfo *cur, unsigned done_mask, int mbw, int mbx, int mby, int x, int y) {
    NbMv r = {0, -1, {0, 0}};
    const MBInfo *m;
    int nx, ny;
    if (y < 0) {
        if (x < 0) { if (!mb_nb_avail(mbs, mbw, mbx, mby, -1, -1)) return r; m = &mbs[(mby - 1) * mbw + mbx - 1]; nx = x + 16; }
        else if (x < 16) { if (!mb_nb_avail(mbs, mbw, mbx, mby, 0, -1)) return r; m = &mbs[(mby - 1) * mbw + mbx]; nx = x; }
        else { if (!mb_nb_avail(mbs, mbw, mbx, mby, 1, -1)) return r; m = &mbs[(mby - 1) * mbw + mbx + 1]; nx = x - 16; }
        ny = y + 16;
    } else if (x < 0) {
        if (!mb_nb_avail(mbs, mbw, mbx, mby, -1, 0)) return r;
        m = &mbs[mby * mbw + mbx - 1]; nx = x + 16; ny = y;
    } else if (x >= 16) {
        return r;
    } else {
        int ras = (y >> 2) * 4 + (x >> 2);
        if (!((done_mask >> ras) & 1)) return r;
        r.avail = 1; r.ref = cur->ref[(y >> 3) * 2 + (x >> 3)];
        r.mv[0] = cur->mv[ras][0]; r.mv[1] = cur->mv[ras][1];
        return r;
    }
    r.avail = 1;
    if (mb_is_intra(m->type)) return r;
    int ras = (ny >> 2) * 4 + (nx >> 2);
    r.ref = m->ref[(ny >> 3) * 2 + (nx >> 3)];
    r.mv[0] = m->mv[ras][0]; r.mv[1] = m->mv[ras][1];
    return r;
}
/* shape: 0 generic/median, 1 = 16x8 partition (by==0 top, else bottom), 2 = 8x16 (bx==0 left). */
static void mvp_generic(const MBInfo *mbs, const MBInfo *cur, unsigned done, int mbw, int mbx, int mby,
                        int bx, int by, int pw, int shape, int refidx, int out[2]) {
    NbMv A = nb_mv(mbs, cur, done, mbw, mbx, mby, bx - 1, by);
    NbMv B = nb_mv(mbs, cur, done, mbw, mbx, mby, bx, by - 1);
    NbMv C = nb_mv(mbs, cur, done, mbw, mbx, mby, bx + pw, by - 1);
    if (!C.avail) C = nb_mv(mbs, cur, done, mbw, mbx, mby, bx - 1, by - 1);
    if (shape == 1) {
        if (by == 0 && B.ref == refidx) { out[0] = B.mv[0]; out[1] = B.mv[1]; return; }
        if (by != 0 && A.ref == refidx) { out[0] = A.mv[0]; out[1] = A.mv[1]; return; }
    } else if (shape == 2) {
        if (bx == 0 && A.ref == refidx) { out[0] = A.mv[0]; out[1] = A.mv[1]; return; }
        if (bx != 0 && C.ref == refidx) { out[0] = C.mv[0]; out[1] = C.mv[1]; return; }
    }
    if (!B.avail && !C.avail && A.avail) { B = A; C = A; }
    int n = (A.ref == refidx) + (B.ref == refidx) + (C.ref == refidx);
    if (n == 1) {
        const NbMv *s = A.ref == refidx ? &A : (B.ref == refidx ? &B : &C);
        out[0] = s->mv[0]; out[1] = s->mv[1];
        return;
    }
    out[0] = median3(A.mv[0], B.mv[0], C.mv[0]);
    out[1] = median3(A.mv[1], B.mv[1], C.mv[1]);
}
void mvp_16x16(const MBInfo *mbs, int mbw, int mbx, int mby, int out[2]) {
    mvp_generic(mbs, NULL, 0, mbw, mbx, mby, 0, 0, 16, 0, 0, out);
}
void mvp_part(const MBInfo *mbs, const MBInfo *cur, int mbw, int mbx, int mby, int bx, int by, int pw, int ph,
              int shape, int out[2]) {
    (void)ph;
    unsigned done = cur->done4;
    mvp_generic(mbs, cur, done, mbw, mbx, mby, bx, by, pw, shape, 0, out);
}
/* 8.4.1.1 P_Skip motion vector */
void pskip_mv(const MBInfo *mbs, int mbw, int mbx, int mby, int out[2]) {
    out[0] = out[1] = 0;
    NbMv A = nb_mv(mbs, NULL, 0, mbw, mbx, mby, -1, 0);
    NbMv B = nb_mv(mbs, NULL, 0, mbw, mbx, mby, 0, -1);
    if (!A.avail || !B.avail) return;  /* mbAddrA or mbAddrB not available: (0, 0) */
    if (A.ref == 0 && A.mv[0] == 0 && A.mv[1] == 0) return;
    if (B.ref == 0 && B.mv[0] == 0 && B.mv[1] == 0) return;
    mvp_16x16(mbs, mbw, mbx, mby, out);
}

/* ================= deblocking (8.7) ================= */
static void filter_line(uint8_t *q, int st, int bS, int alpha, int beta, int tc0, int chroma) {
    int p0 = q[-st], p1 = q[-2 * st], q0 = q[0], q1 = q[st];
    if (!(iabs(p0 - q0) < alpha && iabs(p1 - p0) < beta && iabs(q1 - q0) < beta)) return;
    if (bS < 4) {
        if (chroma) {
            int tc = tc0 + 1;
            int d = clip3(-tc, tc, ((q0 - p0) * 4 + (p1 - q1) + 4) >> 3);
            q[-st] = (uint8_t)clip1(p0 + d); q[0] = (uint8_t)clip1(q0 - d);
        } else {
            int p2 = q[-3 * st], q2 = q[2 * st];
            int ap = iabs(p2 - p0), aq = iabs(q2 - q0);
            int tc = tc0 + (ap < beta) + (aq < beta);
            int d = clip3(-tc, tc, ((q0 - p0) * 4 + (p1 - q1) + 4) >> 3);
            q[-st] = (uint8_t)clip1(p0 + d); q[0] = (uint8_t)clip1(q0 - d);
            if (ap < beta) q[-2 * st] = (uint8_t)(p1 + clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1));
            if (aq < beta) q[st] = (uint8_t)(q1 + clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1));
        }
    } else {
        if (chroma) {
            q[-st] = (uint8_t)((2 * p1 + p0 + q1 + 2) >> 2);
            q[0] = (uint8_t)((2 * q1 + q0 + p1 + 2) >> 2);
        } else {
            int p2 = q[-3 * st], q2 = q[2 * st], p3 = q[-4 * st], q3 = q[3 * st];
            int ap = iabs(p2 - p0), aq = iabs(q2 - q0);
            int small = iabs(p0 - q0) < ((alpha >> 2) + 2);
            if (ap < beta && small) {
                q[-st] = (uint8_t)((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
                q[-2 * st] = (uint8_t)((p2 + p1 + p0 + q0 + 2) >> 2);
                q[-3 * st] = (uint8_t)((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
            } else q[-st] = (uint8_t)((2 * p1 + p0 + q1 + 2) >> 2);
            if (aq < beta && small) {
                q[0] = (uint8_t)((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
                q[st] = (uint8_t)((p0 + q0 + q1 + q2 + 2) >> 2);
                q[2 * st] = (uint8_t)((2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3);
            } else q[0] = (uint8_t)((2 * q1 + q0 + p1 + 2) >> 2);
        }
    }
}
static int mb_qp_dbk(const MBInfo *m) { return m->type == MBT_IPCM ? 0 : m->qp; }
/* bS for the edge between 4x4 blocks (P MB m_p at raster rp) and (Q MB m_q at raster rq). 8.7.2.1 */
static int compute_bs(const MBInfo *mp, int rp, const MBInfo *mq, int rq, int mbedge) {
    if (mb_is_intra(mp->type) || mb_is_intra(mq->type)) return mbedge ? 4 : 3;
    if (mp->nnz[rp] || mq->nnz[rq]) return 2;
    int refp = mp->ref[((rp >> 2) >> 1) * 2 + ((rp & 3) >> 1)], refq = mq->ref[((rq >> 2) >> 1) * 2 + ((rq & 3) >> 1)];
    if (refp != refq) return 1;
    if (iabs(mp->mv[rp][0] - mq->mv[rq][0]) >= 4 || iabs(mp->mv[rp][1] - mq->mv[rq][1]) >= 4) return 1;
    return 0;
}
/* cqp_off: chroma_qp_index_offset (8.7.2.2: QPc of each MB from its QPY + offset; I_PCM QPY = 0).
 * Per MB q, its slice's parameters (8.7, 7.4.3): dbk_idc 1 -> q is not filtered; 2 -> its left / top
 * MB edge is not filtered when the MB across it belongs to another slice; FilterOffsetA/B = dbk_a /
 * dbk_b (slice_alpha_c0_offset_div2 << 1, slice_beta_offset_div2 << 1). */
void deblock_frame(uint8_t *Y, uint8_t *U, uint8_t *V, int ys, int cs, const MBInfo *mbs, int mbw, int mbh,
                   int cqp_off) {
    for (int my = 0; my < mbh; my++)
        for (int mx = 0; mx < mbw; mx++) {
            const MBInfo *q = &mbs[my * mbw + mx];
            if (q->dbk_idc == 1) continue;
            const int off_a = q->dbk_a, off_b = q->dbk_b;
            const int left_ok = mx > 0 && (q->dbk_idc != 2 || mbs[my * mbw + mx - 1].slice_first == q->slice_first);
            const int top_ok = my > 0 && (q->dbk_idc != 2 || mbs[(my - 1) * mbw + mx].slice_first == q->slice_first);
            int qpq = mb_qp_dbk(q), qcq = CHROMA_QP[clip3(0, 51, qpq + cqp_off)];
            int bs[2][4][4]; /* [dir][edge][segment] */
            for (int e = 0; e < 4; e++)
                for (int s = 0; s < 4; s++) {
                    /* vertical edge e (x = 4e), segment s (rows 4s..4s+3) */
                    if (e == 0) bs[0][0][s] = left_ok ? compute_bs(&mbs[my * mbw + mx - 1], s * 4 + 3, q, s * 4, 1) : 0;
                    else bs[0][e][s] = compute_bs(q, s * 4 + e - 1, q, s * 4 + e, 0);
                    if (e == 0) bs[1][0][s] = top_ok ? compute_bs(&mbs[(my - 1) * mbw + mx], 12 + s, q, s, 1) : 0;
                    else bs[1][e][s] = compute_bs(q, (e - 1) * 4 + s, q, e * 4 + s, 0);
                }
            for (int dir = 0; dir < 2; dir++) {
                for (int e = 0; e < 4; e++) {
                    if (e == 0 && ((dir == 0 && !left_ok) || (dir == 1 && !top_ok))) continue;
                    const MBInfo *p = e == 0 ? (dir == 0 ? &mbs[my * mbw + mx - 1] : &mbs[(my - 1) * mbw + mx]) : q;
                    int qpp = mb_qp_dbk(p);
                    int qpav = (qpp + qpq + 1) >> 1;
                    int ia = clip3(0, 51, qpav + off_a), ib = clip3(0, 51, qpav + off_b);
                    int alpha = DBK_ALPHA[ia], beta = DBK_BETA[ib];
                    for (int i = 0; i < 16; i++) {
                        int b = bs[dir][e][i >> 2];
                        if (!b) continue;
                        uint8_t *ptr = dir == 0 ? &Y[(my * 16 + i) * ys + mx * 16 + 4 * e] : &Y[(my * 16 + 4 * e) * ys + mx * 16 + i];
                        filter_line(ptr, dir == 0 ? 1 : ys, b, alpha, beta, b < 4 ? DBK_TC0[ia][b - 1] : 0, 0);
                    }
                    if (e & 1) continue; /* chroma edges at luma 0 and 8 only */
                    int qcp = CHROMA_QP[clip3(0, 51, qpp + cqp_off)];
                    int qcav = (qcp + qcq + 1) >> 1;
                    int ica = clip3(0, 51, qcav + off_a), icb = clip3(0, 51, qcav + off_b);
                    int ca = DBK_ALPHA[ica], cb = DBK_BETA[icb];
                    for (int pl = 0; pl < 2; pl++) {
                        uint8_t *P = pl ? V : U;
                        for (int i = 0; i < 8; i++) {
                            int b = bs[dir][e][i >> 1];
                            if (!b) continue;
                            int ce = e * 2; /* chroma edge offset: 0 or 4 */
                            uint8_t *ptr = dir == 0 ? &P[(my * 8 + i) * cs + mx * 8 + ce] : &P[(my * 8 + ce) * cs + mx * 8 + i];
                            filter_line(ptr, dir == 0 ? 1 : cs, b, ca, cb, b < 4 ? DBK_TC0[ica][b - 1] : 0, 1);
                        }
                    }
                }
            }
        }
}

/* ================= CAVLC (9.2) ================= */
int nc_luma(const MBInfo *mbs, const MBInfo *cur, int mbw, int mbx, int mby, int ras) {
    int bx = ras & 3, by = ras >> 2, na = -1, nb = -1;
    if (bx > 0) na = cur->nnz[ras - 1]; else if (mb_nb_avail(mbs, mbw, mbx, mby, -1, 0)) na = mbs[mby * mbw + mbx - 1].nnz[ras + 3];
    if (by > 0) nb = cur->nnz[ras - 4]; else if (mb_nb_avail(mbs, mbw, mbx, mby, 0, -1)) nb = mbs[(mby - 1) * mbw + mbx].nnz[ras + 12];
    if (na >= 0 && nb >= 0) return (na + nb + 1) >> 1;
    if (na >= 0) return na;
    if (nb >= 0) return nb;
    return 0;
}
int nc_chroma(const MBInfo *mbs, const MBInfo *cur, int mbw, int mbx, int mby, int pl, int blk) {
    int base = 16 + 4 * pl, bx = blk & 1, by = blk >> 1, na = -1, nb = -1;
    if (bx > 0) na = cur->nnz[base + blk - 1]; else if (mb_nb_avail(mbs, mbw, mbx, mby, -1, 0)) na = mbs[mby * mbw + mbx - 1].nnz[base + blk + 1];
    if (by > 0) nb = cur->nnz[base + blk - 2]; else if (mb_nb_avail(mbs, mbw, mbx, mby, 0, -1)) nb = mbs[(mby - 1) * mbw + mbx].nnz[base + blk + 2];
    if (na >= 0 && nb >= 0) return (na + nb + 1) >> 1;
    if (na >= 0) return na;
    if (nb >= 0) return nb;
    return 0;
}
static int nc_class(int nc) { return nc < 2 ? 0 : (nc < 4 ? 1 : (nc < 8 ? 2 : 3)); }

void cavlc_write_block(BW *b, const int16_t *coef, int maxnum, int nc, int *total_out) {
    int lv[16], run[16], tc = 0, t1 = 0, tz = 0;
    int last = -1;
    for (int i = maxnum - 1; i >= 0; i--) if (coef[i]) { last = i; break; }
    /* collect levels from highest frequency down, with run of zeros preceding each */
    for (int i = last; i >= 0; i--) {
        if (coef[i]) {
            lv[tc] = coef[i];
            int r = 0, k = i - 1;
            while (k >= 0 && coef[k] == 0) { r++; k--; }
            run[tc] = r; /* zeros below this coefficient until the next nonzero (or block start) */
            tc++;
        }
    }
    for (int i = 0; i < tc && i < 3; i++) { if (iabs(lv[i]) == 1) t1++; else break; }
    if (last >= 0) { tz = 0; for (int i = 0; i < last; i++) if (!coef[i]) tz++; }
    if (total_out) *total_out = tc;
    if (nc == -1) bw_put(b, CT_DC_CODE[tc * 4 + t1], CT_DC_LEN[tc * 4 + t1]);
    else { int c = nc_class(nc); bw_put(b, CT_CODE[c][tc * 4 + t1], CT_LEN[c][tc * 4 + t1]); }
    if (!tc) return;
    for (int i = 0; i < t1; i++) bw_put(b, lv[i] < 0, 1);
    int sl = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int i = t1; i < tc; i++) {
        int l = lv[i];
        int code = l > 0 ? 2 * l - 2 : -2 * l - 1;
        if (i == t1 && t1 < 3) code -= 2;
        if (sl == 0) {
            if (code < 14) { bw_put(b, 1, code + 1); }
            else if (code < 30) { bw_put(b, 1, 15); bw_put(b, code - 14, 4); }
            else { bw_put(b, 1, 16); bw_put(b, code - 30, 12); }
        } else {
            if (code < (15 << sl)) { bw_put(b, 1, (code >> sl) + 1); bw_put(b, code & ((1 << sl) - 1), sl); }
            else { bw_put(b, 1, 16); bw_put(b, code - (15 << sl), 12); }
        }
        if (sl == 0) sl = 1;
        if (iabs(l) > (3 << (sl - 1)) && sl < 6) sl++;
    }
    if (tc < maxnum) {
        if (nc == -1) bw_put(b, TZ_DC_CODE[tc - 1][tz], TZ_DC_LEN[tc - 1][tz]);
        else bw_put(b, TZ_CODE[tc - 1][tz], TZ_LEN[tc - 1][tz]);
    }
    int zl = tz;
    for (int i = 0; i < tc - 1 && zl > 0; i++) {
        int r = run[i];
        int t = zl > 7 ? 6 : zl - 1;
        bw_put(b, RB_CODE[t][r], RB_LEN[t][r]);
        zl -= r;
    }
}

/* VLC decode helper: find code among (len[],code[]) entries by peeking 16 bits. */
static int vlc_find(BR *r, const uint8_t *len, const uint8_t *code, int n) {
    uint32_t p = br_peek(r, 16);
    for (int i = 0; i < n; i++) {
        int l = len[i];
        if (!l) continue;
        if ((p >> (16 - l)) == code[i]) { r->pos += l; return i; }
    }
    r->err = 1;
    return 0;
}
int cavlc_read_block(BR *r, int16_t *coef, int maxnum, int nc) {
    for (int i = 0; i < maxnum; i++) coef[i] = 0;
    int idx;
    if (nc == -1) idx = vlc_find(r, CT_DC_LEN, CT_DC_CODE, 20);
    else { int c = nc_class(nc); idx = vlc_find(r, CT_LEN[c], CT_CODE[c], 68); }
    int tc = idx >> 2, t1 = idx & 3;
    if (!tc) return 0;
    int lv[16];
    for (int i = 0; i < t1; i++) lv[i] = br_get(r, 1) ? -1 : 1;
    int sl = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int i = t1; i < tc; i++) {
        int prefix = 0;
        while (br_get(r, 1) == 0) { prefix++; if (prefix > 32 || r->err) { r->err = 1; return tc; } }
        int ssize = (prefix == 14 && sl == 0) ? 4 : (prefix >= 15 ? prefix - 3 : sl);
        int code = (imin(15, prefix) << sl);
        if (ssize) code += (int)br_get(r, ssize);
        if (prefix >= 15 && sl == 0) code += 15;
        if (prefix >= 16) code += (1 << (prefix - 3)) - 4096;
        if (i == t1 && t1 < 3) code += 2;
        lv[i] = (code & 1) ? (-code - 1) >> 1 : (code + 2) >> 1;
        if (sl == 0) sl = 1;
        if (iabs(lv[i]) > (3 << (sl - 1)) && sl < 6) sl++;
    }
    int tz = 0;
    if (tc < maxnum) {
        if (nc == -1) tz = vlc_find(r, TZ_DC_LEN[tc - 1], TZ_DC_CODE[tc - 1], 4);
        else tz = vlc_find(r, TZ_LEN[tc - 1], TZ_CODE[tc - 1], 17 - tc);
    }
    int zl = tz, pos = tz + tc - 1;
    if (pos >= maxnum) { r->err = 1; return tc; }
    for (int i = 0; i < tc; i++) {
        int rb = 0;
        if (i < tc - 1 && zl > 0) {
            int t = zl > 7 ? 6 : zl - 1;
            rb = vlc_find(r, RB_LEN[t], RB_CODE[t], t == 6 ? 15 : t + 2);
        } else if (i == tc - 1) rb = zl;
        coef[pos] = (int16_t)lv[i];
        pos -= rb + 1;
        zl -= rb;
        if (pos < -1 || zl < 0) { r->err = 1; return tc; }
    }
    return tc;
}
