/*
 * oracle/asan_driver.c -- TEST INFRASTRUCTURE ONLY. Sanitizer workload for the CPU oracle
 * (`make -C oracle asan-run`, built with -fsanitize=address,undefined; run by
 * tests/test_sanitizers.py). It drives every oracle entry point the tests use on inputs the
 * pytest suite does not reach cheaply:
 *   - encode -> decode round trips at odd geometries (cropping, 1-MB-wide pictures), with IDRs forced
 *     mid-stream and rate-control frame skipping on and off; the decoded picture must equal the
 *     encoder's reconstruction (the same invariant tests/test_oracle_golden.py checks);
 *   - the decoder on damaged input: truncated access units, random bit flips in the slice data,
 *     random bytes behind a valid start code, empty and 1-byte buffers -- it must return, never
 *     read or write out of bounds;
 *   - h264o_cavlc_bits on random blocks (all nC classes, both maxNumCoeff), a too-small cap;
 *   - the wrapper colour conversions (openh264_wrapper.cpp:22-40, :150-195) at odd strides.
 * Exit status 0 = every invariant held and the sanitizers reported nothing (they abort otherwise).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "h264o_api.h"

static uint32_t rng_state = 0x12345678u;
static uint32_t rnd(void) {  /* xorshift32 */
    uint32_t x = rng_state;
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    return rng_state = x;
}

/* moving hash texture: frame t is a window at (3t, 2t) of a fixed pattern, like h264mi/synth.py */
static void synth_frame(uint8_t *f, int w, int h, int t, uint32_t seed) {
    uint8_t *y = f, *u = f + (size_t)w * h, *v = u + (size_t)(w / 2) * (h / 2);
    for (int r = 0; r < h; r++)
        for (int c = 0; c < w; c++) {
            uint32_t x = (uint32_t)(((r + 2 * t) / 3) * 977 + ((c + 3 * t) / 3) * 131) ^ seed;
            x *= 0x9E3779B1u; x ^= x >> 15;
            y[(size_t)r * w + c] = (uint8_t)(64 + (x & 127));
        }
    for (int r = 0; r < h / 2; r++)
        for (int c = 0; c < w / 2; c++) {
            u[(size_t)r * (w / 2) + c] = (uint8_t)(128 + ((r + c + t) & 15));
            v[(size_t)r * (w / 2) + c] = (uint8_t)(120 + ((r * 3 + t) & 31));
        }
}

static int fails = 0;
#define CHECK(c, ...) do { if (!(c)) { fprintf(stderr, "FAIL: " __VA_ARGS__); fprintf(stderr, "\n"); fails++; } } while (0)

static void round_trip(int w, int h, int br, int nf, int skip) {
    const size_t F = (size_t)w * h * 3 / 2, cap = 4 * F + 4096;
    uint8_t *src = malloc(F), *rec = malloc(F), *pic = malloc(F), *out = malloc(cap);
    H264OEnc *e = h264o_enc_create(w, h, br);
    H264ODec *d = h264o_dec_create();
    CHECK(e && d, "create %dx%d", w, h);
    h264o_enc_set_frame_skip(e, skip);
    for (int t = 0; t < nf; t++) {
        synth_frame(src, w, h, t, (uint32_t)(w * 31 + h));
        if (t == nf / 2) h264o_enc_force_idr(e);
        const int n = h264o_enc_encode(e, src, out, (int)cap);
        CHECK(n >= 0, "encode %dx%d frame %d", w, h, t);
        if (n <= 0) continue;  /* skipped by the rate control */
        h264o_enc_recon(e, rec);
        int ow = 0, oh = 0;
        const int rc = h264o_dec_decode(d, out, n, pic, &ow, &oh);
        CHECK(rc == 1 && ow == w && oh == h, "decode %dx%d frame %d: rc %d %dx%d", w, h, t, rc, ow, oh);
        if (rc == 1) CHECK(memcmp(rec, pic, F) == 0, "decoded picture != reconstruction %dx%d frame %d", w, h, t);
        int32_t mi[8 * 4];
        if ((size_t)((w + 15) / 16) * ((h + 15) / 16) <= 4) { h264o_enc_mbinfo(e, mi); h264o_dec_mbinfo(d, mi); }
    }
    int32_t st[6];
    h264o_enc_me_stats(e, st);
    (void)h264o_enc_frames_skipped(e);
    (void)h264o_enc_last_qp(e);
    h264o_enc_destroy(e);
    h264o_dec_destroy(d);
    free(src); free(rec); free(pic); free(out);
}

/* a valid IDR + P pair at 176x144, then damaged copies of the P access unit */
static void damaged_streams(void) {
    const int w = 176, h = 144;
    const size_t F = (size_t)w * h * 3 / 2, cap = 4 * F;
    uint8_t *src = malloc(F), *pic = malloc(F), *au0 = malloc(cap), *au1 = malloc(cap), *bad = malloc(cap);
    H264OEnc *e = h264o_enc_create(w, h, 500000);
    h264o_enc_set_frame_skip(e, 0);
    synth_frame(src, w, h, 0, 7);
    const int n0 = h264o_enc_encode(e, src, au0, (int)cap);
    synth_frame(src, w, h, 1, 7);
    const int n1 = h264o_enc_encode(e, src, au1, (int)cap);
    CHECK(n0 > 0 && n1 > 0, "damaged_streams setup");
    for (int trial = 0; trial < 400; trial++) {
        H264ODec *d = h264o_dec_create();
        int ow, oh;
        (void)h264o_dec_decode(d, au0, n0, pic, &ow, &oh);
        int n = n1;
        memcpy(bad, au1, (size_t)n1);
        switch (trial % 4) {
        case 0: n = 1 + (int)(rnd() % (uint32_t)n1); break;                  /* truncated */
        case 1: for (int k = 0; k < 1 + trial % 9; k++) {                      /* bit flips after the start code + NAL header */
                    const int p = 5 + (int)(rnd() % (uint32_t)(n1 - 5));
                    bad[p] ^= (uint8_t)(1u << (rnd() & 7));
                } break;
        case 2: for (int p = 5; p < n1; p++) bad[p] = (uint8_t)rnd(); break;  /* garbage slice */
        case 3: n = 5 + (int)(rnd() % 64); for (int p = 4; p < n; p++) bad[p] = (uint8_t)rnd(); break;
        }
        const int rc = h264o_dec_decode(d, bad, n, pic, &ow, &oh);
        CHECK(rc >= -1 && rc <= 2, "damaged trial %d rc %d", trial, rc);
        if (rc == 1 || rc == 2) CHECK(ow == w && oh == h, "damaged trial %d size %dx%d", trial, ow, oh);
        h264o_dec_destroy(d);
    }
    H264ODec *d = h264o_dec_create();
    int ow, oh;
    const uint8_t one = 0;
    CHECK(h264o_dec_decode(d, &one, 1, pic, &ow, &oh) <= 0, "1-byte buffer");
    CHECK(h264o_dec_decode(d, au1, n1, pic, &ow, &oh) <= 0, "P slice without a reference");
    h264o_dec_destroy(d);
    h264o_enc_destroy(e);
    free(src); free(pic); free(au0); free(au1); free(bad);
}

static void cavlc_blocks(void) {
    uint8_t bits[1024];
    for (int trial = 0; trial < 20000; trial++) {
        int16_t c[16] = {0};
        const int maxnum = (trial & 1) ? 16 : 15;
        const int nz = (int)(rnd() % 17);
        for (int k = 0; k < nz; k++) {
            const int mag = (rnd() & 7) == 0 ? (int)(rnd() % 3000) : (int)(rnd() % 4);
            c[rnd() % (uint32_t)maxnum] = (int16_t)((rnd() & 1) ? mag : -mag);
        }
        static const int ncs[] = {0, 1, 2, 3, 4, 7, 8, 16};
        const int nc = ncs[trial % 8];
        const int n = h264o_cavlc_bits(c, maxnum, nc, bits, (int)sizeof bits);
        CHECK(n > 0, "cavlc_bits trial %d", trial);
        CHECK(h264o_cavlc_bits(c, maxnum, nc, bits, 1) == -1 || n <= 1, "cavlc_bits small cap trial %d", trial);
    }
    for (int cbp = 0; cbp < 48; cbp++) { (void)h264o_cbp_code(cbp, 0); (void)h264o_cbp_code(cbp, 1); }
}

static void colour(void) {
    static const int sizes[][2] = {{2, 2}, {6, 4}, {64, 48}, {178, 146}};
    for (int s = 0; s < 4; s++) {
        const int w = sizes[s][0], h = sizes[s][1];
        uint8_t *rgba = malloc((size_t)w * h * 4), *yuv = malloc((size_t)w * h * 3 / 2), *back = malloc((size_t)w * h * 4);
        for (size_t i = 0; i < (size_t)w * h * 4; i++) rgba[i] = (uint8_t)rnd();
        h264o_rgba_to_i420(rgba, w, h, yuv);
        const uint8_t *y = yuv, *u = yuv + (size_t)w * h, *v = u + (size_t)(w / 2) * (h / 2);
        h264o_i420_to_rgba(y, u, v, w, h, w, w / 2, back);
        for (size_t i = 3; i < (size_t)w * h * 4; i += 4) CHECK(back[i] == 255, "alpha %dx%d", w, h);
        free(rgba); free(yuv); free(back);
    }
}

int main(void) {
    static const int geo[][2] = {{16, 16}, {48, 32}, {98, 62}, {176, 144}, {352, 288}, {18, 130}};
    for (int g = 0; g < 6; g++) {
        round_trip(geo[g][0], geo[g][1], 300000, 5, 0);
        round_trip(geo[g][0], geo[g][1], 60000, 5, 1);
    }
    round_trip(176, 144, 30000000, 3, 0);  /* QP floor */
    damaged_streams();
    cavlc_blocks();
    colour();
    uint8_t ps[64];
    CHECK(h264o_write_sps(1920, 1080, 1000000, ps) > 0 && h264o_write_pps(ps) > 0, "parameter sets");
    for (int k = 0; k < 200; k++) (void)h264o_rc_qstep2qp((int32_t)(rnd() % 4000000));
    printf("asan_driver: %s (%d failures)\n", fails ? "FAIL" : "ok", fails);
    return fails ? 1 : 0;
}
