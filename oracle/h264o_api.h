/*
 * oracle/h264o_api.h -- TEST INFRASTRUCTURE ONLY. The CPU oracle's C API (loaded by tests/ via
 * ctypes, by __graft_entry__.smoke() as the checker, and by bench.py's cpu_baseline leg). The
 * product library (openh264-wasm_amd/, include/h264mi.h) never includes or links this.
 *
 * Parity status: the encoder restates OpenH264's algorithm at the wrapper's parameters but is
 * "parity unpinned" against OpenH264 itself (no reference tests, fixtures or runnable build --
 * see DESIGN.md §3); the decoder restates the normative H.264 decoding process.
 */
#ifndef H264O_API_H
#define H264O_API_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct H264OEnc H264OEnc;
typedef struct H264ODec H264ODec;

/* encoder: mirrors init_encoder / force_key_frame / encode_frame_yuv_i420 (openh264_wrapper.cpp) */
H264OEnc *h264o_enc_create(int w, int h, int bitrate);
void h264o_enc_destroy(H264OEnc *e);
void h264o_enc_force_idr(H264OEnc *e);
int h264o_enc_encode(H264OEnc *e, const uint8_t *i420, uint8_t *out, int cap); /* bytes, 0 = fail */
void h264o_enc_recon(const H264OEnc *e, uint8_t *i420_out);   /* deblocked recon, tight I420 */
void h264o_enc_mbinfo(const H264OEnc *e, int32_t *out);       /* 8 x int32 per MB */
int h264o_enc_last_qp(const H264OEnc *e);
/* frame skipping is on by default, as in the wrapper's OpenH264 configuration;
 * a skipped frame encodes to 0 bytes */
void h264o_enc_set_frame_skip(H264OEnc *e, int enable);
int h264o_enc_frames_skipped(const H264OEnc *e);
/* motion-search stage counters since creation: cross searches run, cross searches that moved the
 * vector, start points won by a neighbour candidate (A, B or C) */
/* {cross searches, cross searches that moved, neighbour start points won, P_Skip judges run, double-check skips,
 * intra MBs in P slices} */
void h264o_enc_me_stats(const H264OEnc *e, int32_t out[6]);
/* WelsCalculateSingleCtr4x4 (h264.wasm func 1011) over 16 levels in scan order */
int h264o_single_ctr(const int16_t lv[16]);
/* PredictSadSkip (h264.wasm func 331) over the neighbour cache {top-left, top, top-right, left}: reference index (-2
 * outside, -1 intra, 0 inter), skipped flag, skip SAD */
int h264o_predict_sad_skip(const int32_t ref[4], const int32_t sk[4], const int32_t sad[4]);
/* {mv min, mv max low bits, max level, luma single-ctr max, chroma single-ctr max} */
void h264o_pskip_constants(int32_t out[5]);
int h264o_rc_row_delta(int64_t row_bits, int64_t mean);
int h264o_rc_init_qp(int w, int h, int bitrate);
int h264o_rc_idr_params(int w, int h, int bitrate, int *rmin, int *rmax);  /* first IDR QP, IDR QP range */
void h264o_rc_constants(int32_t out[8]);  /* fps, QP min/max, frame window lower/upper, IDR window, IDR ratio, skip ratio */
int h264o_table(const char *name, double *out);  /* the oracle's copy of an OpenH264 table (entry count, -1 unknown) */
/* OpenH264's rate control restated from h264.wasm */
float h264o_logf(float x);                 /* musl logf (func 483) */
int h264o_rc_qstep2qp(int32_t qstep);      /* RcConvertQStep2Qp */
int h264o_enc_gom_state(const H264OEnc *e, int32_t *out, int cap);
/* intra mode decision pieces, for tests: AnalysisVaaInfoIntra of a 16x16 source block, the
 * Intra4x4 choice of one block from its nine mode costs and availability index, the pinned constants */
int h264o_vaa_intra_var(const uint8_t *src, int stride);
int h264o_i4_choose(const int32_t c[9], int avail_index, int32_t *cost);
void h264o_md_constants(int32_t out[3]);
void h264o_enc_set_gom_exact(H264OEnc *e, int enable);  /* MB QPs by OpenH264's GOM rule (funcs 1215 / 1206) */
void h264o_enc_rc_state(const H264OEnc *e, int32_t out[16]);
size_t h264o_write_sps(int w, int h, int bitrate, uint8_t *out);
int h264o_level_idc(int w, int h, int bitrate, int *cs3);
size_t h264o_write_pps(uint8_t *out);

/* decoder: mirrors init_decoder / decode_frame_yuv_i420 */
H264ODec *h264o_dec_create(void);
void h264o_dec_destroy(H264ODec *d);
/* picture output into out_i420 (tight, cropped) -> 1: picture decoded, 2: damaged access unit concealed by a copy of the last picture (frame-copy
 * error concealment), 0: no picture, -1: error with nothing to conceal */
int h264o_dec_decode(H264ODec *d, const uint8_t *data, int size, uint8_t *out_i420, int *w, int *h);
void h264o_dec_mbinfo(const H264ODec *d, int32_t *out);
void h264o_dec_nnz(const H264ODec *d, uint8_t *out);  /* 24 TotalCoeff bytes per MB of the last picture */

/* test-stream helpers (tests/streamgen.py): CAVLC bits of one residual block (0/1 per byte; returns
 * the bit count, -1 if cap is too small) and the coded_block_pattern codeNum of cbp (Table 9-4) */
int h264o_cavlc_bits(const int16_t *coef, int maxnum, int nc, uint8_t *bits, int cap);
int h264o_cbp_code(int cbp, int intra);

/* wrapper colour conversion: rgba_to_yuv (openh264_wrapper.cpp:22-40),
 * yuv_to_rgba_optimized (:150-195) */
void h264o_rgba_to_i420(const uint8_t *rgba, int w, int h, uint8_t *i420_out);
void h264o_i420_to_rgba(const uint8_t *y, const uint8_t *u, const uint8_t *v, int w, int h, int ys, int uvs,
                        uint8_t *rgba_out);

#ifdef __cplusplus
}
#endif
#endif
