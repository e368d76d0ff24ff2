// h264mi_types.h -- HBM data layout shared by the host runtime and the gfx950 kernels.
//
// One "stream" = one independent encoder (or decoder) instance. Every per-stream buffer lives in
// HBM for the lifetime of the instance; a batch of S streams of the same geometry is driven by one
// launch per pipeline stage.
#pragma once
#include <stdint.h>

#define H264MI_MAX_STREAMS 256
#define H264MI_MB_SLOT_DWORDS 640      // per-MB CAVLC scratch (20480 bits; worst case < 17.6 kbit)
#define H264MI_ENC_MAX_MBW 512        // widest encoder picture in MBs (8192 samples, runtime_enc.inc enc_create)
#define H264MI_GRANULES_PER_MB 16      // row-to-row hand-off record (8-byte {tag,payload} granules)
#define H264MI_DBK_GRANULES_PER_MB 24  // deblocking hand-off (luma rows 12..15, chroma rows 6..7)
// Encoder reference planes are stored edge-padded (the picture's border samples replicated, the
// half-sample planes computed from the replicated picture), so every motion-search access stays
// inside the allocation without clamping. The column margins put the origin at 8 (mod 16) luma /
// 4 (mod 8) chroma bytes, so that the window strips the MB kernel loads are 16- / 8-byte aligned.
#define H264MI_LPADX 40
#define H264MI_LPADY 32
#define H264MI_CPADX 20
#define H264MI_CPADY 16

enum { MI_I4 = 0, MI_I16 = 1, MI_P16x16 = 2, MI_PSKIP = 3, MI_P16x8 = 4, MI_P8x16 = 5, MI_P8x8 = 6, MI_IPCM = 7 };

// Per-macroblock side information (128 B). Written by the MB wavefront kernel (encoder) or the
// parse kernel (decoder); read by CAVLC, reconstruction and deblocking. Decoder: the parse kernel
// writes a raw record (i4mode = mode codes in decoding order, 0xff = predicted; mv = mvd at each
// partition's first 4x4 block) and dec_recon_kernel rewrites it with resolved modes / vectors.
struct MbInfo {
    uint8_t type, qp, cbp, i16mode;
    uint8_t cmode, qpc, pad0, pad1;
    int8_t i4mode[16];   // raster 4x4 order; 2 (DC) for non-I4 macroblocks
    int8_t ref[4];       // per 8x8, -1 intra
    uint8_t nnz[24];     // TotalCoeff: luma raster 0..15, Cb 16..19, Cr 20..23
    int16_t mvd[2];      // encoder P16x16 mvd
    uint8_t sub[4];      // decoder P8x8 sub_mb_type
    int16_t mv[16][2];   // raster 4x4, quarter-pel
    int32_t pad2;        // decoder: slice identity + loop-filter parameters (MB_SLICE_*); encoder 0
};
static_assert(sizeof(MbInfo) == 128, "MbInfo layout");

// Quantised levels (scan order). Blocks whose TotalCoeff is 0 are not written and must not be read.
struct MbCoef {
    int16_t luma[16][16];   // raster luma block, scan index (I16: index 0 unused)
    int16_t cac[2][4][16];  // chroma AC, scan index 0 unused
    int16_t lumadc[16];     // I16 DC, scan order
    int16_t cdc[2][4];      // chroma DC
    int16_t pad[8];
};
static_assert(sizeof(MbCoef) == 832, "MbCoef layout");

// OpenH264's RC_BITRATE_MODE state of one stream, restated from the reference's h264.wasm
// (the oracle's Rc in oracle/h264o_enc.c follows the same functions; field comments name the wasm struct
// offsets: rc+N SWelsSvcRc, tl+N its SRCTemporal[0]). The host sets the constants at creation
// (RcInitSequenceParameter, RcInitTlWeight, RcUpdateBitrateFps, RcCalculateIdrQp's table part);
// enc_begin_kernel makes the skip decision and the picture init, enc_pack_kernel the picture update.
struct RcState {
    // constants
    int32_t nmb, mbw, mb_per_gom, gom_count;  // rc+156, rc+160 iNumberMbGom, rc+164 iGomSize
    int32_t skip_qp;                          // rc+188 iSkipQpValue
    int32_t c_bpf, c_min_bits_tl, c_max_bits_tl, c_buffer_size_skip;  // RcUpdateBitrateFps's results
    int32_t tl_weight, gop_num;               // tl+8, rc+180
    int32_t idr_lo, idr_hi, idr_table_qp;     // RcCalculateIdrQp: QP range (clipped) and the first IDR's table QP
    int32_t skip_en;                          // bEnableFrameSkip
    // state
    int32_t skip_flag, continual_skip;        // rc+280, rc+284
    int32_t bpf, min_bits_tl, max_bits_tl, buffer_size_skip;  // rc+40, tl+0, tl+4, rc+228 (set at the first IDR)
    int32_t remaining, vgop_bits, remaining_weights, gop_index, frame_coded_in_vgop;  // rc+60, +56, +112, +184, +172
    int32_t target, bits_level;               // rc+68, rc+72
    int32_t init_qp, last_qscale, qstep, avg_qp, min_frame_qp, max_frame_qp;  // rc+8, +224, +212, +144, +148, +152
    int32_t idr_num, intra_mb_count, pframe_num;  // rc+76, rc+88, tl+24
    int32_t prev_idx;                         // which psrc holds the last coded frame's luma
    int32_t target_bits_slice;                // sl+1372 iTargetBitsSlice (exact GOM mode)
    int64_t fullness;                         // rc+232
    int64_t intra_cmplx, intra_cmplx_mean;    // rc+80, rc+96
    int64_t linear_cmplx, frame_cmplx_mean;   // tl+16, tl+32
    int64_t frame_cmplx;                      // the frame's iFrameComplexity (enc_cmplx_kernel's GOM values)
};

// Per-stream encoder state (device resident; read/updated by the frame-begin and pack kernels).
struct EncState {
    int32_t cur_qp;        // QP of the frame being coded (iGlobalQp: slice QP)
    int32_t cur_idr;       // 1 if the frame being coded is IDR
    int32_t force_idr;     // host request (force_key_frame)
    int32_t first;         // no frame coded yet
    int32_t frame_num, idr_pic_id, poc;
    uint32_t epoch;        // hand-off tag, +1 per coded frame (never 0)
    int32_t bitrate;
    int32_t nal_bytes;     // bytes of the last coded frame (all NAL units, start codes included)
    int32_t err;           // nonzero: a kernel detected an error / timeout
    int32_t cur_skip;      // 1 if the frame being coded is skipped by the rate control (0 bytes out)
    int32_t skipped;       // frames skipped so far
    int32_t inject_err;    // test hook (h264mi_enc_inject_error): the next coded frame fails with this code
                           // (3: through the RBSP-overflow branch of enc_pack_kernel)
    int32_t sps_bytes, pps_bytes;
    uint8_t sps[64], pps[32];
    RcState rc;
};

// Per-stream encoder buffers for one frame step.
struct EncDesc {
    const uint8_t *src;     // tight I420 input (w x h), planes contiguous
    uint8_t *rec[3];        // unfiltered reconstruction (coded size)
    const uint8_t *ref[3];  // deblocked previous frame (coded size)
    uint8_t *dbk[3];        // deblocked output of this frame (coded size) -> next ref
    MbInfo *info;
    MbCoef *coef;
    uint64_t *gran;         // MB-row hand-off granules
    uint64_t *dgran;        // deblocking hand-off granules
    uint32_t *mbbits;       // per-MB CAVLC bits, H264MI_MB_SLOT_DWORDS each
    uint32_t *mblen;        // per-MB bit count (0 = P_Skip)
    uint32_t *rbsp;         // slice RBSP scratch (dwords)
    uint8_t *nal;           // Annex-B output of this frame
    EncState *st;
    int32_t nal_cap;
    int32_t rbsp_cap;       // dwords
    uint8_t *pl[4];         // padded luma reference planes at their origin: integer G, half-sample b
                            // (horizontal), h (vertical), j (centre); rebuilt from dbk after each frame
    uint8_t *plc[2];        // padded chroma reference planes (Cb, Cr) at their origin
    int32_t ps, psc;        // row strides of pl / plc
    int32_t pad3[2];
    uint64_t *egran;        // MB -> deblocking hand-off, 128 granules per MB (deblock.inc DbkSrcGranules)
    int32_t *rowqp;         // MB-row (GOM) QP offsets of the frame being coded (written by the previous pack)
    int32_t *rowbits;       // macroblock_layer() bits per MB row of the last coded frame
    uint64_t *rowq;         // per MB row: {epoch, QPY entering the row} granules (row r publishes r + 1)
    uint8_t *psrc[2];       // coded-size luma of the last coded frame and of the frame being coded (RcState::prev_idx):
                            // the preprocessing's reference picture for the frame complexity (enc_cmplx_kernel)
    uint32_t *gomc;         // per GOM: [0, G) SAD against the last coded source (P), [G, 2G) variance (I)
    uint64_t *bitg;         // exact GOM mode: per MB {epoch, macroblock_layer() bits} granules (the CAVLC waves)
    uint64_t *gomst;        // exact GOM mode: per GOM 4 granules {QP, slice bits before it, target bits, last coded MB + 1}
    // the P_Skip judge's memory: per MB the skip SAD of a skipped MB, -1 for any other, then one word
    // "the picture is P"; the reference picture's (last coded frame) and this frame's (swapped with ref / dbk)
    const int32_t *sksad_ref;
    int32_t *sksad_cur;
};

// One stream's padded reference planes and the picture they are built from (enc_planes.inc).
struct PlanesDesc {
    const uint8_t *src[2][3];  // candidate source pictures (Y, U, V, coded size), src[*parity & 1] (src[0] if parity == nullptr)
    const int32_t *parity;
    const int32_t *active;     // nullptr, or build only if nonzero (decoder: a picture was produced)
    uint8_t *pl[4];            // padded G, b, h, j planes at their origin (H264MI_LPADX/Y margins)
    uint8_t *plc[2];           // padded Cb, Cr at their origin (H264MI_CPADX/Y margins)
    int32_t ps, psc;
};

// Per-stream decoder state + buffers.
struct DecParams {          // SPS/PPS fields the slice layer needs (7.3.2.1, 7.3.2.2)
    int32_t have_sps, have_pps, mbw, mbh, log2_mfn, poc_type, log2_poc, crop[4];
    int32_t dpoaz;         // delta_pic_order_always_zero_flag (POC type 1)
    int32_t nref, qp, cqp, dbkc, red, bfp;
    int32_t has_ref;       // parse-side view: a picture has been decoded before (P slices allowed)
};
struct DecState {
    DecParams ps;          // parameter sets of the picture last reconstructed (host reads crop)
    DecParams psb[2];      // header chain: call k's dec_hdr_kernel reads psb[k & 1], its last wave writes psb[~k & 1]
    int32_t has_ref;       // reconstruction-side: a reference picture exists
    int32_t got_pic;       // 1 if the frame being (or last) reconstructed produced a picture
    int32_t nonref;        // that picture is a non-reference picture (nal_ref_idc 0): it is output, the reference stays
    int32_t err;           // of the current/last frame: 3 = parse error, 2 = unsupported, 1 = wavefront abort
    uint32_t epoch;        // hand-off tag, +1 per reconstructed picture
    int32_t parity;        // pic[parity] = the reference for the next P slice
    int32_t outpar;        // pic[outpar] = the last output picture (parity, or parity ^ 1 after a non-reference one)
};

// One decode call processes up to G frames per stream. Entropy decoding of a frame does not depend
// on other frames' pixels, so all G x S slices are parsed concurrently (one wave each); the
// reconstruction / deblocking passes then run frame by frame. Calls take G-slot groups of a ring of
// frame slots in turn and parse on two alternating HIP streams, so the slice data of consecutive
// calls is entropy-decoded concurrently while earlier calls reconstruct (runtime_dec.inc).
#define H264MI_MAX_NALS 40
#define H264MI_MAX_SLICES 32
struct NalEnt { int32_t start, end, type; uint32_t stop; };  // header byte index, payload end, type, RBSP stop-bit index
// One slice of a picture: dec_scan_kernel (nal), dec_hdr_kernel (header fields), dec_parse_kernel (ok, end_mb).
// info: what every MB record of the slice carries in MbInfo dword 31 (MB_SLICE_* below).
struct SliceEnt {
    int32_t nal;           // index into DecFrame::e
    int32_t first_mb;      // first_mb_in_slice
    int32_t slt;           // slice_type % 5 (0 P, 2 I)
    int32_t qp;            // SliceQPY
    uint32_t data_pos;     // RBSP bit index of slice_data()
    uint32_t info;         // first_mb | idc << 20 | (FilterOffsetA / 2 & 15) << 22 | (FilterOffsetB / 2 & 15) << 26
    int32_t ok;            // slice data parsed without error
    int32_t end_mb;        // one past its last macroblock
};
struct DecFrame {          // per (frame slot, stream): written by dec_scan_kernel, dec_hdr_kernel, dec_parse_kernel
    const uint8_t *nal;
    int32_t nbytes, nnal, nsl, err, got_pic, nonref;
    int32_t hdr_ok;        // parameter sets and every slice header parsed, slice data to follow
    int32_t anyp;          // some slice is a P slice (needs a reference)
    int32_t cqp;           // chroma_qp_index_offset
    int32_t pad_h[5];
    DecParams ps;          // parameter sets in effect for this frame's slices (cropping for the output)
    NalEnt e[H264MI_MAX_NALS];
    SliceEnt sl[H264MI_MAX_SLICES];
    // streamed reconstruction (runtime_dec.inc): {call tag << 32 | MB rows whose records are
    // visible to every CU} (H264MI_PROG_ABORT: the slice data failed, no picture), written by the slice-data
    // waves with agent-scope stores after an L2 write-back; sdone counts the waves done (| failures << 16)
    uint64_t prog;
    uint32_t sdone, pad_p;
};
#define H264MI_PROG_ABORT 0xFFFFFFFFu
// MbInfo dword 31 (pad2) of a decoded MB: its slice's first MB (neighbour availability: a preceding MB
// is in the same slice iff its address >= first) and loop-filter parameters (deblock.inc). 0 for the
// encoder's single-slice pictures.
#define MB_SLICE_FIRST(w) ((int)((w) & 0xFFFFFu))
#define MB_SLICE_IDC(w) ((int)(((w) >> 20) & 3u))
#define MB_SLICE_OFFA(w) (2 * (((int)((w) << 6)) >> 28))   // bits 22..25, signed, x2
#define MB_SLICE_OFFB(w) (2 * (((int)((w) << 2)) >> 28))   // bits 26..29, signed, x2
// one access unit; out / got (optional, device): where dec_output_kernel puts this frame's cropped tight
// I420 picture and its got-picture flag once the frame is reconstructed (every frame of a batched call)
struct DecInput { const uint8_t *nal; const int32_t *size_dev; int32_t size, pad; uint8_t *out; int32_t *got; };

struct DecDesc {
    uint8_t *cur[3];        // unfiltered reconstruction (coded size)
    uint8_t *pic[2][3];     // deblocked pictures (ping-pong by DecState::parity)
    MbInfo *info;
    MbCoef *coef;
    uint64_t *gran;
    uint64_t *dgran;
    DecState *st;
    DecFrame *frm;          // this frame slot's NAL table and parse result
    int32_t cw, ch;         // allocated coded size
    uint64_t *egran;        // MB -> deblocking hand-off, 128 granules per MB (per stream)
    uint8_t *pl[4];         // padded planes of the reference picture (as the encoder's, per stream)
    uint8_t *plc[2];
    int32_t ps, psc;
};
