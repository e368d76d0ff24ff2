/*
 * include/h264mi.h -- C-ABI of libh264mi (openh264-wasm_amd/lib/libh264mi.so), the MI355X-native
 * H.264 encode/decode core that replaces openh264_wrapper.cpp + OpenH264 on the reference's hot
 * path. Plain C types only; no HIP or torch types in any signature.
 *
 * Part 1 -- drop-in wrapper surface. Each declaration below replaces the reference function of the
 * same name (file:line in /root/reference/openh264_wrapper.cpp) with identical argument meaning,
 * ownership and error behaviour, and is what the reference's JS glue binds through
 * Module.cwrap(...) (scripts/encoder_worker.js:27-29, scripts/decoder_worker.js:346-349):
 *   - init_* return 0 on success, -1 on failure;
 *   - the void functions report failure / "no picture" through zeroed out-params;
 *   - the encoded buffer is library-owned and valid until the next encode_* call;
 *   - decoder indices 0..31 (MAX_DECODERS); invalid index = silent no-op.
 */
#ifndef H264MI_H
#define H264MI_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* openh264_wrapper.cpp:198-228 */
int init_encoder(int width, int height, int bitrate);
/* openh264_wrapper.cpp:230-236 */
void force_key_frame(void);
/* openh264_wrapper.cpp:240-251 */
void deinit_decoder(int decoder_index);
/* openh264_wrapper.cpp:253-280 */
int init_decoder(int decoder_index);
/* openh264_wrapper.cpp:315-356 (RGBA8 input, converted with rgba_to_yuv :22-40 on the GPU) */
void encode_frame(unsigned char *rgba_data, int width, int height, unsigned char **out_data, int *out_size);
/* openh264_wrapper.cpp:358-389 (tight I420 input) */
void encode_frame_yuv_i420(unsigned char *yuv_i420_data, int width, int height, unsigned char **out_data, int *out_size);
/* openh264_wrapper.cpp:391-422 (RGBA8 output via yuv_to_rgba_optimized :150-195 on the GPU) */
void decode_frame_optimized(int decoder_index, unsigned char *encoded_data, int size, unsigned char *out_rgba_buffer,
                            int *out_width, int *out_height);
/* openh264_wrapper.cpp:424-464 (tight I420 output) */
void decode_frame_yuv_i420(int decoder_index, unsigned char *encoded_data, int size, unsigned char *out_yuv_buffer,
                           int *out_width, int *out_height);
/* openh264_wrapper.cpp:466-471 */
void free_buffer(void *ptr);

/*
 * Part 1b -- the same nine entry points on an explicit instance. The plain functions above act on
 * one process-wide default instance (the wrapper's globals, openh264_wrapper.cpp:11-18). The
 * reference runs one wasm instance per Worker, each with its own encoder and decoder_pool; a
 * native host that loads this library once per process (the N-API addon) keeps
 * that isolation by creating one instance per Worker. Same argument meaning and error behaviour.
 */
typedef struct h264mi_instance h264mi_instance;
h264mi_instance *h264mi_instance_create(void);
void h264mi_instance_destroy(h264mi_instance *inst);
int h264mi_i_init_encoder(h264mi_instance *inst, int width, int height, int bitrate);
void h264mi_i_force_key_frame(h264mi_instance *inst);
void h264mi_i_deinit_decoder(h264mi_instance *inst, int decoder_index);
int h264mi_i_init_decoder(h264mi_instance *inst, int decoder_index);
void h264mi_i_encode_frame(h264mi_instance *inst, unsigned char *rgba_data, int width, int height, unsigned char **out_data,
                           int *out_size);
void h264mi_i_encode_frame_yuv_i420(h264mi_instance *inst, unsigned char *yuv_i420_data, int width, int height,
                                    unsigned char **out_data, int *out_size);
void h264mi_i_decode_frame_optimized(h264mi_instance *inst, int decoder_index, unsigned char *encoded_data, int size,
                                     unsigned char *out_rgba_buffer, int *out_width, int *out_height);
void h264mi_i_decode_frame_yuv_i420(h264mi_instance *inst, int decoder_index, unsigned char *encoded_data, int size,
                                    unsigned char *out_yuv_buffer, int *out_width, int *out_height);
/* as the two decoders above, with the output buffer's capacity: a picture that does not fit is
   reported as "no picture" (zeroed width/height) instead of overrunning the buffer */
void h264mi_i_decode_frame_optimized_cap(h264mi_instance *inst, int decoder_index, unsigned char *encoded_data, int size,
                                         unsigned char *out_rgba_buffer, size_t out_cap, int *out_width, int *out_height);
void h264mi_i_decode_frame_yuv_i420_cap(h264mi_instance *inst, int decoder_index, unsigned char *encoded_data, int size,
                                        unsigned char *out_yuv_buffer, size_t out_cap, int *out_width, int *out_height);
/* pinned (page-locked) host memory for a host's heap: host<->device copies of frames run at DMA rate */
void *h264mi_host_alloc(size_t bytes);
void h264mi_host_free(void *ptr);

/*
 * Part 2 -- device-resident batch API (no reference counterpart: it is the MI355X-native way to
 * drive the same path for many independent streams whose frames/NAL units already live in HBM).
 * All "d_" pointers are device pointers; hip_stream is a hipStream_t (or NULL for an internal one).
 */
typedef struct h264mi_encoder h264mi_encoder;
h264mi_encoder *h264mi_enc_create(int width, int height, int bitrate, int nstreams, void *hip_stream);
void h264mi_enc_destroy(h264mi_encoder *e);
int h264mi_enc_force_idr(h264mi_encoder *e, int stream);            /* stream < 0: all */
int h264mi_enc_encode(h264mi_encoder *e, const void *d_frames);     /* async; nstreams tight I420 frames back to back */
/* rate-control frame skipping (on by default, as the wrapper's OpenH264): a skipped frame has 0 NAL bytes */
int h264mi_enc_set_frame_skip(h264mi_encoder *e, int enable);
int h264mi_enc_frames_skipped(h264mi_encoder *e, int stream);
/* OpenH264's GOM rate control exactly (WelsRcMbInitGom / WelsRcMbInfoUpdateGom): a P frame's GOM (2 MB rows from
   31 MBs wide) takes its QP from the bits of every MB before it, so a stream keeps one GOM in flight; off (the
   default unless H264MI_GOM_EXACT=1 at creation): this project's MB-row QP plan inside the frame's window */
int h264mi_enc_set_gom_exact(h264mi_encoder *e, int enable);
/* test hook: the next coded frame of stream fails as if its kernels had reported error code (> 0): it
   publishes 0 NAL bytes and the frame after it is an IDR. Code 3 fails it through enc_pack_kernel's
   RBSP-overflow branch itself (the early exit before the slice is assembled) */
int h264mi_enc_inject_error(h264mi_encoder *e, int stream, int code);
int h264mi_enc_sync(h264mi_encoder *e);
int h264mi_enc_nal_bytes(h264mi_encoder *e, int *out_bytes);        /* sync; -2 if a kernel reported an error */
const void *h264mi_enc_nal_ptr(h264mi_encoder *e, int stream);     /* Annex-B bytes of the last frame (device) */
const void *h264mi_enc_recon_ptr(h264mi_encoder *e, int stream);   /* deblocked reconstruction, coded size (device) */
const void *h264mi_enc_input_buffer(h264mi_encoder *e);            /* internal device input area (nstreams frames) */
size_t h264mi_enc_frame_bytes(h264mi_encoder *e);
int h264mi_enc_last_qp(h264mi_encoder *e, int stream);
/* the rate control's state after the last frame step (RC_BITRATE_MODE restated from h264.wasm),
   16 int32 in the oracle's h264o_enc_rc_state order: {skipped, QP, average QP, target bits, remaining bits,
   buffer fullness, continual skips, frame complexity, min / max frame QP, bits per frame, P frames, IDRs,
   skip flag, remaining weights, frames coded in the VGOP} */
int h264mi_enc_rc_state(h264mi_encoder *e, int stream, int *out16);
/* exact GOM mode, the last coded P frame: per GOM {QP, slice bits before it, target bits, last coded MB + 1}
   (4 int32 each, up to cap values; the oracle's h264o_enc_gom_state). Returns the GOM count (out NULL or the
   mode off: nothing copied) */
int h264mi_enc_gom_state(h264mi_encoder *e, int stream, int *out, int cap);
/* RcConvertQStep2Qp as the device computes it (thresholds; the wasm's musl-logf form is the oracle's) */
int h264mi_rc_qstep_to_qp(int qstep);
int h264mi_enc_mbinfo(h264mi_encoder *e, int stream, void *host_out); /* 128 B per MB (h264mi_types.h MbInfo) */
void *h264mi_enc_stream(h264mi_encoder *e);
const int *h264mi_enc_nal_size_dev(h264mi_encoder *e, int stream); /* device address of the NAL byte count */
int h264mi_enc_copy_nals(h264mi_encoder *e, void *d_dst, int slot_bytes, int *d_sizes); /* async: s -> d_dst+s*slot */
int h264mi_enc_set_timing(h264mi_encoder *e, int enable);          /* HIP events around the MB kernel */
int h264mi_enc_kernel_time(h264mi_encoder *e, double *ms_total, int *launches);

typedef struct h264mi_decoder h264mi_decoder;
h264mi_decoder *h264mi_dec_create(int width, int height, int nstreams, void *hip_stream);
/* frame-batched decoder: each call may carry up to max_frames access units per stream. Their slices
   are entropy-decoded concurrently (CAVLC parsing of a frame does not depend on other frames), then
   reconstructed in order; after the call each stream's picture is that of its last frame. */
h264mi_decoder *h264mi_dec_create_batch(int width, int height, int nstreams, int max_frames, void *hip_stream);
/* as h264mi_dec_create_batch with an explicit ring: groups slot groups of max_frames slots (2..16;
   0 = the default, up to 16) and parse_streams entropy-decoding streams (1..16). A caller that waits for
   every call (nothing to overlap) wants groups 2 and parse_streams 1: the C-ABI decoders use that. */
h264mi_decoder *h264mi_dec_create_ring(int width, int height, int nstreams, int max_frames, int groups, int parse_streams,
                                       void *hip_stream);
/* device memory held by a decoder (bytes), and by a C-ABI decoder slot of an instance (0: none yet) */
size_t h264mi_dec_device_bytes(h264mi_decoder *d);
size_t h264mi_i_decoder_device_bytes(h264mi_instance *inst, int decoder_index);
int h264mi_dec_max_frames(h264mi_decoder *d);
int h264mi_dec_ring_groups(h264mi_decoder *d);  /* slot groups in the decoder's ring */
/* number of HIP streams the entropy decoding of consecutive calls rotates over (default 3, 1..16):
   up to that many calls are entropy-decoded concurrently; synchronises the decoder */
int h264mi_dec_set_parse_streams(h264mi_decoder *d, int nstreams);
/* slice-data waves per picture (1..32, default 1; the C-ABI's decoder slots use 8): wave j of a picture
   parses its slices j, j + k, ... -- the slices of a multi-slice picture are independent CAVLC chains
   (7.4.3: no neighbour across a slice edge), so up to k of them are entropy-decoded concurrently */
int h264mi_dec_set_slice_waves(h264mi_decoder *d, int k);
/* streamed reconstruction: the first frame of each call is reconstructed row by row behind its slice data
   (the reconstruction rows wait on the GPU for the rows' records) instead of after the whole parse.
   mode 1: on -- the caller guarantees the reconstruction stream never occupies the parse CUs
   (h264mi_dec_set_parse_cus + a stream from h264mi_stream_create_cus(lo, hi, 1)); 0: off; -1 (the
   default): on while the reconstruction waves of all automatically streamed decoders of the process fit
   in h264mi_dec_set_streamed_budget's budget (one 1080p stream per decoder does), so that the waiting waves can
   never keep the parse from a CU. Applies to the calls enqueued after it (each call captures its mode); it
   synchronises the decoder's streams only when the decoder gives up an automatic share of the budget.
   Returns 0, -1 on a bad argument. h264mi_dec_streamed: the mode in effect. */
int h264mi_dec_set_streamed(h264mi_decoder *d, int mode);
int h264mi_dec_streamed(h264mi_decoder *d);
/* reconstruction gate, for the next decode call only: frame f (< count) of that call is reconstructed once the
   device uint32 *d_counter has reached target + f * step (wrap-safe comparison), or after limit_us microseconds
   of waiting -- a scheduling hint, never a correctness condition. With an encoder's rows counter
   (h264mi_enc_rows_counter) it starts each reconstruction in the tail of a concurrent encoder launch instead of
   beside its densest part. count 0 clears it. The gate is consumed by the next call whether that call succeeds or
   fails; the memory behind d_counter (an encoder's rows counter) must outlive that call's reconstruction (destroy
   the encoder only after synchronising the decoder). Returns 0, -1 on a bad argument. */
int h264mi_dec_set_recon_gate(h264mi_decoder *d, const uint32_t *d_counter, uint32_t target, uint32_t step, int count, int limit_us);
/* automatic streaming's process-wide budget in reconstruction waves (default: a quarter of dec_recon_kernel's
   resident wave slots on the current device, from its CU count and occupancy); waves <= 0 restores the
   default. Applies to later h264mi_dec_set_streamed(-1) / decoder creations. Returns the budget in effect. */
int h264mi_dec_set_streamed_budget(int waves);
/* entropy decoding on reserved CUs: the parse streams get the CU mask bits [cu_lo, cu_hi) (the runtime
   stripes mask bits over the XCDs); cu_lo == cu_hi removes the mask. Pair with wavefront streams from
   h264mi_stream_create_cus(cu_lo, cu_hi, 1) so that encoder / reconstruction workgroups stay off them. */
int h264mi_dec_set_parse_cus(h264mi_decoder *d, int cu_lo, int cu_hi);
/* a HIP stream restricted to CU mask bits [cu_lo, cu_hi), or to every other CU when complement != 0 */
void *h264mi_stream_create_cus(int cu_lo, int cu_hi, int complement);
void h264mi_stream_destroy(void *hip_stream);
void h264mi_dec_destroy(h264mi_decoder *d);
/* async; d_nal[s] / nal_bytes[s] (host array) per stream; a stream with nal_bytes 0 is skipped */
int h264mi_dec_decode(h264mi_decoder *d, const void *const *d_nal, const int *nal_bytes);
/* async; NAL sizes read from device memory (e.g. h264mi_enc_nal_size_dev): no host round trip */
int h264mi_dec_decode_dev(h264mi_decoder *d, const void *const *d_nal, const int *const *d_sizes);
/* async; nframes x nstreams access units, index f * nstreams + s; sizes from the host array
   nal_bytes or, if it is NULL, from device pointers d_sizes */
int h264mi_dec_decode_frames(h264mi_decoder *d, int nframes, const void *const *d_nal, const int *nal_bytes,
                             const int *const *d_sizes);
/* as h264mi_dec_decode_frames, but the inputs are ordered by ready_event (a hipEvent_t recorded by
   the producer) instead of by the decoder's stream: entropy decoding of this call may then overlap
   the reconstruction of the previous one. NULL = h264mi_dec_decode_frames. */
int h264mi_dec_decode_frames_after(h264mi_decoder *d, int nframes, const void *const *d_nal, const int *nal_bytes,
                                   const int *const *d_sizes, void *ready_event);
/* as above with several producers (e.g. encoder lanes on their own HIP streams): the inputs are
   ordered after every one of the nevents hipEvent_t's; nevents 0 = h264mi_dec_decode_frames */
int h264mi_dec_decode_frames_after_n(h264mi_decoder *d, int nframes, const void *const *d_nal, const int *nal_bytes,
                                     const int *const *d_sizes, void *const *ready_events, int nevents);
/* as above, and every frame's picture out: d_out[f * nstreams + s] (device, or NULL) receives frame f's
   cropped tight I420 picture (width x height x 3/2 bytes) once it is reconstructed, d_got[...] (device
   int, or NULL) 1 if that frame produced a picture, else 0 (the buffer is then left untouched) */
int h264mi_dec_decode_frames_out(h264mi_decoder *d, int nframes, const void *const *d_nal, const int *nal_bytes,
                                 const int *const *d_sizes, void *const *ready_events, int nevents, void *const *d_out,
                                 int *const *d_got);
int h264mi_dec_sync(h264mi_decoder *d);
/* HIP-event timing of the decoder's kernels (bench.py): which 0 = dec_recon_kernel, 1 = dec_parse_kernel */
int h264mi_dec_set_timing(h264mi_decoder *d, int enable);
int h264mi_dec_kernel_time(h264mi_decoder *d, int which, double *ms_total, int *launches);
int h264mi_dec_status(h264mi_decoder *d, int *got_pic);             /* sync; per-stream 1 = picture out */
/* diagnostics: parse-kernel cycle counters, 16 per (frame slot, stream): ring_groups x max_frames x nstreams
   slots (env H264MI_PARSE_PROF=1) */
int h264mi_dec_parse_profile(h264mi_decoder *d, uint64_t *out);
/* diagnostics: the padded motion-search reference planes of a stream (luma G, b, h, j then Cb, Cr;
   sizes (cw+80)(ch+64) and (cw/2+40)(ch/2+32)), built from the last coded frame */
int h264mi_enc_ref_planes(h264mi_encoder *e, int stream, void *host_out);
/* diagnostics: dec_recon_kernel section cycle counters, 16 totals (env H264MI_RECON_PROF=1) */
int h264mi_dec_recon_profile(h264mi_decoder *d, uint64_t *out);
/* diagnostics: section cycle counters, 64 totals: 0..15 and 32..51 enc_mb_kernel (tools/enc_prof.py names them), 16..21 the
   encoder's deblocking rows (env H264MI_ENC_PROF=1; H264MI_ENC_PROF_ROW=r counts MB row r only) */
int h264mi_enc_profile(h264mi_encoder *e, uint64_t *out);
/* diagnostics (env H264MI_ENC_TL=1 at creation): the last frame's enc_mb_kernel timeline, {start, end} per
   ticket on the GPU's 100 MHz clock (tickets 0 .. S*mbh-1 MB-row encoders, then the deblocking rows);
   out holds n >= 4 * S * mbh words. -1 when not enabled. */
int h264mi_enc_timeline(h264mi_encoder *e, uint64_t *out, int n);
/* the encoder's progress on the device: a uint32 counting the MB-row workgroups its launches have started since
   creation (S * mbh per frame step; launch k has started all its rows once it reaches (k + 1) * S * mbh).
   Read-only for callers; for h264mi_dec_set_recon_gate. */
const uint32_t *h264mi_enc_rows_counter(h264mi_encoder *e);
const void *h264mi_dec_picture_ptr(h264mi_decoder *d, int stream); /* deblocked picture, coded size (device) */
int h264mi_dec_coded_size(h264mi_decoder *d, int *cw, int *ch);
void *h264mi_dec_stream(h264mi_decoder *d);

/*
 * Device-resident NAL ring: the reference's SharedArrayBuffer frame pool
 * (app.js:52-53, :292-310: FRAME_BUFFER_POOL_SIZE buffers of MAX_FRAME_SIZE bytes + {size, ref_count}
 * per buffer) in HBM. Publishing follows encoder_worker.js:163-202 (size 0 -> nothing; larger than a
 * slot -> dropped; slot ref_count > 0 -> dropped; else copy, size, ref_count = consumers); releasing
 * follows decoder_worker.js:138-164 (Atomics.sub once per consumer). Decisions are taken on the device,
 * in stream order, so neither side synchronises the host. Ticket t uses slot t % slots (the slot
 * advances on a drop too, unlike the JS, so the host knows each ticket's slot without a round trip).
 */
typedef struct h264mi_nal_ring h264mi_nal_ring;
h264mi_nal_ring *h264mi_ring_create(int slots, int slot_bytes);
void h264mi_ring_destroy(h264mi_nal_ring *r);
/* async on the encoder's stream: publish stream's last NAL output; returns the ticket, -1 on bad
   arguments, -2 if ticket - 2*slots is not yet released by all its consumers */
long long h264mi_ring_publish(h264mi_nal_ring *r, h264mi_encoder *e, int stream, int consumers);
const void *h264mi_ring_nal_ptr(h264mi_nal_ring *r, long long ticket);  /* slot bytes (device) */
const int *h264mi_ring_size_dev(h264mi_nal_ring *r, long long ticket);  /* device size word: bytes, 0 = dropped */
/* async on hip_stream: one consumer is done with ticket (every consumer releases every ticket) */
int h264mi_ring_release(h264mi_nal_ring *r, long long ticket, void *hip_stream);
/* sync: counters, and ref_counts[slots] if non-NULL */
int h264mi_ring_stats(h264mi_nal_ring *r, int *published, int *dropped_busy, int *dropped_size, int *ref_counts);
/* Multi-GPU NAL gather (h264mi/shard.py): h264mi_nal_pack concatenates n staged access units (unit u at
   src + u * slot, sizes[u] bytes; sizes on the device) into dst in unit order, unit u at the sum of the
   sizes before it, so a rank sends one message per group; h264mi_nal_unpack is the inverse (rank 0 scatters
   a received packed buffer into slots). One kernel on hip_stream; n <= 8192. Returns 0, -1 on bad arguments. */
int h264mi_nal_pack(void *dst, const void *src, size_t slot, const int32_t *sizes, int n, void *hip_stream);
int h264mi_nal_unpack(void *dst, const void *src, size_t slot, const int32_t *sizes, int n, void *hip_stream);

/* edge colour conversions on the GPU, host buffers (openh264_wrapper.cpp:22-40 and :150-195) */
int h264mi_rgba_to_i420_host(const unsigned char *rgba, int width, int height, unsigned char *out_i420);
int h264mi_i420_to_rgba_host(const unsigned char *i420, int width, int height, unsigned char *out_rgba);

/* library self-description */
const char *h264mi_version(void);

#ifdef __cplusplus
}
#endif
#endif
