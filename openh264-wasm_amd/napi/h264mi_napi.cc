// h264mi_napi.cc -- N-API addon: the reference's Emscripten heap model over libh264mi.
//
// The JS glue (scripts/encoder_worker.js, scripts/decoder_worker.js) talks to the codec through
// cwrap'ed functions whose pointer arguments are byte offsets into one linear heap (HEAPU8), and
// reads results back from that heap (Module.getValue(ptr, 'i32'), HEAPU8.subarray(...)). This addon
// keeps that contract for a native build: each JS environment (main thread or Worker) owns
//   * a heap: pinned host memory (h264mi_host_alloc) exposed to JS as an external ArrayBuffer, with a
//     first-fit allocator behind _malloc / _free (16-byte aligned, offset 0 = NULL);
//   * an h264mi_instance: its own encoder and 32-slot decoder pool, as each Worker of the reference
//     owns a separate wasm instance (openh264_wrapper.cpp:11-18 globals per instance).
// Every entry point takes heap offsets, bounds-checks them, translates them to pointers and calls the
// C-ABI (include/h264mi.h). The encoder's library-owned output (openh264_wrapper.cpp:282-311) is
// mirrored into a grow-only heap block whose offset is written through the out_data slot, as the
// wasm build's pointer is.
#include <node_api.h>
#include <cstdint>
#include <cstring>
#include <map>
#include "../../include/h264mi.h"
#include "heap.h"

namespace {

struct EnvData {
    Heap heap;
    h264mi_instance *inst = nullptr;
    uint32_t enc_out = 0, enc_out_cap = 0;  // heap mirror of the encoder's output buffer
};

void env_finalize(napi_env, void *data, void *) {
    EnvData *d = (EnvData *)data;
    h264mi_instance_destroy(d->inst);
    if (d->heap.base) h264mi_host_free(d->heap.base);
    delete d;
}

EnvData *env_data(napi_env env) {
    void *p = nullptr;
    napi_get_instance_data(env, &p);
    return (EnvData *)p;
}

bool args(napi_env env, napi_callback_info info, int64_t *v, size_t n) {
    napi_value a[8];
    size_t argc = 8;
    if (napi_get_cb_info(env, info, &argc, a, nullptr, nullptr) != napi_ok || argc < n) {
        napi_throw_type_error(env, nullptr, "h264mi: wrong number of arguments");
        return false;
    }
    for (size_t i = 0; i < n; i++) {
        double x = 0;
        if (napi_get_value_double(env, a[i], &x) != napi_ok) {
            napi_throw_type_error(env, nullptr, "h264mi: arguments are numbers (heap offsets / ints)");
            return false;
        }
        // NaN / +-Inf / |x| > 2^53 become -1 (rejected by every bounds check) instead of an undefined conversion
        v[i] = (x == x && x >= -9007199254740992.0 && x <= 9007199254740992.0) ? (int64_t)x : -1;
    }
    return true;
}
napi_value num(napi_env env, double x) { napi_value r; napi_create_double(env, x, &r); return r; }
napi_value undef(napi_env env) { napi_value r; napi_get_undefined(env, &r); return r; }
void put_i32(Heap &h, int64_t off, int32_t v) { if (h.ok(off, 4)) memcpy(h.at(off), &v, 4); }

// createHeap(bytes) -> ArrayBuffer over this environment's pinned heap (once per environment)
napi_value createHeap(napi_env env, napi_callback_info info) {
    int64_t a[1];
    if (!args(env, info, a, 1)) return nullptr;
    EnvData *d = env_data(env);
    if (d->heap.base) { napi_throw_error(env, nullptr, "h264mi: heap already created"); return nullptr; }
    if (a[0] < 4096 || a[0] > ((int64_t)1 << 31)) { napi_throw_range_error(env, nullptr, "h264mi: heap size"); return nullptr; }
    uint8_t *b = (uint8_t *)h264mi_host_alloc((size_t)a[0]);
    if (!b) { napi_throw_error(env, nullptr, "h264mi: pinned heap allocation failed"); return nullptr; }
    memset(b, 0, (size_t)a[0]);
    d->heap.init(b, (size_t)a[0]);
    napi_value ab;
    napi_create_external_arraybuffer(env, b, (size_t)a[0], nullptr, nullptr, &ab);
    return ab;
}
napi_value js_malloc(napi_env env, napi_callback_info info) {
    int64_t a[1];
    if (!args(env, info, a, 1)) return nullptr;
    EnvData *d = env_data(env);
    return num(env, (a[0] < 0 || !d->heap.base) ? 0 : d->heap.alloc((size_t)a[0]));
}
napi_value js_free(napi_env env, napi_callback_info info) {
    int64_t a[1];
    if (!args(env, info, a, 1)) return nullptr;
    if (a[0] > 0) env_data(env)->heap.release((uint32_t)a[0]);
    return undef(env);
}

// ---- the wrapper surface (openh264_wrapper.cpp), offsets in, offsets out
napi_value js_init_encoder(napi_env env, napi_callback_info info) {
    int64_t a[3];
    if (!args(env, info, a, 3)) return nullptr;
    return num(env, h264mi_i_init_encoder(env_data(env)->inst, (int)a[0], (int)a[1], (int)a[2]));
}
napi_value js_force_key_frame(napi_env env, napi_callback_info) {
    h264mi_i_force_key_frame(env_data(env)->inst);
    return undef(env);
}
napi_value js_init_decoder(napi_env env, napi_callback_info info) {
    int64_t a[1];
    if (!args(env, info, a, 1)) return nullptr;
    return num(env, h264mi_i_init_decoder(env_data(env)->inst, (int)a[0]));
}
napi_value js_deinit_decoder(napi_env env, napi_callback_info info) {
    int64_t a[1];
    if (!args(env, info, a, 1)) return nullptr;
    h264mi_i_deinit_decoder(env_data(env)->inst, (int)a[0]);
    return undef(env);
}
template <bool RGBA> napi_value js_encode(napi_env env, napi_callback_info info) {
    int64_t a[5];  // (in, width, height, out_data_slot, out_size_slot)
    if (!args(env, info, a, 5)) return nullptr;
    EnvData *d = env_data(env);
    Heap &h = d->heap;
    put_i32(h, a[3], 0);
    put_i32(h, a[4], 0);
    if (a[1] <= 0 || a[2] <= 0 || a[1] > 16384 || a[2] > 16384) return undef(env);  // (the product cannot overflow)
    const int64_t in_bytes = RGBA ? a[1] * a[2] * 4 : a[1] * a[2] * 3 / 2;
    if (!h.ok(a[0], in_bytes) || !h.ok(a[3], 4) || !h.ok(a[4], 4)) return undef(env);
    unsigned char *out = nullptr;
    int n = 0;
    if (RGBA) h264mi_i_encode_frame(d->inst, h.at(a[0]), (int)a[1], (int)a[2], &out, &n);
    else h264mi_i_encode_frame_yuv_i420(d->inst, h.at(a[0]), (int)a[1], (int)a[2], &out, &n);
    if (n <= 0 || !out) return undef(env);  // failure or skipped frame: size 0 (openh264_wrapper.cpp:360-361)
    if ((uint32_t)n > d->enc_out_cap) {
        if (d->enc_out) h.release(d->enc_out);
        d->enc_out = h.alloc((size_t)n);
        d->enc_out_cap = d->enc_out ? (uint32_t)n : 0;
        if (!d->enc_out) return undef(env);
    }
    memcpy(h.at(d->enc_out), out, (size_t)n);
    put_i32(h, a[3], (int32_t)d->enc_out);
    put_i32(h, a[4], n);
    return undef(env);
}
template <bool RGBA> napi_value js_decode(napi_env env, napi_callback_info info) {
    int64_t a[6];  // (decoder_index, nal, size, out, out_w_slot, out_h_slot)
    if (!args(env, info, a, 6)) return nullptr;
    EnvData *d = env_data(env);
    Heap &h = d->heap;
    put_i32(h, a[4], 0);
    put_i32(h, a[5], 0);
    if (a[2] <= 0 || !h.ok(a[1], a[2]) || !h.ok(a[3], 1) || !h.ok(a[4], 4) || !h.ok(a[5], 4)) return undef(env);
    int w = 0, hh = 0;
    // the caller sizes `out` by the configured geometry (decoder_worker.js:171-181); the library
    // writes w*h*1.5 (or *4) bytes of the decoded picture and refuses a picture that would run past
    // the end of the heap
    const size_t cap = h.size - (size_t)a[3];
    if (RGBA) h264mi_i_decode_frame_optimized_cap(d->inst, (int)a[0], h.at(a[1]), (int)a[2], h.at(a[3]), cap, &w, &hh);
    else h264mi_i_decode_frame_yuv_i420_cap(d->inst, (int)a[0], h.at(a[1]), (int)a[2], h.at(a[3]), cap, &w, &hh);
    put_i32(h, a[4], w);
    put_i32(h, a[5], hh);
    return undef(env);
}
napi_value js_free_buffer(napi_env env, napi_callback_info info) {
    int64_t a[1];
    if (!args(env, info, a, 1)) return nullptr;
    // openh264_wrapper.cpp:466-471 frees a heap pointer; heap blocks come from _malloc
    if (a[0] > 0) env_data(env)->heap.release((uint32_t)a[0]);
    return undef(env);
}
napi_value js_version(napi_env env, napi_callback_info) {
    napi_value r;
    napi_create_string_utf8(env, h264mi_version(), NAPI_AUTO_LENGTH, &r);
    return r;
}

napi_value Init(napi_env env, napi_value exports) {
    EnvData *d = new EnvData();
    d->inst = h264mi_instance_create();
    napi_set_instance_data(env, d, env_finalize, nullptr);
    const napi_property_descriptor p[] = {
        {"createHeap", nullptr, createHeap, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"malloc", nullptr, js_malloc, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"free", nullptr, js_free, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"init_encoder", nullptr, js_init_encoder, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"force_key_frame", nullptr, js_force_key_frame, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"init_decoder", nullptr, js_init_decoder, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"deinit_decoder", nullptr, js_deinit_decoder, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"encode_frame", nullptr, js_encode<true>, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"encode_frame_yuv_i420", nullptr, js_encode<false>, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"decode_frame_optimized", nullptr, js_decode<true>, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"decode_frame_yuv_i420", nullptr, js_decode<false>, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"free_buffer", nullptr, js_free_buffer, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"version", nullptr, js_version, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
    };
    napi_define_properties(env, exports, sizeof(p) / sizeof(p[0]), p);
    return exports;
}

}  // namespace

NAPI_MODULE_INIT() { return Init(env, exports); }
