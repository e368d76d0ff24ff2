// h264.js -- drop-in for the Emscripten-generated scripts/h264.js, over the native libh264mi.
//
// The reference's glue (scripts/encoder_worker.js, scripts/decoder_worker.js, scripts/app.js) uses
// this surface of the Emscripten Module, and nothing else:
//   importScripts('h264.js')                               encoder_worker.js:23, decoder_worker.js:342
//   Module.onRuntimeInitialized = () => {...}              encoder_worker.js:25, decoder_worker.js:343
//   Module.cwrap(name, 'number' | null, ['number', ...])   encoder_worker.js:27-29, decoder_worker.js:346-349
//   Module._malloc(n) / Module._free(p)                    encoder_worker.js:99-108, decoder_worker.js:157-186
//   Module.getValue(p, 'i32')                              encoder_worker.js:164-165, decoder_worker.js:197-198
//   bare HEAPU8 (.set / .subarray with heap offsets)       encoder_worker.js:118, 144, 186; decoder_worker.js:163, 204, 208
// Here every pointer is still a byte offset into one heap, but the heap is pinned host memory owned
// by the N-API addon (lib/h264mi.node, napi/h264mi_napi.cc) and each JS environment (main thread
// or Worker) gets its own heap and its own encoder/decoder state, as each Worker of the reference
// gets its own wasm instance. The codec work runs on the GPU through include/h264mi.h.
'use strict';
(function (root) {
    const path = require('path');
    const addon = require(process.env.H264MI_NODE || path.join(__dirname, '..', 'lib', 'h264mi.node'));
    const Module = root.Module && typeof root.Module === 'object' ? root.Module : {};
    const bytes = Module.INITIAL_MEMORY || 256 * 1024 * 1024;  // Emscripten's option name for the heap size
    const buffer = addon.createHeap(bytes);
    const HEAP8 = new Int8Array(buffer), HEAPU8 = new Uint8Array(buffer);
    const HEAP16 = new Int16Array(buffer), HEAPU16 = new Uint16Array(buffer);
    const HEAP32 = new Int32Array(buffer), HEAPU32 = new Uint32Array(buffer);
    const HEAPF32 = new Float32Array(buffer), HEAPF64 = new Float64Array(buffer);
    Object.assign(Module, { HEAP8, HEAPU8, HEAP16, HEAPU16, HEAP32, HEAPU32, HEAPF32, HEAPF64, buffer });

    Module._malloc = (n) => addon.malloc(n);
    Module._free = (p) => addon.free(p);
    // the exports of the wasm build (h264.js@73423), Emscripten-style leading underscore
    const EXPORTS = ['init_encoder', 'force_key_frame', 'init_decoder', 'deinit_decoder', 'encode_frame',
        'encode_frame_yuv_i420', 'decode_frame_optimized', 'decode_frame_yuv_i420', 'free_buffer'];
    for (const n of EXPORTS) Module['_' + n] = addon[n];

    // All-number signatures return the raw export, as Emscripten's cwrap does (h264.js@71869).
    Module.cwrap = (ident, returnType, argTypes) => {
        const f = Module['_' + ident];
        if (typeof f !== 'function') throw new Error(`h264mi: no export named ${ident}`);
        const numeric = (t) => t === null || t === undefined || t === 'number';
        if (numeric(returnType) && (argTypes || []).every(numeric)) return f;
        throw new Error(`h264mi: cwrap(${ident}) with non-numeric types is not part of the wrapper's surface`);
    };
    Module.ccall = (ident, returnType, argTypes, args) => Module.cwrap(ident, returnType, argTypes)(...args);
    Module.getValue = (ptr, type = 'i8') => {
        switch (type) {
            case 'i1': case 'i8': return HEAP8[ptr];
            case 'i16': return HEAP16[ptr >> 1];
            case 'i32': case '*': return HEAP32[ptr >> 2];
            case 'float': return HEAPF32[ptr >> 2];
            case 'double': return HEAPF64[ptr >> 3];
            default: throw new Error(`h264mi: getValue type ${type}`);
        }
    };
    Module.setValue = (ptr, value, type = 'i8') => {
        switch (type) {
            case 'i1': case 'i8': HEAP8[ptr] = value; break;
            case 'i16': HEAP16[ptr >> 1] = value; break;
            case 'i32': case '*': HEAP32[ptr >> 2] = value; break;
            case 'float': HEAPF32[ptr >> 2] = value; break;
            case 'double': HEAPF64[ptr >> 3] = value; break;
            default: throw new Error(`h264mi: setValue type ${type}`);
        }
    };
    Module.version = addon.version();

    root.Module = Module;
    root.HEAPU8 = HEAPU8;  // the glue reads and writes the heap through the bare global
    // Emscripten initialises the runtime asynchronously; the glue assigns onRuntimeInitialized after
    // importScripts returns (encoder_worker.js:23-25), so the callback runs on a later turn.
    setImmediate(() => {
        Module.calledRun = true;
        if (typeof Module.onRuntimeInitialized === 'function') Module.onRuntimeInitialized();
    });
    if (typeof module === 'object' && module.exports) module.exports = Module;
})(typeof globalThis !== 'undefined' ? globalThis : this);
