// replay_workers.js -- headless replay of the reference glue's worker protocol over the native Module
// (openh264-wasm_amd/js/h264.js -> lib/h264mi.node -> libh264mi.so on the GPU).
//
// Main thread (the part of scripts/app.js that feeds workers): a SharedArrayBuffer ring of
// FRAME_BUFFER_POOL_SIZE x MAX_FRAME_SIZE slots plus an Int32Array control block {size, refcount}
// per slot (app.js:52-53, 292-310); one encoder Worker; D decoder Workers that decode the same
// stream under global stream indices 0..S-1 split across them (decoder_worker.js:51).
// Workers: the call sequences of scripts/encoder_worker.js (:25-31 cwrap, :93-100 init, :127-147
// encode_yuv, :163-202 read-back through getValue + HEAPU8 into the ring) and scripts/decoder_worker.js
// (:343-361 cwrap + 4-byte slots, :137-225 decode into a heap buffer, :197-208 read-back, :295-309
// cleanup), each Worker with its own heap and codec instance, as with separate wasm instances.
//
//   node replay_workers.js <in.yuv> <width> <height> <frames> <outdir> <streams> <decoder_workers> [rgba]
// writes <outdir>/enc.h264 (all access units), <outdir>/dec_<s>.yuv or .rgba per stream index s.
'use strict';
const path = require('path');
const fs = require('fs');
const { Worker, isMainThread, parentPort, workerData } = require('worker_threads');
const JS_DIR = path.join(__dirname, '..', '..', 'openh264-wasm_amd', 'js');
const FRAME_BUFFER_POOL_SIZE = 40, MAX_FRAME_SIZE = 2 * 1024 * 1024;

if (isMainThread) {
    const [inYuv, W, H, N, outDir, S, D, mode] = process.argv.slice(2);
    const w = +W, h = +H, nf = +N, ns = +S, nd = +D, rgba = mode === 'rgba';
    fs.mkdirSync(outDir, { recursive: true });
    const yuv = fs.readFileSync(inYuv), fsz = w * h * 3 / 2;
    const encodedFrameSAB = new SharedArrayBuffer(FRAME_BUFFER_POOL_SIZE * MAX_FRAME_SIZE);
    const controlSAB = new SharedArrayBuffer(FRAME_BUFFER_POOL_SIZE * 2 * 4);
    const sab = { type: 'init_sab', encodedFrameSAB, controlSAB, FRAME_BUFFER_POOL_SIZE, MAX_FRAME_SIZE, numStreams: ns };
    const enc = new Worker(__filename, { workerData: { role: 'enc' } });
    const decs = [];
    for (let k = 0; k < nd; k++) {
        const streams = [];
        for (let s = k; s < ns; s += nd) streams.push(s);
        decs.push({ worker: new Worker(__filename, { workerData: { role: 'dec', id: k, streams, outDir, rgba } }), streams });
    }
    const all = [enc, ...decs.map((d) => d.worker)];
    let ready = 0, t = 0, pending = 0, cleaned = 0;
    const encOut = fs.openSync(path.join(outDir, 'enc.h264'), 'w');
    const sizes = [];
    const next = () => {
        if (t >= nf) { for (const x of all) x.postMessage({ type: 'cleanup' }); return; }
        const yuvData = yuv.buffer.slice(yuv.byteOffset + t * fsz, yuv.byteOffset + (t + 1) * fsz);
        enc.postMessage({ type: 'encode_yuv', yuvData, width: w, height: h }, [yuvData]);
        t++;
    };
    const onMsg = (m) => {
        if (m.type === 'ready' && ++ready === all.length) {
            for (const x of all) x.postMessage(sab);
            enc.postMessage({ type: 'init', width: w, height: h });
        } else if (m.type === 'init_done') {
            next();
        } else if (m.type === 'encoded') {
            const view = new Uint8Array(encodedFrameSAB, m.bufferIndex * MAX_FRAME_SIZE, m.encodedSize);
            fs.writeSync(encOut, Buffer.from(view));
            sizes.push(m.encodedSize);
            pending = ns;
            for (const d of decs)
                for (const s of d.streams)
                    d.worker.postMessage({ type: 'decode', bufferIndex: m.bufferIndex, streamIndex: s, encodedSize: m.encodedSize, width: w, height: h });
        } else if (m.type === 'skipped') {
            sizes.push(0);
            next();
        } else if (m.type === 'decoded') {
            if (--pending === 0) next();
        } else if (m.type === 'cleanup_done' && ++cleaned === all.length) {
            fs.closeSync(encOut);
            fs.writeFileSync(path.join(outDir, 'sizes.json'), JSON.stringify(sizes));
            for (const x of all) x.terminate();
            console.log(`replay ok: ${sizes.length} frames, ${ns} decoder streams on ${nd} workers`);
        } else if (m.type === 'error') {
            console.error('worker error:', m.message);
            process.exit(1);
        }
    };
    for (const x of all) { x.on('message', onMsg); x.on('error', (e) => { console.error(e); process.exit(1); }); }
} else {
    // ---- a Worker's global scope as the reference glue sees it
    global.self = global;
    self.postMessage = (m) => parentPort.postMessage(m);
    global.importScripts = (...files) => { for (const f of files) require(path.join(JS_DIR, f)); };
    parentPort.on('message', (data) => { try { self.onmessage({ data }); } catch (e) { self.postMessage({ type: 'error', message: String(e.stack || e) }); } });
    if (workerData.role === 'enc') encoderWorker(); else decoderWorker(workerData);
}

function encoderWorker() {
    let wasmReady = false, initEncoder, encodeFrameYuv, controlView, frameDataViews = [], pool = 0, maxSize = 0, numStreams = 1;
    let yuvBufferPtr = 0, yuvBufferSize = 0, encodedDataPtr_ptr = 0, encodedSize_ptr = 0, current = 0;
    importScripts('h264.js');                                                          // encoder_worker.js:23
    Module.onRuntimeInitialized = () => {                                              // :25-31
        initEncoder = Module.cwrap('init_encoder', 'number', ['number', 'number', 'number']);
        encodeFrameYuv = Module.cwrap('encode_frame_yuv_i420', null, ['number', 'number', 'number', 'number', 'number']);
        wasmReady = true;
        self.postMessage({ type: 'ready' });
    };
    self.onmessage = (e) => {
        const d = e.data;
        if (d.type === 'init_sab') {                                                   // :35-47
            controlView = new Int32Array(d.controlSAB); pool = d.FRAME_BUFFER_POOL_SIZE; maxSize = d.MAX_FRAME_SIZE; numStreams = d.numStreams;
            for (let i = 0; i < pool; i++) frameDataViews[i] = new Uint8Array(d.encodedFrameSAB, i * maxSize, maxSize);
            return;
        }
        if (!wasmReady) return;
        if (d.type === 'cleanup') {                                                    // :61-76
            if (yuvBufferPtr) Module._free(yuvBufferPtr);
            if (encodedDataPtr_ptr) Module._free(encodedDataPtr_ptr);
            if (encodedSize_ptr) Module._free(encodedSize_ptr);
            self.postMessage({ type: 'cleanup_done' });
            return;
        }
        if (d.type === 'init') {                                                       // :93-100
            if (initEncoder(d.width, d.height, 1000000) !== 0) throw new Error('encoder init failed');
            encodedDataPtr_ptr = Module._malloc(4);
            encodedSize_ptr = Module._malloc(4);
            self.postMessage({ type: 'init_done' });
        } else if (d.type === 'encode_yuv') {                                          // :127-147
            const yuvArray = new Uint8Array(d.yuvData);
            if (yuvArray.length > yuvBufferSize) {
                if (yuvBufferPtr) Module._free(yuvBufferPtr);
                yuvBufferPtr = Module._malloc(yuvArray.length);
                yuvBufferSize = yuvArray.length;
            }
            HEAPU8.set(yuvArray, yuvBufferPtr);
            encodeFrameYuv(yuvBufferPtr, d.width, d.height, encodedDataPtr_ptr, encodedSize_ptr);
            const encodedDataPtr = Module.getValue(encodedDataPtr_ptr, 'i32');         // :163-202
            const encodedSize = Module.getValue(encodedSize_ptr, 'i32');
            if (encodedSize <= 0 || encodedSize > maxSize) { self.postMessage({ type: 'skipped' }); return; }
            if (Atomics.load(controlView, current * 2 + 1) > 0) throw new Error('ring slot still referenced');
            frameDataViews[current].set(HEAPU8.subarray(encodedDataPtr, encodedDataPtr + encodedSize));
            controlView[current * 2] = encodedSize;
            controlView[current * 2 + 1] = numStreams;
            self.postMessage({ type: 'encoded', bufferIndex: current, encodedSize });
            current = (current + 1) % pool;
        }
    };
}

function decoderWorker({ id, streams, outDir, rgba }) {
    let wasmReady = false, initDecoder, decodeFrame, decodeFrameYuv, deinitDecoderWasm, controlView, frameDataViews = [];
    let decodedWidth_ptr = 0, decodedHeight_ptr = 0, encodedBufferPtr = 0, encodedBufferSize = 0, outPtr = 0, outSize = 0;
    const files = new Map();
    importScripts('h264.js');                                                          // decoder_worker.js:342
    Module.onRuntimeInitialized = () => {                                              // :343-361
        initDecoder = Module.cwrap('init_decoder', 'number', ['number']);
        decodeFrame = Module.cwrap('decode_frame_optimized', null, ['number', 'number', 'number', 'number', 'number', 'number']);
        decodeFrameYuv = Module.cwrap('decode_frame_yuv_i420', null, ['number', 'number', 'number', 'number', 'number', 'number']);
        deinitDecoderWasm = Module.cwrap('deinit_decoder', 'number', ['number']);
        decodedWidth_ptr = Module._malloc(4);
        decodedHeight_ptr = Module._malloc(4);
        for (const s of streams) {
            if (initDecoder(s) !== 0) throw new Error(`decoder ${s} init failed`);
            files.set(s, fs.openSync(path.join(outDir, `dec_${s}.${rgba ? 'rgba' : 'yuv'}`), 'w'));
        }
        wasmReady = true;
        self.postMessage({ type: 'ready' });
    };
    self.onmessage = (e) => {
        const d = e.data;
        if (d.type === 'init_sab') {
            controlView = new Int32Array(d.controlSAB);
            for (let i = 0; i < d.FRAME_BUFFER_POOL_SIZE; i++) frameDataViews[i] = new Uint8Array(d.encodedFrameSAB, i * d.MAX_FRAME_SIZE, d.MAX_FRAME_SIZE);
            return;
        }
        if (d.type === 'cleanup') {                                                    // :295-309
            for (const p of [encodedBufferPtr, outPtr, decodedWidth_ptr, decodedHeight_ptr]) if (p) Module._free(p);
            for (const s of streams) { deinitDecoderWasm(s); fs.closeSync(files.get(s)); }
            self.postMessage({ type: 'cleanup_done' });
            return;
        }
        if (d.type !== 'decode' || !wasmReady) return;
        const { bufferIndex, streamIndex, encodedSize, width, height } = d;            // :137-190
        const encodedDataArray = frameDataViews[bufferIndex].subarray(0, encodedSize);
        if (encodedDataArray.length > encodedBufferSize) {
            if (encodedBufferPtr) Module._free(encodedBufferPtr);
            encodedBufferPtr = Module._malloc(encodedDataArray.length);
            encodedBufferSize = encodedDataArray.length;
        }
        HEAPU8.set(encodedDataArray, encodedBufferPtr);
        Atomics.sub(controlView, bufferIndex * 2 + 1, 1);
        const need = rgba ? width * height * 4 : width * height * 1.5;
        if (need > outSize) {
            if (outPtr) Module._free(outPtr);
            outPtr = Module._malloc(need);
            outSize = need;
        }
        if (rgba) decodeFrame(streamIndex, encodedBufferPtr, encodedDataArray.length, outPtr, decodedWidth_ptr, decodedHeight_ptr);
        else decodeFrameYuv(streamIndex, encodedBufferPtr, encodedDataArray.length, outPtr, decodedWidth_ptr, decodedHeight_ptr);
        const dw = Module.getValue(decodedWidth_ptr, 'i32'), dh = Module.getValue(decodedHeight_ptr, 'i32');  // :197-208
        if (dw > 0 && dh > 0) {
            const n = rgba ? dw * dh * 4 : dw * dh * 1.5;
            fs.writeSync(files.get(streamIndex), Buffer.from(HEAPU8.subarray(outPtr, outPtr + n)));
        }
        self.postMessage({ type: 'decoded', streamIndex });
    };
}
