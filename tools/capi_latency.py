"""Single-call latency of the drop-in C-ABI (the reference's call pattern: one frame per call, the
caller waits for each -- scripts/encoder_worker.js:148, scripts/decoder_worker.js:179,189).

usage: capi_latency.py [w h bitrate nframes]  -> one JSON line with per-call ms (median / max) for
encode_frame_yuv_i420, decode_frame_yuv_i420 and decode_frame_optimized (host buffers, PCIe included; frame 0
excluded as warm-up), and idr_decode_ms: frame 0's IDR decoded again once warm.
"""
import ctypes, json, os, sys, time
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'openh264-wasm_amd'))


def main(w=1920, h=1080, br=1000000, nf=12):
    import torch
    import h264mi
    from h264mi.synth import SyntheticStream
    torch.cuda.set_device(0)
    L = h264mi.lib()
    assert L.init_encoder(w, h, br) == 0 and L.init_decoder(0) == 0 and L.init_decoder(1) == 0
    src = SyntheticStream(0, w, h)
    frames = [np.ascontiguousarray(src.frame(t)) for t in range(nf)]
    yuv = np.zeros(w * h * 3 // 2, np.uint8)
    rgba = np.zeros(w * h * 4, np.uint8)
    ow, oh = ctypes.c_int(), ctypes.c_int()
    te, td, tr, sizes = [], [], [], []
    for t, f in enumerate(frames):
        p = ctypes.POINTER(ctypes.c_ubyte)()
        sz = ctypes.c_int(0)
        t0 = time.perf_counter()
        L.encode_frame_yuv_i420(f.ctypes.data_as(ctypes.c_void_p), w, h, ctypes.byref(p), ctypes.byref(sz))
        t1 = time.perf_counter()
        nal = np.frombuffer(ctypes.string_at(p, sz.value), np.uint8).copy() if sz.value > 0 else np.zeros(1, np.uint8)
        t2 = time.perf_counter()
        L.decode_frame_yuv_i420(0, nal.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(sz.value),
                                yuv.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ow), ctypes.byref(oh))
        t3 = time.perf_counter()
        L.decode_frame_optimized(1, nal.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(sz.value),
                                 rgba.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ow), ctypes.byref(oh))
        t4 = time.perf_counter()
        if t > 0:  # frame 0 pays one-time allocation
            te.append((t1 - t0) * 1e3); td.append((t3 - t2) * 1e3); tr.append((t4 - t3) * 1e3)
        sizes.append(sz.value)
        if t == 0:
            idr = nal
    # the IDR's single-call decode once warm: frame 0's access unit decoded again (an IDR restarts the stream)
    t0 = time.perf_counter()
    L.decode_frame_yuv_i420(0, idr.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(int(idr.size)),
                            yuv.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ow), ctypes.byref(oh))
    t_idr = (time.perf_counter() - t0) * 1e3
    assert (ow.value, oh.value) == (w, h), 'IDR re-decode gave no picture'
    st = lambda v: {'median_ms': round(float(np.median(v)), 3), 'max_ms': round(float(np.max(v)), 3)}
    print(json.dumps({'width': w, 'height': h, 'bitrate': br, 'frames': nf, 'nal_bytes': sizes,
                      'idr_decode_ms': round(t_idr, 3), 'encode_frame_yuv_i420': st(te), 'decode_frame_yuv_i420': st(td), 'decode_frame_optimized': st(tr),
                      'note': 'host buffers in and out (PCIe included), one frame per call, caller waits'}))


if __name__ == '__main__':
    main(*[int(x) for x in sys.argv[1:]])
