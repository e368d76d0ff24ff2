"""h264mi -- Python host bindings of libh264mi (MI355X-native H.264 encode/decode core).

Layering:
  * ``lib/libh264mi.so`` -- HIP kernels for gfx950 + runtime + the C-ABI declared in
    ``include/h264mi.h``.
  * ``Module`` (this file) -- mirrors the Emscripten ``Module`` object the reference's workers use
    (``cwrap``/``_malloc``/``_free``/``getValue``/``HEAPU8``; scripts/encoder_worker.js:27-29,
    decoder_worker.js:346-349) so call sequences read exactly like the reference's glue.
  * ``BatchEncoder`` / ``BatchDecoder`` -- the device-resident multi-stream API (frames and NAL
    units already in HBM) used by bench.py and the multi-GPU path.

There is no CPU fallback: importing this module on a machine without the built library raises.
"""
import atexit
import ctypes
import os
import sys
import weakref

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('H264MI_LIB') or os.path.join(os.path.dirname(_HERE), 'lib', 'libh264mi.so')  # env: diagnostics

_lib = None


def lib():
    """Load libh264mi.so (fails loudly when it is missing -- there is no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f'libh264mi.so not built ({LIB_PATH}); run openh264-wasm_amd/build.py')
        L = ctypes.CDLL(LIB_PATH)
        vp, i, cp = ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p
        sig = {
            'init_encoder': (i, [i, i, i]),
            'force_key_frame': (None, []),
            'init_decoder': (i, [i]),
            'deinit_decoder': (None, [i]),
            'encode_frame': (None, [vp, i, i, vp, vp]),
            'encode_frame_yuv_i420': (None, [vp, i, i, vp, vp]),
            'decode_frame_optimized': (None, [i, vp, i, vp, vp, vp]),
            'decode_frame_yuv_i420': (None, [i, vp, i, vp, vp, vp]),
            'free_buffer': (None, [vp]),
            'h264mi_enc_create': (vp, [i, i, i, i, vp]),
            'h264mi_enc_destroy': (None, [vp]),
            'h264mi_enc_force_idr': (i, [vp, i]),
            'h264mi_enc_encode': (i, [vp, vp]),
            'h264mi_enc_set_frame_skip': (i, [vp, i]),
            'h264mi_enc_frames_skipped': (i, [vp, i]),
            'h264mi_enc_set_gom_exact': (i, [vp, i]),
            'h264mi_enc_inject_error': (i, [vp, i, i]),
            'h264mi_enc_sync': (i, [vp]),
            'h264mi_enc_nal_bytes': (i, [vp, vp]),
            'h264mi_enc_nal_ptr': (vp, [vp, i]),
            'h264mi_enc_recon_ptr': (vp, [vp, i]),
            'h264mi_enc_input_buffer': (vp, [vp]),
            'h264mi_enc_frame_bytes': (ctypes.c_size_t, [vp]),
            'h264mi_enc_last_qp': (i, [vp, i]),
            'h264mi_enc_rc_state': (i, [vp, i, vp]),
            'h264mi_enc_gom_state': (i, [vp, i, vp, i]),
            'h264mi_rc_qstep_to_qp': (i, [i]),
            'h264mi_enc_mbinfo': (i, [vp, i, vp]),
            'h264mi_enc_ref_planes': (i, [vp, i, vp]),
            'h264mi_enc_stream': (vp, [vp]),
            'h264mi_enc_nal_size_dev': (vp, [vp, i]),
            'h264mi_enc_copy_nals': (i, [vp, vp, i, vp]),
            'h264mi_enc_set_timing': (i, [vp, i]),
            'h264mi_enc_kernel_time': (i, [vp, vp, vp]),
            'h264mi_dec_decode_dev': (i, [vp, vp, vp]),
            'h264mi_dec_create': (vp, [i, i, i, vp]),
            'h264mi_dec_destroy': (None, [vp]),
            'h264mi_dec_create_batch': (vp, [i, i, i, i, vp]),
            'h264mi_dec_create_ring': (vp, [i, i, i, i, i, i, vp]),
            'h264mi_dec_device_bytes': (ctypes.c_size_t, [vp]),
            'h264mi_dec_ring_groups': (i, [vp]),
            'h264mi_i_decoder_device_bytes': (ctypes.c_size_t, [vp, i]),
            'h264mi_instance_create': (vp, []),
            'h264mi_instance_destroy': (None, [vp]),
            'h264mi_dec_decode_frames': (i, [vp, i, vp, vp, vp]),
            'h264mi_dec_decode_frames_after': (i, [vp, i, vp, vp, vp, vp]),
            'h264mi_dec_decode_frames_after_n': (i, [vp, i, vp, vp, vp, vp, i]),
            'h264mi_dec_decode_frames_out': (i, [vp, i, vp, vp, vp, vp, i, vp, vp]),
            'h264mi_dec_recon_profile': (i, [vp, vp]),
            'h264mi_dec_max_frames': (i, [vp]),
            'h264mi_dec_set_parse_streams': (i, [vp, i]),
            'h264mi_dec_set_slice_waves': (i, [vp, i]),
            'h264mi_dec_set_streamed': (i, [vp, i]),
            'h264mi_dec_streamed': (i, [vp]),
            'h264mi_dec_set_streamed_budget': (i, [i]),
            'h264mi_nal_pack': (i, [vp, vp, ctypes.c_size_t, vp, i, vp]),
            'h264mi_nal_unpack': (i, [vp, vp, ctypes.c_size_t, vp, i, vp]),
            'h264mi_dec_set_parse_cus': (i, [vp, i, i]),
            'h264mi_stream_create_cus': (vp, [i, i, i]),
            'h264mi_stream_destroy': (None, [vp]),
            'h264mi_dec_decode': (i, [vp, vp, vp]),
            'h264mi_dec_sync': (i, [vp]),
            'h264mi_dec_set_timing': (i, [vp, i]),
            'h264mi_dec_kernel_time': (i, [vp, i, vp, vp]),
            'h264mi_dec_status': (i, [vp, vp]),
            'h264mi_dec_parse_profile': (i, [vp, vp]),
            'h264mi_enc_profile': (i, [vp, vp]),
            'h264mi_enc_timeline': (i, [vp, vp, i]),
            'h264mi_dec_picture_ptr': (vp, [vp, i]),
            'h264mi_dec_coded_size': (i, [vp, vp, vp]),
            'h264mi_dec_stream': (vp, [vp]),
            'h264mi_rgba_to_i420_host': (i, [vp, i, i, vp]),
            'h264mi_i420_to_rgba_host': (i, [vp, i, i, vp]),
            'h264mi_ring_create': (vp, [i, i]),
            'h264mi_ring_destroy': (None, [vp]),
            'h264mi_ring_publish': (ctypes.c_longlong, [vp, vp, i, i]),
            'h264mi_ring_nal_ptr': (vp, [vp, ctypes.c_longlong]),
            'h264mi_ring_size_dev': (vp, [vp, ctypes.c_longlong]),
            'h264mi_ring_release': (i, [vp, ctypes.c_longlong, vp]),
            'h264mi_ring_stats': (i, [vp, vp, vp, vp, vp]),
            'h264mi_version': (cp, []),
            'h264mi_enc_rows_counter': (vp, [vp]),
            'h264mi_dec_set_recon_gate': (i, [vp, vp, ctypes.c_uint32, ctypes.c_uint32, i, i]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


# Teardown order. GPU objects (encoders, decoders, rings, CU-masked streams) are released explicitly by
# close(), or at interpreter exit by the atexit hook below -- which runs before the HIP runtime and torch
# unload. __del__ does nothing once the interpreter is finalising: freeing device memory or destroying
# streams and events from a finaliser that runs during library unload is what crashed profiled runs at
# exit (rocprofv3 logs: SIGSEGV in __cxa_finalize).
_live = weakref.WeakSet()
_streams = []  # handles from h264mi_stream_create_cus not yet destroyed


def _close_all():
    for o in list(_live):
        try:
            o.close()
        except Exception:
            pass
    while _streams:
        h = _streams.pop()
        try:
            _hiprt().hipStreamSynchronize(ctypes.c_void_p(h))
            lib().h264mi_stream_destroy(ctypes.c_void_p(h))
        except Exception:
            pass


atexit.register(_close_all)


def _finalising():
    return sys.is_finalizing()


EXPORTED = ('init_encoder', 'force_key_frame', 'init_decoder', 'deinit_decoder', 'encode_frame',
            'encode_frame_yuv_i420', 'decode_frame_optimized', 'decode_frame_yuv_i420', 'free_buffer')


class Module:
    """Emscripten-``Module``-shaped facade over the C-ABI (the reference's JS glue surface).

    ``HEAPU8`` is a bytearray arena; ``_malloc`` returns offsets into it; ``cwrap`` returns callables
    that translate arena offsets to native pointers (and native output pointers back into arena
    offsets, e.g. the encoded buffer of encode_frame*), exactly as the workers expect
    (encoder_worker.js:163-187 reads the encoded buffer via getValue + HEAPU8.subarray).
    """

    def __init__(self, heap_bytes=64 << 20):
        self._L = lib()
        self.HEAPU8 = bytearray(heap_bytes)
        self._heap = (ctypes.c_ubyte * heap_bytes).from_buffer(self.HEAPU8)
        self._base = ctypes.addressof(self._heap)
        self._brk = 16
        self._freelist = {}  # offset -> size (first-fit)
        self._sizes = {}
        self._out_off, self._out_cap = 0, 0

    # -- heap management (Module._malloc / Module._free)
    def _malloc(self, n):
        n = (max(1, int(n)) + 15) & ~15
        for off, sz in sorted(self._freelist.items()):
            if sz >= n:
                del self._freelist[off]
                if sz > n:
                    self._freelist[off + n] = sz - n
                self._sizes[off] = n
                return off
        off = self._brk
        if off + n > len(self.HEAPU8):
            raise MemoryError('h264mi Module heap exhausted')
        self._brk += n
        self._sizes[off] = n
        return off

    def _free(self, off):
        n = self._sizes.pop(off, None)
        if n:
            self._freelist[off] = n

    def getValue(self, ptr, typ='i32'):
        assert typ == 'i32'
        return int.from_bytes(self.HEAPU8[ptr:ptr + 4], 'little', signed=True)

    def setValue(self, ptr, value, typ='i32'):
        assert typ == 'i32'
        self.HEAPU8[ptr:ptr + 4] = int(value).to_bytes(4, 'little', signed=True)

    def _p(self, off):
        return ctypes.c_void_p(self._base + off)

    def cwrap(self, name, ret, args):
        if name not in EXPORTED:
            raise KeyError(f'{name} is not exported by libh264mi')
        f = getattr(self._L, name)
        if name in ('encode_frame', 'encode_frame_yuv_i420'):
            def enc(src, w, h, out_pp, out_size_p, _f=f):
                native = ctypes.POINTER(ctypes.c_ubyte)()
                size = ctypes.c_int(0)
                _f(self._p(src), w, h, ctypes.byref(native), ctypes.byref(size))
                if size.value <= 0:
                    self.setValue(out_pp, 0)
                    self.setValue(out_size_p, 0)
                    return None
                if size.value > self._out_cap:  # library-owned output mirrored into the heap
                    if self._out_cap:
                        self._free(self._out_off)
                    self._out_off, self._out_cap = self._malloc(size.value), size.value
                ctypes.memmove(self._base + self._out_off, native, size.value)
                self.setValue(out_pp, self._out_off)
                self.setValue(out_size_p, size.value)
                return None
            return enc
        if name in ('decode_frame_optimized', 'decode_frame_yuv_i420'):
            def dec(idx, nal, size, out, w_p, h_p, _f=f):
                _f(idx, self._p(nal), size, self._p(out), self._p(w_p), self._p(h_p))
                return None
            return dec
        if name == 'free_buffer':
            return lambda ptr: None  # the reference glue never frees the library-owned buffer
        return lambda *a: f(*a)

    def on_runtime_initialized(self, cb):
        cb()


class BatchEncoder:
    """S independent encoder streams of one geometry, frames and NAL units resident in HBM."""

    def __init__(self, width, height, bitrate, nstreams, stream=None):
        import torch
        self.w, self.h, self.S = width, height, nstreams
        self.frame_bytes = width * height * 3 // 2
        self._L = lib()
        hs = stream.cuda_stream if stream is not None else torch.cuda.current_stream().cuda_stream
        self._e = self._L.h264mi_enc_create(width, height, bitrate, nstreams, ctypes.c_void_p(hs))
        if not self._e:
            raise RuntimeError('h264mi_enc_create failed')
        _live.add(self)

    def encode(self, frames):
        """frames: uint8 CUDA tensor holding S tight I420 frames back to back (async)."""
        assert frames.is_cuda and frames.numel() >= self.S * self.frame_bytes
        if self._L.h264mi_enc_encode(self._e, ctypes.c_void_p(frames.data_ptr())) != 0:
            raise RuntimeError('h264mi_enc_encode failed')

    def force_idr(self, stream=-1):
        self._L.h264mi_enc_force_idr(self._e, stream)

    def set_frame_skip(self, on):
        """rate-control frame skipping (on by default, as the wrapper's encoder)"""
        if self._L.h264mi_enc_set_frame_skip(self._e, 1 if on else 0) != 0:
            raise RuntimeError('h264mi_enc_set_frame_skip failed')

    def inject_error(self, s=0, code=2):
        """test hook: stream s's next coded frame fails (0 bytes out, then an IDR)"""
        if self._L.h264mi_enc_inject_error(self._e, s, code) != 0:
            raise RuntimeError('h264mi_enc_inject_error failed')

    def set_gom_exact(self, on):
        """OpenH264's exact GOM rate control (h264mi_enc_set_gom_exact)"""
        if self._L.h264mi_enc_set_gom_exact(self._e, 1 if on else 0) != 0:
            raise RuntimeError('h264mi_enc_set_gom_exact failed')

    def gom_state(self, s=0):
        """exact GOM mode: the last P frame's per-GOM [QP, slice bits before it, target bits, last coded MB + 1]
        (h264mi_enc_gom_state)"""
        G = self._L.h264mi_enc_gom_state(self._e, s, None, 0)
        out = (ctypes.c_int * (4 * max(G, 1)))()
        if G < 0 or self._L.h264mi_enc_gom_state(self._e, s, out, 4 * G) != G:
            raise RuntimeError('h264mi_enc_gom_state failed')
        return [list(out[4 * g:4 * g + 4]) for g in range(G)]

    def frames_skipped(self, s=0):
        return self._L.h264mi_enc_frames_skipped(self._e, s)

    def rows_counter(self):
        """device address of the encoder's rows-started counter (h264mi_enc_rows_counter): S * mbh per frame step"""
        return self._L.h264mi_enc_rows_counter(self._e)

    def nal_sizes(self):
        out = (ctypes.c_int * self.S)()
        rc = self._L.h264mi_enc_nal_bytes(self._e, out)
        if rc != 0:
            raise RuntimeError(f'encoder kernels reported an error ({rc})')
        return list(out)

    def nal_ptr(self, s):
        return self._L.h264mi_enc_nal_ptr(self._e, s)

    def nal_ptrs(self):
        return [self.nal_ptr(s) for s in range(self.S)]

    def nal_bytes(self, s, size):
        """Copy stream s's last NAL output to host bytes (testing / C-ABI style use)."""
        import torch
        buf = torch.empty(size, dtype=torch.uint8)
        _hip_memcpy_d2h(buf.data_ptr(), self.nal_ptr(s), size)
        return bytes(buf.numpy())

    def nal_size_ptrs(self):
        return [self._L.h264mi_enc_nal_size_dev(self._e, s) for s in range(self.S)]

    def copy_nals(self, dst, slot, sizes=None):
        """async device copy of every stream's NAL into dst[s*slot:(s+1)*slot] (uint8 CUDA tensor);
        byte counts into sizes (int32 CUDA tensor of S) when given"""
        sp = ctypes.c_void_p(sizes.data_ptr()) if sizes is not None else None
        if self._L.h264mi_enc_copy_nals(self._e, ctypes.c_void_p(dst.data_ptr()), slot, sp) != 0:
            raise RuntimeError('h264mi_enc_copy_nals failed')

    def set_timing(self, on):
        self._L.h264mi_enc_set_timing(self._e, 1 if on else 0)

    def kernel_time(self):
        ms, n = ctypes.c_double(), ctypes.c_int()
        if self._L.h264mi_enc_kernel_time(self._e, ctypes.byref(ms), ctypes.byref(n)) != 0:
            raise RuntimeError('h264mi_enc_kernel_time failed')
        return ms.value, n.value

    def recon_ptr(self, s):
        return self._L.h264mi_enc_recon_ptr(self._e, s)

    def last_qp(self, s=0):
        return self._L.h264mi_enc_last_qp(self._e, s)

    RC_FIELDS = ('skipped', 'qp', 'avg_qp', 'target', 'remaining', 'fullness', 'continual', 'cmplx', 'min_qp',
                 'max_qp', 'bpf', 'pframes', 'idrs', 'skip_flag', 'remaining_weights', 'coded_in_vgop')

    def rc_state(self, s=0):
        """stream s's rate-control state after the last frame step (h264mi_enc_rc_state)"""
        out = (ctypes.c_int * 16)()
        if self._L.h264mi_enc_rc_state(self._e, s, out) != 0:
            raise RuntimeError('h264mi_enc_rc_state failed')
        return dict(zip(self.RC_FIELDS, list(out)))

    def close(self):
        if self._e:
            self._L.h264mi_enc_destroy(self._e)
            self._e = None

    def __del__(self):
        if _finalising():
            return
        try:
            self.close()
        except Exception:
            pass


def masked_stream(cu_lo, cu_hi, complement=False):
    """A torch stream (ExternalStream over h264mi_stream_create_cus) restricted to CU mask bits
    [cu_lo, cu_hi), or to every other CU. Pairs with BatchDecoder.set_parse_cus."""
    import torch
    h = lib().h264mi_stream_create_cus(cu_lo, cu_hi, 1 if complement else 0)
    if not h:
        raise RuntimeError('h264mi_stream_create_cus failed')
    _streams.append(h)
    return torch.cuda.ExternalStream(h)


def destroy_stream(st):
    """Synchronise and destroy a stream made by masked_stream() (close its users first)."""
    h = st.cuda_stream
    if h in _streams:
        _streams.remove(h)
        st.synchronize()
        lib().h264mi_stream_destroy(ctypes.c_void_p(h))


class BatchDecoder:
    """S independent decoder streams of one geometry; NAL units in HBM. max_frames > 1 enables
    decode_frames(): several access units per stream per call, entropy-decoded concurrently."""

    def __init__(self, width, height, nstreams, stream=None, max_frames=1, groups=0, parse_streams=3):
        """groups: slot groups of max_frames frames in the decoder's ring (0 = default, up to 16; 2 for a
        caller that waits for every call); parse_streams: HIP streams entropy decoding rotates over"""
        import torch
        self.w, self.h, self.S, self.B = width, height, nstreams, max_frames
        self._L = lib()
        hs = stream.cuda_stream if stream is not None else torch.cuda.current_stream().cuda_stream
        self._d = self._L.h264mi_dec_create_ring(width, height, nstreams, max_frames, groups, parse_streams, ctypes.c_void_p(hs))
        if not self._d:
            raise RuntimeError('h264mi_dec_create failed')
        _live.add(self)
        cw, ch = ctypes.c_int(), ctypes.c_int()
        self._L.h264mi_dec_coded_size(self._d, ctypes.byref(cw), ctypes.byref(ch))
        self.cw, self.ch = cw.value, ch.value

    def decode(self, nal_ptrs, nal_sizes):
        """nal_ptrs: device addresses (ints); nal_sizes: host ints (async)."""
        ptrs = (ctypes.c_void_p * self.S)(*nal_ptrs)
        sizes = (ctypes.c_int * self.S)(*nal_sizes)
        if self._L.h264mi_dec_decode(self._d, ptrs, sizes) != 0:
            raise RuntimeError('h264mi_dec_decode failed')

    def decode_dev(self, nal_ptrs, size_ptrs):
        """async; sizes read on the device from size_ptrs (e.g. BatchEncoder.nal_size_ptrs())"""
        ptrs = (ctypes.c_void_p * self.S)(*nal_ptrs)
        sz = (ctypes.c_void_p * self.S)(*size_ptrs)
        if self._L.h264mi_dec_decode_dev(self._d, ptrs, sz) != 0:
            raise RuntimeError('h264mi_dec_decode_dev failed')

    def decode_frames(self, nal_ptrs, nal_sizes=None, size_ptrs=None, ready_event=None, out_ptrs=None, got_ptrs=None):
        """async; n frames per stream: nal_ptrs[f * S + s] (device addresses), sizes either host ints
        (nal_sizes) or device int32 addresses (size_ptrs). n <= max_frames. Inputs are ordered after
        the decoder's stream, or, if ready_event (a torch.cuda.Event recorded by the producer, or a
        list of them, one per producer stream) is given, after those events only. out_ptrs / got_ptrs
        (device addresses, same indexing): every frame's cropped tight I420 picture and got flag."""
        m = len(nal_ptrs)
        assert m % self.S == 0 and m // self.S <= self.B
        ptrs = (ctypes.c_void_p * m)(*nal_ptrs)
        sizes = (ctypes.c_int * m)(*nal_sizes) if nal_sizes is not None else None
        sp = (ctypes.c_void_p * m)(*size_ptrs) if size_ptrs is not None else None
        evs = [] if ready_event is None else (list(ready_event) if isinstance(ready_event, (list, tuple)) else [ready_event])
        ev = (ctypes.c_void_p * max(1, len(evs)))(*[e.cuda_event for e in evs])
        op = (ctypes.c_void_p * m)(*out_ptrs) if out_ptrs is not None else None
        gp = (ctypes.c_void_p * m)(*got_ptrs) if got_ptrs is not None else None
        if self._L.h264mi_dec_decode_frames_out(self._d, m // self.S, ptrs, sizes, sp, ev, len(evs), op, gp) != 0:
            raise RuntimeError('h264mi_dec_decode_frames failed')

    def set_parse_cus(self, lo, hi):
        """entropy decoding on CU mask bits [lo, hi) (see h264mi_dec_set_parse_cus)"""
        if self._L.h264mi_dec_set_parse_cus(self._d, lo, hi) != 0:
            raise RuntimeError('h264mi_dec_set_parse_cus failed')

    def set_recon_gate(self, counter, target, step, count, limit_us=4000):
        """for the next decode call: frame f < count reconstructs once the device uint32 at `counter` reaches
        target + f * step (h264mi_dec_set_recon_gate; a scheduling hint, bounded by limit_us)"""
        if self._L.h264mi_dec_set_recon_gate(self._d, counter, target & 0xffffffff, step & 0xffffffff, count, limit_us) != 0:
            raise RuntimeError('h264mi_dec_set_recon_gate failed')

    def set_streamed(self, mode):
        """streamed reconstruction (h264mi_dec_set_streamed): 1 on (the reconstruction stream is kept off the
        parse CUs), 0 off, -1 automatic"""
        if self._L.h264mi_dec_set_streamed(self._d, mode) != 0:
            raise RuntimeError('h264mi_dec_set_streamed failed')

    def streamed(self):
        return self._L.h264mi_dec_streamed(self._d)

    def set_slice_waves(self, k):
        """slice-data waves per picture (h264mi_dec_set_slice_waves): a multi-slice picture's slices in parallel"""
        if self._L.h264mi_dec_set_slice_waves(self._d, k) != 0:
            raise RuntimeError('h264mi_dec_set_slice_waves failed')

    def set_parse_streams(self, n):
        if self._L.h264mi_dec_set_parse_streams(self._d, n) != 0:
            raise RuntimeError('h264mi_dec_set_parse_streams failed')

    def set_timing(self, on):
        self._L.h264mi_dec_set_timing(self._d, 1 if on else 0)

    def kernel_time(self, which=0):
        """(total ms, launches) of dec_recon_kernel (which 0) or dec_parse_kernel (1) since set_timing"""
        ms, n = ctypes.c_double(), ctypes.c_int()
        if self._L.h264mi_dec_kernel_time(self._d, which, ctypes.byref(ms), ctypes.byref(n)) != 0:
            raise RuntimeError('h264mi_dec_kernel_time failed')
        return ms.value, n.value

    def device_bytes(self):
        return self._L.h264mi_dec_device_bytes(self._d)

    def ring_groups(self):
        return self._L.h264mi_dec_ring_groups(self._d)

    def status(self):
        got = (ctypes.c_int * self.S)()
        rc = self._L.h264mi_dec_status(self._d, got)
        return rc, list(got)

    def picture_ptr(self, s):
        """Device pointer of stream s's last decoded picture (coded size, planes contiguous)."""
        return self._L.h264mi_dec_picture_ptr(self._d, s)

    def picture_i420(self, s):
        """Cropped tight I420 of stream s's last picture, as host bytes."""
        import numpy as np
        p = self._L.h264mi_dec_picture_ptr(self._d, s)
        cw, ch = self.cw, self.ch
        buf = np.empty(cw * ch * 3 // 2, np.uint8)
        _hip_memcpy_d2h(buf.ctypes.data, p, buf.size)  # planes are contiguous: Y, U, V at coded size
        y = buf[:cw * ch].reshape(ch, cw)[:self.h, :self.w]
        u = buf[cw * ch:cw * ch * 5 // 4].reshape(ch // 2, cw // 2)[:self.h // 2, :self.w // 2]
        v = buf[cw * ch * 5 // 4:].reshape(ch // 2, cw // 2)[:self.h // 2, :self.w // 2]
        return np.concatenate([y.ravel(), u.ravel(), v.ravel()]).tobytes()

    def close(self):
        if self._d:
            self._L.h264mi_dec_destroy(self._d)
            self._d = None

    def __del__(self):
        if _finalising():
            return
        try:
            self.close()
        except Exception:
            pass


class NalRing:
    """Device-resident NAL ring: the reference's SharedArrayBuffer frame pool (app.js:52-53,
    :292-310) with encoder_worker.js:163-202 publish and decoder_worker.js:138-164 release semantics,
    decided on the device. Tickets are returned by publish(); decoders read nal_ptr(t)/size_ptr(t)
    (size 0 = dropped, decoders skip it) and every consumer calls release(t) afterwards."""

    def __init__(self, slots=40, slot_bytes=2 << 20):
        self._L = lib()
        self.slots, self.slot_bytes = slots, slot_bytes
        self._r = self._L.h264mi_ring_create(slots, slot_bytes)
        if not self._r:
            raise RuntimeError('h264mi_ring_create failed')
        _live.add(self)

    def publish(self, enc, stream, consumers):
        t = self._L.h264mi_ring_publish(self._r, enc._e, stream, consumers)
        if t < 0:
            raise RuntimeError(f'h264mi_ring_publish failed ({t})')
        return t

    def nal_ptr(self, t):
        return self._L.h264mi_ring_nal_ptr(self._r, t)

    def size_ptr(self, t):
        return self._L.h264mi_ring_size_dev(self._r, t)

    def release(self, t, stream=None):
        import torch
        hs = stream.cuda_stream if stream is not None else torch.cuda.current_stream().cuda_stream
        if self._L.h264mi_ring_release(self._r, t, ctypes.c_void_p(hs)) != 0:
            raise RuntimeError('h264mi_ring_release failed')

    def stats(self):
        p, b, z = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        refs = (ctypes.c_int * self.slots)()
        if self._L.h264mi_ring_stats(self._r, ctypes.byref(p), ctypes.byref(b), ctypes.byref(z), refs) != 0:
            raise RuntimeError('h264mi_ring_stats failed')
        return {'published': p.value, 'dropped_busy': b.value, 'dropped_size': z.value, 'ref_counts': list(refs)}

    def close(self):
        if self._r:
            self._L.h264mi_ring_destroy(self._r)
            self._r = None

    def __del__(self):
        if _finalising():
            return
        try:
            self.close()
        except Exception:
            pass


def _hip_memcpy_d2h(dst, src, n):
    import torch
    t = torch.cuda.current_stream()
    t.synchronize()
    hip = _hiprt()
    rc = hip.hipMemcpy(ctypes.c_void_p(dst), ctypes.c_void_p(src), ctypes.c_size_t(n), 2)
    if rc != 0:
        raise RuntimeError(f'hipMemcpy failed ({rc})')


_hip = None


def _hiprt():
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL('libamdhip64.so')
        _hip.hipMemcpy.restype = ctypes.c_int
        _hip.hipStreamSynchronize.restype = ctypes.c_int
        _hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    return _hip


def version():
    return lib().h264mi_version().decode()
