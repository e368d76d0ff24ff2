"""ctypes wrapper of the CPU oracle (oracle/h264o_api.h) -- TEST INFRASTRUCTURE ONLY."""
import ctypes
import numpy as np

vp = ctypes.c_void_p


class Oracle:
    def __init__(self, path):
        L = ctypes.CDLL(path)
        L.h264o_enc_create.restype = vp
        L.h264o_enc_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.h264o_enc_destroy.argtypes = [vp]
        L.h264o_enc_force_idr.argtypes = [vp]
        L.h264o_enc_encode.argtypes = [vp, vp, vp, ctypes.c_int]
        L.h264o_enc_recon.argtypes = [vp, vp]
        L.h264o_enc_mbinfo.argtypes = [vp, vp]
        L.h264o_enc_last_qp.argtypes = [vp]
        L.h264o_enc_set_frame_skip.argtypes = [vp, ctypes.c_int]
        L.h264o_enc_frames_skipped.argtypes = [vp]
        L.h264o_enc_me_stats.argtypes = [vp, vp]
        L.h264o_rc_init_qp.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.h264o_rc_qstep2qp.argtypes = [ctypes.c_int32]
        L.h264o_logf.argtypes = [ctypes.c_float]
        L.h264o_logf.restype = ctypes.c_float
        L.h264o_enc_set_gom_exact.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.h264o_enc_rc_state.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.h264o_enc_gom_state.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.h264o_write_sps.restype = ctypes.c_size_t
        L.h264o_write_sps.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, vp]
        L.h264o_write_pps.restype = ctypes.c_size_t
        L.h264o_write_pps.argtypes = [vp]
        L.h264o_dec_create.restype = vp
        L.h264o_dec_destroy.argtypes = [vp]
        L.h264o_dec_decode.argtypes = [vp, vp, ctypes.c_int, vp, vp, vp]
        L.h264o_dec_mbinfo.argtypes = [vp, vp]
        L.h264o_rgba_to_i420.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp]
        L.h264o_i420_to_rgba.argtypes = [vp, vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp]
        self.L = L

    def encoder(self, w, h, br):
        return OEnc(self.L, w, h, br)

    def decoder(self):
        return ODec(self.L)

    def rgba_to_i420(self, rgba, w, h):
        out = np.zeros(w * h * 3 // 2, np.uint8)
        rgba = np.ascontiguousarray(rgba, np.uint8)
        self.L.h264o_rgba_to_i420(rgba.ctypes.data, w, h, out.ctypes.data)
        return out

    def i420_to_rgba(self, i420, w, h):
        i420 = np.ascontiguousarray(i420, np.uint8)
        out = np.zeros(w * h * 4, np.uint8)
        y = i420.ctypes.data
        self.L.h264o_i420_to_rgba(y, y + w * h, y + w * h + (w // 2) * (h // 2), w, h, w, w // 2, out.ctypes.data)
        return out


class OEnc:
    def __init__(self, L, w, h, br):
        self.L, self.w, self.h = L, w, h
        self.e = vp(L.h264o_enc_create(w, h, br))
        assert self.e.value
        self.buf = np.zeros(w * h * 4 + 65536, np.uint8)

    def encode(self, i420):
        i420 = np.ascontiguousarray(i420, np.uint8)
        n = self.L.h264o_enc_encode(self.e, i420.ctypes.data, self.buf.ctypes.data, self.buf.size)
        return self.buf[:n].tobytes()

    def force_idr(self):
        self.L.h264o_enc_force_idr(self.e)

    def set_frame_skip(self, on):
        self.L.h264o_enc_set_frame_skip(self.e, 1 if on else 0)

    def set_gom_exact(self, on):
        self.L.h264o_enc_set_gom_exact(self.e, 1 if on else 0)

    RC_FIELDS = ('skipped', 'qp', 'avg_qp', 'target', 'remaining', 'fullness', 'continual', 'cmplx', 'min_qp',
                 'max_qp', 'bpf', 'pframes', 'idrs', 'skip_flag', 'remaining_weights', 'coded_in_vgop')

    def rc_state(self):
        """the rate control's state after the last encode call (oracle h264o_enc_rc_state)"""
        out = (ctypes.c_int32 * 16)()
        self.L.h264o_enc_rc_state(self.e, out)
        return dict(zip(self.RC_FIELDS, list(out)))

    def gom_state(self):
        """exact GOM mode: the last P frame's per-GOM [QP, slice bits before it, target bits, last coded MB + 1]"""
        G = self.L.h264o_enc_gom_state(self.e, None, 0)
        out = (ctypes.c_int32 * (4 * max(G, 1)))()
        self.L.h264o_enc_gom_state(self.e, out, 4 * G)
        return [list(out[4 * g:4 * g + 4]) for g in range(G)]

    def recon(self):
        out = np.zeros(self.w * self.h * 3 // 2, np.uint8)
        self.L.h264o_enc_recon(self.e, out.ctypes.data)
        return out

    def last_qp(self):
        return self.L.h264o_enc_last_qp(self.e)

    def __del__(self):
        try:
            self.L.h264o_enc_destroy(self.e)
        except Exception:
            pass


class ODec:
    def __init__(self, L):
        self.L = L
        self.d = vp(L.h264o_dec_create())
        self.out = np.zeros(4096 * 2304 * 3 // 2, np.uint8)

    def decode(self, nal):
        """-> (rc, tight I420 bytes or None, w, h)"""
        a = np.frombuffer(nal, np.uint8).copy() if len(nal) else np.zeros(1, np.uint8)
        w, h = ctypes.c_int(0), ctypes.c_int(0)
        rc = self.L.h264o_dec_decode(self.d, a.ctypes.data, len(nal), self.out.ctypes.data, ctypes.byref(w), ctypes.byref(h))
        if rc in (1, 2):  # 2: damaged access unit concealed by a copy of the last picture
            return rc, self.out[:w.value * h.value * 3 // 2].copy(), w.value, h.value
        return rc, None, w.value, h.value

    def __del__(self):
        try:
            self.L.h264o_dec_destroy(self.d)
        except Exception:
            pass
