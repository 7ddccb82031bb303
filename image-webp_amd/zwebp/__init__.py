"""zwebp -- MI355X-native VP8 lossy block-transform pipeline (Python host side).

Thin ctypes layer over the C ABI in ``include/zwebp.h`` (``zwebp/libzwebp.so``,
built by ``make -C image-webp_amd``).  The names mirror the reference crate's
public surface for the lossy path:

  ===============================  =============================================
  here                             reference (zenwebp 0.2.0)
  ===============================  =============================================
  ``encode_frame_lossy``           ``encoder/vp8.rs:3132`` encode_frame_lossy
  ``EncoderParams.lossy``          ``encoder/api.rs:445`` EncoderParams::lossy
  ``WebPEncoder.encode``           ``encoder/api.rs:1291`` WebPEncoder::encode
  ``vp8_decode_frame``             ``decoder/vp8.rs:1526`` Vp8Decoder::decode_frame
  ``WebPDecoder``                  ``decoder/api.rs:306-906`` WebPDecoder (lossy)
  ``decode_rgb/decode_rgba``       ``decoder/api.rs:938-993``
  ``UpsamplingMethod``             ``decoder/api.rs:268``
  ``yuv_to_rgb``                   ``decoder/yuv.rs:82/:402`` fill_rgb_buffer_*
  ``rgb_to_yuv420``                ``decoder/yuv.rs:656`` convert_image_yuv
  ``loop_filter_frame``            ``decoder/vp8.rs:1172`` filter_row_in_cache
  ``EncodingError/DecodingError``  ``encoder/api.rs:35``, ``decoder/api.rs:79``
  ===============================  =============================================

Every call runs on the GPU.  There is no CPU fallback: if the library is not
built, or no HIP device is visible, the first call raises.
"""
import ctypes
import os
import threading
import weakref

import numpy as np

__all__ = [
    "ColorType", "EncoderParams", "WebPEncoder", "ZwError", "EncodingError", "DecodingError", "Context",
    "Frame", "Pipeline", "encode_frame_lossy", "encode_batch", "vp8_decode_frame", "decode_batch",
    "rgb_to_yuv420", "loop_filter_frame", "quant_blocks", "transform_quant_blocks", "library_path", "load_library",
    "UpsamplingMethod", "WebPDecoder", "decode_rgb", "decode_rgba", "vp8_decode_rgb", "decode_rgb_batch",
    "decode_rgb_batch_into", "decode_rgba_into", "decode_rgb_into",
    "yuv_to_rgb", "webp_parse", "encode_frame_lossless", "encode_alpha",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libzwebp.so"


class ColorType:
    """ColorType (encoder/api.rs:83-92), same discriminants as the C ABI."""
    L8 = 0
    La8 = 1
    Rgb8 = 2
    Rgba8 = 3
    BYTES = {0: 1, 1: 2, 2: 3, 3: 4}


_ERRS = {
    1: "InvalidDimensions", 2: "InvalidBufferSize", 3: "InvalidArgument", 4: "DeviceError",
    5: "Unsupported", 6: "OutOfMemory", 10: "Vp8MagicInvalid", 11: "ColorSpaceInvalid",
    12: "LumaPredictionModeInvalid", 13: "IntraPredictionModeInvalid", 14: "ChromaPredictionModeInvalid",
    15: "BitStreamError", 16: "UnsupportedFeature", 17: "NotEnoughInitData",
}


class ZwError(Exception):
    def __init__(self, code, what=""):
        self.code = code
        self.name = _ERRS.get(code, "Unknown")
        super().__init__(f"{what}: {self.name} (code {code})" if what else f"{self.name} (code {code})")


class EncodingError(ZwError):
    pass


class DecodingError(ZwError):
    pass


def library_path():
    return os.environ.get("ZWEBP_LIB", os.path.join(_HERE, LIB_NAME))


class _Frame(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint16), ("height", ctypes.c_uint16),
                ("y_stride", ctypes.c_uint32), ("uv_stride", ctypes.c_uint32), ("mb_rows", ctypes.c_uint32),
                ("y", ctypes.c_void_p), ("u", ctypes.c_void_p), ("v", ctypes.c_void_p),
                ("filter_type", ctypes.c_uint8), ("filter_level", ctypes.c_uint8),
                ("sharpness_level", ctypes.c_uint8), ("pad", ctypes.c_uint8)]


class _Bytes(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_size_t)]


class _Image(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_size_t), ("width", ctypes.c_uint32),
                ("height", ctypes.c_uint32), ("color", ctypes.c_int)]


class _EncParams(ctypes.Structure):
    _fields_ = [("use_lossy", ctypes.c_int), ("lossy_quality", ctypes.c_uint8), ("method", ctypes.c_uint8),
                ("use_predictor_transform", ctypes.c_int)]


class _Metadata(ctypes.Structure):
    _fields_ = [("icc", ctypes.c_void_p), ("icc_len", ctypes.c_size_t), ("exif", ctypes.c_void_p),
                ("exif_len", ctypes.c_size_t), ("xmp", ctypes.c_void_p), ("xmp_len", ctypes.c_size_t)]


class _WebpInfo(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32), ("has_alpha", ctypes.c_int),
                ("is_lossy", ctypes.c_int), ("is_lossless", ctypes.c_int), ("is_animated", ctypes.c_int),
                ("vp8_offset", ctypes.c_uint64), ("vp8_len", ctypes.c_uint64)]


# (name, restype, argtypes) for every symbol in include/zwebp.h
_VP, _SZ, _U32, _I, _U8 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint8
SIGNATURES = [
    ("zw_ctx_create", _I, [_I, ctypes.POINTER(_VP)]),
    ("zw_ctx_destroy", None, [_VP]),
    ("zw_ctx_release_buffers", None, [_VP]),
    ("zw_strerror", ctypes.c_char_p, [_I]),
    ("zw_bytes_free", None, [ctypes.POINTER(_Bytes)]),
    ("zw_frame_free", None, [ctypes.POINTER(_Frame)]),
    ("zw_encode_frame_lossy", _I, [_VP, _VP, _SZ, _U32, _U32, _I, _U8, _U8, ctypes.POINTER(_Bytes)]),
    ("zw_encode_frame_lossy_ex", _I, [_VP, _VP, _SZ, _U32, _U32, _I, _U8, _U8, _I, ctypes.POINTER(_Bytes)]),
    ("zw_encode_webp", _I, [_VP, _VP, _SZ, _U32, _U32, _I, _U8, _U8, ctypes.POINTER(_Bytes)]),
    ("zw_encode_webp_ex", _I, [_VP, _VP, _SZ, _U32, _U32, _I, ctypes.POINTER(_EncParams), ctypes.POINTER(_Metadata),
                               ctypes.POINTER(_Bytes)]),
    ("zw_encode_frame_lossless", _I, [_VP, _SZ, _U32, _U32, _I, _I, ctypes.POINTER(_Bytes)]),
    ("zw_encode_alpha", _I, [_VP, _SZ, _U32, _U32, _I, ctypes.POINTER(_Bytes)]),
    ("zw_encode_batch", _I, [_VP, _I, ctypes.POINTER(_Image), _U8, _U8, ctypes.POINTER(_Bytes)]),
    ("zw_encode_batch_ex", _I, [_VP, _I, ctypes.POINTER(_Image), _U8, _U8, _I, ctypes.POINTER(_Bytes)]),
    ("zw_encode_webp_batch", _I, [_VP, _I, ctypes.POINTER(_Image), _U8, _U8, ctypes.POINTER(_Bytes)]),
    ("zw_vp8_decode_frame", _I, [_VP, _VP, _SZ, ctypes.POINTER(_Frame)]),
    ("zw_vp8_decode_batch", _I, [_VP, _I, ctypes.POINTER(_VP), ctypes.POINTER(_SZ), ctypes.POINTER(_Frame)]),
    ("zw_vp8_decode_rgb", _I, [_VP, _VP, _SZ, _I, _I, ctypes.POINTER(_Bytes), ctypes.POINTER(_U32),
                               ctypes.POINTER(_U32)]),
    ("zw_vp8_decode_rgb_batch", _I, [_VP, _I, ctypes.POINTER(_VP), ctypes.POINTER(_SZ), _I, _I,
                                     ctypes.POINTER(_Bytes), _VP, _VP]),
    ("zw_vp8_decode_rgb_batch_into", _I, [_VP, _I, ctypes.POINTER(_VP), ctypes.POINTER(_SZ), _I, _I,
                                          ctypes.POINTER(_VP), ctypes.POINTER(_SZ), _U32, _VP, _VP]),
    ("zw_webp_parse", _I, [_VP, _SZ, ctypes.POINTER(_WebpInfo)]),
    ("zw_webp_decode_into", _I, [_VP, _VP, _SZ, _I, _I, _VP, _SZ, _U32, ctypes.POINTER(_U32),
                                 ctypes.POINTER(_U32)]),
    ("zw_webp_decode", _I, [_VP, _VP, _SZ, _I, _I, ctypes.POINTER(_Bytes), ctypes.POINTER(_U32),
                            ctypes.POINTER(_U32)]),
    ("zw_decode_rgb_kernel_ms", _I, [_VP, ctypes.POINTER(ctypes.c_float)]),
    ("zw_yuv_to_rgb", _I, [_VP, _VP, _VP, _VP, _U32, _U32, _U32, _U32, _I, _I, _VP]),
    ("zw_rgb_to_yuv420", _I, [_VP, _VP, _U32, _U32, _I, _VP, _VP, _VP]),
    ("zw_transform_quant_blocks", _I, [_VP, _SZ, _VP, _VP, _I, _I, _I, _I, _VP, _VP]),
    ("zw_transform_quant_blocks_device", _I, [_VP, _VP, _SZ, _VP, _VP, _I, _I, _I, _I, _VP, _VP]),
    ("zw_transform_quant_mbs", _I, [_VP, _I, _U32, _U32, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP]),
    ("zw_xmb_seg_table_bytes", _SZ, [_I]),
    ("zw_xmb_seg_table", _I, [_I, _VP, _VP]),
    ("zw_transform_quant_mbs_device", _I, [_VP, _VP, _I, _U32, _U32, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP]),
    ("zw_transform_quant_mbs_rgb", _I, [_VP, _I, _U32, _U32, _I, _VP, _VP, _VP, _VP, _VP, _VP, _VP]),
    ("zw_transform_quant_mbs_rgb_device", _I, [_VP, _VP, _I, _U32, _U32, _I, _VP, _SZ, _VP, _VP, _VP, _VP, _VP, _VP]),
    ("zw_quant_blocks", _I, [_VP, _I, _VP, _VP, _I, _I, _I, _U32, _I, _I, _I, _VP, _VP, _VP]),
    ("zw_loop_filter_frame", _I, [_VP, _VP, _VP, _VP, _U32, _U32, _VP, _I, _I, _I, _I, _I, _VP, _I, _I, _I]),
    ("zw_pipe_create", _I, [_VP, _I, _U32, _U32, _I, _U8, _U8, ctypes.POINTER(_VP)]),
    ("zw_pipe_destroy", None, [_VP]),
    ("zw_pipe_input_device_ptr", _VP, [_VP]),
    ("zw_pipe_upload", _I, [_VP, _I, _VP, _SZ]),
    ("zw_pipe_set_container", _I, [_VP, _I, ctypes.POINTER(_VP)]),
    ("zw_pipe_set_token_partitions", _I, [_VP, _I]),
    ("zw_decode_kernel_times", _I, [_VP, _VP]),
    ("zw_decode_stage_times", _I, [_VP, _VP]),
    ("zw_decode_token_ms", _I, [_VP, _VP]),
    ("zw_decode_token_stages", _I, [_VP, _VP]),
    ("zw_dbg_tokl_frame", _I, [_VP, _SZ, ctypes.POINTER(_I)]),
    ("zw_dbg_seam_stats", _I, [_VP, _I]),
    ("zw_pipe_encode", _I, [_VP]),
    ("zw_pipe_encode_repeat", _I, [_VP, _I]),
    ("zw_pipe_encode_host", _I, [_VP, _I, _VP]),
    ("zw_pipe_run_pass1", _I, [_VP, _I]),
    ("zw_pipe_run_device", _I, [_VP]),
    ("zw_pipe_output", _I, [_VP, _I, ctypes.POINTER(_Bytes)]),
    ("zw_pipe_read_planes", _I, [_VP, _I, _I, _VP, _VP, _VP]),
    ("zw_pipe_read_mbinfo", _I, [_VP, _I, _I, _VP, _VP]),
    ("zw_pipe_read_alpha", _I, [_VP, _I, _VP]),
    ("zw_pipe_enable_debug", _I, [_VP]),
    ("zw_pipe_read_debug", _I, [_VP, _I, _VP]),
    ("zw_pipe_read_segments", _I, [_VP, _I, _VP]),
    ("zw_pipe_read_probs", _I, [_VP, _I, _VP, ctypes.POINTER(_I)]),
    ("zw_pipe_kernel_times", _I, [_VP, ctypes.POINTER(ctypes.c_float), _I]),
    ("zw_pipe_lanes", _I, [_VP]),
    ("zw_pipe_launch_frames", _I, [_VP]),
    ("zw_host_threads", _I, []),
]

_LIB = None


def load_library():
    """Load libzwebp.so (no device access).  Raises if it is not built."""
    global _LIB
    if _LIB is None:
        path = library_path()
        if not os.path.exists(path):
            raise ImportError(f"zwebp: HIP library not built ({path}); run `make -C image-webp_amd`")
        L = ctypes.CDLL(path)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def _check(rc, what, cls=ZwError):
    if rc != 0:
        raise cls(rc, what)


def host_threads():
    """Host worker threads per process (zw_host_threads)."""
    return load_library().zw_host_threads()


class Context:
    """One HIP device + stream (zw_ctx).  Not thread-safe; one per thread."""

    def __init__(self, device=0):
        L = load_library()
        h = ctypes.c_void_p()
        _check(L.zw_ctx_create(device, ctypes.byref(h)), "zw_ctx_create")
        self._h = h
        self._lib = L
        self.device = device

    @property
    def handle(self):
        return self._h

    def release_buffers(self):
        """Free the grow-only device scratch / pinned staging (zw_ctx_release_buffers)."""
        if self._h:
            self._lib.zw_ctx_release_buffers(self._h)

    def close(self):
        if self._h:
            self._lib.zw_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_DEFAULT = {}


def _ctx(ctx):
    """The caller's context, else this thread's default one (a zw_ctx is not
    thread-safe, and ctypes releases the GIL during every call)."""
    if ctx is not None:
        return ctx
    key = (os.getpid(), threading.get_ident())
    if key not in _DEFAULT:
        dev = int(os.environ.get("LOCAL_RANK", "0")) if os.environ.get("ZWEBP_DEVICE") is None else int(
            os.environ["ZWEBP_DEVICE"])
        _DEFAULT[key] = Context(dev)
    return _DEFAULT[key]


def _take_bytes(L, b):
    out = ctypes.string_at(b.data, b.len) if b.len else b""
    L.zw_bytes_free(ctypes.byref(b))
    return out


def _as_u8(data):
    if isinstance(data, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(data), np.uint8)
    return np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)


def encode_frame_lossy(data, width, height, color, quality=75, method=4, ctx=None, token_partitions=1):
    """encode_frame_lossy (encoder/vp8.rs:3132): raw VP8 frame bytes.
    token_partitions (1, 2, 4, 8): MB row y's tokens in partition y % n
    (vp8.rs:352-354, :1419-1421; the reference fixes 1), coded on parallel
    host threads; 1 gives the reference's bytes."""
    c = _ctx(ctx)
    L = c._lib
    a = _as_u8(data)
    out = _Bytes()
    _check(L.zw_encode_frame_lossy_ex(c.handle, _ptr(a), a.size, width, height, color, quality, method,
                                      token_partitions, ctypes.byref(out)), "encode_frame_lossy", EncodingError)
    return _take_bytes(L, out)


def encode_batch(images, width, height, color, quality=75, method=4, ctx=None, token_partitions=1):
    """Encode many same-sized frames in one device pass; returns list of VP8 frames."""
    c = _ctx(ctx)
    L = c._lib
    arrs = [_as_u8(im) for im in images]
    n = len(arrs)
    imgs = (_Image * n)()
    for i, a in enumerate(arrs):
        imgs[i] = _Image(a.ctypes.data, a.size, width, height, color)
    outs = (_Bytes * n)()
    _check(L.zw_encode_batch_ex(c.handle, n, imgs, quality, method, token_partitions, outs), "encode_batch",
           EncodingError)
    return [_take_bytes(L, outs[i]) for i in range(n)]


def encode_webp_batch(images, width, height, color, quality=75, method=4, ctx=None):
    """n WebPEncoder::encode calls with EncoderParams::lossy(quality, method) in
    one device pass: a RIFF container per frame (VP8X + ALPH for LA8 / RGBA8)."""
    c = _ctx(ctx)
    L = c._lib
    arrs = [_as_u8(im) for im in images]
    n = len(arrs)
    imgs = (_Image * n)()
    for i, a in enumerate(arrs):
        imgs[i] = _Image(a.ctypes.data, a.size, width, height, color)
    outs = (_Bytes * n)()
    _check(L.zw_encode_webp_batch(c.handle, n, imgs, quality, method, outs), "encode_webp_batch", EncodingError)
    return [_take_bytes(L, outs[i]) for i in range(n)]


class EncoderParams:
    """EncoderParams (encoder/api.rs:415-458).  The default is lossless (VP8L),
    quality 95, method 4, predictor transform on, as in the reference."""

    def __init__(self, use_predictor_transform=True, use_lossy=False, lossy_quality=95, method=4):
        self.use_predictor_transform = use_predictor_transform
        self.use_lossy = use_lossy
        self.lossy_quality = lossy_quality
        self.method = method

    @classmethod
    def lossy(cls, quality, method=4):
        return cls(True, True, quality, method)

    @classmethod
    def lossless(cls):
        return cls()

    @classmethod
    def default(cls):
        return cls()

    def _c(self):
        return _EncParams(int(self.use_lossy), self.lossy_quality, self.method, int(self.use_predictor_transform))


class WebPEncoder:
    """WebPEncoder (encoder/api.rs:1244-1398) writing to a bytearray-like sink:
    new / set_params / set_icc_profile / set_exif_metadata / set_xmp_metadata / encode."""

    def __init__(self, writer=None, ctx=None):
        self.writer = writer if writer is not None else bytearray()
        self.params = EncoderParams.default()
        self.ctx = ctx
        self.icc = self.exif = self.xmp = b""

    def set_params(self, params):
        self.params = params

    def set_icc_profile(self, icc):
        self.icc = bytes(icc)

    def set_exif_metadata(self, exif):
        self.exif = bytes(exif)

    def set_xmp_metadata(self, xmp):
        self.xmp = bytes(xmp)

    def encode(self, data, width, height, color):
        # lossless encodes are host entropy coding and need no device
        c = _ctx(self.ctx) if self.params.use_lossy else None
        L = c._lib if c is not None else load_library()
        a = _as_u8(data)
        bufs = [np.frombuffer(m, np.uint8) if m else None for m in (self.icc, self.exif, self.xmp)]
        md = _Metadata(*[x for b in bufs for x in ((b.ctypes.data if b is not None else None),
                                                   (b.size if b is not None else 0))])
        out = _Bytes()
        prm = self.params._c()
        _check(L.zw_encode_webp_ex(c.handle if c is not None else None, _ptr(a) if a.size else None, a.size, width,
                                   height, color, ctypes.byref(prm), ctypes.byref(md), ctypes.byref(out)),
               "WebPEncoder.encode", EncodingError)
        self.writer += _take_bytes(L, out)
        return self.writer


def encode_frame_lossless(data, width, height, color, use_predictor_transform=True):
    """encode_frame_lossless (encoder/api.rs:945): the VP8L bitstream (host coder, no device)."""
    L = load_library()
    a = _as_u8(data)
    out = _Bytes()
    _check(L.zw_encode_frame_lossless(_ptr(a) if a.size else None, a.size, width, height, color,
                                      int(use_predictor_transform), ctypes.byref(out)), "encode_frame_lossless",
           EncodingError)
    return _take_bytes(L, out)


def encode_alpha(data, width, height, color):
    """encode_alpha_lossless (encoder/api.rs:1175): the ALPH chunk payload (host coder, no device)."""
    L = load_library()
    a = _as_u8(data)
    out = _Bytes()
    _check(L.zw_encode_alpha(_ptr(a) if a.size else None, a.size, width, height, color, ctypes.byref(out)),
           "encode_alpha_lossless", EncodingError)
    return _take_bytes(L, out)


class Frame:
    """Decoded keyframe (decoder/vp8.rs:153-183): MB-aligned Y/U/V planes."""

    def __init__(self, width, height, ybuf, ubuf, vbuf, y_stride, uv_stride, filter_type, filter_level,
                 sharpness_level):
        self.width, self.height = width, height
        self.ybuf, self.ubuf, self.vbuf = ybuf, ubuf, vbuf
        self.y_stride, self.uv_stride = y_stride, uv_stride
        self.filter_type, self.filter_level, self.sharpness_level = filter_type, filter_level, sharpness_level


def _take_frame(L, f):
    """Zero-copy: the planes are numpy views of the library's buffer, freed
    (zw_frame_free) when the last view goes away."""
    ysz = f.y_stride * f.mb_rows * 16
    csz = f.uv_stride * f.mb_rows * 8
    buf = (ctypes.c_uint8 * (ysz + 2 * csz)).from_address(f.y)
    owner = _Frame()
    ctypes.pointer(owner)[0] = f
    weakref.finalize(buf, L.zw_frame_free, owner)
    a = np.ctypeslib.as_array(buf)
    return Frame(f.width, f.height, a[:ysz], a[ysz:ysz + csz], a[ysz + csz:], f.y_stride, f.uv_stride,
                 f.filter_type, f.filter_level, f.sharpness_level)


def vp8_decode_frame(data, ctx=None):
    """Vp8Decoder::decode_frame (decoder/vp8.rs:1526)."""
    c = _ctx(ctx)
    L = c._lib
    a = _as_u8(data)
    f = _Frame()
    _check(L.zw_vp8_decode_frame(c.handle, _ptr(a) if a.size else None, a.size, ctypes.byref(f)),
           "decode_frame", DecodingError)
    return _take_frame(L, f)


def decode_batch(frames, ctx=None):
    c = _ctx(ctx)
    L = c._lib
    arrs = [_as_u8(d) for d in frames]
    n = len(arrs)
    ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrs])
    lens = (ctypes.c_size_t * n)(*[a.size for a in arrs])
    outs = (_Frame * n)()
    _check(L.zw_vp8_decode_batch(c.handle, n, ptrs, lens, outs), "decode_batch", DecodingError)
    return [_take_frame(L, outs[i]) for i in range(n)]


def decode_kernel_times(ctx=None):
    """Device ms of the last decode batch on `ctx`: (k_dec_recon, k_loopfilter)."""
    c = _ctx(ctx)
    ms = (ctypes.c_float * 2)()
    _check(c._lib.zw_decode_kernel_times(c.handle, ms), "decode_kernel_times")
    return float(ms[0]), float(ms[1])


def decode_token_ms(ctx=None):
    """Device ms of the last decode batch's token parse (k_dec_tokl; 0 when
    the host parsed the tokens)."""
    c = _ctx(ctx)
    ms = ctypes.c_float()
    _check(c._lib.zw_decode_token_ms(c.handle, ctypes.byref(ms)), "decode_token_ms")
    return float(ms.value)


def dbg_tokl_frame(vp8):
    """Test hook (CPU only): (host parse code, match) for the device token
    parse's state machine stepped on the host over one VP8 frame; match 1 =
    records equal to the host parser's (or both failed), 0 = differ, -1 = a
    frame the device parse does not take."""
    L = load_library()
    a = _as_u8(vp8)
    m = ctypes.c_int(-1)
    rc = L.zw_dbg_tokl_frame(_ptr(a) if a.size else None, a.size, ctypes.byref(m))
    return rc, m.value


def dbg_seam_stats(reset=False):
    """Test hook: the encode seam's counters (batches led, frames in them, the
    largest batch) since the last reset."""
    L = load_library()
    out = (ctypes.c_uint64 * 3)()
    _check(L.zw_dbg_seam_stats(out, 1 if reset else 0), "dbg_seam_stats")
    return int(out[0]), int(out[1]), int(out[2])


def decode_token_stages(ctx=None):
    """Device time of the last batch's token parse by stage (ms): stage 1
    (k_dec_tok1, the decision chains), the count pass + offsets (k_dec_tok2
    count, scans, and the host's wait for the total), the record pass."""
    c = _ctx(ctx)
    ms = (ctypes.c_float * 3)()
    _check(c._lib.zw_decode_token_stages(c.handle, ms), "decode_token_stages")
    return float(ms[0]), float(ms[1]), float(ms[2])


def decode_stage_times(ctx=None):
    """Host stages of the last decode batch on `ctx`, wall ms summed over its
    chunks: (parse, download, fan-out)."""
    c = _ctx(ctx)
    ms = (ctypes.c_float * 3)()
    _check(c._lib.zw_decode_stage_times(c.handle, ms), "decode_stage_times")
    return float(ms[0]), float(ms[1]), float(ms[2])


class UpsamplingMethod:
    """UpsamplingMethod (decoder/api.rs:268-279): Bilinear (fancy, default) / Simple."""
    Bilinear = 0
    Simple = 1


def _take_image(L, b, w, h, bpp):
    """Zero-copy view of the library's image buffer (zw_bytes_free when unreferenced)."""
    if not b.len:
        L.zw_bytes_free(ctypes.byref(b))
        return np.zeros((h, w, bpp), np.uint8)
    buf = (ctypes.c_uint8 * b.len).from_address(b.data)
    owner = _Bytes(b.data, b.len)
    weakref.finalize(buf, L.zw_bytes_free, owner)
    return np.ctypeslib.as_array(buf).reshape(h, w, bpp)


def vp8_decode_rgb(data, bpp=3, upsampling=UpsamplingMethod.Bilinear, ctx=None):
    """decode_frame + Frame::fill_rgb / fill_rgba (decoder/vp8.rs:200-258) on the device: (h, w, bpp) u8."""
    c = _ctx(ctx)
    L = c._lib
    a = _as_u8(data)
    out, w, h = _Bytes(), ctypes.c_uint32(), ctypes.c_uint32()
    _check(L.zw_vp8_decode_rgb(c.handle, _ptr(a) if a.size else None, a.size, bpp, upsampling, ctypes.byref(out),
                               ctypes.byref(w), ctypes.byref(h)), "decode_rgb", DecodingError)
    return _take_image(L, out, w.value, h.value, bpp)


def decode_rgb_batch(frames, bpp=3, upsampling=UpsamplingMethod.Bilinear, ctx=None):
    """vp8_decode_rgb over a batch (runs of frames of one size, one device pass each)."""
    c = _ctx(ctx)
    L = c._lib
    arrs = [_as_u8(d) for d in frames]
    n = len(arrs)
    ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrs])
    lens = (ctypes.c_size_t * n)(*[a.size for a in arrs])
    outs = (_Bytes * n)()
    ws, hs = (ctypes.c_uint32 * n)(), (ctypes.c_uint32 * n)()
    _check(L.zw_vp8_decode_rgb_batch(c.handle, n, ptrs, lens, bpp, upsampling, outs, ws, hs), "decode_rgb_batch",
           DecodingError)
    return [_take_image(L, outs[i], ws[i], hs[i], bpp) for i in range(n)]


def _writable_u8(buf):
    a = np.asarray(buf)
    if a.dtype != np.uint8 or not a.flags.c_contiguous or not a.flags.writeable:
        raise ValueError("output must be a writable C-contiguous uint8 buffer")
    return a


def decode_rgb_batch_into(frames, outs, bpp=3, upsampling=UpsamplingMethod.Bilinear, stride_bytes=None, ctx=None):
    """decode_rgb_batch into the caller's buffers (decode_rgba_into / decode_rgb_into,
    decoder/api.rs:1004-1128): outs[i] is a writable uint8 array of at least
    stride * height bytes, rows stride_bytes apart (one stride for every
    buffer; default the widest frame's width * bpp).  Returns [(width, height)]
    per frame."""
    c = _ctx(ctx)
    L = c._lib
    arrs = [_as_u8(d) for d in frames]
    dst = [_writable_u8(o) for o in outs]
    n = len(arrs)
    if len(dst) != n or n == 0:
        raise ValueError("one output buffer per frame")
    if stride_bytes is None:
        stride_bytes = max(webp_frame_width(a) for a in arrs) * bpp
    ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrs])
    lens = (ctypes.c_size_t * n)(*[a.size for a in arrs])
    optr = (ctypes.c_void_p * n)(*[o.ctypes.data for o in dst])
    olen = (ctypes.c_size_t * n)(*[o.nbytes for o in dst])
    ws, hs = (ctypes.c_uint32 * n)(), (ctypes.c_uint32 * n)()
    _check(L.zw_vp8_decode_rgb_batch_into(c.handle, n, ptrs, lens, bpp, upsampling, optr, olen, int(stride_bytes),
                                          ws, hs), "decode_rgb_batch_into", DecodingError)
    return [(ws[i], hs[i]) for i in range(n)]


def webp_frame_width(vp8):
    """Width field of a VP8 key-frame header (frame tag + start code + 14-bit width);
    0 for a frame too short to hold one (the decode then reports the error)."""
    a = _as_u8(vp8)
    return int(a[6]) | ((int(a[7]) & 0x3F) << 8) if a.size >= 10 else 0


def _decode_into(data, output, stride_bytes, bpp, ctx):
    c = _ctx(ctx)
    a = _as_u8(data)
    o = _writable_u8(output)
    w, h = ctypes.c_uint32(), ctypes.c_uint32()
    _check(c._lib.zw_webp_decode_into(c.handle, _ptr(a) if a.size else None, a.size, bpp, UpsamplingMethod.Bilinear,
                                      o.ctypes.data, o.nbytes, int(stride_bytes), ctypes.byref(w), ctypes.byref(h)),
           "decode_into", DecodingError)
    return w.value, h.value


def decode_rgba_into(data, output, stride_bytes, ctx=None):
    """decode_rgba_into (decoder/api.rs:1004): decode into `output` with row stride; (width, height)."""
    return _decode_into(data, output, stride_bytes, 4, ctx)


def decode_rgb_into(data, output, stride_bytes, ctx=None):
    """decode_rgb_into (decoder/api.rs:1067): decode into `output` with row stride; (width, height)."""
    return _decode_into(data, output, stride_bytes, 3, ctx)


def decode_rgb_kernel_ms(ctx=None):
    """Device ms of the last RGB decode batch's k_yuv2rgb launch."""
    c = _ctx(ctx)
    ms = ctypes.c_float()
    _check(c._lib.zw_decode_rgb_kernel_ms(c.handle, ctypes.byref(ms)), "decode_rgb_kernel_ms")
    return float(ms.value)


def webp_parse(data):
    """WebPDecoder::new's container parse (decoder/api.rs:334-510): dict of the header facts."""
    L = load_library()
    a = _as_u8(data)
    info = _WebpInfo()
    rc = L.zw_webp_parse(_ptr(a) if a.size else None, a.size, ctypes.byref(info))
    _check(rc, "WebPDecoder::new", DecodingError)
    return {f: getattr(info, f) for f, _ in _WebpInfo._fields_}


def _webp_decode(data, bpp, upsampling, ctx):
    c = _ctx(ctx)
    L = c._lib
    a = _as_u8(data)
    out, w, h = _Bytes(), ctypes.c_uint32(), ctypes.c_uint32()
    _check(L.zw_webp_decode(c.handle, _ptr(a) if a.size else None, a.size, bpp, upsampling, ctypes.byref(out),
                            ctypes.byref(w), ctypes.byref(h)), "decode", DecodingError)
    return _take_image(L, out, w.value, h.value, bpp), w.value, h.value


def decode_rgba(data, ctx=None):
    """decode_rgba (decoder/api.rs:938): (flat RGBA bytes, width, height); lossy files."""
    img, w, h = _webp_decode(data, 4, UpsamplingMethod.Bilinear, ctx)
    return img.reshape(-1), w, h


def decode_rgb(data, ctx=None):
    """decode_rgb (decoder/api.rs:973): (flat RGB bytes, width, height); lossy files."""
    img, w, h = _webp_decode(data, 3, UpsamplingMethod.Bilinear, ctx)
    return img.reshape(-1), w, h


class WebPDecoder:
    """WebPDecoder (decoder/api.rs:306-906), lossy subset: new / dimensions / has_alpha /
    is_lossy / output_buffer_size / set_lossy_upsampling / read_image."""

    def __init__(self, data, ctx=None):
        self._data = _as_u8(data)
        self._ctx = ctx
        self._info = webp_parse(self._data)
        self._up = UpsamplingMethod.Bilinear

    def dimensions(self):
        return self._info["width"], self._info["height"]

    def has_alpha(self):
        return bool(self._info["has_alpha"])

    def is_lossy(self):
        return bool(self._info["is_lossy"])

    def output_buffer_size(self):
        w, h = self.dimensions()
        return w * h * (4 if self.has_alpha() else 3)

    def set_lossy_upsampling(self, method):
        self._up = method

    def read_image(self, buf=None):
        """Decodes into `buf` (a writable u8 buffer of output_buffer_size()) or returns a new array."""
        bpp = 4 if self.has_alpha() else 3
        img, _, _ = _webp_decode(self._data, bpp, self._up, self._ctx)
        flat = img.reshape(-1)
        if buf is None:
            return flat
        dst = np.frombuffer(buf, np.uint8) if not isinstance(buf, np.ndarray) else buf.reshape(-1)
        if dst.size != flat.size:
            raise DecodingError(3, "read_image: buffer size")  # ImageTooLarge / InvalidParameter in the reference
        dst[:] = flat
        return dst


def yuv_to_rgb(y, u, v, width, height, y_stride, uv_stride, bpp=3, upsampling=UpsamplingMethod.Bilinear, ctx=None):
    """fill_rgb_buffer_fancy / _simple (decoder/yuv.rs:82 / :402) on the device: (h, w, bpp) u8."""
    c = _ctx(ctx)
    y, u, v = _as_u8(y), _as_u8(u), _as_u8(v)
    out = np.zeros(width * height * bpp, np.uint8)
    _check(c._lib.zw_yuv_to_rgb(c.handle, _ptr(y), _ptr(u), _ptr(v), width, height, y_stride, uv_stride, bpp,
                                upsampling, _ptr(out)), "yuv_to_rgb")
    return out.reshape(height, width, bpp)


def rgb_to_yuv420(img, width, height, bpp, ctx=None):
    """convert_image_yuv (decoder/yuv.rs:656): MB-padded Y, U, V planes."""
    c = _ctx(ctx)
    mbw, mbh = (width + 15) // 16, (height + 15) // 16
    y = np.zeros(mbw * 16 * mbh * 16, np.uint8)
    u = np.zeros(mbw * 8 * mbh * 8, np.uint8)
    v = np.zeros(mbw * 8 * mbh * 8, np.uint8)
    a = _as_u8(img)
    if a.size != width * height * bpp:
        raise EncodingError(2, "rgb_to_yuv420")
    _check(c._lib.zw_rgb_to_yuv420(c.handle, _ptr(a), width, height, bpp, _ptr(y), _ptr(u), _ptr(v)),
           "rgb_to_yuv420")
    return y, u, v


def quant_blocks(coeffs, ctx0, ctype, first, use_trellis, lambda_, q_dc, q_ac, matrix_type, probs=None, ctx=None):
    """Quantise (n,16) natural-order coefficient blocks on the GPU.

    Returns (levels zigzag (n,16) int32, dequantised natural (n,16) int32)."""
    c = _ctx(ctx)
    co = np.ascontiguousarray(coeffs, dtype=np.int32).reshape(-1, 16)
    n = co.shape[0]
    cx = np.ascontiguousarray(np.broadcast_to(np.asarray(ctx0, np.uint8), (n,)))
    pr = None if probs is None else np.ascontiguousarray(probs, dtype=np.uint8).reshape(-1)
    lv = np.zeros((n, 16), np.int32)
    dq = np.zeros((n, 16), np.int32)
    ut = 2 if use_trellis == 2 else (1 if use_trellis else 0)  # 2: lane-parallel trellis kernel
    _check(c._lib.zw_quant_blocks(c.handle, n, _ptr(co), _ptr(cx), ctype, first, ut, lambda_,
                                  q_dc, q_ac, matrix_type, _ptr(pr), _ptr(lv), _ptr(dq)), "quant_blocks")
    return lv, dq


def transform_quant_blocks(src, pred, q_dc, q_ac, matrix_type=0, first=0, ctx=None):
    """Streaming DCT+quant pass on (n,16) u8 source/prediction blocks.

    Returns (levels (n,16) int16 zigzag, recon (n,16) uint8)."""
    c = _ctx(ctx)
    s = np.ascontiguousarray(src, dtype=np.uint8).reshape(-1, 16)
    p = np.ascontiguousarray(pred, dtype=np.uint8).reshape(-1, 16)
    assert s.shape == p.shape
    n = s.shape[0]
    lv = np.zeros((n, 16), np.int16)
    rc = np.zeros((n, 16), np.uint8)
    _check(c._lib.zw_transform_quant_blocks(c.handle, n, _ptr(s), _ptr(p), q_dc, q_ac, matrix_type, first,
                                            _ptr(lv), _ptr(rc)), "transform_quant_blocks")
    return lv, rc


def transform_quant_blocks_device(n, d_src, d_pred, q_dc, q_ac, matrix_type, first, d_levels, d_recon, stream=None,
                                  ctx=None):
    """Device-pointer form (e.g. torch tensor .data_ptr()); asynchronous on `stream` (int handle or None)."""
    c = _ctx(ctx)
    _check(c._lib.zw_transform_quant_blocks_device(c.handle, stream, n, d_src, d_pred, q_dc, q_ac, matrix_type, first,
                                                   d_levels, d_recon), "transform_quant_blocks_device")


def transform_quant_mbs(y, u, v, recs, seg_qi, nframes, mbw, mbh, ctx=None):
    """Streaming DCT+quant pass over per-MB records (zw_transform_quant_mbs):
    the encoder's final transform with the trellis off, every MB independent.

    y/u/v: MB-padded source planes of nframes frames; recs: (nframes*mbw*mbh, 96)
    uint8 records (zwebp.xmb.build_records); seg_qi: (nframes, 4) quantizer
    indices.  Returns (levels (nframes*nmb, 25, 16) int16 zigzag, ry, ru, rv)."""
    c = _ctx(ctx)
    nmb = mbw * mbh
    y, u, v = (np.ascontiguousarray(a, dtype=np.uint8).reshape(-1) for a in (y, u, v))
    r = np.ascontiguousarray(recs, dtype=np.uint8).reshape(-1)
    q = np.ascontiguousarray(seg_qi, dtype=np.int32).reshape(-1)
    if y.size != nframes * nmb * 256 or u.size != nframes * nmb * 64 or v.size != u.size:
        raise ValueError("planes must be MB-padded, nframes frames")
    if r.size != nframes * nmb * 96 or q.size != nframes * 4:
        raise ValueError("one 96-byte record per MB and 4 quantizer indices per frame")
    lv = np.zeros((nframes * nmb, 25, 16), np.int16)
    ry, ru, rv = np.zeros_like(y), np.zeros_like(u), np.zeros_like(v)
    _check(c._lib.zw_transform_quant_mbs(c.handle, nframes, mbw, mbh, _ptr(y), _ptr(u), _ptr(v), _ptr(r), _ptr(q),
                                         _ptr(lv), _ptr(ry), _ptr(ru), _ptr(rv)), "transform_quant_mbs")
    return lv, ry, ru, rv


def xmb_seg_table(seg_qi):
    """Host quantiser table of zw_transform_quant_mbs_device for (nframes, 4) indices (uint8 bytes)."""
    L = load_library()
    q = np.ascontiguousarray(seg_qi, dtype=np.int32).reshape(-1, 4)
    n = q.shape[0]
    out = np.zeros(L.zw_xmb_seg_table_bytes(n), np.uint8)
    _check(L.zw_xmb_seg_table(n, _ptr(q), _ptr(out)), "xmb_seg_table")
    return out


def transform_quant_mbs_device(nframes, mbw, mbh, d_y, d_u, d_v, d_recs, d_segs, d_levels, d_ry, d_ru, d_rv,
                               stream=None, ctx=None):
    """Device-pointer form of transform_quant_mbs; asynchronous on `stream` (int handle or None)."""
    c = _ctx(ctx)
    _check(c._lib.zw_transform_quant_mbs_device(c.handle, stream, nframes, mbw, mbh, d_y, d_u, d_v, d_recs, d_segs,
                                                d_levels, d_ry, d_ru, d_rv), "transform_quant_mbs_device")


def transform_quant_mbs_rgb(img, width, height, bpp, recs, seg_qi, nframes, ctx=None):
    """The streaming pass fused with convert_image_yuv (zw_transform_quant_mbs_rgb):
    nframes RGB (bpp 3) / RGBA (bpp 4) frames of width x height pixels in, the
    same (levels, ry, ru, rv) as transform_quant_mbs on the encoder's MB-padded
    planes of those frames."""
    c = _ctx(ctx)
    mbw, mbh = (width + 15) // 16, (height + 15) // 16
    nmb = mbw * mbh
    im = np.ascontiguousarray(img, dtype=np.uint8).reshape(-1)
    r = np.ascontiguousarray(recs, dtype=np.uint8).reshape(-1)
    q = np.ascontiguousarray(seg_qi, dtype=np.int32).reshape(-1)
    if im.size != nframes * width * height * bpp:
        raise ValueError("nframes frames of width x height x bpp bytes")
    if r.size != nframes * nmb * 96 or q.size != nframes * 4:
        raise ValueError("one 96-byte record per MB and 4 quantizer indices per frame")
    lv = np.zeros((nframes * nmb, 25, 16), np.int16)
    ry = np.zeros(nframes * nmb * 256, np.uint8)
    ru, rv = np.zeros(nframes * nmb * 64, np.uint8), np.zeros(nframes * nmb * 64, np.uint8)
    _check(c._lib.zw_transform_quant_mbs_rgb(c.handle, nframes, width, height, bpp, _ptr(im), _ptr(r), _ptr(q),
                                             _ptr(lv), _ptr(ry), _ptr(ru), _ptr(rv)), "transform_quant_mbs_rgb")
    return lv, ry, ru, rv


def transform_quant_mbs_rgb_device(nframes, width, height, bpp, d_img, img_stride, d_recs, d_segs, d_levels, d_ry,
                                   d_ru, d_rv, stream=None, ctx=None):
    """Device-pointer form of transform_quant_mbs_rgb; asynchronous on `stream`."""
    c = _ctx(ctx)
    _check(c._lib.zw_transform_quant_mbs_rgb_device(c.handle, stream, nframes, width, height, bpp, d_img, img_stride,
                                                    d_recs, d_segs, d_levels, d_ry, d_ru, d_rv),
           "transform_quant_mbs_rgb_device")


def loop_filter_frame(y, u, v, mbw, mbh, mb_flags, filter_type, filter_level, sharpness, segments_enabled=0,
                      seg_delta_values=0, seg_lf_level=(0, 0, 0, 0), lf_adj_enabled=0, ref_delta0=0, mode_delta0=0,
                      ctx=None):
    """In-place VP8 loop filter (decoder/vp8.rs:1172-1345) of MB-aligned planes.

    mb_flags: (mbw*mbh, 4) uint8 rows of (luma_mode, segment, skip, non_zero_dct)."""
    c = _ctx(ctx)
    fl = np.ascontiguousarray(mb_flags, dtype=np.uint8).reshape(-1)
    assert fl.size == mbw * mbh * 4
    for p, n in ((y, mbw * mbh * 256), (u, mbw * mbh * 64), (v, mbw * mbh * 64)):
        assert p.dtype == np.uint8 and p.flags.c_contiguous and p.size == n
    lf = np.asarray(seg_lf_level, dtype=np.int8)
    _check(c._lib.zw_loop_filter_frame(c.handle, _ptr(y), _ptr(u), _ptr(v), mbw, mbh, _ptr(fl), filter_type,
                                       filter_level, sharpness, segments_enabled, seg_delta_values, _ptr(lf),
                                       lf_adj_enabled, ref_delta0, mode_delta0), "loop_filter_frame")


class Pipeline:
    """Device-resident batch encoder (zw_pipe): n frames of one size in HBM."""

    def __init__(self, nframes, width, height, color=ColorType.Rgba8, quality=75, method=4, ctx=None):
        self.ctx = _ctx(ctx)
        L = self._lib = self.ctx._lib
        h = ctypes.c_void_p()
        _check(L.zw_pipe_create(self.ctx.handle, nframes, width, height, color, quality, method, ctypes.byref(h)),
               "zw_pipe_create", EncodingError)
        self._h = h
        self.n, self.width, self.height, self.color = nframes, width, height, color
        self.mbw, self.mbh = (width + 15) // 16, (height + 15) // 16

    @property
    def input_ptr(self):
        """Device pointer of the packed input frames (n * w*h*bpp bytes)."""
        return self._lib.zw_pipe_input_device_ptr(self._h)

    def upload(self, i, img):
        a = _as_u8(img)
        _check(self._lib.zw_pipe_upload(self._h, i, _ptr(a), a.size), "zw_pipe_upload")

    def set_container(self, host_frames=None, enable=True):
        """Outputs become WebP containers (WebPEncoder::encode, lossy params);
        for LA8 / RGBA8 the ALPH chunk is encoded from host_frames[i], which the
        pipeline keeps referenced."""
        self._host_frames = [_as_u8(f) for f in host_frames] if host_frames is not None else None
        ptrs = None
        if self._host_frames is not None:
            ptrs = (ctypes.c_void_p * len(self._host_frames))(*[f.ctypes.data for f in self._host_frames])
        _check(self._lib.zw_pipe_set_container(self._h, 1 if enable else 0, ptrs), "zw_pipe_set_container",
               EncodingError)

    def set_token_partitions(self, n):
        """Token partitions (1, 2, 4, 8) of every frame (zw_pipe_set_token_partitions)."""
        _check(self._lib.zw_pipe_set_token_partitions(self._h, n), "zw_pipe_set_token_partitions", EncodingError)

    def encode(self):
        _check(self._lib.zw_pipe_encode(self._h), "zw_pipe_encode", EncodingError)

    def encode_repeat(self, n):
        """Encode the batch n times back to back with batch k+1's GPU passes
        overlapping batch k's host token emission (streaming throughput)."""
        _check(self._lib.zw_pipe_encode_repeat(self._h, int(n)), "zw_pipe_encode_repeat", EncodingError)

    def encode_host(self, batches):
        """PCIe-inclusive streaming encode (zw_pipe_encode_host): batches is a list
        of nb lists of n host frames; batch b+1 is uploaded while batch b encodes.
        Outputs (output(i)) are the last batch's."""
        nb = len(batches)
        arrs = [_as_u8(im) for bt in batches for im in bt]
        if nb == 0 or len(arrs) != nb * self.n:
            raise ValueError("nb batches of n frames")
        want = self.width * self.height * (1, 2, 3, 4)[self.color]
        if any(a.size != want for a in arrs):
            raise ValueError("every frame must be width*height*bpp bytes")
        ptrs = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
        _check(self._lib.zw_pipe_encode_host(self._h, nb, ptrs), "zw_pipe_encode_host", EncodingError)

    def run_pass1(self, write_recon=True):
        _check(self._lib.zw_pipe_run_pass1(self._h, 1 if write_recon else 0), "zw_pipe_run_pass1", EncodingError)

    def run_device(self):
        _check(self._lib.zw_pipe_run_device(self._h), "zw_pipe_run_device", EncodingError)

    def output(self, i):
        b = _Bytes()
        _check(self._lib.zw_pipe_output(self._h, i, ctypes.byref(b)), "zw_pipe_output")
        return _take_bytes(self._lib, b)

    def planes(self, i, which=0):
        ys, cs = self.mbw * self.mbh * 256, self.mbw * self.mbh * 64
        y, u, v = np.zeros(ys, np.uint8), np.zeros(cs, np.uint8), np.zeros(cs, np.uint8)
        _check(self._lib.zw_pipe_read_planes(self._h, i, which, _ptr(y), _ptr(u), _ptr(v)), "zw_pipe_read_planes")
        return y, u, v

    def mbinfo(self, i, pass_=2):
        nmb = self.mbw * self.mbh
        modes = np.zeros((nmb, 20), np.uint8)
        levels = np.zeros((nmb, 25, 16), np.int16)
        _check(self._lib.zw_pipe_read_mbinfo(self._h, i, pass_, _ptr(modes), _ptr(levels)), "zw_pipe_read_mbinfo")
        return modes, levels

    def alpha(self, i):
        a = np.zeros(self.mbw * self.mbh, np.uint8)
        _check(self._lib.zw_pipe_read_alpha(self._h, i, _ptr(a)), "zw_pipe_read_alpha")
        return a

    def enable_debug(self):
        _check(self._lib.zw_pipe_enable_debug(self._h), "zw_pipe_enable_debug")

    def i4_dump(self, i):
        d = np.zeros(self.mbw * self.mbh * 16 * 34, np.int32)
        _check(self._lib.zw_pipe_read_debug(self._h, i, _ptr(d)), "zw_pipe_read_debug")
        return d.reshape(self.mbw * self.mbh, 16, 34)

    def segments(self, i):
        """(4,) int32 quantizer index of each segment of frame i (last encode)."""
        q = np.zeros(4, np.int32)
        _check(self._lib.zw_pipe_read_segments(self._h, i, _ptr(q)), "read_segments")
        return q

    def probs(self, i):
        pr = np.zeros(4 * 8 * 3 * 11, np.uint8)
        sp = ctypes.c_int()
        _check(self._lib.zw_pipe_read_probs(self._h, i, _ptr(pr), ctypes.byref(sp)), "zw_pipe_read_probs")
        return pr, sp.value

    @property
    def lanes(self):
        return self._lib.zw_pipe_lanes(self._h)

    @property
    def launch_frames(self):
        return self._lib.zw_pipe_launch_frames(self._h)

    def kernel_times(self):
        ms = (ctypes.c_float * 9)()
        n = self._lib.zw_pipe_kernel_times(self._h, ms, 9)
        _check(n, "zw_pipe_kernel_times")
        # ms: rgb2yuv, analysis+segments, pass1, pass2 (device); fetch1, stats, fetch2, emit (host wall);
        # emission CPU ms per batch (all lanes' workers)
        return list(ms)

    def close(self):
        if self._h:
            self._lib.zw_pipe_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
