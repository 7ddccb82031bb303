"""ctypes binding of the oracle (oracle/liboracle.so) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_LIB = None


class MbInfo(ctypes.Structure):
    _fields_ = [("luma_mode", ctypes.c_uint8), ("bpred", ctypes.c_uint8 * 16),
                ("chroma_mode", ctypes.c_uint8), ("segment", ctypes.c_uint8),
                ("skip", ctypes.c_uint8), ("non_zero_dct", ctypes.c_uint8)]


class EncDebug(ctypes.Structure):
    _fields_ = [("src_y", ctypes.c_void_p), ("src_u", ctypes.c_void_p), ("src_v", ctypes.c_void_p),
                ("recon_y", ctypes.c_void_p), ("recon_u", ctypes.c_void_p), ("recon_v", ctypes.c_void_p),
                ("recon1_y", ctypes.c_void_p),
                ("mb_alpha", ctypes.c_void_p), ("seg_map", ctypes.c_void_p),
                ("p1_info", ctypes.c_void_p), ("p2_info", ctypes.c_void_p),
                ("levels", ctypes.c_void_p), ("i4_dump", ctypes.c_void_p),
                ("p1_stats", ctypes.c_uint32 * (4 * 8 * 3 * 11)),
                ("final_probs", ctypes.c_uint8 * (4 * 8 * 3 * 11)),
                ("seg_quant_index", ctypes.c_int * 4),
                ("segments_enabled", ctypes.c_int), ("filter_level", ctypes.c_int),
                ("base_quant_index", ctypes.c_int), ("skip_prob", ctypes.c_int),
                ("p1_top_derr_last", ctypes.c_int8 * 1),
                ("derr_in", ctypes.c_void_p)]


class FrameHdr(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int), ("mbw", ctypes.c_int), ("mbh", ctypes.c_int),
                ("filter_type", ctypes.c_int), ("filter_level", ctypes.c_int), ("sharpness", ctypes.c_int),
                ("segments_enabled", ctypes.c_int), ("seg_delta_values", ctypes.c_int),
                ("seg_lf_level", ctypes.c_int * 4), ("seg_quant_level", ctypes.c_int * 4),
                ("lf_adj_enabled", ctypes.c_int), ("ref_delta0", ctypes.c_int), ("mode_delta0", ctypes.c_int),
                ("num_partitions", ctypes.c_int)]


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(ROOT, "oracle", "liboracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(path)
        L.or_encode.restype = ctypes.c_int
        L.or_encode.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p]
        L.or_encode_parts.restype = ctypes.c_int
        L.or_encode_parts.argtypes = L.or_encode.argtypes[:7] + [ctypes.c_int] + L.or_encode.argtypes[7:]
        L.or_decode.argtypes = [ctypes.c_void_p, ctypes.c_size_t] + [ctypes.c_void_p] * 8
        L.or_decode_header.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.or_free.argtypes = [ctypes.c_void_p]
        for n in ("or_fdct_c", "or_fdct_sse2_c", "or_idct_c", "or_idct_scalar_c", "or_wht_c", "or_iwht_c"):
            getattr(L, n).argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.or_rgb_to_yuv420_c.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 3
        L.or_loop_filter_c.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.or_yuv_to_rgb_fancy_c.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
        L.or_yuv_to_rgb_simple_c.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
        L.or_analyze.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.or_bool_encoder_kat.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        L.or_trellis_kat.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.c_void_p]
        L.or_quant_blocks_c.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.or_debug_struct_size.restype = ctypes.c_size_t
        assert L.or_debug_struct_size() == ctypes.sizeof(EncDebug), "EncDebug layout mismatch"
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def blocks(fn, arr):
    a = np.ascontiguousarray(arr, dtype=np.int32).copy()
    getattr(lib(), fn)(_p(a), a.size // 16)
    return a


def quant_blocks(coeffs, ctx0, ctype, first, use_trellis, lambda_, q_dc, q_ac, matrix_type, probs=None):
    co = np.ascontiguousarray(coeffs, dtype=np.int32).reshape(-1, 16)
    n = co.shape[0]
    cx = np.ascontiguousarray(np.broadcast_to(np.asarray(ctx0, np.uint8), (n,)))
    pr = None if probs is None else np.ascontiguousarray(probs, dtype=np.uint8).reshape(-1)
    lv = np.zeros((n, 16), np.int32)
    dq = np.zeros((n, 16), np.int32)
    lib().or_quant_blocks_c(n, _p(co), _p(cx), ctype, first, 1 if use_trellis else 0, lambda_, q_dc, q_ac,
                            matrix_type, _p(pr), _p(lv), _p(dq))
    return lv, dq


def rgb_to_yuv420(img, w, h, bpp):
    mbw, mbh = (w + 15) // 16, (h + 15) // 16
    y = np.zeros(mbw * 16 * mbh * 16, np.uint8)
    u = np.zeros(mbw * 8 * mbh * 8, np.uint8)
    v = np.zeros(mbw * 8 * mbh * 8, np.uint8)
    img = np.ascontiguousarray(img, dtype=np.uint8)
    lib().or_rgb_to_yuv420_c(_p(img), w, h, bpp, _p(y), _p(u), _p(v))
    return y, u, v


def encode(img, w, h, color, quality=75, method=4, debug=False, nparts=1):
    """Returns (rc, vp8_bytes, debug_dict_or_None).  nparts: token partitions (1, 2, 4, 8)."""
    L = lib()
    img = np.ascontiguousarray(img, dtype=np.uint8)
    out = ctypes.c_void_p()
    n = ctypes.c_size_t()
    dbg = None
    keep = {}
    if debug:
        mbw, mbh = (w + 15) // 16, (h + 15) // 16
        ys, cs = mbw * 16 * mbh * 16, mbw * 8 * mbh * 8
        keep = dict(src_y=np.zeros(ys, np.uint8), src_u=np.zeros(cs, np.uint8), src_v=np.zeros(cs, np.uint8),
                    recon_y=np.zeros(ys, np.uint8), recon_u=np.zeros(cs, np.uint8), recon_v=np.zeros(cs, np.uint8),
                    recon1_y=np.zeros(ys, np.uint8),
                    mb_alpha=np.zeros(mbw * mbh, np.uint8), seg_map=np.zeros(mbw * mbh, np.uint8),
                    levels=np.zeros(mbw * mbh * 25 * 16, np.int32),
                    i4_dump=np.zeros(mbw * mbh * 16 * 34, np.int32),
                    derr_in=np.zeros(mbw * mbh * 8, np.int8))
        p1 = (MbInfo * (mbw * mbh))()
        p2 = (MbInfo * (mbw * mbh))()
        dbg = EncDebug()
        for k, a in keep.items():
            setattr(dbg, k, a.ctypes.data)
        dbg.p1_info = ctypes.addressof(p1)
        dbg.p2_info = ctypes.addressof(p2)
        keep["p1_info"] = p1
        keep["p2_info"] = p2
    rc = L.or_encode_parts(_p(img), img.size, w, h, color, quality, method, nparts, ctypes.byref(out),
                           ctypes.byref(n), ctypes.byref(dbg) if dbg is not None else None)
    data = b""
    if rc == 0:
        data = ctypes.string_at(out.value, n.value)
        L.or_free(out)
    if debug and rc == 0:
        keep["p1_stats"] = np.ctypeslib.as_array(dbg.p1_stats).copy()
        keep["final_probs"] = np.ctypeslib.as_array(dbg.final_probs).copy()
        keep["seg_quant_index"] = list(dbg.seg_quant_index)
        keep["segments_enabled"] = dbg.segments_enabled
        keep["filter_level"] = dbg.filter_level
        keep["base_quant_index"] = dbg.base_quant_index
        keep["skip_prob"] = dbg.skip_prob
        return rc, data, keep
    return rc, data, None


def decode_header(vp8):
    h = FrameHdr()
    buf = np.frombuffer(vp8, np.uint8).copy()
    rc = lib().or_decode_header(_p(buf), buf.size, ctypes.byref(h))
    return rc, h


def decode(vp8, want_unfiltered=False, want_info=False):
    rc, h = decode_header(vp8)
    if rc != 0:
        return rc, None
    mbw, mbh = h.mbw, h.mbh
    y = np.zeros(mbw * 16 * mbh * 16, np.uint8)
    u = np.zeros(mbw * 8 * mbh * 8, np.uint8)
    v = np.zeros(mbw * 8 * mbh * 8, np.uint8)
    uy = uu = uv = None
    if want_unfiltered:
        uy, uu, uv = np.zeros_like(y), np.zeros_like(u), np.zeros_like(v)
    info = (MbInfo * (mbw * mbh))() if want_info else None
    buf = np.frombuffer(vp8, np.uint8).copy()
    hdr = FrameHdr()
    rc = lib().or_decode(_p(buf), buf.size, _p(y), _p(u), _p(v), _p(uy), _p(uu), _p(uv),
                         ctypes.addressof(info) if info is not None else None, ctypes.byref(hdr))
    res = dict(y=y, u=u, v=v, hdr=hdr, mbw=mbw, mbh=mbh, uy=uy, uu=uu, uv=uv, info=info)
    return rc, res


def yuv_to_rgb_fancy(y, u, v, w, h, bpp=3):
    """fill_rgb_buffer_fancy on MB-aligned planes; cropped (w*h) planes are padded."""
    mbw, mbh = (w + 15) // 16, (h + 15) // 16
    if y.size == w * h and (w % 16 or h % 16):
        cw, ch = (w + 1) // 2, (h + 1) // 2
        Y = np.zeros((mbh * 16, mbw * 16), np.uint8)
        U = np.zeros((mbh * 8, mbw * 8), np.uint8)
        V = np.zeros((mbh * 8, mbw * 8), np.uint8)
        Y[:h, :w] = y.reshape(h, w)
        U[:ch, :cw] = u.reshape(ch, cw)
        V[:ch, :cw] = v.reshape(ch, cw)
        y, u, v = Y.reshape(-1), U.reshape(-1), V.reshape(-1)
    y, u, v = (np.ascontiguousarray(a, dtype=np.uint8) for a in (y, u, v))
    out = np.zeros(w * h * bpp, np.uint8)
    lib().or_yuv_to_rgb_fancy_c(_p(y), _p(u), _p(v), w, h, bpp, _p(out))
    return out


def yuv_to_rgb_simple(y, u, v, w, h, bpp=3):
    """fill_rgb_buffer_simple (decoder/yuv.rs:402); planes MB-padded (stride mbw*16 / mbw*8)."""
    y = np.ascontiguousarray(y, np.uint8)
    u = np.ascontiguousarray(u, np.uint8)
    v = np.ascontiguousarray(v, np.uint8)
    out = np.zeros(w * h * bpp, np.uint8)
    lib().or_yuv_to_rgb_simple_c(_p(y), _p(u), _p(v), w, h, bpp, _p(out))
    return out


def _bytes_out(fn, *args):
    L = lib()
    out, n = ctypes.c_void_p(), ctypes.c_size_t()
    rc = fn(*args, ctypes.byref(out), ctypes.byref(n))
    data = ctypes.string_at(out.value, n.value) if rc == 0 and out.value else b""
    if out.value:
        L.or_free(out)
    return rc, data


def encode_lossless(img, w, h, color, use_predictor=True, implicit_dims=False):
    """encode_frame_lossless (encoder/api.rs:945): (rc, VP8L bitstream bytes)."""
    L = lib()
    L.or_encode_frame_lossless.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p]
    a = np.ascontiguousarray(img, dtype=np.uint8).reshape(-1)
    return _bytes_out(L.or_encode_frame_lossless, _p(a) if a.size else None, a.size, w, h, color,
                      int(use_predictor), int(implicit_dims))


def encode_alpha(img, w, h, color):
    """encode_alpha_lossless (encoder/api.rs:1175): (rc, ALPH chunk payload)."""
    L = lib()
    L.or_encode_alpha.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_void_p]
    a = np.ascontiguousarray(img, dtype=np.uint8).reshape(-1)
    return _bytes_out(L.or_encode_alpha, _p(a) if a.size else None, a.size, w, h, color)


def rust_sort_unstable_by_key(keys):
    """<[(usize, u32)]>::sort_unstable_by_key(|&(_, k)| k) as restated in the
    oracle (Rust 1.92 ipnsort; api.rs:259-260).  Returns (indexes, keys)."""
    L = lib()
    L.or_rust_sort_unstable_by_key.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    k = np.ascontiguousarray(keys, dtype=np.uint32).copy()
    idx = np.arange(len(k), dtype=np.uint32)
    if len(k):
        L.or_rust_sort_unstable_by_key(_p(idx), _p(k), len(k))
    return idx, k


def riff_vp8_chunk(data):
    """Extract the 'VP8 ' chunk payload from a RIFF WebP file."""
    assert data[:4] == b"RIFF" and data[8:12] == b"WEBP"
    off = 12
    while off + 8 <= len(data):
        tag = data[off:off + 4]
        size = int.from_bytes(data[off + 4:off + 8], "little")
        if tag == b"VP8 ":
            return data[off + 8:off + 8 + size]
        off += 8 + size + (size & 1)
    raise ValueError("no VP8 chunk")


def xform_mbs(y, u, v, recs, seg_qi, nframes, mbw, mbh):
    """Streaming final transform over per-MB records (checker of zw_transform_quant_mbs).
    Returns (levels (nframes*nmb, 25, 16) int16 zigzag, ry, ru, rv)."""
    nmb = mbw * mbh
    y, u, v = (np.ascontiguousarray(a, dtype=np.uint8).reshape(-1) for a in (y, u, v))
    r = np.ascontiguousarray(recs, dtype=np.uint8).reshape(-1)
    q = np.ascontiguousarray(seg_qi, dtype=np.int32).reshape(-1)
    assert r.size == nframes * nmb * 96 and q.size == nframes * 4
    lv = np.zeros((nframes * nmb, 25, 16), np.int16)
    ry, ru, rv = np.zeros_like(y), np.zeros_like(u), np.zeros_like(v)
    lib().or_xform_mbs(nframes, mbw, mbh, _p(y), _p(u), _p(v), _p(r), _p(q), _p(lv), _p(ry), _p(ru), _p(rv))
    return lv, ry, ru, rv
