"""C-ABI boundary checks that need no GPU: libzwebp.so loads, exports every
entry point include/zwebp.h declares, the Python mirror binds all of them, and
the product refuses to run without a device (no CPU fallback)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "zwebp.h")
LIB = os.path.join(ROOT, "image-webp_amd", "zwebp", "libzwebp.so")


def _declared():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(zw_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "image-webp_amd")])
    return ctypes.CDLL(LIB)


def test_header_declares_boundary():
    names = _declared()
    for must in ("zw_encode_frame_lossy", "zw_encode_webp", "zw_encode_batch", "zw_vp8_decode_frame",
                 "zw_rgb_to_yuv420", "zw_loop_filter_frame", "zw_ctx_create", "zw_ctx_destroy"):
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_mirror_binds_every_symbol():
    import zwebp
    bound = {n for n, _, _ in zwebp.SIGNATURES}
    assert bound == set(_declared())
    zwebp.load_library()


def test_no_cpu_fallback_without_device(lib):
    """Without a HIP device the context cannot be created (ZW_EDEVICE)."""
    import zwebp
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a device is visible")
    except ImportError:
        pass
    with pytest.raises(zwebp.ZwError) as e:
        zwebp.Context(0)
    assert e.value.code == 4


def test_strerror(lib):
    import zwebp
    L = zwebp.load_library()
    assert L.zw_strerror(0) == b"ok"
    assert L.zw_strerror(10) == b"invalid VP8 magic"


def test_product_does_not_link_oracle():
    """The product library must not depend on the test oracle."""
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    assert " or_" not in out
    deps = subprocess.run(["ldd", LIB], capture_output=True, text=True).stdout
    assert "oracle" not in deps


def test_free_functions_take_plain_malloc_buffers(lib):
    """zw_bytes_free / zw_frame_free keep the C contract for buffers that did
    not come from the decoded-frame pool (the encoder's outputs, a binding's
    own malloc): they are free()d and the fields cleared; a null frame is a
    no-op.  No device is touched."""
    import zwebp
    L = zwebp.load_library()
    libc = ctypes.CDLL(None)
    libc.malloc.restype = ctypes.c_void_p
    libc.malloc.argtypes = [ctypes.c_size_t]
    for _ in range(4):
        b = zwebp._Bytes()
        b.data = libc.malloc(1 << 20)
        b.len = 1 << 20
        L.zw_bytes_free(ctypes.byref(b))
        assert not b.data and b.len == 0
        f = zwebp._Frame()
        f.y = libc.malloc(3 << 20)
        L.zw_frame_free(ctypes.byref(f))
        assert not f.y and not f.u and not f.v
    L.zw_frame_free(ctypes.byref(zwebp._Frame()))
    L.zw_bytes_free(ctypes.byref(zwebp._Bytes()))
