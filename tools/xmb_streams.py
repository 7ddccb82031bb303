#!/usr/bin/env python3
"""k_xform_mb's copy calibration split by stream (ZW_XMB_VARIANT, RGBA source,
256 x 1920x1080 frames resident in HBM): each variant moves ONE of the pass's
streams with the pass's own access pattern -- 94 the 96-B records in, 92 the
RGBA pixels in (the pass's 8-px x 2-row items, no conversion), 93 the same
pixels with 64 x 16 contiguous bytes per load instruction, 97 the pixels in and
converted into the LDS tiles as the pass does, 96 the levels out (800 B/MB),
95 the reconstruction out (384 B/MB) -- beside the whole copy (99), the pass
itself (0) and torch's own copy / fill of a like-sized buffer.  Prints one JSON
line: ms per launch and GB/s of the stream's bytes."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-webp_amd"))


def main():
    import numpy as np
    import torch
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    import zwebp
    w, h, F, reps = 1920, 1080, 256, 10
    mbw, mbh = (w + 15) // 16, (h + 15) // 16
    nmb = mbw * mbh
    g = torch.Generator(device=dev).manual_seed(1)
    img = torch.randint(0, 256, (F * w * h * 4,), dtype=torch.uint8, device=dev, generator=g)
    recs = torch.zeros(F * nmb * 96, dtype=torch.uint8, device=dev)
    segs = torch.from_numpy(zwebp.xmb_seg_table(np.full((F, 4), 40, np.int32))).to(dev)
    lv = torch.empty(F * nmb * 400, dtype=torch.int16, device=dev)
    oY = torch.empty(F * nmb * 256, dtype=torch.uint8, device=dev)
    oU = torch.empty(F * nmb * 64, dtype=torch.uint8, device=dev)
    oV = torch.empty_like(oU)
    ctx = zwebp.Context(0)
    L = ctx._lib
    st = torch.cuda.Stream(dev)

    def launch():
        r = L.zw_transform_quant_mbs_rgb_device(ctx.handle, st.cuda_stream, F, w, h, 4, img.data_ptr(), w * h * 4,
                                                recs.data_ptr(), segs.data_ptr(), lv.data_ptr(), oY.data_ptr(),
                                                oU.data_ptr(), oV.data_ptr())
        if r:
            raise RuntimeError(f"launch failed {r}")

    def timed(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(st):
            a.record(st)
            for _ in range(reps):
                fn()
            b.record(st)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    mbs = F * nmb
    pix = F * w * h * 4
    legs = {"0": pix + mbs * (96 + 800 + 384), "99": pix + mbs * (96 + 800 + 384), "94": mbs * 96, "92": pix,
            "93": pix, "97": pix, "96": mbs * 800, "95": mbs * 384}
    out = {}
    for v, nbytes in legs.items():
        os.environ["ZW_XMB_VARIANT"] = v
        ms = timed(launch)
        out[v] = {"ms": ms, "gbs": nbytes / ms / 1e6, "bytes": nbytes}
    os.environ.pop("ZW_XMB_VARIANT", None)
    # torch references on a buffer the size of the pixel stream
    dst = torch.empty_like(img)
    with torch.cuda.stream(st):
        ms = timed(lambda: dst.copy_(img))
    out["torch_copy"] = {"ms": ms, "gbs": 2 * pix / ms / 1e6, "bytes": 2 * pix}
    with torch.cuda.stream(st):
        ms = timed(lambda: dst.fill_(7))
    out["torch_fill"] = {"ms": ms, "gbs": pix / ms / 1e6, "bytes": pix}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
