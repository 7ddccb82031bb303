#!/usr/bin/env python3
"""Benchmark: 1080p lossy VP8 encodes/s at Q75 method 4 (BASELINE.json metric).

One step = one full encode of a batch of `--frames` synthetic 1920x1080 RGBA
frames already resident in HBM: rgb->yuv, analysis, segments, pass 1, device
statistics + host probabilities, pass 2 (mode search + DCT/quant/trellis +
recon) and host token emission to finished VP8 bitstreams.  value = frames
encoded by all ranks / max-over-ranks wall time of the K timed steps.  The K
steps run as a stream (Pipeline.encode_repeat): step k+1's GPU passes are
queued before step k's host token emission, as a serving deployment would run
consecutive batches; every step's bitstreams are complete inside the timed
region.  --sequential times K independent encode() calls instead.

Output check: after the timed region every bitstream of the batch is hashed
and compared with tests/golden/bench_digests.json (SHA-256 of the oracle's
bitstream for each synthetic frame, tools/make_bench_digests.py); the line
carries "verified": true only if every frame matched.

Multi-GPU: one process per GPU (torch.distributed.run); frames are sharded by
rank (independent frames, no data-path collective); a barrier brackets the
timed region and the max time is taken with an all-reduce.
  default          weak scaling: every rank encodes its own `--frames` frames
                   per step (global frames [rank*F, (rank+1)*F)).
  --total-frames T strong scaling (BASELINE config 5: 4096 x 3840x2160 over N
                   GPUs): a step encodes T frames in total, rank r the block
                   shard_range(T, r, N), in device batches of `--batch` frames.

`roofline`: the timed step's dominant kernel, k_encode_pass2_fp (pass 2 in
frame pairs: the RD mode search fused with the final DCT+quant+recon) against
HBM at SURVEY 8(d)'s 1568 algorithmic bytes per MB, with its VALU-issue
fraction from profiles/r06_encode_pmc.json: the kernel is bound by each wave's
dependent chains, far from the HBM roof by design.
`roofline_dct_quant_pass`: SURVEY.md 8(d)'s designated HBM-bound pass, the streaming
DCT+quant pass over per-MB records (k_xform_mb + k_xform_mb_i4q) on 256 frames
resident in HBM, BASELINE config 2's form: the synthetic RGBA frames in
(convert_image_yuv fused), levels + reconstructed YUV out.  ALGORITHMIC bytes =
the RGBA read (w*h*4 per frame) + levels 800 + recon 384 per MB (8(d)'s
fused-RGB->YUV form) / the average launch time from HIP events on the launch
stream.  The 96-byte record is traffic the pass moves but 8(d) does not count
(achieved_incl_records).  `yuv_planes_form` is the same pass from Y/U/V planes
at 1568 B/MB.  `copy_ceiling` runs the same loads and stores with no transform
arithmetic (ZW_XMB_VARIANT=99).  `traffic` is the PMC-measured HBM bytes per
launch from profiles/r05_xmb_pmc.json scaled to this launch.  Every frame's
levels and reconstruction are hashed against the oracle's digests.
`roofline_blocks`: k_fdct_quant, the same arithmetic on 4x4 blocks with the
prediction materialised (64 B per block counted, 16 B of prediction moved).
`encode_roofline`: the step's dominant kernel, k_encode_pass2_fp (RD mode search
fused with the final DCT+quant+recon), against the VALU issue peak of 2
wave-instructions per CU-cycle (4 SIMD32, a wave64 VALU op every 2 cycles per
SIMD): `frac` from one rocprofv3 --pmc dispatch (SQ_INSTS_VALU over that
dispatch's GRBM_GUI_ACTIVE cycles, clock_ghz from its timestamps;
profiles/r06_encode_pmc.json), `frac_live` the same instruction count over this
run's launch time at that clock.
cpu_baseline times the C restatement of the reference encoder (oracle/, -O3)
on a bounded sample of the same frames.
"""
import argparse
import hashlib
import json
import os

# Two pipeline lanes x (kernel + copy stream) plus the runtime's own streams:
# ask HIP for 8 hardware queues (default 4) so no two busy streams share one.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "image-webp_amd"))

ALG_BYTES_PER_MB = 1568           # src YUV 384 + levels 800 + recon 384
ALG_BYTES_PER_BLOCK = 64          # the same per 4x4 block: src 16 + levels 32 + recon 16
PRED_BYTES_PER_BLOCK = 16         # materialised prediction: moved, not counted (8(d))
XMB_RECORD_BYTES = 96             # k_xform_mb's per-MB record (modes, borders, diffusion terms): moved, not counted
HBM_PEAK_GBS = 8000.0
VALU_PEAK_PER_CU_CYCLE = 2.0      # wave64 VALU instructions: 4 SIMD32 x 1 per 2 cycles
CLOCK_GHZ = 2.4
XFORM_PMC = os.path.join(ROOT, "profiles", "r04_xform_pmc_traffic.json")
ENCODE_PMC = os.path.join(ROOT, "profiles", "r06_encode_pmc.json")
# FETCH_SIZE / WRITE_SIZE passes of the frame-pair encode kernels (tools/gpu_pmc_enc_traffic.sh)
ENCODE_TRAFFIC = os.path.join(ROOT, "profiles", "r06_encode_traffic.json")
DIGESTS = os.path.join(ROOT, "tests", "golden", "bench_digests.json")
XMB_PMC = os.path.join(ROOT, "profiles", "r05_xmb_pmc.json")


def pmc_traffic(path, units):
    """PMC-measured HBM bytes per launch (profiles/<file>: traffic_bytes over
    `units` of the profiled launch, scaled to `units`), or None when absent."""
    try:
        with open(path) as f:
            d = json.load(f)
        return d["traffic_bytes"] / d["units"] * units
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        return None


def encode_traffic(kernel, mbs):
    """PMC-measured HBM bytes of `kernel` over `mbs` MBs (ENCODE_TRAFFIC, per MB of
    the profiled frame-pair launch), or None when no profile is committed."""
    try:
        with open(ENCODE_TRAFFIC) as f:
            return json.load(f)[kernel]["traffic_bytes_per_mb"] * mbs
    except (OSError, KeyError, ValueError):
        return None


def xform_traffic(blocks):
    """PMC-measured HBM bytes of one k_fdct_quant launch over `blocks` blocks
    (profiles/, scaled per block), or None when no profile is committed."""
    try:
        with open(XFORM_PMC) as f:
            d = json.load(f)
        return d["traffic_bytes"] / d["blocks"] * blocks
    except (OSError, KeyError, ValueError):
        return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--frames", type=int, default=int(os.environ.get("ZW_BENCH_FRAMES", "1024")),
                    help="frames per rank per step (weak scaling)")
    ap.add_argument("--total-frames", type=int, default=0,
                    help="strong scaling: frames per step over all ranks (BASELINE config 5: 4096)")
    ap.add_argument("--batch", type=int, default=512, help="device batch in --total-frames mode (512: frame pairs)")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--quality", type=int, default=75)
    ap.add_argument("--method", type=int, default=4)
    ap.add_argument("--distinct", type=int, default=4, help="distinct synthetic frames per rank")
    ap.add_argument("--cpu-seconds", type=float, default=float(os.environ.get("ZW_BENCH_CPU_SECONDS", "12")))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="only the timed encode (no roofline / decode / single-frame side measurements)")
    ap.add_argument("--sequential", action="store_true",
                    help="time K separate encode() calls (no overlap between consecutive batches)")
    return ap.parse_args()


def cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    share = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if omp > 0:
        share = min(share, omp)
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "cpu_share": share}


def cpu_config1(O, q, m, digests, budget_s=4.0):
    """BASELINE config 1: the CPU reference path on a 768x512 frame (the Kodak
    size; Kodak is absent here, so synth_rgba frames stand in) -- the oracle's
    per-frame time on one core beside the reference's published 65 ms
    (README.md:87-93, CLAUDE.md:10-17), and its bitstreams against the digests."""
    from zwebp.shard import frame_seed
    from zwebp.synth import synth_rgba
    w, h = 768, 512
    seeds = [frame_seed(i) for i in range(4)]
    imgs = [synth_rgba(w, h, sd) for sd in seeds]
    ok = 0
    for img, sd in zip(imgs, seeds):
        rc, bs, _ = O.encode(img, w, h, 3, q, m)
        ok += rc == 0 and hashlib.sha256(bs).hexdigest() == digests.get(f"{w}x{h}/q{q}m{m}/{sd:#010x}")
    n = 0
    t0 = time.perf_counter()
    while True:
        O.encode(imgs[n % 4], w, h, 3, q, m)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 200:
            break
    return {"workload": f"{w}x{h} synth_rgba RGBA Q{q} m{m}, oracle/ C restatement (-O3), 1 thread",
            "ms_per_frame": el / n * 1e3, "frames_timed": n, "published_reference_ms": 65.0,
            "published_source": "reference README.md:87-93 (768x512 Kodak, Q75 m4, SIMD Rust, unspecified x86)",
            "verified": ok == 4, "verification": {"frames_checked": 4, "matched": int(ok)}}


def cpu_baseline(imgs, w, h, q, m, budget_s, digests=None):
    """Oracle (C restatement of the reference CPU encoder, -O3), bounded sample:
    (i) one frame on one thread, (ii) one frame per thread over the job's CPU share,
    (iii) BASELINE config 1 (768x512) on one thread beside the published figure."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    info = cpu_info()
    n = 0
    t0 = time.perf_counter()
    while True:
        rc, _, _ = O.encode(imgs[n % len(imgs)], w, h, 3, q, m)
        assert rc == 0
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 64:
            break
    out = {"value": n / el, "unit": "encodes/s", "cores": 1, "kind": "port",
           "sample": f"{n} synthetic {w}x{h} RGBA frames, Q{q} m{m}, oracle/ C restatement (-O3), 1 thread, {el:.1f} s",
           **info}
    # a batch over the visible cores, one frame per thread (ctypes
    # releases the GIL; the oracle keeps no global state), capped at the job's
    # per-process CPU share (OMP_NUM_THREADS on the GPU box: 16 of the machine's cores)
    nt = info["cpu_share"]
    if nt > 1:
        from concurrent.futures import ThreadPoolExecutor
        stop = time.perf_counter() + budget_s * 0.75
        counts = [0] * nt

        def worker(t):
            i = t
            while time.perf_counter() < stop:
                rc, _, _ = O.encode(imgs[i % len(imgs)], w, h, 3, q, m)
                assert rc == 0
                counts[t] += 1
                i += nt

        t0 = time.perf_counter()
        with ThreadPoolExecutor(nt) as ex:
            list(ex.map(worker, range(nt)))
        el = time.perf_counter() - t0
        out["batch_all_cores"] = {"value": sum(counts) / el, "unit": "encodes/s", "cores": nt,
                                  "sample": f"{sum(counts)} frames, one frame per thread, {nt} threads "
                                            f"(job CPU share of {info['affinity_cpus']} visible), {el:.1f} s"}
    out["config1"] = cpu_config1(O, q, m, digests or {})
    return out


def timed_launches(torch, dev, stream, fn, reps):
    """Average ms of fn() over reps launches, HIP events on `stream` (the launch stream)."""
    fn()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) / reps


def dct_quant_pass(ctx, torch, dev, frames, nmb, reps=5):
    """Streaming DCT+quant pass (k_fdct_quant) over `frames` frames' worth of 4x4
    blocks (24 per MB), device-resident synthetic src/pred; HIP events on the
    launch stream.  Algorithmic bytes per block: 16 src + 32 levels + 16 recon
    (the 16 B of materialised prediction are reported, not counted).  The copy
    ceiling is variant 99 (same loads and stores, no arithmetic) on the same buffers."""
    import zwebp
    n = frames * nmb * 24
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED)
    base = torch.randint(0, 256, (n, 1), dtype=torch.int16, device=dev, generator=g)
    src = (base + torch.randint(-40, 41, (n, 16), dtype=torch.int16, device=dev, generator=g)).clamp(0, 255).to(torch.uint8)
    pred = (base + torch.randint(-20, 21, (n, 16), dtype=torch.int16, device=dev, generator=g)).clamp(0, 255).to(torch.uint8)
    del base
    lv = torch.empty((n, 16), dtype=torch.int16, device=dev)
    rc = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(dev)  # a real (non-null) stream: the kernel and the events share it
    sh = stream.cuda_stream

    def run():
        zwebp.transform_quant_blocks_device(n, src.data_ptr(), pred.data_ptr(), 24, 30, 0, 0, lv.data_ptr(),
                                            rc.data_ptr(), stream=sh, ctx=ctx)

    ms = timed_launches(torch, dev, stream, run, reps)
    prev = os.environ.get("ZW_XFORM_VARIANT")
    os.environ["ZW_XFORM_VARIANT"] = "99"
    try:
        ms_copy = timed_launches(torch, dev, stream, run, reps)
    finally:
        if prev is None:
            os.environ.pop("ZW_XFORM_VARIANT", None)
        else:
            os.environ["ZW_XFORM_VARIANT"] = prev
    del src, pred, lv, rc
    torch.cuda.empty_cache()
    alg = n * ALG_BYTES_PER_BLOCK
    moved = n * (ALG_BYTES_PER_BLOCK + PRED_BYTES_PER_BLOCK)
    ach = alg / (ms * 1e-3) / 1e9
    ach_moved = moved / (ms * 1e-3) / 1e9
    copy_gbs = moved / (ms_copy * 1e-3) / 1e9
    return {"kernel": "k_fdct_quant", "workload": f"{frames} frames x {nmb} MBs x 24 4x4 blocks, Q75 Y1 matrix",
            "blocks": n, "ms_per_launch": ms, "achieved": ach, "frac": ach / HBM_PEAK_GBS, "alg_bytes_per_launch": alg,
            "achieved_incl_pred": ach_moved, "frac_incl_pred": ach_moved / HBM_PEAK_GBS,
            "copy_ceiling": {"kernel": "k_fdct_quant_copy (ZW_XFORM_VARIANT=99: same 32 B read + 48 B written "
                                       "per block, no arithmetic)", "ms_per_launch": ms_copy,
                             "achieved": copy_gbs, "frac": copy_gbs / HBM_PEAK_GBS,
                             "pass_over_copy": ms_copy / ms}}


def xmb_pass(ctx, torch, dev, pipe, nd, seeds, w, h, q, m, frames=256, reps=10, digests=None, imgs=None):
    """SURVEY 8(d)'s HBM-roofline pass: the streaming DCT+quant pass over per-MB
    records (k_xform_mb + k_xform_mb_i4q) on `frames` frames resident in HBM, in
    both source forms:
      "rgba": BASELINE config 2 -- the synthetic RGBA frames in, convert_image_yuv
              fused into the pass (zw_transform_quant_mbs_rgb_device); algorithmic
              bytes per frame = the RGBA read w*h*4 + levels 800 + recon 384 per MB
              (8(d)'s fused form, with the true RGBA size instead of 1 024 B/MB);
      "yuv":  the MB-padded Y/U/V planes in (zw_transform_quant_mbs_device);
              1 568 B/MB (source 384 + levels 800 + recon 384).
    The records carry the modes, segments and reconstructed borders the timed
    encode chose for its first `nd` distinct frames (Pipeline.mbinfo / planes)
    and deterministic error-diffusion inputs (zwebp.xmb.synthetic_derr); frame
    i is distinct frame i % nd.  The 96-byte record is traffic the pass moves
    but 8(d) does not count.  HIP events on the launch stream; the copy ceiling
    (ZW_XMB_VARIANT=99) moves the same bytes without the transform arithmetic.
    Outside the timed region every frame's levels and reconstruction are hashed
    against the oracle's digests (make_bench_digests.py) -- the same digests for
    both forms, since the fused conversion must give the pipe's planes."""
    import numpy as np
    import zwebp
    from zwebp.xmb import build_records, synthetic_derr
    mbw, mbh = (w + 15) // 16, (h + 15) // 16
    nmb = mbw * mbh
    recs, srcs, sq = [], [], []
    for i in range(nd):
        md = pipe.mbinfo(i, 2)[0]
        ry, ru, rv = pipe.planes(i, 1)
        recs.append(build_records(mbw, mbh, md, ry, ru, rv, synthetic_derr(nmb, seeds[i])))
        srcs.append(pipe.planes(i, 0))
        sq.append(pipe.segments(i))
    pick = [i % nd for i in range(frames)]
    tR = torch.from_numpy(np.concatenate([recs[i].reshape(-1) for i in pick])).to(dev)
    tS = torch.from_numpy(zwebp.xmb_seg_table(np.stack([sq[i] for i in pick]))).to(dev)
    lv = torch.empty(frames * nmb * 400, dtype=torch.int16, device=dev)
    oY = torch.empty(frames * nmb * 256, dtype=torch.uint8, device=dev)
    oU = torch.empty(frames * nmb * 64, dtype=torch.uint8, device=dev)
    oV = torch.empty_like(oU)
    stream = torch.cuda.Stream(dev)
    sh = stream.cuda_stream
    mbs = frames * nmb

    def check():
        ok = bad = miss = 0
        if digests is None:
            return ok, bad, miss
        L = lv.view(frames, nmb * 400).cpu().numpy()
        Y, U, V = (t.view(frames, -1).cpu().numpy() for t in (oY, oU, oV))
        for f in range(frames):
            want = digests.get(f"xmb/{w}x{h}/q{q}m{m}/{seeds[pick[f]]:#010x}")
            if want is None:
                miss += 1
                continue
            hsh = hashlib.sha256()
            for a in (L[f], Y[f], U[f], V[f]):
                hsh.update(a.tobytes())
            ok, bad = (ok + 1, bad) if hsh.hexdigest() == want else (ok, bad + 1)
        return ok, bad, miss

    def leg(run, alg, src_moved, name):
        lv.zero_()
        ms = timed_launches(torch, dev, stream, run, reps)
        ok, bad, miss = check()
        prev = os.environ.get("ZW_XMB_VARIANT")
        os.environ["ZW_XMB_VARIANT"] = "99"
        try:
            ms_copy = timed_launches(torch, dev, stream, run, reps)
        finally:
            if prev is None:
                os.environ.pop("ZW_XMB_VARIANT", None)
            else:
                os.environ["ZW_XMB_VARIANT"] = prev
        moved = src_moved + mbs * (1184 + XMB_RECORD_BYTES)
        ach = alg / (ms * 1e-3) / 1e9
        copy_gbs = moved / (ms_copy * 1e-3) / 1e9
        return {"kernel": "k_xform_mb + k_xform_mb_i4q", "source": name,
                "workload": f"{frames} frames x {nmb} MBs ({w}x{h}), the timed encode's modes",
                "mbs_per_launch": mbs, "alg_bytes_per_launch": alg, "alg_bytes_per_mb": alg / mbs,
                "record_bytes_per_mb": XMB_RECORD_BYTES, "ms_per_launch": ms, "achieved": ach,
                "frac": ach / HBM_PEAK_GBS, "achieved_incl_records": moved / (ms * 1e-3) / 1e9,
                "verified": bad == 0 and miss == 0 and ok == frames,
                "verification": {"frames_checked": ok + bad + miss, "matched": ok, "mismatched": bad,
                                 "no_digest": miss},
                "copy_ceiling": {"kernel": "k_xform_mb<copy> (ZW_XMB_VARIANT=99: the same bytes in and out, "
                                           "levels as one contiguous run, no transform arithmetic)", "ms_per_launch": ms_copy, "achieved": copy_gbs,
                                 "frac": copy_gbs / HBM_PEAK_GBS, "pass_over_copy": ms_copy / ms}}

    out = {}
    if imgs is not None:
        fb = w * h * 4
        tI = torch.from_numpy(np.concatenate([np.ascontiguousarray(imgs[i]).reshape(-1) for i in pick])).to(dev)

        def run_rgba():
            zwebp.transform_quant_mbs_rgb_device(frames, w, h, 4, tI.data_ptr(), fb, tR.data_ptr(), tS.data_ptr(),
                                                 lv.data_ptr(), oY.data_ptr(), oU.data_ptr(), oV.data_ptr(),
                                                 stream=sh, ctx=ctx)
        out["rgba"] = leg(run_rgba, frames * (fb + 1184 * nmb), frames * fb, "RGBA frames (fused convert_image_yuv)")
        del tI
    tY = torch.from_numpy(np.concatenate([srcs[i][0] for i in pick])).to(dev)
    tU = torch.from_numpy(np.concatenate([srcs[i][1] for i in pick])).to(dev)
    tV = torch.from_numpy(np.concatenate([srcs[i][2] for i in pick])).to(dev)

    def run_yuv():
        zwebp.transform_quant_mbs_device(frames, mbw, mbh, tY.data_ptr(), tU.data_ptr(), tV.data_ptr(), tR.data_ptr(),
                                         tS.data_ptr(), lv.data_ptr(), oY.data_ptr(), oU.data_ptr(), oV.data_ptr(),
                                         stream=sh, ctx=ctx)
    out["yuv"] = leg(run_yuv, mbs * ALG_BYTES_PER_MB, mbs * 384, "MB-padded Y/U/V planes")
    del tY, tU, tV, tR, tS, lv, oY, oU, oV
    torch.cuda.empty_cache()
    return out


def device_tokens_leg(ctx, streams, frames, tags, digests):
    """Batch decode where the device token parse takes part (k_dec_tok1, one
    frame's decision chain per lane, then k_dec_tok2, every MB replayed from its
    snapshot): the chain of one frame takes about as long as the whole launch,
    whatever its frame count, so the auto split hands the device the frames the
    host would not finish in that time.  The same batch with ZW_DEC_TOKENS=host
    for comparison.  Planes of a sample of frames across the host and device
    shares (every 61st) are hashed against the oracle's decode digests."""
    import zwebp
    batch = [streams[i % len(streams)] for i in range(frames)]
    res = {}
    vy = [0, 0, 0]
    for mode in ("host", "auto"):
        old = os.environ.get("ZW_DEC_TOKENS")
        if mode == "host":
            os.environ["ZW_DEC_TOKENS"] = "host"
        else:
            os.environ.pop("ZW_DEC_TOKENS", None)
        try:
            zwebp.decode_batch(batch[:256], ctx=ctx)  # (warm-up: pool, staging)
            t0 = time.perf_counter()
            dec = zwebp.decode_batch(batch, ctx=ctx)
            el = time.perf_counter() - t0
            st = zwebp.decode_stage_times(ctx=ctx)
            ts = zwebp.decode_token_stages(ctx=ctx)
            res[mode] = {"decodes_per_s": frames / el, "device_token_ms": zwebp.decode_token_ms(ctx=ctx),
                         "device_token_stages_ms": {"k_dec_tok1": ts[0], "count_and_offsets": ts[1],
                                                    "records": ts[2]},
                         "host_parse_ms": st[0], "download_ms": st[1], "fanout_ms": st[2]}
            if mode == "auto" and tags is not None:
                for i in range(0, frames, 61):
                    want = digests.get("dec_yuv/" + tags[i % len(streams)])
                    if want is None:
                        vy[2] += 1
                        continue
                    hsh = hashlib.sha256()
                    for a in (dec[i].ybuf, dec[i].ubuf, dec[i].vbuf):
                        hsh.update(bytes(a))
                    vy[0 if hsh.hexdigest() == want else 1] += 1
            del dec
        finally:
            if old is None:
                os.environ.pop("ZW_DEC_TOKENS", None)
            else:
                os.environ["ZW_DEC_TOKENS"] = old
    return {"batch_frames": frames, "auto": res["auto"], "host_only": res["host"],
            "speedup": res["auto"]["decodes_per_s"] / res["host"]["decodes_per_s"],
            "verified": vy[1] + vy[2] == 0 and vy[0] > 0,
            "verification": {"sampled_frames": vy[0] + vy[1] + vy[2], "matched": vy[0], "mismatched": vy[1],
                             "no_digest": vy[2], "against": "dec_yuv/ oracle digests"}}


def decode_path(ctx, streams, frames, w, h, with_cpu, tags=None, digests=None):
    """SURVEY config 3: the decode path on this GPU.  Host bool decoding + MB
    records up, k_dec_recon (dequant, iWHT/iDCT, prediction) + k_loopfilter,
    planes down.  Single frame end to end, plus a batch for the kernels'
    throughput; algorithmic bytes 1208 B/MB (levels 800 + side info 24 + YUV 384).
    Outside the timed calls, every decoded frame's Y/U/V planes and RGBA image
    (stream i = the bench's distinct frame tags[i]) are hashed against the
    oracle's decode digests."""
    import zwebp
    one = [streams[0]]
    dec1 = zwebp.decode_batch(one, ctx=ctx)
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        zwebp.decode_batch(one, ctx=ctx)
    single_ms = (time.perf_counter() - t0) / reps * 1e3
    rk1, lf1 = zwebp.decode_kernel_times(ctx=ctx)
    # the pipelined batch rate over `pipe_frames` (parse of chunk c beside the
    # device work and download of chunk c-1; a longer batch amortises the first
    # chunk's unoverlapped parse and the last chunk's download)
    pipe_frames = 4 * frames
    pbatch = [streams[i % len(streams)] for i in range(pipe_frames)]
    # warm-up of the timed size: grows the pinned staging buffers, and its frames,
    # freed on return, leave their buffers in the library's frame pool for the
    # timed call (a decode loop's steady state; ZW_DEC_POOL_MB=0 turns it off)
    zwebp.decode_batch(pbatch, ctx=ctx)
    t0 = time.perf_counter()
    decb = zwebp.decode_batch(pbatch, ctx=ctx)  # pipelined chunks (parse / device / download overlap)
    el = time.perf_counter() - t0
    st = zwebp.decode_stage_times(ctx=ctx)
    tok_ms = zwebp.decode_token_ms(ctx=ctx)
    tok_st = zwebp.decode_token_stages(ctx=ctx)
    thr = zwebp.host_threads()
    fbytes = len(decb[0].ybuf) + len(decb[0].ubuf) + len(decb[0].vbuf)
    stages = {"host_parse_ms": st[0], "download_ms": st[1], "fanout_ms": st[2], "host_threads": thr,
              "parse_ms_per_frame_per_thread": st[0] * thr / pipe_frames,  # (over every frame of the batch)
              # the host chunks' parse and the device token parse run side by side
              "parse_bound_decodes_per_s": pipe_frames / (max(st[0], tok_ms) * 1e-3) if max(st[0], tok_ms) > 0
              else None,
              "download_gbs": pipe_frames * fbytes / (st[1] * 1e-3) / 1e9 if st[1] > 0 else None,
              "download_bound_decodes_per_s": pipe_frames / (st[1] * 1e-3) if st[1] > 0 else None,
              "device_token_ms": tok_ms, "device_token_stages_ms": {"k_dec_tok1": tok_st[0],
                                                                      "count_and_offsets": tok_st[1],
                                                                      "records": tok_st[2]},
              "token_split": os.environ.get("ZW_DEC_TOKENS", "auto"),
              "note": "wall ms summed over chunks; the parse (the host bool decoder's serial chain, every "
                      "host thread) of chunk c overlaps the download + fan-out of chunk c-1; host_parse_ms counts "
                      "the host-parsed frames only; device_token_ms: the device token parse (k_dec_tok1 + "
                      "k_dec_tok2) for the frames whose tokens the device parsed (0: none; the auto split "
                      "leaves a batch to the host when the host alone finishes first)"}
    batch = pbatch[:frames]
    vy = [0, 0, 0]  # matched, mismatched, no digest

    def tally(v, i, *arrs):
        want = digests.get(f"{i}") if digests is not None else None
        if want is None:
            v[2] += 1
            return
        hsh = hashlib.sha256()
        for a in arrs:
            hsh.update(np.ascontiguousarray(a).tobytes())
        v[0 if hsh.hexdigest() == want else 1] += 1

    import numpy as np
    if tags is not None:
        for i, fr in enumerate(dec1 + decb):
            j = 0 if i == 0 else (i - 1) % len(streams)
            tally(vy, "dec_yuv/" + tags[j], fr.ybuf, fr.ubuf, fr.vbuf)
    del decb, dec1
    dev_tok = device_tokens_leg(ctx, streams, 16 * frames, tags, digests)
    # kernel throughput: the whole batch as one launch of the per-frame kernels
    env0 = {k: os.environ.get(k) for k in ("ZW_DEC_CHUNK", "ZW_DEC_ROWS")}
    os.environ["ZW_DEC_CHUNK"], os.environ["ZW_DEC_ROWS"] = str(frames), "0"
    try:
        zwebp.decode_batch(batch, ctx=ctx)
        rk, lf = zwebp.decode_kernel_times(ctx=ctx)
    finally:
        for k, v in env0.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    nmb = ((w + 15) // 16) * ((h + 15) // 16) * frames
    ach = 1208 * nmb / ((rk + lf) * 1e-3) / 1e9
    out = {"verified": False, "verification": None,
           "single_frame_ms": single_ms, "single_frame_kernel_ms": {"k_dec_recon": rk1, "k_loopfilter": lf1},
           "batch_frames": pipe_frames, "batch_decodes_per_s": pipe_frames / el, "batch_stages": stages,
           "batch_kernel_ms": {"k_dec_recon": rk, "k_loopfilter": lf, "launch": "whole batch, one workgroup per frame"},
           "kernel_frames_per_s": frames / ((rk + lf) * 1e-3),
           "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                        "alg_bytes_per_mb": 1208},
           "device_tokens": dev_tok}
    # decode to packed RGBA (fancy upsampling on the device, k_yuv2rgb) into the
    # caller's reused buffers (decode_rgba_into, api.rs:1004), and into fresh
    # per-frame buffers (decode_rgba's Vec per call: page faults on 8 MB each);
    # k_yuv2rgb algorithmic bytes per pixel: Y 1 + U,V 0.5 read, RGBA 4 written
    bufs = [np.empty(w * h * 4, np.uint8) for _ in range(frames)]
    zwebp.decode_rgb_batch_into(batch, bufs, 4, zwebp.UpsamplingMethod.Bilinear, ctx=ctx)
    t0 = time.perf_counter()
    zwebp.decode_rgb_batch_into(batch, bufs, 4, zwebp.UpsamplingMethod.Bilinear, ctx=ctx)
    el_rgb = time.perf_counter() - t0
    yk = zwebp.decode_rgb_kernel_ms(ctx=ctx)
    vr = [0, 0, 0]
    if tags is not None:
        for i, b in enumerate(bufs):
            tally(vr, "dec_rgba/" + tags[i % len(streams)], b)
    del bufs
    out["verified"] = tags is not None and vy[1] + vy[2] + vr[1] + vr[2] == 0 and vy[0] > 0 and vr[0] > 0 and \
        dev_tok["verified"]
    out["verification"] = {"yuv": {"matched": vy[0], "mismatched": vy[1], "no_digest": vy[2]},
                           "rgba": {"matched": vr[0], "mismatched": vr[1], "no_digest": vr[2]},
                           "against": "dec_yuv/ and dec_rgba/ oracle digests (decode_frame, fill_rgba fancy)"}
    zwebp.decode_rgb_batch(batch, 4, zwebp.UpsamplingMethod.Bilinear, ctx=ctx)
    t0 = time.perf_counter()
    zwebp.decode_rgb_batch(batch, 4, zwebp.UpsamplingMethod.Bilinear, ctx=ctx)
    el_alloc = time.perf_counter() - t0
    yb = 5.5 * w * h * frames
    out["rgba"] = {"batch_decodes_per_s": frames / el_rgb, "batch_decodes_per_s_alloc": frames / el_alloc,
                   "note": "into reused caller buffers (decode_rgba_into); _alloc: a buffer per frame returned "
                           "to the caller (after a warm-up call, from the library's frame pool)",
                   "k_yuv2rgb_ms": yk,
                   "roofline": {"bound": "hbm", "achieved": yb / (yk * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": yb / (yk * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                "alg_bytes_per_px": 5.5}}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as O
        t0 = time.perf_counter()
        rc, r = O.decode(bytes(one[0]))
        out["cpu_baseline_single_frame_ms"] = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        O.yuv_to_rgb_fancy(r["y"], r["u"], r["v"], w, h, 4)
        out["rgba"]["cpu_baseline_fancy_upsample_ms"] = (time.perf_counter() - t0) * 1e3
    ctx.release_buffers()
    return out


def single_frame(ctx, img, w, h, q, m, seed, digests, reps=3):
    """Latency of one frame through the drop-in seam (zw_encode_frame_lossy,
    encode_frame_lossy vp8.rs:3132: the row-parallel kernels) and through a
    persistent one-frame pipeline (encode + output, buffers reused).  The
    seam's outputs (1 and 8 token partitions) are hashed against the oracle's
    digests outside the timed loops."""
    import zwebp
    tag = f"{w}x{h}/q{q}m{m}/{seed:#010x}"
    out1 = zwebp.encode_frame_lossy(img, w, h, zwebp.ColorType.Rgba8, q, m, ctx=ctx)
    t0 = time.perf_counter()
    for _ in range(reps):
        zwebp.encode_frame_lossy(img, w, h, zwebp.ColorType.Rgba8, q, m, ctx=ctx)
    seam_ms = (time.perf_counter() - t0) / reps * 1e3
    # the same seam with 8 token partitions, coded on parallel host threads
    out8 = zwebp.encode_frame_lossy(img, w, h, zwebp.ColorType.Rgba8, q, m, ctx=ctx, token_partitions=8)
    t0 = time.perf_counter()
    for _ in range(reps):
        zwebp.encode_frame_lossy(img, w, h, zwebp.ColorType.Rgba8, q, m, ctx=ctx, token_partitions=8)
    parts8_ms = (time.perf_counter() - t0) / reps * 1e3
    p = zwebp.Pipeline(1, w, h, zwebp.ColorType.Rgba8, q, m, ctx=ctx)
    p.upload(0, img)
    p.encode()
    t0 = time.perf_counter()
    for _ in range(reps):
        p.encode()
        p.output(0)
    pipe_ms = (time.perf_counter() - t0) / reps * 1e3
    k = p.kernel_times()
    p.close()
    v1 = hashlib.sha256(out1).hexdigest() == digests.get(tag)
    v8 = hashlib.sha256(out8).hexdigest() == digests.get("p8/" + tag)
    return {"encode_frame_lossy_ms": seam_ms, "encode_frame_lossy_8_partitions_ms": parts8_ms,
            "pipeline_1_frame_ms": pipe_ms,
            "kernel_ms": {"rgb2yuv": k[0], "analysis_segments": k[1], "encode_pass1": k[2], "encode_pass2": k[3]},
            "verified": v1 and v8, "verification": {"seam_1_partition": v1, "seam_8_partitions": v8,
                                                    "against": "oracle digests " + tag + " / p8/" + tag},
            "note": "one frame: the row-parallel encode kernels (one wave per MB row, rows handed over through "
                    "global memory); pass 1 is bounded by the chroma raster chain (quirk A5) on one wave"}


def host_resident(pipe, host_imgs, nb, w, h, q, m, seeds, digests):
    """PCIe-inclusive rate (zw_pipe_encode_host): the same batch encoded from
    host memory, as WebPEncoder::encode(&[u8]) callers hand frames over
    (encoder/api.rs:1291).  Each of the batch's frames is its own pageable host
    buffer (frame i holds the synthetic frame seeds[i % D]); per batch every
    frame crosses PCIe again; nb is the headline's batch count (--steps), so the
    pipeline's fill and drain weigh as they do in `value`.  Each lane's uploader thread copies batch b+1 into
    the second device input buffer while batch b's passes run.  RGBA frames
    cross as RGB by default (the uploader drops the alpha bytes, which the VP8
    payload does not read, while staging; rgb2yuv reads 3 bytes a pixel):
    `pinned_rgba` is the same pinned leg with ZW_UPLOAD_PACK=0, every byte
    sent.  The last batch's bitstreams are hashed against the oracle's digests."""
    import numpy as np
    import torch
    n = pipe.n
    out = {}
    for kind in ("pageable", "pinned", "pinned_rgba"):
        if kind == "pinned_rgba":
            os.environ["ZW_UPLOAD_PACK"] = "0"
        if kind == "pageable":
            frames = [np.array(host_imgs[i % len(host_imgs)], copy=True).reshape(-1) for i in range(n)]
        else:  # a serving system's page-locked input ring: no copy through the staging slots
            frames = []
            for i in range(n):
                t = torch.empty(host_imgs[0].size, dtype=torch.uint8, pin_memory=True)
                t.numpy()[:] = np.asarray(host_imgs[i % len(host_imgs)]).reshape(-1)
                frames.append(t.numpy())
        pipe.encode_host([frames])  # warm-up: allocates the second input buffer, streams, staging
        t0 = time.perf_counter()
        pipe.encode_host([frames] * nb)
        el = time.perf_counter() - t0
        os.environ.pop("ZW_UPLOAD_PACK", None)
        ok, bad, miss = verify(pipe, n, seeds, w, h, q, m, digests)
        fb = frames[0].size if kind == "pinned_rgba" else frames[0].size // 4 * 3
        del frames
        out[kind] = {"encodes_per_s": n * nb / el, "frames": n * nb, "batches": nb, "ms_per_batch": el / nb * 1e3,
                     "h2d_bytes_per_frame": fb, "h2d_gbs": n * nb * fb / el / 1e9,
                     "verified": bad == 0 and miss == 0 and ok == n,
                     "verification": {"frames_checked": ok + bad + miss, "matched": ok, "mismatched": bad,
                                      "no_digest": miss, "against": "tests/golden/bench_digests.json (last batch)"}}
    out["encodes_per_s"] = out["pageable"]["encodes_per_s"]
    out["verified"] = all(out[k]["verified"] for k in ("pageable", "pinned", "pinned_rgba"))
    out["note"] = ("zw_pipe_encode_host: every frame crosses PCIe per batch on the DMA engines, packed to RGB "
                   "through two pinned slots per uploader thread (pinned_rgba: ZW_UPLOAD_PACK=0, page-locked "
                   "frames straight to the engines as RGBA); the uploads of batch b+1 overlap batch b's kernels")
    return out


def seam_threads(threads=(1, 4, 16, 64), seconds=3.0, hw_queues=16):
    """encode_frame_lossy (vp8.rs:3132) as callers use it: T host threads, one
    context each (a context is not thread-safe), every call one 1080p frame from
    host memory, all on this one GPU; tools/seam_threads.py, run as a child
    process so that it gets its own HIP runtime with `hw_queues` hardware
    queues: each context's streams then keep a queue of their own, where with the
    bench's 8 a long pass-1 launch of one call blocks the calls queued behind it
    (measured at T = 16: 135 encodes/s with 8 queues, 273-290 with 16 or 32).
    Every output is hashed against the oracle's digest."""
    import subprocess
    env = dict(os.environ, GPU_MAX_HW_QUEUES=str(hw_queues))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "seam_threads.py"), str(seconds)] +
                       [str(t) for t in threads], env=env, capture_output=True, text=True, timeout=600)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"verified": False, "error": (r.stdout + r.stderr)[-800:]}
    d = json.loads(lines[-1])
    d["verified"] = all(v["verified"] for v in d["threads"].values())
    d["note"] = ("T threads x T contexts, zw_encode_frame_lossy per call (host RGBA in, VP8 bytes out): up to 16 "
                 "calls in flight run on their own (row-parallel kernels sharing the GPU), calls beyond that are "
                 "seam-batched into shared pipeline batches (T = 64: 195 encodes/s unbatched, ~670 batched); "
                 "child process with GPU_MAX_HW_QUEUES=%d" % hw_queues)
    return d


def container_rgba(pipe, host_imgs, steps, w, h, q, m, seeds, digests):
    """Full-container rate (WebPEncoder::encode with EncoderParams::lossy on
    RGBA input, api.rs:1291-1398): the pipe's container mode adds, per frame on
    the emission threads, the ALPH chunk (encode_alpha_lossless of the host copy
    of the frame's alpha plane) and the VP8X container.  Same device-resident
    inputs as the headline line; every whole RIFF file (VP8X + ALPH + VP8) is
    hashed against the oracle's digest outside the timed region."""
    import struct
    n = pipe.n
    pipe.set_container([host_imgs[i % len(host_imgs)] for i in range(n)])
    try:
        pipe.encode_repeat(1)
        t0 = time.perf_counter()
        pipe.encode_repeat(steps)
        el = time.perf_counter() - t0
        ok = bad = miss = 0
        alph_bytes = 0
        for i in range(n):
            c = pipe.output(i)
            if i == 0:
                off = 12
                while off + 8 <= len(c):
                    tag, ln = c[off:off + 4], struct.unpack("<I", c[off + 4:off + 8])[0]
                    if tag == b"ALPH":
                        alph_bytes = ln
                    off += 8 + ln + (ln & 1)
            want = digests.get(f"riff/{w}x{h}/q{q}m{m}/{seeds[i % len(seeds)]:#010x}")
            if want is None:
                miss += 1
            elif hashlib.sha256(c).hexdigest() == want:
                ok += 1
            else:
                bad += 1
        k = pipe.kernel_times()
    finally:
        pipe.set_container(None, enable=False)
    return {"container_rgba_encodes_per_s": n * steps / el, "frames": n * steps, "ms_per_batch": el / steps * 1e3,
            "host_emit_ms_per_batch": float(k[7]), "alph_bytes_frame0": alph_bytes,
            "verified": bad == 0 and miss == 0 and ok == n,
            "verification": {"files_checked": ok + bad + miss, "matched": ok, "mismatched": bad, "no_digest": miss,
                             "against": "riff/... oracle digests (RIFF + VP8X + ALPH + VP8)"},
            "note": "RIFF + VP8X + ALPH + VP8 per frame; inputs resident in HBM, alpha planes read from host memory"}


def container_alpha(ctx, w, h, q, m, frames, steps, seeds, digests):
    """The container leg on frames with a real alpha plane (synth_rgba kind
    "alpha": a cut-out with a soft noisy edge and a ramp band; the headline's
    frames have alpha = 255, whose ALPH chunk is ~0.9 KB): every emission
    thread codes each frame's ALPH (encode_alpha_lossless, api.rs:1175-1221)
    beside its VP8 tokens.  Own `frames`-frame pipe, device-resident input;
    whole RIFF files hashed against the oracle's riffa/ digests.  alph_ms_per_frame
    times zw_encode_alpha alone on one host thread."""
    import struct
    import zwebp
    from zwebp.synth import synth_rgba
    imgs = [synth_rgba(w, h, sd, "alpha") for sd in seeds]
    p = zwebp.Pipeline(frames, w, h, zwebp.ColorType.Rgba8, q, m, ctx=ctx)
    try:
        for i in range(frames):
            p.upload(i, imgs[i % len(imgs)])
        p.set_container([imgs[i % len(imgs)] for i in range(frames)])
        p.encode_repeat(1)
        t0 = time.perf_counter()
        p.encode_repeat(steps)
        el = time.perf_counter() - t0
        k = p.kernel_times()
        ok = bad = miss = 0
        alph_bytes = 0
        for i in range(frames):
            c = p.output(i)
            if i == 0:
                off = 12
                while off + 8 <= len(c):
                    tag, ln = c[off:off + 4], struct.unpack("<I", c[off + 4:off + 8])[0]
                    if tag == b"ALPH":
                        alph_bytes = ln
                    off += 8 + ln + (ln & 1)
            want = digests.get(f"riffa/{w}x{h}/q{q}m{m}/{seeds[i % len(seeds)]:#010x}")
            if want is None:
                miss += 1
            elif hashlib.sha256(c).hexdigest() == want:
                ok += 1
            else:
                bad += 1
    finally:
        p.close()
    zwebp.encode_alpha(imgs[0], w, h, zwebp.ColorType.Rgba8)
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        zwebp.encode_alpha(imgs[0], w, h, zwebp.ColorType.Rgba8)
    alph_ms = (time.perf_counter() - t0) / reps * 1e3
    return {"encodes_per_s": frames * steps / el, "frames": frames * steps, "ms_per_batch": el / steps * 1e3,
            "host_emit_ms_per_batch": float(k[7]), "alph_bytes_frame0": alph_bytes, "alph_ms_per_frame": alph_ms,
            "verified": bad == 0 and miss == 0 and ok == frames,
            "verification": {"files_checked": ok + bad + miss, "matched": ok, "mismatched": bad, "no_digest": miss,
                             "against": "riffa/... oracle digests (RIFF + VP8X + ALPH + VP8)"},
            "note": "RGBA frames with a cut-out alpha plane (synth_rgba kind 'alpha'); emission threads code VP8 tokens "
                    "and the ALPH chunk per frame"}


def batch_leg(ctx, w, h, q, m, frames, steps, seeds, digests, first_seed_index=0):
    """A device-resident batch of `frames` w x h frames (distinct synthetic
    frames seeds[i % len(seeds)]), `steps` pipelined batches timed after one
    warm-up, every bitstream hashed against the oracle's digests afterwards.
    BASELINE config 5 at N=1 (3840x2160) and the GPU side of config 1 (768x512)."""
    import zwebp
    from zwebp.synth import synth_rgba
    imgs = [synth_rgba(w, h, sd) for sd in seeds]
    p = zwebp.Pipeline(frames, w, h, zwebp.ColorType.Rgba8, q, m, ctx=ctx)
    try:
        for i in range(frames):
            p.upload(i, imgs[i % len(imgs)])
        p.encode_repeat(1)
        t0 = time.perf_counter()
        p.encode_repeat(steps)
        el = time.perf_counter() - t0
        k = p.kernel_times()
        ok, bad, miss = verify(p, frames, seeds, w, h, q, m, digests)
        nbytes = sum(len(p.output(i)) for i in range(min(frames, len(seeds))))
        threads = zwebp.host_threads()
        emit_s = float(k[7]) * 1e-3
        emit_cpu_s = float(k[8]) * 1e-3
        # the pass kernels' time per batch (launches of launch_frames frames run back to
        # back on the kernel stream): the GPU-side bound of ms_per_batch
        kspan = (float(k[2]) + float(k[3])) * frames / max(1, p.launch_frames)
        return {"workload": f"{w}x{h} RGBA Q{q} m{m}, {frames} frames per device batch, {steps} pipelined batches",
                "encodes_per_s": frames * steps / el, "ms_per_batch": el / steps * 1e3,
                "pass_kernels_ms_per_batch": kspan, "ms_per_batch_over_pass_kernels": (el / steps * 1e3) / kspan
                if kspan > 0 else None,
                "frames_per_step": frames, "launch_frames": p.launch_frames,
                "kernel_ms_per_launch_span": {"encode_pass1": float(k[2]), "encode_pass2": float(k[3])},
                "host_emit_ms_per_batch": float(k[7]), "host_emit_cpu_ms_per_batch": float(k[8]),
                "host_threads": threads,
                "host_emit_frames_per_s_per_core": frames / emit_cpu_s if emit_cpu_s > 0 else None,
                "host_emit_frames_per_s_per_core_wall": frames / (emit_s * threads) if emit_s > 0 else None,
                "avg_frame_bytes": nbytes / max(1, min(frames, len(seeds))),
                "verified": bad == 0 and miss == 0 and ok == frames,
                "verification": {"frames_checked": ok + bad + miss, "matched": ok, "mismatched": bad,
                                 "no_digest": miss, "against": "tests/golden/bench_digests.json (oracle SHA-256)"}}
    finally:
        p.close()


def encode_roofline(p2_ms, launch_frames, nmb):
    """k_encode_pass2 against the VALU issue peak.  `frac` comes from ONE
    rocprofv3 --pmc dispatch (committed summary): SQ_INSTS_VALU over that
    dispatch's own GRBM_GUI_ACTIVE cycles x 256 CUs x 2 per cycle, with the clock
    the dispatch ran at (its cycles over its timestamps).  `frac_live` prices the
    same instruction count over this run's launch time at that clock."""
    try:
        with open(ENCODE_PMC) as f:
            pmc = json.load(f)
        kern = "k_encode_pass2_fp" if "k_encode_pass2_fp" in pmc else "k_encode_pass2"
        d = pmc[kern]
    except (OSError, KeyError, ValueError):
        return None
    mbs = launch_frames * nmb
    insts = d["valu_insts_per_mb"] * mbs
    cus = 256
    clock = d.get("clock_ghz", CLOCK_GHZ)
    peak = VALU_PEAK_PER_CU_CYCLE * cus * clock  # G wave-instructions / s at the dispatch's clock
    achieved_pmc = d["valu_insts_per_mb"] * mbs / (d["dispatch_ms"] * 1e-3) / 1e9 if d.get("dispatch_ms") else None
    achieved = insts / (p2_ms * 1e-3) / 1e9
    return {"kernel": kern, "bound": "valu",
            "achieved": achieved_pmc if achieved_pmc is not None else achieved, "peak": peak,
            "unit": "G wave64-VALU-instructions/s",
            "frac": d.get("valu_issue_frac", achieved / peak),
            "clock_ghz": clock, "pmc_dispatch_ms": d.get("dispatch_ms"),
            "frac_live": achieved / peak, "ms_per_launch": p2_ms,
            "valu_insts_per_mb": d["valu_insts_per_mb"], "mbs_per_launch": mbs,
            "hbm_achieved": ALG_BYTES_PER_MB * mbs / (p2_ms * 1e-3) / 1e9,
            "hbm_frac": ALG_BYTES_PER_MB * mbs / (p2_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "source": "profiles/r06_encode_pmc.json (rocprofv3 --pmc SQ_INSTS_VALU + GRBM_GUI_ACTIVE in one "
                      "pass, one 512-frame frame-pair dispatch; clock from its timestamps; tools/gpu_pmc_encode.sh)"}


def launch_kernel_times(ctx, imgs, w, h, q, m, frames):
    """Per-launch device times on a one-lane pipeline of `frames` frames (the
    timed run's two lanes overlap their launches, which blurs per-kernel event
    times): ms of rgb2yuv, analysis+segments, pass 1, pass 2 per chunk of
    `launch_frames` frames.  With two chunks (512 frames) the passes run as the
    headline runs them, one frame-pair launch over both chunks
    (k_encode_pass1_fp / k_encode_pass2_fp), their time given per chunk."""
    import zwebp
    old = os.environ.get("ZW_PIPE_LANES")
    os.environ["ZW_PIPE_LANES"] = "1"
    try:
        p = zwebp.Pipeline(frames, w, h, zwebp.ColorType.Rgba8, q, m, ctx=ctx)
    finally:
        if old is None:
            os.environ.pop("ZW_PIPE_LANES", None)
        else:
            os.environ["ZW_PIPE_LANES"] = old
    try:
        for i in range(frames):
            p.upload(i, imgs[i % len(imgs)])
        p.run_device()
        best = None
        for _ in range(2):
            p.run_device()
            k = p.kernel_times()
            best = k if best is None or k[3] < best[3] else best
        return {"rgb2yuv": best[0], "analysis_segments": best[1], "encode_pass1": best[2], "encode_pass2": best[3],
                "launch_frames": p.launch_frames, "pass_launch_frames": frames if frames >= 2 * p.launch_frames
                else p.launch_frames}
    finally:
        p.close()


def load_digests():
    try:
        with open(DIGESTS) as f:
            return json.load(f)["digests"]
    except (OSError, KeyError, ValueError):
        return {}


def verify(pipe, nframes, seeds, w, h, q, m, digests):
    """Hash every output bitstream of the batch; frame i was uploaded from the
    synthetic frame seeds[i % len(seeds)].  Returns (matched, mismatched, missing)."""
    ok = bad = missing = 0
    for i in range(nframes):
        key = f"{w}x{h}/q{q}m{m}/{seeds[i % len(seeds)]:#010x}"
        want = digests.get(key)
        if want is None:
            missing += 1
            continue
        if hashlib.sha256(pipe.output(i)).hexdigest() == want:
            ok += 1
        else:
            bad += 1
    return ok, bad, missing


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch
    import torch.distributed as dist
    import zwebp
    from zwebp.shard import frame_seed, gather_counts, rank_frames, reduce_max
    from zwebp.synth import synth_rgba

    # ZW_BENCH_BACKEND / ZW_BENCH_DEVICE: rehearsal of the N>1 path on fewer GPUs
    # (e.g. gloo with every rank on device 0); the driver's runs use RCCL, one GPU per rank
    backend = os.environ.get("ZW_BENCH_BACKEND", "nccl")
    local = int(os.environ.get("ZW_BENCH_DEVICE", str(local)))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group(backend, init_method="env://")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    red_dev = dev if backend == "nccl" else None

    w, h = a.width, a.height
    # frames of this rank per step: its own F (weak) or its block of the T total (strong, config 5)
    first, n_rank = rank_frames(rank, world, a.frames, a.total_frames)
    if a.total_frames > 0:
        B = max(1, min(a.batch, n_rank))
        nbatch, rem = divmod(n_rank, B)
        scaling = "strong"
    else:
        B, nbatch, rem = a.frames, 1, 0
        scaling = "weak"
    ctx = zwebp.Context(local)
    D = max(1, min(a.distinct, B))
    seeds = [frame_seed(first + i) for i in range(D)]
    imgs = [synth_rgba(w, h, sd) for sd in seeds]
    pipes = []
    if n_rank > 0:
        pipes.append((zwebp.Pipeline(B, w, h, zwebp.ColorType.Rgba8, a.quality, a.method, ctx=ctx), nbatch))
    if rem:
        pipes.append((zwebp.Pipeline(rem, w, h, zwebp.ColorType.Rgba8, a.quality, a.method, ctx=ctx), 1))
    for pipe, _ in pipes:
        for i in range(pipe.n):
            pipe.upload(i, imgs[i % D])
    nmb = ((w + 15) // 16) * ((h + 15) // 16)

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(a.warmup):
        for pipe, nb in pipes:
            pipe.encode_repeat(nb)
    barrier()
    kt = np.zeros(9)
    t0 = time.perf_counter()
    if a.sequential:
        for _ in range(a.steps):
            for pipe, nb in pipes:
                for _ in range(nb):
                    pipe.encode()
            kt += np.array(pipes[0][0].kernel_times()) if pipes else 0
    else:
        # streaming: batch k+1's GPU passes overlap batch k's host token emission;
        # every batch is complete (bitstreams emitted) when this returns
        for pipe, nb in pipes:
            pipe.encode_repeat(nb * a.steps)
        if pipes:
            kt += np.array(pipes[0][0].kernel_times()) * a.steps
    barrier()
    el = time.perf_counter() - t0
    el = reduce_max(el, red_dev)
    frames_done = n_rank * a.steps
    total_frames = int(sum(c[0] for c in gather_counts([frames_done], red_dev)))

    # output check (outside the timed region): every bitstream of every pipe
    digests = load_digests()
    vok = vbad = vmiss = 0
    for pipe, _ in pipes:
        r = verify(pipe, pipe.n, seeds, w, h, a.quality, a.method, digests)
        vok, vbad, vmiss = vok + r[0], vbad + r[1], vmiss + r[2]
    vc = gather_counts([vok, vbad, vmiss], red_dev)
    vok, vbad, vmiss = (sum(c[i] for c in vc) for i in range(3))
    bytes_out = sum(len(pipes[0][0].output(i)) for i in range(min(B, D))) if pipes else 0

    if rank == 0:
        k = kt / max(a.steps, 1)  # ms per launch: rgb2yuv, analysis+segments, pass1, pass2
        p2_ms = float(k[3])
        per_launch = pipes[0][0].launch_frames
        threads = zwebp.host_threads()
        emit_s = float(k[7]) * 1e-3
        emit_cpu_s = float(k[8]) * 1e-3  # the emission workers' thread CPU time per batch
        line = {
            "metric": f"{w}x{h} lossy encodes/s (Q{a.quality}, method {a.method})",
            "value": total_frames / el,
            "unit": "encodes/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": el / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "verified": vbad == 0 and vmiss == 0 and vok > 0,
            "verification": {"frames_checked": vok + vbad + vmiss, "matched": vok, "mismatched": vbad,
                             "no_digest": vmiss, "against": "tests/golden/bench_digests.json (oracle SHA-256)"},
            "config": {"workload": f"encode_frame_lossy {w}x{h} RGBA Q{a.quality} m{a.method}",
                       "frames_per_step": total_frames // max(a.steps, 1),
                       "frames_per_step_per_gpu": n_rank, "device_batch": B, "distinct_frames": D,
                       "mbs_per_frame": nmb, "parallelism": f"frames sharded over {world} GPU(s)",
                       "steps_pipelined": not a.sequential,
                       "pipeline_lanes": pipes[0][0].lanes if pipes else 0,
                       **({"total_frames": a.total_frames} if a.total_frames else {})},
            "kernel_ms_per_step": {"rgb2yuv": float(k[0]), "analysis_segments": float(k[1]),
                                   "encode_pass1": float(k[2]), "encode_pass2": p2_ms, "launch_frames": per_launch},
            "kernel_ms_per_step_note": "HIP-event spans per launch on each lane's stream in the pipelined two-lane "
                                       "run: a span includes waiting for the other lane's kernels, so the phases "
                                       "do not add up to the step; kernel_ms_per_launch has one-lane kernel times",
            "host_ms_per_step": {"fetch_pass1": float(k[4]), "stats_probs": float(k[5]),
                                 "fetch_pass2": float(k[6]), "emit": float(k[7]), "threads": threads,
                                 "emit_cpu": float(k[8])},
            # frames per second of CPU time the emission workers ran (thread CPU clocks):
            # what one core sustains; the wall form (emit wall x threads) also counts the
            # workers' waits for a CPU while the two lanes' emissions overlap
            "host_emit_frames_per_s_per_core": B / emit_cpu_s if emit_cpu_s > 0 else None,
            "host_emit_frames_per_s_per_core_wall": B / (emit_s * threads) if emit_s > 0 else None,
            "avg_frame_bytes": bytes_out / max(1, min(B, D)),
        }
        # the extra legs are single-GPU measurements: only the N=1 run carries them
        extras = not a.no_extras and world == 1
        if extras:
            q, m = a.quality, a.method
            tags = [f"{w}x{h}/q{q}m{m}/{sd:#010x}" for sd in seeds]
            lk = launch_kernel_times(ctx, imgs, w, h, q, m, min(B, 512))
            line["kernel_ms_per_launch"] = lk
            er = encode_roofline(lk["encode_pass2"], lk["launch_frames"], nmb)
            line["encode_roofline"] = er
            xa = xmb_pass(ctx, torch, dev, pipes[0][0], min(B, D), seeds, w, h, q, m, 256, 10, digests, imgs)
            xm = xa["rgba"]
            # the timed step's dominant kernel (pass 2 in frame pairs) against HBM, with its
            # VALU-issue figures: it is bound by each wave's dependent chains, not by bytes
            mbs2 = lk["launch_frames"] * nmb
            ach2 = ALG_BYTES_PER_MB * mbs2 / (lk["encode_pass2"] * 1e-3) / 1e9
            line["roofline"] = {"bound": "hbm", "achieved": ach2, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": ach2 / HBM_PEAK_GBS,
                                "traffic": encode_traffic((er or {}).get("kernel", "k_encode_pass2_fp"), mbs2),
                                "traffic_note": "per chunk: FETCH_SIZE x 2 + WRITE_SIZE of a 512-frame launch "
                                                "(r06_encode_traffic.json), scaled to the chunk's MBs; 3.8 x the "
                                                "algorithmic bytes (level-cost tables, row state, the ZwMbOut records "
                                                "with their side data) at 0.05 of HBM: bytes do not bound this kernel",
                                "kernel": (er or {}).get("kernel", "k_encode_pass2_fp"),
                                "alg_bytes_per_mb": ALG_BYTES_PER_MB,
                                "alg_bytes_note": "Y/U/V source 384 + levels 800 + reconstruction 384 per MB "
                                                  "(SURVEY 8(d)), per 256-frame chunk of the pass",
                                "ms_per_chunk": lk["encode_pass2"], "mbs_per_chunk": mbs2,
                                "pass_launch_frames": lk.get("pass_launch_frames"),
                                "valu_issue_frac": er["frac"] if er else None,
                                "valu_insts_per_mb": er["valu_insts_per_mb"] if er else None,
                                "note": "the RD mode search (I16/I4/chroma candidates, trellis) is latency- and "
                                        "issue-bound (VALU issue frac above, from r06_encode_pmc.json); the HBM-bound "
                                        "DCT+quant pass SURVEY 8(d) designates is roofline_dct_quant_pass"}
            line["roofline_dct_quant_pass"] = {"bound": "hbm", "achieved": xm["achieved"], "peak": HBM_PEAK_GBS,
                                "unit": "GB/s",
                                "frac": xm["frac"], "traffic": pmc_traffic(XMB_PMC, xm["mbs_per_launch"]),
                                "kernel": "k_xform_mb<RGBA> + k_xform_mb_i4q (BASELINE config 2: RGBA in, "
                                          "DCT/quant/IDCT, levels + reconstructed YUV out)",
                                "workload": xm["workload"], "mbs_per_launch": xm["mbs_per_launch"],
                                "alg_bytes_per_mb": xm["alg_bytes_per_mb"],
                                "alg_bytes_note": "RGBA read (w*h*4 per frame) + levels 800 + recon 384 per MB: "
                                                  "SURVEY 8(d)'s fused-RGB->YUV form",
                                "alg_bytes_per_launch": xm["alg_bytes_per_launch"],
                                "ms_per_launch": xm["ms_per_launch"],
                                "record_bytes_per_mb": XMB_RECORD_BYTES,
                                "achieved_incl_records": xm["achieved_incl_records"],
                                "copy_ceiling": xm["copy_ceiling"], "verified": xm["verified"],
                                "verification": xm["verification"],
                                "traffic_source": "profiles/r05_xmb_pmc.json (rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE)",
                                "yuv_planes_form": xa["yuv"],
                                "fused_path": {"kernel": "k_encode_pass2 (RD search fused with the final "
                                                         "DCT+quant+recon, the timed step's dominant kernel)",
                                               "hbm_frac": er["hbm_frac"] if er else None,
                                               "valu_frac": er["frac"] if er else None}}
            dq = dct_quant_pass(ctx, torch, dev, 256, nmb)
            line["roofline_blocks"] = {"kernel": "k_fdct_quant (4x4 blocks, prediction materialised in HBM)",
                                       "achieved": dq["achieved"], "frac": dq["frac"],
                                       "traffic": xform_traffic(dq["blocks"]), "blocks_per_launch": dq["blocks"],
                                       "alg_bytes_per_block": ALG_BYTES_PER_BLOCK, "ms_per_launch": dq["ms_per_launch"],
                                       "achieved_incl_pred": dq["achieved_incl_pred"],
                                       "copy_ceiling": dq["copy_ceiling"],
                                       "traffic_source": "profiles/r04_xform_pmc_traffic.json (rocprofv3 --pmc)"}
            line["single_frame"] = single_frame(ctx, imgs[0], w, h, q, m, seeds[0], digests)
            streams = [bytes(pipes[0][0].output(i)) for i in range(min(B, D))]  # VP8 frames, before container mode
            line["container_rgba"] = container_rgba(pipes[0][0], imgs, 2, w, h, q, m, seeds, digests)
            line["container_rgba"]["real_alpha"] = container_alpha(ctx, w, h, q, m, 256, 3, seeds, digests)
            line["host_resident"] = host_resident(pipes[0][0], imgs, max(3, a.steps), w, h, q, m, seeds, digests)
            for k in ("pageable", "pinned", "pinned_rgba"):  # against the HBM-resident headline
                line["host_resident"][k]["of_value"] = line["host_resident"][k]["encodes_per_s"] / line["value"]
            line["seam_threads"] = seam_threads()
            line["decode_path"] = decode_path(ctx, streams, 256, w, h, not a.no_cpu_baseline, tags, digests)
            del streams
            for pipe, _ in pipes:  # free the headline batch before the 4K leg
                pipe.close()
            pipes = []
            s4 = [frame_seed(i) for i in range(4)]
            # (8 pipelined batches each: a 2-batch leg measured mostly the pipeline's fill and
            # drain; 512 frames a batch, so the passes run in frame pairs as in the headline:
            # at 4K the leg is config 5's whole 4 096-frame job at N = 1)
            line["config5_4k_n1"] = batch_leg(ctx, 3840, 2160, q, m, 512, 8, s4, digests)
            line["config1_768x512_gpu"] = batch_leg(ctx, 768, 512, q, m, 512, 8, s4, digests)
            c5 = line["config5_4k_n1"]
            fpc = c5.get("host_emit_frames_per_s_per_core")
            line["host_budget"] = {
                "threads_per_rank": threads,
                "emit_frames_per_s_per_core_1080p": line["host_emit_frames_per_s_per_core"],
                "emit_frames_per_s_per_core_4k": fpc,
                "cores_for_8x_this_gpu_1080p": 8 * line["value"] / line["host_emit_frames_per_s_per_core"]
                if line["host_emit_frames_per_s_per_core"] else None,
                "cores_for_8x_this_gpu_4k": 8 * c5["encodes_per_s"] / fpc if fpc else None,
                "note": "host cores the bool coder needs to keep 8 GPUs at this GPU's measured rate, from the "
                        "emission workers' thread CPU time (the CPU the entropy stage consumes per frame); "
                        "threads per rank = affinity CPUs / LOCAL_WORLD_SIZE, capped by OMP_NUM_THREADS"}
        line["cpu_baseline"] = None
        if not a.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(imgs, w, h, a.quality, a.method, a.cpu_seconds, digests)
        if extras:
            cb = line["cpu_baseline"] or {}
            line["configs"] = {
                "1_768x512_cpu_reference_path": {"verified": bool(cb.get("config1", {}).get("verified")) and
                                                 line["config1_768x512_gpu"]["verified"],
                                                 "see": "cpu_baseline.config1, config1_768x512_gpu"},
                "2_1080p_dct_quant_idct_kernels": {"verified": line["roofline_dct_quant_pass"]["verified"] and
                                                   line["roofline_dct_quant_pass"]["yuv_planes_form"]["verified"],
                                                   "see": "roofline_dct_quant_pass"},
                "3_1080p_decode_path": {"verified": line["decode_path"]["verified"], "see": "decode_path"},
                "4_1080p_batch_encode": {"verified": line["verified"] and line["single_frame"]["verified"] and
                                         line["container_rgba"]["verified"] and line["host_resident"]["verified"]
                                         and line["container_rgba"]["real_alpha"]["verified"]
                                         and line["seam_threads"]["verified"],
                                         "see": "value, single_frame, container_rgba, host_resident, seam_threads"},
                "5_4k_batch_n1": {"verified": line["config5_4k_n1"]["verified"], "see": "config5_4k_n1 (N=1 anchor "
                                  "of the 4096-frame split; the driver's SCALE run measures N=2/4/8)"}}
        print(json.dumps(line), flush=True)
    for pipe, _ in pipes:
        pipe.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
