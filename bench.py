#!/usr/bin/env python3
"""Benchmark: 1080p lossy VP8 encodes/s at Q75 method 4 (BASELINE.json metric).

One step = one full encode of a batch of `--frames` synthetic 1920x1080 RGBA
frames already resident in HBM: rgb->yuv, analysis, segments, pass 1, host
statistics/probabilities, pass 2 (mode search + DCT/quant/trellis + recon) and
host token emission to finished VP8 bitstreams.  value = frames encoded by all
ranks / max-over-ranks wall time of the K timed steps.  The K steps run as a
stream (Pipeline.encode_repeat): step k+1's GPU passes are queued before step
k's host token emission, as a serving deployment would run consecutive
batches; every step's bitstreams are complete inside the timed region.
--sequential times K independent encode() calls instead.

Multi-GPU: one process per GPU (torch.distributed.run); frames are sharded by
rank (independent frames, no data-path collective); a barrier brackets the
timed region and the max time is taken with an all-reduce.

The `roofline` object is SURVEY.md 8(d)'s designated HBM-bound kernel, the
streaming DCT+quant pass k_fdct_quant: 80 algorithmic bytes per 4x4 block
(16 src + 16 pred + 32 levels + 16 recon) x blocks per launch / average launch
time from HIP events on the launch stream, over 256 frames' worth of blocks
(24 per MB) resident in HBM; `traffic` is the PMC-measured HBM bytes per launch
from profiles/ (FETCH_SIZE x2 + WRITE_SIZE, tools/gpu_pmc_xform.sh), scaled to
this launch size.  `encode_kernel` reports the step's dominant kernel
(k_encode pass 2, whose final DCT+quant is fused with the RD mode search)
against the same HBM peak using 8(d)'s 1568 B/MB -- it is VALU-latency bound,
not HBM bound.
cpu_baseline times the C restatement of the reference encoder (oracle/, 1
thread) on a bounded sample of the same frames.
"""
import argparse
import json
import os

# Two pipeline lanes x (kernel + copy stream) plus the runtime's own streams:
# ask HIP for 8 hardware queues (default 4) so no two busy streams share one.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "image-webp_amd"))

ALG_BYTES_PER_MB = 1568
HBM_PEAK_GBS = 8000.0
XFORM_PMC = os.path.join(ROOT, "profiles", "r01_xform_pmc_traffic.json")


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
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--frames", type=int, default=int(os.environ.get("ZW_BENCH_FRAMES", "1024")))
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--quality", type=int, default=75)
    ap.add_argument("--method", type=int, default=4)
    ap.add_argument("--distinct", type=int, default=4, help="distinct synthetic frames per rank")
    ap.add_argument("--cpu-seconds", type=float, default=float(os.environ.get("ZW_BENCH_CPU_SECONDS", "12")))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sequential", action="store_true",
                    help="time K separate encode() calls (no overlap between consecutive batches)")
    return ap.parse_args()


def cpu_baseline(imgs, w, h, q, m, budget_s):
    """Oracle (C port of the reference CPU encoder), 1 thread, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
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
           "sample": f"{n} synthetic {w}x{h} RGBA frames, Q{q} m{m}, oracle/ C restatement, 1 thread, {el:.1f} s"}
    # a batch over the host cores, one frame per thread (ctypes
    # releases the GIL; the oracle keeps no global state).  16 = the box's CPU share.
    nt = min(16, len(os.sched_getaffinity(0)))
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
                                  "sample": f"{sum(counts)} frames, one frame per thread, {nt} threads, {el:.1f} s"}
    return out


def dct_quant_pass(ctx, torch, dev, frames, nmb, reps=5):
    """Streaming DCT+quant pass (k_fdct_quant) over `frames` frames' worth of 4x4
    blocks (24 per MB), device-resident synthetic src/pred; HIP events on the
    launch stream.  Algorithmic bytes per block: 16 src + 16 pred + 32 levels + 16 recon."""
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
    torch.cuda.synchronize(dev)

    def run():
        zwebp.transform_quant_blocks_device(n, src.data_ptr(), pred.data_ptr(), 24, 30, 0, 0, lv.data_ptr(),
                                            rc.data_ptr(), stream=sh, ctx=ctx)

    run()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        run()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    byts = n * 80
    ach = byts / (ms * 1e-3) / 1e9
    del src, pred, lv, rc
    torch.cuda.empty_cache()
    return {"kernel": "k_fdct_quant", "workload": f"{frames} frames x {nmb} MBs x 24 4x4 blocks, Q75 Y1 matrix",
            "blocks": n, "ms_per_launch": ms, "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": ach / HBM_PEAK_GBS, "alg_bytes_per_launch": byts}


def decode_path(ctx, streams, frames, w, h, with_cpu):
    """SURVEY config 3: the decode path on this GPU.  Host bool decoding + MB
    records up, k_dec_recon (dequant, iWHT/iDCT, prediction) + k_loopfilter,
    planes down.  Single frame end to end, plus a batch for the kernels'
    throughput; algorithmic bytes 1208 B/MB (levels 800 + side info 24 + YUV 384)."""
    import zwebp
    one = [streams[0]]
    zwebp.decode_batch(one, ctx=ctx)
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        zwebp.decode_batch(one, ctx=ctx)
    single_ms = (time.perf_counter() - t0) / reps * 1e3
    rk1, lf1 = zwebp.decode_kernel_times(ctx=ctx)
    batch = [streams[i % len(streams)] for i in range(frames)]
    zwebp.decode_batch(batch, ctx=ctx)  # warm-up: grows the pinned staging buffers
    t0 = time.perf_counter()
    zwebp.decode_batch(batch, ctx=ctx)  # pipelined chunks (parse / device / download overlap)
    el = time.perf_counter() - t0
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
    out = {"single_frame_ms": single_ms, "single_frame_kernel_ms": {"k_dec_recon": rk1, "k_loopfilter": lf1},
           "batch_frames": frames, "batch_decodes_per_s": frames / el,
           "batch_kernel_ms": {"k_dec_recon": rk, "k_loopfilter": lf, "launch": "whole batch, one workgroup per frame"},
           "kernel_frames_per_s": frames / ((rk + lf) * 1e-3),
           "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                        "alg_bytes_per_mb": 1208}}
    # decode to packed RGBA (decode_rgba: fancy upsampling on the device, k_yuv2rgb);
    # k_yuv2rgb algorithmic bytes per pixel: Y 1 + U,V 0.5 read, RGBA 4 written
    zwebp.decode_rgb_batch(batch, 4, zwebp.UpsamplingMethod.Bilinear, ctx=ctx)
    t0 = time.perf_counter()
    zwebp.decode_rgb_batch(batch, 4, zwebp.UpsamplingMethod.Bilinear, ctx=ctx)
    el_rgb = time.perf_counter() - t0
    yk = zwebp.decode_rgb_kernel_ms(ctx=ctx)
    yb = 5.5 * w * h * frames
    out["rgba"] = {"batch_decodes_per_s": frames / el_rgb, "k_yuv2rgb_ms": yk,
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
    return out


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch
    import torch.distributed as dist
    import zwebp
    from zwebp.shard import frame_seed, reduce_max
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

    w, h, F = a.width, a.height, a.frames
    ctx = zwebp.Context(local)
    pipe = zwebp.Pipeline(F, w, h, zwebp.ColorType.Rgba8, a.quality, a.method, ctx=ctx)
    # weak scaling: rank r owns global frames [r*F, (r+1)*F); `distinct` of them are generated
    imgs = [synth_rgba(w, h, frame_seed(rank * F + i)) for i in range(min(a.distinct, F))]
    for i in range(F):
        pipe.upload(i, imgs[i % len(imgs)])
    nmb = pipe.mbw * pipe.mbh

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(a.warmup):
        pipe.encode()
    barrier()
    kt = np.zeros(8)
    t0 = time.perf_counter()
    if a.sequential:
        for _ in range(a.steps):
            pipe.encode()
            kt += np.array(pipe.kernel_times())
    else:
        # streaming: step k+1's GPU passes overlap step k's host token emission;
        # all K batches are complete (bitstreams emitted) when this returns
        pipe.encode_repeat(a.steps)
        kt += np.array(pipe.kernel_times()) * a.steps
    barrier()
    el = time.perf_counter() - t0
    el = reduce_max(el, red_dev)
    total_frames = F * a.steps * world
    bytes_out = sum(len(pipe.output(i)) for i in range(min(F, 4)))

    if rank == 0:
        k = kt / max(a.steps, 1)  # ms per launch: rgb2yuv, analysis+segments, pass1, pass2
        p2_ms = float(k[3])
        per_launch = pipe.launch_frames  # frames covered by one k_encode_pass2 launch (one lane chunk)
        achieved = ALG_BYTES_PER_MB * nmb * per_launch / (p2_ms * 1e-3) / 1e9 if p2_ms > 0 else 0.0
        dq = dct_quant_pass(ctx, torch, dev, 256, nmb)
        dec = decode_path(ctx, [bytes(pipe.output(i)) for i in range(min(F, 4))], 256, w, h,
                          not a.no_cpu_baseline)
        cpu = None
        if not a.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(imgs, w, h, a.quality, a.method, a.cpu_seconds)
        line = {
            "metric": f"{w}x{h} lossy encodes/s (Q{a.quality}, method {a.method})",
            "value": total_frames / el,
            "unit": "encodes/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": el / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {"workload": f"encode_frame_lossy {w}x{h} RGBA Q{a.quality} m{a.method}",
                       "frames_per_step_per_gpu": F, "distinct_frames": len(imgs), "mbs_per_frame": nmb,
                       "parallelism": f"frames sharded over {world} GPU(s)",
                       "steps_pipelined": not a.sequential},
            "roofline": {"bound": "hbm", "achieved": dq["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": dq["frac"], "traffic": xform_traffic(dq["blocks"]),
                         "kernel": "k_fdct_quant", "workload": dq["workload"], "blocks_per_launch": dq["blocks"],
                         "alg_bytes_per_launch": dq["alg_bytes_per_launch"], "ms_per_launch": dq["ms_per_launch"],
                         "traffic_source": "profiles/r01_xform_pmc_traffic.json (rocprofv3 --pmc)"},
            "cpu_baseline": cpu,
            "decode_path": dec,
            "encode_kernel": {"kernel": "k_encode_pass2", "bound": "valu", "hbm_achieved": achieved,
                              "hbm_frac": achieved / HBM_PEAK_GBS, "unit": "GB/s",
                              "alg_bytes_per_launch": ALG_BYTES_PER_MB * nmb * per_launch,
                              "launch_frames": per_launch, "ms_per_launch": p2_ms},
            "kernel_ms_per_step": {"rgb2yuv": float(k[0]), "analysis_segments": float(k[1]),
                                   "encode_pass1": float(k[2]), "encode_pass2": p2_ms},
            "host_ms_per_step": {"fetch_pass1": float(k[4]), "stats_probs": float(k[5]),
                                 "fetch_pass2": float(k[6]), "emit": float(k[7])},
            "avg_frame_bytes": bytes_out / min(F, 4),
        }
        print(json.dumps(line), flush=True)
    lanes = pipe.lanes
    pipe.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
