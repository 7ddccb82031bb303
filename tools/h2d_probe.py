#!/usr/bin/env python3
"""H2D / D2H copy rates on this box (torch copies, 256 MB): pageable and pinned host memory."""
import time
import torch

dev = torch.device("cuda", 0)
n = 256 << 20
d = torch.empty(n, dtype=torch.uint8, device=dev)
for kind in ("pageable", "pinned"):
    h = torch.empty(n, dtype=torch.uint8, pin_memory=(kind == "pinned"))
    h.fill_(1)
    for direction in ("h2d", "d2h"):
        best = 1e9
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if direction == "h2d":
                d.copy_(h, non_blocking=(kind == "pinned"))
            else:
                h.copy_(d, non_blocking=(kind == "pinned"))
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        print(f"{kind} {direction}: {n / best / 1e9:.1f} GB/s", flush=True)
