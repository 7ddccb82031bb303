#!/usr/bin/env python3
"""Summarise tools/gpu_ab2.sh bench logs: python tools/ab_summary.py gpurun_out/ab_*.log"""
import json
import sys

for f in sys.argv[1:]:
    line = next((l for l in open(f) if l.startswith("{")), None)
    if line is None:
        print(f, "no bench line")
        continue
    d = json.loads(line)
    k = d.get("kernel_ms_per_step", {})
    print(f, round(d["value"], 1), d.get("verified"), {a: round(b, 2) for a, b in k.items()})
