#!/usr/bin/env python3
"""profiles/r05_xmb_pmc.json (the bench line's `roofline.traffic` source) from
tools/xmb_pmc_summary.py's per-kernel JSON: the RGBA form's HBM bytes per launch
= k_xform_mb<4,0> + the median k_xform_mb_i4q dispatch, the Y/U/V form's per MB
from k_xform_mb<0,0> (the second template argument was a bool before round 5).
usage: xmb_pmc_headline.py SUMMARY.json > profiles/r05_xmb_pmc.json"""
import json
import sys

S = json.load(open(sys.argv[1]))
MBS = 256 * 8160
ALG_RGBA = 1920 * 1080 * 4 / 8160 + 800 + 384  # SURVEY 8(d)'s fused-RGB form, bytes per MB


def pick(*subs):
    ks = [k for k in S if any(k.replace(" ", "").startswith(sub) for sub in subs)]
    assert len(ks) == 1, (subs, list(S))
    return S[ks[0]]


main, i4 = pick("k_xform_mb<4,0>", "k_xform_mb<4,false>"), pick("k_xform_mb_i4")
yuv = pick("k_xform_mb<0,0>", "k_xform_mb<0,false>")
tot = main["hbm_read_bytes"] + main["hbm_write_bytes"] + i4["hbm_read_bytes"] + i4["hbm_write_bytes"]
print(json.dumps({
    "kernel": "k_xform_mb<RGBA> + k_xform_mb_i4q (one launch: 256 1080p frames)",
    "units": MBS, "unit": "MB",
    "traffic_bytes": tot, "traffic_bytes_per_mb": tot / MBS, "alg_bytes_per_mb": ALG_RGBA,
    "breakdown": {
        "k_xform_mb<4,0>": {"hbm_read_bytes": main["hbm_read_bytes"], "hbm_write_bytes": main["hbm_write_bytes"]},
        "k_xform_mb_i4q (median of its dispatches)": {"hbm_read_bytes": i4["hbm_read_bytes"],
                                                     "hbm_write_bytes": i4["hbm_write_bytes"]}},
    "yuv_form": {"kernel": "k_xform_mb<YUV>", "traffic_bytes_per_mb": yuv["traffic_bytes_per_mb"], "alg_bytes_per_mb": 1568},
    "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over tools/xmb_bench.py --reps 3; "
              "FETCH_SIZE doubled (gfx950 counts half the bytes of wide streaming reads, MI355X_MICROARCH.md HBM "
              "section), WRITE_SIZE as is; KiB -> bytes; median per dispatch",
    "source": "tools/gpu_pmc_xmb.sh -> tools/xmb_pmc_summary.py -> tools/xmb_pmc_headline.py; full counters in "
              "profiles/r05_xmb_pmc_summary.json",
}, indent=1))
