#!/usr/bin/env python3
"""Compare the frame-0 record dumps of the device and host token parses
(ZW_DEC_TOKENS_DUMP=<p>: <p>.dev, <p>.host): the first MB whose record differs.
usage: python tools/cmp_recs.py <p> nmb"""
import sys

import numpy as np

p, nmb = sys.argv[1], int(sys.argv[2])


def load(path):
    b = open(path, "rb").read()
    mo = np.frombuffer(b[: 4 * (nmb + 1)], np.uint32)
    return mo, b[4 * (nmb + 1):]


md, rd = load(p + ".dev")
mh, rh = load(p + ".host")
print("bytes dev", md[-1], "host", mh[-1])
for i in range(nmb):
    a = rd[md[i]: md[i + 1]]
    b = rh[mh[i]: mh[i + 1]]
    if a != b or md[i] != mh[i]:
        print("first difference at MB", i, "offsets", md[i], mh[i], "sizes", len(a), len(b))
        ha, hb = np.frombuffer(a[:80], np.uint8), np.frombuffer(b[:80], np.uint8)
        print("dev hdr ", ha.tolist())
        print("host hdr", hb.tolist())
        print("dev lv ", np.frombuffer(a[80:], np.int16).tolist())
        print("host lv", np.frombuffer(b[80:], np.int16).tolist())
        sys.exit(1)
print("identical")
