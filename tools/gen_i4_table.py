#!/usr/bin/env python3
"""Derive the (mode, pixel) -> value-vector index table used by the device I4
predictor.  Each of the ten 4x4 intra predictors (prediction.rs:568-855) is a
per-pixel choice among edge pixels, avg3 of three consecutive edge pixels and
avg2 of two consecutive edge pixels (DC and TM are computed directly).

Edge vector E = [L3, L2, L1, L0, P, A0 .. A7] (13 entries).
Value vector V:  V[0..12]  = E
                 V[13..23] = avg3(E[k], E[k+1], E[k+2]), k = 0..10
                 V[24..35] = avg2(E[k], E[k+1]),         k = 0..11
                 V[36]     = avg3(A6, A7, A7)
                 V[37]     = avg3(L2, L3, L3)
Prints a C initializer for I4_IDX[10][16] (255 = DC, 254 = TM).
"""
E = ["L3", "L2", "L1", "L0", "P", "A0", "A1", "A2", "A3", "A4", "A5", "A6", "A7"]
pos = {e: i for i, e in enumerate(E)}


def avg3(a, b, c):
    if b == "A7" and a == "A6" and c == "A7":
        return 36
    if b == "L3" and ((a == "L2" and c == "L3") or (a == "L3" and c == "L2")):
        return 37
    i, j, k = pos[a], pos[b], pos[c]
    if j == i + 1 and k == j + 1:
        return 13 + i
    if j == i - 1 and k == j - 1:
        return 13 + k
    raise ValueError((a, b, c))


def avg2(a, b):
    i, j = pos[a], pos[b]
    lo = min(i, j)
    assert abs(i - j) == 1
    return 24 + lo


def preds():
    l0, l1, l2, l3, p = "L0", "L1", "L2", "L3", "P"
    a = ["A%d" % i for i in range(8)]
    e = [l3, l2, l1, l0, p, a[0], a[1], a[2], a[3]]
    d = [[None] * 16 for _ in range(10)]
    d[0] = [255] * 16
    d[1] = [254] * 16
    ve = [avg3(p, a[0], a[1]), avg3(a[0], a[1], a[2]), avg3(a[1], a[2], a[3]), avg3(a[2], a[3], a[4])]
    d[2] = [ve[x] for y in range(4) for x in range(4)]
    he = [avg3(p, l0, l1), avg3(l0, l1, l2), avg3(l1, l2, l3), 37]
    d[3] = [he[y] for y in range(4) for x in range(4)]
    ld = [avg3(a[0], a[1], a[2]), avg3(a[1], a[2], a[3]), avg3(a[2], a[3], a[4]), avg3(a[3], a[4], a[5]),
          avg3(a[4], a[5], a[6]), avg3(a[5], a[6], a[7]), 36]
    d[4] = [ld[y + x] for y in range(4) for x in range(4)]
    rd = [avg3(e[0], e[1], e[2]), avg3(e[1], e[2], e[3]), avg3(e[2], e[3], e[4]), avg3(e[3], e[4], e[5]),
          avg3(e[4], e[5], e[6]), avg3(e[5], e[6], e[7]), avg3(e[6], e[7], e[8])]
    d[5] = [rd[3 - y + x] for y in range(4) for x in range(4)]
    q = [None] * 16
    e0, e1, e2, e3, e4, e5, e6, e7, e8 = e
    q[12] = avg3(e1, e2, e3); q[8] = avg3(e2, e3, e4)
    q[13] = q[4] = avg3(e3, e4, e5); q[9] = q[0] = avg2(e4, e5)
    q[14] = q[5] = avg3(e4, e5, e6); q[10] = q[1] = avg2(e5, e6)
    q[15] = q[6] = avg3(e5, e6, e7); q[11] = q[2] = avg2(e6, e7)
    q[7] = avg3(e6, e7, e8); q[3] = avg2(e7, e8)
    d[6] = q
    q = [None] * 16
    a0, a1, a2, a3, a4, a5, a6, a7 = a
    q[0] = avg2(a0, a1); q[4] = avg3(a0, a1, a2)
    q[8] = q[1] = avg2(a1, a2); q[5] = q[12] = avg3(a1, a2, a3)
    q[9] = q[2] = avg2(a2, a3); q[13] = q[6] = avg3(a2, a3, a4)
    q[10] = q[3] = avg2(a3, a4); q[14] = q[7] = avg3(a3, a4, a5)
    q[11] = avg3(a4, a5, a6); q[15] = avg3(a5, a6, a7)
    d[7] = q
    q = [None] * 16
    q[12] = avg2(e0, e1); q[13] = avg3(e0, e1, e2)
    q[8] = q[14] = avg2(e1, e2); q[9] = q[15] = avg3(e1, e2, e3)
    q[10] = q[4] = avg2(e2, e3); q[11] = q[5] = avg3(e2, e3, e4)
    q[6] = q[0] = avg2(e3, e4); q[7] = q[1] = avg3(e3, e4, e5)
    q[2] = avg3(e4, e5, e6); q[3] = avg3(e5, e6, e7)
    d[8] = q
    q = [None] * 16
    q[0] = avg2(l0, l1); q[1] = avg3(l0, l1, l2)
    q[2] = q[4] = avg2(l1, l2); q[3] = q[5] = avg3(l1, l2, l3)
    q[6] = q[8] = avg2(l2, l3); q[7] = q[9] = 37
    for k in (10, 11, 12, 13, 14, 15):
        q[k] = pos[l3]
    d[9] = q
    return d


if __name__ == "__main__":
    d = preds()
    for m in range(10):
        assert all(v is not None for v in d[m]), m
    print("static const uint8_t I4_IDX[10][16] = {")
    for m in range(10):
        print("    {" + ", ".join(str(v) for v in d[m]) + "},")
    print("};")
