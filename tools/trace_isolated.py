"""Per-kernel durations from a rocprofv3 kernel-trace CSV, split into launches
that ran alone on the GPU and launches that overlapped another pass kernel
(the pipeline's two lanes run their pass launches concurrently, so only the
isolated ones compare with bench.py's per-launch kernel times).

    python tools/trace_isolated.py gpurun_out/bprof/bench_kernel_trace.csv
"""
import collections
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    spans = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    passes = [(s, e) for s, e, n in spans if n.startswith("k_encode_pass")]
    groups = collections.defaultdict(lambda: ([], []))
    for s, e, n in spans:
        name = n.split("(")[0]
        if not (name.startswith("k_encode_pass") or name.startswith("void k_xform_mb")
                or name in ("k_dec_recon", "k_loopfilter", "k_pack_scan", "k_pack_write")):
            continue
        alone = sum(1 for a, b in passes if a < e and b > s) - (1 if name.startswith("k_encode_pass") else 0) == 0
        groups[name][0 if alone else 1].append((e - s) / 1e6)
    print("%-28s %8s %-40s %8s %10s" % ("kernel", "isolated", "isolated duration clusters (ms: count)", "overlap", "mean ms"))
    for name, (iso, ov) in sorted(groups.items()):
        clusters = collections.Counter()
        for d in iso:
            key = next((k for k in clusters if abs(k - d) <= 0.03 * k), d)
            clusters[key] += 1
        med = {}
        for k in clusters:
            vals = sorted(d for d in iso if abs(k - d) <= 0.03 * k)
            med[k] = vals[len(vals) // 2]
        desc = ", ".join("%.2f: %d" % (med[k], c) for k, c in sorted(clusters.items()))
        allv = iso + ov
        print("%-28s %8d %-40s %8d %10.3f" % (name[:28], len(iso), desc[:40], len(ov), sum(allv) / len(allv)))
        if len(desc) > 40:
            print("%38s%s" % ("", desc))


if __name__ == "__main__":
    main(sys.argv[1])
