"""Per-render kernel timeline of a rocprofv3 --kernel-trace CSV (diagnostic).

usage: python tools/timeline.py <dir with *_kernel_trace.csv> [render index]
Renders are split at k_mark launches (one per render's tail); prints for
the chosen render: wall span, busy time per kernel, idle gaps between
consecutive kernels on the same queue, and the tail (k_mark -> last kernel).
"""
import collections
import csv
import glob
import os
import sys


def load(d):
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("nori::", "").strip()
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", r.get("Stream_Id", "0"))))
    rows.sort()
    return rows


def main():
    rows = load(sys.argv[1])
    marks = [i for i, r in enumerate(rows) if r[2].startswith("k_mark")]
    sel = int(sys.argv[2]) if len(sys.argv) > 2 else len(marks) - 1
    # a render: from the first kernel after the previous render's last splat/finish to this render's last kernel
    end_i = marks[sel]
    while end_i + 1 < len(rows) and not rows[end_i + 1][2].startswith("k_shade"):
        end_i += 1
    start_i = marks[sel - 1] if sel > 0 else 0
    while start_i < len(rows) and not rows[start_i][2].startswith("k_shade"):
        start_i += 1
    if sel > 0:
        while start_i < end_i and not rows[start_i][2].startswith("k_shade"):
            start_i += 1
    seg = rows[start_i:end_i + 1]
    t0, t1 = seg[0][0], max(r[1] for r in seg)
    busy = collections.defaultdict(float)
    count = collections.Counter()
    for s, e, n, q in seg:
        busy[n.split("<")[0]] += (e - s) / 1e6
        count[n.split("<")[0]] += 1
    print(f"render {sel}: {len(seg)} kernels, wall {(t1 - t0) / 1e6:.3f} ms")
    for n in sorted(busy, key=lambda k: -busy[k]):
        print(f"  {n:16s} {count[n]:5d} launches  {busy[n]:8.3f} ms")
    # union of busy intervals (any queue) -> idle time
    iv = sorted((s, e) for s, e, _, _ in seg)
    cover, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            cover += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    cover += ce - cs
    print(f"  device busy (union) {cover / 1e6:.3f} ms, idle {(t1 - t0 - cover) / 1e6:.3f} ms")
    m = [r for r in seg if r[2].startswith("k_mark")][0]
    print(f"  tail: k_mark at +{(m[0] - t0) / 1e6:.3f} ms, render ends +{(t1 - t0) / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
