"""Per-kernel sums of the counters collected by tools/gpu_pmc_sq.sh (all groups of a tag)."""
import collections
import csv
import glob
import sys

tag = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(f"gpurun_out/pmcsq_{tag}_*/run_counter_collection.csv")):
    seen = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void nori::", "")[:28]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        key = (k, r["Dispatch_Id"])
        if key not in seen:
            agg[k]["_ms_" + f] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            agg[k]["_n_" + f] += 1
        seen[key] += 1
for k, d in agg.items():
    if d.get("SQ_WAVES", 1e9) < 1000:
        continue
    ms = [v for c, v in d.items() if c.startswith("_ms_")]
    print(f"{k}: ms/pass={sum(ms) / len(ms):.2f}")
    w = d.get("SQ_WAVES")
    for c, v in sorted(d.items()):
        if c.startswith("_"):
            continue
        extra = f"  per-wave {v / w:.1f}" if w and c != "SQ_WAVES" else ""
        print(f"   {c:28s} {v:16.0f}{extra}")
