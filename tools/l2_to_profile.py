"""Summarise tools/gpu_l2.sh into profiles/l2_<tag>.json (L2 hit rate per kernel).

usage: python tools/l2_to_profile.py <tag> [bench args recorded in the method]
"""
import collections
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    f = os.path.join(ROOT, "gpurun_out", f"l2_{tag}", "run_counter_collection.csv")
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("nori::", "").strip()
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    commit = os.environ.get("NORI_PROFILE_COMMIT") or subprocess.run(
        ["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip() or None
    out = {"tag": tag, "commit": commit,
           "method": "rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace of `bench.py --roofline-only "
                     + " ".join(sys.argv[2:]) + "` (one pass), summed over launches",
           "kernels": {}}
    for k, d in acc.items():
        req = d.get("TCC_HIT_sum", 0.0) + d.get("TCC_MISS_sum", 0.0)
        if req <= 0:
            continue
        out["kernels"][k] = {"l2_hit_rate": round(d.get("TCC_HIT_sum", 0.0) / req, 4), "tcc_requests": int(req)}
    p = os.path.join(ROOT, "profiles", f"l2_{tag}.json")
    json.dump(out, open(p, "w"), indent=1)
    print(p)
    for k, v in out["kernels"].items():
        print(f"  {k:40s} hit {v['l2_hit_rate']:.3f}  requests {v['tcc_requests']}")


if __name__ == "__main__":
    main()
