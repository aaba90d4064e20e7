"""Summarise rocprofv3 runs into profiles/ (committed evidence for bench.py).

usage: python tools/pmc_to_profile.py <tag>
  reads gpurun_out/pmc_<tag>_FETCH_SIZE/, gpurun_out/pmc_<tag>_WRITE_SIZE/ (tools/gpu_pmc.sh)
  and gpurun_out/prof_<tag>/ (tools/gpu_prof.sh, kernel trace + stats) if present;
  writes profiles/pmc_<tag>.json and copies the kernel-stats CSV to profiles/.

HBM bytes per launch follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes of a wide
(16 B/lane) coalesced read, so it is doubled; WRITE_SIZE is exact for 16 B/lane
stores.  Each counter comes from its own rocprofv3 pass.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("nori::", "")
    return n.strip()


def per_kernel(path, counter):
    acc = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        a = acc[short(r["Kernel_Name"])]
        a[0] += 1
        a[1] += float(r["Counter_Value"])
        a[2] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    return acc


def main():
    tag = sys.argv[1]
    import subprocess
    commit = os.environ.get("NORI_PROFILE_COMMIT")  # set when summarising on the GPU box (no .git there)
    if not commit:
        try:
            commit = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                                    text=True).stdout.strip() or None
        except OSError:
            commit = None
    out = {"tag": tag, "commit": commit, "method": "rocprofv3 --pmc FETCH_SIZE (pass 1) / WRITE_SIZE (pass 2) --kernel-trace; "
                                  "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH correction)",
           "kernels": {}}
    f = os.path.join(ROOT, "gpurun_out", f"pmc_{tag}_FETCH_SIZE", "run_counter_collection.csv")
    w = os.path.join(ROOT, "gpurun_out", f"pmc_{tag}_WRITE_SIZE", "run_counter_collection.csv")
    if os.path.exists(f) and os.path.exists(w):
        fk, wk = per_kernel(f, "FETCH_SIZE"), per_kernel(w, "WRITE_SIZE")
        for k in fk:
            if k not in wk or k.startswith("__amd"):
                continue
            n = fk[k][0]
            fetch_b = 2 * fk[k][1] * 1024 / n
            write_b = wk[k][1] * 1024 / wk[k][0]
            out["kernels"][k] = {"launches": n, "fetch_bytes_per_launch": fetch_b,
                                 "write_bytes_per_launch": write_b,
                                 "hbm_bytes_per_launch": fetch_b + write_b,
                                 "profiled_ms_per_launch": fk[k][2] / n}
    # SQ instruction counters (tools/gpu_pmc_sq.sh groups), when collected
    import glob
    for d in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", f"pmcsq_{tag}_[0-9]*"))):
        path = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for ctr in ("SQ_INSTS_VALU", "SQ_WAVES", "SQ_INSTS_SALU", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES", "SQ_INSTS_SMEM",
                    "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_SCA",
                    "SQ_INSTS_BRANCH", "SQ_BUSY_CYCLES", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
            for k, (n, v, ms) in per_kernel(path, ctr).items():
                if k.startswith("__amd") or n == 0:
                    continue
                e = out["kernels"].setdefault(k, {})
                e[ctr.lower() + "_per_launch"] = v / n
    prof = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    stats = os.path.join(prof, "run_kernel_stats.csv")
    if os.path.exists(stats):
        dst = os.path.join(ROOT, "profiles", f"rocprof_{tag}_kernel_stats.csv")
        shutil.copy(stats, dst)
        for r in csv.DictReader(open(stats)):
            k = short(r["Name"])
            if k.startswith("__amd"):
                continue
            e = out["kernels"].setdefault(k, {})
            e["trace_calls"] = int(r["Calls"])
            e["trace_avg_ms"] = float(r["AverageNs"]) / 1e6
            e["trace_total_ms"] = float(r["TotalDurationNs"]) / 1e6
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    dst = os.path.join(ROOT, "profiles", f"pmc_{tag}.json")
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
