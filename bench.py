"""Headline benchmark: Msamples/s on cbox_path_mis 512x512 @ 512 spp.

A step = one full render of the workload (512x512 pixels x 512 sample passes
= 134,217,728 camera samples of path_mis, scenes/pa4/cbox/cbox_path_mis.xml
with its mirror and dielectric spheres) from resident scene data to the
filtered RGBW film in HBM.

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): one process
per GPU; rank r renders the disjoint sample passes [r*spp, (r+1)*spp) of the
same frame (weak scaling: per-GPU work is fixed) and the RGBW films are summed
over RCCL (all_reduce) -- the reference's ImageBlock::put(block) merge
(block.cpp:124-133).  value = samples of all ranks / max-over-ranks time.

Extra fields:
  roofline     -- extension-ray traversal kernel (k_extend), algorithmic bytes
                  per launch (48 B per ray + BVH bytes) over its average
                  HIP-event launch time, against 8 TB/s HBM peak.
  cpu_baseline -- the CPU oracle (reference structure: sample-outer passes,
                  32x32 blocks, per-block pcg32 streams) timed on this host on
                  a bounded sample of the same workload (rank 0, N=1 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "nori-ray-tracer_amd"))

import nori_amd  # noqa: E402

METRIC = "Msamples/sec on cbox_path_mis 512×512@512spp; per-pixel L2 vs CPU ref"
SCENE = os.path.join(ROOT, "scenes", "pa4", "cbox", "cbox_path_mis.xml")
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(width, height, target_s):
    """Oracle in reference (BLOCK stream) mode on a bounded number of passes."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    threads = min(16, os.cpu_count() or 1)
    scene = nori_amd.load_scene(SCENE, width, height, 1)
    o = pyoracle.OracleScene(scene)
    o.render(passes=1, rng="block", threads=threads, variance_pass=True)
    t1 = o.last_stats["ms_render"] / 1e3
    passes = int(max(1, min(512, target_s / max(t1, 1e-3))))
    o.render(passes=passes, rng="block", threads=threads, variance_pass=True)
    st = o.last_stats
    return {
        "value": st["samples"] / (st["ms_render"] / 1e3) / 1e6,
        "unit": "Msamples/s",
        "cores": st["threads"],
        "kind": "port",
        "sample": f"{width}x{height} x {passes} passes of the same scene ({st['samples']} samples, "
                  f"{st['ms_render'] / 1e3:.1f} s), reference stream layout, serial variance pass included; "
                  f"CPU: {cpu_model()}",
    }


def parity_check():
    """Small-size per-pixel L2 of the GPU image against the oracle (same streams)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    s = nori_amd.load_scene(SCENE, 128, 128, 16)
    with nori_amd.GpuRenderer(s, 0) as r:
        gpu = nori_amd.develop(s, r.render())
    cpu = nori_amd.develop(s, pyoracle.OracleScene(s).render(rng="wave"))
    return {"l2": float(np.mean((gpu - cpu) ** 2)), "config": "128x128@16spp, identical WAVE streams"}


def load_traffic(stats):
    """HBM bytes per k_extend launch from the committed rocprofv3 PMC pass, if any."""
    p = os.path.join(ROOT, "profiles", "pmc_extend.json")
    try:
        d = json.load(open(p))
        return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--height", type=int, default=512)
    ap.add_argument("--spp", type=int, default=512)
    ap.add_argument("--pool", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    torch = None
    if world > 1:
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))

    scene = nori_amd.load_scene(SCENE, args.width, args.height, args.spp)
    r = nori_amd.GpuRenderer(scene, local)
    film_shape = scene.film_shape()
    film_t = None
    if world > 1:
        film_t = torch.zeros(film_shape, dtype=torch.float32, device=f"cuda:{local}")

    def step(timing=False):
        if world > 1:
            from nori_amd import distributed as nd

            film_t.zero_()
            torch.cuda.synchronize()
            pb, pc = nd.pass_range(rank, args.spp)
            r.render(passes=pc, pass_begin=pb, device_ptr=film_t.data_ptr(), path_pool=args.pool, timing=timing)
            nd.reduce_film(film_t, dist)
        else:
            r.render(passes=args.spp, path_pool=args.pool, timing=timing)
        return r.last_stats

    def sync():
        if world > 1:
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        st = step()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # one extra, untimed step with per-kernel HIP events for the roofline
    ts = step(timing=True)
    samples_per_step = args.width * args.height * args.spp
    value = world * samples_per_step * args.steps / elapsed / 1e6

    if rank == 0:
        launches = max(ts["iterations"], 1)
        bytes_total = ts["rays_closest"] * 48 + launches * ts["scene_bytes"]
        achieved = bytes_total / (ts["ms_extend"] / 1e3) / 1e9 if ts["ms_extend"] > 0 else 0.0
        traffic = load_traffic(ts)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: the reference's cbox_path_mis scene file, no external assets",
            "config": {"workload": f"cbox_path_mis {args.width}x{args.height}@{args.spp}spp",
                       "scene": "scenes/pa4/cbox/cbox_path_mis.xml", "integrator": "path_mis",
                       "parallelism": f"pass-range sharding x{world}, RCCL film all_reduce" if world > 1
                       else "single GPU", "path_pool": args.pool or 4194304},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "k_extend (closest-hit traversal)",
                         "bytes_per_launch": bytes_total / launches,
                         "avg_launch_ms": ts["ms_extend"] / launches, "launches": launches},
            "kernel_ms": {"extend": ts["ms_extend"], "shadow": ts["ms_shadow"], "shade": ts["ms_shade"],
                          "splat": ts["ms_splat"], "finish": ts["ms_finish"], "wall": ts["ms_total"]},
            "rays_per_sample": {"closest": ts["rays_closest"] / samples_per_step,
                                "shadow": ts["rays_shadow"] / samples_per_step,
                                "finisher": ts["rays_finish"] / samples_per_step},
            "wavefront_iterations": ts["iterations"],
        }
        if world == 1 and not args.no_parity:
            out["parity"] = parity_check()
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.width, args.height, args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    r.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
