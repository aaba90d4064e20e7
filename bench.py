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
  roofline     -- the dominant kernel (most HIP-event time in the last timed
                  step; k_shade on this workload): algorithmic HBM bytes per
                  launch over its average launch time against the 8 TB/s HBM
                  peak (launch times inside the timed region, where two pool
                  parts on two streams share the chip; `isolated_frac` uses the
                  serialised launch time of the committed counter passes), `traffic` = measured HBM bytes per launch from the
                  committed rocprofv3 PMC summary (profiles/pmc_r01.json), and
                  a per-kernel table (the traversal kernels are VALU-bound:
                  VALU issue rate against the issue peak).
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


PROFILE = os.path.join(ROOT, "profiles", "pmc_r01.json")  # committed rocprofv3 evidence (tools/pmc_to_profile.py)
VALU_PEAK = 256 * 4 * 2.4e9 / 2 * 64  # lane-instr/s: 256 CUs x 4 SIMDs, a wave64 VALU op per 2 cycles


def profiled(prefix):
    """Per-launch rocprofv3 numbers of the kernel whose name starts with `prefix`, if committed."""
    try:
        d = json.load(open(PROFILE))
    except (OSError, ValueError):
        return None
    for k, v in d.get("kernels", {}).items():
        if k.startswith(prefix):
            return dict(v, name=k)
    return None


def roofline(ts, samples):
    """Roofline of the dominant kernel (most HIP-event time) of the timing render.

    Algorithmic HBM bytes per kernel:
      k_shade : per path read ray_o, ray_d, thr, rng, hit (16 B each) + work (4 B) = 84 B,
                per surviving path write ray_o, ray_d, thr, rng + work = 68 B,
                per shadow ray 48 B (origin, direction, payload), per new sample 16 B
                record + 4 B pixel index
      k_extend: per ray read ray_o, ray_d (32 B), write hit (16 B)
      k_shadow: per shadow ray read ray_o, ray_d, payload (48 B)
    The traversal kernels are VALU-bound (scan over the primitive list); their
    VALU issue rate (SQ_INSTS_VALU x 64 lanes per launch, rocprofv3) is given
    against the issue peak.
    """
    launches = max(ts["iterations"] * max(ts.get("stream_parts", 1), 1), 1)  # per kernel
    rc, rs = ts["rays_closest"], ts["rays_shadow"]
    kern = {
        "shade": ("k_shade", ts["ms_shade"], rc * (84 + 68) + rs * 48 + samples * 20),
        "extend": ("k_extend", ts["ms_extend"], rc * 48),
        "shadow": ("k_shadow", ts["ms_shadow"], rs * 48),
    }
    rows = {}
    for key, (name, ms, nbytes) in kern.items():
        if ms <= 0:
            continue
        prof = profiled(name)
        avg = ms / launches
        row = {"ms": ms, "avg_launch_ms": avg, "bytes_per_launch": nbytes / launches,
               "achieved_GBs": nbytes / launches / (avg / 1e3) / 1e9}
        if prof:
            row["traffic_bytes_per_launch"] = prof.get("hbm_bytes_per_launch")
            row["rocprof_avg_launch_ms"] = prof.get("trace_avg_ms")
            # the counter passes serialise the kernels: this launch time has no
            # second stream beside it (the timed region overlaps two pool parts)
            iso = prof.get("profiled_ms_per_launch")
            if iso:
                row["isolated_launch_ms"] = iso
                row["isolated_achieved_GBs"] = nbytes / launches / (iso / 1e3) / 1e9
            if prof.get("sq_insts_valu_per_launch") and prof.get("trace_avg_ms"):
                rate = prof["sq_insts_valu_per_launch"] * 64 / (prof["trace_avg_ms"] / 1e3)
                row["valu_lane_instr_per_s"] = rate
                row["valu_issue_frac"] = rate / VALU_PEAK
        rows[name] = row
    dom = max(rows, key=lambda k: rows[k]["ms"])
    d = rows[dom]
    return {"bound": "hbm", "kernel": dom, "achieved": d["achieved_GBs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": d["achieved_GBs"] / HBM_PEAK_GBS, "traffic": d.get("traffic_bytes_per_launch"),
            "isolated_frac": (d["isolated_achieved_GBs"] / HBM_PEAK_GBS) if "isolated_achieved_GBs" in d else None,
            "bytes_per_launch": d["bytes_per_launch"], "avg_launch_ms": d["avg_launch_ms"], "launches": launches,
            "kernels": rows}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # default warm-up: 2 renders -- the first render after a context's first
    # render runs ~17 ms (~40 %) longer with identical kernel times
    # (tools/step_times.py); from the third on the step time is steady
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
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
    for i in range(args.steps):
        # the last timed step also records HIP events around every kernel (on
        # the renderer's stream) for the per-kernel times of the roofline;
        # their small overhead stays inside the timed region
        ts = step(timing=(i == args.steps - 1))
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    samples_per_step = args.width * args.height * args.spp
    value = world * samples_per_step * args.steps / elapsed / 1e6

    if rank == 0:
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
            "roofline": roofline(ts, samples_per_step),
            "kernel_ms": {"extend": ts["ms_extend"], "shadow": ts["ms_shadow"], "shade": ts["ms_shade"],
                          "splat": ts["ms_splat"], "finish": ts["ms_finish"], "wall": ts["ms_total"]},
            "rays_per_sample": {"closest": ts["rays_closest"] / samples_per_step,
                                "shadow": ts["rays_shadow"] / samples_per_step,
                                "finisher": ts["rays_finish"] / samples_per_step},
            "wavefront_iterations": ts["iterations"],
            "stream_parts": ts.get("stream_parts", 1),
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
