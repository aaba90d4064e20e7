"""Headline benchmark: Msamples/s on cbox_path_mis 512x512 @ 512 spp.

A step = one full render of the workload (default: 512x512 pixels x 512
sample passes = 134,217,728 camera samples of path_mis on
scenes/pa4/cbox/cbox_path_mis.xml, with its mirror and dielectric spheres),
from resident scene data to the filtered RGBW film in HBM.  --config c3|c4|c5
benches the other single-GPU-sized BASELINE configs (nori_amd.configs).

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N, or plain
`python bench.py --gpus N`, which starts that launcher itself before any GPU
call): one process per GPU.  STRONG scaling: the frame is fixed and split over the ranks
by libnori_gpu itself (nori_gpu_render_sharded: rank r renders sample passes
[P r/N, P (r+1)/N), or --shard blocks: every N-th 32x32 block of the spiral
order), and the library sums the RGBW films into rank 0 with RCCL over xGMI --
the reference's ImageBlock::put(block) merge (block.cpp:124-133).  The step
time includes that sum.  value = the frame's samples / max-over-ranks time.
torch.distributed (gloo) only carries the communicator id, the barriers and
the max of the rank times.

Extra fields:
  roofline     -- the traversal kernel k_extend (north_star's target) against
                  the 8 TB/s HBM peak: algorithmic bytes per launch (48 B per
                  extension ray + the scene's primitive/node bytes, SURVEY.md
                  8(d)) over its average launch time, from HIP events in an
                  extra render after the timed region with ONE pool part (the
                  timed renders run two parts on two streams, so a kernel's
                  event time there includes the other part's kernels);
                  `traffic` = measured HBM bytes per launch of the committed
                  rocprofv3 counter passes of `bench.py --roofline-only`
                  (profiles/).  `kernels` holds k_shade / k_shadow alike.
  cpu_baseline -- the CPU oracle (reference structure: sample-outer passes,
                  32x32 blocks, per-block pcg32 streams, serial variance
                  sweep) timed on this host's usable cores on a bounded
                  number of passes of the same workload (rank 0, N=1 only).
  parity       -- C2: the film of the last timed step (512x512@512spp) against
                  the oracle's render of the same configuration on identical
                  WAVE streams (~10 s on 16 host threads): per-pixel L2, the
                  L2 without the worst 0.01 % of the pixels, and the fraction
                  of pixels equal to 1e-3 relative.  Other configs: a reduced
                  size (the oracle would take minutes).
"""
import argparse
import json
import math
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "nori-ray-tracer_amd"))

import nori_amd  # noqa: E402
from nori_amd import configs  # noqa: E402
from nori_amd import distributed as nd  # noqa: E402
from nori_amd._abi import BLOCK_SIZE  # noqa: E402

METRIC = "Msamples/sec on cbox_path_mis 512×512@512spp; per-pixel L2 vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
PROFILE_TAG = "r06"  # committed rocprofv3 evidence: profiles/pmc_<tag>[_<config>].json (tools/pmc_to_profile.py)
VALU_PEAK = 256 * 4 * 2.4e9 / 2 * 64  # lane-instr/s: 256 CUs x 4 SIMDs, a wave64 VALU op per 2 cycles


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def usable_cpus():
    """(threads used, affinity-mask CPUs, cgroup CPU quota or None)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    threads = aff if quota is None else max(1, min(aff, int(math.ceil(quota))))
    return threads, aff, quota


def cpu_baseline(xml, width, height, target_s):
    """Oracle in reference (BLOCK stream) mode on a bounded number of passes."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    threads, aff, quota = usable_cpus()
    scene = nori_amd.load_scene(xml, width, height, 1)
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
                  f"{st['threads']} threads = the process's usable CPUs (affinity mask {aff}, cgroup quota "
                  f"{quota if quota is not None else 'none'}); CPU: {cpu_model()}",
    }


def image_parity(gpu, cpu):
    """Per-pixel L2 (mean over pixels of the mean squared RGB difference), the
    same without the worst 0.01 % of the pixels, and the fraction of pixels
    equal to 1e-3 relative (tests/nori_test_util.image_parity's bars)."""
    d = np.mean((np.asarray(gpu, np.float64) - np.asarray(cpu, np.float64)) ** 2, axis=-1).ravel()
    k = max(1, int(d.size * 1e-4))
    trimmed = float(np.sort(d)[:-k].mean()) if d.size > k else 0.0
    match = float(np.mean(np.all(np.isclose(gpu, cpu, rtol=1e-3, atol=1e-5), axis=-1)))
    return {"l2": float(d.mean()), "l2_trimmed": trimmed, "pixel_match": match, "tolerance": 1e-3,
            "bars": {"l2": 1e-5, "l2_trimmed": 1e-9, "pixel_match": 0.99}}


def oracle_wave_image(scene):
    """The oracle's image of `scene` on the GPU's WAVE streams (all usable threads)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    t0 = time.perf_counter()
    img = nori_amd.develop(scene, pyoracle.OracleScene(scene).render(rng="wave", threads=usable_cpus()[0]))
    return img, time.perf_counter() - t0


def parity_check(xml, width, height, spp):
    """Per-pixel L2 of a GPU render against the oracle on identical WAVE streams (reduced size)."""
    s = nori_amd.load_scene(xml, width, height, spp)
    with nori_amd.GpuRenderer(s, 0) as r:
        gpu = nori_amd.develop(s, r.render())
    cpu, secs = oracle_wave_image(s)
    return dict(image_parity(gpu, cpu), config=f"{width}x{height}@{spp}spp of the benched scene, identical WAVE streams",
                oracle_s=secs)


def parity_full(scene, film, W, H, spp):
    """Per-pixel L2 of the film the last TIMED step produced against the oracle
    at the benched size itself, on identical WAVE streams (render.cpp:194-250:
    every (pass, pixel) sample owns its pcg32 stream on both sides)."""
    gpu = nori_amd.develop(scene, film)
    cpu, secs = oracle_wave_image(scene)
    return dict(image_parity(gpu, cpu), config=f"{W}x{H}@{spp}spp (the benched configuration: the last timed "
                f"step's film), identical WAVE streams", oracle_s=secs)


# the kernels a row of the roofline stands for: the scan-mode scenes' trace
# kernels run as the scene-specialised hipRTC kernels (csrc/rtc.hip)
KERNEL_NAMES = {"k_extend": ("nori_rtc_extend_scan", "k_extend"), "k_shadow": ("nori_rtc_shadow_scan", "k_shadow"),
                "k_shade": ("k_shade",)}


def profiled(name, config="c2"):
    """Per-launch rocprofv3 numbers of the kernel `name` stands for (KERNEL_NAMES), if committed for this config."""
    fname = f"pmc_{PROFILE_TAG}.json" if config == "c2" else f"pmc_{PROFILE_TAG}_{config}.json"
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", fname)))
    except (OSError, ValueError):
        return None
    for prefix in KERNEL_NAMES.get(name, (name,)):
        for k, v in d.get("kernels", {}).items():
            if k.startswith(prefix) and "hbm_bytes_per_launch" in v:
                return dict(v, name=k, file=f"profiles/{fname}", commit=d.get("commit"))
    return None


def roofline(ts, samples, config="c2"):
    """Per-kernel roofline rows of an isolated (one pool part) timing render.

    Algorithmic HBM bytes:
      k_extend: per extension ray read ray_o, ray_d (32 B), write hit (16 B);
                plus the scene's node + primitive bytes once per launch
      k_shadow: per shadow ray read ray_o, ray_d, payload (48 B) (+ the scene)
      k_shade : per path read ray_o, ray_d, thr, hit (16 B each) + the pcg32 state high
                word (4 B) + the pixel index its stream increment is recomputed from
                (4 B) = 72 B, per surviving path write ray_o, ray_d, thr + rng = 52 B,
                per shadow ray 48 B, per new sample 16 B record + 4 B pixel index
    """
    launches = max(ts["iterations"] * max(ts.get("stream_parts", 1), 1), 1)
    rc, rs, scene = ts["rays_closest"], ts["rays_shadow"], ts["scene_bytes"]
    kern = {
        "k_extend": (ts["ms_extend"], rc * 48 + scene * launches),
        "k_shadow": (ts["ms_shadow"], rs * 48 + scene * launches),
        "k_shade": (ts["ms_shade"], rc * (72 + 52) + rs * 48 + samples * 20),
    }
    rows = {}
    for name, (ms, nbytes) in kern.items():
        if ms <= 0:
            continue
        avg = ms / launches
        row = {"ms_per_step": ms, "launches": launches, "avg_launch_ms": avg, "bytes_per_launch": nbytes / launches,
               "achieved_GBs": nbytes / launches / (avg / 1e3) / 1e9}
        row["frac"] = row["achieved_GBs"] / HBM_PEAK_GBS
        prof = profiled(name, config)
        if prof:
            row["traffic_bytes_per_launch"] = prof.get("hbm_bytes_per_launch")
            row["rocprof_avg_launch_ms"] = prof.get("trace_avg_ms")
            # the counters come from the committed profile, collected at the commit recorded in it
            # ("commit"): when the kernel sources changed after that commit they describe the older kernel
            row["profile"] = {"file": prof["file"], "commit": prof.get("commit"), "kernel": prof["name"]}
            if prof.get("sq_insts_valu_per_launch") and prof.get("trace_avg_ms"):
                rate = prof["sq_insts_valu_per_launch"] * 64 / (prof["trace_avg_ms"] / 1e3)
                row["valu_issue_frac"] = rate / VALU_PEAK
        rows[name] = row
    d = rows["k_extend"]
    # the render's tail: the film splat (16 B record read per sample) beside the finisher
    tail = {"ms_splat": ts.get("ms_splat", 0.0), "ms_finish": ts.get("ms_finish", 0.0)}
    if tail["ms_splat"] > 0:
        tail["splat_record_GBs"] = samples * 16 / (tail["ms_splat"] / 1e3) / 1e9
    return {"tail": tail, "bound": "hbm", "kernel": "k_extend", "achieved": d["achieved_GBs"], "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": d["frac"], "traffic": d.get("traffic_bytes_per_launch"), "traffic_profile": d.get("profile"),
            "bytes_per_launch": d["bytes_per_launch"], "avg_launch_ms": d["avg_launch_ms"], "launches": launches,
            "measured": "HIP events on the launch stream, one extra render after the timed region with one pool "
                        "part (NORI_POOL_PARTS=1): kernels serialised on one stream",
            "ms_per_step_isolated": ts["ms_total"], "kernels": rows}


def free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(gpus, env, device_count, argv, port=None):
    """How this invocation runs: None = in this process (one GPU, or this is
    already rank RANK of a torch.distributed.run job), else the argv of the
    launcher to run as a child (one process per GPU).  Raises SystemExit on
    an inconsistent request: --gpus != WORLD_SIZE, or more GPUs than the node
    has (device_count, counted without initialising HIP)."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus {gpus} < 1")
    world = env.get("WORLD_SIZE")
    if world is not None:
        if int(world) != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}: pass the launcher's process count")
        if int(env.get("LOCAL_WORLD_SIZE", world)) > device_count:
            raise SystemExit(f"bench.py: {env.get('LOCAL_WORLD_SIZE', world)} ranks on this node but only "
                             f"{device_count} GPU(s) visible")
        return None
    if gpus > device_count:
        raise SystemExit(f"bench.py: --gpus {gpus} but only {device_count} GPU(s) visible")
    if gpus == 1:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port or free_port()}", os.path.abspath(__file__), *argv]


def hip_runtime():
    libs = sorted({l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l})
    return libs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # default warm-up: 2 renders -- the first render after a context's first
    # render runs ~17 ms (~40 %) longer with identical kernel times
    # (tools/step_times.py); from the third on the step time is steady
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=sorted(configs.CONFIGS))
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--pool", type=int, default=0)
    ap.add_argument("--shard", default="passes", choices=["passes", "blocks"])
    ap.add_argument("--cpu-seconds", type=float, default=6.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--roofline-only", action="store_true",
                    help="profiling helper: one warm-up and one measuring render with one pool part "
                         "(the render bench.py's roofline times), then exit")
    args = ap.parse_args()

    # one process per GPU: a plain `bench.py --gpus N` starts the launcher
    # itself (a child process, before this process touches the GPU) and
    # exits with its status; torch.cuda.device_count() does not initialise HIP
    import torch

    plan = launch_plan(args.gpus, os.environ, torch.cuda.device_count(), sys.argv[1:])
    if plan is not None:
        import subprocess

        sys.exit(subprocess.run(plan).returncode)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    tmp = tempfile.mkdtemp(prefix="nori_bench_")
    xml, label, W, H, spp = configs.config_scene(args.config, tmp, args.width, args.height, args.spp)
    scene = nori_amd.load_scene(xml, W, H, spp)
    r = nori_amd.GpuRenderer(scene, local)

    if args.roofline_only:
        os.environ["NORI_POOL_PARTS"] = "1"
        r.render(path_pool=args.pool)
        r.render(path_pool=args.pool, timing=True)
        print(json.dumps({"roofline_only": True, "workload": label, "stats": r.last_stats}), flush=True)
        r.close()
        return

    dist = None
    comm = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group(backend="gloo")
        comm = nd.film_comm(dist, local)
    film = torch.zeros(scene.film_shape(), dtype=torch.float32, device=f"cuda:{local}")
    torch.cuda.synchronize()
    share = nd.shard(scene, rank, world, args.shard) if world > 1 else (0, spp, None)
    nbx = -(-W // BLOCK_SIZE)
    share_samples = share[1] * (W * H if share[2] is None else sum(
        min(BLOCK_SIZE, W - (b % nbx) * BLOCK_SIZE) *
        min(BLOCK_SIZE, H - (b // nbx) * BLOCK_SIZE) for b in share[2]))

    def step(timing=False):
        if world > 1:
            r.render_sharded(comm, film.data_ptr(), mode=args.shard, root=0, path_pool=args.pool, timing=timing)
        else:
            film.zero_()
            torch.cuda.synchronize()
            r.render(passes=spp, path_pool=args.pool, device_ptr=film.data_ptr(), timing=timing)
        st = r.last_stats
        assert st["samples"] == share_samples, (st["samples"], share_samples)
        return st

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    sync()
    t0 = time.perf_counter()
    invalid = 0
    for _ in range(args.steps):
        invalid += step()["invalid_samples"]
    sync()
    elapsed = time.perf_counter() - t0
    last = r.last_stats
    film_host = film.cpu().numpy() if rank == 0 and world == 1 else None  # the last timed step's image
    rank_ms = [elapsed / args.steps * 1e3]
    comm_ranks = None
    if world > 1:
        t = torch.zeros(world, dtype=torch.float64)
        t[rank] = elapsed
        dist.all_reduce(t)  # every rank's time (gloo)
        rank_ms = [float(x) / args.steps * 1e3 for x in t]
        elapsed = float(t.max())
        nr = torch.zeros(world, dtype=torch.int64)
        nr[rank] = comm.ranks()[0]
        dist.all_reduce(nr)
        comm_ranks = nr.tolist()  # the communicator size each rank's library reports

    samples_per_step = W * H * spp
    value = samples_per_step * args.steps / elapsed / 1e6

    roof = None
    if rank == 0 and not args.no_roofline:
        os.environ["NORI_POOL_PARTS"] = "1"
        r.render(passes=share[1], pass_begin=share[0], blocks=share[2], path_pool=args.pool)
        r.render(passes=share[1], pass_begin=share[0], blocks=share[2], path_pool=args.pool, timing=True)
        ts = r.last_stats
        os.environ.pop("NORI_POOL_PARTS")
        roof = roofline(ts, share_samples, args.config)
    if world > 1:
        dist.barrier()

    if rank == 0:
        out = {
            "metric": METRIC if args.config == "c2" else f"Msamples/sec on {label}",
            "value": value,
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: the reference's scene files (C3/C4: generated mesh / env map, nori_amd.configs)",
            "config": {"workload": label, "scene": os.path.relpath(xml, ROOT) if xml.startswith(ROOT) else
                       os.path.basename(xml), "integrator": scene.integrator,
                       "parallelism": f"{args.shard}-sharded x{world}, RCCL film reduce in libnori_gpu" if world > 1
                       else "single GPU", "path_pool": last.get("path_pool")},
            "samples_per_step": samples_per_step,
            "invalid_samples": invalid,
            "roofline": roof,
            "kernel_ms_isolated": {k: roof["kernels"][k]["ms_per_step"] for k in roof["kernels"]} if roof else None,
            "rays_per_sample": {"closest": last["rays_closest"] / share_samples,
                                "shadow": last["rays_shadow"] / share_samples,
                                "finisher": last["rays_finish"] / share_samples},
            # whole-job ray throughput (all ranks' rays over the step time)
            "grays_per_s": {k: world * last[f"rays_{k}"] / (elapsed / args.steps) / 1e9
                            for k in ("closest", "shadow", "finish")},
            "per_rank_ms_per_step": rank_ms,
            "comm_nranks_per_rank": comm_ranks,
            # scan-mode scenes: the scan kernels specialised for the scene through hipRTC at context
            # creation (csrc/rtc.hip), outside the timed region; cached per process and on disk
            "scan_kernels": {"specialised": bool(last.get("scan_rtc")), "compile_ms": last.get("ms_scan_rtc"),
                             "from_cache": bool(last.get("scan_rtc_cached"))},
            "wavefront_iterations": last["iterations"],
            "stream_parts": last.get("stream_parts", 1),
            "hip_runtime": hip_runtime(),
        }
        if world == 1 and not args.no_parity and args.config == "c2":
            out["parity"] = parity_full(scene, film_host, W, H, spp)
        elif world == 1 and not args.no_parity:
            small = {"c2": (512, 512, 16), "c3": (128, 128, 4), "c4": (128, 128, 8), "c5": (160, 120, 8)}
            pw, ph, ps = small[args.config]
            pxml = xml if args.config != "c3" else configs.heightfield_scene(tmp, n=512, width=pw, height=ph, spp=ps)
            if args.config == "c4":
                pxml = configs.envmap_scene(tmp, pw, ph, ps)
            out["parity"] = parity_check(pxml, pw, ph, ps)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(xml, W, H, args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    r.close()
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
