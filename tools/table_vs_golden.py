"""Render the reference's table scene on the GPU and compare with the reference golden EXR
(scenes/pa4/table/ref/*_512spp.exr, rendered by the course solution)."""
import sys
import time
import os
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nori-ray-tracer_amd"))
import nori_amd  # noqa: E402

for integ in sys.argv[1:] or ["path_mis"]:
    s = nori_amd.load_scene(os.path.join(ROOT, "scenes", "pa4", "table", f"table_{integ}.xml"))
    ref = nori_amd.read_exr(os.path.join(ROOT, "scenes", "pa4", "table", "ref", f"table_{integ}_512spp.exr"))
    with nori_amd.GpuRenderer(s, 0) as r:
        t = time.time()
        img = nori_amd.develop(s, r.render())
        dt = time.time() - t
        st = r.last_stats
    d = img - ref
    rel = float(np.mean(d ** 2 / (ref ** 2 + 1e-2)))
    k = 8
    bm = lambda a: a[: a.shape[0] // k * k, : a.shape[1] // k * k].reshape(a.shape[0] // k, k, a.shape[1] // k, k, 3).mean(axis=(1, 3))
    bd = bm(img) - bm(ref)
    print(f"{integ}: {dt:.2f}s {st['samples']/dt/1e6:.0f} Msamples/s  mean gpu {img.mean(axis=(0,1))} ref {ref.mean(axis=(0,1))}"
          f" relMSE {rel:.3e} L2 {float(np.mean(d**2)):.3e} bias {float(d.mean()):.3e}"
          f" 8x8-block |diff| p50 {np.median(np.abs(bd)):.3e} p99 {np.quantile(np.abs(bd), .99):.3e}", flush=True)
    np.save(os.path.join(ROOT, "gpurun_out", f"table_{integ}.npy"), img)
