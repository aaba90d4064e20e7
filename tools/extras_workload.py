"""Workload for the rocprofv3 summary of the widened kernels (photon mapper
and denoiser): cbox photon mapping at 800x600, 32 spp, 1M photons (the
reference's cbox_pmap configuration with 1M instead of 10M photons), then the
NL-means denoiser on an 800x600 16-spp path_mis render.
Run: rocprofv3 --kernel-trace --stats -d gpurun_out/prof_extras -- python3 tools/extras_workload.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "nori-ray-tracer_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

import nori_amd  # noqa: E402
import synth  # noqa: E402

out = os.path.join(ROOT, "gpurun_out", "extras")
os.makedirs(out, exist_ok=True)
xml = synth.cbox_variant(out, "pmap", integrator="photonmapper",
                         integrator_props='<integer name="photonCount" value="1000000"/>'
                                          '<float name="photonRadius" value="0.05"/>', width=800, height=600)
s = nori_amd.load_scene(xml, 0, 0, 32)
t0 = time.perf_counter()
with nori_amd.GpuRenderer(s, 0) as r:
    t1 = time.perf_counter()
    img = nori_amd.develop(s, r.render())
    t2 = time.perf_counter()
print(f"photonmapper 800x600 32spp 1M photons: create {t1 - t0:.3f} s, render {t2 - t1:.3f} s", flush=True)
p = nori_amd.load_scene(os.path.join(ROOT, "scenes/pa4/cbox/cbox_path_mis.xml"), 800, 600, 16)
stats = np.zeros((600, 800, 8), np.float32)
with nori_amd.GpuRenderer(p, 0) as r:
    noisy = nori_amd.develop(p, r.render(variance=stats))
var = nori_amd.variance_gray(nori_amd.film_variance(p, stats))
for i in range(3):
    t0 = time.perf_counter()
    nori_amd.denoise(noisy, var)
    print(f"denoise 800x600 (host buffers): {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
