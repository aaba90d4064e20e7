"""Render a scene XML on GPU 0 and print Msamples/s and per-kernel times.
usage: python tools/scene_bench.py <scene.xml> [spp] [width height]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "nori-ray-tracer_amd")]
import nori_amd  # noqa: E402

xml = sys.argv[1]
kw = {}
if len(sys.argv) > 2:
    kw["spp"] = int(sys.argv[2])
if len(sys.argv) > 4:
    kw["width"], kw["height"] = int(sys.argv[3]), int(sys.argv[4])
s = nori_amd.load_scene(xml, **kw)
r = nori_amd.GpuRenderer(s, 0)
r.render(passes=1)  # warm-up
t = time.time()
r.render()
dt = time.time() - t
st = r.last_stats
r.render(timing=True)
ts = r.last_stats
r.close()
print(json.dumps({"scene": os.path.basename(xml), "render_s": dt, "Msamples_per_s": st["samples"] / dt / 1e6,
                  "bvh_depth": st["bvh_depth"],
                  "kernel_ms": {k: round(ts[k], 2) for k in ("ms_extend", "ms_shadow", "ms_shade", "ms_splat", "ms_finish")}}))
