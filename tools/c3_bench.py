"""Config C3: a 512x512 height field (524,288 triangles) with the
microfacet parameters of ttest-microfacet.xml inside the Cornell box, path_mis,
512x512 @ 128 spp on one GPU.  Prints scene load / BVH build / render times."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "nori-ray-tracer_amd"), os.path.join(ROOT, "tests")]
import nori_amd  # noqa: E402
import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 128
out = os.path.join(ROOT, "gpurun_out", "c3")
t = time.time()
xml = synth.heightfield_scene(out, n=n, width=512, height=512, spp=spp)
t_gen = time.time() - t
t = time.time()
s = nori_amd.load_scene(xml)
t_load = time.time() - t
t = time.time()
bi = nori_amd.bvh_info(s)
t_bvh = time.time() - t
t = time.time()
r = nori_amd.GpuRenderer(s, 0)
t_create = time.time() - t
r.render(passes=1)  # warm-up
t = time.time()
r.render()
t_render = time.time() - t
st = r.last_stats
r.render(timing=True)
ts = r.last_stats
r.close()
print(json.dumps({"config": f"C3 heightfield n={n} ({2 * n * n} tris) 512x512@{spp}spp path_mis",
                  "gen_s": t_gen, "load_s": t_load, "bvh_build_s (host, threaded)": t_bvh, "bvh_sah": bi["sah_cost"],
                  "create_s (HIP init + BVH build + upload)": t_create,
                  "render_s": t_render, "Msamples_per_s": st["samples"] / t_render / 1e6,
                  "bvh_nodes": st["bvh_nodes"], "bvh_depth": st["bvh_depth"],
                  "rays_per_sample": (st["rays_closest"] + st["rays_shadow"]) / st["samples"],
                  "kernel_ms": {k: ts[k] for k in ("ms_extend", "ms_shadow", "ms_shade", "ms_splat", "ms_finish")},
                  "iterations": st["iterations"]}, indent=1))
