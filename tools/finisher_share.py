"""Per-kernel time of one render of each BASELINE config (timing render, one
pool part): how much of the render the tail finisher takes.
usage: python tools/finisher_share.py [config ...]"""
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "nori-ray-tracer_amd")]
import nori_amd  # noqa: E402
from nori_amd import configs  # noqa: E402

os.environ["NORI_POOL_PARTS"] = "1"
tmp = tempfile.mkdtemp()
for cfg in sys.argv[1:] or ["c2", "c3", "c4", "c5"]:
    xml, label, W, H, spp = configs.config_scene(cfg, tmp, 0, 0, 0)
    s = nori_amd.load_scene(xml, W, H, spp)
    with nori_amd.GpuRenderer(s, 0) as r:
        r.render()
        r.render(timing=True)
        st = r.last_stats
    print(json.dumps({"config": cfg, "workload": label, "ms_total": round(st["ms_total"], 2),
                      **{k: round(st[k], 2) for k in ("ms_extend", "ms_shadow", "ms_shade", "ms_splat", "ms_finish")},
                      "iterations": st["iterations"], "rays_finish_per_sample": st["rays_finish"] / st["samples"]}),
          flush=True)
