"""Per-step wall times of the headline render (diagnostic): warm-up, then
renders with HIP-event timing, host-timed one by one, with per-kernel sums."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nori-ray-tracer_amd"))
import nori_amd  # noqa: E402

s = nori_amd.load_scene(os.path.join(ROOT, "scenes", "pa4", "cbox", "cbox_path_mis.xml"), 512, 512, 512)
r = nori_amd.GpuRenderer(s, 0)
r.render()
for i in range(5):
    if i == 3:
        time.sleep(0.5)  # an idle gap: does the next render slow down again?
    t = time.perf_counter()
    r.render(timing=True)
    st = r.last_stats
    print(f"step {i}: host {1e3 * (time.perf_counter() - t):.1f} ms, total {st['ms_total']:.1f}, "
          f"shade {st['ms_shade']:.1f} extend {st['ms_extend']:.1f} shadow {st['ms_shadow']:.1f} "
          f"splat {st['ms_splat']:.1f} finish {st['ms_finish']:.1f}, iterations {st['iterations']}", flush=True)
r.close()
