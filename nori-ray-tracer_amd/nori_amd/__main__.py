"""Command line mirror of `nori_euler <scene.xml>` (src/main_euler.cpp:24-60 ->
RenderThread::renderScene, render.cpp:135-280):

    python -m nori_amd scene.xml [--width W --height H --spp N] [--gpus G] [--png]

Parses the scene, renders it on the GPU(s) and writes `<stem>.exr` and
`<stem>_variance.exr` next to the XML (render.cpp:158-169), plus `<stem>.png`
with --png (Bitmap::saveToLDR, the hdrToLdr tool).  With --gpus G > 1 one
context per device renders a slice of the sample passes on its own host
thread and the RGBW films are summed (ImageBlock::put(block), block.cpp:124-133).
"""
import argparse
import os
import sys
import threading
import time

import numpy as np

from . import GpuRenderer, NoriError, develop, device_count, film_variance, load_scene, write_exr, write_png


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m nori_amd", description=__doc__.split("\n\n")[0])
    ap.add_argument("scene")
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--png", action="store_true", help="also write <stem>.png (sRGB, 8 bit)")
    a = ap.parse_args(argv)
    try:
        scene = load_scene(a.scene, a.width, a.height, a.spp)
        n = max(1, min(a.gpus, device_count()))
        spp = scene.spp
        renderers = [GpuRenderer(scene, d) for d in range(n)]
        films = [np.zeros(scene.film_shape(), np.float32) for _ in range(n)]
        stats = [np.zeros((scene.height, scene.width, 8), np.float32) for _ in range(n)]
        errors = []

        def run(i):
            b, e = spp * i // n, spp * (i + 1) // n
            try:
                if e > b:
                    renderers[i].render(passes=e - b, pass_begin=b, out=films[i], variance=stats[i])
            except NoriError as err:
                errors.append(err)

        print("Rendering .. ", end="", flush=True)
        t0 = time.time()
        threads = [threading.Thread(target=run, args=(i,)) for i in range(n)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if errors:
            raise errors[0]
        print(f"done. (took {1e3 * (time.time() - t0):.1f}ms)")
        for r in renderers:
            r.close()
        image = develop(scene, np.sum(films, axis=0))
        stem = os.path.splitext(a.scene)[0]
        print(f"Writing a {scene.width}x{scene.height} OpenEXR file to \"{stem}.exr\"")
        write_exr(stem + ".exr", image)
        write_exr(stem + "_variance.exr", film_variance(scene, np.sum(stats, axis=0)))
        if a.png:
            print(f"Writing a {scene.width}x{scene.height} PNG file to \"{stem}.png\"")
            write_png(stem + ".png", image)
    except NoriError as e:
        print(f"Fatal error: {e}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
