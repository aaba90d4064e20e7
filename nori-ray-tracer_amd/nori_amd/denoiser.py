"""Command-line NL-means denoiser on the GPU, the drop-in for
denoiser/denoiser.py:

    python -m nori_amd.denoiser --img_path scene.exr --var_path scene_variance.png

Same arguments and parameters as the script (r = 3, f = 3, k = 0.02,
denoiser.py:22-28); the image is read from EXR and scaled by 1/255 as the
script does; the variance image is an 8-bit PNG (what hdrToLdr writes from
`<stem>_variance.exr`, decoded here and taken to grey the way OpenCV's
imread + COLOR_RGB2GRAY does) or directly the `_variance.exr`.  The script
shows its result in a window; here it is written to `<stem>_denoised.exr`
(in the input's scale) and optionally a PNG.  --textbook selects the
textbook variance terms instead of the script's (nori_gpu.h, nori_denoise).
"""
import argparse
import os
import struct
import sys
import zlib

import numpy as np

from . import denoise, read_exr, variance_gray, write_exr, write_png


def read_png_rgb8(path):
    """8-bit RGB / RGBA non-interlaced PNG -> (H, W, 3) uint8 (all five row filters)."""
    data = open(path, "rb").read()
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        raise ValueError(f"{path}: not a PNG file")
    pos, idat, hdr = 8, b"", None
    while pos < len(data):
        n, kind = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        if kind == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif kind == b"IDAT":
            idat += body
        pos += 12 + n
    w, h, depth, ctype, _, _, interlace = hdr
    if depth != 8 or ctype not in (2, 6) or interlace:
        raise ValueError(f"{path}: only 8-bit RGB/RGBA non-interlaced PNGs are supported")
    bpp = 3 if ctype == 2 else 4
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + bpp * w)
    img = np.zeros((h, bpp * w), np.int32)
    for y in range(h):
        f, line = raw[y, 0], raw[y, 1:].astype(np.int32)
        prev = img[y - 1] if y else np.zeros(bpp * w, np.int32)
        if f == 0:
            cur = line
        elif f == 2:
            cur = (line + prev) & 255
        else:
            cur = np.zeros(bpp * w, np.int32)
            for x in range(bpp * w):
                a = cur[x - bpp] if x >= bpp else 0
                c = prev[x - bpp] if x >= bpp else 0
                if f == 1:
                    pred = a
                elif f == 3:
                    pred = (a + prev[x]) >> 1
                else:  # Paeth
                    p = a + prev[x] - c
                    pa, pb, pc = abs(p - a), abs(p - prev[x]), abs(p - c)
                    pred = a if pa <= pb and pa <= pc else (prev[x] if pb <= pc else c)
                cur[x] = (line[x] + pred) & 255
        img[y] = cur
    return img.reshape(h, w, bpp)[..., :3].astype(np.uint8)


def png_gray(rgb8):
    """imread (B, G, R order) + COLOR_RGB2GRAY + / 255 (denoiser.py:20-21)."""
    bgr = rgb8[..., ::-1].astype(np.int64)
    g = (4899 * bgr[..., 0] + 9617 * bgr[..., 1] + 1868 * bgr[..., 2] + (1 << 13)) >> 14
    return (g / 255.0).astype(np.float32)


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m nori_amd.denoiser")
    ap.add_argument("--img_path", required=True, help="image to denoise (.exr)")
    ap.add_argument("--var_path", required=True, help="per-pixel variance (.png from hdrToLdr, or .exr)")
    ap.add_argument("--out", default=None, help="output EXR (default <stem>_denoised.exr)")
    ap.add_argument("--png", action="store_true", help="also write an sRGB PNG")
    ap.add_argument("--textbook", action="store_true", help="textbook variance terms instead of the script's")
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args(argv)
    img = read_exr(a.img_path)
    if a.var_path.lower().endswith(".exr"):
        var = variance_gray(read_exr(a.var_path))
    else:
        var = png_gray(read_png_rgb8(a.var_path))
    if var.shape != img.shape[:2]:
        print(f"error: variance {var.shape} does not match image {img.shape[:2]}", file=sys.stderr)
        return 1
    out = denoise(img, var, mode=1 if a.textbook else 0, device=a.device)
    dst = a.out or os.path.splitext(a.img_path)[0] + "_denoised.exr"
    write_exr(dst, out)
    if a.png:
        write_png(os.path.splitext(dst)[0] + ".png", out)
    print(f"wrote {dst}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
