"""advancedCamera (advancedCamera.cpp) against the reference's own report
renders of its Cornell box (report-project/images/*.png, copied as data to
tests/golden/project/report_*.png; parameters from report-project.html:
479-520; scene scenes/project/adv_cam/cbox_adv_cam.xml = the reference's
scenes/project/cbox_adv_cam.xml with the pa4 cbox meshes).

The report images are cropped screenshots of partial (~15 %) renders, so the
pin is qualitative but discriminating: each screenshot is aligned with our
800x600 render of the same parameters, compared on 20x20-block means of the
8-bit image, and must match that render better than our renders of the other
parameter sets (depth of field at other focal distances / lens radii, no
lens, barrel distortion).

Not pinned: report_distortion_only.png ("m_distortion = (3, 3)").  The
checkout's advancedCamera.cpp:141-168 solves r (1 + k1 r^2 + k2 r^4) = y by
Newton's method and scales the near-plane point by r / y < 1 for positive
k: the view zooms in (our render, the oracle's, and the code's own
arithmetic agree), while the screenshot shows the opposite -- a barrel
zoom-out with 19 % of the pixels in an unmapped black border.  No
parameter pair of the checkout's formula reproduces it (searched on the
oracle: (3, 3) RMS 54 LDR levels, border IoU 0.00; the nearest, (-3, -3) and
(-1, -1), RMS 39-41 and IoU <= 0.47), so it was rendered by another version
of the camera."""
import os

import numpy as np
import pytest

import nori_amd
from conftest import ROOT

pytestmark = pytest.mark.gpu
XML = os.path.join(ROOT, "scenes", "project", "adv_cam", "cbox_adv_cam.xml")
GOLD = os.path.join(ROOT, "tests", "golden", "project")
VARIANTS = {  # report image -> camera properties
    "cbox_ref": {},
    "dof_only": {"focalDist": 5.7, "lensRadius": 0.35},
    "dof_fd5_7_lr0_1": {"focalDist": 5.7, "lensRadius": 0.1},
    "dof_fd5_7_lr0_9": {"focalDist": 5.7, "lensRadius": 0.9},
    "dof_fd5_lr0_35": {"focalDist": 5.0, "lensRadius": 0.35},
    "distortion_only": {"distortion": (3, 3)},
}


def _scene(tmp_path, props, spp=64):
    src = open(XML).read()
    extra = ""
    for k, v in props.items():
        if isinstance(v, tuple):
            extra += f'<vector name="{k}" value="{v[0]}, {v[1]}"/>'
        else:
            extra += f'<float name="{k}" value="{v}"/>'
    src = src.replace('<integer name="height" value="600"/>', '<integer name="height" value="600"/>' + extra)
    src = src.replace('value="../../pa4/', f'value="{os.path.join(ROOT, "scenes", "pa4")}/')
    path = tmp_path / ("adv_%d.xml" % abs(hash(tuple(sorted(props.items())))))
    path.write_text(src)
    return nori_amd.load_scene(str(path), 800, 600, spp)


@pytest.fixture(scope="module")
def renders(tmp_path_factory):
    out = {}
    tmp = tmp_path_factory.mktemp("advcam")
    for name, props in VARIANTS.items():
        s = _scene(tmp, props)
        with nori_amd.GpuRenderer(s, 0) as r:
            out[name] = nori_amd.ldr_bytes(nori_amd.develop(s, r.render())).astype(np.float64)
    return out


def _shot(name):
    from nori_test_util import read_png
    return read_png(os.path.join(GOLD, f"report_{name}.png"))[..., :3].astype(np.float64)


def _align(ours, shot):
    """Offset of the screenshot (a crop) inside our 800x600 render: least
    squares on a 4x subsampled grey image."""
    h, w = shot.shape[:2]
    g, gs = ours.mean(-1), shot.mean(-1)
    return min((np.mean((g[dy:dy + h:4, dx:dx + w:4] - gs[::4, ::4]) ** 2), dy, dx)
               for dy in range(0, 600 - h + 1) for dx in range(0, 800 - w + 1))


def _block_err(ours, shot, dy, dx, b=20):
    h, w = shot.shape[:2]
    o = ours[dy:dy + h, dx:dx + w]
    hh, ww = h // b * b, w // b * b
    bo = o[:hh, :ww].reshape(hh // b, b, ww // b, b, 3).mean((1, 3))
    bs = shot[:hh, :ww].reshape(hh // b, b, ww // b, b, 3).mean((1, 3))
    return float(np.sqrt(np.mean((bo - bs) ** 2)))


@pytest.mark.parametrize("name", [n for n in VARIANTS if n != "distortion_only"])
def test_report_render_is_best_explained_by_its_parameters(renders, name):
    shot = _shot(name)
    err = {}
    for other, ours in renders.items():
        _, dy, dx = _align(ours, shot)
        err[other] = _block_err(ours, shot, dy, dx)
    print(name, {k: round(v, 2) for k, v in err.items()})
    best = min(err, key=err.get)
    assert best == name, err
    assert err[name] < 4.0, err[name]  # LDR levels of 20x20-block means (measured 1.3-2.0)
