"""The axis-plane proofs (kernels.hip plane_may_hit, pair_candidate) hold for
kappa = (|P| + |Q|) / |P - Q| <= 32 of a triangle's normal products, which
runtime.hip axis_plane checks.  The Cornell box's rectangles have kappa = 1;
here skewed sliver triangles in y = const planes span kappa 1.5 .. 64: the
host must class exactly those with kappa <= 32 as plane triangles
(nori_scene_scan_list), and for every one it accepted, both culls must imply
rejection by the reference's Moller-Trumbore test on random, grazing and
edge-aimed rays -- including slivers at the accepted limit."""
import os

import numpy as np

import nori_amd
from conftest import scene_path
from test_pair_filter import pair_candidate, random_rays, targeted_rays
from test_plane_cull import may_hit, moller_trumbore

f32 = np.float32
KAPPAS = [1.5, 4.0, 16.0, 30.0, 31.5, 31.9, 32.2, 33.0, 40.0, 64.0]


def kappa(e1, e2, A=1):
    B, C = (A + 1) % 3, (A + 2) % 3
    P, Q = float(e1[B]) * float(e2[C]), float(e1[C]) * float(e2[B])
    return (abs(P) + abs(Q)) / abs(P - Q)


def sliver_scene(tmp):
    """Slivers with edges e1 = s R (1, 1), e2 = s R (1 + eps, 1) in the (x, z)
    plane (rotated by R), kappa = (2 + eps) / eps; coordinates on a 2^-12 grid
    so the edges are exact float differences."""
    rng = np.random.default_rng(3)
    q = 2.0 ** -12
    verts, faces, want = [], [], []
    for i, k in enumerate(KAPPAS):
        for j in range(2):
            y = 0.2 + 0.1 * i + 0.03 * j
            eps = 2.0 / (k - 1.0)
            th = rng.uniform(0, 2 * np.pi)
            R = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
            s = rng.uniform(0.3, 0.6)
            a, b = s * R @ np.array([1.0, 1.0]), s * R @ np.array([1.0 + eps, 1.0])
            v0 = np.array([rng.uniform(-0.4, 0.0), rng.uniform(-0.4, 0.0)])
            pts = [v0, v0 + a, v0 + b]
            pts = [np.round(p / q) * q for p in pts]
            base = len(verts) + 1
            for p in pts:
                verts.append((p[0], y, p[1]))
            faces.append((base, base + 1, base + 2))
    obj = os.path.join(tmp, "slivers.obj")
    with open(obj, "w") as f:
        f.write("".join(f"v {float(x):.9g} {float(y):.9g} {float(z):.9g}\n" for x, y, z in np.asarray(verts, np.float32)))
        f.write("".join(f"f {i} {j} {k}\n" for i, j, k in faces))
    with open(scene_path("pa4", "cbox", "cbox_path_mis.xml")) as f:
        xml = f.read().replace('"meshes/', '"' + scene_path("pa4", "cbox", "meshes") + "/")
    xml = xml.replace("</scene>", f'<mesh type="obj"><string name="filename" value="{obj}"/>'
                      '<bsdf type="diffuse"/></mesh>\n</scene>')
    path = os.path.join(tmp, "slivers.xml")
    with open(path, "w") as f:
        f.write(xml)
    return path


def test_kappa_limit_and_culls(built, tmp_path):
    s = nori_amd.load_scene(sliver_scene(str(tmp_path)), 32, 32, 1)
    L = nori_amd.scan_list(s)
    rec = L["records"]
    npairs = len(L["plane_c"])
    in_pair = {}
    for i in range(L["tris"]):
        r = rec[i]
        if not r[4:7].any() or r[1] < 0.19 or r[1] > 1.3:  # padding, and the box's own walls / light
            continue
        k = kappa(r[4:7], r[8:11])
        in_pair[i] = (i < 2 * npairs, k)
    assert len(in_pair) == 2 * len(KAPPAS)
    for i, (paired, k) in in_pair.items():
        assert paired == (k <= 32.0), (i, k, paired)
    assert any(30 < k <= 32 and p for p, k in in_pair.values())  # slivers at the limit are accepted
    rng = np.random.default_rng(17)
    checked = 0
    for g in range(npairs):
        A = int(np.searchsorted(L["plane_end"], g, side="right"))
        recs = [rec[2 * g], rec[2 * g + 1]]
        if not any((2 * g + e) in in_pair for e in range(2)):
            continue
        f, c = L["plane_f"][g], L["plane_c"][g]
        for o, d in (random_rays(rng, 100000), targeted_rays(rng, recs, A, 120000)):
            o[:10000, A] = c
            mint = np.maximum(f32(1e-4), f32(1e-4) * np.abs(o).max(axis=1)).astype(f32)
            mint[10000:12000] = 0.0
            maxt = np.full(len(o), np.inf, f32)
            O, D = (o[:, 0], o[:, 1], o[:, 2]), (d[:, 0], d[:, 1], d[:, 2])
            hit = np.zeros(len(o), bool)
            for r in recs:
                if r[4:7].any():
                    hit |= moller_trumbore(r[0:3], r[4:7], r[8:11], O, D, mint, maxt)[0]
            assert not (hit & ~may_hit(o[:, A], d[:, A], c, mint, maxt)).any()
            assert not (hit & ~pair_candidate(A, f, o, d, mint, maxt)).any()
            checked += int(hit.sum())
    assert checked > 10000
