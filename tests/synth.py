"""Deterministic synthetic scenes (the reference's large assets are missing:
ajax.obj is listed in .MISSING_LARGE_BLOBS, so config C3 uses a generated
height field of the same scale -- SURVEY.md 8d).

heightfield_scene(n): an n x n grid height field (2*n*n triangles) with
z = sum of four fixed sines, inside the Cornell box walls and light of
scenes/pa4/cbox, shaded with the microfacet parameters of
scenes/pa3/tests/ttest-microfacet.xml (alpha 0.1, intIOR 1.5,
extIOR 1.000277, kd 0.1 0.2 0.15).  n = 512 gives 524,288 triangles.
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
CBOX = os.path.join(os.path.dirname(HERE), "scenes", "pa4", "cbox")


def heightfield_obj(path, n):
    xs = np.linspace(-0.8, 0.8, n + 1, dtype=np.float64)
    X, Z = np.meshgrid(xs, xs)
    Y = (0.35 + 0.08 * np.sin(7.1 * X + 0.3) * np.cos(5.3 * Z - 0.7) + 0.05 * np.sin(13.7 * X * Z + 1.1)
         + 0.03 * np.cos(23.1 * Z + 0.2) + 0.02 * np.sin(31.3 * X - 0.5))
    v = np.stack([X.ravel(), Y.ravel(), Z.ravel()], 1)
    idx = np.arange((n + 1) * (n + 1)).reshape(n + 1, n + 1) + 1
    a, b, c, d = idx[:-1, :-1].ravel(), idx[:-1, 1:].ravel(), idx[1:, 1:].ravel(), idx[1:, :-1].ravel()
    faces = np.concatenate([np.stack([a, b, c], 1), np.stack([a, c, d], 1)])
    with open(path, "w") as f:
        f.write("".join(f"v {x:.6f} {y:.6f} {z:.6f}\n" for x, y, z in v))
        f.write("".join(f"f {i} {j} {k}\n" for i, j, k in faces))
    return len(faces)


def heightfield_scene(outdir, n=64, integrator="path_mis", width=256, height=256, spp=16):
    os.makedirs(outdir, exist_ok=True)
    obj = os.path.join(outdir, f"heightfield_{n}.obj")
    if not os.path.exists(obj):
        heightfield_obj(obj, n)
    xml = os.path.join(outdir, f"heightfield_{n}_{integrator}.xml")
    m = os.path.join(CBOX, "meshes")
    with open(xml, "w") as f:
        f.write(f"""<?xml version='1.0' encoding='utf-8'?>
<scene>
  <integrator type="{integrator}"/>
  <camera type="perspective">
    <float name="fov" value="27.7856"/>
    <transform name="toWorld">
      <scale value="-1,1,1"/>
      <lookat target="0, 0.893051, 4.41198" origin="0, 0.919769, 5.41159" up="0, 1, 0"/>
    </transform>
    <integer name="height" value="{height}"/>
    <integer name="width" value="{width}"/>
  </camera>
  <sampler type="independent"><integer name="sampleCount" value="{spp}"/></sampler>
  <mesh type="obj"><string name="filename" value="{m}/walls.obj"/>
    <bsdf type="diffuse"><color name="albedo" value="0.725 0.71 0.68"/></bsdf></mesh>
  <mesh type="obj"><string name="filename" value="{m}/rightwall.obj"/>
    <bsdf type="diffuse"><color name="albedo" value="0.161 0.133 0.427"/></bsdf></mesh>
  <mesh type="obj"><string name="filename" value="{m}/leftwall.obj"/>
    <bsdf type="diffuse"><color name="albedo" value="0.630 0.065 0.05"/></bsdf></mesh>
  <mesh type="obj"><string name="filename" value="{obj}"/>
    <bsdf type="microfacet">
      <float name="alpha" value="0.1"/><float name="intIOR" value="1.5"/>
      <float name="extIOR" value="1.000277"/><color name="kd" value="0.1, 0.2, 0.15"/>
    </bsdf></mesh>
  <mesh type="obj"><string name="filename" value="{m}/light.obj"/>
    <emitter type="area"><color name="radiance" value="15 15 15"/></emitter></mesh>
</scene>
""")
    return xml
