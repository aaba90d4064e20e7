"""The BASELINE.json configurations as scene files.

C2 is the reference's own scene file; the others need assets the reference
checkout lacks, so they are generated deterministically:

* C3 -- ajax.obj (~544k triangles) is listed in .MISSING_LARGE_BLOBS:
  heightfield_scene(n) is an n x n grid height field (2 n^2 triangles, n = 512
  gives 524,288) with z = sum of four fixed sines, inside the Cornell box walls
  and light of scenes/pa4/cbox, shaded with the microfacet parameters of
  scenes/pa3/tests/ttest-microfacet.xml (alpha 0.1, intIOR 1.5, extIOR
  1.000277, kd 0.1 0.2 0.15).
* C4 -- envmaptext.exr / sky.exr are missing: envmap_scene() puts the
  Disney-sphere Cornell box of scenes/project/disney inside a sky sphere
  carrying a fixed-formula lat-long map (envmap_image), the pattern of
  scenes/project/envmap.xml.
* C5 -- scenes/project/volumetric/volumetric.xml as committed.

config_scene(name, outdir) returns (xml path, workload label) for
"c2" | "c3" | "c4" | "c5" at the BASELINE sizes.
"""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SCENES = os.path.join(ROOT, "scenes")
CBOX = os.path.join(SCENES, "pa4", "cbox")


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


DISNEY = os.path.join(SCENES, "project", "disney")


def envmap_image(rows=256, cols=512):
    """Lat-long HDR map of fixed formula (the reference's envmaptext.exr / sky.exr
    are missing): rows index theta in [0, pi] (the envmap's `m_width` axis),
    cols index phi in [0, 2 pi).  Sky gradient + a sun lobe + a warm horizon band."""
    th = (np.arange(rows, dtype=np.float64) + 0.5) / rows * np.pi
    ph = (np.arange(cols, dtype=np.float64) + 0.5) / cols * 2 * np.pi
    T, P = np.meshgrid(th, ph, indexing="ij")
    d = np.stack([np.sin(T) * np.cos(P), np.sin(T) * np.sin(P), np.cos(T)], -1)
    sun = np.array([0.3, 0.5, 0.81])
    sun /= np.linalg.norm(sun)
    lobe = np.exp(40.0 * (d @ sun - 1.0))
    sky = 0.4 + 0.6 * np.clip(np.cos(T), 0, 1)
    band = np.exp(-((T - np.pi / 2) / 0.15) ** 2)
    img = np.stack([0.35 * sky + 0.8 * band + 30 * lobe,
                    0.55 * sky + 0.5 * band + 28 * lobe,
                    0.95 * sky + 0.2 * band + 24 * lobe], -1)
    return img.astype(np.float32)


def envmap_scene(outdir, width=128, height=128, spp=16, integrator="path_mis", rows=256, cols=512, radius=30.0):
    """Config C4: the Disney-sphere Cornell box of
    scenes/project/disney inside an env-mapped sky sphere, as in the reference's
    scenes/project/envmap.xml pattern (envmap emitter on a radius-30 sphere)."""
    from . import write_exr

    os.makedirs(outdir, exist_ok=True)
    exr = os.path.join(outdir, f"sky_{rows}x{cols}.exr")
    if not os.path.exists(exr):
        write_exr(exr, envmap_image(rows, cols))
    src = open(os.path.join(DISNEY, "cbox_path_mis.xml")).read()
    src = src.replace('value="meshes/', f'value="{os.path.join(DISNEY, "meshes")}/')
    src = src.replace('<integrator type="path_mis"/>', f'<integrator type="{integrator}"/>')
    src = src.replace('<integer name="height" value="600"/>', f'<integer name="height" value="{height}"/>')
    src = src.replace('<integer name="width" value="800"/>', f'<integer name="width" value="{width}"/>')
    src = src.replace('<integer name="sampleCount" value="1024"/>', f'<integer name="sampleCount" value="{spp}"/>')
    sky = f"""
	<mesh type="sphere">
		<point name="center" value="0,1,0"/>
		<float name="radius" value="{radius}"/>
		<emitter type="envmap">
			<string name="filename" value="{exr}"/>
		</emitter>
	</mesh>
</scene>"""
    src = src.replace("</scene>", sky)
    xml = os.path.join(outdir, f"envmap_{integrator}.xml")
    with open(xml, "w") as f:
        f.write(src)
    return xml


def cbox_variant(outdir, name, integrator="path_mis", camera_type="perspective", camera_props="",
                 integrator_props="", extra="", width=0, height=0):
    """scenes/pa4/cbox/cbox_path_mis.xml with another integrator and camera
    plugin (thinlens.cpp / advancedCamera.cpp properties in `camera_props`,
    e.g. lensRadius / focalDist / distortion / chromaticAberation) and extra
    scene children (free-standing point/spot emitters)."""
    import re

    os.makedirs(outdir, exist_ok=True)
    src = open(os.path.join(CBOX, "cbox_path_mis.xml")).read()
    src = src.replace('value="meshes/', f'value="{os.path.join(CBOX, "meshes")}/')
    src = src.replace('<integrator type="path_mis"/>',
                      f'<integrator type="{integrator}">{integrator_props}</integrator>')
    src = src.replace('<camera type="perspective">', f'<camera type="{camera_type}">{camera_props}')
    if width:
        src = re.sub(r'<integer name="width" value="\d+"/>', f'<integer name="width" value="{width}"/>', src)
    if height:
        src = re.sub(r'<integer name="height" value="\d+"/>', f'<integer name="height" value="{height}"/>', src)
    src = src.replace("</scene>", extra + "\n</scene>")
    xml = os.path.join(outdir, f"{name}.xml")
    with open(xml, "w") as f:
        f.write(src)
    return xml


# name -> (scene, width, height, spp, label); BASELINE.json configs[1..4]
CONFIGS = {
    "c2": ("cbox", 512, 512, 512, "cbox_path_mis 512x512@512spp"),
    "c3": ("heightfield", 512, 512, 128, "C3 heightfield 524288 tris microfacet path_mis 512x512@128spp"),
    "c4": ("envmap", 1024, 1024, 1024, "C4 disney + envmap path_mis 1024x1024@1024spp"),
    "c5": ("volumetric", 800, 600, 2048, "C5 volumetric 800x600@2048spp"),
}


def config_scene(name, outdir, width=0, height=0, spp=0):
    """(xml path, label, width, height, spp) of BASELINE config `name`; sizes override when > 0."""
    kind, w, h, s, label = CONFIGS[name]
    w, h, s = width or w, height or h, spp or s
    if kind == "cbox":
        xml = os.path.join(CBOX, "cbox_path_mis.xml")
    elif kind == "heightfield":
        xml = heightfield_scene(outdir, n=512, width=w, height=h, spp=s)
    elif kind == "envmap":
        xml = envmap_scene(outdir, w, h, s)
    else:
        xml = os.path.join(SCENES, "project", "volumetric", "volumetric.xml")
    if (w, h, s) != CONFIGS[name][1:4]:
        label = f"{label.rsplit(' ', 1)[0]} {w}x{h}@{s}spp"
    return xml, label, w, h, s
