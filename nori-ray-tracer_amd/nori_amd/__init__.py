"""nori_amd -- MI355X wavefront path tracer behind Nori's scene/plugin API.

Host-side mirror of the reference's render entry points:

* :func:`load_scene` -- ``loadFromXML`` + ``Scene::activate`` (parser.cpp:28,
  scene.cpp:43); the XML `type` names, properties and defaults are Nori's.
* :class:`GpuRenderer` -- one HIP context per device (``nori_gpu_create``);
  ``render`` replaces ``RenderThread::renderScene``'s pass loop
  (render.cpp:173-250) and returns the RGBW image block with its filter
  border (``ImageBlock``, block.h:48).
* :class:`RenderThread` -- ``renderScene(xml)`` writing ``<stem>.exr`` like
  render.cpp:158-261, with ``getProgress``/``stopRendering``.

All compute goes through ``lib/libnori_gpu.so`` (C ABI, include/nori_gpu.h);
there is no CPU fallback: without the library or a GPU the calls raise.
"""
import ctypes as C
import os
import threading
import time

import numpy as np

from . import _abi
from ._abi import NoriError, check, lib  # noqa: F401

__all__ = ["load_scene", "Scene", "GpuRenderer", "RenderThread", "NoriError", "device_count",
           "develop", "write_exr", "write_png", "read_exr", "film_variance", "ldr_bytes", "variance_gray",
           "denoise", "read_image"]


def _fptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


class Scene:
    """A loaded, flattened scene (owner of the nori_scene handle)."""

    def __init__(self, handle, path):
        self._h = C.c_void_p(handle)
        self.path = path
        self.desc_ptr = lib().nori_scene_get_desc(self._h)
        self.desc = self.desc_ptr.contents
        # kept on the instance: at interpreter exit the module globals may be gone before __del__ runs
        self._free = lib().nori_scene_free

    def __del__(self):
        h, free = getattr(self, "_h", None), getattr(self, "_free", None)
        if h is not None and h.value and free is not None:
            free(h)
            self._h = None

    # convenience views
    @property
    def width(self):
        return self.desc.camera.width

    @property
    def height(self):
        return self.desc.camera.height

    @property
    def spp(self):
        return self.desc.sample_count

    @property
    def border(self):
        return lib().nori_film_border(self.desc_ptr)

    @property
    def integrator(self):
        return _abi.INTEGRATOR_NAMES[self.desc.integrator]

    def film_shape(self):
        b = self.border
        return (self.height + 2 * b, self.width + 2 * b, 4)

    def positions(self):
        n = self.desc.num_vertices
        return np.ctypeslib.as_array(self.desc.positions, shape=(n, 3)).copy()

    def indices(self):
        n = self.desc.num_triangles
        return np.ctypeslib.as_array(self.desc.indices, shape=(n, 3)).copy()

    def shapes(self):
        return [self.desc.shapes[i] for i in range(self.desc.num_shapes)]

    def bsdfs(self):
        return [self.desc.bsdfs[i] for i in range(self.desc.num_bsdfs)]

    def emitters(self):
        return [self.desc.emitters[i] for i in range(self.desc.num_emitters)]

    def filter_table(self):
        t = np.zeros(_abi.FILTER_RESOLUTION + 1, np.float32)
        check(lib().nori_filter_table(self.desc_ptr, _fptr(t)))
        return t

    def num_blocks(self):
        bs = _abi.BLOCK_SIZE
        return ((self.width + bs - 1) // bs) * ((self.height + bs - 1) // bs)


def load_scene(path, width=0, height=0, spp=0):
    """Parse a Nori XML scene; width/height/spp > 0 override the XML values."""
    h = C.c_void_p()
    check(lib().nori_scene_load_xml(os.fsencode(path), int(width), int(height), int(spp), C.byref(h)))
    return Scene(h.value, path)


def device_count():
    n = C.c_int(0)
    check(lib().nori_gpu_device_count(C.byref(n)))
    return n.value


def develop(scene, rgbw):
    """ImageBlock::toBitmap (block.cpp:76-82): RGB / W without the border."""
    rgbw = np.ascontiguousarray(rgbw, dtype=np.float32)
    if rgbw.shape != scene.film_shape():
        raise ValueError(f"film shape {rgbw.shape} != {scene.film_shape()}")
    out = np.zeros((scene.height, scene.width, 3), np.float32)
    check(lib().nori_film_develop(scene.desc_ptr, _fptr(rgbw), _fptr(out)))
    return out


def write_exr(path, rgb):
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    check(lib().nori_write_exr(os.fsencode(path), _fptr(rgb), rgb.shape[1], rgb.shape[0]))


def write_png(path, rgb):
    """Bitmap::saveToLDR (bitmap.cpp:109-139): sRGB curve, 8-bit RGB PNG."""
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    check(lib().nori_write_png(os.fsencode(path), _fptr(rgb), rgb.shape[1], rgb.shape[0]))


def film_variance(scene, stats):
    """Variance of each pixel's mean (H, W, 3) from the (H, W, 8) sample
    statistics GpuRenderer.render(variance=...) accumulates (nori_film_variance)."""
    stats = np.ascontiguousarray(stats, dtype=np.float32)
    if stats.shape != (scene.height, scene.width, 8):
        raise ValueError(f"statistics shape {stats.shape} != {(scene.height, scene.width, 8)}")
    out = np.zeros((scene.height, scene.width, 3), np.float32)
    check(lib().nori_film_variance(scene.desc_ptr, _fptr(stats), _fptr(out)))
    return out


def ldr_bytes(rgb):
    """The 8-bit sRGB values Bitmap::saveToLDR writes (bitmap.cpp:122-139;
    nori_write_png): (uint8) clamp(255 * GammaCorrect(v) + 0.5, 0, 255), float32."""
    v = np.asarray(rgb, np.float32)
    with np.errstate(invalid="ignore"):
        g = np.where(v <= np.float32(0.0031308), np.float32(12.92) * v,
                     np.float32(1.055) * np.power(np.maximum(v, 0).astype(np.float32), np.float32(1.0 / 2.4))
                     - np.float32(0.055)).astype(np.float32)
    return np.clip(np.float32(255) * g + np.float32(0.5), 0, 255).astype(np.uint8)


def variance_gray(var_rgb):
    """The variance image denoiser.py:19-21 reads: the `<stem>_variance.exr`
    taken to an 8-bit PNG by hdrToLdr (saveToLDR), loaded by OpenCV as BGR
    and converted with COLOR_RGB2GRAY -- so the blue byte takes the red
    weight -- then divided by 255.  OpenCV's 8-bit grey conversion is fixed
    point: (4899 c0 + 9617 c1 + 1868 c2 + 2^13) >> 14.  (OpenCV is not in
    this image: this step is a restatement, unpinned.)"""
    return variance_gray_bytes(ldr_bytes(var_rgb))


def variance_gray_bytes(rgb8):
    """variance_gray() of an 8-bit RGB image as stored in a PNG (H, W, 3)."""
    bgr = np.asarray(rgb8).astype(np.int64)[..., ::-1]
    gray = (4899 * bgr[..., 0] + 9617 * bgr[..., 1] + 1868 * bgr[..., 2] + (1 << 13)) >> 14
    return (gray.astype(np.float64) / 255.0).astype(np.float32)


def denoise(img, var, radius=3, patch=3, k=0.02, mode=0, device=0, script_scale=True):
    """NL-means denoiser (denoiser/denoiser.py) on the GPU (nori_denoise).

    img: (H, W, 3) linear image; var: (H, W) per-pixel variance in the
    script's units (variance_gray()).  script_scale: divide the image by 255
    first, as the script does with its EXR input (denoiser.py:16), and return
    the result in the input's scale.  mode 0 = the script's distance (both
    variance terms 2 var(neighbour)), 1 = the textbook form."""
    img = np.ascontiguousarray(img, dtype=np.float32)
    var = np.ascontiguousarray(var, dtype=np.float32)
    if img.ndim != 3 or img.shape[2] != 3 or var.shape != img.shape[:2]:
        raise ValueError(f"image {img.shape} / variance {var.shape}: expected (H, W, 3) and (H, W)")
    src = np.ascontiguousarray(img / np.float32(255)) if script_scale else img
    out = np.empty_like(src)
    check(lib().nori_denoise(device, _fptr(src), _fptr(var), img.shape[1], img.shape[0], radius, patch, k, mode,
                             _fptr(out)))
    return out * np.float32(255) if script_scale else out


class BvhInfo(C.Structure):
    _fields_ = [("ref_nodes", C.c_uint32), ("device_nodes", C.c_uint32), ("depth", C.c_uint32),
                ("num_prims", C.c_uint32), ("sah_cost", C.c_float), ("pad", C.c_uint32), ("order_hash", C.c_uint64)]


def bvh_info(scene):
    """Host build of the scene's BVH as the GPU context builds it (nori_scene_bvh_info)."""
    info = BvhInfo()
    check(lib().nori_scene_bvh_info(scene.desc_ptr, C.byref(info)))
    return {k: getattr(info, k) for k, _ in BvhInfo._fields_ if k != "pad"}


class ScanInfo(C.Structure):
    _fields_ = [("records", C.c_uint32), ("pairs", C.c_uint32), ("plane_end", C.c_uint32 * 3), ("tris", C.c_uint32)]


def scan_list(scene):
    """The small-scene scan list as the GPU context builds it (nori_scene_scan_list): a dict with
    records (n, 12) float32, plane_c (pairs,), plane_f (pairs, 8), plane_end (3,), tris; records is
    empty for a BVH scene."""
    info = ScanInfo()
    check(lib().nori_scene_scan_list(scene.desc_ptr, C.byref(info), None, None, None))
    rec = np.zeros((info.records, 12), np.float32)
    pc = np.zeros(max(info.pairs, 1), np.float32)
    pf = np.zeros((max(info.pairs, 1), 8), np.float32)
    check(lib().nori_scene_scan_list(scene.desc_ptr, C.byref(info), _fptr(rec), _fptr(pc), _fptr(pf)))
    return {"records": rec, "plane_c": pc[:info.pairs], "plane_f": pf[:info.pairs],
            "plane_end": np.array(list(info.plane_end)), "tris": info.tris}


def scan_rtc(scene, arch="gfx950"):
    """Compile the scene's scan kernels specialised for its scan list for `arch` (the hipRTC program
    GpuRenderer loads for scan-mode scenes; no device needed): (code object bytes, milliseconds);
    (0, 0.0) for a BVH scene."""
    n, ms = C.c_size_t(), C.c_double()
    check(lib().nori_scene_scan_rtc(scene.desc_ptr, arch.encode(), C.byref(n), C.byref(ms)))
    return n.value, ms.value


def read_exr(path):
    """R, G, B planes of an OpenEXR file as a (height, width, 3) float32 array (nori_read_exr)."""
    w, h = C.c_int(), C.c_int()
    check(lib().nori_read_exr(os.fsencode(path), C.byref(w), C.byref(h), None))
    out = np.zeros((h.value, w.value, 3), np.float32)
    check(lib().nori_read_exr(os.fsencode(path), C.byref(w), C.byref(h), _fptr(out)))
    return out


def read_image(path):
    """An image texture file decoded like the reference's stbi_load(.., STBI_rgb): (height, width, 3) uint8
    (nori_read_image; baseline JPEG or 8-bit PNG)."""
    w, h = C.c_int(), C.c_int()
    check(lib().nori_read_image(os.fsencode(path), C.byref(w), C.byref(h), None))
    out = np.zeros((h.value, w.value, 3), np.uint8)
    check(lib().nori_read_image(os.fsencode(path), C.byref(w), C.byref(h),
                                out.ctypes.data_as(C.POINTER(C.c_uint8))))
    return out


class GpuRenderer:
    """HIP context holding one scene on one device (nori_gpu_create)."""

    def __init__(self, scene, device=0):
        self.scene = scene  # keeps the host arrays alive
        h = C.c_void_p()
        check(lib().nori_gpu_create(scene.desc_ptr, int(device), C.byref(h)))
        self._h = h
        self._destroy = lib().nori_gpu_destroy  # usable in __del__ at interpreter exit
        self.device = device
        self.last_stats = None

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def render(self, passes=None, pass_begin=0, blocks=None, seed=0, out=None, path_pool=0,
               device_ptr=None, timing=False, variance=None):
        """Render passes [pass_begin, pass_begin+passes) of `blocks` (all if None).

        Returns the RGBW film (H+2b, W+2b, 4) as float32, accumulated into
        `out` when given.  With `device_ptr` (an int device address, e.g. a
        torch tensor's data_ptr()) the film is accumulated on the GPU instead.
        `variance`: an (H, W, 8) float32 array (host mode) or an int device
        address (device mode) that the per-pixel sample statistics are added
        into (see film_variance).
        """
        rd, ids = self._desc(passes, pass_begin, blocks, seed, path_pool, timing)
        if variance is not None:
            if device_ptr is not None:
                rd.variance_out = int(variance)
            else:
                assert (isinstance(variance, np.ndarray) and variance.dtype == np.float32 and variance.flags.c_contiguous
                        and variance.shape == (self.scene.height, self.scene.width, 8))
                rd.variance_out = variance.ctypes.data
        st = _abi.Stats()
        if device_ptr is not None:
            rd.output_on_device = 1
            check(lib().nori_gpu_render(self._h, C.byref(rd), C.c_void_p(int(device_ptr)), C.byref(st)))
            self.last_stats = st.as_dict()
            return None
        if out is None:
            out = np.zeros(self.scene.film_shape(), np.float32)
        assert out.dtype == np.float32 and out.flags.c_contiguous and out.shape == self.scene.film_shape()
        check(lib().nori_gpu_render(self._h, C.byref(rd), out.ctypes.data_as(C.c_void_p), C.byref(st)))
        self.last_stats = st.as_dict()
        return out

    def _desc(self, passes, pass_begin, blocks, seed, path_pool, timing):
        rd = _abi.RenderDesc()
        rd.pass_begin = int(pass_begin)
        rd.pass_count = int(self.scene.spp if passes is None else passes)
        ids = None
        if blocks is not None:
            ids = np.ascontiguousarray(np.asarray(blocks, dtype=np.uint32))
            rd.num_blocks = ids.size
            rd.block_ids = ids.ctypes.data_as(C.POINTER(C.c_uint32))
        rd.seed = int(seed)
        rd.path_pool = int(path_pool)
        rd.timing = int(bool(timing))
        return rd, ids

    def render_sharded(self, comm, device_ptr, passes=None, pass_begin=0, blocks=None, mode="passes", root=0,
                       seed=0, path_pool=0, timing=False, variance=None):
        """This rank's share of the frame into the device film at `device_ptr`
        (zeroed first), then the RCCL sum of every rank's film into root's
        (root=-1: into every rank's) -- nori_gpu_render_sharded.  A cancel or
        failure on any rank raises NoriError on every rank (no rank hangs in
        the sum).  `variance` must stay None: the library rejects per-pixel
        statistics for sharded renders (they are not summed across ranks)."""
        rd, ids = self._desc(passes, pass_begin, blocks, seed, path_pool, timing)
        if variance is not None:
            rd.variance_out = int(variance)
        st = _abi.Stats()
        check(lib().nori_gpu_render_sharded(self._h, comm.handle, C.byref(rd), _abi.SHARD_MODES[mode], int(root),
                                            C.c_void_p(int(device_ptr)), C.byref(st)))
        self.last_stats = st.as_dict()

    def trace(self, rays, any_hit=False):
        """Scene::rayIntersect on a batch: rays (n, 8) = o.xyz, mint, d.xyz, maxt."""
        rays = np.ascontiguousarray(rays, dtype=np.float32)
        n = rays.shape[0]
        hits = (_abi.Hit * n)()
        check(lib().nori_gpu_trace(self._h, _fptr(rays), n, int(bool(any_hit)), hits))
        a = np.frombuffer(hits, dtype=np.dtype([("t", "<f4"), ("prim", "<i4"), ("u", "<f4"), ("v", "<f4")]))
        return a.copy()

    def cancel(self):
        check(lib().nori_gpu_cancel(self._h))

    def progress(self):
        return lib().nori_gpu_progress(self._h)


class RenderThread:
    """Mirror of nori::RenderThread (render.h:29-52) over the GPU path."""

    def __init__(self, device=0):
        self.device = device
        self._thread = None
        self._renderer = None
        self._status = 0  # 0 idle, 1 rendering, 2 stop requested, 3 done
        self.error = None
        self.image = None
        self.variance = None

    def renderScene(self, filename, width=0, height=0, spp=0):
        """Writes <stem>.exr and <stem>_variance.exr (render.cpp:158-169, 256-276;
        the variance image is the variance of each pixel's mean, deviation D5)."""
        scene = load_scene(filename, width, height, spp)
        stem = os.path.splitext(filename)[0]

        def run():
            try:
                self._renderer = GpuRenderer(scene, self.device)
                t0 = time.time()
                print("Rendering .. ", end="", flush=True)
                stats = np.zeros((scene.height, scene.width, 8), np.float32)
                film = self._renderer.render(variance=stats)
                print(f"done. (took {1e3 * (time.time() - t0):.1f}ms)")
                self.image = develop(scene, film)
                write_exr(stem + ".exr", self.image)
                self.variance = film_variance(scene, stats)
                write_exr(stem + "_variance.exr", self.variance)
            except NoriError as e:
                self.error = e
            finally:
                if self._renderer is not None:
                    self._renderer.close()
                self._status = 3

        self._status = 1
        self._thread = threading.Thread(target=run)
        self._thread.start()

    def isBusy(self):
        if self._status == 3:
            self._thread.join()
            self._status = 0
        return self._status != 0

    def isRenderingDone(self):
        return self._status == 3

    def getProgress(self):
        r = self._renderer
        return r.progress() if (r is not None and self._status in (1, 2)) else 1.0

    def stopRendering(self):
        if self._status in (1, 2) and self._renderer is not None:
            self._status = 2
            self._renderer.cancel()
            self._thread.join()
            self._status = 0
