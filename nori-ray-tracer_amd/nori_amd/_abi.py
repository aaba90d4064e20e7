"""ctypes mirror of include/nori_gpu.h (ABI version 7, _abi.ABI_VERSION).

The structures below must match the C declarations field for field; the
test suite checks their sizes against the library (tests/test_abi.py).
"""
import ctypes as C
import os

ABI_VERSION = 7

NORI_OK = 0
NORI_ERR_INVALID = -1
NORI_ERR_IO = -2
NORI_ERR_PARSE = -3
NORI_ERR_UNSUPPORTED = -4
NORI_ERR_HIP = -5
NORI_ERR_CANCELLED = -6
NORI_ERR_OOM = -7

SHAPE_MESH, SHAPE_SPHERE = 0, 1
BSDF_DIFFUSE, BSDF_MIRROR, BSDF_DIELECTRIC, BSDF_MICROFACET, BSDF_DISNEY = range(5)
EMITTER_AREA, EMITTER_ENVMAP, EMITTER_POINT, EMITTER_SPOT = 0, 1, 2, 3
TEXTURE_CONSTANT, TEXTURE_CHECKERBOARD, TEXTURE_IMAGE = 0, 1, 2
WRAP_REPEAT, WRAP_CLAMP = 0, 1
CAMERA_PERSPECTIVE, CAMERA_THINLENS, CAMERA_ADVANCED = 0, 1, 2
(INTEGRATOR_PATH_MATS, INTEGRATOR_PATH_MIS, INTEGRATOR_VOLUMETRIC, INTEGRATOR_NORMALS, INTEGRATOR_AV,
 INTEGRATOR_DIRECT, INTEGRATOR_DIRECT_EMS, INTEGRATOR_DIRECT_MATS, INTEGRATOR_DIRECT_MIS,
 INTEGRATOR_PHOTONMAPPER) = range(10)
INTEGRATOR_NAMES = {0: "path_mats", 1: "path_mis", 2: "volumetric", 3: "normals", 4: "av", 5: "direct",
                    6: "direct_ems", 7: "direct_mats", 8: "direct_mis", 9: "photonmapper"}
RNG_WAVE, RNG_BLOCK = 0, 1
BLOCK_SIZE = 32
FILTER_RESOLUTION = 32


class ShapeDesc(C.Structure):
    _fields_ = [("type", C.c_int32), ("tri_offset", C.c_uint32), ("tri_count", C.c_uint32),
                ("vtx_offset", C.c_uint32), ("vtx_count", C.c_uint32), ("has_normals", C.c_int32),
                ("has_uvs", C.c_int32), ("center", C.c_float * 3), ("radius", C.c_float),
                ("bsdf", C.c_int32), ("emitter", C.c_int32), ("normal_map", C.c_int32)]


class ImageDesc(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("wrap", C.c_int32),
                ("rgb", C.POINTER(C.c_uint8))]


class BsdfDesc(C.Structure):
    _fields_ = [("type", C.c_int32), ("albedo", C.c_float * 3), ("int_ior", C.c_float),
                ("ext_ior", C.c_float), ("alpha", C.c_float), ("kd", C.c_float * 3),
                ("base_color", C.c_float * 3), ("metallic", C.c_float), ("specular", C.c_float),
                ("roughness", C.c_float), ("sheen", C.c_float), ("sheen_tint", C.c_float),
                ("specular_tint", C.c_float), ("albedo_texture", C.c_int32), ("tex_value2", C.c_float * 3),
                ("tex_delta", C.c_float * 2), ("tex_scale", C.c_float * 2), ("albedo_image", C.c_int32)]


class EmitterDesc(C.Structure):
    _fields_ = [("type", C.c_int32), ("shape", C.c_int32), ("radiance", C.c_float * 3),
                ("weight", C.c_float), ("lum_scale", C.c_float * 3), ("env_rows", C.c_int32),
                ("env_cols", C.c_int32), ("env_rgb", C.POINTER(C.c_float)),
                ("position", C.c_float * 3), ("power", C.c_float * 3), ("direction", C.c_float * 3),
                ("cos_falloff_start", C.c_float), ("cos_total_width", C.c_float)]


class CameraDesc(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("fov", C.c_float),
                ("near_clip", C.c_float), ("far_clip", C.c_float),
                ("camera_to_world", C.c_float * 16), ("sample_to_camera", C.c_float * 16),
                ("filter_type", C.c_int32), ("filter_radius", C.c_float),
                ("filter_p0", C.c_float), ("filter_p1", C.c_float),
                ("camera_type", C.c_int32), ("lens_radius", C.c_float), ("focal_distance", C.c_float),
                ("distortion", C.c_float * 2), ("chromatic", C.c_float * 3)]


class MediumDesc(C.Structure):
    _fields_ = [("present", C.c_int32), ("sigma_a", C.c_float * 3), ("sigma_s", C.c_float * 3),
                ("box_min", C.c_float * 3), ("box_max", C.c_float * 3)]


class SceneDesc(C.Structure):
    _fields_ = [("abi_version", C.c_uint32), ("num_vertices", C.c_uint32),
                ("positions", C.POINTER(C.c_float)), ("normals", C.POINTER(C.c_float)),
                ("uvs", C.POINTER(C.c_float)), ("num_triangles", C.c_uint32),
                ("indices", C.POINTER(C.c_uint32)), ("num_shapes", C.c_uint32),
                ("shapes", C.POINTER(ShapeDesc)), ("num_bsdfs", C.c_uint32),
                ("bsdfs", C.POINTER(BsdfDesc)), ("num_emitters", C.c_uint32),
                ("emitters", C.POINTER(EmitterDesc)), ("camera", CameraDesc),
                ("medium", MediumDesc), ("integrator", C.c_int32), ("sample_count", C.c_uint32),
                ("av_length", C.c_float), ("photon_count", C.c_uint32), ("photon_radius", C.c_float),
                ("num_images", C.c_uint32), ("images", C.POINTER(ImageDesc))]


class RenderDesc(C.Structure):
    _fields_ = [("pass_begin", C.c_uint32), ("pass_count", C.c_uint32), ("num_blocks", C.c_uint32),
                ("block_ids", C.POINTER(C.c_uint32)), ("seed", C.c_uint64),
                ("output_on_device", C.c_int32), ("path_pool", C.c_uint32), ("timing", C.c_int32),
                ("variance_out", C.c_void_p)]


class Stats(C.Structure):
    _fields_ = [("samples", C.c_uint64), ("invalid_samples", C.c_uint64), ("rays_closest", C.c_uint64),
                ("rays_shadow", C.c_uint64), ("rays_finish", C.c_uint64), ("iterations", C.c_uint64),
                ("scene_bytes", C.c_uint64),
                ("bvh_nodes", C.c_uint32), ("bvh_depth", C.c_uint32), ("stream_parts", C.c_uint32),
                ("path_pool", C.c_uint32), ("ms_total", C.c_double),
                ("ms_extend", C.c_double), ("ms_shadow", C.c_double), ("ms_shade", C.c_double),
                ("ms_splat", C.c_double), ("ms_finish", C.c_double),
                ("scan_rtc", C.c_uint32), ("scan_rtc_cached", C.c_uint32), ("ms_scan_rtc", C.c_double),
                ("nee_inline", C.c_uint32), ("reserved0", C.c_uint32)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class Hit(C.Structure):
    _fields_ = [("t", C.c_float), ("prim", C.c_int32), ("u", C.c_float), ("v", C.c_float)]


# exported entry points: name -> (restype, argtypes)
SIGNATURES = {
    "nori_gpu_last_error": (C.c_char_p, []),
    "nori_gpu_abi_version": (C.c_int, []),
    "nori_scene_load_xml": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    "nori_scene_get_desc": (C.POINTER(SceneDesc), [C.c_void_p]),
    "nori_scene_free": (None, [C.c_void_p]),
    "nori_film_border": (C.c_int, [C.POINTER(SceneDesc)]),
    "nori_filter_table": (C.c_int, [C.POINTER(SceneDesc), C.POINTER(C.c_float)]),
    "nori_film_develop": (C.c_int, [C.POINTER(SceneDesc), C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    "nori_write_exr": (C.c_int, [C.c_char_p, C.POINTER(C.c_float), C.c_int, C.c_int]),
    "nori_write_png": (C.c_int, [C.c_char_p, C.POINTER(C.c_float), C.c_int, C.c_int]),
    "nori_film_variance": (C.c_int, [C.POINTER(SceneDesc), C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    "nori_denoise": (C.c_int, [C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_int, C.c_int, C.c_int,
                               C.c_int, C.c_float, C.c_int, C.POINTER(C.c_float)]),
    "nori_read_exr": (C.c_int, [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_float)]),
    "nori_read_image": (C.c_int, [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_uint8)]),
    "nori_scene_bvh_info": (C.c_int, [C.c_void_p, C.c_void_p]),
    "nori_scene_scan_list": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_float),
                                       C.POINTER(C.c_float)]),
    "nori_scene_scan_rtc": (C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(C.c_size_t), C.POINTER(C.c_double)]),
    "nori_gpu_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "nori_gpu_create": (C.c_int, [C.POINTER(SceneDesc), C.c_int, C.POINTER(C.c_void_p)]),
    "nori_gpu_render": (C.c_int, [C.c_void_p, C.POINTER(RenderDesc), C.c_void_p, C.POINTER(Stats)]),
    "nori_gpu_trace": (C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.c_uint32, C.c_int, C.POINTER(Hit)]),
    "nori_gpu_cancel": (C.c_int, [C.c_void_p]),
    "nori_gpu_progress": (C.c_float, [C.c_void_p]),
    "nori_gpu_destroy": (None, [C.c_void_p]),
    "nori_gpu_comm_id": (C.c_int, [C.POINTER(C.c_ubyte)]),
    "nori_gpu_comm_create": (C.c_int, [C.POINTER(C.c_ubyte), C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    "nori_gpu_comm_rank": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "nori_gpu_comm_destroy": (None, [C.c_void_p]),
    "nori_gpu_comm_library": (C.c_char_p, []),
    "nori_gpu_shard_desc": (C.c_int, [C.POINTER(SceneDesc), C.POINTER(RenderDesc), C.c_int, C.c_int, C.c_int,
                                      C.POINTER(RenderDesc), C.POINTER(C.c_uint32)]),
    "nori_gpu_render_sharded": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(RenderDesc), C.c_int, C.c_int,
                                          C.c_void_p, C.POINTER(Stats)]),
    "nori_gpu_comm_status_word": (C.c_int, [C.c_int, C.c_int]),
    "nori_gpu_comm_timeout": (C.c_double, [C.c_int, C.c_double, C.c_double, C.c_double]),
}

COMM_ID_BYTES = 128
SHARD_PASSES, SHARD_BLOCKS = 0, 1
SHARD_MODES = {"passes": SHARD_PASSES, "blocks": SHARD_BLOCKS}

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# NORI_GPU_LIB: another in-tree build of the library (tuning variants under lib/)
LIB_PATH = os.environ.get("NORI_GPU_LIB") or os.path.join(PKG_DIR, "lib", "libnori_gpu.so")

_lib = None


def _one_hip_runtime():
    """Make libnori_gpu share the process's single HIP runtime with PyTorch.

    PyTorch-ROCm ships its own libamdhip64 / libhsa-runtime64 (torch/lib,
    found through its $ORIGIN rpath by file name), while libnori_gpu needs
    them by SONAME (libamdhip64.so.7), which the loader resolves to /opt/rocm.
    Loaded in that order a process maps TWO HIP runtimes, and whichever
    initialises second sees no device ("No HIP GPUs are available").  So when
    torch is installed, its runtime is mapped first (RTLD_GLOBAL): libnori_gpu's
    SONAME dependency then binds to it, and a later `import torch` finds the
    same files already mapped.  NORI_HIP_RUNTIME=system keeps /opt/rocm's."""
    if os.environ.get("NORI_HIP_RUNTIME", "") == "system":
        return
    import importlib.util

    spec = importlib.util.find_spec("torch")  # locates torch without importing it
    if spec is None or not spec.origin:
        return
    tlib = os.path.join(os.path.dirname(spec.origin), "lib")
    for name in ("libhsa-runtime64.so", "libamdhip64.so"):
        path = os.path.join(tlib, name)
        if os.path.exists(path):
            C.CDLL(path, mode=os.RTLD_NOW | os.RTLD_GLOBAL)


def lib():
    """Load libnori_gpu.so from the package tree; fail loudly if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libnori_gpu.so not built: {LIB_PATH} (run __graft_entry__.build())")
        _one_hip_runtime()
        l = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        if l.nori_gpu_abi_version() != ABI_VERSION:
            raise RuntimeError("libnori_gpu ABI version mismatch")
        _lib = l
    return _lib


class NoriError(RuntimeError):
    """NoriException (common.h:150-155) surfaced from an int status code."""

    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def check(code):
    if code != NORI_OK:
        raise NoriError(code, lib().nori_gpu_last_error().decode(errors="replace"))
    return code
