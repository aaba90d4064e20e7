"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The oracle consumes the same flattened scene description as the
GPU path (the C ABI's nori_scene_desc), so the XML/OBJ boundary is shared and
everything after it -- BVH, sampling, integrators, film -- is restated
independently in C (oracle/nori_oracle.c).
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


class OracleStats(C.Structure):
    _fields_ = [("samples", C.c_uint64), ("invalid_samples", C.c_uint64), ("rays_closest", C.c_uint64),
                ("rays_shadow", C.c_uint64), ("bounces", C.c_uint64), ("ms_render", C.c_double),
                ("threads", C.c_int)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        l = C.CDLL(LIB_PATH)
        vp, u32, u64, f32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_float
        pf, pd = C.POINTER(C.c_float), C.POINTER(C.c_double)
        sig = {
            "oracle_scene_create": (C.c_int, [vp, C.POINTER(vp)]),
            "oracle_scene_free": (None, [vp]),
            "oracle_scene_node_count": (u32, [vp]),
            "oracle_scene_bvh_stats": (C.c_int, [vp, C.POINTER(u32), C.POINTER(C.c_float), C.POINTER(u64)]),
            "oracle_render": (C.c_int, [vp, C.c_int, u64, u32, u32, C.POINTER(u32), u32, C.c_int, C.c_int, pf,
                                        C.POINTER(OracleStats)]),
            "oracle_trace": (C.c_int, [vp, pf, u32, C.c_int, vp]),
            "oracle_wave_samples": (C.c_int, [vp, u64, C.POINTER(u64), u32, pf]),
            "oracle_pcg32_seed": (None, [C.POINTER(u64), u64, u64]),
            "oracle_pcg32_next": (u32, [C.POINTER(u64)]),
            "oracle_pcg32_next_float": (f32, [C.POINTER(u64)]),
            "oracle_scene_ttest": (C.c_int, [vp, u32, pd, pd]),
            "oracle_bsdf_ttest": (C.c_int, [vp, f32, u32, pd, pd]),
            "oracle_bsdf_sample": (C.c_int, [vp, pf, pf, u32, pf]),
            "oracle_bsdf_eval_pdf": (C.c_int, [vp, pf, pf, u32, pf]),
            "oracle_photon_map": (C.c_int, [vp, C.POINTER(u64), C.POINTER(u32), C.POINTER(pf)]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(l, name)
            fn.restype, fn.argtypes = res, args
        _lib = l
    return _lib


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


class Pcg32:
    """pcg32 (ext/pcg32/pcg32.h) through the oracle's C implementation."""

    def __init__(self, initstate=None, initseq=1):
        self.st = (C.c_uint64 * 2)(0x853c49e6748fea9b, 0xda3e39cb94b95bdb)
        if initstate is not None:
            lib().oracle_pcg32_seed(self.st, initstate, initseq)

    def next_uint(self, bound=None):
        if bound is None:
            return lib().oracle_pcg32_next(self.st)
        threshold = ((1 << 32) - bound) % bound  # pcg32.h:68-90
        while True:
            r = lib().oracle_pcg32_next(self.st)
            if r >= threshold:
                return r % bound

    def next_float(self):
        return lib().oracle_pcg32_next_float(self.st)

    def shuffle(self, items):  # pcg32.h:166-170
        items = list(items)
        for i in range(len(items) - 1, 0, -1):
            j = self.next_uint(i + 1)
            items[i], items[j] = items[j], items[i]
        return items


class OracleScene:
    """Oracle view of a scene loaded through nori_amd.load_scene (keeps it alive)."""

    def __init__(self, scene):
        self.scene = scene
        h = C.c_void_p()
        rc = lib().oracle_scene_create(C.cast(scene.desc_ptr, C.c_void_p), C.byref(h))
        if rc != 0:
            raise RuntimeError(f"oracle_scene_create failed: {rc}")
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None) is not None and _lib is not None:
            _lib.oracle_scene_free(self._h)
            self._h = None

    def render(self, passes=None, pass_begin=0, rng="wave", seed=0, blocks=None, threads=0,
               variance_pass=False, out=None):
        mode = 0 if rng == "wave" else 1
        passes = self.scene.spp if passes is None else passes
        if out is None:
            out = np.zeros(self.scene.film_shape(), np.float32)
        ids, nb = None, 0
        if blocks is not None:
            arr = np.ascontiguousarray(np.asarray(blocks, dtype=np.uint32))
            ids, nb = arr.ctypes.data_as(C.POINTER(C.c_uint32)), arr.size
            self._keep = arr
        st = OracleStats()
        rc = lib().oracle_render(self._h, mode, seed, pass_begin, passes, ids, nb, threads, int(variance_pass),
                                 _fp(out), C.byref(st))
        if rc != 0:
            raise RuntimeError(f"oracle_render failed: {rc}")
        self.last_stats = st.as_dict()
        return out

    def trace(self, rays, any_hit=False):
        rays = np.ascontiguousarray(rays, dtype=np.float32)
        n = rays.shape[0]
        out = np.zeros(n, dtype=np.dtype([("t", "<f4"), ("prim", "<i4"), ("u", "<f4"), ("v", "<f4")]))
        rc = lib().oracle_trace(self._h, _fp(rays), n, int(bool(any_hit)), out.ctypes.data_as(C.c_void_p))
        if rc != 0:
            raise RuntimeError("oracle_trace failed")
        return out

    def wave_samples(self, sample_ids, seed=0):
        ids = np.ascontiguousarray(np.asarray(sample_ids, dtype=np.uint64))
        out = np.zeros((ids.size, 5), np.float32)
        lib().oracle_wave_samples(self._h, seed, ids.ctypes.data_as(C.POINTER(C.c_uint64)), ids.size, _fp(out))
        return out

    def ttest(self, n=100000):
        m, v = C.c_double(), C.c_double()
        lib().oracle_scene_ttest(self._h, n, C.byref(m), C.byref(v))
        return m.value, v.value

    def node_count(self):
        return lib().oracle_scene_node_count(self._h)

    def photon_map(self):
        """(emitted photons, photons n x 9: position, direction, power after PhotonData)."""
        e, n, p = C.c_uint64(), C.c_uint32(), C.POINTER(C.c_float)()
        rc = lib().oracle_photon_map(self._h, C.byref(e), C.byref(n), C.byref(p))
        if rc != 0:
            raise RuntimeError(f"oracle_photon_map: {rc}")
        return e.value, np.ctypeslib.as_array(p, shape=(n.value, 9)).copy()

    def bvh_stats(self):
        """(reachable nodes, BVH::statistics SAH cost, FNV-1a hash of the leaf-order primitive ids)."""
        n, sah, h = C.c_uint32(), C.c_float(), C.c_uint64()
        rc = lib().oracle_scene_bvh_stats(self._h, C.byref(n), C.byref(sah), C.byref(h))
        if rc != 0:
            raise RuntimeError(f"oracle_scene_bvh_stats: {rc}")
        return n.value, sah.value, h.value


def bsdf_ttest(bsdf_desc, angle_deg, n=100000):
    m, v = C.c_double(), C.c_double()
    lib().oracle_bsdf_ttest(C.byref(bsdf_desc), angle_deg, n, C.byref(m), C.byref(v))
    return m.value, v.value


def bsdf_sample(bsdf_desc, wi, u2):
    wi = np.ascontiguousarray(wi, np.float32)
    u2 = np.ascontiguousarray(u2, np.float32)
    out = np.zeros((wi.shape[0], 5), np.float32)
    lib().oracle_bsdf_sample(C.byref(bsdf_desc), _fp(wi), _fp(u2), wi.shape[0], _fp(out))
    return out


def bsdf_eval_pdf(bsdf_desc, wi, wo):
    wi = np.ascontiguousarray(wi, np.float32)
    wo = np.ascontiguousarray(wo, np.float32)
    out = np.zeros((wi.shape[0], 4), np.float32)
    lib().oracle_bsdf_eval_pdf(C.byref(bsdf_desc), _fp(wi), _fp(wo), wi.shape[0], _fp(out))
    return out
