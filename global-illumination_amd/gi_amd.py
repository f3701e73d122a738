"""Python mirror of the reference's renderer interface over the C-ABI of include/gi.h.

Names follow the reference (ReillyBova/Global-Illumination, src/):
  ParseArgs        utils/io_utils.cpp:16-212
  ReadScene        utils/io_utils.cpp:219-250
  MapPhotons       photonmap.cpp:260-436
  RenderImage      render.cpp:155-259
  EstimateRadiance utils/photon_utils.cpp:72-162      (batched test seam)
  FindClosestQuick R3Shapes/R3Kdtree.cpp:688-848      (batched test seam)
  Intersects       R3Graphics/R3Scene.cpp:471-479     (batched test seam)

The shared library libgi_amd.so (HIP, gfx950) is loaded from this directory; there is no CPU
fallback: if the library or a GPU is missing every entry point raises.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GI_AMD_LIB") or os.path.join(_HERE, "libgi_amd.so")  # GI_AMD_LIB: experiment builds

GI_OK, GI_ERR_ARG, GI_ERR_IO, GI_ERR_HIP, GI_ERR_STATE, GI_ERR_UNSUPPORTED, GI_ERR_ALLOC = range(7)
DISK, CONE, GAUSS = 0, 1, 2
GLOBAL, CAUSTIC = 0, 1

EXPORTED = [
    "gi_params_default", "gi_parse_args", "gi_create", "gi_create_devices", "gi_device_info",
    "gi_destroy", "gi_last_error",
    "gi_set_params", "gi_read_scene", "gi_scene_info", "gi_map_photons", "gi_set_photon_map",
    "gi_get_photon_map", "gi_get_kd_tree", "gi_set_progress", "gi_render_image", "gi_render_tiles",
    "gi_render_tiles_packed", "gi_compose_tiles", "gi_quantize",
    "gi_estimate_radiance_batch", "gi_knn_batch", "gi_knn_bench", "gi_intersect_batch",
    "gi_math_probe", "gi_release_scratch",
    "gi_write_image",
]


class GiParams(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "verbose", "threads", "fresnel", "ambient", "direct_illum", "transmissive_illum",
        "specular_illum", "indirect_illum", "caustic_illum", "direct_photon_illum", "fast_global",
        "irradiance_cache", "shadows", "soft_shadows", "light_test", "shadow_test", "monte_carlo",
        "max_monte_depth", "recursive_shadows", "distrib_transmissive", "transmissive_test",
        "distrib_specular", "specular_test", "depth_of_field", "dof_test", "global_photon_count",
        "caustic_photon_count", "max_photon_depth", "indirect_test", "global_estimate_size",
        "global_filter", "caustic_estimate_size", "caustic_filter", "gpus")] + [
        (n, C.c_double) for n in (
            "ir_air", "prob_absorb", "focus_depth", "aperture_radius", "global_estimate_dist",
            "caustic_estimate_dist", "filter_const_a", "filter_const_b", "filter_const_k")] + [
        ("seed", C.c_uint64)]


PHOTON_DTYPE = np.dtype([("pos", "<f4", 3), ("rgbe", "u1", 4), ("dir", "<u2"), ("flags", "<u2")])
assert PHOTON_DTYPE.itemsize == 20

QUERY_DTYPE = np.dtype([
    ("point", "<f8", 3), ("normal", "<f8", 3), ("exact_bounce", "<f8", 3), ("cos_theta", "<f8"),
    ("kd", "<f8", 3), ("ks", "<f8", 3), ("shininess", "<f8"), ("max_dist", "<f8"),
    ("k", "<i4"), ("filter", "<i4")])


GI_MAX_DEVICES = 64


class DeviceSet(C.Structure):
    _fields_ = [("count", C.c_int32), ("devices", C.c_int32 * GI_MAX_DEVICES)]


class PhotonStats(C.Structure):
    _fields_ = [("global_stored", C.c_int64), ("caustic_stored", C.c_int64),
                ("global_emitted", C.c_int64), ("caustic_emitted", C.c_int64),
                ("total_s", C.c_double), ("trace_s", C.c_double), ("kd_s", C.c_double),
                ("irradiance_s", C.c_double)]


class RenderStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "screen_rays", "shadow_rays", "monte_carlo_rays", "transmissive_samples",
        "specular_samples", "indirect_samples", "caustic_samples", "knn_queries",
        "knn_photons", "knn_visited")] + [("render_s", C.c_double), ("knn_kernel_ms", C.c_double),
                           ("knn_kernel_launches", C.c_double)] + [
        ("knn_map_queries", C.c_uint64 * 2), ("knn_map_photons", C.c_uint64 * 2),
        ("knn_map_visited", C.c_uint64 * 2), ("knn_map_kernel_ms", C.c_double * 2),
        ("knn_map_launches", C.c_double * 2), ("knn_map_fallback_ms", C.c_double * 2),
        ("knn_map_fallback_queries", C.c_uint64 * 2), ("knn_map_kind", C.c_int32 * 2),
        ("knn_map_pass2_ms", C.c_double * 2), ("knn_map_pass2_queries", C.c_uint64 * 2),
        ("device_render_s_max", C.c_double), ("device_render_s_min", C.c_double),
        ("gather_s", C.c_double)]


def _stats_dict(st):
    out = {}
    for f, _ in type(st)._fields_:
        v = getattr(st, f)
        out[f] = list(v) if isinstance(v, C.Array) else v
    return out


_lib = None


def lib():
    """Load libgi_amd.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C global-illumination_amd`")
        # One HIP runtime per process: torch ships its own libamdhip64 (soname libamdhip64.so.7,
        # but its libraries NEED it under the unversioned name), so a process that loads this
        # library first and torch later ends up with two runtimes, and torch then sees no GPU.
        # When torch is importable it is loaded first and the library binds to its runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        L.gi_params_default.argtypes = [P(GiParams)]
        L.gi_parse_args.argtypes = [C.c_int, P(C.c_char_p), P(GiParams), P(C.c_char_p),
                                    P(C.c_char_p), P(C.c_int), P(C.c_int), P(C.c_int),
                                    P(C.c_int), P(C.c_char_p)]
        L.gi_create.argtypes = [P(C.c_void_p), C.c_int]
        L.gi_create_devices.argtypes = [P(C.c_void_p), P(DeviceSet)]
        L.gi_device_info.argtypes = [C.c_void_p, C.c_int, P(C.c_int), C.c_void_p, C.c_void_p,
                                     C.c_void_p, P(C.c_int)]
        L.gi_destroy.argtypes = [C.c_void_p]
        L.gi_destroy.restype = None
        L.gi_last_error.argtypes = [C.c_void_p]
        L.gi_last_error.restype = C.c_char_p
        L.gi_set_params.argtypes = [C.c_void_p, P(GiParams)]
        L.gi_read_scene.argtypes = [C.c_void_p, C.c_char_p, C.c_int]
        L.gi_scene_info.argtypes = [C.c_void_p, P(C.c_int), P(C.c_int), P(C.c_int),
                                    P(C.c_double)]
        L.gi_map_photons.argtypes = [C.c_void_p, P(PhotonStats)]
        L.gi_set_photon_map.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int64]
        L.gi_get_photon_map.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int64,
                                        P(C.c_int64)]
        L.gi_get_kd_tree.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int64, C.c_void_p,
                                     C.c_int64, P(C.c_int32), P(C.c_int64)]
        L.gi_render_image.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                      C.c_void_p, P(RenderStats)]
        L.gi_render_tiles.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                      C.c_int, C.c_void_p, P(RenderStats)]
        L.gi_render_tiles_packed.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                             C.c_int, C.c_int, C.c_void_p, C.c_int64,
                                             P(C.c_int64), P(RenderStats)]
        L.gi_compose_tiles.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                       C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
        L.gi_quantize.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.gi_estimate_radiance_batch.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_void_p,
                                                 C.c_void_p, C.c_void_p, C.c_void_p]
        L.gi_knn_batch.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_int,
                                   C.c_double, C.c_void_p, C.c_void_p, C.c_void_p]
        L.gi_knn_bench.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_void_p,
                                   C.c_void_p, C.c_int, C.c_int, C.c_int, P(C.c_double),
                                   P(C.c_double), P(C.c_double)]
        L.gi_release_scratch.argtypes = [C.c_void_p]
        L.gi_math_probe.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_void_p,
                                    C.c_void_p]
        L.gi_intersect_batch.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_void_p]
        L.gi_write_image.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_void_p]
        _lib = L
    return _lib


def default_params():
    p = GiParams()
    lib().gi_params_default(C.byref(p))
    return p


def ParseArgs(argv):
    """Return (params, scene, output, width, height, aa, real_material); raises ValueError with
    the reference's message on a bad flag (io_utils.cpp:186-188)."""
    p = default_params()
    args = ["photonmap"] + list(argv)
    arr = (C.c_char_p * len(args))(*[a.encode() for a in args])
    scene, out, err = C.c_char_p(), C.c_char_p(), C.c_char_p()
    w, h, aa, real = C.c_int(1024), C.c_int(1024), C.c_int(2), C.c_int(0)
    rc = lib().gi_parse_args(len(args), arr, C.byref(p), C.byref(scene), C.byref(out),
                             C.byref(w), C.byref(h), C.byref(aa), C.byref(real), C.byref(err))
    if rc != GI_OK:
        raise ValueError(err.value.decode() if err.value else f"gi_parse_args rc={rc}")
    return p, scene.value.decode(), out.value.decode(), w.value, h.value, aa.value, real.value


class GiError(RuntimeError):
    pass


class Renderer:
    """One context: scene, photon maps and render scratch on one HIP device, or on a device
    set (`devices=[...]`, gi_create_devices: tiles dealt across the devices, gathered onto the
    first)."""

    def __init__(self, device=0, params=None, devices=None):
        self._ctx = C.c_void_p()
        if devices is not None:
            ds = DeviceSet()
            ds.count = len(devices)
            for i, d in enumerate(devices):
                ds.devices[i] = d
            rc = lib().gi_create_devices(C.byref(self._ctx), C.byref(ds))
            if rc != GI_OK:
                raise GiError(f"gi_create_devices failed (rc={rc}) for devices {list(devices)}")
        else:
            rc = lib().gi_create(C.byref(self._ctx), device)
            if rc != GI_OK:
                raise GiError(f"gi_create failed (rc={rc}): no usable HIP device {device}")
        self.params = params if params is not None else default_params()
        self._check(lib().gi_set_params(self._ctx, C.byref(self.params)))

    def device_info(self):
        """What the context drives (gi_device_info): HIP ordinals, PCI bus ids, RCCL user rank
        per device, and the RCCL communicator's rank count (0 without RCCL)."""
        n = C.c_int(0)
        self._check(lib().gi_device_info(self._ctx, 0, C.byref(n), None, None, None, None))
        k = n.value
        dev, bus, rk = (C.c_int * k)(), (C.c_int * k)(), (C.c_int * k)()
        cc = C.c_int(0)
        self._check(lib().gi_device_info(self._ctx, k, C.byref(n), dev, bus, rk, C.byref(cc)))
        return {"devices": list(dev), "pci_bus": list(bus), "comm_rank": list(rk),
                "comm_count": cc.value}

    def release_scratch(self):
        """Free the device scratch of renders and map builds; scene and maps stay resident."""
        self._check(lib().gi_release_scratch(self._ctx))

    def close(self):
        if self._ctx:
            lib().gi_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != GI_OK:
            msg = lib().gi_last_error(self._ctx)
            raise GiError(f"rc={rc}: {msg.decode() if msg else ''}")

    def set_params(self, params):
        self.params = params
        self._check(lib().gi_set_params(self._ctx, C.byref(params)))

    def ReadScene(self, path, real_material=False):
        self._check(lib().gi_read_scene(self._ctx, path.encode(), int(real_material)))
        nn, nl, npr, r = C.c_int(), C.c_int(), C.c_int(), C.c_double()
        self._check(lib().gi_scene_info(self._ctx, C.byref(nn), C.byref(nl), C.byref(npr),
                                        C.byref(r)))
        return {"nodes": nn.value, "lights": nl.value, "shapes": npr.value, "radius": r.value}

    def MapPhotons(self):
        st = PhotonStats()
        self._check(lib().gi_map_photons(self._ctx, C.byref(st)))
        return {f: getattr(st, f) for f, _ in PhotonStats._fields_}

    def photon_map(self, which):
        n = C.c_int64()
        self._check(lib().gi_get_photon_map(self._ctx, which, None, 0, C.byref(n)))
        out = np.zeros(n.value, dtype=PHOTON_DTYPE)
        self._check(lib().gi_get_photon_map(self._ctx, which, out.ctypes.data, n.value,
                                            C.byref(n)))
        return out

    def kd_tree(self, which):
        """(nodes [2L, 8] float32, perm [n] int32 kd position -> emission index, nleaves)"""
        nl, n = C.c_int32(), C.c_int64()
        self._check(lib().gi_get_kd_tree(self._ctx, which, None, 0, None, 0, C.byref(nl), C.byref(n)))
        nodes = np.zeros((2 * nl.value, 8), dtype=np.float32)
        perm = np.zeros(n.value, dtype=np.int32)
        self._check(lib().gi_get_kd_tree(self._ctx, which, nodes.ctypes.data, nodes.size,
                                         perm.ctypes.data, n.value, C.byref(nl), C.byref(n)))
        return nodes, perm, nl.value

    def set_photon_map(self, which, photons):
        photons = np.ascontiguousarray(photons, dtype=PHOTON_DTYPE)
        self._check(lib().gi_set_photon_map(self._ctx, which, photons.ctypes.data, len(photons)))

    def RenderImage(self, aa, width, height, want_float=False):
        rgb = np.zeros((height, width, 3), dtype=np.uint8)
        rgbf = np.zeros((height, width, 3), dtype=np.float32) if want_float else None
        st = RenderStats()
        self._check(lib().gi_render_image(self._ctx, aa, width, height, rgb.ctypes.data,
                                          rgbf.ctypes.data if want_float else None,
                                          C.byref(st)))
        stats = _stats_dict(st)
        return (rgb, rgbf, stats) if want_float else (rgb, stats)

    def render_tiles(self, aa, width, height, tile, shard, nshards, rgbf=None):
        if rgbf is None:
            rgbf = np.zeros((height, width, 3), dtype=np.float32)
        st = RenderStats()
        self._check(lib().gi_render_tiles(self._ctx, aa, width, height, tile, shard, nshards,
                                          rgbf.ctypes.data, C.byref(st)))
        return rgbf, _stats_dict(st)

    def shard_pixels(self, width, height, tile, shard, nshards):
        """Pixels of one tile shard (gi_render_tiles_packed with a null buffer)."""
        n = C.c_int64(0)
        self._check(lib().gi_render_tiles_packed(self._ctx, 0, width, height, tile, shard,
                                                 nshards, None, 0, C.byref(n), None))
        return n.value

    def render_tiles_packed(self, aa, width, height, tile, shard, nshards, dev_ptr, capacity):
        """Render a tile shard into a device buffer (`dev_ptr`, 16 B per pixel, e.g. the
        data_ptr() of a CUDA tensor on this context's device). Returns (pixels, stats)."""
        n = C.c_int64(0)
        st = RenderStats()
        self._check(lib().gi_render_tiles_packed(self._ctx, aa, width, height, tile, shard,
                                                 nshards, C.c_void_p(dev_ptr), capacity,
                                                 C.byref(n), C.byref(st)))
        return n.value, _stats_dict(st)

    def compose_tiles(self, width, height, tile, nshards, dev_ptr, stride, want_float=False):
        """Full frame from nshards packed shard buffers at dev_ptr (device, stride pixels
        apart). Returns rgb8 [, rgbf]."""
        rgb = np.zeros((height, width, 3), dtype=np.uint8)
        rgbf = np.zeros((height, width, 3), dtype=np.float32) if want_float else None
        self._check(lib().gi_compose_tiles(self._ctx, width, height, tile, nshards,
                                           C.c_void_p(dev_ptr), stride, rgb.ctypes.data,
                                           rgbf.ctypes.data if want_float else None))
        return (rgb, rgbf) if want_float else rgb

    def EstimateRadiance(self, which, queries):
        q = np.ascontiguousarray(queries, dtype=QUERY_DTYPE)
        n = len(q)
        out = np.zeros((n, 3), dtype=np.float64)
        nf = np.zeros(n, dtype=np.int32)
        md = np.zeros(n, dtype=np.float32)
        self._check(lib().gi_estimate_radiance_batch(self._ctx, which, n, q.ctypes.data,
                                                     out.ctypes.data, nf.ctypes.data,
                                                     md.ctypes.data))
        return out, nf, md

    def FindClosestQuick(self, which, points, k, max_dist):
        pts = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 3)
        n = len(pts)
        idx = np.zeros((n, k), dtype=np.int32)
        d2 = np.zeros((n, k), dtype=np.float32)
        nf = np.zeros(n, dtype=np.int32)
        self._check(lib().gi_knn_batch(self._ctx, which, n, pts.ctypes.data, k, max_dist,
                                       idx.ctypes.data, d2.ctypes.data, nf.ctypes.data))
        return idx, d2, nf

    def knn_bench(self, which, points, normals=None, materials=None, mode=0, kernel=-1,
                  iters=3):
        """Time the k-NN estimate kernel on resident queries (diagnostics; gi_knn_bench)."""
        pts = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 3)
        nrm = None if normals is None else np.ascontiguousarray(normals, dtype=np.float64)
        mat = None if materials is None else np.ascontiguousarray(materials, dtype=np.int32)
        ms, fq, vq = C.c_double(), C.c_double(), C.c_double()
        self._check(lib().gi_knn_bench(
            self._ctx, which, len(pts), pts.ctypes.data,
            None if nrm is None else nrm.ctypes.data, None if mat is None else mat.ctypes.data,
            mode, kernel, iters, C.byref(ms), C.byref(fq), C.byref(vq)))
        return ms.value, fq.value, vq.value

    def Intersects(self, org, dirs):
        org = np.ascontiguousarray(org, dtype=np.float64).reshape(-1, 3)
        dirs = np.ascontiguousarray(dirs, dtype=np.float64).reshape(-1, 3)
        n = len(org)
        hit = np.zeros(n, dtype=np.int32)
        t = np.zeros(n, dtype=np.float64)
        p = np.zeros((n, 3), dtype=np.float64)
        nr = np.zeros((n, 3), dtype=np.float64)
        m = np.zeros(n, dtype=np.int32)
        self._check(lib().gi_intersect_batch(self._ctx, n, org.ctypes.data, dirs.ctypes.data,
                                             hit.ctypes.data, t.ctypes.data, p.ctypes.data,
                                             nr.ctypes.data, m.ctypes.data))
        return hit, t, p, nr, m


MATH_FNS = {"acos": 0, "sin": 1, "cos": 2, "pow": 3, "atan2": 4, "sqrt": 5, "tan": 6, "asin": 7}


def math_probe(renderer, fn, x, y=None):
    """The device's fp64 acos / sin / cos / pow / atan2 / sqrt of host inputs (gi_math_probe)."""
    x = np.ascontiguousarray(x, dtype=np.float64).ravel()
    y = np.ascontiguousarray(np.zeros_like(x) if y is None else y, dtype=np.float64).ravel()
    out = np.zeros_like(x)
    renderer._check(lib().gi_math_probe(renderer._ctx, MATH_FNS[fn], len(x), x.ctypes.data,
                                        y.ctypes.data, out.ctypes.data))
    return out


def write_image(path, rgb):
    """rgb: uint8 [H, W, 3] with row 0 = image row y=0 (bottom), like R2Image."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    h, w, _ = rgb.shape
    rc = lib().gi_write_image(path.encode(), w, h, rgb.ctypes.data)
    if rc != GI_OK:
        raise GiError(f"gi_write_image({path}) rc={rc}")
