"""ctypes binding of oracle/liboracle.so -- the CPU restatement used ONLY as the checker in
tests (and bench.py's cpu_baseline leg). Never imported by the product."""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(ORACLE_DIR, "liboracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-C", ORACLE_DIR, "-s"])
        L = C.CDLL(path)
        L.oracle_run.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.c_void_p, C.c_int64,
                                 C.c_void_p, C.c_int]
        L.oracle_map_photons.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.c_void_p, C.c_int64,
                                         C.POINTER(C.c_int64), C.c_void_p, C.c_int64,
                                         C.POINTER(C.c_int64), C.c_void_p]
        L.oracle_estimate_radiance.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64,
                                               C.c_double, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_knn.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int,
                                 C.c_double, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_intersect.argtypes = [C.c_char_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_rgbe_encode.argtypes = [C.c_void_p, C.c_void_p]
        L.oracle_rgbe_decode.argtypes = [C.c_void_p, C.c_void_p]
        L.oracle_direction_lut.argtypes = [C.c_void_p]
        L.oracle_math.argtypes = [C.c_int, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_parse_args.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.c_void_p,
                                        C.POINTER(C.c_int), C.POINTER(C.c_int),
                                        C.POINTER(C.c_int), C.POINTER(C.c_int)]
        _lib = L
    return _lib


def _argv(args):
    a = ["oracle"] + list(args)
    return len(a), (C.c_char_p * len(a))(*[x.encode() for x in a])


def render(args, width, height):
    """Run the oracle pipeline; returns (rgb uint8 [H,W,3] row 0 = bottom, stats dict)."""
    n, argv = _argv(args)
    rgb = np.zeros((height, width, 3), dtype=np.uint8)
    st = np.zeros(16, dtype=np.float64)
    rc = lib().oracle_run(n, argv, rgb.ctypes.data, rgb.size, st.ctypes.data, 0)
    assert rc == 0, rc
    keys = ["trace_s", "kd_s", "render_s", "global_stored", "caustic_stored", "screen_rays",
            "shadow_rays", "monte_carlo_rays", "transmissive_samples", "specular_samples",
            "indirect_samples", "caustic_samples", "knn_queries", "knn_photons", "w", "h"]
    return rgb, dict(zip(keys, st.tolist()))


def map_photons(args, cap=1 << 23):
    from gi_amd import PHOTON_DTYPE
    n, argv = _argv(args)
    g = np.zeros(cap, dtype=PHOTON_DTYPE)
    c = np.zeros(cap, dtype=PHOTON_DTYPE)
    gn, cn = C.c_int64(), C.c_int64()
    em = np.zeros(2, dtype=np.int64)
    rc = lib().oracle_map_photons(n, argv, g.ctypes.data, cap, C.byref(gn), c.ctypes.data, cap,
                                  C.byref(cn), em.ctypes.data)
    assert rc == 0, rc
    return g[:gn.value].copy(), c[:cn.value].copy(), em


def estimate_radiance(photons, queries, filter_k=1.0):
    from gi_amd import PHOTON_DTYPE, QUERY_DTYPE
    ph = np.ascontiguousarray(photons, dtype=PHOTON_DTYPE)
    q = np.ascontiguousarray(queries, dtype=QUERY_DTYPE)
    out = np.zeros((len(q), 3))
    nf = np.zeros(len(q), dtype=np.int32)
    md = np.zeros(len(q), dtype=np.float32)
    lib().oracle_estimate_radiance(ph.ctypes.data, len(ph), q.ctypes.data, len(q), filter_k,
                                   out.ctypes.data, nf.ctypes.data, md.ctypes.data)
    return out, nf, md


def knn(photons, points, k, max_dist):
    from gi_amd import PHOTON_DTYPE
    ph = np.ascontiguousarray(photons, dtype=PHOTON_DTYPE)
    pts = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 3)
    idx = np.zeros((len(pts), k), dtype=np.int32)
    d2 = np.zeros((len(pts), k), dtype=np.float32)
    nf = np.zeros(len(pts), dtype=np.int32)
    lib().oracle_knn(ph.ctypes.data, len(ph), pts.ctypes.data, len(pts), k, max_dist,
                     idx.ctypes.data, d2.ctypes.data, nf.ctypes.data)
    return idx, d2, nf


def intersect(scene, org, dirs):
    org = np.ascontiguousarray(org, dtype=np.float64).reshape(-1, 3)
    dirs = np.ascontiguousarray(dirs, dtype=np.float64).reshape(-1, 3)
    n = len(org)
    hit = np.zeros(n, dtype=np.int32)
    t = np.zeros(n)
    p = np.zeros((n, 3))
    nr = np.zeros((n, 3))
    m = np.zeros(n, dtype=np.int32)
    rc = lib().oracle_intersect(scene.encode(), n, org.ctypes.data, dirs.ctypes.data,
                                hit.ctypes.data, t.ctypes.data, p.ctypes.data, nr.ctypes.data,
                                m.ctypes.data)
    assert rc == 0
    return hit, t, p, nr, m


def parse_args(args):
    from gi_amd import GiParams
    n, argv = _argv(args)
    p = GiParams()
    w, h, aa, real = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    rc = lib().oracle_parse_args(n, argv, C.byref(p), C.byref(w), C.byref(h), C.byref(aa),
                                 C.byref(real))
    return rc, p, w.value, h.value, aa.value, real.value


def rgbe_encode(rgb):
    out = np.zeros(4, dtype=np.uint8)
    v = np.ascontiguousarray(rgb, dtype=np.float64)
    lib().oracle_rgbe_encode(v.ctypes.data, out.ctypes.data)
    return out


def rgbe_decode(b):
    v = np.ascontiguousarray(b, dtype=np.uint8)
    out = np.zeros(3)
    lib().oracle_rgbe_decode(v.ctypes.data, out.ctypes.data)
    return out


def direction_lut():
    out = np.zeros((65536, 3))
    lib().oracle_direction_lut(out.ctypes.data)
    return out


MATH_FNS = {"acos": 0, "sin": 1, "cos": 2, "pow": 3, "atan2": 4, "sqrt": 5, "tan": 6, "asin": 7}


def math(fn, x, y=None):
    """gi_math.h's fp64 function `fn` on the host (the oracle's, and the device's, sequence)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.zeros_like(x) if y is None else np.ascontiguousarray(y, dtype=np.float64)
    out = np.empty_like(x)
    rc = lib().oracle_math(MATH_FNS[fn], len(x), x.ctypes.data, y.ctypes.data, out.ctypes.data)
    assert rc == 0
    return out


def set_diag(mc_class=-1, window=None, flags=0):
    """Diagnostic switches of the restatement (oracle_set_diag / oracle_set_diag_flags; DESIGN.md
    6.2): keep only Monte Carlo contributions of one path class (-1 = all), render only the
    output-pixel window (x0, y0, x1, y1; row 0 = bottom; None = whole image), flags bit 0 = no
    Fresnel split inside MonteCarlo_PathTrace. Hypothesis tests only: every parity test runs
    with the defaults, which are restored by set_diag()."""
    L = lib()
    L.oracle_set_diag.argtypes = [C.c_int] * 5
    L.oracle_set_diag_flags.argtypes = [C.c_int]
    L.oracle_set_diag(mc_class, *(window or (0, 0, 0, 0)))
    L.oracle_set_diag_flags(flags)


def render_float(args, width, height):
    """One render (no photon map unless the flags need one) returning the box-filtered clamped
    float image [H, W, 3] (row 0 = bottom) and the 8-bit one."""
    L = lib()
    L.oracle_run_tags.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.c_void_p, C.c_int,
                                  C.c_void_p, C.c_void_p, C.c_int64]
    n, argv = _argv(args)
    tags = (C.c_int * 1)(-100)
    f = np.zeros((height, width, 3), np.float32)
    rgb = np.zeros((height, width, 3), np.uint8)
    rc = L.oracle_run_tags(n, argv, tags, 1, f.ctypes.data, rgb.ctypes.data, width * height)
    assert rc == 0, rc
    return f, rgb
