"""The host C library's fp64 functions, one ctypes call per element (the reference's <cmath>
calls on Linux), and the argument sets the renderer feeds gi_math.h's functions."""
import ctypes as C

import numpy as np

# max |gi_math - glibc| in ulps of the glibc result, measured (tests/test_cpu_math.py)
ULP_BOUND = {"sin": 1, "cos": 1, "acos": 1, "asin": 2, "tan": 2, "atan2": 2, "pow": 1, "sqrt": 0}


def glibc(fn, x, y=None):
    libm = C.CDLL("libm.so.6")
    f = getattr(libm, fn)
    two = fn in ("pow", "atan2")
    f.argtypes = [C.c_double, C.c_double] if two else [C.c_double]
    f.restype = C.c_double
    if two:
        return np.array([f(float(a), float(b)) for a, b in zip(x, y)])
    return np.array([f(float(a)) for a in x])


def cases(n=20000, seed=11):
    """{fn: (x, y)} over the argument ranges the samplers, Fresnel / Phong terms and direction
    codes use (graphics_utils.cpp:95-216, photon_utils.cpp:56-60, illumination_utils.cpp)."""
    rng = np.random.default_rng(seed)
    u, v = rng.random(n), rng.random(n)
    k = rng.integers(1, 10000, n)
    third = n // 3
    pow_x = np.concatenate([u[:third], u[third:2 * third], (2 * u[2 * third:] - 1) * 0.5])
    pow_y = np.concatenate([1.0 / (k[:third] + 1.0), v[third:2 * third] * 5000.0,
                            np.where(rng.random(n - 2 * third) < 0.5, 2.0, 5.0)])
    return {
        "acos": (2.0 * u - 1.0, None),                   # acos(cos theta), acos(z), acos(sqrt u)
        "asin": (2.0 * u - 1.0, None),                   # TransmissiveBounce's asin(sin phi)
        "sin": (np.concatenate([u[:third] * np.pi, (2 * u[third:] - 1) * 7.0]), None),
        "cos": (np.concatenate([u[:third] * 2 * np.pi, (2 * u[third:] - 1) * 7.0]), None),
        "tan": ((2.0 * u - 1.0) * 1.5, None),            # tan(phi), |phi| < pi/2
        "atan2": (2.0 * u - 1.0, 2.0 * v - 1.0),         # the direction code's atan2(y, x)
        "pow": (pow_x, pow_y),                           # u^(1/(n+1)), Phong ca^n, r0^2, (1-c)^5
        "sqrt": (u, None),
    }


def ulps(a, ref):
    """|a - ref| in ulps of ref (NaN == NaN counts as 0)."""
    a, ref = np.asarray(a), np.asarray(ref)
    both_nan = np.isnan(a) & np.isnan(ref)
    sp = np.spacing(np.abs(ref))
    d = np.where(a == ref, 0.0, np.abs(a - ref) / np.where(sp > 0, sp, 5e-324))
    return np.where(both_nan, 0.0, d)
