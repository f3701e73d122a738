"""gi_math.h, the fp64 sin / cos / tan / asin / acos / atan2 / pow that the device kernels and the
oracle restatement share (tools/gen_gi_math.py), on the host: accuracy against the C library on
the renderer's argument ranges, and the special values the call sites reach.

Sharing one operation sequence makes the device and the oracle agree bit for bit
(tests/test_gpu_scenes.py::test_device_math_equals_oracle_math); the reference itself calls the
C library, so this file bounds how far the shared sequence is from it."""
import numpy as np
import pytest

import libm_ref
import oracle_lib


@pytest.mark.parametrize("fn", ["acos", "asin", "sin", "cos", "tan", "atan2", "pow", "sqrt"])
def test_gi_math_within_bound_of_glibc(fn):
    x, y = libm_ref.cases()[fn]
    ours = oracle_lib.math(fn, x, y)
    ref = libm_ref.glibc(fn, x, np.zeros_like(x) if y is None else y)
    u = libm_ref.ulps(ours, ref)
    print(f"\n{fn}: max {u.max():.2f} ulp, {np.mean(ours != ref):.3f} of results differ from glibc")
    assert u.max() <= libm_ref.ULP_BOUND[fn], (fn, float(u.max()))


def test_gi_math_special_values():
    m = oracle_lib.math
    pi = np.pi
    assert m("acos", [1.0, -1.0, 0.0]).tolist() == [0.0, pi, pi / 2]
    assert m("asin", [1.0, -1.0, 0.0, -0.0]).tolist() == [pi / 2, -pi / 2, 0.0, -0.0]
    assert np.isnan(m("acos", [1.0000000000000002])[0]) and np.isnan(m("asin", [-1.5])[0])
    at = m("atan2", [0.0, -0.0, 0.0, -0.0, 1.0, -1.0], [0.0, 0.0, -0.0, -0.0, 0.0, -0.0])
    assert at.tolist() == [0.0, -0.0, pi, -pi, pi / 2, -pi / 2]
    assert np.signbit(at[1])
    assert m("atan2", [0.0, -0.0], [-1.0, -1.0]).tolist() == [pi, -pi]
    p = m("pow", [0.0, 2.0, 1.0, -2.0, -2.0, -0.5, 0.3, 0.999],
          [2.0, 0.0, 1e300, 3.0, 2.0, 5.0, 5000.0, 5000.0])
    assert p[:6].tolist() == [0.0, 1.0, 1.0, -8.0, 4.0, -0.03125]
    assert p[6] == 0.0 and abs(p[7] / 0.0067211119598655882 - 1) < 1e-15
    assert np.isnan(m("pow", [-2.0], [0.5])[0])
    # signed zero and infinite operands, as glibc's pow (C99 F.9.4.4): -0.0 reaches
    # pow through EstimateRadiance's clamp `if (ca < 0) ca = 0`
    xs = [-0.0, -0.0, -0.0, -0.0, 0.0, -np.inf, -np.inf, -np.inf, -1.0, -1.0, 0.5, 2.0, -0.5]
    ys = [3.0, -3.0, 2.0, 0.5, -2.0, 3.0, 0.5, -3.0, np.inf, -np.inf, np.inf, -np.inf, -np.inf]
    got = m("pow", xs, ys)
    with np.errstate(divide="ignore"):
        want = np.power(np.array(xs), np.array(ys))
    assert got.tolist() == want.tolist() and (np.signbit(got) == np.signbit(want)).all(), got
    assert m("sin", [0.0, -0.0]).tolist() == [0.0, -0.0] and np.signbit(m("sin", [-0.0])[0])
    assert m("cos", [0.0]).tolist() == [1.0] and m("tan", [0.0]).tolist() == [0.0]
