"""Every scene the reference ships (input/*.scn, committed under tests/scenes as byte copies) plus
a synthetic circle scene, through the drop-in path on the device vs the oracle restatement on the
same RNG streams (f3 of SURVEY.md 8(f); .scn grammar R3Scene.cpp:1462-1953, .off R3Mesh.cpp:4075+).

Each scene renders a small direct-only image and a small full-GI image (own photon maps, every
estimator on), so every loader command, light type, primitive and material combination the
reference's inputs use runs at least once on the GPU. Both must be bit-identical to the oracle's,
with equal stored photon counts: the device and the oracle share gi_math.h's transcendentals
(before r04 a one-ulp difference between ROCm's math library and glibc forked the long bounce
chains of cylinder.scn, and the stack / violin maps by a few photons)."""
import glob
import os

import numpy as np
import pytest

import libm_ref
import oracle_lib
from gpu_util import compare_exact, run_gpu, INP

pytestmark = pytest.mark.gpu

EXTRA = os.path.join(os.path.dirname(INP), "scenes_extra")
SCENES = sorted(os.path.basename(p) for p in glob.glob(os.path.join(INP, "*.scn")))
ALL = [os.path.join(INP, s) for s in SCENES] + [os.path.join(EXTRA, "circles.scn")]
FAST = ["-lt", "4", "-ss", "4", "-tt", "4", "-st", "4", "-md", "32"]


def test_all_reference_scenes_present():
    assert len(SCENES) == 38


@pytest.mark.parametrize("path", ALL, ids=os.path.basename)
def test_scene_direct_only_matches_oracle(renderer, path):
    args = [path, "/tmp/s.png", "-resolution", "32", "24", "-aa", "0", "-no_indirect",
            "-no_caustic", "-seed", "2"] + FAST
    g, gst, _ = run_gpu(renderer, args)
    o, ost = oracle_lib.render(args, 32, 24)
    assert gst["screen_rays"] == ost["screen_rays"]
    compare_exact(g, o)


@pytest.mark.parametrize("path", ALL, ids=os.path.basename)
def test_scene_full_gi_matches_oracle(renderer, path):
    args = [path, "/tmp/s.png", "-resolution", "24", "16", "-aa", "0", "-global", "3000",
            "-caustic", "3000", "-it", "4", "-seed", "4"] + FAST
    g, gst, gp = run_gpu(renderer, args)
    o, ost = oracle_lib.render(args, 24, 16)
    if gp is not None:
        for k in ("global_stored", "caustic_stored"):
            assert gp[k] == ost[k], (k, gp[k], ost[k])
    assert gst["screen_rays"] == ost["screen_rays"]
    for k in ("shadow_rays", "monte_carlo_rays", "indirect_samples", "caustic_samples"):
        assert gst[k] == ost[k], (k, gst[k], ost[k])
    compare_exact(g, o)


def test_circle_intersections_match_oracle(renderer):
    """R3Intersects(ray, R3Circle) (R3Isect.cpp:837-879; gi_device.h ray_circle): rays aimed at
    points inside, on and just outside each circle of circles.scn, from both sides."""
    path = os.path.join(EXTRA, "circles.scn")
    renderer.ReadScene(path)
    rng = np.random.default_rng(12)
    circles = [((0, 0.01, 0), (0, 1, 0), 1.0), ((-1.5, 1, -1), (1, 0, 0.3), 0.8),
               ((1.5, 1, -1), (-1, 0.2, 0.4), 0.7), ((0, 2, -2), (0, 0, 1), 0.5),
               ((0.5, 0.6, 1), (0, 1, 1), 0.3)]
    org, dirs = [], []
    for c, nrm, r in circles:
        c, nrm = np.array(c, float), np.array(nrm, float) / np.linalg.norm(nrm)
        u = np.cross(nrm, [0.3, 0.5, 0.7])
        u /= np.linalg.norm(u)
        v = np.cross(nrm, u)
        n = 1500
        ang = rng.random(n) * 2 * np.pi
        rad = r * np.concatenate([np.sqrt(rng.random(n // 3)), 1 + (rng.random(n // 3) - 0.5) * 1e-5,
                                  1.0 + rng.random(n - 2 * (n // 3)) * 0.2])
        tgt = c + (np.cos(ang) * rad)[:, None] * u + (np.sin(ang) * rad)[:, None] * v
        side = np.where(rng.random(n) < 0.5, 1.0, -1.0)[:, None]
        o = tgt + side * nrm * 2.0 + rng.normal(size=(n, 3)) * 0.5
        org.append(o)
        dirs.append(tgt - o)
    org, d = np.concatenate(org), np.concatenate(dirs)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    gh, gt, gp, gn, gm = renderer.Intersects(org, d)
    oh, ot, op, on, om = oracle_lib.intersect(path, org, d)
    assert gh.sum() > 0.5 * len(gh)
    np.testing.assert_array_equal(gh, oh)
    both = gh == 1
    np.testing.assert_allclose(gt[both], ot[both], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(gn[both], on[both], atol=1e-12)
    np.testing.assert_array_equal(gm[both], om[both])


def test_device_math_equals_oracle_math(renderer):
    """The device evaluates gi_math.h's fp64 sin / cos / tan / asin / acos / atan2 / pow (the
    functions the samplers, Fresnel / Phong terms and StorePhoton call: graphics_utils.cpp:
    95-216, photon_utils.cpp:56-60) with the same operation sequence as the oracle, so the two
    agree bit for bit on every input; both stay within libm_ref.ULP_BOUND of glibc. (Before
    r04 the device called ROCm's math library, within one ulp of glibc but not equal to it, and
    that ulp forked the long bounce chains of cylinder.scn.)"""
    import gi_amd
    for fn, (x, y) in libm_ref.cases().items():
        yy = np.zeros_like(x) if y is None else y
        dev = gi_amd.math_probe(renderer, fn, x, yy)
        np.testing.assert_array_equal(dev, oracle_lib.math(fn, x, yy), err_msg=fn)
        u = libm_ref.ulps(dev, libm_ref.glibc(fn, x, yy))
        assert u.max() <= libm_ref.ULP_BOUND[fn], (fn, float(u.max()))
