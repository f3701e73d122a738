"""The oracle restatement checked against what the reference itself left behind and against
independent invariants:
  * (the reference's own rendered figures pin the shading: tests/test_cpu_gallery.py);
  * RGBE codec and direction table known answers (graphics_utils.cpp:50-77,
    photon_utils.cpp:253-272);
  * the kd-tree FindClosestQuick restatement equals a brute-force k-NN."""
import os

import numpy as np
import pytest

import oracle_lib
import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
SCN = os.path.join(ROOT, "tests", "scenes")


def test_rgbe_known_answers():
    assert list(oracle_lib.rgbe_encode([1.0, 0.5, 0.25])) == [128, 64, 32, 129]
    assert list(oracle_lib.rgbe_encode([0.0, 0.0, 0.0])) == [0, 0, 0, 0]
    np.testing.assert_array_equal(oracle_lib.rgbe_decode([128, 64, 32, 129]), [1.0, 0.5, 0.25])
    np.testing.assert_array_equal(oracle_lib.rgbe_decode([9, 9, 9, 0]), [0, 0, 0])
    rng = np.random.default_rng(0)
    for _ in range(200):
        c = rng.random(3) * 10 ** rng.uniform(-6, 6)
        back = oracle_lib.rgbe_decode(oracle_lib.rgbe_encode(c))
        assert np.all(back <= c * (1 + 1e-12))
        assert np.all(c - back <= c.max() / 128 + 1e-300)


def test_direction_lut():
    lut = oracle_lib.direction_lut()
    np.testing.assert_allclose(np.linalg.norm(lut, axis=1), 1.0, atol=1e-15)
    # code phi*256+theta: theta=0 -> +z, theta=255 -> -z
    np.testing.assert_allclose(lut[0], [0, 0, 1], atol=1e-12)
    np.testing.assert_allclose(lut[255, 2], -1.0, atol=1e-12)


@pytest.mark.parametrize("k,r", [(50, 2.5), (225, 0.225), (7, 0.05)])
def test_kdtree_equals_bruteforce(k, r):
    ph = synth.photon_map(4000, seed=k)
    q = synth.queries(200, seed=1)["point"]
    idx, d2, nf = oracle_lib.knn(ph, q, k, r)
    P = ph["pos"].astype(np.float32)
    r2 = np.float32(r * r)
    for i in range(len(q)):
        qf = q[i].astype(np.float32)
        dx = (qf[0] - P[:, 0]).astype(np.float32)
        dy = (qf[1] - P[:, 1]).astype(np.float32)
        dz = (qf[2] - P[:, 2]).astype(np.float32)
        # the restatement's metric is fmaf(dz, dz, fmaf(dy, dy, dx * dx)) in fp32; the exact
        # fp64 sum of the fp32 products rounded once to fp32 equals it except on rare last-ulp
        # ties, which the rtol below absorbs (the k-NN *set* is checked exactly on the GPU)
        d = (dx * dx).astype(np.float64) + (dy.astype(np.float64) * dy) + (dz.astype(np.float64) * dz)
        df = d.astype(np.float32)
        sel = np.sort(df[df <= r2])[:k]
        assert nf[i] == len(sel)
        np.testing.assert_allclose(d2[i, :nf[i]], sel, rtol=1e-6)
