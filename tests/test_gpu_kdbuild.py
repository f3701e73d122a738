"""Photon-map kd tree built on the device (gi_kdbuild.hip; SURVEY.md 8(f) f1, reference tree:
R3Kdtree.cpp:1552-1671 InsertPoints, median split along the node box's longest axis).

Checked on the tree the k-NN kernels read (gi_get_kd_tree):
- structure: perm is a permutation; every leaf box is the tight box of its photons; every
  internal box is the union of its children; split = the median pivot (the smallest coordinate
  of the upper half), the left child's photons <= split <= the right child's along the axis; the
  axis is the longest extent of the node's box (x, then y / z only when strictly longer);
- k-NN sets through the device-built tree equal the host-built tree's (GI_HOST_KD=1) and
  the oracle's, up to photons tied at the K-th distance;
- a full-GI render on the device-built maps matches the oracle like the host-built ones did.
"""
import os

import numpy as np
import pytest

import gi_amd
import gpu_util
import oracle_lib
import synth
from gi_amd import GLOBAL, CAUSTIC

pytestmark = pytest.mark.gpu


def _positions(ph):
    return np.asarray(ph["pos"], dtype=np.float32)


def check_tree(nodes, perm, L, ph):
    n = len(ph)
    assert sorted(perm.tolist()) == list(range(n))
    pos = _positions(ph)[perm]  # kd order
    levels = L.bit_length() - 1
    lo_of = lambda v, d: ((v - (1 << d)) * (L >> d)) * n // L
    hi_of = lambda v, d: ((v - (1 << d) + 1) * (L >> d)) * n // L
    for d in range(levels + 1):
        for v in range(1 << d, 1 << (d + 1)):
            lo, hi = lo_of(v, d), hi_of(v, d)
            box_lo, box_hi = nodes[v, 0:3], nodes[v, 4:7]
            if hi == lo:
                assert np.all(np.isinf(box_lo)) and np.all(box_lo > 0)
                assert np.all(np.isinf(box_hi)) and np.all(box_hi < 0)
                continue
            seg = pos[lo:hi]
            np.testing.assert_array_equal(box_lo, seg.min(0))
            np.testing.assert_array_equal(box_hi, seg.max(0))
            if d == levels:
                continue
            ax = int(nodes[v, 7:8].view(np.int32)[0])
            ext = box_hi - box_lo
            want = 0
            if ext[1] > ext[want]:
                want = 1
            if ext[2] > ext[want]:
                want = 2
            assert ax == want, (v, ax, want)
            mid = ((v - (1 << d)) * (L >> d) + (L >> (d + 1))) * n // L
            split = nodes[v, 3]
            if mid < hi:  # the median pivot: the smallest coordinate of the upper half
                assert split == pos[mid:hi, ax].min()
            assert np.all(pos[lo:mid, ax] <= split) and np.all(pos[mid:hi, ax] >= split)
            # children boxes union = this box
            c0, c1 = nodes[2 * v], nodes[2 * v + 1]
            np.testing.assert_array_equal(np.minimum(c0[0:3], c1[0:3]), box_lo)
            np.testing.assert_array_equal(np.maximum(c0[4:7], c1[4:7]), box_hi)


@pytest.fixture(scope="module")
def host_renderer():
    old = os.environ.get("GI_HOST_KD")
    os.environ["GI_HOST_KD"] = "1"
    try:
        r = gi_amd.Renderer(0)
    finally:
        if old is None:
            del os.environ["GI_HOST_KD"]
        else:
            os.environ["GI_HOST_KD"] = old
    yield r
    r.close()


def _dup_map(n, seed):
    """photons with many exactly repeated positions and coordinates (ties in every sort)"""
    ph = synth.photon_map(n, seed=seed)
    pts = np.asarray(ph["pos"])
    pts[n // 2:] = pts[: n - n // 2]
    pts[:, 1] = np.round(pts[:, 1] * 8) / 8
    ph["pos"] = pts
    return ph


@pytest.mark.parametrize("n,which", [(0, GLOBAL), (1, GLOBAL), (63, GLOBAL), (64, GLOBAL),
                                     (65, CAUSTIC), (1000, GLOBAL), (20001, CAUSTIC),
                                     (50000, GLOBAL)])
def test_device_tree_structure(renderer, n, which):
    ph = synth.photon_map(n, seed=n + 11)
    renderer.set_photon_map(which, ph)
    nodes, perm, L = renderer.kd_tree(which)
    check_tree(nodes, perm, L, ph)


def test_device_tree_structure_with_ties(renderer):
    ph = _dup_map(9000, 5)
    renderer.set_photon_map(GLOBAL, ph)
    nodes, perm, L = renderer.kd_tree(GLOBAL)
    check_tree(nodes, perm, L, ph)


def test_device_build_is_deterministic(renderer):
    ph = _dup_map(30000, 9)
    renderer.set_photon_map(GLOBAL, ph)
    a = renderer.kd_tree(GLOBAL)
    renderer.set_photon_map(GLOBAL, ph)
    b = renderer.kd_tree(GLOBAL)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])


def _same_sets(gi, gd, gn, oi, od, on):
    np.testing.assert_array_equal(gn, on)
    for i in range(len(gn)):
        m = gn[i]
        np.testing.assert_array_equal(np.sort(gd[i, :m]), np.sort(od[i, :m]))
        a = gi[i, :m][np.lexsort((gi[i, :m], gd[i, :m]))]
        b = oi[i, :m][np.lexsort((oi[i, :m], od[i, :m]))]
        dk = np.sort(gd[i, :m])[m - 1] if m else 0
        mism = a != b
        assert np.all(np.sort(gd[i, :m])[mism] == dk)


@pytest.mark.parametrize("k,r", [(50, 2.5), (225, 0.225)])
def test_knn_device_tree_vs_host_tree_and_oracle(renderer, host_renderer, k, r):
    ph = _dup_map(40000, k)
    q = synth.queries(700, seed=k + 1)["point"]
    renderer.set_photon_map(GLOBAL, ph)
    host_renderer.set_photon_map(GLOBAL, ph)
    g = renderer.FindClosestQuick(GLOBAL, q, k, r)
    h = host_renderer.FindClosestQuick(GLOBAL, q, k, r)
    o = oracle_lib.knn(ph, q, k, r)
    _same_sets(*g, *h)
    _same_sets(*g, *o)


def test_cornell_maps_device_tree(renderer):
    """MapPhotons on cornell (global + caustic): device trees valid, render matches the oracle"""
    args = [gpu_util.scene("cornell.scn"), "/tmp/kd.png", "-resolution", "40", "40", "-aa", "0",
            "-global", "60000", "-caustic", "60000", "-it", "8", "-tt", "4", "-st", "4",
            "-seed", "3"]
    rgb, st, pst = gpu_util.run_gpu(renderer, args)
    for m in (GLOBAL, CAUSTIC):
        nodes, perm, L = renderer.kd_tree(m)
        check_tree(nodes, perm, L, renderer.photon_map(m))
    ref, _ = oracle_lib.render(args, 40, 40)
    gpu_util.compare(rgb, ref, 0.97, 0.99, 0.5)


@pytest.mark.parametrize("n,which", [(5000, GLOBAL), (70001, CAUSTIC)])
def test_device_tree_equals_host_tree_without_ties(renderer, host_renderer, n, which):
    """tie-free photons: the same median splits, axes, boxes and leaf sets from both builds"""
    rng = np.random.default_rng(n)
    ph = synth.photon_map(n, seed=n)
    # distinct coordinates along every axis
    ph["pos"] = np.stack([(rng.permutation(n) + 0.25) / n for _ in range(3)], 1).astype(np.float32)
    assert all(len(np.unique(ph["pos"][:, k])) == n for k in range(3))
    renderer.set_photon_map(which, ph)
    host_renderer.set_photon_map(which, ph)
    dn, dp, dl = renderer.kd_tree(which)
    hn, hp, hl = host_renderer.kd_tree(which)
    assert dl == hl
    np.testing.assert_array_equal(dn, hn)
    for l in range(dl):  # the same photons in every leaf (order inside a leaf may differ)
        s0, s1 = l * n // dl, (l + 1) * n // dl
        assert sorted(dp[s0:s1].tolist()) == sorted(hp[s0:s1].tolist())
