"""Every k-NN kernel the render and the test seams launch, against the oracle
(R3Kdtree::FindClosestQuick, R3Kdtree.cpp:688-848; EstimateRadiance photon_utils.cpp:72-162).

The kernel is chosen when a context is created (gi_host.cpp run_knn): GI_KNN_KERNEL 7 = chunk
kernel with lane select + per-lane fallback (the K <= 64 default), 3 = per-lane kernel (list
mode), 8 = large-K chunk kernel + query-per-wave fallback (the K > 64 default), 1 = query per
wave, 0 = per-lane with global-memory heaps (any K). GI_CHUNK_MINSUB sets how far an
overflowing chunk is split (1 = down to single queries, 64 = straight to the fallback);
GI_KNN_DK=0 turns off the start from per-photon K-th distance bounds; GI_CHUNK_FB_ALL=1 sends
every query of the chunk kernel to its fallback (the query-per-wave kernel; GI_FB_WAVE=0: the
per-lane kernel); GI_CHUNK_DK_EXACT=0 keeps the large-K chunk
kernel's centre bound at the per-photon dk bound (default: refined to the exact d_K(c)). Each
must return the oracle's k-NN sets exactly
(the fp32 metric is shared; only photons tied at the k-th distance may differ) and its
EstimateRadiance within rtol 1e-10 (fp64 sums in a different order). Leaf sizes are varied
too, because the result set may not depend on the tree shape."""
import os

import numpy as np
import pytest

import gi_amd
import oracle_lib
import synth
from gi_amd import GLOBAL, DISK, CONE

pytestmark = pytest.mark.gpu

VARIANTS = [
    {"GI_KNN_KERNEL": "0", "GI_LEAF_SIZE": "16"},
    {"GI_KNN_KERNEL": "1", "GI_LEAF_SIZE": "512"},
    {"GI_KNN_KERNEL": "1", "GI_KNN_DK": "0"},
    {"GI_KNN_KERNEL": "3", "GI_LEAF_SIZE": "32"},
    {"GI_KNN_KERNEL": "7"},
    {"GI_KNN_KERNEL": "7", "GI_LEAF_SIZE": "50"},
    {"GI_KNN_KERNEL": "7", "GI_CHUNK_MINSUB": "1"},
    {"GI_KNN_KERNEL": "7", "GI_CHUNK_DK": "0"},
    {"GI_KNN_KERNEL": "7", "GI_CHUNK_FB_ALL": "1", "GI_KNN_DK": "0"},
    # the per-lane kernel as the last fallback (the query-per-wave kernel is the default)
    {"GI_KNN_KERNEL": "7", "GI_FB_WAVE": "0"},
    {"GI_KNN_KERNEL": "7", "GI_FB_WAVE": "0", "GI_CHUNK_FB_ALL": "1", "GI_LEAF_SIZE": "32"},
    {"GI_KNN_KERNEL": "8"},
    {"GI_KNN_KERNEL": "8", "GI_CHUNK_DK_EXACT": "0"},
    {"GI_KNN_KERNEL": "8", "GI_LEAF_SIZE": "128"},
    {"GI_KNN_KERNEL": "8", "GI_CHUNK_MINSUB_BIG": "1"},
    # every overflowing large-K chunk handed to the query-per-wave fallback whole
    {"GI_KNN_KERNEL": "8", "GI_CHUNK_MINSUB_BIG": "64"},
    # a third large-K chunk pass (512 -> 1024 -> 1024 candidates: the pass chain's ping-pong)
    {"GI_KNN_KERNEL": "8", "GI_CHUNK_CAP_BIG3": "1024", "GI_LEAF_SIZE": "128"},
]


def make_renderer(env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return gi_amd.Renderer(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("env", VARIANTS, ids=lambda e: "-".join(f"{k[3:]}{v}" for k, v in e.items()))
@pytest.mark.parametrize("n,k,r", [(20000, 50, 2.5), (50000, 225, 0.225), (3000, 50, 0.05),
                                   (7, 50, 2.5), (100, 1, 0.3)])
def test_variant_knn_sets(env, n, k, r):
    r_ = make_renderer(env)
    try:
        ph = synth.photon_map(n, seed=n + 1)
        q = synth.queries(700, seed=k + 3)["point"]
        r_.set_photon_map(GLOBAL, ph)
        gi, gd, gn = r_.FindClosestQuick(GLOBAL, q, k, r)
    finally:
        r_.close()
    oi, od, on = oracle_lib.knn(ph, q, k, r)
    np.testing.assert_array_equal(gn, on)
    for i in range(len(q)):
        m = gn[i]
        np.testing.assert_array_equal(np.sort(gd[i, :m]), od[i, :m])
        order = np.lexsort((gi[i, :m], gd[i, :m]))
        got = gi[i, :m][order]
        mism = got != oi[i, :m]
        assert np.all(gd[i, :m][order][mism] == od[i, m - 1]), (i, got[mism])


@pytest.mark.parametrize("env", VARIANTS, ids=lambda e: "-".join(f"{k[3:]}{v}" for k, v in e.items()))
@pytest.mark.parametrize("filt,k,r", [(DISK, 50, 2.5), (CONE, 50, 0.3)])
def test_variant_estimate(env, filt, k, r):
    r_ = make_renderer(env)
    try:
        ph = synth.photon_map(30000, seed=11)
        q = synth.queries(900, seed=5, k=k, r=r, filt=filt, spec=True)
        fk = 1.25 if filt == CONE else 1.0
        p = gi_amd.default_params()
        p.filter_const_k = fk
        r_.set_params(p)
        r_.set_photon_map(GLOBAL, ph)
        g, gn, gm = r_.EstimateRadiance(GLOBAL, q)
    finally:
        r_.close()
    o, on, om = oracle_lib.estimate_radiance(ph, q, filter_k=fk)
    np.testing.assert_array_equal(gn, on)
    np.testing.assert_array_equal(gm, om)
    np.testing.assert_allclose(g, o, rtol=1e-10, atol=1e-300)


def clustered_queries(n, seed, k, r, filt):
    """Dense queries on one face (the regime the chunk kernel is built for): 64 consecutive
    Morton-sorted queries span much less than a K-neighbourhood."""
    q = synth.queries(n, seed=seed, k=k, r=r, filt=filt, spec=True)
    rng = np.random.default_rng(seed)
    pts = np.zeros((n, 3))
    pts[:, 0] = 0.4 + rng.random(n) * 0.2
    pts[:, 1] = 0.0
    pts[:, 2] = 0.5 + rng.random(n) * 0.2
    q["point"] = pts
    q["normal"] = np.tile([0.0, 1.0, 0.0], (n, 1))
    return q


@pytest.mark.parametrize("env", VARIANTS, ids=lambda e: "-".join(f"{k[3:]}{v}" for k, v in e.items()))
@pytest.mark.parametrize("filt,k,r", [(DISK, 50, 2.5), (CONE, 32, 0.05), (DISK, 225, 0.225),
                                      (DISK, 64, 0.05), (DISK, 64, 2.5)])
def test_variant_dense_queries(env, filt, k, r):
    r_ = make_renderer(env)
    try:
        ph = synth.photon_map(200000, seed=13)
        q = clustered_queries(8192, 17, k, r, filt)
        fk = 1.25 if filt == CONE else 1.0
        p = gi_amd.default_params()
        p.filter_const_k = fk
        r_.set_params(p)
        r_.set_photon_map(GLOBAL, ph)
        g, gn, gm = r_.EstimateRadiance(GLOBAL, q)
    finally:
        r_.close()
    o, on, om = oracle_lib.estimate_radiance(ph, q, filter_k=fk)
    np.testing.assert_array_equal(gn, on)
    np.testing.assert_array_equal(gm, om)
    np.testing.assert_allclose(g, o, rtol=1e-10, atol=1e-300)


@pytest.mark.parametrize("env", VARIANTS, ids=lambda e: "-".join(f"{k[3:]}{v}" for k, v in e.items()))
@pytest.mark.parametrize("k,filt", [(50, DISK), (8, CONE), (50, CONE)])
def test_variant_tied_distances(env, k, filt):
    """Photons and queries snapped to a coarse grid on one face: ~40 photons share each
    position and many keys share one d2, so the K-th distance is tied across many photons
    (the lane select's bracket cannot split them and hands such queries to the fallback).
    Which tied photon is kept follows the kd order, and the GPU and oracle kd builds order
    photons with equal coordinates differently, so every photon carries the same power and
    direction: the estimate then depends only on the multiset of the K smallest d2, which is
    unique, and must match exactly."""
    r_ = make_renderer(env)
    try:
        ph = synth.photon_map(40000, seed=23)
        rng = np.random.default_rng(29)
        pts = np.zeros((len(ph), 3), dtype=np.float32)
        pts[:, 0] = np.round(0.3 + rng.random(len(ph)) * 0.3, 2)
        pts[:, 2] = np.round(0.4 + rng.random(len(ph)) * 0.3, 2)
        ph["pos"] = pts
        ph["rgbe"][:] = ph["rgbe"][0]
        ph["dir"][:] = ph["dir"][0]
        q = clustered_queries(4096, 31, k, 0.2, filt)
        q["point"] = np.round(q["point"], 2)
        fk = 1.25 if filt == CONE else 1.0
        p = gi_amd.default_params()
        p.filter_const_k = fk
        r_.set_params(p)
        r_.set_photon_map(GLOBAL, ph)
        g, gn, gm = r_.EstimateRadiance(GLOBAL, q)
    finally:
        r_.close()
    o, on, om = oracle_lib.estimate_radiance(ph, q, filter_k=fk)
    np.testing.assert_array_equal(gn, on)
    np.testing.assert_array_equal(gm, om)
    np.testing.assert_allclose(g, o, rtol=1e-10, atol=1e-300)


def focus_map(n_focus, n_halo, seed):
    """A caustic focus: n_focus photons in a disk of radius 0.01 on the floor, inside a sparse
    halo of n_halo photons (the C2 glass-sphere caustic, where the queries at the focus rim
    overflow every LDS chunk capacity and reach the streaming pass and the wave fallback)."""
    rng = np.random.default_rng(seed)
    ph = synth.photon_map(n_focus + n_halo, seed=seed)
    pts = np.zeros((n_focus + n_halo, 3), dtype=np.float32)
    a = rng.random(n_focus) * 2 * np.pi
    rr = 0.01 * np.sqrt(rng.random(n_focus))
    pts[:n_focus, 0] = 0.5 + rr * np.cos(a)
    pts[:n_focus, 2] = 0.6 + rr * np.sin(a)
    pts[n_focus:, 0] = 0.3 + rng.random(n_halo) * 0.4
    pts[n_focus:, 2] = 0.4 + rng.random(n_halo) * 0.4
    ph["pos"] = pts
    return ph


@pytest.mark.parametrize("env", [{}, {"GI_LEAF_SIZE": "64"}, {"GI_KNN_KERNEL": "1"}],
                         ids=["auto", "leaf64", "wave"])
@pytest.mark.parametrize("filt,k,r", [(DISK, 225, 0.225), (CONE, 100, 0.1), (DISK, 225, 0.02)])
def test_caustic_focus_rim(env, filt, k, r):
    """Queries on the rim of a dense focus (0.005-0.05 from its centre, 64 Morton-adjacent
    queries far closer together than a K-neighbourhood) against the oracle."""
    r_ = make_renderer(env)
    try:
        ph = focus_map(150000, 30000, 41)
        n = 6000
        q = clustered_queries(n, 43, k, r, filt)
        rng = np.random.default_rng(47)
        a = rng.random(n) * 2 * np.pi
        rr = 0.005 + rng.random(n) * 0.045
        pts = np.zeros((n, 3))
        pts[:, 0] = 0.5 + rr * np.cos(a)
        pts[:, 2] = 0.6 + rr * np.sin(a)
        q["point"] = pts
        fk = 1.25 if filt == CONE else 1.0
        p = gi_amd.default_params()
        p.filter_const_k = fk
        r_.set_params(p)
        r_.set_photon_map(GLOBAL, ph)
        g, gn, gm = r_.EstimateRadiance(GLOBAL, q)
    finally:
        r_.close()
    o, on, om = oracle_lib.estimate_radiance(ph, q, filter_k=fk)
    np.testing.assert_array_equal(gn, on)
    np.testing.assert_array_equal(gm, om)
    # 150,000 photons within 0.01: some queries' K-th and (K+1)-th fp32 d2 are equal. The device
    # keeps the tied photon with the smaller kd index, the oracle (like the reference) the one
    # its traversal meets first, so only untied queries must agree
    _, od, onn = oracle_lib.knn(ph, q["point"], k + 1, r)
    tied = (onn == k + 1) & (od[:, k - 1] == od[:, k])
    assert tied.mean() < 0.01
    np.testing.assert_allclose(g[~tied], o[~tied], rtol=1e-10, atol=1e-300)


@pytest.mark.parametrize("name,extra", [
    ("stilllife.scn", ["-global", "20000", "-caustic", "40000"]),                 # Ks = 1, n = 100
    ("jensen.scn", ["-global", "5000", "-caustic", "20000", "-cf", "cone", "1.25"]),  # cone filter
])
def test_general_form_miss_rerenders(name, extra):
    """an instance without the general estimate form (KnnArgs::general == 0) that
    meets a query needing it (specular term, cone / Gauss filter) writes NaN and counts it
    (ST_GEN_MISS); render_common then re-renders with the general instances. GI_KNN_GENERAL=-1
    makes the host claim that no query needs the general form, so every such query misses: the
    image must still equal the normal context's, bit for bit, with no NaN."""
    from gpu_util import run_gpu, scene
    args = [scene(name), "/tmp/x.png", "-resolution", "24", "24", "-aa", "0", "-it", "8",
            "-tt", "4", "-st", "4", "-lt", "4", "-ss", "4", "-seed", "2"] + extra
    outs = []
    for env in ({}, {"GI_KNN_GENERAL": "-1"}):
        r = make_renderer(env)
        try:
            g, f, st, _ = run_gpu(r, args, want_float=True)
            assert np.isfinite(f).all()
            outs.append((g, st))
        finally:
            r.close()
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    for key in ("knn_queries", "knn_photons", "shadow_rays", "monte_carlo_rays"):
        assert outs[0][1][key] == outs[1][1][key], key
