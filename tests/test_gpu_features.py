"""Device features and configurations beyond the headline path, each compared with the oracle
restatement on the same command line and RNG streams (8-bit images; thresholds as in
test_gpu_render.py), plus the reference's own figures as pins for the device path."""
import os

import numpy as np
import pytest

import gallery
import gi_amd
import oracle_lib
from gpu_util import compare_exact, run_gpu, scene

pytestmark = pytest.mark.gpu


# --- the reference's figures (tests/gallery.py) --------------------------------------------
@pytest.mark.parametrize("fig", sorted(gallery.PINNED))
def test_gallery_figure_pins_device(renderer, fig, tmp_path):
    """The device render of each direct-lighting figure's scene meets the same pin as the
    restatement (unsaturated mask, 1 LSB on >= 99.3 %), and equals the restatement's render."""
    scn = gallery.gained_scene(gallery.PINNED[fig], gallery.LIGHT_GAIN, str(tmp_path))
    args = [scn, "/tmp/x.png"] + gallery.FIG_ARGS
    g, _st, _ = run_gpu(renderer, args)
    s = gallery.pin_stats(g, gallery.figure(fig))
    assert s["within1_unsat"] >= 0.993, s
    assert s["exact_unsat"] >= 0.85, s
    assert s["zero_agree"] >= 0.999, s
    o, _ = oracle_lib.render(args + ["-threads", "16"], 512, 512)
    compare_exact(g, o)


@pytest.mark.parametrize("scn,light", [
    ("dirlight1.scn", ("dir", 1.0, np.array([0.710, -0.580, -0.410]))),
    ("pointlight2.scn", ("point", 2.0, np.array([-0.866, 1.0, 0.5])))])
def test_known_answer_floor_pixels_device(renderer, scn, light):
    """Floor pixels computed by hand from the reference's Phong/attenuation formulas
    (tests/gallery.py floor_known_answers) equal the device's 8-bit output exactly."""
    exp = gallery.floor_known_answers(light, 64, 64)
    g, _st, _ = run_gpu(renderer, [scene(scn), "/tmp/x.png", "-resolution", "64", "64", "-aa",
                                   "0", "-no_indirect", "-no_caustic", "-no_specular"])
    got = np.array([g[j, i, 2] for i, j, _ in exp])
    want = np.array([v for _, _, v in exp])
    assert (got == want).all(), np.nonzero(got != want)


# --- BASELINE configs as configured --------------------------------------------------------
def test_c1_exact_command(renderer):
    """C1 exactly: cornell.scn 256x256 aa 0, direct only, default -tt/-st 128."""
    args = [scene("cornell.scn"), "/tmp/c1.png", "-resolution", "256", "256", "-aa", "0",
            "-no_indirect", "-no_caustic", "-seed", "1"]
    g, gst, _ = run_gpu(renderer, args)
    o, ost = oracle_lib.render(args + ["-threads", "16"], 256, 256)
    compare_exact(g, o)
    for k in ("screen_rays", "shadow_rays", "transmissive_samples", "specular_samples"):
        assert gst[k] == ost[k], k


def test_c4_with_caustic_map(renderer):
    """C4's scene with its caustic map (stilllife: five specular solids, Ks = 1): caustic photons
    are stored after specular bounces and the caustic estimate runs in the render."""
    args = [scene("stilllife.scn"), "/tmp/x.png", "-resolution", "24", "24", "-aa", "0",
            "-global", "20000", "-caustic", "40000", "-it", "8", "-tt", "8", "-st", "8",
            "-seed", "2"]
    g, gst, gp = run_gpu(renderer, args)
    o, ost = oracle_lib.render(args + ["-threads", "16"], 24, 24)
    assert gp["caustic_stored"] == ost["caustic_stored"] > 30000
    assert gp["global_stored"] == ost["global_stored"]
    assert gst["knn_map_queries"][1] > 0
    compare_exact(g, o)


# --- render features -----------------------------------------------------------------------
@pytest.mark.parametrize("name,extra", [
    # irradiance cache (photonmap.cpp:381-413, EstimateCachedRadiance photon_utils.cpp:165-246)
    ("cornell.scn", ["-cache", "-global", "20000", "-caustic", "20000", "-it", "16"]),
    # photon visualisation: the global map estimated at the primary hit (raytracer.cpp:151-167)
    ("cornell.scn", ["-photon_viz", "-global", "20000", "-caustic", "20000", "-it", "8"]),
    # fast global: maps store after the first diffuse bounce, no indirect sampling
    ("cornell.scn", ["-fast_global", "-global", "20000", "-caustic", "20000"]),
    # cone and Gaussian filters in a full render (photon_utils.cpp:105-158)
    ("cornell.scn", ["-gf", "cone", "1.25", "-cf", "gauss", "-global", "20000", "-caustic",
                     "20000", "-it", "16"]),
    ("cornell.scn", ["-gf", "gauss", "-cf", "cone", "2", "-global", "20000", "-caustic",
                     "20000", "-it", "16"]),
    # hard lights without shadow rays (light Reflection only), soft lights as hard
    ("cornell.scn", ["-no_shadow", "-no_indirect", "-no_caustic"]),
    ("jensen.scn", ["-no_ss", "-no_indirect", "-no_caustic"]),
    ("jensen.scn", ["-no_shadow", "-no_indirect", "-no_caustic"]),
    # -real: materials normalised so that kd + ks + kt <= 1 (R3Scene.cpp:1741-1755)
    ("stilllife.scn", ["-real", "-global", "20000", "-no_caustic", "-it", "8"]),
    # circular area light with soft shadows (illumination_utils.cpp:91-262), and its photons
    ("softshadow.scn", ["-no_indirect", "-no_caustic", "-lt", "16", "-ss", "16"]),
    ("softshadow.scn", ["-no_ss", "-no_indirect", "-no_caustic"]),
    ("softshadow.scn", ["-global", "20000", "-no_caustic", "-it", "16", "-lt", "4", "-ss", "4"]),
    # spot / directional photon emission feeding a full render
    ("spotlight2.scn", ["-global", "20000", "-no_caustic", "-it", "16"]),
    ("dirlight2.scn", ["-global", "20000", "-no_caustic", "-it", "16"]),
    # rotated / scaled / nested scene-graph transforms (R3SceneNode.cpp:420-510)
    ("transform.scn", ["-no_indirect", "-no_caustic"]),
    ("transform.scn", ["-global", "20000", "-no_caustic", "-it", "8"]),
])
def test_feature_matches_oracle(renderer, name, extra):
    args = [scene(name), "/tmp/x.png", "-resolution", "24", "24", "-aa", "1", "-tt", "8",
            "-st", "8", "-seed", "6"] + extra
    g, gst, gp = run_gpu(renderer, args)
    o, ost = oracle_lib.render(args + ["-threads", "16"], 24, 24)
    if gp is not None:
        assert gp["global_stored"] == ost["global_stored"]
        assert gp["caustic_stored"] == ost["caustic_stored"]
    assert gst["screen_rays"] == ost["screen_rays"]
    assert gst["shadow_rays"] == ost["shadow_rays"]
    assert g.max() > 0
    compare_exact(g, o)


@pytest.mark.parametrize("name,extra", [
    ("spotlight1.scn", []), ("dirlight1.scn", []), ("softshadow.scn", []),
    ("pointlight2.scn", []), ("jensen.scn", [])])
def test_emission_per_light_type(renderer, name, extra):
    """EmitPhotons per light type (photontracer.cpp:198-360): spot (Phong lobe + cutoff
    rejection), directional (disk at 3 R_scene), circular area (disk point + cosine direction),
    point, rect -- the device map equals the restatement's photon for photon."""
    # global map only: the caustic map is not compared here, and spotlight1.scn's Ks = 0.2
    # walls store one caustic photon per ~47,000 emitted (the restatement traced 942 M of them)
    args = [scene(name), "/tmp/x.png", "-global", "20000", "-no_caustic", "-seed", "13"] + extra
    p, sc, *_ = gi_amd.ParseArgs(args)
    renderer.set_params(p)
    renderer.ReadScene(sc)
    renderer.MapPhotons()
    gg = renderer.photon_map(gi_amd.GLOBAL)
    og, oc, _em = oracle_lib.map_photons(args)
    assert len(gg) == len(og) > 10000
    np.testing.assert_array_equal(gg["pos"], og["pos"])
    np.testing.assert_array_equal(gg["rgbe"], og["rgbe"])
    np.testing.assert_array_equal(gg["dir"], og["dir"])
    gc = renderer.photon_map(gi_amd.CAUSTIC)
    assert len(gc) == len(oc)


def test_cache_map_matches_oracle(renderer):
    """-cache precompute: each global photon's power becomes own power + EstimateIrradiance at
    its position (photonmap.cpp:381-413); the cached map equals the restatement's."""
    args = [scene("cornell.scn"), "/tmp/x.png", "-cache", "-global", "30000", "-caustic",
            "1000", "-seed", "3"]
    p, sc, *_ = gi_amd.ParseArgs(args)
    renderer.set_params(p)
    renderer.ReadScene(sc)
    renderer.MapPhotons()
    gg = renderer.photon_map(gi_amd.GLOBAL)
    og, _oc, _em = oracle_lib.map_photons(args)
    assert len(gg) == len(og)
    # irradiance sums differ from the restatement's only in summation order (rtol ~1e-15), which
    # can move an RGBE mantissa across a truncation step on a handful of photons
    assert (gg["rgbe"] == og["rgbe"]).all(axis=1).mean() > 0.995


def test_intersections_transform_scene(renderer):
    """Rotated / scaled / nested begin-end nodes: hit, t (world frame, rescaled), normal by the
    forward affine (Q11) and material inheritance (-1)."""
    rng = np.random.default_rng(1)
    info = renderer.ReadScene(scene("transform.scn"))
    n = 6000
    org = rng.normal(size=(n, 3)) * info["radius"] * 0.7
    tgt = rng.normal(size=(n, 3)) * info["radius"] * 0.3
    d = tgt - org
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    gh, gt, gp, gn, gm = renderer.Intersects(org, d)
    oh, ot, op, on, om = oracle_lib.intersect(scene("transform.scn"), org, d)
    assert gh.sum() > 0.2 * n
    assert (gh == oh).mean() > 0.999
    both = (gh == 1) & (oh == 1)
    np.testing.assert_allclose(gt[both], ot[both], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(gn[both], on[both], atol=1e-9)
    assert (gm[both] == om[both]).mean() > 0.999


# --- large photon maps (C3 4 M caustic, C4 2 M + 10 M, C5 8 M) -------------------------------
@pytest.mark.parametrize("name,extra,res", [
    ("jensen.scn", ["-caustic", "4000000", "-lt", "4", "-ss", "4"], 16),
])
def test_large_map_render_matches_oracle(renderer, name, extra, res):
    """C3's 4 M-photon caustic map: identical stored counts, and a reduced-resolution render whose
    caustic estimates run at C3's photon density (K = 225 over a 4 M map) equals the oracle's."""
    args = [scene(name), "/tmp/x.png", "-resolution", str(res), str(res), "-aa", "0",
            "-it", "8", "-tt", "8", "-st", "8", "-seed", "1"] + extra
    g, gst, gp = run_gpu(renderer, args)
    o, ost = oracle_lib.render(args + ["-threads", "16"], res, res)
    assert gp["caustic_stored"] == ost["caustic_stored"] >= 4000000
    assert gp["global_stored"] == ost["global_stored"]
    assert gst["knn_map_queries"][1] > 0
    compare_exact(g, o)


@pytest.mark.parametrize("name,extra,goal_g,goal_c", [
    ("stilllife.scn", ["-global", "2000000"], 2000000, 10000000),        # C4 maps
    ("teapot.scn", ["-global", "8000000", "-no_caustic"], 8000000, 0),    # C5 map
])
def test_large_map_properties(renderer, name, extra, goal_g, goal_c):
    """C4 / C5 map sizes (8-12 M photons): every goal reached, a k-NN sample equals brute force
    over the device's own map, and a small render is finite, clamped and lit."""
    args = [scene(name), "/tmp/x.png", "-resolution", "16", "16", "-aa", "0", "-it", "8",
            "-tt", "8", "-st", "8", "-seed", "1"] + extra
    g, f, gst, gp = run_gpu(renderer, args, want_float=True)
    assert gp["global_stored"] >= goal_g
    assert gp["caustic_stored"] >= goal_c
    assert np.isfinite(f).all() and f.min() >= 0 and f.max() <= 1
    assert g.mean() > 1
    assert gst["knn_map_queries"][0] > 0
    if goal_c:
        assert gst["knn_map_queries"][1] > 0
    # exact k-NN sets on the big map against a brute force over the same photons
    ph = renderer.photon_map(gi_amd.GLOBAL)
    rng = np.random.default_rng(0)
    q = ph["pos"][rng.integers(0, len(ph), 64)].astype(np.float64) + rng.normal(size=(64, 3)) * 1e-3
    k = 50
    idx, d2, nf = renderer.FindClosestQuick(gi_amd.GLOBAL, q, k, 2.5)
    P = ph["pos"].astype(np.float32)
    for i in range(len(q)):
        qf = q[i].astype(np.float32)
        dd = ((qf - P).astype(np.float64) ** 2).sum(1).astype(np.float32)
        kth = np.sort(dd)[k - 1]
        assert nf[i] == k
        np.testing.assert_allclose(np.sort(d2[i]), np.sort(dd)[:k], rtol=1e-5)
        assert (dd[idx[i]] <= kth * (1 + 1e-5)).all()


def _off_triangles(path):
    with open(path) as f:
        toks = [t for line in f for t in line.split("#")[0].split()]
    assert toks[0] == "OFF"
    nv, nf = int(toks[1]), int(toks[2])
    v = np.array(toks[4:4 + 3 * nv], dtype=float).reshape(nv, 3)
    pos, tris = 4 + 3 * nv, []
    for _ in range(nf):
        k = int(toks[pos])
        tris.append([int(x) for x in toks[pos + 1:pos + 1 + k]])
        pos += 1 + k
    return v, np.array(tris)


@pytest.mark.parametrize("scn,off", [("teapot.scn", "teapot.off"), ("violin.scn", "violinBody.off"),
                                     ("violin.scn", "strings.off")])
@pytest.mark.parametrize("kind", ["surface", "edges", "outside"])
def test_mesh_bvh_matches_linear_loop(renderer, kind, scn, off):
    """The device walks each mesh of >= 16 triangles through its BVH (gi_device.h ray_mesh_bvh);
    the result must be R3Intersects(ray, R3TriangleArray)'s linear loop exactly: Q2 self-hits
    from rays leaving the surface (whole mesh missed), rays through shared edges and vertices
    (equal-t ties go to the lowest triangle index), and rays from outside."""
    rng = np.random.default_rng({"surface": 1, "edges": 2, "outside": 3}[kind])
    v, f = _off_triangles(scene(off))
    renderer.ReadScene(scene(scn))
    n = 6000
    tri = f[rng.integers(0, len(f), n)]
    a, b, c = v[tri[:, 0]], v[tri[:, 1]], v[tri[:, 2]]
    if kind == "surface":
        u = rng.random((n, 2))
        m = u.sum(1) > 1
        u[m] = 1 - u[m]
        org = a + u[:, :1] * (b - a) + u[:, 1:] * (c - a)
        d = rng.normal(size=(n, 3))
    elif kind == "edges":
        w = rng.random((n, 1))
        tgt = np.where(rng.random((n, 1)) < 0.5, a + w * (b - a), a)  # on an edge or a vertex
        org = tgt + rng.normal(size=(n, 3)) * 3.0
        d = tgt - org
    else:
        tgt = a + rng.random((n, 1)) * (b - a)
        org = rng.normal(size=(n, 3)) * 10.0
        d = tgt - org
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    gh, gt, gp, gn, gm = renderer.Intersects(org, d)
    oh, ot, op, on, om = oracle_lib.intersect(scene(scn), org, d)
    np.testing.assert_array_equal(gh, oh)
    both = gh == 1
    assert both.sum() > (0.05 if kind == "surface" else 0.3) * n
    np.testing.assert_array_equal(gt[both], ot[both])
    np.testing.assert_array_equal(gn[both], on[both])
    np.testing.assert_array_equal(gp[both], op[both])


@pytest.mark.parametrize("devices,name,extra", [
    ([0, 0], "cornell.scn", ["-global", "40000", "-caustic", "40000", "-it", "16"]),
    ([0, 0, 0], "jensen.scn", ["-global", "4000", "-caustic", "40000", "-lt", "4", "-ss", "4",
                               "-it", "8"]),
])
def test_device_set_matches_one_device(devices, name, extra):
    """gi_create_devices: photon emission split across the set, maps replicated, 16x16 tiles
    dealt (tx + ty) % ndev and gathered onto the first device. On one GPU the set repeats device 0 (the
    gather is then a peer copy; distinct devices use RCCL send/recv): the image, the f32 frame,
    the photon maps and every -v counter equal the single-device render's."""
    args = [scene(name), "/tmp/x.png", "-resolution", "40", "24", "-aa", "1", "-tt", "8",
            "-st", "8", "-seed", "8"] + extra
    p, sc, _o, w, h, aa, real = gi_amd.ParseArgs(args)
    out = []
    for devs in (None, devices):
        r = gi_amd.Renderer(0, p, devices=devs)
        try:
            r.ReadScene(sc, real)
            ps = r.MapPhotons()
            rgb, f, st = r.RenderImage(aa, w, h, want_float=True)
            maps = [r.photon_map(m) for m in (gi_amd.GLOBAL, gi_amd.CAUSTIC)]
            out.append((rgb, f, st, ps, maps))
        finally:
            r.close()
    (r1, f1, s1, p1, m1), (r2, f2, s2, p2, m2) = out
    for m in (0, 1):
        assert len(m1[m]) == len(m2[m])
        assert (m1[m].tobytes() == m2[m].tobytes())
    assert p1["global_stored"] == p2["global_stored"]
    np.testing.assert_array_equal(f1, f2)
    np.testing.assert_array_equal(r1, r2)
    for k in ("screen_rays", "shadow_rays", "monte_carlo_rays", "transmissive_samples",
              "specular_samples", "indirect_samples", "caustic_samples", "knn_queries",
              "knn_photons"):
        assert s1[k] == s2[k], k


@pytest.mark.parametrize("name,extra,rate0", [
    ("stilllife.scn", ["-global", "300000", "-caustic", "300000"], None),
    ("display.scn", ["-global", "50000", "-caustic", "200000", "-pd", "5"], None),
    ("jensen.scn", ["-global", "20000", "-caustic", "100000"], "0.0001"),
])
def test_single_pass_photon_maps_equal_two_pass(name, extra, rate0, monkeypatch):
    """Single-pass photon tracing (one atomic per wave per bounce, then a sort on (emission
    index, store ordinal); gi_host.cpp trace_batch_dev) builds the maps the count pass + scan +
    re-trace (GI_PHOTON_2PASS=1, r03) built: byte for byte, in the same emission order, with the
    same emitted counts. Covers several lights and emission rounds (stilllife), a short -pd
    (few ordinal bits), and launches that overflow their first slot estimate and are re-run
    (GI_PHOTON_RATE0)."""
    import gpu_util
    args = [gpu_util.scene(name), "/tmp/x.png", "-seed", "3"] + extra
    p, sc, *_ = gi_amd.ParseArgs(args)
    out = []
    for env in ({"GI_PHOTON_2PASS": "1"}, {"GI_PHOTON_2PASS": "0"}):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        if rate0 and env["GI_PHOTON_2PASS"] == "0":
            monkeypatch.setenv("GI_PHOTON_RATE0", rate0)
        r = gi_amd.Renderer(0, p)
        try:
            r.ReadScene(sc)
            st = r.MapPhotons()
            out.append((st, [r.photon_map(m) for m in (gi_amd.GLOBAL, gi_amd.CAUSTIC)]))
        finally:
            r.close()
    (s2, m2), (s1, m1) = out
    for k in ("global_stored", "caustic_stored", "global_emitted", "caustic_emitted"):
        assert s1[k] == s2[k], k
    assert s1["caustic_stored"] > 0
    for a, b in zip(m1, m2):
        assert len(a) == len(b)
        assert a.tobytes() == b.tobytes()
