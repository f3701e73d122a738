"""Device render / photon tracing / ray casting vs the oracle restatement on the same inputs
and RNG streams. Images are compared on the 8-bit output (R2Image::SetPixelRGB truncation):
the device code is compiled without FP contraction (like the reference's x86 build) and shares
gi_math.h's transcendentals with the oracle, so images, photon maps and counters are asserted
bit-identical (compare_exact). Before r04 the device called ROCm's math library, one ulp from
glibc, and the thresholds here had to leave room for the Monte Carlo paths that forked on it."""
import os

import numpy as np
import pytest

import gi_amd
import gi_dist
import oracle_lib
from gpu_util import compare_exact, run_gpu, scene

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,extra", [
    ("cornell.scn", []), ("jensen.scn", ["-lt", "8", "-ss", "8"]), ("stilllife.scn", []),
    ("pointlight1.scn", []), ("spotlight1.scn", []), ("dirlight1.scn", []),
    ("cylinder.scn", []), ("lines.scn", [])])
def test_direct_only_matches_oracle(renderer, name, extra):
    args = [scene(name), "/tmp/x.png", "-resolution", "48", "48", "-aa", "0", "-no_indirect",
            "-no_caustic", "-tt", "8", "-st", "8", "-seed", "3"] + extra
    g, gst, _ = run_gpu(renderer, args)
    o, ost = oracle_lib.render(args, 48, 48)
    compare_exact(g, o)
    assert gst["screen_rays"] == ost["screen_rays"]


def test_full_gi_cornell_matches_oracle(renderer):
    args = [scene("cornell.scn"), "/tmp/x.png", "-resolution", "24", "24", "-aa", "1",
            "-global", "20000", "-caustic", "20000", "-it", "16", "-tt", "8", "-st", "8",
            "-seed", "5"]
    g, gst, gp = run_gpu(renderer, args)
    o, ost = oracle_lib.render(args, 24, 24)
    assert gp["global_stored"] == ost["global_stored"]
    assert gp["caustic_stored"] == ost["caustic_stored"]
    compare_exact(g, o)
    # the same RNG streams and bit-identical paths: the same queries, and the same photons found
    assert gst["knn_queries"] == ost["knn_queries"]
    assert gst["knn_photons"] == ost["knn_photons"]


def test_photon_maps_match_oracle(renderer):
    args = [scene("cornell.scn"), "/tmp/x.png", "-global", "30000", "-caustic", "30000",
            "-seed", "11"]
    p, sc, *_ = gi_amd.ParseArgs(args)
    renderer.set_params(p)
    renderer.ReadScene(sc)
    renderer.MapPhotons()
    gg = renderer.photon_map(gi_amd.GLOBAL)
    gc = renderer.photon_map(gi_amd.CAUSTIC)
    og, oc, em = oracle_lib.map_photons(args)
    for a, b in ((gg, og), (gc, oc)):
        assert len(a) == len(b)
        np.testing.assert_array_equal(a["pos"], b["pos"])
        np.testing.assert_array_equal(a["rgbe"], b["rgbe"])
        np.testing.assert_array_equal(a["dir"], b["dir"])


@pytest.mark.parametrize("name", ["cornell.scn", "stilllife.scn", "teapot.scn", "jensen.scn",
                                  "cylinder.scn"])
def test_intersections_match_oracle(renderer, name):
    rng = np.random.default_rng(0)
    info = renderer.ReadScene(scene(name))
    n = 4000
    org = rng.normal(size=(n, 3)) * info["radius"] * 0.5
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    gh, gt, gp, gn, gm = renderer.Intersects(org, d)
    oh, ot, op, on, om = oracle_lib.intersect(scene(name), org, d)
    assert (gh == oh).mean() > 0.999
    both = (gh == 1) & (oh == 1)
    np.testing.assert_allclose(gt[both], ot[both], rtol=1e-9, atol=1e-12)
    assert (gm[both] == om[both]).mean() > 0.999
    np.testing.assert_allclose(gn[both], on[both], atol=1e-9)


def test_tiles_compose_full_image(renderer):
    args = [scene("cornell.scn"), "/tmp/x.png", "-resolution", "40", "24", "-aa", "1",
            "-no_indirect", "-no_caustic", "-tt", "4", "-st", "4"]
    p, sc, _o, w, h, aa, _r = gi_amd.ParseArgs(args)
    renderer.set_params(p)
    renderer.ReadScene(sc)
    full, ff, _ = renderer.RenderImage(aa, w, h, want_float=True)
    acc = np.zeros((h, w, 3), dtype=np.float32)
    owner = gi_dist.tile_owner_map(w, h, 16, 3)
    for s in range(3):
        part, _ = renderer.render_tiles(aa, w, h, 16, s, 3)
        # the shard touches exactly the pixels gi_dist assigns to it (bench.py's gather)
        assert not part[owner != s].any()
        np.testing.assert_array_equal(part[owner == s], ff[owner == s])
        acc += part
    np.testing.assert_array_equal(acc, ff)


# Full-GI parity on the other BASELINE configs, shrunk to oracle-friendly sizes:
# C3 jensen (rect light with soft shadows + glass caustics), C4 stilllife (boxes and meshes under
# translate nodes, 4 point lights), C5 teapot (1,452-triangle mesh, depth of field).
@pytest.mark.parametrize("name,extra", [
    ("jensen.scn", ["-global", "4000", "-caustic", "20000", "-lt", "4", "-ss", "4", "-it", "16"]),
    ("stilllife.scn", ["-global", "20000", "-no_caustic", "-it", "16"]),
    ("teapot.scn", ["-global", "20000", "-no_caustic", "-it", "8", "-dof", "2", "8.0", "0.05"]),
])
def test_full_gi_configs_match_oracle(renderer, name, extra):
    args = [scene(name), "/tmp/x.png", "-resolution", "20", "20", "-aa", "0", "-tt", "8",
            "-st", "8", "-seed", "9"] + extra
    g, gst, gp = run_gpu(renderer, args)
    o, ost = oracle_lib.render(args, 20, 20)
    if gp is not None:
        assert gp["global_stored"] == ost["global_stored"]
        assert gp["caustic_stored"] == ost["caustic_stored"]
    assert gst["screen_rays"] == ost["screen_rays"]
    compare_exact(g, o)


def test_cylinder_and_line_cases_match_oracle(renderer):
    """R3Intersects(ray, R3Cylinder) (R3Isect.cpp:1025-1200) branch coverage: rays aimed at the
    side and caps from outside, from inside the cylinder, from above/below the caps, parallel to
    the axis (inside and outside), and rays aimed at the radius-1e-3 `line` cylinders."""
    rng = np.random.default_rng(5)
    renderer.ReadScene(scene("cylinder.scn"))
    n = 3000
    # targets on the unit cylinder (axis y, y in [-0.5, 0.5]) and on the cube-edge lines
    phi = rng.random(n) * 2 * np.pi
    side = np.stack([np.cos(phi), rng.random(n) - 0.5, np.sin(phi)], 1)
    cap = np.stack([np.sqrt(rng.random(n)) * np.cos(phi), np.sign(rng.random(n) - 0.5) * 0.5,
                    np.sqrt(rng.random(n)) * np.sin(phi)], 1)
    a, b = np.array([-1.0, -1.0, -1.0]), np.array([1.0, -1.0, -1.0])
    on_line = a + rng.random((n, 1)) * (b - a)
    targets = np.concatenate([side, cap, on_line])
    org = targets + rng.normal(size=targets.shape) * 3.0
    d = targets - org
    inside = np.stack([rng.random(n) * 0.5 - 0.25, rng.random(n) - 0.5, rng.random(n) * 0.5 - 0.25], 1)
    d_in = rng.normal(size=(n, 3))
    par_o = np.stack([rng.random(n) * 3 - 1.5, np.full(n, 2.0), rng.random(n) * 3 - 1.5], 1)
    par_d = np.tile([0.0, -1.0, 0.0], (n, 1))
    org = np.concatenate([org, inside, par_o])
    d = np.concatenate([d, d_in, par_d])
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    gh, gt, gp, gn, gm = renderer.Intersects(org, d)
    oh, ot, op, on, om = oracle_lib.intersect(scene("cylinder.scn"), org, d)
    assert gh.sum() > 0.3 * len(gh)
    assert (gh == oh).mean() > 0.9995
    both = (gh == 1) & (oh == 1)
    np.testing.assert_allclose(gt[both], ot[both], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(gn[both], on[both], atol=1e-9)


@pytest.mark.parametrize("name,extra", [
    ("cornell.scn", ["-global", "20000", "-caustic", "20000"]),
    ("jensen.scn", ["-global", "4000", "-caustic", "20000", "-lt", "4", "-ss", "4"])])
def test_indirect_continuation_queue_is_exact(name, extra):
    """ind_kernel's continuation queue (GI_SPLIT_IND=1, default) only regroups the bounces of
    MonteCarlo_IndirectSample (montecarlo.cpp:177-305) that follow a glass/mirror hit: the f32
    image and every -v counter equal the one-loop-per-lane kernel's (GI_SPLIT_IND=0), also when
    the queue starts far too small (GI_IND_FRAC) and the batch is re-run with more room, and
    when the Monte Carlo paths' sub-paths skip their lean first-bounce kernel (GI_MC_SUB=0).
    The Monte Carlo paths (MonteCarlo_PathTrace, montecarlo.cpp:16-171) give the same image and
    counters in the persistent kernel (a lane takes the next path when its own ends; jensen's
    default, and forced with a 3-block grid: thousands of refills per wave) and one path per lane
    (GI_MC_PERSIST=0), also with their sub-paths going straight to ind_cont_kernel."""
    args = [scene(name), "/tmp/x.png", "-resolution", "32", "32", "-aa", "1", "-it", "32",
            "-tt", "8", "-st", "8", "-seed", "4"] + extra
    p, sc, _o, w, h, aa, real = gi_amd.ParseArgs(args)
    out = []
    keys = ("GI_SPLIT_IND", "GI_IND_FRAC", "GI_MC_SUB", "GI_MC_PERSIST")
    old = {k: os.environ.get(k) for k in keys}
    try:
        for env in ({"GI_SPLIT_IND": "0"}, {"GI_SPLIT_IND": "1"},
                    {"GI_SPLIT_IND": "1", "GI_IND_FRAC": "0.00001"},
                    {"GI_SPLIT_IND": "1", "GI_MC_SUB": "0"}, {"GI_MC_PERSIST": "0"},
                    {"GI_MC_PERSIST": "3"}, {"GI_MC_PERSIST": "3", "GI_MC_SUB": "0"}):
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(env)
            r = gi_amd.Renderer(0, p)
            try:
                r.ReadScene(sc, real)
                r.MapPhotons()
                _rgb, f, st = r.RenderImage(aa, w, h, want_float=True)
                out.append((f, st))
            finally:
                r.close()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    for other in out[1:]:
        np.testing.assert_array_equal(out[0][0], other[0])
        for k in ("screen_rays", "shadow_rays", "monte_carlo_rays", "transmissive_samples",
                  "specular_samples", "indirect_samples", "caustic_samples", "knn_queries"):
            assert out[0][1][k] == other[1][k], k
    assert out[1][1]["transmissive_samples"] > 0


@pytest.mark.parametrize("scene", ["cornell.scn", "jensen.scn", "stilllife.scn", "transform.scn"])
def test_element_pretest_is_exact(scene, monkeypatch):
    """scene_intersect's division-free element box pre-test (elem_maybe_hit) only skips elements
    the reference's box test would skip: renders with it forced on and off are identical."""
    import gi_amd
    import gpu_util
    args = [gpu_util.scene(scene), "/tmp/pt.png", "-resolution", "40", "32", "-aa", "0",
            "-global", "30000", "-caustic", "30000", "-it", "4", "-tt", "4", "-st", "4",
            "-seed", "9"]
    out = []
    for v in ("1", "0"):
        monkeypatch.setenv("GI_ELEM_PRETEST", v)
        r = gi_amd.Renderer(0)
        try:
            _, f, _, _ = gpu_util.run_gpu(r, args, want_float=True)
        finally:
            r.close()
        out.append(f)
    np.testing.assert_array_equal(out[0], out[1])


@pytest.mark.parametrize("scene", ["cornell.scn", "jensen.scn"])
@pytest.mark.parametrize("var,vals", [("GI_ROW_ORDER", ("1", "0")), ("GI_SURF_KEY", ("1", "0")),
                                      ("GI_SURF_KEY_C", ("1", "0"))])
def test_knn_launch_order_is_exact(scene, var, vals, monkeypatch):
    """How the photon lookups (PhotonMap_EstimateRadiance, photonmap.cpp) are grouped into
    launches does not change any result: the global list's valid slots compacted from the
    indirect row masks before the sort (GI_ROW_ORDER=1, default) against the sort of every slot
    with the empty ones last (gi_sort.hip morton_order_valid), and the surface keys (face, depth
    slab, 2-D Hilbert curve in the face's plane; global list GI_SURF_KEY, caustic list
    GI_SURF_KEY_C) against the 3-D curve. The f32 image and the -v counters
    are equal; -tt/-st 4 give Monte Carlo paths, -it 16 many empty slots. (r06: the r04 order over
    every slot, the early estimate of the deterministic slots and other key resolutions, all
    measured slower and shown exact here in r05, were removed with their knobs.)"""
    import gi_amd
    import gpu_util
    args = [gpu_util.scene(scene), "/tmp/so.png", "-resolution", "40", "32", "-aa", "1",
            "-global", "30000", "-caustic", "30000", "-it", "16", "-tt", "4", "-st", "4",
            "-seed", "5"]
    out = []
    for v in vals:
        monkeypatch.setenv(var, v)
        r = gi_amd.Renderer(0)
        try:
            _, f, st, _ = gpu_util.run_gpu(r, args, want_float=True)
        finally:
            r.close()
        out.append((f, st))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    for k in ("monte_carlo_rays", "indirect_samples", "caustic_samples", "knn_queries"):
        assert out[0][1][k] == out[1][1][k], k
    assert out[0][1]["monte_carlo_rays"] > 0


def test_c5_settings_match_oracle(renderer):
    """C5's sampling settings at an oracle-sized resolution: teapot.scn, aa 3 (64 subsamples per
    pixel, render.cpp:174-178), depth of field with 4 aperture samples at the C5 focus and
    aperture (-dof 4 12.2282 0.025, render.cpp:104-117, Q7), global map only."""
    args = [scene("teapot.scn"), "/tmp/x.png", "-resolution", "10", "8", "-aa", "3", "-global",
            "20000", "-no_caustic", "-it", "4", "-dof", "4", "12.2282", "0.025", "-seed", "6"]
    g, gst, gp = run_gpu(renderer, args)
    o, ost = oracle_lib.render(args, 10, 8)
    assert gp["global_stored"] == ost["global_stored"]
    assert gst["screen_rays"] == ost["screen_rays"] > 0  # primary hits (render.cpp:119-121)
    compare_exact(g, o)


def _threads():
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return min(n, int(omp)) if omp.isdigit() and int(omp) > 0 else n


C2_MAPS = ["-global", "1000000", "-caustic", "1000000"]


def test_c2_config_matches_oracle(renderer):
    """C2 exactly as bench.py runs it (cornell.scn, aa 2, 1M global + 1M caustic photons, every
    other flag at the reference default: -it 256, -tt/-st 128, K 50 / 225) at an oracle-sized
    16 x 16 resolution: photon maps of the same size, the same per-sample work."""
    args = [scene("cornell.scn"), "/tmp/x.png", "-resolution", "16", "16", "-aa", "2",
            "-seed", "1", "-threads", str(_threads())] + C2_MAPS
    g, gst, gp = run_gpu(renderer, args)
    o, ost = oracle_lib.render(args, 16, 16)
    assert gp["global_stored"] == ost["global_stored"] >= 1000000
    assert gp["caustic_stored"] == ost["caustic_stored"] >= 1000000
    assert gst["screen_rays"] == ost["screen_rays"]
    for k in ("shadow_rays", "monte_carlo_rays", "transmissive_samples", "specular_samples",
              "indirect_samples", "caustic_samples", "knn_queries", "knn_photons"):
        assert gst[k] == ost[k], (k, gst[k], ost[k])
    compare_exact(g, o)


def test_c2_full_frame_properties(renderer):
    """The full C2 frame (1024^2, aa 2, 1M + 1M photons): finite and clamped to [0, 1] per pixel
    (render.cpp:236-249), the same image twice over the resident maps, and the same image from
    a two-entry device set on one GPU (tiles dealt over the set and gathered, render.cpp:90).
    Three C2-sized contexts share the card over the test, so the session renderer's scratch
    from earlier tests is released first (gi_release_scratch)."""
    import gc
    import hashlib
    gc.collect()
    renderer.release_scratch()
    args = [scene("cornell.scn"), "/tmp/x.png", "-resolution", "1024", "1024", "-aa", "2",
            "-seed", "1"] + C2_MAPS
    p, sc, _o, w, h, aa, real = gi_amd.ParseArgs(args)
    hashes = []
    for devs in (None, [0, 0]):
        r = gi_amd.Renderer(0, p, devices=devs)
        try:
            r.ReadScene(sc, real)
            ps = r.MapPhotons()
            assert ps["global_stored"] >= 1000000 and ps["caustic_stored"] >= 1000000
            runs = 2 if devs is None else 1
            for _ in range(runs):
                rgb, f, st = r.RenderImage(aa, w, h, want_float=True)
                assert rgb.shape == (h, w, 3) and f.shape == (h, w, 3)
                assert np.isfinite(f).all() and f.min() >= 0.0 and f.max() <= 1.0
                assert st["screen_rays"] > 0.9 * w * h * 4 ** aa
                hashes.append(hashlib.sha256(rgb.tobytes()).hexdigest())
        finally:
            r.close()
    assert len(set(hashes)) == 1, hashes


def test_batch_rerun_on_slot_guard_is_exact(monkeypatch):
    """A batch whose path slots (with the indirect tiles' padding to the largest indirect count
    of each 64-primary tile) exceed the 32-bit guard is re-run at half the primary samples
    instead of failing (gi_host.cpp render_pixels): with the guard lowered (GI_SLOT_LIMIT) the
    image and every counter equal the unconstrained render's. The frame is 37 x 21 (partial
    tiles), -it 96 makes the indirect counts vary inside tiles (diffuse vs glass / background)."""
    args = [scene("cornell.scn"), "/tmp/x.png", "-resolution", "37", "21", "-aa", "1",
            "-global", "20000", "-caustic", "20000", "-it", "96", "-tt", "8", "-st", "8",
            "-seed", "2"]
    p, sc, _o, w, h, aa, real = gi_amd.ParseArgs(args)
    out = []
    for lim in (None, "60000"):
        if lim:
            monkeypatch.setenv("GI_SLOT_LIMIT", lim)
        r = gi_amd.Renderer(0, p)
        try:
            r.ReadScene(sc, real)
            r.MapPhotons()
            rgb, f, st = r.RenderImage(aa, w, h, want_float=True)
            out.append((f, st, rgb))
        finally:
            r.close()
    np.testing.assert_array_equal(out[0][0], out[1][0])
    for k in ("screen_rays", "shadow_rays", "monte_carlo_rays", "transmissive_samples",
              "specular_samples", "indirect_samples", "caustic_samples", "knn_queries"):
        assert out[0][1][k] == out[1][1][k], k
    o, _ = oracle_lib.render(args, w, h)
    compare_exact(out[1][2], o)


def test_knn_instances_without_general_form_are_exact(monkeypatch):
    """The k-NN kernels run instances compiled without EstimateRadiance's general form (pow:
    specular term, cone / Gauss filters; KnnArgs::general == 0) when the host finds the disk
    filter and diffuse-only query materials (cornell.scn: the walls; the glass sphere takes no
    queries). Forcing the general instances (GI_KNN_GENERAL=1) gives the same f32 image and
    counters."""
    args = [scene("cornell.scn"), "/tmp/x.png", "-resolution", "40", "30", "-aa", "1",
            "-global", "50000", "-caustic", "100000", "-it", "16", "-tt", "8", "-st", "8",
            "-seed", "4"]
    p, sc, _o, w, h, aa, real = gi_amd.ParseArgs(args)
    out = []
    for gen in ("0", "1"):
        monkeypatch.setenv("GI_KNN_GENERAL", gen)
        r = gi_amd.Renderer(0, p)
        try:
            r.ReadScene(sc, real)
            r.MapPhotons()
            _rgb, f, st = r.RenderImage(aa, w, h, want_float=True)
            out.append((f, st))
        finally:
            r.close()
    assert np.isfinite(out[0][0]).all()
    np.testing.assert_array_equal(out[0][0], out[1][0])
    for k in ("knn_queries", "knn_photons", "caustic_samples", "indirect_samples"):
        assert out[0][1][k] == out[1][1][k], k
