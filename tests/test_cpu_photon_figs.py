"""The photon-map layers of the oracle restatement pinned on the reference's own figures
(tests/photon_figs.py explains the figures, their flags and the statistic).

The oracle's renders at photon_figs.SEEDS are committed (tests/golden/photon_figs/
oracle_blocks.npz, made by tools/photon_figs_oracle.py): they take ~20 min of CPU. Here:
- every figure with oracle seeds passes the statistical pin, except the ones listed in
  KNOWN_MISSES with the reason (DESIGN.md section 6 reports every figure's numbers);
- the criterion is attainable: each oracle seed, standing in for the figure against the other
  seeds, passes it too (leave-one-out);
- the committed blocks are the current oracle's: seed 1 of three cheap figures is re-rendered
  and must give the committed block means exactly;
- the figures show the scenes named for them: display.scn's glass and mirror spheres are black
  in the figures rendered without transmission/specular (camera, geometry, materials agree).
"""
import numpy as np
import pytest

import oracle_lib
import photon_figs as pf

STATS = dict(np.load(pf.STATS))
WITH_SEEDS = [n for n in pf.FIGS if n + "/seeds" in STATS]

KNOWN_MISSES = pf.KNOWN_MISSES


def _pin(name):
    return pf.pin(STATS[name + "/figure"].astype(float), STATS[name + "/seeds"].astype(float),
                  STATS[name + "/mask"])


def test_every_figure_has_stats():
    for n in pf.FIGS:
        assert n + "/figure" in STATS and n + "/mask" in STATS, n
        if pf.FIGS[n][4]:
            assert STATS[n + "/seeds"].shape[0] == len(pf.seeds(n)), n
    assert len(WITH_SEEDS) >= 25


@pytest.mark.parametrize("name", WITH_SEEDS)
def test_figure_pin(name):
    r = _pin(name)
    if name in KNOWN_MISSES:
        pytest.xfail(KNOWN_MISSES[name] + f" ({r})")
    assert r["blocks"] > 0.5 * STATS[name + "/mask"].size * 3 * 0.5, r
    assert r["ok"], r


@pytest.mark.parametrize("name", WITH_SEEDS)
def test_criterion_is_attainable(name):
    """Each oracle seed as the 'figure' against the other seeds: at most one of the eight may
    miss, else the criterion would be stricter than the restatement's own spread."""
    loo = pf.leave_one_out(STATS[name + "/seeds"].astype(float), STATS[name + "/mask"])
    assert sum(not r["ok"] for r in loo) <= 1, [round(r["z_frac"], 3) for r in loo]


@pytest.mark.parametrize("name", ["fig_23a", "fig_28", "fig_29a", "fig_26a", "fig_33a-ii"])
def test_committed_blocks_are_the_oracles(name):
    args, w, h = pf.render_args(name, pf.SEEDS[0], threads=8)
    rgb, _ = oracle_lib.render(args, w, h)
    np.testing.assert_array_equal(pf.render_blocks(rgb, name).astype(np.float32),
                                  STATS[name + "/seeds"][0])


def test_fig_25b_was_traced_without_fresnel():
    """The caustic layer fig_25b (README.md:362-365) against the restatement with the photon
    tracer's Fresnel split on (photontracer.cpp:82-93, FRESNEL true: the r03 configuration,
    committed as FRESNEL_EVIDENCE) and off (-no_fresnel): on, the figure's level is 0.888 of the
    restatement's and the pin fails; off, it is within 1 % and 99 % of the blocks sit within
    |z| < 3. The per-path split (tools/caustic_decompose.py path:) puts the whole
    deficit on the photons whose one specular bounce is a Fresnel reflection off the glass."""
    on = _pin(pf.FRESNEL_EVIDENCE)
    off = _pin("fig_25b")
    assert not on["ok"] and on["ratio"] < 0.92, on
    assert off["ok"] and abs(off["ratio"] - 1) < 0.01 and off["z_frac"] > 0.99, off


def test_direct_layer_needs_no_gain():
    """fig_25a (= fig_27a = fig_30a), display.scn's direct layer under its rect light: the
    restatement matches it at gain 1 (ratio within 1 %), so the 0.9545 gain of the
    point / directional-light figures (gallery.py) is not a property of the lighting code."""
    r = _pin("fig_25a")
    assert r["ok"] and abs(r["ratio"] - 1) < 0.01, r


@pytest.mark.parametrize("row", ["a", "b"])
def test_filters_share_the_unfiltered_gain(row):
    """fig_33 row `row` (README.md:451-456): the cone (k = 1.25) and Gauss filtered caustic
    layers pass at the same light gain as the unfiltered one (GAIN, fitted on none of them
    separately), so their normalisations (photon_utils.cpp:103-158) match the reference's."""
    rs = [_pin(f"fig_33{row}-{c}") for c in ("i", "ii", "iii")]
    assert all(r["ok"] for r in rs), rs


@pytest.mark.parametrize("name", ["fig_28", "fig_29a", "fig_29c", "fig_30b"])
def test_figures_show_the_named_scene(name):
    """display.scn's glass and mirror spheres (Kd = 0) are black in these figures: the primary
    hits the restatement's camera and geometry put on them are black in the figure too."""
    from pngio import read_png
    import os
    scene, res, _aa, _B, _cpu, _f = pf.FIGS[name]
    diffuse = pf.diffuse_hit_mask(os.path.join(pf.SCN, scene), res, res, oracle_lib.intersect)
    o, d = pf.camera_rays(os.path.join(pf.SCN, scene), res, res)
    hit = oracle_lib.intersect(os.path.join(pf.SCN, scene), o, d)[0].reshape(res, res)[::-1]
    nondiff = (~diffuse) & (hit > 0)
    # away from silhouettes (anti-aliased edges and the spheres' soft indirect glow)
    core = nondiff.copy()
    for ax in (0, 1):
        for s in (-2, 2):
            core &= np.roll(nondiff, s, axis=ax)
    fig = read_png(os.path.join(pf.GOLD, name + ".png"))[..., :3].max(-1)
    assert core.sum() > 0.02 * res * res
    assert (fig[core] <= 8).mean() > 0.97, (fig[core] <= 8).mean()
    assert fig[diffuse].mean() > 10


def test_calibration_figures_are_named():
    """The figures the unstated settings were fitted on are marked (photon_figs.CALIBRATION),
    and the held-out pins outnumber them."""
    assert set(pf.CALIBRATION) <= set(pf.FIGS)
    held = [n for n in pf.FIGS if pf.role(n) == "held-out"]
    assert len(held) >= 30 and len(pf.CALIBRATION) == 3

