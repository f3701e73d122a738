"""The oracle restatement pinned against what the reference itself produced: its gallery figures
(tests/gallery.py explains how they were rendered and the one global gain between figure and
code) and pixel values computed by hand from the reference's light formulas."""
import numpy as np
import pytest

import gallery
import oracle_lib


@pytest.mark.parametrize("fig", sorted(gallery.PINNED))
def test_gallery_figure_pins_restatement(fig, tmp_path):
    """Mask: pixels unsaturated in either image. Tolerance: 1 LSB on >= 99.3 % of them (one global
    gain cannot reproduce every truncation boundary), exact on >= 85 %, and the black (shadow /
    back-facing / outside) mask equal on >= 99.9 % of all pixels."""
    scn = gallery.gained_scene(gallery.PINNED[fig], gallery.LIGHT_GAIN, str(tmp_path))
    rgb, _ = oracle_lib.render([scn, "/tmp/x.png"] + gallery.FIG_ARGS + ["-threads", "8"],
                               512, 512)
    s = gallery.pin_stats(rgb, gallery.figure(fig))
    assert s["n_unsat"] > 10000, s
    assert s["within1_unsat"] >= 0.993, s
    assert s["exact_unsat"] >= 0.85, s
    assert s["zero_agree"] >= 0.999, s


def test_gallery_needs_the_gain_and_no_mirror_term(tmp_path):
    """The two departures are real: without the gain, or with the glossy mirror term on, the same
    comparison fails (so the pin is not loose enough to accept anything)."""
    fig = gallery.figure("fig_7b")
    base = [gallery.gained_scene("dirlight2.scn", 1.0, str(tmp_path)), "/tmp/x.png"]
    rgb, _ = oracle_lib.render(base + gallery.FIG_ARGS + ["-threads", "8"], 512, 512)
    assert gallery.pin_stats(rgb, fig)["within1_unsat"] < 0.2
    scn = gallery.gained_scene("dirlight2.scn", gallery.LIGHT_GAIN, str(tmp_path))
    args = [a for a in gallery.FIG_ARGS if a != "-no_specular"] + ["-st", "16"]
    rgb, _ = oracle_lib.render([scn, "/tmp/x.png"] + args + ["-threads", "8"], 512, 512)
    assert gallery.pin_stats(rgb, fig)["within1_unsat"] < 0.97


def test_spot_figures_come_from_other_scene_files():
    """fig_6a shows the sphere lit; with spotlight1.scn as shipped (spot at (-0.866, 2, 0.5)
    aimed at (0,-1,0), cutoff 0.331 rad) every sphere point lies outside the cone, so the
    current reference (R3SpotLight::IntensityAtPoint, R3SpotLight.cpp:105-115) leaves it black."""
    P = np.array([-0.866, 2.0, 0.5])
    D = np.array([0.0, -1.0, 0.0])
    rng = np.random.default_rng(0)
    v = rng.normal(size=(20000, 3))
    pts = gallery.SPHERE_C + gallery.SPHERE_R * v / np.linalg.norm(v, axis=1, keepdims=True)
    ml = pts - P
    cos_a = (ml / np.linalg.norm(ml, axis=1, keepdims=True)) @ D
    assert (cos_a < np.cos(0.331)).all()
    fig = gallery.figure("fig_6a")
    # the sphere's disc in the figure (centre column/row 256, radius ~ 0.2 / (2 tan 0.25) * 256)
    assert fig[200:260, 256:300, :].max() >= 200


@pytest.mark.parametrize("scene,light", [
    ("dirlight1.scn", ("dir", 1.0, np.array([0.710, -0.580, -0.410]))),
    # pointlight2: the blue channel comes only from its (0 0 2) light at (-0.866, 1, 0.5)
    ("pointlight2.scn", ("point", 2.0, np.array([-0.866, 1.0, 0.5])))])
def test_known_answer_floor_pixels(scene, light):
    """Floor pixels computed by hand from the reference formulas (tests/gallery.py
    floor_known_answers) equal the restatement's 8-bit output exactly."""
    exp = gallery.floor_known_answers(light, 64, 64)
    assert len(exp) > 1000
    rgb, _ = oracle_lib.render([gallery.SCN + "/" + scene, "/tmp/x.png", "-resolution", "64",
                                "64", "-aa", "0", "-no_indirect", "-no_caustic",
                                "-no_specular"], 64, 64)
    got = np.array([rgb[j, i, 2] for i, j, _ in exp])
    want = np.array([v for _, _, v in exp])
    assert (got == want).all(), np.nonzero(got != want)
    assert len(set(want.tolist())) >= 5  # not a flat field: attenuation / angle / specular vary
