"""The reference's own renders of its photon-map layers as statistical parity pins.

The reference ships no tests, but its README figures were rendered by the reference code with
the parameters their captions state (README.md:341-481). Those captions cover exactly the
photon-map half of the hot path:
  fig_22a-d  global map (5,000 photons) visualised directly, k = 1 / 8 / 64 / 128, r = the box
             (README.md:341-344): k-NN set + EstimateRadiance, photon power normalisation
  fig_23a-d  the same map, k = 64, r = 0.05 / 0.25 / 0.5 / 1 (README.md:346-349): the radius
             rule Q4 (photon_utils.cpp:85-96) and the pi r^2 normalisation
  fig_24a-c  caustic maps visualised: 300 / 300 k / 100 M photons, k = 10 / 200 / 500,
             r = 1 / 1 / 0.5, lights brightened (README.md:357-360)
  fig_25a-c  direct layer / caustic layer (10 M caustic photons, 225 / 0.225) / both, 512^2,
             4 samples per pixel (README.md:362-365); fig_27a and fig_30a are fig_25a's file
  fig_26a-c  -fast_global maps visualised, 300 / 300 k / 100 M photons (README.md:373-376)
  fig_27b-c  -fast_global layer (10 M photons, 225 / 0.225) and direct + it (README.md:378-381)
  fig_28     global map visualised, ~2,048 photons, 50 / 2.5, 1024^2 (README.md:390-391)
  fig_29a-c  indirect layer (MonteCarlo_IndirectSample -> global k-NN), 8 / 64 / 1,024
             samples, 512^2, 1 sample per pixel (README.md:393-396)
  fig_30b-c  indirect layer, 320 samples, 4 samples per pixel, and direct + it (README.md:398-401)
  fig_33     caustic maps (300 / 300 k / 30 M photons, k 10 / 200 / 500, r 1 / 1 / 0.5) with no
             filter / the cone filter (k = 1.25) / the Gauss filter (README.md:451-456): the only
             reference evidence for photon_utils.cpp:103-158's cone and Gauss code
The figures' scenes are input/jensen.scn (22, 23, 33: glass + mirror sphere, rect light) and
input/display.scn (24-30: + gloss sphere and frosted box): the camera, geometry and materials
match pixel for pixel (test_cpu_photon_figs.py checks the silhouettes).

Settings the captions do not state, established by fitting:
  * the photon tracer's Fresnel split is off (-no_fresnel; photontracer.cpp:82-93 with
    FRESNEL false): fig_25b misses by 11 % with it (ratio 0.888) and matches with it off (ratio
    1.001, median |z| 0.06); split by photon path, the whole deficit is the photons whose one
    specular bounce is a Fresnel reflection off the glass (fitted weight 0.12 against ~1 for
    every other path class; tools/caustic_decompose.py). fig_24b's gain fit drops from 24,679 to
    1,919 (sum of squared block residuals) with it off. Every other photon figure passes either
    way and all are rendered with it off. In these layers -no_transmissive -no_specular leave the
    renderer no Fresnel term, so the flag acts only on the photon tracer;
  * fig_24 / fig_33 ("intensity of the lights increased"): light colours x 4 (GAIN): the fitted
    factor is 4.00 on fig_24b and 4.08 on fig_33b-i;
  * aa: 4 samples per pixel (aa 1) where stated; fig_24 / fig_26 at aa 0 (their render times,
    0.16-6.9 s for 512^2, and the fit: fig_24b loss 1,919 at aa 0 vs 2,555 at aa 1); fig_33 at
    aa 1 (fit: 1,955 vs 2,905); else the default aa 2;
  * the direct layer fig_25a needs no gain: over its 1,972 purely diffuse blocks the restatement
    equals it to 0.12 LSB RMS, ratio 1.000 (so the 0.9545 gain of the point / directional-light
    figures, gallery.py, belongs to those four scene files, not to the lighting code).

Flags not in the captions: the layer is isolated with -no_direct / -no_indirect / -no_caustic
(a figure shows no other layer), and -no_transmissive -no_specular: the glass and mirror sphere
pixels do not depend on the photon maps in these layers, so they are masked out of the
comparison (every 16 x 16 block that holds a primary hit on a non-diffuse material; for the
figures with the direct layer, PURE, every block not purely diffuse: the frosted box and gloss
sphere's direct light depends on transmission / reflection) and need not be path traced.

The RNG of the reference is unseeded (RNScalar.cpp:99-131), so a figure is one random draw;
the pin is statistical (SURVEY.md 8(d) stochastic criterion): the oracle renders each figure's
configuration at S seeds; per 16 x 16 block and channel, z = (figure - mean) / sd over the
seeds; over the unsaturated blocks of diffuse surfaces the figure must have |z| < 3 on
>= Z_FRAC of them and its summed block means within RATIO_TOL of the oracle's (or within three
standard deviations of the oracle's own summed level over the seeds, where that is wider: the
300-photon maps of fig_24a / 26a / 33a vary by +-10 % in total from draw to draw).

Each configuration is rendered exactly as the figure was: the figure's resolution and aa, the
8-bit truncating quantisation per pixel (R2Image::SetPixelRGB), then both images are averaged
over the same blocks. (Rendering the blocks directly at a higher aa would skip the per-pixel
truncation, which lowers a figure's block means by up to 0.5 LSB.)
The CPU oracle renders the figures it can afford at every seed (`cpu` in FIGS); the heaviest
(fig_24c, fig_26c: 100 M photons; fig_33c: 30 M; fig_29c, fig_30b-c: 1,024 and 4 x 320
importance samples per pixel) are pinned by the GPU twin, whose renders equal the oracle's bit
for bit on the same seeds (tests/test_gpu_photon_figs.py checks that on the cheap figures).
"""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "photon_figs")
SCN = os.path.join(ROOT, "tests", "scenes")
STATS = os.path.join(GOLD, "oracle_blocks.npz")

Z_FRAC = 0.90
RATIO_TOL = 0.06
SEEDS = list(range(1, 9))

# Figures the restatement does not reproduce within the criterion, and why.
KNOWN_MISSES = {}

# fig_25b rendered WITH the photon tracer's Fresnel split (the r03 configuration): the evidence
# that the figure was not (test_fig_25b_was_traced_without_fresnel)
FRESNEL_EVIDENCE = "fig_25b+fresnel"

_NF = ["-no_fresnel"]
_PV = ["-photon_viz", "-no_direct", "-no_indirect", "-no_caustic", "-no_transmissive",
       "-no_specular", "-global", "5000"] + _NF
_IND = ["-no_direct", "-no_caustic", "-no_transmissive", "-no_specular", "-global", "2176",
        "-gs", "50", "-gd", "2.5"] + _NF
_DIR = ["-no_indirect", "-no_caustic", "-no_transmissive", "-no_specular"]
_CL = ["-no_direct", "-no_indirect", "-no_transmissive", "-no_specular"] + _NF   # caustic layer
_FG = ["-photon_viz", "-fast_global", "-no_direct", "-no_indirect", "-no_caustic",
       "-no_transmissive", "-no_specular"] + _NF


def _cau(n, k, r):
    return ["-caustic", str(n), "-cs", str(k), "-cd", str(r)]


def _glo(n, k, r):
    return ["-global", str(n), "-gs", str(k), "-gd", str(r)]


# name -> scene, figure resolution, aa, block size, rendered by the CPU oracle, reference flags
FIGS = {
    "fig_22a": ("jensen.scn", 512, 2, 16, True, _PV + ["-gs", "1", "-gd", "5.5"]),
    "fig_22b": ("jensen.scn", 512, 2, 16, True, _PV + ["-gs", "8", "-gd", "5.5"]),
    "fig_22c": ("jensen.scn", 512, 2, 16, True, _PV + ["-gs", "64", "-gd", "5.5"]),
    "fig_22d": ("jensen.scn", 512, 2, 16, True, _PV + ["-gs", "128", "-gd", "5.5"]),
    "fig_23a": ("jensen.scn", 512, 2, 16, True, _PV + ["-gs", "64", "-gd", "0.05"]),
    "fig_23b": ("jensen.scn", 512, 2, 16, True, _PV + ["-gs", "64", "-gd", "0.25"]),
    "fig_23c": ("jensen.scn", 512, 2, 16, True, _PV + ["-gs", "64", "-gd", "0.5"]),
    "fig_23d": ("jensen.scn", 512, 2, 16, True, _PV + ["-gs", "64", "-gd", "1"]),
    "fig_24a": ("display.scn", 512, 0, 16, True, _CL + _cau(300, 10, 1)),
    "fig_24b": ("display.scn", 512, 0, 16, True, _CL + _cau(300000, 200, 1)),
    "fig_24c": ("display.scn", 512, 0, 16, False, _CL + _cau(100000000, 500, 0.5)),
    "fig_25a": ("display.scn", 512, 1, 16, True, _DIR),
    "fig_25b": ("display.scn", 512, 1, 16, True, _CL + _cau(10000000, 225, 0.225)),
    "fig_25c": ("display.scn", 512, 1, 16, True,
                ["-no_indirect", "-no_transmissive", "-no_specular"] + _NF +
                _cau(10000000, 225, 0.225)),
    "fig_26a": ("display.scn", 512, 0, 16, True, _FG + _glo(300, 10, 1)),
    "fig_26b": ("display.scn", 512, 0, 16, True, _FG + _glo(300000, 200, 1)),
    "fig_26c": ("display.scn", 512, 0, 16, False, _FG + _glo(100000000, 500, 0.5)),
    "fig_27b": ("display.scn", 512, 1, 16, True, _FG + _glo(10000000, 225, 0.225)),
    "fig_27c": ("display.scn", 512, 1, 16, True,
                ["-photon_viz", "-fast_global", "-no_indirect", "-no_caustic", "-no_transmissive",
                 "-no_specular"] + _NF + _glo(10000000, 225, 0.225)),
    "fig_28": ("display.scn", 1024, 0, 32, True,
               ["-photon_viz", "-no_direct", "-no_indirect", "-no_caustic", "-no_transmissive",
                "-no_specular", "-global", "2176", "-gs", "50", "-gd", "2.5"] + _NF),
    "fig_29a": ("display.scn", 512, 0, 16, True, _IND + ["-it", "8"]),
    "fig_29b": ("display.scn", 512, 0, 16, True, _IND + ["-it", "64"]),
    "fig_29c": ("display.scn", 512, 0, 16, False, _IND + ["-it", "1024"]),
    "fig_30b": ("display.scn", 512, 1, 16, False, _IND + ["-it", "320"]),
    "fig_30c": ("display.scn", 512, 1, 16, False,
                ["-no_caustic", "-no_transmissive", "-no_specular", "-global", "2176", "-gs",
                 "50", "-gd", "2.5", "-it", "320"] + _NF),
}
_FILTERS = {"i": [], "ii": ["-cf", "cone", "1.25"], "iii": ["-cf", "gauss"]}
for _row, (_n, _k, _r, _cpu) in {"a": (300, 10, 1, True), "b": (300000, 200, 1, True),
                                 "c": (30000000, 500, 0.5, False)}.items():
    for _col, _filt in _FILTERS.items():
        FIGS[f"fig_33{_row}-{_col}"] = ("jensen.scn", 512, 1, 16, _cpu,
                                        _CL + _cau(_n, _k, _r) + _filt)

# Calibration figures: the figures a setting the captions do not state was fitted
# on. They pass partly by construction, so they are counted as calibrations, not as independent
# pins; every other figure is held out (DESIGN.md 6.1 "role").
CALIBRATION = {
    "fig_24b": "light gain 4 fitted on it (4.00) and -no_fresnel chosen with it",
    "fig_33b-i": "light gain fitted on it (4.08; 4 used)",
    "fig_25b": "-no_fresnel chosen on it (the r03 miss)",
}


def role(name):
    return "calibration" if name.split("+")[0] in CALIBRATION else "held-out"


# light colours x GAIN (the captions' "intensity of the lights ... increased")
GAIN = {n: 4.0 for n in FIGS if n.startswith(("fig_24", "fig_33"))}
# figures with the direct layer: mask every block that is not purely diffuse
PURE = {"fig_25a", "fig_25c", "fig_27c", "fig_30c"}
# seeds per figure where not len(SEEDS): four for the 100 M-photon figures (each map takes ~10 s
# to trace on the GPU); 32 for the 300-photon maps, whose summed level varies by +-10 % from draw
# to draw, so that the level tolerance (three standard deviations over the seeds) is estimated
# from enough draws
N_SEEDS = {"fig_24c": 4, "fig_26c": 4, "fig_24a": 32, "fig_26a": 32, "fig_33a-i": 32,
           "fig_33a-ii": 32, "fig_33a-iii": 32}

# fig_25b with the Fresnel split on (FRESNEL_EVIDENCE): the r03 configuration
EVIDENCE = {FRESNEL_EVIDENCE: ("display.scn", 512, 1, 16, True,
                               [f for f in FIGS["fig_25b"][5] if f != "-no_fresnel"])}


def config(name):
    return FIGS[name] if name in FIGS else EVIDENCE[name]


def scene_path(name, tmp_dir=None):
    """The figure's scene file; a copy with the lights x GAIN[name] where the figure was
    rendered brighter (written to tmp_dir)."""
    import tempfile
    scene = config(name)[0]
    if name not in GAIN:
        return os.path.join(SCN, scene)
    import gallery
    return gallery.gained_scene(scene, GAIN[name], tmp_dir or tempfile.gettempdir())


def render_args(name, seed, threads=None, tmp_dir=None):
    """Reference command line of figure `name`'s configuration at `seed`.
    Returns (args, width, height)."""
    _scene, res, aa, _B, _cpu, flags = config(name)
    args = [scene_path(name, tmp_dir), "/tmp/pf.png", "-resolution", str(res), str(res), "-aa",
            str(aa), "-seed", str(seed)] + flags
    if threads:
        args += ["-threads", str(threads)]
    return args, res, res


def seeds(name):
    return list(range(1, 1 + N_SEEDS.get(name, len(SEEDS))))


def blocks(img_top_down, name):
    """Block means [n, n, 3] of an 8-bit image in file (top-down) row order."""
    _scene, res, _aa, B, _cpu, _f = config(name)
    n = res // B
    return img_top_down.astype(float).reshape(n, B, n, B, 3).mean((1, 3))


def figure_file(name):
    """The committed figure of `name` (fig_27a / fig_30a are fig_25a's file; the evidence
    configurations use their figure's)."""
    return os.path.join(GOLD, name.split("+")[0] + ".png")


def figure_blocks(name):
    """Block means of the committed figure."""
    from pngio import read_png
    return blocks(read_png(figure_file(name))[..., :3], name)


def render_blocks(rgb_bottom_up, name):
    """Block means of a render (rows bottom-up, as R2Image) in figure row order."""
    return blocks(rgb_bottom_up[::-1], name)


def camera_rays(scene_path, W, H):
    """Primary rays through the pixel grid, Threadable_RayTracer (render.cpp:64-98) with the
    R3Triad camera axes (R3Triad.cpp:72-79), the default focus depth 100 and yfov = xfov
    (R3Scene.cpp:1892). Rows bottom-up."""
    cam = None
    for line in open(scene_path):
        t = line.split()
        if t and t[0] == "camera":
            cam = [float(x) for x in t[1:11]]
    e, tw, up, xfov = np.array(cam[0:3]), np.array(cam[3:6]), np.array(cam[6:9]), cam[9]
    tw = tw / np.linalg.norm(tw)
    z = -tw
    r = np.cross(up, z)
    r /= np.linalg.norm(r)
    u = np.cross(z, r)
    F = 100.0
    i, j = np.meshgrid(np.arange(W), np.arange(H))
    dx = 2.0 * (i - W // 2) / W
    dy = 2.0 * (j - H // 2) / H
    fp = (e + tw * F)[None, None] + r * (np.tan(xfov) * F * dx)[..., None] \
        + u * (np.tan(xfov) * F * dy)[..., None]
    d = fp - e
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    o = np.broadcast_to(e, d.shape).reshape(-1, 3).copy()
    return o, d.reshape(-1, 3)


def materials(scene_path):
    """[(max Kd, purely diffuse)] per material id, id -1 last (R3default_brdf: Kd 0.8,
    R3Brdf.cpp:13-15). Material lines: ka kd ks kt ke n ir texture (R3Scene.cpp:1607-1650)."""
    out = []
    for line in open(scene_path):
        t = line.split()
        if t and t[0] == "material":
            v = [float(x) for x in t[1:16]]
            out.append((max(v[3:6]), max(v[3:6]) > 0 and max(v[6:15]) == 0))
    return out + [(0.8, True)]


def material_kd(scene_path):
    return np.array([m[0] for m in materials(scene_path)])


def diffuse_hit_mask(scene_path, W, H, intersect, pure=False):
    """[H, W] top-down: True where the primary ray hits a diffuse material (the only pixels a
    photon-map layer can light); with `pure`, a purely diffuse one (no Ks, Kt or emission).
    `intersect` = oracle_lib.intersect or the device's."""
    o, d = camera_rays(scene_path, W, H)
    hit, _t, _p, _n, m = intersect(scene_path, o, d)
    mats = materials(scene_path)
    ok_m = np.array([(p if pure else kd > 0) for kd, p in mats])
    ok = np.where(hit > 0, ok_m[m], False)
    return ok.reshape(H, W)[::-1]


def block_mask(name, intersect):
    """Blocks entirely on diffuse (PURE figures: purely diffuse) surfaces, [n, n] top-down."""
    scene, res, _aa, B, _cpu, _f = config(name)
    m = diffuse_hit_mask(os.path.join(SCN, scene), res, res, intersect,
                         pure=name.split("+")[0] in PURE)
    n = res // B
    return m.reshape(n, B, n, B).all((1, 3))


def pin(fig_b, seed_b, mask):
    """Statistical pin of a figure's block means against renders at several seeds.
    fig_b [n, n, 3], seed_b [S, n, n, 3], mask [n, n]. Returns a dict of the criterion's
    quantities; `ok` = the figure passes."""
    mu = seed_b.mean(0)
    sd = seed_b.std(0, ddof=1)
    use = mask[..., None] & (fig_b < 250) & (mu < 250) & (fig_b + mu > 0)
    z = (fig_b - mu) / np.maximum(sd, 0.5)
    az = np.abs(z[use])
    ratio = float(fig_b[use].sum() / max(mu[use].sum(), 1e-9))
    frac = float((az < 3).mean())
    # level tolerance: RATIO_TOL, or three standard deviations of the restatement's own summed
    # level over the seeds where that is wider (a 300-photon map's total varies +-10 % per draw)
    tot = np.array([b[use].sum() for b in seed_b])
    tol = max(RATIO_TOL, 3.0 * float(tot.std(ddof=1) / max(tot.mean(), 1e-9)))
    return {"z_frac": frac, "median_abs_z": float(np.median(az)), "ratio": ratio,
            "ratio_tol": round(tol, 4), "blocks": int(use.sum()),
            "ok": frac >= Z_FRAC and abs(ratio - 1) <= tol}


def leave_one_out(seed_b, mask):
    """The same statistic with each seed in turn playing the figure against the others: what
    a draw of the restatement itself scores (the criterion's calibration)."""
    out = []
    for j in range(len(seed_b)):
        rest = np.delete(seed_b, j, axis=0)
        out.append(pin(seed_b[j], rest, mask))
    return out
