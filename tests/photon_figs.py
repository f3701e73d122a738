"""The reference's own renders of its photon-map layers as statistical parity pins.

The reference ships no tests, but its README figures were rendered by the reference code with
the parameters their captions state (README.md:341-401). Those captions cover exactly the
photon-map half of the hot path:
  fig_22a-d  global map (5,000 photons) visualised directly, k = 1 / 8 / 64 / 128, r = the box
             (README.md:341-344): k-NN set + EstimateRadiance, photon power normalisation
  fig_23a-d  the same map, k = 64, r = 0.05 / 0.25 / 0.5 / 1 (README.md:346-349): the radius
             rule Q4 (photon_utils.cpp:85-96) and the pi r^2 normalisation
  fig_25b    caustic layer, 10 M caustic photons, 225 / 0.225, 512^2, 4 samples per pixel
             (README.md:362-365)
  fig_28     global map visualised, ~2,048 photons, 50 / 2.5, 1024^2 (README.md:390-391)
  fig_29a-c  indirect layer (MonteCarlo_IndirectSample -> global k-NN), 8 / 64 / 1,024
             samples, 512^2, 1 sample per pixel (README.md:393-396)
  fig_30b    indirect layer, 320 samples, 512^2, 4 samples per pixel (README.md:398-401)
The figures' scenes are input/jensen.scn (22, 23: glass + mirror sphere, rect light) and
input/display.scn (25, 28-30: + gloss sphere and frosted box): the camera, geometry and
materials match pixel for pixel (test_cpu_photon_figs.py checks the silhouettes).

Flags not in the captions: the layer is isolated with -no_direct / -no_indirect / -no_caustic
(a figure shows no other layer), and -no_transmissive -no_specular: the glass and mirror sphere
pixels do not depend on the photon maps in these layers, so they are masked out of the
comparison (every 16 x 16 block that holds a primary hit on a non-diffuse material) and need
not be path traced. aa is the caption's where stated (1 spp = aa 0, 4 = aa 1), else the
reference's default aa 2 (the direct-lighting figures were rendered at aa 2, gallery.py).

The RNG of the reference is unseeded (RNScalar.cpp:99-131), so a figure is one random draw;
the pin is statistical (SURVEY.md 8(d) stochastic criterion): the oracle renders each figure's
configuration at S seeds; per 16 x 16 block and channel, z = (figure - mean) / sd over the
seeds; over the unsaturated blocks of diffuse surfaces the figure must have |z| < 3 on
>= Z_FRAC of them and its summed block means within RATIO_TOL of the oracle's (no gain: unlike
the direct-lighting figures, these need none).

Each configuration is rendered exactly as the figure was: the figure's resolution and aa, the
8-bit truncating quantisation per pixel (R2Image::SetPixelRGB), then both images are averaged
over the same blocks. (Rendering the blocks directly at a higher aa would skip the per-pixel
truncation, which lowers a figure's block means by up to 0.5 LSB: 15 % of fig_25b's level.)
The CPU oracle renders the figures it can afford at every seed (`cpu` in FIGS); the two
heaviest indirect layers (fig_29c, fig_30b: 1,024 and 4 x 320 importance samples per pixel)
are pinned by the GPU twin, whose renders equal the oracle's bit for bit on the same seeds
(tests/test_gpu_photon_figs.py checks that on the cheap figures).
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
KNOWN_MISSES = {
    "fig_25b": "the caustic layer matches where it is bright (blocks >= 10 LSB: figure / "
               "restatement 1.01-1.02) but the faint wall caustics (< 3 LSB) sit 0.2-0.35 LSB "
               "lower in the figure; 8-bit truncation of every subsample (an older RenderImage) "
               "does not explain it (ratio 0.888 -> 0.915); not reproduced",
}

_PV = ["-photon_viz", "-no_direct", "-no_indirect", "-no_caustic", "-no_transmissive",
       "-no_specular", "-global", "5000"]
_IND = ["-no_direct", "-no_caustic", "-no_transmissive", "-no_specular", "-global", "2176",
        "-gs", "50", "-gd", "2.5"]

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
    "fig_25b": ("display.scn", 512, 1, 16, True,
                ["-no_direct", "-no_indirect", "-no_transmissive", "-no_specular", "-caustic",
                 "10000000", "-cs", "225", "-cd", "0.225"]),
    "fig_28": ("display.scn", 1024, 0, 32, True,
               ["-photon_viz", "-no_direct", "-no_indirect", "-no_caustic", "-no_transmissive",
                "-no_specular", "-global", "2176", "-gs", "50", "-gd", "2.5"]),
    "fig_29a": ("display.scn", 512, 0, 16, True, _IND + ["-it", "8"]),
    "fig_29b": ("display.scn", 512, 0, 16, True, _IND + ["-it", "64"]),
    "fig_29c": ("display.scn", 512, 0, 16, False, _IND + ["-it", "1024"]),
    "fig_30b": ("display.scn", 512, 1, 16, False, _IND + ["-it", "320"]),
}


def render_args(name, seed, threads=None):
    """Reference command line of figure `name`'s configuration at `seed`.
    Returns (args, width, height)."""
    scene, res, aa, _B, _cpu, flags = FIGS[name]
    args = [os.path.join(SCN, scene), "/tmp/pf.png", "-resolution", str(res), str(res), "-aa",
            str(aa), "-seed", str(seed)] + flags
    if threads:
        args += ["-threads", str(threads)]
    return args, res, res


def blocks(img_top_down, name):
    """Block means [n, n, 3] of an 8-bit image in file (top-down) row order."""
    _scene, res, _aa, B, _cpu, _f = FIGS[name]
    n = res // B
    return img_top_down.astype(float).reshape(n, B, n, B, 3).mean((1, 3))


def figure_blocks(name):
    """Block means of the committed figure."""
    from pngio import read_png
    return blocks(read_png(os.path.join(GOLD, name + ".png"))[..., :3], name)


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


def material_kd(scene_path):
    kd = []
    for line in open(scene_path):
        t = line.split()
        if t and t[0] == "material":
            kd.append(max(float(x) for x in t[4:7]))
    return np.array(kd + [0.8])  # id -1 -> R3default_brdf, Kd 0.8 (R3Brdf.cpp:13-15)


def diffuse_hit_mask(scene_path, W, H, intersect):
    """[H, W] top-down: True where the primary ray hits a diffuse material (the only pixels a
    photon-map layer can light). `intersect` = oracle_lib.intersect or the device's."""
    o, d = camera_rays(scene_path, W, H)
    hit, _t, _p, _n, m = intersect(scene_path, o, d)
    kd = material_kd(scene_path)
    ok = np.where(hit > 0, kd[m] > 0, False)
    return ok.reshape(H, W)[::-1]


def block_mask(name, intersect):
    """Blocks entirely on diffuse surfaces, [n, n] top-down."""
    scene, res, _aa, B, _cpu, _f = FIGS[name]
    m = diffuse_hit_mask(os.path.join(SCN, scene), res, res, intersect)
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
    return {"z_frac": frac, "median_abs_z": float(np.median(az)), "ratio": ratio,
            "blocks": int(use.sum()), "ok": frac >= Z_FRAC and abs(ratio - 1) <= RATIO_TOL}


def leave_one_out(seed_b, mask):
    """The same statistic with each seed in turn playing the figure against the others: what
    a draw of the restatement itself scores (the criterion's calibration)."""
    out = []
    for j in range(len(seed_b)):
        rest = np.delete(seed_b, j, axis=0)
        out.append(pin(seed_b[j], rest, mask))
    return out
