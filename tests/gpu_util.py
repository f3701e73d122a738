"""Helpers shared by the -m gpu parity tests: run one reference command line through the C-ABI
(gi_amd.Renderer) and compare 8-bit images with the oracle's."""
import os

import numpy as np

import gi_amd

INP = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "scenes")


def scene(name):
    return os.path.join(INP, name)


def run_gpu(renderer, args, want_float=False):
    """ParseArgs -> ReadScene -> MapPhotons (when the flags need a map) -> RenderImage, the
    reference's main flow (photonmap.cpp:440-500). Returns (rgb8, render stats, photon stats)."""
    p, sc, _out, w, h, aa, real = gi_amd.ParseArgs(args)
    renderer.set_params(p)
    renderer.ReadScene(sc, real)
    pst = None
    if p.indirect_illum or p.caustic_illum or p.direct_photon_illum:
        pst = renderer.MapPhotons()
    if want_float:
        rgb, f, st = renderer.RenderImage(aa, w, h, want_float=True)
        return rgb, f, st, pst
    rgb, st = renderer.RenderImage(aa, w, h)
    return rgb, st, pst


# Per-pixel L2 tolerance (BASELINE.json north_star: "matches the reference CPU render within a
# stated per-pixel L2 tolerance under a fixed RNG seed"): the per-pixel L2 distance is
# sqrt(sum over RGB of (a - b)^2) in 8-bit units; its RMS over the image must stay within
# L2_RMS_TOL. (A pixel whose path diverges after a one-ulp difference can be far off, so the
# bound is on the image RMS, next to the exact / within-1-LSB fractions.) Observed on MI355X in
# r02: 0.0 in all 35 image comparisons of test_gpu_render.py / test_gpu_features.py (every
# image bit-exact; profiles/r02_parity_l2.jsonl).
L2_RMS_TOL = 0.5


def l2_stats(a, b):
    d = a.astype(float) - b.astype(float)
    l2 = np.sqrt((d * d).sum(-1))
    return float(np.sqrt((l2 * l2).mean())), float(l2.max())


def compare_exact(a, b):
    """The device image equals the oracle's bit for bit (every pixel, every channel): the two
    share the RNG streams, the operation order and, since r04, gi_math.h's transcendentals."""
    compare(a, b, 1.0, 1.0, 0.0, l2_rms_tol=0.0)


def compare(a, b, exact_frac, le1_frac, mean_tol, l2_rms_tol=None):
    """8-bit image parity: fraction of pixels exact / within 1 LSB (max over channels), the
    mean level and the RMS of the per-pixel L2 distance."""
    d = np.abs(a.astype(int) - b.astype(int))
    rms, mx = l2_stats(a, b)
    log = os.environ.get("GI_PARITY_LOG")
    if log:
        import json
        with open(log, "a") as f:
            f.write(json.dumps({"test": os.environ.get("PYTEST_CURRENT_TEST", "?"), "l2_rms": rms,
                                "l2_max": mx, "exact": float((d.max(-1) == 0).mean())}) + "\n")
    assert (d.max(-1) == 0).mean() >= exact_frac, (d.max(-1) == 0).mean()
    assert (d.max(-1) <= 1).mean() >= le1_frac, (d.max(-1) <= 1).mean()
    assert abs(a.astype(float).mean() - b.astype(float).mean()) <= mean_tol
    tol = l2_rms_tol if l2_rms_tol is not None else L2_RMS_TOL
    if tol is not None:
        assert rms <= tol, (rms, tol)
