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


def compare(a, b, exact_frac, le1_frac, mean_tol):
    """8-bit image parity: fraction of pixels exact / within 1 LSB (max over channels) and the
    mean level."""
    d = np.abs(a.astype(int) - b.astype(int))
    assert (d.max(-1) == 0).mean() >= exact_frac, (d.max(-1) == 0).mean()
    assert (d.max(-1) <= 1).mean() >= le1_frac, (d.max(-1) <= 1).mean()
    assert abs(a.astype(float).mean() - b.astype(float).mean()) <= mean_tol
