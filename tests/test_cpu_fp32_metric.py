"""What the fp32 photon positions and fp32 k-NN metric change against the reference's fp64 ones
(VERDICT r03 weak 1).

The reference stores each photon's hit point as an fp64 R3Point and ranks neighbours by the fp64
R3SquaredDistance (photon_utils.cpp:53-54, R3Kdtree.cpp:688-784). This repo (device and oracle)
stores fp32 positions and ranks by the fp32 metric fma(dz,dz, fma(dy,dy, dx*dx)). On C2's maps
(cornell.scn, 1M global + 1M caustic photons, K = 50 / 225, r = 2.5 / 0.225) and 4,096 primary
hit points of the C2 frame this test measures, per map:
  - metric only: the oracle's fp32 K-set vs the exact fp64 K-set of the same fp32 positions;
  - metric + positions: the same against fp64 positions drawn uniformly inside each fp32
    position's rounding cell (the reference's unknown fp64 originals round to the stored fp32
    values, so they lie in that cell);
the fraction of queries whose K-set changes and the relative change of the disk-filter estimate
sum(power * |N.I|) / (pi r^2) (photon_utils.cpp:85-150). Printed numbers are in DESIGN.md 5."""
import os

import numpy as np
import pytest
from scipy.spatial import cKDTree

import oracle_lib
import photon_figs as pf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCN = os.path.join(ROOT, "tests", "scenes", "cornell.scn")
NQ = 4096


def rgbe_to_rgb(b):
    """RGBE_to_RNRgb (graphics_utils.cpp:64-77), vectorised."""
    e = b[:, 3].astype(int)
    s = np.where(e > 0, np.ldexp(1.0, e - 136), 0.0)
    return b[:, :3].astype(float) * s[:, None]


def estimate(idx, d2, nf, k, r, ph_rgb, inc, normal, cos_theta):
    """Disk-filter EstimateRadiance (photon_utils.cpp:72-162) without the BRDF factor kd."""
    out = np.zeros((len(idx), 3))
    for q in range(len(idx)):
        n = nf[q]
        if n == 0:
            continue
        sel = idx[q, :n]
        r2 = r * r if n < k else max(float(d2[q, :n].max()), 1e-6)
        perp = inc[sel] @ normal[q]
        keep = ~(((cos_theta[q] < 0) & (perp < 0)) | ((cos_theta[q] > 0) & (perp > 0)))
        out[q] = (ph_rgb[sel][keep] * np.abs(perp[keep])[:, None]).sum(0) / (np.pi * r2)
    return out


def fp64_knn(pos64, pts, k, r):
    """Exact fp64 K-nearest within r (ties by index, as the oracle's sorted output)."""
    tree = cKDTree(pos64)
    d, i = tree.query(pts, k=k, distance_upper_bound=r)
    nf = np.isfinite(d).sum(1)
    d2 = np.where(np.isfinite(d), d * d, -1.0)
    i = np.where(np.isfinite(d), i, -1)
    return i.astype(np.int64), d2, nf


def in_cell(pos32, rng):
    """fp64 points uniformly inside each fp32 value's rounding cell."""
    p = pos32.astype(np.float64)
    up = np.nextafter(pos32, np.float32(np.inf)).astype(np.float64)
    dn = np.nextafter(pos32, np.float32(-np.inf)).astype(np.float64)
    lo, hi = (p + dn) / 2, (p + up) / 2
    return lo + (hi - lo) * rng.random(p.shape)


@pytest.fixture(scope="module")
def c2_maps():
    args = [SCN, "/tmp/x.png", "-global", "1000000", "-caustic", "1000000", "-seed", "1",
            "-threads", str(len(os.sched_getaffinity(0)))]
    g, c, _em = oracle_lib.map_photons(args)
    return g, c


@pytest.fixture(scope="module")
def c2_queries():
    """Primary hits at NQ random pixels of the 1024^2 C2 frame (every cornell surface is
    diffuse except the two spheres, whose hits are dropped)."""
    o, d = pf.camera_rays(SCN, 1024, 1024)
    rng = np.random.default_rng(7)
    pick = rng.choice(len(o), NQ * 2, replace=False)
    hit, _t, p, n, m = oracle_lib.intersect(SCN, o[pick], d[pick])
    kd = pf.material_kd(SCN)
    ok = (hit > 0) & (kd[m] > 0)
    p, n, dd = p[ok][:NQ], n[ok][:NQ], d[pick][ok][:NQ]
    cos_theta = (n * -dd).sum(1)
    return p, n, cos_theta


@pytest.mark.parametrize("which,k,r", [("global", 50, 2.5), ("caustic", 225, 0.225)])
def test_fp32_metric_effect_on_c2(c2_maps, c2_queries, which, k, r):
    ph = c2_maps[0] if which == "global" else c2_maps[1]
    pts, normal, cos_theta = c2_queries
    lut = oracle_lib.direction_lut()
    inc = lut[ph["dir"].astype(int)]
    rgb = rgbe_to_rgb(ph["rgbe"])
    i32, d32, n32 = oracle_lib.knn(ph, pts, k, r)
    e32 = estimate(i32, d32, n32, k, r, rgb, inc, normal, cos_theta)
    res = {}
    for name, pos in (("metric", ph["pos"].astype(np.float64)),
                      ("metric+positions", in_cell(ph["pos"], np.random.default_rng(3)))):
        i64, d64, n64 = fp64_knn(pos, pts, k, r)
        e64 = estimate(i64, d64, n64, k, r, rgb, inc, normal, cos_theta)
        changed = np.array([set(i32[q, :n32[q]]) != set(i64[q, :n64[q]]) for q in range(len(pts))])
        den = np.abs(e64).sum(1)
        rel = np.abs(e32 - e64).sum(1) / np.maximum(den, 1e-300)
        rel = rel[den > 0]
        res[name] = (changed.mean(), float(np.median(rel)), float(rel.max()),
                     float((n32 != n64).mean()))
        print(f"\n{which} K={k}: {name}: K-set changed {changed.mean():.4%} of {len(pts)} "
              f"queries, count changed {(n32 != n64).mean():.4%}, estimate rel. change median "
              f"{np.median(rel):.2e} max {rel.max():.2e}")
        # the fp32 metric is a rounding-level perturbation: sets move only at near-ties
        assert changed.mean() < 0.02
        assert rel.max() < 0.05
    assert (n32 > 0).mean() > 0.9
