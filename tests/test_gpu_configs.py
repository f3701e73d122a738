"""BASELINE configs C3, C4 and C5 with their exact flags against committed oracle fixtures
(tests/golden/configs/*.npz, written by tools/make_config_fixtures.py in the build container),
plus full-size property checks of each config.

Each fixture is the config's command line verbatim (photon-map sizes, aa, DOF; every other flag
at the reference default, photonmap.cpp:27-106) at an oracle-sized resolution. The device render
must equal the oracle's image bit for bit (compare_exact), with equal stored photon counts and
equal render counters (screen, shadow and Monte Carlo rays, sample fans, k-NN queries and photons
returned): both sides share the RNG streams, the operation order and gi_math.h. No CPU rendering
runs on the GPU box for these.

  C3  jensen.scn    aa 2, -caustic 4000000: -lt/-ss 128 rect-light fans (the occluder mask),
                    -it 256, -tt/-st 128 through the glass and mirror spheres
  C4  stilllife.scn aa 2, -global 2000000 with the default 10 M caustic map
  C5  teapot.scn    aa 3, -global 8000000 -dof 4 12.2282 0.025 -no_caustic
"""
import hashlib
import json
import os

import numpy as np
import pytest

import gi_amd
from gpu_util import compare_exact, run_gpu, scene

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "configs")
COUNTERS = ("screen_rays", "shadow_rays", "monte_carlo_rays", "transmissive_samples",
            "specular_samples", "indirect_samples", "caustic_samples", "knn_queries",
            "knn_photons")


def fixture(cid):
    z = np.load(os.path.join(GOLD, cid + ".npz"))
    args = [str(x) for x in z["args"]]
    args[0] = scene(args[0])
    return args, z["rgb"], json.loads(str(z["stats"]))


@pytest.mark.parametrize("cid", ["c3", "c4", "c5"])
def test_config_matches_oracle_fixture(renderer, cid):
    args, rgb_o, ost = fixture(cid)
    g, gst, gp = run_gpu(renderer, args)
    assert g.shape == rgb_o.shape
    assert gp["global_stored"] == ost["global_stored"]
    assert gp["caustic_stored"] == ost["caustic_stored"]
    diff = {k: (gst[k], int(ost[k])) for k in COUNTERS if gst[k] != int(ost[k])}
    compare_exact(g, rgb_o)
    assert not diff, diff


def _hash(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def test_c3_full_frame_properties(renderer):
    """The full C3 frame (jensen.scn 1024^2 aa 2, 4 M caustic photons, every other flag at its
    default): finite, clamped to [0, 1], every primary sample traced, the same image twice."""
    import gc
    gc.collect()
    renderer.release_scratch()
    args = [scene("jensen.scn"), "/tmp/x.png", "-resolution", "1024", "1024", "-aa", "2",
            "-caustic", "4000000", "-seed", "1"]
    p, sc, _o, w, h, aa, real = gi_amd.ParseArgs(args)
    r = gi_amd.Renderer(0, p)
    try:
        r.ReadScene(sc, real)
        ps = r.MapPhotons()
        assert ps["caustic_stored"] >= 4000000
        hs = []
        for _ in range(2):
            rgb, f, st = r.RenderImage(aa, w, h, want_float=True)
            assert np.isfinite(f).all() and f.min() >= 0.0 and f.max() <= 1.0
            assert st["screen_rays"] > 0.9 * w * h * 4 ** aa
            assert st["shadow_rays"] > 100 * st["screen_rays"]   # 128 + 128 fans per diffuse hit
            assert st["knn_map_queries"][1] > 0
            hs.append(_hash(rgb))
        assert hs[0] == hs[1]
    finally:
        r.close()


@pytest.mark.parametrize("cid,res,shard", [("c4", 2048, 0), ("c5", 4096, 1)])
def test_full_tile_shard_properties(renderer, cid, res, shard):
    """One GPU's share of the full C4 / C5 frame (tile shard s of 8 through
    gi_render_tiles_packed, the torchrun ranks' entry point): every owned pixel written,
    finite, clamped, its u8 word the truncation of its f32 RGB (SetPixelRGB), and C5's shard
    rendered with 4 DOF samples per subsample."""
    import gc
    import torch
    gc.collect()
    renderer.release_scratch()
    args, _rgb, _st = fixture(cid)
    i = args.index("-resolution")
    args[i + 1] = args[i + 2] = str(res)
    p, sc, _o, w, h, aa, real = gi_amd.ParseArgs(args)
    r = gi_amd.Renderer(0, p)
    try:
        r.ReadScene(sc, real)
        r.MapPhotons()
        n = r.shard_pixels(w, h, 16, shard, 8)
        assert n == (w * h) // 8
        buf = torch.full((n, 4), -1.0, dtype=torch.float32, device="cuda:0")
        npx, st = r.render_tiles_packed(aa, w, h, 16, shard, 8, buf.data_ptr(), n)
        torch.cuda.synchronize()
        assert npx == n
        b = buf.cpu().numpy()
        rgb = b[:, :3]
        assert np.isfinite(rgb).all() and rgb.min() >= 0.0 and rgb.max() <= 1.0
        u8 = b[:, 3].view(np.uint32)
        got = np.stack([u8 & 255, (u8 >> 8) & 255, (u8 >> 16) & 255], -1).astype(np.int64)
        # the u8 word is trunc(255 r) of the fp64 pixel value r (R2Image::SetPixelRGB), the f32
        # words r rounded to fp32: equal truncations except where 255 r lies within fp32
        # rounding of an integer
        x = rgb.astype(np.float64) * 255.0
        want = np.floor(x).astype(np.int64)
        edge = np.abs(x - np.rint(x)) < 1e-4
        assert (np.abs(got - want) <= 1).all()
        assert (got == want)[~edge].all()
        assert st["screen_rays"] > 0
        if cid == "c5":
            assert p.dof_test == 4
        assert rgb.mean() > 0.01
    finally:
        r.close()
