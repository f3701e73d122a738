"""The Monte Carlo specular layer pinned on the reference's own render (tests/mc_figs.py):
gallery/tests/specular.png against the oracle restatement's draws at eight seeds, whose block
statistics tools/mc_figs_oracle.py committed (tests/golden/mc_figs/oracle_blocks.npz)."""
import os

import numpy as np

import mc_figs as mf
import oracle_lib

STATS = dict(np.load(mf.STATS))


def test_specular_figure_is_a_draw_of_the_restatement():
    """specular.scn at aa 0 with -no_ds: every 16 x 16 block within |z| < 3 of the eight
    seeds, level ratio 1 within RATIO_TOL, and the figure's pixels agree with seed 1's as
    closely as seed 1's agree with seed 2's (exact and within 1 LSB)."""
    r = mf.pin(STATS["specular/figure"].astype(float), STATS["specular/seeds"].astype(float))
    assert r["ok"] and r["z_frac"] >= 0.99 and abs(r["ratio"] - 1) < 0.002, r
    fig_px, seed_px = STATS["specular/pix_figure"], STATS["specular/pix_seeds"]
    assert (fig_px >= seed_px - 0.005).all(), (fig_px, seed_px)


def test_specular_figure_was_rendered_without_distributed_specular():
    """Evidence for the -no_ds setting: with SpecularIllumination's Phong-lobe sampling on (the
    default) the same statistic fails, and the figure's pixels agree with a draw far less than
    two draws agree with each other."""
    r = mf.pin(STATS["specular+ds/figure"].astype(float), STATS["specular+ds/seeds"].astype(float))
    assert not r["ok"] and r["z_frac"] < 0.8, r
    assert STATS["specular+ds/pix_figure"][0] < STATS["specular+ds/pix_seeds"][0] - 0.05


def test_committed_blocks_are_the_current_oracle():
    """Seed 1 of the specular pin re-rendered now equals the committed blocks (the file is the
    current restatement's)."""
    threads = len(os.sched_getaffinity(0))
    args, w, h = mf.render_args("specular", 1, threads=threads)
    rgb, _ = oracle_lib.render(args, w, h)
    np.testing.assert_allclose(mf.blocks(rgb[::-1]), STATS["specular/seeds"][0], atol=1e-4)
