"""GPU twin of test_cpu_photon_figs.py: the device renders every photon-map figure's
configuration (tests/photon_figs.py) at the same seeds through the C ABI.

- Figures the CPU oracle rendered: the device's block means equal the oracle's committed ones
  seed for seed (the renders are bit-exact with the restatement on the same RNG streams; a rare
  one-ulp fork of a Monte Carlo path may move one pixel by a few LSB: mean |diff| <= 0.02 LSB).
- Every figure, including the ones the CPU cannot afford (fig_24c, fig_26c: 100 M photons, at
  four seeds; fig_33c: 30 M; fig_29c, fig_30b-c: 1,024 and 4 x 320 importance samples per
  pixel): the device's own renders pin the figure with the same statistic and criterion.
Only the committed block statistics are read (tests/golden/photon_figs/oracle_blocks.npz), not
the figure files."""
import json
import os

import numpy as np
import pytest

import photon_figs as pf
from gpu_util import run_gpu

pytestmark = pytest.mark.gpu

STATS = dict(np.load(pf.STATS))
KNOWN_MISSES = pf.KNOWN_MISSES


def device_blocks(renderer, name, tmp_dir):
    out = []
    for s in pf.seeds(name):
        args, _w, _h = pf.render_args(name, s, tmp_dir=str(tmp_dir))
        rgb, _st, _ps = run_gpu(renderer, args)
        out.append(pf.render_blocks(rgb, name))
    return np.stack(out)


@pytest.mark.parametrize("name", list(pf.FIGS))
def test_device_figure_pin(renderer, name, tmp_path):
    dev = device_blocks(renderer, name, tmp_path)
    if name + "/seeds" in STATS:
        ora = STATS[name + "/seeds"].astype(float)
        d = np.abs(dev - ora)
        assert d.mean() <= 0.02 and d.max() <= 1.0, (d.mean(), d.max())
    r = pf.pin(STATS[name + "/figure"].astype(float), dev, STATS[name + "/mask"])
    log = os.environ.get("GI_FIG_LOG")
    if log:
        with open(log, "a") as f:
            f.write(json.dumps(dict(r, figure=name, role=pf.role(name))) + "\n")
    if name in KNOWN_MISSES:
        pytest.xfail(KNOWN_MISSES[name] + f" ({r})")
    assert r["ok"], r
