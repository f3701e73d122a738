#!/usr/bin/env python3
"""Per-pixel agreement of GPU renders with the oracle on the same RNG streams (diagnostics)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "global-illumination_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import gi_amd  # noqa: E402
import oracle_lib  # noqa: E402

S = os.path.join(ROOT, "tests", "scenes")
CASES = [
    ("cornell direct", ["cornell.scn", "-resolution", "64", "64", "-aa", "0", "-no_indirect", "-no_caustic", "-tt", "8", "-st", "8"]),
    ("jensen direct", ["jensen.scn", "-resolution", "48", "48", "-aa", "0", "-no_indirect", "-no_caustic", "-lt", "8", "-ss", "8", "-tt", "8", "-st", "8"]),
    ("cornell full", ["cornell.scn", "-resolution", "32", "32", "-aa", "1", "-global", "20000", "-caustic", "20000", "-it", "16", "-tt", "8", "-st", "8"]),
    ("teapot full", ["teapot.scn", "-resolution", "32", "32", "-aa", "0", "-global", "20000", "-no_caustic", "-it", "8"]),
]
r = gi_amd.Renderer(0)
for name, a in CASES:
    args = [os.path.join(S, a[0]), "/tmp/x.png"] + a[1:] + ["-seed", "3"]
    p, sc, _o, w, h, aa, real = gi_amd.ParseArgs(args)
    r.set_params(p)
    r.ReadScene(sc, real)
    if p.indirect_illum or p.caustic_illum:
        r.MapPhotons()
    g, _ = r.RenderImage(aa, w, h)
    o, _ = oracle_lib.render(args, w, h)
    d = np.abs(g.astype(int) - o.astype(int)).max(-1)
    print(f"{name:16s} exact={np.mean(d == 0):.5f} le1={np.mean(d <= 1):.5f} max={d.max()} "
          f"meandiff={g.astype(float).mean() - o.astype(float).mean():+.4f}", flush=True)
r.close()
