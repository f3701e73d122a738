#!/usr/bin/env python3
"""Glass-layer exploration: render jensen.scn variants of fig_12 / fig_14
on the device at several seeds and keep the full 8-bit images, so that the per-sample noise of
the glass and mirror spheres can be measured from seed-to-seed differences on the CPU
(tools/glass_fit.py). The device equals the oracle restatement bit for bit (the -m gpu suite),
so these images stand for the restatement's.

usage (GPU box): python tools/glass_explore.py OUT_DIR [variant-prefix ...]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "global-illumination_amd"))

import gi_amd  # noqa: E402
from gpu_util import run_gpu  # noqa: E402

SCN = os.path.join(ROOT, "tests", "scenes")
XSCN = os.path.join(ROOT, "tests", "scenes_extra")
NOGI = ["-no_indirect", "-no_caustic"]


def variants():
    V = {}
    for aa in (0, 1, 2):
        for n in (8, 32, 128):
            t = ["-tt", str(n), "-st", str(n)]
            V[f"a{aa}_on_t{n}"] = ("jensen.scn", aa, NOGI + t)
            V[f"a{aa}_off_t{n}"] = ("jensen.scn", aa, NOGI + t + ["-no_fresnel"])
            V[f"a{aa}_onrs_t{n}"] = ("jensen.scn", aa, NOGI + t + ["-no_rs"])
        for fr in ("on", "off"):
            f = [] if fr == "on" else ["-no_fresnel"]
            V[f"a{aa}_{fr}_nodtds"] = ("jensen.scn", aa, NOGI + f + ["-no_dt", "-no_ds"])
            V[f"a{aa}_{fr}_nods"] = ("jensen.scn", aa, NOGI + f + ["-no_ds"])
            V[f"a{aa}_{fr}_nodt"] = ("jensen.scn", aa, NOGI + f + ["-no_dt"])
    # scene variants (tests/scenes_extra): a lit front wall behind the camera
    for n in (8, 128):
        t = ["-tt", str(n), "-st", str(n)]
        V[f"fw_a1_on_t{n}"] = ("X:jensen_frontwall.scn", 1, NOGI + t)
    V["fw_a1_off_t128"] = ("X:jensen_frontwall.scn", 1, NOGI + ["-no_fresnel"])
    # material variants of jensen.scn written to /tmp: glass (material 3) / mirror (4) shininess
    for g in (100, 200, 300, 400, 500, 700):
        for n in (8, 32, 128):
            V[f"gn{g}_a1_on_t{n}"] = (f"G:{g}", 1, NOGI + ["-tt", str(n), "-st", str(n)])
    for m in (500, 700, 1500):
        for n in (8, 32, 128):
            V[f"mn{m}_a1_on_t{n}"] = (f"M:{m}", 1, NOGI + ["-tt", str(n), "-st", str(n)])
    # per-pixel sample-count candidates: tt = st = k per subsample at aa 0 / 1 / 2
    for aa, ks in ((0, (8, 16, 32, 64, 128)), (1, (1, 2, 4, 8, 16, 32)), (2, (1, 2, 4, 8))):
        for k in ks:
            V[f"cand_a{aa}_k{k}"] = ("jensen.scn", aa, NOGI + ["-tt", str(k), "-st", str(k)])
    return V


def material_variant(kind, n):
    """jensen.scn with the glass (kind G, material 3) or mirror (M, material 4) shininess n"""
    lines = open(os.path.join(SCN, "jensen.scn")).read().splitlines()
    mats = [i for i, l in enumerate(lines) if l.startswith("material")]
    i = mats[3 if kind == "G" else 4]
    t = lines[i].split()
    t[16] = str(n)  # material ka kd ks kt e n ir texture: n is the 16th value
    lines[i] = " ".join(t)
    path = f"/tmp/jensen_{kind}{n}.scn"
    open(path, "w").write("\n".join(lines) + "\n")
    return path


def main():
    out = sys.argv[1]
    pref = sys.argv[2:]
    seeds = [int(s) for s in os.environ.get("SEEDS", "1,2").split(",")]
    os.makedirs(out, exist_ok=True)
    r = gi_amd.Renderer(0)
    V = variants()
    t00 = time.time()
    for name, (sc, aa, flags) in V.items():
        if pref and not any(name.startswith(p) for p in pref):
            continue
        t0 = time.time()
        if sc[:2] in ("G:", "M:"):
            path = material_variant(sc[0], int(sc[2:]))
        elif sc.startswith("X:"):
            path = os.path.join(XSCN, sc[2:])
        else:
            path = os.path.join(SCN, sc)
        imgs = []
        for s in seeds:
            args = [path, "/tmp/ge.png", "-resolution", "512", "512", "-aa", str(aa),
                    "-seed", str(s)] + flags
            rgb, _st, _ps = run_gpu(r, args)
            imgs.append(rgb[::-1].copy())  # figure row order (top-down)
        np.savez_compressed(os.path.join(out, name + ".npz"), imgs=np.stack(imgs),
                            seeds=np.array(seeds), flags=" ".join(flags), scene=sc, aa=aa)
        print(f"{name}: {time.time() - t0:.1f} s (total {time.time() - t00:.0f} s)", flush=True)
    r.close()


if __name__ == "__main__":
    main()
