"""Oracle fixtures for the BASELINE configs C3, C4 and C5 with their exact flags (VERDICT r04
"Next round" item 1): each one is the config's command line verbatim -- photon-map sizes, aa,
DOF and every other flag at the reference default (photonmap.cpp:27-106) -- at an oracle-sized
resolution. The oracle restatement (tests/oracle_lib.py, test infrastructure) renders each one
once here in the build container; the image, its counters and the stored photon counts go to
tests/golden/configs/<id>.npz, and tests/test_gpu_configs.py compares the device render with
them (no CPU rendering on the GPU box).

  C3  jensen.scn   32x32 aa 2  -caustic 4000000                      (lt/ss 128, it 256, tt/st 128)
  C4  stilllife    16x16 aa 2  -global 2000000                       (caustic default 10 M)
  C5  teapot.scn   8x8   aa 3  -global 8000000 -dof 4 12.2282 0.025 -no_caustic

usage: python tools/make_config_fixtures.py [c3 c4 c5] [--threads 8]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "global-illumination_amd"))

import oracle_lib  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "configs")

# id -> (scene, width, height, flags after the resolution); the flags are BASELINE.json's
CONFIGS = {
    "c3": ("jensen.scn", 32, 32, ["-aa", "2", "-caustic", "4000000"]),
    "c4": ("stilllife.scn", 16, 16, ["-aa", "2", "-global", "2000000"]),
    "c5": ("teapot.scn", 8, 8, ["-aa", "3", "-global", "8000000", "-dof", "4", "12.2282",
                                "0.025", "-no_caustic"]),
}
SEED = "1"


def command(cid, scene_dir):
    """The config's argv (without the program name), scene path under scene_dir."""
    sc, w, h, flags = CONFIGS[cid]
    return [os.path.join(scene_dir, sc), "/tmp/%s.png" % cid, "-resolution", str(w), str(h),
            "-seed", SEED] + flags


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("ids", nargs="*", default=sorted(CONFIGS))
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    os.makedirs(OUT, exist_ok=True)
    for cid in a.ids:
        sc, w, h, _ = CONFIGS[cid]
        args = command(cid, os.path.join(ROOT, "tests", "scenes"))
        t0 = time.time()
        rgb, st = oracle_lib.render(args + ["-threads", str(a.threads)], w, h)
        wall = time.time() - t0
        # the argv is stored with the scene's file name only (the test resolves it)
        rel = [sc] + args[1:]
        np.savez_compressed(os.path.join(OUT, cid + ".npz"), rgb=rgb,
                            args=np.array(rel), stats=json.dumps(st))
        print(cid, "%.1f s" % wall, json.dumps(st), flush=True)


if __name__ == "__main__":
    main()
