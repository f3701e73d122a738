#!/usr/bin/env python3
"""Would overlapping batches help? Two independent C2 frames on one GPU (two contexts, two host
threads, their own streams) back to back and concurrently: if the concurrent pair takes well under
twice one frame, the path kernels and the k-NN kernels of different batches share the CUs
productively (GPU box diagnostics).

usage: tools/concurrency_probe.py [--res 1024] [--aa 2]
"""
import argparse
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "global-illumination_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--aa", type=int, default=2)
    a = ap.parse_args()
    import gi_amd
    scene = os.path.join(ROOT, "tests", "scenes", "cornell.scn")
    args = [scene, "/tmp/x.png", "-global", "1000000", "-caustic", "1000000"]
    p, sc, _o, _w, _h, _aa, real = gi_amd.ParseArgs(args)
    rs = []
    for _ in range(2):
        r = gi_amd.Renderer(0, p)
        r.ReadScene(sc, real)
        r.MapPhotons()
        r.RenderImage(a.aa, a.res, a.res)  # warmup: buffers sized
        rs.append(r)
    t = time.time()
    for r in rs:
        r.RenderImage(a.aa, a.res, a.res)
    seq = time.time() - t
    out = [None, None]

    def run(i):
        out[i] = rs[i].RenderImage(a.aa, a.res, a.res)

    th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    t = time.time()
    for x in th:
        x.start()
    for x in th:
        x.join()
    conc = time.time() - t
    print(f"two frames sequential {seq:.3f} s, concurrent {conc:.3f} s, ratio {conc / seq:.3f}",
          flush=True)


if __name__ == "__main__":
    main()
