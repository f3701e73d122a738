#!/usr/bin/env python3
"""Caustic k-NN fallback diagnostics (GPU box): render one frame with GI_DUMP_FB set, so the
host writes the query positions of the caustic launch with the most query-per-wave fallback
queries; save them with the caustic photon map and its kd tree for offline analysis.

usage: tools/caustic_fb_dump.py [--scene cornell.scn --res 1024 --aa 2 --global N --caustic N]
writes gpurun_out/fb/<tag>.npz: fb (final fallback queries, xyz f32, <= 2M, list order),
p2 (second-pass queries, subsampled to <= 1M, list order, stride p2_stride), photons (xyz f32,
kd order), nodes [2L, 8] f32, nleaves, hdr (nq, nfb, nfb2, map).
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "global-illumination_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell.scn")
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--aa", type=int, default=2)
    ap.add_argument("--global-photons", type=int, default=1000000)
    ap.add_argument("--caustic-photons", type=int, default=1000000)
    ap.add_argument("--tag", default="c2")
    ap.add_argument("--extra", default="")
    a = ap.parse_args()
    raw = "/tmp/gi_fb_dump.bin"
    if os.path.exists(raw):
        os.remove(raw)
    os.environ["GI_DUMP_FB"] = raw
    import gi_amd
    scene = os.path.join(ROOT, "tests", "scenes", a.scene)
    args = [scene, "/tmp/x.png", "-global", str(a.global_photons), "-caustic",
            str(a.caustic_photons)] + a.extra.split()
    p, sc, _o, _w, _h, _aa, real = gi_amd.ParseArgs(args)
    r = gi_amd.Renderer(0, p)
    r.ReadScene(sc, real)
    r.MapPhotons()
    t = time.time()
    _rgb, st = r.RenderImage(a.aa, a.res, a.res)
    print(f"frame {time.time() - t:.2f} s", flush=True)
    with open(raw, "rb") as f:
        hdr = np.frombuffer(f.read(32), dtype=np.int64)
        nq, nfb, nfb2, mp = (int(x) for x in hdr)
        q2 = np.frombuffer(f.read(16 * nfb2), dtype=np.float32).reshape(-1, 4)
        q1 = np.frombuffer(f.read(16 * nfb), dtype=np.float32).reshape(-1, 4)
    print(f"launch: nq {nq} second pass {nfb} fallback {nfb2} map {mp}", flush=True)
    fb = np.ascontiguousarray(q2[:2_000_000, :3])
    stride = max(1, (len(q1) + 999_999) // 1_000_000)
    p2 = np.ascontiguousarray(q1[::stride, :3])
    nodes, perm, nl = r.kd_tree(mp)
    ph = r.photon_map(mp)
    pos = np.ascontiguousarray(ph["pos"], dtype=np.float32)[perm]  # kd order
    os.makedirs(os.path.join(ROOT, "gpurun_out", "fb"), exist_ok=True)
    out = os.path.join(ROOT, "gpurun_out", "fb", f"{a.tag}.npz")
    np.savez_compressed(out, fb=fb, p2=p2, p2_stride=stride, photons=pos, nodes=nodes, nleaves=nl,
                        hdr=hdr)
    print("wrote", out, os.path.getsize(out), flush=True)


if __name__ == "__main__":
    main()
