#!/usr/bin/env python3
"""Benchmark: Mpixel-samples/s on cornell.scn at 1024x1024, aa=2, 1M global + 1M caustic
photons (BASELINE.json configs[1] = SURVEY.md C2).

A step = one full frame (RenderImage, render.cpp:155-259) over the resident scene and photon
maps. With N ranks (torchrun, one process per GPU) the frame's 16x16-pixel tiles are dealt
round-robin (tile % N, the reference's column interleave render.cpp:90 re-cut as tiles); each
rank renders its tiles and the image is gathered to rank 0 with one RCCL reduce over xGMI
(disjoint tiles, so the sum is a gather). Total work per step is fixed -> "scaling": "strong".
The photon maps are built once per rank from the same seed (identical, no communication) and
their build time is reported separately (photon_map_s), as SURVEY.md §8(d) prescribes.

Extra JSON fields: roofline (k-NN radiance kernel, algorithmic bytes = 16 B per photon
returned), cpu_baseline (the oracle/ C++ restatement on this host's cores).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "global-illumination_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

SCENE = os.path.join(ROOT, "tests", "scenes", "cornell.scn")
HBM_PEAK_GBPS = 8000.0
BYTES_PER_PHOTON = 16   # compulsory photon record gather
BYTES_PER_SAMPLE = 12   # f32 RGB pixel write


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--aa", type=int, default=2)
    ap.add_argument("--global-photons", type=int, default=1000000)
    ap.add_argument("--caustic-photons", type=int, default=1000000)
    ap.add_argument("--tile", type=int, default=16)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-res", type=int, default=8, help="CPU baseline sample: res x res px")
    ap.add_argument("--cpu-threads", type=int, default=0)
    return ap.parse_args()


def cpu_baseline(a):
    """Oracle restatement (port) of the reference path timed on this host: same scene, flags
    and photon counts, on a res x res pixel sample of the same image plane (uniform sub-grid,
    identical per-sample workload)."""
    import oracle_lib
    threads = a.cpu_threads or min(16, os.cpu_count() or 1)
    args = [SCENE, "/tmp/cpu.png", "-resolution", str(a.cpu_res), str(a.cpu_res), "-aa",
            str(a.aa), "-global", str(a.global_photons), "-caustic", str(a.caustic_photons),
            "-threads", str(threads), "-seed", str(a.seed)]
    _, st = oracle_lib.render(args, a.cpu_res, a.cpu_res)
    samples = a.cpu_res * a.cpu_res * 4 ** a.aa
    return {"value": samples / st["render_s"] / 1e6, "unit": "Mpixel-samples/s",
            "cores": threads, "kind": "port",
            "sample": f"cornell.scn {a.cpu_res}x{a.cpu_res} aa={a.aa} ({samples} pixel-samples), "
                      f"{a.global_photons}+{a.caustic_photons} photons; render {st['render_s']:.2f} s, "
                      f"photon map {st['trace_s'] + st['kd_s']:.2f} s on {threads} threads"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    import gi_amd

    args = [SCENE, "/tmp/bench.png", "-resolution", str(a.res), str(a.res), "-aa", str(a.aa),
            "-global", str(a.global_photons), "-caustic", str(a.caustic_photons),
            "-seed", str(a.seed)]
    p, sc, _o, w, h, aa, real = gi_amd.ParseArgs(args)
    r = gi_amd.Renderer(local, p)
    r.ReadScene(sc, real)
    t0 = time.perf_counter()
    pst = r.MapPhotons()
    photon_s = time.perf_counter() - t0

    def step():
        if world == 1:
            rgb, st = r.RenderImage(aa, w, h)
            return st
        import torch
        img, st = r.render_tiles(aa, w, h, a.tile, rank, world)
        dev = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
        t = torch.from_numpy(img).to(dev)
        dist.reduce(t, dst=0)
        if rank == 0:
            t.cpu()
        return st

    def barrier():
        if dist is not None:
            dist.barrier()
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize()
        except ImportError:
            pass

    for _ in range(a.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    agg = {"knn_photons": 0, "knn_queries": 0, "knn_visited": 0, "knn_kernel_ms": 0.0,
           "knn_kernel_launches": 0.0}
    for _ in range(a.steps):
        st = step()
        for k in agg:
            agg[k] += st[k]
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64,
                          device=("cuda" if torch.cuda.is_available() else "cpu"))
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        ag = torch.tensor([agg["knn_photons"], agg["knn_queries"], agg["knn_kernel_ms"]],
                          dtype=torch.float64, device=tt.device)
        dist.all_reduce(ag)  # sums over ranks (kernel ms summed over GPUs)
        agg["knn_photons"], agg["knn_queries"], agg["knn_kernel_ms"] = [float(x) for x in ag.tolist()]
    samples_per_frame = w * h * 4 ** aa * p.dof_test
    value = samples_per_frame * a.steps / elapsed / 1e6
    ms_per_step = elapsed / a.steps * 1000.0

    if rank == 0:
        # roofline of the dominant kernel (k-NN radiance estimate), HIP-event timed in-library
        knn_s = agg["knn_kernel_ms"] / 1000.0
        alg_bytes = agg["knn_photons"] * BYTES_PER_PHOTON
        achieved = alg_bytes / knn_s / 1e9 if knn_s > 0 else 0.0
        if world > 1:
            achieved *= 1.0  # bytes and kernel seconds both summed over GPUs: per-GPU rate
        roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5), "traffic": None,
                    "kernel": "knn_kernel<true> (k-NN + EstimateRadiance)",
                    "bytes_per_unit": "16 B per photon returned",
                    "photons_per_frame": agg["knn_photons"] / a.steps,
                    "queries_per_frame": agg["knn_queries"] / a.steps,
                    "visited_per_query": agg["knn_visited"] / max(1, agg["knn_queries"]),
                    "knn_ms_per_frame": agg["knn_kernel_ms"] / a.steps / max(1, world)}
        cpu = None
        if not a.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(a)
        line = {
            "metric": "Mpixel-samples/sec (and ms/frame) at 1024^2 aa=2, 1M+1M photons",
            "value": round(value, 4), "unit": "Mpixel-samples/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms_per_step, 2),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f64 (shading/geometry), f32 (photon positions)", "data": "synthetic",
            "config": {"workload": f"cornell.scn {w}x{h} aa={aa} "
                                   f"{a.global_photons}+{a.caustic_photons} photons",
                       "pixel_samples_per_frame": samples_per_frame,
                       "parallelism": f"tiles{a.tile}x{a.tile} % {world}",
                       "photon_map_s": round(photon_s, 3),
                       "global_stored": pst["global_stored"],
                       "caustic_stored": pst["caustic_stored"]},
            "roofline": roofline, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    r.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
