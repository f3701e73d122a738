#!/usr/bin/env python3
"""Benchmark: Mpixel-samples/s on cornell.scn at 1024x1024, aa=2, 1M global + 1M caustic
photons (BASELINE.json configs[1] = SURVEY.md C2).

A step = one full frame (RenderImage, render.cpp:155-259) over the resident scene and photon
maps. The frame's 16x16-pixel output tiles are dealt round-robin over the GPUs (tile % N, the
reference's column interleave render.cpp:90 re-cut as tiles); total work per step is fixed ->
"scaling": "strong". Two ways to run N GPUs:
- torchrun (WORLD_SIZE set; the driver's N>1 launch): one process per GPU. Each rank renders its
  tiles into a packed device buffer (gi_render_tiles_packed) and rank 0 gathers the packed
  buffers over RCCL/xGMI (one gather, 1/N of the frame per rank) and composes the frame on its
  GPU (gi_dist.py).
- `--gpus N` without WORLD_SIZE: the drop-in's own device set in one process (gi_create_devices,
  render.cpp:188-199's thread fork re-cut as devices): one host thread per device, ncclSend /
  ncclRecv tile gather onto device 0. GI_DEVICES="0,0" names the devices explicitly (tests).
The photon maps are built once (per rank, from the same seed: identical, no communication) and
their build time is reported separately (photon_map_s), as SURVEY.md §8(d) prescribes.

Extra JSON fields: roofline (k-NN radiance kernel, algorithmic bytes = 16 B per photon
returned), cpu_baseline (the oracle/ C++ restatement on this host's cores).
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "global-illumination_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

SCENES = os.path.join(ROOT, "tests", "scenes")
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
    ap.add_argument("--scene", default="cornell.scn", help="scene under tests/scenes (C2: cornell)")
    ap.add_argument("--extra", default="", help="extra reference flags, e.g. '-dof 4 12.2 0.025'")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-res", type=int, default=32,
                    help="CPU baseline sample: res x res px at the same aa (BASELINE.md section 3)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--shard", default="",
                    help="S/N: render only tile shard S of N on this GPU (one GPU's share of an "
                         "N-GPU frame, e.g. C5's 0/8); value = that shard's pixel-samples/s")
    ap.add_argument("--balance", type=int, default=0,
                    help="N: render every tile shard s/N of the frame in turn on this GPU and print "
                         "the per-shard times (min/mean/max: an N-GPU frame takes the slowest)")
    return ap.parse_args()


def shard_balance(a):
    """Shard balance of an N-GPU frame measured on one GPU (render.cpp:90's interleave re-cut as
    16x16 tiles, tile (tx, ty) on GPU (tx + ty) % N): each shard rendered `steps` times after one warmup render of
    shard 0 (buffer growth), its time the median. Prints one JSON line."""
    import torch
    import gi_amd
    N = a.balance
    args = [os.path.join(SCENES, a.scene), "/tmp/bench.png", "-resolution", str(a.res),
            str(a.res), "-aa", str(a.aa), "-global", str(a.global_photons), "-caustic",
            str(a.caustic_photons), "-seed", str(a.seed)] + a.extra.split()
    p, sc, _o, w, h, aa, real = gi_amd.ParseArgs(args)
    r = gi_amd.Renderer(0, p)
    r.ReadScene(sc, real)
    t0 = time.perf_counter()
    r.MapPhotons()
    photon_s = time.perf_counter() - t0
    npix = [r.shard_pixels(w, h, a.tile, s, N) for s in range(N)]
    buf = torch.zeros((max(npix), 4), dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()
    for _ in range(a.warmup):
        r.render_tiles_packed(aa, w, h, a.tile, 0, N, buf.data_ptr(), max(npix))
    torch.cuda.synchronize()
    times = []
    for s in range(N):
        ts = []
        for _ in range(max(1, a.steps)):
            t1 = time.perf_counter()
            r.render_tiles_packed(aa, w, h, a.tile, s, N, buf.data_ptr(), max(npix))
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t1)
        times.append(float(np.median(ts)))
        print(f"shard {s}/{N}: {npix[s]} px, {times[-1] * 1e3:.1f} ms", flush=True)
    mean = float(np.mean(times))
    spf = w * h * 4 ** aa * p.dof_test
    line = {"metric": "shard balance (ms per shard, one GPU each)",
            "config": {"workload": f"{a.scene} {w}x{h} aa={aa} "
                                   f"{a.global_photons}+{a.caustic_photons} photons {a.extra}".strip(),
                       "tile": a.tile, "nshards": N, "photon_map_s": round(photon_s, 3),
                       "assignment": f"tile (tx, ty) -> shard (tx + ty) % {N}"},
            "shard_ms": [round(t * 1e3, 1) for t in times], "shard_pixels": npix,
            "min_ms": round(min(times) * 1e3, 1), "mean_ms": round(mean * 1e3, 1),
            "max_ms": round(max(times) * 1e3, 1), "max_over_mean": round(max(times) / mean, 4),
            "sum_ms": round(sum(times) * 1e3, 1),
            "frame_Mpx_samples_per_s_at_N": round(spf / max(times) / 1e6, 3)}
    print(json.dumps(line), flush=True)
    r.close()


# the kernels of the FETCH_SIZE pass behind roofline.traffic (profiles/knn_traffic.json): the
# chunk k-NN passes and, when it was taken, the per-lane last fallback (the query-per-wave
# kernel since r06's final tree; 0.1 ms of a ~40 ms launch)
ROOFLINE_KERNELS = ["knn_chunk_lane_kernel", "knn_lane_kernel"]

# k-NN launch sequences by gi_render_stats.knn_map_kind (run_knn in gi_host.cpp)
KNN_KINDS = {
    7: "gi::knn_chunk_lane_kernel<4,240> -> knn_chunk_lane_kernel<2,480> -> knn_wave_kernel<128> fallback",
    8: "gi::knn_chunk_big_kernel<512> -> knn_chunk_big_kernel<1024> -> knn_wave_kernel<512> fallback",
    3: "gi::knn_lane_kernel<8,4>",
    1: "gi::knn_wave_kernel + knn_list_estimate_kernel",
    0: "gi::knn_kernel (global-memory heaps)",
    9: "gi::cached_kernel (irradiance cache)",
    -1: "none",
}

# CPU-baseline calibration: the restatement vs the reference binary on the
# survey's C2 sample (cornell 64x64 aa=0, 1M + 1M photons, 8 threads) in the build container.
# NOT a same-session measurement: the reference's 72.62 s is the survey session's
# (SURVEY.md section 6), and the reference cannot be rebuilt since (it needs GL/glu.h, DESIGN.md
# section 6), while the restatement's 81.42 s is round 5's. The container's per-core speed moved
# ~1.9x between those sessions (round 2's own restatement: 52.70 s then, ~100 s in round 5;
# profiles/r05_cpu_calibration.json drift_check), so the ratio is only known within
# [81.42 / (72.62 x 1.9), 81.42 / 72.62] = [0.59, 1.12]. No reference-equivalent rate is derived.
CPU_CALIBRATION = {"same_session": False, "restatement_s": 81.417, "restatement_session": "r05",
                   "reference_s": 72.62, "reference_session": "survey (SURVEY.md section 6)",
                   "cross_session_ratio": round(81.417 / 72.62, 3),
                   "container_drift": 1.9,
                   "ratio_band": [round(81.417 / (72.62 * 1.9), 2), round(81.417 / 72.62, 2)],
                   "status": "unpinned: no same-session reference timing is possible here",
                   "measured": "r05, profiles/r05_cpu_calibration.json",
                   "sample": "cornell 64x64 aa=0 1M+1M photons, 8 threads, build container"}

# image_sha16 of the 1-GPU frame per workload (BENCH_r05 and the GPU suite's C2 hash): a run on N
# GPUs must compose the same image (tiles dealt over the GPUs, the same RNG streams per sample)
EXPECTED_SHA16 = {
    ("cornell.scn", 1024, 2, 1000000, 1000000, 1, ""): "8b2810dafe63a3e9",
}


def load_traffic(a, qpl):
    """HBM bytes per launch of the roofline kernel from a committed PMC pass
    (tools/pmc_traffic.py -> profiles/knn_traffic.json), if it was taken on this workload."""
    path = os.path.join(ROOT, "profiles", "knn_traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    wl = t.get("workload", {})
    if (wl.get("res"), wl.get("aa"), wl.get("global"), wl.get("caustic")) != (
            a.res, a.aa, a.global_photons, a.caustic_photons):
        return None
    if t.get("kernel") != " + ".join(ROOFLINE_KERNELS):
        return None  # measured on an earlier kernel
    bpq = t.get("bytes_per_query")
    if not bpq:
        return None
    return bpq * qpl  # the PMC pass's bytes per query, at this run's launch size


def host_threads():
    """CPU threads this process may use: its affinity set, capped by a cgroup CPU quota and by
    the host's declared CPU share (OMP_NUM_THREADS, set on the GPU boxes) when those are set (a
    container can see more CPUs than it may run)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(a):
    """Oracle restatement (port) of the reference path timed on this host: same scene, flags
    and photon counts, on a res x res pixel sample of the same image plane (uniform sub-grid,
    identical per-sample workload)."""
    import oracle_lib
    threads = a.cpu_threads or host_threads()
    args = [os.path.join(SCENES, a.scene), "/tmp/cpu.png", "-resolution", str(a.cpu_res),
            str(a.cpu_res), "-aa", str(a.aa), "-global", str(a.global_photons), "-caustic",
            str(a.caustic_photons), "-threads", str(threads), "-seed", str(a.seed)] + a.extra.split()
    _, st = oracle_lib.render(args, a.cpu_res, a.cpu_res)
    dof = 1
    ex = a.extra.split()
    if "-dof" in ex:
        dof = max(1, int(ex[ex.index("-dof") + 1]))
    samples = a.cpu_res * a.cpu_res * 4 ** a.aa * dof
    value = samples / st["render_s"] / 1e6
    full = a.res * a.res * 4 ** a.aa * dof
    return {"value": value, "unit": "Mpixel-samples/s",
            "cores": threads, "kind": "port", "cpu_model": cpu_model(),
            "host_cpus_visible": os.cpu_count(),
            "sample": f"{a.scene} {a.cpu_res}x{a.cpu_res} aa={a.aa} ({samples} pixel-samples), "
                      f"{a.global_photons}+{a.caustic_photons} photons; render {st['render_s']:.2f} s, "
                      f"photon map {st['trace_s'] + st['kd_s']:.2f} s on {threads} threads",
            "full_frame_s_extrapolated": round(full / (value * 1e6), 1),
            "calibration": CPU_CALIBRATION if a.scene == "cornell.scn" else None}


def device_list(n):
    """Devices of the single-process device set: GI_DEVICES (e.g. "0,0") or 0..n-1."""
    env = os.environ.get("GI_DEVICES")
    if env:
        return [int(x) for x in env.split(",") if x.strip()]
    return list(range(n))


def main():
    a = parse()
    if a.balance:
        return shard_balance(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    devices = None
    if world > 1:
        import torch
        import torch.distributed as dist
        # GI_BENCH_SAME_GPU=1 maps every rank onto GPU 0 and GI_BENCH_BACKEND=gloo carries the
        # gather through host memory (tests on a one-GPU box; RCCL needs distinct GPUs)
        if os.environ.get("GI_BENCH_SAME_GPU") == "1":
            local = 0
        backend = os.environ.get("GI_BENCH_BACKEND") or (
            "nccl" if torch.cuda.is_available() else "gloo")
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
        n_gpus = world
        mode = "torchrun"
    elif a.gpus > 1 or os.environ.get("GI_DEVICES"):
        devices = device_list(a.gpus)
        n_gpus = len(devices)
        mode = "device-set"
    else:
        n_gpus = 1
        mode = "single"
    import gi_amd

    args = [os.path.join(SCENES, a.scene), "/tmp/bench.png", "-resolution", str(a.res),
            str(a.res), "-aa", str(a.aa), "-global", str(a.global_photons), "-caustic",
            str(a.caustic_photons), "-seed", str(a.seed)] + a.extra.split()
    p, sc, _o, w, h, aa, real = gi_amd.ParseArgs(args)
    r = gi_amd.Renderer(local, p, devices=devices)
    r.ReadScene(sc, real)
    t0 = time.perf_counter()
    pst = r.MapPhotons()
    photon_s = time.perf_counter() - t0

    dev = None
    if world > 1:
        import torch
        dev = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
    last = {}

    shard = None
    if a.shard:
        if world > 1 or n_gpus > 1:
            raise SystemExit("--shard measures one GPU's share: run it on one GPU")
        shard = tuple(int(x) for x in a.shard.split("/"))
        import torch
        npix_shard = r.shard_pixels(w, h, a.tile, shard[0], shard[1])
        shard_buf = torch.zeros((npix_shard, 4), dtype=torch.float32, device="cuda:0")
        torch.cuda.synchronize()

    def step():
        if shard is not None:
            _n, st = r.render_tiles_packed(aa, w, h, a.tile, shard[0], shard[1],
                                           shard_buf.data_ptr(), npix_shard)
            return st
        if world == 1:
            rgb, st = r.RenderImage(aa, w, h)
            last["rgb"] = rgb
            return st
        import gi_dist
        img, st = gi_dist.render_sharded(r, aa, w, h, a.tile, rank, world, dist, dev)
        if img is not None:
            last["rgb"] = img[0] if isinstance(img, tuple) else None
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

    # the first frame (the drop-in CLI renders exactly one), reported as first_frame_ms: its
    # device buffers grow during it (started right after another process that
    # held >100 GB of the GPU exits, an allocation can wait seconds for the driver to clear
    # that memory)
    first_ms = None
    for i in range(a.warmup):
        if i == 0:
            barrier()
            tf = time.perf_counter()
        step()
        if i == 0:
            barrier()
            first_ms = round((time.perf_counter() - tf) * 1e3, 1)
    barrier()
    t0 = time.perf_counter()
    keys = ("q0", "q1", "ph0", "ph1", "vis0", "vis1", "ms0", "ms1", "n0", "n1", "fb0", "fb1",
            "fbq0", "fbq1", "p2ms0", "p2ms1", "p2q0", "p2q1", "devmax", "devmin", "gather")
    agg = dict.fromkeys(keys, 0.0)
    kind = [-1, -1]
    step_ms = []
    for _ in range(a.steps):
        ts = time.perf_counter()
        st = step()
        step_ms.append(round((time.perf_counter() - ts) * 1e3, 1))
        kind = list(st.get("knn_map_kind", kind))
        for m in (0, 1):
            agg[f"q{m}"] += st["knn_map_queries"][m]
            agg[f"ph{m}"] += st["knn_map_photons"][m]
            agg[f"vis{m}"] += st["knn_map_visited"][m]
            agg[f"ms{m}"] += st["knn_map_kernel_ms"][m]
            agg[f"n{m}"] += st["knn_map_launches"][m]
            agg[f"fb{m}"] += st["knn_map_fallback_ms"][m]
            agg[f"fbq{m}"] += st["knn_map_fallback_queries"][m]
            agg[f"p2ms{m}"] += st["knn_map_pass2_ms"][m]
            agg[f"p2q{m}"] += st["knn_map_pass2_queries"][m]
        agg["devmax"] += st["device_render_s_max"]
        agg["devmin"] += st["device_render_s_min"]
        agg["gather"] += st["gather_s"]
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        dv = "cuda" if dist.get_backend() == "nccl" else "cpu"
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dv)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        ag = torch.tensor([agg[k] for k in keys], dtype=torch.float64, device=dv)
        dist.all_reduce(ag)  # sums over ranks (kernel ms summed over GPUs)
        agg = dict(zip(keys, [float(x) for x in ag.tolist()]))
    samples_per_frame = w * h * 4 ** aa * p.dof_test
    samples_per_step = samples_per_frame
    if shard is not None:
        samples_per_step = npix_shard * 4 ** aa * p.dof_test
    value = samples_per_step * a.steps / elapsed / 1e6
    ms_per_step = elapsed / a.steps * 1000.0

    # what ran where: every rank's HIP device and PCI bus, the RCCL
    # communicator's rank count, so a multi-GPU line proves N distinct GPUs took part
    info = r.device_info()
    if dist is not None:
        import torch
        me = {"rank": rank, "local_rank": local, "device": info["devices"][0],
              "pci_bus": info["pci_bus"][0], "hostname": os.uname().nodename}
        allr = [None] * world
        dist.all_gather_object(allr, me)
        topo = {"mode": "torchrun", "backend": dist.get_backend(), "comm_count": dist.get_world_size(),
                "ranks": allr, "distinct_pci_bus": len({(x["hostname"], x["pci_bus"]) for x in allr})}
    else:
        topo = dict(info, mode=mode, distinct_pci_bus=len(set(info["pci_bus"])))

    if rank == 0:
        # roofline of the dominant kernel: the global-map k-NN radiance estimate
        # (knn_chunk_kernel + per-lane fallback, K=50), HIP-event timed in-library on the
        # render stream
        def kstats(m):
            ms = agg[f"ms{m}"]
            launches = max(1.0, agg[f"n{m}"])
            photons = agg[f"ph{m}"]
            ach = photons * BYTES_PER_PHOTON / (ms / 1000.0) / 1e9 if ms > 0 else 0.0
            return {"achieved_GBps": round(ach, 2),
                    "launches": agg[f"n{m}"],
                    "avg_launch_ms": round(ms / launches, 3),
                    "alg_bytes_per_launch": photons * BYTES_PER_PHOTON / launches,
                    "queries_per_launch": agg[f"q{m}"] / launches,
                    "photons_per_query": photons / max(1.0, agg[f"q{m}"]),
                    "visited_per_query": agg[f"vis{m}"] / max(1.0, agg[f"q{m}"]),
                    "second_pass_avg_ms": round(agg[f"p2ms{m}"] / launches, 3),
                    "second_pass_query_frac": round(agg[f"p2q{m}"] / max(1.0, agg[f"q{m}"]), 4),
                    "fallback_avg_ms": round(agg[f"fb{m}"] / launches, 3),
                    "fallback_query_frac": round(agg[f"fbq{m}"] / max(1.0, agg[f"q{m}"]), 4),
                    "ms_per_frame": ms / a.steps / max(1, n_gpus)}
        g, c = kstats(0), kstats(1)
        traffic = load_traffic(a, g["queries_per_launch"])
        roofline = {"bound": "hbm", "achieved": g["achieved_GBps"], "peak": HBM_PEAK_GBPS,
                    "unit": "GB/s", "frac": round(g["achieved_GBps"] / HBM_PEAK_GBPS, 5),
                    "traffic": traffic,
                    "kernel": KNN_KINDS.get(kind[0], str(kind[0])) +
                              " (global map k-NN + EstimateRadiance; avg_launch_ms = their sum)",
                    "bytes_per_unit": "16 B per photon returned (SURVEY.md 8(d))",
                    "global": g, "caustic_kernel": dict(c, kernel=KNN_KINDS.get(kind[1], str(kind[1])))}
        # frame-level figure, BASELINE.md section 3.4: every k-NN photon returned (both maps) x 16 B
        # plus the 12-B output pixel per sample, over the whole frame's wall time, against the
        # N GPUs' aggregate peak
        frame_bytes = (agg["ph0"] + agg["ph1"]) * BYTES_PER_PHOTON + \
            BYTES_PER_SAMPLE * samples_per_step * a.steps
        frame_ach = frame_bytes / elapsed / 1e9
        roofline["frame_achieved"] = round(frame_ach, 2)
        roofline["frame_frac"] = round(frame_ach / (HBM_PEAK_GBPS * n_gpus), 5)
        roofline["frame_bytes_per_sample"] = round(frame_bytes / (samples_per_step * a.steps), 1)
        cpu = None
        if not a.no_cpu_baseline and n_gpus == 1:
            cpu = cpu_baseline(a)
        rgb = last.get("rgb")
        sha = hashlib.sha256(rgb.tobytes()).hexdigest()[:16] if rgb is not None else None
        want = EXPECTED_SHA16.get((a.scene, a.res, a.aa, a.global_photons, a.caustic_photons,
                                   a.seed, a.extra.strip()))
        check = None
        if sha is not None and want is not None:
            check = {"expected_1gpu": want, "equal": sha == want}
        par = {"single": "1 GPU",
               "device-set": f"one process, device set {devices}: tiles{a.tile}x{a.tile} % {n_gpus}, "
                             "ncclSend/ncclRecv tile gather onto device 0",
               "torchrun": f"one process per GPU: tiles{a.tile}x{a.tile} % {n_gpus}, packed shards "
                           "gathered to rank 0 over RCCL"}[mode]
        line = {
            "metric": "Mpixel-samples/sec (and ms/frame) at 1024^2 aa=2, 1M+1M photons",
            "value": round(value, 4), "unit": "Mpixel-samples/s", "n_gpus": n_gpus,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms_per_step, 2),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f64 (shading/geometry), f32 (photon positions)",
            "data": f"reference input scene tests/scenes/{a.scene} (no synthetic data; photon maps "
                    "traced from it with a fixed seed)",
            "config": {"workload": f"{a.scene} {w}x{h} aa={aa} "
                                   f"{a.global_photons}+{a.caustic_photons} photons {a.extra}".strip(),
                       "pixel_samples_per_frame": samples_per_frame,
                       "parallelism": par,
                       "photon_map_s": round(photon_s, 3),
                       "global_stored": pst["global_stored"],
                       "caustic_stored": pst["caustic_stored"]},
            "image_sha16": sha,
            "image_check": check,
            "topology": topo,
            "roofline": roofline, "cpu_baseline": cpu,
            "step_ms": step_ms,
            # the first (cold) frame, what the drop-in CLI renders: first warmup step
            "first_frame_ms": first_ms,
        }
        if shard is not None:
            line["shard"] = {"shard": shard[0], "nshards": shard[1], "pixels": npix_shard,
                             "pixel_samples_per_step": samples_per_step,
                             "ms_per_shard": round(ms_per_step, 1),
                             "note": f"one GPU rendering tile shard {shard[0]} of {shard[1]}: an "
                                     f"{shard[1]}-GPU frame takes about the slowest shard's time"}
        if mode == "device-set":
            line["device_set"] = {"devices": devices,
                                  "device_render_ms_max": round(agg["devmax"] / a.steps * 1e3, 2),
                                  "device_render_ms_min": round(agg["devmin"] / a.steps * 1e3, 2),
                                  "gather_ms": round(agg["gather"] / a.steps * 1e3, 3),
                                  "knn_kernel_ms_per_device_per_frame":
                                      round((agg["ms0"] + agg["ms1"]) / a.steps / n_gpus, 2)}
        print(json.dumps(line), flush=True)
    r.close()
    if dist is not None:
        dist.destroy_process_group()
    if rank == 0 and check is not None and not check["equal"]:
        raise SystemExit(f"image_sha16 {sha} differs from the 1-GPU frame's {want} "
                         f"({n_gpus} GPUs, {mode})")


if __name__ == "__main__":
    main()
