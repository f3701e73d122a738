"""Multi-GPU measurement paths on one MI355X (render.cpp:90, 188-199).

- gi_render_tiles_packed + gi_compose_tiles (the torchrun path of bench.py / gi_dist.py): every
  shard rendered into a packed device buffer, composed on the device, equals gi_render_image bit
  for bit.
- bench.py's N-GPU modes reach the image the one-GPU run renders: `--gpus 2` with GI_DEVICES=0,0
  (the drop-in's device set in one process, peer-copy gather) and torchrun with two gloo ranks
  on the same GPU (packed shards, the gather through host memory since both ranks share one
  device; the RCCL gather itself needs distinct GPUs and runs on the driver's 8-GPU node).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import gi_amd
import gpu_util

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("nshards,tile", [(1, 16), (3, 16), (4, 8)])
def test_packed_shards_compose_full_image(renderer, nshards, tile):
    import torch
    args = [gpu_util.scene("cornell.scn"), "/tmp/p.png", "-resolution", "53", "37", "-aa", "1",
            "-global", "20000", "-caustic", "20000", "-it", "8", "-tt", "4", "-st", "4",
            "-seed", "3"]
    ref, reff, _st, _ = gpu_util.run_gpu(renderer, args, want_float=True)
    w, h = 53, 37
    sizes = [renderer.shard_pixels(w, h, tile, s, nshards) for s in range(nshards)]
    assert sum(sizes) == w * h
    m = max(sizes)
    buf = torch.zeros((nshards, m, 4), dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()
    for s in range(nshards):
        n, st = renderer.render_tiles_packed(1, w, h, tile, s, nshards,
                                             buf[s].data_ptr(), m)
        assert n == sizes[s]
        assert st["screen_rays"] > 0
    rgb, rgbf = renderer.compose_tiles(w, h, tile, nshards, buf.data_ptr(), m, want_float=True)
    np.testing.assert_array_equal(rgb, ref)
    np.testing.assert_array_equal(rgbf, reff)


def test_packed_capacity_is_checked(renderer):
    import torch
    buf = torch.zeros((4, 4), dtype=torch.float32, device="cuda:0")
    with pytest.raises(gi_amd.GiError):
        renderer.render_tiles_packed(0, 32, 32, 16, 0, 2, buf.data_ptr(), 4)


BENCH = ["--res", "48", "--aa", "1", "--steps", "1", "--warmup", "0", "--no-cpu-baseline",
         "--global-photons", "30000", "--caustic-photons", "30000"]


def run_bench(extra_args, env_extra, launcher=None, timeout=600):
    env = dict(os.environ)
    env.update(env_extra)
    cmd = (launcher or [sys.executable]) + [os.path.join(ROOT, "bench.py")] + BENCH + extra_args
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_device_set_matches_one_gpu():
    one = run_bench(["--gpus", "1"], {})
    two = run_bench(["--gpus", "2"], {"GI_DEVICES": "0,0"})
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["image_sha16"] == one["image_sha16"]
    assert two["device_set"]["devices"] == [0, 0]
    assert two["device_set"]["gather_ms"] >= 0.0
    assert two["roofline"]["global"]["queries_per_launch"] > 0
    # the line says what ran where (gi_device_info): both entries on GPU 0, one PCI bus; with
    # distinct devices comm_count is the RCCL communicator's rank count
    topo = two["topology"]
    assert topo["mode"] != "single" and topo["devices"] == [0, 0]
    assert len(topo["pci_bus"]) == 2 and topo["distinct_pci_bus"] == 1
    assert topo["comm_count"] in (0, 2)


def test_bench_torchrun_packed_matches_one_gpu():
    one = run_bench(["--gpus", "1"], {})
    launcher = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
                "2", "--master-addr", "127.0.0.1", "--master-port", "29533"]
    # two ranks on one GPU: LOCAL_RANK 1 is mapped onto the same device; gloo carries the gather
    two = run_bench(["--gpus", "2"], {"GI_BENCH_BACKEND": "gloo", "GI_BENCH_SAME_GPU": "1"},
                    launcher=launcher)
    assert two["n_gpus"] == 2
    assert two["image_sha16"] == one["image_sha16"]
    topo = two["topology"]
    assert topo["mode"] == "torchrun" and topo["comm_count"] == 2
    assert sorted(x["rank"] for x in topo["ranks"]) == [0, 1]
