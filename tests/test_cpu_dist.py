"""Multi-rank tile sharding and gather (gi_dist.py) on CPU with the gloo backend, world size
2 and 3. The renderer is replaced by a stand-in with gi_render_tiles' contract: a full-size f32
image that holds this rank's tiles and zeros elsewhere (gi_host.cpp gi_render_tiles). Each rank
sends only its own pixels (checked: the gathered buffers hold 1/world of the frame). The
device-side composition of real tiles is covered by test_gpu_render.py, and the single-process
device-set gather by test_gpu_features.py."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import gi_dist


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def reference_image(w, h):
    ys, xs = np.mgrid[0:h, 0:w]
    return np.stack([xs * 0.01, ys * 0.02, (xs + ys) * 0.003], -1).astype(np.float32)


class FakeTiles:
    def render_tiles(self, aa, w, h, tile, rank, world):
        own = gi_dist.tile_owner_map(w, h, tile, world) == rank
        return np.where(own[..., None], reference_image(w, h), 0.0).astype(np.float32), \
            {"pixels": int(own.sum())}


class FakePacked:
    """gi_render_tiles_packed / gi_compose_tiles contract on host memory: the shard's pixels in
    packed order, 16 B each (f32 RGB + u8 RGB bits), written through a raw pointer."""
    packed_host_memory = True   # opts in to the packed path with a CPU device

    @staticmethod
    def _view(ptr, n):
        import ctypes as C
        return np.ctypeslib.as_array((C.c_float * (4 * n)).from_address(ptr)).reshape(n, 4)

    def render_tiles_packed(self, aa, w, h, tile, rank, world, ptr, cap):
        pix = gi_dist.shard_pixel_list(w, h, tile, rank, world)
        assert len(pix) <= cap
        ref = reference_image(w, h)
        v = self._view(ptr, cap)
        for i, (x, y) in enumerate(pix):
            v[i, :3] = ref[y, x]
        return len(pix), {"pixels": len(pix)}

    def compose_tiles(self, w, h, tile, world, ptr, stride, want_float=True):
        full = np.zeros((h, w, 3), dtype=np.float32)
        v = self._view(ptr, stride * world).reshape(world, stride, 4)
        for s in range(world):
            for i, (x, y) in enumerate(gi_dist.shard_pixel_list(w, h, tile, s, world)):
                full[y, x] = v[s, i, :3]
        return (full * 255).astype(np.uint8), full


class DevicePacked(FakeTiles):
    """A renderer whose packed entry points take device pointers only (like gi_amd.Renderer):
    given a CPU device, render_sharded must take the host path and never call them."""
    def render_tiles_packed(self, *a):
        raise AssertionError("packed path taken with a CPU device")

    def compose_tiles(self, *a, **k):
        raise AssertionError("packed path taken with a CPU device")


def _worker(rank, world, port, w, h, tile, q, packed=False):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sent = []
        real_gather = dist.gather

        def spy(t, parts=None, dst=0):
            sent.append(t.numel())
            return real_gather(t, parts, dst=dst)
        dist.gather = spy
        if packed == "device_only":
            import torch
            img, st = gi_dist.render_sharded(DevicePacked(), 0, w, h, tile, rank, world, dist,
                                             torch.device("cpu"))
        elif packed:
            import torch
            img, st = gi_dist.render_sharded(FakePacked(), 0, w, h, tile, rank, world, dist,
                                             torch.device("cpu"))
            img = None if img is None else img[1]
        else:
            img, st = gi_dist.render_sharded(FakeTiles(), 0, w, h, tile, rank, world, dist)
        q.put((rank, st["pixels"], None if img is None else img, sent))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("packed", [False, True, "device_only"],
                         ids=["host", "packed", "cpu_device_host_path"])
@pytest.mark.parametrize("world,w,h,tile", [(2, 70, 45, 16), (3, 64, 64, 16), (8, 130, 72, 16)])
def test_sharded_gather_equals_full_frame(world, w, h, tile, packed):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, w, h, tile, q, packed))
             for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort(key=lambda x: x[0])
    assert sum(o[1] for o in out) == w * h             # every pixel rendered exactly once
    np.testing.assert_array_equal(out[0][2], reference_image(w, h))
    assert all(o[2] is None for o in out[1:])
    # one gather per rank of at most the largest shard (not the whole frame)
    biggest = int(np.bincount(gi_dist.tile_owner_map(w, h, tile, world).ravel()).max())
    for o in out:
        assert o[3] == [biggest * (4 if packed is True else 3)]
        assert biggest * world < w * h + tile * tile * world


def test_shard_pixel_list_matches_owner_map():
    w, h, tile, world = 70, 45, 16, 3
    own = gi_dist.tile_owner_map(w, h, tile, world)
    seen = np.zeros((h, w), dtype=int)
    for s in range(world):
        pix = gi_dist.shard_pixel_list(w, h, tile, s, world)
        assert len(pix) == gi_dist.shard_sizes(w, h, tile, world)[s]
        for x, y in pix:
            assert own[y, x] == s
            seen[y, x] += 1
    assert np.all(seen == 1)


def test_tile_owner_map_diagonal():
    m = gi_dist.tile_owner_map(40, 20, 16, 2)
    # 3 x 2 tiles, owner = (tile x + tile y) % 2
    assert m[0, 0] == 0 and m[0, 16] == 1 and m[0, 32] == 0
    assert m[16, 0] == 1 and m[16, 16] == 0 and m[16, 39] == 1
    # 64 tiles per row (C2's 1024^2 in 16^2 tiles) on 8 ranks: every run of 8 tiles along a row
    # or a column meets all 8 ranks (t % 8 would give each rank whole tile columns)
    m = gi_dist.tile_owner_map(1024, 1024, 16, 8)[::16, ::16]
    for k in range(0, 64, 8):
        assert sorted(m[5, k:k + 8]) == list(range(8))
        assert sorted(m[k:k + 8, 7]) == list(range(8))
    assert np.bincount(m.ravel()).tolist() == [512] * 8
