"""Multi-GPU image-tile sharding for RenderImage (one process per GPU, torchrun).

The reference's render threads each take the column interleave i % THREADS
(render.cpp:90). Here the frame is cut into tile x tile output-pixel tiles instead, and rank r
renders tiles t with t % world == r (gi_render_tiles, gi_host.cpp). Tile t sits at
((t % ntx) * tile, (t // ntx) * tile). Each rank then sends ONLY its own pixels -- packed in
row-major order of the pixels it owns, 1/world of the image -- to rank 0 with one gather (RCCL
over xGMI on GPUs, gloo on CPU), and rank 0 scatters them into the frame. There is no other
communication: every rank builds the identical photon maps from the same seed.

(The single-process drop-in does the same over a device set in C++: gi_create_devices.)
"""
import numpy as np


def tile_owner_map(width, height, tile, world):
    """[height, width] int array: the rank that renders each output pixel."""
    ntx = (width + tile - 1) // tile
    ys, xs = np.mgrid[0:height, 0:width]
    t = (ys // tile) * ntx + (xs // tile)
    return (t % world).astype(np.int32)


def gather_tiles_to_rank0(img, owner, dist, device=None):
    """Gather every rank's own pixels of its partial f32 image [h, w, 3] (zeros elsewhere) onto
    rank 0. Each rank sends a [max_count, 3] buffer (its pixels first, padding after: the shard
    sizes differ by at most one tile). Returns the full image on rank 0, None elsewhere."""
    import torch
    rank, world = dist.get_rank(), dist.get_world_size()
    counts = np.bincount(owner.ravel(), minlength=world)
    m = int(counts.max())
    buf = np.zeros((m, 3), dtype=np.float32)
    buf[:counts[rank]] = img[owner == rank]
    t = torch.from_numpy(buf)
    if device is not None:
        t = t.to(device)
    if rank == 0:
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.gather(t, parts, dst=0)
        full = np.zeros(img.shape, dtype=np.float32)
        for r in range(world):
            full[owner == r] = parts[r][:counts[r]].cpu().numpy()
        return full
    dist.gather(t, None, dst=0)
    return None


def render_sharded(renderer, aa, width, height, tile, rank, world, dist, device=None):
    """One frame on `world` ranks: this rank's tiles, then the tile gather to rank 0.
    Returns (full f32 image on rank 0 / None, this rank's render stats)."""
    img, st = renderer.render_tiles(aa, width, height, tile, rank, world)
    owner = tile_owner_map(width, height, tile, world)
    return gather_tiles_to_rank0(img, owner, dist, device), st
