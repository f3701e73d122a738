"""Multi-GPU image-tile sharding for RenderImage (one process per GPU).

The reference's render threads each take the column interleave i % THREADS
(render.cpp:90). Here the frame is cut into tile x tile output-pixel tiles instead, and rank r
renders tiles t with t % world == r (gi_render_tiles, gi_host.cpp). Tile t sits at
((t % ntx) * tile, (t // ntx) * tile). Each rank holds a full-size f32 image that is zero
outside its tiles, so one sum-reduce to rank 0 is the gather. There is no other
communication: every rank builds the identical photon maps from the same seed.
"""
import numpy as np


def tile_owner_map(width, height, tile, world):
    """[height, width] int array: the rank that renders each output pixel."""
    ntx = (width + tile - 1) // tile
    ys, xs = np.mgrid[0:height, 0:width]
    t = (ys // tile) * ntx + (xs // tile)
    return (t % world).astype(np.int32)


def gather_to_rank0(img, dist, device=None):
    """Sum-reduce each rank's partial f32 image [h, w, 3] onto rank 0 (disjoint tiles, so
    the sum is the gather). `dist` is torch.distributed (RCCL on GPUs, gloo on CPU). Returns
    the full image on rank 0, None elsewhere."""
    import torch
    t = torch.from_numpy(np.ascontiguousarray(img, dtype=np.float32))
    if device is not None:
        t = t.to(device)
    dist.reduce(t, dst=0)
    if dist.get_rank() == 0:
        return t.cpu().numpy()
    return None


def render_sharded(renderer, aa, width, height, tile, rank, world, dist, device=None):
    """One frame on `world` ranks: this rank's tiles, then the gather to rank 0.
    Returns (full f32 image on rank 0 / None, this rank's render stats)."""
    img, st = renderer.render_tiles(aa, width, height, tile, rank, world)
    return gather_to_rank0(img, dist, device), st
