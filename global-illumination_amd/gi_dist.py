"""Multi-GPU image-tile sharding for RenderImage (one process per GPU, torchrun).

The reference's render threads each take the column interleave i % THREADS
(render.cpp:90). Here the frame is cut into tile x tile output-pixel tiles instead, dealt
diagonally: tile (tx, ty) goes to rank (tx + ty) % world, so every run of `world` tiles along a
row or a column meets every rank (a plain t % world deals whole tile columns when the row's tile
count is a multiple of world, and the glass sphere's expensive tiles then fall on few ranks).
Tile t sits at ((t % ntx) * tile, (t // ntx) * tile).
There is no other communication: every rank builds the identical photon maps from the same
seed, and each rank sends only its own pixels to rank 0 in one gather.

Device path (GPU ranks, RCCL): gi_render_tiles_packed leaves the shard in a device buffer,
16 B per owned pixel (f32 RGB + the u8 RGB), so only 1/world of the frame is sent and nothing
goes through host memory before rank 0. Rank 0 gathers the packed buffers into one device tensor
and gi_compose_tiles scatters them into the frame on its device.

Host path (gloo on CPU, and renderers without the packed entry point): gi_render_tiles' full
f32 image holding this rank's tiles, its own pixels picked out on the host.

(The single-process drop-in does the same over a device set in C++: gi_create_devices.)
"""
import numpy as np


def tile_owner_map(width, height, tile, world):
    """[height, width] int array: the rank that renders each output pixel."""
    ntx = (width + tile - 1) // tile
    ys, xs = np.mgrid[0:height, 0:width]
    return (((ys // tile) + (xs // tile)) % world).astype(np.int32)


def shard_pixel_list(width, height, tile, shard, world):
    """[(x, y)] of one shard in its packed order (gi_host.cpp shard_pixels): tiles by id,
    rows then columns inside a tile."""
    ntx, nty = (width + tile - 1) // tile, (height + tile - 1) // tile
    out = []
    for t in range(ntx * nty):
        if (t % ntx + t // ntx) % world != shard:
            continue
        x0, y0 = (t % ntx) * tile, (t // ntx) * tile
        for y in range(y0, min(height, y0 + tile)):
            for x in range(x0, min(width, x0 + tile)):
                out.append((x, y))
    return out


def shard_sizes(width, height, tile, world):
    """Pixels each rank owns (its packed buffer length)."""
    return np.bincount(tile_owner_map(width, height, tile, world).ravel(), minlength=world)


def gather_tiles_to_rank0(img, owner, dist, device=None):
    """Host path: gather every rank's own pixels of its partial f32 image [h, w, 3] (zeros
    elsewhere) onto rank 0. Each rank sends a [max_count, 3] buffer (its pixels first, then
    padding to the largest shard: with the diagonal deal, tile (tx, ty) on rank (tx + ty) % N,
    shard sizes can differ by more than one tile). Returns the full image on rank 0, None
    elsewhere."""
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


def render_sharded_packed(renderer, aa, width, height, tile, rank, world, dist, device):
    """Device path: this rank's tiles packed into a buffer on `device`, one gather of the
    packed buffers onto rank 0, composed there. Returns ((rgb8, rgbf) on rank 0 / None, this
    rank's render stats)."""
    import torch
    m = int(shard_sizes(width, height, tile, world).max())
    buf = torch.zeros((m, 4), dtype=torch.float32, device=device)
    if device.type == "cuda":
        torch.cuda.synchronize(device)  # the library writes on its own stream
    _n, st = renderer.render_tiles_packed(aa, width, height, tile, rank, world,
                                          buf.data_ptr(), m)
    # gloo has no device buffers: its gather goes through host copies (tests on one GPU)
    host = device.type == "cuda" and dist.get_backend() != "nccl"
    send = buf.cpu() if host else buf
    if rank == 0:
        allb = torch.empty((world, m, 4), dtype=torch.float32, device=send.device)
        dist.gather(send, list(allb.unbind(0)), dst=0)
        if host:
            allb = allb.to(device)
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        return renderer.compose_tiles(width, height, tile, world, allb.data_ptr(), m,
                                      want_float=True), st
    dist.gather(send, None, dst=0)
    return None, st


def render_sharded(renderer, aa, width, height, tile, rank, world, dist, device=None):
    """One frame on `world` ranks: this rank's tiles, then the tile gather to rank 0.
    Returns (full image on rank 0 / None, this rank's render stats): (rgb8, rgbf) on the
    device path, the f32 image on the host path.

    The packed path hands raw data_ptr()s to gi_render_tiles_packed / gi_compose_tiles, which
    take DEVICE pointers (gi.h): it is taken only for a CUDA device, or for a renderer that says
    its packed entry points read host memory (`packed_host_memory`, the CPU test stand-in)."""
    packed_ok = device is not None and hasattr(renderer, "render_tiles_packed") and (
        device.type == "cuda" or getattr(renderer, "packed_host_memory", False))
    if packed_ok:
        return render_sharded_packed(renderer, aa, width, height, tile, rank, world, dist, device)
    img, st = renderer.render_tiles(aa, width, height, tile, rank, world)
    owner = tile_owner_map(width, height, tile, world)
    return gather_tiles_to_rank0(img, owner, dist, device), st
