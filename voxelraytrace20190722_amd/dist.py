"""Multi-GPU frame partition: which rank renders what, the
packed per-rank buffers, and their re-assembly on rank 0.

The device path (bench.py, RCCL) is `vrt_render_tiles_device` + one
`gather` + `vrt_unpack_tiles_device`; these numpy helpers state the same
layouts on the host.  They are the reference for tests/test_dist.py (gloo,
world_size 2, CPU) and the host-staged gloo rehearsal of bench.py, and
tests/test_gpu.py checks that the device buffers equal them bit for bit.

Primary frames: the render area is 8x8-pixel tiles t = ty*ntx + tx (ntx =
nx//8, nty = ny//8); tile t belongs to rank t % nranks; a rank's buffer holds
its tiles in order k = 0.. (t = rank + k*nranks), 64 pixels each, row-major
inside the tile, 3 floats per pixel, `tiles_per_rank * 192` floats (unused
tail zero).  Secondary frames (config 5): the same tile deal (tile t ->
rank t % nranks); every rank writes only the pixels of its tiles into a
zeroed image, so a SUM reduce re-assembles it exactly.
"""
import numpy as np


def tile_grid(nx, ny):
    return nx // 8, ny // 8


def tiles_per_rank(nx, ny, nranks):
    """== vrt_tiles_per_rank (ceil(ntiles / nranks))."""
    ntx, nty = tile_grid(nx, ny)
    return (ntx * nty + nranks - 1) // nranks


def rank_tiles(nx, ny, rank, nranks):
    ntx, nty = tile_grid(nx, ny)
    return np.arange(rank, ntx * nty, nranks)


def pack_tiles_host(img, rank, nranks):
    """This rank's packed tile buffer from a full (ny, nx, 3) image."""
    ny, nx = img.shape[:2]
    ntx, _ = tile_grid(nx, ny)
    tpr = tiles_per_rank(nx, ny, nranks)
    buf = np.zeros((tpr, 64, 3), np.float32)
    for k, t in enumerate(rank_tiles(nx, ny, rank, nranks)):
        tx, ty = t % ntx, t // ntx
        buf[k] = img[ty * 8:ty * 8 + 8, tx * 8:tx * 8 + 8].reshape(64, 3)
    return buf.reshape(-1)


def unpack_tiles_host(gathered, nx, ny, nranks):
    """== vrt_unpack_tiles_device: (nranks, tiles_per_rank*192) -> (ny, nx, 3);
    pixels outside the tile grid are zero."""
    ntx, nty = tile_grid(nx, ny)
    tpr = tiles_per_rank(nx, ny, nranks)
    g = np.asarray(gathered, np.float32).reshape(nranks, tpr, 8, 8, 3)
    img = np.zeros((ny, nx, 3), np.float32)
    for t in range(ntx * nty):
        r, k = t % nranks, t // nranks
        tx, ty = t % ntx, t // ntx
        img[ty * 8:ty * 8 + 8, tx * 8:tx * 8 + 8] = g[r, k]
    return img


def secondary_mask(nx, ny, rank, nranks):
    """(ny, nx) bool: the pixels `rank` computes in a config-5 frame."""
    ntx, nty = tile_grid(nx, ny)
    t = np.arange(ntx * nty).reshape(nty, ntx)
    mine = np.repeat(np.repeat((t % nranks) == rank, 8, 0), 8, 1)
    m = np.zeros((ny, nx), bool)
    m[:nty * 8, :ntx * 8] = mine
    return m
