"""Multi-GPU frame partition: which rank renders what, the
packed per-rank buffers, and their re-assembly on rank 0.

The device path (bench.py, RCCL) is `vrt_render_tiles_device` + one
`gather` + `vrt_unpack_tiles_device`; these numpy helpers state the same
layouts on the host.  They are the reference for tests/test_dist.py (gloo,
world_size 2, CPU) and the host-staged gloo rehearsal of bench.py, and
tests/test_gpu.py checks that the device buffers equal them bit for bit.

The tile deal (include/vrt.h, vrt_internal.h `tile_deal`): the render area
is the ntx x nty grid of 8x8-pixel tiles (ntx = nx//8, nty = ny//8).  With
G = the library's deal block (G = 1 for one rank), the whole G x G blocks of
tiles are dealt round-robin in block raster order (block j -> rank
j % nranks; from 2 ranks on rank 0 gets fewer, see deal_weight); the tiles outside the whole-block region -- the right strip
(rows above the bottom strip), then the bottom strip, each in raster order
-- continue the deal one tile at a time (leftover i -> rank (F + i) %
nranks, F = whole blocks).  A rank's k-th tile: its blocks' tiles first
(block order, row-major inside a block), then its leftover tiles.  A rank's
buffer holds its tiles in that order, 64 pixels each, row-major inside the
tile, 3 floats per pixel, `tiles_per_rank * 192` floats (the largest share;
unused tail zero).  Secondary frames (config 5): the same deal and the same
packed layout with 1 float per pixel (`tiles_per_rank * 64` floats): every
rank renders its pixels, packs its tiles (vrt_pack_tiles_c_device), one
gather brings the buffers to rank 0, which re-assembles the visibility image
(vrt_unpack_tiles_c_device) -- the primary frame's collective.
"""
import numpy as np


def tile_grid(nx, ny):
    return nx // 8, ny // 8


def deal_block():
    """G of the library's tile deal (vrt_tile_deal_block)."""
    from ._ffi import lib
    return int(lib().vrt_tile_deal_block())


def deal_weight(nranks):
    """(m, V) of the weighted deal (vrt_internal.h VRT_DEAL_WEIGHT): from 2
    ranks on, rank 0 -- which also gathers and re-assembles the frame -- gets
    (m-1)/m of another rank's blocks, m = max(2, SPAN // nranks); the whole
    blocks run in periods of V = m*nranks - 1 turns, position p of a period
    going to rank nranks-1 - p % nranks.  (0, 0): plain round robin.  The
    switch and SPAN are the library build's (vrt_build_flag), as deal_block's
    G is, so a variant build and these helpers deal the same tiles."""
    from .api import build_flag
    if nranks < 2 or not build_flag("VRT_DEAL_WEIGHT"):
        return 0, 0
    m = max(2, int(build_flag("VRT_DEAL_SPAN")) // nranks)
    return m, m * nranks - 1


def deal_owner(nx, ny, nranks, g=None):
    """(nty, ntx) arrays: each tile's rank and its index k in that rank's list."""
    ntx, nty = tile_grid(nx, ny)
    g = (deal_block() if g is None else g) if nranks > 1 else 1
    bx, by = ntx // g, nty // g
    nfull = bx * by
    rank = np.zeros((nty, ntx), np.int64)
    slot = np.zeros((nty, ntx), np.int64)
    counts = np.zeros(nranks, np.int64)
    m, period = deal_weight(nranks)
    for j in range(nfull):  # whole blocks, block raster order
        r = nranks - 1 - (j % period) % nranks if period else j % nranks
        y0, x0 = (j // bx) * g, (j % bx) * g
        for w in range(g * g):
            ty, tx = y0 + w // g, x0 + w % g
            rank[ty, tx] = r
            slot[ty, tx] = counts[r]
            counts[r] += 1
    leftovers = [(ty, tx) for ty in range(by * g) for tx in range(bx * g, ntx)]
    leftovers += [(ty, tx) for ty in range(by * g, nty) for tx in range(ntx)]
    for i, (ty, tx) in enumerate(leftovers):
        r = (nfull + i) % nranks
        rank[ty, tx] = r
        slot[ty, tx] = counts[r]
        counts[r] += 1
    return rank, slot, counts


def tiles_per_rank(nx, ny, nranks, g=None):
    """== vrt_tiles_per_rank (the largest share)."""
    return int(deal_owner(nx, ny, nranks, g)[2].max()) if (nx // 8) * (ny // 8) else 0


def rank_tiles(nx, ny, rank, nranks, g=None):
    """This rank's tiles (ty*ntx + tx) in its order k = 0, 1, ..."""
    ntx, _ = tile_grid(nx, ny)
    rk, sl, cnt = deal_owner(nx, ny, nranks, g)
    ty, tx = np.nonzero(rk == rank)
    order = np.argsort(sl[ty, tx])
    return (ty * ntx + tx)[order]


def pack_tiles_host(img, rank, nranks, g=None):
    """This rank's packed tile buffer from a full (ny, nx, 3) image, or from a
    (ny, nx) / (ny, nx, c) image of c floats per pixel (== vrt_pack_tiles_c_device)."""
    ny, nx = img.shape[:2]
    c = 1 if img.ndim == 2 else img.shape[2]
    ntx, _ = tile_grid(nx, ny)
    tpr = tiles_per_rank(nx, ny, nranks, g)
    buf = np.zeros((tpr, 64, c), np.float32)
    for k, t in enumerate(rank_tiles(nx, ny, rank, nranks, g)):
        tx, ty = t % ntx, t // ntx
        buf[k] = img[ty * 8:ty * 8 + 8, tx * 8:tx * 8 + 8].reshape(64, c)
    return buf.reshape(-1)


def unpack_tiles_host(gathered, nx, ny, nranks, g=None, comps=3):
    """== vrt_unpack_tiles_device (comps = 3) / vrt_unpack_tiles_c_device:
    (nranks, tiles_per_rank*64*comps) -> (ny, nx, comps), (ny, nx) for
    comps = 1; pixels outside the tile grid are zero."""
    ntx, nty = tile_grid(nx, ny)
    tpr = tiles_per_rank(nx, ny, nranks, g)
    rk, sl, _ = deal_owner(nx, ny, nranks, g)
    gg = np.asarray(gathered, np.float32).reshape(nranks, tpr, 8, 8, comps)
    img = np.zeros((ny, nx, comps), np.float32)
    for ty in range(nty):
        for tx in range(ntx):
            img[ty * 8:ty * 8 + 8, tx * 8:tx * 8 + 8] = gg[rk[ty, tx], sl[ty, tx]]
    return img[:, :, 0] if comps == 1 else img


def secondary_mask(nx, ny, rank, nranks, g=None):
    """(ny, nx) bool: the pixels `rank` computes in a config-5 frame."""
    ntx, nty = tile_grid(nx, ny)
    rk, _, _ = deal_owner(nx, ny, nranks, g)
    mine = np.repeat(np.repeat(rk == rank, 8, 0), 8, 1)
    m = np.zeros((ny, nx), bool)
    m[:nty * 8, :ntx * 8] = mine
    return m
