"""GPU parity tests (MI355X): the HIP path, called through the C ABI, against
the reference-pinned KATs, the golden fixtures and the live oracle.

Bar: bit-exact for every id, hit point, normal and colour (the shading is
float32 arithmetic reproduced op for op; the 1e-5 RGB tolerance the north
star allows is not needed and not used)."""
import numpy as np
import pytest

import pyoracle as po
import voxelraytrace20190722_amd as vrt
from conftest import golden

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def scene_from(z):
    return vrt.SceneData(z["pos"], z["nrm"], z["uv"], z["mat"], z["mat_tex"], z["mat_kd"], z["tex_dims"],
                         z["tex_off"], z["tex_data"])


def test_device_visible():
    assert vrt.device_count() >= 1


def test_device_mt_matches_reference_kat():
    z = golden("kat_raytri.npz")
    out, _ = vrt.device_selftest(mt_in=z["inp"])
    assert np.array_equal(out.view(np.uint64), z["out"].view(np.uint64))


def test_device_sat_matches_reference_kat():
    z = golden("kat_tribox.npz")
    _, out = vrt.device_selftest(sat_in=z["inp"])
    assert np.array_equal(out, z["out"])


@pytest.mark.parametrize("name", ["proxy", "soup"])
def test_render_matches_golden_fixture(name):
    z = golden(f"scene_{name}.npz")
    tree = vrt.VoxelOctree(scene_from(z), int(z["depth"]))
    k = 0
    while f"cam{k}" in z:
        c = z[f"cam{k}"]
        fw, fh, nx, ny = z[f"film{k}"]
        cam = vrt.Camera(float(c[0]), c[1:4], c[4:7], c[7:10])
        film = vrt.Film(float(fw), float(fh), int(nx), int(ny))
        rgb, so = tree.render(cam, film, samples=True, counters=True)
        assert np.array_equal(so["hit"], z[f"s{k}_hit"]), k
        assert np.array_equal(so["tri"], z[f"s{k}_tri"]), k
        assert np.array_equal(so["voxel"], z[f"s{k}_voxel"]), k
        assert np.array_equal(so["counters"], z[f"s{k}_counters"]), k
        assert np.array_equal(bits(so["rgb"]), bits(z[f"s{k}_rgb"])), k
        assert np.array_equal(bits(rgb), bits(z[f"img{k}"])), k
        k += 1


@pytest.fixture(scope="module")
def proxy_small():
    return vrt.SceneData.proxy(0.25, 2)


@pytest.mark.parametrize("depth", [1, 4, 6, 8])
def test_render_matches_oracle_live(proxy_small, depth):
    tree = vrt.VoxelOctree(proxy_small, depth)
    osc = po.Scene(proxy_small, depth)
    mn, mx = tree.root_box
    for pose, (nx, ny) in [(0, (48, 48)), (5, (64, 40)), (13, (40, 64))]:
        fov, eye, spot, up = vrt.sweep_pose(mn, mx, pose, 16)
        cam = vrt.Camera(fov, eye, spot, up)
        rgb, so = tree.render(cam, vrt.Film(1, 1, nx, ny), samples=True, counters=True)
        oc = po.camera(fov, eye, spot, up)
        orgb, oso = osc.render(oc, 1.0, 1.0, nx, ny, film_index=1, nthreads=8)
        for key in ("hit", "tri", "voxel", "counters"):
            assert np.array_equal(so[key], oso[key]), (depth, pose, key)
        assert np.array_equal(bits(so["rgb"]), bits(oso["rgb"]))
        assert np.array_equal(bits(rgb), bits(orgb))


@pytest.mark.parametrize("depth,detail", [(3, 0.25), (6, 0.25), (6, 1.0), (8, 0.25)])
def test_production_kernel_both_record_formats(depth, detail):
    """The uninstrumented k_render (uniform-leaf loads, per-scene RefRec48 /
    RefRec64 records) against the oracle: both leaf-record formats occur."""
    sd = vrt.SceneData.proxy(detail, 2)
    tree = vrt.VoxelOctree(sd, depth)
    info = tree.info
    wide = info.tri_refs >= 8 * max(1, info.nonempty_leaves)
    assert wide == (depth <= 6), (depth, info.tri_refs, info.nonempty_leaves)
    osc = po.Scene(sd, depth)
    mn, mx = tree.root_box
    for pose in (2, 9):
        fov, eye, spot, up = vrt.sweep_pose(mn, mx, pose, 16)
        rgb, so = tree.render(vrt.Camera(fov, eye, spot, up), vrt.Film(1, 1, 64, 64), samples=True)
        orgb, oso = osc.render(po.camera(fov, eye, spot, up), 1.0, 1.0, 64, 64, film_index=1, nthreads=8)
        for key in ("hit", "tri", "voxel"):
            assert np.array_equal(so[key], oso[key]), (depth, pose, key)
        assert np.array_equal(bits(rgb), bits(orgb)), (depth, pose)


def _random_rays(rng, n, mn, mx):
    c = (mn + mx) / 2
    ext = (mx - mn) / 2
    o = (c + rng.uniform(-1.3, 1.3, (n, 3)) * ext).astype(np.float32)
    d = rng.normal(0, 1, (n, 3)).astype(np.float32)
    zero = rng.random(n) < 0.15
    d[zero, rng.integers(0, 3, zero.sum())] = 0.0
    ax = rng.random(n) < 0.05
    d[ax] = 0.0
    d[ax, rng.integers(0, 3, ax.sum())] = 1.0
    rays = np.zeros((n, 8), np.float32)
    for i in range(n):
        tmin = 0.0 if i % 4 else float(rng.uniform(0, 0.3))
        tmax = vrt.FLT_MAX if i % 7 else float(rng.uniform(0.5, 3))
        rays[i] = vrt.make_ray(o[i], d[i], tmin, tmax)
    return rays


@pytest.mark.parametrize("depth", [5, 7, 9])
def test_ray_march_batch_matches_oracle(proxy_small, depth):
    tree = vrt.VoxelOctree(proxy_small, depth)
    osc = po.Scene(proxy_small, depth)
    mn, mx = tree.root_box
    rng = np.random.default_rng(depth)
    rays = _random_rays(rng, 6000, mn, mx)
    g = tree.ray_march(rays)
    o = osc.ray_march(rays)
    assert o["hit"].sum() > 1000
    assert np.array_equal(g["hit"], o["hit"])
    assert np.array_equal(g["tri"], o["tri"])
    assert np.array_equal(g["voxel"], o["voxel"])
    assert np.array_equal(bits(g["hit_p"]), bits(o["hit_p"]))
    assert np.array_equal(bits(g["normal"]), bits(o["normal"]))
    # secondary rays from the hit points (config 5 pattern: tmin = leaf size)
    h = o["hit"] == 1
    res = float(np.min((mx - mn) / 2.0 ** depth))
    sec = np.zeros((int(h.sum()), 8), np.float32)
    for j, (p, n) in enumerate(zip(o["hit_p"][h], o["normal"][h])):
        sec[j] = vrt.make_ray(p, n + rng.normal(0, 0.5, 3).astype(np.float32), res, vrt.FLT_MAX)
    g2, o2 = tree.ray_march(sec), osc.ray_march(sec)
    for key in ("hit", "tri", "voxel"):
        assert np.array_equal(g2[key], o2[key]), key
    assert np.array_equal(bits(g2["hit_p"]), bits(o2["hit_p"]))


def _extreme_rays(rng, n, mn, mx):
    """Raw rays (no normalisation) outside the kernels' fast path: huge and
    overflowing direction components (travorder distances +-inf and NaN),
    denormal and zero components, far origins, NaN / inf components, and
    odd [tmin, tmax] ranges."""
    c = (mn + mx) / 2
    ext = (mx - mn) / 2
    rays = np.zeros((n, 8), np.float32)
    for i in range(n):
        o = (c + rng.uniform(-1.2, 1.2, 3) * ext).astype(np.float32)
        d = rng.normal(0, 1, 3).astype(np.float32)
        k = i % 9
        if k == 0:
            d = (d / np.abs(d).max() * 3e38).astype(np.float32)  # distances overflow, +inf - inf = NaN
        elif k == 1:
            d[rng.integers(0, 3)] = np.float32(2e38) * np.sign(d[0] + 0.1)
        elif k == 2:
            d[rng.integers(0, 3)] = np.float32(1e-41)  # denormal component
        elif k == 3:
            d[:] = 0
            d[rng.integers(0, 3)] = 1e-40
        elif k == 4:
            o = (o * np.float32(1e20)).astype(np.float32)  # far origin (> 2^60)
            d = (c - o).astype(np.float32)
        elif k == 5:
            d[rng.integers(0, 3)] = np.nan
        elif k == 6:
            o[rng.integers(0, 3)] = np.inf
        elif k == 7:
            d = (d * np.float32(1e19)).astype(np.float32)  # |d| just above 2^64
        rays[i, :3], rays[i, 3:6] = o, d
        rays[i, 6], rays[i, 7] = [(0.0, vrt.FLT_MAX), (-np.inf, np.inf), (0.5, 0.1), (0.0, 0.2)][i % 4]
    return rays


def _same_f32(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    both_nan = np.isnan(a) & np.isnan(b)
    return bool(np.all(both_nan | (bits(a) == bits(b))))


@pytest.mark.parametrize("depth", [4, 7])
def test_ray_march_extreme_rays_match_oracle(proxy_small, depth):
    """The exact (non-fast) traversal path, including libstdc++'s insertion
    sort on NaN distances, against the oracle's literal restatement."""
    tree = vrt.VoxelOctree(proxy_small, depth)
    osc = po.Scene(proxy_small, depth)
    mn, mx = tree.root_box
    rays = _extreme_rays(np.random.default_rng(100 + depth), 2700, mn, mx)
    g, o = tree.ray_march(rays), osc.ray_march(rays)
    assert o["hit"].sum() > 50
    for key in ("hit", "tri", "voxel"):
        assert np.array_equal(g[key], o[key]), key
    assert _same_f32(g["hit_p"], o["hit_p"])
    assert _same_f32(g["normal"], o["normal"])


@pytest.mark.parametrize("nranks,nx,ny", [(2, 200, 120), (3, 200, 120), (8, 200, 120), (3, 204, 122)])
def test_tile_partition_reassembles_image(proxy_small, nranks, nx, ny):
    """Per-rank tile renders + rank-major gather + unpack == one image render
    (sides that are multiples of 8: the 16-B chunk unpack k_unpack4; 204 x
    122: the per-pixel k_unpack, pixels outside the 8 * (n/8) area zero)."""
    import torch
    tree = vrt.VoxelOctree(proxy_small, 7)
    mn, mx = tree.root_box
    fov, eye, spot, up = vrt.sweep_pose(mn, mx, 2, 16)
    cam = vrt.Camera(fov, eye, spot, up)
    film = vrt.Film(1, 1, nx, ny)  # 25 x 15 tiles
    tpr = vrt.tiles_per_rank(film, nranks)
    dev = torch.device("cuda:0")
    gathered = torch.zeros((nranks, tpr * 192), dtype=torch.float32, device=dev)
    for r in range(nranks):
        tree.render_tiles_device(cam, film, r, nranks, 0, gathered[r].data_ptr(), None)
    img = torch.full((ny, nx, 3), 7.0, dtype=torch.float32, device=dev)
    vrt.unpack_tiles_device(film, nranks, gathered.data_ptr(), img.data_ptr(), None)
    torch.cuda.synchronize()
    direct = tree.render(cam, film)
    assert np.array_equal(bits(img.cpu().numpy()), bits(direct))
    # the device buffers are exactly the host statement of the layout
    from voxelraytrace20190722_amd import dist as vd
    g = gathered.cpu().numpy()
    for r in range(nranks):
        assert np.array_equal(bits(g[r]), bits(vd.pack_tiles_host(direct, r, nranks)))
    assert np.array_equal(bits(vd.unpack_tiles_host(g, nx, ny, nranks)), bits(direct))


def test_full_size_frame_properties():
    """1920x1080 at max_depth 8 on the full proxy: deterministic, equal to the
    image_layout device render, and a random pixel sample equals the oracle."""
    import torch
    sd = vrt.SceneData.proxy(1.0, 1)
    tree = vrt.VoxelOctree(sd, 8)
    mn, mx = tree.root_box
    fov, eye, spot, up = vrt.sweep_pose(mn, mx, 0, 16)
    cam = vrt.Camera(fov, eye, spot, up)
    film = vrt.Film(1, 1, 1920, 1080)
    a, so = tree.render(cam, film, samples=True)
    b = tree.render(cam, film)
    assert np.array_equal(bits(a), bits(b))
    d = torch.zeros((1080, 1920, 3), dtype=torch.float32, device="cuda:0")
    tree.render_tiles_device(cam, film, 0, 1, 1, d.data_ptr(), None)
    torch.cuda.synchronize()
    assert np.array_equal(bits(d.cpu().numpy()), bits(a))
    assert so["hit"].mean() > 0.5
    # spot-check 3000 random samples against the oracle at full size
    osc = po.Scene(sd, 8)
    oc = po.camera(fov, eye, spot, up)
    rng = np.random.default_rng(0)
    px = rng.integers(0, 1920, 750)
    py = rng.integers(0, 1080, 750)
    rays = np.concatenate([po.gen_rays4(oc, 1.0, 1.0, 1920, 1080, int(x), int(y)) for x, y in zip(px, py)])
    o = osc.ray_march(rays)
    idx = ((py.astype(np.int64) * 1920 + px)[:, None] * 4 + np.arange(4)).reshape(-1)
    assert np.array_equal(so["tri"][idx], o["tri"])
    assert np.array_equal(so["voxel"][idx], o["voxel"])
    assert np.array_equal(bits(so["rgb"][idx]), bits(osc.shade(rays)))


def test_4k_depth9_frame_sample_matches_oracle():
    """BASELINE configs[2] size (3840x2160, max_depth 9): device tile render
    == image render, and 2000 random samples equal the oracle's."""
    import torch
    sd = vrt.SceneData.proxy(1.0, 1)
    tree = vrt.VoxelOctree(sd, 9)
    mn, mx = tree.root_box
    fov, eye, spot, up = vrt.sweep_pose(mn, mx, 7, 16)
    cam = vrt.Camera(fov, eye, spot, up)
    film = vrt.Film(1, 1, 3840, 2160)
    a, so = tree.render(cam, film, samples=True)
    d = torch.zeros((2160, 3840, 3), dtype=torch.float32, device="cuda:0")
    tree.render_tiles_device(cam, film, 0, 1, 1, d.data_ptr(), None)
    torch.cuda.synchronize()
    assert np.array_equal(bits(d.cpu().numpy()), bits(a))
    osc = po.Scene(sd, 9)
    oc = po.camera(fov, eye, spot, up)
    rng = np.random.default_rng(1)
    px = rng.integers(0, 3840, 500)
    py = rng.integers(0, 2160, 500)
    rays = np.concatenate([po.gen_rays4(oc, 1.0, 1.0, 3840, 2160, int(x), int(y)) for x, y in zip(px, py)])
    o = osc.ray_march(rays)
    idx = ((py.astype(np.int64) * 3840 + px)[:, None] * 4 + np.arange(4)).reshape(-1)
    assert np.array_equal(so["tri"][idx], o["tri"])
    assert np.array_equal(so["voxel"][idx], o["voxel"])
    assert np.array_equal(bits(so["rgb"][idx]), bits(osc.shade(rays)))


def test_edge_scenes():
    # single triangle filling the view, empty scene (all sky), depth 11
    one = vrt.SceneData(np.array([[-5, -5, -1, 5, -5, -1, 0, 5, -1]], np.float32), np.ones((1, 9), np.float32))
    cam = vrt.Camera(vrt.to_radian(60), (0, 0, 1), (0, 0, 0), (0, 1, 0))
    film = vrt.Film(1, 1, 32, 32)
    for depth in (1, 11):
        tree = vrt.VoxelOctree(one, depth)
        osc = po.Scene(one, depth)
        rgb, so = tree.render(cam, film, samples=True, counters=True)
        orgb, oso = osc.render(po.camera(vrt.to_radian(60), (0, 0, 1), (0, 0, 0), (0, 1, 0)), 1.0, 1.0, 32, 32)
        assert np.array_equal(bits(rgb), bits(orgb))
        assert np.array_equal(so["counters"], oso["counters"])
    empty = vrt.SceneData(np.zeros((0, 9), np.float32), np.zeros((0, 9), np.float32))
    tree = vrt.VoxelOctree(empty, 5)
    rgb, so = tree.render(cam, film, samples=True)
    assert so["hit"].sum() == 0
    osc = po.Scene(empty, 5)
    orgb = osc.render(po.camera(vrt.to_radian(60), (0, 0, 1), (0, 0, 0), (0, 1, 0)), 1.0, 1.0, 32, 32,
                      samples=False)
    assert np.array_equal(bits(rgb), bits(orgb))


def test_secondary_matches_golden_fixture():
    z = golden("secondary_proxy.npz")
    tree = vrt.VoxelOctree(scene_from(z), int(z["depth"]))
    c = z["cam"]
    fw, fh, nx, ny = z["film"]
    cam = vrt.Camera(float(c[0]), c[1:4], c[4:7], c[7:10])
    vis, rays, d = tree.render_secondary(cam, vrt.Film(float(fw), float(fh), int(nx), int(ny)),
                                         spp=int(z["spp"]), ids=True)
    assert rays == int(z["rays"])
    for k in ("hit", "tri", "voxel"):
        assert np.array_equal(d[k], z[k]), k
    assert np.array_equal(bits(vis), bits(z["vis"]))


@pytest.mark.parametrize("spp", [1, 17, 64])
def test_secondary_matches_oracle_live(proxy_small, spp):
    tree = vrt.VoxelOctree(proxy_small, 7)
    osc = po.Scene(proxy_small, 7)
    mn, mx = tree.root_box
    fov, eye, spot, up = vrt.sweep_pose(mn, mx, 9, 16)
    film = vrt.Film(1, 1, 40, 24)
    vis, rays, d = tree.render_secondary(vrt.Camera(fov, eye, spot, up), film, spp=spp, ids=True)
    ovis, orays, od = osc.render_secondary(po.camera(fov, eye, spot, up), 1.0, 1.0, 40, 24, spp=spp)
    assert rays == orays
    for k in ("hit", "tri", "voxel"):
        assert np.array_equal(d[k], od[k]), k
    assert np.array_equal(bits(vis), bits(ovis))


@pytest.mark.parametrize("depth", [3, 6, 8])
def test_secondary_occlusion_walk_matches_ordered_walk(proxy_small, depth):
    """Without per-ray ids the kernel runs the occlusion walk (any-hit,
    direction-sign order): every ray's hit boolean -- hence the visibility
    image -- must equal the ordered walk's and the oracle's."""
    tree = vrt.VoxelOctree(proxy_small, depth)
    osc = po.Scene(proxy_small, depth)
    mn, mx = tree.root_box
    for pose in (3, 11):
        fov, eye, spot, up = vrt.sweep_pose(mn, mx, pose, 16)
        cam = vrt.Camera(fov, eye, spot, up)
        film = vrt.Film(1, 1, 48, 32)
        vis_any, rays_any = tree.render_secondary(cam, film, spp=64)
        vis, rays, d = tree.render_secondary(cam, film, spp=64, ids=True)
        ovis, orays, _ = osc.render_secondary(po.camera(fov, eye, spot, up), 1.0, 1.0, 48, 32, spp=64)
        assert rays_any == rays == orays
        assert np.array_equal(bits(vis_any), bits(vis)), (depth, pose)
        assert np.array_equal(bits(vis_any), bits(ovis)), (depth, pose)
        assert 0 < d["hit"].sum() < d["hit"].size  # both outcomes occur


@pytest.mark.parametrize("depth", [6, 8])
@pytest.mark.parametrize("flags,spp", [(0, 64), (vrt.TEST_SPILL_ALL, 64), (0, 17), (0, 1),
                                       (vrt.TEST_SPILL_ALL | vrt.TEST_STREAM_LEFTOVER, 64),
                                       (vrt.TEST_SEC_DEFER, 64), (vrt.TEST_SEC_DEFER, 17),
                                       (vrt.TEST_SEC_DEFER | vrt.TEST_SPILL_ALL, 64)])
def test_secondary_compaction_matches_oracle(proxy_small, depth, flags, spp):
    """Config-5 ray compaction: rays still walking when few
    lanes of their wave are go to a queue with their walk state and are
    resumed 64 to a wave.  Every ray's hit boolean and the visibility image
    equal the oracle's; flags=TEST_SPILL_ALL stops every wave at its first
    ended ray (and every resume round but the last), so nearly all rays are
    saved and resumed mid-walk at least once: the resume round walks them 64 to
    a wave as one stream: a pool of subtree pieces handed to idle lanes, a
    slot refilled with the next saved ray as soon as its ray ends
    (resume_stream); TEST_STREAM_LEFTOVER sends every odd
    chunk to the batch pool (occl_pool) launched after it; spp < 64 starts
    with idle lanes; TEST_SEC_DEFER sends every odd pixel from the fast-only
    walk kernel to the exact-walk launch after it (k_secondary_defer), as a
    pixel with a ray off the fast walk is."""
    tree = vrt.VoxelOctree(proxy_small, depth)
    osc = po.Scene(proxy_small, depth)
    mn, mx = tree.root_box
    fov, eye, spot, up = vrt.sweep_pose(mn, mx, 6, 16)
    film = vrt.Film(1, 1, 96, 64)
    vrt.set_test_flags(flags)
    try:
        vis, rays, d = tree.render_secondary(vrt.Camera(fov, eye, spot, up), film, spp=spp, ids="hit")
        counts = tree.secondary_spill_counts()
        stats = tree.secondary_spill_stats()
    finally:
        vrt.set_test_flags(0)
    ovis, orays, od = osc.render_secondary(po.camera(fov, eye, spot, up), 1.0, 1.0, 96, 64, spp=spp)
    if flags & vrt.TEST_SEC_DEFER:  # every odd pixel with a primary hit went to the exact-walk launch
        assert stats["deferred_pixels"] > 96 * 64 // 8, stats
    else:  # the fast-only kernel ran: no pixel of this view has a ray off the fast walk
        assert stats["deferred_pixels"] <= 4, stats
    assert rays == orays
    assert np.array_equal(d["hit"], od["hit"])
    assert np.array_equal(bits(vis), bits(ovis))
    assert vrt.build_flag("VRT_SEC_SPILL_T") > 0  # the compaction is built in
    if flags & vrt.TEST_SPILL_ALL:  # every wave stops at its first ended ray: most rays are saved
        # (of the pixels the fast-only kernel walks: half of them with TEST_SEC_DEFER)
        assert counts[0] > rays // (40 if flags & vrt.TEST_SEC_DEFER else 20), (counts, rays)
    # the one streaming resume round walks every saved ray to its end: no
    # later queue is ever filled
    assert counts[1:] == [0, 0, 0], counts


@pytest.mark.parametrize("nx,ny,nranks", [(72, 40, 3), (512, 40, 8)])
def test_secondary_rank_partition_sums_to_image(proxy_small, nx, ny, nranks):
    """Each rank writes exactly the pixels of its 8x8 tiles (dist.py
    secondary_mask); the parts sum to the single-rank image.  72x40 / 3
    ranks: ragged edge strips dealt tile by tile; 512x40 / 8 ranks: whole
    4x4-tile blocks with rank 0 dealt the lighter share (include/vrt.h)."""
    import torch
    from voxelraytrace20190722_amd import dist as vd
    tree = vrt.VoxelOctree(proxy_small, 6)
    mn, mx = tree.root_box
    fov, eye, spot, up = vrt.sweep_pose(mn, mx, 4, 16)
    cam = vrt.Camera(fov, eye, spot, up)
    film = vrt.Film(1, 1, nx, ny)
    ref, _ = tree.render_secondary(cam, film, spp=64)
    dev = torch.device("cuda:0")
    prim = torch.zeros(nx * ny * 8, dtype=torch.float32, device=dev)
    acc = torch.zeros((ny, nx), dtype=torch.float32, device=dev)
    for r in range(nranks):
        part = torch.zeros((ny, nx), dtype=torch.float32, device=dev)
        tree.render_secondary_device(cam, film, 64, r, nranks, prim.data_ptr(), part.data_ptr(), None)
        torch.cuda.synchronize()
        m = vd.secondary_mask(nx, ny, r, nranks)
        pa = part.cpu().numpy()
        assert np.all(pa[~m] == 0) and np.all(pa[m] > 0) == np.all(ref[m] > 0)
        acc += part
    assert np.array_equal(bits(acc.cpu().numpy()), bits(ref))


def test_obj_ingest_render_matches_oracle(tmp_path):
    """OBJ/MTL/TGA -> vrt_obj_load (tinyobj-exact) -> octree -> GPU render,
    bit-exact against the oracle on the same ingested soup; the corpus soup
    itself is pinned to the reference's LoadObj by tests/test_ingest.py."""
    import ingest_corpus as ic
    cases = ic.write_obj_corpus(str(tmp_path / "corpus"))
    scenes = [vrt.obj2voxel(str(tmp_path / "corpus" / cases["polys"][0]))]
    proxy = vrt.SceneData.proxy(0.05, 3)
    scenes.append(vrt.obj2voxel(ic.write_scene_obj(str(tmp_path / "proxy"), proxy)))
    assert scenes[1].ntri == proxy.ntri and len(scenes[1].tex_off) == len(proxy.tex_off)
    for sd in scenes:
        tree = vrt.VoxelOctree(sd, 7)
        osc = po.Scene(sd, 7)
        mn, mx = tree.root_box
        for pose in (2, 9):
            fov, eye, spot, up = vrt.sweep_pose(mn, mx, pose, 16)
            rgb, so = tree.render(vrt.Camera(fov, eye, spot, up), vrt.Film(1, 1, 48, 40), samples=True)
            orgb, oso = osc.render(po.camera(fov, eye, spot, up), 1.0, 1.0, 48, 40, film_index=1, nthreads=8)
            for key in ("hit", "tri", "voxel"):
                assert np.array_equal(so[key], oso[key]), key
            assert np.array_equal(bits(rgb), bits(orgb))
            assert so["hit"].mean() > 0.2


def test_device_rgbe_pack_matches_reference_writer(tmp_path):
    """k_rgbe (device stbiw__linear_to_rgbe) + host RLE == stbi_write_hdr:
    reference fixture images, plus an edge image (NaN, +-inf, huge,
    negative, below the 1e-32 cut, denormals, exact powers of two)."""
    import torch
    z = golden("hdr_ref.npz")
    imgs = [z[f"img{i}"] for i in range(6)]
    edge = np.random.default_rng(4).random((7, 33, 3)).astype(np.float32)
    specials = [np.nan, np.inf, -np.inf, 3e38, -1.0, 1e-33, 1e-40, 0.5, 1.0, 2.0, 255.99, 1e-32, 1.0000001e-32]
    for k, v in enumerate(specials):
        edge[k % 7, (3 * k) % 33, k % 3] = v
    edge[6, :, :] = np.float32(2.0) ** np.arange(-40, 59, 3)[:33, None].astype(np.float32)
    imgs.append(edge)
    for i, img in enumerate(imgs):
        img = np.ascontiguousarray(img, np.float32)
        h, w = img.shape[:2]
        comp = 1 if img.ndim == 2 else img.shape[2]
        d = torch.from_numpy(img.reshape(-1).copy()).cuda()
        out = torch.zeros(h * w * 4, dtype=torch.uint8, device="cuda")
        vrt.rgbe_device(d.data_ptr(), w, h, comp, out.data_ptr())
        torch.cuda.synchronize()
        got = out.cpu().numpy().reshape(h, w, 4)
        assert np.array_equal(got, po.linear_to_rgbe_img(img)), i
        p = tmp_path / f"d{i}.hdr"
        assert vrt.write_hdr_device(p, d.data_ptr(), w, h, comp)
        want = z[f"bytes{i}"].tobytes() if i < 6 else vrt.hdr_bytes(img)
        assert p.read_bytes() == want, i


# ---- full trace() ----
LIGHT = (vrt.to_radian(60), (1.0, 10.0, 1.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0))  # VRT/main.cc:80-83


@pytest.mark.parametrize("depth,light_n", [(5, 96), (6, 128), (8, 256)])
def test_lightmap_and_trace_match_oracle(proxy_small, depth, light_n):
    """Light pass + filter: every node's coverage and illum[6] bit-exact vs
    the oracle's canonical-order sums; then the cone-tracing render."""
    tree = vrt.VoxelOctree(proxy_small, depth)
    osc = po.Scene(proxy_small, depth)
    hits = tree.lightmap(vrt.Camera(*LIGHT), vrt.Film(1, 1, light_n, light_n))
    ohits = osc.lightmap(po.camera(*LIGHT), 1.0, 1.0, light_n, light_n, nthreads=8)
    assert hits == ohits > 0
    k, cov, ill = tree.lightmap_nodes()
    ok, ocov, oill = osc.lightmap_nodes()
    assert np.array_equal(k, ok)
    assert np.array_equal(bits(cov), bits(ocov))
    assert np.array_equal(bits(ill), bits(oill))
    res = tree.min_voxel(6)
    assert res == osc.min_voxel(6)
    mn, mx = tree.root_box
    cams = [(vrt.to_radian(90), (1.0, 1.3, -0.2), (0.0, 0.4, 0.0), (0.0, 1.0, 0.0))]
    cams += [vrt.sweep_pose(mn, mx, i, 16) for i in (3, 10)]
    for fov, eye, spot, up in cams:
        rgb, so = tree.render_trace(vrt.Camera(fov, eye, spot, up), vrt.Film(1, 1, 40, 32), res, samples=True)
        orgb, oso = osc.render_trace(po.camera(fov, eye, spot, up), 1.0, 1.0, 40, 32, res, nthreads=8)
        assert np.array_equal(so["hit"], oso["hit"])
        assert np.array_equal(bits(so["rgb"]), bits(oso["rgb"]))
        assert np.array_equal(bits(rgb), bits(orgb))


def test_trace_step_table_follows_min_voxel_and_film(proxy_small):
    """The cone step table (k_cone_steps) is kept per trace set and rebuilt
    only when (mindist, maxdist) change: renders alternating the cone step
    (min_voxel) and the film size (the records move, the table stays at its
    fixed offset) each match the oracle bit for bit."""
    tree = vrt.VoxelOctree(proxy_small, 6)
    osc = po.Scene(proxy_small, 6)
    tree.lightmap(vrt.Camera(*LIGHT), vrt.Film(1, 1, 96, 96))
    osc.lightmap(po.camera(*LIGHT), 1.0, 1.0, 96, 96, nthreads=8)
    res = tree.min_voxel(6)
    view = (vrt.to_radian(90), (1.0, 1.3, -0.2), (0.0, 0.4, 0.0), (0.0, 1.0, 0.0))
    for mv, (nx, ny) in [(res, (40, 32)), (2.0 * res, (40, 32)), (res, (48, 40)), (res, (40, 32)),
                         (0.5 * res, (48, 40))]:
        rgb = tree.render_trace(vrt.Camera(*view), vrt.Film(1, 1, nx, ny), mv)
        orgb, _ = osc.render_trace(po.camera(*view), 1.0, 1.0, nx, ny, mv, nthreads=8)
        assert np.array_equal(bits(rgb), bits(orgb)), (mv, nx, ny)


def test_trace_step_table_survives_failed_frame(proxy_small):
    """A frame that fails after its trace set's scratch is set up (here: a
    light film too large for the light pass, rejected before any kernel
    runs) must not mark the set's cone step table as built: the next frames
    on both sets (trace frames alternate the scene's two sets) with the same
    min_voxel match the oracle (the key used to be committed
    before k_cone_steps was enqueued)."""
    import torch
    tree = vrt.VoxelOctree(proxy_small, 6)
    osc = po.Scene(proxy_small, 6)
    res = tree.min_voxel(6)
    view = (vrt.to_radian(90), (1.0, 1.3, -0.2), (0.0, 0.4, 0.0), (0.0, 1.0, 0.0))
    film = vrt.Film(1, 1, 40, 32)
    img = torch.zeros((32, 40, 3), device="cuda")
    with pytest.raises(vrt.VrtError):
        tree.trace_frame_device(vrt.Camera(*LIGHT), vrt.Film(1, 1, 32768, 32768), vrt.Camera(*view), film, 0, 1, 1,
                                img.data_ptr(), res)
    osc.lightmap(po.camera(*LIGHT), 1.0, 1.0, 96, 96, nthreads=8)
    want, _ = osc.render_trace(po.camera(*view), 1.0, 1.0, 40, 32, res, nthreads=8)
    for k in range(3):  # sets 1, 0, 1 after the failed frame took set 0
        img.zero_()
        tree.trace_frame_device(vrt.Camera(*LIGHT), vrt.Film(1, 1, 96, 96), vrt.Camera(*view), film, 0, 1, 1,
                                img.data_ptr(), res)
        torch.cuda.synchronize()
        assert np.array_equal(bits(img.cpu().numpy()), bits(want)), k
    assert np.array_equal(bits(tree.render_trace(vrt.Camera(*view), film, res)), bits(want))


@pytest.mark.parametrize("depth,light_n", [(5, 96), (8, 128)])
def test_lightmap_tail_walk_matches_oracle(proxy_small, depth, light_n):
    """The light pass's tail launch (k_light_tail: one sample per wave, the
    leaf records split over the lanes) for every sample (TEST_LIGHT_TAIL):
    the light map is bit-exact vs the oracle, as with the budgeted walk."""
    tree = vrt.VoxelOctree(proxy_small, depth)
    osc = po.Scene(proxy_small, depth)
    ohits = osc.lightmap(po.camera(*LIGHT), 1.0, 1.0, light_n, light_n, nthreads=8)
    ok, ocov, oill = osc.lightmap_nodes()
    vrt.set_test_flags(vrt.TEST_LIGHT_TAIL)
    try:
        hits = tree.lightmap(vrt.Camera(*LIGHT), vrt.Film(1, 1, light_n, light_n))
    finally:
        vrt.set_test_flags(0)
    assert hits == ohits > 0
    k, cov, ill = tree.lightmap_nodes()
    assert np.array_equal(k, ok)
    assert np.array_equal(bits(cov), bits(ocov))
    assert np.array_equal(bits(ill), bits(oill))


def test_trace_device_tiles_reassemble(proxy_small):
    import torch
    tree = vrt.VoxelOctree(proxy_small, 6)
    tree.lightmap(vrt.Camera(*LIGHT), vrt.Film(1, 1, 64, 64))
    cam = vrt.Camera(vrt.to_radian(90), (1.0, 1.3, -0.2), (0.0, 0.4, 0.0), (0.0, 1.0, 0.0))
    film = vrt.Film(1, 1, 48, 40)
    direct = tree.render_trace(cam, film)
    n = 3
    tpr = vrt.tiles_per_rank(film, n)
    g = torch.zeros(n * tpr * 192, device="cuda")
    for r in range(n):
        tree.render_trace_device(cam, film, r, n, 0, g[r * tpr * 192:].data_ptr())
    img = torch.zeros(48 * 40 * 3, device="cuda")
    vrt.unpack_tiles_device(film, n, g.data_ptr(), img.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(bits(img.cpu().numpy().reshape(40, 48, 3)), bits(direct))


def test_trace_frame_one_call_matches_two_calls_and_oracle(proxy_small):
    """vrt_trace_frame_device (light map + filter beside the view's primary
    march, then the cones) equals vrt_lightmap_build + vrt_render_trace_device
    and the oracle, bit for bit: a whole-image frame, then 3 ranks' tile
    shares re-assembled, then frames queued back to back on one stream with
    alternating views (the next frame's light pass waits for the previous
    frame's cones, which read the light map), on two streams (frames in
    flight over the scene's two light-map / record sets), then the separate
    light-map build and render again."""
    import torch
    tree = vrt.VoxelOctree(proxy_small, 6)
    osc = po.Scene(proxy_small, 6)
    lfilm = vrt.Film(1, 1, 96, 96)
    ohits = osc.lightmap(po.camera(*LIGHT), 1.0, 1.0, 96, 96, nthreads=8)
    res = tree.min_voxel(6)
    mn, mx = tree.root_box
    views = [(vrt.to_radian(90), (1.0, 1.3, -0.2), (0.0, 0.4, 0.0), (0.0, 1.0, 0.0)), vrt.sweep_pose(mn, mx, 5, 16)]
    film = vrt.Film(1, 1, 48, 40)
    want = [osc.render_trace(po.camera(*v), 1.0, 1.0, 48, 40, res, nthreads=8, samples=False) for v in views]
    st = torch.cuda.Stream()
    img = torch.zeros((40, 48, 3), device="cuda")
    hits = tree.trace_frame_device(vrt.Camera(*LIGHT), lfilm, vrt.Camera(*views[0]), film, 0, 1, 1, img.data_ptr(),
                                   res, st.cuda_stream)
    st.synchronize()
    assert hits == ohits > 0
    assert np.array_equal(bits(img.cpu().numpy()), bits(want[0]))
    assert np.array_equal(bits(tree.render_trace(vrt.Camera(*views[0]), film, res)), bits(want[0]))
    n = 3
    tpr = vrt.tiles_per_rank(film, n)
    g = torch.zeros(n * tpr * 192, device="cuda")
    for r in range(n):
        tree.trace_frame_device(vrt.Camera(*LIGHT), lfilm, vrt.Camera(*views[1]), film, r, n, 0,
                                g[r * tpr * 192:].data_ptr(), res, st.cuda_stream)
    full = torch.zeros(48 * 40 * 3, device="cuda")
    st.synchronize()
    vrt.unpack_tiles_device(film, n, g.data_ptr(), full.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(bits(full.cpu().numpy().reshape(40, 48, 3)), bits(want[1]))
    # frames in flight over the scene's two light-map / record sets with
    # three different light passes (camera, film) cycling against the sets'
    # period of two, so every frame's light map differs from the one in the
    # other set: a frame whose cones read the other set's map, or a light
    # pass that overwrites a set still being read, changes its image (ADVICE
    # r4).  Each frame is compared with its own oracle image.
    light2 = (vrt.to_radian(45), (-2.0, 8.0, 3.0), (0.0, 0.5, 0.0), (0.0, 1.0, 0.0))
    lights = [(LIGHT, 96), (light2, 96), (LIGHT, 64)]
    wantl = {}
    for li, (lc, ln) in enumerate(lights):
        osc.lightmap(po.camera(*lc), 1.0, 1.0, ln, ln, nthreads=8)
        for vi, v in enumerate(views):
            wantl[li, vi] = osc.render_trace(po.camera(*v), 1.0, 1.0, 48, 40, res, nthreads=8, samples=False)
    assert not np.array_equal(bits(wantl[0, 0]), bits(wantl[1, 0]))  # the light maps differ
    assert not np.array_equal(bits(wantl[0, 0]), bits(wantl[2, 0]))
    outs = [torch.zeros((40, 48, 3), device="cuda") for _ in range(6)]
    sts = [st, torch.cuda.Stream()]  # the two light-map sets alternate, frames on two streams
    for k, o in enumerate(outs):
        lc, ln = lights[k % 3]
        tree.trace_frame_device(vrt.Camera(*lc), vrt.Film(1, 1, ln, ln), vrt.Camera(*views[k % 2]), film, 0, 1, 1,
                                o.data_ptr(), res, sts[k % 2].cuda_stream)
    # lm_cur hand-off: a render right behind the frames uses the last frame's
    # light map (lights[5 % 3]), on a third stream
    last = torch.zeros((40, 48, 3), device="cuda")
    st3 = torch.cuda.Stream()
    tree.render_trace_device(vrt.Camera(*views[0]), film, 0, 1, 1, last.data_ptr(), res, st3.cuda_stream)
    torch.cuda.synchronize()
    for k, o in enumerate(outs):
        assert np.array_equal(bits(o.cpu().numpy()), bits(wantl[k % 3, k % 2])), k
    assert np.array_equal(bits(last.cpu().numpy()), bits(wantl[5 % 3, 0]))
    assert tree.lightmap(vrt.Camera(*LIGHT), lfilm) == ohits
    assert np.array_equal(bits(tree.render_trace(vrt.Camera(*views[1]), film, res)), bits(want[1]))


# ---- GPU octree build ----
@pytest.mark.parametrize("depth", [1, 2, 5, 8, 9])
def test_device_build_equals_host_build(proxy_small, depth):
    """VRT_BUILD_DEVICE produces the host build's octree array for array:
    node boxes, child/leaf words, content masks, leaf lists, info."""
    scenes = [proxy_small, scene_from(golden("scene_soup.npz"))]
    for sd in scenes:
        h = vrt.VoxelOctree(sd, depth)
        g = vrt.VoxelOctree(sd, depth, build_on_device=True)
        for x, y in zip(h.nodes(), g.nodes()):
            assert np.array_equal(bits(x), bits(y))
        for x, y in zip(h.leaves(), g.leaves()):
            assert np.array_equal(x, y)
        for f in ("nodes", "internal", "leaves", "nonempty_leaves", "tri_refs"):
            assert getattr(h.info, f) == getattr(g.info, f), f
        assert g.info.build_device_ms > 0
    # and it renders identically
    mn, mx = g.root_box
    fov, eye, spot, up = vrt.sweep_pose(mn, mx, 5, 16)
    cam, film = vrt.Camera(fov, eye, spot, up), vrt.Film(1, 1, 40, 40)
    assert np.array_equal(bits(h.render(cam, film)), bits(g.render(cam, film)))


def test_device_build_edge_scenes():
    one = vrt.SceneData(np.float32([[0, 0, 0, 1, 0, 0.5, 0, 1, 1]]), np.float32([[0, 0, 1] * 3]))
    flat = vrt.SceneData(np.float32([[0, 0, 0, 1, 0, 0, 0, 1, 0], [1, 1, 0, 0, 1, 0, 1, 0, 0]]),
                         np.tile(np.float32([0, 0, 1]), (2, 3)))
    empty = vrt.SceneData(np.zeros((0, 9), np.float32), np.zeros((0, 9), np.float32))
    # a zero-thickness scene splits into all 8 children at every level (both
    # z halves of a flat box coincide): 8^(depth-1) leaves, so keep it shallow
    for sd, depths in ((one, (1, 4, 9)), (flat, (1, 3, 5)), (empty, (1, 11))):
        for depth in depths:
            h = vrt.VoxelOctree(sd, depth)
            g = vrt.VoxelOctree(sd, depth, build_on_device=True)
            for x, y in zip(h.nodes(), g.nodes()):
                assert np.array_equal(bits(x), bits(y))
            for x, y in zip(h.leaves(), g.leaves()):
                assert np.array_equal(x, y)


def _small_soup(n=1500, seed=11):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-1, 1, (n, 1, 3))
    pos = (c + rng.normal(0, 0.05, (n, 3, 3))).astype(np.float32).reshape(n, 9)
    nrm = rng.normal(0, 1, (n, 9)).astype(np.float32)
    return vrt.SceneData(pos, nrm)


@pytest.mark.parametrize("depth", [10, 11])
def test_maximum_depth_matches_oracle(depth):
    """max_depth up to VRT_MAX_DEPTH (11: voxel ids pack 10 bits per axis;
    the LDS stack holds max_depth - 2 live entries): a soup of small
    triangles at the finest grids -- camera renders (per-sample ids, counters,
    RGB bits) and batched arbitrary rays against the oracle."""
    sd = _small_soup()
    tree = vrt.VoxelOctree(sd, depth)
    osc = po.Scene(sd, depth)
    mn, mx = tree.root_box
    for pose in (3, 11):
        fov, eye, spot, up = vrt.sweep_pose(mn, mx, pose, 16)
        rgb, so = tree.render(vrt.Camera(fov, eye, spot, up), vrt.Film(1, 1, 48, 48), samples=True,
                              counters=True)
        orgb, oso = osc.render(po.camera(fov, eye, spot, up), 1.0, 1.0, 48, 48, film_index=1, nthreads=8)
        assert so["hit"].sum() > 1000, pose
        for key in ("hit", "tri", "voxel", "counters"):
            assert np.array_equal(so[key], oso[key]), (depth, pose, key)
        assert np.array_equal(bits(rgb), bits(orgb)), (depth, pose)
    rays = _random_rays(np.random.default_rng(depth), 4000, mn, mx)
    g = tree.ray_march(rays)
    o = osc.ray_march(rays)
    assert o["hit"].sum() > 300
    for key in ("hit", "tri", "voxel"):
        assert np.array_equal(g[key], o[key]), key
    assert np.array_equal(bits(g["hit_p"]), bits(o["hit_p"]))


def test_trace_main_frame_256_matches_oracle():
    """The reference main() frame at 256x256 on the full sponza-proxy
    (depth 6, light map 512^2): light map, filter and the cone-traced image
    bit-exact vs the oracle's canonical order -- every cone step of 262,144
    samples x 6 cones through the descent tables (TraceParams::ctab)."""
    sd = vrt.SceneData.proxy(1.0, 1)
    tree = vrt.VoxelOctree(sd, 6)
    osc = po.Scene(sd, 6)
    hits = tree.lightmap(vrt.Camera(*LIGHT), vrt.Film(1, 1, 512, 512))
    assert hits == osc.lightmap(po.camera(*LIGHT), 1.0, 1.0, 512, 512, nthreads=16) > 0
    res = tree.min_voxel(6)
    cam = (vrt.to_radian(90), (1.0, 1.3, -0.2), (0.0, 0.4, 0.0), (0.0, 1.0, 0.0))
    rgb = tree.render_trace(vrt.Camera(*cam), vrt.Film(1, 1, 256, 256), res)
    orgb = osc.render_trace(po.camera(*cam), 1.0, 1.0, 256, 256, res, nthreads=16, samples=False)
    assert np.array_equal(bits(rgb), bits(orgb))
    # every light-pass and primary-pass sample through the 8-lane tail walks
    vrt.set_test_flags(vrt.TEST_LIGHT_TAIL | vrt.TEST_PRIM_TAIL)
    try:
        assert tree.lightmap(vrt.Camera(*LIGHT), vrt.Film(1, 1, 512, 512)) == hits
        rgb2 = tree.render_trace(vrt.Camera(*cam), vrt.Film(1, 1, 256, 256), res)
    finally:
        vrt.set_test_flags(0)
    assert np.array_equal(bits(rgb2), bits(orgb))
