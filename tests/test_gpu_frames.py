"""GPU parity at the BASELINE.json configuration sizes, whole frame, bit for
bit against the oracle (every sample's hit / triangle / voxel id and RGB
bits, and the film), plus the pins that are not frame renders: the kernels'
travorder / min_element code against the real libstdc++ std::sort /
std::min_element, the device octree build against the oracle's, and
concurrent renders of one scene on two streams.

Configs (BASELINE.json "configs"):
  C1 256x256, max_depth 6 ("64^3"), main()'s view camera
  C2 1920x1080, max_depth 8 ("256^3"), two sweep poses
  C3 3840x2160, max_depth 9 ("512^3"), one sweep pose
  C4 = C3 split over 8 ranks (tile partition + rank-major gather + unpack)
  C5 1920x1080, max_depth 8, 64 secondary rays per hit pixel (visibility)
The oracle runs on the box's host cores (16 threads: the GPU box's CPU
share), a few seconds per frame."""
import os

import numpy as np
import pytest

import pyoracle as po
import voxelraytrace20190722_amd as vrt
from conftest import golden

pytestmark = pytest.mark.gpu

NTH = max(1, min(16, os.cpu_count() or 1))
MAIN_CAM = (vrt.to_radian(90), (1.0, 1.3, -0.2), (0.0, 0.4, 0.0), (0.0, 1.0, 0.0))  # VRT/main.cc:108-112


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.fixture(scope="module")
def proxy():
    return vrt.SceneData.proxy(1.0, 1)


_SCENES = {}


def scenes(sd, depth):
    """(device octree, oracle scene) per depth, built once per module."""
    if depth not in _SCENES:
        _SCENES[depth] = (vrt.VoxelOctree(sd, depth), po.Scene(sd, depth))
    return _SCENES[depth]


def _device_image(tree, cam, film, nranks=1):
    """The production path: vrt_render_tiles_device (persistent kernel for
    small-leaf scenes) into a device image; nranks > 1 renders every rank's
    tiles and reassembles them with vrt_unpack_tiles_device."""
    import torch
    dev = torch.device("cuda:0")
    img = torch.zeros((film.ny, film.nx, 3), dtype=torch.float32, device=dev)
    if nranks == 1:
        tree.render_tiles_device(cam, film, 0, 1, 1, img.data_ptr(), None)
    else:
        tpr = vrt.tiles_per_rank(film, nranks)
        g = torch.zeros((nranks, tpr * 192), dtype=torch.float32, device=dev)
        for r in range(nranks):
            tree.render_tiles_device(cam, film, r, nranks, 0, g[r].data_ptr(), None)
        vrt.unpack_tiles_device(film, nranks, g.data_ptr(), img.data_ptr(), None)
    torch.cuda.synchronize()
    return img.cpu().numpy()


def _whole_frame(sd, depth, pose, nx, ny, film_index=1):
    tree, osc = scenes(sd, depth)
    if pose is None:
        fov, eye, spot, up = MAIN_CAM
    else:
        mn, mx = tree.root_box
        fov, eye, spot, up = vrt.sweep_pose(mn, mx, pose, 16)
    cam = vrt.Camera(fov, eye, spot, up)
    film = vrt.Film(1, 1, nx, ny)
    rgb, so = tree.render(cam, film, samples=True)
    orgb, oso = osc.render(po.camera(fov, eye, spot, up), 1.0, 1.0, nx, ny, film_index=film_index,
                           nthreads=NTH)
    for key in ("hit", "tri", "voxel"):
        assert np.array_equal(so[key], oso[key]), key
    assert np.array_equal(bits(so["rgb"]), bits(oso["rgb"]))
    assert np.array_equal(bits(rgb), bits(orgb))
    assert 0.3 < so["hit"].mean() <= 1.0
    # the production launch (the one bench.py times) gives the same film
    assert np.array_equal(bits(_device_image(tree, cam, film)), bits(orgb))
    return tree, cam, film, orgb


def test_c1_256_depth6_whole_frame(proxy):
    """C1: 256x256 at max_depth 6 (main()'s own depth, VRT/main.cc:67-70).
    A square film, so the oracle uses the reference's own Film indexing
    y*ny+x (VRT/camera.cc:19) and the image is the reference's image."""
    _whole_frame(proxy, 6, None, 256, 256, film_index=0)
    _whole_frame(proxy, 6, 4, 256, 256, film_index=0)


@pytest.mark.parametrize("pose", [0, 9])
def test_c2_1080p_depth8_whole_frame(proxy, pose):
    _whole_frame(proxy, 8, pose, 1920, 1080)


def test_c3_c4_4k_depth9_whole_frame_and_8_ranks(proxy):
    """C3 whole frame, then C4: the same frame as 8 ranks' tiles (the tile
    deal of include/vrt.h: 4x4-tile blocks, rank 0 dealt 5/6 of a share),
    gathered rank-major and unpacked, equals it bit for bit."""
    tree, cam, film, orgb = _whole_frame(proxy, 9, 7, 3840, 2160)
    assert np.array_equal(bits(_device_image(tree, cam, film, nranks=8)), bits(orgb))


def test_c5_1080p_depth8_secondary_whole_frame(proxy):
    """C5: per pixel one primary hit, then 64 secondary rays (the
    VRT/voxel_octree.cc:600-603 pattern); the visibility image and the ray
    count equal the oracle's, through both the host entry point and the
    device entry point bench.py times."""
    import torch
    tree, osc = scenes(proxy, 8)
    mn, mx = tree.root_box
    fov, eye, spot, up = vrt.sweep_pose(mn, mx, 5, 16)
    cam = vrt.Camera(fov, eye, spot, up)
    film = vrt.Film(1, 1, 1920, 1080)
    vis, rays = tree.render_secondary(cam, film, spp=64)
    counts = tree.secondary_spill_counts()
    ovis, orays = osc.render_secondary(po.camera(fov, eye, spot, up), 1.0, 1.0, 1920, 1080, spp=64,
                                       nthreads=NTH, ids=False)
    assert rays == orays > 1920 * 1080 * 32
    assert np.array_equal(bits(vis), bits(ovis))
    # the default build compacts (VRT_SEC_SPILL_T > 0) and streams the saved
    # rays: phase A stopped rays, and the one streaming round left queue 1
    # empty -- a build with the compaction off fails here
    assert vrt.build_flag("VRT_SEC_SPILL_T") > 0
    assert counts[0] > 0, counts
    assert counts[1:] == [0, 0, 0], counts
    prim = torch.zeros(1920 * 1080 * 8, dtype=torch.float32, device="cuda:0")
    dvis = torch.zeros((1080, 1920), dtype=torch.float32, device="cuda:0")
    tree.render_secondary_device(cam, film, 64, 0, 1, prim.data_ptr(), dvis.data_ptr(), None)
    torch.cuda.synchronize()
    assert np.array_equal(bits(dvis.cpu().numpy()), bits(ovis))
    # the compaction scratch is sized from the queue's use, not for every ray
    # (DESIGN §4.3): at most 1 GiB for a 1080p frame, one set for calls that
    # do not overlap
    assert tree.scratch_bytes()[1] <= 1 << 30, tree.scratch_bytes()


def test_two_streams_share_one_scene(proxy):
    """Renders of one scene on two streams, launched back to back without a
    host sync and cycling the work-queue ring several times, each equal the
    oracle's image of its pose (the persistent kernel's queues are per
    launch, vrt_internal.h WorkQueue)."""
    import torch
    tree, osc = scenes(proxy, 8)
    assert tree.info.tri_refs < 8 * tree.info.nonempty_leaves  # small leaves: the persistent kernel
    mn, mx = tree.root_box
    film = vrt.Film(1, 1, 320, 200)
    poses = [vrt.sweep_pose(mn, mx, i, 16) for i in (1, 6)]
    want = [osc.render(po.camera(*p), 1.0, 1.0, 320, 200, nthreads=NTH, samples=False) for p in poses]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    n = 20  # > 2 x the ring's 8 slots
    outs = [torch.zeros((200, 320, 3), dtype=torch.float32, device="cuda:0") for _ in range(n)]
    torch.cuda.synchronize()  # the zero fills ran on torch's stream, the renders use others
    for k in range(n):
        st = streams[k % 2]
        tree.render_tiles_device(vrt.Camera(*poses[k % 2]), film, 0, 1, 1, outs[k].data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    for k in range(n):
        assert np.array_equal(bits(outs[k].cpu().numpy()), bits(want[k % 2])), k
    # and the host entry point (scene stream) interleaved with device launches
    a = tree.render(vrt.Camera(*poses[0]), film)
    assert np.array_equal(bits(a), bits(want[0]))


def test_frames_in_flight_match_oracle(proxy):
    """bench.py's schedule: 3 frames in flight on 3 streams with the
    half-chip grid hint (vrt_scene_set_frames_in_flight), 1080p frames of 3
    poses and 8-rank shares of a 4th -- every frame equals the oracle's
    image of its pose; the hint is then reset."""
    import torch
    tree, osc = scenes(proxy, 8)
    mn, mx = tree.root_box
    film = vrt.Film(1, 1, 1920, 1080)
    poses = [vrt.sweep_pose(mn, mx, i, 16) for i in (2, 7, 12, 15)]
    want = [osc.render(po.camera(*p), 1.0, 1.0, 1920, 1080, nthreads=NTH, samples=False) for p in poses]
    tree.set_frames_in_flight(3)
    try:
        streams = [torch.cuda.Stream() for _ in range(3)]
        outs = [torch.zeros((1080, 1920, 3), dtype=torch.float32, device="cuda:0") for _ in range(9)]
        tpr = vrt.tiles_per_rank(film, 8)
        g = torch.zeros((8, tpr * 192), dtype=torch.float32, device="cuda:0")
        torch.cuda.synchronize()  # the zero fills ran on torch's stream, the renders use others
        for k in range(9):
            tree.render_tiles_device(vrt.Camera(*poses[k % 3]), film, 0, 1, 1, outs[k].data_ptr(),
                                     streams[k % 3].cuda_stream)
        # 8 ranks' shares of pose 4 on the 3 streams, reassembled
        for r in range(8):
            tree.render_tiles_device(vrt.Camera(*poses[3]), film, r, 8, 0, g[r].data_ptr(), streams[r % 3].cuda_stream)
        torch.cuda.synchronize()
        img = torch.zeros((1080, 1920, 3), dtype=torch.float32, device="cuda:0")
        vrt.unpack_tiles_device(film, 8, g.data_ptr(), img.data_ptr(), None)
        torch.cuda.synchronize()
        for k in range(9):
            assert np.array_equal(bits(outs[k].cpu().numpy()), bits(want[k % 3])), k
        assert np.array_equal(bits(img.cpu().numpy()), bits(want[3]))
    finally:
        tree.set_frames_in_flight(1)


@pytest.mark.parametrize("flags", [0, vrt.TEST_SPILL_ALL, vrt.TEST_SEC_DEFER])
def test_c5_frames_in_flight_match_oracle(proxy, flags):
    """bench.py's config-5 schedule: frames of 3 poses issued on 3 streams
    without a host sync (one primary-record / visibility buffer pair per
    stream), the film changing from 640x360 to 1280x720 partway (per-frame
    scratch sized anew) -- every visibility image equals the oracle's.
    flags=TEST_SPILL_ALL: nearly every ray is saved and resumed (the
    compaction is the default build's path: vrt_build_flag), through the
    scene's alternating scratch sets.  flags=TEST_SEC_DEFER: every odd pixel
    goes to the exact walk, which runs on each scratch set's side stream
    beside the streaming resume (forked from and joined back into the
    frame's stream) while the other streams' frames run."""
    import torch
    tree, osc = scenes(proxy, 8)
    mn, mx = tree.root_box
    poses = [vrt.sweep_pose(mn, mx, i, 16) for i in (3, 9, 14)]
    films = [(640, 360)] * 4 + [(1280, 720)] * 4
    want = {}
    for k, (nx, ny) in enumerate(films):
        key = (k % 3, nx, ny)
        if key not in want:
            want[key] = osc.render_secondary(po.camera(*poses[k % 3]), 1.0, 1.0, nx, ny, spp=64, nthreads=NTH,
                                             ids=False)[0]
    streams = [torch.cuda.Stream() for _ in range(3)]
    outs = []
    vrt.set_test_flags(flags)
    try:
        for k, (nx, ny) in enumerate(films):
            prim = torch.zeros(nx * ny * 8, dtype=torch.float32, device="cuda:0")
            vis = torch.zeros((ny, nx), dtype=torch.float32, device="cuda:0")
            outs.append((prim, vis, k, nx, ny))
        torch.cuda.synchronize()  # the zero fills ran on torch's stream
        for prim, vis, k, nx, ny in outs:
            tree.render_secondary_device(vrt.Camera(*poses[k % 3]), vrt.Film(1, 1, nx, ny), 64, 0, 1,
                                         prim.data_ptr(), vis.data_ptr(), streams[k % 3].cuda_stream)
        torch.cuda.synchronize()
    finally:
        vrt.set_test_flags(0)
    for prim, vis, k, nx, ny in outs:
        assert np.array_equal(bits(vis.cpu().numpy()), bits(want[(k % 3, nx, ny)])), (k, nx, ny)


def test_forced_defer_pass_matches_oracle(proxy):
    """The persistent fast-path kernel defers a unit whose rays need the
    exact march (a non-zero denormal direction component); k_render_defer
    renders the deferred units afterwards.  With every unit forced onto that
    path (VRT_TEST_FORCE_DEFER) the images still equal the oracle's: a small
    film (deferred list within its capacity) and a 1080p film (32,400 units:
    more than the list holds, so the fallback re-renders every unit)."""
    tree, osc = scenes(proxy, 8)
    mn, mx = tree.root_box
    try:
        vrt.set_test_flags(vrt.TEST_FORCE_DEFER)
        for (nx, ny, pose) in ((64, 48, 2), (1920, 1080, 11)):
            p = vrt.sweep_pose(mn, mx, pose, 16)
            want = osc.render(po.camera(*p), 1.0, 1.0, nx, ny, nthreads=NTH, samples=False)
            got = _device_image(tree, vrt.Camera(*p), vrt.Film(1, 1, nx, ny))
            assert np.array_equal(bits(got), bits(want)), (nx, ny)
    finally:
        vrt.set_test_flags(0)
    # the count was reset: a normal launch of the same slot ring renders fully
    p = vrt.sweep_pose(mn, mx, 3, 16)
    want = osc.render(po.camera(*p), 1.0, 1.0, 320, 200, nthreads=NTH, samples=False)
    for _ in range(10):  # cycles the 8-slot ring
        got = _device_image(tree, vrt.Camera(*p), vrt.Film(1, 1, 320, 200))
        assert np.array_equal(bits(got), bits(want))


def test_naturally_deferred_rays_match_oracle(proxy):
    """Rays with an exactly zero direction component (the reference's FLT_MIN
    substitution, outside the fast-only kernel's finite-slab contract) are
    deferred and rendered by k_render_defer on a grid sized by the host's
    bound (vrt_camera_defer_bound), without any test flag: a camera built so
    that d_y cancels on a line of sample-1 rays (nx = 5 ny), and the sweep
    pose whose 1080p frame holds one such ray.  A frame with bound 0 runs
    without the deferred pass; all are bit-exact."""
    tree, osc = scenes(proxy, 8)
    mn, mx = tree.root_box
    fov, eye, spot, up = vrt.sweep_pose(mn, mx, 5, 16)
    cam = vrt.Camera(fov, eye, spot, up)
    ocam = po.camera(fov, eye, spot, up)
    for k, v in ((1, 0.5), (5, 0.5), (9, 0.0)):  # s.y = u.y = 0.5, nf.y = 0
        cam.c.C[k] = v
        ocam[k] = v
    for nx, ny in ((400, 80), (1280, 256)):
        f = vrt.Film(1, 1, nx, ny)
        assert cam.defer_bound(f) > 0
        want = osc.render(ocam, 1.0, 1.0, nx, ny, nthreads=NTH, samples=False)
        got = _device_image(tree, cam, f)
        assert np.array_equal(bits(got), bits(want)), (nx, ny)
    bounds = [vrt.Camera(*vrt.sweep_pose(mn, mx, k, 16)).defer_bound(vrt.Film(1, 1, 1920, 1080)) for k in range(16)]
    for pose in (int(np.argmax(bounds)), int(np.argmin(bounds))):
        p = vrt.sweep_pose(mn, mx, pose, 16)
        want = osc.render(po.camera(*p), 1.0, 1.0, 1920, 1080, nthreads=NTH, samples=False)
        got = _device_image(tree, vrt.Camera(*p), vrt.Film(1, 1, 1920, 1080))
        assert np.array_equal(bits(got), bits(want)), (pose, bounds[pose])


def _frame_ms(tree, cam, film, img, n):
    """Mean device time of n production launches into img (HIP events)."""
    import torch
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for k in range(n):
        ev[k][0].record()
        tree.render_tiles_device(cam, film, 0, 1, 1, img.data_ptr(), torch.cuda.current_stream().cuda_stream)
        ev[k][1].record()
    torch.cuda.synchronize()
    return float(np.mean([a.elapsed_time(b) for a, b in ev]))


def test_fully_deferred_frame_runs_on_the_whole_chip(proxy):
    """A 1080p frame whose every unit is deferred (VRT_TEST_FORCE_DEFER: the
    camera-independent way to make every wave take the exact path) is
    re-rendered by k_render_defer on a grid as large as the persistent
    launch's, so it is bit-exact vs the oracle and takes less than 2x the
    normal frame (one 4-wave workgroup took ~40x)."""
    import torch
    tree, osc = scenes(proxy, 8)
    mn, mx = tree.root_box
    p = vrt.sweep_pose(mn, mx, 13, 16)
    cam, film = vrt.Camera(*p), vrt.Film(1, 1, 1920, 1080)
    want = osc.render(po.camera(*p), 1.0, 1.0, 1920, 1080, nthreads=NTH, samples=False)
    img = torch.zeros((1080, 1920, 3), dtype=torch.float32, device="cuda:0")
    _frame_ms(tree, cam, film, img, 2)
    normal = _frame_ms(tree, cam, film, img, 8)
    assert np.array_equal(bits(img.cpu().numpy()), bits(want))
    try:
        vrt.set_test_flags(vrt.TEST_FORCE_DEFER)
        img.zero_()
        deferred = _frame_ms(tree, cam, film, img, 8)
        assert np.array_equal(bits(img.cpu().numpy()), bits(want))
    finally:
        vrt.set_test_flags(0)
    print(f"normal {normal:.3f} ms, every unit deferred {deferred:.3f} ms")
    assert deferred < 2.0 * normal, (normal, deferred)


@pytest.mark.parametrize("flags", [vrt.TEST_FAIL_LAUNCH, vrt.TEST_FAIL_LAUNCH | vrt.TEST_FORCE_DEFER])
def test_failed_launch_leaves_work_queue_usable(proxy, flags):
    """A launch that fails after its first kernel was enqueued (test hook
    VRT_TEST_FAIL_LAUNCH; with FORCE_DEFER its deferred list is non-empty
    too) reports VRT_E_DEVICE, and its work-queue slot is reset on the
    stream: the next 12 launches (every slot of the ring, the failed one
    included) equal the oracle's image."""
    import torch
    tree, osc = scenes(proxy, 8)
    mn, mx = tree.root_box
    p = vrt.sweep_pose(mn, mx, 8, 16)
    cam, film = vrt.Camera(*p), vrt.Film(1, 1, 320, 200)
    want = osc.render(po.camera(*p), 1.0, 1.0, 320, 200, nthreads=NTH, samples=False)
    img = torch.zeros((200, 320, 3), dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()
    try:
        vrt.set_test_flags(flags)
        for _ in range(3):
            with pytest.raises(vrt.VrtError):
                tree.render_tiles_device(cam, film, 0, 1, 1, img.data_ptr(), None)
    finally:
        vrt.set_test_flags(0)
    torch.cuda.synchronize()
    for _ in range(12):
        assert np.array_equal(bits(_device_image(tree, cam, film)), bits(want))


@pytest.mark.parametrize("near,far", [(0.05, vrt.FLT_MAX), (0.0, 2.5), (-1.0, 1e30)])
def test_general_persistent_kernel_nonstandard_range_matches_oracle(proxy, near, far):
    """A camera with near != +0 or far != FLT_MAX makes rays outside the
    fast kernel's standard range: the production launch is then the general
    persistent kernel (k_render_p<false>, render_kind), whose images must
    equal the oracle's too (Camera's near / far are the rays' tmin / tmax,
    VRT/camera.cc:65-75)."""
    tree, osc = scenes(proxy, 8)
    mn, mx = tree.root_box
    p = vrt.sweep_pose(mn, mx, 6, 16)
    cam = vrt.Camera(*p, near, far)
    want = osc.render(po.camera(*p, near, far), 1.0, 1.0, 400, 240, nthreads=NTH, samples=False)
    got = _device_image(tree, cam, vrt.Film(1, 1, 400, 240))
    assert np.array_equal(bits(got), bits(want))
    rgb, so = tree.render(cam, vrt.Film(1, 1, 400, 240), samples=True)  # the grid kernel (per-sample outputs)
    assert np.array_equal(bits(rgb), bits(want))


def _pack(seq):
    w = 0
    for k, c in enumerate(seq):
        w |= int(c) << (3 * k)
    return w


def test_device_travorder_and_min_element_match_libstdcxx():
    """The kernels' own child-order code (insertion-sort emulation of the
    exact path; rank, two-slot and 4-slot-network orders of the NaN-free fast
    paths) and the leaf loop's first-minimum rule, against the real
    libstdc++ std::sort / std::min_element (tests/golden/travorder_std.npz)."""
    z = golden("travorder_std.npz")
    dist, mask, order = z["dist"], z["mask"], z["order"]
    out, am = vrt.device_selftest_order(dist, mask, z["depth"], z["length"])
    assert np.array_equal(am, z["argmin"])
    nan = np.isnan(dist).any(1)
    checked = {"exact": 0, "rank": 0, "two": 0, "net4": 0}
    for i in range(len(dist)):
        full = order[i]
        hit = [c for c in full if (mask[i] >> c) & 1]
        assert out[i, 0] == _pack(full), i
        assert out[i, 1] == _pack(hit) | (len(hit) << 24), i
        checked["exact"] += 1
        if nan[i]:
            continue  # the fast paths run only on NaN-free distances (fast_ok)
        assert out[i, 2] == _pack(hit) | (len(hit) << 24), i
        fp = 0
        for p, c in enumerate(full):
            fp |= p << (3 * int(c))
        assert out[i, 5] == fp, i
        checked["rank"] += 1
        if len(hit) <= 2:
            assert out[i, 3] == _pack(hit), i
            checked["two"] += 1
        if len(hit) <= 4:
            assert out[i, 4] == _pack(hit), i
            checked["net4"] += 1
    assert min(checked.values()) > 500, checked


@pytest.mark.parametrize("depth", [1, 2, 3, 5, 7, 8, 9])
def test_device_build_matches_oracle(depth):
    """§8 f3: the GPU octree build (VRT_BUILD_DEVICE) against the oracle's
    recursive insert()/split() restatement directly: node counts, root box,
    every non-empty leaf's voxel id and triangle list (input order)."""
    sd = vrt.SceneData.proxy(0.25, 2)
    z = golden("scene_soup.npz")
    soup = vrt.SceneData(z["pos"], z["nrm"], z["uv"], z["mat"], z["mat_tex"], z["mat_kd"], z["tex_dims"],
                         z["tex_off"], z["tex_data"])
    for s in (sd, soup):
        g = vrt.VoxelOctree(s, depth, build_on_device=True)
        o = po.Scene(s, depth)
        info, box = o.info()
        assert [g.info.nodes, g.info.internal, g.info.leaves, g.info.nonempty_leaves, g.info.tri_refs] == \
            list(info)
        assert np.array_equal(np.concatenate(g.root_box).view(np.uint32), box.view(np.uint32))
        for x, y in zip(g.leaves(), o.leaves()):
            assert np.array_equal(x, y)
        assert g.info.build_device_ms > 0


def test_host_output_path_matches_oracle(proxy):
    """vrt_render into a host array (the render_mt replacement a C++ caller
    gets): tile-row bands on two streams, pinned staging, threaded copy-out.
    Films of several shapes in a row (the kept device image is re-zeroed on a
    shape change: pixels outside the tile grid stay 0), each equal to the
    oracle's image; a film without a whole tile is all zero."""
    tree, osc = scenes(proxy, 8)
    mn, mx = tree.root_box
    for k, (nx, ny) in enumerate([(1920, 1080), (204, 122), (64, 8), (1920, 1080), (7, 7), (333, 250)]):
        p = vrt.sweep_pose(mn, mx, 3 + k, 16)
        got = tree.render(vrt.Camera(*p), vrt.Film(1, 1, nx, ny))
        want = osc.render(po.camera(*p), 1.0, 1.0, nx, ny, nthreads=NTH, samples=False)
        assert np.array_equal(bits(got), bits(want)), (nx, ny)
    # batched ray_march through the kept buffers: two sizes, then the first again
    cam = vrt.Camera(*vrt.sweep_pose(mn, mx, 2, 16))
    f = vrt.Film(1, 1, 64, 48)
    rays = np.concatenate([cam.gen_rays4(f, px, py) for py in range(48) for px in range(0, 64, 4)])
    for n in (len(rays), 17, len(rays)):
        got = tree.ray_march(rays[:n])
        want = osc.ray_march(rays[:n])
        for key in ("hit", "tri", "voxel"):
            assert np.array_equal(got[key], want[key]), (n, key)


@pytest.mark.parametrize("nx,ny,depth", [(1920, 1080, 8), (3840, 2160, 9), (204, 122, 8)])
def test_multi_device_frame_one_device_matches_oracle(proxy, nx, ny, depth):
    """vrt_scene_create_multi / vrt_render_multi with device_mask = 1: a
    1-device RCCL communicator (ncclCommInitAll) and the same path as N
    devices -- share render, ncclGather to rank 0 (in place), unpack -- equal
    to the oracle's image, through the host and the device entry points."""
    import torch
    m = vrt.MultiOctree(proxy, depth, device_mask=1)
    try:
        assert m.devices == [0]
        osc = scenes(proxy, depth)[1]
        mn, mx = m.root_box
        for pose in (4, 10):
            p = vrt.sweep_pose(mn, mx, pose, 16)
            want = osc.render(po.camera(*p), 1.0, 1.0, nx, ny, nthreads=NTH, samples=False)
            got = m.render(vrt.Camera(*p), vrt.Film(1, 1, nx, ny))
            assert np.array_equal(bits(got), bits(want)), pose
            img = torch.full((ny, nx, 3), 7.0, dtype=torch.float32, device="cuda:0")
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            m.render_device(vrt.Camera(*p), vrt.Film(1, 1, nx, ny), img.data_ptr(), s.cuda_stream)
            s.synchronize()
            assert np.array_equal(bits(img.cpu().numpy()), bits(want)), pose
    finally:
        m.close()


_MULTI_WANT = {}


def _multi_want(proxy, depth, nx, ny, pose):
    key = (depth, nx, ny, pose)
    if key not in _MULTI_WANT:
        tree, osc = scenes(proxy, depth)
        mn, mx = tree.root_box
        p = vrt.sweep_pose(mn, mx, pose, 16)
        _MULTI_WANT[key] = osc.render(po.camera(*p), 1.0, 1.0, nx, ny, nthreads=NTH, samples=False)
    return _MULTI_WANT[key]


@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_multi_device_frame_virtual_ranks_match_oracle(proxy, nranks):
    """The n > 1 branch of vrt_render_multi / vrt_render_multi_device
    (per-rank send buffers, rank-major receive buffer, n-rank unpack) run on
    one GPU with VRT_TEST_VIRTUAL_RANKS: n replicas on device 0, the gather
    done by device copies ordered like the collective.  Film sizes change
    204x122 -> 1920x1080 (buffers regrow) -> 204x122, through the host entry
    point, then three frames queued on one stream without a host sync (each
    rank's send buffer reused while rank 0 unpacks the previous frame)."""
    import torch
    depth = 8
    m = vrt.MultiOctree(proxy, depth, device_mask=1, virtual_ranks=nranks)
    try:
        assert m.devices == [0] * nranks
        mn, mx = m.root_box
        seq = [(204, 122, 4), (1920, 1080, 10), (204, 122, 7)]
        for nx, ny, pose in seq:
            got = m.render(vrt.Camera(*vrt.sweep_pose(mn, mx, pose, 16)), vrt.Film(1, 1, nx, ny))
            assert np.array_equal(bits(got), bits(_multi_want(proxy, depth, nx, ny, pose))), (nx, ny, pose)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        imgs = []
        for nx, ny, pose in [(1920, 1080, 10), (204, 122, 4), (1920, 1080, 3)]:
            img = torch.full((ny, nx, 3), 7.0, dtype=torch.float32, device="cuda:0")
            m.render_device(vrt.Camera(*vrt.sweep_pose(mn, mx, pose, 16)), vrt.Film(1, 1, nx, ny),
                            img.data_ptr(), s.cuda_stream)
            imgs.append((img, nx, ny, pose))
        s.synchronize()
        for img, nx, ny, pose in imgs:
            assert np.array_equal(bits(img.cpu().numpy()), bits(_multi_want(proxy, depth, nx, ny, pose))), \
                (nx, ny, pose)
    finally:
        m.close()


def test_multi_device_frame_two_devices_matches_oracle(proxy):
    """A real 2-device frame (device_mask 0b11: a 2-rank RCCL communicator,
    ncclGather across devices).  Skipped on a one-GPU box."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("fewer than 2 devices visible")
    depth = 8
    m = vrt.MultiOctree(proxy, depth, device_mask=0b11)
    try:
        assert m.devices == [0, 1]
        mn, mx = m.root_box
        for nx, ny, pose in [(1920, 1080, 10), (204, 122, 4)]:
            cam, film = vrt.Camera(*vrt.sweep_pose(mn, mx, pose, 16)), vrt.Film(1, 1, nx, ny)
            want = _multi_want(proxy, depth, nx, ny, pose)
            assert np.array_equal(bits(m.render(cam, film)), bits(want)), (nx, ny, pose)
            img = torch.full((ny, nx, 3), 7.0, dtype=torch.float32, device="cuda:0")
            s = torch.cuda.Stream(device="cuda:0")
            m.render_device(cam, film, img.data_ptr(), s.cuda_stream)
            s.synchronize()
            assert np.array_equal(bits(img.cpu().numpy()), bits(want)), (nx, ny, pose)
    finally:
        m.close()
