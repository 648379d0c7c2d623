"""Python mirror of the reference's hot-path interface over libvrt.so.

Names follow the reference (VRT/x = VoxelRayTrace20190722/x):
  Camera(fov, eye, spot, up, near, far), Camera.gen_rays4/gen_rays1  VRT/camera.h:70-84
  Film(w, h, nx, ny)                                                 VRT/camera.h:24-39
  ray_march_init(scene, max_depth) -> VoxelOctree                    VRT/voxel_octree.h:85-86
  ray_march(tree, rays)                                              VRT/voxel_octree.h:87-89
  render(tree, cam, film)     the per-pixel loop of VRT/main.cc:118-123 (primary shading)
  intersect_triangle3 / tri_box_overlap                              VRT/raytri.h:5, tribox2.h:6
  write_hdr                                                          VRT/stb_image_write.h:178
Errors raise VrtError (the reference exit()s or returns false).
"""
import ctypes as C
import numpy as np

from . import _ffi
from ._ffi import VrtError, check, lib, ptr

FLT_MAX = float(np.finfo(np.float32).max)


def to_radian(degree):
    """jql::to_radian: degree * pi / 180.f in float (VRT/graphics_math.h:896-899)."""
    d = np.float32(degree)
    return float(np.float32(np.float32(d * np.float32(3.1415926535897932384626)) / np.float32(180.0)))


def _f3(v):
    a = np.ascontiguousarray(np.asarray(v, dtype=np.float32).reshape(3))
    return a


class Film:
    """Film(w, h, nx, ny) (VRT/camera.h:24-39)."""

    def __init__(self, w, h, nx, ny):
        self.w, self.h, self.nx, self.ny = float(w), float(h), int(nx), int(ny)
        self.c = _ffi.Film(self.w, self.h, self.nx, self.ny)


class Camera:
    """Camera(fov, eye, spot, up, near=0, far=FLT_MAX) (VRT/camera.cc:65-75)."""

    def __init__(self, fov, eye, spot, up, near=0.0, far=FLT_MAX):
        self.c = _ffi.Camera()
        self.eye, self.spot, self.up = _f3(eye), _f3(spot), _f3(up)
        check(lib().vrt_camera_init(float(fov), ptr(self.eye, _ffi.f32p), ptr(self.spot, _ffi.f32p),
                                    ptr(self.up, _ffi.f32p), float(near), float(far),
                                    C.byref(self.c)), "vrt_camera_init")

    @staticmethod
    def _rays(arr):
        out = np.zeros((len(arr), 8), dtype=np.float32)
        for i, r in enumerate(arr):
            out[i, 0:3] = r.o[:]
            out[i, 3:6] = r.d[:]
            out[i, 6] = r.tmin
            out[i, 7] = r.tmax
        return out

    def gen_rays4(self, film, px, py):
        """4 rays {o, d, tmin, tmax} as a (4, 8) float32 array (VRT/camera.cc:95-112)."""
        arr = (_ffi.Ray * 4)()
        check(lib().vrt_gen_rays4(C.byref(self.c), C.byref(film.c), int(px), int(py), arr),
              "vrt_gen_rays4")
        return self._rays(arr)

    def defer_bound(self, film):
        """vrt_camera_defer_bound: an upper bound on the rays of the film the
        fast-only render defers (0: no deferred pass is launched)."""
        n = C.c_int64()
        check(lib().vrt_camera_defer_bound(C.byref(self.c), C.byref(film.c), C.byref(n)), "vrt_camera_defer_bound")
        return n.value

    def gen_rays1(self, film, px, py):
        arr = (_ffi.Ray * 1)()
        check(lib().vrt_gen_rays1(C.byref(self.c), C.byref(film.c), int(px), int(py), arr),
              "vrt_gen_rays1")
        return self._rays(arr)


def make_ray(o, d, tmin=0.0, tmax=FLT_MAX):
    """jql::Ray(o, d, tmin, tmax): normalises d (VRT/graphics_math.h:1159-1166)."""
    r = _ffi.Ray()
    o, d = _f3(o), _f3(d)
    check(lib().vrt_make_ray(ptr(o, _ffi.f32p), ptr(d, _ffi.f32p), float(tmin), float(tmax),
                             C.byref(r)), "vrt_make_ray")
    return np.array(list(r.o) + list(r.d) + [r.tmin, r.tmax], dtype=np.float32)


class SceneData:
    """Triangle soup + materials + textures (the obj2voxel output the
    reference builds its octree from, VRT/voxel_octree.cc:305-371)."""

    def __init__(self, pos, nrm, uv=None, mat=None, mat_tex=None, mat_kd=None,
                 tex_dims=None, tex_off=None, tex_data=None):
        self.pos = np.ascontiguousarray(np.asarray(pos, np.float32).reshape(-1, 9))
        n = self.pos.shape[0]
        self.nrm = np.ascontiguousarray(np.asarray(nrm, np.float32).reshape(n, 9))
        self.uv = None if uv is None else np.ascontiguousarray(np.asarray(uv, np.float32).reshape(n, 6))
        self.mat = None if mat is None else np.ascontiguousarray(np.asarray(mat, np.int32).reshape(n))
        self.mat_tex = np.ascontiguousarray(np.asarray([-1] if mat_tex is None else mat_tex, np.int32))
        self.mat_kd = np.ascontiguousarray(
            np.asarray([[0.8, 0.8, 0.8]] if mat_kd is None else mat_kd, np.float32).reshape(-1, 3))
        self.tex_dims = np.ascontiguousarray(np.asarray([] if tex_dims is None else tex_dims,
                                                        np.int32).reshape(-1, 3))
        self.tex_off = np.ascontiguousarray(np.asarray([] if tex_off is None else tex_off, np.int64))
        self.tex_data = np.ascontiguousarray(np.asarray([] if tex_data is None else tex_data, np.uint8))

    @property
    def ntri(self):
        return self.pos.shape[0]

    def desc(self):
        d = _ffi.SceneDesc()
        d.ntri = self.ntri
        d.pos = ptr(self.pos, _ffi.f32p)
        d.nrm = ptr(self.nrm, _ffi.f32p)
        d.uv = ptr(self.uv, _ffi.f32p)
        d.mat = ptr(self.mat, _ffi.i32p)
        d.nmat = len(self.mat_tex)
        d.mat_tex = ptr(self.mat_tex, _ffi.i32p)
        d.mat_kd = ptr(self.mat_kd, _ffi.f32p)
        d.ntex = len(self.tex_off)
        d.tex_dims = ptr(self.tex_dims, _ffi.i32p) if len(self.tex_off) else None
        d.tex_off = ptr(self.tex_off, _ffi.i64p) if len(self.tex_off) else None
        d.tex_data = ptr(self.tex_data, _ffi.u8p) if len(self.tex_off) else None
        d.tex_bytes = int(self.tex_data.size)
        return d

    @classmethod
    def proxy(cls, detail=1.0, seed=1):
        """The deterministic sponza-proxy atrium (vrt_proxy_scene)."""
        L = lib()
        nt, nm, nx, tb = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int64()
        check(L.vrt_proxy_scene(float(detail), int(seed), C.byref(nt), None, None, None, None,
                                C.byref(nm), None, None, C.byref(nx), None, None, None,
                                C.byref(tb)), "vrt_proxy_scene(count)")
        n = nt.value
        pos = np.zeros((n, 9), np.float32)
        nrm = np.zeros((n, 9), np.float32)
        uv = np.zeros((n, 6), np.float32)
        mat = np.zeros(n, np.int32)
        mt = np.zeros(nm.value, np.int32)
        kd = np.zeros((nm.value, 3), np.float32)
        td = np.zeros((nx.value, 3), np.int32)
        to = np.zeros(nx.value, np.int64)
        tx = np.zeros(tb.value, np.uint8)
        check(L.vrt_proxy_scene(float(detail), int(seed), C.byref(nt), ptr(pos, _ffi.f32p),
                                ptr(nrm, _ffi.f32p), ptr(uv, _ffi.f32p), ptr(mat, _ffi.i32p),
                                C.byref(nm), ptr(mt, _ffi.i32p), ptr(kd, _ffi.f32p), C.byref(nx),
                                ptr(td, _ffi.i32p), ptr(to, _ffi.i64p), ptr(tx, _ffi.u8p),
                                C.byref(tb)), "vrt_proxy_scene")
        return cls(pos, nrm, uv, mat, mt, kd, td, to, tx)

    @classmethod
    def from_obj(cls, path):
        """obj2voxel(path) + textures (VRT/voxel_octree.cc:305-388)."""
        with ObjModel(path) as m:
            return m.scene_data()


class ObjModel:
    """tinyobj::LoadObj result (+ the obj2voxel soup unless parse_only)
    through vrt_obj_load.  Usable as a context manager; arrays returned are
    copies, so they outlive the handle."""

    def __init__(self, path, parse_only=False):
        self.h = C.c_void_p()
        flags = _ffi.VRT_OBJ_PARSE_ONLY if parse_only else 0
        check(lib().vrt_obj_load(str(path).encode(), flags, C.byref(self.h)), f"vrt_obj_load({path})")
        self.info = _ffi.ObjInfo()
        check(lib().vrt_obj_info(self.h, C.byref(self.info)), "vrt_obj_info")

    def close(self):
        if self.h:
            lib().vrt_obj_free(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown: module globals already gone
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def attrib(self):
        """(vertices (n,3), normals (n,3), texcoords (n,2)) float32."""
        v, vn, vt = _ffi.f32p(), _ffi.f32p(), _ffi.f32p()
        check(lib().vrt_obj_attrib(self.h, C.byref(v), C.byref(vn), C.byref(vt)), "vrt_obj_attrib")
        i = self.info

        def arr(p, n, k):
            if n == 0:
                return np.zeros((0, k), np.float32)
            return np.ctypeslib.as_array(p, (n * k,)).reshape(n, k).copy()
        return arr(v, i.nvert, 3), arr(vn, i.nnormal, 3), arr(vt, i.ntexcoord, 2)

    def faces(self):
        """Per triangle: idx (n,3,3) {v,vn,vt} per corner, material id, shape."""
        n = self.info.nface
        idx = np.zeros((n, 3, 3), np.int32)
        mat = np.zeros(n, np.int32)
        shp = np.zeros(n, np.int32)
        check(lib().vrt_obj_faces(self.h, ptr(idx, _ffi.i32p), ptr(mat, _ffi.i32p), ptr(shp, _ffi.i32p)),
              "vrt_obj_faces")
        return idx, mat, shp

    def materials(self):
        out = []
        for i in range(self.info.nmat):
            name, tex = C.c_char_p(), C.c_char_p()
            kd = np.zeros(3, np.float32)
            check(lib().vrt_obj_material(self.h, i, C.byref(name), ptr(kd, _ffi.f32p), C.byref(tex)),
                  "vrt_obj_material")
            out.append({"name": name.value.decode(errors="surrogateescape"), "kd": kd,
                        "texname": tex.value.decode(errors="surrogateescape")})
        return out

    def texture_paths(self):
        out = []
        for i in range(self.info.ntex):
            p = C.c_char_p()
            check(lib().vrt_obj_texture_path(self.h, i, C.byref(p)), "vrt_obj_texture_path")
            out.append(p.value.decode(errors="surrogateescape"))
        return out

    def warnings(self):
        return lib().vrt_obj_warnings(self.h).decode(errors="replace")

    def scene_data(self):
        d = _ffi.SceneDesc()
        check(lib().vrt_obj_scene_desc(self.h, C.byref(d)), "vrt_obj_scene_desc")
        n, nm, nt = d.ntri, d.nmat, d.ntex

        def cp(p, count, dt):
            if count == 0:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(p, (count,)).copy()
        return SceneData(cp(d.pos, n * 9, np.float32), cp(d.nrm, n * 9, np.float32), cp(d.uv, n * 6, np.float32),
                         cp(d.mat, n, np.int32), cp(d.mat_tex, nm, np.int32), cp(d.mat_kd, nm * 3, np.float32),
                         cp(d.tex_dims, nt * 3, np.int32), cp(d.tex_off, nt, np.int64),
                         cp(d.tex_data, d.tex_bytes, np.uint8))


def obj2voxel(path):
    """The reference's obj2voxel (VRT/voxel_octree.cc:305-371) as SceneData."""
    return SceneData.from_obj(path)


def _image_out(rc, where, w, h, c, p):
    check(rc, where)
    try:
        n = w.value * h.value * c.value
        a = np.ctypeslib.as_array(p, (n,)).copy()
    finally:
        lib().vrt_image_free(p)
    return a.reshape(h.value, w.value, c.value)


def load_image(path):
    """stbi_load(path, .., 0) for TGA (VRT/voxel_octree.cc:373-388):
    uint8 (h, w, channels), row 0 = top."""
    w, h, c, p = C.c_int32(), C.c_int32(), C.c_int32(), _ffi.u8p()
    rc = lib().vrt_tga_load(str(path).encode(), C.byref(w), C.byref(h), C.byref(c), C.byref(p))
    return _image_out(rc, f"vrt_tga_load({path})", w, h, c, p)


def tga_decode(data):
    """stbi_load_from_memory for TGA bytes."""
    buf = np.frombuffer(bytes(data), np.uint8)
    w, h, c, p = C.c_int32(), C.c_int32(), C.c_int32(), _ffi.u8p()
    rc = lib().vrt_tga_decode(ptr(buf, _ffi.u8p) if buf.size else (C.c_uint8 * 1)(), buf.size, C.byref(w),
                              C.byref(h), C.byref(c), C.byref(p))
    return _image_out(rc, "vrt_tga_decode", w, h, c, p)


class VoxelOctree:
    """The octree built by gi::ray_march_init and resident on one device
    (device < 0: host-only, for inspecting the build)."""

    def __init__(self, scene, max_depth, device=0, build_on_device=False):
        self.scene = scene  # keeps the arrays alive for the descriptor
        h = C.c_void_p()
        d = scene.desc()
        flags = _ffi.VRT_BUILD_DEVICE if build_on_device else 0
        check(lib().vrt_scene_create_ex(C.byref(d), int(max_depth), int(device), flags, C.byref(h)),
              "vrt_scene_create")
        self.h = h
        self.max_depth = int(max_depth)
        self.info = _ffi.SceneInfo()
        check(lib().vrt_scene_info(self.h, C.byref(self.info)), "vrt_scene_info")

    def close(self):
        if self.h:
            lib().vrt_scene_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def root_box(self):
        return (np.array(self.info.root_min[:], np.float32), np.array(self.info.root_max[:], np.float32))

    def nodes(self):
        """The flattened octree as uploaded: (boxes (n,6) f32, word a, word b) per
        node in BFS child-block order."""
        n = self.info.nodes
        box = np.zeros((n, 6), np.float32)
        a = np.zeros(n, np.uint32)
        b = np.zeros(n, np.uint32)
        check(lib().vrt_scene_nodes(self.h, ptr(box, _ffi.f32p), ptr(a, _ffi.u32p), ptr(b, _ffi.u32p)),
              "vrt_scene_nodes")
        return box, a, b

    def leaves(self):
        """(voxel ids, counts, concatenated triangle lists) of the non-empty leaves."""
        nl, nr = self.info.nonempty_leaves, self.info.tri_refs
        vox = np.zeros(nl, np.uint32)
        cnt = np.zeros(nl, np.uint32)
        tris = np.zeros(max(nr, 1), np.int32)
        check(lib().vrt_scene_leaves(self.h, ptr(vox, _ffi.u32p), ptr(cnt, _ffi.u32p),
                                     ptr(tris, _ffi.i32p)), "vrt_scene_leaves")
        return vox, cnt, tris[:nr]

    def ray_march(self, rays):
        """Batched gi::ray_march over (n, 8) rays {o, d, tmin, tmax} (d normalised)."""
        rays = np.ascontiguousarray(np.asarray(rays, np.float32).reshape(-1, 8))
        n = rays.shape[0]
        out = np.zeros((max(n, 1), 9), np.uint32)
        check(lib().vrt_ray_march_batch(self.h, rays.ctypes.data_as(C.POINTER(_ffi.Ray)), n,
                                        out.ctypes.data_as(C.POINTER(_ffi.Hit))),
              "vrt_ray_march_batch")
        out = out[:n]
        return {"hit": out[:, 0].astype(np.int32), "tri": out[:, 1].view(np.int32).copy(),
                "voxel": out[:, 2].copy(), "hit_p": out[:, 3:6].view(np.float32).copy(),
                "normal": out[:, 6:9].view(np.float32).copy()}

    def render(self, cam, film, samples=False, counters=False, out=None):
        """Primary render -> (ny, nx, 3) float32 image (+ per-sample dict).
        out: a C-contiguous (ny, nx, 3) float32 array to render into (a film
        reused across frames, as the reference's Film is)."""
        nx, ny = film.nx, film.ny
        if out is not None:
            assert out.shape == (ny, nx, 3) and out.dtype == np.float32 and out.flags.c_contiguous
            rgb = out
        else:
            rgb = np.zeros((ny, nx, 3), np.float32)
        smp = None
        st = None
        so = None
        if samples or counters:
            ns = nx * ny * 4
            so = {}
            s = _ffi.Samples()
            if samples:
                so["hit"] = np.zeros(ns, np.int32)
                so["tri"] = np.zeros(ns, np.int32)
                so["voxel"] = np.zeros(ns, np.uint32)
                so["rgb"] = np.zeros((ns, 3), np.float32)
                s.hit = ptr(so["hit"], _ffi.i32p)
                s.tri = ptr(so["tri"], _ffi.i32p)
                s.voxel = ptr(so["voxel"], _ffi.u32p)
                s.rgb = ptr(so["rgb"], _ffi.f32p)
            if counters:
                so["counters"] = np.zeros((ns, 4), np.uint32)
                s.counters = ptr(so["counters"], _ffi.u32p)
                st = _ffi.Stats()
            smp = C.byref(s)
        check(lib().vrt_render(self.h, C.byref(cam.c), C.byref(film.c), ptr(rgb, _ffi.f32p), smp,
                               C.byref(st) if st is not None else None), "vrt_render")
        if so is not None and st is not None:
            so["stats"] = {"rays": st.rays, "aabb_tests": st.aabb_tests, "leaves": st.leaves,
                           "tri_tests": st.tri_tests, "hits": st.hits, "kernel_ms": st.kernel_ms}
        return (rgb, so) if so is not None else rgb

    def render_secondary(self, cam, film, spp=64, ids=False):
        """Config 5: per-pixel sky visibility from `spp` stochastic secondary
        rays -> (ny, nx) float32 image, rays traced (+ per-ray id dict).
        ids=True: per-ray hit, triangle and voxel ids (the ordered walk);
        ids="hit": per-ray hit booleans only (the occlusion walk with its
        compaction, as without ids)."""
        nx, ny = film.nx, film.ny
        vis = np.zeros((ny, nx), np.float32)
        rays = C.c_int64()
        d = None
        if ids:
            ns = nx * ny * spp
            d = {"hit": np.zeros(ns, np.int32)}
            if ids != "hit":
                d.update(tri=np.zeros(ns, np.int32), voxel=np.zeros(ns, np.uint32))
        check(lib().vrt_render_secondary(self.h, C.byref(cam.c), C.byref(film.c), int(spp), ptr(vis, _ffi.f32p),
                                         ptr(d["hit"], _ffi.i32p) if d else None,
                                         ptr(d["tri"], _ffi.i32p) if d and "tri" in d else None,
                                         ptr(d["voxel"], _ffi.u32p) if d and "voxel" in d else None,
                                         C.byref(rays)),
              "vrt_render_secondary")
        return (vis, rays.value, d) if ids else (vis, rays.value)

    def render_secondary_device(self, cam, film, spp, rank, nranks, d_prim_ptr, d_vis_ptr, stream_ptr=None):
        check(lib().vrt_render_secondary_device(self.h, C.byref(cam.c), C.byref(film.c), int(spp), int(rank),
                                                int(nranks), C.c_void_p(d_prim_ptr), C.c_void_p(d_vis_ptr),
                                                C.c_void_p(stream_ptr) if stream_ptr else None),
              "vrt_render_secondary_device")

    def render_tiles_device(self, cam, film, rank, nranks, image_layout, d_out_ptr, stream_ptr=None):
        check(lib().vrt_render_tiles_device(self.h, C.byref(cam.c), C.byref(film.c), int(rank),
                                            int(nranks), int(image_layout), C.c_void_p(d_out_ptr),
                                            C.c_void_p(stream_ptr) if stream_ptr else None),
              "vrt_render_tiles_device")

    def set_frames_in_flight(self, n):
        """Launch hint (vrt_scene_set_frames_in_flight): n >= 2 frames kept
        in flight on different streams -> half-chip persistent grids."""
        check(lib().vrt_scene_set_frames_in_flight(self.h, int(n)), "vrt_scene_set_frames_in_flight")

    def secondary_spill_counts(self):
        """Records appended to each config-5 compaction queue (phase A, resume
        rounds 1..3) by the last secondary launch (vrt_secondary_spill_counts)."""
        c = (C.c_int64 * 4)()
        check(lib().vrt_secondary_spill_counts(self.h, c), "vrt_secondary_spill_counts")
        return list(c)

    def secondary_spill_stats(self):
        """The last config-5 launch's compaction (vrt_secondary_spill_stats):
        {records, finished_in_place, chunks_taken, chunks_allocated,
        leftover_chunks, record_bytes, deferred_pixels}."""
        c = (C.c_int64 * 7)()
        check(lib().vrt_secondary_spill_stats(self.h, c), "vrt_secondary_spill_stats")
        return dict(zip(("records", "finished_in_place", "chunks_taken", "chunks_allocated", "leftover_chunks",
                         "record_bytes", "deferred_pixels"), list(c)))

    def scratch_bytes(self):
        """(total, compaction) device bytes of scratch the scene keeps between
        calls (vrt_scene_scratch_bytes)."""
        t, sp = C.c_int64(), C.c_int64()
        check(lib().vrt_scene_scratch_bytes(self.h, C.byref(t), C.byref(sp)), "vrt_scene_scratch_bytes")
        return t.value, sp.value

    def last_kernel_ms(self):
        ms = C.c_float()
        check(lib().vrt_last_kernel_ms(self.h, C.byref(ms)), "vrt_last_kernel_ms")
        return ms.value

    # ---- full trace() ----
    def min_voxel(self, levels=0):
        """The reference's Res: min(root.size() / 2^levels) (VRT/main.cc:69-70)."""
        r = C.c_float()
        check(lib().vrt_scene_min_voxel(self.h, int(levels), C.byref(r)), "vrt_scene_min_voxel")
        return r.value

    def lightmap(self, light_cam, light_film):
        """Light pass + cone_trace_init_filter on the device; returns hit samples."""
        h = C.c_int64()
        check(lib().vrt_lightmap_build(self.h, C.byref(light_cam.c), C.byref(light_film.c), C.byref(h)),
              "vrt_lightmap_build")
        return h.value

    def lightmap_nodes(self):
        """(key depth<<32|vox, coverage, illum (n,6,3)) sorted by key."""
        n = self.info.nodes
        key = np.zeros(n, np.uint64)
        cov = np.zeros(n, np.float32)
        ill = np.zeros((n, 6, 3), np.float32)
        check(lib().vrt_lightmap_nodes(self.h, key.ctypes.data_as(C.POINTER(C.c_uint64)), ptr(cov, _ffi.f32p),
                                       ptr(ill, _ffi.f32p)), "vrt_lightmap_nodes")
        o = np.argsort(key, kind="stable")
        return key[o], cov[o], ill[o]

    def render_trace(self, cam, film, min_voxel=0.0, samples=False):
        """trace() render (cone tracing) -> (ny, nx, 3) [+ per-sample hit / rgb]."""
        rgb = np.zeros((film.ny, film.nx, 3), np.float32)
        ns = film.nx * film.ny * 4
        hit = np.zeros(ns, np.int32) if samples else None
        srgb = np.zeros((ns, 3), np.float32) if samples else None
        check(lib().vrt_render_trace(self.h, C.byref(cam.c), C.byref(film.c), float(min_voxel), ptr(rgb, _ffi.f32p),
                                     ptr(hit, _ffi.i32p), ptr(srgb, _ffi.f32p)), "vrt_render_trace")
        return (rgb, {"hit": hit, "rgb": srgb}) if samples else rgb

    def render_trace_device(self, cam, film, rank, nranks, image_layout, d_out_ptr, min_voxel=0.0,
                            stream_ptr=None):
        check(lib().vrt_render_trace_device(self.h, C.byref(cam.c), C.byref(film.c), float(min_voxel), int(rank),
                                            int(nranks), int(image_layout), C.c_void_p(d_out_ptr),
                                            None if stream_ptr is None else C.c_void_p(stream_ptr)),
              "vrt_render_trace_device")

    def trace_frame_device(self, light_cam, light_film, cam, film, rank, nranks, image_layout, d_out_ptr,
                           min_voxel=0.0, stream_ptr=None):
        """The reference main() frame in one call (vrt_trace_frame_device):
        light map + filter beside the view's primary march, then the cones;
        returns the light pass's hit count."""
        hits = C.c_int64()
        check(lib().vrt_trace_frame_device(self.h, C.byref(light_cam.c), C.byref(light_film.c), C.byref(cam.c),
                                           C.byref(film.c), float(min_voxel), int(rank), int(nranks),
                                           int(image_layout), C.c_void_p(d_out_ptr),
                                           None if stream_ptr is None else C.c_void_p(stream_ptr), C.byref(hits)),
              "vrt_trace_frame_device")
        return hits.value


class MultiOctree:
    """The octree replicated on every device of a mask, with an RCCL
    communicator over them (vrt_scene_create_multi): one frame = every
    device's share of the tile deal + one ncclGather to the first device +
    unpack there -- render_mt (VRT/camera.h:42-68) over a node's GPUs."""

    def __init__(self, scene, max_depth, device_mask=1, build_on_device=False, virtual_ranks=None):
        """virtual_ranks=n (test hook, VRT_TEST_VIRTUAL_RANKS_N): n ranks on
        the one device of device_mask, the RCCL gather replaced by
        device-to-device copies -- the n-rank frame on a one-GPU box."""
        self.scene = scene
        h = C.c_void_p()
        d = scene.desc()
        flags = _ffi.VRT_BUILD_DEVICE if build_on_device else 0
        if virtual_ranks:
            prev = lib().vrt_test_flags()  # restored afterwards: a caller's own test flags stay set
            lib().vrt_set_test_flags((prev & 0xFF & ~TEST_VIRTUAL_RANKS) | TEST_VIRTUAL_RANKS
                                     | (int(virtual_ranks) << 8))
            try:
                rc = lib().vrt_scene_create_multi(C.byref(d), int(max_depth), int(device_mask), flags, C.byref(h))
            finally:
                lib().vrt_set_test_flags(prev)
        else:
            rc = lib().vrt_scene_create_multi(C.byref(d), int(max_depth), int(device_mask), flags, C.byref(h))
        check(rc, "vrt_scene_create_multi")
        self.h = h
        n = C.c_int32()
        check(lib().vrt_multi_devices(self.h, C.byref(n), None), "vrt_multi_devices")
        devs = np.zeros(n.value, np.int32)
        check(lib().vrt_multi_devices(self.h, C.byref(n), ptr(devs, _ffi.i32p)), "vrt_multi_devices")
        self.devices = [int(x) for x in devs]
        s0 = C.c_void_p()
        check(lib().vrt_multi_scene(self.h, 0, C.byref(s0)), "vrt_multi_scene")
        self.info = _ffi.SceneInfo()
        check(lib().vrt_scene_info(s0, C.byref(self.info)), "vrt_scene_info")

    def close(self):
        if self.h:
            lib().vrt_multi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def root_box(self):
        return (np.array(self.info.root_min[:], np.float32), np.array(self.info.root_max[:], np.float32))

    def render(self, cam, film):
        """The whole frame -> (ny, nx, 3) float32 host image."""
        rgb = np.zeros((film.ny, film.nx, 3), np.float32)
        check(lib().vrt_render_multi(self.h, C.byref(cam.c), C.byref(film.c), ptr(rgb, _ffi.f32p)),
              "vrt_render_multi")
        return rgb

    def render_device(self, cam, film, d_image_ptr, stream_ptr=None):
        """The whole frame into a device image on the first device."""
        check(lib().vrt_render_multi_device(self.h, C.byref(cam.c), C.byref(film.c), C.c_void_p(d_image_ptr),
                                            C.c_void_p(stream_ptr) if stream_ptr else None),
              "vrt_render_multi_device")


def multi_tile_map(film, device_mask):
    """The deal of a frame over a device mask as (nty, ntx) arrays: each
    tile's device and its index in that device's buffer (vrt_multi_tile_map)."""
    ntx, nty = film.nx // 8, film.ny // 8
    dv = np.zeros((nty, ntx), np.int32)
    sl = np.zeros((nty, ntx), np.int32)
    check(lib().vrt_multi_tile_map(C.byref(film.c), int(device_mask), ptr(dv, _ffi.i32p), ptr(sl, _ffi.i32p)),
          "vrt_multi_tile_map")
    return dv, sl


def ray_march_init(scene, max_depth, device=0):
    """gi::ray_march_init(root, voxels, max_depth) (VRT/voxel_octree.cc:67-75)."""
    return VoxelOctree(scene, max_depth, device)


def ray_march(tree, rays):
    """gi::ray_march over a batch of rays (VRT/voxel_octree.cc:131-188)."""
    return tree.ray_march(rays)


def render(tree, cam, film, **kw):
    return tree.render(cam, film, **kw)


def tiles_per_rank(film, nranks):
    return lib().vrt_tiles_per_rank(C.byref(film.c), int(nranks))


def tile_deal_map(film, nranks):
    """The library's tile deal as (nty, ntx) arrays: each tile's rank and its
    index in that rank's packed buffer (vrt_tile_deal_map)."""
    ntx, nty = film.nx // 8, film.ny // 8
    rk = np.zeros((nty, ntx), np.int32)
    sl = np.zeros((nty, ntx), np.int32)
    check(lib().vrt_tile_deal_map(C.byref(film.c), int(nranks), ptr(rk, _ffi.i32p), ptr(sl, _ffi.i32p)),
          "vrt_tile_deal_map")
    return rk, sl


def unpack_tiles_device(film, nranks, d_gathered_ptr, d_image_ptr, stream_ptr=None):
    check(lib().vrt_unpack_tiles_device(C.byref(film.c), int(nranks), C.c_void_p(d_gathered_ptr),
                                        C.c_void_p(d_image_ptr),
                                        C.c_void_p(stream_ptr) if stream_ptr else None),
          "vrt_unpack_tiles_device")


def pack_tiles_c_device(film, rank, nranks, comps, d_image_ptr, d_packed_ptr, stream_ptr=None):
    """Rank `rank`'s tiles of a (ny, nx, comps) device image -> its packed
    buffer (vrt_pack_tiles_c_device; config 5: comps = 1)."""
    check(lib().vrt_pack_tiles_c_device(C.byref(film.c), int(rank), int(nranks), int(comps), C.c_void_p(d_image_ptr),
                                        C.c_void_p(d_packed_ptr), C.c_void_p(stream_ptr) if stream_ptr else None),
          "vrt_pack_tiles_c_device")


def unpack_tiles_c_device(film, nranks, comps, d_gathered_ptr, d_image_ptr, stream_ptr=None):
    """Rank 0 after the gather: nranks packed buffers -> the (ny, nx, comps)
    image (vrt_unpack_tiles_c_device)."""
    check(lib().vrt_unpack_tiles_c_device(C.byref(film.c), int(nranks), int(comps), C.c_void_p(d_gathered_ptr),
                                          C.c_void_p(d_image_ptr), C.c_void_p(stream_ptr) if stream_ptr else None),
          "vrt_unpack_tiles_c_device")


def intersect_triangle3(orig, direction, v0, v1, v2):
    """VRT/raytri.h:5-7 -> (ret, t, u, v); t/u/v only meaningful when ret == 1."""
    a = [np.ascontiguousarray(np.asarray(x, np.float64).reshape(3)) for x in (orig, direction, v0, v1, v2)]
    t, u, v = C.c_double(), C.c_double(), C.c_double()
    r = lib().intersect_triangle3(*[ptr(x, _ffi.f64p) for x in a], C.byref(t), C.byref(u), C.byref(v))
    return r, t.value, u.value, v.value


def tri_box_overlap(center, half, tri):
    """VRT/tribox2.h:6 -> 1/0."""
    c = np.ascontiguousarray(np.asarray(center, np.float32).reshape(3))
    h = np.ascontiguousarray(np.asarray(half, np.float32).reshape(3))
    t = np.ascontiguousarray(np.asarray(tri, np.float32).reshape(9))
    return lib().triBoxOverlap(ptr(c, _ffi.f32p), ptr(h, _ffi.f32p), ptr(t, _ffi.f32p))


def hdr_bytes(img):
    """The exact bytes stbi_write_hdr would write for img (h, w, comp)."""
    img = np.ascontiguousarray(np.asarray(img, np.float32))
    h, w = img.shape[:2]
    comp = 1 if img.ndim == 2 else img.shape[2]
    n = lib().vrt_write_hdr_mem(w, h, comp, ptr(img, _ffi.f32p), None, 0)
    if n == 0:
        raise VrtError(_ffi.VRT_E_INVALID, "vrt_write_hdr_mem")
    buf = np.zeros(-n, np.uint8)
    n2 = lib().vrt_write_hdr_mem(w, h, comp, ptr(img, _ffi.f32p), ptr(buf, _ffi.u8p), -n)
    assert n2 == -n
    return buf.tobytes()


def hdr_bytes_from_rgbe(rgbe):
    """stbi_write_hdr bytes from packed RGBE (h, w, 4) uint8 (vrt_write_hdr_rgbe_mem)."""
    rgbe = np.ascontiguousarray(np.asarray(rgbe, np.uint8))
    h, w = rgbe.shape[:2]
    n = lib().vrt_write_hdr_rgbe_mem(w, h, ptr(rgbe, _ffi.u8p), None, 0)
    if n == 0:
        raise VrtError(_ffi.VRT_E_INVALID, "vrt_write_hdr_rgbe_mem")
    buf = np.zeros(-n, np.uint8)
    assert lib().vrt_write_hdr_rgbe_mem(w, h, ptr(rgbe, _ffi.u8p), ptr(buf, _ffi.u8p), -n) == -n
    return buf.tobytes()


def rgbe_device(d_img_ptr, w, h, comp, d_rgbe_ptr, stream_ptr=None):
    """k_rgbe: pack a device float image (w*h*comp) into w*h*4 RGBE bytes."""
    check(lib().vrt_rgbe_device(C.c_void_p(d_img_ptr), int(w), int(h), int(comp), C.c_void_p(d_rgbe_ptr),
                                None if stream_ptr is None else C.c_void_p(stream_ptr)), "vrt_rgbe_device")


def write_hdr_device(path, d_img_ptr, w, h, comp=3, stream_ptr=None):
    """stbi_write_hdr of a device-resident image: RGBE packed on the GPU,
    4 bytes/pixel copied back, RLE on the host.  Byte-identical to write_hdr."""
    import torch
    rgbe = torch.empty(int(w) * int(h) * 4, dtype=torch.uint8, device="cuda")
    rgbe_device(d_img_ptr, w, h, comp, rgbe.data_ptr(), stream_ptr)
    torch.cuda.synchronize()
    host = rgbe.cpu().numpy()
    return lib().vrt_write_hdr_rgbe(str(path).encode(), int(w), int(h), ptr(host, _ffi.u8p)) == 1


def write_hdr(path, img):
    """stbi_write_hdr(path, w, h, comp, data): True on success."""
    img = np.ascontiguousarray(np.asarray(img, np.float32))
    h, w = img.shape[:2]
    comp = 1 if img.ndim == 2 else img.shape[2]
    return lib().vrt_write_hdr(str(path).encode(), w, h, comp, ptr(img, _ffi.f32p)) == 1


def sweep_pose(root_min, root_max, i, n):
    """Camera-sweep pose i of n -> (fov, eye, spot, up)."""
    mn, mx = _f3(root_min), _f3(root_max)
    eye, spot, up = np.zeros(3, np.float32), np.zeros(3, np.float32), np.zeros(3, np.float32)
    fov = C.c_float()
    check(lib().vrt_sweep_pose(ptr(mn, _ffi.f32p), ptr(mx, _ffi.f32p), int(i), int(n), ptr(eye, _ffi.f32p),
                               ptr(spot, _ffi.f32p), ptr(up, _ffi.f32p), C.byref(fov)), "vrt_sweep_pose")
    return fov.value, eye, spot, up


def device_selftest_order(dist, hit_mask, depth=None, lengths=None, device=0):
    """The kernels' travorder sort and min_element code on arbitrary inputs
    (vrt_device_selftest_order): dist (n, 8) f32, hit_mask (n,) -> (n, 6)
    u32 order words; depth (m, k) f32 + lengths (m,) -> (m,) first argmin."""
    dist = np.ascontiguousarray(np.asarray(dist, np.float32).reshape(-1, 8))
    hm = np.ascontiguousarray(np.asarray(hit_mask, np.uint32).reshape(-1))
    n = dist.shape[0]
    assert hm.shape[0] == n
    orders = np.zeros((n, 6), np.uint32)
    m, stride, dep, ln, am = 0, 0, None, None, None
    if depth is not None:
        dep = np.ascontiguousarray(np.asarray(depth, np.float32))
        m, stride = dep.shape
        ln = np.ascontiguousarray(np.asarray(lengths, np.int32).reshape(-1))
        assert ln.shape[0] == m
        am = np.zeros(m, np.int32)
    check(lib().vrt_device_selftest_order(device, ptr(dist, _ffi.f32p), ptr(hm, _ffi.u32p), n,
                                          ptr(orders, _ffi.u32p), ptr(dep, _ffi.f32p), ptr(ln, _ffi.i32p), m,
                                          stride, ptr(am, _ffi.i32p)), "vrt_device_selftest_order")
    return orders, am


def build_id():
    """Source hash libvrt.so was built from (tools/build_id.py)."""
    return lib().vrt_build_id().decode()


def build_flag(name):
    """A path-selecting compile-time switch of libvrt.so's kernel build
    (vrt_build_flag), e.g. "VRT_SEC_SPILL_T" (config 5's compaction
    threshold; 0 = no compaction)."""
    v = C.c_int64()
    check(lib().vrt_build_flag(name.encode(), C.byref(v)), "vrt_build_flag")
    return v.value


TEST_FORCE_DEFER = 1  # include/vrt.h VRT_TEST_FORCE_DEFER
TEST_FAIL_LAUNCH = 2  # include/vrt.h VRT_TEST_FAIL_LAUNCH
TEST_SPILL_ALL = 4  # include/vrt.h VRT_TEST_SPILL_ALL
TEST_VIRTUAL_RANKS = 8  # include/vrt.h VRT_TEST_VIRTUAL_RANKS (count << 8)
TEST_STREAM_LEFTOVER = 16  # include/vrt.h VRT_TEST_STREAM_LEFTOVER
TEST_LIGHT_TAIL = 32  # include/vrt.h VRT_TEST_LIGHT_TAIL
TEST_PRIM_TAIL = 64  # include/vrt.h VRT_TEST_PRIM_TAIL
TEST_SEC_DEFER = 128  # include/vrt.h VRT_TEST_SEC_DEFER


def set_test_flags(flags):
    """Test hook (vrt_set_test_flags): flags read by every later launch."""
    check(lib().vrt_set_test_flags(int(flags)), "vrt_set_test_flags")


def test_flags():
    """The current vrt_set_test_flags value (vrt_test_flags)."""
    return int(lib().vrt_test_flags())


def device_count():
    n = C.c_int32()
    check(lib().vrt_device_count(C.byref(n)), "vrt_device_count")
    return n.value


def device_selftest(mt_in=None, sat_in=None, device=0):
    """Run the kernels' own MT / SAT code on the device over n cases."""
    n = len(mt_in) if mt_in is not None else len(sat_in)
    mt_out = np.zeros((n, 4), np.float64) if mt_in is not None else None
    sat_out = np.zeros(n, np.int32) if sat_in is not None else None
    mi = None if mt_in is None else np.ascontiguousarray(np.asarray(mt_in, np.float64).reshape(n, 15))
    si = None if sat_in is None else np.ascontiguousarray(np.asarray(sat_in, np.float32).reshape(n, 15))
    check(lib().vrt_device_selftest(int(device), ptr(mi, _ffi.f64p), ptr(mt_out, _ffi.f64p),
                                    ptr(si, _ffi.f32p), ptr(sat_out, _ffi.i32p), n), "vrt_device_selftest")
    return mt_out, sat_out
