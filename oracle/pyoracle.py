"""TEST INFRASTRUCTURE ONLY: ctypes binding of oracle/liboracle.so (the CPU
restatement, vrt_oracle.c) and of oracle/_ref/libvrtref.so (the reference's
own raytri.cc / tribox2.cc / stb_image_write.h, compiled unmodified).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product (libvrt.so, voxelraytrace20190722_amd) never does.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libvrtref.so")

f32p = C.POINTER(C.c_float)
f64p = C.POINTER(C.c_double)
i32p = C.POINTER(C.c_int32)
u32p = C.POINTER(C.c_uint32)
i64p = C.POINTER(C.c_int64)
u8p = C.POINTER(C.c_uint8)
P = C.c_void_p

_o = None
_r = None


def _p(a, t):
    return None if a is None else a.ctypes.data_as(t)


def oracle():
    global _o
    if _o is None:
        if not os.path.exists(ORACLE_SO):
            raise ImportError(f"{ORACLE_SO} missing: run `make -C oracle`")
        L = C.CDLL(ORACLE_SO)
        sig = {
            "ora_intersect_triangle3": (C.c_int, [f64p] * 8),
            "ora_tri_box_overlap": (C.c_int, [f32p, f32p, f32p]),
            "ora_camera_init": (None, [C.c_float, f32p, f32p, f32p, C.c_float, C.c_float, f32p]),
            "ora_gen_rays4": (C.c_int, [f32p, C.c_float, C.c_float, C.c_int, C.c_int, C.c_int, C.c_int, f32p]),
            "ora_gen_rays1": (C.c_int, [f32p, C.c_float, C.c_float, C.c_int, C.c_int, C.c_int, C.c_int, f32p]),
            "ora_make_ray": (None, [f32p, f32p, C.c_float, C.c_float, f32p]),
            "ora_aabb_isect": (C.c_int, [f32p, f32p]),
            "ora_sort8": (None, [f32p, i32p]),
            "ora_first_min": (C.c_int, [f32p, C.c_int]),
            "ora_scene_create": (P, [f32p, f32p, f32p, i32p, C.c_int, C.c_int]),
            "ora_scene_set_materials": (None, [P, C.c_int, i32p, f32p, C.c_int, i32p, i64p, u8p, C.c_int64]),
            "ora_scene_destroy": (None, [P]),
            "ora_scene_info": (None, [P, i64p, f32p]),
            "ora_scene_leaves": (None, [P, u32p, u32p, i32p]),
            "ora_ray_march": (None, [P, f32p, C.c_int, i32p, i32p, u32p, f32p, f32p, u32p]),
            "ora_shade": (None, [P, f32p, C.c_int, f32p]),
            "ora_render": (None, [P, f32p, C.c_float, C.c_float, C.c_int, C.c_int, C.c_int, C.c_int,
                                  f32p, i32p, i32p, u32p, f32p, u32p]),
            "ora_render_rows": (C.c_double, [P, f32p, C.c_float, C.c_float, C.c_int, C.c_int, C.c_int,
                                             C.c_int, C.c_int, f32p]),
            "ora_linear_to_rgbe": (None, [f32p, u8p]),
            "ora_pcg_next": (C.c_uint32, [C.POINTER(C.c_uint64)]),
            "ora_uniform_m11": (C.c_float, [C.POINTER(C.c_uint64)]),
            "ora_random_point_in_unit_sphere": (None, [C.POINTER(C.c_uint64), f32p]),
            "ora_render_secondary": (C.c_int64, [P, f32p, C.c_float, C.c_float, C.c_int, C.c_int, C.c_int,
                                                 C.c_int, f32p, i32p, i32p, u32p]),
            "ora_lightmap": (C.c_int64, [P, f32p, C.c_float, C.c_float, C.c_int, C.c_int, C.c_int]),
            "ora_lightmap_filter": (None, [P]),
            "ora_lightmap_nodes": (None, [P, C.POINTER(C.c_uint64), f32p, f32p]),
            "ora_min_voxel": (C.c_float, [P, C.c_int]),
            "ora_shade_trace": (None, [P, f32p, C.c_int, C.c_float, f32p]),
            "ora_render_trace": (None, [P, f32p, C.c_float, C.c_float, C.c_int, C.c_int, C.c_float, C.c_int,
                                        f32p, i32p, f32p]),
        }
        for k, (res, args) in sig.items():
            f = getattr(L, k)
            f.restype = res
            f.argtypes = args
        _o = L
    return _o


def sort8(dist):
    """travorder's std::sort of the 8 Items by dist -> child order (8,)."""
    d = np.ascontiguousarray(np.asarray(dist, np.float32).reshape(8))
    o = np.zeros(8, np.int32)
    oracle().ora_sort8(_p(d, f32p), _p(o, i32p))
    return o


def first_min(depth):
    """ray_march_isect's std::min_element index (-1 if empty)."""
    d = np.ascontiguousarray(np.asarray(depth, np.float32).reshape(-1))
    return int(oracle().ora_first_min(_p(d, f32p), d.shape[0]))


def reference_available():
    return os.path.exists(REF_SO)


def reference():
    """The reference's own primitives (oracle/_ref/libvrtref.so)."""
    global _r
    if _r is None:
        if not os.path.exists(REF_SO):
            raise ImportError(f"{REF_SO} missing (built only where /root/reference exists)")
        L = C.CDLL(REF_SO)
        L.ref_intersect_triangle3.restype = C.c_int
        L.ref_intersect_triangle3.argtypes = [f64p] * 6 + [C.POINTER(C.c_int)]
        L.ref_tri_box_overlap.restype = C.c_int
        L.ref_tri_box_overlap.argtypes = [f32p, f32p, f32p]
        L.ref_write_hdr_mem.restype = C.c_long
        L.ref_write_hdr_mem.argtypes = [C.c_int, C.c_int, C.c_int, f32p, u8p, C.c_long]
        L.ref_load_obj.restype = C.POINTER(_RefObj)
        L.ref_load_obj.argtypes = [C.c_char_p, C.c_char_p]
        L.ref_free_obj.restype = None
        L.ref_free_obj.argtypes = [C.POINTER(_RefObj)]
        L.ref_stbi_load.restype = u8p
        L.ref_stbi_load.argtypes = [C.c_char_p, i32p, i32p, i32p]
        L.ref_stbi_load_mem.restype = u8p
        L.ref_stbi_load_mem.argtypes = [u8p, C.c_int, i32p, i32p, i32p]
        L.ref_stbi_free.restype = None
        L.ref_stbi_free.argtypes = [u8p]
        L.ref_stbi_failure.restype = C.c_char_p
        _r = L
    return _r


class _RefObj(C.Structure):
    _fields_ = [("ok", C.c_int32), ("nv", C.c_int64), ("nvn", C.c_int64), ("nvt", C.c_int64),
                ("v", f32p), ("vn", f32p), ("vt", f32p), ("nshape", C.c_int32), ("nface", C.c_int64),
                ("fv", i32p), ("idx", i32p), ("mat", i32p), ("shape", i32p), ("nmat", C.c_int32),
                ("kd", f32p), ("name", C.POINTER(C.c_char_p)), ("tex", C.POINTER(C.c_char_p)),
                ("warn", C.c_char_p), ("err", C.c_char_p)]


def ref_load_obj(path, mtl_basedir):
    """tinyobj::LoadObj(.., path, mtl_basedir, triangulate=true) of the
    reference (compiled in place), flattened to numpy."""
    L = reference()
    q = L.ref_load_obj(str(path).encode(), None if mtl_basedir is None else str(mtl_basedir).encode())
    o = q.contents
    try:
        def arr(p, n, dt):
            return np.ctypeslib.as_array(p, (n,)).astype(dt) if n else np.zeros(0, dt)
        out = {"ok": bool(o.ok), "v": arr(o.v, o.nv * 3, np.float32).reshape(-1, 3),
               "vn": arr(o.vn, o.nvn * 3, np.float32).reshape(-1, 3),
               "vt": arr(o.vt, o.nvt * 2, np.float32).reshape(-1, 2), "nshape": o.nshape,
               "fv": arr(o.fv, o.nface, np.int32), "idx": arr(o.idx, o.nface * 9, np.int32).reshape(-1, 3, 3),
               "mat": arr(o.mat, o.nface, np.int32), "shape": arr(o.shape, o.nface, np.int32),
               "kd": arr(o.kd, o.nmat * 3, np.float32).reshape(-1, 3),
               "names": [o.name[i].decode(errors="surrogateescape") for i in range(o.nmat)],
               "texnames": [o.tex[i].decode(errors="surrogateescape") for i in range(o.nmat)],
               "warn": o.warn.decode(errors="replace"), "err": o.err.decode(errors="replace")}
    finally:
        L.ref_free_obj(q)
    return out


def _stbi_out(L, p, w, h, c):
    if not p:
        return None, L.ref_stbi_failure().decode()
    try:
        a = np.ctypeslib.as_array(p, (w.value * h.value * c.value,)).copy()
    finally:
        L.ref_stbi_free(p)
    return a.reshape(h.value, w.value, c.value), ""


def ref_stbi_load(path):
    """stbi_load(path, &w, &h, &c, 0) -> (uint8 (h, w, c) or None, failure reason)."""
    L = reference()
    w, h, c = C.c_int(), C.c_int(), C.c_int()
    p = L.ref_stbi_load(str(path).encode(), C.byref(w), C.byref(h), C.byref(c))
    return _stbi_out(L, p, w, h, c)


def ref_stbi_load_mem(data):
    L = reference()
    buf = np.frombuffer(bytes(data), np.uint8).copy()
    w, h, c = C.c_int(), C.c_int(), C.c_int()
    p = L.ref_stbi_load_mem(_p(buf, u8p) if buf.size else (C.c_uint8 * 1)(), buf.size, C.byref(w), C.byref(h),
                            C.byref(c))
    return _stbi_out(L, p, w, h, c)


# ---------------------------------------------------------------- primitives
def intersect_triangle3(q):
    """q: (15,) float64 {orig, dir, v0, v1, v2} -> (ret, t, u, v)."""
    q = np.ascontiguousarray(q, np.float64)
    t, u, v = C.c_double(), C.c_double(), C.c_double()
    r = oracle().ora_intersect_triangle3(*[_p(q[3 * k:3 * k + 3], f64p) for k in range(5)],
                                         C.byref(t), C.byref(u), C.byref(v))
    return r, t.value, u.value, v.value


def tri_box_overlap(q):
    """q: (15,) float32 {center, half, tri[9]} -> 1/0."""
    q = np.ascontiguousarray(q, np.float32)
    return oracle().ora_tri_box_overlap(_p(q[0:3], f32p), _p(q[3:6], f32p), _p(q[6:15], f32p))


def ref_intersect_triangle3(q):
    q = np.ascontiguousarray(q, np.float64)
    out = np.zeros(3)
    r = reference().ref_intersect_triangle3(*[_p(q[3 * k:3 * k + 3], f64p) for k in range(5)],
                                            _p(out, f64p), None)
    return r, out[0], out[1], out[2]


def ref_tri_box_overlap(q):
    q = np.ascontiguousarray(q, np.float32)
    return reference().ref_tri_box_overlap(_p(q[0:3], f32p), _p(q[3:6], f32p), _p(q[6:15], f32p))


def ref_hdr_bytes(img):
    img = np.ascontiguousarray(np.asarray(img, np.float32))
    h, w = img.shape[:2]
    comp = 1 if img.ndim == 2 else img.shape[2]
    n = reference().ref_write_hdr_mem(w, h, comp, _p(img, f32p), None, 0)
    buf = np.zeros(-n, np.uint8)
    n2 = reference().ref_write_hdr_mem(w, h, comp, _p(img, f32p), _p(buf, u8p), -n)
    assert n2 == -n
    return buf.tobytes()


def linear_to_rgbe_img(img):
    """stbiw__linear_to_rgbe per pixel of an (h, w, comp) float image ->
    (h, w, 4) uint8 (comp 1/2: grey; comp >= 3: first three channels)."""
    img = np.asarray(img, np.float32)
    if img.ndim == 2:
        img = img[:, :, None]
    h, w, c = img.shape
    lin = np.ascontiguousarray(np.repeat(img[:, :, :1], 3, 2) if c < 3 else img[:, :, :3]).reshape(-1, 3)
    out = np.zeros((h * w, 4), np.uint8)
    f = oracle().ora_linear_to_rgbe
    for i in range(h * w):
        f(_p(lin[i], f32p), _p(out[i], u8p))
    return out.reshape(h, w, 4)


def uniform_draws(seed, n):
    st = C.c_uint64(seed)
    return np.array([oracle().ora_uniform_m11(C.byref(st)) for _ in range(n)], np.float32)


def sphere_points(seed, n):
    st = C.c_uint64(seed)
    out = np.zeros((n, 3), np.float32)
    for i in range(n):
        oracle().ora_random_point_in_unit_sphere(C.byref(st), _p(out[i], f32p))
    return out


# ---------------------------------------------------------------- camera
def camera(fov, eye, spot, up, near=0.0, far=float(np.finfo(np.float32).max)):
    cam = np.zeros(19, np.float32)
    e, s, u = (np.ascontiguousarray(np.asarray(x, np.float32)) for x in (eye, spot, up))
    oracle().ora_camera_init(float(fov), _p(e, f32p), _p(s, f32p), _p(u, f32p), float(near), float(far),
                             _p(cam, f32p))
    return cam


def gen_rays4(cam, film_w, film_h, nx, ny, px, py):
    out = np.zeros((4, 8), np.float32)
    oracle().ora_gen_rays4(_p(cam, f32p), film_w, film_h, nx, ny, px, py, _p(out, f32p))
    return out


def gen_rays1(cam, film_w, film_h, nx, ny, px, py):
    out = np.zeros((1, 8), np.float32)
    oracle().ora_gen_rays1(_p(cam, f32p), film_w, film_h, nx, ny, px, py, _p(out, f32p))
    return out


def make_ray(o, d, tmin, tmax):
    out = np.zeros(8, np.float32)
    o = np.ascontiguousarray(o, np.float32)
    d = np.ascontiguousarray(d, np.float32)
    oracle().ora_make_ray(_p(o, f32p), _p(d, f32p), tmin, tmax, _p(out, f32p))
    return out


def aabb_isect(box, ray):
    box = np.ascontiguousarray(box, np.float32)
    ray = np.ascontiguousarray(ray, np.float32)
    return oracle().ora_aabb_isect(_p(box, f32p), _p(ray, f32p))


# ---------------------------------------------------------------- scene
class Scene:
    """The oracle's octree over a SceneData-like object."""

    def __init__(self, sd, max_depth):
        L = oracle()
        self.sd = sd
        self.max_depth = int(max_depth)
        uv = sd.uv if sd.uv is not None else np.zeros((sd.ntri, 6), np.float32)
        mat = sd.mat if sd.mat is not None else np.zeros(sd.ntri, np.int32)
        self._uv, self._mat = np.ascontiguousarray(uv), np.ascontiguousarray(mat)
        self.h = L.ora_scene_create(_p(sd.pos, f32p), _p(sd.nrm, f32p), _p(self._uv, f32p),
                                    _p(self._mat, i32p), sd.ntri, max_depth)
        ntex = len(sd.tex_off)
        L.ora_scene_set_materials(self.h, len(sd.mat_tex), _p(sd.mat_tex, i32p), _p(sd.mat_kd, f32p), ntex,
                                  _p(sd.tex_dims, i32p) if ntex else None,
                                  _p(sd.tex_off, i64p) if ntex else None,
                                  _p(sd.tex_data, u8p) if ntex else None, int(sd.tex_data.size))

    def close(self):
        if self.h:
            oracle().ora_scene_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self):
        info = np.zeros(5, np.int64)
        box = np.zeros(6, np.float32)
        oracle().ora_scene_info(self.h, _p(info, i64p), _p(box, f32p))
        return info, box

    def leaves(self):
        info, _ = self.info()
        vox = np.zeros(info[3], np.uint32)
        cnt = np.zeros(info[3], np.uint32)
        tris = np.zeros(max(info[4], 1), np.int32)
        oracle().ora_scene_leaves(self.h, _p(vox, u32p), _p(cnt, u32p), _p(tris, i32p))
        return vox, cnt, tris[:info[4]]

    def ray_march(self, rays):
        rays = np.ascontiguousarray(np.asarray(rays, np.float32).reshape(-1, 8))
        n = rays.shape[0]
        hit = np.zeros(n, np.int32)
        tri = np.zeros(n, np.int32)
        vox = np.zeros(n, np.uint32)
        hp = np.zeros((n, 3), np.float32)
        nr = np.zeros((n, 3), np.float32)
        cnt = np.zeros((n, 4), np.uint32)
        oracle().ora_ray_march(self.h, _p(rays, f32p), n, _p(hit, i32p), _p(tri, i32p), _p(vox, u32p),
                               _p(hp, f32p), _p(nr, f32p), _p(cnt, u32p))
        return {"hit": hit, "tri": tri, "voxel": vox, "hit_p": hp, "normal": nr, "counters": cnt}

    def shade(self, rays):
        rays = np.ascontiguousarray(np.asarray(rays, np.float32).reshape(-1, 8))
        out = np.zeros((rays.shape[0], 3), np.float32)
        oracle().ora_shade(self.h, _p(rays, f32p), rays.shape[0], _p(out, f32p))
        return out

    def render(self, cam, film_w, film_h, nx, ny, film_index=1, nthreads=8, samples=True):
        rgb = np.zeros((ny, nx, 3), np.float32)
        ns = nx * ny * 4
        so = None
        if samples:
            so = {"hit": np.zeros(ns, np.int32), "tri": np.zeros(ns, np.int32),
                  "voxel": np.zeros(ns, np.uint32), "rgb": np.zeros((ns, 3), np.float32),
                  "counters": np.zeros((ns, 4), np.uint32)}
        oracle().ora_render(self.h, _p(cam, f32p), film_w, film_h, nx, ny, film_index, nthreads,
                            _p(rgb, f32p),
                            _p(so["hit"], i32p) if so else None, _p(so["tri"], i32p) if so else None,
                            _p(so["voxel"], u32p) if so else None, _p(so["rgb"], f32p) if so else None,
                            _p(so["counters"], u32p) if so else None)
        return (rgb, so) if so else rgb

    def render_secondary(self, cam, film_w, film_h, nx, ny, spp=64, nthreads=8, ids=True):
        vis = np.zeros((ny, nx), np.float32)
        ns = nx * ny * spp
        d = {"hit": np.zeros(ns, np.int32), "tri": np.zeros(ns, np.int32),
             "voxel": np.zeros(ns, np.uint32)} if ids else None
        rays = oracle().ora_render_secondary(self.h, _p(cam, f32p), film_w, film_h, nx, ny, spp, nthreads,
                                             _p(vis, f32p), _p(d["hit"], i32p) if d else None,
                                             _p(d["tri"], i32p) if d else None,
                                             _p(d["voxel"], u32p) if d else None)
        return (vis, rays, d) if ids else (vis, rays)

    def render_rows(self, cam, film_w, film_h, nx, ny, row_stride, row_phase, nthreads):
        rgb = np.zeros((ny, nx, 3), np.float32)
        sec = oracle().ora_render_rows(self.h, _p(cam, f32p), film_w, film_h, nx, ny, row_stride,
                                       row_phase, nthreads, _p(rgb, f32p))
        return sec, rgb

    # ---- full trace() ----
    def lightmap(self, cam, film_w, film_h, nx, ny, nthreads=8, filter=True):
        """Light pass in canonical order (+ cone_trace_init_filter); returns hits."""
        hits = oracle().ora_lightmap(self.h, _p(cam, f32p), film_w, film_h, nx, ny, nthreads)
        if filter:
            oracle().ora_lightmap_filter(self.h)
        return hits

    def lightmap_nodes(self):
        """(key depth<<32|vox, coverage, illum (n,6,3)) sorted by key."""
        n = int(self.info()[0][0])
        key = np.zeros(n, np.uint64)
        cov = np.zeros(n, np.float32)
        ill = np.zeros((n, 6, 3), np.float32)
        oracle().ora_lightmap_nodes(self.h, key.ctypes.data_as(C.POINTER(C.c_uint64)), _p(cov, f32p),
                                    _p(ill, f32p))
        o = np.argsort(key, kind="stable")
        return key[o], cov[o], ill[o]

    def min_voxel(self, levels=None):
        return float(oracle().ora_min_voxel(self.h, self.max_depth if levels is None else int(levels)))

    def shade_trace(self, rays, res):
        rays = np.ascontiguousarray(np.asarray(rays, np.float32).reshape(-1, 8))
        out = np.zeros((rays.shape[0], 3), np.float32)
        oracle().ora_shade_trace(self.h, _p(rays, f32p), rays.shape[0], res, _p(out, f32p))
        return out

    def render_trace(self, cam, film_w, film_h, nx, ny, res, nthreads=8, samples=True):
        rgb = np.zeros((ny, nx, 3), np.float32)
        ns = nx * ny * 4
        hit = np.zeros(ns, np.int32) if samples else None
        srgb = np.zeros((ns, 3), np.float32) if samples else None
        oracle().ora_render_trace(self.h, _p(cam, f32p), film_w, film_h, nx, ny, res, nthreads, _p(rgb, f32p),
                                  _p(hit, i32p), _p(srgb, f32p))
        return (rgb, {"hit": hit, "rgb": srgb}) if samples else rgb
