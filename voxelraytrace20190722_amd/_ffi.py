"""ctypes binding of libvrt.so (include/vrt.h).

This is the reference-side binding a Python caller would add for the C ABI
(INTEGRATION.md shows the C/C++ and ctypes forms).  There is no fallback: if
the HIP library is missing, importing the package's API raises.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libvrt.so")

VRT_OK = 0
VRT_E_INVALID = -1
VRT_E_NOMEM = -2
VRT_E_DEVICE = -3
VRT_E_NODEVICE = -4
VRT_E_IO = -5
VRT_MAX_DEPTH = 11

f32p = C.POINTER(C.c_float)
f64p = C.POINTER(C.c_double)
i32p = C.POINTER(C.c_int32)
u32p = C.POINTER(C.c_uint32)
i64p = C.POINTER(C.c_int64)
u8p = C.POINTER(C.c_uint8)


class SceneDesc(C.Structure):
    _fields_ = [("ntri", C.c_int32), ("pos", f32p), ("nrm", f32p), ("uv", f32p),
                ("mat", i32p), ("nmat", C.c_int32), ("mat_tex", i32p),
                ("mat_kd", f32p), ("ntex", C.c_int32), ("tex_dims", i32p),
                ("tex_off", i64p), ("tex_data", u8p), ("tex_bytes", C.c_int64)]


class Ray(C.Structure):
    _fields_ = [("o", C.c_float * 3), ("d", C.c_float * 3),
                ("tmin", C.c_float), ("tmax", C.c_float)]


class Camera(C.Structure):
    _fields_ = [("C", C.c_float * 16), ("fov", C.c_float), ("near_", C.c_float),
                ("far_", C.c_float), ("origin", C.c_float * 3)]


class Film(C.Structure):
    _fields_ = [("w", C.c_float), ("h", C.c_float), ("nx", C.c_int32),
                ("ny", C.c_int32)]


class Hit(C.Structure):
    _fields_ = [("hit", C.c_int32), ("tri", C.c_int32), ("voxel", C.c_uint32),
                ("hit_p", C.c_float * 3), ("normal", C.c_float * 3)]


class SceneInfo(C.Structure):
    _fields_ = [("nodes", C.c_int64), ("internal", C.c_int64),
                ("leaves", C.c_int64), ("nonempty_leaves", C.c_int64),
                ("tri_refs", C.c_int64), ("max_depth", C.c_int32),
                ("device", C.c_int32), ("root_min", C.c_float * 3),
                ("root_max", C.c_float * 3), ("device_bytes", C.c_int64),
                ("build_ms", C.c_double), ("upload_ms", C.c_double),
                ("build_device_ms", C.c_double)]


class Samples(C.Structure):
    _fields_ = [("hit", i32p), ("tri", i32p), ("voxel", u32p), ("rgb", f32p),
                ("counters", u32p)]


class Stats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("aabb_tests", C.c_uint64),
                ("leaves", C.c_uint64), ("tri_tests", C.c_uint64),
                ("hits", C.c_uint64), ("kernel_ms", C.c_double)]


class ObjInfo(C.Structure):
    _fields_ = [("nvert", C.c_int64), ("nnormal", C.c_int64), ("ntexcoord", C.c_int64),
                ("nshape", C.c_int32), ("nface", C.c_int64), ("nmat", C.c_int32),
                ("has_soup", C.c_int32), ("nsoup_mat", C.c_int32), ("ntex", C.c_int32),
                ("tex_bytes", C.c_int64)]


VRT_OBJ_PARSE_ONLY = 1
VRT_BUILD_DEVICE = 1

_P = C.c_void_p
SIGNATURES = {
    "vrt_device_count": (C.c_int, [i32p]),
    "vrt_scene_create": (C.c_int, [C.POINTER(SceneDesc), C.c_int, C.c_int, C.POINTER(_P)]),
    "vrt_scene_create_ex": (C.c_int, [C.POINTER(SceneDesc), C.c_int, C.c_int, C.c_int, C.POINTER(_P)]),
    "vrt_scene_destroy": (None, [_P]),
    "vrt_scene_info": (C.c_int, [_P, C.POINTER(SceneInfo)]),
    "vrt_scene_leaves": (C.c_int, [_P, u32p, u32p, i32p]),
    "vrt_scene_nodes": (C.c_int, [_P, f32p, u32p, u32p]),
    "vrt_camera_init": (C.c_int, [C.c_float, f32p, f32p, f32p, C.c_float, C.c_float,
                                  C.POINTER(Camera)]),
    "vrt_gen_rays4": (C.c_int, [C.POINTER(Camera), C.POINTER(Film), C.c_int, C.c_int,
                                C.POINTER(Ray)]),
    "vrt_gen_rays1": (C.c_int, [C.POINTER(Camera), C.POINTER(Film), C.c_int, C.c_int,
                                C.POINTER(Ray)]),
    "vrt_make_ray": (C.c_int, [f32p, f32p, C.c_float, C.c_float, C.POINTER(Ray)]),
    "vrt_aabb_isect": (C.c_int, [f32p, C.POINTER(Ray)]),
    "vrt_render": (C.c_int, [_P, C.POINTER(Camera), C.POINTER(Film), f32p,
                             C.POINTER(Samples), C.POINTER(Stats)]),
    "vrt_tiles_per_rank": (C.c_int, [C.POINTER(Film), C.c_int]),
    "vrt_tile_deal_block": (C.c_int, []),
    "vrt_scene_set_frames_in_flight": (C.c_int, [C.c_void_p, C.c_int]),
    "vrt_tile_deal_map": (C.c_int, [C.POINTER(Film), C.c_int, i32p, i32p]),
    "vrt_render_tiles_device": (C.c_int, [_P, C.POINTER(Camera), C.POINTER(Film), C.c_int,
                                          C.c_int, C.c_int, _P, _P]),
    "vrt_unpack_tiles_device": (C.c_int, [C.POINTER(Film), C.c_int, _P, _P, _P]),
    "vrt_pack_tiles_c_device": (C.c_int, [C.POINTER(Film), C.c_int, C.c_int, C.c_int, _P, _P, _P]),
    "vrt_unpack_tiles_c_device": (C.c_int, [C.POINTER(Film), C.c_int, C.c_int, _P, _P, _P]),
    "vrt_last_kernel_ms": (C.c_int, [_P, f32p]),
    "vrt_render_secondary": (C.c_int, [_P, C.POINTER(Camera), C.POINTER(Film), C.c_int, f32p, i32p,
                                       i32p, u32p, i64p]),
    "vrt_render_secondary_device": (C.c_int, [_P, C.POINTER(Camera), C.POINTER(Film), C.c_int, C.c_int,
                                              C.c_int, _P, _P, _P]),
    "vrt_ray_march_batch": (C.c_int, [_P, C.POINTER(Ray), C.c_int64, C.POINTER(Hit)]),
    "vrt_ray_march_batch_device": (C.c_int, [_P, _P, C.c_int64, _P, _P]),
    "vrt_device_selftest": (C.c_int, [C.c_int, f64p, f64p, f32p, i32p, C.c_int64]),
    "vrt_write_hdr": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, f32p]),
    "stbi_write_hdr": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, f32p]),
    "vrt_build_id": (C.c_char_p, []),
    "vrt_build_flag": (C.c_int, [C.c_char_p, i64p]),
    "vrt_test_flags": (C.c_int, []),
    "vrt_set_test_flags": (C.c_int, [C.c_int]),
    "vrt_camera_defer_bound": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_int64)]),
    "vrt_secondary_spill_counts": (C.c_int, [_P, i64p]),
    "vrt_secondary_spill_stats": (C.c_int, [_P, i64p]),
    "vrt_scene_scratch_bytes": (C.c_int, [_P, i64p, i64p]),
    "vrt_device_selftest_order": (C.c_int, [C.c_int, f32p, u32p, C.c_int64, u32p, f32p, i32p, C.c_int64,
                                            C.c_int32, i32p]),
    "vrt_write_hdr_mem": (C.c_int64, [C.c_int, C.c_int, C.c_int, f32p, u8p, C.c_int64]),
    "vrt_rgbe_device": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, _P, _P]),
    "vrt_write_hdr_rgbe": (C.c_int, [C.c_char_p, C.c_int, C.c_int, u8p]),
    "vrt_write_hdr_rgbe_mem": (C.c_int64, [C.c_int, C.c_int, u8p, u8p, C.c_int64]),
    "intersect_triangle3": (C.c_int, [f64p, f64p, f64p, f64p, f64p, f64p, f64p, f64p]),
    "triBoxOverlap": (C.c_int, [f32p, f32p, f32p]),
    "vrt_proxy_scene": (C.c_int, [C.c_double, C.c_uint32, i32p, f32p, f32p, f32p, i32p,
                                  i32p, i32p, f32p, i32p, i32p, i64p, u8p, i64p]),
    "vrt_sweep_pose": (C.c_int, [f32p, f32p, C.c_int, C.c_int, f32p, f32p, f32p, f32p]),
    "vrt_lightmap_build": (C.c_int, [_P, C.POINTER(Camera), C.POINTER(Film), i64p]),
    "vrt_lightmap_nodes": (C.c_int, [_P, C.POINTER(C.c_uint64), f32p, f32p]),
    "vrt_scene_min_voxel": (C.c_int, [_P, C.c_int, f32p]),
    "vrt_render_trace": (C.c_int, [_P, C.POINTER(Camera), C.POINTER(Film), C.c_float, f32p, i32p, f32p]),
    "vrt_render_trace_device": (C.c_int, [_P, C.POINTER(Camera), C.POINTER(Film), C.c_float, C.c_int, C.c_int,
                                          C.c_int, _P, _P]),
    "vrt_trace_frame_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_float,
                                         C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_int64)]),
    "vrt_obj_load": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(_P)]),
    "vrt_obj_free": (None, [_P]),
    "vrt_obj_info": (C.c_int, [_P, C.POINTER(ObjInfo)]),
    "vrt_obj_attrib": (C.c_int, [_P, C.POINTER(f32p), C.POINTER(f32p), C.POINTER(f32p)]),
    "vrt_obj_faces": (C.c_int, [_P, i32p, i32p, i32p]),
    "vrt_obj_material": (C.c_int, [_P, C.c_int, C.POINTER(C.c_char_p), f32p, C.POINTER(C.c_char_p)]),
    "vrt_obj_texture_path": (C.c_int, [_P, C.c_int, C.POINTER(C.c_char_p)]),
    "vrt_obj_warnings": (C.c_char_p, [_P]),
    "vrt_obj_scene_desc": (C.c_int, [_P, C.POINTER(SceneDesc)]),
    "vrt_tga_load": (C.c_int, [C.c_char_p, i32p, i32p, i32p, C.POINTER(u8p)]),
    "vrt_tga_decode": (C.c_int, [u8p, C.c_int64, i32p, i32p, i32p, C.POINTER(u8p)]),
    "vrt_image_free": (None, [u8p]),
    "vrt_scene_create_multi": (C.c_int, [C.POINTER(SceneDesc), C.c_int, C.c_uint32, C.c_int, C.POINTER(_P)]),
    "vrt_multi_destroy": (None, [_P]),
    "vrt_multi_devices": (C.c_int, [_P, i32p, i32p]),
    "vrt_multi_scene": (C.c_int, [_P, C.c_int, C.POINTER(_P)]),
    "vrt_render_multi": (C.c_int, [_P, C.POINTER(Camera), C.POINTER(Film), f32p]),
    "vrt_render_multi_device": (C.c_int, [_P, C.POINTER(Camera), C.POINTER(Film), _P, _P]),
    "vrt_multi_tile_map": (C.c_int, [C.POINTER(Film), C.c_uint32, i32p, i32p]),
    "vrt_status_string": (C.c_char_p, [C.c_int]),
    "vrt_last_error": (C.c_char_p, []),
}

_lib = None


class VrtError(RuntimeError):
    def __init__(self, status, where):
        msg = ""
        if _lib is not None:
            msg = _lib.vrt_last_error().decode(errors="replace")
            st = _lib.vrt_status_string(status).decode()
        else:
            st = str(status)
        super().__init__(f"{where}: {st} ({status}) {msg}".strip())
        self.status = status


def lib():
    """Load libvrt.so (built by `make` / __graft_entry__.build()).  Raises if
    it is missing -- there is deliberately no CPU fallback."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} not built: run `make` at the repo root "
                "(or __graft_entry__.build()); the HIP path has no fallback")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(status, where):
    if status != VRT_OK:
        raise VrtError(status, where)
    return status


def ptr(a, t):
    """numpy array -> ctypes pointer (None for None)."""
    if a is None:
        return None
    return a.ctypes.data_as(t)
