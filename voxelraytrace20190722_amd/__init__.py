"""MI355X-native drop-in for jqly/VoxelRayTrace20190722's per-pixel
voxel-octree ray-march + ray/triangle hit loop.

The compute path is libvrt.so (HIP kernels for gfx950 behind the C ABI in
include/vrt.h); this package is its Python binding.  Importing the API loads
the library and raises if it is missing: there is no CPU fallback.
"""
from ._ffi import VrtError, lib, LIB_PATH  # noqa: F401
from .api import (  # noqa: F401
    FLT_MAX, Camera, Film, MultiOctree, ObjModel, SceneData, VoxelOctree, multi_tile_map, build_id, build_flag, test_flags, device_count, device_selftest,
    device_selftest_order,
    hdr_bytes, hdr_bytes_from_rgbe, intersect_triangle3, load_image, make_ray, obj2voxel, ray_march, ray_march_init,
    TEST_FORCE_DEFER, TEST_FAIL_LAUNCH, TEST_SPILL_ALL, TEST_STREAM_LEFTOVER, TEST_LIGHT_TAIL, TEST_PRIM_TAIL, TEST_SEC_DEFER, TEST_VIRTUAL_RANKS, render, set_test_flags, sweep_pose, tga_decode, tile_deal_map, tiles_per_rank, to_radian, tri_box_overlap,
    unpack_tiles_device, pack_tiles_c_device, unpack_tiles_c_device, write_hdr, rgbe_device, write_hdr_device,
)

__all__ = [
    "VrtError", "lib", "LIB_PATH", "FLT_MAX", "Camera", "Film", "SceneData", "VoxelOctree", "MultiOctree",
    "multi_tile_map",
    "device_count", "device_selftest", "hdr_bytes", "intersect_triangle3", "make_ray",
    "ray_march", "ray_march_init", "render", "sweep_pose", "tile_deal_map", "tiles_per_rank", "to_radian",
    "tri_box_overlap", "unpack_tiles_device", "pack_tiles_c_device", "unpack_tiles_c_device", "write_hdr", "ObjModel", "obj2voxel", "load_image",
    "tga_decode", "hdr_bytes_from_rgbe", "rgbe_device", "write_hdr_device", "build_id", "build_flag", "test_flags", "device_selftest_order", "set_test_flags",
]
