#!/usr/bin/env python3
"""Phase breakdown of the persistent fast march from a VRT_PHASE_STAMPS=1
diagnostic build (make fullvariant NAME=diag DEFS=-DVRT_PHASE_STAMPS=1):
renders the bench sweep through that library, reads vrt_diag_phases and
prints per-unit (= ray-wave) averages and lane utilisation.

usage: tools/diag_phases.py build/variants/libvrt_diag.so [--width --height --depth]
"""
import argparse
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import voxelraytrace20190722_amd as vrt  # noqa: E402
from voxelraytrace20190722_amd import _ffi  # noqa: E402
from ab import load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--poses", type=int, default=16)
    a = ap.parse_args()
    L = load(a.lib)
    L.vrt_diag_phases.restype = C.c_int
    L.vrt_diag_phases.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    sd = vrt.SceneData.proxy(1.0, 1)
    h = C.c_void_p()
    d = sd.desc()
    assert L.vrt_scene_create(C.byref(d), a.depth, 0, C.byref(h)) == 0
    info = _ffi.SceneInfo()
    L.vrt_scene_info(h, C.byref(info))
    film = _ffi.Film(1.0, 1.0, a.width, a.height)
    img = torch.zeros((a.height, a.width, 3), dtype=torch.float32, device="cuda:0")
    st = torch.cuda.current_stream()
    buf = (C.c_ulonglong * 24)()
    cams = []
    for i in range(a.poses):
        fov, eye, spot, up = vrt.sweep_pose(info.root_min[:], info.root_max[:], i, a.poses)
        cam = _ffi.Camera()
        L.vrt_camera_init(fov, eye.ctypes.data_as(_ffi.f32p), spot.ctypes.data_as(_ffi.f32p),
                          up.ctypes.data_as(_ffi.f32p), 0.0, vrt.FLT_MAX, C.byref(cam))
        cams.append(cam)
    for cam in cams:  # warm-up
        L.vrt_render_tiles_device(h, C.byref(cam), C.byref(film), 0, 1, 1, C.c_void_p(img.data_ptr()),
                                  C.c_void_p(st.cuda_stream))
    torch.cuda.synchronize()
    L.vrt_diag_phases(buf, 1)
    for cam in cams:
        L.vrt_render_tiles_device(h, C.byref(cam), C.byref(film), 0, 1, 1, C.c_void_p(img.data_ptr()),
                                  C.c_void_p(st.cuda_stream))
    torch.cuda.synchronize()
    assert L.vrt_diag_phases(buf, 0) == 0
    g = [int(x) for x in buf]
    n = max(1, g[11])
    out = {
        "units": n,
        "inner_iters_per_unit_wave": g[0] / n, "inner_lane_util": g[1] / (64 * max(1, g[0])),
        "leaf_phases_per_unit_wave": g[2] / n, "leaf_phase_lane_util": g[3] / (64 * max(1, g[2])),
        "tri_tests_per_ray": g[5] / (64 * n), "tri_loop_iters_per_unit_wave": g[6] / n,
        "tri_loop_lane_util": g[7] / (64 * max(1, g[6])),
        "cycles_per_unit": g[10] / n, "cycles_inner_frac": g[8] / max(1, g[10]),
        "cycles_leaf_frac": g[9] / max(1, g[10]),
        "cycles_other_frac": 1 - (g[8] + g[9]) / max(1, g[10]),
        # wave iterations of the node-visit loop per unit (ray-wave) in which
        # some lane does X: the blocks X runs issue once per such iteration
        "visit_iters_per_unit": g[12] / n, "pop_iters_per_unit": g[13] / n,
        "linebox_skip_iters_per_unit": g[14] / n, "expand_iters_per_unit": g[15] / n,
        "order2_iters_per_unit": g[16] / n, "rank8_iters_per_unit": g[17] / n,
        "net4_iters_per_unit": g[18] / n, "leaf_stop_iters_per_unit": g[19] / n,
    }
    # a persistent wave's time per unit: dequeue, setup (tile, ray, vote),
    # the march call (root + walk), shading + film store
    span = max(1, g[20] + g[21] + g[22] + g[23])
    out.update({"unit_cycles_wave": span / n, "dequeue_frac": g[20] / span, "setup_frac": g[21] / span,
                "march_frac": g[22] / span, "shade_store_frac": g[23] / span})
    print(json.dumps({k: round(v, 4) if isinstance(v, float) else v for k, v in out.items()}, indent=1))


if __name__ == "__main__":
    main()
