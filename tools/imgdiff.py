#!/usr/bin/env python3
"""Render every sweep pose with two libvrt.so builds into zeroed buffers and
report, per pose, how many pixels differ (bit-wise) and where.
usage: tools/imgdiff.py libA.so libB.so [--width 1920 --height 1080 --depth 8 --poses 16]"""
import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import voxelraytrace20190722_amd as vrt  # noqa: E402
from voxelraytrace20190722_amd import _ffi  # noqa: E402
from ab import load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs=2)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--poses", type=int, default=16)
    a = ap.parse_args()
    sd = vrt.SceneData.proxy(1.0, 1)
    film = _ffi.Film(1.0, 1.0, a.width, a.height)
    libs = [load(p) for p in a.libs]
    hs = []
    for L in libs:
        h = C.c_void_p()
        d = sd.desc()
        assert L.vrt_scene_create(C.byref(d), a.depth, 0, C.byref(h)) == 0
        hs.append(h)
    info = _ffi.SceneInfo()
    libs[0].vrt_scene_info(hs[0], C.byref(info))
    st = torch.cuda.current_stream()
    for i in range(a.poses):
        fov, eye, spot, up = vrt.sweep_pose(info.root_min[:], info.root_max[:], i, a.poses)
        cam = _ffi.Camera()
        libs[0].vrt_camera_init(fov, eye.ctypes.data_as(_ffi.f32p), spot.ctypes.data_as(_ffi.f32p),
                                up.ctypes.data_as(_ffi.f32p), 0.0, vrt.FLT_MAX, C.byref(cam))
        ims = []
        for L, h in zip(libs, hs):
            img = torch.full((a.height, a.width, 3), float("nan"), dtype=torch.float32, device="cuda")
            assert L.vrt_render_tiles_device(h, C.byref(cam), C.byref(film), 0, 1, 1, C.c_void_p(img.data_ptr()),
                                             C.c_void_p(st.cuda_stream)) == 0, L.vrt_last_error()
            torch.cuda.synchronize()
            ims.append(img.cpu().numpy().view(np.uint32))
        bad = np.any(ims[0] != ims[1], axis=2)
        nanA = np.isnan(ims[0].view(np.float32)).any(axis=2).sum()
        nanB = np.isnan(ims[1].view(np.float32)).any(axis=2).sum()
        ys, xs = np.nonzero(bad)
        print(f"pose {i}: {bad.sum()} pixels differ, unwritten A {nanA} B {nanB}",
              "" if not len(ys) else f"tiles {sorted(set(zip((ys // 8).tolist(), (xs // 8).tolist())))[:6]}")


if __name__ == "__main__":
    main()
