#!/usr/bin/env python3
"""A/B timing of libvrt.so build variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  Each variant library is loaded with
its own ctypes handle; every variant's image must be bit-identical to the
first one's (the baseline) or the run fails.

usage: tools/ab.py lib1.so lib2.so ... [--rounds 6] [--width 1920 --height 1080 --depth 8]
"""
import argparse
import ctypes as C
import json
import time
import os
import sys

import numpy as np
import torch  # one HIP runtime: torch's

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import voxelraytrace20190722_amd as vrt  # noqa: E402
from voxelraytrace20190722_amd import _ffi  # noqa: E402


def load(path):
    L = C.CDLL(os.path.abspath(path))
    for name, (res, args) in _ffi.SIGNATURES.items():
        if hasattr(L, name):
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--poses", type=int, default=16)
    ap.add_argument("--width", type=int, default=None, help="default 1920 (1024 for --mode trace)")
    ap.add_argument("--height", type=int, default=None, help="default 1080 (1024 for --mode trace)")
    ap.add_argument("--depth", type=int, default=None, help="default 8 (6 for --mode trace, as bench.py)")
    ap.add_argument("--detail", type=float, default=1.0)
    ap.add_argument("--mode", default="primary", choices=["primary", "secondary", "trace"])
    ap.add_argument("--light-n", type=int, default=2048, help="--mode trace: light film side (VRT/main.cc:79)")
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--no-check", action="store_true", help="timing-only variants (images may differ)")
    ap.add_argument("--ranks", type=int, default=1,
                    help="primary mode: time every rank's share of an N-rank frame separately (launch by launch; "
                         "per pose the slowest rank counts, as in an N-GPU step), images re-assembled with each "
                         "variant's own vrt_unpack_tiles_device for the parity check")
    ap.add_argument("--share-ranks", type=int, default=0,
                    help="primary mode: time rank shares of an N-rank frame as the rehearsal runs them -- K "
                         "frames of one rank's share with frames in flight (--fl streams), wall clock per step; "
                         "the variant's figure is the max over --share-of ranks (an N-GPU step waits for the "
                         "slowest rank)")
    ap.add_argument("--share-of", default="0,1", help="ranks whose shares --share-ranks times")
    ap.add_argument("--fl", type=int, default=3, help="--share-ranks: frames in flight")
    ap.add_argument("--steps", type=int, default=64, help="--share-ranks: frames per timed run")
    a = ap.parse_args()
    tr = a.mode == "trace"
    a.width = a.width or (1024 if tr else 1920)
    a.height = a.height or (1024 if tr else 1080)
    a.depth = a.depth or (6 if tr else 8)
    sd = vrt.SceneData.proxy(a.detail, 1)
    film = _ffi.Film(1.0, 1.0, a.width, a.height)
    libs = [load(p) for p in a.libs]
    scenes = []
    for L in libs:
        h = C.c_void_p()
        d = sd.desc()
        rc = L.vrt_scene_create(C.byref(d), a.depth, 0, C.byref(h))
        assert rc == 0, L.vrt_last_error()
        scenes.append(h)
    info = _ffi.SceneInfo()
    libs[0].vrt_scene_info(scenes[0], C.byref(info))
    if a.mode == "trace":
        return trace_ab(a, libs, scenes, film)
    cams = []
    for i in range(a.poses):
        fov, eye, spot, up = vrt.sweep_pose(info.root_min[:], info.root_max[:], i, a.poses)
        cam = _ffi.Camera()
        libs[0].vrt_camera_init(fov, eye.ctypes.data_as(_ffi.f32p), spot.ctypes.data_as(_ffi.f32p),
                                up.ctypes.data_as(_ffi.f32p), 0.0, vrt.FLT_MAX, C.byref(cam))
        cams.append(cam)
    if a.share_ranks >= 1:  # 1: the whole frame, frames in flight (the bench's schedule)
        return share_ab(a, libs, scenes, film, cams)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    sec = a.mode == "secondary"
    imgs = [torch.zeros((a.height, a.width) if sec else (a.height, a.width, 3), dtype=torch.float32, device=dev)
            for _ in libs]
    prim = torch.zeros(a.width * a.height * 8, dtype=torch.float32, device=dev)
    R = a.ranks if not sec else 1
    tprs = [L.vrt_tiles_per_rank(C.byref(film), R) for L in libs]
    packs = [torch.zeros((R, tpr * 192), dtype=torch.float32, device=dev) for tpr in tprs]
    times = {p: [] for p in a.libs}
    ref = None
    for r in range(a.rounds + 1):
        for vi, (L, h, p) in enumerate(zip(libs, scenes, a.libs)):
            evs = []
            for ci, cam in enumerate(cams):
                if R > 1:
                    pe = []
                    for rk in range(R):
                        e0 = torch.cuda.Event(enable_timing=True)
                        e1 = torch.cuda.Event(enable_timing=True)
                        e0.record(st)
                        rc = L.vrt_render_tiles_device(h, C.byref(cam), C.byref(film), rk, R, 0,
                                                       C.c_void_p(packs[vi][rk].data_ptr()),
                                                       C.c_void_p(st.cuda_stream))
                        assert rc == 0, L.vrt_last_error()
                        e1.record(st)
                        pe.append((e0, e1))
                    evs.append(pe)
                    if r == 0 and ci == a.poses - 1:
                        L.vrt_unpack_tiles_device(C.byref(film), R, C.c_void_p(packs[vi].data_ptr()),
                                                  C.c_void_p(imgs[vi].data_ptr()), C.c_void_p(st.cuda_stream))
                        torch.cuda.synchronize()
                        im = imgs[vi].cpu().numpy().view(np.uint32)
                        if ref is None:
                            ref = im
                        elif not a.no_check and not np.array_equal(im, ref):
                            raise SystemExit(f"variant {p} differs from baseline {a.libs[0]}")
                    continue
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(st)
                if sec:
                        rc = L.vrt_render_secondary_device(h, C.byref(cam), C.byref(film), a.spp, 0, 1,
                                                           C.c_void_p(prim.data_ptr()),
                                                           C.c_void_p(imgs[vi].data_ptr()),
                                                           C.c_void_p(st.cuda_stream))
                else:
                        rc = L.vrt_render_tiles_device(h, C.byref(cam), C.byref(film), 0, 1, 1,
                                                       C.c_void_p(imgs[vi].data_ptr()), C.c_void_p(st.cuda_stream))
                assert rc == 0, L.vrt_last_error()
                e1.record(st)
                evs.append((e0, e1))
                if r == 0 and ci == a.poses - 1:
                    torch.cuda.synchronize()
                    im = imgs[vi].cpu().numpy().view(np.uint32)
                    if ref is None:
                        ref = im
                    elif not a.no_check and not np.array_equal(im, ref):
                        raise SystemExit(f"variant {p} differs from baseline {a.libs[0]}")
            torch.cuda.synchronize()
            if r > 0 and R > 1:  # per pose the slowest rank's launch
                times[p].append(sum(max(s.elapsed_time(e) for s, e in pe) for pe in evs) / len(evs))
            elif r > 0:  # round 0 = warm-up + parity
                times[p].append(sum(s.elapsed_time(e) for s, e in evs) / len(evs))
    base = np.median(times[a.libs[0]])
    out = {}
    for p in a.libs:
        t = np.array(times[p])
        out[os.path.basename(p)] = {"median_ms": round(float(np.median(t)), 4), "min_ms": round(float(t.min()), 4),
                                    "speedup": round(float(base / np.median(t)), 3),
                                    "mrays": round(a.width * a.height * 4 / np.median(t) / 1e3, 1)}
    print(json.dumps(out, indent=1))


def share_ab(a, libs, scenes, film, cams):
    """--share-ranks R: per variant and round, K frames of rank r's share of
    an R-rank frame (the pose sweep, frames in flight on --fl streams, each
    frame its own packed buffer), wall clock around them; per rank the median
    over rounds, the variant's figure the max over the ranks.  Parity: every
    rank's share of the last pose re-assembled and compared with the first
    variant's image."""
    dev = torch.device("cuda:0")
    R, F = a.share_ranks, a.fl
    ranks = [int(x) for x in a.share_of.split(",")]
    streams = [torch.cuda.Stream(dev) for _ in range(F)]
    tpr = [L.vrt_tiles_per_rank(C.byref(film), R) for L in libs]
    packs = [torch.zeros((max(F, R), t * 192), dtype=torch.float32, device=dev) for t in tpr]
    img = torch.zeros((a.height, a.width, 3), dtype=torch.float32, device=dev)
    for L, h in zip(libs, scenes):
        assert L.vrt_scene_set_frames_in_flight(h, F) == 0, L.vrt_last_error()
    ref = None
    times = {p: {r: [] for r in ranks} for p in a.libs}
    for rd in range(a.rounds + 1):
        for vi, (L, h, p) in enumerate(zip(libs, scenes, a.libs)):
            if rd == 0:  # warm-up + parity: every rank's share of the last pose
                s0 = streams[0].cuda_stream
                for rk in range(R):
                    rc = L.vrt_render_tiles_device(h, C.byref(cams[-1]), C.byref(film), rk, R, 0,
                                                   C.c_void_p(packs[vi][rk].data_ptr()), C.c_void_p(s0))
                    assert rc == 0, L.vrt_last_error()
                L.vrt_unpack_tiles_device(C.byref(film), R, C.c_void_p(packs[vi].data_ptr()),
                                          C.c_void_p(img.data_ptr()), C.c_void_p(s0))
                torch.cuda.synchronize()
                im = img.cpu().numpy().view(np.uint32)
                if ref is None:
                    ref = im
                elif not a.no_check and not np.array_equal(im, ref):
                    raise SystemExit(f"variant {p} differs from baseline {a.libs[0]}")
                continue
            for rk in ranks:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for k in range(a.steps):
                    s = streams[k % F]
                    rc = L.vrt_render_tiles_device(h, C.byref(cams[k % len(cams)]), C.byref(film), rk, R, 0,
                                                   C.c_void_p(packs[vi][k % F].data_ptr()),
                                                   C.c_void_p(s.cuda_stream))
                    assert rc == 0, L.vrt_last_error()
                torch.cuda.synchronize()
                times[p][rk].append((time.perf_counter() - t0) * 1e3 / a.steps)
    out = {}
    base = None
    for p in a.libs:
        per = {r: float(np.median(times[p][r])) for r in ranks}
        mx = max(per.values())
        base = base or mx
        out[os.path.basename(p)] = {"max_step_ms": round(mx, 4), "speedup": round(base / mx, 3),
                                    "per_rank_ms": {r: round(v, 4) for r, v in per.items()}}
    print(json.dumps(out, indent=1))


def mkcam(L, fov, eye, spot, up):
    cam = _ffi.Camera()
    f3 = lambda v: np.ascontiguousarray(np.asarray(v, np.float32))  # noqa: E731
    e, s_, u = f3(eye), f3(spot), f3(up)
    L.vrt_camera_init(fov, e.ctypes.data_as(_ffi.f32p), s_.ctypes.data_as(_ffi.f32p), u.ctypes.data_as(_ffi.f32p),
                      0.0, vrt.FLT_MAX, C.byref(cam))
    return cam


def trace_ab(a, libs, scenes, film):
    """--mode trace: the reference main() frame's cone-traced render
    (vrt_render_trace_device, light map built once per variant), timed per
    launch; images must be bit-identical across variants."""
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    light = mkcam(libs[0], vrt.to_radian(60), (1, 10, 1), (0, 0, 0), (0, 1, 0))
    lfilm = _ffi.Film(1.0, 1.0, a.light_n, a.light_n)
    view = mkcam(libs[0], vrt.to_radian(90), (1.0, 1.3, -0.2), (0.0, 0.4, 0.0), (0.0, 1.0, 0.0))
    for L, h in zip(libs, scenes):
        hits = C.c_int64()
        assert L.vrt_lightmap_build(h, C.byref(light), C.byref(lfilm), C.byref(hits)) == 0, L.vrt_last_error()
    imgs = [torch.zeros((a.height, a.width, 3), dtype=torch.float32, device=dev) for _ in libs]
    times = {p: [] for p in a.libs}
    ltimes = {p: [] for p in a.libs}
    ftimes = {p: [] for p in a.libs}
    ref = None
    for r in range(a.rounds + 1):
        for vi, (L, h, p) in enumerate(zip(libs, scenes, a.libs)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            hits = C.c_int64()
            assert L.vrt_lightmap_build(h, C.byref(light), C.byref(lfilm), C.byref(hits)) == 0, L.vrt_last_error()
            torch.cuda.synchronize()
            if r > 0:
                ltimes[p].append((time.perf_counter() - t0) * 1e3)
            evs = []
            for _ in range(4):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(st)
                rc = L.vrt_render_trace_device(h, C.byref(view), C.byref(film), 0.0, 0, 1, 1,
                                               C.c_void_p(imgs[vi].data_ptr()), C.c_void_p(st.cuda_stream))
                assert rc == 0, L.vrt_last_error()
                e1.record(st)
                evs.append((e0, e1))
            torch.cuda.synchronize()
            if r == 0:
                im = imgs[vi].cpu().numpy().view(np.uint32)
                if ref is None:
                    ref = im
                elif not a.no_check and not np.array_equal(im, ref):
                    raise SystemExit(f"variant {p} differs from baseline {a.libs[0]}")
            else:
                times[p].append(sum(s_.elapsed_time(e_) for s_, e_ in evs) / len(evs))
            # the whole frame in one call (vrt_trace_frame_device), 4 frames
            if hasattr(L, "vrt_trace_frame_device"):
                t0 = time.perf_counter()
                for _ in range(4):
                    rc = L.vrt_trace_frame_device(h, C.byref(light), C.byref(lfilm), C.byref(view), C.byref(film),
                                                  0.0, 0, 1, 1, C.c_void_p(imgs[vi].data_ptr()),
                                                  C.c_void_p(st.cuda_stream), None)
                    assert rc == 0, L.vrt_last_error()
                torch.cuda.synchronize()
                if r > 0:
                    ftimes[p].append((time.perf_counter() - t0) * 1e3 / 4)
    base = np.median(times[a.libs[0]])
    fbase = np.median(ftimes[a.libs[0]]) if ftimes[a.libs[0]] else None
    lbase = np.median(ltimes[a.libs[0]])
    print(json.dumps({os.path.basename(p): {"median_ms": round(float(np.median(t)), 4),
                                            "min_ms": round(float(np.min(t)), 4),
                                            "speedup": round(float(base / np.median(t)), 3),
                                            "lightmap_wall_ms": round(float(np.median(ltimes[p])), 4),
                                            "lightmap_speedup": round(float(lbase / np.median(ltimes[p])), 3),
                                            "frame_wall_ms": (round(float(np.median(ftimes[p])), 4)
                                                              if ftimes[p] else None),
                                            "frame_speedup": (round(float(fbase / np.median(ftimes[p])), 3)
                                                              if ftimes[p] and fbase else None)}
                      for p, t in times.items()}, indent=1))


if __name__ == "__main__":
    main()
