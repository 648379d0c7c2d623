#!/usr/bin/env python3
"""CPU-baseline calibration (SURVEY §8(d) CPU baseline (1)):
the oracle's per-pixel primary render (oracle/vrt_oracle.c) timed under two
schedulers on the same frames and the same cores --

  (a) the reference's own: render_mt's 64 tile tasks posted to a
      tp::ThreadPool built from the reference's thread_pool_cpp headers,
      included unmodified (oracle/pool_calib.cc -> oracle/_ref/libpoolcalib.so;
      a new pool per frame, hardware_concurrency workers, VRT/camera.h:42-68);
  (b) bench.py's cpu_baseline: the oracle's atomic-counter scheduler over
      min(nproc, 64) pthreads (ora_render_rows, vrt_oracle.c run_job).

ratio = (b)'s frame time / (a)'s, per pose and as the median; every frame of
(a) is checked bit for bit against (b)'s.  bench.py's cpu_baseline value x
ratio is the rate the reference's own scheduler reaches with this oracle on
the same cores.  Runs where /root/reference exists (the pool is built from
it); writes tests/golden/cpu_calibration.json.

    python3 tools/cpu_calibration.py [--width 1920 --height 1080 --depth 8 --poses 4 --reps 3]
"""
import argparse
import ctypes as C
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as po  # noqa: E402
import voxelraytrace20190722_amd as vrt  # noqa: E402

POOL_SO = os.path.join(ROOT, "oracle", "_ref", "libpoolcalib.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--poses", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3, help="interleaved timed runs per pose and scheduler")
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "cpu_calibration.json"))
    ap.add_argument("--box-workers", type=int, default=256,
                    help="the GPU box's hardware_concurrency (its pool's worker count; the box's bench runs the "
                         "oracle scheduler on min(that, 64) threads): the 'box-shaped' configuration")
    a = ap.parse_args()
    if not os.path.exists(POOL_SO):
        raise SystemExit(f"{POOL_SO} missing: `make -C oracle` where /root/reference exists")
    po.oracle()  # liboracle.so first: libpoolcalib.so resolves ora_render_tile to it
    L = C.CDLL(POOL_SO)
    L.pc_render_mt.restype = C.c_double
    L.pc_render_mt.argtypes = [C.c_void_p, po.f32p, C.c_float, C.c_float, C.c_int, C.c_int, C.c_int, po.f32p]
    L.pc_default_workers.restype = C.c_int
    workers = L.pc_default_workers()
    nproc = os.cpu_count() or 1
    nth = max(1, min(nproc, 64))
    sd = vrt.SceneData.proxy(1.0, 1)
    osc = po.Scene(sd, a.depth)
    info = osc.info()
    mn, mx = info[1][:3], info[1][3:]
    W, H = a.width, a.height
    rays = W * H * 4

    def measure(pool_workers, oracle_threads):
        rows = []
        for pi in range(a.poses):
            fov, eye, spot, up = vrt.sweep_pose(mn, mx, pi, 16)
            cam = po.camera(fov, eye, spot, up)
            pool_rgb = np.zeros((H, W, 3), np.float32)
            t_pool, t_sched = [], []
            # one warm-up each, then interleaved timed runs
            L.pc_render_mt(C.c_void_p(osc.h), po._p(cam, po.f32p), 1.0, 1.0, W, H, pool_workers,
                           po._p(pool_rgb, po.f32p))
            osc.render_rows(cam, 1.0, 1.0, W, H, 1, 0, oracle_threads)
            for _ in range(a.reps):
                t_pool.append(L.pc_render_mt(C.c_void_p(osc.h), po._p(cam, po.f32p), 1.0, 1.0, W, H, pool_workers,
                                             po._p(pool_rgb, po.f32p)))
                t0 = time.perf_counter()
                _, srgb = osc.render_rows(cam, 1.0, 1.0, W, H, 1, 0, oracle_threads)
                t_sched.append(time.perf_counter() - t0)
            same = bool(np.array_equal(pool_rgb.view(np.uint32), srgb.view(np.uint32)))
            if not same:
                raise SystemExit(f"pose {pi}: the pool-driven frame differs from the oracle scheduler's")
            tp_, ts_ = float(np.median(t_pool)), float(np.median(t_sched))
            rows.append({"pose": pi, "pool_s": round(tp_, 4), "oracle_sched_s": round(ts_, 4),
                         "ratio": round(ts_ / tp_, 4), "pool_runs_s": [round(x, 4) for x in t_pool],
                         "oracle_sched_runs_s": [round(x, 4) for x in t_sched], "bit_identical": same})
            print(json.dumps(rows[-1]), flush=True)
        return {"pool_workers": pool_workers or workers, "oracle_threads": oracle_threads,
                "calibration_ratio": round(float(np.median([r["ratio"] for r in rows])), 4),
                "pool_mrays_per_s": round(rays / np.median([r["pool_s"] for r in rows]) / 1e6, 3),
                "oracle_sched_mrays_per_s": round(rays / np.median([r["oracle_sched_s"] for r in rows]) / 1e6, 3),
                "per_pose": rows}

    native = measure(0, nth)
    box = measure(a.box_workers, max(1, min(a.box_workers, 64)))
    out = {
        "what": "oracle per-pixel primary render (vrt_oracle.c) under the reference's own thread_pool_cpp "
                "(render_mt: 64 tile tasks, a new pool per frame) vs under bench.py's cpu_baseline scheduler "
                "(atomic tile counter over min(hardware_concurrency, 64) pthreads), same frames, same cores",
        "calibration_ratio": box["calibration_ratio"],
        "ratio_def": "oracle-scheduler frame time / thread_pool_cpp frame time (median over poses of the "
                     "per-pose medians); > 1: the reference's pool renders the same frame faster; "
                     "calibration_ratio = the box-shaped configuration's",
        "native": native,
        "box_shaped": box,
        "box_shaped_def": f"the thread counts the GPU box uses: pool of {a.box_workers} workers (its "
                          f"hardware_concurrency) vs the oracle scheduler on {min(a.box_workers, 64)} threads, "
                          f"here on {nproc} CPUs",
        "nproc": nproc,
        "cpu_model": next((ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo")
                           if ln.startswith("model name")), platform.processor()),
        "config": {"width": W, "height": H, "max_depth": a.depth, "poses": a.poses, "reps": a.reps,
                   "scene": "sponza-proxy", "tris": sd.ntri},
        "script": "tools/cpu_calibration.py (run where /root/reference exists: the pool is compiled from it)",
    }
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({"calibration_ratio": out["calibration_ratio"],
                      **{k: {x: out[k][x] for x in ("pool_workers", "oracle_threads", "calibration_ratio",
                                                    "pool_mrays_per_s", "oracle_sched_mrays_per_s")}
                         for k in ("native", "box_shaped")}}), flush=True)


if __name__ == "__main__":
    main()
