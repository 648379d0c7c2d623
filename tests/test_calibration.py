"""The CPU-baseline calibration against the reference's own scheduler
(tools/cpu_calibration.py): the committed fixture is
self-consistent, and -- where the reference exists and oracle/_ref was built
from it -- the oracle render driven by the reference's thread_pool_cpp
(render_mt's 64 tile tasks) equals the oracle scheduler's frame bit for bit."""
import ctypes as C
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as po  # noqa: E402
import voxelraytrace20190722_amd as vrt  # noqa: E402

CALIB = os.path.join(ROOT, "tests", "golden", "cpu_calibration.json")
POOL_SO = os.path.join(ROOT, "oracle", "_ref", "libpoolcalib.so")


@pytest.fixture(scope="module")
def proxy_small():
    return vrt.SceneData.proxy(0.25, 2)


def test_calibration_fixture_is_consistent():
    c = json.load(open(CALIB))
    for k in ("native", "box_shaped"):
        rows = c[k]["per_pose"]
        assert rows and all(r["bit_identical"] for r in rows)
        for r in rows:
            assert r["ratio"] == pytest.approx(r["oracle_sched_s"] / r["pool_s"], rel=2e-3)
        assert c[k]["calibration_ratio"] == pytest.approx(float(np.median([r["ratio"] for r in rows])), abs=1e-4)
    assert c["calibration_ratio"] == c["box_shaped"]["calibration_ratio"]
    assert c["box_shaped"]["pool_workers"] == 256 and c["box_shaped"]["oracle_threads"] == 64


@pytest.mark.skipif(not os.path.exists(POOL_SO), reason="oracle/_ref/libpoolcalib.so is built only where "
                                                        "/root/reference exists")
@pytest.mark.parametrize("workers", [0, 3, 80])
def test_reference_pool_drives_the_oracle_render_bit_exact(proxy_small, workers):
    po.oracle()
    L = C.CDLL(POOL_SO)
    L.pc_render_mt.restype = C.c_double
    L.pc_render_mt.argtypes = [C.c_void_p, po.f32p, C.c_float, C.c_float, C.c_int, C.c_int, C.c_int, po.f32p]
    osc = po.Scene(proxy_small, 5)
    mn, mx = osc.info()[1][:3], osc.info()[1][3:]
    fov, eye, spot, up = vrt.sweep_pose(mn, mx, 3, 16)
    cam = po.camera(fov, eye, spot, up)
    W, H = 72, 56
    rgb = np.zeros((H, W, 3), np.float32)
    assert L.pc_render_mt(C.c_void_p(osc.h), po._p(cam, po.f32p), 1.0, 1.0, W, H, workers, po._p(rgb, po.f32p)) > 0
    _, want = osc.render_rows(cam, 1.0, 1.0, W, H, 1, 0, 4)
    assert np.array_equal(rgb.view(np.uint32), want.view(np.uint32))
    assert rgb.any()
    osc.close()
