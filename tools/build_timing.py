"""Host vs GPU octree build time on the sponza-proxy."""
import json
import sys
import time

import torch  # noqa: F401  (one HIP runtime)

sys.path.insert(0, ".")
import voxelraytrace20190722_amd as vrt  # noqa: E402

sd = vrt.SceneData.proxy(1.0, 1)
out = {}
for depth in (6, 8, 9, 10):
    row = {}
    for dev in (False, True):
        best = None
        for _ in range(3):
            t = time.perf_counter()
            tr = vrt.VoxelOctree(sd, depth, build_on_device=dev)
            wall = (time.perf_counter() - t) * 1e3
            rec = {"build_ms": round(tr.info.build_ms, 2), "gpu_ms": round(tr.info.build_device_ms, 2),
                   "create_ms": round(wall, 1), "nodes": tr.info.nodes, "refs": tr.info.tri_refs}
            tr.close()
            if best is None or rec["build_ms"] < best["build_ms"]:
                best = rec
        row["device" if dev else "host"] = best
    out[f"depth{depth}"] = row
    print(json.dumps({depth: row}), flush=True)
json.dump(out, open("gpurun_out/build_timing.json", "w"), indent=1)
