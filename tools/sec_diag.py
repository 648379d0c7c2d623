#!/usr/bin/env python3
"""Config-5 compaction diagnostic: one 1080p depth-8 secondary frame per
pose, the compaction queue counts of each (vrt_secondary_spill_counts) and
the frame time.  usage: tools/sec_diag.py [--poses 4] [--width 1920 --height 1080]"""
import argparse
import os
import sys
import time

import torch  # one HIP runtime: torch's

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraytrace20190722_amd as vrt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--poses", type=int, default=4)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--depth", type=int, default=8)
    a = ap.parse_args()
    sd = vrt.SceneData.proxy(1.0, 1)
    tree = vrt.VoxelOctree(sd, a.depth)
    mn, mx = tree.root_box
    film = vrt.Film(1, 1, a.width, a.height)
    dev = torch.device("cuda:0")
    prim = torch.zeros(a.width * a.height * 8, dtype=torch.float32, device=dev)
    vis = torch.zeros((a.height, a.width), dtype=torch.float32, device=dev)
    tot = []
    for i in range(a.poses):
        fov, eye, spot, up = vrt.sweep_pose(mn, mx, i, 16)
        cam = vrt.Camera(fov, eye, spot, up)
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tree.render_secondary_device(cam, film, 64, 0, 1, prim.data_ptr(), vis.data_ptr(), None)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
        st = tree.secondary_spill_stats()
        tot.append(st)
        print(f"pose {i}: {ms:.2f} ms, spill stats {st}", flush=True)
    n = len(tot)
    rec = sum(t["records"] for t in tot) / n
    fin = sum(t["finished_in_place"] for t in tot) / n
    print(f"mean per frame: {rec:.0f} records ({rec * tot[0]['record_bytes'] / 1e9:.3f} GB of records), "
          f"{fin:.0f} finished in place", flush=True)


if __name__ == "__main__":
    main()
