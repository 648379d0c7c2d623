import sys, os, time
sys.path.insert(0, os.getcwd())
import torch
import numpy as np
import voxelraytrace20190722_amd as vrt
sd = vrt.SceneData.proxy(0.25, 2)
for depth in (7,):
    tree = vrt.VoxelOctree(sd, depth)
    print("scene ok", tree.info.nodes, flush=True)
    mn, mx = tree.root_box
    fov, eye, spot, up = vrt.sweep_pose(mn, mx, 9, 16)
    cam = vrt.Camera(fov, eye, spot, up)
    for ids in (False, True):
        for spp in (1, 64):
            t = time.time()
            vis, rays, *_ = tree.render_secondary(cam, vrt.Film(1, 1, 40, 24), spp=spp, ids=ids)
            print("secondary", depth, ids, spp, rays, round(time.time() - t, 3), flush=True)
