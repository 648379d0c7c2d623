"""The multi-rank frame through the HIP path (tests/test_dist.py checks the
same protocol with oracle-rendered ranks): two gloo ranks sharing cuda:0,
each rendering its share of the tile deal with vrt_render_tiles_device and
its config-5 pixels with vrt_render_secondary_device; rank 0 gathers the
packed tile buffers (gloo, host-staged) and re-assembles them on the device
with vrt_unpack_tiles_device; config 5's pixels take the same path with 1
float per pixel (vrt_pack_tiles_c_device / vrt_unpack_tiles_c_device) --
both bit-exact vs the oracle's single-process images."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import pyoracle as po
import voxelraytrace20190722_amd as vrt
from conftest import golden

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    z = golden("scene_soup.npz")
    sd = vrt.SceneData(z["pos"], z["nrm"], z["uv"], z["mat"], z["mat_tex"], z["mat_kd"], z["tex_dims"],
                       z["tex_off"], z["tex_data"])
    depth = int(z["depth"])
    c = z["cam0"]
    fov, eye, spot, up = float(c[0]), tuple(map(float, c[1:4])), tuple(map(float, c[4:7])), tuple(map(float, c[7:10]))
    cam = vrt.Camera(fov, eye, spot, up)
    nx, ny = 44, 36  # 5 x 4 tiles + a ragged border outside the tile grid
    film = vrt.Film(1, 1, nx, ny)
    dev = torch.device("cuda:0")
    tree = vrt.VoxelOctree(sd, depth, device=0)
    # primary: this rank's tiles on the device -> gather -> device unpack on rank 0
    nt = vrt.tiles_per_rank(film, world)
    buf = torch.zeros(nt * 192, dtype=torch.float32, device=dev)
    tree.render_tiles_device(cam, film, rank, world, 0, buf.data_ptr(), None)
    torch.cuda.synchronize()
    host = buf.cpu()
    gl = [torch.empty_like(host) for _ in range(world)] if rank == 0 else None
    dist.gather(host, gl, dst=0)
    # config 5: this rank's pixels (the rest of its image left as NaN), its
    # tiles packed on the device (1 float per pixel) -> gather -> device
    # unpack on rank 0, as the primary frame
    prim = torch.zeros(nx * ny * 8, dtype=torch.float32, device=dev)
    part = torch.full((ny, nx), float("nan"), dtype=torch.float32, device=dev)
    tree.render_secondary_device(cam, film, 4, rank, world, prim.data_ptr(), part.data_ptr(), None)
    sbuf = torch.zeros(nt * 64, dtype=torch.float32, device=dev)
    vrt.pack_tiles_c_device(film, rank, world, 1, part.data_ptr(), sbuf.data_ptr(), None)
    torch.cuda.synchronize()
    shost = sbuf.cpu()
    sgl = [torch.empty_like(shost) for _ in range(world)] if rank == 0 else None
    dist.gather(shost, sgl, dst=0)
    if rank == 0:
        g = torch.stack(gl).to(dev)
        img = torch.zeros((ny, nx, 3), dtype=torch.float32, device=dev)
        vrt.unpack_tiles_device(film, world, g.data_ptr(), img.data_ptr(), None)
        sg = torch.stack(sgl).to(dev)
        svis = torch.full((ny, nx), float("nan"), dtype=torch.float32, device=dev)
        vrt.unpack_tiles_c_device(film, world, 1, sg.data_ptr(), svis.data_ptr(), None)
        torch.cuda.synchronize()
        t = svis.cpu()
        osc = po.Scene(sd, depth)
        pcam = po.camera(fov, eye, spot, up)
        ref = osc.render(pcam, 1.0, 1.0, nx, ny, film_index=1, nthreads=2, samples=False)
        ref[8 * (ny // 8):] = 0
        ref[:, 8 * (nx // 8):] = 0
        vis, _ = osc.render_secondary(pcam, 1.0, 1.0, nx, ny, spp=4, nthreads=2, ids=False)
        res = {"primary": bool(np.array_equal(img.cpu().numpy().view(np.uint32), ref.view(np.uint32))),
               "secondary": bool(np.array_equal(t.numpy().view(np.uint32), vis.view(np.uint32)))}
        with open(os.path.join(outdir, "res.json"), "w") as f:
            json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


def test_frame_protocol_gloo_hip_ranks(tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    res = json.load(open(tmp_path / "res.json"))
    assert res == {"primary": True, "secondary": True}
