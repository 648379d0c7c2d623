#!/usr/bin/env python3
"""Benchmark: Mrays/s of the primary-ray hot path (camera ray generation +
voxel-octree ray march + Moller-Trumbore + primary shading + Film
accumulation) at 1920x1080 on the sponza-proxy, max_depth 8 ("256^3",
BASELINE.json configs[1]), over the 16-pose camera sweep.

One process per GPU.  A step = one 1920x1080 frame (4 samples / pixel) at
sweep pose (step % 16): each rank renders its share of the 8x8-pixel tiles
(tile t -> rank t % N), then one RCCL gather of the per-rank tile buffers to
rank 0, which re-assembles the image (scaling "strong": the frame is fixed).
Inputs (octree, triangles, textures) are resident in HBM before timing.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line on stdout; diagnostics go to stderr.
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch  # noqa: E402  (import torch before libvrt: one HIP runtime)
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import voxelraytrace20190722_amd as vrt  # noqa: E402

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=32)
    p.add_argument("--warmup", type=int, default=4)
    p.add_argument("--width", type=int, default=None, help="default 1920 (1024 for --mode trace)")
    p.add_argument("--height", type=int, default=None, help="default 1080 (1024 for --mode trace)")
    p.add_argument("--depth", type=int, default=None,
                   help="max_depth; default 8 = '256^3' (6 for --mode trace, as VRT/main.cc:67)")
    p.add_argument("--light-n", type=int, default=2048, help="light film side (--mode trace, VRT/main.cc:79)")
    p.add_argument("--detail", type=float, default=1.0, help="proxy tessellation (1.0 ~ 262k tris)")
    p.add_argument("--scene", default=os.environ.get("VRT_SCENE", ""),
                   help="OBJ file to render instead of the sponza-proxy (e.g. the real sponza.obj); "
                        "also read from $VRT_SCENE")
    p.add_argument("--poses", type=int, default=16)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-counters", action="store_true")
    p.add_argument("--mode", default="primary", choices=["primary", "secondary", "trace"],
                   help="primary: BASELINE configs 1-4 (4 spp primary render); secondary: config 5; "
                        "trace: the reference's full main() frame (light map + filter + cone tracing)")
    p.add_argument("--spp", type=int, default=64, help="secondary rays per hit pixel (--mode secondary)")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="nccl (RCCL over xGMI, the real path) or gloo (host-staged rehearsal)")
    p.add_argument("--save-image", default="", help="rank 0 writes the last frame as .hdr")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    a = p.parse_args()
    trace = a.mode == "trace"
    a.width = a.width or (1024 if trace else 1920)
    a.height = a.height or (1024 if trace else 1080)
    a.depth = a.depth or (6 if trace else 8)
    return a


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={a.gpus}; using WORLD_SIZE")
    local = local % max(1, torch.cuda.device_count())  # gloo rehearsal: ranks may share a GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    # ---- scene: built on the host, uploaded once (excluded from timing)
    t0 = time.time()
    if a.scene:
        sd = vrt.obj2voxel(a.scene)  # tinyobj-exact ingest
        scene_name = os.path.basename(a.scene)
    else:
        sd = vrt.SceneData.proxy(a.detail, 1)
        scene_name = "sponza-proxy"
    h = hashlib.sha256()
    for arr in (sd.pos, sd.nrm, sd.uv, sd.mat, sd.mat_tex, sd.mat_kd, sd.tex_dims, sd.tex_data):
        if arr is not None:
            h.update(np.ascontiguousarray(arr).tobytes())
    scene_hash = h.hexdigest()[:16]
    tree = vrt.VoxelOctree(sd, a.depth, device=local)
    info = tree.info
    log(f"[rank {rank}] scene {scene_name} ({scene_hash}): {sd.ntri} tris, depth {a.depth}: {info.nodes} nodes, "
        f"{info.nonempty_leaves} non-empty leaves, {info.tri_refs} refs, "
        f"{info.device_bytes / 2**20:.1f} MiB on device; build {info.build_ms:.0f} ms, "
        f"upload {info.upload_ms:.0f} ms ({time.time() - t0:.1f} s total)")
    mn, mx = tree.root_box
    cams = []
    for i in range(a.poses):
        fov, eye, spot, up = vrt.sweep_pose(mn, mx, i, a.poses)
        cams.append(vrt.Camera(fov, eye, spot, up))
    trace = a.mode == "trace"
    if trace:
        # VRT/main.cc:79-83 (light camera + film) and :108-112 (view camera)
        light_cam = vrt.Camera(vrt.to_radian(60), (1, 10, 1), (0, 0, 0), (0, 1, 0))
        light_film = vrt.Film(1, 1, a.light_n, a.light_n)
        cams = [vrt.Camera(vrt.to_radian(90), (1.0, 1.3, -0.2), (0.0, 0.4, 0.0), (0.0, 1.0, 0.0))]
        a.poses = 1
        res = tree.min_voxel(a.depth)
        light_ms = []
    film = vrt.Film(1.0, 1.0, a.width, a.height)
    W8, H8 = 8 * (a.width // 8), 8 * (a.height // 8)
    rays_per_frame = W8 * H8 * 4

    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    tpr = vrt.tiles_per_rank(film, world)
    secondary = a.mode == "secondary"
    img = torch.zeros((a.height, a.width) if secondary else (a.height, a.width, 3), dtype=torch.float32,
                      device=dev)
    if secondary:
        # config 5: rays per frame are data dependent (64 per primary hit):
        # count them per pose once, outside the timed region
        frame_rays = {}
        for pi in sorted({k % a.poses for k in range(a.steps)}):
            _, frame_rays[pi] = tree.render_secondary(cams[pi], film, spp=a.spp)
        prim = torch.zeros(W8 * H8 * 8, dtype=torch.float32, device=dev)
        visb = [torch.zeros((a.height, a.width), dtype=torch.float32, device=dev) for _ in range(2)]
    elif world > 1:
        # double-buffered: the RCCL gather of frame k (on the NCCL stream)
        # overlaps the render of frame k+1 (on the compute stream)
        tiles = [torch.zeros(tpr * 192, dtype=torch.float32, device=dev) for _ in range(2)]
        gathered = ([torch.zeros((world, tpr * 192), dtype=torch.float32, device=dev) for _ in range(2)]
                    if rank == 0 else None)
        gl = [list(g.unbind(0)) for g in gathered] if rank == 0 else [None, None]  # in-place views
    works = [None, None]
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(a.steps)]

    def finish(b):
        """Rank 0: re-assemble the frame gathered into buffer b."""
        if works[b] is None:
            return
        works[b].wait()  # stream-wait on the collective, no host block
        works[b] = None
        if rank == 0:
            if secondary:
                img.copy_(visb[b])
            else:
                vrt.unpack_tiles_device(film, world, gathered[b].data_ptr(), img.data_ptr(), sp)

    def step_secondary(k, timed):
        cam = cams[k % a.poses]
        if timed:
            ev[k][0].record(stream)
        if world == 1:
            tree.render_secondary_device(cam, film, a.spp, 0, 1, prim.data_ptr(), img.data_ptr(), sp)
            if timed:
                ev[k][1].record(stream)
            return
        b = k & 1
        finish(b)
        if rank == 0:
            visb[b].zero_()  # the previous reduce summed into rank 0's buffer
        # each rank writes only its own pixels (64-pixel chunks, round-robin);
        # the others stay +0.0, so a SUM reduce assembles the image exactly
        tree.render_secondary_device(cam, film, a.spp, rank, world, prim.data_ptr(), visb[b].data_ptr(), sp)
        if timed:
            ev[k][1].record(stream)
        finish(1 - b)
        if a.dist_backend == "nccl":
            works[b] = dist.reduce(visb[b], dst=0, op=dist.ReduceOp.SUM, async_op=True)
        else:
            host = visb[b].cpu()
            dist.reduce(host, dst=0, op=dist.ReduceOp.SUM)
            if rank == 0:
                img.copy_(host)

    def render(cam, rk, nr, layout, ptr_):
        if trace:
            tree.render_trace_device(cam, film, rk, nr, layout, ptr_, res, sp)
        else:
            tree.render_tiles_device(cam, film, rk, nr, layout, ptr_, sp)

    def step(k, timed):
        if secondary:
            return step_secondary(k, timed)
        cam = cams[k % a.poses]
        if trace:
            # light pass + filter (blocking, on the scene's own stream; every
            # rank builds the whole light map -- the final render is sharded)
            torch.cuda.current_stream(dev).synchronize()
            t0_ = time.perf_counter()
            tree.lightmap(light_cam, light_film)
            if timed:
                light_ms.append((time.perf_counter() - t0_) * 1e3)
        if timed:
            ev[k][0].record(stream)
        if world == 1:
            render(cam, 0, 1, 1, img.data_ptr())
            if timed:
                ev[k][1].record(stream)
            return
        b = k & 1
        finish(b)  # frame k-2 used this buffer pair
        render(cam, rank, world, 0, tiles[b].data_ptr())
        if timed:
            ev[k][1].record(stream)
        finish(1 - b)  # frame k-1: its gather overlapped this render
        if a.dist_backend == "nccl":
            works[b] = dist.gather(tiles[b], gl[b], dst=0, async_op=True)
        else:  # gloo rehearsal (several ranks on one GPU): host-staged gather
            host = tiles[b].cpu()
            hl = [torch.empty_like(host) for _ in range(world)] if rank == 0 else None
            dist.gather(host, hl, dst=0)
            if rank == 0:
                gathered[b].copy_(torch.stack(hl))
                vrt.unpack_tiles_device(film, world, gathered[b].data_ptr(), img.data_ptr(), sp)

    def drain():
        finish(0)
        finish(1)

    for k in range(a.warmup):
        step(k, False)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(a.steps):
        step(k, True)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if a.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kms = np.array([s.elapsed_time(e) for s, e in ev])  # render kernel, ms

    # ---- algorithmic bytes from the instrumented kernel's
    # reference-equivalent counters, per pose actually rendered
    roof = None
    if not a.no_counters and not secondary and not trace:
        poses_used = sorted({k % a.poses for k in range(a.steps)})
        b_rank = []
        cnt_tot = np.zeros(4)
        for pi in poses_used:
            _, so = tree.render(cams[pi], film, counters=True)
            c = so["counters"].reshape(a.height, a.width, 4, 4)
            # this rank's tiles only
            ty, tx = np.divmod(np.arange((a.width // 8) * (a.height // 8)), a.width // 8)
            mine = (np.arange(len(tx)) % world) == rank
            m = np.zeros((H8 // 8, W8 // 8), bool)
            m[ty[mine], tx[mine]] = True
            mask = np.repeat(np.repeat(m, 8, 0), 8, 1)
            cc = c[:H8, :W8][mask].reshape(-1, 4).astype(np.float64)
            s = cc.sum(0)
            cnt_tot += s
            npx = mask.sum()
            b_rank.append(28 * s[0] + 8 * s[1] + 40 * s[2] + 68 * s[3] + 12 * npx)
        pose_b = dict(zip(poses_used, b_rank))
        bytes_per_launch = np.mean([pose_b[k % a.poses] for k in range(a.steps)])
        achieved = bytes_per_launch / (kms.mean() * 1e-3) / 1e9
        traffic = None
        measured = None
        key = f"{a.width}x{a.height}_d{a.depth}_n{world}"
        try:
            traffic = json.load(open(a.traffic_json)).get(key)
        except Exception:
            pass
        try:
            # the bound the kernel actually hits (rocprofv3 PMC of this
            # workload, tools/summarize_prof.py): VALU issue, not HBM
            measured = json.load(open(os.path.join(os.path.dirname(a.traffic_json), "pmc_derived.json"))).get(key)
        except Exception:
            pass
        nr = cnt_tot[3] and (cnt_tot / (len(poses_used) * rays_per_frame / world))
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                "algorithmic_bytes_per_launch": round(float(bytes_per_launch)),
                "measured": measured,
                "per_ray": {"A": round(float(nr[0]), 2), "L": round(float(nr[1]), 2),
                            "T": round(float(nr[2]), 2), "H": round(float(nr[3]), 3)}}

    # ---- CPU baseline: the oracle (C restatement of the reference path,
    # render_mt-style 8x8 tiles over pthreads) on a bounded row sample
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu and trace:
        # one whole reference frame on the oracle: light pass (16 threads for
        # the marches, canonical-order sums), filter, cone-tracing render
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle as po
        osc = po.Scene(sd, a.depth)
        nth = max(1, min(a.cpu_threads, os.cpu_count() or 1))
        t0_ = time.perf_counter()
        osc.lightmap(po.camera(vrt.to_radian(60), (1, 10, 1), (0, 0, 0), (0, 1, 0)), 1.0, 1.0, a.light_n,
                     a.light_n, nthreads=nth)
        t1_ = time.perf_counter()
        # bounded: the cone-traced view at half width and height (same camera,
        # 1/4 of the samples), its time scaled x4 to the full film
        hw, hh = a.width // 2, a.height // 2
        osc.render_trace(po.camera(vrt.to_radian(90), (1.0, 1.3, -0.2), (0.0, 0.4, 0.0), (0.0, 1.0, 0.0)),
                         1.0, 1.0, hw, hh, res, nthreads=nth, samples=False)
        t2_ = time.perf_counter()
        tr = (t2_ - t1_) * (a.width * a.height) / (hw * hh)
        cpu = {"value": round(1.0 / ((t1_ - t0_) + tr), 5), "unit": "frames/s", "cores": nth, "kind": "port",
               "sample": f"light map {a.light_n}^2 x4 + filter ({t1_ - t0_:.1f} s) + cone-traced {hw}x{hh} x4 "
                         f"({t2_ - t1_:.1f} s, scaled x{(a.width * a.height) / (hw * hh):.0f} to "
                         f"{a.width}x{a.height}) by oracle/vrt_oracle.c over {nth} threads"}
        osc.close()
    if rank == 0 and world == 1 and not a.no_cpu and not secondary and not trace:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle as po
        osc = po.Scene(sd, a.depth)
        fov, eye, spot, up = vrt.sweep_pose(mn, mx, 0, a.poses)
        oc = po.camera(fov, eye, spot, up)
        nth = max(1, min(a.cpu_threads, os.cpu_count() or 1))
        # bounded sample: whole frames of the sweep (poses 0,1,..) until the
        # target CPU time is spent, at least one frame
        cpu_rays, sec, frames = 0, 0.0, 0
        while frames == 0 or (sec < a.cpu_seconds and frames < a.poses):
            fov, eye, spot, up = vrt.sweep_pose(mn, mx, frames % a.poses, a.poses)
            oc = po.camera(fov, eye, spot, up)
            s_, _ = osc.render_rows(oc, 1.0, 1.0, a.width, a.height, 1, 0, nth)
            sec += s_
            cpu_rays += rays_per_frame
            frames += 1
        cpu = {"value": round(cpu_rays / sec / 1e6, 4), "unit": "Mrays/s", "cores": nth, "kind": "port",
               "sample": f"{frames} full {a.width}x{a.height} x4 spp frames (sweep poses 0..{frames - 1}, "
                         f"{cpu_rays} rays, {sec:.1f} s) rendered by oracle/vrt_oracle.c with render_mt's "
                         f"8x8 tiles over {nth} threads"}
        osc.close()

    data_desc = (f"OBJ scene {a.scene} (tinyobj-exact ingest)" if a.scene else
                 "synthetic: deterministic sponza-proxy atrium (sponza.obj absent)")
    if rank == 0 and a.save_image:
        vrt.write_hdr(a.save_image, img.cpu().numpy())
    if rank == 0:
        coll = "rccl" if a.dist_backend == "nccl" else "gloo"
        n_side = int(round(2 ** a.depth))
        if trace:
            value = a.steps / elapsed
            out = {
                "metric": f"frames/s of the reference main() frame: light map {a.light_n}^2 x4 + filter + "
                          f"cone-traced {a.width}x{a.height} x4 (Sponza {int(round(2 ** a.depth))}^3 octree)",
                "value": round(value, 3), "unit": "frames/s", "n_gpus": world, "steps": a.steps,
                "warmup": a.warmup, "ms_per_step": round(elapsed * 1e3 / a.steps, 3),
                "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32+f64",
                "data": data_desc,
                "config": {"workload": f"full trace(): {scene_name} ({sd.ntri} tris), max_depth {a.depth}",
                           "scene_hash": scene_hash,
                           "mode": a.mode, "width": a.width, "height": a.height, "light_n": a.light_n,
                           "max_depth": a.depth, "tris": sd.ntri,
                           "parallelism": f"replicated light map, screen tiles x{world}"},
                "light_ms_mean": round(float(np.mean(light_ms)), 3),
                "trace_kernel_ms_mean": round(float(kms.mean()), 3),
                "roofline": None,
                "cpu_baseline": cpu,
            }
            print(json.dumps(out), flush=True)
            if world > 1:
                dist.destroy_process_group()
            return
        if secondary:
            per_step = [frame_rays[k % a.poses] for k in range(a.steps)]
            total_rays = int(sum(per_step))
            mean_rays = total_rays / a.steps
            metric = (f"Mrays/s at {a.width}x{a.height} Sponza {n_side}^3 octree "
                      f"(1 primary + {a.spp} stochastic secondary rays per hit pixel)")
            workload = (f"config 5: {a.width}x{a.height} primary hit + {a.spp} spp secondary rays, "
                        f"{scene_name} ({sd.ntri} tris), max_depth {a.depth}")
            par = f"pixel chunks x{world}" + (f" + {coll} sum-reduce" if world > 1 else "")
        else:
            total_rays = rays_per_frame * a.steps
            mean_rays = rays_per_frame
            metric = f"Mrays/s at {a.width}x{a.height} Sponza {n_side}^3 octree (primary rays, 4 spp)"
            workload = (f"primary render {a.width}x{a.height} x4 spp, {scene_name} ({sd.ntri} tris), "
                        f"max_depth {a.depth} (\"{n_side}^3\")")
            par = f"screen tiles x{world}" + (f" + {coll} gather" if world > 1 else "")
        value = total_rays / elapsed / 1e6
        out = {
            "metric": metric,
            "value": round(value, 2), "unit": "Mrays/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed * 1e3 / a.steps, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32+f64",
            "data": data_desc + ", 16-pose camera sweep",
            "config": {"workload": workload, "mode": a.mode, "scene_hash": scene_hash,
                       "width": a.width, "height": a.height, "max_depth": a.depth,
                       "rays_per_frame": int(round(mean_rays)), "tris": sd.ntri, "poses": a.poses,
                       "parallelism": par},
            "kernel_ms_mean": round(float(kms.mean()), 4),
            "kernel_mrays_per_s": round(mean_rays / world / (kms.mean() * 1e-3) / 1e6, 2),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
