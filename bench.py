#!/usr/bin/env python3
"""Benchmark: Mrays/s of the primary-ray hot path (camera ray generation +
voxel-octree ray march + Moller-Trumbore + primary shading + Film
accumulation) at 1920x1080 on the sponza-proxy, max_depth 8 ("256^3",
BASELINE.json configs[1]), over the 16-pose camera sweep.

One process per GPU.  A step = one 1920x1080 frame (4 samples / pixel) at
sweep pose (step % 16): each rank renders its share of the 8x8-pixel tiles
(the tile deal of include/vrt.h: 4x4-tile blocks round-robin, rank 0 lighter
from 4 ranks on), then one RCCL gather of the per-rank tile buffers to rank
0, which re-assembles the image (scaling "strong": the frame is fixed).
Inputs (octree, triangles, textures) are resident in HBM before timing.

    python bench.py [--gpus N --steps K --warmup W]   (N > 1: spawns N rank processes)
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
N_CU = 256              # MI355X compute units (4 SIMD-32 each)
# VALU issue peak: one wave64 VALU instruction per 2 cycles per SIMD
# (MI355X_MICROARCH.md "Wave scheduling"), 4 SIMDs per CU
VALU_WAVE_INSTR_PER_CYCLE = N_CU * 4 / 2
MAX_CLOCK_GHZ = 2.4     # MI355X max engine clock (MI355X_MICROARCH.md chip table)
# SALU issue peak: one scalar unit per CU (MI355X_MICROARCH.md glossary,
# "CU"), one scalar instruction per cycle
SALU_INSTR_PER_CYCLE = N_CU * 1


CPU_NOTE = ("kind 'port': oracle/vrt_oracle.c, the C restatement of the reference path, scheduled as render_mt "
            "(64 tile tasks over min(hardware_concurrency, 64) threads taking tiles from an atomic counter); the "
            "reference's own per-pixel code (camera.cc, voxel_octree.cc) cannot be built here without stand-ins "
            "for headers libstdc++ 11 lacks (SURVEY §8(c), DESIGN §2), but its scheduler can: "
            "calibration_ratio = this scheduler's frame time / the reference's thread_pool_cpp's (compiled "
            "unmodified, driving the same oracle render, tools/cpu_calibration.py in the build container; "
            "the reference never travels to the GPU box), so value x ratio = the reference scheduler's rate")
CALIB_JSON = os.path.join(ROOT, "tests", "golden", "cpu_calibration.json")


def cpu_calibration():
    """The committed thread_pool_cpp calibration (tools/cpu_calibration.py):
    {calibration_ratio, ...} or None."""
    try:
        c = json.load(open(CALIB_JSON))
    except (OSError, ValueError):
        return None
    b = c.get("box_shaped", {})
    return {"calibration_ratio": c.get("calibration_ratio"),
            "calibration": {"source": "tests/golden/cpu_calibration.json (tools/cpu_calibration.py)",
                            "measured_on": f"{c.get('nproc')} CPUs of the build container ({c.get('cpu_model')})",
                            "config": c.get("config"),
                            "box_shaped": {k: b.get(k) for k in ("pool_workers", "oracle_threads", "calibration_ratio")},
                            "native": {k: c.get("native", {}).get(k) for k in ("pool_workers", "oracle_threads",
                                                                              "calibration_ratio")},
                            "ratio_def": c.get("ratio_def")}}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------
# Live rocprofv3 PMC passes over this same workload (rank 0, N=1): the
# roofline numbers come from counters of this run's code, not from files.
# One counter group per pass (MI355X_MICROARCH.md "rocprofv3 PMC slots":
# FETCH_SIZE and WRITE_SIZE never share a pass), no tracing combined.
# ---------------------------------------------------------------------------
PMC_PASSES = [  # (name, counters, optional)
    ("sq", ["SQ_INSTS_VALU", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_INSTS_VMEM_RD",
            "SQ_INSTS_LDS", "SQ_INSTS_SALU", "GRBM_GUI_ACTIVE"], False),
    ("fetch", ["FETCH_SIZE"], False),
    ("write", ["WRITE_SIZE"], False),
    ("tcc", ["TCC_HIT_sum", "TCC_MISS_sum"], False),
    # lane utilisation and the fp64 share of the VALU issue (fp64 add / mul /
    # fma issue at half the fp32 rate: each takes two issue slots)
    ("valu", ["SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
              "SQ_INSTS_VALU_TRANS_F64", "SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU"], True),
]
# helper kernels never counted as the measured kernel
HELPERS = ("k_render_defer", "k_primary1", "k_unpack", "k_unit_order")


def workload_args(a):
    out = ["--width", str(a.width), "--height", str(a.height), "--depth", str(a.depth),
           "--detail", str(a.detail), "--poses", str(a.poses), "--mode", a.mode, "--spp", str(a.spp),
           "--light-n", str(a.light_n)]
    if a.scene:
        out += ["--scene", a.scene]
    if a.rehearse_ranks > 1:
        out += ["--rehearse-ranks", str(a.rehearse_ranks)]
    return out


def short_name(kn):
    """'void vrt::k_render_p<true>(vrt::RenderParams)' -> 'k_render_p<true>'"""
    kn = kn.split("(")[0]
    return kn.split("::")[-1] if "vrt::" in kn else kn


def pmc_per_kernel(out_dir, steps):
    """Per-frame counter totals per kernel (short name) over the timed
    frames' dispatches in the rocprofv3 *counter_collection.csv files under
    out_dir (one file per pass), plus dispatches per frame and launch
    geometry.  The child runs warm-up 0, but a mode may launch a kernel
    before its timed region (config 5 renders each pose once to count its
    rays): of a kernel's n dispatches in a pass, the last
    floor(n / steps) * steps (dispatch ids are in launch order) are the
    timed frames' and the earlier ones are dropped."""
    import csv
    tot, disp, meta = {}, {}, {}
    for root, _, files in os.walk(out_dir):
        for f in files:
            if not f.endswith("counter_collection.csv"):
                continue
            by_k = {}
            for r in csv.DictReader(open(os.path.join(root, f))):
                kn = short_name(r["Kernel_Name"])
                by_k.setdefault(kn, []).append(r)
                meta[kn] = {"kernel": r["Kernel_Name"], "grid": int(r["Grid_Size"]), "wg": int(r["Workgroup_Size"]),
                            "lds": int(r["LDS_Block_Size"]),
                            # rocprofv3's VGPR_Count on gfx950 is half the allocated
                            # VGPRs (40 / 48 / 32 for the 80 / 96 / 64 the ISA
                            # reports for k_render_p / k_light / k_cones_film): both
                            "vgpr": 2 * int(r["VGPR_Count"]), "rocprof_vgpr_count": int(r["VGPR_Count"]),
                            "sgpr": int(r["SGPR_Count"]), "scratch": int(r["Scratch_Size"])}
            for kn, rows in by_k.items():
                ids = sorted({int(r["Dispatch_Id"]) for r in rows})
                keep = len(ids) // steps * steps if len(ids) >= steps else len(ids)
                kept = set(ids[len(ids) - keep:])
                t = tot.setdefault(kn, {})
                for r in rows:
                    if int(r["Dispatch_Id"]) in kept:
                        t[r["Counter_Name"]] = t.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                disp[kn] = keep / steps
    return ({k: {c: v / steps for c, v in t.items()} for k, t in tot.items()}, disp, meta)


def pmc_means(out_dir, kernel_prefix, steps):
    """Per-dispatch means of the counters of the one kernel whose short name
    starts with kernel_prefix (helpers excluded) -> (means, dispatch info)
    or (None, None)."""
    per, nd, meta = pmc_per_kernel(out_dir, steps)
    ks = [k for k in per if k.startswith(kernel_prefix) and not k.startswith(HELPERS)]
    if len(ks) != 1 or abs(nd[ks[0]] - 1.0) > 1e-9:
        return None, None
    return per[ks[0]], meta[ks[0]]


def kernel_stats(out_dir):
    """rocprofv3 --kernel-trace --stats summary -> {short name: (calls, avg ms, total ms)}."""
    import csv
    out = {}
    for root, _, files in os.walk(out_dir):
        for f in files:
            if f.endswith("kernel_stats.csv"):
                for r in csv.DictReader(open(os.path.join(root, f))):
                    out[short_name(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]) / 1e6,
                                                  float(r["TotalDurationNs"]) / 1e6)
    return out


def run_pmc(a, save_dir=""):
    """Run the timed region of this workload (warm-up 0, the same `steps`
    frames, so the same pose mix, one frame in flight) once per counter group
    under rocprofv3 --pmc, plus one --kernel-trace --stats pass, each in a
    child process (tracing never combined with counters).  Returns the
    per-frame counters per kernel, the kernel-trace summary and each pass's
    own kernel time, or None and the reason when a required pass fails."""
    import shutil
    import signal
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    tmp = tempfile.mkdtemp(prefix="vrt_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    child = [sys.executable, os.path.abspath(__file__), "--no-cpu", "--no-counters", "--no-pmc", "--no-d9",
             "--frames-in-flight", "1", "--frames-in-flight-secondary", "1", "--frames-in-flight-trace", "1",
             "--warmup", "0", "--steps",
             str(a.steps), *workload_args(a)]
    per, nd, meta, child_ms, skipped = {}, {}, {}, {}, []
    stats = None
    passes = [(n, ["--pmc", *c], opt) for n, c, opt in PMC_PASSES] + [("ktrace", ["--kernel-trace", "--stats"], False)]
    for name, popt, optional in passes:
        out_dir = os.path.join(tmp, name)
        cmd = [prof, *popt, "--output-format", "csv", "-d", out_dir, "-o", name, "--", *child]
        t0 = time.time()
        p = subprocess.Popen(cmd, cwd="/tmp", env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                             start_new_session=True, text=True)
        try:
            so, se = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.communicate()
            if optional:
                skipped.append(f"{name}: timed out")
                continue
            return None, f"pmc pass {name} timed out"
        if p.returncode != 0:
            why = f"pmc pass {name} rc={p.returncode}: {se.strip().splitlines()[-1:] if se else ''}"
            if optional:
                skipped.append(why)
                continue
            return None, why
        line = [ln for ln in so.splitlines() if ln.startswith("{")]
        if line:
            j = json.loads(line[-1])
            child_ms[name] = j.get("trace_kernel_ms_mean", j.get("kernel_ms_mean"))
        if name == "ktrace":
            stats = kernel_stats(out_dir)
        else:
            got, n_, m_ = pmc_per_kernel(out_dir, a.steps)
            for k, v in got.items():
                per.setdefault(k, {}).update(v)
            nd.update(n_)
            meta.update(m_)
        log(f"[pmc] pass {name}: {time.time() - t0:.1f} s")
        if save_dir:
            os.makedirs(save_dir, exist_ok=True)
            for root, _, files in os.walk(out_dir):
                for f in files:
                    if f.endswith(".csv") and "agent_info" not in f:
                        shutil.copy(os.path.join(root, f), os.path.join(save_dir, f"{name}_{f}"))
    shutil.rmtree(tmp, ignore_errors=True)
    # the clock comes from GRBM_GUI_ACTIVE of the "sq" pass over that pass's
    # own kernel time (profiled passes run at their own clock)
    return {"per_kernel": per, "per_frame_dispatches": nd, "dispatch": meta, "child_kernel_ms": child_ms.get("sq"),
            "kernel_stats": stats, "skipped": skipped}, None


def roofline_from_pmc(pmc, kernel, single_ms, out_bytes, ref_bytes, launch_ms=None, child_ms=None):
    """The measured roofline of one kernel (short name): VALU issue (the
    limiter) -- its VALU wave-instructions per frame
    (SQ_INSTS_VALU) over its time per frame alone on the GPU (single_ms: one
    frame in flight, HIP events in this process; rocprofv3's kernel-trace
    average of the same command is reported next to it), against the issue
    peak at the max engine clock -- and HBM traffic (FETCH_SIZE x2 per
    MI355X_MICROARCH.md §HBM + WRITE_SIZE; rocprofv3 reports KiB) over the
    same time as a fraction of the 8 TB/s peak.  Also: the fp64-weighted
    issue fraction (fp64 VALU ops take two issue slots), the lane
    utilisation of the VALU instructions, the issue fraction at the measured
    clock, and (launch_ms) the same with frames in flight."""
    m = pmc["per_kernel"][kernel]
    t = single_ms * 1e-3
    rd = 2 * m["FETCH_SIZE"] * 1024
    wr = m["WRITE_SIZE"] * 1024
    traffic = rd + wr
    cycles = m["GRBM_GUI_ACTIVE"] / 8                          # summed over the 8 XCDs
    cms = child_ms or pmc.get("child_kernel_ms") or single_ms
    clock = cycles / (cms * 1e-3) / 1e9                        # GHz in the profiled pass
    valu = m["SQ_INSTS_VALU"]
    achieved = valu / t / 1e9                                  # G wave-instr/s
    peak = VALU_WAVE_INSTR_PER_CYCLE * MAX_CLOCK_GHZ           # G wave-instr/s
    hbm = traffic / t / 1e9
    h, mi = m.get("TCC_HIT_sum", 0.0), m.get("TCC_MISS_sum", 0.0)
    f64 = [m.get(c) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                              "SQ_INSTS_VALU_TRANS_F64")]
    out = {
        "bound": "valu",
        "achieved": round(achieved, 1), "peak": round(peak, 1), "unit": "G wave-instr/s",
        "frac": round(achieved / peak, 4),
        "peak_def": f"{N_CU} CUs x 4 SIMDs x 1/2 wave64 VALU instr/cycle x {MAX_CLOCK_GHZ} GHz max clock",
        "valu_frac": round(achieved / peak, 4),
        "time_basis": {"single_launch_ms": round(single_ms, 4),
                       "note": "one frame in flight: the kernel alone on the GPU (HIP events on its stream)"},
        "issue_frac_at_clock": round(valu / (VALU_WAVE_INSTR_PER_CYCLE * cycles), 4),
        "clock_ghz_profiled": round(clock, 3),
        "valu_instr_per_launch": round(valu),
        "traffic": round(traffic),
        "hbm": {"achieved": round(hbm, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(hbm / PEAK_HBM_GBS, 4),
                "read_bytes": round(rd), "read_bytes_raw": round(rd / 2), "write_bytes": round(wr)},
        "traffic_over_output": round(traffic / out_bytes, 2),
        "l2_hit": round(h / (h + mi), 4) if h + mi > 0 else None,
        "valu_instr_per_wave": round(valu / max(1.0, m["SQ_WAVES"]), 1),
        "avg_waves_per_cu": round(4 * m["SQ_WAVE_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8) / N_CU, 2),
        "reference_equivalent_bytes_per_launch": ref_bytes,
        "kernel": pmc["dispatch"].get(kernel, {}).get("kernel"),
        "dispatch": pmc["dispatch"].get(kernel),
        "source": "live rocprofv3 --pmc passes of this bench command (counters per timed dispatch)",
    }
    if all(v is not None for v in f64):
        n64 = sum(f64)
        out["fp64_instr_per_launch"] = round(n64)
        out["frac_fp64_weighted"] = round((valu + n64) / t / 1e9 / peak, 4)
    if m.get("SQ_THREAD_CYCLES_VALU") and m.get("SQ_ACTIVE_INST_VALU"):
        lu = m["SQ_THREAD_CYCLES_VALU"] / (64.0 * m["SQ_ACTIVE_INST_VALU"])
        out["lane_utilisation"] = round(lu, 4)
        out["lane_util_def"] = "SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU)"
        out["frac_active_lanes"] = round(achieved / peak * lu, 4)
    ks = pmc.get("kernel_stats") or {}
    if kernel in ks:
        calls, avg, _ = ks[kernel]
        out["time_basis"]["rocprof_kernel_trace_avg_ms"] = round(avg, 4)
        out["time_basis"]["rocprof_calls"] = calls
    if launch_ms is not None and launch_ms != single_ms:
        out["time_basis"]["launch_ms"] = round(launch_ms, 4)
        out["time_basis"]["frac_at_launch_ms"] = round(valu / (launch_ms * 1e-3) / 1e9 / peak, 4)
    if m.get("SQ_INSTS_SALU") is not None:
        # the scalar pipe: one scalar unit per CU issues for all its waves, so
        # a kernel heavy in loop / exec-mask control can be bound there before
        # its VALU issue is; `bound` names the busier of the two pipes and the
        # top-level achieved / peak / frac are that pipe's
        salu = m["SQ_INSTS_SALU"]
        s_ach = salu / t / 1e9
        s_peak = SALU_INSTR_PER_CYCLE * MAX_CLOCK_GHZ
        out["salu_frac"] = round(s_ach / s_peak, 4)
        out["salu"] = {"achieved": round(s_ach, 1), "peak": round(s_peak, 1), "unit": "G instr/s",
                       "frac": round(s_ach / s_peak, 4), "instr_per_launch": round(salu),
                       "issue_frac_at_clock": round(salu / (SALU_INSTR_PER_CYCLE * cycles), 4),
                       "peak_def": f"{N_CU} CUs x 1 scalar unit x 1 SALU instr/cycle x {MAX_CLOCK_GHZ} GHz max clock"}
        out["valu"] = {"achieved": out["achieved"], "peak": out["peak"], "unit": "G wave-instr/s",
                       "frac": out["valu_frac"], "peak_def": out["peak_def"]}
        if out["salu_frac"] > out["valu_frac"]:
            out.update({"bound": "salu", "achieved": out["salu"]["achieved"], "peak": out["salu"]["peak"],
                        "unit": "G instr/s", "frac": out["salu_frac"], "peak_def": out["salu"]["peak_def"]})
    if pmc.get("skipped"):
        out["pmc_skipped"] = pmc["skipped"]
    return out


def cpu_info():
    """nproc, usable CPUs (affinity), the cgroup CPU quota and the model."""
    n = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = n
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except Exception:
        pass
    model = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return {"nproc": n, "affinity": aff, "cgroup_quota_cpus": quota, "model": model}


def eff_cores(nth, ci):
    """CPUs the CPU baseline can actually use: its threads, capped by the
    affinity mask and the job's cgroup CPU quota (16 on the GPU box, whose
    nproc is 256)."""
    q = ci["cgroup_quota_cpus"]
    return int(min(nth, ci["affinity"], q if q else nth))


def nccl_options():
    try:
        return dist.ProcessGroupNCCL.Options(is_high_priority_stream=True)
    except Exception:  # noqa: BLE001 -- an older torch: default streams
        return None


def ranks_seen(backend, dev):
    """ranks counted by an all_reduce over the process group"""
    t = torch.ones(1, dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(t)
    return int(t.item())


RANK_FIELDS = ("share_render_ms", "collective_ms", "unpack_ms", "elapsed_s")


def per_rank_report(world, backend, dev, rank, vals):
    """Every rank's diagnostic numbers (RANK_FIELDS) gathered to every rank
    (all_gather: each rank calls) -> the per-rank list rank 0 prints.  share:
    the mean render span of this rank's share (HIP events on its stream);
    collective: from the end of the render to the frame's gather / reduce
    being waited for on its stream (queued behind that stream's next render,
    so it includes that render); unpack: rank 0's re-assembly kernel (0
    elsewhere)."""
    t = torch.tensor([float(rank)] + [float(v) for v in vals], dtype=torch.float64,
                     device=dev if backend == "nccl" else "cpu")
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    rows = []
    for o in out:
        v = o.tolist()
        rows.append({"rank": int(v[0]), **{k: round(x, 4) for k, x in zip(RANK_FIELDS, v[1:])}})
    return rows


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
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="CPU-baseline workers; 0 = hardware_concurrency (os.cpu_count()), as the reference's "
                        "thread pool; at most 64 are ever busy (render_mt posts 64 tile tasks)")
    p.add_argument("--cpu-frames", type=int, default=5, help="CPU-baseline frames timed after 1 warm-up (>= 5)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-counters", action="store_true")
    p.add_argument("--no-pmc", action="store_true", help="skip the live rocprofv3 PMC passes (roofline)")
    p.add_argument("--pmc-save", default="", help="copy the PMC passes' CSVs into this directory")
    p.add_argument("--no-d9", action="store_true",
                   help="skip the max_depth+1 ('true N^3 leaves', SURVEY §8(a)) line of the primary bench")
    p.add_argument("--mode", default="primary", choices=["primary", "secondary", "trace"],
                   help="primary: BASELINE configs 1-4 (4 spp primary render); secondary: config 5; "
                        "trace: the reference's full main() frame (light map + filter + cone tracing)")
    p.add_argument("--spp", type=int, default=64, help="secondary rays per hit pixel (--mode secondary)")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="nccl (RCCL over xGMI, the real path) or gloo (host-staged rehearsal)")
    p.add_argument("--save-image", default="", help="rank 0 writes the last frame as .hdr")
    p.add_argument("--frames-in-flight", type=int, default=3,
                   help="consecutive frames on this many HIP streams (own output buffers), so a frame's "
                        "ramp-down overlaps the next frame's launch; 1 = one stream")
    p.add_argument("--rehearse-rank", type=int, default=-1,
                   help="with --rehearse-ranks: whose share to render (0: rank 0, which also gathers and "
                        "unpacks; from 4 ranks on the deal gives it fewer tiles than the others; -1 (default): "
                        "every rank's in turn, the reported step = the slowest rank's)")
    p.add_argument("--rehearse-repeats", type=int, default=3,
                   help="with --rehearse-ranks: timed runs per rank's share, interleaved over the ranks; a rank's "
                        "step is the median of its runs (all printed in rehearsal.per_rank)")
    p.add_argument("--rehearse-render-only", action="store_true",
                   help="with --rehearse-ranks: time the share's renders alone (no gather, no unpack)")
    p.add_argument("--frames-in-flight-trace", type=int, default=1,
                   help="frames in flight for --mode trace (the scene keeps two light-map / record sets, so a "
                        "frame's light pass can run beside the previous frame's cones; round 4: 1 / 2 in flight "
                        "160.7 / 156.1 frames/s)")
    p.add_argument("--frames-in-flight-secondary", type=int, default=1,
                   help="frames in flight for --mode secondary (round 4, streaming resume round: 1 / 2 / 3 in "
                        "flight 17.81 / 17.85 / 18.08 ms per frame)")
    p.add_argument("--rehearse-ranks", type=int, default=0,
                   help="single-GPU rehearsal of the N-rank path (WORLD_SIZE 1): render rank 0's share of the "
                        "tiles as one of R ranks, RCCL gather over a 1-rank process group, unpack of R rank "
                        "buffers -- the per-rank GPU and host cost of the multi-GPU step without the xGMI "
                        "transfer (reported as 'rehearsal', never as the N-GPU value)")
    p.add_argument("--abi-multi", action="store_true",
                   help="one process over every visible GPU through the library's own multi-device frame "
                        "(vrt_scene_create_multi + vrt_render_multi_device: scene per device, RCCL gather, "
                        "unpack on device 0) -- the C++ caller's render_mt replacement (primary mode)")
    p.add_argument("--abi-multi-virtual", type=int, default=0,
                   help="with --abi-multi on one GPU: N virtual ranks (VRT_TEST_VIRTUAL_RANKS: the N-rank "
                        "path with device copies in place of the gather), reported as a rehearsal")
    p.add_argument("--dry-run", action="store_true",
                   help="launcher check only: form the process group (gloo), count the ranks, print one line; "
                        "no GPU is used")
    a = p.parse_args()
    trace = a.mode == "trace"
    a.width = a.width or (1024 if trace else 1920)
    a.height = a.height or (1024 if trace else 1080)
    a.depth = a.depth or (6 if trace else 8)
    return a


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_ranks(n):
    """`bench.py --gpus N` started without a launcher (no WORLD_SIZE): run
    N rank processes of this same command line (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, one GPU each), as
    torch.distributed.run would, and exit with the worst exit code.  Called
    before anything touches the GPU; the ranks are child processes (no exec
    from this process)."""
    import signal
    import subprocess
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env,
                                      start_new_session=True))
    rc = 0
    try:
        for p in procs:
            rc = max(rc, abs(p.wait()))
            if rc:  # a failed rank: the others would wait for it in a collective
                for q in procs:
                    if q.poll() is None:
                        os.killpg(q.pid, signal.SIGTERM)
    finally:
        for q in procs:
            if q.poll() is None:
                os.killpg(q.pid, signal.SIGKILL)
    return rc


def abi_multi(a):
    """--abi-multi: the library's own multi-device frame in ONE process over
    every visible GPU (vrt_scene_create_multi: the octree built once and
    uploaded per device, one RCCL communicator; vrt_render_multi_device per
    frame: every device's share of the tile deal, ncclGather to device 0,
    unpack there) -- what a C++ caller of render_mt's replacement gets.  K
    frames of the sweep queued on one stream of device 0 (wall clock around
    them, then a sync); the last frame is compared bit for bit with the
    single-device render of the same pose.  --abi-multi-virtual N on one GPU:
    N virtual ranks (device copies in place of the gather), a rehearsal."""
    ndev = torch.cuda.device_count()
    virt = a.abi_multi_virtual if a.abi_multi_virtual > 1 else 0
    n = virt or ndev
    mask = 1 if virt else (1 << ndev) - 1
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    sd = vrt.obj2voxel(a.scene) if a.scene else vrt.SceneData.proxy(a.detail, 1)
    t0 = time.time()
    m = vrt.MultiOctree(sd, a.depth, device_mask=mask, virtual_ranks=virt or None)
    log(f"[abi-multi] {n} ranks on devices {m.devices}: scene replicated + communicator in {time.time() - t0:.1f} s")
    mn, mx = m.root_box
    cams = [vrt.Camera(*vrt.sweep_pose(mn, mx, i, a.poses)) for i in range(a.poses)]
    film = vrt.Film(1.0, 1.0, a.width, a.height)
    rays = 8 * (a.width // 8) * 8 * (a.height // 8) * 4
    st = torch.cuda.Stream(dev)
    imgs = [torch.zeros((a.height, a.width, 3), dtype=torch.float32, device=dev) for _ in range(2)]
    for k in range(a.warmup):
        m.render_device(cams[k % a.poses], film, imgs[k % 2].data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    t_start = time.perf_counter()
    for k in range(a.steps):
        ev[k][0].record(st)
        m.render_device(cams[k % a.poses], film, imgs[k % 2].data_ptr(), st.cuda_stream)
        ev[k][1].record(st)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    span = float(np.mean([x.elapsed_time(y) for x, y in ev]))
    last = (a.steps - 1) % a.poses
    tree = vrt.VoxelOctree(sd, a.depth, device=0)
    ref = torch.zeros_like(imgs[0])
    tree.render_tiles_device(cams[last], film, 0, 1, 1, ref.data_ptr(), None)
    torch.cuda.synchronize()
    same = bool(torch.equal(imgs[(a.steps - 1) % 2].view(torch.int32), ref.view(torch.int32)))
    tree.close()
    m.close()
    if not same:
        raise SystemExit("abi-multi: the multi-device frame differs from the single-device render")
    value = rays * a.steps / elapsed / 1e6
    out = {"metric": f"Mrays/s at {a.width}x{a.height} Sponza {int(round(2 ** a.depth))}^3 octree (primary rays, "
                     f"4 spp), in-library multi-device frame",
           "value": None if virt else round(value, 2), "unit": "Mrays/s", "n_gpus": 1 if virt else n,
           "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed * 1e3 / a.steps, 4),
           "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32+f64",
           "data": "synthetic: deterministic sponza-proxy atrium (sponza.obj absent), 16-pose camera sweep",
           "config": {"workload": f"primary render {a.width}x{a.height} x4 spp, max_depth {a.depth}",
                      "parallelism": (f"vrt_render_multi_device: {n} ranks, scene per device, "
                                      + ("device copies for the gather (VRT_TEST_VIRTUAL_RANKS rehearsal on one GPU)"
                                         if virt else "RCCL ncclGather to device 0 + unpack"))},
           "abi_multi": {"ranks": n, "devices": mask, "virtual": bool(virt), "call_span_ms_mean": round(span, 4),
                         "last_frame_bit_exact_vs_single_device": same},
           "build_id": vrt.build_id()}
    if virt:
        out["metric"] = "rehearsal: " + out["metric"]
        out["abi_multi"]["frames_per_s_one_gpu"] = round(a.steps / elapsed, 2)
    print(json.dumps(out), flush=True)


def main():
    a = parse()
    if a.abi_multi:
        if "WORLD_SIZE" in os.environ and os.environ["WORLD_SIZE"] != "1":
            raise SystemExit("--abi-multi runs in one process over every visible GPU (no launcher)")
        return abi_multi(a)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        # never fall back silently to one rank: N GPUs means N rank processes
        sys.exit(spawn_ranks(a.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus={a.gpus}: launch one rank per GPU "
                         f"(torch.distributed.run --nproc-per-node {a.gpus}, or bench.py --gpus {a.gpus} alone)")
    if a.dry_run:
        # launcher check without a GPU: the process group forms and every
        # rank is counted (gloo on the host)
        per_rank = None
        if world > 1:
            dist.init_process_group("gloo")
            seen = ranks_seen("gloo", None)
            per_rank = per_rank_report(world, "gloo", None, rank, [0.0] * len(RANK_FIELDS))
        else:
            seen = 1
        if rank == 0:
            line = {"dry_run": True, "n_gpus": a.gpus, "ranks_seen": seen}
            if per_rank:
                line["per_rank"] = per_rank
            print(json.dumps(line), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    local = local % max(1, torch.cuda.device_count())  # gloo rehearsal: ranks may share a GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    rehearse = world == 1 and a.rehearse_ranks > 1 and a.mode in ("primary", "secondary")
    if world > 1:
        if a.dist_backend == "nccl":
            # the collectives' stream at high priority: their kernels are
            # dispatched ahead of the next render's persistent workgroups
            dist.init_process_group("nccl", device_id=dev, pg_options=nccl_options())
        else:
            dist.init_process_group("gloo")
        assert dist.get_world_size() == a.gpus, (dist.get_world_size(), a.gpus)
    elif rehearse:
        # a 1-rank RCCL group: the gather below runs through RCCL exactly as
        # in the N-rank step (its payload stays on this GPU)
        dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev,
                                pg_options=nccl_options())
    # the number of tile shares the frame is dealt into
    nshare = a.rehearse_ranks if rehearse else world

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
    # frames in flight: frame k runs on streams[k % nfl] with its own output
    # buffers, so frame k+1's persistent grid fills the CUs while frame k's
    # last (latency-bound) units finish -- a launch's ramp-down is ~0.2 ms
    # whatever its size.  Every frame is still one full launch.
    nfl = 1 if a.dist_backend == "gloo" else max(1, a.frames_in_flight_trace if trace else a.frames_in_flight)
    if a.mode == "secondary" and a.frames_in_flight_secondary is not None:
        nfl = max(1, a.frames_in_flight_secondary)
    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(nfl - 1)]
    if a.mode == "primary":
        tree.set_frames_in_flight(nfl)  # half-chip persistent grids when frames overlap
    tpr = vrt.tiles_per_rank(film, nshare)
    secondary = a.mode == "secondary"
    img_shape = (a.height, a.width) if secondary else (a.height, a.width, 3)
    imgs = [torch.zeros(img_shape, dtype=torch.float32, device=dev) for _ in range(nfl)]
    img = imgs[0]
    # multi-rank buffers: two per frame in flight, so the render that reuses
    # frame k's buffer (frame k + nbuf, on frame k's stream) finds frame k's
    # collective long finished instead of waiting for it
    nbuf = max(2, 2 * nfl)
    if secondary:
        # config 5: rays per frame are data dependent (64 per primary hit):
        # count them per pose once, outside the timed region
        frame_rays = {}
        for pi in sorted({k % a.poses for k in range(a.steps)}):
            _, frame_rays[pi] = tree.render_secondary(cams[pi], film, spp=a.spp)
        prims = [torch.zeros(W8 * H8 * 8, dtype=torch.float32, device=dev) for _ in range(nbuf)]
        visb = [torch.zeros((a.height, a.width), dtype=torch.float32, device=dev) for _ in range(nbuf)]
        if nshare > 1:
            # each rank packs its tiles' pixels (1 float each) and one gather
            # brings them to rank 0, as the primary frame
            tiles = [torch.zeros(tpr * 64, dtype=torch.float32, device=dev) for _ in range(nbuf)]
            gathered = ([torch.zeros((nshare, tpr * 64), dtype=torch.float32, device=dev) for _ in range(nbuf)]
                        if rank == 0 else None)
            gl = [list(g[:world].unbind(0)) for g in gathered] if rank == 0 else [None] * nbuf
    elif nshare > 1:
        # the RCCL gather of frame k (on the NCCL stream) overlaps the render
        # of frame k+1
        tiles = [torch.zeros(tpr * 192, dtype=torch.float32, device=dev) for _ in range(nbuf)]
        gathered = ([torch.zeros((nshare, tpr * 192), dtype=torch.float32, device=dev) for _ in range(nbuf)]
                    if rank == 0 else None)
        # in-place views (a rehearsal's 1-rank group gathers into row 0 only)
        gl = [list(g[:world].unbind(0)) for g in gathered] if rank == 0 else [None] * nbuf
    works = [None] * nbuf
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(a.steps)]
    # N-rank diagnostics on every DIAG_EVERY-th timed frame (each event record
    # costs host time in a step of ~0.15 ms): the collective complete on the
    # stream that waits for it, and rank 0's unpack span
    DIAG_EVERY = 8
    frame_of = [None] * nbuf
    ev_coll = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    ev_unp = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.steps)]
    coll_done, unp_done = [], []
    torch.cuda.synchronize()  # buffers were zeroed on torch's stream; frames run on several

    def sl(k):
        """frame k's stream slot and buffer slot"""
        return k % nfl, k % nbuf

    def finish(b, s):
        """Frame in buffer b: its collective complete on stream s (a stream
        wait, no host block); rank 0 then re-assembles the frame there.  Called
        on the stream of frame k with the buffer of frame k - nfl (the same
        stream's previous frame), right after frame k's render is queued, so
        no render waits for a collective -- only for the re-assembly queued
        behind the previous render on its own stream (rank 0), and the buffer
        is reused (frame k - nfl + nbuf, same stream) after it."""
        if works[b] is None:
            return
        with torch.cuda.stream(s):
            works[b].wait()
        works[b] = None
        k = frame_of[b]
        frame_of[b] = None
        if k is not None:
            ev_coll[k].record(s)
            coll_done.append(k)
        # rank 0 re-assembles; a rehearsal of rank r >= 1's share does what
        # that rank does -- render + gather send, no unpack
        if rank == 0 and not (rehearse and cur["share"] != 0):
            if k is not None:
                ev_unp[k][0].record(s)
            if secondary:
                vrt.unpack_tiles_c_device(film, nshare, 1, gathered[b].data_ptr(), imgs[b % nfl].data_ptr(),
                                          s.cuda_stream)
            else:
                vrt.unpack_tiles_device(film, nshare, gathered[b].data_ptr(), imgs[b % nfl].data_ptr(),
                                        s.cuda_stream)
            if k is not None:
                ev_unp[k][1].record(s)
                unp_done.append(k)

    def step_secondary(k, timed):
        cam = cams[k % a.poses]
        j, b = sl(k)
        s = streams[j]
        if timed:
            ev[k][0].record(s)
        if nshare == 1:
            tree.render_secondary_device(cam, film, a.spp, 0, 1, prims[j].data_ptr(), imgs[j].data_ptr(),
                                         s.cuda_stream)
            if timed:
                ev[k][1].record(s)
            return
        finish(b, s)  # frame k - nbuf used these buffers (finished already, same stream)
        # this rank's pixels (its tiles of the deal), packed by tile
        tree.render_secondary_device(cam, film, a.spp, cur["share"], nshare, prims[b].data_ptr(),
                                     visb[b].data_ptr(), s.cuda_stream)
        vrt.pack_tiles_c_device(film, cur["share"], nshare, 1, visb[b].data_ptr(), tiles[b].data_ptr(),
                                s.cuda_stream)
        if timed:
            ev[k][1].record(s)
        if a.dist_backend == "nccl":
            with torch.cuda.stream(s):
                works[b] = dist.gather(tiles[b], gl[b], dst=0, async_op=True)
            frame_of[b] = k if (timed and k % DIAG_EVERY == 0) else None
            finish(sl(k - nfl)[1], s)  # this stream's previous frame: its gather overlapped this render
        else:  # gloo (several ranks on one GPU): host-staged gather
            host = tiles[b].cpu()
            hl = [torch.empty_like(host) for _ in range(world)] if rank == 0 else None
            dist.gather(host, hl, dst=0)
            if rank == 0:
                gathered[b].copy_(torch.stack(hl))
                vrt.unpack_tiles_c_device(film, world, 1, gathered[b].data_ptr(), img.data_ptr(), sp)

    def render(cam, rk, nr, layout, ptr_, s):
        if trace:
            # the whole main() frame: light map + filter beside the view's
            # primary march, then the cones (vrt_trace_frame_device)
            tree.trace_frame_device(light_cam, light_film, cam, film, rk, nr, layout, ptr_, res, s.cuda_stream)
        else:
            tree.render_tiles_device(cam, film, rk, nr, layout, ptr_, s.cuda_stream)

    def step(k, timed):
        if secondary:
            return step_secondary(k, timed)
        cam = cams[k % a.poses]
        j, b = sl(k)
        s = streams[j]
        if timed:
            ev[k][0].record(s)
        if nshare == 1:
            render(cam, 0, 1, 1, imgs[j].data_ptr(), s)
            if timed:
                ev[k][1].record(s)
            return
        finish(b, s)  # frame k - nbuf used this buffer pair (finished already, same stream)
        render(cam, cur["share"], nshare, 0, tiles[b].data_ptr(), s)
        if timed:
            ev[k][1].record(s)
        if rehearse and a.rehearse_render_only:
            pass  # diagnostic: the share's renders alone
        elif a.dist_backend == "nccl":
            # frame k's gather is queued as soon as its render is: the NCCL
            # stream waits for this render only, so its kernel is ready before
            # the next frame's render and runs beside it
            with torch.cuda.stream(s):
                works[b] = dist.gather(tiles[b], gl[b], dst=0, async_op=True)
            frame_of[b] = k if (timed and k % DIAG_EVERY == 0) else None
            finish(sl(k - nfl)[1], s)  # this stream's previous frame: its gather overlapped this render
        else:  # gloo rehearsal (several ranks on one GPU): host-staged gather
            host = tiles[b].cpu()
            hl = [torch.empty_like(host) for _ in range(world)] if rank == 0 else None
            dist.gather(host, hl, dst=0)
            if rank == 0:
                gathered[b].copy_(torch.stack(hl))
                vrt.unpack_tiles_device(film, world, gathered[b].data_ptr(), img.data_ptr(), sp)

    def drain():
        for b in range(nbuf):
            finish(b, stream)

    def timed_run():
        """W warm-up steps, then K timed steps between barrier + synchronize
        -> (max-over-ranks elapsed s, this rank's elapsed s, host enqueue s)"""
        coll_done.clear()
        unp_done.clear()
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
        # host time to enqueue the K steps: close to `elapsed` means the host
        # loop, not the GPU, sets the pace
        host_enq = time.perf_counter() - t_start
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t_start
        elapsed_local = elapsed
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev if a.dist_backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed, elapsed_local, host_enq

    # the share a step renders: this rank's, or in a rehearsal the rehearsed
    # rank's (--rehearse-rank -1: every rank's in turn, the step = the
    # slowest, as an N-GPU step waits for its slowest rank)
    cur = {"share": rank}
    reh_rows = []
    if rehearse:
        order = list(range(nshare)) if a.rehearse_rank < 0 else [a.rehearse_rank]
        # every rank's share timed --rehearse-repeats times, the repeats
        # interleaved over the ranks (a momentary slowdown of the box lands
        # on one repeat of one rank, not on one rank's only run); a rank's
        # step = the median of its repeats, all of them printed
        reps = {r_: [] for r_ in order}
        for rep_ in range(max(1, a.rehearse_repeats)):
            for r_ in order:
                cur["share"] = r_
                el_, ell_, he_ = timed_run()
                kms_ = np.array([s.elapsed_time(e) for s, e in ev])
                coll_ = float(np.mean([ev[k][1].elapsed_time(ev_coll[k]) for k in coll_done])) if coll_done else 0.0
                unp_ = float(np.mean([ev_unp[k][0].elapsed_time(ev_unp[k][1]) for k in unp_done])) if unp_done else 0.0
                reps[r_].append((el_, ell_, he_, kms_, coll_, unp_))
                log(f"[rehearsal] rank {r_}'s share, repeat {rep_}: {el_ * 1e3 / a.steps:.4f} ms per step")
        runs = []
        for r_ in order:
            rr = sorted(reps[r_], key=lambda x: x[0])
            el_, ell_, he_, kms_, coll_, unp_ = rr[(len(rr) - 1) // 2]  # the median run (lower median)
            runs.append((el_, ell_, he_, kms_, coll_, unp_))
            reh_rows.append({"share_of_rank": r_, "ms_per_step": round(el_ * 1e3 / a.steps, 4),
                             "repeats_ms_per_step": [round(x[0] * 1e3 / a.steps, 4) for x in reps[r_]],
                             "share_render_ms": round(float(kms_.mean()), 4), "collective_ms": round(coll_, 4),
                             "unpack_ms": round(unp_, 4), "host_enqueue_ms_per_step": round(he_ * 1e3 / a.steps, 4)})
        worst = max(range(len(runs)), key=lambda i: runs[i][0])
        elapsed, elapsed_local, host_enq, kms_w, _, _ = runs[worst]
        cur["share"] = order[worst]
        coll_w, unp_w = runs[worst][4], runs[worst][5]
    else:
        elapsed, elapsed_local, host_enq = timed_run()
    # render launch span (HIP events on its stream), ms
    kms = kms_w if rehearse else np.array([s.elapsed_time(e) for s, e in ev])
    if trace:  # the light map alone (blocking build), for reference beside the overlapped frame
        for _ in range(4):
            torch.cuda.synchronize()
            t0_ = time.perf_counter()
            tree.lightmap(light_cam, light_film)
            light_ms.append((time.perf_counter() - t0_) * 1e3)
    per_rank = None
    if world > 1 or (rehearse and not a.rehearse_render_only):
        if rehearse:
            coll_ms, unp_ms = coll_w, unp_w
        else:
            coll_ms = float(np.mean([ev[k][1].elapsed_time(ev_coll[k]) for k in coll_done])) if coll_done else 0.0
            unp_ms = float(np.mean([ev_unp[k][0].elapsed_time(ev_unp[k][1]) for k in unp_done])) if unp_done else 0.0
        vals = [float(kms.mean()), coll_ms, unp_ms, elapsed_local]
        if world > 1:
            per_rank = per_rank_report(world, a.dist_backend, dev, rank, vals)
            seen = ranks_seen(a.dist_backend, dev)
        else:
            per_rank = [{"rank": 0, "share_of_rank": cur["share"],
                         **{k_: round(v_, 4) for k_, v_ in zip(RANK_FIELDS, vals)}}]
    # the scene's device memory after the timed frames: octree + triangles +
    # textures, and the scratch it keeps between calls (config 5's
    # compaction queues among it)
    scr, spl = tree.scratch_bytes()
    dev_bytes = {"scene": int(info.device_bytes), "scratch": int(scr), "compaction_scratch": int(spl)}
    # per-frame device time: the launch span with one frame in flight; with
    # several, spans overlap (a span also holds the wait for the CUs the
    # previous frame still occupies), so the frame time is the step time
    frame_ms = float(kms.mean()) if nfl == 1 else elapsed * 1e3 / a.steps

    # ---- algorithmic bytes from the instrumented kernel's
    # reference-equivalent counters, per pose actually rendered
    # the "true N^3 leaves" depth (max_depth + 1, SURVEY §8(a) depth
    # convention): the same sweep timed on a second octree, reported in the
    # same line (N=1 primary bench only)
    d9 = None
    if world == 1 and not rehearse and not secondary and not trace and not a.no_d9:
        tree9 = vrt.VoxelOctree(sd, a.depth + 1, device=local)
        tree9.set_frames_in_flight(nfl)
        img9 = [torch.zeros_like(img) for _ in range(nfl)]
        for k in range(a.warmup):
            tree9.render_tiles_device(cams[k % a.poses], film, 0, 1, 1, img9[k % nfl].data_ptr(),
                                      streams[k % nfl].cuda_stream)
        ev9 = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(a.steps)]
        torch.cuda.synchronize()
        t9 = time.perf_counter()
        for k in range(a.steps):  # the same frames-in-flight schedule as the headline
            s9 = streams[k % nfl]
            ev9[k][0].record(s9)
            tree9.render_tiles_device(cams[k % a.poses], film, 0, 1, 1, img9[k % nfl].data_ptr(), s9.cuda_stream)
            ev9[k][1].record(s9)
        torch.cuda.synchronize()
        e9 = time.perf_counter() - t9
        k9 = np.mean([s.elapsed_time(e) for s, e in ev9])
        n_side9 = int(round(2 ** a.depth))
        d9 = {"max_depth": a.depth + 1,
              "convention": f"true {n_side9}^3 leaves (max_depth = log2 N + 1; the headline uses the author's "
                            f"max_depth = log2 N, VRT/main.cc:67-70)",
              "value": round(rays_per_frame * a.steps / e9 / 1e6, 2), "unit": "Mrays/s",
              "ms_per_step": round(e9 * 1e3 / a.steps, 4), "kernel_ms_mean": round(float(k9), 4),
              "nodes": tree9.info.nodes, "tri_refs": tree9.info.tri_refs}
        tree9.close()
        del img9

    # the host-buffer entry point (vrt_render: device image -> host array
    # over PCIe, per call); reported next to the HBM-resident value, never as it
    host_out = None
    if world == 1 and not rehearse and not secondary and not trace and not a.no_d9:
        n_h = min(a.steps, 16)
        hrgb = np.zeros((a.height, a.width, 3), np.float32)  # the caller's film, reused every frame
        tree.render(cams[0], film, out=hrgb)  # warm-up (first touch of the film's pages)
        th = time.perf_counter()
        for k in range(n_h):
            tree.render(cams[k % a.poses], film, out=hrgb)
        eh = (time.perf_counter() - th) / n_h
        host_out = {"ms_per_step": round(eh * 1e3, 4), "value": round(rays_per_frame / eh / 1e6, 2),
                    "unit": "Mrays/s", "frames": n_h,
                    "note": "vrt_render into the caller's host float RGB film, reused every frame (24.9 MB at 1080p over PCIe per frame): "
                            "4 tile-row bands on 2 streams, each copied D2H into pinned staging as it is "
                            "rendered, then to the caller's array by 4 host threads"}

    # one launch alone: the same frames with one frame in flight (the
    # roofline's time_basis; equal to frame_ms when nfl == 1)
    single_ms = frame_ms
    if world == 1 and not rehearse and not secondary and not trace and nfl > 1 and not a.no_pmc:
        tree.set_frames_in_flight(1)
        for k in range(2):
            render(cams[k % a.poses], 0, 1, 1, imgs[0].data_ptr(), stream)
        ev1 = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
        torch.cuda.synchronize()
        for k in range(a.steps):
            ev1[k][0].record(stream)
            render(cams[k % a.poses], 0, 1, 1, imgs[0].data_ptr(), stream)
            ev1[k][1].record(stream)
        torch.cuda.synchronize()
        single_ms = float(np.mean([s_.elapsed_time(e_) for s_, e_ in ev1]))
        tree.set_frames_in_flight(nfl)

    roof = None
    ref_bytes, per_ray = None, None
    if not a.no_counters and not rehearse and not secondary and not trace:
        poses_used = sorted({k % a.poses for k in range(a.steps)})
        b_rank, cnt_pose = [], {}
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
            cnt_pose[pi] = s
            npx = mask.sum()
            b_rank.append(28 * s[0] + 8 * s[1] + 40 * s[2] + 68 * s[3] + 12 * npx)
        pose_b = dict(zip(poses_used, b_rank))
        # SURVEY §8(d)'s per-ray model (28A + 8L + 40T + 68H + 12 B/pixel):
        # what the reference's data structure would move, not what this
        # design loads (child boxes are derived, never loaded) -- reported,
        # never divided by the HBM peak
        ref_bytes = round(float(np.mean([pose_b[k % a.poses] for k in range(a.steps)])))
        # per ray over the same timed frames (a pose counted as often as it
        # is rendered), so ref_bytes = the model applied to these counters
        nr = np.mean([cnt_pose[k % a.poses] for k in range(a.steps)], axis=0) / (rays_per_frame / world)
        per_ray = {"A": round(float(nr[0]), 2), "L": round(float(nr[1]), 2),
                   "T": round(float(nr[2]), 2), "H": round(float(nr[3]), 3)}
    trace_kernels = None
    if rank == 0 and world == 1 and not a.no_pmc:
        pmc, why = run_pmc(a, a.pmc_save)
        out_bytes = (W8 * H8 * 4) if secondary else (W8 * H8 * 12 // nshare)
        if pmc:
            pk = pmc["per_kernel"]
            ks = pmc.get("kernel_stats") or {}
            cand = [k for k in pk if not k.startswith(HELPERS) and "SQ_INSTS_VALU" in pk[k] and "FETCH_SIZE" in pk[k]
                    and "vrt::" in pmc["dispatch"].get(k, {}).get("kernel", "")]
            if trace or secondary:
                # the frame's kernels (trace: light pass, light map, render;
                # config 5: primary hits, the secondary walk and its resume
                # rounds), each against its own rocprof time; the line's
                # roofline = the one with the most VALU work per frame (kernel
                # time would pick the light pass of a trace frame, stretched
                # by the primary march it runs beside, not on the frame's
                # critical path)
                trace_kernels = {}
                for k in cand:
                    if k in ks:
                        calls, avg, tot = ks[k]
                        # the timed frames' dispatches of k per frame (the
                        # PMC pass counts them; config 5 also renders each
                        # pose once untimed for its ray count) x the
                        # kernel-trace average duration
                        per = pmc["per_frame_dispatches"].get(k) or calls / a.steps
                        fms = avg * per
                        r_ = roofline_from_pmc(pmc, k, fms, out_bytes, None, child_ms=fms)
                        r_["time_basis"] = {"rocprof_ms_per_frame": round(fms, 4),
                                            "dispatches_per_frame": round(per, 2),
                                            "rocprof_avg_ms": round(avg, 4), "rocprof_calls": calls,
                                            "note": "rocprofv3 kernel trace of this command (one frame in flight)"}
                        trace_kernels[k] = r_
                dom = max(trace_kernels, key=lambda k: trace_kernels[k]["valu_instr_per_launch"]
                          * trace_kernels[k]["time_basis"]["dispatches_per_frame"]) if trace_kernels else None
                roof = dict(trace_kernels[dom]) if dom else None
                if roof and trace:
                    roof["traffic_over_output"] = None  # the frame writes only the 1024^2 image
            else:
                dom = max(cand, key=lambda k: pk[k]["SQ_INSTS_VALU"]) if cand else None
                roof = roofline_from_pmc(pmc, dom, single_ms, out_bytes, ref_bytes,
                                         launch_ms=frame_ms) if dom else None
            if roof is None:
                why = f"no measured kernel among {sorted(pk)}"
            else:
                if per_ray:
                    roof["per_ray"] = per_ray
                roof["build_id"] = vrt.build_id()
        if not pmc or roof is None:
            log(f"[pmc] no roofline: {why}")
            roof = {"bound": "valu", "achieved": None, "peak": None, "unit": "G wave-instr/s", "frac": None,
                    "traffic": None, "unavailable": why, "reference_equivalent_bytes_per_launch": ref_bytes}

    # ---- CPU baseline: the oracle (C restatement of the reference path,
    # render_mt-style 8x8 tiles over pthreads) on a bounded row sample
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu and trace:
        # one whole reference frame on the oracle: light pass (16 threads for
        # the marches, canonical-order sums), filter, cone-tracing render
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle as po
        osc = po.Scene(sd, a.depth)
        ci = cpu_info()
        nth = max(1, min(a.cpu_threads or ci["nproc"], 64))  # as the primary baseline below
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
        cpu = {"value": round(1.0 / ((t1_ - t0_) + tr), 5), "unit": "frames/s", "cores": eff_cores(nth, ci), "threads": nth, "kind": "port", "note": CPU_NOTE,
               "nproc": ci["nproc"], "cgroup_quota_cpus": ci["cgroup_quota_cpus"], "cpu_model": ci["model"],
               "sample": f"light map {a.light_n}^2 x4 + filter ({t1_ - t0_:.1f} s) + cone-traced {hw}x{hh} x4 "
                         f"({t2_ - t1_:.1f} s, scaled x{(a.width * a.height) / (hw * hh):.0f} to "
                         f"{a.width}x{a.height}) by oracle/vrt_oracle.c over {nth} threads"}
        osc.close()
    if rank == 0 and world == 1 and not rehearse and not a.no_cpu and secondary:
        # config 5 on the oracle: render_secondary (primary hit + spp rays
        # per pixel, VRT/voxel_octree.cc:600-603 pattern) over min(nproc, 64)
        # threads, 1 warm-up + >= cpu_frames whole frames of the sweep; value
        # = rays traced / the median frame time; each frame's visibility
        # image checked bit for bit against the GPU's of the same pose
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle as po
        ci = cpu_info()
        osc = po.Scene(sd, a.depth)
        nth = max(1, min(a.cpu_threads or ci["nproc"], 64))

        def oframe(pi):
            fov, eye, spot, up = vrt.sweep_pose(mn, mx, pi, a.poses)
            t0_ = time.perf_counter()
            vis, nr = osc.render_secondary(po.camera(fov, eye, spot, up), 1.0, 1.0, a.width, a.height, spp=a.spp,
                                           nthreads=nth, ids=False)
            return time.perf_counter() - t0_, vis, nr

        warm_s, _, _ = oframe(0)
        times, rates, frames = [], [], 0
        gvis = torch.zeros((a.height, a.width), dtype=torch.float32, device=dev)
        gprim = torch.zeros(W8 * H8 * 8, dtype=torch.float32, device=dev)
        while frames < max(5, a.cpu_frames):
            pi = frames % a.poses
            s_, ovis, nr = oframe(pi)
            times.append(s_)
            rates.append(nr / s_)
            gvis.zero_()
            tree.render_secondary_device(cams[pi], film, a.spp, 0, 1, gprim.data_ptr(), gvis.data_ptr(), sp)
            torch.cuda.synchronize()
            if not np.array_equal(gvis.cpu().numpy().view(np.uint32), ovis.view(np.uint32)):
                raise SystemExit(f"GPU visibility image of pose {pi} differs from the CPU oracle frame")
            if nr != frame_rays.get(pi, nr):
                raise SystemExit(f"pose {pi}: oracle traced {nr} rays, the GPU count is {frame_rays[pi]}")
            frames += 1
        med = float(np.median(times))
        cpu = {"value": round(float(np.median(rates)) / 1e6, 4), "unit": "Mrays/s", "cores": eff_cores(nth, ci), "threads": nth, "kind": "port", "note": CPU_NOTE,
               "nproc": ci["nproc"], "affinity_cpus": ci["affinity"], "cgroup_quota_cpus": ci["cgroup_quota_cpus"],
               "cpu_model": ci["model"],
               "frame_s": {"warmup": round(warm_s, 3), "median": round(med, 3), "min": round(min(times), 3),
                           "max": round(max(times), 3)},
               "sample": f"1 warm-up + {frames} full {a.width}x{a.height} frames x (1 primary + {a.spp} secondary "
                         f"rays per hit pixel) (sweep poses 0..{frames - 1}, median rate), oracle/vrt_oracle.c "
                         f"render_secondary over {nth} threads; all {frames} visibility images bit-identical to "
                         f"the GPU's of the same pose"}
        osc.close()
    if rank == 0 and world == 1 and not rehearse and not a.no_cpu and not secondary and not trace:
        # The reference's scheduler: thread_pool_cpp with hardware_concurrency
        # workers (thread_pool_options.hpp:50-54) takes render_mt's 64 tile
        # tasks (VRT/camera.h:42-68), so min(nproc, 64) threads are ever
        # busy.  1 warm-up frame, then >= cpu_frames whole frames of the
        # sweep (more while the time budget lasts); value = rays per frame /
        # the median frame time.  Each frame is also checked bit for bit
        # against the GPU's image of the same pose.
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle as po
        ci = cpu_info()
        osc = po.Scene(sd, a.depth)
        nth = max(1, min(a.cpu_threads or ci["nproc"], 64))

        def oframe(pi):
            fov, eye, spot, up = vrt.sweep_pose(mn, mx, pi, a.poses)
            return osc.render_rows(po.camera(fov, eye, spot, up), 1.0, 1.0, a.width, a.height, 1, 0, nth)

        warm_s, _ = oframe(0)
        times, checked, frames = [], 0, 0
        gimg = torch.zeros_like(img)
        while frames < max(5, a.cpu_frames) or (sum(times) < a.cpu_seconds and frames < a.poses):
            pi = frames % a.poses
            s_, orgb = oframe(pi)
            times.append(s_)
            tree.render_tiles_device(cams[pi], film, 0, 1, 1, gimg.data_ptr(), sp)
            torch.cuda.synchronize()
            g = gimg.cpu().numpy()
            if not np.array_equal(g.view(np.uint32), orgb.view(np.uint32)):
                raise SystemExit(f"GPU image of pose {pi} differs from the CPU oracle frame")
            checked += 1
            frames += 1
        med = float(np.median(times))
        cpu = {"value": round(rays_per_frame / med / 1e6, 4), "unit": "Mrays/s", "cores": eff_cores(nth, ci), "threads": nth, "kind": "port", "note": CPU_NOTE,
               "nproc": ci["nproc"], "affinity_cpus": ci["affinity"], "cgroup_quota_cpus": ci["cgroup_quota_cpus"],
               "cpu_model": ci["model"],
               "frame_s": {"warmup": round(warm_s, 3), "median": round(med, 3), "min": round(min(times), 3),
                           "max": round(max(times), 3)},
               "sample": f"1 warm-up + {frames} full {a.width}x{a.height} x4 spp frames (sweep poses 0..{frames - 1},"
                         f" {rays_per_frame} rays each, median frame), oracle/vrt_oracle.c with render_mt's 64 "
                         f"tile tasks over {nth} threads (hardware_concurrency = {ci['nproc']}, capped at the 64 "
                         f"tasks); all {checked} frames bit-identical to the GPU image of the same pose"}
        cal = cpu_calibration()
        if cal and cal["calibration_ratio"]:
            cpu.update(cal)
            cpu["reference_scheduler_value"] = round(cpu["value"] * cal["calibration_ratio"], 4)
        osc.close()

    data_desc = (f"OBJ scene {a.scene} (tinyobj-exact ingest)" if a.scene else
                 "synthetic: deterministic sponza-proxy atrium (sponza.obj absent)")
    if rank == 0 and a.save_image:
        last = imgs[(a.steps - 1) % nfl] if nfl > 1 else img
        vrt.write_hdr(a.save_image, last.cpu().numpy())
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
                "frame_span_ms_mean": round(float(kms.mean()), 3),
                "note": "one vrt_trace_frame_device call per frame: light pass + sort + filter on the scene "
                        "stream beside the view's primary march on the frame stream, then the cone-traced "
                        "shading (every rank builds the whole light map; the render is sharded); "
                        "light_ms_mean = vrt_lightmap_build alone, measured separately",
                "roofline": roof,
                "roofline_per_kernel": trace_kernels,
                "cpu_baseline": cpu,
                "device_bytes": dev_bytes,
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
            par = f"pixel tiles x{world}" + (f" + {coll} gather" if world > 1 else "")
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
            "value": round(value, 2), "unit": "Mrays/s", "n_gpus": world, "ranks_seen": seen if world > 1 else 1,
            "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed * 1e3 / a.steps, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32+f64",
            "data": data_desc + ", 16-pose camera sweep",
            "config": {"workload": workload, "mode": a.mode, "scene_hash": scene_hash,
                       "width": a.width, "height": a.height, "max_depth": a.depth,
                       "rays_per_frame": int(round(mean_rays)), "tris": sd.ntri, "poses": a.poses,
                       "parallelism": par},
            "kernel_ms_mean": round(float(kms.mean()), 4),
            "frames_in_flight": nfl,
            "host_enqueue_ms_per_step": round(host_enq * 1e3 / a.steps, 4),
            "frame_ms": round(frame_ms, 4),
            "kernel_mrays_per_s": round(mean_rays / world / (frame_ms * 1e-3) / 1e6, 2),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if secondary and trace_kernels:
            out["roofline_per_kernel"] = trace_kernels
        out["device_bytes"] = dev_bytes
        if per_rank:
            out["per_rank"] = per_rank
        if d9:
            out["depth_plus1"] = d9
        if host_out:
            out["host_output"] = host_out
        if rehearse:
            # not an N-GPU measurement: one rank's share of every frame plus
            # the RCCL call sequence, on one GPU; the xGMI transfer is absent
            out["metric"] = "rehearsal: " + metric
            out["value"] = None
            who = "every rank's share in turn (step = the slowest)" if a.rehearse_rank < 0 else \
                f"rank {a.rehearse_rank}'s share"
            out["config"]["parallelism"] = (f"{who} of {nshare} screen-tile shares + "
                                            f"rccl gather (1-rank group)")
            out["rehearsal"] = {
                "ranks": nshare, "share_of_rank": cur["share"],
                "shares_rehearsed": [r_["share_of_rank"] for r_ in reh_rows],
                "step_is": ("max over the rehearsed ranks' steps" if len(reh_rows) > 1 else "the one rehearsed rank's step")
                + f" (each rank's step: the median of its {max(1, a.rehearse_repeats)} interleaved timed runs)",
                "per_rank": reh_rows,
                "frames_per_s": round(a.steps / elapsed, 2),
                "projected_Mrays_per_s_without_xgmi": round(value, 2),
                "share_kernel_ms_mean": round(float(kms.mean()), 4),
                "note": "per-rank step of the N-rank path on one GPU, each rank's share in turn doing what that rank "
                        "does: render of its tiles + RCCL gather (1-rank group: no xGMI transfer) + on rank 0 the "
                        "unpack of N rank buffers; a real N-GPU step adds the xGMI transfer into rank 0"}
            out["kernel_mrays_per_s"] = round(mean_rays / nshare / (frame_ms * 1e-3) / 1e6, 2)
        out["build_id"] = vrt.build_id()
        print(json.dumps(out), flush=True)
    if world > 1 or rehearse:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
