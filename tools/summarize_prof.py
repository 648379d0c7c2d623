#!/usr/bin/env python3
"""Summarise a tools/prof.sh run (gpurun_out/prof_TAG) into profiles/:
  profiles/TAG_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/TAG_summary.json       per-dispatch means of every PMC counter for
                                  the render kernel + derived figures
(bench.py measures its roofline live with its own PMC passes; this tool
summarises the separate tools/prof.sh runs.)

FETCH_SIZE / WRITE_SIZE are KiB.  MI355X_MICROARCH.md §HBM: on gfx950
FETCH_SIZE reads 1/2 of the bytes of a wide coalesced stream; other access
widths are uncalibrated.  We report raw and x2-corrected reads and take the
corrected figure (an upper bound for this gather-style access) as `traffic`.
usage: summarize_prof.py TAG [--kernel k_render] [--key 1920x1080_d8_n1]
"""
import argparse
import collections
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--kernel", default="k_render<false, false>")
    ap.add_argument("--key", default="1920x1080_d8_n1")
    ap.add_argument("--src", default=None)
    a = ap.parse_args()
    src = a.src or os.path.join(ROOT, "gpurun_out", f"prof_{a.tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "trace_kernel_stats.csv"),
                os.path.join(dst, f"{a.tag}_kernel_stats.csv"))
    stats = {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "trace_kernel_stats.csv"))):
        if a.kernel in r["Name"]:
            stats = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                     "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
    ctr = collections.defaultdict(list)
    meta = {}
    for d in sorted(os.listdir(src)):
        f = os.path.join(src, d, f"{d}_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            if a.kernel in r["Kernel_Name"]:
                ctr[r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta = {"grid": int(r["Grid_Size"]), "wg": int(r["Workgroup_Size"]),
                        "lds": int(r["LDS_Block_Size"]), "vgpr": int(r["VGPR_Count"]),
                        "sgpr": int(r["SGPR_Count"]), "scratch": int(r["Scratch_Size"])}
    mean = {k: sum(v) / len(v) for k, v in ctr.items()}
    out = {"kernel": a.kernel, "trace": stats, "dispatch": meta, "pmc_mean_per_dispatch": mean}
    der = {}
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        rd_raw = mean["FETCH_SIZE"] * 1024
        wr = mean["WRITE_SIZE"] * 1024
        der["hbm_read_bytes_raw"] = rd_raw
        der["hbm_read_bytes_x2"] = 2 * rd_raw
        der["hbm_write_bytes"] = wr
        der["hbm_bytes_per_launch"] = 2 * rd_raw + wr
        if stats:
            der["hbm_GBps"] = der["hbm_bytes_per_launch"] / stats["avg_ns"]
    if "TCC_HIT_sum" in mean:
        h, m = mean["TCC_HIT_sum"], mean["TCC_MISS_sum"]
        der["l2_hit_rate"] = h / (h + m)
    if "GRBM_GUI_ACTIVE" in mean and stats:
        der["clock_GHz"] = mean["GRBM_GUI_ACTIVE"] / 8 / stats["avg_ns"]
    if "SQ_INSTS_VALU" in mean and stats and "clock_GHz" in der:
        wi_s = mean["SQ_INSTS_VALU"] / (stats["avg_ns"] * 1e-9)
        peak = 256 * 4 * der["clock_GHz"] * 1e9 / 2  # one wave64 VALU per 2 cycles per SIMD
        der["valu_wave_instr_per_s"] = wi_s
        der["valu_issue_frac"] = wi_s / peak
        der["valu_per_wave"] = mean["SQ_INSTS_VALU"] / mean.get("SQ_WAVES", 1)
    if "SQ_WAVE_CYCLES" in mean and "GRBM_GUI_ACTIVE" in mean:
        der["avg_waves_per_cu"] = 4 * mean["SQ_WAVE_CYCLES"] / (mean["GRBM_GUI_ACTIVE"] / 8) / 256
    out["derived"] = der
    json.dump(out, open(os.path.join(dst, f"{a.tag}_summary.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
