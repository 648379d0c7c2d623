#!/usr/bin/env python3
"""Recompute a bench line's roofline from the files it was measured with:
the saved rocprofv3 PMC CSVs and kernel-trace stats (bench.py --pmc-save
DIR) and the bench's own JSON line (time basis, steps, build id).  Writes
DIR/summary.json with the per-frame counters of the measured kernel and the
re-derived roofline next to the one the bench printed; they must agree.

usage: tools/pmc_summary.py BENCH_JSON PMC_DIR
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    bj, d = sys.argv[1], sys.argv[2]
    line = json.loads([ln for ln in open(bj) if ln.startswith("{")][-1])
    r = line["roofline"]
    steps = line["steps"]
    per, nd, meta = bench.pmc_per_kernel(d, steps)
    stats = bench.kernel_stats(d)
    kern = bench.short_name(r["kernel"])
    mode = line["config"]["mode"]
    w8, h8 = line["config"]["width"] // 8 * 8, line["config"]["height"] // 8 * 8
    out_bytes = w8 * h8 * (4 if mode == "secondary" else 12)
    tb = r["time_basis"]
    # the profiled pass's own kernel time is not in the CSVs: take the clock
    # the bench reported to rebuild it
    m = per[kern]
    child_ms = m["GRBM_GUI_ACTIVE"] / 8 / (r["clock_ghz_profiled"] * 1e9) * 1e3
    pmc = {"per_kernel": per, "dispatch": meta, "kernel_stats": stats, "child_kernel_ms": child_ms}
    if "rocprof_ms_per_frame" in tb:  # trace / config 5: per-kernel rocprof time per frame
        t = tb["rocprof_ms_per_frame"]
        again = bench.roofline_from_pmc(pmc, kern, t, out_bytes, None, child_ms=child_ms)
    else:
        again = bench.roofline_from_pmc(pmc, kern, tb["single_launch_ms"], out_bytes,
                                        r.get("reference_equivalent_bytes_per_launch"),
                                        launch_ms=tb.get("launch_ms"), child_ms=child_ms)
    keys = ("achieved", "peak", "frac", "issue_frac_at_clock", "traffic", "l2_hit", "frac_fp64_weighted",
            "lane_utilisation", "valu_frac", "salu_frac")
    check = {k: (r.get(k), again.get(k)) for k in keys}
    check["hbm_frac"] = (r["hbm"]["frac"], again["hbm"]["frac"])
    check["bound_is_salu"] = (float(r["bound"] == "salu"), float(again["bound"] == "salu"))
    ok = all(abs((a or 0) - (b or 0)) <= 1e-3 * max(1.0, abs(a or 0)) for a, b in check.values())
    trace_avg = stats.get(kern, (None, None, None))[1]
    summ = {"bench_json": os.path.basename(bj), "build_id": line.get("build_id"), "kernel": meta[kern]["kernel"],
            "dispatch": meta[kern], "steps": steps, "time_basis": tb,
            "rocprof_kernel_trace_avg_ms": trace_avg,
            "pmc_per_frame": m, "bench_vs_recomputed": check, "agree": ok}
    json.dump(summ, open(os.path.join(d, "summary.json"), "w"), indent=1)
    print(json.dumps({"agree": ok, **{k: v for k, v in check.items()}}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
