#!/usr/bin/env python3
"""Recompute a bench line's roofline from the files it was measured with:
the saved rocprofv3 PMC CSVs (bench.py --pmc-save DIR) and the bench's own
JSON line (kernel time, steps, build id).  Writes DIR/summary.json with the
per-dispatch counter means and the re-derived roofline next to the one the
bench printed; they must agree.

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
    kern = "k_secondary" if line["config"]["mode"] == "secondary" else "k_render"
    means, meta = bench.pmc_means(d, kern, line["steps"])
    rows = line["config"]["width"] // 8 * 8, line["config"]["height"] // 8 * 8
    out_bytes = rows[0] * rows[1] * (4 if kern == "k_secondary" else 12)
    # the profiled pass's own kernel time is not in the CSVs: take the clock
    # the bench reported to rebuild it
    child_ms = means["GRBM_GUI_ACTIVE"] / 8 / (r["clock_ghz_profiled"] * 1e9) * 1e3
    # the per-frame time the bench divided by (frame_ms; the launch span with
    # one frame in flight, older lines)
    frame_ms = line.get("frame_ms", line["kernel_ms_mean"])
    again = bench.roofline_from_pmc({"means": means, "child_kernel_ms": child_ms, "dispatch": meta},
                                    frame_ms, out_bytes, r.get("reference_equivalent_bytes_per_launch"))
    keys = ("achieved", "peak", "frac", "issue_frac_at_clock", "traffic", "l2_hit", "traffic_over_output")
    check = {k: (r.get(k), again.get(k)) for k in keys}
    check["hbm_frac"] = (r["hbm"]["frac"], again["hbm"]["frac"])
    ok = all(abs((a or 0) - (b or 0)) <= 1e-3 * max(1.0, abs(a or 0)) for a, b in check.values())
    summ = {"bench_json": os.path.basename(bj), "build_id": line.get("build_id"), "kernel": meta.get("kernel"),
            "dispatch": meta, "steps": line["steps"], "kernel_ms_mean": line["kernel_ms_mean"],
            "frame_ms": frame_ms,
            "pmc_mean_per_dispatch": means, "bench_vs_recomputed": check, "agree": ok}
    json.dump(summ, open(os.path.join(d, "summary.json"), "w"), indent=1)
    print(json.dumps({"agree": ok, **{k: v for k, v in check.items()}}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
