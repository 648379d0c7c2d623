#!/usr/bin/env python3
"""Per-frame kernel timelines from a rocprofv3 `--kernel-trace` CSV: the
last N frames, a frame running from one launch of the anchor kernel to the
next, times in microseconds from the frame's anchor launch (negative: work
that started before it, e.g. the next frame's light pass beside the shading).

usage: tools/timeline.py KERNEL_TRACE_CSV OUT_JSON [--anchor k_cones_film] [--frames 3]
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("out")
    ap.add_argument("--anchor", default="k_cones_film")
    ap.add_argument("--frames", type=int, default=3)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda x: int(x["Start_Timestamp"]))
    idx = [i for i, x in enumerate(rows) if a.anchor in x["Kernel_Name"]]
    frames = []
    for f0, f1 in list(zip(idx, idx[1:]))[-a.frames:]:
        t0 = int(rows[f0]["Start_Timestamp"])
        frames.append([{"kernel": x["Kernel_Name"][:60], "queue": int(x["Queue_Id"]),
                        "start_us": round((int(x["Start_Timestamp"]) - t0) / 1e3, 1),
                        "end_us": round((int(x["End_Timestamp"]) - t0) / 1e3, 1)}
                       for x in rows[f0:f1 + 1]])
    json.dump(frames, open(a.out, "w"), indent=0)
    for fr in frames:
        print(f"frame: {len(fr)} kernels, anchor to next anchor {fr[-1]['start_us']:.1f} us")


if __name__ == "__main__":
    main()
