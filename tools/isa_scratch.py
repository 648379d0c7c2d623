#!/usr/bin/env python3
"""Where a kernel's scratch (register spill) accesses sit relative to its
loops, from `make isa`'s listing (build/obj/vrt_kernels.s).

A loop is a backward branch: `s_branch` / `s_cbranch_*` at line i to a label
at line j < i covers lines j..i.  Every scratch_load / scratch_store is
printed with the number of loops that contain it and the innermost loop's
size, so a spill store inside the DFS / leaf loops shows up as depth >= 2
(the persistent unit loop is depth 1).

    python3 tools/isa_scratch.py KERNEL_SYMBOL_PREFIX [build/obj/vrt_kernels.s]
"""
import re
import sys


def kernel_body(path, sym):
    out, on = [], False
    for ln in open(path):
        if not on and ln.startswith(sym) and ln.split(";")[0].rstrip().endswith(":"):
            on = True
        if on:
            out.append(ln.rstrip("\n"))
            if "s_endpgm" in ln:
                break
    return out


def main():
    sym = sys.argv[1]
    path = sys.argv[2] if len(sys.argv) > 2 else "build/obj/vrt_kernels.s"
    body = kernel_body(path, sym)
    if not body:
        raise SystemExit(f"{sym}: not found in {path}")
    labels = {}
    for i, ln in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", ln)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, ln in enumerate(body):
        m = re.search(r"\bs_(?:c)?branch\w*\s+(\.LBB\w+)", ln)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))
    n_ld = n_st = 0
    for i, ln in enumerate(body):
        m = re.search(r"\b(scratch_(load|store)_\w+)", ln)
        if not m:
            continue
        if m.group(2) == "load":
            n_ld += 1
        else:
            n_st += 1
        inside = [(a, b) for a, b in loops if a <= i <= b]
        inner = min((b - a for a, b in inside), default=0)
        print(f"line {i:6d}  {m.group(1):24s} loops {len(inside)}  innermost {inner} lines")
    print(f"{body[0]} {len(body)} lines, {len(loops)} loops, {n_st} scratch stores, {n_ld} scratch loads")


if __name__ == "__main__":
    main()
