#!/usr/bin/env python3
"""Per-basic-block instruction mix of one kernel from `make isa`'s listing
(build/obj/vrt_kernels.s): for every block its loop (the compiler's
"in Loop: Header=BBx Depth=n" annotation) and its VALU / SALU / VMEM / LDS /
branch counts, then the totals per loop header.  Used for the instruction
budget of DESIGN §4.1 (which blocks a node visit, a pop and a leaf record
execute).

    python3 tools/isa_blocks.py KERNEL_SYMBOL [build/obj/vrt_kernels.s] [--blocks]
"""
import collections
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


def kind(op):
    if op.startswith(("v_mfma",)):
        return "mfma"
    if op.startswith("v_readlane") or op.startswith("v_readfirstlane") or op.startswith("v_writelane"):
        return "xlane"
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load", "s_store")):
        return "smem"
    if op.startswith("s_waitcnt") or op.startswith("s_nop"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other"


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    sym = args[0]
    path = args[1] if len(args) > 1 else "build/obj/vrt_kernels.s"
    body = kernel_body(path, sym)
    if not body:
        raise SystemExit(f"{sym}: not found in {path}")
    blocks = []  # (label, header, depth, Counter)
    cur = None
    for ln in body[1:]:
        m = re.match(r"^(\.LBB\w+|; %bb\.\d+):\s*(?:;\s*(.*))?$", ln.strip()) or \
            re.match(r"^(\.LBB\w+):\s*(?:;\s*(.*))?$", ln)
        if m:
            note = m.group(2) or ""
            h = re.search(r"Header=(\w+) Depth=(\d+)", note)
            hd = re.search(r"Loop Header: Depth=(\d+)", note)
            header = h.group(1) if h else (m.group(1).lstrip(".").replace("LBB", "BB") if hd else "-")
            depth = int(h.group(2)) if h else (int(hd.group(1)) if hd else 0)
            cur = [m.group(1).replace("; %", ""), header, depth, collections.Counter()]
            blocks.append(cur)
            continue
        t = ln.strip()
        if t.startswith(";") and cur is not None:
            hd = re.search(r"Loop Header: Depth=(\d+)", t)
            if hd:  # a loop header's own annotation follows its label
                cur[1] = cur[0].lstrip(".").replace("LBB", "BB")
                cur[2] = int(hd.group(1))
            continue
        if not t or t.startswith("."):
            continue
        op = t.split()[0]
        if cur is None:
            cur = ["entry", "-", 0, collections.Counter()]
            blocks.append(cur)
        cur[3][kind(op)] += 1
    cols = ("valu", "salu", "xlane", "vmem", "smem", "lds", "branch", "wait")
    if "--blocks" in sys.argv:
        print(f"{'block':14s} {'loop':10s} d " + " ".join(f"{c:>6s}" for c in cols))
        for lab, hdr, d, c in blocks:
            print(f"{lab:14s} {hdr:10s} {d} " + " ".join(f"{c[x]:6d}" for x in cols))
    per = collections.OrderedDict()
    for lab, hdr, d, c in blocks:
        k = (hdr, d)
        per.setdefault(k, collections.Counter()).update(c)
    print(f"{'loop header':14s} d " + " ".join(f"{c:>6s}" for c in cols))
    for (hdr, d), c in per.items():
        print(f"{hdr:14s} {d} " + " ".join(f"{c[x]:6d}" for x in cols))


if __name__ == "__main__":
    main()
