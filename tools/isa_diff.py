#!/usr/bin/env python3
"""Compare the gfx950 code of every kernel in two `make isa` listings
(build/obj/vrt_kernels.s): per kernel symbol, its instruction stream with
basic-block numbering and comments normalised.  Used to show that a source
clean-up (dead compile-time alternatives removed) leaves the built kernels
unchanged.

usage: tools/isa_diff.py before.s after.s
"""
import re
import sys


def kernels(path):
    out, cur, name = {}, None, None
    for ln in open(path):
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            name, cur = m.group(1), []
            continue
        if name is None:
            continue
        if ln.startswith(".Lfunc_end"):
            out[name] = cur
            name, cur = None, None
            continue
        s = ln.split(";")[0].rstrip()
        if not s.strip() or s.strip().startswith(".loc") or s.strip().startswith(".file"):
            continue
        s = re.sub(r"\.LBB\d+_(\d+)", r".LBB_\1", s)
        s = re.sub(r"\.Ltmp\d+", ".Ltmp", s)
        cur.append(s)
    return out


def main():
    a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
    same, diff = [], []
    for k in sorted(set(a) | set(b)):
        if k not in a or k not in b:
            diff.append((k, "only in " + ("after" if k not in a else "before")))
        elif a[k] != b[k]:
            diff.append((k, f"{len(a[k])} vs {len(b[k])} lines"))
        else:
            same.append(k)
    print(f"{len(same)} kernels identical")
    for k, why in diff:
        print(f"DIFFERS {k}: {why}")
    return 1 if diff else 0


if __name__ == "__main__":
    sys.exit(main())
