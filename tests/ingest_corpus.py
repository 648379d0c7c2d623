"""Deterministic OBJ / MTL / TGA inputs for the ingest parity tests
(SURVEY.md §8 rows f2, f4).  Every case targets a rule of tinyobjloader
v1.4.0 (VRT/tiny_obj_loader.h) or stb_image's TGA path (VRT/stb_image.h)
that decides output bits: the non-correctly-rounded float parser, ear
clipping, shape export / face dropping, material mapping, TGA variants.

write_obj_corpus(dir) / tga_corpus() are used by tests/test_ingest.py and
by tests/golden/make_golden.py (which records the reference's outputs)."""
import os
import struct

import numpy as np

# ----------------------------------------------------------------- numbers
FLOAT_SPELLINGS = [
    "0", "-0", "+0", "1", "-1", "+3.1417e+2", "-0.0E-3", "1.0324", "-1.41", "11e2", "1.", "1.e3",
    ".5", "-.5", "1e", "1e+", "abc", "1.5x", "--1", "+-1", "nan", "inf", "-inf", "0x1p3",
    "0.1", "0.2", "0.3", "0.7", "123456789.123456789", "0.000000001", "1e-7", "1e-38", "1e-45",
    "3.4028235e38", "3.5e38", "1e39", "1e-50", "7e-46", "0.12345678901234567890", "99999999.5",
    "16777217", "16777217.0", "1.00000005960464477539", "2.5e-1", "2.5E1", "000012.000", "-000.0001",
    "4.9406564584124654e-324", "1e308", "1e309", "1e-400", "12345678912345678912345",
    "0.30000001192092896", "1.17549435e-38", "1.1754942e-38", "6.103515625e-05", "1e22", "1e23",
    "8.589973e9", "-2.2250738585072014e-308", "5e-324", "1E0", "1e-0", "1e+00", "7.", "7.e",
]


def float_lines(rng, n=1500):
    """`v x y z` lines: numbers printed the ways exporters print them plus
    the edge spellings above (some of which tryParseDouble rejects)."""
    from decimal import Decimal
    out = []
    for i in range(n):
        k = i % 7
        if k == 6:
            # exact decimal of the midpoint of two adjacent floats: a correctly
            # rounded parser ties to even, tryParseDouble's last-bit error
            # often rounds the other way (double rounding)
            a = (rng.standard_normal(3) * 10 ** rng.uniform(-3, 3, 3)).astype(np.float32)
            b = np.nextafter(a, np.float32(np.inf), dtype=np.float32)
            xs = [str(Decimal(float(x)) / 2 + Decimal(float(y)) / 2) for x, y in zip(a, b)]
        elif k == 0:
            xs = [FLOAT_SPELLINGS[(i // 6 * 3 + j) % len(FLOAT_SPELLINGS)] for j in range(3)]
        elif k == 1:
            xs = ["%.9g" % x for x in rng.standard_normal(3) * 10 ** rng.uniform(-6, 6)]
        elif k == 2:
            xs = ["%.17g" % x for x in rng.standard_normal(3) * 10 ** rng.uniform(-30, 30)]
        elif k == 3:
            xs = ["%.6f" % x for x in rng.uniform(-50, 50, 3)]
        elif k == 4:
            xs = ["%.12e" % x for x in rng.standard_normal(3) * 10 ** rng.uniform(-300, 300)]
        else:
            d = rng.integers(1, 25, 3)
            xs = [("-" if rng.random() < 0.5 else "") + str(rng.integers(0, 10 ** 6)) + "." +
                  "".join(str(c) for c in rng.integers(0, 10, int(dd))) for dd in d]
        sep = [" ", "\t", "  ", " \t "][i % 4]
        out.append("v" + sep + sep.join(xs))
    return out


# ---------------------------------------------------------------- polygons
def polygon(rng, kind, n):
    """Planar polygon in a random 3D frame: convex, star (concave),
    self-intersecting, collinear runs, duplicate corners, tiny scale."""
    t = np.sort(rng.uniform(0, 2 * np.pi, n))
    if kind in ("convex", "dup"):
        r = np.ones(n)
    elif kind == "star":
        r = np.where(np.arange(n) % 2 == 0, 1.0, rng.uniform(0.2, 0.6))
    elif kind == "bowtie":
        t = rng.permutation(t)
        r = np.ones(n)
    elif kind == "collinear":
        r = np.ones(n)
        t[1:3] = t[0]
    else:  # tiny
        r = np.ones(n) * 1e-4
    p2 = np.stack([r * np.cos(t), r * np.sin(t)], 1)
    if kind == "collinear" and n >= 4:
        p2[1] = p2[0] * 0.6 + p2[3] * 0.4
        p2[2] = p2[0] * 0.3 + p2[3] * 0.7
    elif kind == "collinear":
        p2[2] = (p2[0] + p2[1]) * 0.5
    if kind == "dup":
        p2[2] = p2[1]
    q, _ = np.linalg.qr(rng.standard_normal((3, 3)))
    axis = rng.integers(0, 4)
    if axis < 3:  # axis-aligned planes hit the axis-choice branches exactly
        q = np.eye(3)[[axis, (axis + 1) % 3, (axis + 2) % 3]].T
    p3 = np.concatenate([p2, np.zeros((n, 1))], 1) @ q.T + rng.uniform(-5, 5, 3)
    return p3.astype(np.float32)


def _fmt(x):
    return "%.9g" % float(x)


def mesh_obj(rng, nfaces=400, with_normals=True, forms=("v/vt/vn", "v//vn")):
    """Geometry: polygons of all kinds, index forms and relative indices."""
    lines, nv, nvn, nvt = [], 0, 0, 0
    kinds = ["convex", "star", "bowtie", "collinear", "dup", "tiny"]
    for f in range(nfaces):
        kind = kinds[f % len(kinds)]
        n = 3 if f % 7 == 0 else int(rng.integers(4, 10))
        p = polygon(rng, kind, n)
        for q in p:
            lines.append("v " + " ".join(_fmt(x) for x in q))
        nrm = rng.standard_normal((n, 3)).astype(np.float32)
        for q in nrm:
            lines.append("vn " + " ".join(_fmt(x) for x in q))
        uv = rng.uniform(-1, 2, (n, 2)).astype(np.float32)
        for q in uv:
            lines.append("vt " + " ".join(_fmt(x) for x in q))
        rel = f % 3 == 1
        form = forms[f % len(forms)] if with_normals else "v/vt"
        corners = []
        for k in range(n):
            iv = (k - n) if rel else nv + k + 1
            ivn = (k - n) if rel else nvn + k + 1
            ivt = (k - n) if rel else nvt + k + 1
            corners.append({"v/vt/vn": f"{iv}/{ivt}/{ivn}", "v//vn": f"{iv}//{ivn}",
                            "v/vt": f"{iv}/{ivt}", "v": f"{iv}"}[form])
        lines.append("f " + " ".join(corners))
        nv, nvn, nvt = nv + n, nvn + n, nvt + n
    return lines


# ------------------------------------------------------------------- files
MTL_A = """# materials
newmtl red
Kd 0.8 0.1 0.1
map_Kd tex_a.tga

newmtl green   \t
\tKd 0.1 0.8 0.1
Ka 1 1 1
illum 2
map_Kd -bm 0.5 -s 1 2 3 -o 0.1 0.2 0.3 -clamp on -type sphere -imfchan r -mm 0 1 -colorspace srgb tex_b.tga

newmtl blue
Kd 0.1 0.1 0.8 0.5
map_Ka amb.tga
newmtl red
Kd 0.5 0.5 0.5
newmtl plain
Kd 0.25
newmtl spaced
Kd 1e-1 2E-1 +3e-1
map_Kd dir with space/tex c.tga
newmtl grey8
Kd 0.3 0.3 0.3
map_Kd sub\\tex_g.tga
"""

MTL_B = "newmtl from_b\r\nKd 0.9 0.9 0.1\r\nmap_Kd tex_a.tga\r\n"


def write_text(path, lines, nl="\n", final_newline=True):
    s = nl.join(lines) + (nl if final_newline else "")
    with open(path, "wb") as f:
        f.write(s.encode())


def write_obj_corpus(d, seed=17):
    """Writes the OBJ/MTL/TGA corpus into directory d; returns
    {name: (obj file, parse_only)} -- parse_only for files obj2voxel
    would reject (faces without normals / out-of-range indices)."""
    rng = np.random.default_rng(seed)
    os.makedirs(os.path.join(d, "sub"), exist_ok=True)
    os.makedirs(os.path.join(d, "dir with space"), exist_ok=True)
    with open(os.path.join(d, "a.mtl"), "w") as f:
        f.write(MTL_A)
    with open(os.path.join(d, "b.mtl"), "wb") as f:
        f.write(MTL_B.encode())
    # textures the materials name (decoded by the product like stbi_load)
    for name, w, h, c in [("tex_a.tga", 13, 7, 3), ("tex_b.tga", 8, 8, 4), ("dir with space/tex c.tga", 5, 9, 3),
                          ("sub/tex_g.tga", 6, 4, 1)]:
        px = rng.integers(0, 256, (h, w, c)).astype(np.uint8)
        with open(os.path.join(d, name), "wb") as f:
            f.write(tga_encode(px, rle=(c == 4), bottom_up=(w % 2 == 1)))
    cases = {}

    # 1. number spellings (positions only; a triangle fan referencing them)
    lines = ["# floats"] + float_lines(rng)
    lines += ["vn 0 0 1", "vt 0.5 0.5"]
    lines += [f"f {i}/1/1 {i + 1}/1/1 {i + 2}/1/1" for i in range(1, 1400, 3)]
    write_text(os.path.join(d, "floats.obj"), lines)
    cases["floats"] = ("floats.obj", False)

    # 2. polygons + materials + groups/objects, LF endings
    body = mesh_obj(rng, 420)
    fl = [i for i, ln in enumerate(body) if ln.startswith("f ")]
    out = ["mtllib missing.mtl a.mtl", "o first"]
    mats = ["red", "green", "blue", "plain", "spaced", "grey8", "nosuch", "red "]
    for j, i0 in enumerate(fl):
        start = fl[j - 1] + 1 if j else 0
        out += body[start:i0]
        if j % 9 == 0:
            out.append(f"usemtl {mats[(j // 9) % len(mats)]}")
        if j % 23 == 5:
            out.append(f"g grp{j} extra")
        if j % 31 == 7:
            out.append(f"o obj{j}")
        if j % 29 == 3:
            out += ["s 1", "l 1 2 3", "# comment", "", "   ", "s off"]
        out.append(body[i0])
    write_text(os.path.join(d, "polys.obj"), out)
    cases["polys"] = ("polys.obj", False)

    # 3. shape-export corner cases: usemtl then `o` with no new faces drops
    #    the shape; `g` without a name is ignored; lines keep a shape alive
    q = ["v 0 0 0", "v 1 0 0", "v 1 1 0", "v 0 1 0", "v 0.5 0.5 1", "vn 0 0 1", "vt 0 0"]
    tri = "f 1/1/1 2/1/1 3/1/1"
    quad = "f 1//1 2//1 3//1 4//1"
    lines = q + ["mtllib b.mtl a.mtl", "usemtl red", tri, "usemtl green", "o dropped", quad,
                 "usemtl blue", "g", tri, "usemtl from_b", "l 1 2", "usemtl red", "o kept_by_line", tri,
                 "g g1", "g g2", quad, "f 1//1 2//1", "usemtl plain", "o after_short", "f 5//1 4//1 3//1",
                 "usemtl red", "usemtl red", tri]
    write_text(os.path.join(d, "shapes.obj"), lines)
    cases["shapes"] = ("shapes.obj", False)

    # 4. CRLF / lone CR / tabs / no final newline / vertex colours
    lines = ["v 0 0 0 1 0 0", "v\t1\t0\t0", "v 1 1 0 0.5 0.5", "v 0 1 0", "vn 0 0 1", "vt 0.25 0.75 0.5",
             "mtllib a.mtl", "usemtl green", "f\t1/1/1\t2/1/1 3/1/1  4/1/1\t", "usemtl blue", "f -4/-1/-1 -2/-1/-1 -1/-1/-1"]
    with open(os.path.join(d, "endings.obj"), "wb") as f:
        f.write(("\r\n".join(lines[:5]) + "\r" + "\n".join(lines[5:])).encode())
    cases["endings"] = ("endings.obj", False)

    # 5. no mtllib at all: faces have material -1 (default material)
    lines = ["v 0 0 0", "v 2 0 0", "v 0 2 0", "v 2 2 1", "vn 0 0 1", "f 1//1 2//1 4//1 3//1"]
    write_text(os.path.join(d, "nomat.obj"), lines, final_newline=False)
    cases["nomat"] = ("nomat.obj", False)

    # 6. parse-only: faces without normals, forward references
    body = mesh_obj(rng, 60, with_normals=False)
    write_text(os.path.join(d, "nonormals.obj"), ["f 1 2 3 4 5", "f 2 3 4", "g early"] + body)
    cases["nonormals"] = ("nonormals.obj", True)
    return cases


# ---------------------------------------------------------------------- TGA
def tga_encode(px, rle=False, bottom_up=True, id_len=0):
    """Minimal true-colour / grey TGA writer (BGR(A) order) for test inputs."""
    h, w, c = px.shape
    grey = c in (1, 2)
    typ = (3 if grey else 2) + (8 if rle else 0)
    hdr = struct.pack("<BBBHHBHHHHBB", id_len, 0, typ, 0, 0, 0, 0, 0, w, h, 8 * c, 0 if bottom_up else 32)
    rows = px[::-1] if bottom_up else px
    data = rows.copy()
    if c >= 3:
        data[..., [0, 2]] = data[..., [2, 0]]
    flat = data.reshape(-1, c)
    if not rle:
        body = flat.tobytes()
    else:
        body = bytearray()
        i = 0
        while i < len(flat):
            j = i
            while j + 1 < len(flat) and j - i < 127 and np.array_equal(flat[j + 1], flat[i]):
                j += 1
            if j > i:
                body += bytes([0x80 | (j - i)]) + flat[i].tobytes()
                i = j + 1
            else:
                k = i
                while k + 1 < len(flat) and k - i < 127 and not np.array_equal(flat[k + 1], flat[k]):
                    k += 1
                body += bytes([k - i]) + flat[i:k + 1].tobytes()
                i = k + 1
        body = bytes(body)
    return hdr + b"I" * id_len + body


def _hdr(id_len, cmap, typ, pal_start, pal_len, pal_bits, w, h, bpp, desc):
    return struct.pack("<BBBHHBHHHHBB", id_len, cmap, typ, pal_start, pal_len, pal_bits, 0, 0, w, h, bpp, desc)


def _rle_stream(rng, npx, bpp_bytes, make_px):
    out = bytearray()
    left = npx
    while left > 0:
        n = int(min(left, rng.integers(1, 129)))
        if rng.random() < 0.5:
            out += bytes([0x80 | (n - 1)]) + make_px()
        else:
            out += bytes([n - 1]) + b"".join(make_px() for _ in range(n))
        left -= n
    return bytes(out)


def tga_corpus(seed=23):
    """[(name, bytes)]: every TGA layout stb accepts, plus rejects and
    truncated RLE / palette streams (stb reads zeros past EOF)."""
    rng = np.random.default_rng(seed)
    cases = []
    for c in (1, 2, 3, 4):
        for rle in (False, True):
            for bu in (False, True):
                h, w = int(rng.integers(1, 17)), int(rng.integers(1, 23))
                px = rng.integers(0, 256, (h, w, c)).astype(np.uint8)
                if rle:
                    px[:, : w // 2] = px[0, 0]
                cases.append((f"tc{c}_rle{int(rle)}_bu{int(bu)}", tga_encode(px, rle, bu, id_len=int(rng.integers(0, 4)))))
    # 8-bit true-colour image type (grey through type 2), 15/16-bit 5-5-5
    for typ, bpp in ((2, 8), (10, 8), (2, 15), (2, 16), (10, 16), (3, 16), (11, 16), (3, 24), (3, 32)):
        h, w = 5, 7
        npx = h * w
        bb = (bpp + 7) // 8
        for desc in (0, 32):
            if typ >= 8:
                body = _rle_stream(rng, npx, bb, lambda: rng.integers(0, 256, bb).astype(np.uint8).tobytes())
            else:
                body = rng.integers(0, 256, npx * bb).astype(np.uint8).tobytes()
            cases.append((f"t{typ}_b{bpp}_d{desc}", _hdr(0, 1 - 1, typ, 0, 0, 0, w, h, bpp, desc) + body))
    # colour-mapped: palette entry size x index size x RLE, palette offset
    for pal_bits in (8, 15, 16, 24, 32):
        for idx_bits in (8, 16):
            for typ in (1, 9):
                h, w, pal_len, pal_start = 6, 9, int(rng.integers(3, 40)), int(rng.integers(0, 3))
                eb = (pal_bits + 7) // 8
                pal = rng.integers(0, 256, pal_len * eb).astype(np.uint8).tobytes()
                ib = idx_bits // 8

                def one():  # some indices past the palette (stb maps them to 0)
                    k = int(rng.integers(0, pal_len + 3))
                    return k.to_bytes(ib, "little")
                npx = h * w
                body = _rle_stream(rng, npx, ib, one) if typ == 9 else b"".join(one() for _ in range(npx))
                desc = 32 if rng.random() < 0.5 else 0
                cases.append((f"cm{pal_bits}_i{idx_bits}_t{typ}",
                              _hdr(2, 1, typ, pal_start, pal_len, pal_bits, w, h, idx_bits, desc) + b"ID" +
                              b"\0" * pal_start + pal + body))
    # truncated streams (RLE and palette-indexed read zeros past the end)
    full = tga_encode(rng.integers(0, 256, (8, 8, 3)).astype(np.uint8), rle=True, bottom_up=True)
    cases.append(("rle_truncated", full[: len(full) * 2 // 3]))
    cases.append(("header_only_rle", _hdr(0, 0, 10, 0, 0, 0, 4, 4, 24, 0)))
    cases.append(("cm_no_indices", _hdr(0, 1, 1, 0, 4, 24, 3, 3, 8, 0) + bytes(range(12))))
    # rejects: stb's tga_test says no -> stbi_load fails
    for name, hdr in [("bad_cmap2", _hdr(0, 2, 2, 0, 0, 0, 4, 4, 24, 0)),
                      ("bad_type4", _hdr(0, 0, 4, 0, 0, 0, 4, 4, 24, 0)),
                      ("bad_bpp12", _hdr(0, 0, 2, 0, 0, 0, 4, 4, 12, 0)),
                      ("bad_w0", _hdr(0, 0, 2, 0, 0, 0, 0, 4, 24, 0)),
                      ("bad_h0", _hdr(0, 0, 2, 0, 0, 0, 4, 0, 24, 0)),
                      ("bad_cm_type2", _hdr(0, 1, 2, 0, 4, 24, 4, 4, 8, 0)),
                      ("bad_cm_idx24", _hdr(0, 1, 1, 0, 4, 24, 4, 4, 24, 0)),
                      ("bad_cm_pal12", _hdr(0, 1, 1, 0, 4, 12, 4, 4, 8, 0)),
                      ("cm_short_palette", _hdr(0, 1, 1, 0, 200, 24, 4, 4, 8, 0) + bytes(30)),
                      ("empty", b""), ("short", b"\0\0\2")]:
        cases.append((name, hdr))
    return cases


def write_scene_obj(d, sd, name="scene"):
    """SceneData -> OBJ + MTL + TGA textures (one `v/vt/vn` corner per
    triangle vertex, one usemtl run per material change): the way a user's
    asset reaches obj2voxel.  Returns the OBJ path."""
    os.makedirs(os.path.join(d, "textures"), exist_ok=True)
    with open(os.path.join(d, f"{name}.mtl"), "w") as f:
        for m in range(len(sd.mat_tex)):
            f.write(f"newmtl m{m}\nKd {' '.join(_fmt(x) for x in sd.mat_kd[m])}\n")
            t = int(sd.mat_tex[m])
            if t >= 0:
                f.write(f"map_Kd textures/t{t}.tga\n")
    for t in range(len(sd.tex_off)):
        w, h, c = (int(x) for x in sd.tex_dims[t])
        px = sd.tex_data[sd.tex_off[t]: sd.tex_off[t] + w * h * c].reshape(h, w, c)
        with open(os.path.join(d, "textures", f"t{t}.tga"), "wb") as f:
            f.write(tga_encode(px, rle=bool(t % 2), bottom_up=True))
    n = sd.ntri
    uv = sd.uv if sd.uv is not None else np.zeros((n, 6), np.float32)
    mat = sd.mat if sd.mat is not None else np.zeros(n, np.int32)
    lines = [f"mtllib {name}.mtl", f"o {name}"]
    lines += ["v " + " ".join(_fmt(x) for x in p) for p in sd.pos.reshape(-1, 3)]
    lines += ["vn " + " ".join(_fmt(x) for x in p) for p in sd.nrm.reshape(-1, 3)]
    lines += ["vt " + " ".join(_fmt(x) for x in p) for p in uv.reshape(-1, 2)]
    cur = None
    for i in range(n):
        if mat[i] != cur:
            cur = mat[i]
            lines.append(f"usemtl m{cur}")
        a = 3 * i + 1
        lines.append(f"f {a}/{a}/{a} {a + 1}/{a + 1}/{a + 1} {a + 2}/{a + 2}/{a + 2}")
    path = os.path.join(d, f"{name}.obj")
    write_text(path, lines)
    return path
