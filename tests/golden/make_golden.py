"""Regenerate the committed golden fixtures (run in the dev container, where
/root/reference exists):

    python tests/golden/make_golden.py          # everything
    python tests/golden/make_golden.py ingest   # ingest_ref.npz only

* kat_raytri.npz / kat_tribox.npz / hdr_ref.npz -- outputs of the
  REFERENCE's own raytri.cc, tribox2.cc and stb_image_write.h, compiled
  unmodified into oracle/_ref/libvrtref.so (oracle/Makefile).
* scene_*.npz -- small scenes (inputs) with per-sample outputs of the oracle
  restatement (oracle/vrt_oracle.c): hit, triangle id, voxel id, per-sample
  RGB, reference-equivalent counters and the accumulated image.  The oracle's
  floating-point leaves are pinned by the KATs above; see DESIGN.md.
* ingest_ref.npz -- tinyobj::LoadObj and stbi_load outputs of the
  REFERENCE (tiny_obj_loader.cc / stb_image.h compiled unmodified into
  oracle/_ref/libvrtref.so) on the tests/ingest_corpus.py inputs.
Only inputs and outputs are stored -- no reference source.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pyoracle as po  # noqa: E402

import voxelraytrace20190722_amd as vrt  # noqa: E402


def kat_raytri(n=6000, seed=7):
    rng = np.random.default_rng(seed)
    cases = []
    # float-widened inputs, as Triangle::isect passes them
    a = rng.standard_normal((n // 3, 15)).astype(np.float32).astype(np.float64)
    cases.append(a)
    # small-integer grids: edge / vertex / coplanar / parallel hits
    b = (rng.integers(-3, 4, (n // 3, 15)) * 0.5).astype(np.float64)
    cases.append(b)
    # near-degenerate determinants around +-1e-6 and rays along axes
    c = rng.standard_normal((n - 2 * (n // 3), 15)).astype(np.float32).astype(np.float64)
    c[:, 3:6] = 0.0
    ax = rng.integers(0, 3, len(c))
    c[np.arange(len(c)), 3 + ax] = rng.choice([-1.0, 1.0], len(c))
    scale = 10.0 ** rng.uniform(-4.5, -2.0, len(c))
    c[:, 9:15] = c[:, 6:9].repeat(2, 0).reshape(len(c), 6) + (c[:, 9:15] * scale[:, None])
    cases.append(c)
    # rays aimed at a point of the triangle (hits, incl. near-edge / vertex
    # barycentrics and hits behind the origin)
    m = n // 2
    tri = rng.standard_normal((m, 9)).astype(np.float32)
    w = rng.dirichlet([1, 1, 1], m)
    w[: m // 4] = np.round(w[: m // 4] * 8) / 8  # on edges / vertices
    tgt = (w[:, :1] * tri[:, 0:3] + w[:, 1:2] * tri[:, 3:6] + w[:, 2:3] * tri[:, 6:9])
    org = rng.standard_normal((m, 3)) * 3
    d = tgt - org
    d[: m // 8] *= -1  # target behind the origin: a hit with t < 0
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    cases.append(np.concatenate([org, d, tri], 1).astype(np.float32).astype(np.float64))
    q = np.ascontiguousarray(np.concatenate(cases))
    out = np.zeros((len(q), 4))
    for i in range(len(q)):
        r, t, u, v = po.ref_intersect_triangle3(q[i])
        out[i] = (r, t, u, v) if r == 1 else (r, 0, 0, 0)
    return q, out


def kat_tribox(n=8000, seed=11):
    rng = np.random.default_rng(seed)
    a = rng.standard_normal((n // 2, 15)).astype(np.float32)
    b = (rng.integers(-4, 5, (n - n // 2, 15)) * 0.25).astype(np.float32)
    q = np.ascontiguousarray(np.concatenate([a, b]))
    q[:, 3:6] = np.abs(q[:, 3:6])
    out = np.array([po.ref_tri_box_overlap(q[i]) for i in range(len(q))], np.int32)
    return q, out


def hdr_cases(seed=3):
    rng = np.random.default_rng(seed)
    imgs = []
    for (h, w, c) in [(5, 7, 3), (9, 40, 3), (16, 300, 3), (4, 130, 1), (6, 64, 4), (3, 9, 2)]:
        x = (rng.random((h, w, c)) * 4).astype(np.float32)
        x[:, : w // 3] = 0.25  # long runs
        x[0, :] = 0.0
        x[1, ::3] = 1e-33      # below the rgbe threshold
        imgs.append(x)
    return imgs


def downsample_textures(sd, step):
    dims, offs, data = [], [], []
    o = 0
    for t in range(len(sd.tex_off)):
        w, h, c = sd.tex_dims[t]
        img = sd.tex_data[sd.tex_off[t]: sd.tex_off[t] + w * h * c].reshape(h, w, c)[::step, ::step]
        img = np.ascontiguousarray(img)
        dims.append([img.shape[1], img.shape[0], c])
        offs.append(o)
        data.append(img.reshape(-1))
        o += img.size
    return vrt.SceneData(sd.pos, sd.nrm, sd.uv, sd.mat, sd.mat_tex, sd.mat_kd, np.array(dims, np.int32),
                         np.array(offs, np.int64), np.concatenate(data))


def soup(n=2500, seed=5):
    """Random triangle soup in a box with an untextured and a 1-channel material."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(-1, 1, (n, 1, 3))
    pos = (c + rng.normal(0, 0.08, (n, 3, 3))).astype(np.float32).reshape(n, 9)
    nrm = rng.normal(0, 1, (n, 9)).astype(np.float32)
    uv = rng.uniform(-2.5, 3.5, (n, 6)).astype(np.float32)
    mat = rng.integers(0, 3, n).astype(np.int32)
    tex = np.concatenate([rng.integers(0, 256, 16 * 12 * 1), rng.integers(0, 256, 8 * 8 * 4)]).astype(np.uint8)
    return vrt.SceneData(pos, nrm, uv, mat, np.array([0, -1, 1], np.int32),
                         np.array([[0.2, 0.4, 0.6], [0.9, 0.3, 0.1], [0, 0, 0]], np.float32),
                         np.array([[16, 12, 1], [8, 8, 4]], np.int32), np.array([0, 192], np.int64), tex)


def scene_fixture(name, sd, depth, cams, films):
    osc = po.Scene(sd, depth)
    rec = {"pos": sd.pos, "nrm": sd.nrm, "uv": sd.uv, "mat": sd.mat, "mat_tex": sd.mat_tex,
           "mat_kd": sd.mat_kd, "tex_dims": sd.tex_dims, "tex_off": sd.tex_off, "tex_data": sd.tex_data,
           "depth": np.int32(depth)}
    info, box = osc.info()
    rec["tree_info"] = info
    rec["root_box"] = box
    for k, ((fov, eye, spot, up), (fw, fh, nx, ny)) in enumerate(zip(cams, films)):
        cam = po.camera(fov, eye, spot, up)
        rgb, so = osc.render(cam, fw, fh, nx, ny, film_index=1, nthreads=8)
        rec[f"cam{k}"] = np.array([fov, *eye, *spot, *up], np.float32)
        rec[f"film{k}"] = np.array([fw, fh, nx, ny], np.float32)
        rec[f"img{k}"] = rgb
        for key in ("hit", "tri", "voxel", "rgb", "counters"):
            rec[f"s{k}_{key}"] = so[key]
    np.savez_compressed(os.path.join(HERE, f"scene_{name}.npz"), **rec)
    return rec


def pcg_std():
    """Draws of the real libstdc++ uniform_real_distribution<float> over the
    jql::PCG engine (tests/golden/pcg_std.cpp compiled with g++)."""
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "pcg_std")
        subprocess.run(["g++", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(HERE, "pcg_std.cpp")],
                       check=True)
        out = subprocess.run([exe, "64", "48", "64"], check=True, capture_output=True, text=True).stdout
    seeds, draws, pts = [], [], {}
    for ln in out.splitlines():
        f = ln.split()
        if f[0] == "U":
            seeds.append(int(f[1]))
            draws.append([float.fromhex(x) for x in f[2:]])
        else:
            pts.setdefault(int(f[1]), []).append([float.fromhex(x) for x in f[2:5]])
    return (np.array(seeds, np.uint64), np.array(draws, np.float32),
            np.array([pts[s] for s in seeds], np.float32))


def _ftok(x):
    """float32 -> a token travorder_std.cpp reads back bit-exactly."""
    x = np.float32(x)
    if np.isnan(x):
        return "nanx%08x" % int(np.array(x).view(np.uint32))
    if np.isinf(x):
        return "inf" if x > 0 else "-inf"
    return float(x).hex()


def travorder_cases(seed=20190722):
    """Adversarial inputs for travorder's std::sort and ray_march_isect's
    std::min_element: ties, +-0, +-inf, NaN (several payloads/signs, any
    position), denormals, presorted / reversed runs, plus plain random."""
    rng = np.random.default_rng(seed)
    nan_bits = np.array([0x7fc00000, 0xffc00000, 0x7f800001, 0x7fc00123], np.uint32).view(np.float32)
    special = np.concatenate([np.float32([0.0, -0.0, np.inf, -np.inf, 1.0, -1.0, 1e-45, -1e-45, 1.17549435e-38,
                                          3.4028235e38, -3.4028235e38, 0.5, 0.5, 2.0]), nan_bits])
    dist = []
    for k in range(4096):
        kind = k % 8
        if kind == 0:
            d = rng.normal(0, 1, 8)
        elif kind == 1:  # heavy ties
            d = rng.choice(np.float32([0.0, -0.0, 1.0, 1.0, 2.0]), 8)
        elif kind == 2:  # specials everywhere
            d = rng.choice(special, 8)
        elif kind == 3:  # one or two NaNs in random positions, finite otherwise
            d = rng.normal(0, 3, 8)
            for _ in range(1 + (k // 8) % 2):
                d[rng.integers(0, 8)] = rng.choice(nan_bits)
        elif kind == 4:  # presorted / reversed / constant runs with ties
            d = np.sort(rng.integers(-3, 4, 8).astype(np.float32))
            d = d[::-1] if (k // 8) % 2 else d
        elif kind == 5:  # denormals and signed zeros
            d = rng.choice(np.float32([1e-45, 2e-45, -1e-45, 0.0, -0.0, 1e-40]), 8)
        elif kind == 6:  # infinities among finite values
            d = rng.normal(0, 1, 8)
            d[rng.integers(0, 8, 3)] = rng.choice(np.float32([np.inf, -np.inf]), 3)
        else:  # realistic: travorder distances of children of one box
            c = rng.uniform(-1, 1, 3)
            h = rng.uniform(0.01, 1)
            o = rng.uniform(-2, 2, 3)
            dd = rng.normal(0, 1, 3)
            dd /= np.linalg.norm(dd)
            d = [np.float32(dd[0]) * np.float32(c[0] + (h if ci & 4 else -h) - o[0])
                 + np.float32(dd[1]) * np.float32(c[1] + (h if ci & 2 else -h) - o[1])
                 + np.float32(dd[2]) * np.float32(c[2] + (h if ci & 1 else -h) - o[2]) for ci in range(8)]
        dist.append(np.asarray(d, np.float32))
    dist = np.array(dist, np.float32)
    # hit masks: any, and ones with <= 2 / <= 4 children (the fast paths)
    mask = rng.integers(0, 256, len(dist)).astype(np.uint32)
    for k in range(len(dist)):
        if k % 3 == 1:
            mask[k] &= mask[k] - 1  # fewer bits
            mask[k] &= rng.integers(0, 256)
        elif k % 3 == 2:
            bits = rng.choice(8, rng.integers(0, 3), replace=False)
            mask[k] = np.uint32(sum(1 << int(b) for b in bits))
    depth = np.zeros((2048, 16), np.float32)
    length = np.zeros(2048, np.int32)
    for j in range(2048):
        n = j % 17
        length[j] = n
        kind = (j // 17) % 4
        if kind == 0:
            v = rng.uniform(0, 5, n)
        elif kind == 1:
            v = rng.choice(np.float32([1.0, 1.0, 2.0, 0.0, -0.0]), n)
        elif kind == 2:
            v = rng.choice(special, n)
        else:
            v = rng.uniform(0, 2, n).astype(np.float32)
            if n:
                v[rng.integers(0, n)] = rng.choice(nan_bits)
        depth[j, :n] = v
    return dist, mask, depth, length


def travorder_std():
    """The real libstdc++ std::sort / std::min_element on travorder_cases()
    (tests/golden/travorder_std.cpp compiled with g++)."""
    import subprocess
    import tempfile
    dist, mask, depth, length = travorder_cases()
    lines = ["S " + " ".join(_ftok(x) for x in d) for d in dist]
    lines += [f"M {n} " + " ".join(_ftok(x) for x in depth[j, :n]) for j, n in enumerate(length)]
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "travorder_std")
        subprocess.run(["g++", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(HERE, "travorder_std.cpp")],
                       check=True)
        out = subprocess.run([exe], input="\n".join(lines) + "\n", check=True, capture_output=True,
                             text=True).stdout.splitlines()
    order = np.array([[int(x) for x in ln.split()[1:]] for ln in out if ln[0] == "S"], np.int32)
    argmin = np.array([int(ln.split()[1]) for ln in out if ln[0] == "M"], np.int32)
    assert order.shape == (len(dist), 8) and argmin.shape == (len(length),)
    np.savez_compressed(os.path.join(HERE, "travorder_std.npz"), dist=dist, mask=mask, order=order,
                        depth=depth, length=length, argmin=argmin)


def secondary_fixture(sd, depth, cam, film, spp, name):
    osc = po.Scene(sd, depth)
    c = po.camera(*cam)
    vis, rays, d = osc.render_secondary(c, film[0], film[1], film[2], film[3], spp=spp, nthreads=8)
    rec = {"pos": sd.pos, "nrm": sd.nrm, "uv": sd.uv, "mat": sd.mat, "mat_tex": sd.mat_tex,
           "mat_kd": sd.mat_kd, "tex_dims": sd.tex_dims, "tex_off": sd.tex_off, "tex_data": sd.tex_data,
           "depth": np.int32(depth), "cam": np.array([cam[0], *cam[1], *cam[2], *cam[3]], np.float32),
           "film": np.array(film, np.float32), "spp": np.int32(spp), "vis": vis, "rays": np.int64(rays),
           "hit": d["hit"], "tri": d["tri"], "voxel": d["voxel"]}
    np.savez_compressed(os.path.join(HERE, f"secondary_{name}.npz"), **rec)


def ingest_fixture():
    """tinyobj::LoadObj (reference, compiled in place) on the deterministic
    OBJ/MTL corpus of tests/ingest_corpus.py, and stbi_load_from_memory on
    its TGA corpus.  Inputs are regenerated by the tests; their SHA-256 is
    stored so a drifting generator cannot silently change the cases."""
    import hashlib
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ingest_corpus as ic
    rec = {}
    with tempfile.TemporaryDirectory() as td:
        cases = ic.write_obj_corpus(td)
        for name, (fn, _parse_only) in sorted(cases.items()):
            path = os.path.join(td, fn)
            rec[f"{name}_sha"] = np.array(hashlib.sha256(open(path, "rb").read()).hexdigest())
            r = po.ref_load_obj(path, td + "/")
            assert r["ok"], (name, r["err"])
            for k in ("v", "vn", "vt", "idx", "mat", "shape", "kd"):
                rec[f"{name}_{k}"] = r[k]
            rec[f"{name}_nshape"] = np.int32(r["nshape"])
            rec[f"{name}_names"] = np.array(r["names"], dtype=str)
            rec[f"{name}_texnames"] = np.array(r["texnames"], dtype=str)
    for name, data in ic.tga_corpus():
        img, _why = po.ref_stbi_load_mem(data)
        rec[f"tga_{name}_sha"] = np.array(hashlib.sha256(data).hexdigest())
        rec[f"tga_{name}_ok"] = np.int32(img is not None)
        if img is not None:
            rec[f"tga_{name}_img"] = img
    np.savez_compressed(os.path.join(HERE, "ingest_ref.npz"), **rec)


def main():
    if not po.reference_available():
        raise SystemExit("oracle/_ref/libvrtref.so missing: run `make` where /root/reference exists")
    if sys.argv[1:] == ["ingest"]:
        ingest_fixture()
        return
    if sys.argv[1:] == ["travorder"]:
        travorder_std()
        return
    travorder_std()
    ingest_fixture()
    q, out = kat_raytri()
    np.savez_compressed(os.path.join(HERE, "kat_raytri.npz"), inp=q, out=out)
    q, out = kat_tribox()
    np.savez_compressed(os.path.join(HERE, "kat_tribox.npz"), inp=q, out=out)
    rec = {}
    for i, img in enumerate(hdr_cases()):
        rec[f"img{i}"] = img
        rec[f"bytes{i}"] = np.frombuffer(po.ref_hdr_bytes(img), np.uint8)
    np.savez_compressed(os.path.join(HERE, "hdr_ref.npz"), **rec)

    main_cam = (vrt.to_radian(90), (1.0, 1.3, -0.2), (0.0, 0.4, 0.0), (0.0, 1.0, 0.0))
    sd = downsample_textures(vrt.SceneData.proxy(0.02, 1), 8)
    tree = vrt.VoxelOctree(sd, 6, device=-1)
    mn, mx = tree.root_box
    sweep = [(f, tuple(e), tuple(s), tuple(u)) for f, e, s, u in
             (vrt.sweep_pose(mn, mx, i, 16) for i in (3, 11))]
    scene_fixture("proxy", sd, 6, [main_cam, sweep[0], sweep[1]],
                  [(1.0, 1.0, 64, 64), (1.0, 1.0, 48, 32), (1.0, 1.0, 40, 56)])
    sd2 = soup()
    scene_fixture("soup", sd2, 7,
                  [(vrt.to_radian(70), (0.1, 0.2, 2.8), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0)),
                   (vrt.to_radian(100), (0.05, 0.0, 0.02), (1.0, 0.3, 0.2), (0.0, 1.0, 0.0))],
                  [(1.0, 1.0, 40, 40), (1.0, 1.0, 33, 27)])
    seeds, draws, pts = pcg_std()
    np.savez_compressed(os.path.join(HERE, "pcg_std.npz"), seeds=seeds, draws=draws, points=pts)
    secondary_fixture(sd, 6, main_cam, (1.0, 1.0, 24, 16), 64, "proxy")
    for f in sorted(os.listdir(HERE)):
        print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
