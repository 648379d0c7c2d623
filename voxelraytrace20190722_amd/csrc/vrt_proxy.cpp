// vrt_proxy.cpp -- deterministic synthetic inputs: the "sponza-proxy" atrium
// (Asset/sponza/sponza.obj is absent from the reference, see
// .MISSING_LARGE_BLOBS) and the camera-sweep poses.
//
// The atrium lives in the frame the reference's cameras expect (its scaled
// Sponza: x in [-1.92, 1.80], y in [-0.13, 1.43], z in [-1.11, 1.19];
// VRT/main.cc:76-78,112-115): a tiled floor, outer walls, two storeys of
// colonnades with arches on both long sides, balcony slabs, hanging curtains,
// vases and wall ornaments.  Every textured material uses a procedural 8-bit
// texture (1, 3 and 4 channels, tiled and negative uvs) so every branch of
// texel_fetch / unit_cycle is exercised; one material is untextured (Kd).
#include "../../include/vrt.h"

#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

constexpr double kPi = 3.14159265358979323846;

struct V {
        float x, y, z;
};

struct Mesh {
        std::vector<float> pos, nrm, uv;
        std::vector<int32_t> mat;
        void tri(V a, V b, V c, V na, V nb, V nc, float ua, float va, float ub,
                 float vb, float uc, float vc, int m)
        {
                const V p[3] = { a, b, c }, n[3] = { na, nb, nc };
                for (int i = 0; i < 3; ++i) {
                        pos.insert(pos.end(), { p[i].x, p[i].y, p[i].z });
                        nrm.insert(nrm.end(), { n[i].x, n[i].y, n[i].z });
                }
                uv.insert(uv.end(), { ua, va, ub, vb, uc, vc });
                mat.push_back(m);
        }
        // grid patch: P(s,t), N(s,t), UV = (u0 + s*us, v0 + t*vs)
        template <class FP, class FN>
        void patch(int ns, int nt, FP P, FN N, float u0, float us, float v0,
                   float vs, int m)
        {
                for (int j = 0; j < nt; ++j)
                        for (int i = 0; i < ns; ++i) {
                                const double s0 = (double)i / ns, s1 = (double)(i + 1) / ns;
                                const double t0 = (double)j / nt, t1 = (double)(j + 1) / nt;
                                const V a = P(s0, t0), b = P(s1, t0), c = P(s1, t1), d = P(s0, t1);
                                const V na = N(s0, t0), nb = N(s1, t0), nc = N(s1, t1), nd = N(s0, t1);
                                const float ua = (float)(u0 + s0 * us), ub = (float)(u0 + s1 * us);
                                const float va = (float)(v0 + t0 * vs), vb = (float)(v0 + t1 * vs);
                                tri(a, b, c, na, nb, nc, ua, va, ub, va, ub, vb, m);
                                tri(a, c, d, na, nc, nd, ua, va, ub, vb, ua, vb, m);
                        }
        }
        // axis-aligned box, 6 subdivided faces
        void box(V lo, V hi, int sub, float uvs, int m)
        {
                const float x0 = lo.x, y0 = lo.y, z0 = lo.z, x1 = hi.x, y1 = hi.y, z1 = hi.z;
                auto L = [](double a, double b, double t) { return (float)(a + (b - a) * t); };
                // +y, -y
                patch(sub, sub, [&](double s, double t) { return V{ L(x0, x1, s), y1, L(z1, z0, t) }; },
                      [](double, double) { return V{ 0, 2, 0 }; }, 0, uvs * (x1 - x0), 0, uvs * (z1 - z0), m);
                patch(sub, sub, [&](double s, double t) { return V{ L(x0, x1, s), y0, L(z0, z1, t) }; },
                      [](double, double) { return V{ 0, -1, 0 }; }, 0, uvs * (x1 - x0), 0, uvs * (z1 - z0), m);
                // +x, -x
                patch(sub, sub, [&](double s, double t) { return V{ x1, L(y0, y1, t), L(z1, z0, s) }; },
                      [](double, double) { return V{ 1, 0, 0 }; }, 0, uvs * (z1 - z0), 0, uvs * (y1 - y0), m);
                patch(sub, sub, [&](double s, double t) { return V{ x0, L(y0, y1, t), L(z0, z1, s) }; },
                      [](double, double) { return V{ -3, 0, 0 }; }, 0, uvs * (z1 - z0), 0, uvs * (y1 - y0), m);
                // +z, -z
                patch(sub, sub, [&](double s, double t) { return V{ L(x0, x1, s), L(y0, y1, t), z1 }; },
                      [](double, double) { return V{ 0, 0, 1 }; }, 0, uvs * (x1 - x0), 0, uvs * (y1 - y0), m);
                patch(sub, sub, [&](double s, double t) { return V{ L(x1, x0, s), L(y0, y1, t), z0 }; },
                      [](double, double) { return V{ 0, 0, -1 }; }, 0, uvs * (x1 - x0), 0, uvs * (y1 - y0), m);
        }
        // vertical cylinder column with base/capital bulges
        void column(float cx, float cz, float y0, float y1, float r, int seg, int rings, int m)
        {
                auto R = [&](double t) {
                        double rr = r;
                        if (t < 0.08) rr *= 1.0 + 0.35 * (1.0 - t / 0.08);
                        if (t > 0.90) rr *= 1.0 + 0.30 * ((t - 0.90) / 0.10);
                        rr *= 1.0 + 0.03 * std::sin(t * 40.0);  // fluting-ish
                        return rr;
                };
                patch(seg, rings,
                      [&](double s, double t) {
                              const double a = 2 * kPi * s, rr = R(t);
                              return V{ (float)(cx + rr * std::cos(a)), (float)(y0 + (y1 - y0) * t),
                                        (float)(cz + rr * std::sin(a)) };
                      },
                      [&](double s, double) {
                              const double a = 2 * kPi * s;
                              return V{ (float)(1.7 * std::cos(a)), 0.f, (float)(1.7 * std::sin(a)) };
                      },
                      -0.5f, 2.0f, 0.0f, 3.0f, m);
        }
        // semicircular arch (thick half-annulus) in the plane z = zc, spanning
        // x in [xa, xb], springing at height ys, depth dz
        void arch(float xa, float xb, float ys, float zc, float dz, float th, int seg, int m)
        {
                const double cx = 0.5 * (xa + xb), rin = 0.5 * (xb - xa), rout = rin + th;
                auto P = [&](double rr, double a, double z) {
                        return V{ (float)(cx - rr * std::cos(a)), (float)(ys + rr * std::sin(a)), (float)z };
                };
                const double z0 = zc - 0.5 * dz, z1 = zc + 0.5 * dz;
                // intrados (inner) and extrados (outer) surfaces
                patch(seg, 4, [&](double s, double t) { return P(rin, kPi * s, z0 + (z1 - z0) * t); },
                      [&](double s, double) { return V{ (float)std::cos(kPi * s), (float)-std::sin(kPi * s), 0.f }; },
                      0, 4, 0, 1, m);
                patch(seg, 4, [&](double s, double t) { return P(rout, kPi * s, z1 + (z0 - z1) * t); },
                      [&](double s, double) { return V{ (float)-std::cos(kPi * s), (float)std::sin(kPi * s), 0.f }; },
                      0, 4, 0, 1, m);
                // the two faces (annulus sectors)
                patch(seg, 3, [&](double s, double t) { return P(rin + (rout - rin) * t, kPi * s, z0); },
                      [](double, double) { return V{ 0, 0, -1 }; }, 0, 4, 0, 0.5f, m);
                patch(seg, 3, [&](double s, double t) { return P(rout + (rin - rout) * t, kPi * s, z1); },
                      [](double, double) { return V{ 0, 0, 1 }; }, 0, 4, 0, 0.5f, m);
        }
        void sphere(V c, float r, int seg, int rings, int m)
        {
                patch(seg, rings,
                      [&](double s, double t) {
                              const double a = 2 * kPi * s, b = kPi * (t - 0.5);
                              return V{ (float)(c.x + r * std::cos(b) * std::cos(a)), (float)(c.y + r * std::sin(b)),
                                        (float)(c.z + r * std::cos(b) * std::sin(a)) };
                      },
                      [&](double s, double t) {
                              const double a = 2 * kPi * s, b = kPi * (t - 0.5);
                              return V{ (float)(std::cos(b) * std::cos(a)), (float)std::sin(b),
                                        (float)(std::cos(b) * std::sin(a)) };
                      },
                      0, 1, 0, 1, m);
        }
        // hanging curtain in the plane z = zc with a wave along x
        void curtain(float x0, float x1, float ytop, float ybot, float zc, float amp, int ns, int nt, int m)
        {
                patch(ns, nt,
                      [&](double s, double t) {
                              const double w = amp * std::sin(s * 6 * kPi) * (0.3 + 0.7 * t);
                              return V{ (float)(x0 + (x1 - x0) * s), (float)(ytop + (ybot - ytop) * t), (float)(zc + w) };
                      },
                      [&](double s, double t) {
                              const double dw = amp * 6 * kPi * std::cos(s * 6 * kPi) * (0.3 + 0.7 * t) / (x1 - x0);
                              return V{ (float)-dw, 0.f, 1.f };
                      },
                      0, 1, 0, 1, m);
        }
};

struct Tex {
        int w, h, c;
        std::vector<uint8_t> px;
};

uint32_t hash32(uint32_t x)
{
        x ^= x >> 16;
        x *= 0x7feb352dU;
        x ^= x >> 15;
        x *= 0x846ca68bU;
        x ^= x >> 16;
        return x;
}

Tex make_tex(int kind, int w, int h, int c, uint32_t seed)
{
        Tex t{ w, h, c, std::vector<uint8_t>((size_t)w * h * c) };
        for (int y = 0; y < h; ++y)
                for (int x = 0; x < w; ++x) {
                        const uint32_t n = hash32((uint32_t)(x + 7919 * y) ^ seed) & 63;
                        int r = 128, g = 128, b = 128, a = 255;
                        switch (kind) {
                        case 0: {  // floor tiles
                                const bool chk = ((x / (w / 8)) + (y / (h / 8))) & 1;
                                r = chk ? 190 : 120; g = chk ? 180 : 110; b = chk ? 160 : 100;
                                break;
                        }
                        case 1: {  // bricks
                                const int bh = h / 16, bw = w / 8;
                                const int row = y / bh, off = (row & 1) * bw / 2;
                                const bool mortar = (y % bh) < 2 || ((x + off) % bw) < 2;
                                r = mortar ? 200 : 150; g = mortar ? 195 : 80; b = mortar ? 185 : 60;
                                break;
                        }
                        case 2: {  // column stone, vertical stripes
                                const int s = (x * 12 / w) & 1;
                                r = 200 - 30 * s; g = 190 - 30 * s; b = 170 - 25 * s;
                                break;
                        }
                        case 3: case 4: case 5: {  // fabric red / green / blue
                                const int s = ((x / 6) ^ (y / 6)) & 1;
                                r = kind == 3 ? 170 + 30 * s : 40; g = kind == 4 ? 150 + 30 * s : 40;
                                b = kind == 5 ? 160 + 30 * s : 50;
                                break;
                        }
                        case 6: {  // arch: gradient
                                r = 100 + 100 * x / w; g = 90 + 80 * y / h; b = 80;
                                break;
                        }
                        case 7: {  // roof RGBA
                                r = 140; g = 70 + (y * 60 / h); b = 50; a = 128 + (x & 127);
                                break;
                        }
                        default: {  // grey (1-channel ornaments)
                                r = g = b = 60 + (int)((x * 131 + y * 71) % 150);
                                break;
                        }
                        }
                        const int v[4] = { r + (int)n - 32, g + (int)n - 32, b + (int)n - 32, a };
                        for (int k = 0; k < c; ++k) {
                                int q = c == 1 ? v[0] : v[k];
                                q = q < 0 ? 0 : (q > 255 ? 255 : q);
                                t.px[((size_t)y * w + x) * c + k] = (uint8_t)q;
                        }
                }
        return t;
}

enum Mat {
        M_FLOOR, M_BRICK, M_COLUMN, M_FAB_R, M_FAB_G, M_FAB_B, M_ARCH, M_ROOF,
        M_ORN, M_VASE_KD, M_COUNT
};

void build(double detail, uint32_t seed, Mesh &me, std::vector<Tex> &texs,
           std::vector<int32_t> &mat_tex, std::vector<float> &mat_kd)
{
        // detail 1.0 ~ 262k triangles (Sponza's count)
        const double q = 0.9 * std::sqrt(detail > 0.01 ? detail : 0.01);
        auto S = [&](int n) { int v = (int)std::lround(n * q); return v < 3 ? 3 : v; };
        const float X0 = -1.92f, X1 = 1.80f, Y0 = -0.13f, Y1 = 1.43f, Z0 = -1.11f, Z1 = 1.19f;
        const float yf = 0.0f;     // ground floor level
        const float y2 = 0.62f;    // second storey
        // floor slab (top subdivided, uv tiled 0..8 with negative offset)
        me.patch(S(110), S(68), [&](double s, double t) {
                         return V{ (float)(X0 + (X1 - X0) * s), yf, (float)(Z1 + (Z0 - Z1) * t) }; },
                 [](double, double) { return V{ 0, 1, 0 }; }, -2.0f, 9.0f, -1.5f, 6.0f, M_FLOOR);
        me.box(V{ X0, Y0, Z0 }, V{ X1, yf - 0.001f, Z1 }, S(4), 1.0f, M_BRICK);
        // outer walls (inner faces subdivided), end walls with ornaments
        const float wt = 0.05f;
        me.box(V{ X0, yf, Z0 }, V{ X1, Y1 - 0.10f, Z0 + wt }, S(40), 2.0f, M_BRICK);
        me.box(V{ X0, yf, Z1 - wt }, V{ X1, Y1 - 0.10f, Z1 }, S(40), 2.0f, M_BRICK);
        me.box(V{ X0, yf, Z0 }, V{ X0 + wt, Y1 - 0.10f, Z1 }, S(28), 2.0f, M_BRICK);
        me.box(V{ X1 - wt, yf, Z0 }, V{ X1, Y1 - 0.10f, Z1 }, S(28), 2.0f, M_BRICK);
        // roof rims on the long sides (sloped, RGBA texture)
        for (int side = 0; side < 2; ++side) {
                const float zw = side ? Z1 : Z0, zi = side ? Z1 - 0.55f : Z0 + 0.55f;
                me.patch(S(96), S(10), [&](double s, double t) {
                                 return V{ (float)(X0 + (X1 - X0) * s), (float)(Y1 - 0.10 + 0.10 * t),
                                           (float)(zw + (zi - zw) * t) }; },
                         [&](double, double) { return V{ 0.f, 1.f, side ? -0.3f : 0.3f }; },
                         0.f, 12.f, 0.f, 1.f, M_ROOF);
        }
        // colonnades: both long sides, two storeys
        const int ncol = 11;
        const float colr = 0.055f;
        for (int side = 0; side < 2; ++side) {
                const float zc = side ? Z1 - 0.55f : Z0 + 0.55f;
                for (int storey = 0; storey < 2; ++storey) {
                        const float ya = storey ? y2 + 0.02f : yf;
                        const float yb = storey ? Y1 - 0.25f : y2 - 0.10f;
                        const float xs0 = X0 + 0.35f, xs1 = X1 - 0.35f;
                        for (int i = 0; i < ncol; ++i) {
                                const float cx = xs0 + (xs1 - xs0) * i / (ncol - 1);
                                me.column(cx, zc, ya, yb, storey ? colr * 0.8f : colr, S(40), S(26), M_COLUMN);
                                if (i + 1 < ncol) {
                                        const float nx = xs0 + (xs1 - xs0) * (i + 1) / (ncol - 1);
                                        me.arch(cx + colr, nx - colr, yb - 0.5f * (nx - cx - 2 * colr) + 0.02f,
                                                zc, 0.12f, 0.03f, S(40), M_ARCH);
                                }
                        }
                        // entablature beam above the arches
                        me.box(V{ xs0 - 0.1f, yb, zc - 0.07f }, V{ xs1 + 0.1f, yb + 0.05f, zc + 0.07f }, S(24), 4.0f,
                               M_ARCH);
                }
                // balcony slab between the wall and the colonnade
                const float za = side ? zc - 0.06f : Z0 + wt, zb = side ? Z1 - wt : zc + 0.06f;
                me.box(V{ X0 + wt, y2 - 0.04f, za }, V{ X1 - wt, y2, zb }, S(24), 3.0f, M_FLOOR);
                // curtains hanging between upper columns
                for (int i = 1; i + 1 < ncol; i += 2) {
                        const float xs0 = X0 + 0.35f, xs1 = X1 - 0.35f;
                        const float a = xs0 + (xs1 - xs0) * i / (ncol - 1) + 0.06f;
                        const float b = xs0 + (xs1 - xs0) * (i + 1) / (ncol - 1) - 0.06f;
                        me.curtain(a, b, y2 - 0.05f, y2 - 0.45f, side ? zc - 0.12f : zc + 0.12f, 0.02f, S(48), S(32),
                                   M_FAB_R + (i / 2) % 3);
                }
        }
        // vases on the floor (untextured Kd material for two of them)
        for (int i = 0; i < 16; ++i) {
                const float x = X0 + 0.6f + (X1 - X0 - 1.2f) * (i % 8) / 7.0f;
                const float z = (i < 8) ? -0.25f : 0.30f;
                me.sphere(V{ x, 0.07f, z }, 0.07f, S(36), S(18), (i % 8 == 3) ? M_VASE_KD : M_ORN);
        }
        // wall ornaments ("lion heads") on the end walls
        for (int i = 0; i < 6; ++i) {
                const float y = 0.35f + 0.25f * (i / 2), z = (i & 1) ? -0.35f : 0.35f;
                me.sphere(V{ X0 + wt + 0.02f, y, z }, 0.06f, S(36), S(18), M_ORN);
                me.sphere(V{ X1 - wt - 0.02f, y, z }, 0.06f, S(36), S(18), M_ORN);
        }
        // a sparse hanging lattice of small boxes across the open courtyard
        for (int i = 0; i < 24; ++i) {
                const uint32_t h = hash32(seed + (uint32_t)i);
                const float x = X0 + 0.4f + (X1 - X0 - 0.8f) * ((h & 1023) / 1023.0f);
                const float z = -0.3f + 0.6f * (((h >> 10) & 1023) / 1023.0f);
                const float y = 0.9f + 0.3f * (((h >> 20) & 1023) / 1023.0f);
                me.box(V{ x - 0.02f, y, z - 0.02f }, V{ x + 0.02f, y + 0.04f, z + 0.02f }, S(3), 8.0f, M_ROOF);
        }

        // textures: kind, size, channels
        const int kinds[M_COUNT - 1][4] = {
                { 0, 512, 512, 3 },  { 1, 512, 512, 3 }, { 2, 256, 1024, 3 },
                { 3, 256, 256, 3 },  { 4, 256, 256, 4 }, { 5, 256, 256, 3 },
                { 6, 512, 256, 3 },  { 7, 256, 256, 4 }, { 8, 256, 256, 1 },
        };
        for (int t = 0; t < M_COUNT - 1; ++t)
                texs.push_back(make_tex(kinds[t][0], kinds[t][1], kinds[t][2], kinds[t][3], seed * 31u + (uint32_t)t));
        for (int m = 0; m < M_COUNT; ++m) {
                mat_tex.push_back(m == M_VASE_KD ? -1 : m);
                mat_kd.insert(mat_kd.end(), { 0.8f, 0.65f, 0.3f });
        }
}

}  // namespace

extern "C" int vrt_proxy_scene(double detail, uint32_t seed, int32_t *ntri,
                               float *pos, float *nrm, float *uv, int32_t *mat,
                               int32_t *nmat, int32_t *mat_tex, float *mat_kd,
                               int32_t *ntex, int32_t *tex_dims,
                               int64_t *tex_off, uint8_t *tex_data,
                               int64_t *tex_bytes)
{
        if (!ntri || !nmat || !ntex || !tex_bytes || !(detail > 0))
                return VRT_E_INVALID;
        Mesh me;
        std::vector<Tex> texs;
        std::vector<int32_t> mt;
        std::vector<float> kd;
        build(detail, seed, me, texs, mt, kd);
        int64_t tb = 0;
        for (auto &t : texs)
                tb += (int64_t)t.px.size();
        const int32_t nt = (int32_t)me.mat.size();
        if (pos) {
                if (!nrm || !uv || !mat || !mat_tex || !mat_kd || !tex_dims || !tex_off || !tex_data ||
                    *ntri < nt || *nmat < (int32_t)mt.size() || *ntex < (int32_t)texs.size() || *tex_bytes < tb)
                        return VRT_E_INVALID;
                std::memcpy(pos, me.pos.data(), me.pos.size() * sizeof(float));
                std::memcpy(nrm, me.nrm.data(), me.nrm.size() * sizeof(float));
                std::memcpy(uv, me.uv.data(), me.uv.size() * sizeof(float));
                std::memcpy(mat, me.mat.data(), me.mat.size() * sizeof(int32_t));
                std::memcpy(mat_tex, mt.data(), mt.size() * sizeof(int32_t));
                std::memcpy(mat_kd, kd.data(), kd.size() * sizeof(float));
                int64_t o = 0;
                for (size_t t = 0; t < texs.size(); ++t) {
                        tex_dims[3 * t] = texs[t].w;
                        tex_dims[3 * t + 1] = texs[t].h;
                        tex_dims[3 * t + 2] = texs[t].c;
                        tex_off[t] = o;
                        std::memcpy(tex_data + o, texs[t].px.data(), texs[t].px.size());
                        o += (int64_t)texs[t].px.size();
                }
        }
        *ntri = nt;
        *nmat = (int32_t)mt.size();
        *ntex = (int32_t)texs.size();
        *tex_bytes = tb;
        return VRT_OK;
}

extern "C" int vrt_sweep_pose(const float mn[3], const float mx[3], int i,
                              int n, float eye[3], float spot[3], float up[3],
                              float *fov)
{
        if (!mn || !mx || !eye || !spot || !up || !fov || n < 1)
                return VRT_E_INVALID;
        const double a = 2 * kPi * (double)(i % n) / n;
        const double cx = 0.5 * (mn[0] + mx[0]), cy = 0.5 * (mn[1] + mx[1]), cz = 0.5 * (mn[2] + mx[2]);
        const double rx = 0.35 * (mx[0] - mn[0]), rz = 0.30 * (mx[2] - mn[2]);
        eye[0] = (float)(cx + rx * std::cos(a));
        eye[1] = (float)(mn[1] + 0.4 * (mx[1] - mn[1]));
        eye[2] = (float)(cz + rz * std::sin(a));
        spot[0] = (float)cx;
        spot[1] = (float)cy;
        spot[2] = (float)cz;
        up[0] = 0.f;
        up[1] = 1.f;
        up[2] = 0.f;
        // fov 90 degrees via jql::to_radian (degree * pi / 180.f)
        *fov = 90.f * 3.1415926535897932384626f / 180.f;
        return VRT_OK;
}
