// vrt_math.h -- the reference's floating-point contract, written once for
// both the host (legacy symbols, camera, octree build) and the gfx950
// kernels.  Every function performs exactly the IEEE operations, in exactly
// the order, of the cited reference code; compile with -ffp-contract=off and
// without fast-math (hipcc's default correctly-rounded f32 div/sqrt).
//
// VRT/x = /root/reference/VoxelRayTrace20190722/x
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define VRT_HD __host__ __device__ __forceinline__

namespace vrt {

struct f3 {
        float x, y, z;
};

VRT_HD f3 mk3(float x, float y, float z) { return f3{ x, y, z }; }
VRT_HD f3 operator+(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
VRT_HD f3 operator-(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
VRT_HD f3 operator*(f3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
VRT_HD f3 operator-(f3 a) { return mk3(-a.x, -a.y, -a.z); }

// dot = value_sum(p*q): `sum{0}; sum += p_k*q_k` (VRT/graphics_math.h:532-549)
VRT_HD float dot(f3 a, f3 b)
{
        float s = 0.0f;
        s += a.x * b.x;
        s += a.y * b.y;
        s += a.z * b.z;
        return s;
}
// VRT/graphics_math.h:576-586: sqrtf(dot(v,v)); v / length (per component)
VRT_HD float length(f3 a) { return sqrtf(dot(a, a)); }
VRT_HD f3 normalize(f3 a)
{
        const float l = length(a);
        return mk3(a.x / l, a.y / l, a.z / l);
}
// VRT/graphics_math.h:588-592
VRT_HD f3 cross(f3 p, f3 q)
{
        return mk3(p.y * q.z - q.y * p.z, p.z * q.x - q.z * p.x,
                   p.x * q.y - q.x * p.y);
}
// jql::clamp (VRT/graphics_math.h:904-909)
VRT_HD float clampf(float s, float lo, float hi)
{
        return s > hi ? hi : (s < lo ? lo : s);
}
VRT_HD int clampi(int s, int lo, int hi)
{
        return s > hi ? hi : (s < lo ? lo : s);
}
// std::min / std::max as used by jql::min/max (VRT/graphics_math.h:920-946)
VRT_HD float std_min(float a, float b) { return (b < a) ? b : a; }
VRT_HD float std_max(float a, float b) { return (a < b) ? b : a; }

// FLT_MIN / FLT_MAX without <cfloat> in device code
constexpr float kFltMin = 1.17549435082228750797e-38f;
constexpr float kFltMax = 3.40282346638528859812e+38f;

// ---------------------------------------------------------------------
// fp64 Moller-Trumbore, VRT/raytri.cc:197-249 (intersect_triangle3).
// Returns 1 and writes t,u,v on a hit; 0 otherwise (u,v may be written).
// ---------------------------------------------------------------------
VRT_HD int mt_isect(const double o[3], const double d[3], const double v0[3],
                    const double v1[3], const double v2[3], double *t,
                    double *u, double *v)
{
        const double e1x = v1[0] - v0[0], e1y = v1[1] - v0[1], e1z = v1[2] - v0[2];
        const double e2x = v2[0] - v0[0], e2y = v2[1] - v0[1], e2z = v2[2] - v0[2];
        const double px = d[1] * e2z - d[2] * e2y;
        const double py = d[2] * e2x - d[0] * e2z;
        const double pz = d[0] * e2y - d[1] * e2x;
        const double det = e1x * px + e1y * py + e1z * pz;
        const double tx = o[0] - v0[0], ty = o[1] - v0[1], tz = o[2] - v0[2];
        const double inv_det = 1.0 / det;
        const double qx = ty * e1z - tz * e1y;
        const double qy = tz * e1x - tx * e1z;
        const double qz = tx * e1y - ty * e1x;
        double uu, vv;
        if (det > 0.000001) {
                uu = tx * px + ty * py + tz * pz;
                *u = uu;
                if (uu < 0.0 || uu > det)
                        return 0;
                vv = d[0] * qx + d[1] * qy + d[2] * qz;
                *v = vv;
                if (vv < 0.0 || uu + vv > det)
                        return 0;
        } else if (det < -0.000001) {
                uu = tx * px + ty * py + tz * pz;
                *u = uu;
                if (uu > 0.0 || uu < det)
                        return 0;
                vv = d[0] * qx + d[1] * qy + d[2] * qz;
                *v = vv;
                if (vv > 0.0 || uu + vv < det)
                        return 0;
        } else {
                return 0;
        }
        *t = (e2x * qx + e2y * qy + e2z * qz) * inv_det;
        *u = uu * inv_det;
        *v = vv * inv_det;
        return 1;
}

// ---------------------------------------------------------------------
// fp32 triangle/box SAT, VRT/tribox2.cc:52-196 (triBoxOverlap).
// ---------------------------------------------------------------------
VRT_HD bool sat_sep(float pa, float pb, bool swap_cmp, float rad)
{
        float mn, mx;
        if (!swap_cmp) {  // if(p0<p2) {min=p0; max=p2;} else {...}
                if (pa < pb) { mn = pa; mx = pb; } else { mn = pb; mx = pa; }
        } else {          // AXISTEST_Z12: if(p2<p1) {min=p2; max=p1;} else {...}
                if (pb < pa) { mn = pb; mx = pa; } else { mn = pa; mx = pb; }
        }
        return mn > rad || mx < -rad;
}

VRT_HD int tri_box_overlap(const float c[3], const float h[3], const float tv[9])
{
        float v0[3], v1[3], v2[3], e0[3], e1[3], e2[3];
        for (int k = 0; k < 3; ++k) {
                v0[k] = tv[k] - c[k];
                v1[k] = tv[3 + k] - c[k];
                v2[k] = tv[6 + k] - c[k];
        }
        for (int k = 0; k < 3; ++k) {
                e0[k] = v1[k] - v0[k];
                e1[k] = v2[k] - v1[k];
                e2[k] = v0[k] - v2[k];
        }
        // X tests project on (y,z), Y tests on (x,z), Z tests on (x,y)
        auto X = [&](float a, float b, const float *va, const float *vb, float fa, float fb) {
                return sat_sep(a * va[1] - b * va[2], a * vb[1] - b * vb[2], false, fa * h[1] + fb * h[2]);
        };
        auto Y = [&](float a, float b, const float *va, const float *vb, float fa, float fb) {
                return sat_sep(-a * va[0] + b * va[2], -a * vb[0] + b * vb[2], false, fa * h[0] + fb * h[2]);
        };
        auto Z = [&](float a, float b, const float *va, const float *vb, float fa, float fb, bool z12) {
                return sat_sep(a * va[0] - b * va[1], a * vb[0] - b * vb[1], z12, fa * h[0] + fb * h[1]);
        };
        float fx = fabsf(e0[0]), fy = fabsf(e0[1]), fz = fabsf(e0[2]);
        if (X(e0[2], e0[1], v0, v2, fz, fy)) return 0;      // AXISTEST_X01
        if (Y(e0[2], e0[0], v0, v2, fz, fx)) return 0;      // AXISTEST_Y02
        if (Z(e0[1], e0[0], v1, v2, fy, fx, true)) return 0; // AXISTEST_Z12
        fx = fabsf(e1[0]); fy = fabsf(e1[1]); fz = fabsf(e1[2]);
        if (X(e1[2], e1[1], v0, v2, fz, fy)) return 0;      // AXISTEST_X01
        if (Y(e1[2], e1[0], v0, v2, fz, fx)) return 0;      // AXISTEST_Y02
        if (Z(e1[1], e1[0], v0, v1, fy, fx, false)) return 0; // AXISTEST_Z0
        fx = fabsf(e2[0]); fy = fabsf(e2[1]); fz = fabsf(e2[2]);
        if (X(e2[2], e2[1], v0, v1, fz, fy)) return 0;      // AXISTEST_X2
        if (Y(e2[2], e2[0], v0, v1, fz, fx)) return 0;      // AXISTEST_Y1
        if (Z(e2[1], e2[0], v1, v2, fy, fx, true)) return 0; // AXISTEST_Z12
        for (int k = 0; k < 3; ++k) {  // FINDMINMAX, bullet 1
                float mn = v0[k], mx = v0[k];
                if (v1[k] < mn) mn = v1[k];
                if (v1[k] > mx) mx = v1[k];
                if (v2[k] < mn) mn = v2[k];
                if (v2[k] > mx) mx = v2[k];
                if (mn > h[k] || mx < -h[k])
                        return 0;
        }
        // bullet 2: planeBoxOverlap(normal, d, boxhalfsize)
        const float n0 = e0[1] * e1[2] - e0[2] * e1[1];
        const float n1 = e0[2] * e1[0] - e0[0] * e1[2];
        const float n2 = e0[0] * e1[1] - e0[1] * e1[0];
        const float dd = -(n0 * v0[0] + n1 * v0[1] + n2 * v0[2]);
        const float n[3] = { n0, n1, n2 };
        float vmin[3], vmax[3];
        for (int q = 0; q < 3; ++q) {
                if (n[q] > 0.0f) { vmin[q] = -h[q]; vmax[q] = h[q]; }
                else { vmin[q] = h[q]; vmax[q] = -h[q]; }
        }
        if (n0 * vmin[0] + n1 * vmin[1] + n2 * vmin[2] + dd > 0.0f)
                return 0;
        if (n0 * vmax[0] + n1 * vmax[1] + n2 * vmax[2] + dd >= 0.0f)
                return 1;
        return 0;
}

// ---------------------------------------------------------------------
// AABB3D::isect(ray, nullptr), VRT/graphics_math.h:1312-1332.
// ---------------------------------------------------------------------
VRT_HD float dinv_of(float d)  // std::replace(d, 0.f, FLT_MIN); 1.f / d
{
        return 1.f / (d == 0.f ? kFltMin : d);
}

VRT_HD bool slab_hit(float t0, float t1, float tmin, float tmax)
{
        if (t0 > t1)
                return false;
        return (t0 >= tmin && t0 <= tmax) || (t1 >= tmin && t1 <= tmax);
}

VRT_HD bool aabb_isect(const float bmin[3], const float bmax[3], f3 o,
                       f3 dinv, float tmin, float tmax)
{
        const float oo[3] = { o.x, o.y, o.z }, di[3] = { dinv.x, dinv.y, dinv.z };
        float at0[3], at1[3];
        for (int k = 0; k < 3; ++k) {
                const float a = (bmin[k] - oo[k]) * di[k];
                const float b = (bmax[k] - oo[k]) * di[k];
                at0[k] = std_min(a, b);
                at1[k] = std_max(a, b);
        }
        float t0 = at0[0], t1 = at1[0];  // max_element / min_element
        if (t0 < at0[1]) t0 = at0[1];
        if (t0 < at0[2]) t0 = at0[2];
        if (at1[1] < t1) t1 = at1[1];
        if (at1[2] < t1) t1 = at1[2];
        return slab_hit(t0, t1, tmin, tmax);
}

// ---------------------------------------------------------------------
// Texture addressing, VRT/voxel_octree.cc:392-422.
// unit_cycle subtracts/adds 1 one step at a time; for |s| < 2^24 every step
// but the last upward one is exact, so the loop equals the closed form
// below bit for bit (tests/test_host.py checks it against the loop).  For
// |s| >= 2^24 the reference loop can fail to terminate; we stop after 64
// steps there (documented deviation on inputs the reference hangs on).
// ---------------------------------------------------------------------
VRT_HD float unit_cycle(float s)
{
        if (s > 1.f) {
                if (s < 16777216.f) {
                        s = s - (ceilf(s) - 1.f);
                } else {
                        for (int i = 0; i < 64 && s > 1.f; ++i)
                                s -= 1.f;
                }
        }
        if (s < 0.f) {
                if (s > -16777216.f) {
                        s = (s + (ceilf(-s) - 1.f)) + 1.f;
                } else {
                        for (int i = 0; i < 64 && s < 0.f; ++i)
                                s += 1.f;
                }
        }
        return s;
}

// jql::barycentric, VRT/graphics_math.h:1082-1100
VRT_HD f3 barycentric(f3 p, f3 a, f3 b, f3 c)
{
        const f3 v0 = b - a, v1 = c - a, v2 = p - a;
        const float d00 = dot(v0, v0), d01 = dot(v0, v1), d11 = dot(v1, v1);
        const float d20 = dot(v2, v0), d21 = dot(v2, v1);
        const float denom = d00 * d11 - d01 * d01;
        if (denom == 0)
                return mk3(0.f, 0.f, 0.f);
        f3 bc;
        bc.y = (d11 * d20 - d01 * d21) / denom;
        bc.z = (d00 * d21 - d01 * d20) / denom;
        bc.x = 1.0f - bc.y - bc.z;
        return bc;
}

// Sky on a miss, VRT/main.cc:18-20: t = 0.5 * (d.y + 1.0) in double, then
// lerp((1,1,1), (.6,.8,1), t) = v0 + (v1 - v0) * t.
VRT_HD f3 sky(float dy)
{
        const float t = (float)(0.5 * ((double)dy + 1.0));
        return mk3(1.0f + (0.6f - 1.0f) * t, 1.0f + (0.8f - 1.0f) * t,
                   1.0f + (1.0f - 1.0f) * t);
}

// Camera::gen_rays4 / gen_rays1 direction for pixel (px,py), sample (sx,sy)
// (VRT/camera.cc:77-112): x = px - nx/2, y = (ny-1-py) - ny/2 (int math),
// x_ = (x+sx)/nx, y_ = (y+sy)/ny, then vector_transform(C_, {x_, y_, z}) =
// `result{}; result += C[i]*v[i]` for the 4 columns, then Ray normalises.
VRT_HD f3 camera_dir(const float s[3], const float u[3], const float nf[3],
                     const float e[3], float z, int nx, int ny, int px, int py,
                     float sx, float sy)
{
        const float x = (float)(px - nx / 2);
        const float y = (float)((ny - 1 - py) - ny / 2);
        const float x_ = (x + sx) / (float)nx;
        const float y_ = (y + sy) / (float)ny;
        float dv[3];
        for (int q = 0; q < 3; ++q) {
                float acc = 0.0f;
                acc += s[q] * x_;
                acc += u[q] * y_;
                acc += nf[q] * z;
                acc += e[q] * 0.0f;
                dv[q] = acc;
        }
        return normalize(mk3(dv[0], dv[1], dv[2]));
}

// gen_rays4 sample offsets Vec2{1,5}/8, {3,1}/8, {7,3}/8, {5,7}/8
VRT_HD float sample_x(int s)
{
        return (s == 0) ? 0.125f : (s == 1) ? 0.375f : (s == 2) ? 0.875f : 0.625f;
}
VRT_HD float sample_y(int s)
{
        return (s == 0) ? 0.625f : (s == 1) ? 0.125f : (s == 2) ? 0.375f : 0.875f;
}

}  // namespace vrt
