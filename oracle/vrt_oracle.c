/*
 * vrt_oracle.c -- TEST INFRASTRUCTURE ONLY (see vrt_oracle.h for the pinning
 * statement).  A literal CPU restatement of the reference's primary-ray hot
 * path, written for readability against the cited reference lines, not for
 * speed.  Build: gcc -O2 -ffp-contract=off -fno-fast-math (x86-64 SSE, no FMA:
 * the reference's /fp:precise MSVC x64 build has the same single-rounding
 * float semantics).
 *
 * Citations: VRT/x = /root/reference/VoxelRayTrace20190722/x
 */
#define _POSIX_C_SOURCE 200809L
#include "vrt_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------ */
/* jql vector arithmetic (VRT/graphics_math.h)                          */
/* ------------------------------------------------------------------ */
typedef struct { float x, y, z; } v3;

static v3 mk(float x, float y, float z) { v3 r = { x, y, z }; return r; }
static v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3 muls(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
/* dot = value_sum(p*q): sum{0}; sum += each product (VRT/graphics_math.h:532-549) */
static float dot(v3 a, v3 b)
{
        float s = 0.0f;
        s += a.x * b.x;
        s += a.y * b.y;
        s += a.z * b.z;
        return s;
}
/* length / normalize: VRT/graphics_math.h:576-586 (per-component division) */
static float length(v3 a) { return sqrtf(dot(a, a)); }
static v3 normalize(v3 a)
{
        float l = length(a);
        return mk(a.x / l, a.y / l, a.z / l);
}
/* cross: VRT/graphics_math.h:588-592 */
static v3 cross(v3 p, v3 q)
{
        return mk(p.y * q.z - q.y * p.z, p.z * q.x - q.z * p.x,
                  p.x * q.y - q.x * p.y);
}
/* jql::clamp(s,min,max) = s > max ? max : (s < min ? min : s)
 * (VRT/graphics_math.h:904-909) */
static float clampf_(float s, float lo, float hi)
{
        return s > hi ? hi : (s < lo ? lo : s);
}
static int clampi_(int s, int lo, int hi)
{
        return s > hi ? hi : (s < lo ? lo : s);
}
/* std::min(a,b) = (b < a) ? b : a ; std::max(a,b) = (a < b) ? b : a */
static float stdmin(float a, float b) { return (b < a) ? b : a; }
static float stdmax(float a, float b) { return (a < b) ? b : a; }
static v3 vget(const float *p) { return mk(p[0], p[1], p[2]); }

/* ------------------------------------------------------------------ */
/* VRT/raytri.cc:197-249  intersect_triangle3 (fp64 Moller-Trumbore)    */
/* ------------------------------------------------------------------ */
#define ORA_EPS 0.000001
int ora_intersect_triangle3(const double orig[3], const double dir[3],
                            const double vert0[3], const double vert1[3],
                            const double vert2[3], double *t, double *u,
                            double *v)
{
        double e1[3], e2[3], tv[3], pv[3], qv[3], det, inv_det;
        /* SUB(edge1, vert1, vert0); SUB(edge2, vert2, vert0) */
        for (int k = 0; k < 3; ++k) {
                e1[k] = vert1[k] - vert0[k];
                e2[k] = vert2[k] - vert0[k];
        }
        /* CROSS(pvec, dir, edge2) */
        pv[0] = dir[1] * e2[2] - dir[2] * e2[1];
        pv[1] = dir[2] * e2[0] - dir[0] * e2[2];
        pv[2] = dir[0] * e2[1] - dir[1] * e2[0];
        det = e1[0] * pv[0] + e1[1] * pv[1] + e1[2] * pv[2];
        for (int k = 0; k < 3; ++k)
                tv[k] = orig[k] - vert0[k];
        inv_det = 1.0 / det; /* division before the det test (raytri.cc:194) */
        qv[0] = tv[1] * e1[2] - tv[2] * e1[1];
        qv[1] = tv[2] * e1[0] - tv[0] * e1[2];
        qv[2] = tv[0] * e1[1] - tv[1] * e1[0];
        if (det > ORA_EPS) {
                *u = tv[0] * pv[0] + tv[1] * pv[1] + tv[2] * pv[2];
                if (*u < 0.0 || *u > det)
                        return 0;
                *v = dir[0] * qv[0] + dir[1] * qv[1] + dir[2] * qv[2];
                if (*v < 0.0 || *u + *v > det)
                        return 0;
        } else if (det < -ORA_EPS) {
                *u = tv[0] * pv[0] + tv[1] * pv[1] + tv[2] * pv[2];
                if (*u > 0.0 || *u < det)
                        return 0;
                *v = dir[0] * qv[0] + dir[1] * qv[1] + dir[2] * qv[2];
                if (*v > 0.0 || *u + *v < det)
                        return 0;
        } else {
                return 0;
        }
        *t = (e2[0] * qv[0] + e2[1] * qv[1] + e2[2] * qv[2]) * inv_det;
        *u *= inv_det;
        *v *= inv_det;
        return 1;
}

/* ------------------------------------------------------------------ */
/* VRT/tribox2.cc:52-196  triBoxOverlap (fp32 SAT, Akenine-Moller)      */
/* ------------------------------------------------------------------ */
static int plane_box_overlap(const float n[3], float d, const float mb[3])
{
        float vmin[3], vmax[3];
        for (int q = 0; q < 3; ++q) {
                if (n[q] > 0.0f) {
                        vmin[q] = -mb[q];
                        vmax[q] = mb[q];
                } else {
                        vmin[q] = mb[q];
                        vmax[q] = -mb[q];
                }
        }
        if (n[0] * vmin[0] + n[1] * vmin[1] + n[2] * vmin[2] + d > 0.0f)
                return 0;
        if (n[0] * vmax[0] + n[1] * vmax[1] + n[2] * vmax[2] + d >= 0.0f)
                return 1;
        return 0;
}

/* One separating-axis test of the 9 edge axes; (pa, pb) are the two
 * projections the reference macro computes (tribox2.cc:77-120), compared in
 * the macro's own order (p0<p2 / p0<p1 / p2<p1). */
static int axis_sep(float pa, float pb, int z12_order, float rad)
{
        float mn, mx;
        if (!z12_order) {
                if (pa < pb) { mn = pa; mx = pb; } else { mn = pb; mx = pa; }
        } else {
                /* AXISTEST_Z12: if(p2<p1) {min=p2; max=p1;} else {min=p1; max=p2;}
                 * called with pa=p1, pb=p2 */
                if (pb < pa) { mn = pb; mx = pa; } else { mn = pa; mx = pb; }
        }
        return (mn > rad || mx < -rad);
}

int ora_tri_box_overlap(const float bc[3], const float bh[3],
                        const float tv[9])
{
        float v0[3], v1[3], v2[3], e0[3], e1[3], e2[3], nrm[3];
        float fex, fey, fez, mn, mx, d;
        for (int k = 0; k < 3; ++k) {
                v0[k] = tv[0 + k] - bc[k];
                v1[k] = tv[3 + k] - bc[k];
                v2[k] = tv[6 + k] - bc[k];
        }
        for (int k = 0; k < 3; ++k) {
                e0[k] = v1[k] - v0[k];
                e1[k] = v2[k] - v1[k];
                e2[k] = v0[k] - v2[k];
        }
#define X_(a, b, va, vb, fa, fb)                                               \
        axis_sep(a * va[1] - b * va[2], a * vb[1] - b * vb[2], 0,            \
                 fa * bh[1] + fb * bh[2])
#define Y_(a, b, va, vb, fa, fb)                                               \
        axis_sep(-a * va[0] + b * va[2], -a * vb[0] + b * vb[2], 0,          \
                 fa * bh[0] + fb * bh[2])
#define Z_(a, b, va, vb, fa, fb, o)                                            \
        axis_sep(a * va[0] - b * va[1], a * vb[0] - b * vb[1], o,            \
                 fa * bh[0] + fb * bh[1])
        /* edge 0: X01, Y02, Z12 */
        fex = fabsf(e0[0]); fey = fabsf(e0[1]); fez = fabsf(e0[2]);
        if (X_(e0[2], e0[1], v0, v2, fez, fey)) return 0;
        if (Y_(e0[2], e0[0], v0, v2, fez, fex)) return 0;
        if (Z_(e0[1], e0[0], v1, v2, fey, fex, 1)) return 0;
        /* edge 1: X01, Y02, Z0 */
        fex = fabsf(e1[0]); fey = fabsf(e1[1]); fez = fabsf(e1[2]);
        if (X_(e1[2], e1[1], v0, v2, fez, fey)) return 0;
        if (Y_(e1[2], e1[0], v0, v2, fez, fex)) return 0;
        if (Z_(e1[1], e1[0], v0, v1, fey, fex, 0)) return 0;
        /* edge 2: X2, Y1, Z12 */
        fex = fabsf(e2[0]); fey = fabsf(e2[1]); fez = fabsf(e2[2]);
        if (X_(e2[2], e2[1], v0, v1, fez, fey)) return 0;
        if (Y_(e2[2], e2[0], v0, v1, fez, fex)) return 0;
        if (Z_(e2[1], e2[0], v1, v2, fey, fex, 1)) return 0;
#undef X_
#undef Y_
#undef Z_
        /* Bullet 1: FINDMINMAX per axis (tribox2.cc:45-50,177-186) */
        for (int k = 0; k < 3; ++k) {
                mn = mx = v0[k];
                if (v1[k] < mn) mn = v1[k];
                if (v1[k] > mx) mx = v1[k];
                if (v2[k] < mn) mn = v2[k];
                if (v2[k] > mx) mx = v2[k];
                if (mn > bh[k] || mx < -bh[k])
                        return 0;
        }
        /* Bullet 2: plane (tribox2.cc:191-193) */
        nrm[0] = e0[1] * e1[2] - e0[2] * e1[1];
        nrm[1] = e0[2] * e1[0] - e0[0] * e1[2];
        nrm[2] = e0[0] * e1[1] - e0[1] * e1[0];
        d = -(nrm[0] * v0[0] + nrm[1] * v0[1] + nrm[2] * v0[2]);
        if (!plane_box_overlap(nrm, d, bh))
                return 0;
        return 1;
}

/* ------------------------------------------------------------------ */
/* Camera (VRT/camera.cc:65-112) and Ray (VRT/graphics_math.h:1150-1167) */
/* ------------------------------------------------------------------ */
void ora_camera_init(float fov, const float eye[3], const float spot[3],
                     const float up[3], float near_, float far_,
                     float cam[19])
{
        v3 e = vget(eye), f = normalize(sub(vget(spot), e));
        v3 s = normalize(cross(f, vget(up)));
        v3 u = normalize(cross(s, f));
        v3 nf = neg(f);
        /* affine_transform(Mat3{s, up_, -forward_}, eye): columns
         * (VRT/graphics_math.h:1002-1016) */
        float C[16] = { s.x, s.y, s.z, 0.f, u.x, u.y, u.z, 0.f,
                        nf.x, nf.y, nf.z, 0.f, e.x, e.y, e.z, 1.f };
        memcpy(cam, C, sizeof C);
        cam[16] = near_;
        cam[17] = far_;
        cam[18] = fov;
}

void ora_make_ray(const float o[3], const float d[3], float tmin, float tmax,
                  float r[8])
{
        v3 dn = normalize(vget(d));
        r[0] = o[0]; r[1] = o[1]; r[2] = o[2];
        r[3] = dn.x; r[4] = dn.y; r[5] = dn.z;
        r[6] = tmin; r[7] = tmax;
}

/* dot(Mat4, Vec4): result{}; result += A[i]*v[i] (VRT/graphics_math.h:552-562) */
static void mat4_vec(const float *C, const float v[4], float out[4])
{
        for (int k = 0; k < 4; ++k) {
                float r = 0.0f;
                for (int i = 0; i < 4; ++i)
                        r += C[4 * i + k] * v[i];
                out[k] = r;
        }
}

static void gen_ray(const float cam[19], float x, float y, float z, float sx,
                    float sy, int nx, int ny, float out[8])
{
        float x_ = (x + sx) / (float)nx;
        float y_ = (y + sy) / (float)ny;
        /* point_transform(C_, {}) (VRT/graphics_math.h:1063-1070) */
        float p[4] = { 0.f, 0.f, 0.f, 1.f }, po[4];
        mat4_vec(cam, p, po);
        float w = po[3];
        float o[3] = { po[0] / w, po[1] / w, po[2] / w };
        /* vector_transform(C_, {x_, y_, z}) (VRT/graphics_math.h:1072-1077) */
        float vv[4] = { x_, y_, z, 0.f }, vo[4];
        mat4_vec(cam, vv, vo);
        ora_make_ray(o, vo, cam[16], cam[17], out);
}

static float cam_z(const float cam[19], float film_h)
{
        /* z = -(film.h / (2 * std::tanf(fov / 2))) (VRT/camera.cc:100) */
        return -(film_h / (2.0f * tanf(cam[18] / 2.0f)));
}

int ora_gen_rays4(const float cam[19], float film_w, float film_h, int nx,
                  int ny, int px, int py, float out[32])
{
        (void)film_w;
        const float x = (float)(px - nx / 2);
        const float y = (float)((ny - 1 - py) - ny / 2);
        const float z = cam_z(cam, film_h);
        static const float S[4][2] = { { 1.f / 8.f, 5.f / 8.f },
                                       { 3.f / 8.f, 1.f / 8.f },
                                       { 7.f / 8.f, 3.f / 8.f },
                                       { 5.f / 8.f, 7.f / 8.f } };
        for (int s = 0; s < 4; ++s)
                gen_ray(cam, x, y, z, S[s][0], S[s][1], nx, ny, out + 8 * s);
        return 4;
}

int ora_gen_rays1(const float cam[19], float film_w, float film_h, int nx,
                  int ny, int px, int py, float out[8])
{
        (void)film_w;
        const float x = (float)(px - nx / 2);
        const float y = (float)((ny - 1 - py) - ny / 2);
        gen_ray(cam, x, y, cam_z(cam, film_h), 0.5f, 0.5f, nx, ny, out);
        return 1;
}

/* ------------------------------------------------------------------ */
/* AABB3D::isect(ray, nullptr): VRT/graphics_math.h:1312-1332           */
/* ------------------------------------------------------------------ */
static int aabb_isect(const float b[6], const float r[8])
{
        float d[3] = { r[3], r[4], r[5] };
        for (int k = 0; k < 3; ++k) /* std::replace(d, 0.f, FLT_MIN) */
                if (d[k] == 0.f)
                        d[k] = FLT_MIN;
        float at0[3], at1[3];
        for (int k = 0; k < 3; ++k) {
                float dinv = 1.f / d[k];
                float t1 = (b[k] - r[k]) * dinv;
                float t2 = (b[3 + k] - r[k]) * dinv;
                at0[k] = stdmin(t1, t2);
                at1[k] = stdmax(t1, t2);
        }
        float t0 = at0[0], t1 = at1[0]; /* max_element / min_element */
        for (int k = 1; k < 3; ++k) {
                if (t0 < at0[k]) t0 = at0[k];
                if (at1[k] < t1) t1 = at1[k];
        }
        if (t0 > t1)
                return 0;
        return (t0 >= r[6] && t0 <= r[7]) || (t1 >= r[6] && t1 <= r[7]);
}
int ora_aabb_isect(const float box[6], const float ray[8])
{
        return aabb_isect(box, ray);
}

/* ------------------------------------------------------------------ */
/* Scene + octree build (VRT/voxel_octree.cc:27-75, 423-431, 486-492)   */
/* ------------------------------------------------------------------ */
typedef struct {
        float box[6];          /* min xyz, max xyz */
        int child;             /* index of first of 8 children, -1 = leaf */
        int depth;
        uint32_t ix, iy, iz;   /* integer coords at this depth */
        int *tris;             /* leaf list (input order) */
        int ntris, cap;
} onode;

typedef struct {
        int tex;  /* -1: Kd */
        float kd[3];
} omat;

typedef struct {
        int w, h, c;
        const uint8_t *data;
} otex;

struct ora_scene {
        int ntri, max_depth;
        float *p;  /* 9 per tri */
        float *n;  /* 9 per tri, normalised (voxel_octree.cc:426) */
        float *t;  /* 6 per tri */
        int *mat;
        onode *nodes;
        int nnodes, capnodes;
        int nmat, ntex;
        omat *mats;
        otex *texs;
        uint8_t *texbytes;
        float *lm_cov;    /* VoxelOctree::coverage per node (full trace) */
        float *lm_illum;  /* VoxelOctree::illum[6] per node, 18 floats */
};

static int new_node(ora_scene *s)
{
        if (s->nnodes == s->capnodes) {
                s->capnodes = s->capnodes ? 2 * s->capnodes : 1024;
                s->nodes = realloc(s->nodes, sizeof(onode) * s->capnodes);
        }
        memset(&s->nodes[s->nnodes], 0, sizeof(onode));
        s->nodes[s->nnodes].child = -1;
        return s->nnodes++;
}

/* Triangle::is_overlap: center=(min+max)*.5f, half=size()/2.f
 * (VRT/voxel_octree.cc:486-492, VRT/graphics_math.h:1252-1260) */
static int tri_overlap(const ora_scene *s, int tri, const float b[6])
{
        float c[3], h[3];
        for (int k = 0; k < 3; ++k) {
                c[k] = (b[k] + b[3 + k]) * .5f;
                h[k] = (b[3 + k] - b[k]) / 2.f;
        }
        return 1 == ora_tri_box_overlap(c, h, s->p + 9 * tri);
}

/* split(): VRT/voxel_octree.cc:27-39 */
static void split(ora_scene *s, int ni)
{
        int first = -1;
        for (int i = 0; i < 8; ++i) {
                int c = new_node(s);
                if (i == 0)
                        first = c;
        }
        onode *nd = &s->nodes[ni];
        float half[3];
        for (int k = 0; k < 3; ++k)
                half[k] = (nd->box[3 + k] - nd->box[k]) / 2; /* size()/2 */
        for (int i = 0; i < 8; ++i) {
                onode *c = &s->nodes[first + i];
                int m[3] = { (i & 4) ? 1 : 0, (i & 2) ? 1 : 0, (i & 1) ? 1 : 0 };
                for (int k = 0; k < 3; ++k) {
                        c->box[k] = nd->box[k] + (float)m[k] * half[k];
                        c->box[3 + k] = c->box[k] + half[k];
                }
                c->depth = nd->depth + 1;
                c->ix = nd->ix * 2 + m[0];
                c->iy = nd->iy * 2 + m[1];
                c->iz = nd->iz * 2 + m[2];
        }
        s->nodes[ni].child = first;
}

/* insert(): VRT/voxel_octree.cc:41-65 */
static void insert(ora_scene *s, int ni, int tri, int cur, int maxd)
{
        if (!tri_overlap(s, tri, s->nodes[ni].box))
                return;
        if (s->nodes[ni].child >= 0) {
                int first = s->nodes[ni].child;
                for (int i = 0; i < 8; ++i)
                        insert(s, first + i, tri, cur + 1, maxd);
                return;
        }
        if (cur == maxd) {
                onode *nd = &s->nodes[ni];
                if (nd->ntris == nd->cap) {
                        nd->cap = nd->cap ? 2 * nd->cap : 4;
                        nd->tris = realloc(nd->tris, sizeof(int) * nd->cap);
                }
                nd->tris[nd->ntris++] = tri;
                return;
        }
        split(s, ni);
        int first = s->nodes[ni].child;
        for (int i = 0; i < 8; ++i)
                insert(s, first + i, tri, cur + 1, maxd);
}

ora_scene *ora_scene_create(const float *pos, const float *nrm,
                            const float *uv, const int32_t *mat, int ntri,
                            int max_depth)
{
        ora_scene *s = calloc(1, sizeof *s);
        s->ntri = ntri;
        s->max_depth = max_depth;
        s->p = malloc(sizeof(float) * 9 * (size_t)(ntri ? ntri : 1));
        s->n = malloc(sizeof(float) * 9 * (size_t)(ntri ? ntri : 1));
        s->t = malloc(sizeof(float) * 6 * (size_t)(ntri ? ntri : 1));
        s->mat = malloc(sizeof(int) * (size_t)(ntri ? ntri : 1));
        memcpy(s->p, pos, sizeof(float) * 9 * (size_t)ntri);
        memcpy(s->t, uv, sizeof(float) * 6 * (size_t)ntri);
        for (int i = 0; i < ntri; ++i) {
                s->mat[i] = mat ? mat[i] : 0;
                for (int v = 0; v < 3; ++v) {
                        v3 nn = normalize(vget(nrm + 9 * i + 3 * v));
                        s->n[9 * i + 3 * v + 0] = nn.x;
                        s->n[9 * i + 3 * v + 1] = nn.y;
                        s->n[9 * i + 3 * v + 2] = nn.z;
                }
        }
        /* ray_march_init: root->aabb = {} then merge every tri AABB
         * (VRT/voxel_octree.cc:67-75; AABB ctor/merge graphics_math.h:1230-1265) */
        int root = new_node(s);
        float rb[6] = { FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX };
        for (int i = 0; i < ntri; ++i) {
                float tb[6] = { FLT_MAX, FLT_MAX, FLT_MAX,
                                -FLT_MAX, -FLT_MAX, -FLT_MAX };
                for (int v = 0; v < 3; ++v)
                        for (int k = 0; k < 3; ++k) {
                                float c = s->p[9 * i + 3 * v + k];
                                tb[k] = stdmin(tb[k], c);
                                tb[3 + k] = stdmax(tb[3 + k], c);
                        }
                for (int k = 0; k < 3; ++k) {
                        rb[k] = stdmin(rb[k], tb[k]);
                        rb[3 + k] = stdmax(rb[3 + k], tb[3 + k]);
                }
        }
        memcpy(s->nodes[root].box, rb, sizeof rb);
        s->nodes[root].depth = 1;
        for (int i = 0; i < ntri; ++i)
                insert(s, root, i, 1, max_depth);
        return s;
}

void ora_scene_set_materials(ora_scene *s, int nmat, const int32_t *mat_tex,
                             const float *mat_kd, int ntex,
                             const int32_t *tex_dims, const int64_t *tex_off,
                             const uint8_t *tex_data, int64_t tex_bytes)
{
        free(s->mats);
        free(s->texs);
        free(s->texbytes);
        s->nmat = nmat;
        s->ntex = ntex;
        s->mats = calloc((size_t)(nmat ? nmat : 1), sizeof(omat));
        s->texs = calloc((size_t)(ntex ? ntex : 1), sizeof(otex));
        s->texbytes = malloc((size_t)(tex_bytes ? tex_bytes : 1));
        if (tex_bytes)
                memcpy(s->texbytes, tex_data, (size_t)tex_bytes);
        for (int m = 0; m < nmat; ++m) {
                s->mats[m].tex = mat_tex[m];
                for (int k = 0; k < 3; ++k)
                        s->mats[m].kd[k] = mat_kd[3 * m + k];
        }
        for (int t = 0; t < ntex; ++t) {
                s->texs[t].w = tex_dims[3 * t];
                s->texs[t].h = tex_dims[3 * t + 1];
                s->texs[t].c = tex_dims[3 * t + 2];
                s->texs[t].data = s->texbytes + tex_off[t];
        }
}

void ora_scene_destroy(ora_scene *s)
{
        if (!s)
                return;
        for (int i = 0; i < s->nnodes; ++i)
                free(s->nodes[i].tris);
        free(s->nodes);
        free(s->p);
        free(s->n);
        free(s->t);
        free(s->mat);
        free(s->mats);
        free(s->texs);
        free(s->texbytes);
        free(s->lm_cov);
        free(s->lm_illum);
        free(s);
}

static uint32_t vox_key(const onode *n)
{
        return n->ix | (n->iy << 10) | (n->iz << 20);
}

void ora_scene_info(const ora_scene *s, int64_t info[5], float root_box[6])
{
        int64_t internal = 0, leaves = 0, nonempty = 0, refs = 0;
        for (int i = 0; i < s->nnodes; ++i) {
                if (s->nodes[i].child >= 0) {
                        internal++;
                } else {
                        leaves++;
                        if (s->nodes[i].ntris) {
                                nonempty++;
                                refs += s->nodes[i].ntris;
                        }
                }
        }
        info[0] = s->nnodes;
        info[1] = internal;
        info[2] = leaves;
        info[3] = nonempty;
        info[4] = refs;
        if (root_box)
                memcpy(root_box, s->nodes[0].box, sizeof(float) * 6);
}

static const ora_scene *g_sort_scene;
static int cmp_leaf(const void *a, const void *b)
{
        uint32_t ka = vox_key(&g_sort_scene->nodes[*(const int *)a]);
        uint32_t kb = vox_key(&g_sort_scene->nodes[*(const int *)b]);
        return ka < kb ? -1 : (ka > kb ? 1 : 0);
}

void ora_scene_leaves(const ora_scene *s, uint32_t *vox, uint32_t *cnt,
                      int32_t *tris)
{
        int nl = 0;
        int *idx = malloc(sizeof(int) * (size_t)(s->nnodes ? s->nnodes : 1));
        for (int i = 0; i < s->nnodes; ++i)
                if (s->nodes[i].child < 0 && s->nodes[i].ntris)
                        idx[nl++] = i;
        g_sort_scene = s;
        qsort(idx, (size_t)nl, sizeof(int), cmp_leaf);
        int64_t o = 0;
        for (int j = 0; j < nl; ++j) {
                const onode *n = &s->nodes[idx[j]];
                vox[j] = vox_key(n);
                cnt[j] = (uint32_t)n->ntris;
                for (int k = 0; k < n->ntris; ++k)
                        tris[o++] = n->tris[k];
        }
        free(idx);
}

/* ------------------------------------------------------------------ */
/* Triangle::isect (VRT/voxel_octree.cc:438-460)                        */
/* ------------------------------------------------------------------ */
typedef struct { v3 hit, normal; } oisect;

static int tri_isect(const ora_scene *s, int tri, const float r[8],
                     oisect *is)
{
        double dt = 0, du = 0, dv = 0;
        double o[3] = { r[0], r[1], r[2] }, d[3] = { r[3], r[4], r[5] };
        const float *P = s->p + 9 * tri;
        double p0[3] = { P[0], P[1], P[2] }, p1[3] = { P[3], P[4], P[5] },
               p2[3] = { P[6], P[7], P[8] };
        if (ora_intersect_triangle3(o, d, p0, p1, p2, &dt, &du, &dv) != 1)
                return 0;
        float u = clampf_((float)du, 0, 1);
        float v = clampf_((float)dv, 0, 1);
        float w = clampf_(1 - u - v, 0, 1);
        const float *N = s->n + 9 * tri;
        /* n_[0]*w + n_[1]*u + n_[2]*v */
        v3 nt = add(add(muls(vget(N), w), muls(vget(N + 3), u)),
                    muls(vget(N + 6), v));
        is->normal = normalize(nt);
        v3 ro = vget(r), rd = vget(r + 3);
        is->hit = add(ro, muls(rd, (float)dt)); /* ray.o + (float)dt * ray.d */
        return 1;
}

/* ------------------------------------------------------------------ */
/* ray_march: VRT/voxel_octree.cc:77-188                                */
/* ------------------------------------------------------------------ */
typedef struct {
        int leaf, tri;
        oisect is;
        uint32_t A, L, T;
} omarch;

/* ray_march_isect (VRT/voxel_octree.cc:99-129): first min of length(hit-o) */
static int march_isect(const ora_scene *s, const onode *leaf, const float r[8],
                       omarch *m)
{
        int best = -1;
        float bestd = 0;
        oisect bis;
        m->L++;
        for (int i = 0; i < leaf->ntris; ++i) {
                oisect is;
                m->T++;
                if (tri_isect(s, leaf->tris[i], r, &is)) {
                        float t = length(sub(is.hit, vget(r)));
                        /* min_element(records, depth <): smallest starts at
                         * the first record; replaced only on strict < */
                        if (best < 0 || t < bestd) {
                                best = leaf->tris[i];
                                bestd = t;
                                bis = is;
                        }
                }
        }
        if (best < 0)
                return 0;
        m->tri = best;
        m->is = bis;
        return 1;
}

/* std::sort(items, items + 8, lhs.dist < rhs.dist) (VRT/voxel_octree.cc:
 * 91-93): for 8 elements libstdc++ runs __insertion_sort alone
 * (stl_algo.h:1855 threshold 16, :1826 move-to-front when val < first, :1806
 * __unguarded_linear_insert shifting while val < prev) -- restated on the
 * child indices.  Pinned against the real libstdc++ by
 * tests/golden/travorder_std.npz. */
void ora_sort8(const float dist[8], int ord[8])
{
        struct { int ci; float dist; } it[8], val;
        for (int ci = 0; ci < 8; ++ci) {
                it[ci].ci = ci;
                it[ci].dist = dist[ci];
        }
        for (int i = 1; i < 8; ++i) {
                val = it[i];
                if (val.dist < it[0].dist) {
                        memmove(&it[1], &it[0], sizeof(it[0]) * (size_t)i);
                        it[0] = val;
                } else {
                        int j = i;
                        while (val.dist < it[j - 1].dist) {
                                it[j] = it[j - 1];
                                --j;
                        }
                        it[j] = val;
                }
        }
        for (int i = 0; i < 8; ++i)
                ord[i] = it[i].ci;
}

/* std::min_element(records, lhs.depth < rhs.depth) (VRT/voxel_octree.cc:
 * 122-125): the first element, replaced only by a strictly smaller one;
 * -1 for an empty range.  Pinned like ora_sort8. */
int ora_first_min(const float *depth, int n)
{
        int best = n > 0 ? 0 : -1;
        for (int i = 1; i < n; ++i)
                if (depth[i] < depth[best])
                        best = i;
        return best;
}

/* travorder (VRT/voxel_octree.cc:77-97): dot(ray.d, child.center() - ray.o)
 * for the 8 children, then the std::sort above */
static void travorder(const ora_scene *s, const onode *nd, const float r[8],
                      int ord[8])
{
        float dist[8];
        v3 o = vget(r), d = vget(r + 3);
        for (int ci = 0; ci < 8; ++ci) {
                const float *b = s->nodes[nd->child + ci].box;
                v3 c = muls(add(vget(b), vget(b + 3)), .5f); /* center() */
                dist[ci] = dot(d, sub(c, o));
        }
        ora_sort8(dist, ord);
}

static int ray_march(const ora_scene *s, const float r[8], omarch *m)
{
        memset(m, 0, sizeof *m);
        m->leaf = -1;
        m->tri = -1;
        const onode *root = &s->nodes[0];
        m->A++;
        if (!aabb_isect(root->box, r))
                return 0;
        if (root->child < 0) {
                if (march_isect(s, root, r, m)) {
                        m->leaf = 0;
                        return 1;
                }
                return 0;
        }
        struct { int node; int ord[8]; int cur; } st[64];
        int sp = 0;
        st[0].node = 0;
        st[0].cur = 0;
        travorder(s, root, r, st[0].ord);
        sp = 1;
        while (sp > 0) {
                int top = sp - 1;
                int ci = st[top].ord[st[top].cur++];
                int child = s->nodes[st[top].node].child + ci;
                if (st[top].cur == 8)
                        --sp;
                const onode *cn = &s->nodes[child];
                m->A++;
                if (!aabb_isect(cn->box, r))
                        continue;
                if (cn->child >= 0) {
                        st[sp].node = child;
                        st[sp].cur = 0;
                        travorder(s, cn, r, st[sp].ord);
                        ++sp;
                        continue;
                }
                if (march_isect(s, cn, r, m)) {
                        m->leaf = child;
                        return 1;
                }
        }
        return 0;
}

void ora_ray_march(const ora_scene *s, const float *rays, int n, int32_t *hit,
                   int32_t *tri, uint32_t *vox, float *hitp, float *nrm,
                   uint32_t *cnt)
{
        for (int i = 0; i < n; ++i) {
                omarch m;
                int h = ray_march(s, rays + 8 * i, &m);
                if (hit) hit[i] = h;
                if (tri) tri[i] = h ? m.tri : -1;
                if (vox) vox[i] = h ? vox_key(&s->nodes[m.leaf]) : 0xFFFFFFFFu;
                if (hitp) {
                        hitp[3 * i + 0] = h ? m.is.hit.x : 0.f;
                        hitp[3 * i + 1] = h ? m.is.hit.y : 0.f;
                        hitp[3 * i + 2] = h ? m.is.hit.z : 0.f;
                }
                if (nrm) {
                        nrm[3 * i + 0] = h ? m.is.normal.x : 0.f;
                        nrm[3 * i + 1] = h ? m.is.normal.y : 0.f;
                        nrm[3 * i + 2] = h ? m.is.normal.z : 0.f;
                }
                if (cnt) {
                        cnt[4 * i + 0] = m.A;
                        cnt[4 * i + 1] = m.L;
                        cnt[4 * i + 2] = m.T;
                        cnt[4 * i + 3] = (uint32_t)h;
                }
        }
}

/* ------------------------------------------------------------------ */
/* Shading: VRT/voxel_octree.cc:392-484, VRT/graphics_math.h:1082-1100, */
/* sky VRT/main.cc:18-20                                                */
/* ------------------------------------------------------------------ */
static float unit_cycle(float s) /* VRT/voxel_octree.cc:392-399 */
{
        while (s > 1.f)
                s -= 1.f;
        while (s < 0.f)
                s += 1.f;
        return s;
}

static v3 barycentric(v3 p, v3 a, v3 b, v3 c)
{
        v3 v0 = sub(b, a), v1 = sub(c, a), v2 = sub(p, a);
        float d00 = dot(v0, v0), d01 = dot(v0, v1), d11 = dot(v1, v1);
        float d20 = dot(v2, v0), d21 = dot(v2, v1);
        float denom = d00 * d11 - d01 * d01;
        if (denom == 0)
                return mk(0, 0, 0); /* "0 area triangle." */
        v3 bc;
        bc.y = (d11 * d20 - d01 * d21) / denom;
        bc.z = (d00 * d21 - d01 * d20) / denom;
        bc.x = 1.0f - bc.y - bc.z;
        return bc;
}

static v3 texel_fetch(const otex *t, float cu, float cv)
{
        int x = clampi_((int)(unit_cycle(cu) * (float)t->w), 0, t->w - 1);
        int y = clampi_((int)(unit_cycle(cv) * (float)t->h), 0, t->h - 1);
        y = t->h - 1 - y;
        const uint8_t *p = t->data + ((size_t)y * t->w + x) * t->c;
        float px[4] = { 0, 0, 0, 0 };
        for (int k = 0; k < t->c && k < 4; ++k)
                px[k] = (float)p[k];
        return mk(px[0] / 255.f, px[1] / 255.f, px[2] / 255.f);
}

static v3 get_albedo(const ora_scene *s, int tri, v3 hit)
{
        const omat *m = &s->mats[s->mat[tri]];
        if (m->tex < 0)
                return mk(m->kd[0], m->kd[1], m->kd[2]);
        const float *P = s->p + 9 * tri, *T = s->t + 6 * tri;
        v3 bc = barycentric(hit, vget(P), vget(P + 3), vget(P + 6));
        bc.x = clampf_(bc.x, 0.f, 1.f);
        bc.y = clampf_(bc.y, 0.f, 1.f);
        bc.z = clampf_(bc.z, 0.f, 1.f);
        /* bc.x * t_[0] + bc.y * t_[1] + bc.z * t_[2] */
        float u = bc.x * T[0] + bc.y * T[2] + bc.z * T[4];
        float v = bc.x * T[1] + bc.y * T[3] + bc.z * T[5];
        return texel_fetch(&s->texs[m->tex], u, v);
}

static v3 shade_sample(const ora_scene *s, const float r[8], int h,
                       const omarch *m)
{
        if (!h) {
                float t = (float)(0.5 * ((double)r[4] + 1.0));
                /* lerp(v0, v1, t) = v0 + (v1 - v0) * t */
                return mk(1.0f + (0.6f - 1.0f) * t, 1.0f + (0.8f - 1.0f) * t,
                          1.0f + (1.0f - 1.0f) * t);
        }
        v3 albedo = get_albedo(s, m->tri, m->is.hit);
        float tmp = dot(m->is.normal, neg(vget(r + 3)));
        tmp = clampf_(tmp, 0.f, 1.f);
        v3 c = muls(albedo, tmp);
        return mk(c.x * 1.f, c.y * 1.f, c.z * 1.f); /* * color(1,1,1) */
}

void ora_shade(const ora_scene *s, const float *rays, int n, float *rgb)
{
        for (int i = 0; i < n; ++i) {
                omarch m;
                int h = ray_march(s, rays + 8 * i, &m);
                v3 c = shade_sample(s, rays + 8 * i, h, &m);
                rgb[3 * i + 0] = c.x;
                rgb[3 * i + 1] = c.y;
                rgb[3 * i + 2] = c.z;
        }
}

/* ------------------------------------------------------------------ */
/* Primary render: VRT/camera.h:42-68 tiles, VRT/main.cc:118-123        */
/* ------------------------------------------------------------------ */
typedef struct {
        const ora_scene *s;
        const float *cam;
        float fw, fh;
        int nx, ny, film_index;
        int row_stride, row_phase; /* render rows with py % stride == phase */
        float *rgb;
        int32_t *s_hit, *s_tri;
        uint32_t *s_vox, *s_cnt;
        float *s_rgb;
        atomic_int next;
} rjob;

static void render_pixel(rjob *j, int px, int py)
{
        float rays[32];
        ora_gen_rays4(j->cam, j->fw, j->fh, j->nx, j->ny, px, py, rays);
        for (int s = 0; s < 4; ++s) {
                omarch m;
                const float *r = rays + 8 * s;
                int h = ray_march(j->s, r, &m);
                v3 c = shade_sample(j->s, r, h, &m);
                size_t si = ((size_t)py * j->nx + px) * 4 + s;
                if (j->s_hit) j->s_hit[si] = h;
                if (j->s_tri) j->s_tri[si] = h ? m.tri : -1;
                if (j->s_vox)
                        j->s_vox[si] = h ? vox_key(&j->s->nodes[m.leaf]) : 0xFFFFFFFFu;
                if (j->s_rgb) {
                        j->s_rgb[3 * si + 0] = c.x;
                        j->s_rgb[3 * si + 1] = c.y;
                        j->s_rgb[3 * si + 2] = c.z;
                }
                if (j->s_cnt) {
                        j->s_cnt[4 * si + 0] = m.A;
                        j->s_cnt[4 * si + 1] = m.L;
                        j->s_cnt[4 * si + 2] = m.T;
                        j->s_cnt[4 * si + 3] = (uint32_t)h;
                }
                /* Film::add(px, py, c * .25f) (VRT/camera.cc:17-20) */
                size_t idx = j->film_index == 0 ? (size_t)py * j->ny + px
                                                : (size_t)py * j->nx + px;
                j->rgb[3 * idx + 0] += c.x * .25f;
                j->rgb[3 * idx + 1] += c.y * .25f;
                j->rgb[3 * idx + 2] += c.z * .25f;
        }
}

/* 8x8 equal tiles, pt = n/8; each tile row-major (VRT/camera.h:45-63).
 * Tiles are handed out dynamically (the reference's pool posts 64 tasks to
 * hardware_concurrency workers); tiles never share pixels (square films). */
static void *render_worker(void *arg)
{
        rjob *j = arg;
        int ptx = j->nx / 8, pty = j->ny / 8;
        for (;;) {
                int t = atomic_fetch_add(&j->next, 1);
                if (t >= 64)
                        break;
                int tx = t % 8, ty = t / 8;
                int x0 = ptx * tx, y0 = pty * ty;
                for (int py = y0; py < y0 + pty; ++py) {
                        if (py % j->row_stride != j->row_phase)
                                continue;
                        for (int px = x0; px < x0 + ptx; ++px)
                                render_pixel(j, px, py);
                }
        }
        return NULL;
}

static void run_job(rjob *j, int nthreads)
{
        atomic_init(&j->next, 0);
        if (nthreads <= 1) {
                render_worker(j);
                return;
        }
        pthread_t *th = malloc(sizeof(pthread_t) * (size_t)nthreads);
        for (int i = 0; i < nthreads; ++i)
                pthread_create(&th[i], NULL, render_worker, j);
        for (int i = 0; i < nthreads; ++i)
                pthread_join(th[i], NULL);
        free(th);
}

void ora_render(const ora_scene *s, const float cam[19], float film_w,
                float film_h, int nx, int ny, int film_index, int nthreads,
                float *rgb, int32_t *s_hit, int32_t *s_tri, uint32_t *s_vox,
                float *s_rgb, uint32_t *s_cnt)
{
        rjob j;
        memset(&j, 0, sizeof j);
        j.s = s;
        j.cam = cam;
        j.fw = film_w;
        j.fh = film_h;
        j.nx = nx;
        j.ny = ny;
        j.film_index = film_index;
        j.row_stride = 1;
        j.row_phase = 0;
        j.rgb = rgb;
        j.s_hit = s_hit;
        j.s_tri = s_tri;
        j.s_vox = s_vox;
        j.s_rgb = s_rgb;
        j.s_cnt = s_cnt;
        memset(rgb, 0, sizeof(float) * 3 * (size_t)nx * ny);
        size_t ns = (size_t)nx * ny * 4;
        if (s_hit) memset(s_hit, 0, sizeof(int32_t) * ns);
        if (s_tri) for (size_t i = 0; i < ns; ++i) s_tri[i] = -1;
        if (s_vox) for (size_t i = 0; i < ns; ++i) s_vox[i] = 0xFFFFFFFFu;
        if (s_rgb) memset(s_rgb, 0, sizeof(float) * 3 * ns);
        if (s_cnt) memset(s_cnt, 0, sizeof(uint32_t) * 4 * ns);
        run_job(&j, nthreads);
}

double ora_render_rows(const ora_scene *s, const float cam[19], float film_w,
                       float film_h, int nx, int ny, int row_stride,
                       int row_phase, int nthreads, float *rgb)
{
        rjob j;
        struct timespec a, b;
        memset(&j, 0, sizeof j);
        j.s = s;
        j.cam = cam;
        j.fw = film_w;
        j.fh = film_h;
        j.nx = nx;
        j.ny = ny;
        j.film_index = 1;
        j.row_stride = row_stride;
        j.row_phase = row_phase;
        j.rgb = rgb;
        clock_gettime(CLOCK_MONOTONIC, &a);
        run_job(&j, nthreads);
        clock_gettime(CLOCK_MONOTONIC, &b);
        return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}

/* One render_mt task (VRT/camera.h:50-60): pixels [x0, x1) x [y0, y1),
 * rows py then columns px, film index y*nx+x; rgb accumulated into.  The
 * caller schedules the tasks (oracle/pool_calib.cc drives it with the
 * reference's own thread_pool_cpp). */
void ora_render_tile(const ora_scene *s, const float cam[19], float film_w,
                     float film_h, int nx, int ny, int x0, int y0, int x1,
                     int y1, float *rgb)
{
        rjob j;
        memset(&j, 0, sizeof j);
        j.s = s;
        j.cam = cam;
        j.fw = film_w;
        j.fh = film_h;
        j.nx = nx;
        j.ny = ny;
        j.film_index = 1;
        j.row_stride = 1;
        j.rgb = rgb;
        for (int py = y0; py < y1; ++py)
                for (int px = x0; px < x1; ++px)
                        render_pixel(&j, px, py);
}

/* stbiw__linear_to_rgbe: VRT/stb_image_write.h:601-616 */
void ora_linear_to_rgbe(const float lin[3], uint8_t rgbe[4])
{
        float mx = lin[1] > lin[2] ? lin[1] : lin[2];
        mx = lin[0] > mx ? lin[0] : mx;
        if (mx < 1e-32f) {
                rgbe[0] = rgbe[1] = rgbe[2] = rgbe[3] = 0;
        } else {
                int e;
                float nrm = (float)frexp(mx, &e) * 256.0f / mx;
                rgbe[0] = (unsigned char)(lin[0] * nrm);
                rgbe[1] = (unsigned char)(lin[1] * nrm);
                rgbe[2] = (unsigned char)(lin[2] * nrm);
                rgbe[3] = (unsigned char)(e + 128);
        }
}

/* ------------------------------------------------------------------ */
/* Config 5: stochastic secondary rays                   */
/* ------------------------------------------------------------------ */
/* jql::PCG::operator() (VRT/graphics_math.h:836-849) */
uint32_t ora_pcg_next(uint64_t *state)
{
        *state = *state * 6364136223846793005ULL + 1442695040888963407ULL;
        const uint64_t s = *state;
        const uint32_t xorshift = (uint32_t)((s ^ (s >> 18u)) >> 27u);
        const uint64_t shift = s >> 59u;
        const int32_t sh32 = (int32_t)(uint32_t)shift; /* reinterpret low 32 bits */
        return (xorshift >> shift) | (xorshift << ((uint32_t)(-sh32) & 31u));
}

/* libstdc++ 11: generate_canonical<float, 24>(pcg) (random.tcc:3348-3380),
 * then uniform_real_distribution<float>{-1,1}: (u * (b - a)) + a. */
float ora_uniform_m11(uint64_t *state)
{
        float sum = 0.0f;
        sum += (float)ora_pcg_next(state) * 1.0f;
        float ret = sum / 4294967296.0f;
        if (ret >= 1.0f)
                ret = nextafterf(1.0f, 0.0f);
        return (ret * (1.0f - -1.0f)) + -1.0f;
}

/* jql::random_point_in_unit_sphere (VRT/graphics_math.h:1208-1216): braced
 * init evaluates d(pcg) left to right; accept when length(r) < 1. */
void ora_random_point_in_unit_sphere(uint64_t *state, float p[3])
{
        for (;;) {
                float x = ora_uniform_m11(state);
                float y = ora_uniform_m11(state);
                float z = ora_uniform_m11(state);
                if (length(mk(x, y, z)) < 1.f) {
                        p[0] = x;
                        p[1] = y;
                        p[2] = z;
                        return;
                }
        }
}

typedef struct {
        const ora_scene *s;
        const float *cam;
        float fw, fh, res;
        int nx, ny, spp;
        float *vis;
        int32_t *s_hit, *s_tri;
        uint32_t *s_vox;
        atomic_int next_row;
        atomic_llong rays;
} sjob;

static void *secondary_worker(void *arg)
{
        sjob *j = arg;
        const int W8 = 8 * (j->nx / 8), H8 = 8 * (j->ny / 8);
        for (;;) {
                const int py = atomic_fetch_add(&j->next_row, 1);
                if (py >= H8)
                        break;
                long long rays = 0;
                for (int px = 0; px < W8; ++px) {
                        float pr[8];
                        ora_gen_rays1(j->cam, j->fw, j->fh, j->nx, j->ny, px, py, pr);
                        omarch m;
                        const size_t pi = (size_t)py * j->nx + px;
                        ++rays;
                        if (!ray_march(j->s, pr, &m)) {
                                j->vis[pi] = 1.0f;
                                continue;
                        }
                        uint64_t st = 0xc01dbeefULL ^ (uint64_t)((uint64_t)py * (uint64_t)j->nx + (uint64_t)px);
                        int misses = 0;
                        for (int s = 0; s < j->spp; ++s) {
                                float p[3], r[8];
                                ora_random_point_in_unit_sphere(&st, p);
                                const float o[3] = { m.is.hit.x, m.is.hit.y, m.is.hit.z };
                                const float d[3] = { m.is.normal.x + p[0], m.is.normal.y + p[1],
                                                     m.is.normal.z + p[2] };
                                ora_make_ray(o, d, j->res, FLT_MAX, r);
                                omarch m2;
                                const int h = ray_march(j->s, r, &m2);
                                ++rays;
                                misses += !h;
                                const size_t si = pi * (size_t)j->spp + s;
                                if (j->s_hit) j->s_hit[si] = h;
                                if (j->s_tri) j->s_tri[si] = h ? m2.tri : -1;
                                if (j->s_vox)
                                        j->s_vox[si] = h ? vox_key(&j->s->nodes[m2.leaf]) : 0xFFFFFFFFu;
                        }
                        j->vis[pi] = (float)misses / (float)j->spp;
                }
                atomic_fetch_add(&j->rays, rays);
        }
        return NULL;
}

int64_t ora_render_secondary(const ora_scene *s, const float cam[19],
                             float film_w, float film_h, int nx, int ny,
                             int spp, int nthreads, float *vis,
                             int32_t *s_hit, int32_t *s_tri, uint32_t *s_vox)
{
        sjob j;
        memset(&j, 0, sizeof j);
        j.s = s;
        j.cam = cam;
        j.fw = film_w;
        j.fh = film_h;
        j.nx = nx;
        j.ny = ny;
        j.spp = spp;
        j.vis = vis;
        j.s_hit = s_hit;
        j.s_tri = s_tri;
        j.s_vox = s_vox;
        /* Res = *min_element(root.aabb.size() / powf(2, D)) (VRT/main.cc:69-70) */
        const float *rb = s->nodes[0].box;
        const float p2 = powf(2.f, (float)s->max_depth);
        float res = (rb[3] - rb[0]) / p2;
        if ((rb[4] - rb[1]) / p2 < res) res = (rb[4] - rb[1]) / p2;
        if ((rb[5] - rb[2]) / p2 < res) res = (rb[5] - rb[2]) / p2;
        j.res = res;
        memset(vis, 0, sizeof(float) * (size_t)nx * ny);
        const size_t ns = (size_t)nx * ny * (size_t)spp;
        if (s_hit) memset(s_hit, 0, sizeof(int32_t) * ns);
        if (s_tri) for (size_t i = 0; i < ns; ++i) s_tri[i] = -1;
        if (s_vox) for (size_t i = 0; i < ns; ++i) s_vox[i] = 0xFFFFFFFFu;
        atomic_init(&j.next_row, 0);
        atomic_init(&j.rays, 0);
        if (nthreads <= 1) {
                secondary_worker(&j);
        } else {
                pthread_t *th = malloc(sizeof(pthread_t) * (size_t)nthreads);
                for (int i = 0; i < nthreads; ++i)
                        pthread_create(&th[i], NULL, secondary_worker, &j);
                for (int i = 0; i < nthreads; ++i)
                        pthread_join(th[i], NULL);
                free(th);
        }
        return (int64_t)atomic_load(&j.rays);
}

/* ------------------------------------------------------------------ */
/* Full trace(): light map, filter, cone tracing     */
/* ------------------------------------------------------------------ */
/* VoxelOctree::illum_d (VRT/voxel_octree.cc:19-20) */
static const float kIllumD[6][3] = { { 1, 0, 0 },  { 0, 1, 0 },  { 0, 0, 1 },
                                     { -1, 0, 0 }, { 0, -1, 0 }, { 0, 0, -1 } };
/* HemiCones (VRT/voxel_octree.cc:256-263): xyz direction, w weight */
static const float kHemi[6][4] = {
        { 0.000000f, 0.000000f, 1.0f, 0.25f },  { 0.000000f, 0.866025f, 0.5f, 0.15f },
        { 0.823639f, 0.267617f, 0.5f, 0.15f },  { 0.509037f, -0.700629f, 0.5f, 0.15f },
        { -0.509037f, -0.700629f, 0.5f, 0.15f }, { -0.823639f, 0.267617f, 0.5f, 0.15f },
};

typedef struct {
        int leaf;   /* -1: no hit */
        v3 illum;   /* get_diffuse(isect, ray, (1,1,1)) */
        v3 normal;  /* isect.normal */
} lsample;

typedef struct {
        const ora_scene *s;
        const float *cam;
        float fw, fh;
        int nx, ny;
        lsample *out;
        atomic_int next;
} ljob;

/* One render_mt task of the light pass (VRT/main.cc:80-97): task
 * t = tx*8 + ty in post order (VRT/camera.h:50-56), pixels row-major,
 * gen_rays4 samples in order.  Sample k of the canonical single-threaded
 * order is stored at out[k]. */
static void *light_worker(void *arg)
{
        ljob *j = arg;
        const int ptx = j->nx / 8, pty = j->ny / 8;
        for (;;) {
                const int t = atomic_fetch_add(&j->next, 1);
                if (t >= 64)
                        break;
                const int tx = t / 8, ty = t % 8;
                size_t k = (size_t)t * (size_t)ptx * (size_t)pty * 4;
                for (int py = pty * ty; py < pty * ty + pty; ++py)
                        for (int px = ptx * tx; px < ptx * tx + ptx; ++px) {
                                float rays[32];
                                ora_gen_rays4(j->cam, j->fw, j->fh, j->nx, j->ny, px, py, rays);
                                for (int q = 0; q < 4; ++q, ++k) {
                                        omarch m;
                                        const float *r = rays + 8 * q;
                                        lsample *o = &j->out[k];
                                        if (!ray_march(j->s, r, &m)) {
                                                o->leaf = -1;
                                                continue;
                                        }
                                        o->leaf = m.leaf;
                                        o->illum = shade_sample(j->s, r, 1, &m);
                                        o->normal = m.is.normal;
                                }
                        }
        }
        return NULL;
}

int64_t ora_lightmap(ora_scene *s, const float cam[19], float film_w,
                     float film_h, int nx, int ny, int nthreads)
{
        free(s->lm_cov);
        free(s->lm_illum);
        s->lm_cov = calloc((size_t)s->nnodes, sizeof(float));
        s->lm_illum = calloc((size_t)s->nnodes * 18, sizeof(float));
        const size_t ns = (size_t)(nx / 8) * (size_t)(ny / 8) * 64 * 4;
        ljob j;
        memset(&j, 0, sizeof j);
        j.s = s;
        j.cam = cam;
        j.fw = film_w;
        j.fh = film_h;
        j.nx = nx;
        j.ny = ny;
        j.out = malloc(sizeof(lsample) * (ns ? ns : 1));
        atomic_init(&j.next, 0);
        if (nthreads <= 1) {
                light_worker(&j);
        } else {
                pthread_t *th = malloc(sizeof(pthread_t) * (size_t)nthreads);
                for (int i = 0; i < nthreads; ++i)
                        pthread_create(&th[i], NULL, light_worker, &j);
                for (int i = 0; i < nthreads; ++i)
                        pthread_join(th[i], NULL);
                free(th);
        }
        /* leaf_ptr->illum[i] += clamp(dot(illum_d[i], n), 0, 1) * illum in
         * the canonical order (the reference's += is racy across tasks) */
        int64_t hits = 0;
        for (size_t k = 0; k < ns; ++k) {
                const lsample *o = &j.out[k];
                if (o->leaf < 0)
                        continue;
                ++hits;
                float *L = s->lm_illum + 18 * (size_t)o->leaf;
                for (int i = 0; i < 6; ++i) {
                        float coeff = dot(vget(kIllumD[i]), o->normal);
                        coeff = clampf_(coeff, 0.f, 1.f);
                        v3 acc = add(vget(L + 3 * i), muls(o->illum, coeff));
                        L[3 * i + 0] = acc.x;
                        L[3 * i + 1] = acc.y;
                        L[3 * i + 2] = acc.z;
                }
        }
        free(j.out);
        return hits;
}

/* cone_trace_init_filter (VRT/voxel_octree.cc:190-214) */
static void filter_node(ora_scene *s, int ni)
{
        onode *nd = &s->nodes[ni];
        float *L = s->lm_illum + 18 * (size_t)ni;
        if (nd->child < 0) {
                if (nd->ntris == 0) {
                        s->lm_cov[ni] = 0;
                        memset(L, 0, sizeof(float) * 18);
                        return;
                }
                s->lm_cov[ni] = 1.f;
                return;
        }
        s->lm_cov[ni] = 0.f;
        memset(L, 0, sizeof(float) * 18);
        const int first = nd->child;
        for (int i = 0; i < 8; ++i) {
                filter_node(s, first + i);
                s->lm_cov[ni] += s->lm_cov[first + i];
                const float *C = s->lm_illum + 18 * (size_t)(first + i);
                for (int f = 0; f < 18; ++f)
                        L[f] += C[f];
        }
        for (int f = 0; f < 18; ++f)
                L[f] /= 8; /* Vec3 /= 8 */
        s->lm_cov[ni] /= 8.f;
}

void ora_lightmap_filter(ora_scene *s)
{
        if (!s->lm_cov) {
                s->lm_cov = calloc((size_t)s->nnodes, sizeof(float));
                s->lm_illum = calloc((size_t)s->nnodes * 18, sizeof(float));
        }
        filter_node(s, 0);
}

void ora_lightmap_nodes(const ora_scene *s, uint64_t *key, float *cov,
                        float *illum)
{
        for (int i = 0; i < s->nnodes; ++i) {
                const onode *n = &s->nodes[i];
                key[i] = ((uint64_t)n->depth << 32) | vox_key(n);
                if (cov) cov[i] = s->lm_cov ? s->lm_cov[i] : 0.f;
                if (illum)
                        for (int f = 0; f < 18; ++f)
                                illum[18 * (size_t)i + f] = s->lm_illum ? s->lm_illum[18 * (size_t)i + f] : 0.f;
        }
}

/* VoxelOctree::compute_illum (VRT/voxel_octree.h:72-82) */
static v3 compute_illum(const ora_scene *s, int ni, v3 d)
{
        v3 r = mk(0, 0, 0);
        const float *L = s->lm_illum + 18 * (size_t)ni;
        for (int i = 0; i < 6; ++i) {
                float coeff = dot(vget(kIllumD[i]), d);
                coeff = clampf_(coeff, 0.f, 1.f);
                r = add(r, muls(vget(L + 3 * i), coeff));
        }
        return r;
}

/* cone_trace(root, cone, min_voxel_size) (VRT/voxel_octree.cc:276-311) */
static v3 cone_march(const ora_scene *s, v3 o, v3 d, float min_voxel)
{
        const float aperture = 0.577350269f, step = .1f, decay = 1.f;
        const float mindist = 1.414f * min_voxel;
        const float *rb = s->nodes[0].box;
        const float maxdist = length(sub(vget(rb + 3), vget(rb)));
        float dist = mindist;
        float opacity = 0.f;
        v3 diffuse = mk(0, 0, 0);
        while (dist < maxdist && opacity < 1.f) {
                const v3 p = add(o, muls(d, dist));
                const float diam = stdmax(mindist, aperture * 2.f * dist);
                if (maxdist < diam)
                        break;
                int split_level = (int)log2f(maxdist / diam);
                int ni = 0;
                while (s->nodes[ni].child >= 0 && split_level) {
                        const float *b = s->nodes[ni].box;
                        const v3 c = muls(add(vget(b), vget(b + 3)), .5f);
                        int i = 0;
                        i += (p.x > c.x ? 4 : 0);
                        i += (p.y > c.y ? 2 : 0);
                        i += (p.z > c.z ? 1 : 0);
                        ni = s->nodes[ni].child + i;
                        split_level--;
                }
                if (split_level == 0) {
                        const v3 illum = compute_illum(s, ni, neg(d));
                        const float transparency = clampf_(1.f - opacity, 0.f, 1.f);
                        const float cov = s->lm_cov[ni];
                        const float a = cov * step;
                        const float w = (1.f / (1 + decay * dist)) * transparency * cov;
                        diffuse = add(diffuse, muls(illum, w));
                        opacity += transparency * a;
                }
                dist += step * diam;
        }
        return diffuse;
}

/* cone_trace(root, isect, min_voxel_size) (VRT/voxel_octree.cc:313-330)
 * with orthonormal_basis (VRT/voxel_octree.cc:265-274) */
static v3 cone_trace_isect(const ora_scene *s, v3 hit, v3 n, float min_voxel)
{
        const float sg = (0.0f > n.z) ? -1.0f : 1.0f;
        const float a0 = -1.0f / (sg + n.z);
        const float a1 = n.x * n.y * a0;
        const v3 t = mk(1.0f + sg * n.x * n.x * a0, sg * a1, -sg * n.x);
        const v3 b = mk(a1, sg + n.y * n.y * a0, -n.y);
        v3 diffuse = mk(0, 0, 0);
        for (int i = 0; i < 6; ++i) {
                /* dot(Mat3{t,b,n}, d) = ((0 + t*d.x) + b*d.y) + n*d.z */
                v3 r = mk(0, 0, 0);
                r = add(r, muls(t, kHemi[i][0]));
                r = add(r, muls(b, kHemi[i][1]));
                r = add(r, muls(n, kHemi[i][2]));
                const v3 cd = normalize(r);
                diffuse = add(diffuse, muls(cone_march(s, hit, cd, min_voxel), kHemi[i][3]));
        }
        return diffuse;
}

float ora_min_voxel(const ora_scene *s, int levels)
{
        const float *rb = s->nodes[0].box;
        const float p2 = powf(2.f, (float)levels);
        float res = (rb[3] - rb[0]) / p2;
        if ((rb[4] - rb[1]) / p2 < res) res = (rb[4] - rb[1]) / p2;
        if ((rb[5] - rb[2]) / p2 < res) res = (rb[5] - rb[2]) / p2;
        return res;
}

/* trace(root, ray, 5, true) (VRT/main.cc:10-30) */
static v3 trace_sample(const ora_scene *s, const float r[8], float res,
                       omarch *m, int *h)
{
        *h = ray_march(s, r, m);
        if (!*h)
                return shade_sample(s, r, 0, m);
        const v3 indirect = cone_trace_isect(s, m->is.hit, m->is.normal, res);
        const v3 direct = compute_illum(s, m->leaf, neg(vget(r + 3)));
        const v3 albedo = get_albedo(s, m->tri, m->is.hit);
        const v3 l = add(indirect, direct);
        return mk(albedo.x * l.x, albedo.y * l.y, albedo.z * l.z);
}

void ora_shade_trace(const ora_scene *s, const float *rays, int n, float res,
                     float *rgb)
{
        for (int i = 0; i < n; ++i) {
                omarch m;
                int h;
                v3 c = trace_sample(s, rays + 8 * i, res, &m, &h);
                rgb[3 * i + 0] = c.x;
                rgb[3 * i + 1] = c.y;
                rgb[3 * i + 2] = c.z;
        }
}

typedef struct {
        const ora_scene *s;
        const float *cam;
        float fw, fh, res;
        int nx, ny;
        float *rgb, *s_rgb;
        int32_t *s_hit;
        atomic_int next;
} tjob;

static void *trace_worker(void *arg)
{
        tjob *j = arg;
        const int ptx = j->nx / 8, pty = j->ny / 8;
        for (;;) {
                const int t = atomic_fetch_add(&j->next, 1);
                if (t >= 64)
                        break;
                const int tx = t / 8, ty = t % 8;
                for (int py = pty * ty; py < pty * ty + pty; ++py)
                        for (int px = ptx * tx; px < ptx * tx + ptx; ++px) {
                                float rays[32];
                                ora_gen_rays4(j->cam, j->fw, j->fh, j->nx, j->ny, px, py, rays);
                                for (int q = 0; q < 4; ++q) {
                                        omarch m;
                                        int h;
                                        const v3 c = trace_sample(j->s, rays + 8 * q, j->res, &m, &h);
                                        const size_t si = ((size_t)py * j->nx + px) * 4 + q;
                                        if (j->s_hit) j->s_hit[si] = h;
                                        if (j->s_rgb) {
                                                j->s_rgb[3 * si + 0] = c.x;
                                                j->s_rgb[3 * si + 1] = c.y;
                                                j->s_rgb[3 * si + 2] = c.z;
                                        }
                                        float *o = j->rgb + ((size_t)py * j->nx + px) * 3;
                                        o[0] += c.x * .25f;
                                        o[1] += c.y * .25f;
                                        o[2] += c.z * .25f;
                                }
                        }
        }
        return NULL;
}

void ora_render_trace(const ora_scene *s, const float cam[19], float film_w,
                      float film_h, int nx, int ny, float res, int nthreads,
                      float *rgb, int32_t *s_hit, float *s_rgb)
{
        tjob j;
        memset(&j, 0, sizeof j);
        j.s = s;
        j.cam = cam;
        j.fw = film_w;
        j.fh = film_h;
        j.res = res;
        j.nx = nx;
        j.ny = ny;
        j.rgb = rgb;
        j.s_rgb = s_rgb;
        j.s_hit = s_hit;
        memset(rgb, 0, sizeof(float) * 3 * (size_t)nx * ny);
        const size_t ns = (size_t)nx * ny * 4;
        if (s_hit) memset(s_hit, 0, sizeof(int32_t) * ns);
        if (s_rgb) memset(s_rgb, 0, sizeof(float) * 3 * ns);
        atomic_init(&j.next, 0);
        if (nthreads <= 1) {
                trace_worker(&j);
        } else {
                pthread_t *th = malloc(sizeof(pthread_t) * (size_t)nthreads);
                for (int i = 0; i < nthreads; ++i)
                        pthread_create(&th[i], NULL, trace_worker, &j);
                for (int i = 0; i < nthreads; ++i)
                        pthread_join(th[i], NULL);
                free(th);
        }
}
